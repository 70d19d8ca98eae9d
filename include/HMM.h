// HMM value model for the MI355X Viterbi backend.
//
// Drop-in for the reference's `class HMM` (reference: Viterbi_impl/HMM.h:7-60).  The public
// members, type aliases and static helpers keep the reference's names, types and meaning so
// that code written against the reference (benchmark/, tests/) compiles unchanged against this
// header.  Probabilities are stored "modified": -log2(p) as fp32, +inf for p == 0.
#pragma once

#include <cmath>
#include <cstddef>
#include <limits>
#include <vector>

class HMM {
  public:
    // Type aliases (reference HMM.h:9-16).
    using Probability_t = float;
    using Mod_prob_t = float;
    using Index_t = size_t;
    using Emit_t = size_t;
    using Mod_prob_vec_t = std::vector<Mod_prob_t>;
    using Index_vec_t = std::vector<Index_t>;
    using Emit_seq_t = std::vector<Emit_t>;
    using Emit_seq_vec_t = std::vector<Emit_seq_t>;

    // Hash of a symbol tuple; keys the level-L precomputed products of the _spec path
    // (reference HMM.h:18-26, boost::hash_combine style mixing, bit-identical result).
    struct Emit_seq_hasher {
        std::size_t operator()(const HMM::Emit_seq_t& key) const {
            std::size_t h = key.size();
            for (const auto sym : key) {
                h ^= sym + 0x9e3779b9 + (h << 6) + (h >> 2);
            }
            return h;
        }
    };

    // Sizes.
    Index_t states_num;
    Index_t emit_num;
    Index_t trans_num;

    // Transitions as COO triples src -> dst (reference HMM.h:32-34).
    Index_vec_t trans_rows;     // source state
    Index_vec_t trans_cols;     // destination state
    Mod_prob_vec_t trans_probs; // -log2 p

    // emissions[symbol][state] (symbol-major, reference HMM.h:35 / data_reader.cpp:55).
    std::vector<Mod_prob_vec_t> emissions;

    // Sparse start distribution (reference HMM.h:36-38).
    Index_t non_zero_start_probs;
    Index_vec_t start_probabilities_cols;
    Mod_prob_vec_t start_probabilities;

    // "Impossible" in the -log2 domain (reference HMM.h:41).
    static constexpr auto zero_prob = std::numeric_limits<HMM::Mod_prob_t>::infinity();

    // Reference tolerance |x - y| <= 1.0, or both +inf (reference HMM.h:43-49).
    static bool almost_equal(HMM::Mod_prob_t x, HMM::Mod_prob_t y) {
        if (x == zero_prob && y == zero_prob) {
            return true;
        }
        return std::fabs(x - y) <= 1.0;
    }

    // p -> -log2(p), p <= 0 -> +inf; fp32 log2 exactly as the reference (HMM.h:51-57).
    static HMM::Mod_prob_t to_modified_prob(HMM::Probability_t p) {
        if (!(p > 0.0)) {
            return zero_prob;
        }
        return -1 * std::log2(p);
    }

    static bool is_not_zero_mod_prob(HMM::Mod_prob_t x) { return !almost_equal(x, zero_prob); }
};
