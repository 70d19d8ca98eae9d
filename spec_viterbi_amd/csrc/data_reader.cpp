// .chmm / .ess readers (host side of the boundary).
//
// Behaviour follows the reference readers (reference: Viterbi_impl/data_reader.cpp:17-79 for
// read_HMM, :93-134 for read_emit_seq): whitespace-separated tokens read with iostream
// extraction (so fp32 parsing goes through the same libstdc++ num_get path), each probability
// mapped with HMM::to_modified_prob, emissions transposed to [symbol][state].  Errors print to
// stderr and return an empty object, as the reference does.
#include "data_reader.h"

#include <fstream>
#include <iostream>

namespace {

// Read `count` (index, probability) pairs of the sparse start distribution.
void read_start_distribution(std::istream& in, HMM& hmm) {
    in >> hmm.non_zero_start_probs;
    hmm.start_probabilities_cols.clear();
    hmm.start_probabilities.clear();
    hmm.start_probabilities_cols.reserve(hmm.non_zero_start_probs);
    hmm.start_probabilities.reserve(hmm.non_zero_start_probs);
    // Loop variables live outside the loop: on a truncated file a failed extraction leaves the
    // previous value in place, exactly like the reference's hoisted locals.
    HMM::Index_t state = 0;
    HMM::Probability_t p = 0;
    for (HMM::Index_t k = 0; k < hmm.non_zero_start_probs; ++k) {
        in >> state >> p;
        hmm.start_probabilities_cols.push_back(state);
        hmm.start_probabilities.push_back(HMM::to_modified_prob(p));
    }
}

// File stores one line per state with emit_num probabilities; keep them symbol-major.
void read_emission_table(std::istream& in, HMM& hmm) {
    in >> hmm.emit_num;
    hmm.emissions.assign(hmm.emit_num, HMM::Mod_prob_vec_t(hmm.states_num, HMM::zero_prob));
    HMM::Probability_t p = 0;
    for (HMM::Index_t state = 0; state < hmm.states_num; ++state) {
        for (HMM::Index_t sym = 0; sym < hmm.emit_num; ++sym) {
            in >> p;
            hmm.emissions[sym][state] = HMM::to_modified_prob(p);
        }
    }
}

// Transition triples "src dst p" kept in file order (duplicates are resolved downstream,
// first occurrence wins, like GrB_Matrix_build(..., GrB_FIRST_FP32)).
void read_transitions(std::istream& in, HMM& hmm) {
    in >> hmm.trans_num;
    hmm.trans_rows.clear();
    hmm.trans_cols.clear();
    hmm.trans_probs.clear();
    hmm.trans_rows.reserve(hmm.trans_num);
    hmm.trans_cols.reserve(hmm.trans_num);
    hmm.trans_probs.reserve(hmm.trans_num);
    HMM::Index_t src = 0;
    HMM::Index_t dst = 0;
    HMM::Probability_t p = 0;
    for (HMM::Index_t e = 0; e < hmm.trans_num; ++e) {
        in >> src >> dst >> p;
        hmm.trans_rows.push_back(src);
        hmm.trans_cols.push_back(dst);
        hmm.trans_probs.push_back(HMM::to_modified_prob(p));
    }
}

} // namespace

HMM read_HMM(const std::string& HMM_file_name) {
    std::ifstream in(HMM_file_name);
    if (!in) {
        std::cerr << "Failed to open file with HMM: " << HMM_file_name << '\n';
        return HMM{};
    }
    HMM hmm{};
    in >> hmm.states_num;
    read_start_distribution(in, hmm);
    read_emission_table(in, hmm);
    read_transitions(in, hmm);
    return hmm;
}

HMM::Emit_seq_vec_t read_emit_seq(const std::string& emit_seq_file_name) {
    std::ifstream in(emit_seq_file_name);
    if (!in) {
        std::cerr << "Failed to open file with emitted sequences: " << emit_seq_file_name << '\n';
        return {};
    }
    size_t count = 0;
    in >> count;

    HMM::Emit_seq_vec_t all;
    all.reserve(count);
    size_t id = 0;
    size_t len = 0;
    HMM::Emit_t sym = 0;
    for (size_t expected = 0; expected < count; ++expected) {
        in >> id;
        if (id != expected) {
            std::cerr << "Error in .ess file " << emit_seq_file_name
                      << ": expected sequence number is " << expected << ", but read " << id
                      << '\n';
            return {};
        }
        in >> len;
        HMM::Emit_seq_t seq;
        seq.reserve(len);
        for (size_t k = 0; k < len; ++k) {
            in >> sym;
            seq.push_back(sym);
        }
        all.push_back(std::move(seq));
    }
    return all;
}
