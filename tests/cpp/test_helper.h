// Shared helpers of the C++ parity tests.  Written against the reference interfaces
// (Viterbi_impl / Viterbi_spec_impl), mirroring the reference's test strategy
// (reference tests/test_helper.h:17-73): four golden fixtures, tolerance HMM::almost_equal.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "HMM.h"
#include "Viterbi_impl.h"
#include "Viterbi_spec_impl.h"
#include "data_reader.h"

namespace hip_test {

inline std::string data_dir(int argc, char** argv) {
    if (argc > 1) return argv[1];
    if (const char* d = std::getenv("SVH_DATA")) return d;
    return "data";
}

// Expected scores of the reference's fixtures (values of reference tests/test_helper.h:17-22).
inline std::vector<HMM::Mod_prob_vec_t> expected_results() {
    return {HMM::Mod_prob_vec_t{25.6574f, 24.4874f, HMM::to_modified_prob(0)},
            HMM::Mod_prob_vec_t{HMM::to_modified_prob(0.04608f), HMM::to_modified_prob(0.10752f)},
            HMM::Mod_prob_vec_t{HMM::to_modified_prob(0.00882f), HMM::to_modified_prob(0.02646f)},
            HMM::Mod_prob_vec_t{HMM::to_modified_prob(0), HMM::to_modified_prob(0.00000282f),
                                HMM::to_modified_prob(0.0000181f), HMM::to_modified_prob(0.00000605f)}};
}
constexpr size_t kLevelsToTest = 3;

inline bool same_answer(const HMM::Mod_prob_vec_t& a, const HMM::Mod_prob_vec_t& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (!HMM::almost_equal(a[i], b[i])) {
            std::fprintf(stderr, "  state %zu: %.7g vs %.7g\n", i, a[i], b[i]);
            return false;
        }
    return true;
}

inline HMM fixture_hmm(const std::string& dir, size_t i) {
    return read_HMM(dir + "/chmm_files/test_chmms/" + std::to_string(i) + "_test_chmm.chmm");
}
inline HMM::Emit_seq_t fixture_seq(const std::string& dir, size_t i) {
    return read_emit_seq(dir + "/ess_files/test_sequences/" + std::to_string(i) + "_test_seq.ess")[0];
}

inline bool test_impl(const Viterbi_impl& impl, const std::string& dir) {
    const auto expected = expected_results();
    for (size_t i = 0; i < expected.size(); ++i) {
        const auto res = impl.run_Viterbi(fixture_hmm(dir, i), fixture_seq(dir, i));
        if (!same_answer(res, expected[i])) {
            std::fprintf(stderr, "test_impl fail %zu\n", i);
            return false;
        }
    }
    return true;
}

inline bool test_spec_impl(Viterbi_spec_impl& impl, const std::string& dir) {
    const auto expected = expected_results();
    for (size_t i = 0; i < expected.size(); ++i) {
        impl.spec_with(fixture_hmm(dir, i));
        const auto res = impl.run_Viterbi_spec(fixture_seq(dir, i));
        if (!same_answer(res, expected[i])) {
            std::fprintf(stderr, "test_spec_impl fail %zu (level %zu)\n", i, impl.get_level());
            return false;
        }
    }
    return true;
}

}  // namespace hip_test
