// Dumps what the REFERENCE reader parses (test infrastructure, oracle/_ref only).
// Usage: ref_reader_dump chmm <file> | ref_reader_dump ess <file>
// Output: one token per line; floats as 8-hex-digit IEEE-754 bit patterns.
#include <cstdio>
#include <cstring>
#include <string>

#include "data_reader.h"  // the reference's header, from -I$(REF)/Viterbi_impl

static void f(float x) {
    unsigned u;
    std::memcpy(&u, &x, 4);
    std::printf("%08x\n", u);
}

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    const std::string mode = argv[1];
    if (mode == "chmm") {
        const HMM h = read_HMM(argv[2]);
        std::printf("%zu\n%zu\n%zu\n%zu\n", h.states_num, h.emit_num, h.start_probabilities.size(),
                    h.trans_probs.size());
        for (size_t i = 0; i < h.start_probabilities.size(); ++i) {
            std::printf("%zu\n", h.start_probabilities_cols[i]);
            f(h.start_probabilities[i]);
        }
        for (const auto& row : h.emissions)
            for (float x : row) f(x);
        for (size_t e = 0; e < h.trans_probs.size(); ++e) {
            std::printf("%zu\n%zu\n", h.trans_rows[e], h.trans_cols[e]);
            f(h.trans_probs[e]);
        }
        return 0;
    }
    if (mode == "ess") {
        const auto seqs = read_emit_seq(argv[2]);
        std::printf("%zu\n", seqs.size());
        for (const auto& s : seqs) {
            std::printf("%zu\n", s.size());
            for (auto x : s) std::printf("%zu\n", x);
        }
        return 0;
    }
    return 2;
}
