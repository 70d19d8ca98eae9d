// Cross-path equality over every .chmm x emit_3_3500_20.ess (counterpart of reference
// tests/test_semantic_equality.cpp): non-spec == spec level 1 (bit-identical here) and
// spec level 2 within HMM::almost_equal, exactly the reference's checks.
#include <dirent.h>

#include <algorithm>
#include <memory>

#include "HIP_impl.h"
#include "HIP_spec_impl.h"
#include "test_helper.h"

int main(int argc, char** argv) {
    const std::string dir = hip_test::data_dir(argc, argv);
    const auto sequences = read_emit_seq(dir + "/ess_files/emit_3_3500_20.ess");
    if (sequences.empty()) return 1;
    std::vector<std::string> models;
    if (DIR* d = opendir((dir + "/chmm_files").c_str())) {
        while (dirent* e = readdir(d)) {
            const std::string name = e->d_name;
            if (name.size() > 5 && name.substr(name.size() - 5) == ".chmm") models.push_back(name);
        }
        closedir(d);
    }
    std::sort(models.begin(), models.end());
    const HIP_impl non_spec;
    for (const auto& name : models) {
        const HMM hmm = read_HMM(dir + "/chmm_files/" + name);
        HIP_spec_impl spec1(1), spec2(2);
        spec1.spec_with(hmm);
        spec2.spec_with(hmm);
        const auto a = non_spec.run_Viterbi_batch(hmm, sequences);
        const auto b = spec1.run_Viterbi_spec_batch(sequences);
        const auto c = spec2.run_Viterbi_spec_batch(sequences);
        for (size_t q = 0; q < sequences.size(); ++q) {
            if (a[q] != b[q]) {
                std::fprintf(stderr, "%s seq %zu: non-spec and spec level 1 differ\n", name.c_str(), q);
                return 1;
            }
            if (!hip_test::same_answer(b[q], c[q])) {
                std::fprintf(stderr, "%s seq %zu: spec levels 1 and 2 differ\n", name.c_str(), q);
                return 1;
            }
        }
        std::printf("%s ok\n", name.c_str());
    }
    std::printf("test_semantic_equality: PASS (%zu models)\n", models.size());
    return 0;
}
