// Golden fixtures through HIP_spec_impl at levels 1..3 (counterpart of reference
// tests/test_GraphBLAS_spec_impl.cpp; spec_with is re-called per fixture).
#include "HIP_spec_impl.h"
#include "test_helper.h"

int main(int argc, char** argv) {
    const std::string dir = hip_test::data_dir(argc, argv);
    bool ok = true;
    for (size_t lvl = 1; lvl <= hip_test::kLevelsToTest; ++lvl) {
        HIP_spec_impl impl(lvl);
        ok &= hip_test::test_spec_impl(impl, dir);
    }
    std::printf("test_HIP_spec_impl: %s\n", ok ? "PASS" : "FAIL");
    return ok ? 0 : 1;
}
