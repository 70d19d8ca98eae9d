// Golden fixtures through HIP_impl (counterpart of reference tests/test_GraphBLAS_impl.cpp).
#include "HIP_impl.h"
#include "test_helper.h"

int main(int argc, char** argv) {
    const HIP_impl impl;
    const bool ok = hip_test::test_impl(impl, hip_test::data_dir(argc, argv));
    std::printf("test_HIP_impl: %s\n", ok ? "PASS" : "FAIL");
    return ok ? 0 : 1;
}
