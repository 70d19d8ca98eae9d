// Fused step kernel family: R=2 light terms per row, HM=2 heavy rows, XM=2 exceptions,
// heavy mode kHeavyUniform.  One family per translation unit so instantiations compile in parallel.
#include "fused_impl.h"

namespace svh {

const void* fused_kernel_r2uni(int smax, bool paths) {
    return paths ? nullptr : fused_family_ptr<2, 2, 2, kHeavyUniform, false>(smax);
}

}  // namespace svh
