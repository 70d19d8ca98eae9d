// Fused step kernel family: R=4 light terms per row, HM=4 heavy rows, XM=4 exceptions,
// heavy mode kHeavyGeneral.  One family per translation unit so instantiations compile in parallel.
#include "fused_impl.h"

namespace svh {

const void* fused_kernel_r4(int smax, bool paths) {
    return paths ? fused_family_ptr<4, 4, 4, kHeavyGeneral, true>(smax)
                 : fused_family_ptr<4, 4, 4, kHeavyGeneral, false>(smax);
}

}  // namespace svh
