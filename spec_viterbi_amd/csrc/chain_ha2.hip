// Chain kernel instantiations with two heavy feeders.
#include "chain_impl.h"

namespace svh {
namespace {
template <int HA>
const void* chain_ptr(int sm, int waves, bool ge) {
    switch (waves) {
        case 1: return chain_ptr_w<1, HA>(sm, ge);
        case 2: return chain_ptr_w<2, HA>(sm, ge);
        case 4: return chain_ptr_w<4, HA>(sm, ge);
        case 8: return chain_ptr_w<8, HA>(sm, ge);
        default: return nullptr;
    }
}
}  // namespace

const void* chain_fn_ha2(int sm, int waves, bool ge) { return chain_ptr<2>(sm, waves, ge); }

}  // namespace svh
