// apply_caps.hip -- the fixed-capacity replay kernels (apply_kernel<false, CAP>, compile-time LDS
// layout per leaf capacity), compiled in parts (-DMTR_CAP_PART=0..kCapParts-1) so the build runs
// them in parallel.  mtr_engine.hip asks each part in turn to launch a class's kernel.
#include <hip/hip_runtime.h>

#include "apply.hip.h"

#ifndef MTR_CAP_PART
#error "MTR_CAP_PART must be defined"
#endif

namespace mtr {

#define MTR_PASTE2(a, b) a##b
#define MTR_PASTE(a, b) MTR_PASTE2(a, b)

// the capacities of this part: C / 32 % kCapParts == MTR_CAP_PART (compile-time selection, so
// each part instantiates only its own kernels)
template <int C>
static bool try_cap(int cap, uint32_t grid, size_t lds, hipStream_t st, const KParams& P) {
    if constexpr ((C / 32) % kCapParts == MTR_CAP_PART) {
        if (cap == C) {
            static bool attr = false;
            if (!attr) {
                (void)hipFuncSetAttribute((const void*)apply_kernel<false, C>,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                attr = true;
            }
            apply_kernel<false, C><<<grid, NT, lds, st>>>(P);
            return true;
        }
    }
    return false;
}

#define MTR_PART_CASE(C) \
    if (try_cap<C>(cap, grid, lds, st, P)) return true;

// launches apply_kernel<false, cap> if this part owns that capacity
bool MTR_PASTE(launch_fixed_cap_p, MTR_CAP_PART)(int cap, uint32_t grid, size_t lds, hipStream_t st,
                                                  const KParams& P) {
    MTR_FIXED_CAPS(MTR_PART_CASE)
    return false;
}

}  // namespace mtr
