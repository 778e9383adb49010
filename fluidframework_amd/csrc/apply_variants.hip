// apply_variants.hip -- the runtime-layout apply kernels (every instantiation that is not a
// fixed-capacity replay kernel of apply_caps.hip), compiled in parts (-DMTR_VARIANT_PART=0..
// kVariantParts-1) so the build runs them in parallel.  mtr_engine.hip names the variant it needs
// (enum ApplyVariant) and asks each part in turn to launch it.
#include <hip/hip_runtime.h>

#include <utility>

#include "apply.hip.h"

#ifndef MTR_VARIANT_PART
#error "MTR_VARIANT_PART must be defined"
#endif

namespace mtr {

#define MTR_PASTE2(a, b) a##b
#define MTR_PASTE(a, b) MTR_PASTE2(a, b)

template <class... Args>
static void go(void (*k)(Args...), bool& attr, uint32_t grid, size_t lds, hipStream_t st, Args... args) {
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(NT), lds, st, args...);
}
template <class... Args>
static void go2(void (*k)(Args...), bool& attr, uint32_t grid, size_t lds, hipStream_t st, Args... args) {
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(2 * NT), lds, st, args...);  // two waves per workgroup
}

template <class... Args>
static void go_team(void (*k)(Args...), bool& attr, uint32_t grid, size_t lds, hipStream_t st, Args... args) {
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k, dim3(grid), dim3(MTR_GW * NT), lds, st, args...);  // an HBM-resident document's team
}

// one variant, instantiated only in the part that owns it (V % kVariantParts)
template <int V>
static bool try_variant(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region) {
    if constexpr (V % kVariantParts == MTR_VARIANT_PART) {
        if (v != V) return false;
        static bool attr = false;
        if constexpr (V == AV_LDS_X) go(apply_kernel<false>, attr, grid, lds, st, P);
        if constexpr (V == AV_HBM_X) go(apply_kernel<true>, attr, grid, lds, st, P);
        if constexpr (V == AV_LDS_LEAN) go(apply_kernel<false, -1>, attr, grid, lds, st, P);
        if constexpr (V == AV_HBM_LEAN) go_team(apply_kernel<true, -1>, attr, grid, lds, st, P);
        if constexpr (V == AV_LDS_DL) go(apply_kernel<false, 0, true>, attr, grid, lds, st, P);
        if constexpr (V == AV_HBM_DL) go(apply_kernel<true, 0, true>, attr, grid, lds, st, P);
        if constexpr (V == AV_LDS_GN) go(apply_kernel<false, 0, false, true>, attr, grid, lds, st, P);
        if constexpr (V == AV_HBM_GN) go(apply_kernel<true, 0, false, true>, attr, grid, lds, st, P);
        if constexpr (V == AV_PAIR_LDS) go(apply_pair_kernel<false>, attr, grid, lds, st, P, region);
        if constexpr (V == AV_PAIR_HBM) go(apply_pair_kernel<true>, attr, grid, lds, st, P, region);
        if constexpr (V == AV_PAIR_LDS_DL) go(apply_pair_kernel<false, true>, attr, grid, lds, st, P, region);
        if constexpr (V == AV_PAIR_HBM_DL) go(apply_pair_kernel<true, true>, attr, grid, lds, st, P, region);
        if constexpr (V == AV_PAIR_LDS_GN) go(apply_pair_kernel<false, false, true>, attr, grid, lds, st, P, region);
        if constexpr (V == AV_PAIR_HBM_GN) go(apply_pair_kernel<true, false, true>, attr, grid, lds, st, P, region);
        if constexpr (V == AV_PAIR2_LDS) go2(apply_pair2_kernel<false>, attr, grid, lds, st, P, region);
        if constexpr (V == AV_PAIR2_HBM) go2(apply_pair2_kernel<true>, attr, grid, lds, st, P, region);
        return true;
    }
    return false;
}

template <int... Vs>
static bool try_all(int v, uint32_t grid, size_t lds, hipStream_t st, const KParams& P, uint32_t region,
                    std::integer_sequence<int, Vs...>) {
    return (try_variant<Vs>(v, grid, lds, st, P, region) || ...);
}

bool MTR_PASTE(launch_variant_p, MTR_VARIANT_PART)(int v, uint32_t grid, size_t lds, hipStream_t st,
                                                    const KParams& P, uint32_t region) {
    return try_all(v, grid, lds, st, P, region, std::make_integer_sequence<int, AV_COUNT>{});
}

}  // namespace mtr
