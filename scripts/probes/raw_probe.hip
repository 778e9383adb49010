// Probe: a lane-0 global store, a wave-scope fence + wave barrier (Eng's wsync), then every lane loads the
// same word.  mode 0: no wait; mode 1: s_waitcnt vmcnt(0) after the store.  warm: the line was loaded first.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(1))) int* gi;
__device__ inline void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ void probe(int* a, int* bad, int iters, int warm, int mode) {
    gi g = (gi)a + blockIdx.x * 1024;
    int miss = 0;
    for (int it = 1; it <= iters; it++) {
        const int slot = (it * 7) & 511;
        int w = 0;
        if (warm) w = g[slot + (threadIdx.x & 15)];
        asm volatile("" :: "v"(w));
        wsync();
        if (threadIdx.x == 0) g[slot] = it;
        if (mode) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wsync();
        const int r = g[slot];
        miss += (r != it);
        wsync();
    }
    if (miss) atomicAdd(bad, miss);
}
int main() {
    int *a, *bad;
    hipMalloc(&a, 4 * 1024 * 1024);
    hipMalloc(&bad, 4);
    for (int mode = 0; mode < 2; mode++)
        for (int warm = 0; warm < 2; warm++) {
            hipMemset(a, 0, 4 * 1024 * 1024);
            hipMemset(bad, 0, 4);
            probe<<<1000, 64>>>(a, bad, 20000, warm, mode);
            int h = 0;
            (void)hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
            printf("mode=%d warm=%d mismatches=%d of %d lane-loads\n", mode, warm, h, 1000 * 64 * 20000);
        }
    return 0;
}
