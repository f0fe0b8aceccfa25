// dev probe: ds_mskor_rtn_b32 as a 16-bit exchange inside a 32-bit LDS word:
// lanes with the same half-word must see the previous same-address lane's value
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
__device__ inline uint32_t mskor_rtn(uint32_t* p, uint32_t mask, uint32_t data) {
    uint32_t r;
    const uint32_t a = (uint32_t) (uintptr_t) p;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n s_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a), "v"(mask), "v"(data) : "memory");
    return r;
}
__global__ void k(const uint32_t* addr, uint32_t* got, int trials, int nslot) {
    __shared__ uint32_t t[1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int tr = blockIdx.x * 4 + w; tr < trials; tr += gridDim.x * 4) {
        uint32_t* tt = t + w * 256;
        for (int i = lane; i < 256; i += 64) tt[i] = 0xffffffffu;
        __builtin_amdgcn_wave_barrier();
        const uint32_t a = addr[tr * 64 + lane] % nslot;       /* half-word slot */
        const uint32_t sh = (a & 1) * 16;
        const uint32_t old = mskor_rtn(&tt[a >> 1], 0xffffu << sh, (uint32_t) lane << sh);
        got[tr * 64 + lane] = (old >> sh) & 0xffff;
        __builtin_amdgcn_wave_barrier();
    }
}
int main() {
    const int trials = 200000;
    for (int nslot = 2; nslot <= 128; nslot *= 4) {
        uint32_t* h = (uint32_t*) malloc(trials * 64 * 4);
        uint32_t* g = (uint32_t*) malloc(trials * 64 * 4);
        srand(nslot);
        for (int i = 0; i < trials * 64; i++) h[i] = rand();
        uint32_t *da, *dg;
        if (hipMalloc(&da, trials * 256) || hipMalloc(&dg, trials * 256)) return 2;
        if (hipMemcpy(da, h, trials * 256, hipMemcpyHostToDevice)) return 2;
        k<<<1024, 256>>>(da, dg, trials, nslot);
        if (hipMemcpy(g, dg, trials * 256, hipMemcpyDeviceToHost)) return 2;
        long bad = 0;
        for (int tr = 0; tr < trials; tr++) {
            uint32_t last[128];
            for (int s = 0; s < 128; s++) last[s] = 0xffffu;
            for (int l = 0; l < 64; l++) {
                uint32_t a = h[tr * 64 + l] % nslot;
                bad += g[tr * 64 + l] != last[a];
                last[a] = l;
            }
        }
        printf("nslot %d: %ld of %d lanes differ\n", nslot, bad, trials * 64);
        hipFree(da); hipFree(dg); free(h); free(g);
    }
    return 0;
}
