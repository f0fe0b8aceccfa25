// dev probe: does one wave's LDS atomic exchange with conflicting addresses
// process lanes in ascending order (lane i gets the previous same-address
// lane's value)?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
__global__ void k(const uint32_t* addr, uint32_t* got, int trials, int nslot) {
    __shared__ uint32_t t[1024];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int tr = blockIdx.x * 4 + w; tr < trials; tr += gridDim.x * 4) {
        uint32_t* tt = t + w * 256;
        for (int i = lane; i < 256; i += 64) tt[i] = 0xffffffffu;
        __builtin_amdgcn_wave_barrier();
        const uint32_t a = addr[tr * 64 + lane] % nslot;
        const uint32_t r = atomicExch(&tt[a], (uint32_t) lane);
        got[tr * 64 + lane] = r;
        __builtin_amdgcn_wave_barrier();
    }
}
int main() {
    const int trials = 200000;
    for (int nslot = 1; nslot <= 64; nslot *= 4) {
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
            uint32_t last[64];
            for (int s = 0; s < 64; s++) last[s] = 0xffffffffu;
            for (int l = 0; l < 64; l++) {
                uint32_t a = h[tr * 64 + l] % nslot;
                bad += g[tr * 64 + l] != last[a];
                last[a] = l;
            }
        }
        printf("nslot %d: %ld of %d lanes differ from ascending-lane order\n", nslot, bad, trials * 64);
        hipFree(da); hipFree(dg); free(h); free(g);
    }
    return 0;
}
