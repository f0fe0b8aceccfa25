#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__device__ static inline uint32_t wave_iscan(uint32_t v)
{
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x142, 0xa, 0xf, false);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x143, 0xc, 0xf, false);
    return v;
}
__global__ void k(const uint32_t* in, uint32_t* out) { out[threadIdx.x] = wave_iscan(in[threadIdx.x]); }
int main() {
  uint32_t h[64], r[64]; for (int i = 0; i < 64; i++) h[i] = (i * 7919u) % 1000;
  uint32_t *di, *dout; hipMalloc(&di, 256); hipMalloc(&dout, 256);
  hipMemcpy(di, h, 256, hipMemcpyHostToDevice); k<<<1, 64>>>(di, dout); hipMemcpy(r, dout, 256, hipMemcpyDeviceToHost);
  uint32_t acc = 0; int bad = 0; for (int i = 0; i < 64; i++) { acc += h[i]; if (r[i] != acc) bad++; }
  printf("scan bad=%d\n", bad); return bad != 0;
}
