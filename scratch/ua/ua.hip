// dev probe: are unaligned LDS dword reads correct on this GPU?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
__global__ void k(uint32_t* out, const uint8_t* in, const uint32_t* offs, int n) {
    __shared__ uint8_t w[8192];
    for (int i = threadIdx.x; i < 8192; i += blockDim.x) w[i] = in[i];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        uint32_t v;
        __builtin_memcpy(&v, w + offs[i], 4);
        out[i] = v;
    }
}
int main() {
    const int n = 65536;
    uint8_t h[8192]; uint32_t ho[n], hr[n];
    for (int i = 0; i < 8192; i++) h[i] = (uint8_t) (i * 131 + 7 + (i >> 8));
    for (int i = 0; i < n; i++) ho[i] = (uint32_t) ((i * 2654435761u) % 8188u);
    uint8_t* din; uint32_t *doff, *dout;
    hipMalloc(&din, 8192); hipMalloc(&doff, n * 4); hipMalloc(&dout, n * 4);
    hipMemcpy(din, h, 8192, hipMemcpyHostToDevice); hipMemcpy(doff, ho, n * 4, hipMemcpyHostToDevice);
    k<<<1, 256>>>(dout, din, doff, n);
    hipMemcpy(hr, dout, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; i++) { uint32_t v; memcpy(&v, h + ho[i], 4); bad += v != hr[i]; }
    printf("unaligned LDS dword reads: %d of %d wrong\n", bad, n);
    return bad != 0;
}
