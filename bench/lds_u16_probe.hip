// Dev probe: does an unaligned 16-bit LDS store (ds_write_b16 at odd addresses) land correctly on gfx950?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
typedef uint16_t __attribute__((aligned(1))) u16u;
__global__ void k(uint8_t* out, int shift) {
    __shared__ uint8_t s[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) s[i] = 0xEE;
    __syncthreads();
    const uint32_t pos = threadIdx.x * 3 + shift;  // odd and even positions
    *(u16u*)(s + pos) = (uint16_t)(0x0100 * ((threadIdx.x + 1) & 0xFF) | (threadIdx.x & 0xFF));
    __syncthreads();
    for (int i = threadIdx.x; i < 256; i += 64) out[i] = s[i];
}
int main() {
    uint8_t* d; hipMalloc(&d, 256);
    uint8_t h[256];
    int bad = 0;
    for (int shift = 0; shift < 2; ++shift) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, shift);
        hipMemcpy(h, d, 256, hipMemcpyDeviceToHost);
        for (int t = 0; t < 64; ++t) {
            const int p = t * 3 + shift;
            if (h[p] != (t & 0xFF) || h[p + 1] != ((t + 1) & 0xFF)) bad++;
        }
    }
    printf("{\"u16_unaligned_lds_bad\": %d}\n", bad);
    return 0;
}
