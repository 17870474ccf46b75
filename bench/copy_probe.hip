// copy_probe.hip — development probe (not part of the product): the HBM ceilings the decode kernel's
// traffic mix can reach on this MI355X, to price its skeleton (round 5). Config 5's decode reads
// ~1.13 GB (input + offsets) and writes ~1.31 GB (decoded bytes + lengths + statuses) per launch.
//   read   : every lane sums 16-byte chunks of a 1.13 GB buffer (grid-stride, 4 chunks in flight)
//   write  : every lane stores 16-byte chunks over a 1.31 GB buffer
//   copy   : reads a 1.13 GB buffer and writes a 1.31 GB one in the same loop (the mix, 8:9.3)
// One workgroup of 1024 threads per CU (256) like the decode kernel, and 2048-thread grids x 2 per
// CU for comparison. Prints one JSON line per variant: microseconds per launch, GB/s of traffic.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(2);                                                                          \
        }                                                                                     \
    } while (0)

// kRd / kWr: read / write the two buffers; chunks are 16 B, nr / nw chunks in each; kNt: nontemporal
// stores (1), loads and stores (2); kF: chunks in flight per lane
template <bool kRd, bool kWr, int kNt = 0, int kF = 4>
__global__ __launch_bounds__(1024) void stream(const uint4* __restrict__ in, uint64_t nr, uint4* __restrict__ out,
                                               uint64_t nw, uint32_t* sink) {
    const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    const uint64_t n = nr > nw ? nr : nw;
    for (uint64_t i = t0; i < n; i += kF * T) {
        uint4 v[kF];
#pragma unroll
        for (int k = 0; k < kF; ++k) {
            const uint64_t j = i + k * T;
            if (kRd && j < nr) {
                if (kNt >= 2) {
                    v[k].x = __builtin_nontemporal_load(&in[j].x);
                    v[k].y = __builtin_nontemporal_load(&in[j].y);
                    v[k].z = __builtin_nontemporal_load(&in[j].z);
                    v[k].w = __builtin_nontemporal_load(&in[j].w);
                } else {
                    v[k] = in[j];
                }
            } else {
                v[k] = make_uint4((uint32_t)j, 1u, 2u, 3u);
            }
        }
#pragma unroll
        for (int k = 0; k < kF; ++k) {
            const uint64_t j = i + k * T;
            if (kWr && j < nw) {
                if (kNt >= 1) {
                    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                    const v4u x = {v[k].x, v[k].y, v[k].z, v[k].w};
                    __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(&out[j]));
                }
                else
                    out[j] = v[k];
            }
            acc += v[k].x ^ v[k].w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

template <bool kRd, bool kWr, int kNt = 0, int kF = 4>
static void run(const char* name, const uint4* in, uint64_t nr, uint4* out, uint64_t nw, uint32_t* sink, int blocks,
                int threads) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((stream<kRd, kWr, kNt, kF>), dim3(blocks), dim3(threads), 0, 0, in, nr, out, nw, sink);
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL((stream<kRd, kWr, kNt, kF>), dim3(blocks), dim3(threads), 0, 0, in, nr, out, nw, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = ms * 1e3 / reps;
    const double bytes = (kRd ? nr * 16.0 : 0) + (kWr ? nw * 16.0 : 0);
    printf("{\"variant\": \"%s\", \"nt\": %d, \"inflight\": %d, \"blocks\": %d, \"threads\": %d, \"us\": %.1f, \"GB_s\": %.1f}\n", name, kNt, kF,
           blocks, threads, us, bytes / us * 1e-3);
}

int main() {
    const uint64_t rb = 1127000000ull, wb = 1312000000ull;
    const uint64_t nr = rb / 16, nw = wb / 16;
    uint4 *in, *out;
    uint32_t* sink;
    CK(hipMalloc(&in, nr * 16));
    CK(hipMalloc(&out, nw * 16));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(in, 1, nr * 16));
    for (int cfg = 0; cfg < 2; ++cfg) {
        const int blocks = cfg ? 512 : 256, threads = 1024;
        run<true, false>("read", in, nr, out, nw, sink, blocks, threads);
        run<false, true>("write", in, nr, out, nw, sink, blocks, threads);
        run<true, true>("copy", in, nr, out, nw, sink, blocks, threads);
        run<false, true, 1>("write", in, nr, out, nw, sink, blocks, threads);
        run<true, true, 1>("copy", in, nr, out, nw, sink, blocks, threads);
        run<true, true, 2>("copy", in, nr, out, nw, sink, blocks, threads);
        run<true, true, 0, 8>("copy", in, nr, out, nw, sink, blocks, threads);
        run<true, true, 1, 8>("copy", in, nr, out, nw, sink, blocks, threads);
        run<true, false, 0, 8>("read", in, nr, out, nw, sink, blocks, threads);
    }
    // the float4 copy of the microarchitecture guide: one 16-byte chunk per thread, a grid over the buffer
    run<true, true, 0, 1>("copy_flat", in, nr, out, nr, sink, (int)((nr + 1023) / 1024), 1024);
    run<true, true, 1, 1>("copy_flat", in, nr, out, nr, sink, (int)((nr + 1023) / 1024), 1024);
    run<true, true, 0, 1>("copy_flat256", in, nr, out, nr, sink, (int)((nr + 255) / 256), 256);
    return 0;
}
