// ta_probe.hip — development probe (not part of the product): what per-lane streams cost the
// vector-memory path on gfx950, to choose between a decode design where every lane streams its own
// contiguous literal range (16-B loads / stores at 64 different addresses per wave-instruction)
// and one where a wave moves coalesced 1-KiB pieces.
//
// Each of 256 x 1024 lanes owns a contiguous input stream of S bytes and an output stream of
// S * 4 / 3 bytes. Per iteration a lane loads `kLd` 16-byte chunks of its input (register staging,
// written to a per-lane LDS ring the next iteration), does `kAlu` dependent VALU operations on a
// value it read from the ring (the decode's stand-in), and stores `kSt` 16-byte chunks of output.
// Variant "coal": the same bytes per wave, but lane t of a wave takes chunk t of the wave's
// contiguous 1-KiB piece (the wave owns 64 consecutive lane streams' bytes).
// Prints one JSON line per variant: microseconds per launch and GB/s moved.
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

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// kCoal = 0: lane streams; 1: wave-coalesced pieces. S: input bytes per lane (multiple of 16 * kLd).
template <int kLd, int kSt, int kAlu, int kCoal>
__global__ __launch_bounds__(1024) void probe(const uint8_t* in, uint8_t* out, uint32_t S, uint32_t in_bytes,
                                              uint32_t out_bytes, uint32_t* sink) {
    __shared__ uint32_t ring[16 * 1024];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint64_t gl = (uint64_t)blockIdx.x * 1024 + tid;
    const uint64_t gw = gl >> 6;
    const __amdgpu_buffer_rsrc_t ri = rsrc(in, in_bytes), ro = rsrc(out, out_bytes);
    const uint32_t iters = S / (16u * kLd);
    u32x4 P[kLd];
    for (int k = 0; k < kLd; ++k) P[k] = u32x4{0, 0, 0, 0};
    uint32_t acc = tid, h = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        // previous iteration's chunks to the ring
        for (int k = 0; k < kLd; ++k) {
            ring[((h + 4 * k + 0) & 15u) * 1024 + tid] = P[k].x;
            ring[((h + 4 * k + 1) & 15u) * 1024 + tid] = P[k].y;
            ring[((h + 4 * k + 2) & 15u) * 1024 + tid] = P[k].z;
            ring[((h + 4 * k + 3) & 15u) * 1024 + tid] = P[k].w;
        }
        h += 4 * kLd;
        for (int k = 0; k < kLd; ++k) {
            uint32_t off;
            if (kCoal)  // wave piece: 64 lanes x 16 B contiguous, pieces of the wave's span in order
                off = (uint32_t)((gw * 64ull * S) + ((uint64_t)it * kLd + k) * 1024ull + lane * 16ull);
            else  // the lane's own stream
                off = (uint32_t)(gl * S + ((uint64_t)it * kLd + k) * 16ull);
            P[k] = __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, 0);
        }
        uint32_t v = ring[((h + tid) & 15u) * 1024 + tid];
#pragma unroll
        for (int a = 0; a < kAlu; ++a) v = __builtin_amdgcn_alignbit(v, acc, a + 1) ^ (v >> 3);
        acc += v;
        for (int k = 0; k < kSt; ++k) {
            uint32_t off;
            if (kCoal)
                off = (uint32_t)((gw * 64ull * S * 4 / 3) + ((uint64_t)it * kSt + k) * 1024ull + lane * 16ull);
            else
                off = (uint32_t)(gl * (S * 4 / 3) + ((uint64_t)it * kSt + k) * 16ull);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{acc, v, acc ^ v, it}, ro, off, 0, 0);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;  // keep the work
}

template <int kLd, int kSt, int kAlu, int kCoal>
static void run(const char* name, const uint8_t* in, uint8_t* out, uint32_t S, uint32_t ib, uint32_t ob,
                uint32_t* sink) {
    dim3 g(256), b(1024);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((probe<kLd, kSt, kAlu, kCoal>), g, b, 0, 0, in, out, S, ib, ob, sink);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 10;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((probe<kLd, kSt, kAlu, kCoal>), g, b, 0, 0, in, out, S, ib, ob, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / reps;
    const uint32_t iters = S / (16u * kLd);
    const double rd = 262144.0 * iters * kLd * 16, wr = 262144.0 * iters * kSt * 16;
    printf("{\"variant\": \"%s\", \"S\": %u, \"us\": %.1f, \"read_GBs\": %.0f, \"write_GBs\": %.0f, "
           "\"vmem_instr_per_cu\": %.0f, \"cycles_per_vmem_instr_at_2.4GHz\": %.1f}\n",
           name, S, us, rd / us / 1e3, wr / us / 1e3, 1024.0 / 64 * iters * (kLd + kSt),
           us * 2400.0 / (1024.0 / 64 * iters * (kLd + kSt)));
    fflush(stdout);
}

int main() {
    const uint32_t S = 3328;  // ~ a config-5 lane range (122 literals x 27 B), multiple of 32
    const uint32_t ib = 262144u * S, ob = 262144u * (S * 4 / 3);
    uint8_t *in, *out;
    uint32_t* sink;
    CK(hipMalloc(&in, ib));
    CK(hipMalloc(&out, ob));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(in, 1, ib));
    run<2, 0, 0, 0>("lane_ld32", in, out, S, ib, ob, sink);
    run<2, 0, 0, 1>("coal_ld32", in, out, S, ib, ob, sink);
    run<2, 2, 0, 0>("lane_ld32_st32", in, out, S, ib, ob, sink);
    run<2, 2, 0, 1>("coal_ld32_st32", in, out, S, ib, ob, sink);
    run<1, 1, 0, 0>("lane_ld16_st16", in, out, S, ib, ob, sink);
    run<4, 4, 0, 0>("lane_ld64_st64", in, out, S, ib, ob, sink);
    run<2, 2, 64, 0>("lane_ld32_st32_alu64", in, out, S, ib, ob, sink);
    run<2, 2, 64, 1>("coal_ld32_st32_alu64", in, out, S, ib, ob, sink);
    run<2, 2, 256, 0>("lane_ld32_st32_alu256", in, out, S, ib, ob, sink);
    run<2, 2, 256, 1>("coal_ld32_st32_alu256", in, out, S, ib, ob, sink);
    return 0;
}
