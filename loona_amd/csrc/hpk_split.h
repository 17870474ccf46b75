// hpk_split.h — a workgroup's share of a batch, balanced by bytes rather than by literal count.
//
// A batch with skewed literal lengths (config 3: Zipf lengths to 4 KiB) split into equal literal
// counts gives the busiest of 512 workgroups ~14 % more bytes than the mean, and the kernel waits
// for it. split_by_bytes gives workgroup b the literals [BA, BB) whose weight w(i) = off[i] +
// kPerLit * i (bytes plus a per-literal charge for the metadata work) starts in
// [W * b / G, W * (b + 1) / G): a 256-ary search per boundary (half the workgroup each), 3 rounds
// for 1M literals, one barrier per round.
//
// With offsets that are not non-decreasing (a bad batch) the search still returns a deterministic
// index per boundary, boundary 0 is 0 and boundary G is n: the ranges cover [0, n) with no gap
// (a literal may be seen by two workgroups, which the kernels' bad-offset handling tolerates: both
// write the same verdict).
#pragma once
#include <stdint.h>

namespace hpksplit {

constexpr int kMaxRounds = 6;  // 256^5 > 2^32 literals

// s_cnt: 2 * kMaxRounds words of LDS. All kBlock threads must call it (it has barriers).
template <int kBlock, uint32_t kPerLit>
__device__ __forceinline__ void split_by_bytes(const uint32_t* __restrict__ off, uint32_t n, uint32_t* s_cnt,
                                               uint32_t& BA, uint32_t& BB) {
    static_assert(kBlock % 128 == 0, "two halves of whole waves");
    constexpr uint32_t kHalf = kBlock / 2;
    const uint32_t G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
    const uint32_t s = tid / kHalf, t = tid % kHalf;  // search s finds boundary b + s
    if (tid < 2 * kMaxRounds) s_cnt[tid] = 0;
    const uint32_t o0 = off[0], oN = off[n];
    __syncthreads();
    const uint64_t W = (uint64_t)(oN - o0) + (uint64_t)kPerLit * n;
    const uint32_t k = b + s;
    // the first literal whose weight reaches T; boundaries 0 and G are fixed
    const uint64_t T = (uint64_t)o0 + W * k / G;
    uint32_t lo = 0, hi = n;
    if (k == 0) hi = 0;
    if (k == G || oN < o0) lo = hi = (oN < o0) ? (uint32_t)((uint64_t)n * k / G) : n;  // bad totals: count split
    uint32_t rounds = 1;
    for (uint32_t x = n; x; x /= kHalf) ++rounds;  // block-uniform; enough for the interval to close
    for (uint32_t r = 0; r < rounds && r < (uint32_t)kMaxRounds; ++r) {
        const uint32_t m = hi - lo;
        const uint32_t q = lo + (uint32_t)((uint64_t)m * t / kHalf);
        const bool below = (uint64_t)off[q] + (uint64_t)kPerLit * q < T;
        const uint32_t pop = (uint32_t)__popcll(__ballot(below));
        if ((tid & 63u) == 0 && pop) atomicAdd(&s_cnt[2 * r + s], pop);
        __syncthreads();
        const uint32_t c = s_cnt[2 * r + s];
        if (c) {  // off[q_{c-1}] is below T, off[q_c] (or off[hi]) is not
            const uint32_t qa = lo + (uint32_t)((uint64_t)m * (c - 1u) / kHalf);
            const uint32_t qb = c < kHalf ? lo + (uint32_t)((uint64_t)m * c / kHalf) : hi;
            hi = qb;
            lo = min(qa + 1u, qb);  // (equal probes at c - 1 and c only with offsets out of order)
        } else {
            hi = lo;
        }
    }
    // boundary b from the first half, b + 1 from the second (both halves computed both values
    // identically within their half; exchange through LDS)
    __syncthreads();
    if (t == 0) s_cnt[s] = lo;
    __syncthreads();
    BA = s_cnt[0];
    BB = s_cnt[1];
    __syncthreads();
}

}  // namespace hpksplit
