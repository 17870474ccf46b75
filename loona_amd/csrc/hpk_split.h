// hpk_split.h — a workgroup's share of a batch, balanced by bytes rather than by literal count.
//
// A batch with skewed literal lengths (config 3: Zipf lengths to 4 KiB) split into equal literal
// counts gives the busiest of 512 workgroups ~14 % more bytes than the mean, and the kernel waits
// for it. split_by_bytes gives workgroup b the literals [BA, BB) whose weight w(i) = off[i] +
// kPerLit * i (bytes plus a per-literal charge for the metadata work) starts in
// [W * b / G, W * (b + 1) / G), W the batch's total weight: the first literal whose weight reaches
// each of the two targets, found by a 256-ary search per boundary (half the workgroup each). The
// first round probes a window of +-2 count-shares around the count split's boundary, so a batch
// whose imbalance is within that (config 3: 14 %) takes two rounds — two dependent global reads,
// two barriers; a boundary outside the window goes on with the full search. Every thread tracks both
// boundaries' intervals from the round counts in LDS, so all threads leave the loop together.
//
// With offsets that are not non-decreasing (a bad batch) the search still returns a deterministic
// index per boundary, boundary 0 is 0 and boundary G is n: the ranges cover [0, n) with no gap
// (a literal may be seen by two workgroups, which the kernels' bad-offset handling tolerates: both
// write the same verdict).
#pragma once
#include <stdint.h>

namespace hpksplit {

constexpr int kMaxRounds = 8;  // window round, then 256-ary rounds over up to 2^32 literals

// s_cnt: 2 * kMaxRounds words of LDS. All kBlock threads must call it (it has barriers).
template <int kBlock, uint32_t kPerLit>
__device__ __forceinline__ void split_by_bytes(const uint32_t* __restrict__ off, uint32_t n, uint32_t* s_cnt,
                                               uint32_t& BA, uint32_t& BB) {
    static_assert(kBlock % 128 == 0, "two halves of whole waves");
    constexpr uint32_t kHalf = kBlock / 2;
    const uint32_t G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
    const uint32_t s = tid / kHalf, t = tid % kHalf;  // this thread probes for boundary b + s
    if (tid < 2 * kMaxRounds) s_cnt[tid] = 0;
    const uint32_t o0 = off[0], oN = off[n];
    const bool bad = oN < o0;  // totals out of order: the count split
    const uint64_t W = (uint64_t)(oN - o0) + (uint64_t)kPerLit * n;
    const uint32_t share = n / G;
    const uint32_t h = 2u * share + kHalf;  // the first round's window half-width
    uint64_t T[2];
    uint32_t lo[2], hi[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t k = b + (uint32_t)j;
        T[j] = (uint64_t)o0 + W * k / G;
        const uint32_t i0 = (uint32_t)((uint64_t)n * k / G);
        if (bad || k == 0 || k == G) {
            lo[j] = hi[j] = i0;  // fixed
        } else {
            lo[j] = i0 > h ? i0 - h : 0u;
            hi[j] = n - i0 > h ? i0 + h : n;
        }
    }
    __syncthreads();
    for (uint32_t r = 0; r < (uint32_t)kMaxRounds; ++r) {
        if (lo[0] == hi[0] && lo[1] == hi[1]) break;  // (uniform: every thread has both intervals)
        // round 0 probes [lo, hi] inclusive (the answer may lie outside the window); later rounds
        // probe lo + m t / H with the answer known to be in (probe, hi]
        const uint32_t div = r == 0 ? kHalf - 1u : kHalf;
        const uint32_t ls = s ? lo[1] : lo[0], hs = s ? hi[1] : hi[0];
        const uint32_t q = ls + (uint32_t)((uint64_t)(hs - ls) * t / div);
        const bool below = ls != hs && (uint64_t)off[q] + (uint64_t)kPerLit * q < (s ? T[1] : T[0]);
        const uint32_t pop = (uint32_t)__popcll(__ballot(below));
        if ((tid & 63u) == 0 && pop) atomicAdd(&s_cnt[2 * r + s], pop);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            if (lo[j] == hi[j]) continue;
            const uint32_t c = s_cnt[2 * r + j], m = hi[j] - lo[j];
            if (r == 0 && c == 0) {  // the answer is at or before the window
                hi[j] = lo[j];
                lo[j] = 0;
            } else if (r == 0 && c == kHalf) {  // after it
                lo[j] = min(hi[j] + 1u, n);
                hi[j] = n;
            } else if (c == 0) {
                hi[j] = lo[j];
            } else {
                const uint32_t qa = lo[j] + (uint32_t)((uint64_t)m * (c - 1u) / div);
                const uint32_t qb = c < kHalf ? lo[j] + (uint32_t)((uint64_t)m * c / div) : hi[j];
                hi[j] = qb;
                lo[j] = min(qa + 1u, qb);  // (equal probes at c - 1 and c only with offsets out of order)
            }
        }
    }
    BA = lo[0];
    BB = lo[1];
}

}  // namespace hpksplit
