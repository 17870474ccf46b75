// hpk_decode11.h — decode kernel v11: one large LDS window per fill, output written straight to
// HBM as whole dwords, longest-first queue, two-symbol table step.
//
// Why: with the output image in LDS (v8) a fill could hold ~1,500 literals for 1,024 lanes; every
// fill ends in a tail where most lanes of a wave idle while the wave still issues full
// instructions, and halving the fill size cost +40 % time (bench/kvariants "v8_half_fill").
// Without the image the window is 2.7x larger, so a config-2 workgroup range (~106 KB) is ONE
// fill: one tail per workgroup instead of ~3. The price is the write pattern: every lane stores
// its own literal's dwords, which the L2 does not fully merge (PMC on v5: ~4x the output bytes
// reach HBM), which is affordable while the kernel is far from the HBM roof.
#pragma once
#include "legacy_decode.h"

namespace hpkdec {

template <int kWaves, int kW, int kQ>
struct Geo11 {
    static constexpr int kBlock = kWaves * 64;
    static constexpr int kMetaRounds = (kQ + kBlock - 1) / kBlock;
    static constexpr int kStageRounds = (kW / 16 + kBlock - 1) / kBlock;
    static constexpr int kLutBytes = (int)(HPK_LUT_SIZE * 4);
    static constexpr int kLutOff = kTabBytes;
    static constexpr int kInOff = kTabBytes + kLutBytes;
    static constexpr int kQOff = kInOff + kW;
    static constexpr int kHistOff = kQOff + 8 * kQ;  // 64 bucket counts + 64 bucket bases
    static constexpr int kCtrOff = kHistOff + 512;
    static constexpr int kLdsBytes = kCtrOff + 16;
    static_assert(kLdsBytes <= 163840, "LDS budget (160 KiB per CU on gfx950)");
    static_assert(kW % 16 == 0 && kW < (1 << 17), "window offsets pack in 17 bits");
    static_assert(kQ <= 4096, "fill index packs in 12 bits");
};
constexpr uint32_t kQ11Byte = 0x80000000u;  // queue entry .y flag: byte path
constexpr uint32_t kOutSpan11 = 4u * 65535u;  // output span of a fill: dword index in 16 bits

// lit_step8 with the output gathered in a register and stored to global memory a dword at a
// time (lit_emit_g); L.od is the global dword index, the region dword-aligned and >= the bound.
template <int kStore, class Src>
__device__ __forceinline__ void lit_step11(Lit& L, const Src& src, const uint32_t* __restrict__ lut,
                                           const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8) {
    lit_refill(L, src);
    const uint32_t hi = (uint32_t)(L.win >> 32);
    const uint32_t e = lut[hi >> (32 - HPK_LUT_BITS)];
    const uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u;
    const bool ok1 = L.live & ((e >> 26) != 0u) & (len0 <= L.rem);
    const bool ok2 = ok1 & ((e >> 27) != 0u) & (tot <= L.rem);
    const uint32_t use = ok2 ? tot : ok1 ? len0 : 0u;
    const uint32_t g = (uint32_t)ok1 + (uint32_t)ok2;
    L.win <<= use;
    L.nb -= use;
    L.rem -= use;
    lit_emit_g<kStore>(L, e & 0xFFFFu, g, out8);
    const bool park = L.live & ((e >> 26) == 0u);  // a 13..30-bit code, or EOS
    L.live = park | (ok1 & (L.rem != 0u));
    if (park) {
        lit_refill(L, src);
        const uint32_t w = (uint32_t)(L.win >> 32);
        uint32_t s1, len;
        bool eos;
        lo_decode(w, lo, s1, len, eos);
        if (len > L.rem) {
            L.live = false;  // only padding left
        } else if (eos) {
            L.st = HPK_EOS_IN_STRING;  // huffman.rs:112-116
            L.live = false;
        } else {
            L.win <<= len;
            L.nb -= len;
            L.rem -= len;
            lit_emit_g<kStore>(L, s1, 1u, out8);
            L.live = L.rem != 0u;
        }
    }
}

// kMode: 0 product, 1 stage only, 2 no output stores, 4 checked stores (g_chk).
template <int kMode, int kWaves, int kW, int kQ, int kRefillN, int kChunk, bool kLpt = true>
__global__ __launch_bounds__(kWaves * 64) void hpk_decode11(DecodeArgs a) {
    using G = Geo11<kWaves, kW, kQ>;
    constexpr int R = G::kMetaRounds, S = G::kStageRounds;
    __shared__ __attribute__((aligned(16))) uint8_t smem[G::kLdsBytes];
    uint8_t* s_t8 = smem;
    uint16_t* s_lo = reinterpret_cast<uint16_t*>(smem + kT8Bytes);
    uint32_t* s_lut = reinterpret_cast<uint32_t*>(smem + G::kLutOff);
    uint8_t* s_in = smem + G::kInOff;
    uint2* s_q = reinterpret_cast<uint2*>(smem + G::kQOff);
    uint32_t* s_hist = reinterpret_cast<uint32_t*>(smem + G::kHistOff);
    uint32_t* s_bbase = s_hist + 64;
    // [0] fitting count, [1] queue head, [2] input end of the fill, [3] output end of the fill
    uint32_t* s_ctr = reinterpret_cast<uint32_t*>(smem + G::kCtrOff);
    for (uint32_t t = threadIdx.x; t < kT8Bytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_t8)[t] = reinterpret_cast<const uint4*>(a.t8)[t];
    for (uint32_t t = threadIdx.x; t < kLoBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];
    for (uint32_t t = threadIdx.x; t < (uint32_t)G::kLutBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lut)[t] = reinterpret_cast<const uint4*>(a.lut)[t];

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const LdsSrc lds{reinterpret_cast<const uint32_t*>(s_in)};
    const uint32_t BA = (uint32_t)((uint64_t)a.n * blockIdx.x / gridDim.x);
    const uint32_t BB = (uint32_t)((uint64_t)a.n * (blockIdx.x + 1) / gridDim.x);
    const uint32_t in_end = a.in_off[a.n] + a.in_mis;
    const uint32_t last16 = in_end ? (in_end - 1) >> 4 : 0;
    const uint32_t r_end = a.in_off[BB] + a.in_mis;
    const uint32_t rlast16 = r_end ? (r_end - 1) >> 4 : 0;

    uint32_t cur = BA;
    uint32_t gin = 0, gout = 0;
    if (cur < BB) {
        gin = a.in_off[cur] + a.in_mis;
        gout = a.out_off[cur] + a.out_mis;
    }
    while (cur < BB) {  // block-uniform
        const uint32_t cntl = min((uint32_t)kQ, BB - cur);
        const uint32_t base16 = gin & ~15u;
        const uint32_t ob16 = gout & ~15u;
        // a config-2 workgroup range is one fill, so the fill's loads are simply issued here (all
        // before the first wait); registers are not held across the decode
        Prefetch<R, S> P;
        prefetch_fill<G::kBlock>(P, a, tid, cur, min(cur + (uint32_t)kQ, BB), base16, rlast16);
        lds_barrier();  // previous fill decoded: queue and window free
        if (tid < 64) s_hist[tid] = 0;
        if (tid == 0) {
            s_ctr[0] = 0;
            s_ctr[1] = G::kBlock;
            s_ctr[2] = gin;
            s_ctr[3] = gout;
        }
        lds_barrier();
        uint32_t ex[R], ey[R], pos[R];
        uint32_t kw = 0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = tid + (uint32_t)G::kBlock * r;
            const uint32_t p0 = P.io0[r] + a.in_mis, p1 = P.io1[r] + a.in_mis;
            const uint32_t o0 = P.oo0[r] + a.out_mis, o1 = P.oo1[r] + a.out_mis;
            // fitting literals form a prefix (offsets are non-decreasing)
            const bool fits = t < cntl && p1 - base16 <= (uint32_t)kW && o1 - ob16 <= kOutSpan11;
            pos[r] = 0xFFFFFFFFu;
            if (fits) {
                const uint32_t nbytes = p1 - p0, ocap = o1 - o0;
                // dword path: an aligned region holding hpk_decoded_bound(nbytes) bytes
                const bool dw = ((o0 | ocap) & 3u) == 0 && ocap >= (nbytes * 8u) / 5u && nbytes < 32768u;
                ex[r] = (p0 - base16) | ((dw ? nbytes : 0u) << 17);
                ey[r] = t | (((o0 - ob16) >> 2) << 12) | (dw ? 0u : kQ11Byte);
                if (kLpt) {
                    const uint32_t bk = lpt_bucket(nbytes);
                    pos[r] = (bk << 16) | atomicAdd(&s_hist[bk], 1u);
                } else {
                    pos[r] = t;  // literal order: neighbouring lanes store to neighbouring lines
                }
            }
            const uint64_t fb = __ballot(fits);
            kw += (uint32_t)__popcll(fb);
            if (fb) {  // the wave's last fitting literal ends furthest
                const int hl = 63 - __builtin_clzll(fb);
                const uint32_t e_in = (uint32_t)__builtin_amdgcn_readlane((int)p1, hl);
                const uint32_t e_out = (uint32_t)__builtin_amdgcn_readlane((int)o1, hl);
                if (lane == 0) {
                    atomicMax(&s_ctr[2], e_in);
                    atomicMax(&s_ctr[3], e_out);
                }
            }
        }
        if (lane == 0 && kw) atomicAdd(&s_ctr[0], kw);
        lds_barrier();
        const uint32_t k = s_ctr[0];
        if (k == 0) {  // literal `cur` alone exceeds the window: one lane decodes it from global
            if (tid == 0) {
                const GlobalSrc g{reinterpret_cast<const uint32_t*>(a.in_base), last16 * 4 + 3};
                uint8_t* dst = a.out_base + gout;
                Lit L = {};
                lit_bytes_to(L, g, s_lo, [&](uint32_t j, uint8_t v) { dst[j] = v; },
                             a.out_off[cur + 1] - a.out_off[cur], gin, a.in_off[cur + 1] + a.in_mis - gin);
                a.out_len[cur] = L.cnt;
                a.status[cur] = (uint8_t)lit_status(L);
            }
            cur += 1;
            if (cur < BB) {
                gin = a.in_off[cur] + a.in_mis;
                gout = a.out_off[cur] + a.out_mis;
            }
            continue;
        }
        const uint32_t gin_next = s_ctr[2], gout_next = s_ctr[3];
        if (tid < 64) {  // bucket bases: exclusive scan by wave 0
            const uint32_t v = s_hist[tid];
            uint32_t x = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (lane >= (uint32_t)d) x += y;
            }
            s_bbase[tid] = x - v;
        }
        {
            uint4* l16 = reinterpret_cast<uint4*>(s_in);
#pragma unroll
            for (int r = 0; r < S; ++r)
                if (tid + G::kBlock * r < kW / 16) l16[tid + G::kBlock * r] = P.chunk[r];
        }
        lds_barrier();
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (pos[r] != 0xFFFFFFFFu)
                s_q[kLpt ? s_bbase[pos[r] >> 16] + (pos[r] & 0xFFFFu) : pos[r]] = make_uint2(ex[r], ey[r]);
        const uint32_t cur_next = cur + k;
        lds_barrier();
        if (kMode == 1) {  // diagnostic: no decode; lengths from the staged bytes keep them live
            for (uint32_t t = tid; t < k; t += G::kBlock) {
                const uint2 e = s_q[t];
                a.out_len[cur + (e.y & 0xFFFu)] = (e.x >> 17) + s_in[e.x & 0x1FFFFu];
            }
        } else {
            constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : kDword);
            const uint32_t od_base = ob16 >> 2;
            Lit L = {};  // every field defined: idle lanes still run the (predicated) step
            L.nb = 64;
            uint32_t t = tid;
            uint32_t qb = 0, qe = 0;
            bool act = false;
            uint32_t idx = 0;
            auto begin = [&](uint32_t tt) {
                const uint2 e = s_q[min(tt, k - 1)];
                act = tt < k && !(e.y & kQ11Byte);
                idx = e.y & 0xFFFu;
                lit_begin(L, lds, e.x & 0x1FFFFu, e.x >> 17);
                L.od = od_base + ((e.y >> 12) & 0xFFFFu);
                L.oend = L.od + ((e.x >> 17) * 8u / 5u + 3u) / 4u;
                L.live = L.live && act;
            };
            begin(t);
            for (;;) {
#pragma unroll
                for (int s = 0; s < kRefillN; ++s) lit_step11<kStore>(L, lds, s_lut, s_lo, a.out_base);
                const bool fin = t < k && !L.live;
                if (__any(fin)) {
                    if (fin && act) {
                        if (kStore == kDword && L.accn) reinterpret_cast<uint32_t*>(a.out_base)[L.od] = (uint32_t)L.acc;
                        if (kStore == kChecked && L.accn) {
                            if (L.od < L.oend)
                                reinterpret_cast<uint32_t*>(a.out_base)[L.od] = (uint32_t)L.acc;
                            else
                                chk_report(2, L.od, L.oend, L.cnt);
                        }
                        a.out_len[cur + idx] = L.cnt;
                        a.status[cur + idx] = (uint8_t)lit_status(L);
                    }
                    const bool free_lane = fin || t >= k;
                    const uint64_t fm = __ballot(free_lane);
                    const uint32_t rank =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                    const uint32_t need = (uint32_t)__popcll(fm), have = qe - qb;
                    uint32_t base = qb + rank;
                    if (have < need) {  // wave-uniform
                        uint32_t nb = 0;
                        if (rank == 0 && free_lane) nb = atomicAdd(&s_ctr[1], (uint32_t)kChunk);
                        nb = (uint32_t)__builtin_amdgcn_readlane((int)nb, (int)__builtin_ctzll(fm));
                        if (rank >= have) base = nb + (rank - have);
                        qb = nb + (need - have);
                        qe = nb + kChunk;
                    } else {
                        qb += need;
                    }
                    qb = (uint32_t)__builtin_amdgcn_readfirstlane((int)qb);
                    qe = (uint32_t)__builtin_amdgcn_readfirstlane((int)qe);
                    if (free_lane) {
                        t = base;
                        begin(base);
                    }
                }
                if (!__any(t < k)) break;
            }
            // literals whose output region is unaligned / below the decoded bound (or > 32 KiB
            // encoded): byte stores with a capacity check per byte
            for (uint32_t tt = tid; tt < k; tt += G::kBlock) {
                const uint2 e = s_q[tt];
                if (e.y & kQ11Byte) {
                    const uint32_t i = cur + (e.y & 0xFFFu);
                    const uint32_t sb = a.in_off[i] + a.in_mis - base16;
                    uint8_t* dst = a.out_base + a.out_off[i] + a.out_mis;
                    Lit B = {};
                    lit_bytes_to(B, lds, s_lo, [&](uint32_t j, uint8_t v) { dst[j] = v; }, a.out_off[i + 1] - a.out_off[i],
                                 sb, a.in_off[i + 1] - a.in_off[i]);
                    a.out_len[i] = B.cnt;
                    a.status[i] = (uint8_t)lit_status(B);
                }
            }
        }
        cur = cur_next;
        gin = gin_next;
        gout = gout_next;
    }
}

}  // namespace hpkdec
