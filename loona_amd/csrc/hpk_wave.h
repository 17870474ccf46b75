// hpk_wave.h — decode v25: wave fills. Every wave of the workgroup decodes its own contiguous
// literal range in fills of at most 128 literals (two per lane) with no workgroup barrier between
// the fills, so one wave's memory traffic and setup overlap the other fifteen waves' decoding.
//
// Why (profiles/r03/decomposition_v24_modes.jsonl): the v24 fill kernel spends 631 of its 1,178 us
// per 32M-literal launch in the fill machinery alone (decode switched off), because all 16 waves of
// a workgroup set up, wait at the fill-top barrier for the fill's slowest literal and write back
// together, so the CU's memory path and its LDS/VALU take turns instead of overlapping. A lane
// stream per lane (each lane its own literal range) was ruled out by profiles/r03/
// ta_probe_lane_vs_coalesced.jsonl: 16-byte stores to 64 addresses per instruction run at 45 % of
// the coalesced rate. Here every transfer is still a coalesced wave-wide piece (window loads,
// image write-back, offsets), and every wave runs its own pipeline:
//   * per wave an input window (kWinB bytes, big-endian dwords) and an output image (kImgB bytes,
//     the last 256 the lanes' dummy slots) in LDS; the 16 waves' areas plus the shared tables fill
//     the CU's 160 KiB;
//   * a fill is the longest prefix of the next 128 literals whose input fits the window and whose
//     output regions fit the image; its offsets and window were loaded into registers while the
//     previous fill decoded;
//   * per fill: the offsets are checked (decoder.rs:138-142: a literal's bounds before any Huffman
//     work), the previous fill's image and lengths are written back, the fill's literals are sorted
//     longest-first by a per-wave counting sort (LDS atomics on 32 length classes, in the image),
//     the window is staged and the next fill's loads are issued; then lane i decodes queue slots i
//     and 127 - i (the static snake of v13: the longest with the shortest, both read before the
//     first step) with the two-lookup step of v12 (lit12_step), unconditional byte stores of v14 and
//     the late length/status of v22;
//   * literals of >= long_min encoded bytes whose region holds the decoded bound are listed for the
//     long-literal phase (hpk_long.h) after all waves are done, as v19 did; a workgroup range made
//     mostly of them (config 3) is listed whole without any wave fill;
//   * a literal whose region is below the decoded bound is decoded code by code with a capacity
//     check per byte by the lane that holds it, after the lane loop (HPK_OUTPUT_OVERFLOW);
//   * bad offsets stop the wave (HPK_BAD_OFFSETS for the rest of its range) and, through an LDS flag
//     read at every fill, the workgroup's other waves at their next fill.
// Semantics are huffman.rs:95-161 through lit12_step (hpk_decode12.h).
#pragma once
#include <type_traits>

#include "hpk_decode12.h"


#ifndef HPK_BODY
#define HPK_BODY 1  // v27: unchecked body steps + checked tails (0: v26's checked steps throughout)
#endif
#ifndef HPK_BODY_UNROLL
#define HPK_BODY_UNROLL 4  // body steps between the checks for a lane whose literal's body ended (2: config 5 +2.5 %)
#endif
#ifndef HPK_LUT3
#define HPK_LUT3 1  // v28: the wave kernel's lookups in the LUT3 layout (byte-wide "bits held")
#endif
#ifndef HPK_CW_LANE_DIAG
#define HPK_CW_LANE_DIAG 0  // (measurement only) 2: no copy loop, 3: 16-byte pieces at 16-aligned
                            // addresses, 4: no 16-byte stores
#endif
#ifndef HPK_NT_STORE
#define HPK_NT_STORE 1  // 1: the image write-back as nontemporal 16-byte stores (the output is never re-read)
#endif
#ifndef HPK_NT_LOAD
#define HPK_NT_LOAD 1  // 1: the window prefetch as nontemporal 16-byte loads (each input byte is read once)
#endif
#ifndef HPK_WIN_CUT
#define HPK_WIN_CUT 1  // 1: the window loads stop at the literal chunk's last input byte (round 6: config-5
                       // reads 1.229 -> 1.178 GB per launch, time unchanged)
#endif

namespace hpkdec {

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16(uint4* p, const uint4 v) {
    if (HPK_NT_STORE) {
        const v4u32 x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<v4u32*>(p));
    } else {
        *p = v;
    }
}
__device__ __forceinline__ uint4 ld16(const uint4* p) {
    if (HPK_NT_LOAD) {
        const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p));
        return make_uint4(x.x, x.y, x.z, x.w);
    }
    return *p;
}

template <int kWinB, int kImgB>
struct GeoW {
    static constexpr int kWaves = 16, kBlock = kWaves * 64;
    static constexpr int kWaveBytes = kWinB + kImgB;
    static constexpr int kLutOff = kTabBytes;                    // T8 + LO (kTabBytes), then LUT2
    static constexpr int kWaveOff = kTabBytes + (int)HPK_LUT_SIZE * 4;
    static constexpr int kCtrOff = kWaveOff + kWaves * kWaveBytes;
    static constexpr int kLdsBytes = kCtrOff + 64 + (int)kHugeMax * 4;  // counters, then the huge list
    static constexpr int kImg = kImgB - 256;                     // usable image bytes (dummy slots after)
    static constexpr int kWinRounds = (kWinB / 16 + 63) / 64;    // window chunks per lane
    static constexpr int kFlushRounds = (kImg / 16 + 1 + 63) / 64;
    static_assert(kLdsBytes <= 163840, "LDS budget (160 KiB per CU on gfx950)");
    static_assert(kWinB % 16 == 0 && kImgB % 16 == 0 && kWinB < 65536 && kImgB < 131072, "entry packing");
    // the long-literal phase's rings and queues (hpk_long.h) over the wave areas after the fills
    static_assert(kWaves * kWaveBytes >= huge_lds_bytes<kBlock>(), "huge-phase LDS");
};

// WG counters (s_ctr): [0] bad offsets seen (waves stop at their next fill), [1] long list, front
// (>= long_big bytes), [2] long list, back, [3] long-phase claim, [4]/[5] dense check sums, [6] the
// dense listing found an entry it cannot list, [7] chunks of kChunk literals handed out to the waves,
// [8] huge literals listed (s_huge = s_ctr + 16, at most kHugeMax of them; hpk_huge.h), [9] (kCompact) bytes
// of the workgroup's bound span handed out
// kRank: 0 = counting sort with LDS atomics on 32 length classes of 2 bytes, 1 / 2 = ranks from
// ballots over 16 classes of 4 bytes / 32 classes of 2 bytes (no LDS round trip)
// Inclusive sum over the wave's 64 lanes: DPP row shifts within rows of 16 lanes (zero fill), then the
// rows' totals by readlane.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, uint32_t lane) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
    const uint32_t r1 = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
    const uint32_t r2 = (uint32_t)__builtin_amdgcn_readlane((int)x, 47);
    return x + (lane >= 16u ? r0 : 0u) + (lane >= 32u ? r1 : 0u) + (lane >= 48u ? r2 : 0u);
}

// kCompact (hpk_decode_batch_compact, round 5): a.out_off is the library's bound layout (4-rounded
// decoded bounds); each workgroup packs its output into its own range's bound span [out_off[BA],
// out_off[BB]) from an LDS cursor (s_ctr[9]): every decoded fill takes its decoded total there and is
// gathered into it (compact_fill), every listed literal takes its 4-rounded bound there when it is
// listed (co_off). No device-wide cursor: one atomic per fill on one word would be ~290k per 32M-literal
// launch, against the ~88 per us one word takes (MI355X_MICROARCH.md, dequeue).
template <int kMode, int kWinB, int kImgB, uint32_t kChunk, int kGuided, int kRank, bool kCompact = false>
__global__ __launch_bounds__(1024) void hpk_decode_wave(DecodeArgs a) {
    using G = GeoW<kWinB, kImgB>;
    constexpr int kStore = kMode == 2 ? kNoStore : kPred;
    // kMode 3 (diagnostic builds): per-wave cycle stamps into a.dbg[wave * 16 + i]: 0 total, 1 waiting
    // for the fill's offsets + their checks, 2 write-back, 3 queue, 4 window staging, 5 prefetch issue
    // and queue reads, 6 lane loop, 7 byte path + results, 8 fills, 9 lane-loop rounds, 10 long phase,
    // 11 before the first fill
    // (the sums live in LDS, added by lane 0 with return-less ds_add: held in registers they pushed
    // the kernel over 128 VGPRs, and the spills' waits distorted what they measured)
    __shared__ uint32_t s_dg[kMode == 3 ? G::kWaves * 12 : 1];
    uint32_t tq = kMode == 3 ? (uint32_t)__builtin_amdgcn_s_memtime() : 0u;
    const uint32_t t_start = tq;
    auto dg_add = [&](int i, uint32_t v) {
        if (kMode == 3 && (threadIdx.x & 63u) == 0u) atomicAdd(&s_dg[(threadIdx.x >> 6) * 12u + i], v);
    };
    auto stamp = [&](int i) {
        if (kMode == 3) {
            const uint32_t t = (uint32_t)__builtin_amdgcn_s_memtime();
            dg_add(i, t - tq);
            tq = t;
        }
    };
    constexpr int R = G::kWinRounds, F = G::kFlushRounds;
    __shared__ __attribute__((aligned(16))) uint8_t smem[G::kLdsBytes];
    uint16_t* s_lo = reinterpret_cast<uint16_t*>(smem + kT8Bytes);
    uint32_t* s_lut = reinterpret_cast<uint32_t*>(smem + G::kLutOff);
    uint32_t* s_ctr = reinterpret_cast<uint32_t*>(smem + G::kCtrOff);
    uint32_t* s_huge = s_ctr + 16;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    constexpr int kTab = HPK_LUT3 && HPK_BODY ? 3 : 2;  // the table layout of the fills and the phases after them
    const uint32_t BA = (uint32_t)((uint64_t)a.n * blockIdx.x / gridDim.x);
    const uint32_t BB = (uint32_t)((uint64_t)a.n * (blockIdx.x + 1) / gridDim.x);
    // (round 6) The start's memory round trips overlapped: every wave's first chunk is fixed here (wave wv's
    // c0 literals from BA + wv c0; the static split: its 1/16), and its first literal's offsets, the dense
    // check's offsets and the tables are loaded together (they had been four dependent round trips: tables,
    // the dense check, the first claim's offsets, then the first fill's). Config 2: see DESIGN.md §4.0.
    static_assert(G::kBlock == 1024, "the dense check's two offsets rounds");
    const uint32_t c0 = kGuided == 2 ? kChunk : max(kChunk, (BB - BA) / 32u);
    const uint32_t cur0 = kGuided == 0 ? BA + (uint32_t)((uint64_t)(BB - BA) * wv / G::kWaves) : min(BA + wv * c0, BB);
    const uint32_t ce0 =
        kGuided == 0 ? BA + (uint32_t)((uint64_t)(BB - BA) * (wv + 1) / G::kWaves) : min(cur0 + c0, BB);
    const uint32_t gin0 = a.in_off[cur0];
    const uint32_t gend0 = HPK_WIN_CUT ? a.in_off[ce0] : 0u;
    const uint32_t gout0 = kCompact ? 0u : a.out_off[cur0];
    const uint32_t kd = min(BB - BA, 2048u);  // the dense check's literals: the range's first 2048
    uint32_t dv0[2], dv1[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const uint32_t tt = BA + min(tid + (uint32_t)G::kBlock * r, kd ? kd - 1u : 0u);
        dv0[r] = a.in_off[tt];
        dv1[r] = a.in_off[tt + 1u];
    }
    for (uint32_t t = tid; t < kLoBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];
    for (uint32_t t = tid; t < HPK_LUT_SIZE * 4 / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lut)[t] = reinterpret_cast<const uint4*>(kTab == 3 ? a.lut3 : a.lut2)[t];
    if (tid < 16) s_ctr[tid] = tid == 7 && kGuided ? min(G::kWaves * c0, BB - BA) : 0u;  // [7]: the first chunks
    if (kMode == 3)
        for (uint32_t t = tid; t < (uint32_t)G::kWaves * 12u; t += G::kBlock) s_dg[t] = 0;
    const uint32_t in_end = min(a.in_off[a.n], a.in_cap) + a.in_mis;
    const uint32_t last16 = in_end ? (in_end - 1) >> 4 : 0;  // last 16-B chunk holding a batch byte
    // (kCompact, v34) the bound layout is U(i) = floor(8 (in_off[i] - in_off[0]) / 5) + 4 i, made here
    // from the input offsets (no scan, no out_off array): a literal's region U(i + 1) - U(i) holds its
    // decoded bound, a range's span U(BB) - U(BA) every 4-rounded bound of its literals, and U(n) is
    // hpk_decoded_bound(in_off[n] - in_off[0]) + 4 n (floor(8 d / 5) = d + 3 q + floor(3 r / 5), d = 5 q + r)
    const uint32_t in0 = kCompact ? a.in_off[0] : 0u;
    auto ulay = [&](uint32_t i, uint32_t io) -> uint32_t {
        const uint32_t d = io - in0, q = __umulhi(d, 0xCCCCCCCDu) >> 2;
        return d + 3u * q + (((d - 5u * q) * 39u) >> 6) + 4u * i;
    };
    auto oof = [&](uint32_t i) -> uint32_t { return kCompact ? ulay(i, a.in_off[i]) : a.out_off[i]; };
    if (kCompact && blockIdx.x == 0 && tid == 0) a.co_off[a.n] = ulay(a.n, a.in_off[a.n]);  // the span's end
    const uint32_t wg0 = kCompact && BA < BB ? oof(BA) : 0u;  // (kCompact) the range's bound span
    auto leave = [&](uint32_t i, uint32_t nb) {  // list literal i for the huge / long-literal phase
        if (kCompact) a.co_off[i] = wg0 + atomicAdd(&s_ctr[9], ((nb * 8u) / 5u + 3u) & ~3u);
        if (nb >= HPK_HUGE_MIN && nb < kHugeLimit) {
            const uint32_t h = atomicAdd(&s_ctr[8], 1u);
            if (h < kHugeMax) {
                s_huge[h] = i;
                return;
            }
        }
        if (nb >= a.long_big)
            a.long_list[BA + atomicAdd(&s_ctr[1], 1u)] = i;
        else
            a.long_list[BB - 1u - atomicAdd(&s_ctr[2], 1u)] = i;
    };
    __syncthreads();
    // ---- a range whose first literals hold mostly long-literal bytes (config 3) is listed whole ----
    bool dense = false;
    {
        uint32_t dlb = 0, dtb = 0;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            if (tid + (uint32_t)G::kBlock * r < kd) {
                const uint32_t nb = min(dv1[r] - dv0[r], 1u << 20);  // (bad offsets: bounded)
                dtb += nb;
                dlb += nb >= a.long_min ? nb : 0u;
            }
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            dlb += __shfl_xor(dlb, d);
            dtb += __shfl_xor(dtb, d);
        }
        if (lane == 0 && dtb) {
            atomicAdd(&s_ctr[4], dlb);
            atomicAdd(&s_ctr[5], dtb);
        }
        __syncthreads();
        if (s_ctr[4] > s_ctr[5] / 2u) {  // block-uniform
            // round 6: the list in LPT order (lpt_class_of, longest first) by a counting sort over the wave
            // areas (free before the fills): the long phase takes it front to back, so the longest jobs start
            // first; huge literals to the huge list; validated before anything is allocated
            uint32_t* const s_cls = reinterpret_cast<uint32_t*>(smem + G::kWaveOff);  // counts, then cursors
            if (tid < 64) s_cls[tid] = 0;
            __syncthreads();
            bool no = false;
            for (uint32_t i = BA + tid; i < BB; i += G::kBlock) {
                const uint32_t p0 = a.in_off[i], p1 = a.in_off[i + 1];
                const uint32_t q0 = kCompact ? ulay(i, p0) : a.out_off[i], q1 = kCompact ? ulay(i + 1u, p1) : a.out_off[i + 1];
                const bool ok = p0 <= p1 && p1 <= a.in_cap && q0 <= q1 && q1 <= a.out_cap &&
                                (uint64_t)(q1 - q0) >= (uint64_t)(p1 - p0) * 8u / 5u;
                if (!ok) {
                    no = true;
                    continue;
                }
                const uint32_t nb = p1 - p0;
                if (!(nb >= HPK_HUGE_MIN && nb < kHugeLimit)) atomicAdd(&s_cls[lpt_class_of(nb)], 1u);
            }
            if (__any(no) && lane == 0) s_ctr[6] = 1u;
            __syncthreads();
            dense = s_ctr[6] == 0u;
            if (dense) {
                if (tid < 64) {  // class bases
                    const uint32_t v = tid < 32 ? s_cls[tid] : 0u;
                    uint32_t x = v;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t y = __shfl_up(x, d);
                        if (lane >= (uint32_t)d) x += y;
                    }
                    if (tid < 32) s_cls[32 + tid] = x - v;
                    if (tid == 31) s_ctr[1] = x;  // the front's count
                }
                __syncthreads();
                for (uint32_t i = BA + tid; i < BB; i += G::kBlock) {
                    const uint32_t nb = a.in_off[i + 1] - a.in_off[i];
                    if (kCompact) a.co_off[i] = wg0 + atomicAdd(&s_ctr[9], ((nb * 8u) / 5u + 3u) & ~3u);
                    bool huge = false;
                    if (nb >= HPK_HUGE_MIN && nb < kHugeLimit) {
                        const uint32_t hh = atomicAdd(&s_ctr[8], 1u);
                        if (hh < kHugeMax) {
                            s_huge[hh] = i;
                            huge = true;
                        }
                    }
                    // (huge literals past the huge list's room go to the list's back, LPT class 0 taken last)
                    if (!huge)
                        a.long_list[nb >= HPK_HUGE_MIN && nb < kHugeLimit ? BB - 1u - atomicAdd(&s_ctr[2], 1u)
                                                                          : BA + atomicAdd(&s_cls[32 + lpt_class_of(nb)], 1u)] = i;
                }
                __syncthreads();
            }
            if (!dense) {  // not all listable: the range goes through the wave fills after all
                __syncthreads();
                if (tid == 0) {
                    s_ctr[1] = 0;
                    s_ctr[2] = 0;
                    s_ctr[8] = 0;
                    s_ctr[9] = 0;  // (kCompact: the listing's allocations are void)
                }
                __syncthreads();
            }
        }
    }
    if (!dense) {
        // ---- wave fills ----
        uint8_t* const s_win = smem + G::kWaveOff + wv * G::kWaveBytes;
        uint8_t* const s_img = s_win + kWinB;
        const uint32_t* const win32 = reinterpret_cast<const uint32_t*>(s_win);
        // The lane walk addresses the window and the image from the LDS array's base (its bit and
        // output positions carry the wave's offsets), so a step's window read and byte stores take
        // their base as the instruction's offset instead of a VGPR add each (v26; config 5 924-933 us
        // with the one-chunk claims below, against 988-1001 us for v25: profiles/r03/s2/
        // ab_wave_late_abs_r2.jsonl; with lit12_step's + 1 store offsets a step's block went from 82
        // to 73 VALU in the ISA, and the kernel's 8 B/lane of scratch is gone)
        const uint32_t wbits = (uint32_t)(G::kWaveOff + wv * G::kWaveBytes) * 8u;
        const uint32_t obase = (uint32_t)(G::kWaveOff + wv * G::kWaveBytes + kWinB);
        const uint32_t* const wl32 = reinterpret_cast<const uint32_t*>(smem);
        uint8_t* const ol8 = smem;
        const uint32_t dmy = obase + (uint32_t)G::kImg + lane * 4u;
        // The workgroup's range is handed out in chunks, in order, to whichever wave asks next (an LDS
        // cursor): a static split left the waves the SIMDs' arbitration favours idle at the end while
        // the others finished (11 % of a wave's time). Chunks shrink as the range drains (guided
        // self-scheduling: 1/32 of what is left, at least kChunk literals), so early chunks hold many
        // fills (a chunk's last fill is usually partial) and the last ones even the waves out.
        // (!kGuided: the wave's static 1/16 of the range, then nothing)
        bool given = false;
        auto claim = [&](uint32_t& ca, uint32_t& ce) {
            if (!kGuided) {
                ca = given ? BB : BA + (uint32_t)((uint64_t)(BB - BA) * wv / G::kWaves);
                ce = given ? BB : BA + (uint32_t)((uint64_t)(BB - BA) * (wv + 1) / G::kWaves);
                given = true;
                return;
            }
            uint32_t c = 0;
            if (lane == 0) {
                const uint32_t seen = *(volatile HPK_LDS_AS uint32_t*)(&s_ctr[7]);
                const uint32_t left = BB - BA > seen ? BB - BA - seen : 0u;
                // (2: fixed chunks. Round 6: fixed chunks until 16 were left, then 1/16 of what was left, at
                // least 32 / 48 / 64 literals: config 2 47.1-47.8 / 45.2-45.5 / 44.1-44.6 vs 40.5-41.4 us)
                const uint32_t want = kGuided == 2 ? kChunk : max(kChunk, left / 32u);
                c = atomicAdd(&s_ctr[7], want);
                c = c < BB - BA ? c : BB - BA;
                ce = BA + min(c + want, BB - BA);  // (lane 0's; broadcast below)
            }
            ca = BA + (uint32_t)__builtin_amdgcn_readfirstlane((int)c);
            ce = (uint32_t)__builtin_amdgcn_readfirstlane((int)ce);
        };
        // registers of the next fill: the start offsets of slots lane and lane + 64 (a slot's end is the
        // next slot's start, taken from the neighbouring lane by DPP at the fill's top: round 5, half the
        // offset loads and four VGPRs fewer), the offsets of slot 128 (wave-uniform: scalar loads), the
        // window chunks
        uint32_t io0[2], oo0[2], ie = 0, oe = 0, pcnt = 1, pc = 0;
        uint4 ch[R];
        // clim: the last 16-byte input chunk of the current literal chunk's bytes, where the window loads
        // stop (bytes past it belong to another wave's chunk: loaded here, they were loaded twice). (A ring,
        // a window's first chunks moved in LDS from the previous window's unused tail instead of
        // reloaded, read the same bytes from HBM, +2 % time: those reloads hit the L2)
        constexpr bool kCut = HPK_WIN_CUT != 0;
        constexpr uint32_t kWinC = (uint32_t)kWinB / 16u;
        auto chunk_lim = [&](uint32_t x) {  // x: in_off at the literal chunk's end
            x = min(x, a.in_cap) + a.in_mis;
            return min(last16, x ? (x - 1u) >> 4 : 0u);
        };
        uint32_t clim = kCut ? chunk_lim(gend0) : last16;
        auto prefetch = [&](uint32_t c, uint32_t e, uint32_t base16) {
            const uint32_t cnt = min(128u, e - c);  // >= 1
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t t = c + min(lane + 64u * r, cnt - 1u);
                io0[r] = a.in_off[t];
                if (!kCompact) oo0[r] = a.out_off[t];  // (kCompact: made from io0 in ends())
            }
            ie = a.in_off[c + cnt];
            if (!kCompact) oe = a.out_off[c + cnt];
            pcnt = cnt;
            pc = c;
            const uint4* g16 = reinterpret_cast<const uint4*>(a.in_base);
#pragma unroll
            for (int r = 0; r < R; ++r) ch[r] = ld16(g16 + min((base16 >> 4) + lane + 64u * r, clim));
        };
        // the end offsets of the slots (wave_shl:1, lane i takes lane i + 1's value; lane 63 the next
        // round's first, or slot 128's; a slot at or past the batch's last takes slot 128's)
        uint32_t io1[2], oo1[2];
        auto ends = [&]() {
            if (kCompact) {
#pragma unroll
                for (int r = 0; r < 2; ++r) oo0[r] = ulay(pc + min(lane + 64u * r, pcnt - 1u), io0[r]);
                oe = ulay(pc + pcnt, ie);
            }
            const uint32_t i1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)io0[1]);
            const uint32_t o1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)oo0[1]);
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t ni = (uint32_t)__builtin_amdgcn_update_dpp((int)(r ? ie : i1), (int)io0[r], 0x130, 0xF, 0xF, false);
                const uint32_t no = (uint32_t)__builtin_amdgcn_update_dpp((int)(r ? oe : o1), (int)oo0[r], 0x130, 0xF, 0xF, false);
                const bool last = lane + 64u * r + 1u >= pcnt;
                io1[r] = last ? ie : ni;
                oo1[r] = last ? oe : no;
            }
        };
        // A wave holds one chunk at a time and claims the next when its current one ends (its first
        // offsets are then loaded under the fill's setup): claimed a chunk ahead, the range's last
        // chunks were held by a few waves while the workgroup's others waited (5 % of a wave's time)
        uint32_t cur = cur0, ce = ce0;  // the first chunk (above)
        given = true;
        uint32_t gin = 0, gout = 0;
        uint32_t sens[4] = {0u, 1u, 2u, 3u};  // diagnostic modes 6 / 7 only
        if (cur < ce) {
            gin = gin0 + a.in_mis;
            gout = (kCompact ? ulay(cur, gin0) : gout0) + a.out_mis;
            prefetch(cur, ce, gin & ~15u);
        }
        // the previous fill, not yet written back: literals [pcur, pcur + pk), output [pG0, pG1), and
        // each lane's (up to) two results: length | status << 24 and the literal's index in the fill
        uint32_t pk = 0, pcur = 0, pG0 = 0, pG1 = 0;
        uint32_t rv0 = 0, rv1 = 0, ri0 = 0xFFFFFFFFu, ri1 = 0xFFFFFFFFu;
        uint32_t stop = 0;  // s_ctr[0] as read at the previous fill: another wave saw bad offsets
        stamp(11);
        // (LDS addresses of the per-fill transfers are made from an opaque copy of the lane index, so
        // the compiler recomputes them where they are used instead of hoisting a register per round
        // out of the fill loop: hoisted, they spilled, and every reload waited for all memory traffic)
        auto opaque = [](uint32_t x) {
            asm volatile("" : "+v"(x));
            return x;
        };
        auto flush = [&]() {  // the previous fill's image span and results to global memory
            const uint32_t ob = pG0 & ~15u;
            const uint32_t c0 = ob >> 4, c1 = (pG1 + 15u) >> 4;
            uint4* l16 = reinterpret_cast<uint4*>(s_img) + (opaque(lane) - lane);
            uint4* g16 = reinterpret_cast<uint4*>(a.out_base);
            if (kMode != 2) {
                if (lane < 32) {  // the partial chunks at the two ends, one byte per lane (read before the
                                  // chunks are zeroed below)
                    const uint32_t g = lane < 16 ? c0 << 4 : (c1 - 1u) << 4;
                    const bool partial = !(g >= pG0 && g + 16u <= pG1) && (lane < 16 || c1 - 1u != c0);
                    const uint32_t x = g + (lane & 15u);
                    if (partial && x >= pG0 && x < pG1) a.out_base[x] = s_img[x - ob];
                }
#pragma unroll
                for (int r = 0; r < F; ++r) {
                    const uint32_t ci = c0 + lane + 64u * r;
                    if (ci < c1) {
                        if ((ci << 4) >= pG0 && (ci << 4) + 16u <= pG1) st16(g16 + ci, l16[ci - c0]);
                    }
                }
            }
            if (ri0 != 0xFFFFFFFFu) {
                a.out_len[pcur + ri0] = rv0 & 0xFFFFFFu;
                a.status[pcur + ri0] = (uint8_t)(rv0 >> 24);
            }
            if (ri1 != 0xFFFFFFFFu) {
                a.out_len[pcur + ri1] = rv1 & 0xFFFFFFu;
                a.status[pcur + ri1] = (uint8_t)(rv1 >> 24);
            }
            ri0 = ri1 = 0xFFFFFFFFu;
        };
        // (kCompact) the decoded fill [fcur, fcur + fk) packed into the workgroup's span (round 5, v33):
        // its lengths by literal into the window (dead once the fill is decoded), a wave scan, ONE LDS
        // cursor add for the fill's total; then each lane stores its own two slots' literals (the snake's
        // long-with-short pair) from the image to their destinations in 16-byte stores at any byte address
        // (the hardware's unaligned global accesses): a literal of n >= 16 bytes in pieces at 0, 16, ...
        // and its last piece ending at n (rewriting some of its bytes with the same values), one of 4..15
        // bytes in dwords the same way, a shorter one bytewise; each stored dword from two image dwords by
        // alignbyte; the pair's pieces in one loop. Then offsets / lengths / statuses. (The per-chunk
        // gather this replaced, a map from each 16-byte destination chunk to its literal and five image
        // dwords of each of two literals per chunk, cost 1.37-1.45 ms per config-5 shard against
        // 1.12-1.14: DESIGN §4.1d.) q1 / q2: the lane's two queue entries (image offsets)
        auto compact_fill = [&](uint32_t fcur, uint32_t fk, const uint2 q1, const uint2 q2) {
            uint32_t* const s_len = reinterpret_cast<uint32_t*>(s_win);  // [128] len | status << 24, kListed
            uint32_t* const s_ex = s_len + 128;                           // [128] exclusive prefix sums
            static_assert(256 * 4 <= kWinB, "compact tables in the window");
            s_len[lane] = kListed;
            s_len[lane + 64u] = kListed;
            if (ri0 != 0xFFFFFFFFu) s_len[ri0] = rv0;
            if (ri1 != 0xFFFFFFFFu) s_len[ri1] = rv1;
            const uint32_t l0 = s_len[lane], l1 = s_len[lane + 64u];
            const uint32_t x0 = l0 == kListed ? 0u : l0 & 0xFFFFFFu, x1 = l1 == kListed ? 0u : l1 & 0xFFFFFFu;
            const uint32_t i0 = wave_incl_scan(x0, lane), i1 = wave_incl_scan(x1, lane);
            const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)i0, 63);
            const uint32_t ex0 = i0 - x0, ex1 = t0 + i1 - x1;
            const uint32_t tot = t0 + (uint32_t)__builtin_amdgcn_readlane((int)i1, 63);
            uint32_t u = 0;
            if (lane == 0) u = atomicAdd(&s_ctr[9], tot);
            const uint32_t base = wg0 + (uint32_t)__builtin_amdgcn_readfirstlane((int)u);  // (blob-relative)
            if (tot != 0u) {
                const uint32_t D0 = a.out_mis + base;
                s_ex[lane] = ex0;
                s_ex[lane + 64u] = ex1;
                __builtin_amdgcn_wave_barrier();
                const uint32_t* const img32 = reinterpret_cast<const uint32_t*>(s_img);
                uint32_t js[2], jd[2], jn[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t ri = r ? ri1 : ri0, rv = r ? rv1 : rv0;
                    const bool on = ri != 0xFFFFFFFFu && rv != kListed;
                    js[r] = ((r ? q2.y : q1.y) >> 12) & 0x1FFFFu;
                    jd[r] = D0 + s_ex[on ? ri : 0u];
                    jn[r] = on ? rv & 0xFFFFFFu : 0u;
                }
                // the image dword at byte u (any alignment)
                auto dw_at = [&](uint32_t u) {
                    return __builtin_amdgcn_alignbyte(img32[(u >> 2) + 1u], img32[u >> 2], u & 3u);
                };
                uint32_t sp = js[0], dp = jd[0], np = jn[0], tp = 0;
                bool second = true;
                if (np == 0u) {
                    sp = js[1];
                    dp = jd[1];
                    np = jn[1];
                    second = false;
                }
                while (HPK_CW_LANE_DIAG != 2 && __any(tp < np)) {
                    if (tp < np) {
                        if (np >= 16u) {  // a 16-byte piece at t (the last one ending at n)
                            const uint32_t t = min(tp, np - 16u), u = sp + t;
                            const uint32_t sw = u >> 2, s3 = u & 3u;
                            uint32_t A[5];
#pragma unroll
                            for (int j = 0; j < 5; ++j) A[j] = img32[sw + (uint32_t)j];
                            u32x4u v;
                            v.x = __builtin_amdgcn_alignbyte(A[1], A[0], s3);
                            v.y = __builtin_amdgcn_alignbyte(A[2], A[1], s3);
                            v.z = __builtin_amdgcn_alignbyte(A[3], A[2], s3);
                            v.w = __builtin_amdgcn_alignbyte(A[4], A[3], s3);
                            if (HPK_CW_LANE_DIAG == 3)
                                *reinterpret_cast<u32x4u*>(a.out_base + ((dp + t) & ~15u)) = v;
                            else if (HPK_CW_LANE_DIAG == 4)
                                asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
                            else
                                *reinterpret_cast<u32x4u*>(a.out_base + dp + t) = v;
                            tp += 16u;
                        } else if (np >= 4u) {  // dwords at 0, 4, 8 and the last one ending at n
                            u32u* const g = reinterpret_cast<u32u*>(a.out_base + dp);
                            g[0] = dw_at(sp);
                            if (np >= 8u) g[1] = dw_at(sp + 4u);
                            if (np >= 12u) g[2] = dw_at(sp + 8u);
                            *reinterpret_cast<u32u*>(a.out_base + dp + np - 4u) = dw_at(sp + np - 4u);
                            tp = np;
                        } else {
                            for (uint32_t b = 0; b < np; ++b) a.out_base[dp + b] = s_img[sp + b];
                            tp = np;
                        }
                        if (tp >= np && second) {
                            sp = js[1];
                            dp = jd[1];
                            np = jn[1];
                            tp = 0;
                            second = false;
                        }
                    }
                }
            }
            // offsets, lengths, statuses: stored last (a spill reload in between waits for every older
            // vector-memory operation, these stores included)
            if (lane < fk && l0 != kListed) {
                a.co_off[fcur + lane] = base + ex0;
                a.out_len[fcur + lane] = x0;
                a.status[fcur + lane] = (uint8_t)(l0 >> 24);
            }
            if (lane + 64u < fk && l1 != kListed) {
                a.co_off[fcur + lane + 64u] = base + ex1;
                a.out_len[fcur + lane + 64u] = x1;
                a.status[fcur + lane + 64u] = (uint8_t)(l1 >> 24);
            }
        };
        while (cur < ce) {  // wave-uniform
            const uint32_t cntl = min(128u, ce - cur);
            const uint32_t base16 = gin & ~15u, ob16 = gout & ~15u;
            // 1. offsets: bounds (bad), what fits
            bool bad = false;
            uint32_t ex[2], ey[2];
            bool fits[2];
            ends();
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t t = lane + 64u * r;
                bad |= t < cntl && !(io0[r] <= io1[r] && io1[r] <= a.in_cap && oo0[r] <= oo1[r] && oo1[r] <= a.out_cap);
                const uint32_t p0 = io0[r] + a.in_mis, p1 = io1[r] + a.in_mis;
                const uint32_t o0 = oo0[r] + a.out_mis, o1 = oo1[r] + a.out_mis;
                fits[r] = t < cntl && p1 - base16 <= (uint32_t)kWinB && o1 - ob16 <= (uint32_t)G::kImg;
                const uint32_t nbytes = p1 - p0, ocap = o1 - o0;
                const bool fast = ocap >= (nbytes * 8u) / 5u;
                ex[r] = (p0 - base16) | (nbytes << 16);
                ey[r] = t | ((o0 - ob16) << 12) | (fast ? 0u : kQ7Byte);
            }
            const bool wbad = __any(bad) || stop != 0u;
            stamp(1);
            dg_add(8, 1u);
            if (wbad) {  // the rest of the wave's chunks is void; nothing more is decoded or written here
                if (pk) flush();
                pk = 0;
                if (lane == 0) {
                    *a.err = 1u;
                    s_ctr[0] = 1u;
                }
                for (;;) {  // this chunk's rest, then every chunk still unclaimed
                    for (uint32_t i = cur + lane; i < ce; i += 64u) {
                        a.out_len[i] = 0;
                        a.status[i] = (uint8_t)HPK_BAD_OFFSETS;
                    }
                    claim(cur, ce);
                    if (cur >= ce) break;
                }
                break;
            }
            // the fitting literals form a prefix (offsets are non-decreasing)
            const uint64_t f0 = __ballot(fits[0]), f1 = __ballot(fits[1]);
            const uint32_t k = (uint32_t)__popcll(f0) + (uint32_t)__popcll(f1);  // (wave-uniform)
            if (k == 0) {  // literal `cur` alone exceeds the window or the image
                if (pk) flush();
                pk = 0;
                const uint32_t nb = a.in_off[cur + 1] - a.in_off[cur];
                const bool left = nb >= a.long_min && oof(cur + 1) - oof(cur) >= (nb * 8u) / 5u;
                if (lane == 0) {
                    if (left) {
                        leave(cur, nb);
                    } else {
                        const GlobalSrc g{reinterpret_cast<const uint32_t*>(a.in_base), last16 * 4 + 3};
                        uint8_t* dst = a.out_base + gout;
                        if (kCompact) {  // (never with the library's bound layout: such a literal is listed)
                            const uint32_t o = wg0 + atomicAdd(&s_ctr[9], ((nb * 8u) / 5u + 3u) & ~3u);
                            a.co_off[cur] = o;
                            dst = a.out_base + a.out_mis + o;
                        }
                        Lit L = {};
                        lit_bytes_to(L, g, s_lo, [&](uint32_t j, uint8_t v) { dst[j] = v; },
                                     oof(cur + 1) - oof(cur), gin, a.in_off[cur + 1] + a.in_mis - gin);
                        a.out_len[cur] = L.cnt;
                        a.status[cur] = (uint8_t)lit_status(L);
                    }
                }
                cur += 1;
                if (cur == ce) {  // the next chunk
                    claim(cur, ce);
                    if (kCut && cur < ce) clim = chunk_lim(a.in_off[ce]);
                }
                if (cur < ce) {
                    gin = a.in_off[cur] + a.in_mis;
                    gout = oof(cur) + a.out_mis;
                    prefetch(cur, ce, gin & ~15u);
                }
                continue;
            }
            // the fill's end: the last fitting literal's offsets
            const uint64_t fl = f1 ? f1 : f0;
            const int hl = 63 - __builtin_clzll(fl);
            const uint32_t gin_end = (uint32_t)__builtin_amdgcn_readlane((int)((f1 ? io1[1] : io1[0]) + a.in_mis), hl);
            const uint32_t gout_end =
                (uint32_t)__builtin_amdgcn_readlane((int)((f1 ? oo1[1] : oo1[0]) + a.out_mis), hl);
            // where the next fill starts: right after this one, or at the next chunk
            uint32_t cur_n = cur + k, ce_n = ce, gin_n = gin_end, gout_n = gout_end;
            if (cur_n == ce) {
                claim(cur_n, ce_n);
                if (cur_n < ce_n) {
                    gin_n = a.in_off[cur_n] + a.in_mis;
                    gout_n = oof(cur_n) + a.out_mis;
                    if (kCut) clim = chunk_lim(a.in_off[ce_n]);
                }
            }
            // 2. the window, big-endian dwords: bit P of the stream is bit 31 - P % 32 of dword P / 32
            // (staged before the write-back's stores are issued: its loads' vmcnt wait then covers no
            // store of this fill)
            {
                uint4* l16 = reinterpret_cast<uint4*>(s_win) + (opaque(lane) - lane);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint4 c = ch[r];
                    const uint32_t j = lane + 64u * r;
                    if (j < kWinC)
                        l16[j] = make_uint4(__builtin_bswap32(c.x), __builtin_bswap32(c.y), __builtin_bswap32(c.z),
                                            __builtin_bswap32(c.w));
                }
            }
            stamp(4);
            // 3. the previous fill's write-back (its image is read out before this fill's queue lands there)
            if (pk) flush();
            stamp(2);
            // 4. queue, longest first (kRank 0: a counting sort over 32 length classes of 2 bytes, 996-1015
            // us on config 5 against 1121-1175 us for the ballot ranks, r3h/r3j), long literals listed
            // for the long-literal phase instead
            bool qd[2];
            uint32_t key[2];
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t nbytes = ex[r] >> 16;
                const bool lng = nbytes >= a.long_min && !(ey[r] & kQ7Byte);
                if (fits[r] && lng) leave(cur + lane + 64u * r, nbytes);
                qd[r] = fits[r] && !lng;
                key[r] = kRank == 1 ? min(nbytes >> 2, 15u) : min(nbytes >> 1, 31u);
            }
            uint32_t rank0 = 0, rank1 = 0, kq = 0;
            uint2* const q = reinterpret_cast<uint2*>(s_img + 256);  // 128 entries, in the image
            if (kRank == 0) {  // counting sort: class counts by LDS atomics, bases by a wave scan
                uint32_t* const hist = reinterpret_cast<uint32_t*>(s_img);  // 32 counts, then 32 bases
                if (lane < 32) hist[lane] = 0;
                const uint32_t pa = qd[0] ? atomicAdd(&hist[31u - key[0]], 1u) : 0u;
                const uint32_t pb = qd[1] ? atomicAdd(&hist[31u - key[1]], 1u) : 0u;
                const uint32_t v = lane < 32 ? hist[lane] : 0u;
                // inclusive scan within rows of 16 lanes by DPP row shifts (no bpermute addresses to
                // keep: as shuffles they were hoisted and spilled), then row 1 adds row 0's total
                uint32_t x = v;
                x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
                x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
                x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
                x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
                const uint32_t row0 = (uint32_t)__builtin_amdgcn_readlane((int)x, 15);
                x += lane >= 16u ? row0 : 0u;
                if (lane < 32) hist[32 + lane] = x - v;
                kq = (uint32_t)__builtin_amdgcn_readlane((int)x, 31);
                rank0 = qd[0] ? hist[32 + 31 - key[0]] + pa : 0u;
                rank1 = qd[1] ? hist[32 + 31 - key[1]] + pb : 0u;
            }
#pragma unroll
            for (int c = (kRank == 1 ? 15 : 31); kRank != 0 && c >= 0; --c) {
                const bool h0 = qd[0] && key[0] == (uint32_t)c, h1 = qd[1] && key[1] == (uint32_t)c;
                const uint64_t m0 = __ballot(h0), m1 = __ballot(h1);
                const uint32_t p0 = (uint32_t)__popcll(m0);
                const uint32_t b0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
                const uint32_t b1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
                rank0 = h0 ? kq + b0 : rank0;
                rank1 = h1 ? kq + p0 + b1 : rank1;
                kq += p0 + (uint32_t)__popcll(m1);
            }
            if (qd[0]) q[rank0] = make_uint2(ex[0], ey[0]);
            if (qd[1]) q[rank1] = make_uint2(ex[1], ey[1]);
            stamp(3);
            // 5. the snake's two queue entries per lane (read before the image is decoded over), and
            // the workgroup's stop flag for the next fill
            const uint32_t t1 = lane, t2 = 127u - lane;
            const uint2 e1 = kq ? q[min(t1, kq - 1u)] : make_uint2(0u, 0u);
            const uint2 e2 = kq ? q[min(t2, kq - 1u)] : make_uint2(0u, 0u);
            // (through an LDS-qualified pointer: a volatile read through a generic one is a flat load,
            // and its vmcnt(0) wait made every fill wait for its own write-back's stores)
            stop = *(volatile HPK_LDS_AS uint32_t*)(&s_ctr[0]);
            // 6. the next fill's offsets and window, in flight while this one decodes. Issued
            // unconditionally (past the last chunk: this fill's again, never used): under a branch the
            // registers' old and new values met in copies, and a copy waits for its load (vmcnt(0)
            // right after the loads: every fill waited for the next fill's offsets)
            {
                const bool more = cur_n < ce_n;
                prefetch(more ? cur_n : cur, more ? ce_n : cur + k, (more ? gin_n : gin) & ~15u);
            }
            // 7. lane walks: slots t1 then t2
            Lit12 L, N;
            auto load = [&](Lit12& T, const uint2 e, uint32_t tt) {
                T.act = tt < kq && !(e.y & kQ7Byte);
                T.idx = e.y & 0xFFFu;
                const uint32_t nb = e.x >> 16;
                const uint32_t o = (e.y >> 12) & 0x1FFFFu;
                T.X = wbits + (e.x & 0xFFFFu) * 8u + 31u;
                T.Eb = T.X + (T.act ? nb * 8u : 0u);
                T.o = obase + o;
                T.o0 = obase + o;
                T.st = HPK_OK;
                T.prog = false;
                lit12_load(T, wl32);
            };
            load(L, e1, t1);
            if (!(kMode != 1 && HPK_BODY)) load(N, e2, t2);  // (v28 loads the second literal when it starts)
            bool nv = t2 < kq;
            uint32_t sX = 0, sO = 0, sSt = 0;
            bool s1 = false;
            stamp(5);
            uint32_t Lend = 0;  // the second walk's output end (bytes, image-relative)
            if (kMode != 1 && HPK_BODY) {
                // v27: body steps (lit12_body, no fit tests) while a literal has >= kBodyMin bits left,
                // slot t1's body then slot t2's; then the checked steps (lit12_step) for the two
                // literals' last bits, t1's tail then t2's. A lane's first literal waits between the
                // two phases as (aX, aO, aSt). (Measured and not taken, round 5: accumulated dword
                // stores, dword ORs, both bodies or both tails in one block)
                bool body = L.Eb - L.X >= kBodyMin;
                uint32_t aX = L.X, aO = L.o, aSt = L.st;
                bool aAct = L.act, onA = true;
                for (;;) {
                    dg_add(9, 1u);
#pragma unroll
                    for (int s = 0; s < HPK_BODY_UNROLL; ++s) {
                        if (body)
                            lit12_body<kStore, kTab, (kMode >= 8 && kMode <= 10) ? kMode - 7 : 0>(L, wl32, s_lut, s_lo, ol8,
                                                                                                   body);
                        if (kMode == 6) {
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[0]) : "v"(L.X));
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[1]) : "v"(L.o));
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[2]) : "v"(L.Eb));
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[3]) : "v"(L.d1));
                            }
                        }
                    }
                    if (__any(!body)) {
                        const bool sw = !body & onA;
                        if (sw) {  // the first literal's body is done: it waits, the second one starts (its
                                   // state made from the queue entry here, not carried through the loop)
                            aX = L.X;
                            aO = L.o;
                            aSt = L.st;
                            aAct = L.act;
                            load(L, e2, t2);
                            onA = false;
                            body = L.Eb - L.X >= kBodyMin;
                        }
                        if (!__any(body)) break;
                    }
                }
                // tails: both literals of the lane at once, t1's from where its body stopped (restored
                // into L), t2's (in N) from where its body stopped; a step that proves the walk has
                // ended clears `more`, so no step is spent finding out (usually one step per tail)
                N = L;
                L.X = aX;
                L.o = aO;
                L.st = aSt;
                L.act = aAct;
                L.Eb = wbits + (e1.x & 0xFFFFu) * 8u + 31u + (aAct ? (e1.x >> 16) * 8u : 0u);
                L.o0 = obase + ((e1.y >> 12) & 0x1FFFFu);
                L.idx = e1.y & 0xFFFu;
                if (aSt != HPK_OK) L.Eb = L.X;  // ended in its body (EOS / padding): no tail
                lit12_load(L, wl32);
                L.more = L.Eb - L.X >= 5u;  // (fewer bits than the shortest code: ended)
                N.more = N.Eb - N.X >= 5u;
                while (__any(L.more | N.more)) {
                    if (L.more) lit12_step<kStore, true, kTab, true>(L, wl32, s_lut, s_lo, ol8, dmy);
                    if (N.more) lit12_step<kStore, true, kTab, true>(N, wl32, s_lut, s_lo, ol8, dmy);
                }
                // results in the v26 form: the first slot's end state saved, the second in L
                sX = L.X;
                sO = L.o;
                sSt = L.st;
                s1 = L.act;
                L = N;
                Lend = L.o;
            } else if (kMode != 1) {
                for (;;) {
                    dg_add(9, 1u);
#pragma unroll
                    for (int s = 0; s < 2; ++s) {
                        lit12_step<kStore, true>(L, wl32, s_lut, s_lo, ol8, dmy);
                        // sensitivity diagnostics (libhpk_diag.so): mode 6 adds 16 independent VALU per
                        // step (4 chains of 4), mode 7 adds 2 conflict-free LDS reads per step, off the
                        // walk's dependency chain; the kernel's response says which resource binds
                        if (kMode == 6) {
#pragma unroll
                            for (int q = 0; q < 4; ++q) {
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[0]) : "v"(L.X));
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[1]) : "v"(L.o));
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[2]) : "v"(L.Eb));
                                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(sens[3]) : "v"(L.d1));
                            }
                        } else if (kMode == 7) {
                            const uint32_t r1 = reinterpret_cast<volatile uint32_t*>(smem)[lane];
                            const uint32_t r2 = reinterpret_cast<volatile uint32_t*>(smem)[64u + lane];
                            sens[0] += r1 ^ r2;
                        }
                    }
                    const bool fin = !L.prog;  // no progress in the last step: ended (a fixed point) or idle
                    if (__any(fin)) {
                        const bool sw = fin & nv;
                        if (sw) {
                            sX = L.X;
                            sO = L.o;
                            sSt = L.st;
                            s1 = L.act;
                            L = N;
                            nv = false;
                        }
                        if (!__any(!fin | sw)) break;
                    }
                }
                Lend = L.o;
            }
            stamp(6);
            if ((kMode == 6 || kMode == 7) && (kMode == 7 ? sens[0] : sens[0] ^ sens[1] ^ sens[2] ^ sens[3]) == 0x5EB51u)
                a.status[0] = 9u;  // (never: keeps the diagnostic work alive)
            // results: the first slot's from its saved end state, the second's from the walk
            {
                const uint32_t Eb = wbits + (e1.x & 0xFFFFu) * 8u + 31u + (e1.x >> 16) * 8u;
                const uint32_t st = sSt != HPK_OK ? sSt : residual_status(Eb - sX, win_at(wl32, sX - 31u));
                rv0 = (sO - obase - ((e1.y >> 12) & 0x1FFFFu)) | (st << 24);
                ri0 = s1 ? e1.y & 0xFFFu : 0xFFFFFFFFu;
                rv1 = (Lend - L.o0) | (lit12_status(L) << 24);
                ri1 = L.act ? L.idx : 0xFFFFFFFFu;
            }
            if (kMode == 1) {  // diagnostic: no decode
                rv0 = 0;
                ri0 = t1 < kq ? e1.y & 0xFFFu : 0xFFFFFFFFu;
            }
            // 8. a literal whose region is below the decoded bound: code by code, capacity-checked
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint2 e = r == 0 ? e1 : e2;
                const uint32_t tt = r == 0 ? t1 : t2;
                if (tt < kq && (e.y & kQ7Byte)) {
                    const uint32_t i = e.y & 0xFFFu;
                    const uint32_t o = (e.y >> 12) & 0x1FFFFu;
                    Lit B = {};
                    lit_bytes_to(B, LdsSwapSrc{win32}, s_lo, [&](uint32_t j, uint8_t v) { s_img[o + j] = v; },
                                 oof(cur + i + 1) - oof(cur + i), e.x & 0xFFFFu, e.x >> 16);
                    if (r == 0) {
                        rv0 = B.cnt | (lit_status(B) << 24);
                        ri0 = i;
                    } else {
                        rv1 = B.cnt | (lit_status(B) << 24);
                        ri1 = i;
                    }
                }
            }
            stamp(7);
            if (kCompact) {
                // the next fill's prefetched offsets and window are waited for HERE (they landed during the
                // lane loop): waited for after compact_fill, the wait (vmcnt counts loads and stores in
                // issue order) would cover every store of the fill's write-back
#pragma unroll
                for (int r = 0; r < 2; ++r) asm volatile("" ::"v"(io0[r]), "s"(ie));
#pragma unroll
                for (int r = 0; r < R; ++r) asm volatile("" ::"v"(ch[r].x), "v"(ch[r].y), "v"(ch[r].z), "v"(ch[r].w));
                compact_fill(cur, k, e1, e2);
            } else {
                pk = k;
                pcur = cur;
                pG0 = gout;
                pG1 = gout_end;
            }
            cur = cur_n;
            ce = ce_n;
            gin = gin_n;
            gout = gout_n;
        }
        if (pk) flush();
        stamp(2);
    }
    // ---- the literals left to the long-literal phase ----
    __syncthreads();  // every wave's fills, list entries and stores are out
    const uint32_t c1 = s_ctr[1], c2 = s_ctr[2], nh = min(s_ctr[8], kHugeMax);
    huge_phase<G::kBlock, kTab>(a, s_huge, nh, reinterpret_cast<uint32_t*>(smem + G::kWaveOff), s_lut, s_lo);
    if (c1 + c2) {
        static_assert(G::kWaveOff % 16 == 0, "long-phase rings");
        uint8_t* const area = smem + G::kWaveOff;
        constexpr int kLB = HPK_LONG_WAVES * 64;  // the fill kernel's geometry (hpk_long.h)
        constexpr int kLQ = kLB * (HPK_LONG_RING * 4 + HPK_LONG_OS);
        static_assert(kLQ + HPK_LONG_WAVES * HPK_LONG_CLAIM * 16 <= G::kWaves * G::kWaveBytes, "long-phase LDS");
        long_phase<kLB, HPK_LONG_U, HPK_LONG_RING, kMode == 5 ? 1 : 0, G::kBlock, HPK_LONG_OS, HPK_LONG_CLAIM, kTab>(
            a, BA, BB, c1, c2, &s_ctr[3], reinterpret_cast<uint32_t*>(area), area + kLB * HPK_LONG_RING * 4,
            reinterpret_cast<uint4*>(area + kLQ), s_lut, s_lo);
    }
    stamp(10);
    if (kMode == 3) {
        __syncthreads();  // (every lane 0's adds are in)
        if (lane < 12) {
            const uint32_t v = lane == 0 ? (uint32_t)__builtin_amdgcn_s_memtime() - t_start : s_dg[wv * 12u + lane];
            a.dbg[((uint64_t)blockIdx.x * G::kWaves + wv) * 16u + lane] = v;
        }
    }
}

}  // namespace hpkdec
