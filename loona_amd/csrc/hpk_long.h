// hpk_long.h — long-literal decode phase (v19): one lane per literal, streaming from HBM.
//
// The fill kernel (hpk_decode12 with kLongK) leaves the literals of >= long_min encoded bytes whose
// region holds the decoded bound (and whole ranges dominated by them) to this phase, which the same
// workgroup runs once its fills are done, on its own literal range: it lists them in
// long_list[its range), those of >= long_big bytes from the front (c1 of them) and the others from
// the back (c2), so the longest start first. Measured on config 3 (profiles/r02/rejected/), a
// cooperative walk costs 0.47-0.9 VALU per input bit and wave (speculative segments resync slowly
// on header text: 78 % within 64 bits) against ~0.08 for a lane walk, and a fill of the fill
// kernel waits for its longest literal, decoded by one lane. So here a literal is decoded by ONE
// lane with the fill kernel's two-lookup step, and the parallelism comes from decoding thousands of
// long literals at once. Measured and not taken: a separate launch over all workgroups' lists
// (config 3 0.90 ms, but 4.75 us on every batch with nothing to leave), and claims across
// workgroups inside the fill kernel (a release fence per workgroup to publish its list: config 2
// 61.8 us, config 3 1.00 ms).
//   * 8 waves per workgroup (the other 8 exit), no barriers: a lane that finishes takes the next
//     literal from its wave's LDS queue; a wave whose queue runs dry claims the next 64 entries of
//     the list (an LDS counter);
//   * each lane streams its literal through an input ring in LDS (dword j of lane t at
//     ring[j % kRing][t]: conflict-free). Global loads are issued only at wave-uniform refill points,
//     every kU steps, two 16-byte chunks per lane into registers, and written to the ring at the
//     NEXT refill point: a load has kU steps to land before anything waits on it (a load waited for
//     where a lane needs it stalls the whole wave for the HBM latency at every 16 bytes);
//   * decoded bytes go to a 96-byte output buffer per lane in LDS, a step's bytes as 4 byte
//     stores at fixed offsets from the lane's position (the buffer is the lane's own: the bytes
//     past the decoded ones are overwritten later or never stored out; no dummy slot, no address
//     select), and leave it at refill points as 16-byte stores of
//     whole 16-byte groups of the output (a literal's first and last group bytewise), the partial
//     group moved to the buffer's front: scattered dword stores straight from the step cost a TA
//     cycle per lane and dword (0.8 ms of config 3 in the first measurement);
//   * memory operations are buffer instructions (one VGPR offset) whose operands stay live until
//     the next refill point (pin), and the claim's loads are straight-line: the first version had
//     vmcnt waits for everything (the refill loads included) in the first step of every period,
//     where the compiler re-used registers it could not prove free of a pending memory operation;
//   * a lane's step budget for the period is set at the refill point from its ring's lookahead
//     (a step advances < 2 dwords), not checked in every step;
//   * a literal that ends is finished (padding check, last bytes, length, status) at the next
//     refill point, outside the steps.
// The regions (LDS of the fill kernel, free after its fills): input rings (64 KiB) and output
// buffers (48 KiB) over the input window and the output image, wave queues over the fill queue.
// Semantics are the fill kernel's lane walk (huffman.rs:95-161): the walk stops where no code fits,
// an EOS is EOSInString at once, then >7 residual bits PaddingTooLarge, non-ones InvalidPadding.
#pragma once
// (included by hpk_decode12.h after the lane-walk helpers it uses: lut12, residual_status, lo_decode)
#include "hpk_decode_kernel.h"

namespace hpkdec {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Raw buffer resources (gfx9 dword 3): accesses past num_records bytes are dropped (stores) or read 0
// (loads), and every access is ONE VGPR offset plus its data registers, which the kernel keeps live
// (pin) so that no later instruction overwrites a register a pending store still reads.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

// Bytes [lo, hi) of the 16-byte output group at byte offset gb (v: its four dwords, b[e] = byte e in
// the low byte): whole dwords by dword stores, the rest bytewise (straight-line, no loop).
__device__ __forceinline__ void store_part(__amdgpu_buffer_rsrc_t r, uint32_t gb, uint32_t lo, uint32_t hi,
                                           const uint32_t (&v)[4], const uint32_t (&b)[16]) {
#pragma unroll
    for (uint32_t d = 0; d < 4u; ++d) {
        if (lo <= 4u * d && 4u * d + 4u <= hi) {
            __builtin_amdgcn_raw_buffer_store_b32(v[d], r, gb, 4 * d, 0);
        } else {
#pragma unroll
            for (uint32_t e = 0; e < 4u; ++e)
                if (4u * d + e >= lo && 4u * d + e < hi)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)b[4u * d + e], r, gb, 4 * d + e, 0);
        }
    }
}

// LPT class of a literal listed for this phase (which takes its list front to back): its job size, half the
// literal for one decoded as two halves (HPK_LONG_SPLIT), in 128-byte classes, 0 the longest. The dense
// listings order their lists by it (a counting sort), so the longest jobs start first.
__device__ __forceinline__ uint32_t lpt_class_of(uint32_t nb);

// Keep a value's register live (and unchanged) up to here.
__device__ __forceinline__ void pin(uint32_t x) { asm volatile("" ::"v"(x)); }

#ifndef HPK_LONG_WAVES
#define HPK_LONG_WAVES 8  // waves of the fill kernel's workgroup that run the phase (the others exit)
#endif
#ifndef HPK_LONG_U
#define HPK_LONG_U 8  // steps between refill points
#endif
#ifndef HPK_LONG_CLAIM
#define HPK_LONG_CLAIM 64  // list entries per claim (32 or 64)
#endif
#ifndef HPK_LONG_RING
#define HPK_LONG_RING 32  // input ring dwords per lane
#endif

#ifndef HPK_LONG_TAILPT
#define HPK_LONG_TAILPT 1  // round 6: the steps between refill points are body steps only (>= kBodyMin bits left);
                           // a literal's last bits are walked with checked steps at the refill point, by the
                           // lanes in their tail only (both step kinds in one loop made every step pay both:
                           // some lane of 64 is nearly always in its tail)
#endif

#ifndef HPK_LONG_SPLIT
#define HPK_LONG_SPLIT 0  // round 6: literals of >= this many encoded bytes decoded as two halves (0: off; measured slower
                          // than the LPT list order alone: config 3 930 vs 635 us, profiles/r06/split_rejected/)
#endif

#ifndef HPK_LONG_LEAD
#define HPK_LONG_LEAD 64  // bytes the second half of a split literal walks before its split point (512 bits: a walk
                          // started anywhere in config-3 text met the true one within 512 bits in all of 19,609
                          // samples, within 256 bits in 99.66 %; scripts/sync_stats.py)
#endif

#ifndef HPK_LONG_OS
#define HPK_LONG_OS 80  // output buffer bytes per lane (a multiple of 16; 80: 20-dword stride, 4-way bank aliasing instead of 96's 8-way, config 3 870 vs 883 us)
#endif

// Long-literal phase of fill workgroup g = blockIdx.x (all kBlockAll threads call it, after the
// fills; c1 / c2 = its class counts). kBlock threads decode (one wave queue of kQ entries each in
// s_q), kU steps between refill points, kRing input dwords per lane in s_ring and a kOS-byte
// output buffer per lane in s_out (16-byte aligned). kDiag (diagnostic builds): per-wave counters
// into a.dbg[wave * 16 + i] (scripts/diag_decode.py).
#ifndef HPK_LONG_BODY
#define HPK_LONG_BODY 1  // v28: body steps (no fit tests) while a literal has >= kBodyMin bits left
#endif

__device__ __forceinline__ uint32_t lpt_class_of(uint32_t nb) {
    const uint32_t key = (HPK_LONG_SPLIT && nb >= (uint32_t)HPK_LONG_SPLIT) ? nb >> 1 : nb;
    return 31u - min(key >> 7, 31u);
}

template <int kBlock, int kU, int kRing, int kDiag, int kBlockAll, int kOSz = HPK_LONG_OS, int kClaim = 64,
          int kTab = 2,            // kTab: the layout of s_lut (2 = LUT2, the fill kernel; 3 = LUT3, the wave kernel)
          bool kCompact = false>   // the compacted mode: a claim takes its literals' decoded bounds from a.cursor
__device__ __forceinline__ void long_phase(const DecodeArgs& a, uint32_t ba, uint32_t bb, uint32_t c1, uint32_t c2,
                                           uint32_t* s_claim, uint32_t* s_ring, uint8_t* s_out, uint4* s_q,
                                           uint32_t* s_qx, uint32_t* s_rec, const uint32_t* s_lut,
                                           const uint16_t* s_lo) {
    constexpr uint32_t kChunk = kClaim;        // list entries per claim (at most one per lane)
    constexpr uint32_t kQ = kChunk;            // per-wave queue: a claim is made only once the lanes that
                                               // want a literal have emptied the queue, so it never holds
                                               // more than one claim
    static_assert(kClaim == 32 || kClaim == 64, "claim size");
    // Output buffer per lane: bytes [lb, ob) of the output (lb 16-byte aligned) at [0, ob - lb). A
    // refill point stores every whole 16-byte group and moves the partial one (< 16 bytes) to the
    // front, so a period starts with <= 15 bytes and adds <= 5 per step: 15 + 5 kU + 3 bytes
    // (a step's 4-byte store) must fit.
    constexpr uint32_t kOS = kOSz;
    // (HPK_LONG_TAILPT: a tail at the refill point adds <= 6 bytes; a first half's crossing of its end <= 11:
    // the codes starting in the < 54 bits before it)
    static_assert(15 + 5 * kU + 3 + (HPK_LONG_SPLIT ? 11 : HPK_LONG_TAILPT ? 6 : 0) < (int)kOS, "output buffer");
    static_assert((kRing & (kRing - 1)) == 0 && kRing >= 16, "input ring: a power of two >= 16 dwords");
    static_assert(kBlock % 64 == 0 && kBlock <= kBlockAll, "decoding waves");
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t total = c1 + c2;
    if (total == 0) return;  // (block-uniform: nothing left to this phase)
    if (tid >= (uint32_t)kBlock) return;  // (no barrier follows)
    uint4 (*sq)[kQ] = reinterpret_cast<uint4 (*)[kQ]>(s_q);
    // Split literals (HPK_LONG_SPLIT, round 6). The phase's length is set by each workgroup's longest
    // literal, one lane's serial walk (config 3: ~1,240 steps against ~800 per lane on average, 25 % of the
    // lane-steps idle at the end). A literal of >= HPK_LONG_SPLIT bytes is decoded as two halves by two
    // lanes of the same wave: the first half (kP0) from the literal's start to its first code boundary at
    // or after the split point s (E0); the second half (kLead) from kLeadB bytes before s with no output
    // until its walk reaches a code boundary at or after s (S1, kP1 from there: a walk started anywhere
    // falls into step with the true one within HPK_LONG_LEAD bytes nearly always on header text), its bytes at the provisional offset floor(8 (s - start) / 5) of the region
    // (s - start is a multiple of 5, and the first half's codes all start before s, so its bytes fit
    // below). When both halves are done the wave joins them: S1 == E0 -> the second half's bytes move down
    // to follow the first's; otherwise the walk is redone from E0 (kCont, a true start) by the lane that
    // finished last. An EOS in the second half's lead-in is a 30-bit code, not an error. Per wave: kRecs
    // records of 8 words (o0, E0 - s8 | st0 << 16, S1 - s8, c0, c1, st1, done bits then the literal's index,
    // P1) and one extra word per queue entry (start bit, mode, record).
    constexpr uint32_t kNorm = 0, kP0 = 1, kLead = 2, kP1 = 3, kCont = 4;
    constexpr uint32_t kLeadB = HPK_LONG_LEAD, kRecs = 64, kRecW = 8;
    uint32_t* const qx = s_qx + wv * kQ;
    uint32_t* const rec_base = s_rec + wv * kRecs * kRecW;
    uint64_t recfree = ~0ull;  // wave-uniform: free records
    const uint32_t in_end = min(a.in_off[a.n], a.in_cap) + a.in_mis;
    // (whole 16-byte chunks: a load that reaches past num_records reads 0 in all its dwords)
    const __amdgpu_buffer_rsrc_t r_in = buf_rsrc(a.in_base, (in_end + 15u) & ~15u);
    const __amdgpu_buffer_rsrc_t r_out = buf_rsrc(a.out_base, a.out_cap + a.out_mis);
    const __amdgpu_buffer_rsrc_t r_len = buf_rsrc(a.out_len, min(a.n, 0x3FFFFFFFu) * 4u);
    const __amdgpu_buffer_rsrc_t r_st = buf_rsrc(a.status, a.n);
    uint32_t* ring = s_ring + tid;        // input dword j: ring[(j % kRing) * kBlock]
    uint8_t* const obuf = s_out + tid * kOS;  // output byte p: obuf[p - lb]
    bool more = true;               // wave-uniform: claims may remain
    uint32_t qh = 0, qt = 0;        // wave-uniform: the wave's queue sq[wv][qh, qt) (mod kQ)
    // Lane state. Input positions are relative to the literal's first 16-byte chunk q0: X = bit
    // position + 31 (the fill kernel's convention), the pair (d0, d1) = dwords (X >> 5) - 1 and
    // X >> 5, d2 the next; the ring holds dwords [.., h) (h a multiple of 8), the registers P the next
    // 8. Output positions are byte addresses relative to out_base: o0 the literal's first, ob the
    // next, fl the first not yet stored to global memory, lb the one at the buffer's front.
    bool act = false, live = false, pend = false, done = false;
    uint32_t idx = 0, X = 0, Eb = 0, d0 = 0, d1 = 0, d2 = 0, st = HPK_OK, q0 = 0, span = 0, h = 0;
    uint32_t mode = kNorm, rec = 0, sbX = 0;  // (HPK_LONG_SPLIT) the lane's part of a split literal, its
                                              // record, the split point in its X coordinates
    uint32_t o0 = 0, ob = 0, fl = 0, lb = 0;
    u32x4 P0 = {}, P1 = {};
    unsigned long long dg[12] = {};  // kDiag: 0 cycles, 1 points, 2 lane-steps, 3 stalled, 4 idle (no literal),
                                     // 9 waiting for a literal's first chunks, 10 ended and waiting, 11 ring-write cycles,
                                     // 5 assign cycles, 6 step cycles, 7 refill cycles, 8 literals
    const unsigned long long dt0 = kDiag ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
        unsigned long long dtp = kDiag ? __builtin_amdgcn_s_memtime() : 0;
        if (kDiag) dg[1] += 1;
        // ---- refill point (wave-uniform) ----
        // 1. the chunks loaded at the previous point go to the ring
        if (pend) {
            if (kDiag) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t b = h & (kRing - 1u);
            ring[(b + 0) * kBlock] = __builtin_bswap32(P0.x);
            ring[(b + 1) * kBlock] = __builtin_bswap32(P0.y);
            ring[(b + 2) * kBlock] = __builtin_bswap32(P0.z);
            ring[(b + 3) * kBlock] = __builtin_bswap32(P0.w);
            ring[(b + 4) * kBlock] = __builtin_bswap32(P1.x);
            ring[(b + 5) * kBlock] = __builtin_bswap32(P1.y);
            ring[(b + 6) * kBlock] = __builtin_bswap32(P1.z);
            ring[(b + 7) * kBlock] = __builtin_bswap32(P1.w);
            h += 8u;
            pend = false;
        }
        if (kDiag) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            dg[11] += t - dtp;
        }
        // 2. a literal whose first chunks just arrived: its window
        if (act && !live && (h != 0 || span == 0)) {
            const uint32_t j = X >> 5;  // 0..4
            d0 = ring[((j - 1u) & (kRing - 1u)) * kBlock];  // (unread when j == 0: X is dword-aligned)
            d1 = ring[j * kBlock];
            d2 = ring[(j + 1u) * kBlock];
            live = true;
        }
        // 2a. (HPK_LONG_SPLIT) halves within 54 bits (a body step's reach) of the split point, the ring holding
        // what they read: lookups that take a table entry's second code only if it starts before the split
        // point (a 13..30-bit code or EOS by the leading-ones table), until the walk reaches the split point
        if (HPK_LONG_SPLIT) {
            for (;;) {
                const bool cr = act && live && !done && (mode == kP0 || mode == kLead) && sbX - X < 54u &&
                                (h * 4u >= span || h >= ((sbX + 30u) >> 5) + 2u);
                if (!__any(cr)) break;
                bool reached = false;
                if (cr) {
                    const uint32_t j0 = X >> 5;
                    const uint32_t d3 = ring[((j0 + 2u) & (kRing - 1u)) * kBlock];
                    const uint32_t w = __builtin_amdgcn_alignbit(d0, d1, ~X);
                    const uint32_t e = s_lut[w >> (32 - HPK_LUT_BITS)];
                    const uint32_t nc = kTab == 3 ? HPK_L3_CODES(e) : HPK_L2_CODES(e);
                    if (nc != 0u) {  // one or two codes of <= 12 bits: the first starts before the split point
                        const uint32_t l0 = kTab == 3 ? HPK_L3_LEN0(e) : HPK_L2_LEN0(e);
                        const uint32_t u = kTab == 3 ? HPK_L3_HELD(e) : HPK_L2_HELD(e);
                        const bool two = nc == 2u && X + l0 < sbX;
                        if (mode == kP0) {
                            uint8_t* const p = obuf + (ob - lb);
                            p[0] = (uint8_t)e;
                            p[1] = (uint8_t)(e >> 16);
                            ob += two ? 2u : 1u;
                        }
                        const uint32_t xn = X + (two ? u : l0);
                        const bool cross = (xn ^ X) > 31u;
                        d0 = cross ? d1 : d0;
                        d1 = cross ? d2 : d1;
                        d2 = cross ? d3 : d2;
                        X = xn;
                        reached = X >= sbX;
                    } else {
                        uint32_t sy, len;
                        bool eos;
                        lo_decode(w, s_lo, sy, len, eos);
                        if (mode == kP0 && eos) {  // the first half's EOS is the literal's (huffman.rs:112-116)
                            st = HPK_EOS_IN_STRING;
                            done = true;
                        } else {  // (an EOS in the lead-in: a 30-bit code, lo_decode's len)
                            if (mode == kP0) {
                                obuf[ob - lb] = (uint8_t)sy;
                                ob += 1u;
                            }
                            X += len;
                            const uint32_t j = X >> 5;
                            d0 = ring[((j - 1u) & (kRing - 1u)) * kBlock];
                            d1 = ring[(j & (kRing - 1u)) * kBlock];
                            d2 = ring[((j + 1u) & (kRing - 1u)) * kBlock];
                            reached = X >= sbX;
                        }
                    }
                }
                if (reached) {
                    if (mode == kP0) {
                        done = true;  // E0 recorded when it is finished (4)
                    } else {          // the second half is at S1: its output starts here
                        rec_base[rec * kRecW + 2] = X - sbX;
                        mode = kP1;
                    }
                }
            }
        }
        // 2b. (HPK_LONG_TAILPT) lanes whose literal has fewer than kBodyMin bits left, all of its chunks in
        // the ring: checked steps (lit12_step's) until the walk ends; the literal is finished in 4 below
        if (HPK_LONG_TAILPT) {
            for (;;) {
                const bool tl = act && live && !done && Eb - X < kBodyMin && h * 4u >= span;
                if (!__any(tl)) break;
                if (tl) {
                    const uint32_t j0 = X >> 5;
                    const uint32_t d3 = ring[((j0 + 2u) & (kRing - 1u)) * kBlock];
                    const uint32_t w = __builtin_amdgcn_alignbit(d0, d1, ~X);
                    const uint32_t rem = Eb - X;
                    const uint32_t e1 = s_lut[w >> (32 - HPK_LUT_BITS)];
                    bool a1, a2;
                    const uint32_t u1 = lut12<kTab>(e1, rem, a1, a2);
                    bool park = !a1 & (rem > (uint32_t)HPK_LUT_BITS);
                    const bool cont = a1 & (a2 | lut_nottwo<kTab>(e1));
                    const uint32_t rem2 = rem - u1;
                    const uint32_t e2 = s_lut[(w << u1) >> (32 - HPK_LUT_BITS)];
                    bool b1, b2;
                    const uint32_t v2 = lut12<kTab>(e2, rem2, b1, b2);
                    park |= cont & !b1 & (rem2 > (uint32_t)HPK_LUT_BITS);
                    b1 &= cont;
                    b2 &= cont;
                    const uint32_t g1 = (uint32_t)a1 + (uint32_t)a2, g2 = (uint32_t)b1 + (uint32_t)b2;
                    uint8_t* const p = obuf + (ob - lb);
                    p[0] = (uint8_t)e1;
                    p[1] = (uint8_t)(e1 >> 16);
                    p[g1] = (uint8_t)e2;
                    p[g1 + 1] = (uint8_t)(e2 >> 16);
                    ob += g1 + g2;
                    const uint32_t xn = X + u1 + (cont ? v2 : 0u);
                    const bool cross = (xn ^ X) > 31u;
                    d0 = cross ? d1 : d0;
                    d1 = cross ? d2 : d1;
                    d2 = cross ? d3 : d2;
                    X = xn;
                    bool prog = a1 | park;
                    // both entries used whole: more codes may follow; otherwise the walk has ended
                    const bool mo = park | (b1 & (b2 | lut_nottwo<kTab>(e2)));
                    if (park) {  // a 13..30-bit code or EOS with > 12 bits left
                        const uint32_t wp = __builtin_amdgcn_alignbit(d0, d1, ~X);
                        uint32_t sy, len;
                        bool eos;
                        lo_decode(wp, s_lo, sy, len, eos);
                        if (len > Eb - X) {  // huffman.rs:128-134
                            st = HPK_PADDING_TOO_LARGE;
                            prog = false;
                        } else if (eos) {  // huffman.rs:112-116
                            st = HPK_EOS_IN_STRING;
                            prog = false;
                        } else {
                            obuf[ob - lb] = (uint8_t)sy;
                            ob += 1u;
                            const uint32_t xp = X + len;
                            const uint32_t j = xp >> 5;
                            d0 = ring[((j - 1u) & (kRing - 1u)) * kBlock];
                            d1 = ring[(j & (kRing - 1u)) * kBlock];
                            d2 = ring[((j + 1u) & (kRing - 1u)) * kBlock];
                            X = xp;
                        }
                    }
                    done = !prog || !mo;
                }
            }
        }
        // 3. output to global memory: a literal's first 16-byte group (it shares it with the previous
        // region) once complete, bytewise; then whole groups as 16-byte stores; the partial group
        // to the buffer's front. Every register a store reads its data from stays live until after
        // the steps (pin).
        u32x4 gv[4];
        uint32_t hv[4], hb[16], tv[4], tb[16], lv = 0, sv = 0;
        uint32_t ha = 0, ga = 0, ta = 0, ia = 0, ja = 0;  // their addresses (pinned too)
        {
            const uint32_t gb = fl & ~15u;  // (== lb: nothing of the literal is stored yet)
            ha = gb;
            if (act && fl != gb && gb + 16u <= ob) {
                const uint32_t* s = reinterpret_cast<const uint32_t*>(obuf);
#pragma unroll
                for (int e = 0; e < 4; ++e) hv[e] = s[e];
#pragma unroll
                for (int e = 0; e < 16; ++e) hb[e] = hv[e >> 2] >> (8 * (e & 3));
                store_part(r_out, gb, fl - gb, 16u, hv, hb);
                fl = gb + 16u;
            }
        }
        {  // (fl is group-aligned here.) All four groups are read before any is stored.
            ga = fl;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t* s = reinterpret_cast<const uint32_t*>(obuf + min((fl - lb) + 16u * k, kOS - 16u));
                gv[k] = u32x4{s[0], s[1], s[2], s[3]};
            }
            uint32_t ng = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (act && ga + 16u * (k + 1) <= ob) {
                    __builtin_amdgcn_raw_buffer_store_b128(gv[k], r_out, ga, 16 * k, 0);
                    ng = k + 1;
                }
            }
            fl += 16u * ng;
            if (act && fl != lb && (fl & 15u) == 0) {  // the partial group (< 16 bytes) to the front
                const uint4 v = *reinterpret_cast<const uint4*>(obuf + (fl - lb));
                *reinterpret_cast<uint4*>(obuf) = v;
                lb = fl;
            }
        }
        // 4. a literal that ended in the last steps: padding check, last bytes, length, status (a half of a
        // split literal: its record instead; the lane that completes the record joins it, 4b)
        bool jown = false;
        if (done) {
            if (st == HPK_OK && mode != kP0 && mode != kLead)
                st = residual_status(Eb - X, __builtin_amdgcn_alignbit(d0, d1, ~X));
            if (ob > fl) {  // [fl, ob) lies in one group, at the buffer's front
                const uint32_t gb = fl & ~15u;
                ta = gb;
                const uint32_t* s = reinterpret_cast<const uint32_t*>(obuf);
#pragma unroll
                for (int e = 0; e < 4; ++e) tv[e] = s[e];
#pragma unroll
                for (int e = 0; e < 16; ++e) tb[e] = tv[e >> 2] >> (8 * (e & 3));
                store_part(r_out, gb, fl - gb, ob - gb, tv, tb);
            }
            lv = ob - o0;
            sv = st;
            ia = idx * 4u;
            ja = idx;
            if (!HPK_LONG_SPLIT || mode == kNorm || mode == kCont) {
                __builtin_amdgcn_raw_buffer_store_b32(lv, r_len, ia, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)sv, r_st, ja, 0, 0);
            } else {
                uint32_t* const R = rec_base + rec * kRecW;
                uint32_t bit;
                if (mode == kP0) {
                    R[1] = ((X - sbX) & 0xFFFFu) | (sv << 16);  // E0 (meaningless after an EOS) and the first half's status
                    R[3] = lv;
                    bit = 1u;
                } else {  // kP1 (a kLead cannot end before its lead-in does; if it did, R[2] has no S1)
                    R[4] = lv;
                    R[5] = sv;
                    bit = 2u;
                }
                jown = (atomicOr(&R[6], bit) | bit) == 3u;
            }
            act = false;
            live = false;
            done = false;
        }
        // 4b. (HPK_LONG_SPLIT) joins, one record at a time by the whole wave: halves that met (S1 == E0) have
        // the second half's bytes moved down behind the first's (16-byte pieces, ascending: a piece's
        // destination never reaches a later piece's source); halves that did not meet have the walk redone
        // from E0 by the lane that completed the record (kCont: a true start at a bit offset, its bytes
        // straight after c0); a first half's EOS is the literal's status at once
        if (HPK_LONG_SPLIT) {
            bool fr = mode == kCont && !act && rec != 0xFFFFFFFFu;  // a continuation finished in 4
            while (__any(jown)) {
                const uint32_t L = (uint32_t)__builtin_ctzll(__ballot(jown));
                const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rec, (int)L);
                const uint32_t* const R = rec_base + r * kRecW;
                const uint32_t ro0 = R[0], e0 = R[1] & 0xFFFFu, s1 = R[2], c0 = R[3];
                const uint32_t li = (uint32_t)__builtin_amdgcn_readlane((int)idx, (int)L);
                bool freed = true;
                uint32_t olen = c0, ost = R[1] >> 16;
                if (ost == HPK_OK && e0 == s1) {  // the second half's bytes moved down behind the first's
                    const uint32_t c1 = R[4], p1 = R[7];
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the halves' stores are done
                    const uint32_t dst = ro0 + c0;
                    for (uint32_t off = 0; off < c1; off += 1024u) {
                        // (every lane's 16-byte piece is read before any is stored; a whole piece's store ends
                        // at or below the next lane's destination, below every later source byte, so the
                        // last lane's bytes, copied after, are still in place)
                        const uint32_t j = off + lane * 16u;
                        const bool whole = j + 16u <= c1;
                        if (whole) {
                            const u32x4u v = *reinterpret_cast<const u32x4u*>(a.out_base + p1 + j);
                            *reinterpret_cast<u32x4u*>(a.out_base + dst + j) = v;
                        }
                        if (!whole)  // (after the whole pieces: see above)
                            for (uint32_t k = j; k < c1; ++k) a.out_base[dst + k] = a.out_base[p1 + k];
                    }
                    olen = c0 + c1;
                    ost = R[5];
                } else if (ost == HPK_OK) {  // the halves did not meet: lane L redoes the walk from E0
                    freed = false;
                    if (lane == L) {
                        const uint32_t sbyte = q0 * 16u + ((sbX - 31u) >> 3);  // (abs, incl. in_mis)
                        const uint32_t pend_b = q0 * 16u + ((Eb - 31u) >> 3);
                        const uint32_t p0 = sbyte + (e0 >> 3);
                        act = true;
                        live = false;
                        mode = kCont;
                        q0 = p0 >> 4;
                        span = pend_b - (q0 << 4);
                        X = (p0 & 15u) * 8u + (e0 & 7u) + 31u;
                        Eb = (pend_b - (q0 << 4)) * 8u + 31u;
                        h = 0;
                        st = HPK_OK;
                        o0 = ro0;
                        ob = ro0 + c0;
                        fl = ob;
                        lb = ob & ~15u;
                    }
                }
                if (freed) {
                    if (lane == 0) {
                        a.out_len[li] = olen;
                        a.status[li] = (uint8_t)ost;
                    }
                    recfree |= 1ull << r;
                }
                if (lane == L) jown = false;
            }
            while (__any(fr)) {  // continuations done: their records free
                const uint32_t L = (uint32_t)__builtin_ctzll(__ballot(fr));
                recfree |= 1ull << (uint32_t)__builtin_amdgcn_readlane((int)rec, (int)L);
                if (lane == L) {
                    fr = false;
                    rec = 0xFFFFFFFFu;
                }
            }
        }
        if (kDiag) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            dg[7] += t - dtp;
            dtp = t;
        }
        // 5. idle lanes take literals from the wave's queue; when it is dry, claim 64 more list entries
#pragma unroll 1
        for (int claims = 0;; ++claims) {
            const bool want = !act;
            if (!__any(want)) break;
            const uint64_t wm = __ballot(want);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(wm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wm, 0u));
            if (want && qh + rank < qt) {
                const uint4 te = sq[wv][(qh + rank) % kQ];
                const uint32_t x = HPK_LONG_SPLIT ? qx[(qh + rank) % kQ] : 0u;
                idx = te.x;
                act = true;
                live = false;
                const uint32_t p0 = te.y + a.in_mis, p1 = te.z + a.in_mis;
                q0 = p0 >> 4;
                span = p1 - (q0 << 4);  // bytes from the first chunk's start to the literal's end
                X = (p0 & 15u) * 8u + 31u;
                Eb = X + (p1 - p0) * 8u;
                h = 0;
                st = HPK_OK;
                o0 = te.w + a.out_mis;
                ob = o0;
                fl = o0;
                lb = o0 & ~15u;
                mode = (x >> 3) & 7u;
                rec = x >> 6;
                // the split point in the lane's X: kLeadB bytes in (kLead), the literal's halfway point (kP0)
                sbX = X + (mode == kP0 ? ((te.z - te.y) / 10u) * 5u : kLeadB) * 8u;
            }
            const uint32_t need = (uint32_t)__popcll(wm);
            const bool enough = need <= qt - qh;
            qh += min(need, qt - qh);
            if (enough || !more || claims == 2) break;  // (at most two claims per refill point)
            // claim the next entries of this workgroup's list (an LDS counter): as many as the queue has room for,
            // two slots each (a literal of >= HPK_LONG_SPLIT bytes is queued as its two halves, kP0 then kLead,
            // with a record, while records last: taken by the next lanes that want work, so the halves of the
            // list's first (longest) literals start together)
            const uint32_t room = HPK_LONG_SPLIT ? (kQ - (qt - qh)) / 2u : kQ - (qt - qh);
            if (room == 0u) break;
            uint32_t rr = 0;
            if (lane == 0) rr = atomicAdd(s_claim, room);
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rr, 0);
            if (r >= total) {
                more = false;
                break;
            }
            // entries r + lane: [0, c1) from the front of the range, then from the back
            const uint32_t e = r + lane;
            const bool ok = lane < room && e < total;
            const uint32_t lpos = ok ? (e < c1 ? ba + e : bb - 1u - (e - c1)) : ba;
            const uint32_t i0 = a.long_list[lpos];  // (a load either way: see the note below)
            const uint32_t i = ok ? i0 : 0u;
            // straight-line loads (no branch around them): a load under a branch leaves the compiler
            // unsure whether its register is still pending, and it then waits for all memory
            // operations (the refill loads included) before the steps reuse the register
            uint4 li;
            if (kCompact) {  // the claim's literals' decoded bounds: one cursor add per claim, offsets to co_off
                li = make_uint4(i, a.in_off[i], a.in_off[i + 1], 0u);
                const uint32_t bd = ok ? ((li.z - li.y) * 8u) / 5u : 0u;
                uint32_t x = bd;
#pragma unroll
                for (int d = 1; d < 64; d <<= 1) {
                    const uint32_t y = __shfl_up(x, d);
                    if (lane >= (uint32_t)d) x += y;
                }
                uint32_t cb = 0;
                if (lane == 63u) cb = atomicAdd(a.cursor, x);
                li.w = (uint32_t)__builtin_amdgcn_readlane((int)cb, 63) + x - bd;
                if (ok) a.co_off[i] = li.w;
            } else {
                li = make_uint4(i, a.in_off[i], a.in_off[i + 1], a.lit_out[i]);
            }
            bool sp = false;
            uint32_t srec = 0;
            if (HPK_LONG_SPLIT) {
                uint64_t cm = __ballot(ok && li.z - li.y >= (uint32_t)HPK_LONG_SPLIT);
                while (cm && recfree) {
                    const uint32_t L = (uint32_t)__builtin_ctzll(cm);
                    const uint32_t rf = (uint32_t)__builtin_ctzll(recfree);
                    recfree &= recfree - 1ull;
                    cm &= cm - 1ull;
                    if (lane == L) {
                        srec = rf;
                        sp = true;
                    }
                }
            }
            const uint32_t k = ok ? (sp ? 2u : 1u) : 0u;
            uint32_t inc = k;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(inc, d);
                if (lane >= (uint32_t)d) inc += y;
            }
            const uint32_t slot = qt + inc - k;
            if (ok) {
                sq[wv][slot % kQ] = li;
                if (HPK_LONG_SPLIT) qx[slot % kQ] = sp ? (kP0 << 3) | (srec << 6) : 0u;
            }
            if (sp) {  // the second half, and the record
                const uint32_t hb = ((li.z - li.y) / 10u) * 5u;  // a multiple of 5 bytes in (>= kLeadB)
                sq[wv][(slot + 1u) % kQ] = make_uint4(li.x, li.y + hb - kLeadB, li.z, li.w + (hb / 5u) * 8u);
                qx[(slot + 1u) % kQ] = (kLead << 3) | (srec << 6);
                uint32_t* const R = rec_base + srec * kRecW;
                R[0] = li.w + a.out_mis;
                R[2] = 0xFFFFFFFFu;
                R[6] = 0u;
                R[7] = li.w + a.out_mis + (hb / 5u) * 8u;
            }
            qt += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        }
        if (kDiag) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            dg[5] += t - dtp;
            dtp = t;
        }
        if (!__any(act)) break;  // no literal left for this wave
        // 6. the next two chunks, while the ring has room for them past the window's first dword
        if (act && h * 4u < span && h + 8u + 1u <= kRing + (X >> 5)) {
            P0 = __builtin_amdgcn_raw_buffer_load_b128(r_in, (q0 + (h >> 2)) * 16u, 0, 0);
            P1 = __builtin_amdgcn_raw_buffer_load_b128(r_in, (q0 + (h >> 2)) * 16u + 16u, 0, 0);
            pend = true;
        }
        // ---- kU steps while the input ring holds what a step can reach: a step advances < 2 dwords
        // (<= 24 bits of lookups + a <= 30-bit long code) and reads up to dword (X >> 5) + 3; the
        // lane's budget of steps is set here, not checked per step (config 3 936.7 vs 1026.9 us) ----
        const uint32_t x5 = X >> 5;
        const uint32_t budget = !(act && live) ? 0u
                                : h * 4u >= span ? (uint32_t)kU
                                : x5 + 4u <= h ? min((uint32_t)kU, ((h - x5 - 4u) >> 1) + 1u) : 0u;
        for (int s = 0; s < kU; ++s) {
            const bool go = (uint32_t)s < budget && !done && (!HPK_LONG_TAILPT || Eb - X >= kBodyMin) &&
                            (!HPK_LONG_SPLIT || !(mode == kP0 || mode == kLead) || sbX - X >= 54u);
            if (kDiag) {
                dg[2] += (unsigned long long)__popcll(__ballot(go));
                dg[3] += (unsigned long long)__popcll(__ballot(act && live && !done && !go));
                dg[4] += (unsigned long long)__popcll(__ballot(!act));
                dg[9] += (unsigned long long)__popcll(__ballot(act && !live));
                dg[10] += (unsigned long long)__popcll(__ballot(act && live && done));
            }
            if (!go) continue;
            const uint32_t j0 = X >> 5;
            const uint32_t d3 = ring[((j0 + 2u) & (kRing - 1u)) * kBlock];
            const uint32_t w = __builtin_amdgcn_alignbit(d0, d1, ~X);
            const uint32_t rem = Eb - X;
            uint32_t e1, e2, u1, u2, g1, g2;
            bool park, prog;
            if (HPK_LONG_TAILPT || (HPK_LONG_BODY && rem >= kBodyMin)) {
                // body step (lit12_body): every code of the two entries ends inside the literal
                e1 = s_lut[w >> (32 - HPK_LUT_BITS)];
                u1 = kTab == 3 ? HPK_L3_HELD(e1) : HPK_L2_HELD(e1);
                e2 = s_lut[(w << u1) >> (32 - HPK_LUT_BITS)];
                u2 = kTab == 3 ? HPK_L3_HELD(e2) : HPK_L2_HELD(e2);
                g1 = kTab == 3 ? HPK_L3_CODES(e1) : HPK_L2_CODES(e1);
                g2 = kTab == 3 ? HPK_L3_CODES(e2) : HPK_L2_CODES(e2);
                park = u2 == 0u;  // (> 12 bits left at e2: kBodyMin - 12)
                prog = true;
            } else {
                e1 = s_lut[w >> (32 - HPK_LUT_BITS)];
                bool a1, a2;
                u1 = lut12<kTab>(e1, rem, a1, a2);
                park = !a1 & (rem > (uint32_t)HPK_LUT_BITS);  // (see lit12_step)
                const bool cont = a1 & (a2 | lut_nottwo<kTab>(e1));
                const uint32_t w2 = w << u1;
                const uint32_t rem2 = rem - u1;
                e2 = s_lut[w2 >> (32 - HPK_LUT_BITS)];
                bool b1, b2;
                const uint32_t v2 = lut12<kTab>(e2, rem2, b1, b2);
                park |= cont & !b1 & (rem2 > (uint32_t)HPK_LUT_BITS);
                b1 &= cont;
                b2 &= cont;
                g1 = (uint32_t)a1 + (uint32_t)a2;
                g2 = (uint32_t)b1 + (uint32_t)b2;
                u2 = cont ? v2 : 0u;
                prog = a1 | park;
            }
            {  // the step's (up to 4) bytes as byte stores into the lane's own buffer (bytes past the
               // ones decoded are overwritten later or never stored out; one unaligned dword store
               // instead: config 3 936.7 vs 889.7 us, gfx950 splits it)
                uint8_t* const p = obuf + (ob - lb);
                p[0] = (uint8_t)e1;
                p[1] = (uint8_t)(e1 >> 16);
                p[g1] = (uint8_t)e2;
                p[g1 + 1] = (uint8_t)(e2 >> 16);
                ob += HPK_LONG_SPLIT && mode == kLead ? 0u : g1 + g2;  // (the lead-in: no output)
            }
            const uint32_t xn = X + u1 + u2;
            const bool cross = (xn ^ X) > 31u;
            d0 = cross ? d1 : d0;
            d1 = cross ? d2 : d1;
            d2 = cross ? d3 : d2;
            X = xn;
            if (park) {  // a 13..30-bit code or EOS: one leading-ones lookup
                const uint32_t wp = __builtin_amdgcn_alignbit(d0, d1, ~X);
                uint32_t sy, len;
                bool eos;
                lo_decode(wp, s_lo, sy, len, eos);
                if (len > Eb - X) {  // nothing fits in the > 12 bits left: huffman.rs:128-134
                    st = HPK_PADDING_TOO_LARGE;
                    prog = false;
                } else if (eos && !(HPK_LONG_SPLIT && mode == kLead)) {  // huffman.rs:112-116
                    st = HPK_EOS_IN_STRING;
                    prog = false;
                } else {  // (an EOS in a lead-in: a 30-bit code)
                    obuf[ob - lb] = (uint8_t)sy;
                    ob += HPK_LONG_SPLIT && mode == kLead ? 0u : 1u;
                    const uint32_t xp = X + len;  // (len <= 30: crosses at most one dword)
                    // the window re-read from the ring (a select from d3 or a fourth dword read beside
                    // the lookup instead: config 3 832-836 vs 817-822 us)
                    const uint32_t j = xp >> 5;
                    d0 = ring[((j - 1u) & (kRing - 1u)) * kBlock];
                    d1 = ring[(j & (kRing - 1u)) * kBlock];
                    d2 = ring[((j + 1u) & (kRing - 1u)) * kBlock];
                    X = xp;
                }
            }
            done = !prog;  // the literal has ended: finished at the next refill point
        }
        if (kDiag) dg[6] += __builtin_amdgcn_s_memtime() - dtp;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pin(gv[k].x);
            pin(gv[k].y);
            pin(gv[k].z);
            pin(gv[k].w);
            pin(hv[k]);
            pin(tv[k]);
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            pin(hb[e]);
            pin(tb[e]);
        }
        pin(lv);
        pin(sv);
        pin(ha);
        pin(ga);
        pin(ta);
        pin(ia);
        pin(ja);
    }
    if (kDiag) {
        dg[0] = __builtin_amdgcn_s_memtime() - dt0;
        const uint32_t gw = blockIdx.x * (uint32_t)(kBlock / 64) + wv;
        if (lane < 12) {
            unsigned long long v = 0;
#pragma unroll
            for (int i = 0; i < 12; ++i) v = lane == (uint32_t)i ? dg[i] : v;
            a.dbg[gw * 16u + lane] = v;
        }
    }
}

}  // namespace hpkdec
