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

// LPT class of a literal listed for this phase (which takes its list front to back): its encoded length in
// 128-byte classes, 0 the longest. The dense listings order their lists by it (a counting sort), so the
// longest literals start first (round 6: config 3 810 -> 635 us; the phase's length had been set by each
// workgroup's longest literal started late, 25 % of its lane-steps idle at the end).
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

#ifndef HPK_LONG_CH
#define HPK_LONG_CH 3  // 16-byte chunks a lane loads per refill point (round 6: 3, config 3 633.0-634.1 vs 641.7-642.4 us)
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

__device__ __forceinline__ uint32_t lpt_class_of(uint32_t nb) { return 31u - min(nb >> 7, 31u); }

template <int kBlock, int kU, int kRing, int kDiag, int kBlockAll, int kOSz = HPK_LONG_OS, int kClaim = 64,
          int kTab = 2,            // kTab: the layout of s_lut (2 = LUT2, the fill kernel; 3 = LUT3, the wave kernel)
          bool kCompact = false,   // the compacted mode: a claim takes its literals' decoded bounds from a.cursor
          int kCh = HPK_LONG_CH>   // 16-byte chunks loaded per lane and refill point
__device__ __forceinline__ void long_phase(const DecodeArgs& a, uint32_t ba, uint32_t bb, uint32_t c1, uint32_t c2,
                                           uint32_t* s_claim, uint32_t* s_ring, uint8_t* s_out, uint4* s_q,
                                           const uint32_t* s_lut, const uint16_t* s_lo) {
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
    // (HPK_LONG_TAILPT: a tail at the refill point adds <= 6 bytes: < kBodyMin bits, codes of >= 5 bits)
    static_assert(15 + 5 * kU + 3 + (HPK_LONG_TAILPT ? 6 : 0) < (int)kOS, "output buffer");
    static_assert((kRing & (kRing - 1)) == 0 && kRing >= 16 && 4 * kCh + 8 <= kRing, "input ring: a power of two >= 16 dwords");
    static_assert(kBlock % 64 == 0 && kBlock <= kBlockAll, "decoding waves");
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t total = c1 + c2;
    if (total == 0) return;  // (block-uniform: nothing left to this phase)
    if (tid >= (uint32_t)kBlock) return;  // (no barrier follows)
    uint4 (*sq)[kQ] = reinterpret_cast<uint4 (*)[kQ]>(s_q);
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
    uint32_t o0 = 0, ob = 0, fl = 0, lb = 0;
    u32x4 P[kCh] = {};  // the chunks loaded at the previous refill point
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
#pragma unroll
            for (int c = 0; c < kCh; ++c) {
                ring[((b + 4 * c + 0) & (kRing - 1u)) * kBlock] = __builtin_bswap32(P[c].x);
                ring[((b + 4 * c + 1) & (kRing - 1u)) * kBlock] = __builtin_bswap32(P[c].y);
                ring[((b + 4 * c + 2) & (kRing - 1u)) * kBlock] = __builtin_bswap32(P[c].z);
                ring[((b + 4 * c + 3) & (kRing - 1u)) * kBlock] = __builtin_bswap32(P[c].w);
            }
            h += 4u * kCh;
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
        // 4. a literal that ended in the last steps: padding check, last bytes, length, status
        if (done) {
            if (st == HPK_OK) st = residual_status(Eb - X, __builtin_amdgcn_alignbit(d0, d1, ~X));
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
            __builtin_amdgcn_raw_buffer_store_b32(lv, r_len, ia, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)sv, r_st, ja, 0, 0);
            act = false;
            live = false;
            done = false;
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
            }
            const uint32_t need = (uint32_t)__popcll(wm);
            const bool enough = need <= qt - qh;
            qh += min(need, qt - qh);
            if (enough || !more || claims == 2) break;  // (at most two claims per refill point)
            // claim the next 64 entries of this workgroup's list (an LDS counter)
            uint32_t rr = 0;
            if (lane == 0) rr = atomicAdd(s_claim, kChunk);
            const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)rr, 0);
            if (r >= total) {
                more = false;
                break;
            }
            // entries r + lane: [0, c1) from the front of the range, then from the back
            const uint32_t e = r + lane;
            const bool ok = lane < kChunk && e < total;
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
            const uint64_t lm = __ballot(ok);
            const uint32_t lr = __builtin_amdgcn_mbcnt_hi((uint32_t)(lm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lm, 0u));
            if (ok) sq[wv][(qt + lr) % kQ] = li;
            qt += (uint32_t)__popcll(lm);
        }
        if (kDiag) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            dg[5] += t - dtp;
            dtp = t;
        }
        if (!__any(act)) break;  // no literal left for this wave
        // 6. the next kCh chunks, while the ring has room for them past the window's first dword
        if (act && h * 4u < span && h + 4u * kCh + 1u <= kRing + (X >> 5)) {
#pragma unroll
            for (int c = 0; c < kCh; ++c)
                P[c] = __builtin_amdgcn_raw_buffer_load_b128(r_in, (q0 + (h >> 2)) * 16u + 16u * c, 0, 0);
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
            const bool go = (uint32_t)s < budget && !done && (!HPK_LONG_TAILPT || Eb - X >= kBodyMin);
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
                ob += g1 + g2;
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
                } else if (eos) {  // huffman.rs:112-116
                    st = HPK_EOS_IN_STRING;
                    prog = false;
                } else {
                    obuf[ob - lb] = (uint8_t)sy;
                    ob += 1u;
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
