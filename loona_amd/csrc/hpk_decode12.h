// hpk_decode12.h — the workgroup-fill decode kernel (decode v24; the v25 wave-fill kernel in
// hpk_wave.h is built on its lane walk) and the lane walk both kernels share.
//
// Per fill a 1024-thread workgroup holds in LDS an input window (big-endian dwords), an image of the
// fill's output span and a queue of up to 2048 literals sorted longest-first; the next fill's offsets
// and window are loaded into registers while the current one decodes (issued from the lane loop, a
// group per round, v23), the previous image is written back with 16-byte stores (its last round from
// the lane loop, v24). Lane i decodes queue slots i and 2 * 1024 - 1 - i (static snake, v13); lengths
// and statuses are made after the lane loop (v22). Literals of >= long_min encoded bytes go to the
// long-literal phase (hpk_long.h, v19).
//   * Lane walk (v12): a lane holds its bit position as X = P + 31 and the dword pair (d0, d1) =
//     window dwords (X >> 5) - 1 and X >> 5, plus the next dword d2. The 32 bits at P are ONE
//     v_alignbit_b32(d0, d1, ~X). A step does two lookups in the two-symbol table (LUT2 layout,
//     hpk_code.h), each decoding up to two codes of <= 12 bits, and advances <= 24 bits, so it crosses
//     at most one dword: the pair then slides by one (v_cndmask) and d2 takes d3, the dword read at the
//     top of the step. A code longer than 12 bits (EOS included) takes the rarely taken branch: one
//     leading-ones lookup. Bits past a literal's end are never masked: a code that runs past the end is,
//     by prefix-freeness, longer than what is left whatever follows, so the walk stops exactly where
//     huffman.rs's bit iterator stops matching (huffman.rs:100-123); the final padding check
//     (huffman.rs:128-160) looks at the residual bits only.
//   * Stores (v14): a step's (up to) four byte stores are unconditional, a byte that is not output
//     going to the lane's dummy slot (no exec-mask branch around each ds_write_b8).
// The variants measured along the way and not taken (whole-wave long literals, the segment stream,
// dynamic slots, dword stores, deferred write-back, ...) were timed in the round 1-3 harness
// (bench/legacy_decode12.h, removed in round 4; git history keeps it); DESIGN.md has their numbers.
#pragma once
#include "hpk_decode_kernel.h"

// Product settings of the fill kernel (each measured against its alternative):
// the next fill's prefetch issued from the lane loop (v23), the last write-back round stored from it
// (v24), workgroups' first fills staggered over 2 phases in ranges of >= 8 fills, lengths and
// statuses made after the lane loop (v22).
#define HPK_FLUSH_LOOP 1
#define HPK_PF_LOOP 1
#define HPK_STAGGER 1
#define HPK_STAGGER_PH 2
#define HPK_LATE_FIN 1
#ifndef HPK_FILL_BODY
#define HPK_FILL_BODY 1  // v28: body steps + two-at-once checked tails in the fill kernel too
#endif

namespace hpkdec {

// a dword and four dwords stored at any byte address (unaligned global stores: the compacted forms)
typedef uint32_t u32u __attribute__((aligned(1)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

// LDS carve-up: Geo7's regions plus a fifth counter (the long-literal queue head).
template <int kWaves, int kW, int kO, int kQ>
struct Geo12 : Geo7<kWaves, kW, kO, kQ, true> {
    using B = Geo7<kWaves, kW, kO, kQ, true>;
    static constexpr int kLdsBytes = B::kCtrOff + 48 + (int)kHugeMax * 4;  // counters, then the huge list
    static_assert(kLdsBytes <= 163840, "LDS budget (160 KiB per CU on gfx950)");
};

__device__ __forceinline__ void put8(uint8_t* __restrict__ out8, uint32_t pos, uint32_t v, uint32_t oend, int kStore) {
    if (kStore == kChecked) {
        if (pos < oend)
            out8[pos] = (uint8_t)v;
        else
            chk_report(1, pos, oend, 0);
    } else if (kStore == kDword || kStore == kPred) {
        out8[pos] = (uint8_t)v;
    } else {
        asm volatile("" ::"v"(v));
    }
}

// The 32 window bits at bit position p (big-endian dwords).
__device__ __forceinline__ uint32_t win_at(const uint32_t* __restrict__ win32, uint32_t p) {
    const uint32_t x = p + 31u;
    const uint32_t* q = win32 + (x >> 5);
    return __builtin_amdgcn_alignbit(q[-1], q[0], ~x);
}

// The codes one table entry decodes with rem bits left: ok1 / ok2 = its first / second code fits
// inside the literal; returns the bits they use.
template <int kTab = 2>  // the table layout: 2 = LUT2, 3 = LUT3 (hpk_code.h)
__device__ __forceinline__ uint32_t lut12(uint32_t e, uint32_t rem, bool& ok1, bool& ok2) {
    // a length field the entry does not hold is 15, past any clamped rem (and t1 >= l1: ok2 => ok1)
    const uint32_t rc = min(rem, HPK_LUT2_CLAMP);
    if (kTab == 3) {
        const uint32_t l1 = HPK_L3_LEN0(e), t1 = HPK_L3_HELD(e);
        ok1 = l1 <= rc;
        ok2 = (t1 <= rc) & (e < HPK_L3_NOTTWO);
        return ok2 ? t1 : (ok1 ? l1 : 0u);
    }
    const uint32_t l1 = HPK_L2_LEN0(e), t1 = HPK_L2_LEN01(e);
    ok1 = l1 <= rc;
    ok2 = t1 <= rc;
    return ok2 ? t1 : (ok1 ? l1 : 0u);
}
template <int kTab>
__device__ __forceinline__ bool lut_nottwo(uint32_t e) {
    return kTab == 3 ? e >= HPK_L3_NOTTWO : e >= HPK_LUT2_NOTTWO;
}
// An entry's second symbol byte, in place for a byte store (LUT2 / LUT3: [23:16])
template <int kTab>
__device__ __forceinline__ uint32_t lut_sym1(uint32_t e) {
    return e >> 16;
}

// The decoded bytes of an entry, packed little-endian and zero above the g = ok1 + ok2 of them.
__device__ __forceinline__ uint32_t lut12_bytes(uint32_t e, uint32_t g) {
    return __builtin_amdgcn_ubfe(__builtin_amdgcn_perm(e, e, 0x0C0C0200u), 0, 8u * g);
}

// Final status at a stop with rem residual bits and window w there (huffman.rs:128-160): at most
// 7 residual bits, all ones (the most significant bits of EOS).
__device__ __forceinline__ uint32_t residual_status(uint32_t rem, uint32_t w) {
    if (rem == 0) return HPK_OK;
    if (rem > 7) return HPK_PADDING_TOO_LARGE;
    return (w | (0xFFFFFFFFu >> rem)) != 0xFFFFFFFFu ? HPK_INVALID_PADDING : HPK_OK;
}

// ------------------------------------------------------------------------------------------
// Lane-per-literal walk.

struct Lit12 {
    uint32_t X;           // bit position in the window + 31
    uint32_t Eb;          // end bit position + 31: rem = Eb - X bits left
    uint32_t d0, d1, d2;  // window dwords (X >> 5) - 1, X >> 5, (X >> 5) + 1
    uint32_t o;           // next output byte in the LDS image
    uint32_t o0;          // first output byte of the literal
    uint32_t oend;        // checked mode: end of the literal's capacity
    uint32_t st;          // hpk_status set by the walk (EOS, or padding found by the long-code branch)
    uint32_t idx;         // literal index in the fill
    bool prog;            // the last step consumed a code or took the long-code branch
    bool more;            // (kMore steps) the walk may go on: the last step used both entries whole, or
                          // decoded a long code; false once a step has proved that no code fits
    bool act;             // holds a fast-path literal not yet finalised
};

// (Re)load the pair and the next dword at X.
__device__ __forceinline__ void lit12_load(Lit12& L, const uint32_t* __restrict__ win32) {
    const uint32_t* p = win32 + (L.X >> 5);
    L.d0 = p[-1];
    L.d1 = p[0];
    L.d2 = p[1];
}

// One step: two lookups (up to four codes of <= 12 bits) and, for a longer code, one leading-ones
// lookup. kStore == kPred: the (up to) four byte stores are unconditional, a byte that is not output
// going to the lane's dummy slot out8[dmy] (no exec-mask branch around each store); kChecked
// (diagnostic mode 4) checks every store against the literal's capacity, kNoStore (mode 2) stores
// nothing.
// (lit12_step's two parts: the lookups and their stores, returning whether a 13..30-bit code or EOS
// starts at the new position; then that code's leading-ones lookup. on = false: the step does nothing
// — no advance, its stores to the dummy slot — so two literals' steps can share one block, lit12_step2.)
template <int kStore, bool kP1, int kTab, bool kMore>
__device__ __forceinline__ bool lit12_step_main(Lit12& L, const uint32_t* __restrict__ win32,
                                                const uint32_t* __restrict__ lut, uint8_t* __restrict__ out8,
                                                uint32_t dmy, bool on = true) {
    const uint32_t d3 = win32[(L.X >> 5) + 2];  // the dword after d2, in case this step crosses one
    const uint32_t w = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
    const uint32_t rem = L.Eb - L.X;
    const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
    bool a1, a2;
    uint32_t u1 = lut12<kTab>(e1, rem, a1, a2);
    a1 &= on;
    a2 &= on;
    u1 = on ? u1 : 0u;
    uint32_t use = u1;
    // a code longer than 12 bits (or EOS) starts here and may still fit (with more than 12 bits
    // left, any code the entry holds fits: no first code <=> the entry has none)
    bool park = on & !a1 & (rem > (uint32_t)HPK_LUT_BITS);
    bool more2 = false;
    if (kStore == kPred) {
        out8[a1 ? L.o : dmy] = (uint8_t)e1;
        if (kP1)
            (out8 + 1)[a2 ? L.o : dmy - 1u] = (uint8_t)lut_sym1<kTab>(e1);
        else
            out8[a2 ? L.o + 1 : dmy] = (uint8_t)lut_sym1<kTab>(e1);
    } else {
        if (a1) put8(out8, L.o, e1, L.oend, kStore);
        if (a2) put8(out8, L.o + 1, lut_sym1<kTab>(e1), L.oend, kStore);
    }
    L.o += (uint32_t)a1 + (uint32_t)a2;
    {
        // the first entry was consumed whole: look the next bits up too
        const bool cont = a1 & (a2 | lut_nottwo<kTab>(e1));
        const uint32_t w2 = w << u1;
        const uint32_t rem2 = rem - u1;
        const uint32_t e2 = lut[w2 >> (32 - HPK_LUT_BITS)];
        bool b1, b2;
        const uint32_t u2 = lut12<kTab>(e2, rem2, b1, b2);
        park |= cont & !b1 & (rem2 > (uint32_t)HPK_LUT_BITS);
        b1 &= cont;
        b2 &= cont;
        // both entries used whole: more codes may follow (otherwise one of them held a code that does
        // not fit, or none with <= 12 bits left: the walk has ended here, huffman.rs:100-123)
        more2 = b1 & (b2 | lut_nottwo<kTab>(e2));
        if (kStore == kPred) {
            out8[b1 ? L.o : dmy] = (uint8_t)e2;
            if (kP1)
                (out8 + 1)[b2 ? L.o : dmy - 1u] = (uint8_t)lut_sym1<kTab>(e2);
            else
                out8[b2 ? L.o + 1 : dmy] = (uint8_t)lut_sym1<kTab>(e2);
        } else {
            if (b1) put8(out8, L.o, e2, L.oend, kStore);
            if (b2) put8(out8, L.o + 1, lut_sym1<kTab>(e2), L.oend, kStore);
        }
        L.o += (uint32_t)b1 + (uint32_t)b2;
        use += cont ? u2 : 0u;
    }
    const uint32_t xn = L.X + use;
    const bool cross = (xn ^ L.X) > 31u;
    L.d0 = cross ? L.d1 : L.d0;
    L.d1 = cross ? L.d2 : L.d1;
    L.d2 = cross ? d3 : L.d2;
    L.X = xn;
    L.prog = a1 | park;
    if (kMore) L.more = park | more2;
    return park;
}

template <int kStore, bool kMore>
__device__ __forceinline__ void lit12_park(Lit12& L, const uint32_t* __restrict__ win32, const uint16_t* __restrict__ lo,
                                           uint8_t* __restrict__ out8) {
    // a 13..30-bit code or EOS: one leading-ones lookup (any code in one read)
    const uint32_t wp = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
    uint32_t s, len;
    bool eos;
    lo_decode(wp, lo, s, len, eos);
    const uint32_t r = L.Eb - L.X;
    if (len > r) {  // nothing fits in the > 12 bits left: huffman.rs:128-134
        L.st = HPK_PADDING_TOO_LARGE;
        L.Eb = L.X;
        if (kMore) L.more = false;
    } else if (eos) {  // huffman.rs:112-116
        L.st = HPK_EOS_IN_STRING;
        L.Eb = L.X;
        if (kMore) L.more = false;
    } else {
        put8(out8, L.o, s, L.oend, kStore);
        L.o += 1;
        L.X += len;
        lit12_load(L, win32);
    }
}

// One step: two lookups (up to four codes of <= 12 bits) and, for a longer code, one leading-ones
// lookup. kStore == kPred: the (up to) four byte stores are unconditional, a byte that is not output
// going to the lane's dummy slot out8[dmy] (no exec-mask branch around each store); kChecked
// (diagnostic mode 4) checks every store against the literal's capacity, kNoStore (mode 2) stores
// nothing.
template <int kStore, bool kP1 = false,   // kP1: a lookup's second byte stored at (address) + 1 by the
          int kTab = 2,                  // store's offset (the wave kernel; in the fill kernel's
          bool kMore = false>            // register budget the extra live dmy - 1 spills); kTab: lut12;
                                         // kMore: set L.more (the tails of decode v27)
__device__ __forceinline__ void lit12_step(Lit12& L, const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                           const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8,
                                           uint32_t dmy = 0) {
    if (lit12_step_main<kStore, kP1, kTab, kMore>(L, win32, lut, out8, dmy)) lit12_park<kStore, kMore>(L, win32, lo, out8);
}

// Body step (decode v27): the same two lookups with NO fit tests, for a literal with at least
// kBodyMin bits left before the step. A step consumes <= 24 bits, so every code the two entries hold
// ends inside the literal, and >= 13 bits are left after it. The stores are unconditional at the
// lane's own output positions: an entry's second byte when it holds one code (or both bytes when it
// holds none) is garbage that the next store overwrites, or lies past the decoded bytes inside the
// literal's own region (see kBodyMin). Lengths come from the entries' "bits held" and "codes held" fields: ~25 VALU per
// step against lit12_step's ~48. A lookup that holds no code (a 13..30-bit code or EOS) takes the
// checked leading-ones branch of lit12_step; `body` says whether the next step may be a body step.
#ifndef HPK_BODY_MIN
#define HPK_BODY_MIN 29
#endif
// 24 bits a step may consume + 5: after a body step >= 5 bits are left, so when the decoded bytes end
// there the decoded length is below the bound (a code is >= 5 bits) and a garbage byte at the next
// output position stays in the region; a lookup holding no code has >= 29 - 12 > 12 bits left, so it
// always takes the leading-ones branch (whose symbol overwrites the garbage)
constexpr uint32_t kBodyMin = HPK_BODY_MIN;

// kDup (diagnostic builds, LDS bank-conflict attribution): one access class of the step issued twice,
// the extra access a volatile one through an LDS-qualified pointer (a volatile access through a generic
// pointer became a flat access, and a later plain store to the same byte let the compiler drop the
// earlier one): 1 the two table reads, 2 the window read, 3 the four byte stores (the same bytes, the
// duplicate first). The conflict cycles a variant adds over the product are that class's.
#ifndef HPK_LDS_AS
#define HPK_LDS_AS __attribute__((address_space(3)))
#endif
#ifndef HPK_LAZY_D3
#define HPK_LAZY_D3 0  // 1: the window dword after d2 read only by the lanes whose step crossed a dword (round 5:
                       // config 5 781-789 vs 769-783 us, profiles/r05/ab_lazy_window_read_rejected.jsonl)
#endif
template <int kStore, int kTab = 2, int kDup = 0>
__device__ __forceinline__ void lit12_body(Lit12& L, const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                           const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8, bool& body) {
    const uint32_t d3 = HPK_LAZY_D3 ? 0u : win32[(L.X >> 5) + 2];
    if (kDup == 2) asm volatile("" ::"v"(((const volatile HPK_LDS_AS uint32_t*)win32)[(L.X >> 5) + 2]));
    const uint32_t w = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
    const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
    const uint32_t u1 = kTab == 3 ? HPK_L3_HELD(e1) : HPK_L2_HELD(e1);
    const uint32_t e2 = lut[(w << u1) >> (32 - HPK_LUT_BITS)];
    if (kDup == 1) {
        const volatile HPK_LDS_AS uint32_t* vl = (const volatile HPK_LDS_AS uint32_t*)lut;
        asm volatile("" ::"v"(vl[w >> (32 - HPK_LUT_BITS)]));
        asm volatile("" ::"v"(vl[(w << u1) >> (32 - HPK_LUT_BITS)]));
    }
    const uint32_t u2 = kTab == 3 ? HPK_L3_HELD(e2) : HPK_L2_HELD(e2);
    const uint32_t o1 = L.o + (kTab == 3 ? HPK_L3_CODES(e1) : HPK_L2_CODES(e1));
    if (kStore != kNoStore) {
        if (kDup == 3) {
            volatile HPK_LDS_AS uint8_t* v8 = (volatile HPK_LDS_AS uint8_t*)out8;
            v8[L.o] = (uint8_t)e1;
            (v8 + 1)[L.o] = (uint8_t)lut_sym1<kTab>(e1);
            v8[o1] = (uint8_t)e2;
            (v8 + 1)[o1] = (uint8_t)lut_sym1<kTab>(e2);
        }
        out8[L.o] = (uint8_t)e1;
        (out8 + 1)[L.o] = (uint8_t)lut_sym1<kTab>(e1);
        out8[o1] = (uint8_t)e2;
        (out8 + 1)[o1] = (uint8_t)lut_sym1<kTab>(e2);
    }
    L.o = o1 + (kTab == 3 ? HPK_L3_CODES(e2) : HPK_L2_CODES(e2));
    const uint32_t xn = L.X + u1 + u2;
    const bool cross = (xn ^ L.X) > 31u;
    L.d0 = cross ? L.d1 : L.d0;
    L.d1 = cross ? L.d2 : L.d1;
    if (HPK_LAZY_D3) {
        if (cross) L.d2 = win32[(xn >> 5) + 1u];
    } else {
        L.d2 = cross ? d3 : L.d2;
    }
    L.X = xn;
    if (u2 == 0u) {  // e2 holds no code (nor e1, if u1 == 0): a 13..30-bit code or EOS at X; > 12 bits are
                     // left (>= kBodyMin - 12 before this lookup), so the leading-ones branch of lit12_step applies
        const uint32_t wp = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
        uint32_t sy, len;
        bool eos;
        lo_decode(wp, lo, sy, len, eos);
        const uint32_t r = L.Eb - L.X;
        if (len > r) {  // nothing fits in the > 12 bits left: huffman.rs:128-134
            L.st = HPK_PADDING_TOO_LARGE;
            L.Eb = L.X;
        } else if (eos) {  // huffman.rs:112-116
            L.st = HPK_EOS_IN_STRING;
            L.Eb = L.X;
        } else {
            if (kStore != kNoStore) out8[L.o] = (uint8_t)sy;
            L.o += 1;
            L.X += len;
            lit12_load(L, win32);
        }
    }
    body = L.Eb - L.X >= kBodyMin;
}

// Final status of a literal whose walk has stopped; a status set by the walk wins.
__device__ __forceinline__ uint32_t lit12_status(const Lit12& L) {
    if (L.st != HPK_OK) return L.st;
    return residual_status(L.Eb - L.X, __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X));
}

}  // namespace hpkdec

#include "hpk_long.h"  // the long-literal phase
#include "hpk_huge.h"  // the huge-literal phase

namespace hpkdec {

// ------------------------------------------------------------------------------------------

// kMode: 0 product; diagnostics (libhpk_diag.so only, never the product library): 1 no decode (fill
// structure only), 2 no output stores, 3 product + 16 per-wave stamps in a.dbg (cycles: total, in
// the decode loop, steps, waiting at the fill-top barrier, before the first fill, fill setup up to
// the entries, fill setup from there to the decode, -, the first fill's two setup parts, the byte
// pass, the last write-back, setup B to the window, to the prefetch, to the write-back issue),
// 4 checked stores (g_chk), 5 product + per-wave counters of the long-literal phase in a.dbg.
// kCompact: the compacted-output mode (hpk_decode_batch_compact): a.out_off is the library's own
// bound layout of the fills' images; every fill, once decoded, takes its decoded total from the device
// cursor and writes its literals' bytes there back to back (compact_flush), with their offsets in
// a.co_off; a listed (huge / long) literal takes its decoded bound when its phase starts it (a
// literal can be listed twice: a fill whose setup is redone lists its long literals again).
constexpr uint32_t kListed = 0xFFFFFFFFu;  // (kCompact) s_lenst mark of a literal listed, not decoded by its fill
template <int kMode, int kWaves, int kW, int kO, int kQ, int kRefillN, bool kCompact = false>
__global__ __launch_bounds__(kWaves * 64) void hpk_decode12(DecodeArgs a) {
    using G = Geo12<kWaves, kW, kO, kQ>;
    constexpr int R = G::kMetaRounds, S = G::kStageRounds;
    constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : kPred);
    // v22: lengths and statuses of the lane literals made after the lane loop (HPK_LATE_FIN)
    constexpr bool kLate = HPK_LATE_FIN && kStore == kPred;
    // the next fill's prefetch issued from the lane loop, a load per round (HPK_PF_LOOP)
    constexpr bool kPfLoop = HPK_PF_LOOP && kLate;
    // HPK_FLUSH_LOOP: the previous fill's last S write-back rounds are read into the window-prefetch
    // registers (free once the window is in LDS) and stored from the lane loop, before the window's
    // prefetch loads reuse those registers
    constexpr int kFD = kPfLoop && !kCompact ? (HPK_FLUSH_LOOP < S ? HPK_FLUSH_LOOP : S) : 0;
    // groups of one fill prefetch: a round of offsets each, the deferred write-back rounds, the window
    constexpr int kPfN = R + kFD + 1;
    // kPred: the image's last 256 bytes are the lanes' dummy slots (one dword apart), not output
    constexpr int kImg = kStore == kPred ? kO - 256 : kO;
    const uint32_t dmy = (uint32_t)kImg + (threadIdx.x & 63u) * 4u;
    unsigned long long t_start = 0, t_dec = 0, n_steps = 0, n_fills = 0, t_pre = 0, t_setA = 0, t_setB = 0,
                       t_A0 = 0, t_B0 = 0, t_tail = 0, t_byte = 0, t_sb1 = 0, t_sb2 = 0, t_sb3 = 0;
    if (kMode == 3) t_start = __builtin_amdgcn_s_memtime();
    __shared__ __attribute__((aligned(16))) uint8_t smem[G::kLdsBytes];
    uint16_t* s_lo = reinterpret_cast<uint16_t*>(smem + kT8Bytes);
    uint32_t* s_lut = reinterpret_cast<uint32_t*>(smem + G::kLutOff);
    uint8_t* s_in = smem + G::kInOff;
    const uint32_t* win32 = reinterpret_cast<const uint32_t*>(s_in);
    uint8_t* s_out = smem + G::kOutOff;
    uint2* s_q = reinterpret_cast<uint2*>(smem + G::kQOff);
    uint32_t* s_lenst = reinterpret_cast<uint32_t*>(smem + G::kLenOff);  // len | status << 24
    uint32_t* s_hist = reinterpret_cast<uint32_t*>(smem + G::kHistOff);
    uint32_t* s_bbase = s_hist + 64;
    // [0] fitting count, [1] lane-queue head, [2] input end of the fill, [3] output end of the
    // fill, [4] long-queue head, ... [11] huge literals listed (s_huge = s_ctr + 12; hpk_huge.h)
    uint32_t* s_ctr = reinterpret_cast<uint32_t*>(smem + G::kCtrOff);
    uint32_t* s_huge = s_ctr + 12;
    for (uint32_t t = threadIdx.x; t < kLoBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];
    for (uint32_t t = threadIdx.x; t < (uint32_t)G::kLutBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lut)[t] = reinterpret_cast<const uint4*>(a.lut2)[t];

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    // (byte-balanced workgroup ranges, hpk_split.h, gained nothing here: DESIGN.md §5)
    const uint32_t BA = (uint32_t)((uint64_t)a.n * blockIdx.x / gridDim.x);
    const uint32_t BB = (uint32_t)((uint64_t)a.n * (blockIdx.x + 1) / gridDim.x);
    // offsets are clamped to the input capacity wherever they bound a read, so bad offsets (caught
    // per fill below) never move a window past the blob
    const uint32_t in_end = min(a.in_off[a.n], a.in_cap) + a.in_mis;
    const uint32_t last16 = in_end ? (in_end - 1) >> 4 : 0;  // last 16-B chunk holding a batch byte
    // last chunk holding a byte of THIS workgroup's literals: windows never read past it
    const uint32_t r_end = min(min(a.in_off[BB], a.in_cap) + a.in_mis, in_end);
    const uint32_t rlast16 = r_end ? (r_end - 1) >> 4 : 0;
    // the range is cut into the fewest fills the window allows, of about equal input size (v16: a
    // greedy cut leaves a small last fill that still costs a whole fill's setup, slowest literal and
    // write-back); the effective window is that size plus a margin for literal granularity
    uint32_t kWe = (uint32_t)kW;
    uint32_t kW0 = kWe;  // the first fill's window
    {
        const uint32_t R = r_end - min((min(a.in_off[BA], a.in_cap) + a.in_mis) & ~15u, r_end);
        const uint32_t nf = (R + (uint32_t)kW - 1u) / (uint32_t)kW;
        if (nf > 1u) kWe = min((uint32_t)kW, (R + nf - 1u) / nf + 512u);
        // HPK_STAGGER: in a range of many fills, workgroup b's first fill is (b % PH) / PH of a window
        // (a whole one for b % PH = 0), so the workgroups' write-back and prefetch bursts (~35 MB over
        // the chip at once when all fills run in step) alternate instead of coinciding (config 5
        // +0.7 % with PH = 2, +0.4 % with 4; a range of a few fills would pay a whole extra fill)
        const uint32_t ph = blockIdx.x % (uint32_t)HPK_STAGGER_PH;
        if (HPK_STAGGER && nf >= 8u && ph) kW0 = kWe * ph / (uint32_t)HPK_STAGGER_PH;
    }

    // write back one decoded fill from the LDS image: the output span [G0, G1) with 16-byte
    // stores (bytewise in the two end chunks, which neighbours own), then out_len and status
    auto flush = [&](uint32_t fcur, uint32_t fk, uint32_t G0, uint32_t G1) {
        const uint32_t ob = G0 & ~15u;
        if (kMode != 2) {
            const uint32_t c0 = ob >> 4, c1 = (G1 + 15) >> 4;
            const uint4* l16 = reinterpret_cast<const uint4*>(s_out);
            uint4* g16 = reinterpret_cast<uint4*>(a.out_base);
#pragma unroll
            for (int r = 0; r < G::kFlushRounds; ++r) {
                const uint32_t ci = c0 + tid + (uint32_t)G::kBlock * r;
                if (ci < c1 && (ci << 4) >= G0 && (ci << 4) + 16u <= G1) g16[ci] = l16[ci - c0];
            }
            if (tid < 32) {  // the partial chunks at the two ends, one byte per lane
                const uint32_t g = tid < 16 ? c0 << 4 : (c1 - 1) << 4;
                const bool partial = !(g >= G0 && g + 16u <= G1) && (tid < 16 || c1 - 1 != c0);
                const uint32_t x = g + (tid & 15u);
                if (partial && x >= G0 && x < G1) a.out_base[x] = s_out[x - ob];
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t i = tid + (uint32_t)G::kBlock * r;
            if (i < fk) {
                const uint32_t v = s_lenst[i];
                a.out_len[fcur + i] = v & 0xFFFFFFu;
                a.status[fcur + i] = (uint8_t)(v >> 24);
            }
        }
    };
    uint32_t pk = 0, pcur = 0, pG0 = 0, pG1 = 0;  // the previous fill, not yet written back
    uint32_t fd_c0 = 0, fd_mask = 0;  // kFD: first image chunk of the deferred rounds' fill, rounds holding data
    Prefetch<R, S> P;
    // kFD: the write-back with its last kFD rounds read into P.chunk (stored by pf_part)
    auto flush_split = [&](uint32_t fcur, uint32_t fk, uint32_t G0, uint32_t G1) {
        const uint32_t ob = G0 & ~15u;
        const uint32_t c0 = ob >> 4, c1 = (G1 + 15) >> 4;
        const uint4* l16 = reinterpret_cast<const uint4*>(s_out);
        uint4* g16 = reinterpret_cast<uint4*>(a.out_base);
        fd_c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)c0);
        fd_mask = 0;
#pragma unroll
        for (int r = 0; r < G::kFlushRounds; ++r) {
            const uint32_t ci = c0 + tid + (uint32_t)G::kBlock * r;
            const bool ok = ci < c1 && (ci << 4) >= G0 && (ci << 4) + 16u <= G1;
            if (r < G::kFlushRounds - kFD) {
                if (ok) g16[ci] = l16[ci - c0];
            } else if (kFD) {
                const int d = r - (G::kFlushRounds - kFD);
                if (ok) {
                    P.chunk[d < S ? d : 0] = l16[ci - c0];
                    fd_mask |= 1u << d;
                }
            }
        }
        if (tid < 32) {  // the partial chunks at the two ends, one byte per lane
            const uint32_t g = tid < 16 ? c0 << 4 : (c1 - 1) << 4;
            const bool partial = !(g >= G0 && g + 16u <= G1) && (tid < 16 || c1 - 1 != c0);
            const uint32_t x = g + (tid & 15u);
            if (partial && x >= G0 && x < G1) a.out_base[x] = s_out[x - ob];
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t i = tid + (uint32_t)G::kBlock * r;
            if (i < fk) {
                const uint32_t v = s_lenst[i];
                a.out_len[fcur + i] = v & 0xFFFFFFu;
                a.status[fcur + i] = (uint8_t)(v >> 24);
            }
        }
    };
    // kCompact: the decoded fill [fcur, fcur + fk) written back compacted (its kq queue entries give the
    // decoded literals' image offsets, written by literal into the window, free once the fill is
    // decoded): a block scan of the lengths in literal order, ONE cursor add for the fill's total, then
    // each thread stores its literals' bytes (round 5: unaligned 16-byte pieces, as the wave kernel's
    // compact_fill; the round-4 per-chunk gather measured 97 us on config 2 against 90-91), lengths,
    // statuses and offsets. Listed literals (kListed) are 0 bytes here.
#ifndef HPK_COMPACT_NOCOPY
#define HPK_COMPACT_NOCOPY 0  // (measurement only: no copy, no lengths)
#endif
    auto compact_flush = [&](uint32_t fcur, uint32_t fk, uint32_t kqc) {
        lds_barrier();  // every length and status of the fill is in s_lenst; the window is free
        uint32_t* const s_iof = reinterpret_cast<uint32_t*>(s_in);  // [kQ] image offsets by literal
        static_assert(kQ * 4 <= kW, "compacted write-back table in the window");
#pragma unroll
        for (int r = 0; r < R; ++r) {  // the image offsets, from the queue (still intact)
            const uint32_t q = tid + (uint32_t)G::kBlock * r;
            if (q < kqc) {
                const uint2 e = s_q[q];
                s_iof[e.y & 0xFFFu] = (e.y >> 12) & 0x1FFFFu;
            }
        }
        const uint32_t wv = tid >> 6;
        uint32_t lst[R], exs[R];
        uint32_t carry = 0;
        auto lenof = [](uint32_t v) { return v == kListed ? 0u : v & 0xFFFFFFu; };
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = tid + (uint32_t)G::kBlock * r;
            lst[r] = t < fk ? s_lenst[t] : kListed;
            uint32_t x = lenof(lst[r]);
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (lane >= (uint32_t)d) x += y;
            }
            if (lane == 63u) s_hist[wv] = x;
            lds_barrier();
            uint32_t pre = 0, tot = 0;
            for (uint32_t q = 0; q < (uint32_t)kWaves; ++q) {
                const uint32_t v = s_hist[q];
                pre += q < wv ? v : 0u;
                tot += v;
            }
            exs[r] = carry + pre + x - lenof(lst[r]);
            carry += tot;
            lds_barrier();  // (s_hist again in the next round)
        }
        if (tid == 0) s_hist[32] = atomicAdd(a.cursor, carry);
        lds_barrier();
        const uint32_t base = s_hist[32];
        const uint32_t D0 = a.out_mis + base;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = tid + (uint32_t)G::kBlock * r;
            if (t < fk && lst[r] != kListed && !HPK_COMPACT_NOCOPY) {
                a.co_off[fcur + t] = base + exs[r];
                a.out_len[fcur + t] = lenof(lst[r]);
                a.status[fcur + t] = (uint8_t)(lst[r] >> 24);
            }
        }
        const uint32_t* const img32 = reinterpret_cast<const uint32_t*>(s_out);
        // (round 5, as the wave kernel's compact_fill) each thread stores literals tid and tid + kBlock
        // from the image in 16-byte pieces at any byte address, a literal's last piece ending at its
        // last byte; 4..15 bytes in dwords the same way, fewer bytewise
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = tid + (uint32_t)G::kBlock * r;
            const uint32_t np = t < fk && !HPK_COMPACT_NOCOPY ? lenof(lst[r]) : 0u;
            const uint32_t sp = np ? s_iof[t] : 0u, dp = D0 + exs[r];
            auto dw_at = [&](uint32_t u) {
                return __builtin_amdgcn_alignbyte(img32[(u >> 2) + 1u], img32[u >> 2], u & 3u);
            };
            if (np >= 16u) {
                for (uint32_t tp = 0; tp < np; tp += 16u) {
                    const uint32_t tt = min(tp, np - 16u), u = sp + tt, sw = u >> 2, s3 = u & 3u;
                    uint32_t A[5];
#pragma unroll
                    for (int j = 0; j < 5; ++j) A[j] = img32[sw + (uint32_t)j];
                    u32x4u v;
                    v.x = __builtin_amdgcn_alignbyte(A[1], A[0], s3);
                    v.y = __builtin_amdgcn_alignbyte(A[2], A[1], s3);
                    v.z = __builtin_amdgcn_alignbyte(A[3], A[2], s3);
                    v.w = __builtin_amdgcn_alignbyte(A[4], A[3], s3);
                    *reinterpret_cast<u32x4u*>(a.out_base + dp + tt) = v;
                }
            } else if (np >= 4u) {
                u32u* const g = reinterpret_cast<u32u*>(a.out_base + dp);
                g[0] = dw_at(sp);
                if (np >= 8u) g[1] = dw_at(sp + 4u);
                if (np >= 12u) g[2] = dw_at(sp + 8u);
                *reinterpret_cast<u32u*>(a.out_base + dp + np - 4u) = dw_at(sp + np - 4u);
            } else {
                for (uint32_t b = 0; b < np; ++b) a.out_base[dp + b] = s_out[sp + b];
            }
        }
    };
    // long literals left to the long-literal phase are listed in a.long_list[BA, BB): those of
    // >= long_big encoded bytes from the front, the others from the back (counts in s_ctr[6], [7])
    auto leave = [&](uint32_t i, uint32_t nb) {
        if (nb >= HPK_HUGE_MIN && nb < kHugeLimit) {  // huge literals: the huge-literal phase's (hpk_huge.h)
            const uint32_t h = atomicAdd(&s_ctr[11], 1u);
            if (h < kHugeMax) {
                s_huge[h] = i;
                return;
            }
        }
        if (nb >= a.long_big)
            a.long_list[BA + atomicAdd(&s_ctr[6], 1u)] = i;
        else
            a.long_list[BB - 1u - atomicAdd(&s_ctr[7], 1u)] = i;
    };
    if (tid == 0) {
        s_ctr[6] = 0;
        s_ctr[7] = 0;
        s_ctr[8] = 0;
        s_ctr[9] = 0;
        s_ctr[11] = 0;
    }

    uint32_t cur = BA;
    uint32_t gin = 0, gout = 0;  // exact input / output start of the fill (blob-relative + mis)
    if (cur < BB) {
        gin = a.in_off[cur] + a.in_mis;
        gout = a.out_off[cur] + a.out_mis;
        prefetch_fill<G::kBlock>(P, a, tid, cur, min(cur + (uint32_t)kQ, BB), gin & ~15u, rlast16);
    }
    if (kMode == 3) t_pre = __builtin_amdgcn_s_memtime() - t_start;
    bool dense_tried = false;  // block-uniform: the range's first fill was checked
    while (cur < BB) {  // block-uniform
        const uint32_t cntl = min((uint32_t)kQ, BB - cur);
        const uint32_t kWf = cur == BA ? kW0 : kWe;
        const uint32_t base16 = gin & ~15u;
        const uint32_t ob16 = gout & ~15u;
        unsigned long long tb0 = 0;
        if (kMode == 3) tb0 = __builtin_amdgcn_s_memtime();
        lds_barrier();  // previous fill decoded and its image read out: every LDS region is free
        if (kMode == 3) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            n_fills += t1 - tb0;  // (mode 3: barrier wait)
            tb0 = t1;
        }
        // the long-list counts before this fill (nothing changes them until the setup below): a fill
        // found bad takes back what its own literals listed
        const uint32_t lcnt6 = s_ctr[6], lcnt7 = s_ctr[7], lcnt11 = s_ctr[11];
        if (tid < 64) s_hist[tid] = 0;
        if (tid == 0) {
            s_ctr[0] = 0;
            s_ctr[1] = G::kBlock;  // lane-queue slots handed out at the start
            s_ctr[2] = gin;
            s_ctr[3] = gout;
            s_ctr[4] = 0;
            s_ctr[5] = 0;
        }
        lds_barrier();
        uint32_t ex[R], ey[R], pos[R];
        uint32_t kw = 0;
        uint32_t dlb = 0, dtb = 0;  // (first fill) long-literal bytes and all bytes of the candidates
        bool bad = false;  // a literal of this fill's range with decreasing offsets or offsets past a capacity
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = tid + (uint32_t)G::kBlock * r;
            if (!dense_tried) {
                const uint32_t nb = min(P.io1[r] - P.io0[r], 1u << 20);  // (bad offsets: bounded)
                dtb += t < cntl ? nb : 0u;
                dlb += t < cntl && nb >= a.long_min ? nb : 0u;
            }
            bad |= t < cntl && !(P.io0[r] <= P.io1[r] && P.io1[r] <= a.in_cap && P.oo0[r] <= P.oo1[r] &&
                                 P.oo1[r] <= a.out_cap);
            const uint32_t p0 = P.io0[r] + a.in_mis, p1 = P.io1[r] + a.in_mis;
            const uint32_t o0 = P.oo0[r] + a.out_mis, o1 = P.oo1[r] + a.out_mis;
            // fitting literals form a prefix (offsets are non-decreasing)
            const bool fits = !bad && t < cntl && p1 - base16 <= kWf && o1 - ob16 <= (uint32_t)kImg;
            pos[r] = 0xFFFFFFFFu;
            if (fits) {
                const uint32_t nbytes = p1 - p0, ocap = o1 - o0;
                // fast path: a region holding hpk_decoded_bound(nbytes) bytes (dword-aligned in
                // start and size for the dword stores, which write up to 3 bytes past the end)
                const bool fast = ocap >= (nbytes * 8u) / 5u;
                ex[r] = (p0 - base16) | (nbytes << 16);
                ey[r] = t | ((o0 - ob16) << 12) | (fast ? 0u : kQ7Byte);
                if (fast && nbytes >= a.long_min) {  // the long-literal phase's (not queued here)
                    leave(cur + t, nbytes);
                    if (kCompact) s_lenst[t] = kListed;
                } else {
                    const uint32_t bk = lpt_bucket(nbytes);
                    pos[r] = (bk << 16) | atomicAdd(&s_hist[bk], 1u);
                }
            }
            const uint64_t fb = __ballot(fits);
            kw += (uint32_t)__popcll(fb);
            if (fb) {  // the wave's last fitting literal ends furthest (offsets non-decreasing)
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
        if (__any(bad) && lane == 0) s_ctr[5] = 1u;
        if (!dense_tried) {
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
                dlb += __shfl_xor(dlb, d);
                dtb += __shfl_xor(dtb, d);
            }
            if (lane == 0) {
                atomicAdd(&s_ctr[8], dlb);
                atomicAdd(&s_ctr[9], dtb);
            }
        }
        lds_barrier();
        if (kMode == 3) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            t_setA += t1 - tb0;  // (mode 3: offsets in, entries made)
            if (cur == BA) t_A0 = t1 - tb0;
            tb0 = t1;
        }
        if (s_ctr[5]) {  // bad offsets (block-uniform): the range's remaining literals are void, nothing
                         // more is decoded or written here (the previous, valid fill is flushed below)
            for (uint32_t i = cur + tid; i < BB; i += G::kBlock) {
                a.out_len[i] = 0;
                a.status[i] = (uint8_t)HPK_BAD_OFFSETS;
            }
            if (tid == 0) {
                *a.err = 1u;
                s_ctr[6] = lcnt6;  // this fill's long literals are void too: not for the long-literal phase
                s_ctr[7] = lcnt7;
                s_ctr[11] = lcnt11;
            }
            break;
        }
        if (!dense_tried) {
            // A range whose first fill's literals hold mostly long-literal bytes (config 3: Zipf
            // lengths) goes to the long-literal phase whole: here every fill would stream the long
            // literals' bytes through the window only to skip them, and wait for its longest short
            // literal. All of the range's literals are listed (validated: offsets in bounds, regions
            // >= the decoded bound); if any is not, the range is decoded by fills after all.
            dense_tried = true;
            if (s_ctr[8] > s_ctr[9] / 2u) {  // block-uniform
                lds_barrier();
                if (tid == 0) {
                    s_ctr[6] = 0;  // (this fill's entries are listed again below)
                    s_ctr[7] = 0;
                    s_ctr[11] = 0;
                    s_ctr[10] = 0;
                }
                if (tid < 64) s_hist[tid] = 0;  // (round 6) LPT classes: counts [0, 32), then cursors
                lds_barrier();
                // round 6: the list in LPT order (lpt_class_of, longest first) by a counting sort: the long phase
                // takes it front to back, so the longest jobs start first; huge literals to the huge list
                bool no = false;
                for (uint32_t i = BA + tid; i < BB; i += G::kBlock) {
                    const uint32_t p0 = a.in_off[i], p1 = a.in_off[i + 1], q0 = a.out_off[i], q1 = a.out_off[i + 1];
                    const bool ok = p0 <= p1 && p1 <= a.in_cap && q0 <= q1 && q1 <= a.out_cap &&
                                    (uint64_t)(q1 - q0) >= (uint64_t)(p1 - p0) * 8u / 5u;
                    if (!ok) {
                        no = true;
                        continue;
                    }
                    const uint32_t nb = p1 - p0;
                    bool huge = false;
                    if (nb >= HPK_HUGE_MIN && nb < kHugeLimit) {
                        const uint32_t hh = atomicAdd(&s_ctr[11], 1u);
                        if (hh < kHugeMax) {
                            s_huge[hh] = i;
                            huge = true;
                        }
                    }
                    if (!huge) atomicAdd(&s_hist[lpt_class_of(nb)], 1u);
                }
                if (__any(no) && lane == 0) s_ctr[10] = 1u;
                lds_barrier();
                if (s_ctr[10] == 0) {
                    if (tid < 64) {  // class bases
                        const uint32_t v = tid < 32 ? s_hist[tid] : 0u;
                        uint32_t x = v;
#pragma unroll
                        for (int d = 1; d < 64; d <<= 1) {
                            const uint32_t y = __shfl_up(x, d);
                            if (lane >= (uint32_t)d) x += y;
                        }
                        if (tid < 32) s_hist[32 + tid] = x - v;
                        if (tid == 31) {
                            s_ctr[6] = x;  // all from the front of the list
                            s_ctr[7] = 0;
                        }
                    }
                    lds_barrier();
                    const uint32_t nh = min(s_ctr[11], kHugeMax);
                    for (uint32_t i = BA + tid; i < BB; i += G::kBlock) {
                        const uint32_t nb = a.in_off[i + 1] - a.in_off[i];
                        bool huge = false;
                        if (nb >= HPK_HUGE_MIN && nb < kHugeLimit)
                            for (uint32_t hh = 0; hh < nh; ++hh) huge |= s_huge[hh] == i;
                        if (!huge) a.long_list[BA + atomicAdd(&s_hist[32 + lpt_class_of(nb)], 1u)] = i;
                    }
                    cur = BB;  // all listed
                    break;
                }
                lds_barrier();
                if (tid == 0) {
                    s_ctr[6] = 0;
                    s_ctr[7] = 0;
                    s_ctr[11] = 0;
                }
                continue;  // this fill again, from its setup (its prefetched offsets and window are still
                           // in the registers)
            }
        }
        const uint32_t k = s_ctr[0];
        if (k == 0) {  // literal `cur` alone exceeds the window: one lane decodes it from global
            bool left = false;
            {  // (unless it is the long-literal phase's)
                const uint32_t nb = a.in_off[cur + 1] - a.in_off[cur];
                left = nb >= a.long_min && a.out_off[cur + 1] - a.out_off[cur] >= (nb * 8u) / 5u;
                if (left && tid == 0) leave(cur, nb);
            }
            if (tid == 0 && !left) {
                const GlobalSrc g{reinterpret_cast<const uint32_t*>(a.in_base), last16 * 4 + 3};
                uint8_t* dst = a.out_base + gout;
                if (kCompact) {  // (a region below the bound cannot happen here: the library makes them)
                    const uint32_t nb = a.in_off[cur + 1] - a.in_off[cur];
                    a.co_off[cur] = atomicAdd(a.cursor, (nb * 8u) / 5u);
                    dst = a.out_base + a.out_mis + a.co_off[cur];
                }
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
                prefetch_fill<G::kBlock>(P, a, tid, cur, min(cur + (uint32_t)kQ, BB), gin & ~15u, rlast16);
            }
            continue;
        }
        const uint32_t gin_next = s_ctr[2], gout_next = s_ctr[3];  // = in/out offsets of cur + k
        // bucket bases (exclusive scan over 64 buckets by wave 0), then scatter the entries
        if (tid < 64) {
            const uint32_t v = s_hist[tid];
            uint32_t x = v;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t y = __shfl_up(x, d);
                if (lane >= (uint32_t)d) x += y;
            }
            s_bbase[tid] = x - v;
        }
        // the window, from the prefetched registers, as big-endian dwords: bit P of the stream
        // is bit 31 - P % 32 of dword P / 32
        {
            uint4* l16 = reinterpret_cast<uint4*>(s_in);
#pragma unroll
            for (int r = 0; r < S; ++r) {
                const uint4 c = P.chunk[r];
                if (tid + G::kBlock * r < kW / 16)
                    l16[tid + G::kBlock * r] = make_uint4(__builtin_bswap32(c.x), __builtin_bswap32(c.y),
                                                          __builtin_bswap32(c.z), __builtin_bswap32(c.w));
            }
        }
        lds_barrier();
        if (kMode == 3) t_sb1 += __builtin_amdgcn_s_memtime() - tb0;  // (mode 3: scan, window in LDS)
        // queue entries: the fill's literals less those left to the long-literal phase
        const uint32_t kq = (uint32_t)__builtin_amdgcn_readfirstlane((int)(s_bbase[63] + s_hist[63]));
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (pos[r] != 0xFFFFFFFFu) s_q[s_bbase[pos[r] >> 16] + (pos[r] & 0xFFFFu)] = make_uint2(ex[r], ey[r]);
        // the next fill's offsets and window: in flight during this fill's decode. Unconditional
        // (clamped past the range end), so no register phi forces a wait on the stores below.
        const uint32_t cur_next = cur + k;
        // (block-uniform: held in scalar registers through the lane loop)
        const uint32_t pf_c = (uint32_t)__builtin_amdgcn_readfirstlane((int)min(cur_next, BB - 1));
        const uint32_t pf_end = min(pf_c + (uint32_t)kQ, BB);
        const uint32_t pf_base = (uint32_t)__builtin_amdgcn_readfirstlane((int)(gin_next & ~15u));
        // kPfLoop: the next fill's loads are issued one per lane-loop round (the first kPfN rounds)
        // instead of all at once here, where every wave's loads and the write-back's stores queued
        // at the CU's memory path together; what the loop does not issue goes out after it
        uint32_t pf_i = 0;  // (wave-uniform) next load of the prefetch to issue
        auto pf_part = [&](uint32_t j) {
            // (addresses from an opaque copy of the round, so they are not hoisted out of the lane
            // loop into registers it does not have)
            uint32_t base = pf_c;
            asm volatile("" : "+s"(base));
            const uint32_t cntl = pf_end - base;
#pragma unroll
            for (int q = 0; q < kPfN; ++q) {
                if (j == (uint32_t)q) {
                    if (q < R) {  // round q of the offsets
                        const uint32_t t = min(tid + (uint32_t)G::kBlock * q, cntl - 1);
                        P.io0[q] = a.in_off[base + t];
                        P.io1[q] = a.in_off[base + t + 1];
                        P.oo0[q] = a.out_off[base + t];
                        P.oo1[q] = a.out_off[base + t + 1];
                    } else if (q < R + kFD) {  // a deferred write-back round (stored before the window's loads)
                        const int d = q - R;
                        if ((fd_mask >> d) & 1u)
                            reinterpret_cast<uint4*>(a.out_base)[fd_c0 + (base - pf_c) + tid +
                                                                 (uint32_t)G::kBlock * (G::kFlushRounds - kFD + d)] =
                                P.chunk[d < S ? d : 0];
                    } else {  // the window chunks
#pragma unroll
                        for (int r = 0; r < S; ++r)
                            P.chunk[r] = reinterpret_cast<const uint4*>(
                                a.in_base)[min((pf_base >> 4) + (base - pf_c) + tid + (uint32_t)G::kBlock * r, rlast16)];
                    }
                }
            }
        };
        if (!kPfLoop) {
            prefetch_fill<G::kBlock>(P, a, tid, pf_c, pf_end, pf_base, rlast16);
            pf_i = kPfN;
        }
        if (kMode == 3) t_sb2 += __builtin_amdgcn_s_memtime() - tb0;  // (mode 3: + queue, prefetch issued)
        // the previous fill's write-back: its image is read out before this fill decodes over it
        fd_mask = 0;
        if (pk) {
            if (kFD)
                flush_split(pcur, pk, pG0, pG1);
            else
                flush(pcur, pk, pG0, pG1);
        }
        if (!kCompact) {  // (the compacted mode writes each fill back once it is decoded: compact_flush)
            pk = k;
            pcur = cur;
            pG0 = gout;
            pG1 = gout_next;
        }
        if (kMode == 3) t_sb3 += __builtin_amdgcn_s_memtime() - tb0;  // (mode 3: + write-back issued)
        lds_barrier();
        unsigned long long td0 = 0;
        if (kMode == 3) {
            td0 = __builtin_amdgcn_s_memtime();
            t_setB += td0 - tb0;  // (mode 3: window, queue, prefetch + write-back issued)
            if (cur == BA) t_B0 = td0 - tb0;
        }
        if (kMode == 1) {  // diagnostic: no decode; lengths from the queue keep the fill live
            for (uint32_t tt = tid; tt < kq; tt += G::kBlock) {
                const uint2 e = s_q[tt];
                s_lenst[e.y & 0xFFFu] = (e.x >> 16) + s_in[e.x & 0xFFFFu];
            }
        }
        // lane walks: lane i decodes queue slots i and 2 * block - 1 - i of the longest-first queue (the
        // longest with the shortest), the second literal's entry and window dwords read before the first
        // step, so a lane moves on without an LDS round trip (v13 static snake)
        if (kMode != 1 && kq) {
            static_assert(kQ <= 2 * G::kBlock, "static snake: two literals per lane at most");
            const uint2* lq = s_q;
            Lit12 L, N;  // the literal being decoded and the lane's next one
            auto load = [&](Lit12& T, uint32_t tt) {
                const uint2 e = lq[min(tt, kq - 1)];
                T.act = tt < kq && !(e.y & kQ7Byte);
                T.idx = e.y & 0xFFFu;
                const uint32_t nb = e.x >> 16;
                const uint32_t ob = (e.y >> 12) & 0x1FFFFu;
                T.X = (e.x & 0xFFFFu) * 8u + 31u;
                T.Eb = T.X + (T.act ? nb * 8u : 0u);
                T.o = ob;
                T.o0 = ob;
                T.oend = ob + nb * 8u / 5u;
                T.st = HPK_OK;
                T.prog = false;
                lit12_load(T, win32);
            };
            const uint32_t t1 = tid;
            load(L, t1);
            const uint32_t t2 = 2u * G::kBlock - 1u - t1;
            bool nv = t2 < kq;  // a second literal is waiting in N
            if (!(kLate && HPK_FILL_BODY)) load(N, t2);  // (v28 loads it when it starts)
            if (kLate && HPK_FILL_BODY) {
                // v28 (as the wave kernel, hpk_wave.h): body steps (lit12_body) while a literal has >=
                // kBodyMin bits left, slot t1's body then slot t2's; then both tails at once with
                // checked steps that clear `more` once the walk has ended
                bool body = L.Eb - L.X >= kBodyMin;
                uint32_t aX = L.X, aO = L.o, aSt = L.st;
                bool aAct = L.act, onA = true;
                for (;;) {
#pragma unroll
                    for (int s = 0; s < kRefillN; ++s)
                        if (body) lit12_body<kStore>(L, win32, s_lut, s_lo, s_out, body);
                    if (kMode == 3) n_steps += kRefillN;
                    if (kPfLoop && pf_i < (uint32_t)kPfN) pf_part(pf_i++);
                    if (__any(!body)) {
                        const bool sw = !body & onA;
                        if (sw) {
                            aX = L.X;
                            aO = L.o;
                            aSt = L.st;
                            aAct = L.act;
                            load(L, t2);
                            onA = false;
                            body = L.Eb - L.X >= kBodyMin;
                        }
                        if (!__any(body)) break;
                    }
                }
                N = L;
                {
                    const uint2 e = lq[min(t1, kq - 1)];
                    L.X = aX;
                    L.o = aO;
                    L.st = aSt;
                    L.act = aAct;
                    L.Eb = aSt != HPK_OK ? aX : (e.x & 0xFFFFu) * 8u + 31u + (aAct ? (e.x >> 16) * 8u : 0u);
                    L.o0 = (e.y >> 12) & 0x1FFFFu;
                    L.idx = e.y & 0xFFFu;
                    lit12_load(L, win32);
                }
                L.more = L.Eb - L.X >= 5u;
                N.more = N.Eb - N.X >= 5u;
                while (__any(L.more | N.more)) {
                    if (L.more) lit12_step<kStore, false, 2, true>(L, win32, s_lut, s_lo, s_out, dmy);
                    if (N.more) lit12_step<kStore, false, 2, true>(N, win32, s_lut, s_lo, s_out, dmy);
                }
                if (L.act) s_lenst[L.idx] = (L.o - L.o0) | (lit12_status(L) << 24);
                if (N.act) s_lenst[N.idx] = (N.o - N.o0) | (lit12_status(N) << 24);
            } else if (kLate) {
                // v22: a lane's first literal that ends leaves only its end state (bit and output
                // positions, walk status) in three registers as the second one starts; lengths and
                // statuses (the padding check) are made once per lane after the loop, not in every
                // finish round a wave takes (a round ran the check whenever any of its lanes finished)
                uint32_t sX = 0, sO = 0, sSt = 0;
                bool s1 = false;  // the first literal's end state is saved
                for (;;) {
#pragma unroll
                    for (int s = 0; s < kRefillN; ++s) lit12_step<kStore>(L, win32, s_lut, s_lo, s_out, dmy);
                    if (kMode == 3) n_steps += kRefillN;
                    if (kPfLoop && pf_i < (uint32_t)kPfN) pf_part(pf_i++);
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
                if (s1) {
                    const uint2 e = lq[t1];
                    const uint32_t Eb = (e.x & 0xFFFFu) * 8u + 31u + (e.x >> 16) * 8u;
                    const uint32_t st = sSt != HPK_OK ? sSt : residual_status(Eb - sX, win_at(win32, sX - 31u));
                    s_lenst[e.y & 0xFFFu] = (sO - ((e.y >> 12) & 0x1FFFFu)) | (st << 24);
                }
                if (L.act) s_lenst[L.idx] = (L.o - L.o0) | (lit12_status(L) << 24);
            } else {
                // (diagnostic modes 2 and 4) a finished literal's length and status made in the round
                for (;;) {
#pragma unroll
                    for (int s = 0; s < kRefillN; ++s) lit12_step<kStore>(L, win32, s_lut, s_lo, s_out, dmy);
                    if (kMode == 3) n_steps += kRefillN;
                    const bool fin = !L.prog;  // no progress in the last step: finished (or idle)
                    if (__any(fin)) {
                        if (fin && L.act) s_lenst[L.idx] = (L.o - L.o0) | (lit12_status(L) << 24);
                        if (fin) {
                            if (nv) {
                                L = N;
                                nv = false;
                            } else {
                                L.act = false;
                            }
                        }
                        // (only a finish changes what is left: the check stays off the step path;
                        // an idle lane makes no progress, so the first pass always gets here)
                        if (!__any(L.act || nv)) break;
                    }
                }
            }
        }
        while (pf_i < (uint32_t)kPfN) pf_part(pf_i++);  // (kPfLoop) the prefetch loads the loop did not issue
        unsigned long long tq0 = 0;
        if (kMode == 3) {
            tq0 = __builtin_amdgcn_s_memtime();
            t_dec += tq0 - td0;
        }
        // literals whose output region is below the decoded bound (or not dword-aligned for the
        // dword stores): byte stores into the image with a capacity check per byte
        for (uint32_t tt = tid; kMode != 1 && tt < kq; tt += G::kBlock) {
            const uint2 e = s_q[tt];
            if (e.y & kQ7Byte) {
                const uint32_t i = e.y & 0xFFFu;
                const uint32_t o = a.out_off[cur + i] + a.out_mis - ob16;
                Lit B = {};
                lit_bytes_to(B, LdsSwapSrc{win32}, s_lo, [&](uint32_t j, uint8_t v) { s_out[o + j] = v; },
                             a.out_off[cur + i + 1] - a.out_off[cur + i], e.x & 0xFFFFu, e.x >> 16);
                s_lenst[i] = B.cnt | (lit_status(B) << 24);
            }
        }
        if (kMode == 3) t_byte += __builtin_amdgcn_s_memtime() - tq0;
        if (kCompact) compact_flush(cur, k, kq);
        cur = cur_next;
        gin = gin_next;
        gout = gout_next;
    }
    if (kMode == 3) t_tail = __builtin_amdgcn_s_memtime();
    if (pk) {
        lds_barrier();
        flush(pcur, pk, pG0, pG1);
    }
    if (kMode == 3 && lane == 0) {
        const uint64_t gwi = (uint64_t)blockIdx.x * kWaves + (tid >> 6);
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        a.dbg[gwi * 16 + 0] = t_end - t_start;
        a.dbg[gwi * 16 + 1] = t_dec;
        a.dbg[gwi * 16 + 2] = n_steps;
        a.dbg[gwi * 16 + 3] = n_fills;
        a.dbg[gwi * 16 + 4] = t_pre;
        a.dbg[gwi * 16 + 5] = t_setA;
        a.dbg[gwi * 16 + 6] = t_setB;
        a.dbg[gwi * 16 + 7] = 0;
        a.dbg[gwi * 16 + 8] = t_A0;
        a.dbg[gwi * 16 + 9] = t_B0;
        a.dbg[gwi * 16 + 10] = t_byte;
        a.dbg[gwi * 16 + 11] = t_end - t_tail;
        a.dbg[gwi * 16 + 12] = t_sb1;
        a.dbg[gwi * 16 + 13] = t_sb2;
        a.dbg[gwi * 16 + 14] = t_sb3;
    }
    {  // the literals this workgroup left to the long-literal phase
        lds_barrier();
        if (tid == 0) s_ctr[5] = 0;  // its claim counter
        __syncthreads();  // (every thread's list entries and stores are out)
        static_assert(kW + kO + 12 * kQ >= huge_lds_bytes<G::kBlock>(), "huge-phase LDS");
        huge_phase<G::kBlock, 2>(a, s_huge, min(s_ctr[11], kHugeMax), reinterpret_cast<uint32_t*>(s_in), s_lut, s_lo);
        // rings, then output buffers, then the wave queues, over the window, image, fill queue and
        // lengths (all free once the fills are done)
        constexpr int kLB = HPK_LONG_WAVES * 64;
        constexpr int kLQ = kLB * (HPK_LONG_RING * 4 + HPK_LONG_OS);
        static_assert(kLQ + HPK_LONG_WAVES * HPK_LONG_CLAIM * 16 <= kW + kO + 12 * kQ && G::kInOff % 16 == 0 &&
                          kW % 16 == 0 && kLQ % 16 == 0 && G::kHistOff == G::kInOff + kW + kO + 12 * kQ,
                      "long-phase LDS");
        long_phase<kLB, HPK_LONG_U, HPK_LONG_RING, kMode == 5 ? 1 : 0, G::kBlock, HPK_LONG_OS, HPK_LONG_CLAIM, 2,
                   kCompact>(
            a, BA, BB, s_ctr[6], s_ctr[7], &s_ctr[5], reinterpret_cast<uint32_t*>(s_in), s_in + kLB * HPK_LONG_RING * 4,
            reinterpret_cast<uint4*>(s_in + kLQ), s_lut, s_lo);
    }
}

}  // namespace hpkdec
