// legacy_decode12.h — development harness copy (not part of the product) of the v12-v24 fill kernel
// with every compile-time variant measured along the way (kCoop whole-wave long literals and the v18
// segment stream, kSched dynamic slots, kAcc dword stores, kDefer, kSpread, HPK_FAST, HPK_RELOAD,
// HPK_DEC_SPLIT, HPK_FLUSH_TOP, HPK_FD_FIRST; DESIGN.md §4.1 has their numbers). The product header
// loona_amd/csrc/hpk_decode12.h keeps only the shipped configuration.
// Original header comment: hpk_decode12.h — decode kernel v12: the v8 fill structure, a bit-position step, and a
// wave-cooperative path for long literals.
//
// Fill structure as v8 (hpk_decode7, now in bench/legacy_decode.h): per fill an LDS input window, an LDS
// image of the fill's output span and a longest-first queue; the next fill's offsets and window
// are prefetched into registers while the current one decodes, the previous image is written
// back with 16-byte stores. What changes:
//   * the window is staged as big-endian dwords; a lane holds its bit position as X = P + 31 and
//     the dword pair (d0, d1) = window dwords (X >> 5) - 1 and X >> 5, plus the next dword d2.
//     The 32 bits at P are ONE v_alignbit_b32(d0, d1, ~X): no 64-bit shifts and no refill
//     bookkeeping (v8 spent ~14 VALU per step on its 64-bit window refill);
//   * a step does kLook lookups in the two-symbol table (LUT2 layout, hpk_code.h), each decoding
//     up to two codes of <= 12 bits; the second lookup reads the window shifted past the first;
//   * a step advances <= 24 bits, so it crosses at most one dword: the pair then slides by one
//     (v_cndmask) and d2 takes d3, the dword read at the top of the step (issued before the table
//     reads, so it has arrived when they have: no extra wait on the serial chain);
//   * output: kAcc = false stores each symbol as a byte into the LDS image; kAcc = true gathers a
//     step's bytes with v_perm and stores whole dwords (fewer LDS stores, more VALU);
//   * a code longer than 12 bits (EOS included) takes the rarely taken branch: one leading-ones
//     lookup on a freshly read pair. Bits past a literal's end are never masked: a code that
//     runs past the end is, by prefix-freeness, longer than what is left whatever follows, so the
//     walk stops exactly where huffman.rs's bit iterator stops matching (huffman.rs:100-123); the
//     final padding check (huffman.rs:128-160) looks at the residual bits only;
//   * long literals (>= 224 encoded bytes: the head of the longest-first queue) are not given to
//     one lane: a whole wave decodes each of them by self-synchronising speculation (long_decode
//     below), so a 4 KiB header value no longer holds a fill for thousands of steps.
#pragma once
#include "../loona_amd/csrc/hpk_decode_kernel.h"
#include "../loona_amd/csrc/hpk_split.h"

#ifndef HPK_FD_FIRST
#define HPK_FD_FIRST 0  // 1: the write-back rounds deferred to the lane loop are the first (always full), not the last
#endif
#ifndef HPK_FLUSH_LOOP
#define HPK_FLUSH_LOOP 1  // write-back rounds (<= 3) stored from the lane loop instead of before it (needs HPK_PF_LOOP; 1: config 5 +1 %, 2 spill)
#endif
#ifndef HPK_FLUSH_TOP
#define HPK_FLUSH_TOP 0  // 1: the previous fill's write-back at the top of a fill (config 5 687 vs 689 GiB/s: no gain)
#endif
#ifndef HPK_PF_LOOP
#define HPK_PF_LOOP 1
#endif
#ifndef HPK_STAGGER
#define HPK_STAGGER 1
#endif
#ifndef HPK_STAGGER_PH
#define HPK_STAGGER_PH 2  // phases: workgroup b's first fill is (b % PH) / PH of a window
#endif
#ifndef HPK_LATE_FIN
#define HPK_LATE_FIN 1  // 0: a finished lane literal's length and status are made in the finish round (v21)
#endif
#ifndef HPK_FAST
#define HPK_FAST 0  // 1: body steps without fit tests + a checked tail pass (measured slower)
#endif
#ifndef HPK_RELOAD
// 1: lane steps read the window's two dwords each step instead of shifting a 3-dword register window
// (5 fewer VALU per step, but the read sits on the step's dependency chain: config 2 46.2 vs 45.6 us,
// config 3 825-829 vs 832-842 us, profiles/r02/v20/decode_reload_ab.jsonl)
#define HPK_RELOAD 0
#endif
#ifndef HPK_DEC_SPLIT
// workgroup ranges balanced by encoded bytes (hpk_split.h): off — measured on config 3 at 857-861 us
// against 859-871 (the fills and the long phase already even the workgroups out) and on config 2
// +4.5 us (the search's two dependent reads before the first fill), profiles/r02/v20/decode_split_ab.jsonl
#define HPK_DEC_SPLIT 0
#endif

namespace hpkdec {

// LDS carve-up: Geo7's regions plus a fifth counter (the long-literal queue head).
template <int kWaves, int kW, int kO, int kQ>
struct Geo12 : Geo7<kWaves, kW, kO, kQ, true> {
    using B = Geo7<kWaves, kW, kO, kQ, true>;
    static constexpr int kLdsBytes = B::kCtrOff + 48;
    static_assert(kLdsBytes <= 163840, "LDS budget (160 KiB per CU on gfx950)");
};

#ifndef HPK_DEFER0
#define HPK_DEFER0 2
#endif

// Longest-first buckets 0..14 hold the literals of >= 224 encoded bytes (lpt_bucket).
constexpr uint32_t kLongBuckets = 15;

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

__device__ __forceinline__ void put32(uint32_t* __restrict__ out32, uint32_t pos, uint32_t v, uint32_t oend, int kStore) {
    if (kStore == kChecked) {
        if (pos < oend)
            out32[pos] = v;
        else
            chk_report(2, pos, oend, 0);
    } else if (kStore == kDword || kStore == kPred) {
        out32[pos] = v;
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

// A window cursor for a walk: X = bit position + 31, the dword pair holding bit X - 31 and the dword
// after it. The 32 bits at the position are one v_alignbit; an advance of <= 32 bits slides the pair
// with the dword read ahead of the step (d3), so a lookup costs one LDS round trip, not three.
struct WinCur {
    uint32_t X, d0, d1, d2;
};
__device__ __forceinline__ void wc_load(WinCur& c, const uint32_t* __restrict__ win32, uint32_t p) {
    c.X = p + 31u;
    const uint32_t* q = win32 + (c.X >> 5);
    c.d0 = q[-1];
    c.d1 = q[0];
    c.d2 = q[1];
}
__device__ __forceinline__ uint32_t wc_bits(const WinCur& c) { return __builtin_amdgcn_alignbit(c.d0, c.d1, ~c.X); }
__device__ __forceinline__ uint32_t wc_next(const uint32_t* __restrict__ win32, const WinCur& c) {
    return win32[(c.X >> 5) + 2];
}
__device__ __forceinline__ void wc_adv(WinCur& c, uint32_t n, uint32_t d3) {
    const uint32_t xn = c.X + n;
    const bool cross = (xn ^ c.X) > 31u;
    c.d0 = cross ? c.d1 : c.d0;
    c.d1 = cross ? c.d2 : c.d1;
    c.d2 = cross ? d3 : c.d2;
    c.X = xn;
}

// The codes one table entry decodes with rem bits left: ok1 / ok2 = its first / second code fits
// inside the literal; returns the bits they use.
__device__ __forceinline__ uint32_t lut12(uint32_t e, uint32_t rem, bool& ok1, bool& ok2) {
    // a length field the entry does not hold is 63, past any clamped rem (and t1 >= l1: ok2 => ok1)
    const uint32_t rc = min(rem, HPK_LUT2_CLAMP);
    const uint32_t l1 = HPK_L2_LEN0(e), t1 = HPK_L2_LEN01(e);
    ok1 = l1 <= rc;
    ok2 = t1 <= rc;
    return ok2 ? t1 : (ok1 ? l1 : 0u);
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
    uint32_t o;           // next output byte (kAcc: next output dword) in the LDS image
    uint32_t o0;          // first output byte of the literal (byte stores)
    uint32_t cnt;         // bytes decoded (kAcc)
    uint32_t acc, accn;   // pending output bytes and their count 0..3 (kAcc)
    uint32_t oend;        // checked mode: end of the literal's capacity (bytes / dwords)
    uint32_t st;          // hpk_status set by the walk (EOS, or padding found by the long-code branch)
    uint32_t idx;         // literal index in the fill
    bool prog;            // the last step consumed a code or took the long-code branch
    bool act;             // holds a fast-path literal not yet finalised
};

// (Re)load the pair and the next dword at X.
__device__ __forceinline__ void lit12_load(Lit12& L, const uint32_t* __restrict__ win32) {
    const uint32_t* p = win32 + (L.X >> 5);
    L.d0 = p[-1];
    L.d1 = p[0];
    L.d2 = p[1];
}

// Append g (<= 4) bytes p (zero above them) to the pending output; store a dword when one is full.
template <int kStore>
__device__ __forceinline__ void acc_push(Lit12& L, uint32_t* __restrict__ out32, uint32_t p, uint32_t g,
                                         uint32_t dmy32 = 0) {
    const uint64_t x = (uint64_t)p << (8u * L.accn);
    const uint32_t lo = L.acc | (uint32_t)x;
    const uint32_t n2 = L.accn + g;  // <= 7
    const bool full = n2 >= 4u;
    if (kStore == kPred)
        out32[full ? L.o : dmy32] = lo;  // unconditional: a dword not yet complete goes to the dummy slot
    else if (full)
        put32(out32, L.o, lo, L.oend, kStore);
    L.o += full ? 1u : 0u;
    L.acc = full ? (uint32_t)(x >> 32) : lo;
    L.accn = n2 & 3u;
    L.cnt += g;
}

// kStore == kPred: the (up to) four byte stores of a step are unconditional, a byte that is not
// output going to the lane's dummy slot out8[dmy] (no exec-mask branch around each store).
template <int kStore, int kLook, bool kAcc>
__device__ __forceinline__ void lit12_step(Lit12& L, const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                           const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8,
                                           uint32_t dmy = 0) {
    uint32_t* out32 = reinterpret_cast<uint32_t*>(out8);
#if HPK_RELOAD
    // the window's two dwords read at each step (no registers shifted on a dword crossing)
    const uint32_t* const wq = win32 + (L.X >> 5);
    const uint32_t w = __builtin_amdgcn_alignbit(wq[-1], wq[0], ~L.X);
#else
    const uint32_t d3 = win32[(L.X >> 5) + 2];  // the dword after d2, in case this step crosses one
    const uint32_t w = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
#endif
    const uint32_t rem = L.Eb - L.X;
    const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
    bool a1, a2;
    const uint32_t u1 = lut12(e1, rem, a1, a2);
    uint32_t use = u1;
    // a code longer than 12 bits (or EOS) starts here and may still fit (with more than 12 bits
    // left, any code the entry holds fits: no first code <=> the entry has none)
    bool park = !a1 & (rem > (uint32_t)HPK_LUT_BITS);
    uint32_t pk = 0, g = 0;
    if (!kAcc && kStore == kPred) {
        out8[a1 ? L.o : dmy] = (uint8_t)e1;
        out8[a2 ? L.o + 1 : dmy] = (uint8_t)(e1 >> 16);
        L.o += (uint32_t)a1 + (uint32_t)a2;
    } else if (!kAcc) {
        if (a1) put8(out8, L.o, e1, L.oend, kStore);
        if (a2) put8(out8, L.o + 1, e1 >> 16, L.oend, kStore);
        L.o += (uint32_t)a1 + (uint32_t)a2;
    } else {
        g = (uint32_t)a1 + (uint32_t)a2;
        pk = lut12_bytes(e1, g);
    }
    if (kLook == 2) {
        // the first entry was consumed whole: look the next bits up too
        const bool cont = a1 & (a2 | (e1 >= HPK_LUT2_NOTTWO));
        const uint32_t w2 = w << u1;
        const uint32_t rem2 = rem - u1;
        const uint32_t e2 = lut[w2 >> (32 - HPK_LUT_BITS)];
        bool b1, b2;
        const uint32_t u2 = lut12(e2, rem2, b1, b2);
        park |= cont & !b1 & (rem2 > (uint32_t)HPK_LUT_BITS);
        b1 &= cont;
        b2 &= cont;
        if (!kAcc && kStore == kPred) {
            out8[b1 ? L.o : dmy] = (uint8_t)e2;
            out8[b2 ? L.o + 1 : dmy] = (uint8_t)(e2 >> 16);
            L.o += (uint32_t)b1 + (uint32_t)b2;
        } else if (!kAcc) {
            if (b1) put8(out8, L.o, e2, L.oend, kStore);
            if (b2) put8(out8, L.o + 1, e2 >> 16, L.oend, kStore);
            L.o += (uint32_t)b1 + (uint32_t)b2;
        } else {
            const uint32_t g2 = (uint32_t)b1 + (uint32_t)b2;
            pk |= lut12_bytes(e2, g2) << (8u * g);
            g += g2;
        }
        use += cont ? u2 : 0u;
    }
    if (kAcc) acc_push<kStore>(L, out32, pk, g, dmy >> 2);
    const uint32_t xn = L.X + use;
#if !HPK_RELOAD
    const bool cross = (xn ^ L.X) > 31u;
    L.d0 = cross ? L.d1 : L.d0;
    L.d1 = cross ? L.d2 : L.d1;
    L.d2 = cross ? d3 : L.d2;
#endif
    L.X = xn;
    L.prog = a1 | park;
    if (park) {  // a 13..30-bit code or EOS: one leading-ones lookup (any code in one read)
#if HPK_RELOAD
        const uint32_t* const pq = win32 + (L.X >> 5);
        const uint32_t wp = __builtin_amdgcn_alignbit(pq[-1], pq[0], ~L.X);
#else
        const uint32_t wp = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
#endif
        uint32_t s, len;
        bool eos;
        lo_decode(wp, lo, s, len, eos);
        const uint32_t r = L.Eb - L.X;
        if (len > r) {  // nothing fits in the > 12 bits left: huffman.rs:128-134
            L.st = HPK_PADDING_TOO_LARGE;
            L.Eb = L.X;
        } else if (eos) {  // huffman.rs:112-116
            L.st = HPK_EOS_IN_STRING;
            L.Eb = L.X;
        } else {
            if (kAcc) {
                acc_push<kStore>(L, out32, s, 1u, dmy >> 2);
            } else {
                put8(out8, L.o, s, L.oend, kStore);
                L.o += 1;
            }
            L.X += len;
            if (!HPK_RELOAD) lit12_load(L, win32);
        }
    }
}

// The body step (v21, kFast): the same two lookups with no per-code fit test. A step commits only
// when every code its two entries hold ends inside the literal (X + held1 + held2 <= Eb: one compare
// for the step); otherwise it changes nothing, and the literal's last bits are left to the checked
// step (lit12_step) in the tail pass after the lane loop, so the step's stores and advances need no
// fit flags, only the held counts. prog = false at a step that stops: it overran the literal's end,
// or no code of <= 12 bits starts here and fewer than 13 bits are left. A stopped walk is a fixed
// point (the same step stops again), so a lane can keep stepping until its wave leaves the loop.
// Stores go in an order that leaves no byte outside the step's output: a slot an entry does not
// fill is written first and then overwritten (sym1 at o + two, then sym0 at o), a second entry with
// no code writes to the dummy slot, and a step that stops writes only there. A park (a longer code
// with >= 13 bits left) lets the first entry's bytes land on o, where the park's own byte goes; an
// error there (EOS, or a code running past the end) leaves them in the literal's own slack: it has
// >= 13 unconsumed bits, so its decoded length is >= 2 below the bound (huffman.rs:95-161).
__device__ __forceinline__ void lit12_fast(Lit12& L, const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                           const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8, uint32_t dmy) {
    const uint32_t d3 = win32[(L.X >> 5) + 2];  // the dword after d2, in case this step crosses one
    const uint32_t w = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
    const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
    const uint32_t h1 = HPK_L2_HELD(e1);
    const uint32_t e2 = lut[(w << h1) >> (32 - HPK_LUT_BITS)];  // (no code: h1 = 0, e2 = e1)
    const uint32_t xn = L.X + h1 + HPK_L2_HELD(e2);
    const bool none2 = e2 >= HPK_LUT2_NONE;
    const bool park = none2 & (xn + (uint32_t)HPK_LUT_BITS < L.Eb);  // >= 13 bits left at xn
    // a step at a longer code (no code in e1: xn = X) needs >= 13 bits; otherwise its codes must fit
    const bool stop = xn + (e1 >> 31) * (uint32_t)(HPK_LUT_BITS + 1) > L.Eb;
    const uint32_t n1 = HPK_L2_CODES(e1);
    const uint32_t b1 = stop ? dmy : L.o;
    out8[b1 + HPK_L2_TWO(e1)] = (uint8_t)(e1 >> 16);
    out8[b1] = (uint8_t)e1;
    const uint32_t b2 = none2 ? dmy : b1 + n1;
    out8[b2 + HPK_L2_TWO(e2)] = (uint8_t)(e2 >> 16);
    out8[b2] = (uint8_t)e2;
    L.o = stop ? L.o : L.o + n1 + HPK_L2_CODES(e2);
    const uint32_t xc = stop ? L.X : xn;
    const bool cross = (xc ^ L.X) > 31u;
    L.d0 = cross ? L.d1 : L.d0;
    L.d1 = cross ? L.d2 : L.d1;
    L.d2 = cross ? d3 : L.d2;
    L.X = xc;
    L.prog = !stop;
    if (park) {  // a 13..30-bit code or EOS with more than 12 bits left: one leading-ones lookup
        const uint32_t wp = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
        uint32_t s, len;
        bool eos;
        lo_decode(wp, lo, s, len, eos);
        if (len > L.Eb - L.X) {  // nothing fits in what is left: huffman.rs:128-134
            L.st = HPK_PADDING_TOO_LARGE;
            L.Eb = L.X;
        } else if (eos) {  // huffman.rs:112-116
            L.st = HPK_EOS_IN_STRING;
            L.Eb = L.X;
        } else {
            out8[L.o] = (uint8_t)s;
            L.o += 1;
            L.X += len;
            lit12_load(L, win32);
        }
    }
}

// Final status of a literal whose walk has stopped; a status set by the walk wins.
__device__ __forceinline__ uint32_t lit12_status(const Lit12& L) {
    if (L.st != HPK_OK) return L.st;
    return residual_status(L.Eb - L.X, __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X));
}

// The same for the step's window as the steps use it (HPK_RELOAD: read from the LDS window).
__device__ __forceinline__ uint32_t lit12_status(const Lit12& L, const uint32_t* __restrict__ win32) {
    if (!HPK_RELOAD) return lit12_status(L);
    if (L.st != HPK_OK) return L.st;
    const uint32_t* const q = win32 + (L.X >> 5);
    return residual_status(L.Eb - L.X, __builtin_amdgcn_alignbit(q[-1], q[0], ~L.X));
}

// ------------------------------------------------------------------------------------------
// Wave-cooperative decode of one long literal (self-synchronising speculation).
//
// The literal's N bits are cut into 64 segments of S >= 32 bits; lane j walks codes from a start
// b_j (speculatively j*S) while they start before e_j = (j+1)*S and records where it stops: the
// first code boundary at or past e_j ("through"), the literal's end, or an EOS. Lane j's true
// start is lane j-1's stop when that one came through; Huffman walks from a wrong position fall
// into step with the true one within a few codes, so after one re-walk from the neighbours' stops
// the starts are all true and a second pass changes nothing. Each round only lanes whose start
// changed walk again, and the loop ends (lane 0's start is always true, and round r fixes lane r).
// A final walk writes the symbols at offsets from a scan of the per-lane counts.

enum SegStop : uint32_t { kThrough = 0, kEnded = 1, kEos = 2, kStuck = 3 };

// One lane's walk over [b, e) of a literal at window bit P0 with N bits; writes its symbols to
// out8[o ...] when kWrite. Returns the stop position; cnt = codes taken, stop = SegStop.
template <bool kWrite>
__device__ __forceinline__ uint32_t seg_walk(const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                             const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8, int kStore,
                                             uint32_t P0, uint32_t N, uint32_t b, uint32_t e, uint32_t o, uint32_t oend,
                                             uint32_t& cnt, uint32_t& stop) {
    uint32_t pos = b;
    cnt = 0;
    stop = kThrough;
    bool run = pos < e;
    WinCur c;
    wc_load(c, win32, P0 + pos);
    // every pass advances >= 5 bits or stops; the guard only bounds the loop for the compiler and
    // any unforeseen input (a segment holds <= 8192 bits)
    for (uint32_t guard = 0; run; ++guard) {
        if (guard > 4096u) {
            stop = kStuck;
            break;
        }
        const uint32_t d3 = wc_next(win32, c);
        const uint32_t w = wc_bits(c);
        const uint32_t rem = N - pos;
        const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
        bool a1, a2;
        lut12(e1, rem, a1, a2);
        uint32_t adv = 0;
        if (a1) {
            const uint32_t l1 = HPK_L2_LEN0(e1);
            if (kWrite) put8(out8, o + cnt, e1, oend, kStore);
            cnt += 1;
            if (a2 && pos + l1 < e) {  // the second code also starts inside the segment
                if (kWrite) put8(out8, o + cnt, e1 >> 16, oend, kStore);
                cnt += 1;
                adv = HPK_L2_LEN01(e1);
            } else {
                adv = l1;
            }
            run = pos + adv < e;
        } else if (e1 >= HPK_LUT2_NONE && rem > (uint32_t)HPK_LUT_BITS) {
            uint32_t s, len;
            bool eos;
            lo_decode(w, lo, s, len, eos);
            if (len > rem) {
                stop = kEnded;
                run = false;
            } else if (eos) {
                stop = kEos;
                run = false;
            } else {
                if (kWrite) put8(out8, o + cnt, s, oend, kStore);
                cnt += 1;
                adv = len;
                run = pos + adv < e;
            }
        } else {  // the next code does not fit: the literal ends here
            stop = kEnded;
            run = false;
        }
        pos += adv;
        wc_adv(c, adv, d3);
    }
    return pos;
}

// A lane's walk state in long_decode: where it stopped, how it stopped, the codes it took, and a
// mask of the code starts it passed in the first 64 bits of its segment.
struct SegWalk {
    uint32_t pos, cnt, stop;
    uint64_t mask;  // bit i: a code started at segment start + i
};

// seg_walk without output, recording code starts in [s0, s0 + 64). With kResume, the walk from b
// stops at the first code start that `old` also passed: from there on the old walk is valid (same
// bits, same boundaries), so its counts, stop and mask are spliced in. A re-walk from a corrected
// start therefore costs the few codes until the two walks fall into step, not the segment.
template <bool kResume>
__device__ __forceinline__ SegWalk seg_record(const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                              const uint16_t* __restrict__ lo, uint32_t P0, uint32_t N, uint32_t s0,
                                              uint32_t b, uint32_t e, const SegWalk& old) {
    SegWalk r = {b, 0u, (uint32_t)kThrough, 0ull};
    // at a code start p: true when the walk joins `old` there (r completed from old)
    auto join = [&](uint32_t p) {
        const uint32_t i = p - s0;
        if (i >= 64u) return false;
        const uint64_t bit = 1ull << i;
        if (kResume && (old.mask & bit)) {
            r.cnt += old.cnt - (uint32_t)__popcll(old.mask & (bit - 1));
            r.mask |= old.mask & ~(bit - 1);
            r.pos = old.pos;
            r.stop = old.stop;
            return true;
        }
        r.mask |= bit;
        return false;
    };
    bool run = r.pos < e;
    WinCur c;
    wc_load(c, win32, P0 + b);
    for (uint32_t guard = 0; run; ++guard) {
        if (guard > 4096u) {
            r.stop = kStuck;
            break;
        }
        if (join(r.pos)) break;
        const uint32_t pos = r.pos;
        const uint32_t d3 = wc_next(win32, c);
        const uint32_t w = wc_bits(c);
        const uint32_t rem = N - pos;
        const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
        bool a1, a2;
        lut12(e1, rem, a1, a2);
        if (a1) {
            const uint32_t p2 = pos + (HPK_L2_LEN0(e1));
            r.cnt += 1;
            r.pos = p2;
            if (a2 && p2 < e) {  // the second code also starts inside the segment
                if (join(p2)) break;
                r.cnt += 1;
                r.pos = pos + (HPK_L2_LEN01(e1));
            }
            run = r.pos < e;
        } else if (e1 >= HPK_LUT2_NONE && rem > (uint32_t)HPK_LUT_BITS) {
            uint32_t sy, len;
            bool eos;
            lo_decode(w, lo, sy, len, eos);
            if (len > rem) {
                r.stop = kEnded;
                run = false;
            } else if (eos) {
                r.stop = kEos;
                run = false;
            } else {
                r.cnt += 1;
                r.pos = pos + len;
                run = r.pos < e;
            }
        } else {  // the next code does not fit: the literal ends here
            r.stop = kEnded;
            run = false;
        }
        wc_adv(c, r.pos - pos, d3);
    }
    return r;
}

// Whole-wave call (all 64 lanes, wave-uniform arguments): the literal's bits start at window bit
// P0 (N bits), its output at image byte o0. Returns out_len and the hpk_status.
//
// A lane's start is only replaced by its left neighbour's stop when that walk came "through" its
// segment; a lane whose left neighbour stopped (end of literal or EOS, possibly a spurious one on
// a not-yet-synchronised walk) keeps its own start and walk. So a spurious stop does not silence
// the lanes after it (a cascade of one lane per round); once corrected, the next lane re-walks
// from the true start and, with the boundary mask, joins its old walk within a few codes. The
// first lane that does not come through holds the literal's true end.
template <uint32_t kLead>
__device__ __forceinline__ void long_decode(const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                            const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8, int kStore,
                                            uint32_t P0, uint32_t N, uint32_t o0, uint32_t& out_len, uint32_t& status,
                                            uint32_t& nround) {
    const uint32_t j = threadIdx.x & 63u;
    const uint32_t S = max(32u, (N + 63u) >> 6);
    const uint32_t s0 = j * S, e = (j + 1) * S;
    uint32_t b = s0;
    SegWalk wk = {b, 0u, (uint32_t)kEnded, 0ull};
    auto walk = [&](bool resume) {
        if (b >= N) {  // nothing left: a stop at the literal's end
            wk = {b, 0u, (uint32_t)kEnded, 0ull};
        } else if (S > 96u) {  // long segments: keep the boundary mask, re-walks join the old walk
            wk = resume ? seg_record<true>(win32, lut, lo, P0, N, s0, b, e, wk)
                        : seg_record<false>(win32, lut, lo, P0, N, s0, b, e, wk);
        } else {  // short segments re-walk whole (cheaper than keeping the mask up)
            wk.pos = seg_walk<false>(win32, lut, lo, out8, kStore, P0, N, b, e, 0, 0, wk.cnt, wk.stop);
        }
    };
    // lead-in: lane j > 0 first walks codes from kLead bits before its segment, so its speculative
    // start is usually already the true one (Huffman walks fall into step within a few codes) and
    // the rounds below mostly just confirm it instead of re-walking
    if (kLead && j > 0 && s0 < N) {
        uint32_t p = s0 > kLead ? s0 - kLead : 0u;
        WinCur c;
        wc_load(c, win32, P0 + p);
        for (uint32_t g = 0; p < s0 && g < kLead; ++g) {
            const uint32_t d3 = wc_next(win32, c);
            const uint32_t w = wc_bits(c);
            const uint32_t rem = N - p;
            const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
            bool a1, a2;
            lut12(e1, rem, a1, a2);
            uint32_t adv = 0;
            if (a1) {
                const uint32_t l1 = HPK_L2_LEN0(e1);
                adv = (a2 && p + l1 < s0) ? HPK_L2_LEN01(e1) : l1;
            } else if (e1 >= HPK_LUT2_NONE && rem > (uint32_t)HPK_LUT_BITS) {
                uint32_t sy, len;
                bool eos;
                lo_decode(w, lo, sy, len, eos);
                if (len > rem || eos) break;
                adv = len;
            } else {
                break;
            }
            p += adv;
            wc_adv(c, adv, d3);
        }
        b = p >= s0 ? p : s0;  // a lead-in cut short leaves the plain speculative start
        wk.pos = b;
    }
    walk(false);
    // lane j's start only changes after lane j-1's stopped changing, so 64 rounds always suffice
    bool stuck = false;
    nround = 0;
    for (uint32_t round = 0;; ++round) {
        nround = round;
        if (round > 64u) {
            stuck = true;
            break;
        }
        const uint32_t lpos = __shfl_up(wk.pos, 1);
        const uint32_t lthrough = __shfl_up((uint32_t)(wk.stop == kThrough), 1);
        const uint32_t nb = j == 0 ? 0u : (lthrough ? lpos : b);
        const bool changed = nb != b;
        if (!__any(changed)) break;
        if (changed) {
            b = nb;
            walk(true);
        }
    }
    // the literal ends in the first lane that does not come through (all through: the last lane)
    const uint64_t nt = __ballot(wk.stop != kThrough);
    const uint32_t L = nt ? (uint32_t)__builtin_ctzll(nt) : 63u;
    const uint32_t c = j <= L ? wk.cnt : 0u;
    uint32_t incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d);
        if (j >= (uint32_t)d) incl += y;
    }
    out_len = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    const uint32_t s_stop = (uint32_t)__builtin_amdgcn_readlane((int)wk.stop, (int)L);
    const uint32_t s_pos = (uint32_t)__builtin_amdgcn_readlane((int)wk.pos, (int)L);
    status = s_stop == kEos ? (uint32_t)HPK_EOS_IN_STRING : residual_status(N - s_pos, win_at(win32, P0 + s_pos));
    if (stuck || __any(j <= L && wk.stop == kStuck)) status = 0x7F;  // never expected: a bad status
    if (c) {
        uint32_t c2, st2;
        seg_walk<true>(win32, lut, lo, out8, kStore, P0, N, b, e, o0 + incl - c, o0 + N / 5u, c2, st2);
    }
}

// ------------------------------------------------------------------------------------------
// (v18 segment stream, below) Symbols of a walk: byte k at bits 8(k % 8) of lo (k < 8) or of hi.
// OR the (<= 2) bytes v in at byte index cnt (0..13) of the 128-bit (lo, hi).
__device__ __forceinline__ void st128_put(uint64_t& lo, uint64_t& hi, uint32_t cnt, uint32_t v) {
    const uint32_t sh = cnt * 8u;
    const uint64_t x = (uint64_t)v;
    lo |= sh < 64u ? x << (sh & 63u) : 0ull;
    hi |= sh >= 64u ? x << ((sh - 64u) & 63u) : (sh > 48u ? x >> ((64u - sh) & 63u) : 0ull);
}

__device__ __forceinline__ void shr128(uint64_t& lo, uint64_t& hi, uint32_t s) {  // s: bits, < 128
    const uint64_t l = s == 0u ? lo : (s < 64u ? (lo >> (s & 63u)) | (hi << ((64u - s) & 63u)) : hi >> ((s - 64u) & 63u));
    const uint64_t h = s < 64u ? hi >> (s & 63u) : 0ull;
    lo = l;
    hi = h;
}

__device__ __forceinline__ void shl128(uint64_t& lo, uint64_t& hi, uint32_t s) {  // s: bits, < 128
    const uint64_t h = s == 0u ? hi : (s < 64u ? (hi << (s & 63u)) | (lo >> ((64u - s) & 63u)) : lo << ((s - 64u) & 63u));
    const uint64_t l = s < 64u ? lo << (s & 63u) : 0ull;
    lo = l;
    hi = h;
}

// One lane's walk over the segment [s0, e) of a literal at window bit P0 with N bits, from bit b
// (s0 <= b <= N, b < s0 + 30). Each step reads the LUT2 entry AND the leading-ones entry of the
// same 32 window bits (both from the window bits, so the reads issue together and a 13..30-bit
// code costs no branch). Out: where and how it stopped (pos, stop: SegStop), the symbols (cnt of
// them, in lo/hi, which must be zero on entry) and the code starts it passed (mask, bit i = s0 + i).
// kJoin: stop at the first code start that the walk of mask `omask` also passed (joined = true,
// pos = that start, jq = that walk's symbols before it).
template <bool kJoin>
__device__ __forceinline__ void walk2(const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                      const uint16_t* __restrict__ lo_tab, uint32_t P0, uint32_t N, uint32_t s0,
                                      uint32_t b, uint32_t e, uint32_t& pos_o, uint32_t& stop_o, uint32_t& cnt_o,
                                      uint64_t& mask_o, uint64_t& lo, uint64_t& hi, uint64_t omask, bool& joined,
                                      uint32_t& jq) {
    uint32_t pos = b, stop = kThrough, cnt = 0;
    uint64_t mask = 0;
    joined = false;
    jq = 0;
    WinCur c;
    wc_load(c, win32, P0 + b);
    bool run = b < e;
    // every step takes a code or stops, and a segment of <= 64 bits holds <= 13 codes
    for (uint32_t guard = 0; run; ++guard) {
        if (guard > 64u) {
            stop = kStuck;
            break;
        }
        const uint32_t i0 = pos - s0;  // < 64
        if (kJoin && ((omask >> i0) & 1ull)) {
            joined = true;
            jq = (uint32_t)__popcll(omask & ((1ull << i0) - 1ull));
            break;
        }
        mask |= 1ull << i0;
        const uint32_t d3 = wc_next(win32, c);
        const uint32_t w = wc_bits(c);
        const uint32_t rem = N - pos;
        const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
        const uint32_t kk = __clz(~w);
        const uint32_t el = lo_tab[min(kk, (uint32_t)HPK_LO_RUNS - 1u) * 32u + ((w << ((kk + 1u) & 31u)) >> 27)];
        const uint32_t l1 = HPK_L2_LEN0(e1), t1 = HPK_L2_LEN01(e1);
        const bool ok1 = (e1 < HPK_LUT2_NONE) & (l1 <= rem);
        const uint32_t i2 = i0 + l1;
        bool ok2 = ok1 & (e1 < HPK_LUT2_NOTTWO) & (t1 <= rem) & (s0 + i2 < e);  // the second code starts in the segment
        bool jn2 = false;
        if (kJoin) {
            jn2 = ok2 & (((omask >> (i2 & 63u)) & 1ull) != 0ull);
            ok2 &= !jn2;
        }
        const bool eos = (kk >= (uint32_t)HPK_LO_RUNS) | ((el & 0x1FFu) == HPK_EOS);
        const uint32_t llen = eos ? 30u : (el >> 9);
        const bool lng = !ok1 & (e1 >= HPK_LUT2_NONE) & (rem > (uint32_t)HPK_LUT_BITS);  // a 13..30-bit code (or EOS)
        const bool lok = lng & !eos & (llen <= rem);
        const uint32_t v = ok1 ? (ok2 ? ((e1 & 0xFFu) | ((e1 >> 8) & 0xFF00u)) : (e1 & 0xFFu)) : (lok ? (el & 0xFFu) : 0u);
        st128_put(lo, hi, cnt, v);
        cnt += ok1 ? (ok2 ? 2u : 1u) : (lok ? 1u : 0u);
        if (ok2) mask |= 1ull << i2;
        const bool stopped = !ok1 & !lok;
        // stopped: EOS decoded (huffman.rs:112-116), or the next code does not fit (the end: padding)
        stop = stopped ? ((lng & eos & (llen <= rem)) ? (uint32_t)kEos : (uint32_t)kEnded) : (uint32_t)kThrough;
        const uint32_t adv = ok1 ? (ok2 ? t1 : l1) : (lok ? llen : 0u);
        pos += adv;
        wc_adv(c, adv, d3);
        if (kJoin && jn2) {
            joined = true;
            jq = (uint32_t)__popcll(omask & ((1ull << i2) - 1ull));
            break;
        }
        run = !stopped & (pos < e);
    }
    pos_o = pos;
    stop_o = stop;
    cnt_o = cnt;
    mask_o = mask;
}

__device__ __forceinline__ void store8p(uint8_t* __restrict__ out8, bool ok, uint32_t pos, uint32_t v, uint32_t dmy,
                                        uint32_t oend, int kStore) {
    if (kStore == kPred)
        out8[ok ? pos : dmy] = (uint8_t)v;
    else if (ok)
        put8(out8, pos, v, oend, kStore);
}

// ------------------------------------------------------------------------------------------
// v18 segment stream (kCoop 3): the queue's head (the fill's longer literals) decoded by whole
// waves as ONE stream of 64-bit segments. A wave takes literals from the queue one after another
// and lays their segments side by side over its 64 lanes, chunk after chunk, so a literal's tail
// and the next literals share a chunk and every lane walks a segment. Within a chunk the lanes of
// one literal are contiguous; the first lane of a literal starts at a true code boundary (bit 0, or
// where the literal's previous chunk stopped). The others start speculatively at their segment
// start and resynchronise: lane j's true start is lane j-1's stop when that came through its
// segment. The lane then re-walks from there until it meets a code start of its current walk
// (join; at once when that walk passed the true start): its symbols are the re-walk's followed by
// the current walk's from the join on, and its stop stays. A lane whose re-walk never joins has a
// new stop, which corrects its right neighbour in the next round. A first lane's start is true, so
// round r fixes the literal's r-th lane at the latest; Huffman walks fall into step within a few
// codes, so most lanes join in round 1 after a few codes. Nothing is walked twice to write: a lane
// keeps its <= 13 symbols in registers; an exclusive scan of the counts gives its place in the
// image. A literal's end lane (its first lane that does not come through) writes its length and
// status; a literal still going at the chunk's end continues, at its true stop, in the wave's next
// chunk.
template <int kStore>
__device__ __forceinline__ void seg_stream(const uint2* __restrict__ q, uint32_t nq, uint32_t* ctr,
                                           const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                           const uint16_t* __restrict__ lo_tab, uint8_t* __restrict__ out8, uint32_t dmy,
                                           uint32_t* __restrict__ lenst, unsigned long long& nround,
                                           unsigned long long& nchunk) {
    const uint32_t j = threadIdx.x & 63u;
    // the wave's open literal, segments still to assign (wave-uniform, scalar registers)
    uint32_t c_ex = 0, c_ey = 0, c_nseg = 0, c_next = 0, c_opos = 0, c_base = 0;
    bool open = false, qdone = false;
    for (;;) {  // chunks
        // 1. lanes -> (literal, segment): the open literal's next segments, then new literals
        uint32_t fill = 0;
        uint32_t l_ex = 0, l_ey = 0, s0 = 0, b = 0, l_f = j, l_last = j, l_base = 0;
        uint32_t l_flags = 0;  // 1: has a segment, 2: the literal's first lane here, 4: more segments follow
        while (fill < 64u) {
            if (!open) {
                if (qdone) break;
                uint32_t t = 0;
                if (j == 0) t = atomicAdd(ctr, 1u);
                t = (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
                if (t >= nq) {
                    qdone = true;
                    break;
                }
                c_ex = (uint32_t)__builtin_amdgcn_readfirstlane((int)q[t].x);
                c_ey = (uint32_t)__builtin_amdgcn_readfirstlane((int)q[t].y);
                if (c_ey & kQ7Byte) continue;  // capacity below the bound: the byte pass
                c_nseg = ((c_ex >> 16) * 8u + 63u) >> 6;
                c_next = 0;
                c_opos = 0;
                c_base = 0;
                open = c_nseg != 0;
                if (!open) {  // an empty literal (not expected here): length 0, status OK
                    if (j == 0) lenst[c_ey & 0xFFFu] = 0;
                    continue;
                }
            }
            const uint32_t take = min(64u - fill, c_nseg - c_next);
            if (j >= fill && j < fill + take) {
                l_ex = c_ex;
                l_ey = c_ey;
                s0 = (c_next + (j - fill)) * 64u;
                b = j == fill ? c_base : s0;
                l_f = fill;
                l_last = fill + take - 1u;
                l_base = c_opos;
                l_flags = 1u | (j == fill ? 2u : 0u) | (c_next + take < c_nseg ? 4u : 0u);
            }
            fill += take;
            c_next += take;
            if (c_next == c_nseg) open = false;
        }
        if (fill == 0) break;
        nchunk += 1;
        const bool l_act = l_flags & 1u, l_ts = l_flags & 2u;
        // 2. speculative walks (the first lane of each literal from its true start)
        const uint32_t P0 = (l_ex & 0xFFFFu) * 8u, N = (l_ex >> 16) * 8u;
        const uint32_t e = s0 + 64u;
        // the lane's output: A (an bytes: a re-walk's head) then W's symbols from index bq on
        uint32_t wpos = 0, wstop = kEnded, wcnt = 0, an = 0, bq = 0;
        uint64_t wmask = 0, wlo = 0, whi = 0, alo = 0, ahi = 0;
        bool jn;
        uint32_t jq;
        if (l_act) walk2<false>(win32, lut, lo_tab, P0, N, s0, b, e, wpos, wstop, wcnt, wmask, wlo, whi, 0ull, jn, jq);
        bool bad = false;
        for (uint32_t round = 1;; ++round) {
            if (round > 65u) {
                bad = true;
                break;
            }
            const uint32_t lpos = __shfl_up(wpos, 1);
            const uint32_t lthr = __shfl_up((uint32_t)(wstop == kThrough), 1);
            const uint32_t nb = (!l_ts && lthr) ? lpos : b;
            const bool changed = l_act & (nb != b);
            if (!__any(changed)) break;
            nround += 1;
            if (changed) {
                b = nb;
                // fold A into W's symbols, then re-walk from nb into A until W's walk is met
                shr128(wlo, whi, 8u * bq);
                shl128(wlo, whi, 8u * an);
                wlo |= alo;
                whi |= ahi;
                wcnt = an + wcnt - bq;
                alo = ahi = 0;
                uint32_t rpos, rstop, rcnt;
                uint64_t rmask;
                walk2<true>(win32, lut, lo_tab, P0, N, s0, nb, e, rpos, rstop, rcnt, rmask, alo, ahi, wmask, jn, jq);
                if (jn) {  // rpos = the join: W's stop and its boundaries from there on stay
                    wmask = rmask | (wmask & ~((1ull << (rpos - s0)) - 1ull));
                    an = rcnt;
                    bq = jq;
                } else {
                    wpos = rpos;
                    wstop = rstop;
                    wcnt = rcnt;
                    wmask = rmask;
                    wlo = alo;
                    whi = ahi;
                    alo = ahi = 0;
                    an = 0;
                    bq = 0;
                }
            }
        }
        // 3. each literal ends in its first lane that does not come through
        const uint64_t nt = __ballot(!l_act | (wstop != kThrough));
        const uint64_t ntf = nt >> l_f;
        const uint32_t endl = ntf ? l_f + (uint32_t)__builtin_ctzll(ntf) : 64u;
        const bool ends = endl <= l_last || !(l_flags & 4u);  // the literal's end is in this chunk
        const uint32_t L = endl <= l_last ? endl : l_last;
        const uint32_t c = (l_act & (j <= L)) ? an + wcnt - bq : 0u;
        bad |= l_act & (j <= L) & (wstop == kStuck);
        shr128(wlo, whi, 8u * bq);
        shl128(wlo, whi, 8u * an);
        wlo |= alo;
        whi |= ahi;
        uint32_t P = c;  // inclusive scan over the wave, then made per literal
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(P, d);
            if (j >= (uint32_t)d) P += y;
        }
        const uint32_t Pf = __shfl(P, (int)(l_f == 0 ? 0u : l_f - 1u));
        const uint32_t before = l_f == 0 ? 0u : Pf;  // symbols of earlier literals in this chunk
        const uint32_t o0 = (l_ey >> 12) & 0x1FFFFu;
        const uint32_t dst = o0 + l_base + (P - c - before);
#pragma unroll
        for (int i = 0; i < 13; ++i) {
            const uint32_t v = (uint32_t)((i < 8 ? wlo >> (8 * i) : whi >> (8 * (i - 8))) & 0xFFull);
            store8p(out8, (uint32_t)i < c, dst + (uint32_t)i, v, dmy, o0 + N / 5u, kStore);
        }
        if (l_act & ends & (j == L)) {
            const uint32_t st = bad ? 0x7Fu
                                    : (wstop == kEos ? (uint32_t)HPK_EOS_IN_STRING
                                                     : residual_status(N - wpos, win_at(win32, P0 + wpos)));
            lenst[l_ey & 0xFFFu] = (l_base + P - before) | (st << 24);
        }
        // 4. the literal at the chunk's end, if it goes on: its true stop and bytes so far
        if (open) {
            const bool go_on = (uint32_t)__builtin_amdgcn_readlane((int)(ends ? 0u : 1u), 63) != 0u;
            if (go_on) {
                c_base = (uint32_t)__builtin_amdgcn_readlane((int)wpos, 63);
                c_opos = (uint32_t)__builtin_amdgcn_readlane((int)(l_base + P - before), 63);
            } else {
                open = false;  // it ended early (an error): its remaining segments are not decoded
            }
        }
    }
}

}  // namespace hpkdec

#include "../loona_amd/csrc/hpk_long.h"  // the long-literal phase (kLongK)

namespace hpkdec {

// ------------------------------------------------------------------------------------------

// kMode: 0 product; diagnostics (never the default): 1 no decode (fill structure only), 2 no
// output stores, 3 product + 16 per-wave stamps in a.dbg (cycles: total, in the decode loops,
// steps, waiting at the fill-top barrier, before the first fill, fill setup up to the entries,
// fill setup from there to the decode, in long literals, the first fill's two setup parts, the
// byte pass, the last write-back),
// 4 checked stores (g_chk), 5 product + per-wave counters of the long-literal phase in a.dbg.
// kCoop: 1 = long literals by whole waves (product), 0 = every literal by one lane (comparison).
// kSched: 0 = lanes take queue slots dynamically (ballot + per-wave reservations), 1 = static
// snake: lane i decodes slots i and 2*block-1-i of the longest-first queue, the second one's
// entry and window dwords prefetched while the first decodes (no refill stall).
// kLongDyn: 1 = a wave done with a long literal takes the next one from an LDS counter (the first
// kWaves are dealt statically), 0 = static round-robin.
// kDefer: 1 = the previous fill's write-back stores are issued from registers during this fill's
// decode, one slot per iteration; 0 = all of them between the two decodes.
// kPredSt: 1 = lane steps store every byte unconditionally (kPred), 0 = exec-masked stores.
// kSpread: 1 = the snake's queue slots interleaved over the waves and the lane phase before the
// long literals (which waves then take dynamically); 0 = contiguous slots per wave, long first.
// kSmallFill: a fill of at most this many literals also gives its literals of >= 64 encoded
// bytes to whole waves (0 = only >= 224 bytes, always).
// kLead: bits of lead-in walk before each speculative segment start of a long literal (0 = none).
// kEven: 1 = fills of about equal input size (fewest the window allows), 0 = greedy full windows.
template <int kMode, int kWaves, int kW, int kO, int kQ, int kRefillN, int kChunk, int kLook, bool kAcc,
          int kCoop = 1, int kSched = 0, int kLongDyn = 1, int kDefer = 1, int kPredSt = 1, int kSpread = 0,
          int kSmallFill = 512, uint32_t kLead = 0, int kEven = 1, int kSegBig = 15, int kSegSmall = 32,
          int kLongK = 0>
__global__ __launch_bounds__(kWaves * 64) void hpk_decode12(DecodeArgs a) {
    using G = Geo12<kWaves, kW, kO, kQ>;
    constexpr int R = G::kMetaRounds, S = G::kStageRounds;
    constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : (kPredSt ? kPred : kDword));
    // v21: body steps without fit tests, the literals' last bits in a checked tail pass (lit12_fast)
    constexpr bool kFast = HPK_FAST && kStore == kPred && !kAcc && kLook == 2 && !HPK_RELOAD && !kDefer;
    // v22: lengths and statuses of the lane literals made after the lane loop (HPK_LATE_FIN)
    constexpr bool kLate = HPK_LATE_FIN && !kFast && kStore == kPred && !kAcc && !HPK_RELOAD && !kDefer && !kSpread;
    // the next fill's prefetch issued from the lane loop, a load per round (HPK_PF_LOOP)
    constexpr bool kPfLoop = HPK_PF_LOOP && kLate;
    // HPK_FLUSH_LOOP: the previous fill's last S write-back rounds are read into the window-prefetch
    // registers (free once the window is in LDS) and stored from the lane loop, before the window's
    // prefetch loads reuse those registers
    constexpr int kFD = kPfLoop ? (HPK_FLUSH_LOOP < S ? HPK_FLUSH_LOOP : S) : 0;
    // groups of one fill prefetch: a round of offsets each, the deferred write-back rounds, the window
    constexpr int kPfN = R + kFD + 1;
    // the previous fill's write-back issued at the top of a fill, before its setup (HPK_FLUSH_TOP)
    constexpr bool kFlushTop = HPK_FLUSH_TOP && !kDefer;
    // kPred: the image's last 256 bytes are the lanes' dummy slots (one dword apart), not output
    constexpr int kImg = kStore == kPred ? kO - 256 : kO;
    const uint32_t dmy = (uint32_t)kImg + (threadIdx.x & 63u) * 4u;
    static_assert(kChunk >= 64, "a refill can hand out 64 slots");
    unsigned long long t_start = 0, t_dec = 0, n_steps = 0, n_fills = 0, t_pre = 0, t_setA = 0, t_setB = 0, t_long = 0,
                       t_A0 = 0, t_B0 = 0, t_tail = 0, t_byte = 0, t_rounds = 0, n_longs = 0, t_sb1 = 0, t_sb2 = 0,
                       t_sb3 = 0;
    if (kMode == 3) t_start = __builtin_amdgcn_s_memtime();
    __shared__ __attribute__((aligned(16))) uint8_t smem[G::kLdsBytes];
    uint16_t* s_lo = reinterpret_cast<uint16_t*>(smem + kT8Bytes);
    uint32_t* s_lut = reinterpret_cast<uint32_t*>(smem + G::kLutOff);
    uint8_t* s_in = smem + G::kInOff;
    const uint32_t* win32 = reinterpret_cast<const uint32_t*>(s_in);
    uint8_t* s_out = smem + G::kOutOff;
    uint32_t* s_out32 = reinterpret_cast<uint32_t*>(s_out);
    uint2* s_q = reinterpret_cast<uint2*>(smem + G::kQOff);
    uint32_t* s_lenst = reinterpret_cast<uint32_t*>(smem + G::kLenOff);  // len | status << 24
    uint32_t* s_hist = reinterpret_cast<uint32_t*>(smem + G::kHistOff);
    uint32_t* s_bbase = s_hist + 64;
    // [0] fitting count, [1] lane-queue head, [2] input end of the fill, [3] output end of the
    // fill, [4] long-queue head
    uint32_t* s_ctr = reinterpret_cast<uint32_t*>(smem + G::kCtrOff);
    for (uint32_t t = threadIdx.x; t < kLoBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];
    for (uint32_t t = threadIdx.x; t < (uint32_t)G::kLutBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lut)[t] = reinterpret_cast<const uint4*>(a.lut2)[t];

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
#if HPK_DEC_SPLIT
    // the workgroup's literals: equal encoded bytes (+ 8 per literal) per workgroup (the lane
    // queue's LDS holds the search's counters; it is set up after)
    uint32_t BA, BB;
    hpksplit::split_by_bytes<G::kBlock, 8>(a.in_off, a.n, reinterpret_cast<uint32_t*>(s_q), BA, BB);
    __syncthreads();
#else
    const uint32_t BA = (uint32_t)((uint64_t)a.n * blockIdx.x / gridDim.x);
    const uint32_t BB = (uint32_t)((uint64_t)a.n * (blockIdx.x + 1) / gridDim.x);
#endif
    // offsets are clamped to the input capacity wherever they bound a read, so bad offsets (caught
    // per fill below) never move a window past the blob
    const uint32_t in_end = min(a.in_off[a.n], a.in_cap) + a.in_mis;
    const uint32_t last16 = in_end ? (in_end - 1) >> 4 : 0;  // last 16-B chunk holding a batch byte
    // last chunk holding a byte of THIS workgroup's literals: windows never read past it
    const uint32_t r_end = min(min(a.in_off[BB], a.in_cap) + a.in_mis, in_end);
    const uint32_t rlast16 = r_end ? (r_end - 1) >> 4 : 0;
    // kEven: the range is cut into the fewest fills the window allows, of about equal input size
    // (a greedy cut leaves a small last fill that still costs a whole fill's setup, slowest literal
    // and write-back); the effective window is that size plus a margin for literal granularity
    uint32_t kWe = (uint32_t)kW;
    uint32_t kW0 = kWe;  // the first fill's window
    if (kEven) {
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
    // kDefer: the same write-back in two halves. flush_read takes the previous fill's image chunks,
    // lengths and end bytes into registers before this fill decodes over the image; flush_slot(s)
    // issues slot s of their stores (s < F: image round s, s == F: lengths, statuses, end bytes),
    // one slot per decode iteration, so the stores drain while the fill decodes instead of
    // stalling every wave at once between two decodes.
    constexpr int F = G::kFlushRounds;
    constexpr int kDefer0 = HPK_DEFER0;  // image rounds [0, kDefer0) are stored by flush_read itself
    static_assert(F <= 16 && R <= 15, "flush slot bits");
    uint4 f_c[F];
    uint32_t f_lv[R];
    uint32_t f_mask = 0, f_pv = 0, f_px = 0;  // bit r: chunk r; bit 16 + r: length r; bit 31: end byte
    uint32_t f_c0 = 0, f_cur = 0;
    int fs = F + 1;  // next slot to issue (F + 1: nothing pending); wave-uniform
    auto flush_read = [&](uint32_t fcur, uint32_t fk, uint32_t G0, uint32_t G1) {
        const uint32_t ob = G0 & ~15u;
        const uint32_t c0 = ob >> 4, c1 = (G1 + 15) >> 4;
        f_c0 = c0;
        f_cur = fcur;
        f_mask = 0;
        if (kMode != 2) {
            const uint4* l16 = reinterpret_cast<const uint4*>(s_out);
#pragma unroll
            for (int r = 0; r < F; ++r) {
                const uint32_t ci = c0 + tid + (uint32_t)G::kBlock * r;
                if (ci < c1 && (ci << 4) >= G0 && (ci << 4) + 16u <= G1) {
                    if (r < kDefer0) {  // the first rounds go out now
                        reinterpret_cast<uint4*>(a.out_base)[ci] = l16[ci - c0];
                    } else {
                        f_c[r] = l16[ci - c0];
                        f_mask |= 1u << r;
                    }
                }
            }
            if (tid < 32) {
                const uint32_t g = tid < 16 ? c0 << 4 : (c1 - 1) << 4;
                const bool partial = !(g >= G0 && g + 16u <= G1) && (tid < 16 || c1 - 1 != c0);
                const uint32_t x = g + (tid & 15u);
                if (partial && x >= G0 && x < G1) {
                    f_pv = s_out[x - ob];
                    f_px = x;
                    f_mask |= 1u << 31;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t i = tid + (uint32_t)G::kBlock * r;
            if (i < fk) {
                f_lv[r] = s_lenst[i];
                f_mask |= 1u << (16 + r);
            }
        }
        fs = 0;
    };
    auto flush_slot = [&](int s) {
        uint4* g16 = reinterpret_cast<uint4*>(a.out_base);
#pragma unroll
        for (int r = 0; r < F; ++r)
            if (s == r && ((f_mask >> r) & 1u)) g16[f_c0 + tid + (uint32_t)G::kBlock * r] = f_c[r];
        if (s == F) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if ((f_mask >> (16 + r)) & 1u) {
                    const uint32_t i = f_cur + tid + (uint32_t)G::kBlock * r;
                    a.out_len[i] = f_lv[r] & 0xFFFFFFu;
                    a.status[i] = (uint8_t)(f_lv[r] >> 24);
                }
            }
            if (f_mask >> 31) a.out_base[f_px] = (uint8_t)f_pv;
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
            if (HPK_FD_FIRST ? r >= kFD : r < G::kFlushRounds - kFD) {
                if (ok) g16[ci] = l16[ci - c0];
            } else if (kFD) {
                const int d = HPK_FD_FIRST ? r : r - (G::kFlushRounds - kFD);
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
    // kLongK: long literals left to the long-literal phase are listed in a.long_list[BA, BB): those of
    // >= long_big encoded bytes from the front, the others from the back (counts in s_ctr[6], [7])
    auto leave = [&](uint32_t i, uint32_t nb) {
        if (nb >= a.long_big)
            a.long_list[BA + atomicAdd(&s_ctr[6], 1u)] = i;
        else
            a.long_list[BB - 1u - atomicAdd(&s_ctr[7], 1u)] = i;
    };
    if (kLongK) {
        if (tid == 0) {
            s_ctr[6] = 0;
            s_ctr[7] = 0;
            s_ctr[8] = 0;
            s_ctr[9] = 0;
        }
    }

    uint32_t cur = BA;
    uint32_t gin = 0, gout = 0;  // exact input / output start of the fill (blob-relative + mis)
    if (cur < BB) {
        gin = a.in_off[cur] + a.in_mis;
        gout = a.out_off[cur] + a.out_mis;
        prefetch_fill<G::kBlock>(P, a, tid, cur, min(cur + (uint32_t)kQ, BB), gin & ~15u, rlast16);
    }
    if (kMode == 3) t_pre = __builtin_amdgcn_s_memtime() - t_start;
    bool dense_tried = false;  // block-uniform (kLongK): the range's first fill was checked
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
        const uint32_t lcnt6 = kLongK ? s_ctr[6] : 0u, lcnt7 = kLongK ? s_ctr[7] : 0u;
        if (kFlushTop && pk) {  // the previous fill's write-back first: its stores drain under this setup
            flush(pcur, pk, pG0, pG1);
            pk = 0;
        }
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
        uint32_t dlb = 0, dtb = 0;  // (kLongK, first fill) long-literal bytes and all bytes of the candidates
        bool bad = false;  // a literal of this fill's range with decreasing offsets or offsets past a capacity
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const uint32_t t = tid + (uint32_t)G::kBlock * r;
            if (kLongK && !dense_tried) {
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
                const bool fast = ocap >= (nbytes * 8u) / 5u && (!kAcc || ((o0 | ocap) & 3u) == 0);
                ex[r] = (p0 - base16) | (nbytes << 16);
                ey[r] = t | ((o0 - ob16) << 12) | (fast ? 0u : kQ7Byte);
                if (kLongK && fast && nbytes >= a.long_min) {  // hpk_decode_long's (not queued here)
                    leave(cur + t, nbytes);
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
        if (kLongK && !dense_tried) {
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
                if (kLongK) {  // this fill's long literals are void too: not for the long-literal phase
                    s_ctr[6] = lcnt6;
                    s_ctr[7] = lcnt7;
                }
            }
            break;
        }
        if (kLongK && !dense_tried) {
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
                    s_ctr[10] = 0;
                }
                lds_barrier();
                bool no = false;
                for (uint32_t i = BA + tid; i < BB; i += G::kBlock) {
                    const uint32_t p0 = a.in_off[i], p1 = a.in_off[i + 1], q0 = a.out_off[i], q1 = a.out_off[i + 1];
                    const bool ok = p0 <= p1 && p1 <= a.in_cap && q0 <= q1 && q1 <= a.out_cap &&
                                    (uint64_t)(q1 - q0) >= (uint64_t)(p1 - p0) * 8u / 5u;
                    if (ok)
                        leave(i, p1 - p0);
                    else
                        no = true;
                }
                if (__any(no) && lane == 0) s_ctr[10] = 1u;
                lds_barrier();
                if (s_ctr[10] == 0) {
                    cur = BB;  // all listed
                    break;
                }
                lds_barrier();
                if (tid == 0) {
                    s_ctr[6] = 0;
                    s_ctr[7] = 0;
                }
                continue;  // this fill again, from its setup (its prefetched offsets and window are still
                           // in the registers)
            }
        }
        const uint32_t k = s_ctr[0];
        if (k == 0) {  // literal `cur` alone exceeds the window: one lane decodes it from global
            bool left = false;
            if (kLongK) {  // (unless it is hpk_decode_long's)
                const uint32_t nb = a.in_off[cur + 1] - a.in_off[cur];
                left = nb >= a.long_min && a.out_off[cur + 1] - a.out_off[cur] >= (nb * 8u) / 5u;
                if (left && tid == 0) leave(cur, nb);
            }
            if (tid == 0 && !left) {
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
        // queue entries: the fill's literals less those left to hpk_decode_long (kLongK)
        const uint32_t kq = kLongK ? (uint32_t)__builtin_amdgcn_readfirstlane((int)(s_bbase[63] + s_hist[63])) : k;
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (pos[r] != 0xFFFFFFFFu) s_q[s_bbase[pos[r] >> 16] + (pos[r] & 0xFFFFu)] = make_uint2(ex[r], ey[r]);
        // the queue's head goes to whole waves: literals of >= 224 bytes; in a fill of few literals
        // (long ones fill the window: lanes would idle) also those of >= 64 bytes (kSmallFill)
        // (kCoop 3, the segment stream: literals of the first kSegBig buckets, kSegSmall in a small fill;
        // bucket b < 48 holds encoded lengths >= 2 (48 - b) + ... : 15 = >= 224 B, 32 = >= 64 B, 48 = >= 32 B)
        const uint32_t lb = kCoop == 3 ? ((kSmallFill && k <= (uint32_t)kSmallFill) ? (uint32_t)kSegSmall : (uint32_t)kSegBig)
                                       : ((kSmallFill && k <= (uint32_t)kSmallFill) ? 32u : kLongBuckets);
        const uint32_t nlong = kCoop ? (uint32_t)__builtin_amdgcn_readfirstlane((int)s_bbase[lb]) : 0u;
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
                                                                 (uint32_t)G::kBlock * (HPK_FD_FIRST ? d : G::kFlushRounds - kFD + d)] =
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
        if (!kFlushTop && pk) {
            if (kDefer)
                flush_read(pcur, pk, pG0, pG1);
            else if (kFD)
                flush_split(pcur, pk, pG0, pG1);
            else
                flush(pcur, pk, pG0, pG1);
        }
        pk = k;
        pcur = cur;
        pG0 = gout;
        pG1 = gout_next;
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
        // long literals first (longest-first): one wave each, the first kWaves dealt round-robin,
        // then taken from an LDS counter as waves come free. Everything that steers this loop is
        // wave-uniform and held in scalar registers (readlane of lane 0, never a branch on a vector
        // value): a divergent loop would run long_decode's cross-lane operations under a partial
        // exec mask.
        // (the long-literal phase and the lane phase are lambdas so that with kDefer the phase
        // holding the write-back registers is a separate code path: long_decode never runs with
        // them live, and the decode keeps its registers)
        auto long_phase = [&]() {
            if (kCoop == 3 && kMode != 1 && nlong) {
                seg_stream<kStore>(s_q, nlong, &s_ctr[4], win32, s_lut, s_lo, s_out, dmy, s_lenst, t_rounds, n_longs);
            } else if (kMode != 1 && nlong) {
                const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
                for (uint32_t jl = wv; jl < nlong;) {
                    const uint32_t ex = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q[jl].x);
                    const uint32_t ey = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_q[jl].y);
                    if (!(ey & kQ7Byte)) {  // (capacity below the bound: the byte pass below)
                        uint32_t len, st, nr;
                        long_decode<kLead>(win32, s_lut, s_lo, s_out, kStore, (ex & 0xFFFFu) * 8u, (ex >> 16) * 8u,
                                           (ey >> 12) & 0x1FFFFu, len, st, nr);
                        if (kMode == 3) {
                            t_rounds += nr;
                            n_longs += 1;
                        }
                        if (lane == 0) s_lenst[ey & 0xFFFu] = len | (st << 24);
                    }
                    if (kLongDyn) {  // the next long literal: one LDS atomic per wave, read from lane 0
                        uint32_t nx = 0;
                        if (lane == 0) nx = atomicAdd(&s_ctr[4], 1u) + (uint32_t)kWaves;
                        jl = (uint32_t)__builtin_amdgcn_readlane((int)nx, 0);
                    } else {
                        jl += kWaves;
                    }
                }
            }
            if (kMode == 3) t_long += __builtin_amdgcn_s_memtime() - td0;
        };
        const uint32_t kl = kq - nlong;  // lane-queue entries s_q[nlong, kq)
        auto lane_phase = [&](auto dtag) {
            constexpr bool D = decltype(dtag)::value;  // issue write-back slots from the loop
            if (kMode != 1 && kl && kSched == 0) {
                const uint2* lq = s_q + nlong;
                Lit12 L;
                uint32_t t = tid;
                uint32_t qb = 0, qe = 0;  // queue slots reserved by this wave, not yet handed out
                // Branch-free (re)start: lanes past the queue read a clamped entry and stay idle (no
                // bits: rem = 0). The loop has no divergent exits, so the ballots see the whole wave.
                auto begin = [&](uint32_t tt) {
                    const uint2 e = lq[min(tt, kl - 1)];
                    L.act = tt < kl && !(e.y & kQ7Byte);
                    L.idx = e.y & 0xFFFu;
                    const uint32_t nb = e.x >> 16;
                    const uint32_t ob = (e.y >> 12) & 0x1FFFFu;
                    L.X = (e.x & 0xFFFFu) * 8u + 31u;
                    L.Eb = L.X + (L.act ? nb * 8u : 0u);
                    L.o = kAcc ? ob >> 2 : ob;
                    L.o0 = ob;
                    L.oend = kAcc ? (ob + nb * 8u / 5u + 3u) >> 2 : ob + nb * 8u / 5u;
                    L.cnt = 0;
                    L.acc = 0;
                    L.accn = 0;
                    L.st = HPK_OK;
                    L.prog = false;
                    lit12_load(L, win32);
                };
                begin(t);
                for (;;) {
    #pragma unroll
                    for (int s = 0; s < kRefillN; ++s) lit12_step<kStore, kLook, kAcc>(L, win32, s_lut, s_lo, s_out, dmy);
                    if (kMode == 3) n_steps += kRefillN;
                    const bool fin = t < kl && !L.prog;
                    if (__any(fin)) {
                        if (fin && L.act) {
                            if (kAcc && L.accn) put32(s_out32, L.o, L.acc, L.oend, kStore);
                            s_lenst[L.idx] = (kAcc ? L.cnt : L.o - L.o0) | (lit12_status(L, win32) << 24);
                        }
                        const bool free_lane = fin || t >= kl;
                        const uint64_t fm = __ballot(free_lane);
                        const uint32_t rank =
                            __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                        // free lanes take the wave's reserved slots [qb, qe) in rank order; when those
                        // run short the wave reserves kChunk more with one LDS atomic
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
                    if (!__any(t < kl)) break;
                }
            }
            if (kMode != 1 && kl && kSched == 1) {
                static_assert(kSched != 1 || kQ <= 2 * G::kBlock, "static snake: two literals per lane at most");
                const uint2* lq = s_q + nlong;
                Lit12 L, N;  // the literal being decoded and the lane's next one (prefetched)
                auto load = [&](Lit12& T, uint32_t tt) {
                    const uint2 e = lq[min(tt, kl - 1)];
                    T.act = tt < kl && !(e.y & kQ7Byte);
                    T.idx = e.y & 0xFFFu;
                    const uint32_t nb = e.x >> 16;
                    const uint32_t ob = (e.y >> 12) & 0x1FFFFu;
                    T.X = (e.x & 0xFFFFu) * 8u + 31u;
                    T.Eb = T.X + (T.act ? nb * 8u : 0u);
                    T.o = kAcc ? ob >> 2 : ob;
                    T.o0 = ob;
                    T.oend = kAcc ? (ob + nb * 8u / 5u + 3u) >> 2 : ob + nb * 8u / 5u;
                    T.cnt = 0;
                    T.acc = 0;
                    T.accn = 0;
                    T.st = HPK_OK;
                    T.prog = false;
                    lit12_load(T, win32);
                };
                // kSpread: consecutive queue slots go to different waves (slot = lane * kWaves + wave),
                // so a short lane queue (few literals below the long threshold) still reaches every wave
                const uint32_t t1 = kSpread ? (tid & 63u) * (uint32_t)kWaves + (tid >> 6) : tid;
                load(L, t1);
                const uint32_t t2 = 2u * G::kBlock - 1u - t1;
                bool nv = t2 < kl;  // a second literal is waiting in N
                load(N, t2);
                if (kFast) {
                    // body steps until every lane's literals have stopped (the first one's stopped state
                    // moves to N when the second starts), then both tails with the checked step, the two
                    // lanes' walks interleaved
                    for (;;) {
    #pragma unroll
                        for (int s = 0; s < kRefillN; ++s) lit12_fast(L, win32, s_lut, s_lo, s_out, dmy);
                        if (kMode == 3) n_steps += kRefillN;
                        const bool fin = !L.prog;
                        if (__any(fin)) {
                            const bool sw = fin & nv;
                            if (sw) {
                                const Lit12 T = L;
                                L = N;
                                N = T;
                                nv = false;
                            }
                            if (!__any(!fin | sw)) break;
                        }
                    }
                    for (;;) {
                        lit12_step<kStore, kLook, kAcc>(L, win32, s_lut, s_lo, s_out, dmy);
                        lit12_step<kStore, kLook, kAcc>(N, win32, s_lut, s_lo, s_out, dmy);
                        if (!__any(L.prog | N.prog)) break;
                    }
                    if (L.act) s_lenst[L.idx] = (L.o - L.o0) | (lit12_status(L) << 24);
                    if (N.act) s_lenst[N.idx] = (N.o - N.o0) | (lit12_status(N) << 24);
                }
                if (kLate) {
                    // v22: a lane's first literal that ends leaves only its end state (bit and output
                    // positions, walk status) in three registers as the second one starts; lengths and
                    // statuses (the padding check) are made once per lane after the loop, not in every
                    // finish round a wave takes (a round ran the check whenever any of its lanes finished)
                    uint32_t sX = 0, sO = 0, sSt = 0;
                    bool s1 = false;  // the first literal's end state is saved
                    for (;;) {
    #pragma unroll
                        for (int s = 0; s < kRefillN; ++s) lit12_step<kStore, kLook, kAcc>(L, win32, s_lut, s_lo, s_out, dmy);
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
                }
                for (; !kFast && !kLate;) {
    #pragma unroll
                    for (int s = 0; s < kRefillN; ++s) lit12_step<kStore, kLook, kAcc>(L, win32, s_lut, s_lo, s_out, dmy);
                    if (kMode == 3) n_steps += kRefillN;
                    if (D && fs <= F) flush_slot(fs++);
                    const bool fin = !L.prog;  // no progress in the last step: finished (or idle)
                    if (__any(fin)) {
                        if (fin && L.act) {
                            if (kAcc && L.accn) put32(s_out32, L.o, L.acc, L.oend, kStore);
                            s_lenst[L.idx] = (kAcc ? L.cnt : L.o - L.o0) | (lit12_status(L, win32) << 24);
                        }
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
        };
        if (kDefer) {
            if (nlong) {  // write-back first, then the long literals
                while (fs <= F) flush_slot(fs++);
                long_phase();
                lane_phase(std::false_type{});
            } else {
                lane_phase(std::true_type{});
            }
        } else if (kSpread) {  // lane literals first; waves then take long literals as they come free
            lane_phase(std::false_type{});
            long_phase();
        } else {
            long_phase();
            lane_phase(std::false_type{});
        }
        if (kDefer)
            while (fs <= F) flush_slot(fs++);  // what the decode loops did not issue
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
        a.dbg[gwi * 16 + 7] = t_long;
        a.dbg[gwi * 16 + 8] = t_A0;
        a.dbg[gwi * 16 + 9] = t_B0;
        a.dbg[gwi * 16 + 10] = t_byte;
        a.dbg[gwi * 16 + 11] = t_end - t_tail;
        a.dbg[gwi * 16 + 12] = kCoop ? t_rounds : t_sb1;
        a.dbg[gwi * 16 + 13] = kCoop ? n_longs : t_sb2;
        a.dbg[gwi * 16 + 14] = t_sb3;
    }
    if constexpr (kLongK != 0) {  // the literals this workgroup left to the long-literal phase
        lds_barrier();
        if (tid == 0) s_ctr[5] = 0;  // its claim counter
        __syncthreads();  // (every thread's list entries and stores are out)
        static_assert(!kLongK || (kW + kO >= 512 * (32 * 4 + HPK_LONG_OS) && G::kInOff % 16 == 0 && kW % 16 == 0),
                      "long-phase LDS");
        long_phase<512, 8, 32, kMode == 5 ? 1 : 0, G::kBlock>(a, BA, BB, s_ctr[6], s_ctr[7], &s_ctr[5],
                                                              reinterpret_cast<uint32_t*>(s_in), s_in + 512 * 32 * 4,
                                                              reinterpret_cast<uint4*>(s_q), s_lut, s_lo);
    }
}

}  // namespace hpkdec
