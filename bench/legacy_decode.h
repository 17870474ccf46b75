// legacy_decode.h — earlier decode kernels kept for comparison runs in bench/kvariants (never
// built into libhpk.so): hpk_decode_kernel (v3-v5: block window + block queue) and hpk_decode7
// (v7-v10: LDS image, longest-first queue, pipelined fills). The product kernel is
// hpk_decode12 (loona_amd/csrc/hpk_decode12.h); the building blocks they share stay in
// loona_amd/csrc/hpk_decode_kernel.h.
#pragma once
#include "../loona_amd/csrc/hpk_decode_kernel.h"

namespace hpkdec {

// lane-walk steps of v3-v10
template <int kStore>
__device__ __forceinline__ void lit_emit(Lit& L, uint32_t packed, uint32_t g, uint8_t* __restrict__ out8) {
    L.acc |= (uint64_t)packed << (8u * L.accn);
    L.accn += g;
    L.cnt += g;
    if (L.accn >= 4u) {
        if (kStore == kDword) {
            reinterpret_cast<uint32_t*>(out8)[L.od] = (uint32_t)L.acc;
        } else if (kStore == kChecked) {
            if (L.od < L.oend)
                reinterpret_cast<uint32_t*>(out8)[L.od] = (uint32_t)L.acc;
            else
                chk_report(1, L.od, L.oend, L.cnt);
        } else {
            asm volatile("" ::"v"((uint32_t)L.acc));
        }
        L.od += 1;
        L.acc >>= 32;
        L.accn -= 4u;
    }
}

// One step: refill, then 4 codes decoded speculatively as if all were 5..8-bit codes: lengths
// from the canonical limits (no memory access on the serial chain), symbols from T8 off that
// chain, running bit offsets c1..c4. The valid prefix (fast code, ends inside the literal, lane
// live) is then consumed and emitted with a handful of selects. The first invalid code either
// runs past the literal's end (only padding left: the lane stops) or is a 10..30-bit code / EOS:
// the lane "parks" and that one code is decoded with the leading-ones table (one branch per
// step, taken only when some lane needs it).
template <int kStore, class Src>
__device__ __forceinline__ void lit_step(Lit& L, const Src& src, const uint8_t* __restrict__ t8,
                                         const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8) {
    lit_refill(L, src);  // >= 32 bits loaded: four 8-bit codes fit
    uint64_t x = L.win;
    uint32_t c[5], sym[4];
    bool fast[4];
    c[0] = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t w = (uint32_t)(x >> 32);
        const uint32_t len = 5u + (w >= HPK_LIM5) + (w >= HPK_LIM6) + (w >= HPK_LIM7);
        fast[i] = w < HPK_LIM8;
        sym[i] = t8[w >> 24];
        c[i + 1] = c[i] + len;
        x <<= len;
    }
    // valid prefix: m_i = lane live and codes 0..i are fast and end inside the literal
    const bool m0 = L.live && fast[0] && c[1] <= L.rem;
    const bool m1 = m0 && fast[1] && c[2] <= L.rem;
    const bool m2 = m1 && fast[2] && c[3] <= L.rem;
    const bool m3 = m2 && fast[3] && c[4] <= L.rem;
    const uint32_t use = m3 ? c[4] : m2 ? c[3] : m1 ? c[2] : m0 ? c[1] : 0u;
    const uint32_t g = m3 ? 4u : m2 ? 3u : m1 ? 2u : m0 ? 1u : 0u;
    // the first invalid code: a long code (park for the LO lookup) or the literal's end
    const bool bad_fast = m2 ? fast[3] : m1 ? fast[2] : m0 ? fast[1] : fast[0];
    const bool park = L.live && !m3 && !bad_fast;
    L.win <<= use;
    L.nb -= use;
    L.rem -= use;
    uint32_t packed = sym[0] | (sym[1] << 8) | (sym[2] << 16) | (sym[3] << 24);
    packed &= g >= 4u ? 0xFFFFFFFFu : ((1u << (8u * g)) - 1u);
    lit_emit<kStore>(L, packed, g, out8);
    L.live = park || (m3 && L.rem != 0u);
    if (park) {  // a 10..30-bit code (or EOS): one lookup in the leading-ones table
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
            lit_emit<kStore>(L, s1, 1u, out8);
            L.live = L.rem != 0u;
        }
    }
}

// Append g (<= 4) bytes to the pending output, garbage-tolerant: bytes of acc above the accn
// valid ones may hold anything (they are masked here before new bytes land on them, and the
// final partial dword only writes inside the literal's own output region, whose bytes past
// out_len are unspecified by the ABI).
template <int kStore>
__device__ __forceinline__ void lit_emit_g(Lit& L, uint32_t packed, uint32_t g, uint8_t* __restrict__ out8) {
    const uint32_t sh = 8u * L.accn;  // accn <= 3 here
    const uint64_t add = (uint64_t)packed << sh;
    const uint32_t lo = ((uint32_t)L.acc & __builtin_amdgcn_ubfe(0xFFFFFFFFu, 0, sh)) | (uint32_t)add;
    L.acc = ((uint64_t)(uint32_t)(add >> 32) << 32) | lo;
    L.accn += g;
    L.cnt += g;
    if (L.accn >= 4u) {
        if (kStore == kDword) {
            reinterpret_cast<uint32_t*>(out8)[L.od] = (uint32_t)L.acc;
        } else if (kStore == kChecked) {
            if (L.od < L.oend)
                reinterpret_cast<uint32_t*>(out8)[L.od] = (uint32_t)L.acc;
            else
                chk_report(1, L.od, L.oend, L.cnt);
        } else {
            asm volatile("" ::"v"((uint32_t)L.acc));
        }
        L.od += 1;
        L.acc >>= 32;
        L.accn -= 4u;
    }
}

// v6 step: the same speculative 4-code decode as lit_step, in 32-bit arithmetic. Code i starts
// at bit c_i = 5i + e_i of the window's top dword (e_i = extra bits of codes 0..i-1 over 5).
// Its 5-bit prefix t_i alone fixes the 5..8-bit length (the canonical limits 0x50/0xB8/0xF8
// end in three zero bits, i.e. t >= 10, 23, 31), so len_i - 5 = popcount(M << (31 - t_i)) with
// M = bits {10, 23, 31}, and 31 - t_i is a bit-field extract of ~hi pre-shifted by 5i: the
// serial chain per code is extract, shift, popcount, subtract. Symbols and the fast test read
// the 8-bit prefix off the chain. f_i = 27 - e_i.
template <int kStore, class Src>
__device__ __forceinline__ void lit_step6(Lit& L, const Src& src, const uint8_t* __restrict__ t8,
                                          const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8) {
    lit_refill(L, src);
    constexpr uint32_t M = (1u << 10) | (1u << 23) | (1u << 31);
    const uint32_t hi = (uint32_t)(L.win >> 32);
    const uint32_t nh = ~hi;
    uint32_t f[5], sym[4];
    bool fast[4], fits[4];
    f[0] = 27;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = __builtin_amdgcn_ubfe(nh << (5 * i), f[i], 5);  // 31 - t_i
        f[i + 1] = f[i] - (uint32_t)__builtin_popcount(M << s);
        const uint32_t b = __builtin_amdgcn_ubfe(hi, f[i] - (3 + 5 * i), 8);
        fast[i] = b < 0xFEu;
        sym[i] = t8[b];
        // code i ends inside the literal: c_{i+1} = 5(i+1) + 27 - f_{i+1} <= rem
        fits[i] = f[i + 1] + L.rem >= 32u + 5u * i;
    }
    const bool m0 = L.live && fast[0] && fits[0];
    const bool m1 = m0 && fast[1] && fits[1];
    const bool m2 = m1 && fast[2] && fits[2];
    const bool m3 = m2 && fast[3] && fits[3];
    const uint32_t g = (uint32_t)m0 + (uint32_t)m1 + (uint32_t)m2 + (uint32_t)m3;
    const uint32_t fg = m3 ? f[4] : m2 ? f[3] : m1 ? f[2] : m0 ? f[1] : 27u;
    const uint32_t use = 5u * g + 27u - fg;
    const bool bad_fast = m2 ? fast[3] : m1 ? fast[2] : m0 ? fast[1] : fast[0];
    const bool park = L.live && !m3 && !bad_fast;
    L.win <<= use;
    L.nb -= use;
    L.rem -= use;
    const uint32_t packed = sym[0] | (sym[1] << 8) | (sym[2] << 16) | (sym[3] << 24);
    lit_emit_g<kStore>(L, packed, g, out8);
    L.live = park || (m3 && L.rem != 0u);
    if (park) {  // a 10..30-bit code (or EOS): one lookup in the leading-ones table
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

// v7 step: lit_step6 without the in-step branch. A lane whose next code is longer than 8 bits
// (~0.8 % of header-value codes, but with 64 lanes x ~3.5 codes per step ~80 % of wave-steps
// saw one) parks and idles until the wave's next refill point, where all parked lanes take
// their leading-ones lookup together (lit_unpark): one branch per kRefillN steps.
template <int kStore, class Src>
__device__ __forceinline__ void lit_step7(Lit& L, const Src& src, const uint8_t* __restrict__ t8,
                                          uint8_t* __restrict__ out8) {
    lit_refill(L, src);
    constexpr uint32_t M = (1u << 10) | (1u << 23) | (1u << 31);
    const uint32_t hi = (uint32_t)(L.win >> 32);
    const uint32_t nh = ~hi;
    uint32_t f[5], sym[4];
    bool fast[4], fits[4];
    f[0] = 27;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = __builtin_amdgcn_ubfe(nh << (5 * i), f[i], 5);  // 31 - t_i
        f[i + 1] = f[i] - (uint32_t)__builtin_popcount(M << s);
        const uint32_t b = __builtin_amdgcn_ubfe(hi, f[i] - (3 + 5 * i), 8);
        fast[i] = b < 0xFEu;
        sym[i] = t8[b];
        fits[i] = f[i + 1] + L.rem >= 32u + 5u * i;
    }
    const bool run = L.live && !L.park;
    const bool m0 = run && fast[0] && fits[0];
    const bool m1 = m0 && fast[1] && fits[1];
    const bool m2 = m1 && fast[2] && fits[2];
    const bool m3 = m2 && fast[3] && fits[3];
    const uint32_t g = (uint32_t)m0 + (uint32_t)m1 + (uint32_t)m2 + (uint32_t)m3;
    const uint32_t fg = m3 ? f[4] : m2 ? f[3] : m1 ? f[2] : m0 ? f[1] : 27u;
    const uint32_t use = 5u * g + 27u - fg;
    // the first invalid code is a long one (park) or runs past the literal (only padding left)
    const bool bad_fast = (m2 && fast[3]) || (m1 && !m2 && fast[2]) || (m0 && !m1 && fast[1]) || (!m0 && fast[0]);
    const bool park = run && !m3 && !bad_fast;
    L.win <<= use;
    L.nb -= use;
    L.rem -= use;
    const uint32_t packed = sym[0] | (sym[1] << 8) | (sym[2] << 16) | (sym[3] << 24);
    lit_emit_g<kStore>(L, packed, g, out8);
    L.live = run ? (park || (m3 && L.rem != 0u)) : L.live;
    L.park = L.park || park;
}

// The parked lanes' long code: one lookup in the leading-ones table.
template <int kStore, class Src>
__device__ __forceinline__ void lit_unpark(Lit& L, const Src& src, const uint16_t* __restrict__ lo,
                                           uint8_t* __restrict__ out8) {
    L.park = false;
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

// v8 step: one lookup in the 12-bit two-symbol table (hpk_code.h LUT) decodes up to two codes
// of <= 12 bits (the VALU work per symbol is a third of the arithmetic steps'; PMC showed those
// saturating the SIMDs' vector issue). Symbols go straight to the LDS output image as bytes (no
// accumulator), each under its own validity mask. A code longer than 12 bits (EOS included)
// takes one leading-ones lookup in the (rarely taken) branch.
template <int kStore, class Src>
__device__ __forceinline__ void lit_step8(Lit& L, const Src& src, const uint32_t* __restrict__ lut,
                                          const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8) {
    lit_refill(L, src);
    const uint32_t hi = (uint32_t)(L.win >> 32);
    const uint32_t e = lut[hi >> (32 - HPK_LUT_BITS)];
    const uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u;
    const bool ok1 = L.live && (e >> 26) != 0u && len0 <= L.rem;
    const bool ok2 = ok1 && (e >> 27) != 0u && tot <= L.rem;
    const uint32_t use = ok2 ? tot : ok1 ? len0 : 0u;
    const uint32_t pos = L.od + L.cnt;
    if (kStore == kChecked) {
        if (ok1 && L.cnt >= L.oend - L.od) chk_report(1, pos, L.oend, L.cnt);
        if (ok2 && L.cnt + 1u >= L.oend - L.od) chk_report(1, pos + 1, L.oend, L.cnt);
    }
    if (kStore != kNoStore) {
        if (ok1) out8[pos] = (uint8_t)e;
        if (ok2) out8[pos + 1] = (uint8_t)(e >> 8);
    } else {
        asm volatile("" ::"v"(e));
    }
    L.cnt += (uint32_t)ok1 + (uint32_t)ok2;
    L.win <<= use;
    L.nb -= use;
    L.rem -= use;
    const bool park = L.live && (e >> 26) == 0u;  // a 13..30-bit code, or EOS
    L.live = park || (ok1 && L.rem != 0u);
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
            if (kStore == kChecked && L.cnt >= L.oend - L.od) chk_report(1, L.od + L.cnt, L.oend, L.cnt);
            if (kStore != kNoStore) out8[L.od + L.cnt] = (uint8_t)s1;
            L.cnt += 1;
            L.win <<= len;
            L.nb -= len;
            L.rem -= len;
            L.live = L.rem != 0u;
        }
    }
}

// ------------------------------------------------------------------------------------------
// v9: bit-position decode, two literals per lane.
//
// PMC on the window-register steps (v6..v8): the SIMDs' vector issue was 70-90 % busy and half
// the wave time sat in s_waitcnt on LDS. v9 keeps no bit window in registers: the input window
// is staged byte-swapped (big-endian dwords), and each step reads the two dwords under the
// literal's bit position P (one ds_read2), shifts them into a 32-bit window, and looks the next
// 12 bits up in the two-symbol table: ~20 VALU per step instead of ~40. Each lane carries TWO
// independent literals whose steps interleave, so one literal's LDS round trips hide behind the
// other's arithmetic.
struct Lit9 {
    uint32_t P;    // bit position in the window (MSB-first over the big-endian dwords)
    uint32_t E;    // end bit position
    uint32_t cnt;  // bytes decoded
    uint32_t od;   // output byte position in the LDS image
    uint32_t oend; // checked mode: end of the output region
    uint32_t w;    // the 32 bits at P from the last step (final padding check)
    uint32_t e;    // the table entry of this step
    uint32_t st;
    bool live;
};

__device__ __forceinline__ uint32_t lit9_window(const uint32_t* __restrict__ win32, uint32_t P) {
    const uint32_t q = P >> 5;
    const uint64_t pair = ((uint64_t)win32[q] << 32) | win32[q + 1];
    return (uint32_t)((pair << (P & 31u)) >> 32);
}

// Main part of a step (no branch): window, table entry, symbols, position.
template <int kStore>
__device__ __forceinline__ void lit9_main(Lit9& L, const uint32_t* __restrict__ win32, const uint32_t* __restrict__ lut,
                                          uint8_t* __restrict__ out8) {
    const uint32_t w = lit9_window(win32, L.P);
    const uint32_t e = lut[w >> (32 - HPK_LUT_BITS)];
    const uint32_t rem = L.E - L.P;
    const uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u;
    const bool ok1 = L.live && (e >> 26) != 0u && len0 <= rem;
    const bool ok2 = ok1 && (e >> 27) != 0u && tot <= rem;
    const uint32_t use = ok2 ? tot : ok1 ? len0 : 0u;
    const uint32_t pos = L.od + L.cnt;
    if (kStore == kChecked) {
        if (ok1 && L.cnt >= L.oend - L.od) chk_report(1, pos, L.oend, L.cnt);
        if (ok2 && L.cnt + 1u >= L.oend - L.od) chk_report(1, pos + 1, L.oend, L.cnt);
    }
    if (kStore != kNoStore) {
        if (ok1) out8[pos] = (uint8_t)e;
        if (ok2) out8[pos + 1] = (uint8_t)(e >> 8);
    } else {
        asm volatile("" ::"v"(e));
    }
    L.cnt += (uint32_t)ok1 + (uint32_t)ok2;
    L.w = w;
    L.e = e;
    L.P += use;
    // a code longer than 12 bits (or EOS) leaves the lane live with the entry's nsym = 0: the
    // park part takes it; otherwise the literal goes on while bits are left
    L.live = L.live && ((e >> 26) == 0u || (ok1 && L.P != L.E));
}

// Both literals of a lane in one step, all LDS reads issued before any LDS write: the byte
// stores into the output image may alias the window / table as far as the compiler knows, so
// reads placed after them could not be hoisted and the two literals' round trips would serialise.
template <int kStore>
__device__ __forceinline__ void lit9_pair(Lit9& A, Lit9& B, const uint32_t* __restrict__ win32,
                                          const uint32_t* __restrict__ lut, uint8_t* __restrict__ out8) {
    const uint32_t qa = A.P >> 5, qb = B.P >> 5;
    const uint32_t a0 = win32[qa], a1 = win32[qa + 1], b0 = win32[qb], b1 = win32[qb + 1];
    const uint32_t wa = (uint32_t)(((((uint64_t)a0 << 32) | a1) << (A.P & 31u)) >> 32);
    const uint32_t wb = (uint32_t)(((((uint64_t)b0 << 32) | b1) << (B.P & 31u)) >> 32);
    const uint32_t ea = lut[wa >> (32 - HPK_LUT_BITS)];
    const uint32_t eb = lut[wb >> (32 - HPK_LUT_BITS)];
    auto one = [&](Lit9& L, uint32_t w, uint32_t e, bool& ok1, bool& ok2, uint32_t& pos) {
        const uint32_t rem = L.E - L.P;
        const uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u;
        // bitwise, not short-circuit: no branches between the two literals' work
        ok1 = L.live & ((e >> 26) != 0u) & (len0 <= rem);
        ok2 = ok1 & ((e >> 27) != 0u) & (tot <= rem);
        const uint32_t use = ok2 ? tot : ok1 ? len0 : 0u;
        pos = L.od + L.cnt;
        if (kStore == kChecked) {
            if (ok1 && L.cnt >= L.oend - L.od) chk_report(1, pos, L.oend, L.cnt);
            if (ok2 && L.cnt + 1u >= L.oend - L.od) chk_report(1, pos + 1, L.oend, L.cnt);
        }
        L.cnt += (uint32_t)ok1 + (uint32_t)ok2;
        L.w = w;
        L.e = e;
        L.P += use;
        L.live = L.live & (((e >> 26) == 0u) | (ok1 & (L.P != L.E)));
    };
    bool a1ok, a2ok, b1ok, b2ok;
    uint32_t pa, pb;
    one(A, wa, ea, a1ok, a2ok, pa);
    one(B, wb, eb, b1ok, b2ok, pb);
    if (kStore != kNoStore) {
        if (a1ok) out8[pa] = (uint8_t)ea;
        if (a2ok) out8[pa + 1] = (uint8_t)(ea >> 8);
        if (b1ok) out8[pb] = (uint8_t)eb;
        if (b2ok) out8[pb + 1] = (uint8_t)(eb >> 8);
    } else {
        asm volatile("" ::"v"(ea), "v"(eb));
    }
}

// Park part: the lanes whose entry had no code (a 13..30-bit code or EOS): leading-ones table.
template <int kStore>
__device__ __forceinline__ void lit9_park(Lit9& L, const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8) {
    const uint32_t w = L.w;
    uint32_t s1, len;
    bool eos;
    lo_decode(w, lo, s1, len, eos);
    const uint32_t rem = L.E - L.P;
    if (len > rem) {
        L.live = false;  // only padding left
    } else if (eos) {
        L.st = HPK_EOS_IN_STRING;  // huffman.rs:112-116
        L.live = false;
    } else {
        if (kStore == kChecked && L.cnt >= L.oend - L.od) chk_report(1, L.od + L.cnt, L.oend, L.cnt);
        if (kStore != kNoStore) out8[L.od + L.cnt] = (uint8_t)s1;
        L.cnt += 1;
        L.P += len;
        L.live = L.P != L.E;
    }
    L.e = 1u << 26;  // handled
}

__device__ __forceinline__ uint32_t lit9_status(const Lit9& L) {
    uint32_t st = L.st;
    const uint32_t rem = L.E - L.P;
    if (st == HPK_OK && rem > 0) {  // huffman.rs:128-160
        if (rem > 7)
            st = HPK_PADDING_TOO_LARGE;
        else if ((L.w | (0xFFFFFFFFu >> rem)) != 0xFFFFFFFFu)
            st = HPK_INVALID_PADDING;
    }
    return st;
}

// The window as lit_begin/lit_refill expect it (raw byte order) for the byte path.
template <int kStore>
__device__ __forceinline__ void lit8_pair(Lit& A, Lit& B, const uint32_t* __restrict__ win32,
                                          const uint32_t* __restrict__ lut, const uint16_t* __restrict__ lo,
                                          uint8_t* __restrict__ out8) {
    // refill both from their prefetched dwords; read the next prefetch dwords
    auto refill_regs = [&](Lit& L) {
        const bool need = L.nb <= 32u;
        const uint64_t add = (uint64_t)__builtin_bswap32(L.nxt) << ((32u - L.nb) & 63u);
        L.win |= need ? add : 0ull;
        L.nb += need ? 32u : 0u;
        L.nxt = need ? L.pf : L.nxt;
        L.q += need ? 1u : 0u;
    };
    refill_regs(A);
    refill_regs(B);
    const uint32_t pfa = win32[A.q], pfb = win32[B.q];
    const uint32_t ha = (uint32_t)(A.win >> 32), hb = (uint32_t)(B.win >> 32);
    const uint32_t ea = lut[ha >> (32 - HPK_LUT_BITS)], eb = lut[hb >> (32 - HPK_LUT_BITS)];
    A.pf = pfa;
    B.pf = pfb;
    auto one = [&](Lit& L, uint32_t e, bool& ok1, bool& ok2, uint32_t& pos) {
        const uint32_t len0 = (e >> 16) & 31u, tot = (e >> 21) & 31u;
        ok1 = L.live & ((e >> 26) != 0u) & (len0 <= L.rem);
        ok2 = ok1 & ((e >> 27) != 0u) & (tot <= L.rem);
        const uint32_t use = ok2 ? tot : ok1 ? len0 : 0u;
        pos = L.od + L.cnt;
        if (kStore == kChecked) {
            if (ok1 && L.cnt >= L.oend - L.od) chk_report(1, pos, L.oend, L.cnt);
            if (ok2 && L.cnt + 1u >= L.oend - L.od) chk_report(1, pos + 1, L.oend, L.cnt);
        }
        L.cnt += (uint32_t)ok1 + (uint32_t)ok2;
        L.win <<= use;
        L.nb -= use;
        L.rem -= use;
        L.park = L.live & ((e >> 26) == 0u);  // a 13..30-bit code, or EOS
        L.live = L.park | (ok1 & (L.rem != 0u));
    };
    bool a1, a2, b1, b2;
    uint32_t pa, pb;
    one(A, ea, a1, a2, pa);
    one(B, eb, b1, b2, pb);
    if (kStore != kNoStore) {
        if (a1) out8[pa] = (uint8_t)ea;
        if (a2) out8[pa + 1] = (uint8_t)(ea >> 8);
        if (b1) out8[pb] = (uint8_t)eb;
        if (b2) out8[pb + 1] = (uint8_t)(eb >> 8);
    } else {
        asm volatile("" ::"v"(ea), "v"(eb));
    }
    if (__any(A.park | B.park)) {
        auto park = [&](Lit& L) {
            L.park = false;
            lit_refill(L, LdsSrc{win32});
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
                if (kStore == kChecked && L.cnt >= L.oend - L.od) chk_report(1, L.od + L.cnt, L.oend, L.cnt);
                if (kStore != kNoStore) out8[L.od + L.cnt] = (uint8_t)s1;
                L.cnt += 1;
                L.win <<= len;
                L.nb -= len;
                L.rem -= len;
                L.live = L.rem != 0u;
            }
        };
        if (A.park) park(A);
        if (B.park) park(B);
    }
}

// Final status of a literal whose walk has stopped (huffman.rs:128-160): at most 7 residual
// bits, all ones (the most significant bits of EOS); an EOS decoded inside wins (st already set).
template <int kStore>
__device__ __forceinline__ void lit_finish(Lit& L, const DecodeArgs& a, uint32_t i) {
    // the last, partial dword lies inside this literal's capacity (aligned, >= decoded bound)
    if (kStore == kDword && L.accn) reinterpret_cast<uint32_t*>(a.out_base)[L.od] = (uint32_t)L.acc;
    if (kStore == kChecked && L.accn) {
        if (L.od < L.oend)
            reinterpret_cast<uint32_t*>(a.out_base)[L.od] = (uint32_t)L.acc;
        else
            chk_report(2, L.od, L.oend, L.cnt);
    }
    if (kStore == kChecked && i >= a.n) {
        chk_report(3, i, a.n, 0);
        return;
    }
    const uint32_t st = lit_status(L);
    a.out_len[i] = L.cnt;
    a.status[i] = (uint8_t)st;
}

// Literal i decoded whole, one code at a time, with byte stores and per-byte capacity checks:
// output regions that are unaligned or below hpk_decoded_bound, and literals too long for the
// LDS window (read from global memory).
template <class Src>
__device__ __forceinline__ void lit_bytes(const Src& src, const uint16_t* lo, const DecodeArgs& a, uint32_t i,
                                          uint32_t sb, uint32_t nbytes) {
    Lit L;
    lit_begin(L, src, sb, nbytes);
    uint32_t o = a.out_off[i] + a.out_mis;
    const uint32_t ocap = a.out_off[i + 1] - a.out_off[i];
    while (L.live) {
        lit_refill(L, src);
        uint32_t sym, len;
        bool eos;
        lo_decode((uint32_t)(L.win >> 32), lo, sym, len, eos);
        if (len > L.rem) break;
        if (eos) {
            L.st = HPK_EOS_IN_STRING;
            break;
        }
        if (L.cnt >= ocap) {
            L.st = HPK_OUTPUT_OVERFLOW;
            break;
        }
        a.out_base[o + L.cnt] = (uint8_t)sym;
        L.cnt += 1;
        L.win <<= len;
        L.nb -= len;
        L.rem -= len;
        L.live = L.rem != 0u;
    }
    L.accn = 0;
    lit_finish<kNoStore>(L, a, i);
}



// Block-level window (v5): the workgroup stages a contiguous run of its literals into one LDS
// window shared by all its waves, and every wave pulls literals from ONE block queue (an LDS
// counter). Waves of a SIMD are arbitrated by age, so with a static per-wave split the youngest
// wave of each SIMD finished ~1.8x later than the oldest; with a shared queue fast waves simply
// take more literals and all finish together.
template <int kWaves, int kData, int kMaxLits>
struct BlockGeometry {
    static constexpr int kBlock = kWaves * 64;
    static constexpr int kMetaRounds = (kMaxLits + kBlock - 1) / kBlock;
    static constexpr int kStageRounds = (kData / 16 + kBlock - 1) / kBlock;
    static constexpr int kQueueOff = kTabBytes + kData;
    static constexpr int kCtrOff = kQueueOff + kMaxLits * 8;
    static constexpr int kLdsBytes = kCtrOff + 16;
    static_assert(kLdsBytes <= 163840, "LDS budget (160 KiB per CU on gfx950)");
    static_assert(kData % 16 == 0 && kData <= (1 << 17), "window offsets pack in 17 bits");
};
constexpr uint32_t kQByte = 0x80000000u;  // queue entry .y flag: byte path

// kMode: 0 = product kernel; diagnostic variants (HPK_DEBUG_MODE, never the default):
//   1 = stage only (no decode), 2 = decode without output stores, 3 = product + per-wave stamps,
//   4 = every global store bounds-checked (first violation recorded in g_chk, store skipped)
template <int kMode, int kWaves, int kData, int kMaxLits, int kRefillN, int kChunk, int kStep = 4>
__global__ __launch_bounds__(kWaves * 64) void hpk_decode_kernel(DecodeArgs a) {
    using G = BlockGeometry<kWaves, kData, kMaxLits>;
    unsigned long long t_start = 0, t_staged = 0;
    if (kMode == 3) t_start = __builtin_amdgcn_s_memtime();
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* s_t8 = smem;
    uint16_t* s_lo = reinterpret_cast<uint16_t*>(smem + kT8Bytes);
    uint8_t* s_data = smem + kTabBytes;
    uint2* s_q = reinterpret_cast<uint2*>(smem + G::kQueueOff);
    uint32_t* s_ctr = reinterpret_cast<uint32_t*>(smem + G::kCtrOff);  // [0] fitting count, [1] queue head
    for (uint32_t t = threadIdx.x; t < kT8Bytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_t8)[t] = reinterpret_cast<const uint4*>(a.t8)[t];
    for (uint32_t t = threadIdx.x; t < kLoBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const LdsSrc lds{reinterpret_cast<const uint32_t*>(s_data)};
    const uint32_t BA = (uint32_t)((uint64_t)a.n * blockIdx.x / gridDim.x);
    const uint32_t BB = (uint32_t)((uint64_t)a.n * (blockIdx.x + 1) / gridDim.x);

    uint32_t cur = BA;
    while (cur < BB) {  // block-uniform
        const uint32_t cntl = min((uint32_t)kMaxLits, BB - cur);
        const uint32_t base16 = (a.in_off[cur] + a.in_mis) & ~15u;
        const uint32_t limit = base16 + kData;
        __syncthreads();  // previous fill fully drained (queue, window and counters free)
        if (tid == 0) {
            s_ctr[0] = 0;
            s_ctr[1] = G::kBlock;
        }
        __syncthreads();
        // offsets: all loads issued first (clamped indices), then used
        uint32_t io0[G::kMetaRounds], io1[G::kMetaRounds], oo0[G::kMetaRounds], oo1[G::kMetaRounds];
#pragma unroll
        for (int r = 0; r < G::kMetaRounds; ++r) {
            const uint32_t t = min(tid + (uint32_t)G::kBlock * r, cntl - 1);
            io0[r] = a.in_off[cur + t];
            io1[r] = a.in_off[cur + t + 1];
            oo0[r] = a.out_off[cur + t];
            oo1[r] = a.out_off[cur + t + 1];
        }
        uint32_t kw = 0;
#pragma unroll
        for (int r = 0; r < G::kMetaRounds; ++r) {
            const uint32_t t = tid + (uint32_t)G::kBlock * r;
            const uint32_t p0 = io0[r] + a.in_mis, p1 = io1[r] + a.in_mis;
            const bool fits = t < cntl && p1 <= limit;
            if (fits) {
                const uint32_t nbytes = p1 - p0;
                const uint32_t o = oo0[r] + a.out_mis, ocap = oo1[r] - oo0[r];
                // dword path needs an aligned region holding hpk_decoded_bound(nbytes) bytes (and a
                // length that packs in 15 bits); byte-path entries carry the length in .y instead
                const bool dw = ((o | ocap) & 3u) == 0 && ocap >= (nbytes * 8u) / 5u && nbytes < 32768u;
                s_q[t] = dw ? make_uint2((p0 - base16) | (nbytes << 17), o >> 2)
                            : make_uint2(p0 - base16, kQByte | nbytes);
            }
            kw += (uint32_t)__popcll(__ballot(fits));
        }
        if (lane == 0 && kw) atomicAdd(&s_ctr[0], kw);
        __syncthreads();
        const uint32_t k = s_ctr[0];
        if (k == 0) {  // literal `cur` alone exceeds the window: one lane decodes it from global
            if (tid == 0) {
                const GlobalSrc g{reinterpret_cast<const uint32_t*>(a.in_base), (a.in_off[a.n] + a.in_mis - 1) >> 2};
                const uint32_t sb = a.in_off[cur] + a.in_mis;
                lit_bytes(g, s_lo, a, cur, sb, a.in_off[cur + 1] + a.in_mis - sb);
            }
            cur += 1;
            continue;
        }
        // stage the window's bytes with 16-byte loads: all loads issued, then all LDS writes.
        // Chunks are 16-byte aligned and each holds a byte of the batch, so no page is crossed.
        const uint2 last = s_q[k - 1];
        const uint32_t endb = (last.x & 0x1FFFFu) + ((last.y & kQByte) ? (last.y & ~kQByte) : (last.x >> 17));
        uint32_t nch = (endb + 15) >> 4;
        if (kMode == 4 && (nch > kData / 16 || base16 + endb > a.in_off[a.n] + a.in_mis + 16)) {
            chk_report(5, nch, endb, base16);
            nch = 0;
        }
        if (nch) {
            const uint4* g16 = reinterpret_cast<const uint4*>(a.in_base + base16);
            uint4* l16 = reinterpret_cast<uint4*>(s_data);
            uint4 chunk[G::kStageRounds];
#pragma unroll
            for (int r = 0; r < G::kStageRounds; ++r) chunk[r] = g16[min(tid + (uint32_t)G::kBlock * r, nch - 1)];
#pragma unroll
            for (int r = 0; r < G::kStageRounds; ++r)
                if (tid + (uint32_t)G::kBlock * r < nch) l16[tid + G::kBlock * r] = chunk[r];
        }
        __syncthreads();
        if (kMode == 3 && t_staged == 0) t_staged = __builtin_amdgcn_s_memtime();
        if (kMode == 1) {  // diagnostic: keep the staged bytes live, write lengths only
            for (uint32_t t = tid; t < k; t += G::kBlock) {
                const uint2 e = s_q[t];
                a.out_len[cur + t] = e.x + s_data[e.x & 0x1FFFFu];
                a.status[cur + t] = 0;
            }
        } else {
            // decode [0, k) from the block queue
            constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : kDword);
            Lit L = {};  // every field defined: idle lanes still run the (predicated) step
            L.nb = 64;
            uint32_t t = tid;
            uint32_t qb = 0, qe = 0;  // queue slots reserved by this wave, not yet handed out
            bool act = false;         // lane holds a dword-path literal not yet finalised
            // Branch-free (re)start: lanes past the queue read a clamped entry and stay idle. Keeping
            // the loop free of divergent exits matters: the ballots below must see the whole wave.
            auto begin = [&](uint32_t tt) {
                const uint2 e = s_q[min(tt, k - 1)];
                act = tt < k && !(e.y & kQByte);
                lit_begin(L, lds, e.x & 0x1FFFFu, e.x >> 17);
                L.od = e.y;
                L.oend = e.y + ((e.x >> 17) * 8u / 5u + 3u) / 4u;
                L.live = L.live && act;
            };
            begin(t);
            for (;;) {
#pragma unroll
                for (int s = 0; s < kRefillN; ++s) {
                    if (kStep == 6)
                        lit_step6<kStore>(L, lds, s_t8, s_lo, a.out_base);
                    else
                        lit_step<kStore>(L, lds, s_t8, s_lo, a.out_base);
                }
                const bool fin = t < k && !L.live;
                if (__any(fin)) {
                    if (fin && act) lit_finish<kStore>(L, a, cur + t);
                    const bool free_lane = fin || t >= k;
                    const uint64_t fm = __ballot(free_lane);
                    const uint32_t rank =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                    // free lanes take the wave's reserved slots [qb, qe) in rank order; when those
                    // run short the wave reserves kChunk more with one LDS atomic (block queue)
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
                    const uint32_t tn = free_lane ? base : t;
                    if (free_lane) {
                        t = tn;
                        begin(tn);
                    }
                }
                if (!__any(t < k)) break;
            }
            // literals whose output region is unaligned / below the decoded bound
            for (uint32_t tt = tid; tt < k; tt += G::kBlock) {
                const uint2 e = s_q[tt];
                if (e.y & kQByte) lit_bytes(lds, s_lo, a, cur + tt, e.x & 0x1FFFFu, e.y & ~kQByte);
            }
        }
        cur += k;
    }
    if (kMode == 3 && lane == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        const uint64_t gwi = (uint64_t)blockIdx.x * kWaves + (tid >> 6);
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.dbg[gwi * 4 + 0] = t_start;
        a.dbg[gwi * 4 + 1] = t_staged;
        a.dbg[gwi * 4 + 2] = t_end;
        a.dbg[gwi * 4 + 3] = ((unsigned long long)xcc << 32) | (BB - BA);
    }
}


// kMode as for v5 (0 product, 1 stage+flush only, 2 no output stores, 3 stamps, 4 checked).
//
// Software pipeline across fills: while fill j decodes, fill j+1's offsets and input window are
// already in flight into registers, and fill j-1's write-back stores drain; only LDS work
// (queue build, window copy, flush reads) sits between two decodes.
template <int kMode, int kWaves, int kW, int kO, int kQ, int kRefillN, int kChunk, int kStep>
__global__ __launch_bounds__(kWaves * 64) void hpk_decode7(DecodeArgs a) {
    using G = Geo7<kWaves, kW, kO, kQ, (kStep >= 8)>;
    constexpr int R = G::kMetaRounds, S = G::kStageRounds;
    unsigned long long t_start = 0, t_staged = 0;
    if (kMode == 3) t_start = __builtin_amdgcn_s_memtime();
    // static LDS: the compiler folds every region offset into the ds instructions' offset fields
    __shared__ __attribute__((aligned(16))) uint8_t smem[G::kLdsBytes];
    uint8_t* s_t8 = smem;
    uint16_t* s_lo = reinterpret_cast<uint16_t*>(smem + kT8Bytes);
    uint8_t* s_in = smem + G::kInOff;
    uint8_t* s_out = smem + G::kOutOff;
    uint32_t* s_out32 = reinterpret_cast<uint32_t*>(s_out);
    uint2* s_q = reinterpret_cast<uint2*>(smem + G::kQOff);
    uint32_t* s_lenst = reinterpret_cast<uint32_t*>(smem + G::kLenOff);  // len | status << 24
    uint32_t* s_hist = reinterpret_cast<uint32_t*>(smem + G::kHistOff);
    uint32_t* s_bbase = s_hist + 64;
    // [0] fitting count, [1] queue head, [2] input end of the fill, [3] output end of the fill
    uint32_t* s_ctr = reinterpret_cast<uint32_t*>(smem + G::kCtrOff);
    for (uint32_t t = threadIdx.x; t < kT8Bytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_t8)[t] = reinterpret_cast<const uint4*>(a.t8)[t];
    for (uint32_t t = threadIdx.x; t < kLoBytes / 16; t += G::kBlock)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];
    uint32_t* s_lut = reinterpret_cast<uint32_t*>(smem + G::kLutOff);
    if (kStep >= 8)
        for (uint32_t t = threadIdx.x; t < (uint32_t)G::kLutBytes / 16; t += G::kBlock)
            reinterpret_cast<uint4*>(s_lut)[t] = reinterpret_cast<const uint4*>(a.lut)[t];

    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u;
    const LdsSrc lds{reinterpret_cast<const uint32_t*>(s_in)};
    const uint32_t BA = (uint32_t)((uint64_t)a.n * blockIdx.x / gridDim.x);
    const uint32_t BB = (uint32_t)((uint64_t)a.n * (blockIdx.x + 1) / gridDim.x);
    const uint32_t in_end = a.in_off[a.n] + a.in_mis;
    const uint32_t last16 = in_end ? (in_end - 1) >> 4 : 0;  // last 16-B chunk holding a batch byte
    // last chunk holding a byte of THIS workgroup's literals: windows never read past it (the
    // next workgroup reads its own range), and the final, unused prefetch collapses onto it
    const uint32_t r_end = a.in_off[BB] + a.in_mis;
    const uint32_t rlast16 = r_end ? (r_end - 1) >> 4 : 0;

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
            if (tid < 2) {  // the partial chunks at the two ends
                const uint32_t g = tid == 0 ? c0 << 4 : (c1 - 1) << 4;
                if (!(g >= G0 && g + 16u <= G1) && (tid == 0 || c1 - 1 != c0)) {
#pragma unroll 1
                    for (uint32_t b = 0; b < 16u; ++b)
                        if (g + b >= G0 && g + b < G1) a.out_base[g + b] = s_out[g + b - ob];
                }
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

    uint32_t cur = BA;
    uint32_t gin = 0, gout = 0;  // exact input / output start of the fill (blob-relative + mis)
    Prefetch<R, S> P;
    if (cur < BB) {
        gin = a.in_off[cur] + a.in_mis;
        gout = a.out_off[cur] + a.out_mis;
        prefetch_fill<G::kBlock>(P, a, tid, cur, min(cur + (uint32_t)kQ, BB), gin & ~15u, rlast16);
    }
    while (cur < BB) {  // block-uniform
        const uint32_t cntl = min((uint32_t)kQ, BB - cur);
        const uint32_t base16 = gin & ~15u;
        const uint32_t ob16 = gout & ~15u;
        lds_barrier();  // previous fill decoded and its image read out: every LDS region is free
        if (tid < 64) s_hist[tid] = 0;
        if (tid == 0) {
            s_ctr[0] = 0;
            s_ctr[1] = kStep >= 9 ? 2 * G::kBlock : G::kBlock;  // slots handed out at the start
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
            const bool fits = t < cntl && p1 - base16 <= (uint32_t)kW && o1 - ob16 <= (uint32_t)kO;
            pos[r] = 0xFFFFFFFFu;
            if (fits) {
                const uint32_t nbytes = p1 - p0, ocap = o1 - o0;
                // fast path: a region holding hpk_decoded_bound(nbytes) bytes (dword-aligned for
                // the accumulator steps, which store whole dwords)
                const bool dw = (kStep >= 8 || ((o0 | ocap) & 3u) == 0) && ocap >= (nbytes * 8u) / 5u;
                ex[r] = (p0 - base16) | (nbytes << 16);
                ey[r] = t | ((o0 - ob16) << 12) | (dw ? 0u : kQ7Byte);
                const uint32_t bk = lpt_bucket(nbytes);
                pos[r] = (bk << 16) | atomicAdd(&s_hist[bk], 1u);
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
        // the window, from the prefetched registers
        {
            uint4* l16 = reinterpret_cast<uint4*>(s_in);
#pragma unroll
            for (int r = 0; r < S; ++r) {
                uint4 c = P.chunk[r];
                if (kStep == 9)  // big-endian dwords: bit P of the stream is bit 31 - P % 32 of dword P / 32
                    c = make_uint4(__builtin_bswap32(c.x), __builtin_bswap32(c.y), __builtin_bswap32(c.z),
                                   __builtin_bswap32(c.w));
                if (tid + G::kBlock * r < kW / 16) l16[tid + G::kBlock * r] = c;
            }
        }
        lds_barrier();
#pragma unroll
        for (int r = 0; r < R; ++r)
            if (pos[r] != 0xFFFFFFFFu) s_q[s_bbase[pos[r] >> 16] + (pos[r] & 0xFFFFu)] = make_uint2(ex[r], ey[r]);
        // the next fill's offsets and window: in flight during this fill's decode. Unconditional
        // (clamped past the range end), so no register phi forces a wait on the stores below.
        const uint32_t cur_next = cur + k;
        {
            const uint32_t c = min(cur_next, BB - 1);
            prefetch_fill<G::kBlock>(P, a, tid, c, min(c + (uint32_t)kQ, BB), gin_next & ~15u, rlast16);
        }
        // the previous fill's write-back: its image is read out before this fill decodes over it
        if (pk) flush(pcur, pk, pG0, pG1);
        pk = k;
        pcur = cur;
        pG0 = gout;
        pG1 = gout_next;
        lds_barrier();
        if (kMode == 3 && t_staged == 0) t_staged = __builtin_amdgcn_s_memtime();
        if (kMode == 1) {  // diagnostic: no decode; lengths from the staged bytes keep them live
            for (uint32_t t = tid; t < k; t += G::kBlock) {
                const uint2 e = s_q[t];
                s_lenst[e.y & 0xFFFu] = (e.x >> 16) + s_in[e.x & 0xFFFFu];
            }
        } else if (kStep == 10) {
            constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : kDword);
            static_assert(kStep != 10 || kChunk >= 128, "a refill can hand out 128 slots (two per lane)");
            const uint32_t* win32 = reinterpret_cast<const uint32_t*>(s_in);
            Lit A = {}, B = {};  // every field defined: idle lanes still run the (predicated) step
            A.nb = 64;
            B.nb = 64;
            uint32_t ta = tid, tb = tid + G::kBlock;
            uint32_t qb = 0, qe = 0;  // queue slots reserved by this wave, not yet handed out
            bool acta = false, actb = false;
            uint32_t ia = 0, ib = 0;
            auto begin = [&](Lit& L, bool& act, uint32_t& idx, uint32_t tt) {
                const uint2 e = s_q[min(tt, k - 1)];
                act = tt < k && !(e.y & kQ7Byte);
                idx = e.y & 0xFFFu;
                lit_begin(L, lds, e.x & 0xFFFFu, e.x >> 16);
                L.park = false;
                L.od = (e.y >> 12) & 0x1FFFFu;
                L.oend = L.od + (e.x >> 16) * 8u / 5u;
                L.live = L.live && act;
            };
            begin(A, acta, ia, ta);
            begin(B, actb, ib, tb);
            for (;;) {
#pragma unroll
                for (int s = 0; s < kRefillN; ++s) lit8_pair<kStore>(A, B, win32, s_lut, s_lo, s_out);
                const bool fa = ta < k && !A.live, fb = tb < k && !B.live;
                if (__any(fa || fb)) {
                    if (fa && acta) s_lenst[ia] = A.cnt | (lit_status(A) << 24);
                    if (fb && actb) s_lenst[ib] = B.cnt | (lit_status(B) << 24);
                    const bool fra = fa || ta >= k, frb = fb || tb >= k;
                    const uint64_t ma = __ballot(fra), mb = __ballot(frb);
                    const uint32_t na = (uint32_t)__popcll(ma);
                    const uint32_t ra = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
                    const uint32_t rb =
                        na + __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
                    const uint32_t need = na + (uint32_t)__popcll(mb), have = qe - qb;
                    uint32_t nb = qb;
                    if (have < need) {  // wave-uniform: reserve kChunk more slots
                        uint32_t g = 0;
                        if (lane == 0) g = atomicAdd(&s_ctr[1], (uint32_t)kChunk);
                        g = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
                        nb = g;
                    }
                    const uint32_t xa = ra < have ? qb + ra : nb + (ra - have);
                    const uint32_t xb = rb < have ? qb + rb : nb + (rb - have);
                    if (have < need) {
                        qb = nb + (need - have);
                        qe = nb + kChunk;
                    } else {
                        qb += need;
                    }
                    qb = (uint32_t)__builtin_amdgcn_readfirstlane((int)qb);
                    qe = (uint32_t)__builtin_amdgcn_readfirstlane((int)qe);
                    if (fra) {
                        ta = xa;
                        begin(A, acta, ia, xa);
                    }
                    if (frb) {
                        tb = xb;
                        begin(B, actb, ib, xb);
                    }
                }
                if (!__any(ta < k || tb < k)) break;
            }
            for (uint32_t tt = tid; tt < k; tt += G::kBlock) {
                const uint2 e = s_q[tt];
                if (e.y & kQ7Byte) {
                    const uint32_t i = e.y & 0xFFFu;
                    const uint32_t o = a.out_off[cur + i] + a.out_mis - ob16;
                    Lit Bt = {};
                    lit_bytes_to(Bt, lds, s_lo, [&](uint32_t j, uint8_t v) { s_out[o + j] = v; },
                                 a.out_off[cur + i + 1] - a.out_off[cur + i], e.x & 0xFFFFu, e.x >> 16);
                    s_lenst[i] = Bt.cnt | (lit_status(Bt) << 24);
                }
            }
        } else if (kStep == 9) {
            constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : kDword);
            static_assert(kStep != 9 || kChunk >= 128, "a refill can hand out 128 slots (two per lane)");
            const uint32_t* win32 = reinterpret_cast<const uint32_t*>(s_in);
            Lit9 A = {}, B = {};
            uint32_t ta = tid, tb = tid + G::kBlock;
            uint32_t qb = 0, qe = 0;  // queue slots reserved by this wave, not yet handed out
            bool acta = false, actb = false;
            uint32_t ia = 0, ib = 0;
            auto begin = [&](Lit9& L, bool& act, uint32_t& idx, uint32_t tt) {
                const uint2 e = s_q[min(tt, k - 1)];
                act = tt < k && !(e.y & kQ7Byte);
                idx = e.y & 0xFFFu;
                L.P = (e.x & 0xFFFFu) * 8u;
                L.E = L.P + (e.x >> 16) * 8u;
                L.cnt = 0;
                L.st = HPK_OK;
                L.w = 0xFFFFFFFFu;
                L.e = 1u << 26;
                L.od = (e.y >> 12) & 0x1FFFFu;
                L.oend = L.od + (e.x >> 16) * 8u / 5u;
                L.live = act && L.P != L.E;
            };
            begin(A, acta, ia, ta);
            begin(B, actb, ib, tb);
            for (;;) {
#pragma unroll
                for (int s = 0; s < kRefillN; ++s) {
                    lit9_pair<kStore>(A, B, win32, s_lut, s_out);
                    const bool pa = A.live && (A.e >> 26) == 0u, pb = B.live && (B.e >> 26) == 0u;
                    if (__any(pa || pb)) {
                        if (pa) lit9_park<kStore>(A, s_lo, s_out);
                        if (pb) lit9_park<kStore>(B, s_lo, s_out);
                    }
                }
                const bool fa = ta < k && !A.live, fb = tb < k && !B.live;
                if (__any(fa || fb)) {
                    if (fa && acta) s_lenst[ia] = A.cnt | (lit9_status(A) << 24);
                    if (fb && actb) s_lenst[ib] = B.cnt | (lit9_status(B) << 24);
                    const bool fra = fa || ta >= k, frb = fb || tb >= k;
                    const uint64_t ma = __ballot(fra), mb = __ballot(frb);
                    const uint32_t na = (uint32_t)__popcll(ma);
                    const uint32_t ra = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
                    const uint32_t rb =
                        na + __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
                    const uint32_t need = na + (uint32_t)__popcll(mb), have = qe - qb;
                    uint32_t nb = qb;
                    if (have < need) {  // wave-uniform: reserve kChunk more slots
                        uint32_t g = 0;
                        if (lane == 0) g = atomicAdd(&s_ctr[1], (uint32_t)kChunk);
                        g = (uint32_t)__builtin_amdgcn_readfirstlane((int)g);
                        nb = g;
                    }
                    // rank r takes qb + r while r < have, else nb + (r - have)
                    const uint32_t xa = ra < have ? qb + ra : nb + (ra - have);
                    const uint32_t xb = rb < have ? qb + rb : nb + (rb - have);
                    if (have < need) {
                        qb = nb + (need - have);
                        qe = nb + kChunk;
                    } else {
                        qb += need;
                    }
                    qb = (uint32_t)__builtin_amdgcn_readfirstlane((int)qb);
                    qe = (uint32_t)__builtin_amdgcn_readfirstlane((int)qe);
                    if (fra) {
                        ta = xa;
                        begin(A, acta, ia, xa);
                    }
                    if (frb) {
                        tb = xb;
                        begin(B, actb, ib, xb);
                    }
                }
                if (!__any(ta < k || tb < k)) break;
            }
            // byte path (capacity below the decoded bound)
            for (uint32_t tt = tid; tt < k; tt += G::kBlock) {
                const uint2 e = s_q[tt];
                if (e.y & kQ7Byte) {
                    const uint32_t i = e.y & 0xFFFu;
                    const uint32_t o = a.out_off[cur + i] + a.out_mis - ob16;
                    Lit Bt = {};
                    lit_bytes_to(Bt, LdsSwapSrc{win32}, s_lo, [&](uint32_t j, uint8_t v) { s_out[o + j] = v; },
                                 a.out_off[cur + i + 1] - a.out_off[cur + i], e.x & 0xFFFFu, e.x >> 16);
                    s_lenst[i] = Bt.cnt | (lit_status(Bt) << 24);
                }
            }
        } else {
            constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : kDword);
            Lit L = {};  // every field defined: idle lanes still run the (predicated) step
            L.nb = 64;
            uint32_t t = tid;
            uint32_t qb = 0, qe = 0;  // queue slots reserved by this wave, not yet handed out
            bool act = false;         // lane holds a dword-path literal not yet finalised
            uint32_t idx = 0;         // its index in the fill
            auto begin = [&](uint32_t tt) {
                const uint2 e = s_q[min(tt, k - 1)];
                act = tt < k && !(e.y & kQ7Byte);
                idx = e.y & 0xFFFu;
                lit_begin(L, lds, e.x & 0xFFFFu, e.x >> 16);
                const uint32_t ob = (e.y >> 12) & 0x1FFFFu;
                L.od = kStep == 8 ? ob : ob >> 2;  // byte (step 8) or dword position in the image
                L.oend = kStep == 8 ? ob + (e.x >> 16) * 8u / 5u : L.od + ((e.x >> 16) * 8u / 5u + 3u) / 4u;
                L.live = L.live && act;
            };
            begin(t);
            for (;;) {
#pragma unroll
                for (int s = 0; s < kRefillN; ++s) {
                    if (kStep == 8)
                        lit_step8<kStore>(L, lds, s_lut, s_lo, s_out);
                    else if (kStep == 7)
                        lit_step7<kStore>(L, lds, s_t8, s_out);
                    else if (kStep == 6)
                        lit_step6<kStore>(L, lds, s_t8, s_lo, s_out);
                    else
                        lit_step<kStore>(L, lds, s_t8, s_lo, s_out);
                }
                if (kStep == 7 && __any(L.park)) {
                    if (L.park) lit_unpark<kStore>(L, lds, s_lo, s_out);
                }
                const bool fin = t < k && !L.live;
                if (__any(fin)) {
                    if (fin && act) {
                        if (kStep != 8 && kStore == kDword && L.accn) s_out32[L.od] = (uint32_t)L.acc;
                        if (kStep != 8 && kStore == kChecked && L.accn) {
                            if (L.od < L.oend && L.od < (uint32_t)kO / 4)
                                s_out32[L.od] = (uint32_t)L.acc;
                            else
                                chk_report(2, L.od, L.oend, L.cnt);
                        }
                        s_lenst[idx] = L.cnt | (lit_status(L) << 24);
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
            // literals whose output region is unaligned / below the decoded bound: byte stores
            // into the image with a capacity check per byte
            for (uint32_t tt = tid; tt < k; tt += G::kBlock) {
                const uint2 e = s_q[tt];
                if (e.y & kQ7Byte) {
                    const uint32_t i = e.y & 0xFFFu;
                    const uint32_t o = a.out_off[cur + i] + a.out_mis - ob16;
                    Lit B = {};
                    lit_bytes_to(B, lds, s_lo, [&](uint32_t j, uint8_t v) { s_out[o + j] = v; },
                                 a.out_off[cur + i + 1] - a.out_off[cur + i], e.x & 0xFFFFu, e.x >> 16);
                    s_lenst[i] = B.cnt | (lit_status(B) << 24);
                }
            }
        }
        cur = cur_next;
        gin = gin_next;
        gout = gout_next;
    }
    if (pk) {
        lds_barrier();
        flush(pcur, pk, pG0, pG1);
    }
    if (kMode == 3 && lane == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        const uint64_t gwi = (uint64_t)blockIdx.x * kWaves + (tid >> 6);
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.dbg[gwi * 4 + 0] = t_start;
        a.dbg[gwi * 4 + 1] = t_staged;
        a.dbg[gwi * 4 + 2] = t_end;
        a.dbg[gwi * 4 + 3] = ((unsigned long long)xcc << 32) | (BB - BA);
    }
}


}  // namespace hpkdec
