// hpk_code.h — the RFC 7541 Appendix B Huffman code and the decode tables derived from it.
//
// The code is canonical (codes assigned in (length, symbol) order, Kraft sum exactly 1), so the
// whole table is determined by the 257 code lengths below; codes are rebuilt from them. The
// reference keeps the same code as 257 explicit (code, len) pairs in
// crates/loona-hpack/src/huffman.rs:222-480 and builds a HashMap<len, HashMap<code, sym>> from
// them on every literal (huffman.rs:58-82, decoder.rs:148). Here the tables are built once per
// context and staged in LDS by the kernels.
//
// Decode tables (built and self-checked below; validated end to end by the golden vectors):
//
//  * LUT  (HPK_LUT_BITS-bit index = the next bits of the stream, MSB-first). Entry (u32):
//        [7:0] sym0  [15:8] sym1  [20:16] len0  [25:21] len0+len1  [27:26] nsym (0,1,2)
//    nsym = 0 means the next code is longer than HPK_LUT_BITS: use the LO table.
//  * LO   ("leading ones") table. Every code is 1^k 0 t with a tail t of at most 5 bits
//    (k = run of leading ones). Index = k*32 + next 5 bits after the terminating 0.
//    Entry (u16): [8:0] symbol (256 = EOS) [13:9] code length. k >= 30 is EOS (30 ones).
//    One lookup decodes ANY codeword, so the fallback is branch-light and cheap.
#pragma once
#include <stdint.h>

#define HPK_NSYM 257
#define HPK_EOS 256
#define HPK_LUT_BITS 12
#define HPK_LUT_SIZE (1u << HPK_LUT_BITS)
#define HPK_LO_RUNS 30
#define HPK_LO_SIZE (HPK_LO_RUNS * 32)

// Canonical limits of the 5..8-bit codes (left-aligned 32-bit window): a window below LIM5 starts
// with a 5-bit code, below LIM6 a 6-bit one, below LIM7 7, below LIM8 8; at or above LIM8 the
// code is 10..30 bits long. These four lengths cover ~99.9 % of header-value symbols, so the
// decoder computes the length arithmetically and reads only the symbol from a table (T8).
#define HPK_LIM5 0x50000000u
#define HPK_LIM6 0xB8000000u
#define HPK_LIM7 0xF8000000u
#define HPK_LIM8 0xFE000000u

// Code length of every symbol 0..255 and EOS (256). RFC 7541 Appendix B, column "len in bits".
static const uint8_t HPK_CODE_LEN[HPK_NSYM] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28, /*   0.. 15 */
    28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28, /*  16.. 31 */
    6,  10, 10, 12, 13, 6,  8,  11, 10, 10, 8,  11, 8,  6,  6,  6,  /*  32.. 47 */
    5,  5,  5,  6,  6,  6,  6,  6,  6,  6,  7,  8,  15, 6,  12, 10, /*  48.. 63 */
    13, 6,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  /*  64.. 79 */
    7,  7,  7,  7,  7,  7,  7,  7,  8,  7,  8,  13, 19, 13, 14, 6,  /*  80.. 95 */
    15, 5,  6,  5,  6,  5,  6,  6,  6,  5,  7,  7,  6,  6,  6,  5,  /*  96..111 */
    6,  7,  6,  5,  5,  6,  7,  7,  7,  7,  7,  15, 11, 14, 13, 28, /* 112..127 */
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23, /* 128..143 */
    24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24, /* 144..159 */
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23, /* 160..175 */
    21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23, /* 176..191 */
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25, /* 192..207 */
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27, /* 208..223 */
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23, /* 224..239 */
    26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26, /* 240..255 */
    30,                                                             /* EOS      */
};

// LUT2: the LUT's content in the layout of the bit-position step (decode v12; fields re-packed in
// v21), chosen so the checked step clamps the bits left to HPK_LUT2_CLAMP and needs one compare per
// code, the unchecked body step (lit12_fast) reads the bits and codes an entry holds with one bfe
// each, and v_perm / ds_write_b8_d16_hi take the two symbols where they are:
//   [7:0] sym0  [11:8] len0  [15:12] bits held  [23:16] sym1  [27:24] len0+len1  [29:28] codes held
//   [30] fewer than two  [31] none
// a length field of a code the entry does not hold is 15 (never <= the clamped bits left); bits held
// is 0 for an entry with no code (a 13..30-bit code or EOS starts here).
#define HPK_LUT2_NOTTWO 0x40000000u  // e >= : fewer than two codes
#define HPK_LUT2_NONE 0x80000000u    // e >= : no code (a 13..30-bit code or EOS starts here)
#define HPK_LUT2_MISSING 15u         // the length field of a code the entry does not hold
#define HPK_LUT2_CLAMP 14u           // bits left are clamped to this before the length compares
#define HPK_L2_LEN0(e) (((e) >> 8) & 15u)
#define HPK_L2_HELD(e) (((e) >> 12) & 15u)
#define HPK_L2_LEN01(e) (((e) >> 24) & 15u)
#define HPK_L2_CODES(e) (((e) >> 28) & 3u)
#define HPK_L2_TWO(e) (((e) >> 29) & 1u)

// LUT3 (decode v28, the wave kernel): the same codes in a layout whose "bits held" is a whole byte, so
// the body step (lit12_body) shifts by it and adds it with sub-dword (SDWA) operand selection, no
// bfe:
//   [7:0] sym0  [15:8] bits held  [23:16] sym1  [25:24] codes held  [29:26] len0 (15: none)
//   [31] fewer than two codes
// The checked step reads len0 from [29:26] and the two codes' length as "bits held" when [31] is
// clear (lutc<kLut3>).
#define HPK_L3_HELD(e) (((e) >> 8) & 0xFFu)
#define HPK_L3_CODES(e) (((e) >> 24) & 3u)
#define HPK_L3_LEN0(e) (((e) >> 26) & 15u)
#define HPK_L3_NOTTWO 0x80000000u

struct hpk_tables {
    uint32_t code[HPK_NSYM];   // right-aligned canonical code
    uint8_t len[HPK_NSYM];     // code length in bits
    uint32_t lut[HPK_LUT_SIZE];
    uint32_t lut2[HPK_LUT_SIZE];
    uint32_t lut3[HPK_LUT_SIZE];
    uint16_t lo[HPK_LO_SIZE];
    uint8_t t8[256];  // symbol of the <=8-bit code that prefixes each 8-bit window (0 past LIM8)
};

// Build canonical codes from lengths, then the LUT and LO tables. Returns 0 on success,
// -1 if the length list is not a complete prefix code (never, for the static table).
static inline int hpk_build_tables(hpk_tables* t) {
    // canonical assignment: sort symbols by (len, sym); counting sort over lengths 1..30
    uint16_t order[HPK_NSYM];
    int n = 0;
    for (int L = 1; L <= 30; ++L)
        for (int s = 0; s < HPK_NSYM; ++s)
            if (HPK_CODE_LEN[s] == L) order[n++] = (uint16_t)s;
    if (n != HPK_NSYM) return -1;
    uint64_t c = 0;
    int prev = HPK_CODE_LEN[order[0]];
    for (int i = 0; i < n; ++i) {
        int s = order[i], L = HPK_CODE_LEN[s];
        if (i) c = (c + 1) << (L - prev);
        prev = L;
        t->code[s] = (uint32_t)c;
        t->len[s] = (uint8_t)L;
    }
    if (c + 1 != (1ull << prev)) return -1;  // complete code: last code is all ones

    // LO table: for every run k of leading ones (0..29) and every 5-bit continuation t5,
    // the unique code that is a prefix of 1^k 0 t5 (tails are <= 5 bits, so it exists).
    for (int k = 0; k < HPK_LO_RUNS; ++k)
        for (int t5 = 0; t5 < 32; ++t5) {
            // 64-bit MSB-aligned window 1^k 0 t5 0... (k+6 <= 35 bits, codes are <= 30 bits,
            // so the device's zero fill past bit 32 only lands on don't-care positions)
            uint64_t w = ((((1ull << k) - 1) << 6) | (uint64_t)t5) << (64 - (k + 6));
            uint16_t e = 0xFFFF;
            for (int s = 0; s < HPK_NSYM; ++s) {
                int L = t->len[s];
                if ((w >> (64 - L)) == t->code[s]) { e = (uint16_t)(s | (L << 9)); break; }
            }
            if (e == 0xFFFF) return -1;
            t->lo[k * 32 + t5] = e;
        }

    // T8: the symbol whose (<= 8-bit) code prefixes each 8-bit window; check the limits too.
    for (uint32_t v = 0; v < 256; ++v) {
        t->t8[v] = 0;
        const uint32_t w = v << 24;
        if (w >= HPK_LIM8) continue;
        const int L = 5 + (w >= HPK_LIM5) + (w >= HPK_LIM6) + (w >= HPK_LIM7);
        int found = -1;
        for (int s = 0; s < 256; ++s)
            if (t->len[s] <= 8 && (w >> (32 - t->len[s])) == t->code[s]) { found = s; break; }
        if (found < 0 || t->len[found] != L) return -1;
        t->t8[v] = (uint8_t)found;
    }

    // LUT: up to two whole codes inside the first HPK_LUT_BITS bits.
    for (uint32_t v = 0; v < HPK_LUT_SIZE; ++v) {
        uint32_t w = v << (32 - HPK_LUT_BITS);  // MSB-aligned, zero beyond
        int s0 = -1, l0 = 0;
        for (int s = 0; s < 256; ++s) {
            int L = t->len[s];
            if (L <= HPK_LUT_BITS && (w >> (32 - L)) == t->code[s]) { s0 = s; l0 = L; break; }
        }
        if (s0 < 0) {
            t->lut[v] = 0;
            t->lut2[v] = 0xC0000000u | (HPK_LUT2_MISSING << 8) | (HPK_LUT2_MISSING << 24);
            continue;
        }
        uint32_t w1 = w << l0;
        int rem = HPK_LUT_BITS - l0, s1 = -1, l1 = 0;
        for (int s = 0; s < 256 && rem >= 5; ++s) {
            int L = t->len[s];
            if (L <= rem && (w1 >> (32 - L)) == t->code[s]) { s1 = s; l1 = L; break; }
        }
        uint32_t e = (uint32_t)s0 | ((uint32_t)l0 << 16);
        uint32_t e2 = (uint32_t)s0 | ((uint32_t)l0 << 8);
        if (s1 >= 0) {
            e |= ((uint32_t)s1 << 8) | ((uint32_t)(l0 + l1) << 21) | (2u << 26);
            e2 |= ((uint32_t)s1 << 16) | ((uint32_t)(l0 + l1) << 24) | ((uint32_t)(l0 + l1) << 12) | (2u << 28);
        } else {
            e |= ((uint32_t)l0 << 21) | (1u << 26);
            e2 |= (HPK_LUT2_MISSING << 24) | ((uint32_t)l0 << 12) | (1u << 28) | HPK_LUT2_NOTTWO;
        }
        t->lut[v] = e;
        t->lut2[v] = e2;
    }
    for (uint32_t v = 0; v < HPK_LUT_SIZE; ++v) {  // LUT3 from LUT2
        const uint32_t e2 = t->lut2[v], codes = HPK_L2_CODES(e2);
        t->lut3[v] = (e2 & 0xFFu) | (HPK_L2_HELD(e2) << 8) | (e2 & 0x00FF0000u) | (codes << 24) |
                     ((codes ? HPK_L2_LEN0(e2) : 15u) << 26) | (codes < 2 ? HPK_L3_NOTTWO : 0u);
    }
    return 0;
}
