// Host check of the decode kernel's two-symbol table (hpk_code.h, LUT2 layout of decode v21): every
// 12-bit prefix is decoded again here, code by code, from the canonical (code, length) pairs the
// builder derives (pinned to the reference's table by tests/test_oracle.py), and each field of the
// entry is compared with what the lane step (lit12_step / lut12) expects. Prints "ok" or the first
// mismatch. Built and run by tests/test_tables.py.
#include <cstdio>

#include "hpk_code.h"

static int first_code(const hpk_tables& t, unsigned bits, int nbits, int& sym, int& len) {
    // the code that prefixes the nbits-bit string `bits` (MSB first), if it fits
    for (int s = 0; s < HPK_NSYM; ++s) {
        const int L = t.len[s];
        if (L <= nbits && (bits >> (nbits - L)) == t.code[s]) {
            sym = s;
            len = L;
            return 1;
        }
    }
    return 0;
}

int main() {
    static hpk_tables t;
    if (hpk_build_tables(&t) != 0) {
        puts("table build failed");
        return 1;
    }
    for (unsigned v = 0; v < HPK_LUT_SIZE; ++v) {
        const unsigned e = t.lut2[v];
        int s0 = -1, l0 = 0, s1 = -1, l1 = 0;
        const int has0 = first_code(t, v, HPK_LUT_BITS, s0, l0) && s0 < 256;
        int has1 = 0;
        if (has0 && HPK_LUT_BITS - l0 >= 5) {
            const unsigned rest = v & ((1u << (HPK_LUT_BITS - l0)) - 1u);
            has1 = first_code(t, rest, HPK_LUT_BITS - l0, s1, l1) && s1 < 256;
        }
        const unsigned codes = has0 ? (has1 ? 2u : 1u) : 0u;
        const unsigned held = has0 ? (unsigned)(l0 + (has1 ? l1 : 0)) : 0u;
        const unsigned want_len0 = has0 ? (unsigned)l0 : HPK_LUT2_MISSING;
        const unsigned want_len01 = has1 ? (unsigned)(l0 + l1) : HPK_LUT2_MISSING;
        const int ok = HPK_L2_CODES(e) == codes && HPK_L2_HELD(e) == held && HPK_L2_LEN0(e) == want_len0 &&
                       HPK_L2_LEN01(e) == want_len01 && (!has0 || (e & 0xFFu) == (unsigned)s0) &&
                       (!has1 || ((e >> 16) & 0xFFu) == (unsigned)s1) && HPK_L2_TWO(e) == (codes == 2u) &&
                       ((e >= HPK_LUT2_NOTTWO) == (codes < 2u)) && ((e >= HPK_LUT2_NONE) == (codes == 0u)) &&
                       HPK_LUT2_MISSING > HPK_LUT2_CLAMP && (unsigned)HPK_LUT_BITS <= HPK_LUT2_CLAMP;
        if (!ok) {
            printf("entry %u = %08x: codes %u held %u len0 %u len01 %u sym0 %d sym1 %d\n", v, e, codes, held, want_len0,
                   want_len01, s0, s1);
            return 1;
        }
    }
    puts("ok");
    return 0;
}
