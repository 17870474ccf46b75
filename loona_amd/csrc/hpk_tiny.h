// hpk_tiny.h — decode v28 for small batches (the granularity of one loona thread's read_headers:
// crates/loona/src/h2/server.rs:1619-1638, a few hundred to a few thousand literals per call).
//
// Round 3 measured the synchronous 1k-literal call at 23 us, 12.5 of them in the fill kernel,
// whose cost at that size is its fixed latency chain: the 18 KiB of tables into LDS, the first
// offsets and window from memory, one fill, the write-back. This kernel has no
// staging at all: one lane per literal, 64-thread workgroups (one wave each, spread over the CUs),
// the input read straight from global memory into a 64-bit bit window (dwords, byte-swapped), one
// LUT2 lookup per iteration (up to two codes) and the leading-ones table for a 13..30-bit code, both
// read from global memory (16 KiB + 1.9 KiB: L1/L2-resident after the first touches), the decoded
// bytes stored straight to the literal's region. Same semantics as the lane walk of the other two
// kernels (huffman.rs:95-161 with the precedence of huffman.rs:112-160), same offset checks
// (decoder.rs:138-142: a literal's bounds before any Huffman work) and statuses.
#pragma once
#include "hpk_decode12.h"

namespace hpkdec {

// One literal per lane. kChk: the literal's region is below the decoded bound, so every byte is
// capacity-checked (HPK_OUTPUT_OVERFLOW), as lit_bytes_to.
__global__ __launch_bounds__(64) void hpk_decode_tiny(DecodeArgs a) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t p0 = a.in_off[i], p1 = a.in_off[i + 1], q0 = a.out_off[i], q1 = a.out_off[i + 1];
    if (!(p0 <= p1 && p1 <= a.in_cap && q0 <= q1 && q1 <= a.out_cap)) {
        a.out_len[i] = 0;
        a.status[i] = (uint8_t)HPK_BAD_OFFSETS;
        *a.err = 1u;
        return;
    }
    const uint32_t nb = p1 - p0, ocap = q1 - q0;
    const bool chk = (uint64_t)ocap < (uint64_t)nb * 8u / 5u;
    const uint32_t in_end = min(a.in_off[a.n], a.in_cap) + a.in_mis;
    const GlobalSrc src{reinterpret_cast<const uint32_t*>(a.in_base), in_end ? (in_end - 1u) >> 2 : 0u};
    uint8_t* const dst = a.out_base + a.out_mis + q0;
    Lit L;
    lit_begin(L, src, p0 + a.in_mis, nb);
    while (L.live) {
        lit_refill(L, src);  // >= 33 bits in the window
        const uint32_t w = (uint32_t)(L.win >> 32);
        const uint32_t e = a.lut2[w >> (32 - HPK_LUT_BITS)];
        bool ok1, ok2;
        uint32_t u = lut12(e, L.rem, ok1, ok2);
        uint32_t g = (uint32_t)ok1 + (uint32_t)ok2;
        if (chk && L.cnt + g > ocap) {  // the region ends inside this entry's codes
            if (L.cnt >= ocap && ok1) {
                L.st = HPK_OUTPUT_OVERFLOW;
                break;
            }
            // room for the first code only: take it; the second one is the overflow, next round
            ok2 = false;
            g = 1u;
            u = HPK_L2_LEN0(e);
        }
        if (ok1) dst[L.cnt] = (uint8_t)e;
        if (ok2) dst[L.cnt + 1u] = (uint8_t)(e >> 16);
        if (!ok1) {
            if (L.rem <= (uint32_t)HPK_LUT_BITS) break;  // nothing fits in the bits left: the end
            // a 13..30-bit code or EOS: one leading-ones lookup (the window holds >= 33 bits)
            uint32_t sy, len;
            bool eos;
            lo_decode(w, a.lo, sy, len, eos);
            if (len > L.rem) break;  // huffman.rs:128-134 (> 12 bits left: PaddingTooLarge below)
            if (eos) {               // huffman.rs:112-116
                L.st = HPK_EOS_IN_STRING;
                break;
            }
            if (chk && L.cnt >= ocap) {
                L.st = HPK_OUTPUT_OVERFLOW;
                break;
            }
            dst[L.cnt] = (uint8_t)sy;
            g = 1u;
            u = len;
        }
        L.cnt += g;
        L.win <<= u;
        L.nb -= u;
        L.rem -= u;
        L.live = L.rem != 0u;
    }
    a.out_len[i] = L.cnt;
    a.status[i] = (uint8_t)lit_status(L);
}

}  // namespace hpkdec
