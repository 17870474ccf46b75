// bench/legacy_wave_mk.h — rejected (v25c): dword output of the wave kernel's lane walk by LDS
// masked OR (ds_mskor_b32), one LDS store per step instead of four byte stores, safe for any region
// alignment. Bit-exact on config 5 / config 2 but slower: 1223-1229 us vs 998-1013 us per 32M-literal
// launch (gpurun_out r3o); kept for the record, not built.
#pragma once
#include "../loona_amd/csrc/hpk_decode12.h"

namespace hpkdec {

// LDS byte address of a pointer into the kernel's shared memory.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// ds_mskor_b32: the LDS dword at `addr` becomes (old & ~mask) | data, atomically (data is zero
// outside mask). No return value, so nothing waits for it; a wave's LDS operations complete in
// order, so the write-back's reads (compiler-issued, waited for) come after it.
__device__ __forceinline__ void lds_mskor(uint32_t addr, uint32_t mask, uint32_t data) {
    asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(addr), "v"(mask), "v"(data));
}

// Dword output (v25c): a lane gathers its literal's bytes on the image's dword grid and stores each
// dword once it is complete, with ONE masked OR (6 LDS cycles) per step instead of four byte
// stores (16 cycles: address + data per ds_write_b8). The masked OR makes any region alignment
// safe: the bytes of a literal's first dword below its first byte belong to the region before it
// (another lane may be writing them), so they are masked off; the last, partial dword is stored
// with the mask of the bytes the literal holds (mk_tail). A step that completes no dword stores to
// the lane's dummy dword (no exec-mask branch).
// Append g (<= 4) decoded bytes p (little-endian, zero above them) at image byte o; acc holds the
// bytes of o's dword below o (zero below the literal's first byte o0).
__device__ __forceinline__ void mk_append(uint32_t& o, uint32_t& acc, uint32_t o0, uint32_t img, uint32_t dmy,
                                          uint32_t p, uint32_t g) {
    const uint32_t n = o & 3u;
    const uint64_t x = (uint64_t)p << (8u * n);
    const uint32_t lo32 = acc | (uint32_t)x;
    const bool full = n + g >= 4u;
    const uint32_t head = (o ^ o0) < 4u ? o0 & 3u : 0u;  // o's dword is the literal's first
    lds_mskor(full ? img + (o & ~3u) : dmy, 0xFFFFFFFFu << (8u * head), lo32);
    acc = full ? (uint32_t)(x >> 32) : lo32;
    o += g;
}

// A literal's last, partial dword (bytes [head, o & 3) of o's dword).
__device__ __forceinline__ void mk_tail(uint32_t o, uint32_t acc, uint32_t o0, uint32_t img) {
    const uint32_t n = o & 3u;
    if (n) {
        const uint32_t head = (o ^ o0) < 4u ? o0 & 3u : 0u;
        const uint32_t mask = ((1u << (8u * n)) - 1u) & (0xFFFFFFFFu << (8u * head));
        lds_mskor(img + (o & ~3u), mask, acc & mask);
    }
}

// lit12_step with dword output: the step's (up to four) bytes are packed with v_perm and appended.
__device__ __forceinline__ void lit12_step_mk(Lit12& L, uint32_t& acc, const uint32_t* __restrict__ win32,
                                              const uint32_t* __restrict__ lut, const uint16_t* __restrict__ lo,
                                              uint32_t img, uint32_t dmy) {
    const uint32_t d3 = win32[(L.X >> 5) + 2];
    const uint32_t w = __builtin_amdgcn_alignbit(L.d0, L.d1, ~L.X);
    const uint32_t rem = L.Eb - L.X;
    const uint32_t e1 = lut[w >> (32 - HPK_LUT_BITS)];
    bool a1, a2;
    const uint32_t u1 = lut12(e1, rem, a1, a2);
    bool park = !a1 & (rem > (uint32_t)HPK_LUT_BITS);
    const bool cont = a1 & (a2 | (e1 >= HPK_LUT2_NOTTWO));
    const uint32_t w2 = w << u1;
    const uint32_t rem2 = rem - u1;
    const uint32_t e2 = lut[w2 >> (32 - HPK_LUT_BITS)];
    bool b1, b2;
    const uint32_t u2 = lut12(e2, rem2, b1, b2);
    park |= cont & !b1 & (rem2 > (uint32_t)HPK_LUT_BITS);
    b1 &= cont;
    b2 &= cont;
    const uint32_t g1 = (uint32_t)a1 + (uint32_t)a2, g2 = (uint32_t)b1 + (uint32_t)b2;
    mk_append(L.o, acc, L.o0, img, dmy, lut12_bytes(e1, g1) | (lut12_bytes(e2, g2) << (8u * g1)), g1 + g2);
    const uint32_t xn = L.X + u1 + (cont ? u2 : 0u);
    const bool cross = (xn ^ L.X) > 31u;
    L.d0 = cross ? L.d1 : L.d0;
    L.d1 = cross ? L.d2 : L.d1;
    L.d2 = cross ? d3 : L.d2;
    L.X = xn;
    L.prog = a1 | park;
    if (park) {  // a 13..30-bit code or EOS: one leading-ones lookup (any code in one read)
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
            mk_append(L.o, acc, L.o0, img, dmy, sy, 1u);
            L.X += len;
            lit12_load(L, win32);
        }
    }
}

}  // namespace hpkdec
