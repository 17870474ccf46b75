// hpk_decode_kernel.h — building blocks of the gfx950 decode kernel (hpk_decode12.h; design
// notes in hpk_decode.hip): kernel arguments, LDS carve-up, the code-by-code byte path, the
// longest-first bucket, fill prefetch. Earlier kernels built on them (v3-v11) are in git history
// (bench/legacy_decode*.h until round 3).
#pragma once
#include <stdint.h>

#include "hpk_device.h"

namespace hpkdec {

// Tables in LDS (once per workgroup): T8 (256 B, symbols of the <= 8-bit codes) and the
// leading-ones table LO (1.9 KiB, any code). 16-byte aligned carve-outs.
constexpr int kT8Bytes = 256;
constexpr int kLoBytes = HPK_LO_SIZE * 2;
constexpr int kTabBytes = ((kT8Bytes + kLoBytes + 15) / 16) * 16;

struct DecodeArgs {
    const uint8_t* in_base;  // in_blob rounded down to 16 bytes
    uint32_t in_mis;         // in_blob - in_base (0..15)
    const uint32_t* in_off;
    uint32_t n;
    uint8_t* out_base;  // out_blob rounded down to 16 bytes
    uint32_t out_mis;   // out_blob - out_base (0..15)
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
    const uint8_t* t8;
    const uint16_t* lo;
    const uint32_t* lut;  // two-symbol table (hpk_code.h), step 8
    const uint32_t* lut2; // the same in the LUT2 layout (decode v12)
    const uint32_t* lut3; // the same in the LUT3 layout (decode v28, the wave kernel's long and huge phases)
    unsigned long long* dbg;  // diagnostic builds only: per-wave timestamps
    uint32_t in_cap, out_cap;  // blob sizes (clamped to HPK_MAX_OFFSET): larger offsets are bad
    uint32_t* err;             // sticky error flag (host-mapped): set to 1 on bad offsets
    // kLongK: literals of >= long_min encoded bytes (region >= the decoded bound) are left to the
    // long-literal phase (hpk_long.h): fill workgroup g lists them in long_list[its literal range),
    // those of >= long_big bytes from the front, the others from the back
    uint32_t* long_list;
    uint32_t long_min, long_big;
    // where the long- and huge-literal phases write literal i: lit_out[i] (out_off; in the compacted
    // mode the compacted offsets co_off, allocated when the literal is listed)
    const uint32_t* lit_out;
    // compacted mode (hpk_decode_batch_compact): co_off[i] = where literal i's bytes went, allocated from
    // the device cursor *cursor per fill (fill literals) or per listed literal (its decoded bound)
    uint32_t* co_off;
    uint32_t* cursor;
};

// Huge literals (hpk_huge.h) listed per workgroup in LDS; more go to the long-literal phase.
constexpr uint32_t kHugeMax = 16;

// Per-lane state of the literal being decoded.
struct Lit {
    uint64_t win;   // next bits, MSB-aligned (bits past the literal: whatever follows)
    uint32_t nb;    // loaded bits in win
    uint32_t nxt;   // next source dword (raw), merged at the next refill
    uint32_t pf;    // the dword after it (raw, read one refill ahead)
    uint32_t q;     // source dword index of pf
    uint32_t rem;   // literal bits not yet consumed
    uint32_t cnt;   // bytes decoded
    uint32_t st;    // hpk_status
    uint64_t acc;   // pending output bytes (little-endian order)
    uint32_t accn;  // bytes in acc
    uint32_t od;    // output dword index (dword stores) or byte position (byte stores)
    uint32_t ocap;  // output capacity (byte stores only)
    uint32_t oend;  // diagnostic mode 4: one past the last output dword of the literal
    bool live;      // still decoding
    bool park;      // step 7: waiting at the next refill point for a leading-ones lookup
};

enum StoreMode { kDword = 0, kNoStore = 1, kChecked = 3, kPred = 4 };  // kPred: kDword, lane steps store
// unconditionally, a byte that is not output going to a per-lane dummy slot

// Bitstream sources: a staged LDS window, or global memory (clamped to the batch).
struct LdsSrc {
    const uint32_t* p;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return p[i]; }
};
struct GlobalSrc {
    const uint32_t* p;
    uint32_t last;  // last dword index holding a byte of the batch: never read past it
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return p[min(i, last)]; }
};


// diagnostic mode 4: record the first out-of-region store instead of performing it
__device__ unsigned long long g_chk[8];
__device__ __forceinline__ void chk_report(uint32_t code, uint32_t a0, uint32_t a1, uint32_t a2) {
    if (atomicCAS(&g_chk[0], 0ull, (unsigned long long)code) == 0ull) {
        g_chk[1] = a0;
        g_chk[2] = a1;
        g_chk[3] = a2;
        g_chk[4] = blockIdx.x;
        g_chk[5] = threadIdx.x;
    }
}

template <class Src>
__device__ __forceinline__ void lit_begin(Lit& L, const Src& src, uint32_t sb, uint32_t nbytes) {
    L.rem = nbytes * 8u;
    L.cnt = 0;
    L.st = HPK_OK;
    L.live = nbytes != 0;
    L.acc = 0;
    L.accn = 0;
    const uint32_t q0 = sb >> 2;
    const uint32_t sk = (sb & 3u) * 8u;
    const uint32_t d0 = src(q0);
    L.nxt = src(q0 + 1);
    L.pf = src(q0 + 2);
    L.q = q0 + 2;
    L.win = ((uint64_t)hpk_bswap32(d0) << 32) << sk;
    L.nb = 32u - sk;
}

// Top the window up to >= 32 bits from the prefetched dword; read the next one.
template <class Src>
__device__ __forceinline__ void lit_refill(Lit& L, const Src& src) {
    const bool need = L.nb <= 32u;
    const uint64_t add = (uint64_t)hpk_bswap32(L.nxt) << ((32u - L.nb) & 63u);
    L.win |= need ? add : 0ull;
    L.nb += need ? 32u : 0u;
    L.nxt = need ? L.pf : L.nxt;
    L.q += need ? 1u : 0u;
    L.pf = src(L.q);
}

// Decode one code of any length from the window (>= 30 loaded bits): leading-ones table.
__device__ __forceinline__ void lo_decode(uint32_t w, const uint16_t* __restrict__ lo, uint32_t& sym,
                                          uint32_t& len, bool& eos) {
    const uint32_t kk = __clz(~w);
    const uint32_t e = lo[min(kk, (uint32_t)HPK_LO_RUNS - 1) * 32 + ((w << ((kk + 1) & 31)) >> 27)];
    eos = kk >= HPK_LO_RUNS || (e & 0x1FFu) == HPK_EOS;
    sym = e & 0xFFu;
    len = eos ? 30u : (e >> 9);
}

// Append g (<= 4) bytes to the pending output; store a whole dword when one is complete.
struct LdsSwapSrc {
    const uint32_t* p;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return __builtin_bswap32(p[i]); }
};

// v10 step: lit_step8 for two literals of a lane at once (kStep 10). All LDS reads of both
// (prefetch dwords, table entries) are issued before any byte store, so the two literals' LDS
// round trips overlap; the long-code branch runs once for both.
__device__ __forceinline__ uint32_t lit_status(const Lit& L) {
    uint32_t st = L.st;
    if (st == HPK_OK && L.rem > 0) {
        if (L.rem > 7) {
            st = HPK_PADDING_TOO_LARGE;
        } else {
            const uint32_t w = (uint32_t)(L.win >> 32) | (0xFFFFFFFFu >> L.rem);
            if (w != 0xFFFFFFFFu) st = HPK_INVALID_PADDING;
        }
    }
    return st;
}

// ------------------------------------------------------------------------------------------
// v7: output staged in LDS too, queue in longest-first order.
//
// PMC on v5 showed 163 MB of HBM writes per launch for 41 MB of output: every lane stores its
// own literal's dwords whenever they complete, so a 64-B sector is written several times (by
// the lane itself as the L2 evicts the half-written line, and by the neighbouring literal's
// lane at the boundary). Here each fill decodes into an LDS image of its output span and the
// workgroup writes the span back with 16-byte stores, exact bytes; out_len and status are
// staged and written back coalesced as well. LDS is then shared by an input window, the
// output image (1.6x + rounding) and the queue, so fills are ~2.5x smaller; the load balance
// that costs is won back by ordering each fill's queue longest-first (a counting sort on the
// encoded length: LPT list scheduling, the tail is made of short literals).
template <int kWaves, int kW, int kO, int kQ, bool kLut = false>
struct Geo7 {
    static constexpr int kBlock = kWaves * 64;
    static constexpr int kMetaRounds = (kQ + kBlock - 1) / kBlock;
    static constexpr int kStageRounds = (kW / 16 + kBlock - 1) / kBlock;
    static constexpr int kFlushRounds = (kO / 16 + 1 + kBlock - 1) / kBlock;
    static constexpr int kLutBytes = kLut ? (int)(HPK_LUT_SIZE * 4) : 0;
    static constexpr int kLutOff = kTabBytes;
    static constexpr int kInOff = kTabBytes + kLutBytes;
    static constexpr int kOutOff = kInOff + kW;
    static constexpr int kQOff = kOutOff + kO;
    static constexpr int kLenOff = kQOff + 8 * kQ;
    static constexpr int kHistOff = kLenOff + 4 * kQ;  // 64 bucket counts + 64 bucket bases
    static constexpr int kCtrOff = kHistOff + 512;
    static constexpr int kLdsBytes = kCtrOff + 16;
    static_assert(kLdsBytes <= 163840, "LDS budget (160 KiB per CU on gfx950)");
    static_assert(kW % 16 == 0 && kW <= 65536, "window offsets and lengths pack in 16 bits");
    static_assert(kO % 16 == 0 && kO <= 131072, "output byte offset packs in 17 bits");
    static_assert(kQ <= 4096, "fill index packs in 12 bits");
};
constexpr uint32_t kQ7Byte = 0x80000000u;  // queue entry .y flag: byte path

// Longest-first bucket of an encoded length (0 = longest): 2-byte classes up to 94 B, then
// 128-byte classes.
__device__ __forceinline__ uint32_t lpt_bucket(uint32_t nbytes) {
    const uint32_t b = nbytes < 96u ? (nbytes >> 1) : min(63u, 48u + ((nbytes - 96u) >> 7));
    return 63u - b;
}

// One literal decoded code by code into a byte destination with a capacity check per byte.
template <class Src, class Dst>
__device__ __forceinline__ void lit_bytes_to(Lit& L, const Src& src, const uint16_t* lo, Dst dst, uint32_t ocap,
                                             uint32_t sb, uint32_t nbytes) {
    lit_begin(L, src, sb, nbytes);
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
        dst(L.cnt, (uint8_t)sym);
        L.cnt += 1;
        L.win <<= len;
        L.nb -= len;
        L.rem -= len;
        L.live = L.rem != 0u;
    }
}

// Workgroup barrier that orders LDS only: outstanding global stores (the previous fill's
// write-back) and prefetch loads stay in flight across it. __syncthreads() would wait for them.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Registers of the next fill, loaded while the current one decodes: the offsets of up to kQ
// literals and the whole kW-byte input window (clamped to the batch).
template <int kMeta, int kStage>
struct Prefetch {
    uint32_t io0[kMeta], io1[kMeta], oo0[kMeta], oo1[kMeta];
    uint4 chunk[kStage];
};

template <int kBlock, int kMeta, int kStage>
__device__ __forceinline__ void prefetch_fill(Prefetch<kMeta, kStage>& P, const DecodeArgs& a, uint32_t tid,
                                              uint32_t cur, uint32_t end, uint32_t base16, uint32_t last16) {
    const uint32_t cntl = end - cur;  // >= 1
#pragma unroll
    for (int r = 0; r < kMeta; ++r) {
        const uint32_t t = min(tid + (uint32_t)kBlock * r, cntl - 1);
        P.io0[r] = a.in_off[cur + t];
        P.io1[r] = a.in_off[cur + t + 1];
        P.oo0[r] = a.out_off[cur + t];
        P.oo1[r] = a.out_off[cur + t + 1];
    }
    const uint4* g16 = reinterpret_cast<const uint4*>(a.in_base);
#pragma unroll
    for (int r = 0; r < kStage; ++r) P.chunk[r] = g16[min((base16 >> 4) + tid + (uint32_t)kBlock * r, last16)];
}

}  // namespace hpkdec
