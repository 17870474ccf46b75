// hpk_decode.hip — gfx950 batched Huffman literal decode (the hot path).
//
// Replaces, for a batch of literals at once, the Huffman branch of decode_string
// (crates/loona-hpack/src/decoder.rs:143-157) i.e. HuffmanDecoder::decode
// (crates/loona-hpack/src/huffman.rs:95-161), with identical results per literal: decoded bytes,
// and status Ok / PaddingTooLarge / InvalidPadding / EOSInString with the reference's precedence.
//
// Work decomposition (kernel template hpk_decode12 in hpk_decode12.h):
//   * one 1024-thread workgroup per CU (16 waves) owns a contiguous literal range (n / CUs); the
//     decode tables (16 KiB two-symbol table, 1.9 KiB leading-ones table) are staged into LDS once;
//   * the range is decoded in fills: a 40 KiB LDS input window (big-endian dwords), an LDS image
//     of the fill's output span and a queue of up to 2048 literals ordered longest-first (counting
//     sort on the encoded length). The next fill's offsets and window are loaded into registers
//     while the current fill decodes, the previous fill's image is written back with 16-byte
//     stores while it decodes; barriers order LDS only;
//   * literals of >= 224 encoded bytes (the queue's head) are decoded one per wave, cooperatively:
//     64 lanes walk 64 segments from speculative starts and re-walk from their neighbours' true
//     stops until nothing changes (Huffman walks resynchronise within a few codes);
//   * the other literals are decoded one per lane out of LDS in a static snake over the
//     longest-first queue: lane i takes slots i and 2*1024-1-i (the longest with the shortest),
//     the second literal's entry and first window dwords read while the first one decodes, so a
//     lane moves on without waiting for LDS;
//   * a step is two lookups in the 12-bit two-symbol table, each decoding up to two codes of
//     <= 12 bits, from a 32-bit window made by ONE v_alignbit out of a register-held dword pair;
//     a code longer than 12 bits (or EOS) takes one leading-ones lookup (any code in one read).
//     Bits past a literal's end are NOT masked: a code that runs past the end is, by
//     prefix-freeness, longer than what is left whatever follows, so the walk stops exactly where
//     huffman.rs's bit iterator stops matching; only the final padding check (huffman.rs:128-160)
//     looks at the residual bits;
//   * a literal whose output capacity is below hpk_decoded_bound (caller-chosen offsets) is decoded
//     after the queue drains, code by code with a capacity check per byte (HPK_OUTPUT_OVERFLOW).
// A literal too large for the window is decoded by one lane straight from global memory.
#include <stdlib.h>

#include "hpk_decode12.h"

using namespace hpkdec;

// Product geometry (v12): 16 waves (one 1024-thread workgroup) per CU; per fill a 40 KiB input
// window, a 77 KiB output image and a 2048-entry longest-first queue, plus the 16 KiB two-symbol
// table; two lookups per step, lanes check for a finished literal every 2 steps, static snake
// schedule, byte stores into the image (bench/kvariants: profiles/r01/kvariants_v1[23]*.jsonl).
#ifndef HPK_REFILLN
#define HPK_REFILLN 2  // lane steps between two finish checks
#endif
constexpr int kWaves = 16, kW = 40960, kO = 79104, kQ = 2048, kRefillN = HPK_REFILLN, kChunk = 64, kLook = 2, kSched = 1;
constexpr bool kAcc = false;
constexpr int kCoop = 0;  // (v16: literals of >= 224 encoded bytes one wave each; v19: hpk_decode_long)
#ifndef HPK_LONGK
#define HPK_LONGK 1
#endif
#ifndef HPK_SPREAD
#define HPK_SPREAD 0
#endif
constexpr int kLongK = HPK_LONGK;  // long literals left to the long-literal phase (hpk_long.h)
constexpr int kSpread = HPK_SPREAD;  // lane-queue slots interleaved over the waves (fills of few literals use every SIMD)
#ifndef HPK_LONG_MIN
#define HPK_LONG_MIN 64  // encoded bytes: literals from here on go to the long-literal phase
#endif
#ifndef HPK_LONG_BIG
#define HPK_LONG_BIG 1024  // the long-literal phase takes these first (longest-first, roughly)
#endif
using Geo = Geo12<kWaves, kW, kO, kQ>;
#ifndef HPK_LONGDYN
#define HPK_LONGDYN 1
#endif
#ifndef HPK_DEFER
#define HPK_DEFER 0
#endif
constexpr int kLongDyn = HPK_LONGDYN;     // long literals: waves take the next one from an LDS counter
constexpr int kDefer = HPK_DEFER;  // the previous fill's write-back issued during this decode
#ifndef HPK_PREDST
#define HPK_PREDST 1
#endif
constexpr int kPredSt = HPK_PREDST;  // unconditional byte stores in the lane step (dummy slots)
#define DEC_KERNEL(m) hpk_decode12<m, kWaves, kW, kO, kQ, kRefillN, kChunk, kLook, kAcc, kCoop, kSched, kLongDyn, kDefer, kPredSt, \
                                   kSpread, 512, 0, 1, 15, 32, kLongK>

#ifdef HPK_DIAG
// Diagnostic build (libhpk_diag.so, `make diag`; never the product library): HPK_DEBUG_MODE selects
// 1 no decode, 2 no output stores, 3 per-wave stamps (16 x u64 per wave, hpk_debug_stamps),
// 4 every store bounds-checked (hpk_debug_check).
static int g_debug_mode = -1;
static unsigned long long* g_dbg = nullptr;
static size_t g_dbg_n = 0;

extern "C" int hpk_debug_check(unsigned long long* host8) {
    return hipMemcpyFromSymbol(host8, HIP_SYMBOL(g_chk), 8 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}

extern "C" int hpk_debug_stamps(unsigned long long* host, size_t cap_entries) {
    if (!g_dbg) return 0;
    size_t n = g_dbg_n < cap_entries ? g_dbg_n : cap_entries;
    if (hipMemcpy(host, g_dbg, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return (int)n;
}
#endif

int hpk_launch_decode(hpk_ctx* c, const hpk_batch& b) {
    DecodeArgs a;
    const uintptr_t ip = (uintptr_t)b.in_blob;
    a.in_base = (const uint8_t*)(ip & ~(uintptr_t)15);
    a.in_mis = (uint32_t)(ip & 15);
    a.in_off = b.in_off;
    a.n = b.n;
    const uintptr_t op = (uintptr_t)b.out_blob;
    a.out_base = (uint8_t*)(op & ~(uintptr_t)15);
    a.out_mis = (uint32_t)(op & 15);
    a.out_off = b.out_off;
    a.out_len = b.out_len;
    a.status = b.status;
    a.t8 = c->d_t8;
    a.lo = c->d_lo;
    a.lut = c->d_lut;
    a.lut2 = c->d_lut2;
    a.dbg = nullptr;
    a.in_cap = b.in_cap;
    a.out_cap = b.out_cap;
    a.err = c->d_err;
    uint32_t* ll = nullptr;
    int lslot = 0;
    if (int rc = hpk_long_list(c, b.n, &ll, &lslot)) return rc;
    a.long_list = ll;
    a.long_min = HPK_LONG_MIN;
    a.long_big = HPK_LONG_BIG;
#ifdef HPK_DIAG
    if (const char* lm = getenv("HPK_LONG_MIN")) a.long_min = (uint32_t)atoi(lm);
    if (const char* lb = getenv("HPK_LONG_BIG")) a.long_big = (uint32_t)atoi(lb);
#endif
    // one workgroup per CU; fewer when the batch is small (>= ~64 literals per workgroup)
    uint64_t blocks = ((uint64_t)b.n + 63) / 64;
    if (blocks > (uint64_t)c->num_cu) blocks = (uint64_t)c->num_cu;
    if (blocks < 1) blocks = 1;
    const dim3 grid((uint32_t)blocks), block(Geo::kBlock);
#ifdef HPK_DIAG
    if (g_debug_mode < 0) {
        const char* dm = getenv("HPK_DEBUG_MODE");
        g_debug_mode = dm ? atoi(dm) : 0;
    }
    switch (g_debug_mode) {
        case 1:
            hipLaunchKernelGGL(DEC_KERNEL(1), grid, block, 0, c->stream, a);
            break;
        case 2:
            hipLaunchKernelGGL(DEC_KERNEL(2), grid, block, 0, c->stream, a);
            break;
        case 3: {
            const size_t need = (size_t)blocks * kWaves * 16;
            if (need > g_dbg_n) {
                (void)hipFree(g_dbg);
                HIP_TRY(hipMalloc(&g_dbg, need * 8));
                g_dbg_n = need;
            }
            a.dbg = g_dbg;
            hipLaunchKernelGGL(DEC_KERNEL(3), grid, block, 0, c->stream, a);
            break;
        }
        case 4:
            hipLaunchKernelGGL(DEC_KERNEL(4), grid, block, 0, c->stream, a);
            break;
        case 5: {  // the product kernel with per-wave counters of the long-literal phase (8 waves)
            const size_t need = (size_t)blocks * 8 * 16;
            if (need > g_dbg_n) {
                (void)hipFree(g_dbg);
                HIP_TRY(hipMalloc(&g_dbg, need * 8));
                g_dbg_n = need;
            }
            HIP_TRY(hipMemsetAsync(g_dbg, 0, need * 8, c->stream));
            a.dbg = g_dbg;
            hipLaunchKernelGGL(DEC_KERNEL(5), grid, block, 0, c->stream, a);
            break;
        }
        default:
            hipLaunchKernelGGL(DEC_KERNEL(0), grid, block, 0, c->stream, a);
    }
#else
    hipLaunchKernelGGL(DEC_KERNEL(0), grid, block, 0, c->stream, a);
#endif
    HIP_TRY(hipGetLastError());
    return hpk_long_list_used(c, lslot);
}
