// hpk_decode.hip — gfx950 batched Huffman literal decode (the hot path).
//
// Replaces, for a batch of literals at once, the Huffman branch of decode_string
// (crates/loona-hpack/src/decoder.rs:143-157) i.e. HuffmanDecoder::decode
// (crates/loona-hpack/src/huffman.rs:95-161), with identical results per literal: decoded bytes,
// and status Ok / PaddingTooLarge / InvalidPadding / EOSInString with the reference's precedence.
//
// Work decomposition (kernel template hpk_decode7 in hpk_decode_kernel.h, step 8):
//   * one 1024-thread workgroup per CU (16 waves) owns a contiguous literal range (n / CUs); the
//     decode tables (16 KiB two-symbol table, 1.9 KiB leading-ones table) are staged into LDS once;
//   * the range is decoded in fills: a 40 KiB LDS input window, an LDS image of the fill's output
//     span and a queue of up to 2048 literals ordered longest-first (counting sort on the encoded
//     length: LPT list scheduling keeps the end-of-fill tail short). The next fill's offsets and
//     window are loaded into registers while the current fill decodes, the previous fill's image
//     is written back with 16-byte stores while it decodes; barriers order LDS only;
//   * lanes decode one literal each out of LDS; free lanes take the next queue slots every 6 steps
//     (ballot + mbcnt) from a per-wave reservation topped up 64 slots at a time with one LDS
//     atomic, so waves the SIMD's age-priority arbitration favours simply take more literals;
//   * a step refills a 64-bit bit window from a dword read one step ahead, looks the next 12 bits
//     up in the two-symbol table and writes up to two symbols straight into the output image; a
//     code longer than 12 bits (or EOS) takes one leading-ones lookup (any code in one read).
//     Bits past a literal's end are NOT masked: a code that runs past the end is, by
//     prefix-freeness, longer than what is left whatever follows, so the walk stops exactly where
//     huffman.rs's bit iterator stops matching; only the final padding check (huffman.rs:128-160)
//     looks at the residual bits, masked;
//   * a literal whose output capacity is below hpk_decoded_bound (caller-chosen offsets) is decoded
//     after the queue drains, code by code with a capacity check per byte (HPK_OUTPUT_OVERFLOW).
// A literal too large for the window is decoded by one lane straight from global memory.
#include <stdlib.h>

#include "hpk_decode_kernel.h"

using namespace hpkdec;

// Product geometry (v8): 16 waves (one 1024-thread workgroup) per CU; per fill a 40 KiB input
// window, a 77 KiB output image and a 2048-entry longest-first queue, plus the 16 KiB two-symbol
// table; lanes refill every 6 steps, waves reserve 64 queue slots at a time (bench/kvariants).
constexpr int kWaves = 16, kW = 40960, kO = 79104, kQ = 2048, kRefillN = 6, kChunk = 64, kStep = 8;
using Geo = Geo7<kWaves, kW, kO, kQ, true>;
#define DEC_KERNEL(m) hpk_decode7<m, kWaves, kW, kO, kQ, kRefillN, kChunk, kStep>

static int g_debug_mode = -1;

int hpk_decode_setup() {
    static int rc = -1;
    static bool done = false;
    if (!done) {
        const char* dm = getenv("HPK_DEBUG_MODE");
        g_debug_mode = dm ? atoi(dm) : 0;
        const void* fns[5] = {reinterpret_cast<const void*>(&DEC_KERNEL(0)), reinterpret_cast<const void*>(&DEC_KERNEL(1)),
                              reinterpret_cast<const void*>(&DEC_KERNEL(2)), reinterpret_cast<const void*>(&DEC_KERNEL(3)),
                              reinterpret_cast<const void*>(&DEC_KERNEL(4))};
        rc = HPK_E_OK;
        for (int i = 0; i < 5 && rc == HPK_E_OK; ++i) {
            (void)fns[i];  // the decode kernel's LDS is static (no dynamic-size attribute needed)
        }
        done = true;
    }
    return rc;
}

// diagnostic stamps buffer (HPK_DEBUG_MODE=3): 4 x u64 per wave
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

int hpk_launch_decode(hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                      const uint32_t* out_off, uint32_t* out_len, uint8_t* status) {
    int rc = hpk_decode_setup();
    if (rc) return rc;
    DecodeArgs a;
    const uintptr_t ip = (uintptr_t)in_blob;
    a.in_base = (const uint8_t*)(ip & ~(uintptr_t)15);
    a.in_mis = (uint32_t)(ip & 15);
    a.in_off = in_off;
    a.n = n;
    const uintptr_t op = (uintptr_t)out_blob;
    a.out_base = (uint8_t*)(op & ~(uintptr_t)15);
    a.out_mis = (uint32_t)(op & 15);
    a.out_off = out_off;
    a.out_len = out_len;
    a.status = status;
    a.t8 = c->d_t8;
    a.lo = c->d_lo;
    a.lut = c->d_lut;
    a.dbg = nullptr;
    // one workgroup per CU; fewer when the batch is small (>= ~64 literals per workgroup)
    uint64_t blocks = ((uint64_t)n + 63) / 64;
    if (blocks > (uint64_t)c->num_cu) blocks = (uint64_t)c->num_cu;
    if (blocks < 1) blocks = 1;
    const dim3 grid((uint32_t)blocks), block(Geo::kBlock);
    const int lds = 0;  // static LDS
    switch (g_debug_mode) {
        case 1:
            hipLaunchKernelGGL(DEC_KERNEL(1), grid, block, lds, c->stream, a);
            break;
        case 2:
            hipLaunchKernelGGL(DEC_KERNEL(2), grid, block, lds, c->stream, a);
            break;
        case 3: {
            const size_t need = (size_t)blocks * kWaves * 4;
            if (need > g_dbg_n) {
                (void)hipFree(g_dbg);
                HIP_TRY(hipMalloc(&g_dbg, need * 8));
                g_dbg_n = need;
            }
            a.dbg = g_dbg;
            hipLaunchKernelGGL(DEC_KERNEL(3), grid, block, lds, c->stream, a);
            break;
        }
        case 4:
            hipLaunchKernelGGL(DEC_KERNEL(4), grid, block, lds, c->stream, a);
            break;
        default:
            hipLaunchKernelGGL(DEC_KERNEL(0), grid, block, lds, c->stream, a);
    }
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}
