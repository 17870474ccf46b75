// hpk_decode.hip — gfx950 batched Huffman literal decode (the hot path).
//
// Replaces, for a batch of literals at once, the Huffman branch of decode_string
// (crates/loona-hpack/src/decoder.rs:143-157) i.e. HuffmanDecoder::decode
// (crates/loona-hpack/src/huffman.rs:95-161), with identical results per literal: decoded bytes,
// and status Ok / PaddingTooLarge / InvalidPadding / EOSInString with the reference's precedence.
//
// Two kernels, identical results (tests/test_gpu.py runs every case through both):
//   * hpk_decode_wave (v25, hpk_wave.h), for large batches: every wave of a 1024-thread workgroup
//     decodes its own fills of <= 128 literals (two per lane, longest with shortest) out of its own
//     LDS window into its own LDS image, with no barrier between fills, so the waves' memory traffic
//     and setup overlap each other's decoding; the workgroup's range is handed out in chunks;
//   * hpk_decode12 (v24, hpk_decode12.h), for small batches: one workgroup-wide fill at a time per
//     CU (40 KiB window, 77 KiB image, 2048-literal longest-first queue), the next fill's loads in
//     flight during the decode, the previous image written back around it.
// Both use the same lane walk (hpk_decode12.h): a step is two lookups in the 12-bit two-symbol
// table, each decoding up to two codes of <= 12 bits, from a 32-bit window made by ONE v_alignbit
// out of a register-held dword pair; a longer code (or EOS) takes one leading-ones lookup. Bits past
// a literal's end are not masked: a code that runs past the end is, by prefix-freeness, longer than
// what is left whatever follows, so the walk stops exactly where huffman.rs's bit iterator stops
// matching; only the final padding check (huffman.rs:128-160) looks at the residual bits. Literals
// of >= 64 encoded bytes go to the long-literal phase (hpk_long.h), one lane each streaming from
// HBM, after the fills; a literal whose output region is below hpk_decoded_bound is decoded code by
// code with a capacity check per byte (HPK_OUTPUT_OVERFLOW).
#include <stdlib.h>

#include <chrono>


#include "hpk_wave.h"
#include "hpk_persist.h"

using namespace hpkdec;

// Workgroup-fill kernel (v24, hpk_decode12.h): 16 waves (one 1024-thread workgroup) per CU; per
// fill a 40 KiB input window, a 77 KiB output image and a 2048-entry longest-first queue, plus the
// 16 KiB two-symbol table; lanes check for a finished literal every 2 steps.
constexpr int kWaves = 16, kW = 40960, kO = 79104, kQ = 2048, kRefillN = 2;
// long-literal phase (hpk_long.h, both kernels): literals of >= HPK_LONG_MIN encoded bytes, those of
// >= HPK_LONG_BIG first (longest-first, roughly)
#ifndef HPK_LONG_MIN
#define HPK_LONG_MIN 64
#endif
#ifndef HPK_LONG_BIG
#define HPK_LONG_BIG 1024
#endif
using Geo = Geo12<kWaves, kW, kO, kQ>;
// Wave-fill kernel (v25, hpk_wave.h): per wave a 3 KiB window and a 5.75 KiB image, the workgroup's
// range handed out in chunks of 224 literals; for batches of at least HPK_WAVE_MIN literals (smaller
// ones keep the workgroup-fill kernel) unless the context says otherwise (hpk_ctx_set_decode_kernel)
constexpr int kWaveWin = 3072, kWaveImg = 5888;
#ifndef HPK_WAVE_MIN
#define HPK_WAVE_MIN 0u  // (round 6: the wave kernel for every batch; it had been 4M: config 2 40.3-40.8 vs 47.1-47.3 us
                         // for the workgroup-fill kernel, 1k-literal synchronous calls 21.5 vs 24.4 us)
#endif
#ifndef HPK_WAVE_GUIDED
#define HPK_WAVE_GUIDED 1  // chunks claimed by the waves (1: guided self-scheduling, 2: fixed HPK_WAVE_CHUNK) vs a static 1/16 each (0)
#endif
#ifndef HPK_WAVE_RANK
#define HPK_WAVE_RANK 0  // longest-first order: 0 LDS counting sort (32 classes), 1/2 ballots (16/32 classes)
#endif
#ifndef HPK_WAVE_CHUNK
#define HPK_WAVE_CHUNK 224u  // least literals per chunk claim
#endif
#define WAVE_KERNEL(m) hpk_decode_wave<m, kWaveWin, kWaveImg, HPK_WAVE_CHUNK, HPK_WAVE_GUIDED, HPK_WAVE_RANK>
// (round 6) batches below HPK_WAVE_GUIDED_MIN literals hand their workgroups' ranges out in fixed chunks of
// about one fill (config 2 with 104-literal chunks: 43.7-43.9 us against 51.1 guided, 44.1-45.0 static, 46.9
// for the workgroup-fill kernel; with the overlapped start, hpk_wave.h, and 96-literal chunks 40.3-40.6)
#ifndef HPK_WAVE_GUIDED_MIN
#define HPK_WAVE_GUIDED_MIN 4000000u
#endif
#ifndef HPK_WAVE_SMALL_CHUNK
#define HPK_WAVE_SMALL_CHUNK 96u  // (config 2: 88 43.1-43.5, 92 40.5-41.0, 96 40.3-40.6, 100 42.4-43.3, 104 43.3-43.9 us)
#endif
#define WAVE_KERNEL_SMALL(m) hpk_decode_wave<m, kWaveWin, kWaveImg, HPK_WAVE_SMALL_CHUNK, 2, HPK_WAVE_RANK>
#define DEC_KERNEL(m) hpk_decode12<m, kWaves, kW, kO, kQ, kRefillN>

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

namespace {
// The compacted mode's bound layout: the exclusive sum over the n + 1 elements "the 4-rounded decoded
// bound of literal i" (0 for i = n; sums mod 2^32), in two passes over in_off: per 4,096-element tile the
// sum of its bounds, one workgroup scanning the tile sums, then every tile scanned again with its base
// (reads 2 x 4 B and writes 4 B per literal; hipcub's scan over a transform iterator took 151 us per
// 32M literals, round 5).
constexpr uint32_t kScanT = 256, kScanK = 16, kScanTile = kScanT * kScanK;

__device__ __forceinline__ uint32_t bound_of(uint32_t a, uint32_t b) {
    const uint64_t nb = (uint64_t)(b - a);  // (decreasing offsets: the decode kernel reports them)
    const uint64_t bd = ((nb * 8u) / 5u + 3u) & ~(uint64_t)3u;
    return bd > 0x7FFFFFFFu ? 0x7FFFFFFFu : (uint32_t)bd;
}

// the tile's offsets into LDS (striped, coalesced), element j's bound = s[j + 1] - s[j] (0 past n)
__device__ __forceinline__ void scan_load(const uint32_t* __restrict__ off, uint32_t n, uint32_t base, uint32_t* s) {
    const uint32_t t = threadIdx.x;
#pragma unroll
    for (uint32_t k = 0; k < kScanK; ++k) {
        const uint32_t j = base + t + kScanT * k;
        s[t + kScanT * k] = j <= n ? off[j] : 0u;
    }
    if (t == 0) s[kScanTile] = base + kScanTile <= n ? off[base + kScanTile] : 0u;
    __syncthreads();
}

// exclusive block scan of one value per thread (256 threads), total to *tot
__device__ __forceinline__ uint32_t block_exscan(uint32_t v, uint32_t* s_w, uint32_t* tot) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, d);
        if (lane >= d) x += y;
    }
    if (lane == 63u) s_w[w] = x;
    __syncthreads();
    uint32_t pre = 0, all = 0;
#pragma unroll
    for (uint32_t q = 0; q < kScanT / 64u; ++q) {
        pre += q < w ? s_w[q] : 0u;
        all += s_w[q];
    }
    *tot = all;
    return pre + x - v;
}

__global__ __launch_bounds__(kScanT) void bound_tile_sums(const uint32_t* __restrict__ off, uint32_t n,
                                                          uint32_t* __restrict__ sums) {
    __shared__ uint32_t s[kScanTile + 1];
    __shared__ uint32_t s_w[kScanT / 64];
    const uint32_t base = blockIdx.x * kScanTile, t = threadIdx.x;
    scan_load(off, n, base, s);
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanK; ++k) {
        const uint32_t l = t * kScanK + k;
        acc += base + l < n ? bound_of(s[l], s[l + 1]) : 0u;
    }
    uint32_t tot;
    (void)block_exscan(acc, s_w, &tot);
    if (t == 0) sums[blockIdx.x] = tot;
}

// one workgroup: the tile sums' exclusive scan, in place
__global__ __launch_bounds__(kScanT) void bound_sums_scan(uint32_t* __restrict__ sums, uint32_t nt) {
    __shared__ uint32_t s_w[kScanT / 64];
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nt; b0 += kScanT * kScanK) {
        const uint32_t t = threadIdx.x;
        uint32_t v[kScanK], acc = 0;
#pragma unroll
        for (uint32_t k = 0; k < kScanK; ++k) {
            const uint32_t j = b0 + t * kScanK + k;
            v[k] = j < nt ? sums[j] : 0u;
            acc += v[k];
        }
        uint32_t tot;
        uint32_t x = carry + block_exscan(acc, s_w, &tot);
#pragma unroll
        for (uint32_t k = 0; k < kScanK; ++k) {
            const uint32_t j = b0 + t * kScanK + k;
            if (j < nt) sums[j] = x;
            x += v[k];
        }
        carry += tot;
        __syncthreads();  // (s_w reused)
    }
}

__global__ __launch_bounds__(kScanT) void bound_tile_scan(const uint32_t* __restrict__ off, uint32_t n,
                                                          const uint32_t* __restrict__ sums, uint32_t* __restrict__ out) {
    __shared__ uint32_t s[kScanTile + 1];
    __shared__ uint32_t s_w[kScanT / 64];
    const uint32_t base = blockIdx.x * kScanTile, t = threadIdx.x;
    scan_load(off, n, base, s);
    uint32_t v[kScanK], acc = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanK; ++k) {
        const uint32_t l = t * kScanK + k;
        v[k] = base + l < n ? bound_of(s[l], s[l + 1]) : 0u;
        acc += v[k];
    }
    uint32_t tot;
    uint32_t x = sums[blockIdx.x] + block_exscan(acc, s_w, &tot);
    __syncthreads();  // (every thread's bounds are read: the tile's offsets give way to its results)
#pragma unroll
    for (uint32_t k = 0; k < kScanK; ++k) {
        s[t * kScanK + k] = x;
        x += v[k];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kScanK; ++k) {
        const uint32_t j = base + t + kScanT * k;
        if (j <= n) out[j] = s[t + kScanT * k];
    }
}
}  // namespace

int hpk_bound_scan(hpk_ctx* c, const uint32_t* in_off, uint32_t n, uint32_t* out, void* tmp, size_t* tmp_bytes) {
    const uint32_t nt = (uint32_t)(((uint64_t)n + 1u + kScanTile - 1u) / kScanTile);  // tiles over n + 1 elements
    if (!out) {
        *tmp_bytes = (size_t)nt * 4u;
        return HPK_E_OK;
    }
    if (*tmp_bytes < (size_t)nt * 4u) return HPK_E_INVAL;
    uint32_t* sums = static_cast<uint32_t*>(tmp);
    hipLaunchKernelGGL(bound_tile_sums, dim3(nt), dim3(kScanT), 0, c->stream, in_off, n, sums);
    hipLaunchKernelGGL(bound_sums_scan, dim3(1), dim3(kScanT), 0, c->stream, sums, nt);
    hipLaunchKernelGGL(bound_tile_scan, dim3(nt), dim3(kScanT), 0, c->stream, in_off, n, (const uint32_t*)sums, out);
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}

// (tests only) the bound layout of device offsets into device memory, synchronously
extern "C" int hpk_test_bound_scan(hpk_ctx* c, const uint32_t* in_off, uint32_t n, uint32_t* out) {
    size_t tmp = 0;
    int rc = hpk_bound_scan(c, in_off, n, nullptr, nullptr, &tmp);
    if (rc) return rc;
    void* t = nullptr;
    HIP_TRY(hipMalloc(&t, tmp ? tmp : 4));
    rc = hpk_bound_scan(c, in_off, n, out, t, &tmp);
    const hipError_t e = hipStreamSynchronize(c->stream);
    (void)hipFree(t);
    return rc ? rc : e == hipSuccess ? HPK_E_OK : HPK_E_DEVICE;
}

static void decode_args(hpk_ctx* c, const hpk_batch& b, DecodeArgs& a) {
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
    a.lut3 = c->d_lut3;
    a.dbg = nullptr;
    a.in_cap = b.in_cap;
    a.out_cap = b.out_cap;
    a.err = c->d_err;
    a.lit_out = b.out_off;
    a.co_off = nullptr;
    a.cursor = nullptr;
}

// one workgroup per CU; fewer when the batch is small (>= ~64 literals or ~32 KiB of input per
// workgroup: a batch of a few huge literals gets one workgroup each, hpk_huge.h)
static uint32_t decode_blocks(hpk_ctx* c, const hpk_batch& b) {
    uint64_t blocks = ((uint64_t)b.n + 63) / 64;
    if (blocks < ((uint64_t)b.in_cap + 32767) / 32768) blocks = ((uint64_t)b.in_cap + 32767) / 32768;
    if (blocks > (uint64_t)b.n) blocks = (uint64_t)b.n;
    // (the small-call mode's persistent workgroups hold sm_wgs CUs: a one-per-CU grid leaves them out, or its
    // last workgroups would wait for a CU the whole time)
    const uint64_t cus = (uint64_t)c->num_cu - (c->sm_launched && c->sm_max ? (uint64_t)c->sm_wgs : 0u);
    if (blocks > cus) blocks = cus;
    if (blocks < 1) blocks = 1;
    return (uint32_t)blocks;
}

// ---- the small-call mode (hpk_persist.h) ----
constexpr int kPersistThreads = 256;

static int persist_launch(hpk_ctx* c, uint32_t base) {
    auto* h = static_cast<PersistCtl*>(c->h_sm);
    if (c->sm_launched) HIP_TRY(hipStreamSynchronize(c->sm_stream));  // (the previous kernel has exited)
    __atomic_store_n(&h->stop, 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&h->done, base, __ATOMIC_RELAXED);
    __atomic_store_n(&h->declined, 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&h->alive, 1u, __ATOMIC_RELEASE);
    const uint32_t init[4] = {0u, base, 0u, 0u};
    HIP_TRY(hipMemcpyAsync(c->d_sm_dev, init, sizeof init, hipMemcpyHostToDevice, c->sm_stream));
    PersistArgs a{static_cast<PersistCtl*>(c->d_sm), c->d_sm_dev, c->d_lut3, c->d_lo, base, c->sm_idle_ms * 100000u};
    hipLaunchKernelGGL(hpk_persist<kPersistThreads>, dim3((uint32_t)c->sm_wgs), dim3(kPersistThreads), 0, c->sm_stream, a);
    HIP_TRY(hipGetLastError());
    c->sm_launched = true;
    return HPK_E_OK;
}

int hpk_persist_start(hpk_ctx* c) { return persist_launch(c, c->sm_req); }

extern "C" uint64_t hpk_test_small_calls(const hpk_ctx* c) { return c ? c->sm_calls : 0u; }

extern "C" int hpk_test_small_stamps(const hpk_ctx* c, uint32_t* out6) {  // (10 values)
    if (!c || !c->h_sm || !out6) return HPK_E_INVAL;
    const auto* h = static_cast<const PersistCtl*>(c->h_sm);
    for (int k = 0; k < 6; ++k) out6[k] = __atomic_load_n(&h->ts[k], __ATOMIC_ACQUIRE);
    for (int k = 0; k < 4; ++k) out6[6 + k] = __atomic_load_n(&h->tl[k], __ATOMIC_ACQUIRE);
    return HPK_E_OK;
}

int hpk_persist_stop(hpk_ctx* c) {
    if (!c->sm_launched) return HPK_E_OK;
    auto* h = static_cast<PersistCtl*>(c->h_sm);
    __atomic_store_n(&h->stop, 1u, __ATOMIC_RELEASE);
    HIP_TRY(hipStreamSynchronize(c->sm_stream));
    c->sm_launched = false;
    return HPK_E_OK;
}

int hpk_persist_call(hpk_ctx* c, const hpk_batch& b, bool* handled) {
    *handled = false;
    if (!c->sm_max || b.n > c->sm_max || b.n == 0) return HPK_E_OK;
    // the kernel does not follow the caller's stream order: the work queued there before this call (a
    // synchronous call waits for it anyway) is finished first
    if (hipStreamQuery(c->stream) != hipSuccess) HIP_TRY(hipStreamSynchronize(c->stream));
    auto* h = static_cast<PersistCtl*>(c->h_sm);
    if (!c->sm_launched || __atomic_load_n(&h->alive, __ATOMIC_ACQUIRE) == 0u)
        if (int rc = persist_launch(c, c->sm_req)) return rc;
    const uintptr_t ip = (uintptr_t)b.in_blob, op = (uintptr_t)b.out_blob;
    h->in_base = (const uint8_t*)(ip & ~(uintptr_t)15);
    h->out_base = (uint8_t*)(op & ~(uintptr_t)15);
    h->in_off = b.in_off;
    h->out_off = b.out_off;
    h->out_len = b.out_len;
    h->status = b.status;
    h->n = b.n;
    h->in_mis = (uint32_t)(ip & 15);
    h->out_mis = (uint32_t)(op & 15);
    h->in_cap = b.in_cap;
    h->out_cap = b.out_cap;
    const uint32_t k = ++c->sm_req;
    __atomic_store_n(&h->req, k, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spins = 0; __atomic_load_n(&h->done, __ATOMIC_ACQUIRE) != k; ++spins) {
        if (__atomic_load_n(&h->alive, __ATOMIC_ACQUIRE) == 0u) {  // it went idle just before the request
            if (int rc = persist_launch(c, k - 1u)) return rc;
        }
        __builtin_ia32_pause();
        if ((spins & 4095u) == 4095u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
            return hpk_set_err_msg("small-call mode: the persistent kernel did not answer", HPK_E_DEVICE);
    }
    *handled = __atomic_load_n(&h->declined, __ATOMIC_ACQUIRE) == 0u;  // (declined: bad offsets, the launch path's)
    c->sm_calls += *handled ? 1u : 0u;
    return HPK_E_OK;
}

// The compacted form: the wave-fill kernel's (each workgroup packs into its range's bound span, no device
// cursor: *wave = 1, out_off[n] is then the bound layout's end) for the batches the region form runs it
// on, else the workgroup-fill kernel's (fills packed from the device cursor, *wave = 0)
bool hpk_compact_wave(const hpk_ctx* c, uint32_t n) {
    return c->decode_kernel == HPK_DECODE_WAVE || (c->decode_kernel == HPK_DECODE_AUTO && n >= HPK_WAVE_MIN);
}

int hpk_launch_decode_compact(hpk_ctx* c, const hpk_batch& b, uint32_t* co_off, uint32_t* long_list, uint32_t* cursor,
                              bool wave) {
    DecodeArgs a;
    decode_args(c, b, a);
    a.lit_out = co_off;
    a.co_off = co_off;
    a.cursor = cursor;
    a.long_list = long_list;
    a.long_min = HPK_LONG_MIN;
    a.long_big = HPK_LONG_BIG;
    if (wave) {
        a.cursor = nullptr;  // (the huge phase takes a listed literal's region from co_off)
        hipLaunchKernelGGL((hpk_decode_wave<0, kWaveWin, kWaveImg, HPK_WAVE_CHUNK, HPK_WAVE_GUIDED, HPK_WAVE_RANK, true>),
                           dim3(decode_blocks(c, b)), dim3(Geo::kBlock), 0, c->stream, a);
    } else {
        hipLaunchKernelGGL((hpk_decode12<0, kWaves, kW, kO, kQ, kRefillN, true>), dim3(decode_blocks(c, b)),
                           dim3(Geo::kBlock), 0, c->stream, a);
    }
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}

int hpk_launch_decode(hpk_ctx* c, const hpk_batch& b) {
    DecodeArgs a;
    decode_args(c, b, a);
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
    const uint32_t blocks = decode_blocks(c, b);
    const dim3 grid(blocks), block(Geo::kBlock);
    bool wave = c->decode_kernel == HPK_DECODE_WAVE || (c->decode_kernel == HPK_DECODE_AUTO && b.n >= HPK_WAVE_MIN);
#ifdef HPK_DIAG
    if (const char* wk = getenv("HPK_DECODE_KERNEL")) wave = wk[0] == 'w';  // "wave" / "fill" (A/B runs)
    if (g_debug_mode < 0) {
        const char* dm = getenv("HPK_DEBUG_MODE");
        g_debug_mode = dm ? atoi(dm) : 0;
    }
    // (A/B runs) HPK_WAVE_VARIANT=v: hand-out v / 3 (0 static, 1 guided), order v % 3 (kRank)
    static const int wave_var = getenv("HPK_WAVE_VARIANT") ? atoi(getenv("HPK_WAVE_VARIANT")) : -1;
    if (wave && wave_var >= 0 && g_debug_mode == 0) {
        switch (wave_var) {
            case 0: hipLaunchKernelGGL((hpk_decode_wave<0, kWaveWin, kWaveImg, 224u, false, 0>), grid, block, 0, c->stream, a); break;
            case 1: hipLaunchKernelGGL((hpk_decode_wave<0, kWaveWin, kWaveImg, 224u, false, 1>), grid, block, 0, c->stream, a); break;
            case 2: hipLaunchKernelGGL((hpk_decode_wave<0, kWaveWin, kWaveImg, 224u, false, 2>), grid, block, 0, c->stream, a); break;
            case 3: hipLaunchKernelGGL((hpk_decode_wave<0, kWaveWin, kWaveImg, 224u, true, 0>), grid, block, 0, c->stream, a); break;
            case 4: hipLaunchKernelGGL((hpk_decode_wave<0, kWaveWin, kWaveImg, 224u, true, 1>), grid, block, 0, c->stream, a); break;
            case 5: hipLaunchKernelGGL((hpk_decode_wave<0, kWaveWin, kWaveImg, 224u, true, 2>), grid, block, 0, c->stream, a); break;
            // (the least chunk of the guided hand-out, 128-1024 literals: within the noise, r3l; the 3072 /
            // 5888 split won over 3328-3840 B windows, whose fourth prefetch round spills, r3i; dword
            // output by LDS masked OR, code in git history: 1223-1229 us, r3o)
            default: hipLaunchKernelGGL((WAVE_KERNEL(0)), grid, block, 0, c->stream, a); break;
        }
        HIP_TRY(hipGetLastError());
        return hpk_long_list_used(c, lslot);
    }
    if (wave) {
        // (every mode runs the kernel the product would: fixed chunks below HPK_WAVE_GUIDED_MIN literals)
#define WAVE_LAUNCH(m)                                                                    \
    do {                                                                                  \
        if (b.n < HPK_WAVE_GUIDED_MIN)                                                    \
            hipLaunchKernelGGL(WAVE_KERNEL_SMALL(m), grid, block, 0, c->stream, a);       \
        else                                                                              \
            hipLaunchKernelGGL(WAVE_KERNEL(m), grid, block, 0, c->stream, a);             \
    } while (0)
        if (g_debug_mode == 1) {
            WAVE_LAUNCH(1);
        } else if (g_debug_mode == 3) {
            const size_t need = (size_t)blocks * kWaves * 16;
            if (need > g_dbg_n) {
                (void)hipFree(g_dbg);
                HIP_TRY(hipMalloc(&g_dbg, need * 8));
                g_dbg_n = need;
            }
            a.dbg = g_dbg;
            WAVE_LAUNCH(3);
        } else if (g_debug_mode == 2)
            WAVE_LAUNCH(2);
        else if (g_debug_mode == 6)
            WAVE_LAUNCH(6);
        else if (g_debug_mode == 7)
            WAVE_LAUNCH(7);
        else if (g_debug_mode == 8)  // LDS conflict attribution (lit12_body's kDup): table reads twice
            WAVE_LAUNCH(8);
        else if (g_debug_mode == 9)  // the window read twice
            WAVE_LAUNCH(9);
        else if (g_debug_mode == 10)  // the byte stores twice
            WAVE_LAUNCH(10);
        else if (g_debug_mode == 5) {  // per-wave counters of the long-literal phase (HPK_LONG_WAVES waves)
            const size_t need = (size_t)blocks * HPK_LONG_WAVES * 16;
            if (need > g_dbg_n) {
                (void)hipFree(g_dbg);
                HIP_TRY(hipMalloc(&g_dbg, need * 8));
                g_dbg_n = need;
            }
            HIP_TRY(hipMemsetAsync(g_dbg, 0, need * 8, c->stream));
            a.dbg = g_dbg;
            if (b.n < HPK_WAVE_GUIDED_MIN)
                hipLaunchKernelGGL(WAVE_KERNEL_SMALL(5), grid, block, 0, c->stream, a);
            else
                WAVE_LAUNCH(5);
        } else if (b.n < HPK_WAVE_GUIDED_MIN)  // (the product's choice)
            hipLaunchKernelGGL(WAVE_KERNEL_SMALL(0), grid, block, 0, c->stream, a);
        else
            WAVE_LAUNCH(0);
        HIP_TRY(hipGetLastError());
        return hpk_long_list_used(c, lslot);
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
    if (wave && b.n < HPK_WAVE_GUIDED_MIN)
        hipLaunchKernelGGL(WAVE_KERNEL_SMALL(0), grid, block, 0, c->stream, a);
    else if (wave)
        hipLaunchKernelGGL(WAVE_KERNEL(0), grid, block, 0, c->stream, a);
    else
        hipLaunchKernelGGL(DEC_KERNEL(0), grid, block, 0, c->stream, a);
#endif
    HIP_TRY(hipGetLastError());
    return hpk_long_list_used(c, lslot);
}
