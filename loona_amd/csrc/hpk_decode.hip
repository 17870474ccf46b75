// hpk_decode.hip — gfx950 batched Huffman literal decode (the hot path).
//
// Replaces, for a batch of literals at once, the Huffman branch of decode_string
// (crates/loona-hpack/src/decoder.rs:143-157) i.e. HuffmanDecoder::decode
// (crates/loona-hpack/src/huffman.rs:95-161), with identical results per literal: decoded bytes,
// and status Ok / PaddingTooLarge / InvalidPadding / EOSInString with the reference's precedence.
//
// Work decomposition:
//   * one 1024-thread workgroup per CU (16 waves); the decode tables (hpk_code.h: 16 KiB
//     two-symbol LUT + 1.9 KiB leading-ones table) are staged into LDS once per workgroup;
//   * every wave owns a contiguous range of literals (≈ n / (16·CUs)) and stages it into its
//     private LDS window in one go: offsets with coalesced dword loads, literal bytes with 16-byte
//     loads, every load issued before the first wait; ranges larger than the window are staged
//     in several fills;
//   * per window the wave builds a queue of 8-byte entries {window offset, length, output
//     position}; lanes decode one literal each out of LDS and pull the next queue entry every
//     kRefill steps (ballot + mbcnt), so long literals do not hold up the other 63 lanes;
//   * a step decodes one or two symbols with one LUT lookup (codes > 12 bits take one extra
//     lookup in the leading-ones table). The bit window is a 64-bit register refilled a dword at
//     a time from a dword read one step ahead. Bits past the literal's end are NOT masked: a code
//     that runs past the end is, by prefix-freeness, longer than what is left whatever follows,
//     so the walk stops exactly where huffman.rs's bit iterator stops matching; only the final
//     padding check (huffman.rs:128-160) looks at the residual bits, masked;
//   * output bytes are packed in a register and stored as aligned dwords. A literal whose output
//     region is not dword-aligned or is smaller than hpk_decoded_bound (caller-chosen offsets)
//     is decoded after the queue drains with byte stores and per-byte capacity checks.
// A literal too large for the LDS window (> ~7 KiB encoded) is decoded by one lane straight from
// global memory with the same step code.
#include <stdlib.h>

#include "hpk_device.h"

namespace {

constexpr int kBlock = 1024;
constexpr int kWaves = kBlock / 64;
constexpr int kStage = 7040;   // bytes of literal data per wave window (multiple of 16)
constexpr int kMaxLits = 256;  // literals per window fill
constexpr int kRefill = 4;     // decode steps between queue refills
constexpr int kMetaRounds = (kMaxLits + 1 + 63) / 64;
constexpr int kStageRounds = (kStage / 16 + 63) / 64;
constexpr int kLutBytes = HPK_LUT_SIZE * 4;
constexpr int kLoBytes = HPK_LO_SIZE * 2;
constexpr int kTabBytes = ((kLutBytes + kLoBytes + 15) / 16) * 16;
constexpr int kQueueBytes = kMaxLits * 8;  // uint2 per literal
constexpr int kWaveBytes = kStage + kQueueBytes;
constexpr int kLdsBytes = kTabBytes + kWaves * kWaveBytes;
constexpr uint32_t kBytePath = 0x80000000u;  // queue flag: decode with byte stores
static_assert(kLdsBytes <= 163840, "LDS budget (160 KiB per CU on gfx950)");
static_assert(kStage % 16 == 0 && kStage < 32768, "window offsets/lengths pack in 15 bits");
static_assert(kMaxLits % 64 == 0, "queue filled in whole rounds of 64");

struct DecodeArgs {
    const uint8_t* in_base;  // in_blob rounded down to 16 bytes
    uint32_t in_mis;         // in_blob - in_base (0..15)
    const uint32_t* in_off;
    uint32_t n;
    uint8_t* out_base;  // out_blob rounded down to 4 bytes
    uint32_t out_mis;   // out_blob - out_base (0..3)
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
    const uint32_t* lut;
    const uint16_t* lo;
    unsigned long long* dbg;  // diagnostic builds only: per-wave timestamps
};

// Per-lane state of the literal being decoded.
struct Lit {
    uint64_t win;   // next bits, MSB-aligned (bits past the literal: whatever follows)
    uint32_t nb;    // loaded bits in win
    uint32_t nxt;   // next source dword (raw), merged at the next refill
    uint32_t pf;    // the dword after it (raw, read one step ahead)
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
};

enum StoreMode { kDword = 0, kNoStore = 1, kBytes = 2, kChecked = 3 };

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

// One decode step of a live lane: one LUT lookup, one or two symbols out.
template <int kStore, class Src>
__device__ __forceinline__ void lit_step(Lit& L, const Src& src, const uint32_t* __restrict__ lut,
                                         const uint16_t* __restrict__ lo, uint8_t* __restrict__ out8) {
    // refill the window from the prefetched dword, read the next one for a later step
    const bool need = L.nb <= 32u;
    const uint64_t add = (uint64_t)hpk_bswap32(L.nxt) << ((32u - L.nb) & 63u);
    L.win |= need ? add : 0ull;
    L.nb += need ? 32u : 0u;
    L.nxt = need ? L.pf : L.nxt;
    L.q += need ? 1u : 0u;
    L.pf = src(L.q);

    const uint32_t w = (uint32_t)(L.win >> 32);
    const uint32_t ent = lut[w >> (32 - HPK_LUT_BITS)];
    uint32_t len = (ent >> 16) & 31u;
    uint32_t syms = ent & 0xFFFFu;  // one-symbol entries carry 0 in the second byte
    bool eos = false;
    if (ent < (1u << 26)) {  // code longer than the LUT index: one leading-ones table lookup
        const uint32_t kk = __clz(~w);
        const uint32_t e = lo[min(kk, (uint32_t)HPK_LO_RUNS - 1) * 32 + ((w << ((kk + 1) & 31)) >> 27)];
        eos = kk >= HPK_LO_RUNS || (e & 0x1FFu) == HPK_EOS;
        syms = e & 0xFFu;
        len = eos ? 30u : (e >> 9);
    }
    const uint32_t total = (ent >> 21) & 31u;
    const bool stop = len > L.rem || eos;  // end of literal (only padding left) or EOS
    // second symbol only if its code ends inside the literal; otherwise the literal ends after
    // the first (the next step decodes that same code and stops), and the extra byte left in
    // acc lies past out_len, inside the capacity
    const bool two = ent >= (2u << 26) && total <= L.rem;
    const uint32_t use = two ? total : len;
    const uint32_t k = two ? 2u : 1u;
    if (eos && len <= L.rem) L.st = HPK_EOS_IN_STRING;  // huffman.rs:112-116
    if (!stop) {
        if (kStore == kBytes) {
            for (uint32_t j = 0; j < k; ++j) {
                if (L.cnt + j >= L.ocap) {
                    L.st = HPK_OUTPUT_OVERFLOW;
                    L.cnt += j;
                    L.live = false;
                    return;
                }
                out8[L.od + j] = (uint8_t)(syms >> (8 * j));
            }
            L.od += k;
        } else {
            L.acc |= (uint64_t)syms << (8u * L.accn);
            L.accn += k;
            if (L.accn >= 4u) {
                if (kStore == kDword)
                    reinterpret_cast<uint32_t*>(out8)[L.od] = (uint32_t)L.acc;
                else if (kStore == kChecked) {
                    if (L.od < L.oend) reinterpret_cast<uint32_t*>(out8)[L.od] = (uint32_t)L.acc;
                    else chk_report(1, L.od, L.oend, L.cnt);
                } else
                    asm volatile("" ::"v"((uint32_t)L.acc));
                L.od += 1;
                L.acc >>= 32;
                L.accn -= 4u;
            }
        }
        L.cnt += k;
        L.win <<= use;
        L.nb -= use;
        L.rem -= use;
    }
    L.live = !stop && L.rem != 0u;
}

template <int kStore>
__device__ __forceinline__ void lit_finish(Lit& L, const DecodeArgs& a, uint32_t i) {
    // the last, partial dword lies inside this literal's capacity (aligned, >= decoded bound)
    if (kStore == kDword && L.accn) reinterpret_cast<uint32_t*>(a.out_base)[L.od] = (uint32_t)L.acc;
    if (kStore == kChecked && L.accn) {
        if (L.od < L.oend) reinterpret_cast<uint32_t*>(a.out_base)[L.od] = (uint32_t)L.acc;
        else chk_report(2, L.od, L.oend, L.cnt);
    }
    if (kStore == kChecked && i >= a.n) {
        chk_report(3, i, a.n, 0);
        return;
    }
    uint32_t st = L.st;
    if (st == HPK_OK && L.rem > 0) {  // huffman.rs:128-160: at most 7 bits, all ones (EOS MSBs)
        if (L.rem > 7) {
            st = HPK_PADDING_TOO_LARGE;
        } else {
            const uint32_t w = (uint32_t)(L.win >> 32) | (0xFFFFFFFFu >> L.rem);
            if (w != 0xFFFFFFFFu) st = HPK_INVALID_PADDING;
        }
    }
    a.out_len[i] = L.cnt;
    a.status[i] = (uint8_t)st;
}

// Literal i decoded whole with byte stores and capacity checks.
template <class Src>
__device__ __forceinline__ void lit_bytes(const Src& src, const uint32_t* lut, const uint16_t* lo,
                                          const DecodeArgs& a, uint32_t i, uint32_t sb, uint32_t nbytes) {
    Lit L;
    lit_begin(L, src, sb, nbytes);
    L.od = a.out_off[i] + a.out_mis;
    L.ocap = a.out_off[i + 1] - a.out_off[i];
    while (L.live) lit_step<kBytes>(L, src, lut, lo, a.out_base);
    lit_finish<kBytes>(L, a, i);
}

struct LdsSrc {
    const uint32_t* p;
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return p[i]; }
};
struct GlobalSrc {
    const uint32_t* p;
    uint32_t last;  // last dword index holding a byte of the batch: never read past it
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const { return p[min(i, last)]; }
};

// kMode: 0 = product kernel; diagnostic variants (HPK_DEBUG_MODE, never the default):
//   1 = stage only (no decode), 2 = decode without output stores, 3 = product + per-wave stamps,
//   4 = every global store bounds-checked (first violation recorded in g_chk, store skipped)
template <int kMode>
__global__ __launch_bounds__(kBlock) void hpk_decode_kernel(DecodeArgs a) {
    unsigned long long t_start = 0, t_staged = 0;
    if (kMode == 3) t_start = __builtin_amdgcn_s_memtime();
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* s_lut = reinterpret_cast<uint32_t*>(smem);
    uint16_t* s_lo = reinterpret_cast<uint16_t*>(smem + kLutBytes);
    for (uint32_t t = threadIdx.x; t < kLutBytes / 16; t += kBlock)
        reinterpret_cast<uint4*>(s_lut)[t] = reinterpret_cast<const uint4*>(a.lut)[t];
    for (uint32_t t = threadIdx.x; t < kLoBytes / 16; t += kBlock)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6;
    uint8_t* wbase = smem + kTabBytes + wv * kWaveBytes;
    uint2* s_q = reinterpret_cast<uint2*>(wbase + kStage);
    const LdsSrc lds{reinterpret_cast<const uint32_t*>(wbase)};

    const uint64_t W = (uint64_t)gridDim.x * kWaves;
    const uint64_t gw = (uint64_t)blockIdx.x * kWaves + wv;
    const uint32_t A = (uint32_t)((uint64_t)a.n * gw / W);
    const uint32_t B = (uint32_t)((uint64_t)a.n * (gw + 1) / W);

    uint32_t cur = A;
    while (cur < B) {
        const uint32_t cntl = min((uint32_t)kMaxLits, B - cur);
        const uint32_t base16 = (a.in_off[cur] + a.in_mis) & ~15u;
        const uint32_t limit = base16 + kStage;
        // all offset loads first (indices clamped, so no branches), then use. Lane l holds the
        // offsets of literal l + 64 r; successors come from lane l+1 or the next round.
        uint32_t io[kMetaRounds], oo[kMetaRounds];
#pragma unroll
        for (int r = 0; r < kMetaRounds; ++r) {
            const uint32_t t = min(lane + 64u * r, cntl);
            io[r] = a.in_off[cur + t] + a.in_mis;
            oo[r] = a.out_off[cur + t] + a.out_mis;
        }
        uint32_t k = 0;
#pragma unroll
        for (int r = 0; r < kMaxLits / 64; ++r) {
            // successors: lane l+1 of this round; for lane 63, lane 0 of the next round, read with
            // v_readlane (a ds_bpermute under lane 63's exec mask would read an inactive lane as 0)
            const uint32_t nio = __shfl_down(io[r], 1);
            const uint32_t noo = __shfl_down(oo[r], 1);
            const uint32_t io1 = lane == 63 ? (uint32_t)__builtin_amdgcn_readlane((int)io[r + 1], 0) : nio;
            const uint32_t oo1 = lane == 63 ? (uint32_t)__builtin_amdgcn_readlane((int)oo[r + 1], 0) : noo;
            const uint32_t t = lane + 64u * r;
            const bool fits = t < cntl && io1 <= limit;
            if (fits) {
                const uint32_t nbytes = io1 - io[r];
                const uint32_t ocap = oo1 - oo[r];
                // dword path needs an aligned region holding hpk_decoded_bound(nbytes) bytes
                const bool dw = ((oo[r] | ocap) & 3u) == 0 && ocap >= (nbytes * 8u) / 5u;
                s_q[t] = make_uint2((io[r] - base16) | (nbytes << 16) | (dw ? 0u : kBytePath), dw ? (oo[r] >> 2) : 0u);
            }
            k += (uint32_t)__popcll(__ballot(fits));
        }
        if (k == 0) {  // literal `cur` alone exceeds the window: decode from global on one lane
            if (lane == 0) {
                const GlobalSrc g{reinterpret_cast<const uint32_t*>(a.in_base), (a.in_off[a.n] + a.in_mis - 1) >> 2};
                const uint32_t sb = a.in_off[cur] + a.in_mis;
                lit_bytes(g, s_lut, s_lo, a, cur, sb, a.in_off[cur + 1] + a.in_mis - sb);
            }
            cur += 1;
            continue;
        }
        // stage the window's bytes with 16-byte loads: all loads issued, then all LDS writes.
        // Chunks are 16-byte aligned and each holds a byte of the batch, so no page is crossed.
        const uint2 last = s_q[k - 1];
        const uint32_t endb = (last.x & 0xFFFFu) + ((last.x >> 16) & 0x7FFFu);
        uint32_t nch = (endb + 15) >> 4;
        if (kMode == 4 && (nch > kStage / 16 || base16 + endb > a.in_off[a.n] + a.in_mis + 16)) {
            chk_report(5, nch, endb, base16);
            nch = 0;
        }
        if (kMode == 4 && k > cntl) chk_report(6, k, cntl, cur);
        if (nch) {
            const uint4* g16 = reinterpret_cast<const uint4*>(a.in_base + base16);
            uint4* l16 = reinterpret_cast<uint4*>(wbase);
            uint4 chunk[kStageRounds];
#pragma unroll
            for (int r = 0; r < kStageRounds; ++r) chunk[r] = g16[min(lane + 64u * r, nch - 1)];
#pragma unroll
            for (int r = 0; r < kStageRounds; ++r)
                if (lane + 64u * r < nch) l16[lane + 64u * r] = chunk[r];
        }

        if (kMode == 3 && t_staged == 0) t_staged = __builtin_amdgcn_s_memtime();
        if (kMode == 1) {  // diagnostic: keep the staged bytes live, write lengths only
            for (uint32_t t = lane; t < k; t += 64) {
                const uint2 e = s_q[t];
                a.out_len[cur + t] = ((e.x >> 16) & 0x7FFFu) + reinterpret_cast<const uint8_t*>(wbase)[e.x & 0xFFFFu];
                a.status[cur + t] = 0;
            }
            cur += k;
            continue;
        }

        // decode [0, k) with the lane queue
        constexpr int kStore = kMode == 2 ? kNoStore : (kMode == 4 ? kChecked : kDword);
        Lit L;
        L.live = false;
        uint32_t t = lane;
        bool act = false;  // lane holds a dword-path literal not yet finalised
        auto begin = [&](uint32_t tt) {
            const uint2 e = s_q[tt];
            act = !(e.x & kBytePath);
            lit_begin(L, lds, e.x & 0xFFFFu, (e.x >> 16) & 0x7FFFu);
            L.od = e.y;
            L.oend = e.y + (((e.x >> 16) & 0x7FFFu) * 8u / 5u + 3u) / 4u;
            if (kMode == 4 && tt >= k) chk_report(4, tt, k, 0);
            L.live = L.live && act;
        };
        if (t < k) begin(t);
        uint32_t next = 64;
        while (__any(t < k)) {
#pragma unroll
            for (int s = 0; s < kRefill; ++s)
                if (L.live) lit_step<kStore>(L, lds, s_lut, s_lo, a.out_base);
            const bool fin = t < k && !L.live;
            if (__any(fin)) {
                if (fin && act) lit_finish<kStore>(L, a, cur + t);
                const bool free_lane = fin || t >= k;
                const uint64_t fm = __ballot(free_lane);
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(fm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)fm, 0u));
                if (free_lane) {
                    t = next + rank;
                    act = false;
                    if (t < k) begin(t);
                }
                next += (uint32_t)__popcll(fm);
            }
        }
        // literals whose output region is unaligned / below the decoded bound
        for (uint32_t tt = lane; tt < k; tt += 64) {
            const uint2 e = s_q[tt];
            if (e.x & kBytePath) lit_bytes(lds, s_lut, s_lo, a, cur + tt, e.x & 0xFFFFu, (e.x >> 16) & 0x7FFFu);
        }
        cur += k;
    }
    if (kMode == 3 && lane == 0) {
        const unsigned long long t_end = __builtin_amdgcn_s_memtime();
        const uint64_t gwi = (uint64_t)blockIdx.x * kWaves + wv;
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        a.dbg[gwi * 4 + 0] = t_start;
        a.dbg[gwi * 4 + 1] = t_staged;
        a.dbg[gwi * 4 + 2] = t_end;
        a.dbg[gwi * 4 + 3] = ((unsigned long long)xcc << 32) | (B - A);
    }
}

}  // namespace

static int g_debug_mode = -1;

int hpk_decode_setup() {
    static int rc = -1;
    static bool done = false;
    if (!done) {
        const char* dm = getenv("HPK_DEBUG_MODE");
        g_debug_mode = dm ? atoi(dm) : 0;
        const void* fns[5] = {reinterpret_cast<const void*>(&hpk_decode_kernel<0>),
                              reinterpret_cast<const void*>(&hpk_decode_kernel<1>),
                              reinterpret_cast<const void*>(&hpk_decode_kernel<2>),
                              reinterpret_cast<const void*>(&hpk_decode_kernel<3>),
                              reinterpret_cast<const void*>(&hpk_decode_kernel<4>)};
        rc = HPK_E_OK;
        for (int i = 0; i < 5 && rc == HPK_E_OK; ++i) {
            hipError_t e = hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
            if (e != hipSuccess) rc = hpk_set_err("hipFuncSetAttribute(decode LDS)", e);
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
    a.out_base = (uint8_t*)(op & ~(uintptr_t)3);
    a.out_mis = (uint32_t)(op & 3);
    a.out_off = out_off;
    a.out_len = out_len;
    a.status = status;
    a.lut = c->d_lut;
    a.lo = c->d_lo;
    a.dbg = nullptr;
    // one workgroup per CU; fewer when the batch is small (>= ~32 literals per wave)
    uint64_t blocks = ((uint64_t)n + kWaves * 32 - 1) / (kWaves * 32);
    if (blocks > (uint64_t)c->num_cu) blocks = (uint64_t)c->num_cu;
    if (blocks < 1) blocks = 1;
    const dim3 grid((uint32_t)blocks), block(kBlock);
    switch (g_debug_mode) {
        case 1:
            hipLaunchKernelGGL(hpk_decode_kernel<1>, grid, block, kLdsBytes, c->stream, a);
            break;
        case 2:
            hipLaunchKernelGGL(hpk_decode_kernel<2>, grid, block, kLdsBytes, c->stream, a);
            break;
        case 3: {
            const size_t need = (size_t)blocks * kWaves * 4;
            if (need > g_dbg_n) {
                (void)hipFree(g_dbg);
                HIP_TRY(hipMalloc(&g_dbg, need * 8));
                g_dbg_n = need;
            }
            a.dbg = g_dbg;
            hipLaunchKernelGGL(hpk_decode_kernel<3>, grid, block, kLdsBytes, c->stream, a);
            break;
        }
        case 4:
            hipLaunchKernelGGL(hpk_decode_kernel<4>, grid, block, kLdsBytes, c->stream, a);
            break;
        default:
            hipLaunchKernelGGL(hpk_decode_kernel<0>, grid, block, kLdsBytes, c->stream, a);
    }
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}
