// hpk_encode.hip — gfx950 batched canonical Huffman encode (RFC 7541 §5.2; the H-bit branch
// crates/loona-hpack/src/encoder.rs:299-307 never takes — the reference has no encoder).
//
// v2 (hpk_encode2): one 1024-thread workgroup per CU owns a contiguous literal range and encodes it
// in tiles of whole literals (<= 32 KiB of input, <= 2048 literals, output span <= the LDS image):
//   * every thread owns 32 consecutive input bytes of the tile (two 16-byte loads, in registers);
//   * a segmented scan of per-byte code lengths over the 1024 threads (literal starts reset it)
//     gives each byte its bit offset inside its literal;
//   * each byte's code is OR-ed into an LDS image of the tile's output span (big-endian dwords,
//     ds_or_b32, one or two per code), clipped at the literal's capacity;
//   * one thread per literal then pads the last byte with EOS's most significant bits (ones) and
//     writes out_len / status; the image goes out with 16-byte stores (bytewise in the span's two
//     end chunks, which neighbouring tiles own).
// A literal too large for a tile is encoded by one lane straight to global memory (v1's loop).
// v1 (hpk_encode_kernel, one lane per literal) stays as the comparison build (HPK_ENCODE_V1=1).
#include <stdlib.h>

#include "hpk_device.h"
#include "hpk_split.h"

namespace {

struct EncodeArgs {
    const uint8_t* in_blob;
    const uint32_t* in_off;
    uint32_t n;
    uint8_t* out_blob;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
    const uint32_t* codes;  // [0,257): right-aligned code, [257,514): length
    // v2: 16-byte aligned bases and the blobs' misalignment (offsets are blob-relative)
    const uint8_t* in_base;
    uint32_t in_mis;
    uint8_t* out_base;
    uint32_t out_mis;
    uint32_t in_cap, out_cap;  // blob sizes (clamped to HPK_MAX_OFFSET): larger offsets are bad
    uint32_t* err;             // sticky error flag (host-mapped): set to 1 on bad offsets
    unsigned long long* prof;  // diagnostic build: cycles per kernel phase (kProf)
};

// diagnostic build: per-wave cycles spent in each phase of hpk_encode2, summed over waves

#define EPROF(i)                                                                  \
    if (kProf) {                                                                  \
        const uint64_t now_ = clock64();                                          \
        if (lane == 0) atomicAdd(&S.prof[wv][i], (unsigned long long)(now_ - tprev)); \
        tprev = now_;                                                             \
    }

// One literal, one lane, global memory: v1's loop (also the large-literal path of v2).
__device__ __forceinline__ void encode_serial(const EncodeArgs& a, const uint32_t* code, const uint8_t* len,
                                              uint32_t i) {
    const uint32_t s = a.in_off[i], e = a.in_off[i + 1];
    const uint32_t o0 = a.out_off[i], ocap = a.out_off[i + 1] - o0;
    uint8_t* out = a.out_blob + o0;
    uint64_t acc = 0;
    int nb = 0;
    uint32_t o = 0;
    uint32_t st = HPK_OK;
    for (uint32_t p = s; p < e; ++p) {
        const uint32_t b = a.in_blob[p];
        acc = (acc << len[b]) | code[b];
        nb += len[b];
        while (nb >= 8) {
            nb -= 8;
            if (o >= ocap) {
                st = HPK_OUTPUT_OVERFLOW;
                break;
            }
            out[o++] = (uint8_t)(acc >> nb);
        }
        if (st) break;
    }
    if (!st && nb) {
        if (o >= ocap)
            st = HPK_OUTPUT_OVERFLOW;
        else
            out[o++] = (uint8_t)((acc << (8 - nb)) | (0xFFu >> nb));
    }
    a.out_len[i] = o;
    a.status[i] = (uint8_t)st;
}

#define ENC_BLOCK 256

#ifdef HPK_DIAG
__global__ __launch_bounds__(ENC_BLOCK) void hpk_encode_kernel(EncodeArgs a) {
    __shared__ uint32_t s_code[256];
    __shared__ uint8_t s_len[256];
    if (threadIdx.x < 256) {
        s_code[threadIdx.x] = a.codes[threadIdx.x];
        s_len[threadIdx.x] = (uint8_t)a.codes[257 + threadIdx.x];
    }
    __syncthreads();
    for (uint32_t i = blockIdx.x * ENC_BLOCK + threadIdx.x; i < a.n; i += gridDim.x * ENC_BLOCK)
        encode_serial(a, s_code, s_len, i);
}
#endif

// ---------------------------------------------------------------------------------------------
// v2

// Geometry: kEB threads per workgroup, kEO bytes of LDS output image, kEQ literals per tile. The
// product runs two workgroups of 512 threads per CU (16 KiB input tiles, 56 KiB images), so one
// workgroup's global-memory waits overlap the other's LDS work; 1024 / 112 KiB / 2048 (one per CU)
// stays for comparison (HPK_ENCODE_CFG=1; v5 dropped the 16-bytes-per-thread geometries: the start
// map has one word per thread).

// Pass 2's phantom runs (bytes a thread holds but does not own: before the tile's first literal,
// after its last) go to kEPh dwords past the image: a run covers at most 32 bytes of 30-bit codes
// (30 dwords), started at dword (tid & 31) so the lanes of a wave do not all hit one address.
constexpr int kEPh = 64;

template <int kEB, int kEO, int kEQ, int kP = 0>
struct EncLds {
    uint32_t img[kEO / 4 + kEPh];  // the tile's output span, big-endian dwords; then the phantom dwords
    uint32_t ioff[kEQ + 3];      // input offsets of the tile's literals, relative to the tile base (+ sentinel)
    uint32_t ooff[kEQ + 2];      // output offsets, relative to the image base
    uint32_t bits[kEQ];          // encoded bits per literal (set by the thread holding its last byte)
    uint2 tab[256];              // (code, length)
    uint32_t code1[256];         // serial path: codes
    uint8_t len1[256];           // serial path: lengths
    uint32_t wf[16], wv[16], wl[16];  // per-wave scan totals
    uint32_t smap[kEB + 1];      // bit j of word h: input byte 32h + j starts a (non-empty) literal of the tile
    uint32_t slast[kEB + 1];     // 1 + the last (non-empty) literal starting in word h's bytes, 0 if none
    uint32_t live[(kEO / 16 + 31) / 32];  // image chunks holding output bytes (the rest is slack)
    uint32_t ctr[4];             // [0] literals in the tile, [1] bad offsets seen, [2] a literal of the tile
                                 // has less room than 30 bits per input byte (pass 2 takes the checked path)
    uint32_t split[2 * hpksplit::kMaxRounds];  // split_by_bytes's counters
    unsigned long long prof[kP ? kEB / 64 : 1][12];  // diagnostic build (kProf): per-wave phase cycles
};


__device__ __forceinline__ void lds_barrier_e() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// OR a code of `len` bits (right-aligned in c) into the big-endian image at bit q.
__device__ __forceinline__ void img_or(uint32_t* img, uint32_t q, uint32_t c, uint32_t len) {
    const uint32_t d = q >> 5, r = q & 31u;
    if (r + len <= 32u) {
        atomicOr(&img[d], c << (32u - r - len));
    } else {
        atomicOr(&img[d], c >> (r + len - 32u));
        atomicOr(&img[d + 1], c << (64u - r - len));
    }
}


template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_e(uint32_t x) {  // out-of-range lanes read 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, kCtrl, 0xF, 0xF, false);
}

template <int kCtrl>
__device__ __forceinline__ void seg_step(uint32_t& f, uint32_t& v, uint32_t& L) {
    const uint32_t pf = dpp_e<kCtrl>(f), pv = dpp_e<kCtrl>(v), pl = dpp_e<kCtrl>(L);
    v = f ? v : v + pv;
    f |= pf;
    L = max(L, pl);
}

// Segmented inclusive scan over the wave's 64 lanes of (f, v) under (f0, v0) . (f1, v1) = (f0 | f1,
// f1 ? v1 : v0 + v1) (f: a literal starts in the lane's bytes, v: code bits since the last start), with
// an inclusive max of L beside it: DPP row shifts within rows of 16 lanes, then the rows' totals by
// readlane (v5: it replaced 12 dependent ds_bpermute shuffles).
__device__ __forceinline__ void wave_seg_scan(uint32_t& f, uint32_t& v, uint32_t& L, uint32_t lane) {
    seg_step<0x111>(f, v, L);  // row_shr:1
    seg_step<0x112>(f, v, L);  // row_shr:2
    seg_step<0x114>(f, v, L);  // row_shr:4
    seg_step<0x118>(f, v, L);  // row_shr:8
    const uint32_t f0 = __builtin_amdgcn_readlane((int)f, 15), v0 = __builtin_amdgcn_readlane((int)v, 15);
    const uint32_t f1 = __builtin_amdgcn_readlane((int)f, 31), v1 = __builtin_amdgcn_readlane((int)v, 31);
    const uint32_t f2 = __builtin_amdgcn_readlane((int)f, 47), v2 = __builtin_amdgcn_readlane((int)v, 47);
    const uint32_t l0 = __builtin_amdgcn_readlane((int)L, 15), l1 = __builtin_amdgcn_readlane((int)L, 31);
    const uint32_t l2 = __builtin_amdgcn_readlane((int)L, 47);
    // the carry into rows 1, 2, 3: row 0, rows 0-1, rows 0-2
    const uint32_t c1f = f0, c1v = v0;
    const uint32_t c2f = f0 | f1, c2v = f1 ? v1 : v0 + v1;
    const uint32_t c3f = c2f | f2, c3v = f2 ? v2 : c2v + v2;
    const uint32_t row = lane >> 4;
    const uint32_t cf = row == 0 ? 0u : row == 1 ? c1f : row == 2 ? c2f : c3f;
    const uint32_t cv = row == 0 ? 0u : row == 1 ? c1v : row == 2 ? c2v : c3v;
    const uint32_t cl = row == 0 ? 0u : row == 1 ? l0 : row == 2 ? max(l0, l1) : max(max(l0, l1), l2);
    v = f ? v : v + cv;
    f |= cf;
    L = max(L, cl);
}

template <int kEB, int kEO, int kEQ, int kEBytes = 32, int kProf = 0>  // kEBytes: input bytes per thread per tile
// (at least 4 waves per SIMD: two 512-thread workgroups per CU fit only under 128 VGPRs)
__global__ __launch_bounds__(kEB, 4) void hpk_encode2(EncodeArgs a) {
    static_assert(kEBytes == 32, "bytes per thread: one start-map word per thread");
    constexpr int kCh = kEBytes / 16;  // 16-byte chunks per thread
    constexpr int kETile = kEB * kEBytes;  // input bytes per tile
    constexpr int kEMeta = kEQ / kEB;      // offset rounds per thread
    static_assert(sizeof(EncLds<kEB, kEO, kEQ, kProf>) <= 163840, "LDS budget (160 KiB per CU on gfx950)");
    static_assert(kEB <= 1024 && kEQ % kEB == 0, "geometry");
    __shared__ __attribute__((aligned(16))) EncLds<kEB, kEO, kEQ, kProf> S;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    uint64_t tprev = kProf ? clock64() : 0;
    if (kProf && tid < (kEB / 64) * 12) (&S.prof[0][0])[tid] = 0;
    if (tid < 256) {
        const uint32_t c = a.codes[tid], l = a.codes[257 + tid];
        S.tab[tid] = make_uint2(c, l);
        S.code1[tid] = c;
        S.len1[tid] = (uint8_t)l;
    }
    {  // the image starts clear; every tile clears what it wrote (its live chunks) after storing them
        uint4* i16 = reinterpret_cast<uint4*>(S.img);
        for (uint32_t c = tid; c < (uint32_t)kEO / 16; c += kEB) i16[c] = make_uint4(0, 0, 0, 0);
    }
    if (tid == 0) {
        S.ctr[0] = 0;
        S.ctr[1] = 0;
        S.ctr[2] = 0;
    }
    for (uint32_t w = tid; w <= (uint32_t)kEB; w += kEB) {
        S.smap[w] = 0;
        S.slast[w] = 0;
    }
    // the workgroup's literals: equal input bytes (+ 16 per literal) per workgroup (split_by_bytes has
    // barriers: the clears above are seen by the first tile)
    uint32_t BA, BB;
    hpksplit::split_by_bytes<kEB, 16>(a.in_off, a.n, S.split, BA, BB);
    EPROF(8);
    const uint32_t in_end = min(a.in_off[a.n], a.in_cap) + a.in_mis;  // (clamped: reads stay in the blob)
    const uint32_t last16 = in_end ? (in_end - 1) >> 4 : 0;  // last 16-B chunk holding a batch byte
    const uint4* g_in = reinterpret_cast<const uint4*>(a.in_base);
    // the next tile's input chunks and offsets are loaded into registers while the current one is
    // encoded (issued before its write-back stores, so the wait for them does not include those)
    uint4 ch[2] = {};
    uint32_t pi0[kEMeta], pi1[kEMeta], po0[kEMeta], po1[kEMeta];
    auto prefetch = [&](uint32_t c, uint32_t base16) {
        const uint32_t cn = min((uint32_t)kEQ, BB - c);
#pragma unroll
        for (int r = 0; r < kCh; ++r) ch[r] = g_in[min((base16 >> 4) + (uint32_t)kCh * tid + (uint32_t)r, last16)];
#pragma unroll
        for (int r = 0; r < kEMeta; ++r) {
            const uint32_t t = min(tid + (uint32_t)kEB * r, cn - 1u);
            pi0[r] = a.in_off[c + t];
            pi1[r] = a.in_off[c + t + 1];
            po0[r] = a.out_off[c + t];
            po1[r] = a.out_off[c + t + 1];
        }
    };
    uint32_t cur = BA;
    uint32_t gin = 0, gout = 0;  // the tile's input / output start (base-relative: + mis)
    if (cur < BB) {
        gin = a.in_off[cur] + a.in_mis;
        gout = a.out_off[cur] + a.out_mis;
        prefetch(cur, gin & ~15u);
    }
    while (cur < BB) {  // block-uniform
        const uint32_t cntl = min((uint32_t)kEQ, BB - cur);
        const uint32_t base16 = gin & ~15u, ob16 = gout & ~15u;
        EPROF(7);
        lds_barrier_e();  // the previous tile's image is out
        EPROF(11);
        // (the counters and the start map were cleared after the previous tile's scan, or before the first
        // tile; the live map is first written in finalize, barriers later: v5b, one barrier fewer per tile)
        for (uint32_t w = tid; w < (uint32_t)((kEO / 16 + 31) / 32); w += kEB) S.live[w] = 0;
        EPROF(0);
        // which literals fit (a prefix: offsets are non-decreasing); each fitting non-empty literal marks
        // its first byte in the start map and its index in its word's slast
        uint32_t kw = 0;
        bool bad = false;  // a literal of the tile's range with decreasing offsets or offsets past a capacity
        bool tight = false;  // a fitting literal with less room than 30 bits per input byte
#pragma unroll
        for (int r = 0; r < kEMeta; ++r) {
            const uint32_t t = tid + (uint32_t)kEB * r;
            bad |= t < cntl && !(pi0[r] <= pi1[r] && pi1[r] <= a.in_cap && po0[r] <= po1[r] && po1[r] <= a.out_cap);
        }
#pragma unroll
        for (int r = 0; r < kEMeta; ++r) {
            const uint32_t t = tid + (uint32_t)kEB * r;
            bool fits = false;
            const uint32_t i0 = pi0[r] + a.in_mis, i1 = pi1[r] + a.in_mis;
            const uint32_t o0 = po0[r] + a.out_mis, o1 = po1[r] + a.out_mis;
            if (t < cntl && !bad) fits = i1 - base16 <= (uint32_t)kETile && o1 - ob16 <= (uint32_t)kEO;
            if (fits) {
                S.ioff[t] = i0 - base16;
                S.ooff[t] = o0 - ob16;
                S.ioff[t + 1] = i1 - base16;  // (the same value literal t + 1 writes)
                S.ooff[t + 1] = o1 - ob16;
                S.bits[t] = 0;
                if (i1 > i0) {
                    const uint32_t x = i0 - base16;
                    atomicOr(&S.smap[x >> 5], 1u << (x & 31u));
                    atomicMax(&S.slast[x >> 5], t + 1u);
                }
                tight |= (o1 - o0) * 8u < 30u * (i1 - i0);
            }
            kw += (uint32_t)__popcll(__ballot(fits));
        }
        if (lane == 0 && kw) atomicAdd(&S.ctr[0], kw);
        if (__any(bad) && lane == 0) S.ctr[1] = 1u;
        if (__any(tight) && lane == 0) S.ctr[2] = 1u;
        const uint4 chc0 = ch[0], chc1 = ch[1];
        EPROF(1);
        lds_barrier_e();
        EPROF(11);
        if (S.ctr[1]) {  // bad offsets (block-uniform): the range's remaining literals are void
            for (uint32_t i = cur + tid; i < BB; i += kEB) {
                a.out_len[i] = 0;
                a.status[i] = (uint8_t)HPK_BAD_OFFSETS;
            }
            if (tid == 0) *a.err = 1u;
            break;
        }
        EPROF(1);
        const uint32_t k = S.ctr[0];
        if (tid == 0) S.ioff[k + 1] = 0xFFFFFFFFu;  // pass 2's literal search stops at the phantom literal k
        if (k == 0) {  // literal `cur` alone exceeds a tile: one lane, global memory
            if (tid == 0) encode_serial(a, S.code1, S.len1, cur);
            cur += 1;
            if (cur < BB) {
                gin = a.in_off[cur] + a.in_mis;
                gout = a.out_off[cur] + a.out_mis;
                prefetch(cur, gin & ~15u);
            }
            continue;
        }
        // the next tile: starts where this one ends
        const uint32_t cur_n = cur + k;
        const uint32_t gin_n = S.ioff[k] + base16, gout_n = S.ooff[k] + ob16;
        if (cur_n < BB) prefetch(cur_n, gin_n & ~15u);
        const uint32_t xb = S.ioff[0], xe = S.ioff[k];  // the tile's input bytes [xb, xe)
        const bool tile_safe = S.ctr[2] == 0u;  // every literal has room for 30 bits per byte (the longest code)
        // this thread's bytes [x0, x1); its word of the start map gives the literal starts among them
        // (v5: it replaced a binary search of ioff and a walk over the literals the thread touches)
        const uint32_t x0 = max(tid * (uint32_t)kEBytes, xb), x1 = min(tid * (uint32_t)kEBytes + kEBytes, xe);
        const bool any = x0 < x1;
        const uint32_t xt = tid * (uint32_t)kEBytes;
        const uint32_t sm = S.smap[tid], snext = S.smap[tid + 1], sl = S.slast[tid];
        // the thread's bytes by constant index (the loops below are unrolled: no register array
        // indexed at run time, which the compiler would put in scratch memory)
        const uint32_t wd[8] = {chc0.x, chc0.y, chc0.z, chc0.w, chc1.x, chc1.y, chc1.z, chc1.w};
        // the literal starts among the thread's bytes after its first (bit j: byte xt + j starts a
        // literal; empty literals add nothing) and the bytes it owns: masks, so the byte loops below have
        // no control flow and their table reads issue back to back
        uint32_t bm = 0, vm = 0, em = 0;  // em bit j: byte xt + j is the last of its literal
        bool f0 = false;       // the thread's first byte starts a literal
        bool ends_here = false;  // the thread's last literal ends at its last byte
        if (any) {
            vm = (uint32_t)(((1ull << (x1 - x0)) - 1ull) << (x0 - xt));
            f0 = (sm >> (x0 - xt)) & 1u;
            bm = sm & vm & ~(1u << (x0 - xt));
            ends_here = x1 == xe || (snext & 1u);
            em = (bm >> 1) | (ends_here ? 1u << (x1 - 1u - xt) : 0u);
        }
        // pass 2's run starts: the literal starts, the tile's first byte when the thread holds bytes
        // before it (the run before is a phantom) and the tile's end when the thread holds bytes after
        // it (the run after is a phantom; x1 < xt + 32 only there)
        const uint32_t bm2 = bm | (any && x0 > xt ? 1u << (x0 - xt) : 0u) |
                             (any && x1 < xt + (uint32_t)kEBytes ? 1u << (x1 - xt) : 0u);
        EPROF(2);
        // pass 1: (a literal starts in the thread's bytes, bits since the last start) = the code
        // lengths of the owned bytes from the last literal start on (mask cm)
        const uint32_t f = (f0 || bm) ? 1u : 0u;
        const uint32_t cm = bm ? vm & ~((1u << (31u - __builtin_clz(bm))) - 1u) : vm;
        uint32_t v = 0;
#pragma unroll 1
        for (uint32_t g = 0; g < (uint32_t)kEBytes / 8u; ++g) {  // 8 bytes at a time (register pressure)
            const uint32_t lo8 = g == 0 ? wd[0] : g == 1 ? wd[2] : g == 2 ? wd[4] : wd[6];
            const uint32_t hi8 = g == 0 ? wd[1] : g == 1 ? wd[3] : g == 2 ? wd[5] : wd[7];
            const uint32_t cm8 = cm >> (8u * g);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t ln = S.len1[((k < 4 ? lo8 : hi8) >> (8 * (k & 3))) & 0xFFu];
                v += ln & (uint32_t)__builtin_amdgcn_sbfe((int)cm8, k, 1);  // ln or 0, no select
            }
        }
        EPROF(3);
        // segmented exclusive scan over the workgroup: the carry into each thread's first literal, and
        // (max scan) 1 + the last literal starting before the thread's bytes
        uint32_t fi = f, vi = v, Li = sl;
        wave_seg_scan(fi, vi, Li, lane);
        if (lane == 63) {
            S.wf[wv] = fi;
            S.wv[wv] = vi;
            S.wl[wv] = Li;
        }
        EPROF(4);
        lds_barrier_e();
        EPROF(11);
        uint32_t cw = 0, cl = 0;  // carry into this wave's lane 0 (the waves' totals read together)
#pragma unroll
        for (uint32_t j = 0; j < (uint32_t)kEB / 64u - 1u; ++j) {
            const uint32_t f = S.wf[j], v = S.wv[j], l = S.wl[j];
            if (j < wv) {
                cw = f ? v : cw + v;
                cl = max(cl, l);
            }
        }
        const uint32_t ef = dpp_e<0x138>(fi), ev = dpp_e<0x138>(vi), el = dpp_e<0x138>(Li);  // wave_shr:1 (lane 0: 0)
        const uint32_t carry = ef ? ev : cw + ev;
        // every thread has read the counters and its start-map words (before the barrier above): clear them
        // for the next tile
        if (tid == 0) {
            S.ctr[0] = 0;
            S.ctr[1] = 0;
            S.ctr[2] = 0;
        }
        for (uint32_t w = tid; w <= (uint32_t)kEB; w += kEB) {
            S.smap[w] = 0;
            S.slast[w] = 0;
        }
        const uint32_t lx = max(cl, el);  // 1 + the last non-empty literal starting before byte xt
        // the literal holding x0: the one starting there (after any empty ones), else the last one
        // started before it
        uint32_t li = 0;
        if (any) {
            if (f0) {
                li = lx;
                while (S.ioff[li + 1] <= x0) ++li;
            } else {
                li = lx - 1u;
            }
        }
        // pass 2: each run of codes (this thread's bytes of one literal) is packed into a 64-bit
        // accumulator aligned to the image's dword grid: whole dwords inside the run are plain
        // stores, the run's first and last (shared with neighbouring runs) are ds_or; a code past
        // the literal's capacity is clipped (rare: the caller's capacity below the bound)
        EPROF(4);
        if (tile_safe) {
            // v3 pass 2 (every literal of the wave's threads has room): per byte, the code is shifted
            // into a 64-bit accumulator holding the bits of the current image dword on (n of them,
            // counted from the dword's start: a run that starts mid-dword begins with n zero bits
            // that the OR leaves alone), and the dword's bits so far go out with one ds_or per byte,
            // so the byte loop has no branch but the run starts'. Every byte of the thread is coded
            // (no ownership mask): bytes outside the tile's literals belong to phantom runs whose
            // dwords land past the image, and a literal's bit count is its run's end position minus
            // its start (no per-byte count). The run-start branch advances to the next literal with
            // offsets read at the previous start (nq: its first bit, nx: the first byte of the
            // literal after it; an empty literal between takes the search).
            uint32_t lj = any && x0 > xt ? li - 1u : li;
            uint32_t nq = S.ooff[lj + 1u] * 8u, nx = S.ioff[lj + 2u];
            bool ph = !any || x0 > xt;  // in a phantom run
            const uint32_t qph = (uint32_t)(kEO / 4 + (tid & 31u)) * 32u;
            uint32_t qs = ph ? qph : S.ooff[li] * 8u;  // the run's literal's first bit
            const uint32_t q = ph ? qph : qs + (f0 ? 0u : carry);
            uint32_t dq = q >> 5, n = q & 31u;
            uint64_t acc = 0;
#pragma unroll 1
            for (uint32_t g = 0; g < (uint32_t)kEBytes / 8u; ++g) {
                const uint32_t lo8 = g == 0 ? wd[0] : g == 1 ? wd[2] : g == 2 ? wd[4] : wd[6];
                const uint32_t hi8 = g == 0 ? wd[1] : g == 1 ? wd[3] : g == 2 ? wd[5] : wd[7];
                const uint32_t bm8 = bm2 >> (8u * g);
                // the group's table reads issue together, ahead of the run-start branches (which
                // would otherwise hold each read back to its own byte)
                uint2 tb[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) tb[j] = S.tab[((j < 4 ? lo8 : hi8) >> (8 * (j & 3))) & 0xFFu];
                // a run starts at byte j: close the previous one
                auto start = [&](int j) {
                    if (n) atomicOr(&S.img[dq], (uint32_t)(acc << (32u - n)));
                    if (!ph) S.bits[lj] = dq * 32u + n - qs;
                    const uint32_t x = xt + 8u * g + (uint32_t)j;
                    if (nx > x) {
                        ++lj;
                        qs = nq;
                    } else {
                        while (S.ioff[lj + 1] <= x) ++lj;  // (empty literals between: bits stay 0)
                        qs = S.ooff[lj] * 8u;
                    }
                    ph = lj >= k;  // (k: the tile's literals) the tile's end: the rest is a phantom
                    qs = ph ? qph : qs;
                    nq = S.ooff[lj + 1u] * 8u;
                    nx = S.ioff[lj + 2u];
                    dq = qs >> 5;
                    n = qs & 31u;
                    acc = 0;
                };
                // one code: the current dword's bits so far — all of them once it is complete — ORed
                // in (a prefix ORs nothing the complete dword does not)
                auto put = [&](uint2 cl) {
                    acc = (acc << cl.y) | cl.x;
                    n += cl.y;  // 5 <= n < 62
                    const bool full = n >= 32u;
                    atomicOr(&S.img[dq], (uint32_t)((acc << (64u - n)) >> 32));
                    dq += full ? 1u : 0u;
                    n &= 31u;
                };
#pragma unroll
                for (int j = 0; j < 8; j += 2) {
                    const uint2 c0 = tb[j], c1 = tb[j + 1];
                    if ((bm8 >> j) & 1u) start(j);
                    // (two codes per OR where a whole wave can — no run start at the second byte, the
                    // two codes within the dword's room — measured slower: config 3 537 vs 503-509 us;
                    // ORing only complete dwords too: 510-514 vs 502-504 us)
                    put(c0);
                    if ((bm8 >> (j + 1)) & 1u) start(j + 1);
                    put(c1);
                }
            }
            if (any && !ph) {
                if (n) atomicOr(&S.img[dq], (uint32_t)(acc << (32u - n)));
                if (ends_here) S.bits[lj] = dq * 32u + n - qs;
            }
        } else if (any) {
            uint32_t lj = li;
            uint32_t bp = f0 ? 0u : carry;
            uint32_t ob = S.ooff[li] * 8u, cap = S.ooff[li + 1] * 8u - ob;
            uint32_t dq = (ob + bp) >> 5, n = (ob + bp) & 31u;
            uint64_t acc = 0;
            bool first = true;
            auto flush_run = [&]() {
                if (n) atomicOr(&S.img[dq], (uint32_t)(acc << (32u - n)));
                n = 0;
                acc = 0;
            };
#pragma unroll 1
            for (uint32_t g = 0; g < (uint32_t)kEBytes / 8u; ++g) {
            const uint32_t lo8 = g == 0 ? wd[0] : g == 1 ? wd[2] : g == 2 ? wd[4] : wd[6];
            const uint32_t hi8 = g == 0 ? wd[1] : g == 1 ? wd[3] : g == 2 ? wd[5] : wd[7];
            const uint32_t vm8 = vm >> (8u * g), bm8 = bm >> (8u * g);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t b = ((k < 4 ? lo8 : hi8) >> (8 * (k & 3))) & 0xFFu;
                const uint32_t code = S.code1[b], ln = S.len1[b];
                if ((vm8 >> k) & 1u) {
                    const uint32_t x = xt + 8u * g + (uint32_t)k;
                    if ((bm8 >> k) & 1u) {  // a new literal: close the run, skip empty literals
                        flush_run();
                        while (S.ioff[lj + 1] <= x) ++lj;
                        bp = 0;
                        ob = S.ooff[lj] * 8u;
                        cap = S.ooff[lj + 1] * 8u - ob;
                        dq = ob >> 5;
                        n = ob & 31u;
                        first = true;
                    }
                    if (bp + ln <= cap) {
                        acc = (acc << ln) | code;
                        n += ln;
                        if (n >= 32u) {
                            const uint32_t w = (uint32_t)(acc >> (n - 32u));
                            if (first)
                                atomicOr(&S.img[dq], w);
                            else
                                S.img[dq] = w;
                            first = false;
                            dq += 1;
                            n -= 32u;
                            acc &= (1ull << n) - 1ull;
                        }
                    } else {  // overflow: close the run, then the bits of this code that still fit
                        flush_run();
                        if (bp < cap) {
                            const uint32_t keep = cap - bp;
                            img_or(S.img, ob + bp, code >> (ln - keep), keep);
                        }
                    }
                    bp += ln;
                    if ((em >> (8u * g + k)) & 1u) S.bits[lj] = bp;  // the literal's last byte
                }
            }
            }
            flush_run();
        }
        EPROF(5);
        lds_barrier_e();
        EPROF(11);
        // per literal: EOS padding, out_len, status
#pragma unroll
        for (int r = 0; r < kEMeta; ++r) {
            const uint32_t t = tid + (uint32_t)kEB * r;
            if (t < k) {
                const uint32_t bits = S.bits[t];
                const uint32_t cap = S.ooff[t + 1] - S.ooff[t];
                const uint32_t nbytes = (bits + 7u) >> 3;
                const bool over = nbytes > cap;
                if (!over && (bits & 7u)) {
                    const uint32_t pad = 8u - (bits & 7u);
                    img_or(S.img, S.ooff[t] * 8u + bits, (1u << pad) - 1u, pad);
                }
                const uint32_t len = over ? cap : nbytes;
                a.out_len[cur + t] = len;
                a.status[cur + t] = (uint8_t)(over ? HPK_OUTPUT_OVERFLOW : HPK_OK);
                if (len) {  // the image chunks holding the output: the only ones stored
                    const uint32_t ca = S.ooff[t] >> 4, cb = (S.ooff[t] + len - 1u) >> 4;
                    for (uint32_t w = ca >> 5; w <= cb >> 5; ++w) {
                        const uint32_t lo = w == (ca >> 5) ? (ca & 31u) : 0u, hi = w == (cb >> 5) ? (cb & 31u) : 31u;
                        atomicOr(&S.live[w], (0xFFFFFFFFu >> (31u - hi)) & (0xFFFFFFFFu << lo));
                    }
                }
            }
        }
        EPROF(6);
        lds_barrier_e();
        EPROF(11);
        {  // write the image back: bytes [G0, G1) of the image (relative to ob16)
            const uint32_t G0 = S.ooff[0], G1 = S.ooff[k];
            const uint32_t c1 = (G1 + 15u) >> 4;
            const uint4* i16 = reinterpret_cast<const uint4*>(S.img);
            uint4* g16 = reinterpret_cast<uint4*>(a.out_base + ob16);
            uint4* m16 = reinterpret_cast<uint4*>(S.img);
            for (uint32_t c = tid; c < c1; c += kEB) {
                // (live chunks only: with encode_offsets' regions, 30 bits per input byte, most of the
                // span is slack no byte of output reaches)
                if ((c << 4) >= G0 && (c << 4) + 16u <= G1 && ((S.live[c >> 5] >> (c & 31u)) & 1u)) {
                    const uint4 w = i16[c];
                    g16[c] = make_uint4(__builtin_bswap32(w.x), __builtin_bswap32(w.y), __builtin_bswap32(w.z),
                                        __builtin_bswap32(w.w));
                    m16[c] = make_uint4(0, 0, 0, 0);
                }
            }
            if (tid < 32) {  // the partial chunks at the two ends, one byte per lane
                const uint32_t g = tid < 16 ? 0u : (c1 - 1u) << 4;
                const bool partial = !(g >= G0 && g + 16u <= G1) && (tid < 16 || c1 - 1u != 0u);
                const uint32_t x = g + (tid & 15u);
                if (partial && x >= G0 && x < G1) {
                    const uint32_t w = S.img[x >> 2];
                    a.out_base[ob16 + x] = (uint8_t)(w >> (24u - 8u * (x & 3u)));
                }
                // then clear them (wave 0's reads above come first: one wave, program order)
                if ((tid & 15u) == 0 && partial) m16[g >> 4] = make_uint4(0, 0, 0, 0);
            }
        }
        EPROF(7);
        cur = cur_n;
        gin = gin_n;
        gout = gout_n;
    }
    if (kProf) {
        __syncthreads();
        if (tid < (kEB / 64) * 12) atomicAdd(&a.prof[tid % 12], S.prof[tid / 12][tid % 12]);
    }
}

#ifdef HPK_DIAG
static int g_encode_v1 = -1, g_encode_cfg = 0;
static unsigned long long* g_eprof = nullptr;  // HPK_ENCODE_PROF=1: hpk_encode2's phase cycles
#endif

}  // namespace

int hpk_launch_encode(hpk_ctx* c, const hpk_batch& b) {
    EncodeArgs a{b.in_blob, b.in_off, b.n, b.out_blob, b.out_off, b.out_len, b.status, c->d_codes};
    const uintptr_t ip = (uintptr_t)b.in_blob, op = (uintptr_t)b.out_blob;
    a.in_base = (const uint8_t*)(ip & ~(uintptr_t)15);
    a.in_mis = (uint32_t)(ip & 15);
    a.out_base = (uint8_t*)(op & ~(uintptr_t)15);
    a.out_mis = (uint32_t)(op & 15);
    a.in_cap = b.in_cap;
    a.out_cap = b.out_cap;
    a.err = c->d_err;
    a.prof = nullptr;
    int cfg = 0;
#ifdef HPK_DIAG
    // diagnostic build only: v1 (one lane per literal, no offset checks) and geometry variants
    if (g_encode_v1 < 0) {
        const char* e = getenv("HPK_ENCODE_V1");
        g_encode_v1 = e && atoi(e) ? 1 : 0;
        const char* w = getenv("HPK_ENCODE_CFG");
        g_encode_cfg = w ? atoi(w) : 0;
    }
    cfg = g_encode_cfg;
    if (g_encode_v1) {
        uint64_t blocks = ((uint64_t)b.n + ENC_BLOCK - 1) / ENC_BLOCK;
        const uint64_t max_blocks = (uint64_t)c->num_cu * 8;
        if (blocks > max_blocks) blocks = max_blocks;
        if (blocks < 1) blocks = 1;
        hipLaunchKernelGGL(hpk_encode_kernel, dim3((uint32_t)blocks), dim3(ENC_BLOCK), 0, c->stream, a);
        HIP_TRY(hipGetLastError());
        return HPK_E_OK;
    }
#endif
    // per = workgroups per CU; fewer when the batch is small (>= ~64 literals per workgroup)
    const int per = cfg == 1 ? 1 : 2;
    uint64_t blocks = ((uint64_t)b.n + 63) / 64;
    // (the small-call mode's persistent workgroups hold sm_wgs CUs, hpk_persist.h: left out of the grid)
    const uint64_t cus = (uint64_t)c->num_cu - (c->sm_launched && c->sm_max ? (uint64_t)c->sm_wgs : 0u);
    if (blocks > cus * per) blocks = cus * per;
    if (blocks < 1) blocks = 1;
    const dim3 grid((uint32_t)blocks);
    switch (cfg) {
#ifdef HPK_DIAG
        case 1:  // one 1024-thread workgroup per CU, 32 KiB tiles
            hipLaunchKernelGGL((hpk_encode2<1024, 112 * 1024, 2048, 32>), grid, dim3(1024), 0, c->stream, a);
            break;
        case 9:  // the product geometry with per-phase cycle counters (hpk_debug_encode_prof)
            if (!g_eprof) HIP_TRY(hipMalloc(&g_eprof, 16 * sizeof(unsigned long long)));
            HIP_TRY(hipMemsetAsync(g_eprof, 0, 16 * sizeof(unsigned long long), c->stream));
            a.prof = g_eprof;
            hipLaunchKernelGGL((hpk_encode2<512, 56 * 1024, 1024, 32, 1>), grid, dim3(512), 0, c->stream, a);
            break;
#endif
        default:  // product: two 512-thread workgroups per CU, 32 bytes per thread
            hipLaunchKernelGGL((hpk_encode2<512, 56 * 1024, 1024, 32>), grid, dim3(512), 0, c->stream, a);
    }
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}

#ifdef HPK_DIAG
// diagnostic build: the phase cycles of the last HPK_ENCODE_CFG=9 launch (16 x u64)
extern "C" int hpk_debug_encode_prof(unsigned long long* host16) {
    if (!g_eprof) return -1;
    return hipMemcpy(host16, g_eprof, 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
