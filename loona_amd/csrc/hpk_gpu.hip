// hpk_gpu.hip — device half of libhpk: gfx950 (CDNA4) Huffman decode/encode kernels and the
// batch C ABI (include/hpk.h).
//
// Decode: one lane per literal, literals dealt to lanes by a per-wave work queue (a lane that
// finishes takes the next literal of its wave's range, chosen by ballot + mbcnt, so a long
// literal does not idle the other 63 lanes). Decode tables (hpk_code.h) are staged once per
// workgroup in LDS: a 2^12-entry two-symbol LUT (16 KiB) plus the 960-entry leading-ones table
// that decodes any longer codeword in one lookup. The literal bits are read through a 64-bit
// big-endian window refilled one aligned dword at a time; bits past the literal's end read as
// ones so the end-of-literal checks match huffman.rs:128-160 exactly.
//
// Encode: one lane per literal, codes from an LDS copy of the 257-entry table, bit-packed
// MSB-first into a 64-bit accumulator and flushed a byte at a time, padded with EOS MSBs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/hpk.h"
#include "hpk_code.h"
#include "hpk_internal.h"

#define HPK_VERSION "hpk 0.1 gfx950 lane-queue decode v1"

static thread_local std::string t_last_error;

static int set_err(const char* what, hipError_t e) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    t_last_error = buf;
    return HPK_E_DEVICE;
}
static int set_err_msg(const char* what, int code) {
    t_last_error = what;
    return code;
}

#define HIP_TRY(call)                                  \
    do {                                               \
        hipError_t _e = (call);                        \
        if (_e != hipSuccess) return set_err(#call, _e); \
    } while (0)

// ------------------------------------------------------------------------------------------
// device decode

struct DecodeArgs {
    const uint32_t* in_words;  // in_blob rounded down to a 4-byte boundary
    uint32_t in_mis;           // in_blob - in_words (0..3)
    const uint32_t* in_off;
    uint32_t n;
    uint8_t* out_blob;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
    const uint32_t* lut;
    const uint16_t* lo;
};

#define DEC_BLOCK 256
#define DEC_WAVES (DEC_BLOCK / 64)

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Decode literal i completely. Returns nothing; writes out bytes, out_len[i], status[i].
__device__ __forceinline__ void decode_literal(const DecodeArgs& a, const uint32_t* __restrict__ s_lut,
                                               const uint16_t* __restrict__ s_lo, uint32_t i) {
    const uint32_t s = a.in_off[i], e = a.in_off[i + 1];
    const uint32_t o0 = a.out_off[i];
    const uint32_t ocap = a.out_off[i + 1] - o0;
    uint8_t* __restrict__ out = a.out_blob + o0;
    uint32_t rem = (e - s) * 8u;  // literal bits not yet consumed
    uint32_t cnt = 0;
    uint32_t st = HPK_OK;
    uint64_t win = 0;
    int nb = 0;
    uint32_t q = 0, qe = 0;
    if (rem) {
        const uint32_t p = s + a.in_mis, pe = e + a.in_mis;
        const uint32_t w0 = bswap32(a.in_words[p >> 2]);
        const int sk = (int)(p & 3u) * 8;
        win = ((uint64_t)w0 << 32) << sk;
        nb = 32 - sk;
        q = (p >> 2) + 1;
        qe = (pe + 3) >> 2;
    }
    while (rem > 0) {
        if (nb <= 32 && q < qe) {
            const uint32_t d = bswap32(a.in_words[q++]);
            win |= (uint64_t)d << (32 - nb);
            nb += 32;
        }
        uint32_t w = (uint32_t)(win >> 32);
        if (rem < 32) w |= 0xFFFFFFFFu >> rem;
        const uint32_t ent = s_lut[w >> (32 - HPK_LUT_BITS)];
        uint32_t nsym = ent >> 26;
        uint32_t sym0 = ent & 0xFFu, sym1 = (ent >> 8) & 0xFFu;
        uint32_t len = (ent >> 16) & 31u, total = (ent >> 21) & 31u;
        if (nsym == 0) {
            const uint32_t k = __clz(~w);
            if (k >= HPK_LO_RUNS) {
                sym0 = HPK_EOS;
                len = 30;
            } else {
                const uint32_t lo = s_lo[k * 32 + ((w << (k + 1)) >> 27)];
                sym0 = lo & 0x1FFu;
                len = lo >> 9;
            }
            total = len;
        }
        if (len > rem) break;
        if (sym0 == HPK_EOS) { st = HPK_EOS_IN_STRING; break; }
        if (cnt >= ocap) { st = HPK_OUTPUT_OVERFLOW; break; }
        out[cnt++] = (uint8_t)sym0;
        if (nsym == 2 && total <= rem) {
            if (cnt >= ocap) { st = HPK_OUTPUT_OVERFLOW; break; }
            out[cnt++] = (uint8_t)sym1;
            len = total;
        }
        win <<= len;
        nb -= (int)len;
        rem -= len;
    }
    if (st == HPK_OK && rem > 0) {
        if (rem > 7) {
            st = HPK_PADDING_TOO_LARGE;
        } else {
            const uint32_t w = (uint32_t)(win >> 32) | (0xFFFFFFFFu >> rem);
            if (w != 0xFFFFFFFFu) st = HPK_INVALID_PADDING;
        }
    }
    a.out_len[i] = cnt;
    a.status[i] = (uint8_t)st;
}

__global__ __launch_bounds__(DEC_BLOCK) void hpk_decode_kernel(DecodeArgs a, uint32_t per_wave) {
    __shared__ __attribute__((aligned(16))) uint32_t s_lut[HPK_LUT_SIZE];
    __shared__ __attribute__((aligned(16))) uint16_t s_lo[HPK_LO_SIZE];
    for (uint32_t t = threadIdx.x; t < HPK_LUT_SIZE / 4; t += DEC_BLOCK)
        reinterpret_cast<uint4*>(s_lut)[t] = reinterpret_cast<const uint4*>(a.lut)[t];
    for (uint32_t t = threadIdx.x; t < HPK_LO_SIZE / 8; t += DEC_BLOCK)
        reinterpret_cast<uint4*>(s_lo)[t] = reinterpret_cast<const uint4*>(a.lo)[t];
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gwave = blockIdx.x * DEC_WAVES + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * DEC_WAVES;
    // each wave owns contiguous chunks of `per_wave` literals, grid-strided
    for (uint64_t base = (uint64_t)gwave * per_wave; base < a.n; base += (uint64_t)nwaves * per_wave) {
        const uint32_t lo_i = (uint32_t)base;
        const uint32_t hi_i = (uint32_t)min<uint64_t>(base + per_wave, a.n);
        // lane work queue: next = lo_i + 64 initially, lanes pull in ballot order
        uint32_t next = lo_i + 64;
        uint32_t mine = lo_i + lane;
        while (true) {
            const bool active = mine < hi_i;
            if (!__any(active)) break;
            if (active) decode_literal(a, s_lut, s_lo, mine);
            // every lane that was active is now free; hand out the next indices
            const uint64_t freed = __ballot(active);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(freed >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)freed, 0u));
            if (active) mine = next + rank;
            next += (uint32_t)__popcll(freed);
        }
    }
}

// ------------------------------------------------------------------------------------------
// device encode

struct EncodeArgs {
    const uint8_t* in_blob;
    const uint32_t* in_off;
    uint32_t n;
    uint8_t* out_blob;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
    const uint32_t* codes;  // [0,257): right-aligned code, [257,514): length
};

#define ENC_BLOCK 256

__global__ __launch_bounds__(ENC_BLOCK) void hpk_encode_kernel(EncodeArgs a) {
    __shared__ uint32_t s_code[256];
    __shared__ uint8_t s_len[256];
    if (threadIdx.x < 256) {
        s_code[threadIdx.x] = a.codes[threadIdx.x];
        s_len[threadIdx.x] = (uint8_t)a.codes[257 + threadIdx.x];
    }
    __syncthreads();
    for (uint32_t i = blockIdx.x * ENC_BLOCK + threadIdx.x; i < a.n; i += gridDim.x * ENC_BLOCK) {
        const uint32_t s = a.in_off[i], e = a.in_off[i + 1];
        const uint32_t o0 = a.out_off[i], ocap = a.out_off[i + 1] - o0;
        uint8_t* out = a.out_blob + o0;
        uint64_t acc = 0;
        int nb = 0;
        uint32_t o = 0;
        uint32_t st = HPK_OK;
        for (uint32_t p = s; p < e; ++p) {
            const uint32_t b = a.in_blob[p];
            acc = (acc << s_len[b]) | s_code[b];
            nb += s_len[b];
            while (nb >= 8) {
                nb -= 8;
                if (o >= ocap) { st = HPK_OUTPUT_OVERFLOW; break; }
                out[o++] = (uint8_t)(acc >> nb);
            }
            if (st) break;
        }
        if (!st && nb) {
            if (o >= ocap) st = HPK_OUTPUT_OVERFLOW;
            else out[o++] = (uint8_t)((acc << (8 - nb)) | (0xFFu >> nb));
        }
        a.out_len[i] = o;
        a.status[i] = (uint8_t)st;
    }
}

// ------------------------------------------------------------------------------------------
// context

struct hpk_ctx {
    int device = 0;
    int num_cu = 256;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    uint32_t* d_lut = nullptr;
    uint16_t* d_lo = nullptr;
    uint32_t* d_codes = nullptr;
    // grow-only scratch for HPK_PTR_HOST calls
    uint8_t* d_in = nullptr;
    size_t d_in_cap = 0;
    uint8_t* d_out = nullptr;
    size_t d_out_cap = 0;
    uint32_t* d_meta = nullptr;  // in_off | out_off | out_len
    size_t d_meta_cap = 0;
    uint8_t* d_st = nullptr;
    size_t d_st_cap = 0;
};

extern "C" const char* hpk_version(void) { return HPK_VERSION; }

extern "C" const char* hpk_last_error(const hpk_ctx*) { return t_last_error.c_str(); }

extern "C" hpk_ctx* hpk_ctx_create(int device) {
    const hpk_tables* t = hpk_get_tables();
    if (!t) { set_err_msg("code table build failed", HPK_E_INVAL); return nullptr; }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) { set_err("hipGetDeviceCount", e); return nullptr; }
    if (device < 0 || device >= ndev) { set_err_msg("device index out of range", HPK_E_INVAL); return nullptr; }
    hpk_ctx* c = new hpk_ctx();
    c->device = device;
    auto fail = [&](const char* what, hipError_t err) {
        set_err(what, err);
        hpk_ctx_destroy(c);
        return (hpk_ctx*)nullptr;
    };
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return fail("hipGetDeviceProperties", e);
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_err_msg("libhpk kernels are built for gfx950 only", HPK_E_NODEVICE);
        delete c;
        return nullptr;
    }
    c->num_cu = prop.multiProcessorCount;
    if ((e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", e);
    c->stream = c->own;
    if ((e = hipMalloc(&c->d_lut, sizeof(t->lut))) != hipSuccess) return fail("hipMalloc lut", e);
    if ((e = hipMalloc(&c->d_lo, sizeof(t->lo))) != hipSuccess) return fail("hipMalloc lo", e);
    if ((e = hipMalloc(&c->d_codes, 2 * 257 * sizeof(uint32_t))) != hipSuccess) return fail("hipMalloc codes", e);
    uint32_t packed[2 * 257];
    for (int s = 0; s < 257; ++s) {
        packed[s] = t->code[s];
        packed[257 + s] = t->len[s];
    }
    if ((e = hipMemcpy(c->d_lut, t->lut, sizeof(t->lut), hipMemcpyHostToDevice)) != hipSuccess) return fail("upload lut", e);
    if ((e = hipMemcpy(c->d_lo, t->lo, sizeof(t->lo), hipMemcpyHostToDevice)) != hipSuccess) return fail("upload lo", e);
    if ((e = hipMemcpy(c->d_codes, packed, sizeof(packed), hipMemcpyHostToDevice)) != hipSuccess) return fail("upload codes", e);
    return c;
}

extern "C" void hpk_ctx_destroy(hpk_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->d_lut);
    (void)hipFree(c->d_lo);
    (void)hipFree(c->d_codes);
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_meta);
    (void)hipFree(c->d_st);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

extern "C" int hpk_ctx_set_stream(hpk_ctx* c, void* s) {
    if (!c) return HPK_E_INVAL;
    c->stream = s ? (hipStream_t)s : c->own;
    return HPK_E_OK;
}

extern "C" void* hpk_ctx_stream(hpk_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int hpk_ctx_sync(hpk_ctx* c) {
    if (!c) return HPK_E_INVAL;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return HPK_E_OK;
}

static int grow(void** p, size_t* cap, size_t need) {
    if (need <= *cap) return HPK_E_OK;
    size_t n = need + need / 4 + 4096;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc(p, n));
    *cap = n;
    return HPK_E_OK;
}

static int check_offsets(const uint32_t* off, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) return set_err_msg("offsets must be non-decreasing", HPK_E_INVAL);
    return HPK_E_OK;
}

static int launch_decode(hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n,
                         uint8_t* out_blob, const uint32_t* out_off, uint32_t* out_len, uint8_t* status) {
    DecodeArgs a;
    const uintptr_t ip = (uintptr_t)in_blob;
    a.in_words = (const uint32_t*)(ip & ~(uintptr_t)3);
    a.in_mis = (uint32_t)(ip & 3);
    a.in_off = in_off;
    a.n = n;
    a.out_blob = out_blob;
    a.out_off = out_off;
    a.out_len = out_len;
    a.status = status;
    a.lut = c->d_lut;
    a.lo = c->d_lo;
    const uint32_t per_wave = 256;
    const uint64_t waves_needed = ((uint64_t)n + per_wave - 1) / per_wave;
    uint64_t blocks = (waves_needed + DEC_WAVES - 1) / DEC_WAVES;
    const uint64_t max_blocks = (uint64_t)c->num_cu * 8;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(hpk_decode_kernel, dim3((uint32_t)blocks), dim3(DEC_BLOCK), 0, c->stream, a, per_wave);
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}

static int launch_encode(hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n,
                         uint8_t* out_blob, const uint32_t* out_off, uint32_t* out_len, uint8_t* status) {
    EncodeArgs a{in_blob, in_off, n, out_blob, out_off, out_len, status, c->d_codes};
    uint64_t blocks = ((uint64_t)n + ENC_BLOCK - 1) / ENC_BLOCK;
    const uint64_t max_blocks = (uint64_t)c->num_cu * 8;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(hpk_encode_kernel, dim3((uint32_t)blocks), dim3(ENC_BLOCK), 0, c->stream, a);
    HIP_TRY(hipGetLastError());
    return HPK_E_OK;
}

typedef int (*launch_fn)(hpk_ctx*, const uint8_t*, const uint32_t*, uint32_t, uint8_t*, const uint32_t*,
                         uint32_t*, uint8_t*);

static int run_batch(launch_fn fn, hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n,
                     uint8_t* out_blob, const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int flags) {
    if (!c || !in_off || !out_off || (n && (!out_len || !status))) return set_err_msg("null argument", HPK_E_INVAL);
    HIP_TRY(hipSetDevice(c->device));
    if (flags & HPK_PTR_DEVICE) {
        if (n == 0) return HPK_E_OK;
        if (!in_blob || !out_blob) return set_err_msg("null blob", HPK_E_INVAL);
        int rc = fn(c, in_blob, in_off, n, out_blob, out_off, out_len, status);
        if (rc) return rc;
        if (!(flags & HPK_ASYNC)) HIP_TRY(hipStreamSynchronize(c->stream));
        return HPK_E_OK;
    }
    // host pointers: validate, stage, run, copy back
    if (check_offsets(in_off, n) || check_offsets(out_off, n)) return HPK_E_INVAL;
    if (n == 0) return HPK_E_OK;
    const size_t in_bytes = in_off[n], out_bytes = out_off[n];
    if ((in_bytes && !in_blob) || (out_bytes && !out_blob)) return set_err_msg("null blob", HPK_E_INVAL);
    int rc;
    if ((rc = grow((void**)&c->d_in, &c->d_in_cap, in_bytes + 16))) return rc;
    if ((rc = grow((void**)&c->d_out, &c->d_out_cap, out_bytes + 16))) return rc;
    if ((rc = grow((void**)&c->d_meta, &c->d_meta_cap, (3 * (size_t)n + 2) * 4))) return rc;
    if ((rc = grow((void**)&c->d_st, &c->d_st_cap, n))) return rc;
    uint32_t* d_in_off = c->d_meta;
    uint32_t* d_out_off = c->d_meta + (n + 1);
    uint32_t* d_len = c->d_meta + 2 * ((size_t)n + 1);
    if (in_bytes) HIP_TRY(hipMemcpyAsync(c->d_in, in_blob, in_bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_in_off, in_off, (n + 1) * 4ull, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_out_off, out_off, (n + 1) * 4ull, hipMemcpyHostToDevice, c->stream));
    if ((rc = fn(c, c->d_in, d_in_off, n, c->d_out, d_out_off, d_len, c->d_st))) return rc;
    if (out_bytes) HIP_TRY(hipMemcpyAsync(out_blob, c->d_out, out_bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(out_len, d_len, n * 4ull, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(status, c->d_st, n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return HPK_E_OK;
}

extern "C" int hpk_decode_batch(hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n,
                                uint8_t* out_blob, const uint32_t* out_off, uint32_t* out_len, uint8_t* status,
                                int flags) {
    return run_batch(launch_decode, c, in_blob, in_off, n, out_blob, out_off, out_len, status, flags);
}

extern "C" int hpk_encode_batch(hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n,
                                uint8_t* out_blob, const uint32_t* out_off, uint32_t* out_len, uint8_t* status,
                                int flags) {
    return run_batch(launch_encode, c, in_blob, in_off, n, out_blob, out_off, out_len, status, flags);
}
