// hpk_cpu.cpp — host half of libhpk: the scalar single-literal entry points (the CPU drop-in for
// HuffmanDecoder::decode, crates/loona-hpack/src/huffman.rs:95-161) and the shared code tables.
//
// The decoder here is table-driven (HPK_LUT_BITS-bit two-symbol LUT + the leading-ones table,
// see hpk_code.h), not the reference's bit-at-a-time hash walk; its results, including the
// error precedence (EOS at once, then >7 residual bits, then non-EOS padding) and the bytes
// decoded before an error, match the reference bit for bit (tests/test_host.py).
#include <string.h>

#include <mutex>
#include <thread>
#include <vector>

#include "../../include/hpk.h"
#include "hpk_code.h"
#include "hpk_internal.h"

static hpk_tables g_tables;
static int g_tables_rc = -1;
static std::once_flag g_tables_once;

const hpk_tables* hpk_get_tables() {
    std::call_once(g_tables_once, [] { g_tables_rc = hpk_build_tables(&g_tables); });
    return g_tables_rc == 0 ? &g_tables : nullptr;
}

extern "C" size_t hpk_decoded_bound(size_t n) { return n * 8 / 5; }
extern "C" size_t hpk_encoded_bound(size_t n) { return (30 * n + 7) / 8; }

extern "C" size_t hpk_huffman_encoded_len(const uint8_t* in, size_t n) {
    const hpk_tables* t = hpk_get_tables();
    if (!t || (!in && n)) return 0;
    uint64_t bits = 0;
    for (size_t i = 0; i < n; ++i) bits += t->len[in[i]];
    return (size_t)((bits + 7) / 8);
}

// Decode core shared by the single-literal API. Reads the literal through a 64-bit MSB-aligned
// window; bits past the end read as ones (the EOS prefix), so a code that runs past the end is
// recognised as "longer than what is left" and ends the walk exactly where the reference's
// bit iterator would stop matching.
int hpk_cpu_decode(const hpk_tables* t, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                   size_t* out_len) {
    uint64_t win = 0;
    int nb = 0;
    size_t p = 0;
    uint64_t rem = (uint64_t)n * 8;
    size_t cnt = 0;
    int st = HPK_OK;
    while (rem > 0) {
        while (nb <= 56 && p < n) {
            win |= (uint64_t)in[p++] << (56 - nb);
            nb += 8;
        }
        uint32_t w = (uint32_t)(win >> 32);
        if (rem < 32) w |= 0xFFFFFFFFu >> rem;
        uint32_t e = t->lut[w >> (32 - HPK_LUT_BITS)];
        uint32_t nsym = e >> 26, sym0, sym1 = 0, len, total;
        if (nsym == 0) {
            uint32_t k = (~w) ? (uint32_t)__builtin_clz(~w) : 32u;
            if (k >= HPK_LO_RUNS) {
                sym0 = HPK_EOS;
                len = 30;
            } else {
                uint16_t lo = t->lo[k * 32 + ((w << (k + 1)) >> 27)];
                sym0 = lo & 0x1FF;
                len = lo >> 9;
            }
            total = len;
        } else {
            sym0 = e & 0xFF;
            sym1 = (e >> 8) & 0xFF;
            len = (e >> 16) & 31;
            total = (e >> 21) & 31;
        }
        if (len > rem) break;
        if (sym0 == HPK_EOS) { st = HPK_EOS_IN_STRING; break; }
        if (cnt >= cap) { st = HPK_OUTPUT_OVERFLOW; break; }
        out[cnt++] = (uint8_t)sym0;
        if (nsym == 2 && total <= rem) {
            if (cnt >= cap) { st = HPK_OUTPUT_OVERFLOW; break; }
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
            uint32_t w = (uint32_t)(win >> 32) | (0xFFFFFFFFu >> rem);
            if (w != 0xFFFFFFFFu) st = HPK_INVALID_PADDING;
        }
    }
    *out_len = cnt;
    return st;
}

extern "C" int hpk_huffman_decode_one(const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                                      size_t* out_len) {
    const hpk_tables* t = hpk_get_tables();
    if (!t) return HPK_E_INVAL;
    if (!out_len || (!in && n) || (!out && cap)) return HPK_E_INVAL;
    return hpk_cpu_decode(t, in, n, out, cap, out_len);
}

int hpk_cpu_encode(const hpk_tables* t, const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                   size_t* out_len) {
    uint64_t acc = 0;
    int nb = 0;
    size_t o = 0;
    // on HPK_E_NOSPACE *out_len = cap: out holds the encoding's first cap bytes (as the device kernels)
    for (size_t i = 0; i < n; ++i) {
        acc = (acc << t->len[in[i]]) | t->code[in[i]];
        nb += t->len[in[i]];
        while (nb >= 8) {
            if (o >= cap) {
                *out_len = o;
                return HPK_E_NOSPACE;
            }
            nb -= 8;
            out[o++] = (uint8_t)(acc >> nb);
        }
    }
    if (nb) {
        if (o >= cap) {
            *out_len = o;
            return HPK_E_NOSPACE;
        }
        out[o++] = (uint8_t)((acc << (8 - nb)) | (0xFFu >> nb));
    }
    *out_len = o;
    return HPK_E_OK;
}

extern "C" int hpk_huffman_encode_one(const uint8_t* in, size_t n, uint8_t* out, size_t cap,
                                      size_t* out_len) {
    const hpk_tables* t = hpk_get_tables();
    if (!t) return HPK_E_INVAL;
    if (!out_len || (!in && n) || (!out && cap)) return HPK_E_INVAL;
    return hpk_cpu_encode(t, in, n, out, cap, out_len);
}

// ------------------------------------------------------------------------------------------
// host batch (thread-per-core over contiguous shards balanced by input bytes)

template <bool kEncode>
static int cpu_batch(const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                     const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int nthreads) {
    const hpk_tables* t = hpk_get_tables();
    if (!t) return HPK_E_INVAL;
    if (!in_off || !out_off || (n && (!out_len || !status))) return HPK_E_INVAL;
    for (uint32_t i = 0; i < n; ++i)
        if (in_off[i + 1] < in_off[i] || out_off[i + 1] < out_off[i]) return HPK_E_INVAL;
    if (n == 0) return HPK_E_OK;
    if ((in_off[n] && !in_blob) || (out_off[n] && !out_blob)) return HPK_E_INVAL;
    if (nthreads <= 0) {  // default: the cores, at most 16, and >= 2048 literals per thread (a thread's start
                          // costs more than decoding a few hundred short literals)
        nthreads = (int)std::thread::hardware_concurrency();
        if (nthreads > 16) nthreads = 16;
        if ((uint32_t)nthreads > n / 2048u + 1u) nthreads = (int)(n / 2048u + 1u);
    }
    if (nthreads < 1) nthreads = 1;
    if ((uint32_t)nthreads > n) nthreads = (int)n;
    auto work = [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; ++i) {
            size_t ol = 0;
            const size_t cap = out_off[i + 1] - out_off[i];
            int st;
            if (kEncode) {
                st = hpk_cpu_encode(t, in_blob + in_off[i], in_off[i + 1] - in_off[i], out_blob + out_off[i], cap, &ol);
                st = st ? HPK_OUTPUT_OVERFLOW : HPK_OK;
            } else {
                st = hpk_cpu_decode(t, in_blob + in_off[i], in_off[i + 1] - in_off[i], out_blob + out_off[i], cap, &ol);
            }
            out_len[i] = (uint32_t)ol;
            status[i] = (uint8_t)st;
        }
    };
    if (nthreads == 1) {
        work(0, n);
        return HPK_E_OK;
    }
    std::vector<std::thread> th;
    const uint64_t total = (uint64_t)in_off[n] - in_off[0];
    uint32_t start = 0;
    for (int k = 0; k < nthreads; ++k) {
        uint32_t end = n;
        if (k != nthreads - 1) {
            const uint64_t target = in_off[0] + total * (uint64_t)(k + 1) / (uint64_t)nthreads;
            end = start;
            while (end < n && in_off[end] < target) ++end;
        }
        th.emplace_back(work, start, end);
        start = end;
    }
    for (auto& x : th) x.join();
    return HPK_E_OK;
}

extern "C" int hpk_decode_batch_cpu(const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                                    const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int nthreads) {
    return cpu_batch<false>(in_blob, in_off, n, out_blob, out_off, out_len, status, nthreads);
}

extern "C" int hpk_encode_batch_cpu(const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                                    const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int nthreads) {
    return cpu_batch<true>(in_blob, in_off, n, out_blob, out_off, out_len, status, nthreads);
}
