/*
 * hpk_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of loona-hpack's Huffman path, used
 * as the parity checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Nothing in the product (loona_amd/, libhpk.so) links, loads or calls this file.
 *
 * Parity pinning: the reference is Rust (bearcove/loona @ 2025-05-09) and no Rust toolchain is
 * available, so it cannot be built (oracle/_ref stays empty). This restatement is pinned by the
 * reference's own vectors, extracted into tests/golden/ by tests/golden/make_golden.py:
 *   - huffman.rs unit KATs incl. every error variant   (huffman.rs:523-707)
 *   - RFC 7541 App. C Huffman literals                  (decoder.rs:1216-1402, 1450-1465)
 *   - the http2jp interop stories (decoded header lists) (fixtures/hpack/interop, decoder.rs:1661-1717)
 *   - the 257-entry (code, len) table itself            (huffman.rs:222-480)
 *
 * Structure follows the reference deliberately, so that timing it is a fair stand-in for
 * "loona-hpack's CPU decoder" (label: "ref-restated"):
 *   - oracle_decoder_new(): one two-level hash map  len -> (code -> symbol) built with 257
 *     inserts, keyed by SipHash-1-3 as Rust's std HashMap is   (huffman.rs:58-88)
 *   - built afresh for every literal, as decode_string does     (decoder.rs:148)
 *   - oracle_decode(): MSB-first bit iterator, after each bit probe the len map and then the
 *     code map; EOS -> EOSInString at once; at the end >7 residual bits -> PaddingTooLarge,
 *     residual != EOS MSBs -> InvalidPadding                    (huffman.rs:95-161, 171-220)
 *   - output pushed byte by byte into a growing buffer          (huffman.rs:98,118)
 * Encode has no reference function (encoder.rs:296-307 never sets the H bit); oracle_encode is
 * the RFC 7541 §5.2 canonical encoding, pinned by re-encoding the interop wire literals.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* The code: RFC 7541 Appendix B as 257 (code, length) pairs, rebuilt canonically from the
 * lengths (the code is canonical: ordered by (length, symbol)). Lengths as a 257-char string
 * over 'A'+len to keep this table independent of the product's copy. */
static const char ORACLE_LENS[] =
    "NX]]]]]]]Y_]]_]]]]]]]]_]]]]]]]]]" /* 0..31 */
    "GKKMNGILKKILIGGGFFFGGGGGGGHIPGMKNGHHHHHHHHHHHHHHHHHHHHHHIHINTNOG" /* 32..95 */
    "PFGFGFGGGFHHGGGFGHGFFGHHHHHPLON]" /* 96..127 */
    "UWUUWWWXWXXXXXYXYYWXYXXXXVWXWXXYWVUWWXXVXWWYVWXXVVWVXWXXUWWWXWWX" /* 128..191 */
    "[[UTWXWZ[[[\\\\[YZTV[\\\\[\\YVV[[]\\\\\\UYUVWVVXWWZZYY[X[\\[[\\\\\\\\\\]\\\\\\\\\\[" /* 192..255 */
    "_" /* 256 = EOS */;

typedef struct { uint32_t code; uint8_t len; } oracle_code;
static oracle_code ORACLE_TABLE[257];
static int oracle_table_ready = 0;
static pthread_once_t oracle_once = PTHREAD_ONCE_INIT;

static void oracle_init_table(void) {
    int n = 0;
    uint64_t c = 0;
    int prev = 0;
    for (int L = 1; L <= 30; ++L)
        for (int s = 0; s < 257; ++s) {
            int ls = ORACLE_LENS[s] - 'A';
            if (ls != L) continue;
            if (n) c = (c + 1) << (L - prev);
            prev = L;
            ORACLE_TABLE[s].code = (uint32_t)c;
            ORACLE_TABLE[s].len = (uint8_t)L;
            ++n;
        }
    oracle_table_ready = (n == 257 && c + 1 == (1ull << prev));
}

int oracle_table(uint32_t* codes, uint8_t* lens) {
    pthread_once(&oracle_once, oracle_init_table);
    for (int s = 0; s < 257; ++s) { codes[s] = ORACLE_TABLE[s].code; lens[s] = ORACLE_TABLE[s].len; }
    return oracle_table_ready ? 0 : -1;
}

/* ------------------------------------------------------------------------------------------ */
/* SipHash-1-3 (the keyed hash behind Rust's std::collections::HashMap) */
#define ROTL(x, b) (uint64_t)(((x) << (b)) | ((x) >> (64 - (b))))
#define SIPROUND                                                              \
    do {                                                                      \
        v0 += v1; v1 = ROTL(v1, 13); v1 ^= v0; v0 = ROTL(v0, 32);             \
        v2 += v3; v3 = ROTL(v3, 16); v3 ^= v2;                                \
        v0 += v3; v3 = ROTL(v3, 21); v3 ^= v0;                                \
        v2 += v1; v1 = ROTL(v1, 17); v1 ^= v2; v2 = ROTL(v2, 32);             \
    } while (0)

static uint64_t siphash13(uint64_t k0, uint64_t k1, const uint8_t* in, size_t len) {
    uint64_t v0 = 0x736f6d6570736575ULL ^ k0, v1 = 0x646f72616e646f6dULL ^ k1;
    uint64_t v2 = 0x6c7967656e657261ULL ^ k0, v3 = 0x7465646279746573ULL ^ k1;
    uint64_t b = ((uint64_t)len) << 56;
    size_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t m;
        memcpy(&m, in + i, 8);
        v3 ^= m; SIPROUND; v0 ^= m;
    }
    for (size_t j = 0; i + j < len; ++j) b |= ((uint64_t)in[i + j]) << (8 * j);
    v3 ^= b; SIPROUND; v0 ^= b;
    v2 ^= 0xff;
    SIPROUND; SIPROUND; SIPROUND;
    return v0 ^ v1 ^ v2 ^ v3;
}

/* Open-addressing map u32 -> i16 with power-of-two growth (load <= 7/8), like hashbrown. */
typedef struct { uint32_t* keys; int16_t* vals; uint8_t* used; uint32_t cap, len; uint64_t k0, k1; } omap;

static uint64_t omap_hash(const omap* m, uint32_t key, int keybytes) {
    uint8_t b[4];
    memcpy(b, &key, 4);
    return siphash13(m->k0, m->k1, b, (size_t)keybytes);
}
static void omap_init(omap* m, uint64_t k0, uint64_t k1) {
    memset(m, 0, sizeof(*m));
    m->k0 = k0; m->k1 = k1;
}
static void omap_free(omap* m) { free(m->keys); free(m->vals); free(m->used); }
static void omap_insert(omap* m, uint32_t key, int16_t val, int keybytes);
static void omap_grow(omap* m, int keybytes) {
    omap old = *m;
    m->cap = old.cap ? old.cap * 2 : 4;
    m->len = 0;
    m->keys = (uint32_t*)calloc(m->cap, 4);
    m->vals = (int16_t*)calloc(m->cap, 2);
    m->used = (uint8_t*)calloc(m->cap, 1);
    for (uint32_t i = 0; i < old.cap; ++i)
        if (old.used[i]) omap_insert(m, old.keys[i], old.vals[i], keybytes);
    omap_free(&old);
}
static void omap_insert(omap* m, uint32_t key, int16_t val, int keybytes) {
    if ((m->len + 1) * 8 > m->cap * 7) omap_grow(m, keybytes);
    uint32_t i = (uint32_t)omap_hash(m, key, keybytes) & (m->cap - 1);
    while (m->used[i] && m->keys[i] != key) i = (i + 1) & (m->cap - 1);
    if (!m->used[i]) { m->used[i] = 1; m->keys[i] = key; ++m->len; }
    m->vals[i] = val;
}
static const int16_t* omap_get(const omap* m, uint32_t key, int keybytes) {
    if (!m->cap) return NULL;
    uint32_t i = (uint32_t)omap_hash(m, key, keybytes) & (m->cap - 1);
    while (m->used[i]) {
        if (m->keys[i] == key) return &m->vals[i];
        i = (i + 1) & (m->cap - 1);
    }
    return NULL;
}

/* HuffmanDecoder { table: HashMap<u8, HashMap<u32, HuffmanCodeSymbol>>, eos_codepoint }.
 * The outer map stores an index into `inner`. */
typedef struct {
    omap outer;
    omap inner[32];
    int ninner;
    uint32_t eos_code;
    uint8_t eos_len;
} oracle_decoder;

static void oracle_decoder_new(oracle_decoder* d, uint64_t seed) {
    pthread_once(&oracle_once, oracle_init_table);
    /* std's RandomState: per-map keys; a per-thread counter stands in for the OS entropy */
    uint64_t k0 = 0x0123456789abcdefULL ^ seed, k1 = 0xfedcba9876543210ULL + seed;
    omap_init(&d->outer, k0, k1);
    d->ninner = 0;
    for (int s = 0; s < 257; ++s) {
        uint8_t L = ORACLE_TABLE[s].len;
        const int16_t* idx = omap_get(&d->outer, L, 1); /* decoder_table.entry(code_len).or_default() */
        int slot;
        if (!idx) {
            slot = d->ninner++;
            omap_init(&d->inner[slot], k0 + 1 + (uint64_t)slot, k1);
            omap_insert(&d->outer, L, (int16_t)slot, 1);
        } else {
            slot = *idx;
        }
        omap_insert(&d->inner[slot], ORACLE_TABLE[s].code, (int16_t)s, 4);
        if (s == 256) { d->eos_code = ORACLE_TABLE[s].code; d->eos_len = L; }
    }
}
static void oracle_decoder_free(oracle_decoder* d) {
    for (int i = 0; i < d->ninner; ++i) omap_free(&d->inner[i]);
    omap_free(&d->outer);
}

/* growing output buffer (Vec<u8> without reserve) */
typedef struct { uint8_t* p; size_t len, cap; } ovec;
static void ovec_push(ovec* v, uint8_t b) {
    if (v->len == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 8;
        v->p = (uint8_t*)realloc(v->p, v->cap);
    }
    v->p[v->len++] = b;
}

enum { O_OK = 0, O_PADDING_TOO_LARGE = 1, O_INVALID_PADDING = 2, O_EOS_IN_STRING = 3, O_OVERFLOW = 4 };

static int oracle_decode_with(oracle_decoder* d, const uint8_t* buf, size_t n, ovec* result) {
    uint32_t current = 0;
    uint8_t current_len = 0;
    /* BitIterator: bytes in order, bits MSB -> LSB (huffman.rs:171-220) */
    for (size_t i = 0; i < n; ++i) {
        for (int pos = 7; pos >= 0; --pos) {
            int bit = (buf[i] >> pos) & 1;
            current_len += 1;
            current <<= 1;
            if (bit) current |= 1;
            const int16_t* slot = omap_get(&d->outer, current_len, 1); /* contains_key + get */
            if (slot) {
                const int16_t* sym = omap_get(&d->inner[*slot], current, 4);
                if (sym) {
                    if (*sym == 256) return O_EOS_IN_STRING;
                    ovec_push(result, (uint8_t)*sym);
                    current = 0;
                    current_len = 0;
                }
            }
        }
    }
    if (current_len > 7) return O_PADDING_TOO_LARGE;
    uint32_t right_align_current = current_len == 0 ? 0 : current << (32 - current_len);
    uint32_t right_align_eos = d->eos_code << (32 - d->eos_len);
    uint32_t mask = current_len == 0 ? 0 : ((1u << current_len) - 1) << (32 - current_len);
    if ((right_align_eos & mask) != right_align_current) return O_INVALID_PADDING;
    return O_OK;
}

static __thread uint64_t oracle_seed = 1;

/* One literal, exactly as decode_string does it: a fresh decoder per call. Returns the status;
 * *out_len = bytes decoded before returning (the symbols pushed so far, also on error). */
int oracle_decode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    oracle_decoder d;
    oracle_decoder_new(&d, oracle_seed++);
    ovec v = {0, 0, 0};
    int st = oracle_decode_with(&d, in, n, &v);
    oracle_decoder_free(&d);
    size_t k = v.len < cap ? v.len : cap;
    if (k) memcpy(out, v.p, k);
    *out_len = k;
    free(v.p);
    if (v.len > cap) return O_OVERFLOW;
    return st;
}

/* RFC 7541 §5.2: concatenate the codes MSB-first; pad the last octet with the most significant
 * bits of EOS (all ones). Returns 0, or -2 if cap is too small. */
int oracle_encode(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
    pthread_once(&oracle_once, oracle_init_table);
    uint64_t acc = 0;
    int nb = 0;
    size_t o = 0;
    for (size_t i = 0; i < n; ++i) {
        const oracle_code* c = &ORACLE_TABLE[in[i]];
        acc = (acc << c->len) | c->code;
        nb += c->len;
        while (nb >= 8) {
            if (o >= cap) return -2;
            out[o++] = (uint8_t)(acc >> (nb - 8));
            nb -= 8;
        }
    }
    if (nb) {
        if (o >= cap) return -2;
        out[o++] = (uint8_t)((acc << (8 - nb)) | (0xFFu >> nb));
    }
    *out_len = o;
    return 0;
}

/* decode_integer (decoder.rs:67-125): N-bit prefix varint, at most 5 octets.
 * Returns 0 ok, 1 InvalidPrefix, 2 NotEnoughOctets, 3 TooManyOctets. */
int oracle_decode_integer(const uint8_t* buf, size_t n, int prefix, uint64_t* value, size_t* consumed) {
    if (prefix < 1 || prefix > 8) return 1;
    if (n == 0) return 2;
    uint8_t mask = prefix == 8 ? 0xFF : (uint8_t)((1u << prefix) - 1);
    uint64_t v = buf[0] & mask;
    if (v < mask) { *value = v; *consumed = 1; return 0; }
    size_t total = 1;
    int m = 0;
    for (size_t i = 1; i < n; ++i) {
        uint8_t b = buf[i];
        total += 1;
        v += (uint64_t)(b & 127) << m;
        m += 7;
        if (!(b & 128)) { *value = v; *consumed = total; return 0; }
        if (total == 5) return 3;
    }
    return 2;
}

/* ------------------------------------------------------------------------------------------ */
/* batch drivers (threads over contiguous literal shards; loona is thread-per-core) */
typedef struct {
    int encode;
    const uint8_t* in_blob; const uint32_t* in_off; uint32_t lo, hi;
    uint8_t* out_blob; const uint32_t* out_off; uint32_t* out_len; uint8_t* status;
} oracle_job;

static void* oracle_worker(void* arg) {
    oracle_job* j = (oracle_job*)arg;
    for (uint32_t i = j->lo; i < j->hi; ++i) {
        size_t ol = 0;
        const uint8_t* in = j->in_blob + j->in_off[i];
        size_t n = j->in_off[i + 1] - j->in_off[i];
        uint8_t* out = j->out_blob + j->out_off[i];
        size_t cap = j->out_off[i + 1] - j->out_off[i];
        int st;
        if (j->encode) {
            st = oracle_encode(in, n, out, cap, &ol);
            st = st ? O_OVERFLOW : O_OK;
        } else {
            st = oracle_decode(in, n, out, cap, &ol);
        }
        j->out_len[i] = (uint32_t)ol;
        j->status[i] = (uint8_t)st;
    }
    return NULL;
}

static void oracle_batch(int encode, const uint8_t* in_blob, const uint32_t* in_off, uint32_t n,
                         uint8_t* out_blob, const uint32_t* out_off, uint32_t* out_len, uint8_t* status,
                         int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    oracle_job jobs[256];
    /* balance by encoded bytes */
    uint64_t total = (uint64_t)in_off[n] - in_off[0];
    uint32_t start = 0;
    for (int t = 0; t < nthreads; ++t) {
        uint64_t target = in_off[0] + total * (uint64_t)(t + 1) / (uint64_t)nthreads;
        uint32_t end = start;
        if (t == nthreads - 1) end = n;
        else while (end < n && in_off[end] < target) ++end;
        jobs[t] = (oracle_job){encode, in_blob, in_off, start, end, out_blob, out_off, out_len, status};
        start = end;
    }
    if (nthreads == 1) { oracle_worker(&jobs[0]); return; }
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, oracle_worker, &jobs[t]);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void oracle_decode_batch(const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                         const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int nthreads) {
    oracle_batch(0, in_blob, in_off, n, out_blob, out_off, out_len, status, nthreads);
}

void oracle_encode_batch(const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                         const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int nthreads) {
    oracle_batch(1, in_blob, in_off, n, out_blob, out_off, out_len, status, nthreads);
}
