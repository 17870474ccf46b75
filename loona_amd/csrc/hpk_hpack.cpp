// hpk_hpack.cpp — two-pass HPACK header-block decoding around the batched Huffman kernel
// (SURVEY §8f-1). Host code: the C ABI's hpk_hdec_* entry points (include/hpk.h).
//
// Reference: hpack::Decoder, crates/loona-hpack/src/decoder.rs:257-555, with its header table
// (crates/loona-hpack/src/lib.rs:43-289). Huffman results never depend on dynamic-table state,
// so the work splits in three:
//   1. scan (per block): walk the field representations (decoder.rs:368-450) with decode_integer
//      (decoder.rs:67-125) and the string framing of decode_string (decoder.rs:135-163): record
//      every field and the byte span of every string; stop at the first integer / length error;
//   2. one Huffman batch for the H-bit strings of ALL blocks (device: hpk_decode_batch through a
//      context; or the library's CPU batch path when the caller passes no context);
//   3. apply (per block, in order per decoder): table lookups, insertions, size updates and the
//      emitted header list, reporting the FIRST error in field order exactly as the reference's
//      single pass would (index integer, then name string or name index, then value string;
//      Huffman status of a string where the reference would have decoded it).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <pthread.h>
#include <unordered_map>
#include <thread>
#include <string>
#include <vector>

#include "../../include/hpk.h"

int hpk_set_err_msg(const char* what, int code);  // hpk_ctx.hip: hpk_last_error's message
// hpk_ctx.hip: the context's page-locked host staging area, grown to at least `bytes` (grow-only)
int hpk_ctx_pinned(hpk_ctx* ctx, size_t bytes, void** p);
// hpk_ctx.hip: a trusted host batch whose chunks can be waited for one by one (not in the C ABI)
int hpk_decode_host_begin(hpk_ctx* c, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off, uint32_t n,
                          uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                          uint8_t* status, int* nchunks, uint32_t* cut);
int hpk_host_chunk_wait(hpk_ctx* c, int j);
int hpk_decode_host_end(hpk_ctx* c);
int hpk_ctx_max_chunks();

namespace {

// RFC 7541 Appendix A (the reference keeps it as STATIC_TABLE, crates/loona-hpack/src/lib.rs).
const char* const kStatic[61][2] = {
    {":authority", ""},
    {":method", "GET"},
    {":method", "POST"},
    {":path", "/"},
    {":path", "/index.html"},
    {":scheme", "http"},
    {":scheme", "https"},
    {":status", "200"},
    {":status", "204"},
    {":status", "206"},
    {":status", "304"},
    {":status", "400"},
    {":status", "404"},
    {":status", "500"},
    {"accept-charset", ""},
    {"accept-encoding", "gzip, deflate"},
    {"accept-language", ""},
    {"accept-ranges", ""},
    {"accept", ""},
    {"access-control-allow-origin", ""},
    {"age", ""},
    {"allow", ""},
    {"authorization", ""},
    {"cache-control", ""},
    {"content-disposition", ""},
    {"content-encoding", ""},
    {"content-language", ""},
    {"content-length", ""},
    {"content-location", ""},
    {"content-range", ""},
    {"content-type", ""},
    {"cookie", ""},
    {"date", ""},
    {"etag", ""},
    {"expect", ""},
    {"expires", ""},
    {"from", ""},
    {"host", ""},
    {"if-match", ""},
    {"if-modified-since", ""},
    {"if-none-match", ""},
    {"if-range", ""},
    {"if-unmodified-since", ""},
    {"last-modified", ""},
    {"link", ""},
    {"location", ""},
    {"max-forwards", ""},
    {"proxy-authenticate", ""},
    {"proxy-authorization", ""},
    {"range", ""},
    {"referer", ""},
    {"refresh", ""},
    {"retry-after", ""},
    {"server", ""},
    {"set-cookie", ""},
    {"strict-transport-security", ""},
    {"transfer-encoding", ""},
    {"user-agent", ""},
    {"vary", ""},
    {"via", ""},
    {"www-authenticate", ""},
};

uint32_t static_len(int i, int part) {  // strlen of kStatic[i][part], computed once
    static const auto lens = [] {
        std::vector<uint32_t> v(122);
        for (int k = 0; k < 61; ++k) {
            v[2 * k] = (uint32_t)strlen(kStatic[k][0]);
            v[2 * k + 1] = (uint32_t)strlen(kStatic[k][1]);
        }
        return v;
    }();
    return lens[2 * i + part];
}

// A fixed set of worker threads for the block calls' parallel passes (spawning 15 threads per
// pass cost more than a small pass). One call at a time uses it; a concurrent caller (loona's
// runtime threads each decode their own connections) spawns its own threads instead.
class Pool {
  public:
    static constexpr int kMax = 16;
    // fn(t) for t in [0, n): t = 0 on the calling thread
    void run(int n, const std::function<void(int)>& fn) {
        if (n <= 1) {
            fn(0);
            return;
        }
        std::unique_lock<std::mutex> busy(use_, std::try_to_lock);
        if (!busy.owns_lock()) {  // in use by another caller
            std::vector<std::thread> th;
            for (int t = 1; t < n; ++t) th.emplace_back(fn, t);
            fn(0);
            for (auto& x : th) x.join();
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            while ((int)th_.size() < kMax - 1) {
                const int id = (int)th_.size() + 1;
                th_.emplace_back([this, id] { work(id); });
            }
            job_ = &fn;
            n_ = n;
            pending_ = n - 1;
            ++gen_;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
        job_ = nullptr;
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& x : th_) x.join();
    }

  private:
    void work(int id) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (id >= n_) continue;
                job = job_;
            }
            (*job)(id);
            std::lock_guard<std::mutex> g(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::mutex use_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> th_;
    const std::function<void(int)>* job_ = nullptr;
    int n_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// One pool per process. After a fork the child inherits the parent's Pool object but none of its
// threads (run() would wait forever for them), and maybe a mutex some parent thread held: the
// pthread_atfork child handler forgets it (leaked, never destroyed: its std::thread handles are
// meaningless in the child) and the child's first call makes a fresh one.
static Pool* g_pool = nullptr;

Pool& pool() {
    static const bool registered = [] {
        pthread_atfork(nullptr, nullptr, [] { __atomic_store_n(&g_pool, (Pool*)nullptr, __ATOMIC_RELEASE); });
        return true;
    }();
    (void)registered;
    Pool* p = __atomic_load_n(&g_pool, __ATOMIC_ACQUIRE);
    if (p) return *p;
    Pool* fresh = new Pool();  // no threads until its first run()
    Pool* expect = nullptr;
    if (__atomic_compare_exchange_n(&g_pool, &expect, fresh, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return *fresh;
    delete fresh;  // another thread installed one first
    return *expect;
}

// decode_integer (decoder.rs:67-125): prefix 1..8, at most 5 octets.
int decode_integer(const uint8_t* p, size_t n, int prefix, uint64_t* value, size_t* consumed) {
    if (prefix < 1 || prefix > 8) return HPK_BLK_INT_INVALID_PREFIX;
    if (n == 0) return HPK_BLK_INT_NOT_ENOUGH_OCTETS;
    const uint32_t mask = prefix == 8 ? 0xFFu : ((1u << prefix) - 1u);
    uint64_t v = p[0] & mask;
    if (v < mask) {
        *value = v;
        *consumed = 1;
        return HPK_BLK_OK;
    }
    size_t total = 1;
    unsigned m = 0;
    for (size_t i = 1; i < n; ++i) {
        const uint8_t b = p[i];
        total += 1;
        v += (uint64_t)(b & 127u) << m;
        m += 7;
        if (!(b & 128u)) {
            *value = v;
            *consumed = total;
            return HPK_BLK_OK;
        }
        if (total == 5) return HPK_BLK_INT_TOO_MANY_OCTETS;
    }
    return HPK_BLK_INT_NOT_ENOUGH_OCTETS;
}

struct Str {
    uint32_t off;       // absolute offset of the string bytes in the blocks buffer
    uint32_t len;
    uint32_t lit : 31;  // index among its scan thread's Huffman strings (huff only; + that thread's base)
    uint32_t huff : 1;
    Str() : off(0), len(0), lit(0), huff(0) {}
};

enum Kind : uint8_t { kIndexed, kLitIncr, kSizeUpdate, kLitNever, kLitPlain };

// Stages of one field in the reference's order; a scan error is recorded with the stage at which
// the reference would have raised it.
enum Stage : uint8_t { kStIndex = 0, kStName = 1, kStValue = 2 };

struct Field {  // 32 bytes (40 until round 3): a batch's fields are written once by the scan and read once by
                // the apply
    uint32_t index = 0;  // header index / name index / new table size (decode_integer's <= 5 octets: < 2^29)
    Str name, value;
    int8_t err = HPK_BLK_OK;  // scan error in this field (the last field scanned)
    Kind kind = kIndexed;
    Stage err_stage = kStIndex;
};
static_assert(sizeof(Field) <= 32, "Field packing");

struct Scan {  // a block's fields: pools[pool][first .. first + n) (one field pool per host thread)
    uint32_t pool = 0, first = 0, n = 0;
    uint32_t lit_end = 0;  // its scan thread's Huffman strings so far, this block's included
};

// decode_string's framing (decoder.rs:135-163) without the Huffman step.
int scan_string(const uint8_t* base, size_t pos, size_t end, Str* s, size_t* consumed) {
    uint64_t len;
    size_t c;
    int e = decode_integer(base + pos, end - pos, 7, &len, &c);
    if (e) return e;
    if (c + len > end - pos) return HPK_BLK_STR_NOT_ENOUGH_OCTETS;
    s->off = (uint32_t)(pos + c);
    s->len = (uint32_t)len;
    s->huff = (base[pos] & 128u) ? 1u : 0u;
    *consumed = c + (size_t)len;
    return HPK_BLK_OK;
}

void scan_fields(const uint8_t* base, size_t begin, size_t end, std::vector<Field>* pool, std::vector<uint32_t>* hoff,
                 std::vector<uint32_t>* hlen);

void scan_block(const uint8_t* base, size_t begin, size_t end, uint32_t pool_id, std::vector<Field>* pool, Scan* out,
                std::vector<uint32_t>* hoff, std::vector<uint32_t>* hlen) {
    out->pool = pool_id;
    out->first = (uint32_t)pool->size();
    scan_fields(base, begin, end, pool, hoff, hlen);
    out->n = (uint32_t)pool->size() - out->first;
    out->lit_end = (uint32_t)hoff->size();
}

void scan_fields(const uint8_t* base, size_t begin, size_t end, std::vector<Field>* pool, std::vector<uint32_t>* hoff,
                 std::vector<uint32_t>* hlen) {
    size_t pos = begin;
    auto add_huff = [&](Str& s) {
        if (!s.huff) return;
        s.lit = (uint32_t)hoff->size();
        hoff->push_back(s.off);
        hlen->push_back(s.len);
    };
    while (pos < end) {
        Field f;
        const uint8_t b = base[pos];
        f.kind = (b & 128u) ? kIndexed : (b & 64u) ? kLitIncr : (b & 32u) ? kSizeUpdate : (b & 16u) ? kLitNever : kLitPlain;
        size_t c = 0;
        if (f.kind == kIndexed || f.kind == kSizeUpdate) {
            uint64_t v = 0;
            f.err = (int8_t)decode_integer(base + pos, end - pos, f.kind == kIndexed ? 7 : 5, &v, &c);
            f.index = (uint32_t)v;
            pool->push_back(f);
            if (f.err) return;
            pos += c;
            continue;
        }
        // decode_literal (decoder.rs:502-527)
        const int prefix = f.kind == kLitIncr ? 6 : 4;
        uint64_t v = 0;
        f.err = (int8_t)decode_integer(base + pos, end - pos, prefix, &v, &c);
        f.index = (uint32_t)v;
        if (f.err) {
            pool->push_back(f);
            return;
        }
        size_t at = pos + c;
        if (f.index == 0) {
            size_t cn;
            f.err = (int8_t)scan_string(base, at, end, &f.name, &cn);
            if (f.err) {
                f.err_stage = kStName;
                pool->push_back(f);
                return;
            }
            add_huff(f.name);
            at += cn;
        }
        size_t cv;
        f.err = (int8_t)scan_string(base, at, end, &f.value, &cv);
        if (f.err) {
            f.err_stage = kStValue;
            pool->push_back(f);
            return;
        }
        add_huff(f.value);
        at += cv;
        pool->push_back(f);
        pos = at;
    }
}

}  // namespace

// Decoder state: the dynamic table (lib.rs:43-164) and the SizeUpdate limit (decoder.rs:316-318).
// The table holds its entries' bytes in one buffer, appended at the end, and the entries (offset,
// name length, value length) in a ring, newest first: an insertion or eviction allocates nothing
// (the reference's VecDeque of owned strings allocates per entry). Evicted bytes are reclaimed by
// moving the live ones (at most max_size bytes) to the buffer's start when the end is reached.
struct hpk_hdec {
    struct Ent {
        uint32_t at, nl, vl;
    };
    std::vector<Ent> ring{std::vector<Ent>(64)};  // capacity a power of two
    uint32_t first = 0, count = 0;                // newest entry at ring[first]
    std::vector<uint8_t> bytes;
    size_t end = 0;                               // bytes[0, end): entries' names and values
    size_t size = 0;
    size_t max_size = 4096;
    bool has_max_allowed = false;
    size_t max_allowed = 0;

    const Ent& at(size_t di) const { return ring[(first + di) & (ring.size() - 1)]; }
    void pop_oldest() {
        const Ent& e = at(count - 1);
        size -= (size_t)e.nl + e.vl + 32;
        count -= 1;
        if (count == 0) end = 0;
    }
    void consolidate() {
        while (size > max_size) pop_oldest();
    }
    // add_header then consolidate (lib.rs:97-117): an entry larger than the limit empties the
    // table. n and v must not point into the table.
    void add(const uint8_t* n, size_t nl, const uint8_t* v, size_t vl) {
        const size_t sz = nl + vl + 32;
        if (sz > max_size) {
            count = 0;
            size = 0;
            end = 0;
            return;
        }
        while (size + sz > max_size) pop_oldest();
        if (end + nl + vl > bytes.size()) {
            const size_t lo = count ? at(count - 1).at : end;  // the oldest live byte
            if (lo) {
                memmove(bytes.data(), bytes.data() + lo, end - lo);
                for (uint32_t k = 0; k < count; ++k) ring[(first + k) & (ring.size() - 1)].at -= (uint32_t)lo;
                end -= lo;
            }
            if (end + nl + vl > bytes.size()) bytes.resize(std::max<size_t>(2 * (end + nl + vl), 8192));
        }
        if (count == ring.size()) {  // grow the ring, newest first at 0
            std::vector<Ent> r(2 * ring.size());
            for (uint32_t k = 0; k < count; ++k) r[k] = at(k);
            ring.swap(r);
            first = 0;
        }
        if (nl) memcpy(bytes.data() + end, n, nl);
        if (vl) memcpy(bytes.data() + end + nl, v, vl);
        first = (first - 1) & (uint32_t)(ring.size() - 1);
        ring[first] = Ent{(uint32_t)end, (uint32_t)nl, (uint32_t)vl};
        count += 1;
        end += nl + vl;
        size += sz;
    }
    // HeaderTable::get_from_table (lib.rs:228-255): 1-based, static then dynamic
    bool get(uint64_t index, const uint8_t** n, size_t* nl, const uint8_t** v, size_t* vl) const {
        if (index == 0) return false;
        const uint64_t ri = index - 1;
        if (ri < 61) {
            *n = (const uint8_t*)kStatic[ri][0];
            *nl = static_len((int)ri, 0);
            *v = (const uint8_t*)kStatic[ri][1];
            *vl = static_len((int)ri, 1);
            return true;
        }
        const uint64_t di = ri - 61;
        if (di >= count) return false;
        const Ent& e = at((size_t)di);
        *n = bytes.data() + e.at;
        *nl = e.nl;
        *v = bytes.data() + e.at + e.nl;
        *vl = e.vl;
        return true;
    }
};

extern "C" hpk_hdec* hpk_hdec_create(void) { return new (std::nothrow) hpk_hdec(); }

extern "C" void hpk_hdec_destroy(hpk_hdec* d) { delete d; }

extern "C" int hpk_hdec_set_max_table_size(hpk_hdec* d, size_t n) {
    if (!d) return HPK_E_INVAL;
    if (d->has_max_allowed && n > d->max_allowed) return HPK_E_INVAL;  // the reference asserts
    d->max_size = n;
    d->consolidate();
    return HPK_E_OK;
}

extern "C" int hpk_hdec_set_max_allowed_table_size(hpk_hdec* d, size_t n) {
    if (!d) return HPK_E_INVAL;
    d->has_max_allowed = true;
    d->max_allowed = n;
    return HPK_E_OK;
}

extern "C" int hpk_hdec_table_size(const hpk_hdec* d, size_t* size, size_t* entries, size_t* max_size) {
    if (!d) return HPK_E_INVAL;
    if (size) *size = d->size;
    if (entries) *entries = d->count;
    if (max_size) *max_size = d->max_size;
    return HPK_E_OK;
}

namespace {

// A thread's output: header bytes and header records appended with plain copies (the vectors' sizes
// are capacities; vector::insert per string cost a fifth of the apply pass).
struct Out {
    std::vector<uint8_t> arena;
    std::vector<hpk_header> headers;
    size_t an = 0, hn = 0;  // bytes / records in use
    void reset(size_t abytes, size_t nhdr) {
        an = hn = 0;
        if (arena.size() < abytes) arena.resize(abytes);
        if (headers.size() < nhdr) headers.resize(nhdr);
    }
};

inline uint32_t put(Out& o, const void* p, size_t n) {
    const uint32_t at = (uint32_t)o.an;
    if (o.an + n > o.arena.size()) o.arena.resize(std::max(2 * o.arena.size(), o.an + n + 4096));
    if (n) memcpy(o.arena.data() + o.an, p, n);
    o.an += n;
    return at;
}

inline void put_header(Out& o, const hpk_header& h) {
    if (o.hn == o.headers.size()) o.headers.resize(2 * o.headers.size() + 1024);
    o.headers[o.hn++] = h;
}

struct Huff {  // the Huffman batch's results (host memory: pageable vectors or the ctx's pinned area)
    const uint8_t* out;
    const uint32_t* oo;
    const uint32_t* len;
    const uint8_t* st;
    const uint32_t* lbase;  // batch index of each scan thread's first string
};

// Pass 3 for one block: the reference's single pass over the scanned fields.
void apply_block(hpk_hdec* d, const uint8_t* base, const Scan& sc, const std::vector<std::vector<Field>>& pools,
                 const Huff& h, Out& o, hpk_block_result* r) {
    const Field* fields = pools[sc.pool].data() + sc.first;
    const uint32_t lb = h.lbase[sc.pool];
    r->first_header = (uint32_t)o.hn;
    r->n_headers = 0;
    r->error = HPK_BLK_OK;
    r->detail = 0;
    auto fail = [&](int e, int detail) {
        r->error = e;
        r->detail = detail;
    };
    // string bytes: raw from the block, Huffman from the batch (status checked by the caller)
    auto str = [&](const Str& s, const uint8_t** p, size_t* n) {
        if (s.huff) {
            *p = h.out + h.oo[lb + s.lit];
            *n = h.len[lb + s.lit];
        } else {
            *p = base + s.off;
            *n = s.len;
        }
    };
    auto huff_err = [&](const Str& s) -> int { return s.huff ? h.st[lb + s.lit] : 0; };
    auto emit = [&](const uint8_t* n, size_t nl, const uint8_t* v, size_t vl) {  // -> the header's index
        hpk_header hd;
        hd.name_len = (uint32_t)nl;
        hd.name_off = put(o, n, nl);
        hd.value_len = (uint32_t)vl;
        hd.value_off = put(o, v, vl);
        put_header(o, hd);
        r->n_headers += 1;
        return hd;
    };
    bool last_was_size_update = false;
    for (size_t fi = 0; fi < sc.n; ++fi) {
        const Field& f = fields[fi];
        last_was_size_update = f.kind == kSizeUpdate;
        if (f.err && f.err_stage == kStIndex) return fail(f.err, 0);
        if (f.kind == kIndexed) {
            const uint8_t *n, *v;
            size_t nl, vl;
            if (!d->get(f.index, &n, &nl, &v, &vl)) return fail(HPK_BLK_HEADER_INDEX_OUT_OF_BOUNDS, 0);
            emit(n, nl, v, vl);
            continue;
        }
        if (f.kind == kSizeUpdate) {  // update_max_dynamic_size (decoder.rs:538-554)
            if (d->has_max_allowed && f.index > d->max_allowed) return fail(HPK_BLK_INVALID_MAX_DYNAMIC_SIZE, 0);
            d->max_size = (size_t)f.index;
            d->consolidate();
            continue;
        }
        // literal: name (literal string or table name), then value
        const uint8_t* np;
        size_t nl;
        if (f.index == 0) {
            if (f.err && f.err_stage == kStName) return fail(f.err, 0);
            if (int hs = huff_err(f.name)) return fail(HPK_BLK_STR_HUFFMAN, hs);
            str(f.name, &np, &nl);
        } else {
            const uint8_t* v;
            size_t vl;
            if (!d->get(f.index, &np, &nl, &v, &vl)) return fail(HPK_BLK_HEADER_INDEX_OUT_OF_BOUNDS, 0);
        }
        if (f.err && f.err_stage == kStValue) return fail(f.err, 0);
        if (int hs = huff_err(f.value)) return fail(HPK_BLK_STR_HUFFMAN, hs);
        const uint8_t* vp;
        size_t vl;
        str(f.value, &vp, &vl);
        const hpk_header hd = emit(np, nl, vp, vl);
        // the insertion reads the header's copies in the output (the table name it came from may be
        // evicted by the insertion itself)
        if (f.kind == kLitIncr)
            d->add(o.arena.data() + hd.name_off, nl, o.arena.data() + hd.value_off, vl);
    }
    if (last_was_size_update) fail(HPK_BLK_SIZE_UPDATE_AT_END, 0);
}

}  // namespace

namespace {
// The output buffers of the last freed hpk_blocks_out (hpk_blocks_out_free), handed to the next
// call that fits in them: the caller-owned results are large (tens of MB for a big batch), and a
// fresh malloc of that size is a fresh mapping whose every page faults on first write.
struct OutCache {
    std::mutex m;
    void* p[3] = {};
    size_t cap[3] = {};  // bytes
    void* take(int k, size_t bytes) {
        {
            std::lock_guard<std::mutex> g(m);
            if (p[k] && cap[k] >= bytes) {
                void* r = p[k];
                p[k] = nullptr;
                cap[k] = 0;
                return r;
            }
        }
        return malloc(bytes ? bytes : 1);
    }
    void give(int k, void* q, size_t bytes) {
        if (!q) return;
        std::lock_guard<std::mutex> g(m);
        if (!p[k] || bytes > cap[k]) {
            free(p[k]);
            p[k] = q;
            cap[k] = bytes;
        } else {
            free(q);
        }
    }
};
OutCache g_out_cache;  // [0] arena, [1] headers, [2] block results

// Scratch of hpk_hdec_decode_blocks, kept per calling thread (loona calls from its runtime
// threads; each keeps its own): steady-state calls reuse capacity instead of page-faulting
// fresh allocations in every pass.
struct BlockScratch {
    std::vector<Scan> scans;
    std::vector<std::vector<Field>> pools;
    std::vector<std::vector<uint32_t>> thoff, thlen;
    std::vector<uint32_t> lbase, in_off, out_off, len, abase, hbase;
    std::vector<uint64_t> tin, tout;
    std::vector<uint8_t> st, in, dec, owner;
    std::vector<Out> outs;
    std::vector<uint64_t> bwork;  // [thread][bucket] apply work (fields + 1 per block) seen by the scan
    std::vector<uint8_t> bthread;  // bucket -> apply thread
    std::vector<uint16_t> bkt;     // block -> its decoder's bucket
};

// Decoders go to apply threads through kBuckets hash buckets of their addresses; the buckets are
// placed on threads longest-first by the work the scan counted in them. (A plain hash of the
// address per thread left the busiest of 16 threads with 1.37-1.56x the mean on config 4, whose
// connections differ in size by two orders of magnitude.)
constexpr int kBucketBits = 9, kBuckets = 1 << kBucketBits;
inline uint32_t dec_bucket(const hpk_hdec* d) {
    return (uint32_t)((((uintptr_t)d >> 4) * 0x9E3779B97F4A7C15ull) >> (64 - kBucketBits));
}
thread_local BlockScratch t_scratch;
}  // namespace

// Timeline of a call with a device context: scan (threads) -> the batch assembled in the pinned
// area (threads) -> the batch's chunks copied in, decoded and copied out on the device while the
// threads apply the blocks whose strings are back (a thread waits for chunk j's results only when
// it reaches a block with a string in it), so the device time hides under the apply pass.
extern "C" int hpk_hdec_decode_blocks(hpk_ctx* ctx, hpk_hdec* const* decs, const uint8_t* blocks,
                                      const uint32_t* block_off, uint32_t nblocks, hpk_blocks_out* out) {
    if (!decs || !block_off || !out || (nblocks && block_off[nblocks] && !blocks)) return HPK_E_INVAL;
    memset(out, 0, sizeof *out);
    for (uint32_t b = 0; b < nblocks; ++b)
        if (!decs[b] || block_off[b + 1] < block_off[b]) return HPK_E_INVAL;
    // Host threads: blocks are independent in pass 1; in pass 3 a decoder's blocks stay on one
    // thread, in order (decoders are independent of each other). Per-thread outputs are joined
    // at the end (a block's headers stay contiguous; blocks need not be in order in the arrays).
    int nth = (int)std::thread::hardware_concurrency();
    if (const char* e = getenv("HPK_HDEC_THREADS")) nth = atoi(e);  // (for measurements)
    if (nth > Pool::kMax) nth = Pool::kMax;
    if (nth < 1) nth = 1;
    if ((uint32_t)nth > nblocks / 256u + 1u) nth = (int)(nblocks / 256u + 1u);
    auto parallel = [&](const std::function<void(int)>& fn) { pool().run(nth, fn); };
    static const bool timing = getenv("HPK_HDEC_TIMING") != nullptr;  // per-pass wall times to stderr
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t_0 = now();
    auto us = [&](std::chrono::steady_clock::time_point a) {
        return (long)std::chrono::duration_cast<std::chrono::microseconds>(now() - a).count();
    };
    // pass 1: scan every block, gather the Huffman strings (contiguous block ranges per thread)
    BlockScratch& W = t_scratch;
    std::vector<Scan>& scans = W.scans;
    scans.resize(nblocks);
    std::vector<std::vector<Field>>& pools = W.pools;
    std::vector<std::vector<uint32_t>>&thoff = W.thoff, &thlen = W.thlen;
    if ((int)pools.size() < nth) {
        pools.resize(nth);
        thoff.resize(nth);
        thlen.resize(nth);
        W.outs.resize(nth);
    }
    W.tin.assign(nth, 0);
    W.tout.assign(nth, 0);
    W.bwork.assign((size_t)nth * kBuckets, 0);
    W.bkt.resize(nblocks);
    // (scan ranges of equal block counts: ranges of equal bytes scanned slower on config 4)
    auto blk0 = [&](int t) { return (uint32_t)((uint64_t)nblocks * t / nth); };
    parallel([&](int t) {
        // the vectors are moved into locals while the thread appends: their headers sit next to
        // the other threads' in the scratch arrays (false sharing on every push_back otherwise)
        const size_t bytes = block_off[blk0(t + 1)] - block_off[blk0(t)];
        std::vector<Field> pool = std::move(pools[t]);
        std::vector<uint32_t> ho = std::move(thoff[t]), hl = std::move(thlen[t]);
        pool.clear();
        ho.clear();
        hl.clear();
        pool.reserve(bytes / 8 + 16);  // ~12 block bytes per field on the interop corpus
        ho.reserve(bytes / 8 + 16);
        hl.reserve(bytes / 8 + 16);
        uint64_t* const bw = W.bwork.data() + (size_t)t * kBuckets;
        for (uint32_t b = blk0(t); b < blk0(t + 1); ++b) {
            scan_block(blocks, block_off[b], block_off[b + 1], (uint32_t)t, &pool, &scans[b], &ho, &hl);
            const uint32_t k = dec_bucket(decs[b]);
            W.bkt[b] = (uint16_t)k;
            bw[k] += scans[b].n + 1u;
        }
        uint64_t ti = 0, to = 0;  // the thread's string bytes and their decoded bounds
        for (uint32_t x : hl) {
            ti += x;
            to += (hpk_decoded_bound(x) + 3) & ~(uint64_t)3;
        }
        W.tin[t] = ti;
        W.tout[t] = to;
        pools[t] = std::move(pool);
        thoff[t] = std::move(ho);
        thlen[t] = std::move(hl);
    });
    std::vector<uint32_t>& lbase = W.lbase;  // each thread's first index in the batch
    lbase.assign(nth + 1, 0);
    std::vector<uint64_t> ibase(nth + 1, 0), obase(nth + 1, 0);
    for (int t = 0; t < nth; ++t) {
        lbase[t + 1] = lbase[t] + (uint32_t)thoff[t].size();
        ibase[t + 1] = ibase[t] + W.tin[t];
        obase[t + 1] = obase[t] + W.tout[t];
    }
    const long us_scan = us(t_0);
    auto t_1 = now();
    // pass 2: one batch for all of them. With a device context the batch is staged in the context's
    // page-locked host area (hpk_ctx_pinned), so its copies are DMA transfers that overlap the kernel
    // chunk by chunk; pageable vectors made HIP bounce every byte through its own staging buffer.
    const uint32_t n = lbase[nth];
    const size_t tot = ibase[nth], otot = obase[nth];
    if (tot >= (1ull << 32) || otot >= (1ull << 32)) return HPK_E_INVAL;
    uint8_t *in, *dec, *st;
    uint32_t *in_off, *out_off, *len;
    const size_t in_b = (tot + 16 + 15) & ~(size_t)15, dec_b = (otot + 16 + 15) & ~(size_t)15;
    const size_t off_b = ((size_t)(n + 1) * 4 + 15) & ~(size_t)15;
    if (ctx) {
        uint8_t* base = nullptr;
        if (int rc = hpk_ctx_pinned(ctx, in_b + dec_b + 3 * off_b + n + 16, (void**)&base)) return rc;
        in = base;
        dec = in + in_b;
        in_off = (uint32_t*)(dec + dec_b);
        out_off = (uint32_t*)((uint8_t*)in_off + off_b);
        len = (uint32_t*)((uint8_t*)out_off + off_b);
        st = (uint8_t*)len + off_b;
    } else {
        W.in.resize(in_b);
        W.dec.resize(dec_b);
        W.in_off.resize(n + 1);
        W.out_off.resize(n + 1);
        W.len.resize(n ? n : 1);
        W.st.resize(n ? n : 1);
        in = W.in.data();
        dec = W.dec.data();
        in_off = W.in_off.data();
        out_off = W.out_off.data();
        len = W.len.data();
        st = W.st.data();
    }
    parallel([&](int t) {  // each thread's strings: offsets from its bases, bytes gathered
        uint64_t io = ibase[t], oo = obase[t];
        const uint32_t* ho = thoff[t].data();
        const uint32_t* hl = thlen[t].data();
        uint32_t* ino = in_off + lbase[t];
        uint32_t* ouo = out_off + lbase[t];
        for (size_t j = 0, m = thlen[t].size(); j < m; ++j) {
            ino[j] = (uint32_t)io;
            ouo[j] = (uint32_t)oo;
            memcpy(in + io, blocks + ho[j], hl[j]);
            io += hl[j];
            oo += (hpk_decoded_bound(hl[j]) + 3) & ~(uint64_t)3;
        }
    });
    in_off[n] = (uint32_t)tot;
    out_off[n] = (uint32_t)otot;
    int chunks = 0;
    std::vector<uint32_t> cut(ctx ? hpk_ctx_max_chunks() + 1 : 1, 0);
    if (n) {
        const int rc = ctx ? hpk_decode_host_begin(ctx, in, in_b, in_off, n, dec, dec_b, out_off, len, st, &chunks,
                                                   cut.data())
                           : hpk_decode_batch_cpu(in, in_off, n, dec, out_off, len, st, 0);
        if (rc) {
            if (ctx && chunks) (void)hpk_decode_host_end(ctx);
            return rc;
        }
    }
    const long us_batch = us(t_1);
    auto t_2 = now();
    // pass 3: apply; thread of a decoder = a hash of its address, its blocks in list order
    std::vector<Out>& outs = W.outs;
    for (int t = 0; t < nth; ++t)  // decoded headers take a few times the block bytes
        outs[t].reset(4 * (size_t)block_off[nblocks] / (size_t)nth + 4096, pools[t].size() + 16);
    // results go straight into the caller's malloc'd buffers (hpk_blocks_out_free)
    out->n_blocks = nblocks;
    out->blocks = (hpk_block_result*)g_out_cache.take(2, (size_t)nblocks * sizeof(hpk_block_result));
    if (!out->blocks) {
        if (chunks) (void)hpk_decode_host_end(ctx);
        return HPK_E_INVAL;
    }
    hpk_block_result* res = out->blocks;
    std::vector<uint8_t>& owner = W.owner;
    owner.resize(nblocks);
    {  // buckets to threads, heaviest first onto the least loaded thread
        uint64_t bsum[kBuckets];
        uint16_t order[kBuckets];
        for (int k = 0; k < kBuckets; ++k) {
            uint64_t x = 0;
            for (int t = 0; t < nth; ++t) x += W.bwork[(size_t)t * kBuckets + k];
            bsum[k] = x;
            order[k] = (uint16_t)k;
        }
        std::sort(order, order + kBuckets, [&](uint16_t x, uint16_t y) { return bsum[x] > bsum[y]; });
        uint64_t load[Pool::kMax] = {};
        W.bthread.resize(kBuckets);
        for (int i = 0; i < kBuckets; ++i) {
            int m = 0;
            for (int t = 1; t < nth; ++t)
                if (load[t] < load[m]) m = t;
            load[m] += bsum[order[i]];
            W.bthread[order[i]] = (uint8_t)m;
        }
    }

    const Huff h{dec, out_off, len, st, lbase.data()};
    std::vector<int> wait_rc(nth, 0);
    parallel([&](int t) {
        Out mine = std::move(outs[t]);  // (a local: no false sharing with the neighbours' headers)
        // this thread's blocks, in order; a block's fields and its Huffman strings are fetched a few
        // blocks ahead (a thread's blocks are scattered over the batch: every string would otherwise
        // be a cache miss on the critical path)
        std::vector<uint32_t> my;
        my.reserve(nblocks / nth + 64);
        const uint16_t* const bk = W.bkt.data();
        const uint8_t* const bt = W.bthread.data();
        for (uint32_t b = 0; b < nblocks; ++b)
            if (bt[bk[b]] == t) {
                my.push_back(b);
                owner[b] = (uint8_t)t;
            }
        auto fetch_fields = [&](uint32_t b) {
            const Field* f = pools[scans[b].pool].data() + scans[b].first;
            for (uint32_t k = 0; k < scans[b].n; k += 1) __builtin_prefetch(f + k);
        };
        auto fetch_strings = [&](uint32_t b) {
            const Field* f = pools[scans[b].pool].data() + scans[b].first;
            const uint32_t lb = lbase[scans[b].pool];
            for (uint32_t k = 0; k < scans[b].n; ++k) {
                if (f[k].name.huff) __builtin_prefetch(dec + out_off[lb + f[k].name.lit]);
                if (f[k].value.huff) __builtin_prefetch(dec + out_off[lb + f[k].value.lit]);
            }
        };
        int waited = 0;  // device chunks whose results this thread has waited for
        for (size_t i = 0; i < my.size() && !wait_rc[t]; ++i) {
            const uint32_t b = my[i];
            if (i + 4 < my.size()) fetch_fields(my[i + 4]);
            if (i + 2 < my.size()) fetch_strings(my[i + 2]);
            const uint32_t lit_end = lbase[scans[b].pool] + scans[b].lit_end;  // the block's strings end
            while (waited < chunks && cut[waited] < lit_end)
                if ((wait_rc[t] = hpk_host_chunk_wait(ctx, waited++))) break;
            if (!wait_rc[t]) apply_block(decs[b], blocks, scans[b], pools, h, mine, &res[b]);
        }
        outs[t] = std::move(mine);
    });
    int rc = chunks ? hpk_decode_host_end(ctx) : HPK_E_OK;
    for (int t = 0; t < nth && !rc; ++t) rc = wait_rc[t];
    if (rc) {  // a device failure: the decoders are left as far as the apply pass got
        g_out_cache.give(2, out->blocks, (size_t)nblocks * sizeof(hpk_block_result));
        memset(out, 0, sizeof *out);
        return rc;
    }
    const long us_apply = us(t_2);
    auto t_3 = now();
    // join the per-thread outputs into the caller's buffers
    std::vector<uint32_t>&abase = W.abase, &hbase = W.hbase;
    abase.assign(nth, 0);
    hbase.assign(nth, 0);
    size_t at = 0, ht = 0;
    for (int t = 0; t < nth; ++t) {
        abase[t] = (uint32_t)at;
        hbase[t] = (uint32_t)ht;
        at += outs[t].an;
        ht += outs[t].hn;
    }
    out->arena_len = at;
    out->n_headers = ht;
    out->arena = (uint8_t*)g_out_cache.take(0, at);
    out->headers = (hpk_header*)g_out_cache.take(1, ht * sizeof(hpk_header));
    if (at >= (1ull << 32) || !out->arena || !out->headers) {
        hpk_blocks_out_free(out);
        return HPK_E_INVAL;
    }
    parallel([&](int t) {
        if (outs[t].an) memcpy(out->arena + abase[t], outs[t].arena.data(), outs[t].an);
        for (size_t j = 0; j < outs[t].hn; ++j) {
            hpk_header hd = outs[t].headers[j];
            hd.name_off += abase[t];
            hd.value_off += abase[t];
            out->headers[hbase[t] + j] = hd;
        }
        for (uint32_t b = blk0(t); b < blk0(t + 1); ++b) res[b].first_header += hbase[owner[b]];
    });
    if (timing)
        fprintf(stderr, "hpk_hdec_decode_blocks: %d threads, scan %ld us, batch %s %ld us, apply %ld us, join %ld us\n",
                nth, us_scan, ctx ? "issue" : "cpu", us_batch, us_apply, us(t_3));
    return HPK_E_OK;
}

extern "C" void hpk_blocks_out_free(hpk_blocks_out* out) {
    if (!out) return;
    g_out_cache.give(0, out->arena, out->arena_len);
    g_out_cache.give(1, out->headers, out->n_headers * sizeof(hpk_header));
    g_out_cache.give(2, out->blocks, (size_t)out->n_blocks * sizeof(hpk_block_result));
    memset(out, 0, sizeof *out);
}

// ---------------------------------------------------------------------------------------------
// Encoder (the response path): hpack::Encoder, crates/loona-hpack/src/encoder.rs:172-335, with
// the H-bit rule as an option. The dynamic table is the reference's (lib.rs:43-164; the same
// eviction as hpk_hdec), the lookup its find_header (lib.rs:261-288): static then dynamic
// (newest first), the first full match, else the LAST name match.
struct hpk_henc {
    std::deque<std::pair<std::string, std::string>> table;  // front = newest
    size_t size = 0;
    size_t max_size = 4096;
    int huffman = 0;

    void consolidate() {
        while (size > max_size) {
            const auto& last = table.back();
            size -= last.first.size() + last.second.size() + 32;
            table.pop_back();
        }
    }
    void add(std::string n, std::string v) {
        size += n.size() + v.size() + 32;
        table.emplace_front(std::move(n), std::move(v));
        consolidate();
    }
    // 1-based index, 0 = no name match; *full = name and value matched
    size_t find(const uint8_t* n, size_t nl, const uint8_t* v, size_t vl, bool* full) const {
        size_t name_match = 0;
        for (size_t i = 0; i < 61; ++i) {
            const char* sn = kStatic[i][0];
            if (strlen(sn) == nl && !memcmp(sn, n, nl)) {
                const char* sv = kStatic[i][1];
                if (strlen(sv) == vl && !memcmp(sv, v, vl)) {
                    *full = true;
                    return i + 1;
                }
                name_match = i + 1;
            }
        }
        for (size_t j = 0; j < table.size(); ++j) {
            const auto& e = table[j];
            if (e.first.size() == nl && !memcmp(e.first.data(), n, nl)) {
                if (e.second.size() == vl && !memcmp(e.second.data(), v, vl)) {
                    *full = true;
                    return 62 + j;
                }
                name_match = 62 + j;
            }
        }
        *full = false;
        return name_match;
    }
};

namespace {

// encode_integer_into (encoder.rs:93-122)
void put_integer(std::vector<uint8_t>& o, size_t value, int prefix, uint8_t leading) {
    const size_t mask = prefix >= 8 ? 0xFFu : ((1u << prefix) - 1u);
    leading &= (uint8_t)~mask;
    if (value < mask) {
        o.push_back((uint8_t)(leading | value));
        return;
    }
    o.push_back((uint8_t)(leading | mask));
    value -= mask;
    while (value >= 128) {
        o.push_back((uint8_t)(value % 128 + 128));
        value /= 128;
    }
    o.push_back((uint8_t)value);
}

// encode_string_literal (encoder.rs:299-307); with huffman, the H-bit form when strictly shorter
void put_string(std::vector<uint8_t>& o, const uint8_t* s, size_t n, int huffman) {
    if (huffman && n) {
        const size_t hl = hpk_huffman_encoded_len(s, n);
        if (hl < n) {
            put_integer(o, hl, 7, 0x80);
            const size_t at = o.size();
            o.resize(at + hl);
            size_t got = 0;
            hpk_huffman_encode_one(s, n, o.data() + at, hl, &got);
            return;
        }
    }
    put_integer(o, n, 7, 0);
    o.insert(o.end(), s, s + n);
}

}  // namespace

extern "C" hpk_henc* hpk_henc_create(int huffman) {
    hpk_henc* e = new (std::nothrow) hpk_henc();
    if (e) e->huffman = huffman ? 1 : 0;
    return e;
}

extern "C" void hpk_henc_destroy(hpk_henc* e) { delete e; }

extern "C" int hpk_henc_set_max_table_size(hpk_henc* e, size_t n) {
    if (!e) return HPK_E_INVAL;
    e->max_size = n;
    e->consolidate();
    return HPK_E_OK;
}

extern "C" int hpk_henc_encode(hpk_henc* e, const uint8_t* fields, const uint32_t* field_off, size_t n, uint8_t* out,
                               size_t cap, size_t* out_len) {
    if (!e || !out_len || (n && !field_off) || (cap && !out)) return HPK_E_INVAL;
    for (size_t k = 0; k < 2 * n; ++k)
        if (field_off[k + 1] < field_off[k]) return HPK_E_INVAL;
    if (n && field_off[2 * n] > field_off[0] && !fields) return HPK_E_INVAL;
    // encode against a copy of the state; commit only when the block fits
    hpk_henc next = *e;
    std::vector<uint8_t> o;
    for (size_t j = 0; j < n; ++j) {
        const uint8_t* nm = fields + field_off[2 * j];
        const size_t nl = field_off[2 * j + 1] - field_off[2 * j];
        const uint8_t* v = fields + field_off[2 * j + 1];
        const size_t vl = field_off[2 * j + 2] - field_off[2 * j + 1];
        bool full = false;
        const size_t idx = next.find(nm, nl, v, vl, &full);
        if (idx == 0) {  // encode_literal with indexing (encoder.rs:279-291), then add_header
            o.push_back(0x40);
            put_string(o, nm, nl, next.huffman);
            put_string(o, v, vl, next.huffman);
            next.add(std::string((const char*)nm, nl), std::string((const char*)v, vl));
        } else if (!full) {  // encode_indexed_name, not indexed (encoder.rs:311-323)
            put_integer(o, idx, 4, 0x00);
            put_string(o, v, vl, next.huffman);
        } else {  // encode_indexed (encoder.rs:329-334)
            put_integer(o, idx, 7, 0x80);
        }
    }
    *out_len = o.size();
    if (o.size() > cap) return HPK_E_NOSPACE;
    if (!o.empty()) memcpy(out, o.data(), o.size());
    *e = std::move(next);
    return HPK_E_OK;
}

// Many response header blocks at once (the batched form of encoder.rs:210-234): the
// table logic runs per block on the host, in order per encoder (it never depends on how a string
// is coded); every string literal of every block whose encoder Huffman-codes is then encoded in
// ONE batch (hpk_encode_batch through ctx, or the library's CPU batch path), and each block is
// assembled with the H-bit form wherever it is strictly shorter — the same bytes as hpk_henc_encode
// block by block.
// Test hook (include/hpk.h): the next n Huffman batches made by hpk_henc_encode_blocks fail as a
// device error would, so tests can check that a failed call leaves every encoder as it was.
static thread_local int t_fail_batches = 0;
extern "C" void hpk_test_fail_batches(int n) { t_fail_batches = n > 0 ? n : 0; }

extern "C" int hpk_henc_encode_blocks(hpk_ctx* ctx, hpk_henc* const* encs, const uint8_t* fields,
                                      const uint32_t* field_off, const uint32_t* hdr_off, uint32_t nblocks,
                                      hpk_henc_out* out) {
    if (!encs || !hdr_off || !out) return HPK_E_INVAL;
    memset(out, 0, sizeof *out);
    const uint32_t nh = hdr_off[nblocks] - hdr_off[0];
    for (uint32_t b = 0; b < nblocks; ++b)
        if (!encs[b] || hdr_off[b + 1] < hdr_off[b]) return HPK_E_INVAL;
    if (nh && !field_off) return HPK_E_INVAL;
    for (uint32_t k = 2 * hdr_off[0]; k < 2 * hdr_off[nblocks]; ++k)
        if (field_off[k + 1] < field_off[k]) return HPK_E_INVAL;
    if (nh && field_off[2 * hdr_off[nblocks]] > field_off[2 * hdr_off[0]] && !fields) return HPK_E_INVAL;
    // Pass 1 runs against a working copy of each distinct encoder (hpk_henc_encode's `next = *e`);
    // the copies replace the encoders only once every block is assembled, so a call that fails in
    // the Huffman batch or the assembly leaves each dynamic table as it was and the peer's decoder
    // never sees an index to an entry whose header was not sent.
    std::unordered_map<hpk_henc*, size_t> slot;
    std::vector<hpk_henc> work;
    std::vector<size_t> wk(nblocks);
    for (uint32_t b = 0; b < nblocks; ++b) {
        auto it = slot.find(encs[b]);
        if (it == slot.end()) {
            it = slot.emplace(encs[b], work.size()).first;
            work.push_back(*encs[b]);
        }
        wk[b] = it->second;
    }
    // pass 1: representation of every header; strings to code are recorded as (field start, length)
    struct Op {
        uint32_t raw_at, raw_len;  // bytes already final (prefix integers) in `raw`
        uint32_t str;              // index into the string list, or UINT32_MAX
    };
    std::vector<uint8_t> raw;
    std::vector<Op> ops;
    std::vector<uint32_t> ops_off(nblocks + 1, 0);
    std::vector<uint32_t> s_at, s_len;  // string k = fields[s_at[k] .. + s_len[k])
    std::vector<uint8_t> s_huff;        // its encoder Huffman-codes
    for (uint32_t b = 0; b < nblocks; ++b) {
        hpk_henc& e = work[wk[b]];
        auto lit = [&](uint32_t at, uint32_t len) {
            ops.push_back(Op{(uint32_t)raw.size(), 0u, (uint32_t)s_at.size()});
            s_at.push_back(at);
            s_len.push_back(len);
            s_huff.push_back((uint8_t)(e.huffman && len));
        };
        for (uint32_t j = hdr_off[b]; j < hdr_off[b + 1]; ++j) {
            const uint32_t na = field_off[2 * j], nl = field_off[2 * j + 1] - na;
            const uint32_t va = field_off[2 * j + 1], vl = field_off[2 * j + 2] - va;
            const uint8_t* nm = fields + na;
            const uint8_t* v = fields + va;
            bool full = false;
            const size_t idx = e.find(nm, nl, v, vl, &full);
            const uint32_t r0 = (uint32_t)raw.size();
            if (idx == 0) {  // literal with incremental indexing (encoder.rs:279-291), then add_header
                raw.push_back(0x40);
                ops.push_back(Op{r0, 1u, UINT32_MAX});
                lit(na, nl);
                lit(va, vl);
                e.add(std::string((const char*)nm, nl), std::string((const char*)v, vl));
            } else if (!full) {  // indexed name, value not indexed (encoder.rs:311-323)
                put_integer(raw, idx, 4, 0x00);
                ops.push_back(Op{r0, (uint32_t)raw.size() - r0, UINT32_MAX});
                lit(va, vl);
            } else {  // indexed (encoder.rs:329-334)
                put_integer(raw, idx, 7, 0x80);
                ops.push_back(Op{r0, (uint32_t)raw.size() - r0, UINT32_MAX});
            }
        }
        ops_off[b + 1] = (uint32_t)ops.size();
    }
    // pass 2: one Huffman batch for the strings of Huffman-coding encoders (u32 offsets: the strings
    // and their encoded bounds must each fit below HPK_MAX_OFFSET)
    const uint32_t ns = (uint32_t)s_at.size();
    std::vector<uint32_t> bi(ns, UINT32_MAX);  // string -> batch index
    std::vector<uint32_t> in_off(1, 0), eo(1, 0);
    std::vector<uint8_t> in;
    uint64_t eo_sum = 0;
    for (uint32_t k = 0; k < ns; ++k) {
        if (!s_huff[k]) continue;
        bi[k] = (uint32_t)in_off.size() - 1;
        in.insert(in.end(), fields + s_at[k], fields + s_at[k] + s_len[k]);
        eo_sum += (hpk_encoded_bound(s_len[k]) + 3) & ~(uint64_t)3;
        if (in.size() > HPK_MAX_OFFSET || eo_sum > HPK_MAX_OFFSET)
            return hpk_set_err_msg("Huffman strings of one call exceed the u32 offset range", HPK_E_INVAL);
        in_off.push_back((uint32_t)in.size());
        eo.push_back((uint32_t)eo_sum);
    }
    const uint32_t nb = (uint32_t)in_off.size() - 1;
    std::vector<uint8_t> enc(eo.back() ? eo.back() : 1), est(nb ? nb : 1);
    std::vector<uint32_t> elen(nb ? nb : 1);
    if (nb) {
        if (in.empty()) in.push_back(0);
        int rc;
        if (t_fail_batches > 0) {
            --t_fail_batches;
            rc = hpk_set_err_msg("injected batch failure (hpk_test_fail_batches)", HPK_E_DEVICE);
        } else {
            rc = ctx ? hpk_encode_batch(ctx, in.data(), in.size(), in_off.data(), nb, enc.data(), enc.size(), eo.data(),
                                        elen.data(), est.data(), HPK_PTR_HOST)
                     : hpk_encode_batch_cpu(in.data(), in_off.data(), nb, enc.data(), eo.data(), elen.data(), est.data(),
                                            0);
        }
        if (rc) return rc;
    }
    // pass 3: assemble every block
    std::vector<uint8_t> o;
    o.reserve(raw.size() + in.size() + 16);
    std::vector<uint32_t> boff(nblocks + 1, 0);
    for (uint32_t b = 0; b < nblocks; ++b) {
        for (uint32_t q = ops_off[b]; q < ops_off[b + 1]; ++q) {
            const Op& op = ops[q];
            if (op.str == UINT32_MAX) {
                o.insert(o.end(), raw.begin() + op.raw_at, raw.begin() + op.raw_at + op.raw_len);
                continue;
            }
            const uint32_t k = op.str, n = s_len[k];
            const uint32_t i = bi[k];
            if (i != UINT32_MAX && est[i] == HPK_OK && elen[i] < n) {  // the H-bit form, strictly shorter
                put_integer(o, elen[i], 7, 0x80);
                o.insert(o.end(), enc.begin() + eo[i], enc.begin() + eo[i] + elen[i]);
            } else {
                put_integer(o, n, 7, 0);
                o.insert(o.end(), fields + s_at[k], fields + s_at[k] + n);
            }
        }
        if (o.size() >= (1ull << 32)) return hpk_set_err_msg("encoded blocks exceed 4 GiB", HPK_E_INVAL);
        boff[b + 1] = (uint32_t)o.size();
    }
    out->block_off = (uint32_t*)malloc((nblocks + 1) * sizeof(uint32_t));
    out->bytes = (uint8_t*)malloc(o.size() ? o.size() : 1);
    if (!out->block_off || !out->bytes) {
        hpk_henc_out_free(out);
        return HPK_E_INVAL;
    }
    memcpy(out->block_off, boff.data(), (nblocks + 1) * sizeof(uint32_t));
    if (!o.empty()) memcpy(out->bytes, o.data(), o.size());
    out->n_blocks = nblocks;
    out->len = o.size();
    // commit: every encoder takes its working copy's table
    for (const auto& kv : slot) *kv.first = std::move(work[kv.second]);
    return HPK_E_OK;
}

extern "C" void hpk_henc_out_free(hpk_henc_out* out) {
    if (!out) return;
    free(out->bytes);
    free(out->block_off);
    memset(out, 0, sizeof *out);
}
