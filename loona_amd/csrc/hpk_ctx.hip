// hpk_ctx.hip — device context and the batch entry points of the C ABI (include/hpk.h).
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include "hpk_device.h"

#define HPK_VERSION "hpk 0.37 gfx950 decode v37 (every batch: wave fills, each wave with its own LDS window and image, longest-first queue, slot end offsets by DPP, nontemporal window loads stopping at the chunk's last byte, nontemporal write-back; chunks by guided self-scheduling from 4M literals, fixed 96-literal chunks below; fills and long-literal phase: body steps with no fit tests while >= 29 bits are left, then checked tails (the long phase's at its refill points); long literals one lane each streaming from HBM after the fills, dense ranges listed longest-first; literals of >= 8 KiB by a whole workgroup in speculative pieces; compacted-output form: wave fills packed per workgroup from an LDS cursor into a bound layout made from the input offsets, each lane storing its two literals in unaligned 16-byte pieces; small-call mode: a persistent kernel behind a host-mapped doorbell); encode v5 (byte-balanced workgroup ranges, start map and DPP segmented scan, run accumulator, LDS image, live chunks only)"

static thread_local std::string t_last_error;

int hpk_set_err(const char* what, hipError_t e) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    t_last_error = buf;
    return HPK_E_DEVICE;
}

int hpk_set_err_msg(const char* what, int code) {
    t_last_error = what;
    return code;
}


extern "C" const char* hpk_version(void) { return HPK_VERSION; }

extern "C" const char* hpk_last_error(const hpk_ctx*) { return t_last_error.c_str(); }

extern "C" hpk_ctx* hpk_ctx_create(int device) {
    const hpk_tables* t = hpk_get_tables();
    if (!t) { hpk_set_err_msg("code table build failed", HPK_E_INVAL); return nullptr; }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) { hpk_set_err("hipGetDeviceCount", e); return nullptr; }
    if (device < 0 || device >= ndev) { hpk_set_err_msg("device index out of range", HPK_E_INVAL); return nullptr; }
    hpk_ctx* c = new hpk_ctx();
    c->device = device;
    auto fail = [&](const char* what, hipError_t err) {
        hpk_set_err(what, err);
        hpk_ctx_destroy(c);
        return (hpk_ctx*)nullptr;
    };
    if ((e = hipSetDevice(device)) != hipSuccess) return fail("hipSetDevice", e);
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return fail("hipGetDeviceProperties", e);
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        hpk_set_err_msg("libhpk kernels are built for gfx950 only", HPK_E_NODEVICE);
        delete c;
        return nullptr;
    }
    c->num_cu = prop.multiProcessorCount;
    if ((e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) != hipSuccess) return fail("hipStreamCreate", e);
    c->stream = c->own;
    if ((e = hipMalloc(&c->d_lut, sizeof(t->lut))) != hipSuccess) return fail("hipMalloc lut", e);
    if ((e = hipMemcpy(c->d_lut, t->lut, sizeof(t->lut), hipMemcpyHostToDevice)) != hipSuccess) return fail("upload lut", e);
    if ((e = hipMalloc(&c->d_lut2, sizeof(t->lut2))) != hipSuccess) return fail("hipMalloc lut2", e);
    if ((e = hipMemcpy(c->d_lut2, t->lut2, sizeof(t->lut2), hipMemcpyHostToDevice)) != hipSuccess)
        return fail("upload lut2", e);
    if ((e = hipMalloc(&c->d_lut3, sizeof(t->lut3))) != hipSuccess) return fail("hipMalloc lut3", e);
    if ((e = hipMemcpy(c->d_lut3, t->lut3, sizeof(t->lut3), hipMemcpyHostToDevice)) != hipSuccess)
        return fail("upload lut3", e);
    if ((e = hipMalloc(&c->d_lo, sizeof(t->lo))) != hipSuccess) return fail("hipMalloc lo", e);
    if ((e = hipMalloc(&c->d_t8, sizeof(t->t8))) != hipSuccess) return fail("hipMalloc t8", e);
    if ((e = hipMemcpy(c->d_t8, t->t8, sizeof(t->t8), hipMemcpyHostToDevice)) != hipSuccess) return fail("upload t8", e);
    if ((e = hipMalloc(&c->d_codes, 2 * 257 * sizeof(uint32_t))) != hipSuccess) return fail("hipMalloc codes", e);
    uint32_t packed[2 * 257];
    for (int s = 0; s < 257; ++s) {
        packed[s] = t->code[s];
        packed[257 + s] = t->len[s];
    }
    if ((e = hipMemcpy(c->d_lo, t->lo, sizeof(t->lo), hipMemcpyHostToDevice)) != hipSuccess) return fail("upload lo", e);
    if ((e = hipMemcpy(c->d_codes, packed, sizeof(packed), hipMemcpyHostToDevice)) != hipSuccess) return fail("upload codes", e);
    if ((e = hipHostMalloc((void**)&c->h_err, 64, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
        return fail("hipHostMalloc err flag", e);
    *c->h_err = 0;
    if ((e = hipHostGetDevicePointer((void**)&c->d_err, c->h_err, 0)) != hipSuccess) return fail("err flag pointer", e);
    return c;
}

// The long-literal list of a launch: one slot per stream (a stream's launches are ordered, so its
// slot is reused without a wait). Completion events are recorded only once a second stream has used
// the context (an event record per launch cost ~1 us of a ~23 us small call); from then on a slot
// taken over by another stream, or grown, waits for its last launch.
int hpk_long_list(hpk_ctx* c, uint32_t n, uint32_t** list, int* slot) {
    int j = -1;
    bool any = false;
    for (int k = 0; k < hpk_ctx::kLongSlots; ++k) {
        if (c->long_list[k] && c->long_stream[k] == c->stream) j = k;
        any |= c->long_list[k] != nullptr;
    }
    if (j < 0) {
        if (any && !c->long_multi) {  // a second stream: events from here on; the past is drained
            // once, here. (Recording an event on each earlier slot's stream would touch a handle the
            // caller may have destroyed since — a stream bound with hpk_ctx_set_stream, created and
            // destroyed by the caller: ADVICE r3.) Launches on a stream the context does not own always
            // record their slot's event (hpk_long_list_used), so the only slots without one were used on
            // the context's own stream: waiting for that stream drains them.
            // Only those slots' (absent) events are cleared: a slot used on another stream keeps its
            // recorded event, which the own-stream wait does not cover.
            c->long_multi = true;
            HIP_TRY(hipStreamSynchronize(c->own));
            for (int k = 0; k < hpk_ctx::kLongSlots; ++k)
                if (c->long_stream[k] == c->own) c->long_ev_set[k] = false;
        }
        j = 0;
        while (j < hpk_ctx::kLongSlots && c->long_list[j]) ++j;
        if (j == hpk_ctx::kLongSlots) {  // all taken: reuse the oldest once its last launch is done
            j = c->long_next;
            c->long_next = (j + 1) % hpk_ctx::kLongSlots;
            if (c->long_ev_set[j]) HIP_TRY(hipEventSynchronize(c->long_ev[j]));
        }
        c->long_stream[j] = c->stream;
    }
    if (c->long_multi && !c->long_ev[j]) HIP_TRY(hipEventCreateWithFlags(&c->long_ev[j], hipEventDisableTiming));
    if (c->long_list_cap[j] < (size_t)n || !c->long_list[j]) {  // grow: the old list may still be in use
        if (int rc = hpk_slot_drain(c, j)) return rc;
        (void)hipFree(c->long_list[j]);
        c->long_list[j] = nullptr;
        c->long_list_cap[j] = 0;
        const size_t cap = (size_t)n + (n >> 2) + 1024;
        HIP_TRY(hipMalloc(&c->long_list[j], cap * sizeof(uint32_t)));
        c->long_list_cap[j] = cap;
    }
    *list = c->long_list[j];
    *slot = j;
    return HPK_E_OK;
}

int hpk_slot_drain(hpk_ctx* c, int j) {
    if (c->long_ev_set[j])
        HIP_TRY(hipEventSynchronize(c->long_ev[j]));
    else if (c->long_list[j])  // a slot without an event was last used on the own stream (foreign
                               // streams always record theirs): wait for that stream, not the caller's
        HIP_TRY(hipStreamSynchronize(c->own));
    return HPK_E_OK;
}

int hpk_long_list_used(hpk_ctx* c, int slot) {
    if (!c->long_multi && c->stream == c->own) return HPK_E_OK;
    // a stream the context does not own always gets its event: the slot is then never waited on
    // through the stream handle, which the caller may destroy
    if (!c->long_ev[slot]) HIP_TRY(hipEventCreateWithFlags(&c->long_ev[slot], hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->long_ev[slot], c->stream));
    c->long_ev_set[slot] = true;
    return HPK_E_OK;
}

extern "C" void hpk_ctx_destroy(hpk_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hpk_persist_stop(c);
    if (c->sm_stream) (void)hipStreamDestroy(c->sm_stream);
    if (c->h_sm) (void)hipHostFree(c->h_sm);
    (void)hipFree(c->d_sm_dev);
    (void)hipStreamSynchronize(c->stream);
    (void)hipFree(c->d_lut);
    (void)hipFree(c->d_lut2);
    (void)hipFree(c->d_lut3);
    (void)hipFree(c->d_lo);
    (void)hipFree(c->d_t8);
    (void)hipFree(c->d_codes);
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_meta);
    (void)hipFree(c->d_st);
    if (c->h_err) (void)hipHostFree(c->h_err);
    if (c->h_pin) (void)hipHostFree(c->h_pin);
    for (int j = 0; j < hpk_ctx::kLongSlots; ++j) {
        if (c->long_ev_set[j]) (void)hipEventSynchronize(c->long_ev[j]);
        if (c->long_list[j]) (void)hipFree(c->long_list[j]);
        (void)hipFree(c->cp_bound[j]);
        (void)hipFree(c->cp_tmp[j]);
        (void)hipFree(c->cp_cursor[j]);
        if (c->long_ev[j]) (void)hipEventDestroy(c->long_ev[j]);
    }
    for (int j = 0; j < hpk_ctx::kMaxChunks; ++j) {
        if (c->ev_in[j]) (void)hipEventDestroy(c->ev_in[j]);
        if (c->ev_run[j]) (void)hipEventDestroy(c->ev_run[j]);
        if (c->ev_out[j]) (void)hipEventDestroy(c->ev_out[j]);
    }
    if (c->h2d) (void)hipStreamDestroy(c->h2d);
    if (c->d2h) (void)hipStreamDestroy(c->d2h);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

extern "C" int hpk_ctx_set_stream(hpk_ctx* c, void* s) {
    if (!c) return HPK_E_INVAL;
    if (s == HPK_STREAM_LEGACY)
        c->stream = (hipStream_t)0;
    else
        c->stream = s ? (hipStream_t)s : c->own;
    return HPK_E_OK;
}

extern "C" int hpk_host_register(void* ptr, size_t bytes) {
    if (!ptr || !bytes) return hpk_set_err_msg("null range", HPK_E_INVAL);
    HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return HPK_E_OK;
}

extern "C" int hpk_host_unregister(void* ptr) {
    if (!ptr) return hpk_set_err_msg("null pointer", HPK_E_INVAL);
    HIP_TRY(hipHostUnregister(ptr));
    return HPK_E_OK;
}

// The context's page-locked host staging area (grow-only): the block-level calls build their
// Huffman batch in it so the batch's copies DMA straight from it. Growing waits for the context's
// stream (the old area may still be the source or target of its copies).
int hpk_ctx_pinned(hpk_ctx* c, size_t bytes, void** p) {
    if (bytes > c->h_pin_cap) {
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->d2h) HIP_TRY(hipStreamSynchronize(c->d2h));
        if (c->h_pin) (void)hipHostFree(c->h_pin);
        c->h_pin = nullptr;
        c->h_pin_cap = 0;
        const size_t cap = bytes + bytes / 4 + (1u << 20);
        HIP_TRY(hipHostMalloc(&c->h_pin, cap, hipHostMallocDefault));
        c->h_pin_cap = cap;
    }
    *p = c->h_pin;
    return HPK_E_OK;
}

extern "C" int hpk_ctx_set_decode_kernel(hpk_ctx* c, int kind) {
    if (!c || kind < HPK_DECODE_AUTO || kind > HPK_DECODE_WAVE) return hpk_set_err_msg("bad decode kernel", HPK_E_INVAL);
    c->decode_kernel = kind;
    return HPK_E_OK;
}

extern "C" void* hpk_ctx_stream(hpk_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int hpk_ctx_set_small_mode(hpk_ctx* c, uint32_t max_literals, int workgroups, uint32_t idle_ms) {
    if (!c) return HPK_E_INVAL;
    HIP_TRY(hipSetDevice(c->device));
    if (max_literals == 0) {
        const int rc = hpk_persist_stop(c);
        c->sm_max = 0;
        return rc;
    }
    if (workgroups < 1 || workgroups > 16 || workgroups >= c->num_cu || idle_ms < 1 || idle_ms > 10000 ||
        max_literals > (uint32_t)workgroups * 256u * 64u)
        return hpk_set_err_msg("small mode: 1-16 workgroups, 1-10000 ms idle, at most 64 literals per lane", HPK_E_INVAL);
    if (!c->h_sm) {
        HIP_TRY(hipStreamCreateWithFlags(&c->sm_stream, hipStreamNonBlocking));
        HIP_TRY(hipHostMalloc(&c->h_sm, 256, hipHostMallocMapped | hipHostMallocCoherent));
        memset(c->h_sm, 0, 256);
        HIP_TRY(hipHostGetDevicePointer(&c->d_sm, c->h_sm, 0));
        HIP_TRY(hipMalloc(&c->d_sm_dev, 128));  // [0..4) counters, [4, 21) the request copy
    }
    if (c->sm_launched && (workgroups != c->sm_wgs || idle_ms != c->sm_idle_ms))
        if (int rc = hpk_persist_stop(c)) return rc;
    c->sm_max = max_literals;
    c->sm_wgs = workgroups;
    c->sm_idle_ms = idle_ms;
    return c->sm_launched ? HPK_E_OK : hpk_persist_start(c);
}

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

static int check_offsets(const uint32_t* off, uint32_t n, size_t cap) {
    for (uint32_t i = 0; i < n; ++i)
        if (off[i + 1] < off[i]) return hpk_set_err_msg("offsets must be non-decreasing", HPK_E_INVAL);
    if (off[n] > cap || off[n] > HPK_MAX_OFFSET) return hpk_set_err_msg("offsets pass the blob's capacity", HPK_E_INVAL);
    return HPK_E_OK;
}

// read and clear the sticky device error flag (the ctx stream must be synchronised)
static int take_err(hpk_ctx* c) {
    if (!__atomic_exchange_n(c->h_err, 0u, __ATOMIC_ACQ_REL)) return HPK_E_OK;
    return hpk_set_err_msg("a batch had non-monotone offsets or offsets past a blob's capacity (HPK_BAD_OFFSETS)",
                           HPK_E_INVAL);
}

extern "C" int hpk_ctx_check(hpk_ctx* c) {
    if (!c) return HPK_E_INVAL;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return take_err(c);
}

typedef int (*launch_fn)(hpk_ctx*, const hpk_batch&);

static uint32_t clamp_cap(size_t cap) { return cap > HPK_MAX_OFFSET ? HPK_MAX_OFFSET : (uint32_t)cap; }

// Host-pointer batches: stage, run and copy back, cut into up to kMaxChunks literal ranges balanced
// by encoded bytes; chunk j's copy-in (h2d stream), kernel (ctx stream) and copy-out (d2h stream)
// overlap with the neighbouring chunks' (PCIe is full duplex), and ev_out[j] marks its results in
// host memory. Offsets stay absolute, so every chunk is the same kernel on a sub-range of the
// scratch buffers. With pageable host memory HIP stages the copies itself and the overlap is small:
// register the arena (hpk_host_register). `trusted`: the offsets were made by the library itself
// (hpk_hdec_decode_blocks), monotone by construction, so the O(n) host checks are skipped.
static int queue_chunks(launch_fn fn, hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint8_t* out_blob,
                        const uint32_t* out_off, uint32_t* out_len, uint8_t* status, uint32_t n, size_t in_bytes,
                        size_t out_bytes, int chunks, const uint32_t* cut, uint32_t* d_in_off, uint32_t* d_out_off,
                        uint32_t* d_len);

static int host_begin(launch_fn fn, hpk_ctx* c, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off,
                      uint32_t n, uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                      uint8_t* status, bool trusted, int* nchunks, uint32_t* cut) {
    *nchunks = 0;
    if (!trusted && (check_offsets(in_off, n, in_cap) || check_offsets(out_off, n, out_cap))) return HPK_E_INVAL;
    if (n == 0) return HPK_E_OK;
    const size_t in_bytes = in_off[n], out_bytes = out_off[n];
    if ((in_bytes && !in_blob) || (out_bytes && !out_blob)) return hpk_set_err_msg("null blob", HPK_E_INVAL);
    int rc;
    if ((rc = grow((void**)&c->d_in, &c->d_in_cap, in_bytes + 16))) return rc;
    if ((rc = grow((void**)&c->d_out, &c->d_out_cap, out_bytes + 16))) return rc;
    if ((rc = grow((void**)&c->d_meta, &c->d_meta_cap, (3 * (size_t)n + 2) * 4))) return rc;
    if ((rc = grow((void**)&c->d_st, &c->d_st_cap, n))) return rc;
    uint32_t* d_in_off = c->d_meta;
    uint32_t* d_out_off = c->d_meta + (n + 1);
    uint32_t* d_len = c->d_meta + 2 * ((size_t)n + 1);
    if (!c->h2d) {
        HIP_TRY(hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking));
        HIP_TRY(hipStreamCreateWithFlags(&c->d2h, hipStreamNonBlocking));
        for (int j = 0; j < hpk_ctx::kMaxChunks; ++j) {
            HIP_TRY(hipEventCreateWithFlags(&c->ev_in[j], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&c->ev_run[j], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&c->ev_out[j], hipEventDisableTiming));
        }
    }
    const size_t kChunkBytes = (size_t)4 << 20;
    int chunks = (int)((in_bytes + out_bytes) / kChunkBytes);
    chunks = chunks < 1 ? 1 : (chunks > hpk_ctx::kMaxChunks ? hpk_ctx::kMaxChunks : chunks);
    if ((uint32_t)chunks > n) chunks = (int)n;
    cut[0] = 0;
    for (int j = 1; j < chunks; ++j) {  // first literal whose end passes j/chunks of the bytes
        const uint64_t target = (uint64_t)in_bytes * j / chunks;
        uint32_t lo = cut[j - 1], hi = n;
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (in_off[mid + 1] < target) lo = mid + 1; else hi = mid;
        }
        cut[j] = lo;
    }
    cut[chunks] = n;
    // A failure after some chunk's copies were queued leaves DMA into and out of the caller's buffers
    // (and the pinned staging area the block decoder reuses) in flight: drain the three streams before
    // returning, so nothing lands after the call has returned.
    auto drain = [&](int rc) {
        (void)hipStreamSynchronize(c->h2d);
        (void)hipStreamSynchronize(c->stream);
        (void)hipStreamSynchronize(c->d2h);
        return rc;
    };
    if (int e = queue_chunks(fn, c, in_blob, in_off, out_blob, out_off, out_len, status, n, in_bytes, out_bytes,
                             chunks, cut, d_in_off, d_out_off, d_len))
        return drain(e);
    *nchunks = chunks;
    return HPK_E_OK;
}

static int queue_chunks(launch_fn fn, hpk_ctx* c, const uint8_t* in_blob, const uint32_t* in_off, uint8_t* out_blob,
                        const uint32_t* out_off, uint32_t* out_len, uint8_t* status, uint32_t n, size_t in_bytes,
                        size_t out_bytes, int chunks, const uint32_t* cut, uint32_t* d_in_off, uint32_t* d_out_off,
                        uint32_t* d_len) {
    int rc;
    HIP_TRY(hipEventRecord(c->ev_run[0], c->stream));  // earlier work on the ctx stream first
    HIP_TRY(hipStreamWaitEvent(c->h2d, c->ev_run[0], 0));
    for (int j = 0; j < chunks; ++j) {
        const uint32_t a = cut[j], b = cut[j + 1];
        if (a < b) {
            const size_t ib = in_off[a], ie = in_off[b], ob = out_off[a], oe = out_off[b];
            if (ie > ib) HIP_TRY(hipMemcpyAsync(c->d_in + ib, in_blob + ib, ie - ib, hipMemcpyHostToDevice, c->h2d));
            HIP_TRY(hipMemcpyAsync(d_in_off + a, in_off + a, (b - a + 1) * 4ull, hipMemcpyHostToDevice, c->h2d));
            HIP_TRY(hipMemcpyAsync(d_out_off + a, out_off + a, (b - a + 1) * 4ull, hipMemcpyHostToDevice, c->h2d));
            HIP_TRY(hipEventRecord(c->ev_in[j], c->h2d));
            HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_in[j], 0));
            const hpk_batch bt{c->d_in, (uint32_t)in_bytes, d_in_off + a, b - a, c->d_out, (uint32_t)out_bytes,
                               d_out_off + a, d_len + a, c->d_st + a};
            if ((rc = fn(c, bt))) return rc;
            HIP_TRY(hipEventRecord(c->ev_run[j], c->stream));
            HIP_TRY(hipStreamWaitEvent(c->d2h, c->ev_run[j], 0));
            if (oe > ob) HIP_TRY(hipMemcpyAsync(out_blob + ob, c->d_out + ob, oe - ob, hipMemcpyDeviceToHost, c->d2h));
            HIP_TRY(hipMemcpyAsync(out_len + a, d_len + a, (b - a) * 4ull, hipMemcpyDeviceToHost, c->d2h));
            HIP_TRY(hipMemcpyAsync(status + a, c->d_st + a, b - a, hipMemcpyDeviceToHost, c->d2h));
        }
        HIP_TRY(hipEventRecord(c->ev_out[j], c->d2h));
    }
    return HPK_E_OK;
}

static int host_end(hpk_ctx* c) {
    HIP_TRY(hipStreamSynchronize(c->d2h));
    return take_err(c);
}

static int run_batch(launch_fn fn, hpk_ctx* c, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off,
                     uint32_t n, uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                     uint8_t* status, int flags) {
    if (!c || !in_off || !out_off || (n && (!out_len || !status))) return hpk_set_err_msg("null argument", HPK_E_INVAL);
    HIP_TRY(hipSetDevice(c->device));
    if (flags & HPK_PTR_DEVICE) {
        if (n == 0) return HPK_E_OK;
        if (!in_blob || !out_blob) return hpk_set_err_msg("null blob", HPK_E_INVAL);
        const hpk_batch b{in_blob, clamp_cap(in_cap), in_off, n, out_blob, clamp_cap(out_cap), out_off, out_len, status};
        if (fn == hpk_launch_decode && !(flags & HPK_ASYNC) && c->sm_max) {  // the small-call mode
            bool handled = false;
            if (int rc = hpk_persist_call(c, b, &handled)) return rc;
            if (handled) return HPK_E_OK;
        }
        int rc = fn(c, b);
        if (rc) return rc;
        if (!(flags & HPK_ASYNC)) {
            HIP_TRY(hipStreamSynchronize(c->stream));
            return take_err(c);
        }
        return HPK_E_OK;
    }
    int chunks;
    uint32_t cut[hpk_ctx::kMaxChunks + 1];
    if (int rc = host_begin(fn, c, in_blob, in_cap, in_off, n, out_blob, out_cap, out_off, out_len, status, false,
                            &chunks, cut))
        return rc;
    return chunks ? host_end(c) : HPK_E_OK;
}

// The block decoder's form (hpk_hpack.cpp): a trusted host batch started here, its chunks' results
// waited for one by one (so the caller applies chunk j's blocks while later chunks still decode),
// then finished. Not part of the C ABI.
int hpk_decode_host_begin(hpk_ctx* c, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off, uint32_t n,
                          uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                          uint8_t* status, int* nchunks, uint32_t* cut) {
    HIP_TRY(hipSetDevice(c->device));
    return host_begin(hpk_launch_decode, c, in_blob, in_cap, in_off, n, out_blob, out_cap, out_off, out_len, status,
                      true, nchunks, cut);
}

int hpk_host_chunk_wait(hpk_ctx* c, int j) {
    HIP_TRY(hipEventSynchronize(c->ev_out[j]));
    return HPK_E_OK;
}

int hpk_decode_host_end(hpk_ctx* c) { return host_end(c); }

int hpk_ctx_max_chunks() { return hpk_ctx::kMaxChunks; }

extern "C" int hpk_decode_batch(hpk_ctx* c, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off, uint32_t n,
                                uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                                uint8_t* status, int flags) {
    return run_batch(hpk_launch_decode, c, in_blob, in_cap, in_off, n, out_blob, out_cap, out_off, out_len, status,
                     flags);
}

// The compacted form (include/hpk.h). The kernels' images keep bound-sized regions (a literal's decoded
// length is known only once it is decoded). Wave-fill kernel (large batches): it makes the bound layout
// from in_off itself, each workgroup packing into its range's span, and writes out_off[n]. Workgroup-fill
// kernel: the bound layout made on the device by a scan of the literals' 4-rounded bounds, the output
// cursor zeroed, the kernel, then the cursor copied to out_off[n].
extern "C" int hpk_decode_batch_compact(hpk_ctx* c, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off,
                                        uint32_t n, uint8_t* out_blob, size_t out_cap, uint32_t* out_off,
                                        uint32_t* out_len, uint8_t* status, int flags) {
    if (!c || !in_off || !out_off || (n && (!out_len || !status))) return hpk_set_err_msg("null argument", HPK_E_INVAL);
    if (!(flags & HPK_PTR_DEVICE)) return hpk_set_err_msg("the compacted form takes device pointers only", HPK_E_INVAL);
    if (n >= 0x7FFFFFFFu) return hpk_set_err_msg("too many literals for the compacted form", HPK_E_INVAL);
    const uint64_t need = (uint64_t)hpk_decoded_bound(in_cap > HPK_MAX_OFFSET ? HPK_MAX_OFFSET : in_cap) + 4ull * n;
    if (need > HPK_MAX_OFFSET) return hpk_set_err_msg("the compacted form's output would pass 4 GiB", HPK_E_INVAL);
    if (out_cap < need) return hpk_set_err_msg("out_cap below hpk_decoded_bound(in_cap) + 4 n", HPK_E_INVAL);
    HIP_TRY(hipSetDevice(c->device));
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(out_off, 0, 4, c->stream));
    } else {
        if (!in_blob || !out_blob) return hpk_set_err_msg("null blob", HPK_E_INVAL);
        // the stream's slot (two calls on two streams must not share the cursor, the bound
        // layout or the scan's scratch), its buffers regrown only once its last launch has completed
        int rc, j;
        uint32_t* ll = nullptr;
        if ((rc = hpk_long_list(c, n, &ll, &j))) return rc;
        if (hpk_compact_wave(c, n)) {  // (the kernel makes its bound layout and writes out_off[n])
            const hpk_batch b{in_blob, clamp_cap(in_cap), in_off, n, out_blob, clamp_cap(out_cap), nullptr, out_len,
                              status};
            if ((rc = hpk_launch_decode_compact(c, b, out_off, ll, nullptr, true))) return rc;
            if ((rc = hpk_long_list_used(c, j))) return rc;
            if (!(flags & HPK_ASYNC)) {
                HIP_TRY(hipStreamSynchronize(c->stream));
                return take_err(c);
            }
            return HPK_E_OK;
        }
        size_t tmp = 0;
        if ((rc = hpk_bound_scan(c, in_off, n, nullptr, nullptr, &tmp))) return rc;
        if (c->cp_bound_cap[j] < ((size_t)n + 1) * 4 || c->cp_tmp_cap[j] < tmp || !c->cp_cursor[j]) {
            if ((rc = hpk_slot_drain(c, j))) return rc;
            if ((rc = grow((void**)&c->cp_bound[j], &c->cp_bound_cap[j], ((size_t)n + 1) * 4))) return rc;
            if ((rc = grow(&c->cp_tmp[j], &c->cp_tmp_cap[j], tmp))) return rc;
            if (!c->cp_cursor[j]) HIP_TRY(hipMalloc(&c->cp_cursor[j], 4));
        }
        tmp = c->cp_tmp_cap[j];
        if ((rc = hpk_bound_scan(c, in_off, n, c->cp_bound[j], c->cp_tmp[j], &tmp))) return rc;
        HIP_TRY(hipMemsetAsync(c->cp_cursor[j], 0, 4, c->stream));
        const hpk_batch b{in_blob, clamp_cap(in_cap), in_off, n, out_blob, clamp_cap(out_cap), c->cp_bound[j], out_len,
                          status};
        if ((rc = hpk_launch_decode_compact(c, b, out_off, ll, c->cp_cursor[j], false))) return rc;
        // the span written: the cursor
        HIP_TRY(hipMemcpyAsync(out_off + n, c->cp_cursor[j], 4, hipMemcpyDeviceToDevice, c->stream));
        if ((rc = hpk_long_list_used(c, j))) return rc;
    }
    if (!(flags & HPK_ASYNC)) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        return take_err(c);
    }
    return HPK_E_OK;
}

extern "C" int hpk_encode_batch(hpk_ctx* c, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off, uint32_t n,
                                uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                                uint8_t* status, int flags) {
    return run_batch(hpk_launch_encode, c, in_blob, in_cap, in_off, n, out_blob, out_cap, out_off, out_len, status,
                     flags);
}

// buffet's buffer arena (crates/buffet/src/bufpool/privatepool.rs:80-108): ONE anonymous mapping of
// num_bufs x buf_size bytes from which a thread's read buffers are carved; page-locked here (pin) so
// batches whose literal or frame bytes sit in it DMA without a staging copy.
struct hpk_arena {
    void* base;
    size_t len;
    int pinned;
};

extern "C" hpk_arena* hpk_arena_create(size_t num_bufs, size_t buf_size, int pin) {
    if (!num_bufs || !buf_size || num_bufs > ((size_t)1 << 40) / buf_size) {
        hpk_set_err_msg("bad arena size", HPK_E_INVAL);
        return nullptr;
    }
    const size_t len = num_bufs * buf_size;
    void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
        hpk_set_err_msg("mmap failed", HPK_E_INVAL);
        return nullptr;
    }
    hpk_arena* a = new hpk_arena{p, len, 0};
    if (pin) {
        const hipError_t e = hipHostRegister(p, len, hipHostRegisterDefault);
        if (e != hipSuccess) {
            hpk_set_err("hipHostRegister arena", e);
            munmap(p, len);
            delete a;
            return nullptr;
        }
        a->pinned = 1;
    }
    return a;
}

extern "C" void* hpk_arena_base(const hpk_arena* a) { return a ? a->base : nullptr; }
extern "C" size_t hpk_arena_len(const hpk_arena* a) { return a ? a->len : 0; }

extern "C" void hpk_arena_destroy(hpk_arena* a) {
    if (!a) return;
    if (a->pinned) (void)hipHostUnregister(a->base);
    munmap(a->base, a->len);
    delete a;
}
