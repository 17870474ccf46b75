// hpk_device.h — shared between the device translation units of libhpk (context, decode, encode).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/hpk.h"
#include "hpk_code.h"
#include "hpk_internal.h"

struct hpk_ctx {
    int device = 0;
    int num_cu = 256;
    int decode_kernel = HPK_DECODE_AUTO;  // hpk_ctx_set_decode_kernel
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    uint32_t* d_lut = nullptr;
    uint32_t* d_lut2 = nullptr;
    uint32_t* d_lut3 = nullptr;
    uint16_t* d_lo = nullptr;
    uint8_t* d_t8 = nullptr;
    uint32_t* d_codes = nullptr;  // [0,257) code, [257,514) length
    // grow-only scratch for HPK_PTR_HOST calls
    uint8_t* d_in = nullptr;
    size_t d_in_cap = 0;
    uint8_t* d_out = nullptr;
    size_t d_out_cap = 0;
    uint32_t* d_meta = nullptr;  // in_off | out_off | out_len
    size_t d_meta_cap = 0;
    uint8_t* d_st = nullptr;
    size_t d_st_cap = 0;
    // page-locked host staging for the block-level calls (hpk_ctx_pinned), grow-only
    void* h_pin = nullptr;
    size_t h_pin_cap = 0;
    // host-pointer pipeline: copy-in and copy-out streams + per-chunk events (created lazily)
    static constexpr int kMaxChunks = 8;
    hipStream_t h2d = nullptr;
    hipStream_t d2h = nullptr;
    hipEvent_t ev_in[kMaxChunks] = {};
    hipEvent_t ev_run[kMaxChunks] = {};
    hipEvent_t ev_out[kMaxChunks] = {};  // chunk j's results are in host memory
    // sticky error flag: host-mapped, written (plain store of 1) by a kernel that saw bad offsets
    uint32_t* h_err = nullptr;
    uint32_t* d_err = nullptr;
    // the long-literal list per stream (calls on different streams may overlap): one u32 per
    // literal of the batch, grow-only. A slot's event is recorded after the launch that used it; a
    // slot taken over from another stream (or grown) is reused only once that event has completed,
    // whatever became of the stream that recorded it.
    static constexpr int kLongSlots = 8;
    hipStream_t long_stream[kLongSlots] = {};
    hipEvent_t long_ev[kLongSlots] = {};
    bool long_ev_set[kLongSlots] = {};
    uint32_t* long_list[kLongSlots] = {};
    size_t long_list_cap[kLongSlots] = {};
    int long_next = 0;
    bool long_multi = false;  // more than one stream has used the context: slots carry events
    // the compacted mode (hpk_decode_batch_compact): the fills' bound layout, the scan's scratch and the
    // output cursor, per slot like the long-literal list (two calls on two streams never share them),
    // grow-only
    uint32_t* cp_bound[kLongSlots] = {};
    size_t cp_bound_cap[kLongSlots] = {};
    void* cp_tmp[kLongSlots] = {};
    size_t cp_tmp_cap[kLongSlots] = {};
    uint32_t* cp_cursor[kLongSlots] = {};
    // the small-call mode (hpk_ctx_set_small_mode, hpk_persist.h): a persistent kernel of sm_wgs
    // workgroups on its own stream takes synchronous device-pointer batches of <= sm_max literals
    uint32_t sm_max = 0;
    int sm_wgs = 0;
    uint32_t sm_idle_ms = 0;
    hipStream_t sm_stream = nullptr;
    void* h_sm = nullptr;           // hpkdec::PersistCtl, coherent host memory
    void* d_sm = nullptr;           // its device-visible address
    uint32_t* d_sm_dev = nullptr;   // [0] workgroups finished, [1] command broadcast, [2] declined request
    uint32_t sm_req = 0;            // the last request issued
    bool sm_launched = false;       // a kernel was launched on sm_stream (it may have exited since)
    uint64_t sm_calls = 0;          // calls it answered (hpk_test_small_calls)
};

// The small-call mode (hpk_decode.hip): hpk_persist_call decodes a synchronous device-pointer batch through
// the persistent kernel if the mode is on, the batch small enough and the caller's stream idle (*handled);
// hpk_persist_stop ends the kernel and waits for it.
int hpk_persist_call(hpk_ctx* c, const struct hpk_batch& b, bool* handled);
int hpk_persist_start(hpk_ctx* c);
int hpk_persist_stop(hpk_ctx* c);

// The long-literal list for the context's current stream, sized for n literals (allocated on
// first use; HPK_E_OK or an error code); *slot is passed to hpk_long_list_used after the launch.
int hpk_long_list(hpk_ctx* c, uint32_t n, uint32_t** list, int* slot);
// Records the slot's event on the context's stream after the launch that reads the list.
int hpk_long_list_used(hpk_ctx* c, int slot);
// Waits until the slot's last launch has completed (before its buffers are freed or regrown).
int hpk_slot_drain(hpk_ctx* c, int slot);

// One batch call as the launchers see it: capacities clamped to HPK_MAX_OFFSET (offsets above
// them are bad whatever the buffer size).
struct hpk_batch {
    const uint8_t* in_blob;
    uint32_t in_cap;
    const uint32_t* in_off;
    uint32_t n;
    uint8_t* out_blob;
    uint32_t out_cap;
    const uint32_t* out_off;
    uint32_t* out_len;
    uint8_t* status;
};

int hpk_set_err(const char* what, hipError_t e);
int hpk_set_err_msg(const char* what, int code);

#define HIP_TRY(call)                                            \
    do {                                                         \
        hipError_t _e = (call);                                  \
        if (_e != hipSuccess) return hpk_set_err(#call, _e);     \
    } while (0)

int hpk_launch_decode(hpk_ctx* c, const hpk_batch& b);
// The compacted mode, co_off the caller's output offsets, long_list the slot's long-literal list (the
// caller took the slot with hpk_long_list and records it used after its last operation on the stream).
// wave (hpk_compact_wave): the wave-fill kernel, which makes its bound layout from in_off itself and
// writes co_off[n]; otherwise the workgroup-fill kernel, b.out_off the bound layout made by
// hpk_bound_scan and cursor the (zeroed) output cursor.
bool hpk_compact_wave(const hpk_ctx* c, uint32_t n);
int hpk_launch_decode_compact(hpk_ctx* c, const hpk_batch& b, uint32_t* co_off, uint32_t* long_list, uint32_t* cursor,
                              bool wave);
// out[i] = sum over j < i of the 4-rounded decoded bound of literal j (n + 1 entries), on the ctx
// stream; tmp == nullptr: *tmp_bytes = the scratch it needs.
int hpk_bound_scan(hpk_ctx* c, const uint32_t* in_off, uint32_t n, uint32_t* out, void* tmp, size_t* tmp_bytes);
int hpk_launch_encode(hpk_ctx* c, const hpk_batch& b);

__device__ __forceinline__ uint32_t hpk_bswap32(uint32_t x) { return __builtin_bswap32(x); }
