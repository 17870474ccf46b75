/*
 * hpk.h — C ABI of the MI355X-native HPACK Huffman codec (RFC 7541 §5.2 + App. B).
 *
 * This is the drop-in boundary for loona-hpack's Huffman string-literal path.
 * Every entry point is `extern "C"`, takes plain pointers and sizes, never
 * throws across the boundary and never panics on input bytes.
 *
 * Reference interfaces each entry point replaces (paths relative to
 * bearcove/loona @ 2025-05-09):
 *
 *   hpk_huffman_decode_one   HuffmanDecoder::new().decode(buf)
 *                            crates/loona-hpack/src/huffman.rs:86-88, :95-161
 *                            called from decode_string, crates/loona-hpack/src/decoder.rs:148-149
 *   hpk_status               HuffmanDecoderError {PaddingTooLarge, InvalidPadding, EOSInString}
 *                            crates/loona-hpack/src/huffman.rs:28-41 (1:1 mapping, 0 = Ok)
 *   hpk_decode_batch         many decode_string Huffman branches at once
 *                            (decoder.rs:143-157), literals gathered across header blocks /
 *                            streams by the caller (crates/loona/src/h2/server.rs:1619-1638)
 *   hpk_huffman_encode_one   NEW: the reference never Huffman-encodes
 *   hpk_encode_batch         (crates/loona-hpack/src/encoder.rs:296-307 writes raw literals);
 *                            this is the H-bit branch encode_string_literal would add.
 *
 * Threading: one hpk_ctx per host thread (loona is !Send, thread-per-core,
 * crates/buffet/src/lib.rs:38-49). A context owns a HIP stream (or borrows
 * one via hpk_ctx_set_stream) and grow-only device scratch buffers.
 */
#ifndef HPK_H
#define HPK_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-literal status (one byte per literal in batch calls) ---------- */
typedef enum hpk_status {
    HPK_OK = 0,                 /* Ok(Vec<u8>)                                 */
    HPK_PADDING_TOO_LARGE = 1,  /* HuffmanDecoderError::PaddingTooLarge  (>7 residual bits) */
    HPK_INVALID_PADDING = 2,    /* HuffmanDecoderError::InvalidPadding   (residual != EOS MSBs) */
    HPK_EOS_IN_STRING = 3,      /* HuffmanDecoderError::EOSInString      (30-bit EOS decoded) */
    HPK_OUTPUT_OVERFLOW = 4,    /* not a reference error: caller's out capacity < decoded size */
    HPK_BAD_OFFSETS = 5         /* not a reference error: device-pointer call whose offsets are not
                                   non-decreasing or pass a blob's capacity; the call's results are
                                   void (see hpk_decode_batch) */
} hpk_status;

/* ---- API return codes (negative = the call itself failed) -------------- */
#define HPK_E_OK 0
#define HPK_E_INVAL (-1)    /* bad argument (null pointer, offsets not monotone, ...) */
#define HPK_E_NOSPACE (-2)  /* single-literal call: `cap` too small               */
#define HPK_E_DEVICE (-3)   /* HIP runtime error; see hpk_last_error()            */
#define HPK_E_NODEVICE (-4) /* no GPU / kernel image for gfx950 not loadable      */

/* ---- flags for batch calls --------------------------------------------- */
#define HPK_PTR_HOST 0x0   /* all buffers are host memory: staged H2D / run / D2H in overlapping
                              chunks on the ctx's copy streams, synchronous                */
#define HPK_PTR_DEVICE 0x1 /* all buffers are device memory: enqueue on the ctx stream */
#define HPK_ASYNC 0x2      /* with HPK_PTR_DEVICE: return without synchronising       */

/* Upper bounds for output capacity. Every HPACK code is >= 5 bits and <= 30 bits. */
size_t hpk_decoded_bound(size_t encoded_len); /* floor(8n/5)    */
size_t hpk_encoded_bound(size_t decoded_len); /* ceil(30n/8)    */

/* Canonical Huffman encoded length of `in` (bytes, incl. EOS-prefix padding). */
size_t hpk_huffman_encoded_len(const uint8_t* in, size_t n);

/* ---- single-literal CPU entry points (the scalar drop-in) --------------- */
/* Decode n bytes. Returns an hpk_status (>= 0) and sets *out_len to the number
 * of bytes written (also on error: the symbols decoded before the error), or a
 * negative HPK_E_* code. `out` may be NULL iff cap == 0. */
int hpk_huffman_decode_one(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* Encode n bytes (MSB-first codes, padded with the most significant bits of
 * EOS). Returns HPK_E_OK or HPK_E_NOSPACE (then *out_len = cap and out holds the encoding's
 * first cap bytes, as the batch calls' HPK_OUTPUT_OVERFLOW). */
int hpk_huffman_encode_one(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len);

/* ---- device context ----------------------------------------------------- */
typedef struct hpk_ctx hpk_ctx;

hpk_ctx* hpk_ctx_create(int device);           /* NULL on failure (see hpk_last_error(NULL)) */
void hpk_ctx_destroy(hpk_ctx* ctx);
/* Run on `hip_stream`: NULL = the ctx's own (non-blocking) stream; HPK_STREAM_LEGACY = the
 * legacy null stream (stream 0, what torch's default stream is). */
#define HPK_STREAM_LEGACY ((void*)(intptr_t)-1)
int hpk_ctx_set_stream(hpk_ctx* ctx, void* hip_stream);
void* hpk_ctx_stream(hpk_ctx* ctx);
int hpk_ctx_sync(hpk_ctx* ctx);
const char* hpk_last_error(const hpk_ctx* ctx); /* thread-local text of the last failure */

/* ---- batch decode --------------------------------------------------------
 * Literal i occupies in_blob[in_off[i] .. in_off[i+1]) and may write
 * out_blob[out_off[i] .. out_off[i+1]) (its capacity; hpk_decoded_bound of
 * its length always suffices). On return out_len[i] = bytes decoded and
 * status[i] = hpk_status. Bytes of a literal's region past out_len[i] are
 * unspecified. Offsets are u32 (one shard): in_off/out_off have n+1 entries,
 * must be non-decreasing and at most HPK_MAX_OFFSET; in_cap / out_cap are the
 * byte sizes of in_blob / out_blob (the reference checks a literal's length
 * against its buffer before any Huffman work, decoder.rs:138-142).
 *
 * Host pointers: offsets and capacities are checked before anything is copied
 * (HPK_E_INVAL). Device pointers: the offsets live in device memory, so the
 * kernels check them as they read them: a literal whose offsets decrease or
 * pass a capacity makes the kernel write HPK_BAD_OFFSETS (out_len 0) for it and
 * for any other literals of the same batch it has not written yet, and nothing
 * is read or written outside [in_blob, in_blob + in_cap) and
 * [out_blob, out_blob + out_cap). The context keeps a sticky error flag: a
 * synchronous call returns HPK_E_INVAL when it is set (and clears it);
 * hpk_ctx_check() does the same after HPK_ASYNC calls. out_len and status
 * must have room for n entries. */
#define HPK_MAX_OFFSET 0xFFFFFFDFu /* offsets + a 16-byte misalignment + a 16-byte chunk stay < 2^32 */
int hpk_decode_batch(hpk_ctx* ctx, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off, uint32_t n,
                     uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                     uint8_t* status, int flags);

/* ---- batch decode, compacted output --------------------------------------
 * The reference returns each literal as an exact-length Vec (huffman.rs:98, 160); this form writes
 * each literal's decoded bytes exactly, in runs with no region slack between a run's literals, instead of
 * into bound-sized regions: on return literal i's bytes are out_blob[out_off[i] .. out_off[i] + out_len[i])
 * and out_off[n] is the end of the span written to. The span is NOT gap-free: see the layouts below
 * (listed literals keep their bound, and the wave-fill kernel's workgroup shares end in unwritten tails).
 * out_off (n+1 entries) is an OUTPUT here. Literals are packed in runs (a fill of the kernel at a
 * time, literal order inside a run, runs in completion order), so out_off is not monotone. A literal
 * the kernel hands to its long- or huge-literal phase keeps a region of its 4-rounded decoded bound,
 * the bytes past its out_len unwritten: every literal of >= 64 encoded bytes, and every literal
 * (short ones too) of a workgroup range the kernel lists whole because most of its input bytes are
 * in such literals. Batches the wave-fill kernel decodes (every batch unless the workgroup-fill kernel is
 * forced by hpk_ctx_set_decode_kernel) are packed per workgroup: workgroup w's runs and listed regions fill
 * its literal range [a, b)'s share [U(a), U(b)) from its start, the rest of the share unwritten, where
 * U(i) = floor(8 (in_off[i] - in_off[0]) / 5) + 4 i (it holds every 4-rounded decoded bound of the
 * range), and out_off[n] = U(n); the workgroup-fill kernel packs every run from one device cursor and
 * out_off[n] is its end.
 * Device pointers only (HPK_PTR_DEVICE, optionally HPK_ASYNC); out_cap must be at least
 * hpk_decoded_bound(in_cap) + 4 * n (HPK_E_INVAL otherwise). Statuses, errors and offsets checks
 * as hpk_decode_batch. */
int hpk_decode_batch_compact(hpk_ctx* ctx, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off,
                             uint32_t n, uint8_t* out_blob, size_t out_cap, uint32_t* out_off, uint32_t* out_len,
                             uint8_t* status, int flags);

/* ---- batch encode --------------------------------------------------------
 * Symmetric: literal i = in_blob[in_off[i] .. in_off[i+1]) is Huffman-encoded
 * into out_blob[out_off[i] ..) with capacity out_off[i+1]-out_off[i]
 * (hpk_encoded_bound suffices). out_len[i] = encoded bytes; status[i] is
 * HPK_OK or HPK_OUTPUT_OVERFLOW (out_len = the capacity, holding the
 * encoding's prefix). Offsets and capacities as hpk_decode_batch. */
int hpk_encode_batch(hpk_ctx* ctx, const uint8_t* in_blob, size_t in_cap, const uint32_t* in_off, uint32_t n,
                     uint8_t* out_blob, size_t out_cap, const uint32_t* out_off, uint32_t* out_len,
                     uint8_t* status, int flags);

/* Which decode kernel a context's batches use. All give identical results (the parity tests run
 * every case through each); they differ in speed. HPK_DECODE_AUTO (the default): the wave-fill kernel
 * for every batch (since round 6; it had been the workgroup-fill kernel below 4M literals). */
#define HPK_DECODE_AUTO 0
#define HPK_DECODE_FILL 1 /* workgroup fills: one fill at a time per CU, barriers between fills */
#define HPK_DECODE_WAVE 2 /* wave fills: every wave its own fills, no barriers between them */
int hpk_ctx_set_decode_kernel(hpk_ctx* ctx, int kind);

/* Small-call mode (opt-in; hpk_persist.h). A persistent kernel of `workgroups` (1-16) workgroups, its
 * decode tables resident in LDS, takes this context's synchronous device-pointer hpk_decode_batch
 * calls of 1..max_literals literals through a host-mapped doorbell (after the work already queued on
 * the context's stream): such a call skips the kernel launch and the stream synchronisation.
 * Results are identical to the launch path's (a batch with bad offsets is handed to the launch path).
 * While the kernel runs it holds `workgroups` CUs, which the context's batch kernels then leave out.
 * It exits after idle_ms (1-10000) without a call (the next small call starts it again), when the
 * mode is turned off (max_literals = 0) or when the context is destroyed. No counterpart in the
 * reference: loona decodes one connection's header block at a time (crates/loona/src/h2/server.rs:
 * 1619-1637), the granularity this mode serves. */
int hpk_ctx_set_small_mode(hpk_ctx* ctx, uint32_t max_literals, int workgroups, uint32_t idle_ms);

/* Read and clear the context's sticky device error flag (after HPK_ASYNC calls; synchronises the
 * ctx stream). Returns HPK_E_OK, HPK_E_INVAL (some call saw bad offsets) or HPK_E_DEVICE.
 * The flag belongs to the context, not to a stream: it reports a bad call made on any stream the
 * context was bound to (hpk_ctx_set_stream) once that call has run, so after async calls on
 * several streams synchronise each of them before relying on the answer; a synchronous call
 * returns (and clears) a flag left by an earlier async call on another stream. */
int hpk_ctx_check(hpk_ctx* ctx);

/* ---- batch calls on the host CPU ----------------------------------------
 * Same layout and results as the device calls, run by `nthreads` host threads over contiguous
 * literal shards balanced by bytes (thread-per-core, like loona). This is the table-driven CPU
 * path ("cpu-fast" in the bench), not the reference restatement. nthreads <= 0: the cores, at most
 * 16 and at least 2048 literals per thread. */
int hpk_decode_batch_cpu(const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                         const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int nthreads);
int hpk_encode_batch_cpu(const uint8_t* in_blob, const uint32_t* in_off, uint32_t n, uint8_t* out_blob,
                         const uint32_t* out_off, uint32_t* out_len, uint8_t* status, int nthreads);

/* ---- pinned host memory ---------------------------------------------------
 * Page-lock a host range (e.g. buffet's buffer arena, crates/buffet/src/bufpool/privatepool.rs:94-108)
 * so HPK_PTR_HOST batches inside it DMA directly and their copies overlap the kernels.
 * Returns HPK_E_OK or HPK_E_DEVICE. */
int hpk_host_register(void* ptr, size_t bytes);
int hpk_host_unregister(void* ptr);

/* buffet's buffer arena (crates/buffet/src/bufpool/privatepool.rs:80-108: one anonymous mmap of
 * num_bufs x buf_size, 64Ki x 4 KiB by default there), page-locked when pin != 0, so the frames
 * and literals read into its buffers DMA straight to the device. NULL on failure. */
typedef struct hpk_arena hpk_arena;
hpk_arena* hpk_arena_create(size_t num_bufs, size_t buf_size, int pin);
void* hpk_arena_base(const hpk_arena* arena);
size_t hpk_arena_len(const hpk_arena* arena);
void hpk_arena_destroy(hpk_arena* arena);

/* ---- HPACK header blocks: two-pass decode -----------------------------------------------
 * hpk_hdec mirrors hpack::Decoder (crates/loona-hpack/src/decoder.rs:257-555; header table
 * crates/loona-hpack/src/lib.rs:43-289): one per connection, holding the dynamic table.
 * hpk_hdec_decode_blocks decodes many header blocks at once — block b is
 * blocks[block_off[b] .. block_off[b+1]) for decoder decs[b]; the blocks of one decoder must be
 * in connection order — with every Huffman string of every block decoded in ONE batch: through
 * `ctx` on the GPU, or, when ctx is NULL, by the library's CPU batch path
 * (hpk_decode_batch_cpu). Per block the result equals Decoder::decode_with_cb on the same state:
 * the headers emitted before the first error, and that error with the reference's precedence
 * (decoder.rs:368-450). Results are returned in library-allocated buffers (hpk_blocks_out_free,
 * which keeps the largest freed buffers for the next call instead of returning them to the
 * allocator). With a context the device batch runs while the blocks whose strings are back are
 * applied: a device failure (HPK_E_DEVICE) mid-call leaves the decoders as far as the apply got,
 * and `out` empty. Host threads: up to 16, HPK_HDEC_THREADS overrides (measurements). */
typedef struct hpk_hdec hpk_hdec;

typedef enum hpk_block_error {   /* DecoderError (decoder.rs:237-253) and its nested kinds */
    HPK_BLK_OK = 0,
    HPK_BLK_HEADER_INDEX_OUT_OF_BOUNDS = 1,  /* HeaderIndexOutOfBounds                         */
    HPK_BLK_INT_TOO_MANY_OCTETS = 2,         /* IntegerDecodingError::TooManyOctets           */
    HPK_BLK_INT_VALUE_TOO_LARGE = 3,         /* IntegerDecodingError::ValueTooLarge (unused)  */
    HPK_BLK_INT_NOT_ENOUGH_OCTETS = 4,       /* IntegerDecodingError::NotEnoughOctets         */
    HPK_BLK_INT_INVALID_PREFIX = 5,          /* IntegerDecodingError::InvalidPrefix           */
    HPK_BLK_STR_NOT_ENOUGH_OCTETS = 6,       /* StringDecodingError::NotEnoughOctets          */
    HPK_BLK_STR_HUFFMAN = 7,                 /* StringDecodingError::HuffmanDecoderError(detail = hpk_status) */
    HPK_BLK_INVALID_MAX_DYNAMIC_SIZE = 8,    /* InvalidMaxDynamicSize                          */
    HPK_BLK_SIZE_UPDATE_AT_END = 9           /* SizeUpdateAtEnd                                */
} hpk_block_error;

typedef struct hpk_header {      /* one emitted (name, value), offsets into hpk_blocks_out.arena */
    uint32_t name_off, name_len, value_off, value_len;
} hpk_header;

typedef struct hpk_block_result {
    uint32_t first_header;       /* index into hpk_blocks_out.headers                         */
    uint32_t n_headers;          /* headers emitted (before the error, if any)               */
    int32_t error;               /* hpk_block_error                                           */
    int32_t detail;              /* hpk_status for HPK_BLK_STR_HUFFMAN, else 0                 */
} hpk_block_result;

typedef struct hpk_blocks_out {
    uint8_t* arena;
    size_t arena_len;
    hpk_header* headers;
    size_t n_headers;
    hpk_block_result* blocks;
    uint32_t n_blocks;
} hpk_blocks_out;

hpk_hdec* hpk_hdec_create(void);                                  /* Decoder::new(): max table 4096 */
void hpk_hdec_destroy(hpk_hdec* dec);
int hpk_hdec_set_max_table_size(hpk_hdec* dec, size_t max_size); /* decoder.rs:296-311 */
int hpk_hdec_set_max_allowed_table_size(hpk_hdec* dec, size_t max_allowed); /* decoder.rs:316-318 */
int hpk_hdec_table_size(const hpk_hdec* dec, size_t* size, size_t* entries, size_t* max_size);
int hpk_hdec_decode_blocks(hpk_ctx* ctx, hpk_hdec* const* decs, const uint8_t* blocks, const uint32_t* block_off,
                           uint32_t nblocks, hpk_blocks_out* out);
void hpk_blocks_out_free(hpk_blocks_out* out);

/* ---- HTTP/2 framing in front of the block decoder ------------------------
 * hpk_h2conn is one connection's header-reading state: its HPACK decoder and a HEADERS block still
 * waiting for CONTINUATION frames. hpk_h2_read_frames takes the bytes received on many
 * connections — connection c's are bytes[off[c] .. off[c+1]), whole frames (RFC 9113 §4.1:
 * 24-bit length, type, flags, 31-bit stream id) followed by at most one incomplete frame — and
 * does what the reference does per connection: the deframer's length check and padding removal
 * (crates/loona/src/h2/server.rs:290-390; Frame::parse crates/loona-h2/src/lib.rs:397-411), the
 * HEADERS priority block (server.rs:895-911), CONTINUATION gathering until END_HEADERS and the
 * concatenation (read_headers, server.rs:1349-1417, 1619-1638; flags lib.rs:139-168). Every
 * complete header block of every connection is then decoded by ONE hpk_hdec_decode_blocks call
 * (one Huffman batch through ctx, or the CPU path when ctx is NULL). Other frame types are
 * skipped. The first connection error stops the connection for this and all later calls (the
 * reference sends GOAWAY); an HPACK decoding error is HPK_H2_COMPRESSION_ERROR and the
 * connection's later blocks of the same call are marked skipped. */
typedef struct hpk_h2conn hpk_h2conn;

typedef enum hpk_h2_error {                   /* H2ConnectionError (crates/loona/src/h2/types.rs:300-370) */
    HPK_H2_OK = 0,
    HPK_H2_FRAME_TOO_LARGE = 1,               /* FrameTooLarge                 -> FRAME_SIZE_ERROR  */
    HPK_H2_PADDED_FRAME_EMPTY = 2,            /* PaddedFrameEmpty              -> FRAME_SIZE_ERROR  */
    HPK_H2_PADDED_FRAME_TOO_SHORT = 3,        /* PaddedFrameTooShort           -> PROTOCOL_ERROR    */
    HPK_H2_PRIORITY_PARSE = 4,                /* ReadAndParse(PrioritySpec)    -> PROTOCOL_ERROR    */
    HPK_H2_HEADERS_INVALID_PRIORITY = 5,      /* HeadersInvalidPriority        -> PROTOCOL_ERROR    */
    HPK_H2_EXPECTED_CONTINUATION_FRAME = 6,   /* ExpectedContinuationFrame     -> PROTOCOL_ERROR    */
    HPK_H2_EXPECTED_CONTINUATION_FOR_STREAM = 7, /* ExpectedContinuationForStream -> PROTOCOL_ERROR */
    HPK_H2_UNEXPECTED_CONTINUATION_FRAME = 8, /* UnexpectedContinuationFrame   -> PROTOCOL_ERROR    */
    HPK_H2_COMPRESSION_ERROR = 9              /* HpackDecodingError            -> COMPRESSION_ERROR */
} hpk_h2_error;

typedef struct hpk_h2_block {   /* one complete header block, in connection order */
    uint32_t conn;              /* index of its connection in the call                        */
    uint32_t stream_id;
    uint32_t end_stream;        /* the HEADERS frame's END_STREAM flag                        */
    uint32_t skipped;           /* 1: after a COMPRESSION_ERROR on its connection: not decoded */
} hpk_h2_block;

typedef struct hpk_h2_out {
    hpk_blocks_out hb;          /* hb.blocks[i] / headers of blocks[i] (hpk_hdec_decode_blocks) */
    hpk_h2_block* blocks;       /* hb.n_blocks entries                                          */
    int32_t* conn_error;        /* per connection: hpk_h2_error (sticky)                        */
    uint32_t* conn_consumed;    /* per connection: bytes of whole frames consumed (the rest is an
                                   incomplete frame: pass it again with more bytes)             */
    uint32_t n_conns;
} hpk_h2_out;

hpk_h2conn* hpk_h2conn_create(void);
void hpk_h2conn_destroy(hpk_h2conn* conn);
hpk_hdec* hpk_h2conn_decoder(hpk_h2conn* conn);                      /* its HPACK decoder */
int hpk_h2conn_set_max_frame_size(hpk_h2conn* conn, uint32_t max);  /* our SETTINGS_MAX_FRAME_SIZE */
int hpk_h2conn_error(const hpk_h2conn* conn);                       /* hpk_h2_error */
int hpk_h2_error_code(int h2_error);                                /* RFC 9113 §7 code for GOAWAY */
int hpk_h2_read_frames(hpk_ctx* ctx, hpk_h2conn* const* conns, const uint8_t* bytes, const uint32_t* off,
                       uint32_t nconn, hpk_h2_out* out);
void hpk_h2_out_free(hpk_h2_out* out);

/* ---- HPACK header blocks: encode (the response path) ----------------------
 * hpk_henc mirrors hpack::Encoder (crates/loona-hpack/src/encoder.rs:172-335): one per
 * connection, holding the dynamic table, with the reference's single strategy (a header found
 * whole in the table -> indexed; name found -> indexed name + literal value, not indexed; else a
 * literal name + value with incremental indexing). String literals (encoder.rs:299-307): with
 * huffman == 0 always raw, byte-identical to the reference; with huffman == 1 the H-bit form
 * (RFC 7541 §5.2) whenever its Huffman encoding is strictly shorter than the raw bytes. */
typedef struct hpk_henc hpk_henc;

hpk_henc* hpk_henc_create(int huffman);                           /* Encoder::new(): max table 4096 */
void hpk_henc_destroy(hpk_henc* enc);
int hpk_henc_set_max_table_size(hpk_henc* enc, size_t max_size); /* encoder.rs:193-197 */
/* Encoder::encode (encoder.rs:210-234) of n headers: header j's name is
 * fields[field_off[2j] .. field_off[2j+1]) and its value fields[field_off[2j+1] .. field_off[2j+2]).
 * Writes the block into out[0 .. cap) and its length to *out_len. Returns HPK_E_OK; HPK_E_NOSPACE
 * with *out_len = the size needed and the encoder state unchanged; HPK_E_INVAL on bad arguments. */
int hpk_henc_encode(hpk_henc* enc, const uint8_t* fields, const uint32_t* field_off, size_t n_headers, uint8_t* out,
                    size_t cap, size_t* out_len);

/* Many responses' header blocks at once: block b encodes headers [hdr_off[b], hdr_off[b+1]) (header j
 * as in hpk_henc_encode) with encoder encs[b]; the blocks of one encoder are encoded in list order.
 * The table logic runs on the host; every string literal of every Huffman-coding encoder goes
 * through ONE hpk_encode_batch on ctx (the CPU batch path when ctx is NULL), and the H-bit form is
 * used where strictly shorter: the bytes equal hpk_henc_encode's block by block. Results in
 * library-allocated buffers: block b is bytes[block_off[b] .. block_off[b+1]). */
typedef struct hpk_henc_out {
    uint8_t* bytes;
    size_t len;
    uint32_t* block_off;
    uint32_t n_blocks;
} hpk_henc_out;
int hpk_henc_encode_blocks(hpk_ctx* ctx, hpk_henc* const* encs, const uint8_t* fields, const uint32_t* field_off,
                           const uint32_t* hdr_off, uint32_t nblocks, hpk_henc_out* out);
void hpk_henc_out_free(hpk_henc_out* out);
/* A failed hpk_henc_encode_blocks (any negative return) leaves every encoder's dynamic table as it
 * was before the call, as a failed hpk_henc_encode does; the blocks are then not sent at all.
 * Testing only: the calling thread's next n Huffman batches inside hpk_henc_encode_blocks fail
 * with HPK_E_DEVICE (n = 0 clears it), so that guarantee can be checked without a device fault. */
void hpk_test_fail_batches(int n);
/* Testing only: the compacted form's internal bound layout of n literals' device offsets in_off
 * (n + 1 entries) into device memory out (n + 1 entries): the exclusive sum mod 2^32 of
 * (floor(8 len / 5) + 3) & ~3, synchronously on the context's stream. */
int hpk_test_bound_scan(hpk_ctx* ctx, const uint32_t* in_off, uint32_t n, uint32_t* out);
/* Testing only: how many decode calls of this context the small-call mode's persistent kernel has
 * answered (hpk_ctx_set_small_mode), so the tests can tell it ran. */
uint64_t hpk_test_small_calls(const hpk_ctx* ctx);
/* Testing only: the small-call mode's device stamps of its last request (100 MHz ticks): workgroup 0 saw
 * it, broadcast it, finished its literals; the last workgroup published it; then workgroup 0's shader-clock
 * cycles from the broadcast to its finish and the same interval in 100 MHz ticks; thread 0's first literal in
 * shader-clock cycles: offsets loaded, staged, walked, stored (10 values). */
int hpk_test_small_stamps(const hpk_ctx* ctx, uint32_t* out6);

/* Library/kernel identification (for logs and the bench JSON). */
const char* hpk_version(void);

#ifdef __cplusplus
}
#endif

#endif /* HPK_H */
