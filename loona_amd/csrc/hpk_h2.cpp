// hpk_h2.cpp — HTTP/2 frame layer in front of the two-pass HPACK decoder. Host code:
// the C ABI's hpk_h2_* entry points (include/hpk.h).
//
// The reference reads header blocks one connection and one stream at a time: its deframer
// (crates/loona/src/h2/server.rs:290-390) cuts frames (Frame::parse, crates/loona-h2/src/lib.rs:
// 397-411), drops the padding of DATA / HEADERS frames, the frame loop strips a HEADERS frame's
// priority block (server.rs:895-911), and read_headers (server.rs:1349-1643) gathers CONTINUATION
// fragments until END_HEADERS (lib.rs:139-168) and calls Decoder::decode_with_cb on the
// concatenation (server.rs:1619-1638). Here one call takes the bytes received on MANY connections,
// does the same framing per connection, and decodes every complete header block of every
// connection with ONE hpk_hdec_decode_blocks call: all their Huffman strings go to the device as one
// batch. A block whose CONTINUATION frames have not all arrived stays with its connection until a
// later call completes it; a connection error stops that connection, as the reference's connection
// task ends with GOAWAY.
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "../../include/hpk.h"

namespace {

enum : uint8_t { kData = 0x0, kHeaders = 0x1, kContinuation = 0x9 };
enum : uint8_t { kEndStream = 0x01, kEndHeaders = 0x04, kPadded = 0x08, kPriority = 0x20 };

uint32_t be24(const uint8_t* p) { return ((uint32_t)p[0] << 16) | ((uint32_t)p[1] << 8) | p[2]; }
uint32_t be31(const uint8_t* p) {
    return (((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]) & 0x7FFFFFFFu;
}

}  // namespace

struct hpk_h2conn {
    hpk_hdec* dec = nullptr;
    uint32_t max_frame_size = 16384;  // RFC 9113 §6.5.2 SETTINGS_MAX_FRAME_SIZE initial value
    // a HEADERS block still waiting for CONTINUATION frames (possibly across calls)
    bool pending = false;
    uint32_t pend_stream = 0;
    uint32_t pend_end_stream = 0;
    std::vector<uint8_t> frag;
    int32_t error = HPK_H2_OK;  // sticky: the reference's connection is gone after its first error
};

extern "C" hpk_h2conn* hpk_h2conn_create(void) {
    hpk_h2conn* c = new (std::nothrow) hpk_h2conn();
    if (!c) return nullptr;
    c->dec = hpk_hdec_create();
    if (!c->dec) {
        delete c;
        return nullptr;
    }
    return c;
}

extern "C" void hpk_h2conn_destroy(hpk_h2conn* c) {
    if (!c) return;
    hpk_hdec_destroy(c->dec);
    delete c;
}

extern "C" hpk_hdec* hpk_h2conn_decoder(hpk_h2conn* c) { return c ? c->dec : nullptr; }

extern "C" int hpk_h2conn_set_max_frame_size(hpk_h2conn* c, uint32_t n) {
    if (!c || n < 16384 || n > 16777215) return HPK_E_INVAL;  // RFC 9113 §6.5.2 bounds
    c->max_frame_size = n;
    return HPK_E_OK;
}

extern "C" int hpk_h2conn_error(const hpk_h2conn* c) { return c ? c->error : HPK_E_INVAL; }

extern "C" int hpk_h2_error_code(int err) {  // H2ConnectionError::as_known_error_code (types.rs:428-456)
    switch (err) {
        case HPK_H2_OK: return 0x0;                             // NO_ERROR
        case HPK_H2_FRAME_TOO_LARGE:                            // FRAME_SIZE_ERROR
        case HPK_H2_PADDED_FRAME_EMPTY: return 0x6;
        case HPK_H2_COMPRESSION_ERROR: return 0x9;              // COMPRESSION_ERROR
        default: return 0x1;                                    // PROTOCOL_ERROR
    }
}

extern "C" int hpk_h2_read_frames(hpk_ctx* ctx, hpk_h2conn* const* conns, const uint8_t* bytes, const uint32_t* off,
                                  uint32_t nconn, hpk_h2_out* out) {
    if (!conns || !off || !out || (nconn && off[nconn] > off[0] && !bytes)) return HPK_E_INVAL;
    memset(out, 0, sizeof *out);
    for (uint32_t c = 0; c < nconn; ++c)
        if (!conns[c] || off[c + 1] < off[c]) return HPK_E_INVAL;
    out->n_conns = nconn;
    out->conn_error = (int32_t*)calloc(nconn ? nconn : 1, sizeof(int32_t));
    out->conn_consumed = (uint32_t*)calloc(nconn ? nconn : 1, sizeof(uint32_t));
    if (!out->conn_error || !out->conn_consumed) {
        hpk_h2_out_free(out);
        return HPK_E_INVAL;
    }
    // 1. framing, connection by connection: complete header blocks are copied into one buffer
    std::vector<uint8_t> blk;
    std::vector<uint32_t> boff(1, 0);
    std::vector<hpk_hdec*> decs;
    std::vector<hpk_h2_block> meta;
    blk.reserve(off[nconn] - off[0]);
    auto emit = [&](uint32_t c, uint32_t sid, uint32_t end_stream, const uint8_t* p, size_t n) {
        blk.insert(blk.end(), p, p + n);
        boff.push_back((uint32_t)blk.size());
        decs.push_back(conns[c]->dec);
        meta.push_back(hpk_h2_block{c, sid, end_stream, 0u});
    };
    std::vector<int32_t> frame_err(nconn, HPK_H2_OK);  // framing errors found this call
    for (uint32_t c = 0; c < nconn; ++c) {
        hpk_h2conn* k = conns[c];
        size_t pos = off[c];
        const size_t end = off[c + 1];
        int32_t err = k->error;
        while (err == HPK_H2_OK && end - pos >= 9) {
            const uint8_t* h = bytes + pos;
            const uint32_t len = be24(h), sid = be31(h + 5);
            const uint8_t type = h[3], flags = h[4];
            if (len > k->max_frame_size) {  // server.rs:318-325
                err = HPK_H2_FRAME_TOO_LARGE;
                break;
            }
            if (end - pos - 9 < len) break;  // the rest of this frame comes with a later call
            const uint8_t* p = h + 9;
            size_t n = len;
            pos += 9 + (size_t)len;
            if ((type == kData || type == kHeaders) && (flags & kPadded)) {  // server.rs:356-382
                if (n == 0) {
                    err = HPK_H2_PADDED_FRAME_EMPTY;
                    break;
                }
                const size_t pad = p[0];
                p += 1;
                n -= 1;
                if (n < pad) {
                    err = HPK_H2_PADDED_FRAME_TOO_SHORT;
                    break;
                }
                n -= pad;
            }
            if (k->pending) {  // read_headers' CONTINUATION loop (server.rs:1376-1417)
                // the stream id is checked before the frame type (server.rs:1391-1397, then 1399-1408):
                // any frame of another stream is ExpectedContinuationForStream, whatever its type
                if (sid != k->pend_stream) {
                    err = HPK_H2_EXPECTED_CONTINUATION_FOR_STREAM;
                    break;
                }
                if (type != kContinuation) {
                    err = HPK_H2_EXPECTED_CONTINUATION_FRAME;
                    break;
                }
                k->frag.insert(k->frag.end(), p, p + n);
                if (flags & kEndHeaders) {
                    emit(c, k->pend_stream, k->pend_end_stream, k->frag.data(), k->frag.size());
                    k->pending = false;
                    k->frag.clear();
                }
                continue;
            }
            if (type == kContinuation) {  // server.rs:1299-1303
                err = HPK_H2_UNEXPECTED_CONTINUATION_FRAME;
                break;
            }
            if (type != kHeaders) continue;  // other frame types: not this layer's business
            if (flags & kPriority) {         // server.rs:895-911, PrioritySpec::parse
                if (n < 5) {
                    err = HPK_H2_PRIORITY_PARSE;
                    break;
                }
                if (be31(p) == sid) {
                    err = HPK_H2_HEADERS_INVALID_PRIORITY;
                    break;
                }
                p += 5;
                n -= 5;
            }
            const uint32_t es = (flags & kEndStream) ? 1u : 0u;
            if (flags & kEndHeaders) {
                emit(c, sid, es, p, n);
            } else {
                k->pending = true;
                k->pend_stream = sid;
                k->pend_end_stream = es;
                k->frag.assign(p, p + n);
            }
        }
        out->conn_consumed[c] = (uint32_t)(pos - off[c]);
        frame_err[c] = err;
        if (err != HPK_H2_OK) k->error = err;
    }
    // 2. every complete block of every connection in one two-pass decode (one Huffman batch)
    const uint32_t nb = (uint32_t)meta.size();
    int rc = nb ? hpk_hdec_decode_blocks(ctx, decs.data(), blk.data(), boff.data(), nb, &out->hb) : HPK_E_OK;
    if (rc) {
        hpk_h2_out_free(out);
        return rc;
    }
    out->blocks = (hpk_h2_block*)malloc((nb ? nb : 1) * sizeof(hpk_h2_block));
    if (!out->blocks) {
        hpk_h2_out_free(out);
        return HPK_E_INVAL;
    }
    if (nb) memcpy(out->blocks, meta.data(), nb * sizeof(hpk_h2_block));
    // 3. a decoding error is a connection error (COMPRESSION_ERROR, types.rs:446): it comes before
    // any framing error of the same call (its block was framed earlier), and the connection's
    // later blocks are never decoded by the reference
    std::vector<uint8_t> dead(nconn, 0);
    for (uint32_t c = 0; c < nconn; ++c) dead[c] = conns[c]->error != HPK_H2_OK && frame_err[c] == HPK_H2_OK;
    for (uint32_t b = 0; b < nb; ++b) {
        const uint32_t c = meta[b].conn;
        if (dead[c]) {
            out->blocks[b].skipped = 1;
            continue;
        }
        if (out->hb.blocks[b].error != HPK_BLK_OK) {
            dead[c] = 1;
            conns[c]->error = HPK_H2_COMPRESSION_ERROR;
            frame_err[c] = HPK_H2_COMPRESSION_ERROR;
        }
    }
    for (uint32_t c = 0; c < nconn; ++c) out->conn_error[c] = conns[c]->error;
    return HPK_E_OK;
}

extern "C" void hpk_h2_out_free(hpk_h2_out* out) {
    if (!out) return;
    hpk_blocks_out_free(&out->hb);
    free(out->blocks);
    free(out->conn_error);
    free(out->conn_consumed);
    memset(out, 0, sizeof *out);
}
