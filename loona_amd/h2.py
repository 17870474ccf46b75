"""HTTP/2 header reading across many connections with one Huffman batch.

Mirrors what loona's h2 server does per connection before it hands a header block to its HPACK
decoder — the deframer (crates/loona/src/h2/server.rs:290-390: frame length check, padding), the
HEADERS priority block (server.rs:895-911) and read_headers' CONTINUATION gathering
(server.rs:1349-1417, 1619-1638) — over the bytes of MANY connections at once, then decodes every
complete header block of every connection with one hpk_hdec_decode_blocks call (include/hpk.h
hpk_h2_read_frames):

    conns = [Connection() for _ in range(n)]
    res = read_frames(conns, [bytes_of_conn0, bytes_of_conn1, ...], codec)   # codec=None: CPU batch
    res.blocks    -> [(conn, stream_id, end_stream, headers | DecoderError | None (skipped))]
    res.errors    -> per connection: H2Error name or None; res.consumed -> bytes used per connection

A connection keeps a HEADERS block whose CONTINUATION frames have not all arrived, and its HPACK
dynamic table, between calls; its first error ends it (the reference sends GOAWAY with
H2Error.code(name)).
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .hpack import _error

ERRORS = {  # hpk_h2_error -> the reference's H2ConnectionError variant
    1: "FrameTooLarge",
    2: "PaddedFrameEmpty",
    3: "PaddedFrameTooShort",
    4: "ReadAndParse(PrioritySpec)",
    5: "HeadersInvalidPriority",
    6: "ExpectedContinuationFrame",
    7: "ExpectedContinuationForStream",
    8: "UnexpectedContinuationFrame",
    9: "HpackDecodingError",
}
CODES = {0x1: "PROTOCOL_ERROR", 0x6: "FRAME_SIZE_ERROR", 0x9: "COMPRESSION_ERROR", 0x0: "NO_ERROR"}


def error_code(name):
    """RFC 9113 §7 error code name the reference's GOAWAY carries for a connection error."""
    inv = {v: k for k, v in ERRORS.items()}
    return CODES[_lib.lib().hpk_h2_error_code(inv[name] if name else 0)]


class Connection:
    """One connection's header-reading state (hpk_h2conn): HPACK decoder + pending CONTINUATION."""

    def __init__(self, max_frame_size: int = 16384):
        self._L = _lib.lib()
        self._h = self._L.hpk_h2conn_create()
        if not self._h:
            raise MemoryError("hpk_h2conn_create")
        if max_frame_size != 16384:
            _lib.check(self._L.hpk_h2conn_set_max_frame_size(self._h, max_frame_size), "hpk_h2conn_set_max_frame_size")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._L.hpk_h2conn_destroy(h)

    @property
    def error(self):
        e = self._L.hpk_h2conn_error(self._h)
        return ERRORS.get(e) if e else None


class Result:
    def __init__(self, blocks, errors, consumed):
        self.blocks, self.errors, self.consumed = blocks, errors, consumed


class Arena:
    """buffet's buffer arena (hpk_arena_create: one anonymous mmap of num_bufs x buf_size, page-locked
    when pin): .view is a writable numpy view of it; read_frames_in() decodes frames in place."""

    def __init__(self, num_bufs=65536, buf_size=4096, pin=True):
        self._L = _lib.lib()
        self._h = self._L.hpk_arena_create(num_bufs, buf_size, 1 if pin else 0)
        if not self._h:
            raise RuntimeError(f"hpk_arena_create failed: {_lib.last_error()}")
        n = self._L.hpk_arena_len(self._h)
        self.base = self._L.hpk_arena_base(self._h)
        self.view = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(self.base))

    def close(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self.view = None
            self._L.hpk_arena_destroy(h)

    def __del__(self):
        self.close()


def read_frames_in(conns, arena, offsets, codec=None) -> Result:
    """read_frames on bytes already in an Arena: connection c's bytes are
    arena.view[offsets[c] : offsets[c+1]] (no copy on the way in)."""
    off32 = np.ascontiguousarray(offsets, dtype=np.uint32)
    return _read(conns, arena.base, off32, codec)


def read_frames(conns, chunks, codec=None) -> Result:
    """Frames received on each connection (chunks[c] = bytes for conns[c]) -> decoded header blocks."""
    L = _lib.lib()
    n = len(conns)
    if len(chunks) != n:
        raise ValueError("one byte chunk per connection")
    off = np.zeros(n + 1, np.int64)
    np.cumsum([len(c) for c in chunks], out=off[1:])
    if off[-1] >= 2**32:
        raise ValueError("the bytes of one call must stay below 4 GiB")
    blob = np.frombuffer(b"".join(bytes(c) for c in chunks) or b"\0", dtype=np.uint8).copy()
    return _read(conns, blob.ctypes.data, off.astype(np.uint32), codec)


def _read(conns, base, off32, codec):
    L = _lib.lib()
    n = len(conns)
    hs = (ctypes.c_void_p * max(n, 1))(*[c._h for c in conns])
    out = _lib.H2Out()
    ctx = codec._h if codec is not None else None
    _lib.check(L.hpk_h2_read_frames(ctx, hs, base, off32.ctypes.data, n, ctypes.byref(out)),
               "hpk_h2_read_frames")
    try:
        arena = ctypes.string_at(out.hb.arena, out.hb.arena_len) if out.hb.arena_len else b""
        blocks = []
        for b in range(out.hb.n_blocks):
            m = out.blocks[b]
            if m.skipped:
                val = None
            else:
                r = out.hb.blocks[b]
                hl = []
                for j in range(r.first_header, r.first_header + r.n_headers):
                    h = out.hb.headers[j]
                    hl.append((arena[h.name_off : h.name_off + h.name_len],
                               arena[h.value_off : h.value_off + h.value_len]))
                val = hl if r.error == 0 else _error(r.error, r.detail)
            blocks.append((m.conn, m.stream_id, bool(m.end_stream), val))
        errors = [ERRORS.get(out.conn_error[c]) if out.conn_error[c] else None for c in range(n)]
        consumed = [out.conn_consumed[c] for c in range(n)]
        return Result(blocks, errors, consumed)
    finally:
        L.hpk_h2_out_free(ctypes.byref(out))


def frame(ftype: int, flags: int, stream_id: int, payload: bytes) -> bytes:
    """One frame: RFC 9113 §4.1 header (24-bit length, type, flags, 31-bit stream id) + payload."""
    n = len(payload)
    return bytes([n >> 16 & 255, n >> 8 & 255, n & 255, ftype, flags]) + (stream_id & 0x7FFFFFFF).to_bytes(4, "big") + \
        bytes(payload)
