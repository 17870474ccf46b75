"""HPACK header blocks: decoding with batched Huffman strings and the response-path
encoder (§8f-2).

Mirrors loona-hpack's `hpack::Decoder` (crates/loona-hpack/src/decoder.rs:257-555):

    d = Decoder()                       # Decoder::new(), dynamic table max 4096
    d.set_max_table_size(256)           # decoder.rs:296-311
    d.set_max_allowed_table_size(4096)  # decoder.rs:316-318
    headers = d.decode(block)           # list[(name, value)] or raises DecoderError

and adds the batched form the GPU is for:

    decode_blocks([(d1, block_a), (d2, block_b), (d1, block_c)], codec)

which decodes every Huffman string of every block in one hpk_decode_batch on `codec`'s device
(or with the library's CPU batch path when codec is None) and then applies each block to its
decoder in order. Error values carry the reference's enum names:
    DecoderError("HeaderIndexOutOfBounds")
    DecoderError("IntegerDecodingError", "TooManyOctets" | "NotEnoughOctets" | ...)
    DecoderError("StringDecodingError", "NotEnoughOctets")
    DecoderError("StringDecodingError", ("HuffmanDecoderError", status))
    DecoderError("InvalidMaxDynamicSize"), DecoderError("SizeUpdateAtEnd")

The encoder mirrors `hpack::Encoder` (crates/loona-hpack/src/encoder.rs:172-335):

    e = Encoder()                       # Encoder::new(): raw string literals, as the reference
    e = Encoder(huffman=True)           # the H-bit form whenever it is strictly shorter
    e.set_max_table_size(256)           # encoder.rs:193-197
    block = e.encode([(b"custom-key", b"custom-value")])   # encoder.rs:210-217

and its batched form for many responses at once (all their Huffman strings in one device batch):

    encode_blocks([(e1, headers_a), (e2, headers_b), (e1, headers_c)], codec)  # -> [bytes]
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_ERR = {
    1: ("HeaderIndexOutOfBounds", None),
    2: ("IntegerDecodingError", "TooManyOctets"),
    3: ("IntegerDecodingError", "ValueTooLarge"),
    4: ("IntegerDecodingError", "NotEnoughOctets"),
    5: ("IntegerDecodingError", "InvalidPrefix"),
    6: ("StringDecodingError", "NotEnoughOctets"),
    8: ("InvalidMaxDynamicSize", None),
    9: ("SizeUpdateAtEnd", None),
}

_DISPLAY = {
    "HeaderIndexOutOfBounds": "Header index out of bounds",
    "InvalidMaxDynamicSize": "Dynamic table size exceeds the maximum size",
    "SizeUpdateAtEnd": "Dynamic table size update at the end of a header block",
}


class DecoderError(Exception):
    """DecoderError (decoder.rs:237-253): .kind = variant name, .detail = nested kind."""

    def __init__(self, kind, detail=None):
        super().__init__(_DISPLAY.get(kind, kind if detail is None else f"{kind}: {detail}"))
        self.kind = kind
        self.detail = detail

    def __eq__(self, other):
        return isinstance(other, DecoderError) and (self.kind, self.detail) == (other.kind, other.detail)

    def __hash__(self):
        return hash((self.kind, self.detail))


def _error(code, detail):
    if code == 7:
        return DecoderError("StringDecodingError", ("HuffmanDecoderError", int(detail)))
    kind, det = _ERR[code]
    return DecoderError(kind, det)


class Decoder:
    """hpack::Decoder: one per connection (holds the dynamic table)."""

    def __init__(self):
        self._L = _lib.lib()
        self._h = self._L.hpk_hdec_create()
        if not self._h:
            raise MemoryError("hpk_hdec_create")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._L.hpk_hdec_destroy(h)

    def set_max_table_size(self, n: int):
        if self._L.hpk_hdec_set_max_table_size(self._h, n) != 0:
            raise AssertionError(f"new_max_size ({n}) > max_allowed_size")  # the reference asserts

    def set_max_allowed_table_size(self, n: int):
        _lib.check(self._L.hpk_hdec_set_max_allowed_table_size(self._h, n), "hpk_hdec_set_max_allowed_table_size")

    def table_size(self):
        """(size in octets per RFC 7541 §4.1, entries, max size)."""
        a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        self._L.hpk_hdec_table_size(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def decode_with_cb(self, buf: bytes, cb, codec=None):
        """decoder.rs:368-450: cb(name, value) for each header; raises the first error."""
        (res,) = _decode_raw([(self, buf)], codec)
        headers, err = res
        for n, v in headers:
            cb(n, v)
        if err is not None:
            raise err

    def decode(self, buf: bytes, codec=None):
        """decoder.rs:461-469: the header list, or DecoderError."""
        (res,) = _decode_raw([(self, buf)], codec)
        headers, err = res
        if err is not None:
            raise err
        return headers


def _decode_raw(pairs, codec):
    L = _lib.lib()
    n = len(pairs)
    off = np.zeros(n + 1, np.int64)
    np.cumsum([len(b) for _, b in pairs], out=off[1:])
    if off[-1] >= 2**32:
        raise ValueError("header blocks of one call must stay below 4 GiB")
    blob = np.frombuffer(b"".join(bytes(b) for _, b in pairs) or b"\0", dtype=np.uint8).copy()
    off32 = off.astype(np.uint32)
    decs = (ctypes.c_void_p * max(n, 1))(*[d._h for d, _ in pairs])
    out = _lib.BlocksOut()
    ctx = codec._h if codec is not None else None
    rc = L.hpk_hdec_decode_blocks(ctx, decs, blob.ctypes.data, off32.ctypes.data, n, ctypes.byref(out))
    _lib.check(rc, "hpk_hdec_decode_blocks")
    try:
        arena = ctypes.string_at(out.arena, out.arena_len) if out.arena_len else b""
        res = []
        for b in range(n):
            r = out.blocks[b]
            hs = []
            for j in range(r.first_header, r.first_header + r.n_headers):
                h = out.headers[j]
                hs.append((arena[h.name_off : h.name_off + h.name_len], arena[h.value_off : h.value_off + h.value_len]))
            res.append((hs, None if r.error == 0 else _error(r.error, r.detail)))
        return res
    finally:
        L.hpk_blocks_out_free(ctypes.byref(out))


def decode_blocks(pairs, codec=None):
    """[(Decoder, block bytes)] -> [header list | DecoderError], all Huffman strings in one batch.
    The blocks of one decoder are applied in list order (connection order)."""
    return [hs if err is None else err for hs, err in _decode_raw(pairs, codec)]


class Encoder:
    """hpack::Encoder: one per connection (holds the dynamic table). huffman=False produces the
    reference's bytes exactly; huffman=True Huffman-codes a string literal when that is shorter."""

    def __init__(self, huffman: bool = False):
        self._L = _lib.lib()
        self._h = self._L.hpk_henc_create(1 if huffman else 0)
        if not self._h:
            raise MemoryError("hpk_henc_create")

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._L.hpk_henc_destroy(h)

    def set_max_table_size(self, n: int):
        _lib.check(self._L.hpk_henc_set_max_table_size(self._h, n), "hpk_henc_set_max_table_size")

    def encode(self, headers) -> bytes:
        """encoder.rs:210-217: the header block for [(name, value)] (bytes)."""
        parts, off = [], [0]
        for name, value in headers:
            for x in (name, value):
                parts.append(bytes(x))
                off.append(off[-1] + len(x))
        if off[-1] >= 2**32:
            raise ValueError("header fields of one block must stay below 4 GiB")
        fields = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8).copy()
        off32 = np.asarray(off, dtype=np.uint32)
        n = len(off) // 2
        cap = 64 + 2 * off[-1] + 8 * n
        while True:
            out = np.empty(cap, np.uint8)
            got = ctypes.c_size_t(0)
            rc = self._L.hpk_henc_encode(self._h, fields.ctypes.data, off32.ctypes.data, n, out.ctypes.data, cap,
                                         ctypes.byref(got))
            if rc == -2:  # HPK_E_NOSPACE: state unchanged, retry with the size needed
                cap = got.value
                continue
            _lib.check(rc, "hpk_henc_encode")
            return out[: got.value].tobytes()


def encode_blocks(pairs, codec=None):
    """[(Encoder, [(name, value)])] -> [block bytes]: the table logic per block on the host (blocks of
    one encoder in list order), every string literal of every Huffman-coding encoder in ONE
    hpk_encode_batch on `codec`'s device (the library's CPU batch path when codec is None); the same
    bytes as Encoder.encode block by block (hpk_henc_encode_blocks)."""
    L = _lib.lib()
    parts, off, hoff = [], [0], [0]
    for _, headers in pairs:
        for name, value in headers:
            for x in (name, value):
                parts.append(bytes(x))
                off.append(off[-1] + len(x))
        hoff.append(hoff[-1] + len(headers))
    if off[-1] >= 2**32:
        raise ValueError("header fields of one call must stay below 4 GiB")
    fields = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8).copy()
    off32 = np.asarray(off, dtype=np.uint32)
    hoff32 = np.asarray(hoff, dtype=np.uint32)
    n = len(pairs)
    encs = (ctypes.c_void_p * max(n, 1))(*[e._h for e, _ in pairs])
    out = _lib.HencOut()
    ctx = codec._h if codec is not None else None
    _lib.check(L.hpk_henc_encode_blocks(ctx, encs, fields.ctypes.data, off32.ctypes.data, hoff32.ctypes.data, n,
                                        ctypes.byref(out)), "hpk_henc_encode_blocks")
    try:
        data = ctypes.string_at(out.bytes, out.len) if out.len else b""
        return [data[out.block_off[b] : out.block_off[b + 1]] for b in range(n)]
    finally:
        L.hpk_henc_out_free(ctypes.byref(out))
