"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of loona-hpack's decode path (and of its
block encoder, encoder.rs, for the response-path tests).

Used by tests/ (small cases) and tests/golden/make_golden.py as a second, independent checker
next to the C oracle (hpk_oracle.c). Never imported by the product package ``loona_amd``.

Parity pinning: loona-hpack is Rust and cannot be built here (no cargo/rustc), so this module
is pinned by the reference's own vectors in tests/golden/ (huffman.rs unit KATs, RFC 7541
App. C blocks from decoder.rs tests, and the http2jp interop stories). Every function cites
the reference lines it restates (paths relative to bearcove/loona @ 2025-05-09).
"""

from __future__ import annotations

import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

# ----------------------------------------------------------------------------------------------
# The Huffman code (RFC 7541 App. B). Pinned against the reference's explicit table
# (crates/loona-hpack/src/huffman.rs:222-480) via tests/golden/huffman_table.json.
_LENS_STR = (
    "NX]]]]]]]Y_]]_]]]]]]]]_]]]]]]]]]"
    "GKKMNGILKKILIGGGFFFGGGGGGGHIPGMKNGHHHHHHHHHHHHHHHHHHHHHHIHINTNOG"
    "PFGFGFGGGFHHGGGFGHGFFGHHHHHPLON]"
    "UWUUWWWXWXXXXXYXYYWXYXXXXVWXWXXYWVUWWXXVXWWYVWXXVVWVXWXXUWWWXWWX"
    "[[UTWXWZ[[[\\\\[YZTV[\\\\[\\YVV[[]\\\\\\UYUVWVVXWWZZYY[X[\\[[\\\\\\\\\\]\\\\\\\\\\["
    "_"
)


def code_table():
    """(code, len) for symbols 0..256, rebuilt canonically from the lengths."""
    lens = [ord(ch) - ord("A") for ch in _LENS_STR]
    assert len(lens) == 257
    order = sorted(range(257), key=lambda s: (lens[s], s))
    table = [None] * 257
    c, prev = 0, lens[order[0]]
    for i, s in enumerate(order):
        if i:
            c = (c + 1) << (lens[s] - prev)
        prev = lens[s]
        table[s] = (c, lens[s])
    return table


TABLE = code_table()
EOS_CODE, EOS_LEN = TABLE[256]

# status values (hpk.h hpk_status <-> huffman.rs:28-41 HuffmanDecoderError)
OK, PADDING_TOO_LARGE, INVALID_PADDING, EOS_IN_STRING = 0, 1, 2, 3


def huffman_decode(buf: bytes):
    """HuffmanDecoder::decode (huffman.rs:95-161): bit-by-bit walk over a len->code->sym map.

    Returns (status, decoded_bytes_so_far)."""
    by_len = {}
    for sym, (code, ln) in enumerate(TABLE):  # from_table, huffman.rs:58-82
        by_len.setdefault(ln, {})[code] = sym
    current, current_len = 0, 0
    out = bytearray()
    for byte in buf:  # BitIterator, huffman.rs:171-220 (MSB first)
        for pos in range(7, -1, -1):
            current_len += 1
            current = (current << 1) | ((byte >> pos) & 1)
            sub = by_len.get(current_len)
            if sub is not None and current in sub:
                sym = sub[current]
                if sym == 256:
                    return EOS_IN_STRING, bytes(out)
                out.append(sym)
                current, current_len = 0, 0
    if current_len > 7:
        return PADDING_TOO_LARGE, bytes(out)
    rac = 0 if current_len == 0 else (current << (32 - current_len)) & 0xFFFFFFFF
    rae = (EOS_CODE << (32 - EOS_LEN)) & 0xFFFFFFFF
    mask = 0 if current_len == 0 else (((1 << current_len) - 1) << (32 - current_len)) & 0xFFFFFFFF
    if (rae & mask) != rac:
        return INVALID_PADDING, bytes(out)
    return OK, bytes(out)


def huffman_encode(data: bytes) -> bytes:
    """RFC 7541 §5.2 canonical encoding, EOS-MSB padding (no reference fn: encoder.rs:296-307)."""
    acc, nb = 0, 0
    for b in data:
        code, ln = TABLE[b]
        acc = (acc << ln) | code
        nb += ln
    pad = (-nb) % 8
    acc = (acc << pad) | ((1 << pad) - 1)
    nb += pad
    return acc.to_bytes(nb // 8, "big") if nb else b""


# ----------------------------------------------------------------------------------------------
# HPACK integer / string / block layer (decoder.rs, lib.rs)


class DecoderError(Exception):
    """DecoderError (decoder.rs:237-253); .kind is a short tag, .detail optional."""

    def __init__(self, kind, detail=None):
        super().__init__(kind if detail is None else f"{kind}:{detail}")
        self.kind = kind
        self.detail = detail


def decode_integer(buf: bytes, prefix: int):
    """decode_integer (decoder.rs:67-125). Returns (value, consumed)."""
    if not 1 <= prefix <= 8:
        raise DecoderError("IntegerDecodingError", "InvalidPrefix")
    if not buf:
        raise DecoderError("IntegerDecodingError", "NotEnoughOctets")
    mask = 0xFF if prefix == 8 else (1 << prefix) - 1
    value = buf[0] & mask
    if value < mask:
        return value, 1
    total, m = 1, 0
    for b in buf[1:]:
        total += 1
        value += (b & 127) << m
        m += 7
        if not b & 128:
            return value, total
        if total == 5:
            raise DecoderError("IntegerDecodingError", "TooManyOctets")
    raise DecoderError("IntegerDecodingError", "NotEnoughOctets")


def decode_string(buf: bytes):
    """decode_string (decoder.rs:135-163). Returns (bytes, consumed)."""
    ln, consumed = decode_integer(buf, 7)
    if consumed + ln > len(buf):
        raise DecoderError("StringDecodingError", "NotEnoughOctets")
    raw = bytes(buf[consumed : consumed + ln])
    if buf[0] & 128:
        st, out = huffman_decode(raw)
        if st != OK:
            raise DecoderError("StringDecodingError", ("HuffmanDecoderError", st))
        return out, consumed + ln
    return raw, consumed + ln


def _load_static_table():
    with open(os.path.join(HERE, "..", "tests", "golden", "static_table.json")) as f:
        return [(n.encode(), v.encode()) for n, v in json.load(f)]


STATIC_TABLE = None


class DynamicTable:
    """DynamicTable (lib.rs:43-164): FIFO, entry size = name + value + 32."""

    def __init__(self, max_size=4096):
        self.table = []  # front = newest
        self.size = 0
        self.max_size = max_size

    def set_max_table_size(self, n):
        self.max_size = n
        self._consolidate()

    def add_header(self, name, value):
        self.size += len(name) + len(value) + 32
        self.table.insert(0, (name, value))
        self._consolidate()

    def _consolidate(self):
        while self.size > self.max_size:
            n, v = self.table.pop()
            self.size -= len(n) + len(v) + 32


class Decoder:
    """Decoder::decode_with_cb / decode (decoder.rs:368-469) with HeaderTable (lib.rs:178-289)."""

    def __init__(self):
        global STATIC_TABLE
        if STATIC_TABLE is None:
            STATIC_TABLE = _load_static_table()
        self.static = STATIC_TABLE
        self.dynamic = DynamicTable()
        self.max_allowed_table_size = None

    def set_max_table_size(self, n):
        """Decoder::set_max_table_size (decoder.rs:325-340); the allowed-size assert is a panic
        there, so it is only restated for the unset case the tests use."""
        assert self.max_allowed_table_size is None or n <= self.max_allowed_table_size
        self.dynamic.set_max_table_size(n)

    def get_from_table(self, index):
        if index == 0:
            raise DecoderError("HeaderIndexOutOfBounds")
        ri = index - 1
        if ri < len(self.static):
            return self.static[ri]
        di = ri - len(self.static)
        if di < len(self.dynamic.table):
            return self.dynamic.table[di]
        raise DecoderError("HeaderIndexOutOfBounds")

    def _decode_literal(self, buf, index):
        prefix = 6 if index else 4
        table_index, consumed = decode_integer(buf, prefix)
        if table_index == 0:
            name, n = decode_string(buf[consumed:])
            consumed += n
        else:
            name = self.get_from_table(table_index)[0]
        value, n = decode_string(buf[consumed:])
        return (name, value), consumed + n

    def decode(self, buf: bytes):
        out = []
        i = 0
        last_was_size_update = False
        while i < len(buf):
            b = buf[i]
            rest = buf[i:]
            last_was_size_update = False
            if b & 128:
                index, consumed = decode_integer(rest, 7)
                out.append(self.get_from_table(index))
            elif b & 64:
                (n, v), consumed = self._decode_literal(rest, True)
                out.append((n, v))
                self.dynamic.add_header(n, v)
            elif b & 32:
                last_was_size_update = True
                new_size, consumed = decode_integer(rest, 5)
                if self.max_allowed_table_size is not None and new_size > self.max_allowed_table_size:
                    raise DecoderError("InvalidMaxDynamicSize")
                self.dynamic.set_max_table_size(new_size)
            else:  # 0001xxxx never indexed, 0000xxxx without indexing
                (n, v), consumed = self._decode_literal(rest, False)
                out.append((n, v))
            i += consumed
        if last_was_size_update:
            raise DecoderError("SizeUpdateAtEnd")
        return out


def encode_integer(value: int, prefix: int, leading: int = 0) -> bytes:
    """encode_integer_into (encoder.rs:93-122)."""
    mask = 0xFF if prefix >= 8 else (1 << prefix) - 1
    leading &= ~mask & 0xFF
    if value < mask:
        return bytes([leading | value])
    out = [leading | mask]
    value -= mask
    while value >= 128:
        out.append(value % 128 + 128)
        value //= 128
    out.append(value)
    return bytes(out)


class Encoder:
    """Encoder (encoder.rs:172-335) with HeaderTable::find_header (lib.rs:261-288). huffman=True
    adds this library's policy on top (not the reference's: encoder.rs:296-307 never Huffman-
    codes): a string literal takes the H-bit form when its Huffman encoding is strictly shorter."""

    def __init__(self, huffman=False):
        global STATIC_TABLE
        if STATIC_TABLE is None:
            STATIC_TABLE = _load_static_table()
        self.static = STATIC_TABLE
        self.dynamic = DynamicTable()
        self.huffman = huffman

    def set_max_table_size(self, n):
        self.dynamic.set_max_table_size(n)

    def find_header(self, name, value):
        matching = None
        for i, (n, v) in enumerate(list(self.static) + list(self.dynamic.table)):
            if n == name:
                if v == value:
                    return i + 1, True
                matching = i + 1
        return (matching, False) if matching is not None else None

    def _string(self, s):
        if self.huffman and s:
            h = huffman_encode(s)
            if len(h) < len(s):
                return encode_integer(len(h), 7, 0x80) + h
        return encode_integer(len(s), 7, 0) + s

    def encode(self, headers):
        out = b""
        for name, value in headers:
            name, value = bytes(name), bytes(value)
            f = self.find_header(name, value)
            if f is None:  # encode_literal(should_index = true) + add_header (encoder.rs:246-253)
                out += bytes([0x40]) + self._string(name) + self._string(value)
                self.dynamic.add_header(name, value)
            elif not f[1]:  # encode_indexed_name(should_index = false) (encoder.rs:254-259, 311-323)
                out += encode_integer(f[0], 4, 0) + self._string(value)
            else:  # encode_indexed (encoder.rs:260-264, 329-334)
                out += encode_integer(f[0], 7, 0x80)
        return out


def huffman_literal_spans(buf: bytes):
    """Walk one header block and list the Huffman literal spans (start, end) of its string
    literals, in field order, without table state (positions never depend on it).
    Stops silently at the first malformed field (errors are the block decoder's job)."""
    spans = []
    i = 0
    try:
        while i < len(buf):
            b = buf[i]
            rest = buf[i:]
            if b & 128:
                _, c = decode_integer(rest, 7)
                i += c
                continue
            if (b & 0xE0) == 0x20:
                _, c = decode_integer(rest, 5)
                i += c
                continue
            prefix = 6 if b & 64 else 4
            idx, c = decode_integer(rest, prefix)
            j = i + c
            strings = 2 if idx == 0 else 1
            for _ in range(strings):
                ln, cc = decode_integer(buf[j:], 7)
                if j + cc + ln > len(buf):
                    return spans
                if buf[j] & 128:
                    spans.append((j + cc, j + cc + ln))
                j += cc + ln
            i = j
    except DecoderError:
        pass
    return spans
