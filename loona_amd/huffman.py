"""Host-side mirror of loona-hpack's Huffman API (crates/loona-hpack/src/huffman.rs).

    HuffmanDecoder().decode(buf) -> bytes        # huffman.rs:86-88, :95-161
    HuffmanDecoderError.{PaddingTooLarge, InvalidPadding, EOSInString}   # huffman.rs:28-41

Same names, argument meaning and error behaviour as the Rust API: `decode` returns the decoded
octets or raises HuffmanDecoderError carrying the same variant the reference returns. Single
literals run on the library's scalar CPU path (hpk_huffman_decode_one); batches go to the GPU
through loona_amd.batch.HuffmanCodec.
"""

from __future__ import annotations

import ctypes
import enum

from . import _lib


class HuffmanDecoderError(Exception):
    """Error variants of HuffmanDecoderError; `.kind` is the variant.

    str() gives the reference's Display text ("Padding too large", "Invalid padding",
    "EOS in string"; huffman.rs:31-40)."""

    class Kind(enum.IntEnum):
        PaddingTooLarge = _lib.HPK_PADDING_TOO_LARGE
        InvalidPadding = _lib.HPK_INVALID_PADDING
        EOSInString = _lib.HPK_EOS_IN_STRING

    _TEXT = {
        Kind.PaddingTooLarge: "Padding too large",
        Kind.InvalidPadding: "Invalid padding",
        Kind.EOSInString: "EOS in string",
    }

    def __init__(self, kind):
        self.kind = HuffmanDecoderError.Kind(kind)
        super().__init__(self._TEXT[self.kind])

    def __eq__(self, other):
        if isinstance(other, HuffmanDecoderError):
            return self.kind == other.kind
        if isinstance(other, HuffmanDecoderError.Kind):
            return self.kind == other
        return NotImplemented

    def __hash__(self):
        return hash(self.kind)


# variant shorthands, so `HuffmanDecoderError.EOSInString` reads as in Rust
HuffmanDecoderError.PaddingTooLarge = HuffmanDecoderError.Kind.PaddingTooLarge
HuffmanDecoderError.InvalidPadding = HuffmanDecoderError.Kind.InvalidPadding
HuffmanDecoderError.EOSInString = HuffmanDecoderError.Kind.EOSInString


def decoded_bound(n: int) -> int:
    return int(_lib.lib().hpk_decoded_bound(n))


def encoded_bound(n: int) -> int:
    return int(_lib.lib().hpk_encoded_bound(n))


class HuffmanDecoder:
    """HuffmanDecoder (huffman.rs:48-161). Stateless between calls, like the reference."""

    def __init__(self):
        self._L = _lib.lib()

    @classmethod
    def new(cls) -> "HuffmanDecoder":
        return cls()

    def decode(self, buf: bytes) -> bytes:
        buf = bytes(buf)
        cap = self._L.hpk_decoded_bound(len(buf))
        out = ctypes.create_string_buffer(max(cap, 1))
        out_len = ctypes.c_size_t(0)
        rc = self._L.hpk_huffman_decode_one(buf, len(buf), out, cap, ctypes.byref(out_len))
        _lib.check(rc, "hpk_huffman_decode_one")
        if rc != _lib.HPK_OK:
            raise HuffmanDecoderError(rc)
        return out.raw[: out_len.value]


def huffman_encode(data: bytes) -> bytes:
    """Canonical RFC 7541 §5.2 encoding (the reference has no encoder: encoder.rs:296-307)."""
    L = _lib.lib()
    data = bytes(data)
    cap = L.hpk_encoded_bound(len(data))
    out = ctypes.create_string_buffer(max(cap, 1))
    out_len = ctypes.c_size_t(0)
    _lib.check(L.hpk_huffman_encode_one(data, len(data), out, cap, ctypes.byref(out_len)), "hpk_huffman_encode_one")
    return out.raw[: out_len.value]


def huffman_encoded_len(data: bytes) -> int:
    data = bytes(data)
    return int(_lib.lib().hpk_huffman_encoded_len(data, len(data)))
