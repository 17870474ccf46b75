"""loona_amd — MI355X-native HPACK Huffman codec for loona's HTTP/2 header path.

The product is libhpk.so (include/hpk.h C ABI; gfx950 kernels in csrc/hpk_decode*.hip and
csrc/hpk_encode.hip). This package is its host-side mirror of the loona-hpack interface:

    from loona_amd import HuffmanDecoder, HuffmanDecoderError, HuffmanCodec
"""

from ._lib import lib  # noqa: F401
from .batch import HuffmanCodec, pack, unpack  # noqa: F401
from .huffman import (  # noqa: F401
    HuffmanDecoder,
    HuffmanDecoderError,
    decoded_bound,
    encoded_bound,
    huffman_encode,
    huffman_encoded_len,
)

__all__ = [
    "HuffmanDecoder",
    "HuffmanDecoderError",
    "HuffmanCodec",
    "huffman_encode",
    "huffman_encoded_len",
    "decoded_bound",
    "encoded_bound",
    "pack",
    "unpack",
    "lib",
]
