"""The response-path block encoder (hpk_henc) on the CPU.

Pinned by encoder.rs's own vectors (its doc example, test_uses_index_on_second_iteration,
test_name_indexed_value_not, test_encode_integer through string-length prefixes) and by the
restatement oracle/hpack_ref.Encoder on every header list of the interop stories; huffman mode is
checked by decoding (the library's hpk_hdec and the decoder.rs restatement) and by the H-bit rule
literal by literal."""

import ctypes

import numpy as np
import pytest

from hpk_util import hpack_ref, load

from loona_amd import _lib, hpack


def stories():
    inter = load("interop.json.gz")
    for enc in sorted(inter):
        for story in inter[enc]:
            yield [[(n.encode(), v.encode()) for n, v in c["headers"]] for c in story["cases"]]


def test_reference_doc_example():
    """encoder.rs:146-170 and test_uses_index_on_second_iteration (encoder.rs:406-430)."""
    e = hpack.Encoder()
    h = [(b"custom-key", b"custom-value")]
    assert e.encode(h) == bytes([0x40, 10]) + b"custom-key" + bytes([12]) + b"custom-value"
    assert e.encode(h) == bytes([0x80 | 62])


def test_reference_name_indexed_value_not():
    """encoder.rs:436-463: the LAST name match (index 3 for :method), value literal, not indexed."""
    assert hpack.Encoder().encode([(b":method", b"PUT")]) == bytes([3, 3]) + b"PUT"
    assert hpack.Encoder().encode([(b":authority", b"example.com")]) == bytes([1, 11]) + b"example.com"


@pytest.mark.parametrize("n,prefix", [(126, b"\x7e"), (127, b"\x7f\x00"), (255, b"\x7f\x80\x01"), (1337, None)])
def test_string_length_prefixes(n, prefix):
    """encode_integer (encoder.rs:346-356) through the 7-bit string length prefix."""
    v = b"v" * n
    got = hpack.Encoder().encode([(b"x-len", v)])
    want = b"\x40" + hpack_ref.encode_integer(5, 7) + b"x-len" + hpack_ref.encode_integer(n, 7) + v
    assert got == want
    if prefix is not None:
        assert got[7 : 7 + len(prefix)] == prefix
    assert hpack_ref.encode_integer(1337, 5) == bytes([31, 154, 10])
    assert hpack_ref.encode_integer(255, 7) == bytes([127, 128, 1])


def test_multiple_headers_decodable():
    """encoder.rs:467-479."""
    h = [(b"custom-key", b"custom-value"), (b":method", b"GET"), (b":path", b"/some/path")]
    for huff in (False, True):
        assert hpack.Decoder().decode(hpack.Encoder(huffman=huff).encode(h)) == h


@pytest.mark.parametrize("huff", [False, True])
def test_interop_stories_match_restatement_and_round_trip(huff):
    """Every interop story's header lists, one encoder per story (connection order): bytes equal to
    the encoder.rs restatement, and the blocks decode back (hpk_hdec and decoder.rs restated)."""
    total = 0
    for lists in stories():
        e, r = hpack.Encoder(huffman=huff), hpack_ref.Encoder(huffman=huff)
        d, rd = hpack.Decoder(), hpack_ref.Decoder()
        for h in lists:
            b = e.encode(h)
            assert b == r.encode(h)
            assert d.decode(b) == h
            assert rd.decode(b) == h
            total += len(b)
    assert total > 0


def test_huffman_only_when_shorter():
    """Literal by literal: the H bit is set exactly when the Huffman form is strictly shorter."""
    rng = np.random.default_rng(9)
    for _ in range(300):
        n = int(rng.integers(0, 40))
        v = bytes(rng.integers(0, 256, n, dtype=np.uint8)) if rng.random() < 0.3 else bytes(
            rng.choice(list(b"abcdefghijklmnopqrstuvwxyz0123456789-/"), n))
        b = hpack.Encoder(huffman=True).encode([(b"x-k", v)])
        # 0x40, then the name literal ("x-k": 20 bits of codes, 3 bytes either way: raw), then the value
        assert len(hpack_ref.huffman_encode(b"x-k")) == 3
        assert b[:5] == b"\x40\x03x-k"
        name_end = 5
        hv = hpack_ref.huffman_encode(v)
        if v and len(hv) < len(v):
            assert b[name_end:] == hpack_ref.encode_integer(len(hv), 7, 0x80) + hv
        else:
            assert b[name_end:] == hpack_ref.encode_integer(len(v), 7) + v


def test_eviction_and_table_size():
    """A small table evicts FIFO (lib.rs:121-139): encoder and a decoder of the same size agree."""
    e, d = hpack.Encoder(huffman=True), hpack.Decoder()
    r = hpack_ref.Encoder(huffman=True)
    for x in (e, d, r):
        x.set_max_table_size(100)
    for k in range(50):
        h = [(b"k%d" % (k % 7), b"v" * (k % 13)), (b"k%d" % ((k + 3) % 7), b"w" * (k % 5))]
        b = e.encode(h)
        assert b == r.encode(h)
        assert d.decode(b) == h
    assert d.table_size()[0] <= 100


def test_nospace_leaves_state_unchanged():
    L = _lib.lib()
    h = L.hpk_henc_create(1)
    try:
        fields = np.frombuffer(b"custom-keycustom-value", np.uint8).copy()
        off = np.array([0, 10, 22], np.uint32)
        out = np.zeros(64, np.uint8)
        got = ctypes.c_size_t(0)
        assert L.hpk_henc_encode(h, fields.ctypes.data, off.ctypes.data, 1, out.ctypes.data, 3, ctypes.byref(got)) == -2
        need = got.value
        assert need > 3
        assert L.hpk_henc_encode(h, fields.ctypes.data, off.ctypes.data, 1, out.ctypes.data, 64, ctypes.byref(got)) == 0
        assert got.value == need and out[0] == 0x40  # still a literal with indexing: nothing was added before
        assert L.hpk_henc_encode(h, fields.ctypes.data, off.ctypes.data, 1, out.ctypes.data, 64, ctypes.byref(got)) == 0
        assert got.value == 1 and out[0] == 0x80 | 62
    finally:
        L.hpk_henc_destroy(h)


def response_lists(seed=3, n=3000):
    """Header lists of the interop stories plus seeded random headers (text, binary, empty)."""
    import random

    rng = random.Random(seed)
    inter = load("interop.json.gz")
    lists = [[(k.encode(), v.encode()) for k, v in c["headers"]] for enc in sorted(inter) for st in inter[enc]
             for c in st["cases"]]
    rng.shuffle(lists)
    lists = lists[:n]
    for _ in range(200):
        hs = []
        for _ in range(rng.randrange(0, 8)):
            k = rng.choice([b"content-type", b"x-req-id", b"set-cookie", b"server", b":status"])
            v = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))) if rng.random() < 0.3 else \
                str(rng.randrange(10**9)).encode()
            hs.append((k, v))
        lists.append(hs)
    return lists


@pytest.mark.parametrize("huffman", [False, True])
def test_encode_blocks_matches_block_by_block(huffman):
    """hpk_henc_encode_blocks (all Huffman strings of all blocks in one batch) == hpk_henc_encode per
    block, with blocks of several encoders interleaved (each encoder's blocks in order)."""
    from loona_amd import hpack

    lists = response_lists()
    k = 7
    batch_encs = [hpack.Encoder(huffman=huffman) for _ in range(k)]
    seq_encs = [hpack.Encoder(huffman=huffman) for _ in range(k)]
    pairs = [(batch_encs[i % k], hs) for i, hs in enumerate(lists)]
    got = hpack.encode_blocks(pairs, None)
    want = [seq_encs[i % k].encode(hs) for i, hs in enumerate(lists)]
    assert got == want
    # and the blocks decode back to the lists through fresh decoders in the same order
    decs = [hpack.Decoder() for _ in range(k)]
    back = hpack.decode_blocks([(decs[i % k], b) for i, b in enumerate(got)], None)
    assert back == lists


@pytest.mark.parametrize("huffman", [False, True])
def test_encode_blocks_match_restatement(huffman):
    """hpk_henc_encode_blocks on the CPU batch path against the encoder.rs restatement
    (oracle/hpack_ref.Encoder; encoder.rs:210-234, string literals encoder.rs:296-307 with the H bit
    when shorter) block by block, on interop lists plus random binary and numeric values."""
    lists = response_lists(seed=5)
    k = 5
    encs = [hpack.Encoder(huffman=huffman) for _ in range(k)]
    refs = [hpack_ref.Encoder(huffman=huffman) for _ in range(k)]
    got = hpack.encode_blocks([(encs[i % k], hs) for i, hs in enumerate(lists)], None)
    want = [refs[i % k].encode(hs) for i, hs in enumerate(lists)]
    assert got == want


@pytest.mark.parametrize("huffman", [False, True])
def test_failed_encode_blocks_leaves_encoders_unchanged(huffman):
    """A batch call that fails after the table pass (here: an injected Huffman-batch failure) must
    leave every encoder's dynamic table as it was (hpk_henc_encode's copy-and-commit): the next call
    gives the bytes fresh encoders give for the same blocks."""
    L = _lib.lib()
    lists = response_lists(seed=11, n=300)
    k = 3
    encs = [hpack.Encoder(huffman=huffman) for _ in range(k)]
    warm = lists[:30]
    hpack.encode_blocks([(encs[i % k], hs) for i, hs in enumerate(warm)], None)
    refs = [hpack_ref.Encoder(huffman=huffman) for _ in range(k)]
    for i, hs in enumerate(warm):
        refs[i % k].encode(hs)
    rest = lists[30:]
    pairs = [(encs[i % k], hs) for i, hs in enumerate(rest)]
    if huffman:  # the injected failure sits in the Huffman batch, which only Huffman encoders make
        L.hpk_test_fail_batches(1)
        try:
            with pytest.raises(RuntimeError, match="injected"):
                hpack.encode_blocks(pairs, None)
        finally:
            L.hpk_test_fail_batches(0)
    got = hpack.encode_blocks(pairs, None)
    assert got == [refs[i % k].encode(hs) for i, hs in enumerate(rest)]
