"""Pin the oracles (C restatement + pure-Python restatement) to the reference's own vectors.

The reference is Rust and cannot be built here; these goldens were extracted from its tests and
fixtures by tests/golden/make_golden.py ("Oracle and parity")."""

import hashlib
import random

import numpy as np
import pytest

from hpk_util import (
    hpack_ref,
    interop_literals,
    load,
    oracle,
    oracle_decode,
    oracle_decode_batch,
    oracle_encode,
    oracle_encode_batch,
    pack,
)


def test_oracle_table_matches_reference_table():
    """huffman.rs:222-480 (code, len) == the oracle's canonical rebuild from lengths."""
    ref = load("huffman_table.json")["table"]
    codes = np.zeros(257, np.uint32)
    lens = np.zeros(257, np.uint8)
    assert oracle().oracle_table(codes.ctypes.data, lens.ctypes.data) == 0
    assert [[int(c), int(ln)] for c, ln in zip(codes, lens)] == ref
    assert [list(t) for t in hpack_ref.TABLE] == ref


@pytest.mark.parametrize("impl", ["c", "py"])
def test_kats(impl):
    """huffman.rs unit tests (huffman.rs:523-707): every single-literal KAT incl. each error."""
    for k in load("kat.json"):
        buf = bytes.fromhex(k["in"])
        st, out = oracle_decode(buf) if impl == "c" else hpack_ref.huffman_decode(buf)
        assert st == k["status"], k
        if k["out"] is not None:
            assert out == bytes.fromhex(k["out"]), k


def test_rfc7541_literals():
    """The 12 App. C Huffman literals (decoder.rs:1216-1402) decode and re-encode exactly."""
    lits = load("rfc7541_blocks.json")["huffman_literals"]
    assert len(lits) == 12
    for x in lits:
        st, out = oracle_decode(bytes.fromhex(x["in"]))
        assert st == 0 and out.hex() == x["out"]
        assert oracle_encode(out).hex() == x["in"]


def test_rfc7541_blocks_python_decoder():
    """Whole-block App. C sequences and block error cases through the Python block decoder."""
    g = load("rfc7541_blocks.json")
    for seq in g["sequences"]:
        d = hpack_ref.Decoder()
        if seq["max_table_size"] is not None:
            d.dynamic.set_max_table_size(seq["max_table_size"])
        for b in seq["blocks"]:
            got = [[n.decode(), v.decode()] for n, v in d.decode(bytes.fromhex(b["wire"]))]
            assert got == b["headers"]
    for e in g["errors"]:
        with pytest.raises(hpack_ref.DecoderError) as ei:
            hpack_ref.Decoder().decode(bytes.fromhex(e["wire"]))
        kind = [ei.value.kind] + ([] if ei.value.detail is None else
                                  list(ei.value.detail) if isinstance(ei.value.detail, tuple) else [ei.value.detail])
        assert kind == e["error"]


def test_error_vectors_c_vs_python():
    """3000 seeded random/perturbed literals: C oracle == Python restatement (status + bytes)."""
    for v in load("error_vectors.json")["vectors"]:
        st, out = oracle_decode(bytes.fromhex(v["in"]))
        assert st == v["status"], v
        assert out.hex() == v["out"], v


def test_closed_form_end_check():
    """after the walk, OK <=> residual <= 7 bits and all ones."""
    rng = random.Random(1)
    for _ in range(2000):
        n = rng.randrange(0, 6)
        b = bytes(rng.getrandbits(8) for _ in range(n))
        st, _ = hpack_ref.huffman_decode(b)
        # recompute the residual by walking with the table
        by = {(c, ln): s for s, (c, ln) in enumerate(hpack_ref.TABLE)}
        cur = ln = 0
        eos = False
        for byte in b:
            for pos in range(7, -1, -1):
                cur = (cur << 1) | ((byte >> pos) & 1)
                ln += 1
                s = by.get((cur, ln))
                if s is not None:
                    if s == 256:
                        eos = True
                        break
                    cur = ln = 0
            if eos:
                break
        if eos:
            assert st == 3
        else:
            ok = ln <= 7 and cur == (1 << ln) - 1
            assert (st == 0) == ok


def test_interop_corpus_digest():
    """All 142,773 interop Huffman literals through the C oracle batch: counts and sha256 of the
    concatenated decoded stream match the digest computed from the reference fixtures."""
    dig = load("interop_digest.json")
    lits = interop_literals()
    assert len(lits) == dig["huffman_literals"]
    blob, off = pack(lits)
    assert int(off[-1]) == dig["encoded_bytes"]
    assert hashlib.sha256(blob.tobytes()).hexdigest() == dig["sha256_encoded"]
    out, oo, ol, st = oracle_decode_batch(blob, off)
    assert not st.any()
    assert int(ol.sum()) == dig["decoded_bytes"]
    h = hashlib.sha256()
    for i in range(len(lits)):
        h.update(out[oo[i] : oo[i] + ol[i]].tobytes())
    assert h.hexdigest() == dig["sha256_decoded"]


def test_interop_reencode_identity():
    """Canonical encode of every decoded interop literal reproduces its wire bytes."""
    lits = interop_literals()
    blob, off = pack(lits)
    out, oo, ol, st = oracle_decode_batch(blob, off)
    dec = [out[oo[i] : oo[i] + ol[i]].tobytes() for i in range(len(lits))]
    dblob, doff = pack(dec)
    eout, eoo, eol, est = oracle_encode_batch(dblob, doff)
    assert not est.any()
    for i in range(0, len(lits)):
        assert eout[eoo[i] : eoo[i] + eol[i]].tobytes() == lits[i]


def test_decode_integer_vectors():
    """decode_integer (decoder.rs:67-125) incl. its error cases (decoder.rs:572-646)."""
    import ctypes

    L = oracle()

    def dec(buf, prefix):
        v = ctypes.c_uint64()
        c = ctypes.c_size_t()
        rc = L.oracle_decode_integer(bytes(buf), len(buf), prefix, ctypes.byref(v), ctypes.byref(c))
        return rc, v.value, c.value

    assert dec([10], 5)[:3] == (0, 10, 1)
    assert dec([31, 154, 10], 5)[:3] == (0, 1337, 3)
    assert dec([31 + 32, 154, 10], 5)[:3] == (0, 1337, 3)
    assert dec([42], 8)[:3] == (0, 42, 1)
    assert dec([0xFF, 0x80, 0x80, 0x80, 0x80, 0x01], 8)[0] == 3  # TooManyOctets
    assert dec([0xFF, 0x80], 8)[0] == 2  # NotEnoughOctets
    assert dec([], 8)[0] == 2
    assert dec([10], 0)[0] == 1 and dec([10], 9)[0] == 1  # InvalidPrefix
    for buf, p in [([10], 5), ([31, 154, 10], 5), ([0xFF, 0x80], 8), ([0xFF, 0x80, 0x80, 0x80, 0x80, 0x01], 8)]:
        try:
            v, c = hpack_ref.decode_integer(bytes(buf), p)
            assert dec(buf, p)[:3] == (0, v, c)
        except hpack_ref.DecoderError as e:
            assert dec(buf, p)[0] == {"NotEnoughOctets": 2, "TooManyOctets": 3, "InvalidPrefix": 1}[e.detail]
