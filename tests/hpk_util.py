"""Test helpers: the C oracle (oracle/liboracle.so, test infrastructure only) and golden loaders."""

import ctypes
import gzip
import json
import os
import sys

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "oracle"))

import hpack_ref  # noqa: E402  (pure-Python oracle)

_oracle = None


def oracle():
    global _oracle
    if _oracle is None:
        # HPK_ORACLE_LIB: the sanitizer build of the same oracle (scripts/sanitize.sh)
        L = ctypes.CDLL(os.environ.get("HPK_ORACLE_LIB", os.path.join(REPO, "oracle", "liboracle.so")))
        L.oracle_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_decode.restype = ctypes.c_int
        L.oracle_encode.argtypes = L.oracle_decode.argtypes
        L.oracle_encode.restype = ctypes.c_int
        for fn in (L.oracle_decode_batch, L.oracle_encode_batch):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
            fn.restype = None
        L.oracle_table.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_table.restype = ctypes.c_int
        L.oracle_decode_integer.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_size_t)]
        L.oracle_decode_integer.restype = ctypes.c_int
        _oracle = L
    return _oracle


def oracle_decode(buf: bytes):
    L = oracle()
    cap = len(buf) * 8 // 5
    out = ctypes.create_string_buffer(max(cap, 1))
    ol = ctypes.c_size_t(0)
    st = L.oracle_decode(bytes(buf), len(buf), out, cap, ctypes.byref(ol))
    return st, out.raw[: ol.value]


def oracle_encode(buf: bytes):
    L = oracle()
    cap = (len(buf) * 30 + 7) // 8
    out = ctypes.create_string_buffer(max(cap, 1))
    ol = ctypes.c_size_t(0)
    assert L.oracle_encode(bytes(buf), len(buf), out, cap, ctypes.byref(ol)) == 0
    return out.raw[: ol.value]


def bound_offsets(in_off, num, den, add):
    in_off = np.asarray(in_off, dtype=np.int64)
    b = (np.diff(in_off) * num + add) // den
    out = np.zeros(len(in_off), dtype=np.int64)
    np.cumsum(b, out=out[1:])
    return out.astype(np.uint32)


def oracle_decode_batch(blob, off, nthreads=8):
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    n = len(off) - 1
    oo = bound_offsets(off, 8, 5, 0)
    out = np.zeros(max(int(oo[-1]), 1), np.uint8)
    ol = np.zeros(max(n, 1), np.uint32)
    st = np.zeros(max(n, 1), np.uint8)
    src = blob if blob.size else np.zeros(1, np.uint8)
    oracle().oracle_decode_batch(src.ctypes.data, off.ctypes.data, n, out.ctypes.data, oo.ctypes.data,
                                 ol.ctypes.data, st.ctypes.data, nthreads)
    return out, oo, ol[:n], st[:n]


def oracle_encode_batch(blob, off, nthreads=8):
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    n = len(off) - 1
    oo = bound_offsets(off, 30, 8, 7)
    out = np.zeros(max(int(oo[-1]), 1), np.uint8)
    ol = np.zeros(max(n, 1), np.uint32)
    st = np.zeros(max(n, 1), np.uint8)
    src = blob if blob.size else np.zeros(1, np.uint8)
    oracle().oracle_encode_batch(src.ctypes.data, off.ctypes.data, n, out.ctypes.data, oo.ctypes.data,
                                 ol.ctypes.data, st.ctypes.data, nthreads)
    return out, oo, ol[:n], st[:n]


def load(name):
    p = os.path.join(GOLDEN, name)
    if name.endswith(".gz"):
        with gzip.open(p) as f:
            return json.load(f)
    with open(p) as f:
        return json.load(f)


_interop_lits = None


def interop_literals():
    """Every Huffman literal of the interop corpus, in corpus order (list of bytes)."""
    global _interop_lits
    if _interop_lits is None:
        inter = load("interop.json.gz")
        lits = []
        for enc in inter:
            for story in inter[enc]:
                for c in story["cases"]:
                    w = bytes.fromhex(c["wire"])
                    for s, e in hpack_ref.huffman_literal_spans(w):
                        lits.append(w[s:e])
        _interop_lits = lits
    return _interop_lits


def pack(lits):
    lens = np.asarray([len(x) for x in lits], dtype=np.int64)
    off = np.zeros(len(lits) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    blob = np.frombuffer(b"".join(lits), dtype=np.uint8).copy()
    return blob, off.astype(np.uint32)


def compare_batches(a, b, what=""):
    """(out_blob, out_off, out_len, status) pairs: identical status, length and valid bytes."""
    oa, ooa, la, sa = a
    ob, oob, lb, sb = b
    n = len(la)
    assert len(lb) == n
    bad = np.nonzero(sa != sb)[0]
    assert bad.size == 0, f"{what}: status differs at {bad[:10]} ({sa[bad[:10]]} vs {sb[bad[:10]]})"
    bad = np.nonzero(la != lb)[0]
    assert bad.size == 0, f"{what}: out_len differs at {bad[:10]} ({la[bad[:10]]} vs {lb[bad[:10]]})"
    # gather valid bytes of each side into compact streams and compare
    def compact(out, oo, ln):
        ln = ln.astype(np.int64)
        starts = np.asarray(oo[:-1], dtype=np.int64)
        tot = int(ln.sum())
        if tot == 0:
            return np.zeros(0, np.uint8)
        ends = np.cumsum(ln)
        idx = np.repeat(starts - (ends - ln), ln) + np.arange(tot)
        return out[idx]
    ca, cb = compact(oa, ooa, la), compact(ob, oob, lb)
    if not np.array_equal(ca, cb):
        first = int(np.nonzero(ca != cb)[0][0])
        lit = int(np.searchsorted(np.cumsum(la.astype(np.int64)), first, side="right"))
        raise AssertionError(f"{what}: decoded bytes differ (first at byte {first}, literal {lit})")
