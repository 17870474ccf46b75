"""Seeded synthetic header-literal workloads (BASELINE.json configs).

Decoded strings are drawn from the empirical byte histogram of the interop fixtures' header
values (data/char_model.json; ≈0.74 encoded/decoded under the RFC 7541 code), then Huffman-
encoded by the library's own canonical encoder (hpk_encode_batch_cpu). Seeds are fixed (PCG64).

  config1  RFC 7541 App. C Huffman literals repeated 10,000x (CPU plumbing case)
  config2  1M short literals, decoded length ~ U[8,64]          (the bench workload)
  config3  1M mixed literals, decoded length ~ Zipf(1.1) over 8..4096, 5 % uniform bytes
  config5  config-2 distribution at any count (256M total over 8 GPUs, weak-scaled per rank)
"""

from __future__ import annotations

import json
import os

import numpy as np

from . import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 7541

APP_C_LITERALS = [  # RFC 7541 C.4.1-C.4.3, C.6.1-C.6.3 (hex)
    "f1e3c2e5f23a6ba0ab90f4ff", "a8eb10649cbf", "25a849e95ba97d7f", "25a849e95bb8e8b4bf", "6402", "aec3771a4b",
    "d07abe941054d444a8200595040b8166e082a62d1bff", "9d29ad171863c78f0b97c8e9ae82ae43d3", "640eff",
    "d07abe941054d444a8200595040b8166e084a62d1bff", "9bd9ab",
    "94e7821dd7f2e6c7b335dfdfcd5b3960d5af27087f3672c1ab270fb5291f9587316065c003ed4ee5b1063d5007",
]


def char_model():
    with open(os.path.join(HERE, "data", "char_model.json")) as f:
        c = np.asarray(json.load(f)["counts"], dtype=np.float64)
    return c / c.sum()


def _offsets(lens):
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    return off


def encode_cpu(dec_blob, dec_off, nthreads=0):
    """Canonical encode of a decoded batch on the host (library CPU path)."""
    L = _lib.lib()
    dec_blob = np.ascontiguousarray(dec_blob, dtype=np.uint8)
    dec_off = np.ascontiguousarray(dec_off, dtype=np.uint32)
    n = len(dec_off) - 1
    lens = np.diff(dec_off.astype(np.int64))
    bound = _offsets((lens * 30 + 7) // 8).astype(np.uint32)
    out = np.empty(max(int(bound[-1]), 1), dtype=np.uint8)
    out_len = np.empty(max(n, 1), dtype=np.uint32)
    st = np.empty(max(n, 1), dtype=np.uint8)
    src = dec_blob if dec_blob.size else np.zeros(1, np.uint8)
    _lib.check(L.hpk_encode_batch_cpu(src.ctypes.data, dec_off.ctypes.data, n, out.ctypes.data, bound.ctypes.data,
                                      out_len.ctypes.data, st.ctypes.data, nthreads), "hpk_encode_batch_cpu")
    assert not st[:n].any()
    # compact
    enc_off = _offsets(out_len[:n].astype(np.int64))
    if enc_off[-1] >= 2**32:
        raise ValueError("encoded shard exceeds 4 GiB")
    starts = bound[:-1].astype(np.int64)
    idx = np.repeat(starts - enc_off[:-1], out_len[:n].astype(np.int64)) + np.arange(enc_off[-1])
    enc_blob = out[idx] if enc_off[-1] else np.zeros(0, np.uint8)
    return enc_blob, enc_off.astype(np.uint32)


class Workload:
    """A batch: encoded literals (the decode input) plus the decoded originals."""

    def __init__(self, name, enc_blob, enc_off, dec_blob=None, dec_off=None, desc=""):
        self.name = name
        self.enc_blob, self.enc_off = enc_blob, enc_off
        self.dec_blob, self.dec_off = dec_blob, dec_off
        self.desc = desc

    @property
    def n(self):
        return len(self.enc_off) - 1

    @property
    def enc_bytes(self):
        return int(self.enc_off[-1])

    @property
    def dec_bytes(self):
        return None if self.dec_off is None else int(self.dec_off[-1])


def _strings(rng, lens, uniform_frac=0.0):
    p = char_model()
    total = int(lens.sum())
    blob = rng.choice(256, size=total, p=p).astype(np.uint8)
    if uniform_frac > 0:
        m = rng.random(total) < uniform_frac
        blob[m] = rng.integers(0, 256, size=int(m.sum()), dtype=np.uint8)
    return blob, _offsets(lens).astype(np.uint32)


def config1(reps=10_000):
    lits = [bytes.fromhex(h) for h in APP_C_LITERALS] * reps
    blob = np.frombuffer(b"".join(lits), dtype=np.uint8).copy()
    off = _offsets(np.asarray([len(x) for x in lits], dtype=np.int64)).astype(np.uint32)
    return Workload("config1", blob, off, desc=f"RFC 7541 App. C Huffman literals x{reps}")


def config2(n=1_000_000, seed=SEED):
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = rng.integers(8, 65, size=n, dtype=np.int64)
    dec_blob, dec_off = _strings(rng, lens)
    enc_blob, enc_off = encode_cpu(dec_blob, dec_off)
    return Workload("config2", enc_blob, enc_off, dec_blob, dec_off,
                    desc=f"{n} short literals, decoded len U[8,64], fixture char model")


def zipf_lengths(rng, n, s=1.1, lo=8, hi=4096):
    k = np.arange(lo, hi + 1, dtype=np.float64)
    w = 1.0 / np.power(k - lo + 1, s)
    w /= w.sum()
    return rng.choice(k.astype(np.int64), size=n, p=w)


def config3(n=1_000_000, seed=SEED + 3):
    rng = np.random.Generator(np.random.PCG64(seed))
    lens = zipf_lengths(rng, n)
    dec_blob, dec_off = _strings(rng, lens, uniform_frac=0.05)
    enc_blob, enc_off = encode_cpu(dec_blob, dec_off)
    return Workload("config3", enc_blob, enc_off, dec_blob, dec_off,
                    desc=f"{n} mixed literals, decoded len Zipf(1.1) 8..4096, 5% uniform bytes")


def config5_shard(n_total=256_000_000, world=8, rank=0, seed=SEED + 5):
    """This rank's contiguous share of the 256M config-2-distribution literals."""
    per = n_total // world
    w = config2(per, seed=seed + rank)
    w.name = "config5"
    w.desc = f"rank {rank}/{world}: {per} of {n_total} config-2 literals"
    return w
