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


# ---------------------------------------------------------------------------------------------
# Device-side generation for the full-size configs (config 5's 32M-literal shards, config 3 at
# 1M): the same distributions as above, drawn with torch's CUDA generator (seeded, deterministic
# per seed and device type) instead of numpy, and encoded by the library's device encoder into
# exact-size regions, so a 32M-literal shard (1.15 GB of strings) is made in well under a second.
# The encoder is parity-tested against the oracle (tests/test_gpu.py); the tests and the bench
# check every decoded byte against the generated strings.


def code_lengths():
    """Bits of each byte's RFC 7541 code (from the library's encoded-length function)."""
    L = _lib.lib()
    return np.array([L.hpk_huffman_encoded_len(bytes([b]) * 8, 8) for b in range(256)], np.int64)


class DeviceWorkload:
    """A batch resident on one GPU: enc_blob/enc_off (the decode input, int32 offsets),
    dec_blob/dec_off (the generated strings, int64 offsets) as torch tensors."""

    def __init__(self, name, enc_blob, enc_off, dec_blob, dec_off, desc=""):
        self.name, self.desc = name, desc
        self.enc_blob, self.enc_off = enc_blob, enc_off
        self.dec_blob, self.dec_off = dec_blob, dec_off
        self.n = int(enc_off.shape[0]) - 1
        self.enc_bytes = int(enc_off[-1].item())
        self.dec_bytes = int(dec_off[-1].item())

    def drop_strings(self):
        self.dec_blob = self.dec_off = None


def _device_strings(g, lens, uniform_frac, device, chunk=1 << 26):
    import torch

    p = char_model()
    cdf = torch.tensor(np.cumsum(p), dtype=torch.float64, device=device)
    cdf[-1] = 2.0  # every u < 1 maps to a byte
    off = torch.zeros(lens.numel() + 1, dtype=torch.int64, device=device)
    torch.cumsum(lens, 0, out=off[1:])
    total = int(off[-1].item())
    blob = torch.empty(total, dtype=torch.uint8, device=device)
    for s in range(0, total, chunk):
        m = min(chunk, total - s)
        u = torch.rand(m, generator=g, device=device, dtype=torch.float64)
        part = torch.searchsorted(cdf, u, right=True).clamp_(max=255).to(torch.uint8)
        if uniform_frac > 0:
            mask = torch.rand(m, generator=g, device=device) < uniform_frac
            part[mask] = torch.randint(0, 256, (int(mask.sum().item()),), generator=g, device=device,
                                       dtype=torch.int64).to(torch.uint8)
        blob[s : s + m] = part
    return blob, off


def _device_encode(codec, dec_blob, dec_off, chunk=1 << 26):
    """Exact encoded lengths (sums of code lengths, device cumsums per chunk of literals), then one
    device encode into regions of exactly that size."""
    import torch

    dev = dec_blob.device
    lens_tab = torch.tensor(code_lengths(), dtype=torch.int64, device=dev)
    n = dec_off.numel() - 1
    bits = torch.empty(n, dtype=torch.int64, device=dev)
    # literal ranges of about `chunk` bytes
    cuts = torch.searchsorted(dec_off, torch.arange(0, int(dec_off[-1].item()) + chunk, chunk, device=dev)).tolist()
    cuts = sorted(set([0] + [min(c, n) for c in cuts] + [n]))
    for a, b in zip(cuts[:-1], cuts[1:]):
        if a == b:
            continue
        x0, x1 = int(dec_off[a].item()), int(dec_off[b].item())
        cs = torch.zeros(x1 - x0 + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens_tab[dec_blob[x0:x1].to(torch.int64)], 0, out=cs[1:])
        o = dec_off[a : b + 1] - x0
        bits[a:b] = cs[o[1:]] - cs[o[:-1]]
    enc_len = (bits + 7) // 8
    enc_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(enc_len, 0, out=enc_off[1:])
    if int(enc_off[-1].item()) >= 2**31 or int(dec_off[-1].item()) >= 2**31:
        raise ValueError("device workloads keep int32 offsets: shard too large")
    enc_off32 = enc_off.to(torch.int32)
    enc_blob = torch.empty(max(int(enc_off[-1].item()), 1), dtype=torch.uint8, device=dev)
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    codec.encode_into(dec_blob, dec_off.to(torch.int32), enc_blob, enc_off32, ol, st, device=True, sync=True)
    if st.any().item() or not torch.equal(ol.to(torch.int64), enc_len):
        raise RuntimeError("device encode of the synthetic batch disagrees with the code-length sums")
    return enc_blob, enc_off32


def device_config2(codec, n=1_000_000, seed=SEED, device="cuda"):
    """Config-2 distribution (decoded length U[8,64], fixture character model) made on the GPU."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    lens = torch.randint(8, 65, (n,), generator=g, device=device, dtype=torch.int64)
    dec_blob, dec_off = _device_strings(g, lens, 0.0, device)
    enc_blob, enc_off = _device_encode(codec, dec_blob, dec_off)
    return DeviceWorkload("config2", enc_blob, enc_off, dec_blob, dec_off,
                          desc=f"{n} short literals, decoded len U[8,64], fixture char model (device-generated)")


def device_config3(codec, n=1_000_000, seed=SEED + 3, device="cuda", rnd=0.05):
    """Config-3 distribution (Zipf(1.1) lengths 8..4096, 5 % uniform bytes) made on the GPU (rnd: the
    uniform-bytes fraction, for measurements)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    k = np.arange(8, 4097, dtype=np.float64)
    w = torch.tensor(1.0 / np.power(k - 7, 1.1), dtype=torch.float64, device=device)
    lens = torch.multinomial(w, n, replacement=True, generator=g) + 8
    dec_blob, dec_off = _device_strings(g, lens, rnd, device)
    enc_blob, enc_off = _device_encode(codec, dec_blob, dec_off)
    return DeviceWorkload("config3", enc_blob, enc_off, dec_blob, dec_off,
                          desc=f"{n} mixed literals, Zipf(1.1) 8..4096, 5% uniform bytes (device-generated)")


CONFIG5_TOTAL = 256_000_000
CONFIG5_SHARDS = 8  # 32M literals each: one launch's u32-offset shard


def config5_shard_seed(s):
    return SEED + 5000 + s


def device_config5_shard(codec, s, device="cuda"):
    """Shard s (0..7) of config 5: 32M config-2-distribution literals, the same data whichever GPU
    of however many makes it (seeded by the shard index)."""
    w = device_config2(codec, CONFIG5_TOTAL // CONFIG5_SHARDS, seed=config5_shard_seed(s), device=device)
    w.name = "config5"
    w.desc = f"config-5 shard {s}/{CONFIG5_SHARDS}: {w.n} config-2 literals (device-generated)"
    return w


def gather_output(out_blob, out_off, out_len, a, b):
    """Decoded bytes of literals [a, b) of a device decode, concatenated (torch, on the device)."""
    import torch

    ln = out_len[a:b].to(torch.int64)
    st = out_off[a:b].to(torch.int64) & 0xFFFFFFFF
    tot = int(ln.sum().item())
    if tot == 0:
        return torch.zeros(0, dtype=torch.uint8, device=out_blob.device)
    excl = torch.cumsum(ln, 0) - ln
    idx = torch.repeat_interleave(st - excl, ln) + torch.arange(tot, device=out_blob.device)
    return out_blob[idx]


def check_decoded(w, out_blob, out_off, out_len, status, chunk=1 << 22):
    """Every literal decoded OK and every decoded byte equals the generated string (device-side)."""
    import torch

    if status[: w.n].any().item():
        raise AssertionError("a literal of the synthetic batch did not decode OK")
    want_len = (w.dec_off[1:] - w.dec_off[:-1])
    if not torch.equal(out_len[: w.n].to(torch.int64), want_len):
        raise AssertionError("decoded lengths differ from the generated strings")
    for a in range(0, w.n, chunk):
        b = min(w.n, a + chunk)
        got = gather_output(out_blob, out_off, out_len, a, b)
        if not torch.equal(got, w.dec_blob[int(w.dec_off[a].item()) : int(w.dec_off[b].item())]):
            raise AssertionError(f"decoded bytes differ from the generated strings in literals [{a}, {b})")
