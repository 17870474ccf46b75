#!/usr/bin/env python3
"""Write a decode-harness input file (bench/kvariants): u32 n, u32 enc_bytes, u32 in_off[n+1], blob."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from loona_amd import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
path = sys.argv[2] if len(sys.argv) > 2 else "/tmp/kin.bin"
n = int(sys.argv[3]) if len(sys.argv) > 3 else None
if cfg.startswith("interop"):  # the interop corpus' Huffman literals (interop_long: >= 224 B only)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from hpk_util import interop_literals, pack  # noqa: E402

    lits = [x for x in interop_literals() if cfg == "interop" or len(x) >= 224]
    blob, off = pack(lits * (n or 1))
    w = synth.Workload(cfg, blob, off)
elif cfg == "mixlong":  # long literals with every error path (tests/test_gpu.py test_long_literals' mix)
    from loona_amd import huffman_encode  # noqa: E402
    from loona_amd.batch import pack  # noqa: E402

    rng = np.random.default_rng(2025)
    lits = []
    for k in rng.integers(224, 6000, size=3000):
        r = rng.random()
        if r < 0.4:
            lits.append(huffman_encode(rng.integers(0, 256, int(k), dtype=np.uint8).tobytes()))
        elif r < 0.7:
            lits.append(huffman_encode(rng.choice(np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;, ", np.uint8),
                                                  int(k)).tobytes()))
        elif r < 0.85:
            lits.append(rng.integers(0, 256, int(k), dtype=np.uint8).tobytes())  # random bytes: padding / EOS errors
        else:
            body = bytearray(huffman_encode(b"accept-encoding: gzip, deflate" * int(k // 30 + 1)))
            body[int(rng.integers(0, len(body)))] = 0xFF
            lits.append(bytes(body))
        lits.append(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8).tobytes())
    lits.append(b"\xff" * 3000)
    lits.append(huffman_encode(bytes([1]) * 800))
    lits.append(huffman_encode(bytes(range(256)) * 40))
    blob, off = pack(lits)
    w = synth.Workload(cfg, blob, off)
else:
    w = getattr(synth, cfg)() if n is None else getattr(synth, cfg)(n=n)
with open(path, "wb") as f:
    np.array([w.n, w.enc_bytes], np.uint32).tofile(f)
    w.enc_off.astype(np.uint32).tofile(f)
    w.enc_blob.tofile(f)
print(path, w.n, w.enc_bytes)
