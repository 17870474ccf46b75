#!/usr/bin/env python3
"""Per-call latency at the batch sizes one loona thread would gather (1k / 5k / 20k
literals), on config-2 literals, median of 200 calls after 20 warm ones:
  device   hpk_decode_batch on device buffers, synchronous (launch + kernel + sync)
  host     hpk_decode_batch on host buffers (H2D, kernel, D2H; pageable numpy)
  pinned   the same from hpk_host_register'ed buffers
  cpu      the library's CPU batch path, 1 thread (what a thread would do without the GPU)
  blocks   hpk_hdec_decode_blocks on interop header blocks holding about that many literals
One JSON line per (size, mode)."""
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from hpk_util import load  # noqa: E402

from loona_amd import HuffmanCodec, _lib, hpack, synth  # noqa: E402
from loona_amd.batch import decode_batch_cpu, decode_offsets_np  # noqa: E402


def med(fn, reps=200, warm=20):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e6


def main():
    L = _lib.lib()
    codec = HuffmanCodec(0, stream="own")
    w = synth.config2(n=20000, seed=77)
    inter = load("interop.json.gz")
    blocks = [bytes.fromhex(c["wire"]) for enc in sorted(inter) for st in inter[enc] for c in st["cases"]]
    for n in (1000, 5000, 20000):
        off = w.enc_off[: n + 1].copy()
        blob = w.enc_blob[: int(off[-1])].copy()
        oo = decode_offsets_np(off)
        db, do, doo = torch.from_numpy(blob).cuda(), torch.from_numpy(off.view(np.int32)).cuda(), \
            torch.from_numpy(oo.view(np.int32)).cuda()
        dout = torch.empty(int(oo[-1]) + 16, dtype=torch.uint8, device="cuda")
        dl = torch.empty(n, dtype=torch.int32, device="cuda")
        ds = torch.empty(n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        r = {"literals": n, "encoded_bytes": int(off[-1])}
        r["device_us"] = round(med(lambda: codec.decode_into(db, do, dout, doo, dl, ds, device=True, sync=True)), 1)
        hout = np.empty(int(oo[-1]) + 16, np.uint8)
        hl = np.empty(n, np.uint32)
        hs = np.empty(n, np.uint8)
        r["host_us"] = round(med(lambda: codec.decode_into(blob, off, hout, oo, hl, hs, device=False)), 1)
        for a in (blob, off, hout, oo, hl, hs):
            assert L.hpk_host_register(a.ctypes.data, a.nbytes) == 0
        r["pinned_us"] = round(med(lambda: codec.decode_into(blob, off, hout, oo, hl, hs, device=False)), 1)
        for a in (blob, off, hout, oo, hl, hs):
            L.hpk_host_unregister(a.ctypes.data)
        r["cpu_1thread_us"] = round(med(lambda: decode_batch_cpu(blob, off, nthreads=1), reps=50), 1)
        # interop blocks holding about n Huffman literals (~8.5 per block)
        nb = max(1, n * 10 // 85)
        pairs_blocks = blocks[:nb]
        decs = [hpack.Decoder() for _ in pairs_blocks]
        r["blocks"] = len(pairs_blocks)
        r["blocks_device_us"] = round(med(lambda: hpack.decode_blocks(list(zip([hpack.Decoder() for _ in pairs_blocks],
                                                                                  pairs_blocks)), codec), reps=30,
                                          warm=3), 1)
        r["blocks_cpu_us"] = round(med(lambda: hpack.decode_blocks(list(zip([hpack.Decoder() for _ in pairs_blocks],
                                                                               pairs_blocks)), None), reps=30, warm=3),
                                   1)
        del decs
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
