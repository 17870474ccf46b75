#!/usr/bin/env python3
"""device time of large literals (16 KiB to 4 MiB encoded, header text; and 256 of
64 KiB in one batch) next to one CPU
thread (the library's table-driven CPU path and the restatement of huffman.rs), every result checked
against the oracle. One JSON line per size: `python scripts/large_time.py [reps]`."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hpk_util import compare_batches, oracle_decode_batch, pack  # noqa: E402  (the checker)
from loona_amd import HuffmanCodec, huffman_encode  # noqa: E402
from loona_amd.batch import decode_batch_cpu  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    rng = np.random.default_rng(1 << 20)
    text = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789-_=;,/.:ABCDEFGHIJ ", np.uint8)
    codec = HuffmanCodec(0, stream=torch.cuda.current_stream())
    for kind in ("wave", "fill"):
        codec.set_decode_kernel(kind)
        for nb, cnt in ((16384, 1), (65536, 1), (1 << 20, 1), (4 << 20, 1), (65536, 256)):
            lit = huffman_encode(rng.choice(text, nb + nb // 3).tobytes())[:nb]
            blob, off = pack([lit] * cnt)
            ref = oracle_decode_batch(blob, off)
            db = torch.from_numpy(blob).cuda()
            do = torch.from_numpy(off.astype(np.int32)).cuda()
            out, oo, ol, st = codec.decode_device(db, do, sync=True)
            compare_batches((out.cpu().numpy(), oo.cpu().numpy().astype(np.uint32), ol[:cnt].cpu().numpy().astype(np.uint32),
                             st[:cnt].cpu().numpy()), ref, "large")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                codec.decode_into(db, do, out, oo, ol, st, device=True, sync=True)
            dev_us = (time.perf_counter() - t0) / reps * 1e6
            t0 = time.perf_counter()
            for _ in range(reps):
                c = decode_batch_cpu(blob, off, nthreads=1)
            cpu_us = (time.perf_counter() - t0) / reps * 1e6
            compare_batches(c, ref, "large cpu")
            t0 = time.perf_counter()
            oracle_decode_batch(blob, off, nthreads=1)
            ora_us = (time.perf_counter() - t0) * 1e6
            print(json.dumps({"kernel": kind, "literals": cnt, "encoded_bytes": nb * cnt, "decoded_bytes": int(ref[2].sum()),
                              "device_sync_call_us": round(dev_us, 1), "cpu_fast_1thread_us": round(cpu_us, 1),
                              "oracle_restatement_1thread_us": round(ora_us, 1),
                              "device_MBps": round(nb * cnt / dev_us, 1), "cpu_fast_MBps": round(nb * cnt / cpu_us, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
