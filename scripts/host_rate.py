#!/usr/bin/env python3
"""Host-inclusive decode rate: the path starts and ends in host memory, so time
hpk_decode_batch(HPK_PTR_HOST) end to end — H2D of in_blob + in_off + out_off, the kernel,
D2H of out_blob + out_len + status, pipelined in chunks by the library — on config 2 (1M
literals), from pageable numpy buffers and from the same buffers page-locked with
hpk_host_register. Prints one JSON line per mode (GiB/s of encoded bytes, like bench.py)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_np  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    w = synth.config2(n=n)
    L = _lib.lib()
    blob = np.ascontiguousarray(w.enc_blob)
    io = np.ascontiguousarray(w.enc_off, dtype=np.uint32)
    oo = decode_offsets_np(io)
    out = np.zeros(int(oo[-1]) + 16, np.uint8)
    ol = np.zeros(n, np.uint32)
    st = np.zeros(n, np.uint8)
    ref_len = np.diff(w.dec_off.astype(np.int64))
    host_bytes = blob.nbytes + io.nbytes + oo.nbytes + int(oo[-1]) + ol.nbytes + st.nbytes
    with HuffmanCodec(0) as c:
        for mode in ("pageable", "pinned"):
            regs = []
            if mode == "pinned":
                for a in (blob, io, oo, out, ol, st):
                    _lib.check(L.hpk_host_register(a.ctypes.data, a.nbytes), "hpk_host_register")
                    regs.append(a)
            c.decode_into(blob, io, out, oo, ol, st, device=False)  # warm (scratch, streams)
            ok = bool(np.array_equal(ol.astype(np.int64), ref_len) and not st.any())
            t0 = time.perf_counter()
            for _ in range(reps):
                c.decode_into(blob, io, out, oo, ol, st, device=False)
            dt = (time.perf_counter() - t0) / reps
            for a in regs:
                _lib.check(L.hpk_host_unregister(a.ctypes.data), "hpk_host_unregister")
            print(json.dumps({"mode": mode, "literals": n, "encoded_bytes": w.enc_bytes, "ms_per_call": round(dt * 1e3, 3),
                              "encoded_GiB_s": round(w.enc_bytes / dt / 2**30, 3),
                              "host_bytes_moved": host_bytes, "pcie_GB_s": round(host_bytes / dt / 1e9, 2),
                              "correct": ok}), flush=True)


if __name__ == "__main__":
    main()
