#!/usr/bin/env python3
"""Small synchronous device calls for the latency trace: `python
scripts/lat_trace.py [reps]` times hpk_decode_batch on device-resident config-2 batches of 1k and
5k literals (the raw C call, arguments made once), synchronous, `reps` calls each after 20 warm
ones, and prints the median wall time per call. Run under `rocprofv3 --hip-trace --kernel-trace`
(scripts/gpu_r3q.sh) to split a call into host work, launch, kernel and synchronisation
(scripts/lat_split.py)."""
import ctypes
import json
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    codec = HuffmanCodec(0, stream="own")
    L = _lib.lib()
    small = os.environ.get("HPK_SMALL_MODE")  # "max,workgroups,idle_ms": the small-call mode (round 6)
    if small:
        mx, wgs, idle = (int(x) for x in small.split(","))
        codec.set_small_mode(mx, wgs, idle)
    w = synth.device_config2(codec, n=20000, seed=91)
    res = []
    for n in (1000, 5000, 20000):
        io = w.enc_off[: n + 1].contiguous()
        blob = w.enc_blob
        oo = decode_offsets_torch(io)
        out = torch.empty(int(oo[-1].item()) + 16, dtype=torch.uint8, device="cuda")
        ol = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        args = (codec._h, ctypes.c_void_p(blob.data_ptr()), blob.numel(), ctypes.c_void_p(io.data_ptr()),
                ctypes.c_uint32(n), ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.c_void_p(oo.data_ptr()),
                ctypes.c_void_p(ol.data_ptr()), ctypes.c_void_p(st.data_ptr()), _lib.HPK_PTR_DEVICE)
        fn = L.hpk_decode_batch
        for _ in range(20):
            assert fn(*args) == 0
        ts = []
        dv = []  # (small-call mode) the device stamps' intervals, us
        st4 = (ctypes.c_uint32 * 10)()
        for _ in range(reps):
            t0 = time.perf_counter()
            fn(*args)
            ts.append(time.perf_counter() - t0)
            if small:
                L.hpk_test_small_stamps(codec._h, st4)
                dv.append([((st4[k + 1] - st4[k]) & 0xFFFFFFFF) / 100.0 for k in range(3)] +
                          [st4[4] / max(st4[5], 1) * 0.1] + [st4[6 + k] / 2400.0 for k in range(4)])  # GHz; us
        assert not st.any().item()
        assert torch.equal(ol.to(torch.int64), (w.dec_off[1 : n + 1] - w.dec_off[:n]).to(torch.int64))
        res.append({"lib": os.path.basename(os.environ.get("HPK_LIB", "libhpk.so")), "small_mode": small or None,
                    "small_calls": int(L.hpk_test_small_calls(codec._h)) if hasattr(L, "hpk_test_small_calls") else None,
                    "literals": n, "calls": reps, "median_us": round(statistics.median(ts) * 1e6, 1),
                    "p10_us": round(sorted(ts)[reps // 10] * 1e6, 1), "p90_us": round(sorted(ts)[reps * 9 // 10] * 1e6, 1)})
        if dv:
            res[-1]["device_us_median"] = {k: round(statistics.median(x[i] for x in dv), 2)
                                           for i, k in enumerate(("broadcast", "decode_wg0", "last_publish", "sclk_ghz",
                                                                      "lit0_offsets", "lit0_staged", "lit0_walk", "lit0_stores"))}
    for r in res:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
