#!/usr/bin/env python3
"""Diagnostics for the decode kernel (not part of the product): time one kernel variant
(HPK_DEBUG_MODE env) on the config-2 batch (DIAG_CONFIG=config3 for the mixed one) and, in mode 3, dump per-wave timestamps."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the diagnostic kernel variants live only in libhpk_diag.so (`make -C loona_amd/csrc diag`)
os.environ.setdefault("HPK_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                              "loona_amd", "libhpk_diag.so"))
from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402

mode = int(os.environ.get("HPK_DEBUG_MODE", "0"))
n = int(os.environ.get("DIAG_N", "1000000"))
w = getattr(synth, os.environ.get("DIAG_CONFIG", "config2"))(n=n)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    codec = HuffmanCodec(0, stream=s)
    blob = torch.from_numpy(w.enc_blob).cuda()
    io = torch.from_numpy(w.enc_off.astype(np.int32)).cuda()
    oo = decode_offsets_torch(io)
    out = torch.empty(int(oo[-1].item()) + 16, dtype=torch.uint8, device="cuda")
    ol = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    for _ in range(5):
        codec.decode_into(blob, io, out, oo, ol, st)
    s.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    K = 20
    for _ in range(K):
        codec.decode_into(blob, io, out, oo, ol, st)
    e1.record(s)
    s.synchronize()
    us = e0.elapsed_time(e1) / K * 1e3
res = {"config": w.name, "mode": mode, "us_per_launch": round(us, 2)}
if mode in (0, 2, 3, 4, 5):
    ok = bool((st.cpu().numpy() == 0).all()) and np.array_equal(ol.cpu().numpy(), np.diff(w.dec_off.astype(np.int64)))
    res["lengths_ok"] = ok
if mode == 4:
    L = _lib.lib()
    L.hpk_debug_check.argtypes = [ctypes.c_void_p]
    chk = np.zeros(8, np.uint64)
    L.hpk_debug_check(chk.ctypes.data)
    res["check"] = [int(x) for x in chk]
if mode == 3:
    L = _lib.lib()
    L.hpk_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(256 * 16 * 16, np.uint64)
    got = L.hpk_debug_stamps(buf.ctypes.data, buf.size)
    st8 = buf[:got].reshape(-1, 16).astype(np.int64)
    names = ["total", "decode", "steps", "barrier_wait", "pre", "setupA", "setupB", "long", "setupA_fill0",
             "setupB_fill0", "byte_pass", "last_flush", "setupB_to_window", "setupB_to_prefetch", "setupB_to_flush"]
    res["stamps_per_wave"] = {nm: {"mean": round(float(st8[:, i].mean()), 1), "max": int(st8[:, i].max())}
                              for i, nm in enumerate(names)}
if mode == 5:  # hpk_decode_long's per-wave counters
    L = _lib.lib()
    L.hpk_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros(256 * 16 * 16, np.uint64)
    got = L.hpk_debug_stamps(buf.ctypes.data, buf.size)
    st8 = buf[:got].reshape(-1, 16).astype(np.int64)
    names = ["cycles", "points", "lane_steps", "stalled", "idle_no_literal", "assign_cyc", "step_cyc", "refill_cyc", "-",
             "idle_first_chunks", "idle_ended", "ringwrite_wait_cyc"]
    res["long_per_wave"] = {nm: {"mean": round(float(st8[:, i].mean()), 1), "max": int(st8[:, i].max()),
                                 "min": int(st8[:, i].min())} for i, nm in enumerate(names)}
    # (round 6) per workgroup (8 long-phase waves each): its slowest wave and its total lane-steps, to tell
    # imbalance across workgroups from imbalance inside one
    if st8.shape[0] % 8 == 0:
        g = st8.reshape(-1, 8, 16)
        wmax, wmean, work = g[:, :, 0].max(1), g[:, :, 0].mean(1), g[:, :, 2].sum(1)
        res["per_workgroup"] = {
            "slowest_wave_cycles": {"mean": round(float(wmax.mean()), 1), "max": int(wmax.max()), "min": int(wmax.min())},
            "mean_wave_cycles": {"mean": round(float(wmean.mean()), 1), "max": round(float(wmean.max()), 1)},
            "lane_steps": {"mean": round(float(work.mean()), 1), "max": int(work.max()), "min": int(work.min())},
            "corr_lane_steps_slowest": round(float(np.corrcoef(work, wmax)[0, 1]), 3),
            "top8_slowest": [int(x) for x in np.sort(wmax)[-8:]]}
print(json.dumps(res), flush=True)
