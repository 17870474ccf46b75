#!/usr/bin/env python3
"""Per-wave phase stamps of the v25 wave-fill decode kernel (diagnostic build, HPK_DEBUG_MODE=3,
HPK_DECODE_KERNEL=wave): `python scripts/wave_stamps.py [config5|c2_4m|config2]`. One JSON line: mean
cycles per wave in each phase and its share of the wave's total."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("HPK_LIB", os.path.join(REPO, "loona_amd", "libhpk_diag.so"))
os.environ["HPK_DEBUG_MODE"] = "3"
os.environ.setdefault("HPK_DECODE_KERNEL", "wave")
from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "config5"
codec = HuffmanCodec(0)
gens = {"config2": synth.device_config2, "c2_4m": lambda c: synth.device_config2(c, n=4_000_000),
        "config5": lambda c: synth.device_config5_shard(c, 0)}
w = gens[wl](codec)
doff = decode_offsets_torch(w.enc_off)
out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
for _ in range(3):
    codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True, sync=True)
synth.check_decoded(w, out, doff, ol, st)
L = _lib.lib()
L.hpk_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(256 * 16 * 16, np.uint64)
got = L.hpk_debug_stamps(buf.ctypes.data, buf.size)
s = buf[:got].reshape(-1, 16).astype(np.int64)
names = ["total", "offsets_wait", "write_back", "queue", "window", "prefetch_issue_qread", "lane_loop",
         "byte_path_results", "fills", "loop_rounds", "long_phase", "before_first_fill"]
tot = s[:, 0].mean()
res = {"workload": wl, "kernel": os.environ["HPK_DECODE_KERNEL"], "waves": int(s.shape[0])}
for i, nm in enumerate(names):
    res[nm] = {"mean": round(float(s[:, i].mean()), 1), "max": int(s[:, i].max()), "min": int(s[:, i].min())}
    if i not in (0, 8, 9):
        res[nm]["share"] = round(float(s[:, i].mean() / tot), 4)
print(json.dumps(res), flush=True)
