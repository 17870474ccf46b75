#!/usr/bin/env python3
"""Per-wave phase stamps of the workgroup-fill decode kernel (diagnostic build, HPK_DEBUG_MODE=3,
HPK_DECODE_KERNEL=fill) on a small batch, where a call's time is the kernel's fixed chain rather
than its work: `python scripts/fill_stamps.py [literals]`. One JSON line: the kernel's event time and
the mean / max s_memtime cycles per wave of each phase (hpk_decode12.h, mode 3)."""
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
os.environ["HPK_DECODE_KERNEL"] = "fill"
from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
codec = HuffmanCodec(0, stream=torch.cuda.current_stream())
w = synth.device_config2(codec, n=n)
doff = decode_offsets_torch(w.enc_off)
out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
for _ in range(20):
    codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True, sync=True)
synth.check_decoded(w, out, doff, ol, st)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
times = []
for _ in range(50):
    ev0.record()
    codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True, sync=False)
    ev1.record()
    torch.cuda.synchronize()
    times.append(ev0.elapsed_time(ev1) * 1e3)
L = _lib.lib()
L.hpk_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
buf = np.zeros(256 * 16 * 16, np.uint64)
got = L.hpk_debug_stamps(buf.ctypes.data, buf.size)
s = buf[:got].reshape(-1, 16).astype(np.int64)
s = s[s[:, 0] > 0]  # the waves of the launched workgroups
names = {0: "total", 1: "decode_loop", 2: "steps", 3: "fill_top_barrier_waits", 4: "before_first_fill", 5: "setup_a", 6: "setup_b",
         10: "byte_path", 11: "last_write_back", 12: "setup_b_to_window", 13: "setup_b_to_prefetch",
         14: "setup_b_to_write_back_issue"}
res = {"literals": n, "kernel_event_us_median": round(float(np.median(times)), 2), "waves": int(s.shape[0])}
for i, nm in names.items():
    res[nm] = {"mean": round(float(s[:, i].mean()), 1), "max": int(s[:, i].max())}
print(json.dumps(res), flush=True)
