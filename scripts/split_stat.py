#!/usr/bin/env python3
"""Dev tool (diagnostic build): config-3 decode time at several split thresholds and the split join's
outcomes (met / A ended with an EOS / rest decoded by one lane, mean meeting distance in bits).
HPK_LIB=loona_amd/libhpk_diag.so HPK_SPLIT_MIN=... python scripts/split_stat.py"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402

L = _lib.lib()
codec = HuffmanCodec(0)
w = synth.device_config3(codec)
doff = decode_offsets_torch(w.enc_off)
out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
buf = (ctypes.c_ulonglong * 4)()
L.hpk_debug_split_stat(buf)
before = list(buf)
codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True, sync=True)
L.hpk_debug_split_stat(buf)
d = [b - a for a, b in zip(before, buf)]
if not os.environ.get("NO_CHECK"):
    synth.check_decoded(w, out, doff, ol, st)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True, sync=False)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"split_min": os.environ.get("HPK_SPLIT_MIN", "default"), "decode_us": round(e0.elapsed_time(e1) / 5 * 1e3, 1),
                  "met": d[0], "a_eos": d[1], "rest": d[2], "mean_meet_bits": round(d[3] / max(d[0], 1), 1)}))
