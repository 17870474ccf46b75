#!/usr/bin/env python3
"""Split-literal join statistics (a library built with -DHPK_SPLIT=1 -DHPK_SPLIT_DIAG=3): config 3
decoded once, then the join's counters: slots, failed walks, A EOS, mean walked bits past the split."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402

codec = HuffmanCodec(0)
w = synth.device_config3(codec)
doff = decode_offsets_torch(w.enc_off)
out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True, sync=True)
ok = True
try:
    synth.check_decoded(w, out, doff, ol, st)
except AssertionError as e:
    ok = str(e)[:200]
L = _lib.lib()
L.hpk_debug_split_stat.argtypes = [ctypes.c_void_p]
buf = np.zeros(4, np.uint64)
L.hpk_debug_split_stat(buf.ctypes.data)
print(json.dumps({"slots": int(buf[0]), "failed": int(buf[1]), "mean_walk_bits_past_split": float(buf[3]) / max(1, int(buf[0])),
                  "checked": ok, "lib": os.environ.get("HPK_LIB")}))
