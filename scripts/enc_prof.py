#!/usr/bin/env python3
"""Diagnostics for the encode kernel (not part of the product): cycles per phase of hpk_encode2,
summed over waves, from the diagnostic library's HPK_ENCODE_CFG=9 variant:
`python scripts/enc_prof.py config3`. One JSON line (phase shares of the total)."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("HPK_LIB", os.path.join(REPO, "loona_amd", "libhpk_diag.so"))
os.environ["HPK_ENCODE_CFG"] = "9"

import numpy as np  # noqa: E402
import torch  # noqa: E402

from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import encode_offsets_torch  # noqa: E402

PHASES = ["top", "meta_fits", "setup", "pass1", "scan", "pass2", "finalize", "writeback", "split", "unused9",
          "unused10", "barrier_waits"]  # (v5: the barriers' waits apart from the phases' work)


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "config3"
    codec = HuffmanCodec(0)
    w = {"config2": synth.device_config2, "config3": synth.device_config3}[wl](codec)
    doff = w.dec_off.to(torch.int32)
    eoff = encode_offsets_torch(doff)
    out = torch.empty(int(eoff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
    ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
    st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        codec.encode_into(w.dec_blob, doff, out, eoff, ol, st, device=True)
    torch.cuda.synchronize()
    assert not st.any().item()
    L = _lib.lib()
    L.hpk_debug_encode_prof.argtypes = [ctypes.c_void_p]
    buf = np.zeros(16, np.uint64)
    assert L.hpk_debug_encode_prof(buf.ctypes.data) == 0
    tot = float(buf[:12].sum())
    print(json.dumps({"workload": wl, "cycles_total": tot,
                      "share": {p: round(float(buf[i]) / tot, 4) for i, p in enumerate(PHASES)}}), flush=True)


if __name__ == "__main__":
    main()
