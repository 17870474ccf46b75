#!/usr/bin/env python3
"""Device decode time of one synthetic workload (device-generated, device-resident), checked
against the generated strings once: `python scripts/dec_time.py config3 [reps]`. One JSON line.
HPK_LIB selects the library (e.g. loona_amd/libhpk_diag.so for the diagnostic modes)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from loona_amd import HuffmanCodec, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "config3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    codec = HuffmanCodec(0)
    w = {"config2": synth.device_config2, "config3": synth.device_config3}[wl](codec)
    doff = decode_offsets_torch(w.enc_off)
    out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
    ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
    st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
    run = lambda: codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True)  # noqa: E731
    run()
    torch.cuda.synchronize()
    synth.check_decoded(w, out, doff, ol, st)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(json.dumps({"workload": wl, "literals": w.n, "encoded_bytes": w.enc_bytes, "decode_us": round(us, 1),
                      "GiB_s": round(w.enc_bytes / us * 1e6 / 2**30, 2), "checked": True,
                      "long_min": os.environ.get("HPK_LONG_MIN", "default")}), flush=True)


if __name__ == "__main__":
    main()
