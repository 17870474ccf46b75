#!/usr/bin/env python3
"""Device encode time of one synthetic workload (device-generated strings, bound-sized output
regions), checked against the decode of its output once: `python scripts/enc_time.py config3 [reps]`."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from loona_amd import HuffmanCodec, synth  # noqa: E402
from loona_amd.batch import encode_offsets_torch  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "config3"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    codec = HuffmanCodec(0)
    w = {"config2": synth.device_config2, "config3": synth.device_config3}[wl](codec)
    doff = w.dec_off.to(torch.int32)
    eoff = encode_offsets_torch(doff)
    out = torch.empty(int(eoff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
    ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
    st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
    run = lambda: codec.encode_into(w.dec_blob, doff, out, eoff, ol, st, device=True)  # noqa: E731
    run()
    torch.cuda.synchronize()
    assert not st.any().item()
    assert torch.equal(ol.to(torch.int64), w.enc_off[1:].to(torch.int64) - w.enc_off[:-1].to(torch.int64))
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(json.dumps({"workload": wl, "literals": w.n, "decoded_bytes": w.dec_bytes, "encode_us": round(us, 1),
                      "GiB_s_of_input": round(w.dec_bytes / us * 1e6 / 2**30, 2), "lengths_checked": True}), flush=True)


if __name__ == "__main__":
    main()
