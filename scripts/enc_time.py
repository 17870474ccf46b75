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
    # the encoded bytes: compacted, equal to the workload's own encoding, and decoding to the strings
    enc2 = synth.gather_output(out, eoff, ol, 0, w.n)
    same = bool(torch.equal(enc2, w.enc_blob[: enc2.numel()])) and enc2.numel() == w.enc_bytes
    from loona_amd.batch import decode_offsets_torch
    e2off = torch.zeros(w.n + 1, dtype=torch.int64, device="cuda")
    e2off[1:] = torch.cumsum(ol.to(torch.int64), 0)
    e2off = e2off.to(torch.int32)
    doo = decode_offsets_torch(e2off)
    dout = torch.empty(int(doo[-1].item()) + 16, dtype=torch.uint8, device="cuda")
    dl = torch.empty(w.n, dtype=torch.int32, device="cuda")
    ds = torch.empty(w.n, dtype=torch.uint8, device="cuda")
    codec.decode_into(enc2, e2off, dout, doo, dl, ds, device=True, sync=True)
    synth.check_decoded(w, dout, doo, dl, ds)
    print(json.dumps({"workload": wl, "literals": w.n, "decoded_bytes": w.dec_bytes, "encode_us": round(us, 1),
                      "GiB_s_of_input": round(w.dec_bytes / us * 1e6 / 2**30, 2), "lengths_checked": True,
                      "bytes_equal_workload_encoding": same, "round_trip_checked": True,
                      "lib": os.path.basename(os.environ.get("HPK_LIB", "libhpk.so"))}), flush=True)


if __name__ == "__main__":
    main()
