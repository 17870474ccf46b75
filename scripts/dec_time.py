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
    gens = {"config2": synth.device_config2, "config3": synth.device_config3,
            "c2_4m": lambda c: synth.device_config2(c, n=4_000_000),
            "config3_text": lambda c: synth.device_config3(c, rnd=0.0),
            "config5": lambda c: synth.device_config5_shard(c, 0)}
    w = gens[wl](codec)
    compact = os.environ.get("HPK_COMPACT", "0") == "1"  # hpk_decode_batch_compact instead
    if compact:
        out, doff, ol, st = codec.decode_compact(w.enc_blob, w.enc_off)
    else:
        doff = decode_offsets_torch(w.enc_off)
        out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device="cuda")
        ol = torch.empty(w.n, dtype=torch.int32, device="cuda")
        st = torch.empty(w.n, dtype=torch.uint8, device="cuda")
        codec.decode_into(w.enc_blob, w.enc_off, out, doff, ol, st, device=True)  # binds the stream, checks args
    torch.cuda.synchronize()
    if os.environ.get("HPK_DEBUG_MODE", "0") in ("0", "3", "4", "5"):
        synth.check_decoded(w, out, doff, ol, st)
    # the raw C call with its arguments made once: Python's per-call work must not pace the launches
    import ctypes
    from loona_amd import _lib
    L = _lib.lib()
    args = (codec._h, ctypes.c_void_p(w.enc_blob.data_ptr()), w.enc_blob.numel(), ctypes.c_void_p(w.enc_off.data_ptr()),
            ctypes.c_uint32(w.n), ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.c_void_p(doff.data_ptr()),
            ctypes.c_void_p(ol.data_ptr()), ctypes.c_void_p(st.data_ptr()), _lib.HPK_PTR_DEVICE | _lib.HPK_ASYNC)
    fn = L.hpk_decode_batch_compact if compact else L.hpk_decode_batch
    run = lambda: fn(*args)  # noqa: E731
    s = torch.cuda.current_stream()
    for _ in range(int(os.environ.get("HPK_WARM", "10"))):  # untimed launches first (clocks: round 5)
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        run()
    e1.record(s)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(json.dumps({"workload": wl, "literals": w.n, "encoded_bytes": w.enc_bytes, "decode_us": round(us, 1),
                      "GiB_s": round(w.enc_bytes / us * 1e6 / 2**30, 2),
                      "checked": os.environ.get("HPK_DEBUG_MODE", "0") in ("0", "3", "4", "5"),
                      "long_min": os.environ.get("HPK_LONG_MIN", "default"),
                      "lib": os.path.basename(os.environ.get("HPK_LIB", "libhpk.so")),
                      "debug_mode": os.environ.get("HPK_DEBUG_MODE", "0"),
                      "kernel": os.environ.get("HPK_DECODE_KERNEL", "auto"),
                      "wave_variant": os.environ.get("HPK_WAVE_VARIANT"), "compact": compact,
                      "written_bytes": int(doff[-1].item()) & 0xFFFFFFFF if compact else None}), flush=True)


if __name__ == "__main__":
    main()
