#!/usr/bin/env python3
"""Bench: device-resident HPACK Huffman literal decode on MI355X (BASELINE.json metric).

One step = one hpk_decode_batch launch over this rank's whole batch of config-2 literals
(1M short literals, decoded length U[8,64], fixture character model) already
resident in HBM. Timed with HIP events on the stream the kernel runs on, between a barrier +
device synchronize on both sides; rank 0 prints one JSON line with the max over ranks.

Multi-GPU (`--gpus N` under torch.distributed.run): weak scaling, each rank decodes its own
1M-literal shard (independent literals, no data-path collective); value = all ranks' encoded
bytes / max time.

Extras on the JSON line:
  roofline      dominant kernel (hpk_decode12): algorithmic bytes per launch
                (sum of enc + dec + 13 per literal) / average launch time, against
                the 8.0 TB/s HBM3E spec peak; traffic = PMC HBM bytes per launch from the
                committed rocprofv3 counter summary (profiles/), null when absent
  cpu_baseline  oracle/hpk_oracle.c ("ref-restated": per-literal hash-map build + bit walk, as
                loona-hpack's HuffmanDecoder) on a bounded prefix of the same batch, host threads
  cpu_fast      the library's own table-driven CPU batch path on the whole batch (same threads)
"""

from __future__ import annotations

import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Huffman header-literal decode GiB/s (device-resident) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s spec, 6.29 measured)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--literals", type=int, default=1_000_000, help="literals per GPU (config 2: 1M)")
    ap.add_argument("--rotate", type=int, default=4,
                    help="distinct input/output copies cycled per step (4 x 84 MB > 256 MiB Infinity Cache)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpus)")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_decode.json"))
    return ap.parse_args()


def cpu_threads(arg):
    if arg > 0:
        return arg
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def run_cpu_baselines(w, threads):
    """Oracle restatement on a bounded prefix + library CPU path on the whole batch."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from hpk_util import oracle_decode_batch  # test infrastructure: the checker, timed as baseline

    from loona_amd import _lib

    # bounded sample: ~40k literals per thread (~1 s of wall, tens of CPU-seconds)
    k = min(w.n, max(50_000, 40_000 * threads))
    off = w.enc_off[: k + 1]
    blob = w.enc_blob[: int(off[-1])]
    oracle_decode_batch(blob[: int(off[1001])], off[:1001], nthreads=threads)  # warm allocator arenas
    t0 = time.perf_counter()
    oracle_decode_batch(blob, off, nthreads=threads)
    dt = time.perf_counter() - t0
    base = {
        "value": round(int(off[-1]) / dt / 2**30, 6),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {k} of the {w.n} config-2 literals ({int(off[-1])} encoded B), oracle/hpk_oracle.c "
                  f"restatement of huffman.rs:95-161 (per-literal HashMap build + bit walk), {threads} threads, "
                  f"{cpu_model()}",
        "seconds": round(dt, 3),
    }
    # library CPU fast path on the whole batch
    L = _lib.lib()
    n = w.n
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(np.diff(w.enc_off.astype(np.int64)) * 8 // 5, out=oo[1:])
    oo = oo.astype(np.uint32)
    out = np.empty(int(oo[-1]) + 1, np.uint8)
    ol = np.empty(n, np.uint32)
    st = np.empty(n, np.uint8)
    L.hpk_decode_batch_cpu(w.enc_blob.ctypes.data, w.enc_off.ctypes.data, n, out.ctypes.data, oo.ctypes.data,
                           ol.ctypes.data, st.ctypes.data, threads)
    t0 = time.perf_counter()
    L.hpk_decode_batch_cpu(w.enc_blob.ctypes.data, w.enc_off.ctypes.data, n, out.ctypes.data, oo.ctypes.data,
                           ol.ctypes.data, st.ctypes.data, threads)
    dt2 = time.perf_counter() - t0
    fast = {"value": round(w.enc_bytes / dt2 / 2**30, 4), "unit": "GiB/s", "cores": threads,
            "kind": "library hpk_decode_batch_cpu (table-driven)", "sample": f"all {n} literals"}
    return base, fast


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from loona_amd import HuffmanCodec, _lib, synth

    w = synth.config2(n=args.literals, seed=synth.SEED + rank)
    n = w.n
    enc_b, dec_b = w.enc_bytes, w.dec_bytes
    algo_bytes = enc_b + dec_b + 13 * n  # enc + dec + in_off + out_off + out_len + status

    stream = torch.cuda.current_stream(dev)
    codec = HuffmanCodec(local, stream=stream)
    R = max(1, args.rotate)
    d_in_off = torch.from_numpy(w.enc_off.astype(np.int64)).to(torch.int32).to(dev)
    from loona_amd.batch import decode_offsets_torch

    d_out_off = decode_offsets_torch(d_in_off)
    out_cap = int(d_out_off[-1].item())
    copies = []
    for r in range(R):
        blob = torch.from_numpy(w.enc_blob).to(dev)
        io = d_in_off.clone()
        oo = d_out_off.clone()
        out = torch.empty(out_cap + 16, dtype=torch.uint8, device=dev)
        ol = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        copies.append((blob, io, out, oo, ol, st))
    torch.cuda.synchronize()

    def step(i):
        blob, io, out, oo, ol, st = copies[i % R]
        codec.decode_into(blob, io, out, oo, ol, st, device=True, sync=False)

    for i in range(args.warmup):
        step(i)
    # correctness gate on the warm path: all literals decode, lengths match the generator
    torch.cuda.synchronize()
    chk_len = copies[0][4].cpu().numpy().astype(np.int64)
    if copies[0][5].any().item() or not np.array_equal(chk_len, np.diff(w.dec_off.astype(np.int64))):
        print(json.dumps({"error": "decode mismatch in bench warmup"}), flush=True)
        sys.exit(2)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    ev_ms = ev0.elapsed_time(ev1)
    t_local = torch.tensor([ev_ms / 1e3, wall], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(enc_b), float(dec_b), float(n), float(algo_bytes)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_local, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    t_ev, t_wall = t_local.tolist()
    all_enc, all_dec, all_n, all_algo = tot.tolist()

    if rank == 0:
        per_launch_s = t_ev / args.steps
        achieved = algo_bytes / per_launch_s / 1e9
        traffic = None
        if os.path.exists(args.pmc):
            try:
                with open(args.pmc) as f:
                    pm = json.load(f)
                # only a summary of this exact kernel build on this workload counts
                if pm.get("literals") == n and pm.get("kernel_version") == _lib.lib().hpk_version().decode():
                    traffic = pm.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        line = {
            "metric": METRIC,
            "value": round(all_enc * args.steps / t_ev / 2**30, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_ev / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": "config2: 1M short Huffman literals per GPU (decoded len U[8,64], interop-fixture "
                            "char model, canonical RFC 7541 encoding), decode, device-resident",
                "literals_per_gpu": n,
                "encoded_bytes_per_gpu": enc_b,
                "decoded_bytes_per_gpu": dec_b,
                "rotate_copies": R,
                "parallelism": f"shard{world} (independent literals, no collective)",
            },
            "decoded_GiB_s": round(all_dec * args.steps / t_ev / 2**30, 3),
            "literals_per_s": round(all_n * args.steps / t_ev, 1),
            "wall_ms_per_step": round(t_wall / args.steps * 1e3, 5),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "hpk_decode12",
                "algorithmic_bytes_per_launch": algo_bytes,
                "avg_launch_us": round(per_launch_s * 1e6, 3),
            },
            "kernel_version": _lib.lib().hpk_version().decode(),
        }
        if not args.no_cpu:
            base, fast = run_cpu_baselines(w, cpu_threads(args.cpu_threads))
            line["cpu_baseline"] = base
            line["cpu_fast"] = fast
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
