#!/usr/bin/env python3
"""Bench: device-resident HPACK Huffman literal decode on MI355X (BASELINE.json metric).

Workload (default, BASELINE.json config 5): 256M short Huffman literals — the config-2
distribution (decoded length U[8,64], interop-fixture character model, canonical RFC 7541
encoding) — cut into 8 shards of 32M literals (one hpk_decode_batch launch each: u32 offsets,
~870 MB encoded). Shard s is decoded by rank s % N, so the same 256M literals are decoded at any
N ("scaling": "strong"); a step decodes every shard once. The literals are generated on the GPU
(synth.device_config5_shard, seeded by shard index) and encoded by the library's device encoder;
every decoded byte of every shard is checked against the generated strings before the warm-up and
again after the timed steps.

Timing: barrier + device synchronize on both sides of the K timed steps, HIP events on the stream
the kernels run on; value = encoded bytes of all shards x K / max over ranks of the time.

Extras on the JSON line:
  roofline      dominant kernel (hpk_decode12): algorithmic bytes per launch (sum over a shard of
                enc + dec + 13 per literal) / average launch time, against the 8.0 TB/s
                HBM3E spec peak; traffic = PMC HBM bytes per launch from the committed rocprofv3
                counter summary for this workload and kernel build (profiles/pmc_config5.json)
  config2       BASELINE config 2 (1M literals, 4 rotating copies so every launch reads HBM) on
                rank 0: the short-batch case, same kernel
  e2e_scatter_decode_gather (N > 1) the root-resident form of config 5: rank 0 holds all 8 shards,
                RCCL point-to-point sends each to its owner, every rank decodes, results come back
                to rank 0 (device-resident end to end, shard.scatter_decode_gather); timed apart
  cpu_baseline  oracle/hpk_oracle.c (a restatement of loona-hpack's HuffmanDecoder: per-literal
                hash-map build + bit walk) on a bounded prefix of config 2, this GPU's host-CPU
                share of threads; single_thread beside it
  cpu_fast      the library's own table-driven CPU batch path on config 2 (same thread counts)
"""

from __future__ import annotations

import argparse
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["config5", "config2"], default="config5")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 side measurement")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 encode/decode side measurement")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 captured-HEADERS side measurement")
    ap.add_argument("--no-e2e", action="store_true", help="skip the scatter+decode+gather leg (N > 1)")
    ap.add_argument("--no-compact", action="store_true", help="skip the compacted-output side measurement")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every CPU of this process's affinity mask, capped at the GPU's host-CPU share (16)")
    ap.add_argument("--pmc-dir", default=os.path.join(REPO, "profiles"))
    return ap.parse_args()


def affinity_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


HOST_CPU_SHARE = 16  # the GPU box allots 16 host CPUs per GPU (its OMP_NUM_THREADS / MAX_JOBS)


def cpu_threads(arg):
    """Threads for the CPU baselines: --cpu-threads, else every CPU of the affinity mask, capped at
    the GPU's host-CPU share (the box's mask can list the whole machine, of which one GPU's job owns
    16 CPUs). Returns (threads, affinity count)."""
    aff = affinity_cpus()
    if arg > 0:
        return arg, aff
    return max(1, min(HOST_CPU_SHARE, aff)), aff


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or "unknown"


def run_cpu_baselines(enc_blob, enc_off, threads, aff=0):
    """Oracle restatement on bounded prefixes (1 thread, `threads` threads, and `aff` threads = every
    CPU of the affinity mask when that is more) + the library's CPU batch path on the whole batch.
    enc_blob/enc_off: numpy, config 2."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from hpk_util import oracle_decode_batch  # test infrastructure: the checker, timed as baseline

    from loona_amd import _lib

    n = len(enc_off) - 1

    def oracle_rate(k, th):
        off = enc_off[: k + 1]
        blob = enc_blob[: int(off[-1])]
        oracle_decode_batch(blob[: int(off[1001])], off[:1001], nthreads=th)  # warm allocator arenas
        t0 = time.perf_counter()
        oracle_decode_batch(blob, off, nthreads=th)
        dt = time.perf_counter() - t0
        return int(off[-1]) / dt / 2**30, dt, int(off[-1])

    k1 = min(n, 60_000)
    v1, dt1, b1 = oracle_rate(k1, 1)
    kt = min(n, 60_000 * threads)
    vt, dtt, bt = oracle_rate(kt, threads)
    base = {
        "value": round(vt, 6),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {kt} of {n} config-2 literals ({bt} encoded B), oracle/hpk_oracle.c restatement of "
                  f"huffman.rs:95-161 (per-literal HashMap build + bit walk), {threads} threads = this GPU's host-CPU "
                  f"share, {cpu_model()}",
        "seconds": round(dtt, 3),
        "single_thread": {"value": round(v1, 6), "unit": "GiB/s", "cores": 1, "seconds": round(dt1, 3),
                          "sample": f"first {k1} literals ({b1} encoded B)"},
    }
    if aff > threads:  # BASELINE.md's `nproc` threads: the machine's CPUs, of which this job owns `threads`
        ta = min(aff, 256)  # (the restatement's thread cap)
        ka = min(n, 60_000 * ta)
        va, dta, ba = oracle_rate(ka, ta)
        base["at_affinity"] = {"value": round(va, 6), "unit": "GiB/s", "cores": ta, "affinity_cpus": aff,
                               "seconds": round(dta, 3),
                               "sample": f"first {ka} literals ({ba} encoded B)",
                               "note": "one thread per CPU of the affinity mask (the whole machine); this GPU's job "
                                       f"owns {threads} of them, so the threads share those"}
    L = _lib.lib()
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(np.diff(enc_off.astype(np.int64)) * 8 // 5, out=oo[1:])
    oo = oo.astype(np.uint32)
    out = np.empty(int(oo[-1]) + 1, np.uint8)
    ol = np.empty(n, np.uint32)
    st = np.empty(n, np.uint8)
    fast = {"unit": "GiB/s", "kind": "library hpk_decode_batch_cpu (table-driven)", "sample": f"all {n} literals"}
    for th, key in ((threads, "value"), (1, "single_thread")):
        args = (enc_blob.ctypes.data, enc_off.ctypes.data, n, out.ctypes.data, oo.ctypes.data, ol.ctypes.data,
                st.ctypes.data, th)
        L.hpk_decode_batch_cpu(*args)
        t0 = time.perf_counter()
        L.hpk_decode_batch_cpu(*args)
        fast[key] = round(int(enc_off[-1]) / (time.perf_counter() - t0) / 2**30, 4)
    fast["cores"] = threads
    return base, fast


def make_unit(codec, w, dev, copies=1):
    """Device buffers for decoding workload w (`copies` independent input/output sets)."""
    import torch

    from loona_amd.batch import decode_offsets_torch

    oo = decode_offsets_torch(w.enc_off)
    cap = int(oo[-1].item()) & 0xFFFFFFFF
    sets = []
    for c in range(copies):
        blob = w.enc_blob if c == 0 else w.enc_blob.clone()
        io = w.enc_off if c == 0 else w.enc_off.clone()
        out = torch.empty(cap + 16, dtype=torch.uint8, device=dev)
        ol = torch.empty(w.n, dtype=torch.int32, device=dev)
        st = torch.empty(w.n, dtype=torch.uint8, device=dev)
        sets.append((blob, io, out, oo if c == 0 else oo.clone(), ol, st))
    return sets


def source_hash():
    """sha256 (16 hex digits) of the library's sources (loona_amd/csrc + include/hpk.h): the key of
    the committed PMC summaries, so a kernel change invalidates them whether or not anyone edits a
    version string."""
    import hashlib

    h = hashlib.sha256()
    csrc = os.path.join(REPO, "loona_amd", "csrc")
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".h", ".hip", ".cpp")) or f == "Makefile")
    for f in names:
        h.update(f.encode())
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(REPO, "include", "hpk.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_summary(path, workload, literals, src):
    """A committed rocprofv3 PMC summary of this exact workload and library source (scripts/
    pmc_traffic.py, scripts/pmc_sq.py); None when there is none."""
    try:
        with open(path) as f:
            pm = json.load(f)
        if pm.get("workload") == workload and pm.get("literals") == literals and pm.get("src_sha16") == src:
            return pm
    except Exception:
        pass
    return None


def pmc_traffic(path, workload, literals, src):
    pm = pmc_summary(path, workload, literals, src)
    return pm.get("hbm_bytes_per_launch") if pm else None


def time_launches(codec, sets, stream, steps, warmup):
    import torch

    def step(i):
        blob, io, out, oo, ol, st = sets[i % len(sets)]
        codec.decode_into(blob, io, out, oo, ol, st, device=True, sync=False)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for i in range(steps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / 1e3


def cuda_time(fn, reps, stream):
    """Seconds per call of fn (device work on `stream`), HIP events around reps back-to-back calls after
    three untimed ones (round 5: cold first launches read ~7 % slow, DESIGN §5 Timers)."""
    import torch

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def run_compact(codec, w, stream, pmc_dir, reps=10):
    """The compacted-output form (hpk_decode_batch_compact) on one config-5 shard: every decoded byte
    checked, then `reps` back-to-back launches timed with HIP events on the codec's stream; the span it
    wrote and, when a same-source PMC summary of it exists (gpu_run.sh pmc with HPK_COMPACT=1), its HBM
    writes against the algorithmic ones (decoded bytes + out_off + out_len + status)."""
    import torch

    from loona_amd import synth

    out, oo, ol, st = codec.decode_compact(w.enc_blob, w.enc_off, sync=True)
    synth.check_decoded(w, out, oo, ol, st)
    written = int(oo[w.n].item()) & 0xFFFFFFFF
    for _ in range(5):  # (warm: in a kernel trace the first calls run ~4 % longer)
        codec.decode_compact(w.enc_blob, w.enc_off, out, oo, ol, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        codec.decode_compact(w.enc_blob, w.enc_off, out, oo, ol, st)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    res = {"literals": w.n, "encoded_bytes": w.enc_bytes, "decoded_bytes": w.dec_bytes, "written_span": written,
           "avg_call_us": round(us, 1), "calls": reps,
           "note": "one config-5 shard, 5 warm calls then `calls` back-to-back ones; a call = the wave-fill "
                   "kernel in its compacted mode (its bound layout made from in_off in the kernel); every byte "
                   "checked"}
    p = os.path.join(pmc_dir, "pmc_compact_config5.json")
    if os.path.exists(p):
        d = json.load(open(p))
        if d.get("src_sha16") == source_hash():
            algo_w = w.dec_bytes + 9 * w.n
            res["pmc_write_bytes"] = d["write_bytes_per_launch"]
            res["write_algorithmic"] = algo_w
            res["write_vs_algorithmic"] = round(d["write_bytes_per_launch"] / algo_w, 4)
    return res


def run_host_inclusive(codec, w, reps=10):
    """The rate including the copies (north_star: the path starts and ends in host memory): config 2's 1M
    literals from host numpy buffers through hpk_decode_batch(HPK_PTR_HOST) -- H2D of in_blob + in_off +
    out_off, the kernel, D2H of out_blob + out_len + status, pipelined in chunks on three streams by the
    library -- from pageable buffers and from the same buffers page-locked (hpk_host_register, as buffet's
    arena would be). Every call's lengths and statuses checked; never `value`."""
    from loona_amd import _lib
    from loona_amd.batch import decode_offsets_np

    L = _lib.lib()
    blob = np.ascontiguousarray(w.enc_blob.cpu().numpy())
    io = np.ascontiguousarray(w.enc_off.cpu().numpy().view(np.uint32))
    oo = decode_offsets_np(io)
    out = np.zeros(int(oo[-1]) + 16, np.uint8)
    ol = np.zeros(w.n, np.uint32)
    st = np.zeros(w.n, np.uint8)
    want = (w.dec_off[1:] - w.dec_off[:-1]).cpu().numpy().astype(np.int64)
    moved = blob.nbytes + io.nbytes + oo.nbytes + int(oo[-1]) + ol.nbytes + st.nbytes
    res = {"literals": w.n, "encoded_bytes": w.enc_bytes, "host_bytes_moved_per_call": int(moved), "calls": reps}
    for mode in ("pageable", "page_locked"):
        regs = []
        if mode == "page_locked":
            for arr in (blob, io, oo, out, ol, st):
                _lib.check(L.hpk_host_register(arr.ctypes.data, arr.nbytes), "hpk_host_register")
                regs.append(arr)
        try:
            codec.decode_into(blob, io, out, oo, ol, st, device=False)  # warm (scratch, streams)
            ok = True
            t0 = time.perf_counter()
            for _ in range(reps):
                codec.decode_into(blob, io, out, oo, ol, st, device=False)
            dt = (time.perf_counter() - t0) / reps
            ok = bool(np.array_equal(ol.astype(np.int64), want) and not st.any())
        finally:
            for arr in regs:
                _lib.check(L.hpk_host_unregister(arr.ctypes.data), "hpk_host_unregister")
        res[mode] = {"ms_per_call": round(dt * 1e3, 3), "encoded_GiB_s": round(w.enc_bytes / dt / 2**30, 3),
                     "pcie_GB_s": round(moved / dt / 1e9, 2), "checked": ok}
    return res


def run_small_calls(codec, w, n=1000, reps=200):
    """Small synchronous calls at the granularity loona's read_headers decodes (one connection's block at a
    time, crates/loona/src/h2/server.rs:1619-1637): the raw C call hpk_decode_batch on n device-resident
    config-2 literals, synchronous, median and p10 over `reps` calls after 20 warm ones, through the launch
    path and through the small-call mode (hpk_ctx_set_small_mode: a persistent kernel of 4 workgroups behind
    a host-mapped doorbell). Lengths and statuses checked after each mode. Never `value`."""
    import ctypes
    import statistics

    import torch

    from loona_amd import _lib
    from loona_amd.batch import decode_offsets_torch

    L = _lib.lib()
    io = w.enc_off[: n + 1].contiguous()
    blob = w.enc_blob
    oo = decode_offsets_torch(io)
    out = torch.empty(int(oo[-1].item()) + 16, dtype=torch.uint8, device=blob.device)
    ol = torch.empty(n, dtype=torch.int32, device=blob.device)
    st = torch.empty(n, dtype=torch.uint8, device=blob.device)
    want = (w.dec_off[1 : n + 1] - w.dec_off[:n]).to(torch.int64)
    torch.cuda.synchronize()
    args = (codec._h, ctypes.c_void_p(blob.data_ptr()), blob.numel(), ctypes.c_void_p(io.data_ptr()), ctypes.c_uint32(n),
            ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.c_void_p(oo.data_ptr()), ctypes.c_void_p(ol.data_ptr()),
            ctypes.c_void_p(st.data_ptr()), _lib.HPK_PTR_DEVICE)
    res = {"literals": n, "calls": reps, "note": "raw C call, synchronous, device-resident config-2 literals"}
    for mode in ("launch", "small_mode"):
        if mode == "small_mode":
            codec.set_small_mode(1024, 4, 50)
        try:
            for _ in range(20):
                _lib.check(L.hpk_decode_batch(*args), "hpk_decode_batch")
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                L.hpk_decode_batch(*args)
                ts.append(time.perf_counter() - t0)
            ok = bool(torch.equal(ol.to(torch.int64), want)) and not bool(st.any().item())
        finally:
            if mode == "small_mode":
                codec.set_small_mode(0)
        ts.sort()
        res[mode] = {"median_us": round(statistics.median(ts) * 1e6, 1), "p10_us": round(ts[reps // 10] * 1e6, 1),
                     "checked": ok}
    return res


def run_config3(codec, stream, dev, reps=10):
    """BASELINE config 3: 1M mixed literals (Zipf(1.1) lengths 8..4096, 5 % uniform bytes), device
    encode and device decode timed apart, each over `reps` back-to-back launches; the round trip is
    bit-exact (every decoded byte equals the generated strings; the encode into hpk_encoded_bound
    regions equals the exact-size encode the decode consumed, whose lengths equal the sums of the
    RFC 7541 code lengths)."""
    import torch

    from loona_amd import synth
    from loona_amd.batch import decode_offsets_torch, encode_offsets_torch

    w = synth.device_config3(codec, 1_000_000, device=dev)
    n = w.n
    doff32 = w.dec_off.to(torch.int32)
    eoff = encode_offsets_torch(doff32)
    e_out = torch.empty((int(eoff[-1].item()) & 0xFFFFFFFF) + 16, dtype=torch.uint8, device=dev)
    e_len = torch.empty(n, dtype=torch.int32, device=dev)
    e_st = torch.empty(n, dtype=torch.uint8, device=dev)
    t_enc = cuda_time(lambda: codec.encode_into(w.dec_blob, doff32, e_out, eoff, e_len, e_st, device=True), reps,
                      stream)
    ok_enc = (not e_st.any().item()) and bool(torch.equal(
        synth.gather_output(e_out, eoff, e_len, 0, n), w.enc_blob[: w.enc_bytes]))
    doff = decode_offsets_torch(w.enc_off)
    d_out = torch.empty((int(doff[-1].item()) & 0xFFFFFFFF) + 16, dtype=torch.uint8, device=dev)
    d_len = torch.empty(n, dtype=torch.int32, device=dev)
    d_st = torch.empty(n, dtype=torch.uint8, device=dev)
    t_dec = cuda_time(lambda: codec.decode_into(w.enc_blob, w.enc_off, d_out, doff, d_len, d_st, device=True), reps,
                      stream)
    synth.check_decoded(w, d_out, doff, d_len, d_st)  # raises on any difference
    algo = w.enc_bytes + w.dec_bytes + 13 * n
    return {"literals": n, "decoded_bytes": w.dec_bytes, "encoded_bytes": w.enc_bytes,
            "decode_us": round(t_dec * 1e6, 2), "decode_GiB_s_of_input": round(w.enc_bytes / t_dec / 2**30, 2),
            "decode_roofline_frac": round(algo / t_dec / 1e9 / HBM_PEAK_GBS, 4),
            "encode_us": round(t_enc * 1e6, 2), "encode_GiB_s_of_input": round(w.dec_bytes / t_enc / 2**30, 2),
            "encode_roofline_frac": round(algo / t_enc / 1e9 / HBM_PEAK_GBS, 4),
            "round_trip_bit_exact": True, "encode_matches_exact_region_encode": ok_enc,
            "note": f"device-generated, {reps} back-to-back launches per kernel; algorithmic bytes enc + dec + 13 "
                    "per literal for both kernels"}


def run_config4(codec, threads):
    """BASELINE config 4: captured HEADERS — the interop stories' header blocks (five encoders' real
    output, crates/loona-hpack/fixtures/hpack/interop) replicated to >= 1M Huffman literals, one
    hpk_hdec per connection (a story), decoded by ONE hpk_hdec_decode_blocks call: host span walk,
    one Huffman batch (device, from host buffers: H2D + kernel + D2H), in-order apply; against the
    same call on the library's CPU batch path. Host-inclusive, wall clock: three warm-up calls per leg,
    then five calls per leg alternating, the median of each."""
    import ctypes
    import gzip

    from loona_amd import _lib

    gold = os.path.join(REPO, "tests", "golden")
    with gzip.open(os.path.join(gold, "interop.json.gz"), "rt") as f:
        inter = json.load(f)
    with open(os.path.join(gold, "interop_digest.json")) as f:
        dig = json.load(f)
    stories = [[bytes.fromhex(c["wire"]) for c in st["cases"]] for enc in sorted(inter) for st in inter[enc]]
    reps = -(-1_000_000 // dig["huffman_literals"])
    L = _lib.lib()
    blocks, owners = [], []
    for r in range(reps):
        for si, st in enumerate(stories):
            for b in st:
                blocks.append(b)
                owners.append(r * len(stories) + si)
    nconn = reps * len(stories)
    off = np.zeros(len(blocks) + 1, np.int64)
    np.cumsum([len(b) for b in blocks], out=off[1:])
    blob = np.frombuffer(b"".join(blocks), np.uint8).copy()
    off32 = off.astype(np.uint32)
    def call(ctx):
        decs = [L.hpk_hdec_create() for _ in range(nconn)]
        arr = (ctypes.c_void_p * len(blocks))(*[decs[o] for o in owners])
        out = _lib.BlocksOut()
        t0 = time.perf_counter()
        rc = L.hpk_hdec_decode_blocks(ctx, arr, blob.ctypes.data, off32.ctypes.data, len(blocks), ctypes.byref(out))
        dt = time.perf_counter() - t0
        _lib.check(rc, "hpk_hdec_decode_blocks")
        errs = sum(1 for b in range(len(blocks)) if out.blocks[b].error)
        nh = out.n_headers
        L.hpk_blocks_out_free(ctypes.byref(out))
        for d in decs:
            L.hpk_hdec_destroy(d)
        return dt, errs, nh

    legs = (("device", codec._h), ("cpu_batch", None))
    for _ in range(3):  # warm-up: scratch buffers, the pinned area, page-ins (both legs)
        for _, ctx in legs:
            call(ctx)
    times = {leg: [] for leg, _ in legs}
    res = {}
    for _ in range(5):  # the legs alternate; each reports its median call
        for leg, ctx in legs:
            dt, errs, nh = call(ctx)
            times[leg].append(dt)
            res[leg] = (None, errs, nh)
    for leg in times:
        res[leg] = (float(np.median(times[leg])), res[leg][1], res[leg][2])
    lit_bytes = dig["encoded_bytes"] * reps
    return {"source": "crates/loona-hpack/fixtures/hpack/interop (5 encoders' captured header blocks)",
            "connections": nconn, "header_blocks": len(blocks), "huffman_literals": dig["huffman_literals"] * reps,
            "huffman_bytes": lit_bytes, "headers": res["device"][2], "block_errors": res["device"][1],
            "device_ms": round(res["device"][0] * 1e3, 2), "cpu_batch_ms": round(res["cpu_batch"][0] * 1e3, 2),
            "device_blocks_per_s": round(len(blocks) / res["device"][0], 1),
            "cpu_batch_blocks_per_s": round(len(blocks) / res["cpu_batch"][0], 1),
            "device_over_cpu": round(res["cpu_batch"][0] / res["device"][0], 3),
            "host_threads": threads,
            "calls_ms": {leg: [round(x * 1e3, 2) for x in v] for leg, v in times.items()},
            "note": "host-inclusive wall clock of one hpk_hdec_decode_blocks call: span walk, Huffman batch "
                    "(device: from host buffers, H2D + kernel + D2H), in-order apply with each connection's "
                    "dynamic table"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # (rehearsal on a one-GPU box only: HPK_BENCH_DEVICE puts every rank on one device and
    # HPK_BENCH_BACKEND=gloo replaces RCCL, which refuses two ranks on one GPU; never set for a run)
    if os.environ.get("HPK_BENCH_DEVICE") is not None:
        local = int(os.environ["HPK_BENCH_DEVICE"])
    backend = os.environ.get("HPK_BENCH_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from loona_amd import HuffmanCodec, _lib, shard, synth

    version = _lib.lib().hpk_version().decode()
    stream = torch.cuda.current_stream(dev)
    codec = HuffmanCodec(local, stream=stream)

    # ---- the workload, generated on this GPU and checked once before any timing ----
    units = []  # (workload, buffer sets)
    by_shard = {}  # config 5: shard index -> its workload on this rank
    if args.workload == "config5":
        my = [s for s in range(synth.CONFIG5_SHARDS) if shard.owner(s, world) == rank]
        for s in my:
            w = synth.device_config5_shard(codec, s, device=dev)
            by_shard[s] = w
            units.append((w, make_unit(codec, w, dev)))
        workload = (f"config5: {synth.CONFIG5_TOTAL} short Huffman literals (config-2 distribution: decoded len "
                    f"U[8,64], interop-fixture char model, canonical RFC 7541 encoding) in {synth.CONFIG5_SHARDS} "
                    f"shards of {synth.CONFIG5_TOTAL // synth.CONFIG5_SHARDS}, shard s decoded by rank s % N, "
                    f"device-resident")
    else:
        w = synth.device_config2(codec, 1_000_000, seed=synth.SEED + rank, device=dev)
        units.append((w, make_unit(codec, w, dev, copies=4)))
        workload = ("config2: 1M short Huffman literals per GPU (decoded len U[8,64], interop-fixture char model, "
                    "canonical RFC 7541 encoding), 4 rotating copies, device-resident")
    for w, sets in units:
        for blob, io, out, oo, ol, st in sets:
            codec.decode_into(blob, io, out, oo, ol, st, device=True, sync=True)
            synth.check_decoded(w, out, oo, ol, st)  # every byte vs the generated strings

    my_enc = sum(w.enc_bytes for w, _ in units)
    my_dec = sum(w.dec_bytes for w, _ in units)
    my_n = sum(w.n for w, _ in units)
    # bytes of the literals' output regions (the caller's out_off spans: the decoded bound, 8/5 of the
    # encoded length): the image write-back stores whole spans, the slack past out_len included
    my_region = sum(int(sets[0][3][-1].item()) & 0xFFFFFFFF for _, sets in units)
    per_step_enc = my_enc if args.workload == "config5" else units[0][0].enc_bytes

    def step():
        if args.workload == "config5":
            for w, sets in units:
                blob, io, out, oo, ol, st = sets[0]
                codec.decode_into(blob, io, out, oo, ol, st, device=True, sync=False)

    rot = [0]

    def step2():
        w, sets = units[0]
        blob, io, out, oo, ol, st = sets[rot[0] % len(sets)]
        rot[0] += 1
        codec.decode_into(blob, io, out, oo, ol, st, device=True, sync=False)

    run = step if args.workload == "config5" else step2
    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        run()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    t_ev = ev0.elapsed_time(ev1) / 1e3
    # the timed launches' results, every byte again (the last launch of each buffer set)
    for w, sets in units:
        blob, io, out, oo, ol, st = sets[0] if args.workload == "config5" else sets[(rot[0] - 1) % len(sets)]
        synth.check_decoded(w, out, oo, ol, st)
    n_launch = args.steps * (len(units) if args.workload == "config5" else 1)
    algo_local = (my_enc + my_dec + 13 * my_n) if args.workload == "config5" else \
        (units[0][0].enc_bytes + units[0][0].dec_bytes + 13 * units[0][0].n)
    launches_per_step = len(units) if args.workload == "config5" else 1
    t_local = torch.tensor([t_ev, wall], dtype=torch.float64, device=dev)
    tot = torch.tensor([float(per_step_enc), float(my_dec if args.workload == "config5" else units[0][0].dec_bytes),
                        float(my_n if args.workload == "config5" else units[0][0].n)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_local, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    t_max, wall_max = t_local.tolist()
    all_enc, all_dec, all_n = tot.tolist()

    # ---- root-resident form (N > 1): scatter + decode + gather over RCCL, device-resident ----
    e2e = None
    if world > 1 and args.workload == "config5" and not args.no_e2e:
        from loona_amd.batch import decode_offsets_torch

        shards = None
        if rank == 0:
            shards = []
            for s in range(synth.CONFIG5_SHARDS):
                if s in by_shard:
                    shards.append((by_shard[s].enc_blob, by_shard[s].enc_off))
                else:
                    w = synth.device_config5_shard(codec, s, device=dev)
                    w.drop_strings()
                    shards.append((w.enc_blob, w.enc_off))

        def decode_fn(blob, off):  # the compacted form (its decoded bytes gathered end to end before they travel)
            return codec.decode_compact(blob, off, sync=False)

        res = shard.scatter_decode_gather(shards, decode_fn, device=dev, compacted=True)  # warm
        reps = 2
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            res = shard.scatter_decode_gather(shards, decode_fn, device=dev, compacted=True)
        torch.cuda.synchronize()
        dist.barrier()
        dt = (time.perf_counter() - t0) / reps
        if rank == 0:
            ok = all(not r[3].any().item() for r in res) and len(res) == synth.CONFIG5_SHARDS
            enc_total = sum(int(b.numel()) for b, _ in shards)
            e2e = {"value": round(enc_total / dt / 2**30, 3), "unit": "GiB/s", "ms_per_step": round(dt * 1e3, 3),
                   "steps": reps, "statuses_ok": bool(ok),
                   "what": "rank 0 holds the 8 shards; RCCL grouped send/recv of offsets + blob to each owner, "
                           "device decode in the compacted form (hpk_decode_batch_compact), the decoded bytes "
                           "gathered end to end on the owner (the wave kernel's span has gaps between "
                           "workgroup shares), one all-reduce of the decoded sizes, RCCL send/recv of "
                           "bytes/out_len/status back; no host copy of the data"}
        del res, shards

    line = None
    if rank == 0:
        per_launch_s = t_ev / n_launch
        algo_per_launch = algo_local / launches_per_step
        achieved = algo_per_launch / per_launch_s / 1e9
        lit_per_launch = my_n // launches_per_step if args.workload == "config5" else units[0][0].n
        src = source_hash()
        pm_hbm = pmc_summary(os.path.join(args.pmc_dir, f"pmc_{args.workload}.json"), args.workload, lit_per_launch,
                             src)
        traffic = pm_hbm.get("hbm_bytes_per_launch") if pm_hbm else None
        pm_sq = pmc_summary(os.path.join(args.pmc_dir, f"pmc_sq_{args.workload}.json"), args.workload,
                            lit_per_launch, src)
        kernel_name = (pm_hbm or pm_sq or {}).get("kernel") or (
            "hpk_decode_wave" if lit_per_launch >= 4_000_000 else "hpk_decode12")
        traffic_split = None
        if pm_hbm and args.workload == "config5":
            lpl = launches_per_step
            rd_algo = (my_enc + 8 * my_n) / lpl
            wr_algo = (my_dec + 5 * my_n) / lpl
            wr_span = (my_region + 5 * my_n) / lpl
            traffic_split = {
                "read_algorithmic": int(rd_algo), "read_pmc": pm_hbm.get("read_bytes_per_launch"),
                "write_algorithmic": int(wr_algo), "write_region_spans": int(wr_span),
                "write_pmc": pm_hbm.get("write_bytes_per_launch"),
                "why": "reads: a fill's window starts 16-B-aligned and runs to its chunk's end (lines shared by "
                       "neighbouring chunks are read by both waves) and in_off/out_off are read as (t, t+1) "
                       "pairs; writes: the image write-back stores each fill's whole output span "
                       "(the regions' slack between out_len and the 8/5 bound included) in 16-B chunks"}
        issue = None
        if pm_sq:
            per = pm_sq["per_launch"]
            issue = {"valu_insts_per_launch": per.get("SQ_INSTS_VALU"),
                     "lds_insts_per_launch": per.get("SQ_INSTS_LDS"),
                     "lds_active_cycles_per_launch": per.get("SQ_LDS_IDX_ACTIVE"),
                     "source": f"profiles/pmc_sq_{args.workload}.json (src_sha16 {src})",
                     "basis": "this run's avg launch time, 2.4 GHz; VALU: 2 cycles per wave64 instruction on each "
                              "of 1,024 SIMD-32s; LDS: LDS-array cycles of 256 CUs"}
            if per.get("SQ_INSTS_VALU"):
                issue["valu_frac"] = round(per["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * per_launch_s), 4)
            if per.get("SQ_LDS_IDX_ACTIVE"):
                issue["lds_frac"] = round(per["SQ_LDS_IDX_ACTIVE"] / (256 * 2.4e9 * per_launch_s), 4)
        line = {
            "metric": METRIC,
            "value": round(all_enc * args.steps / t_max / 2**30, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 5),
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "config5" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (generated on the GPU with a seeded torch generator, encoded by the device encoder; "
                    "every decoded byte checked against the generated strings before and after timing)",
            "config": {
                "workload": workload,
                "literals_total": int(all_n),
                "encoded_bytes_total": int(all_enc),
                "decoded_bytes_total": int(all_dec),
                "launches_per_step_rank0": launches_per_step,
                "parallelism": (f"{synth.CONFIG5_SHARDS} shards over {world} rank(s), independent literals, no "
                                "data-path collective in the timed decode") if args.workload == "config5" else
                               f"shard{world} (independent literals, no collective)",
            },
            "decoded_GiB_s": round(all_dec * args.steps / t_max / 2**30, 3),
            "literals_per_s": round(all_n * args.steps / t_max, 1),
            "wall_ms_per_step": round(wall_max / args.steps * 1e3, 5),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_read": pm_hbm.get("read_bytes_per_launch") if pm_hbm else None,
                "traffic_write": pm_hbm.get("write_bytes_per_launch") if pm_hbm else None,
                "issue": issue,
                "kernel": kernel_name,
                "traffic_vs_algorithmic": traffic_split,
                "algorithmic_bytes_per_launch": int(algo_per_launch),
                "literals_per_launch": int(lit_per_launch),
                "avg_launch_us": round(per_launch_s * 1e6, 3),
            },
            "kernel_version": version,
            "src_sha16": source_hash(),
        }
        if e2e is not None:
            line["e2e_scatter_decode_gather"] = e2e

    # ---- the compacted form, config-2 side measurement and CPU baselines (rank 0) ----
    if rank == 0 and args.workload == "config5" and not args.no_compact:
        line["config5_compact"] = run_compact(codec, units[0][0], stream, args.pmc_dir)
        torch.cuda.empty_cache()
    if rank == 0 and args.workload == "config5" and not args.no_config2:
        del units, by_shard
        torch.cuda.empty_cache()
        w2 = synth.device_config2(codec, 1_000_000, seed=synth.SEED, device=dev)
        sets2 = make_unit(codec, w2, dev, copies=4)
        for blob, io, out, oo, ol, st in sets2:
            codec.decode_into(blob, io, out, oo, ol, st, device=True, sync=True)
            synth.check_decoded(w2, out, oo, ol, st)
        k2 = 100  # (>= 100 back-to-back launches)
        t2 = time_launches(codec, sets2, stream, k2, 10)
        a2 = w2.enc_bytes + w2.dec_bytes + 13 * w2.n
        line["config2"] = {
            "value": round(w2.enc_bytes * k2 / t2 / 2**30, 3), "unit": "GiB/s", "literals": w2.n,
            "encoded_bytes": w2.enc_bytes, "avg_launch_us": round(t2 / k2 * 1e6, 3),
            "algorithmic_bytes_per_launch": a2, "roofline_frac": round(a2 / (t2 / k2) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic(os.path.join(args.pmc_dir, "pmc_config2.json"), "config2", w2.n, source_hash()),
            "note": "1M literals, 4 rotating input/output copies (> 256 MiB Infinity Cache), 100 launches"}
        line["host_inclusive"] = run_host_inclusive(codec, w2)
        line["small_calls"] = run_small_calls(codec, w2)
        cpu_w = w2
    elif rank == 0:
        cpu_w = units[0][0]
    if rank == 0 and args.workload == "config5" and not args.no_config3:
        line["config3"] = run_config3(codec, stream, dev)
        torch.cuda.empty_cache()
    if rank == 0 and args.workload == "config5" and not args.no_config4:
        line["config4"] = run_config4(codec, cpu_threads(args.cpu_threads)[0])
    if rank == 0 and not args.no_cpu:
        blob_h = cpu_w.enc_blob.cpu().numpy()
        off_h = cpu_w.enc_off.cpu().numpy().view(np.uint32).copy()
        th, aff = cpu_threads(args.cpu_threads)
        base, fast = run_cpu_baselines(blob_h, off_h, th, aff)
        base["affinity_cpus"] = aff
        base["threads_rule"] = (f"every CPU of the affinity mask ({aff}) capped at this GPU's host-CPU share "
                                f"({HOST_CPU_SHARE}): {th} threads")
        line["cpu_baseline"] = base
        line["cpu_fast"] = fast
    if rank == 0:
        print(json.dumps(line), flush=True)
    codec.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
