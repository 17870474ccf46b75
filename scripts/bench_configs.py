#!/usr/bin/env python3
"""The BASELINE.json configs other than the headline one, measured on one MI355X.

One JSON line per config (and per leg), into stdout:
  config1  RFC 7541 App. C Huffman literals x10k, CPU only: the oracle restatement of loona-hpack's
           decoder (1 thread, like loona's per-connection decode) and the library's CPU batch path
  config3  1M mixed literals (Zipf 8..4096, 5 % uniform bytes): device encode, device decode
           (device-resident, GiB/s of the bytes each kernel consumes), round trip == input checked
           on the whole batch, device encode == oracle encode on a sample
  config4  captured HEADERS: the interop stories' header blocks (real encoder output) replicated
           to >= 1M Huffman literals, one hpk_hdec per connection: host span walk + ONE device
           Huffman batch + in-order apply (hpk_hdec_decode_blocks), against the same call with the
           library's CPU batch path
  config5  this GPU's share of the 256M-literal job at 8 GPUs (32M config-2 literals, the 1M
           synthetic batch tiled 32x on the device): decode GiB/s at that shard size
Inputs are synthetic and seeded (loona_amd.synth) or the reference's own interop fixtures.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

import torch  # noqa: E402

from loona_amd import HuffmanCodec, _lib, synth  # noqa: E402
from loona_amd.batch import decode_offsets_torch, encode_offsets_torch  # noqa: E402


def emit(d):
    print(json.dumps(d), flush=True)


def cuda_time(fn, reps, stream):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def config1():
    from hpk_util import oracle_decode_batch  # the oracle: test infrastructure, timed as the baseline

    w = synth.config1()
    t0 = time.perf_counter()
    oracle_decode_batch(w.enc_blob, w.enc_off, nthreads=1)
    t_or = time.perf_counter() - t0
    L = _lib.lib()
    n = w.n
    oo = np.zeros(n + 1, np.int64)
    np.cumsum(np.diff(w.enc_off.astype(np.int64)) * 8 // 5, out=oo[1:])
    oo = oo.astype(np.uint32)
    out = np.empty(int(oo[-1]) + 1, np.uint8)
    ol = np.empty(n, np.uint32)
    st = np.empty(n, np.uint8)
    t0 = time.perf_counter()
    L.hpk_decode_batch_cpu(w.enc_blob.ctypes.data, w.enc_off.ctypes.data, n, out.ctypes.data, oo.ctypes.data,
                           ol.ctypes.data, st.ctypes.data, 1)
    t_fast = time.perf_counter() - t0
    assert not st.any()
    emit({"config": "config1", "literals": n, "encoded_bytes": w.enc_bytes,
          "oracle_restated_GiB_s_1thread": round(w.enc_bytes / t_or / 2**30, 4),
          "library_cpu_GiB_s_1thread": round(w.enc_bytes / t_fast / 2**30, 4),
          "note": "CPU only (plumbing case); oracle = restatement of huffman.rs with its per-literal map build"})


def config3(codec, stream):
    from hpk_util import compare_batches, oracle_encode_batch

    w = synth.config3()
    dev = torch.device("cuda", 0)
    d_dec = torch.from_numpy(w.dec_blob).to(dev)
    d_doff = torch.from_numpy(w.dec_off.astype(np.int64)).to(dev)
    d_doff32 = d_doff.to(torch.int32)
    eoff = encode_offsets_torch(d_doff32)
    e_out = torch.empty(int(eoff[-1].item()) + 16, dtype=torch.uint8, device=dev)
    e_len = torch.empty(w.n, dtype=torch.int32, device=dev)
    e_st = torch.empty(w.n, dtype=torch.uint8, device=dev)
    t_enc = cuda_time(lambda: codec.encode_into(d_dec, d_doff32, e_out, eoff, e_len, e_st, device=True), 5, stream)
    assert not e_st.any().item()
    # compact the encoded literals (the decode input), then decode them
    lens = e_len.to(torch.int64)
    enc_off = torch.zeros(w.n + 1, dtype=torch.int64, device=dev)
    torch.cumsum(lens, 0, out=enc_off[1:])
    idx = torch.repeat_interleave(eoff[:-1].to(torch.int64) - enc_off[:-1], lens) + torch.arange(
        int(enc_off[-1].item()), device=dev)
    enc_blob = e_out[idx]
    enc_off32 = enc_off.to(torch.int32)
    doff = decode_offsets_torch(enc_off32)
    d_out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device=dev)
    d_len = torch.empty(w.n, dtype=torch.int32, device=dev)
    d_st = torch.empty(w.n, dtype=torch.uint8, device=dev)
    t_dec = cuda_time(lambda: codec.decode_into(enc_blob, enc_off32, d_out, doff, d_len, d_st, device=True), 5, stream)
    # the same batch as the CPU encoder wrote it (a cross-check of the decode time)
    c_blob = torch.from_numpy(w.enc_blob).to(dev)
    c_off = torch.from_numpy(w.enc_off.astype(np.int64)).to(dev).to(torch.int32)
    t_dec_cpu_enc = cuda_time(lambda: codec.decode_into(c_blob, c_off, d_out, doff, d_len, d_st, device=True), 5, stream)
    codec.decode_into(enc_blob, enc_off32, d_out, doff, d_len, d_st, device=True)
    ok_st = not d_st.any().item()
    ok_len = bool(torch.equal(d_len.to(torch.int64), d_doff[1:] - d_doff[:-1]))
    dl = d_len.to(torch.int64)
    idx2 = torch.repeat_interleave(doff[:-1].to(torch.int64) - d_doff[:-1], dl) + torch.arange(int(d_doff[-1].item()),
                                                                                                device=dev)
    ok_bytes = bool(torch.equal(d_out[idx2], d_dec))
    # device encode == oracle encode on a 20k sample
    k = 20000
    so = w.dec_off[: k + 1]
    sub = (e_out.cpu().numpy(), eoff[: k + 1].cpu().numpy().astype(np.uint32), e_len[:k].cpu().numpy().astype(np.uint32),
           e_st[:k].cpu().numpy())
    compare_batches(sub, oracle_encode_batch(w.dec_blob[: int(so[-1])], so), "config3 encode sample")
    enc_bytes = int(enc_off[-1].item())
    emit({"config": "config3", "literals": w.n, "decoded_bytes": w.dec_bytes, "encoded_bytes": enc_bytes,
          "encode_us": round(t_enc * 1e6, 1), "encode_GiB_s_of_input": round(w.dec_bytes / t_enc / 2**30, 2),
          "decode_us": round(t_dec * 1e6, 1), "decode_GiB_s_of_input": round(enc_bytes / t_dec / 2**30, 2),
          "decode_us_cpu_encoded_copy": round(t_dec_cpu_enc * 1e6, 1),
          "round_trip_bit_exact": ok_st and ok_len and ok_bytes, "encode_matches_oracle_sample": k})


def config4(codec):
    from hpk_util import interop_literals, load  # interop fixtures: the reference's captured blocks

    inter = load("interop.json.gz")
    stories = [[bytes.fromhex(c["wire"]) for c in st["cases"]] for enc in sorted(inter) for st in inter[enc]]
    lits_per_rep = len(interop_literals())
    reps = -(-1_000_000 // lits_per_rep)
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
    res = {}
    for leg, ctx in (("device", codec._h), ("cpu_batch", None)):
        for rep in range(2):  # the first call grows the context's scratch buffers: time the second
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
        res[leg] = (dt, errs, nh)
    lit_bytes = sum(len(x) for x in interop_literals()) * reps
    emit({"config": "config4", "source": "crates/loona-hpack/fixtures/hpack/interop (5 encoders' captured blocks)",
          "connections": nconn, "header_blocks": len(blocks), "huffman_literals": lits_per_rep * reps,
          "huffman_bytes": lit_bytes, "headers": res["device"][2], "errors": res["device"][1],
          "device_blocks_per_s": round(len(blocks) / res["device"][0], 1),
          "device_literal_GiB_s": round(lit_bytes / res["device"][0] / 2**30, 4),
          "cpu_batch_blocks_per_s": round(len(blocks) / res["cpu_batch"][0], 1),
          "note": "host-inclusive: span walk, H2D/D2H of the literal batch, one device decode, in-order apply"})


def config5(codec, stream, tiles=32):
    w = synth.config2()
    dev = torch.device("cuda", 0)
    base = torch.from_numpy(w.enc_blob).to(dev)
    off1 = torch.from_numpy(w.enc_off.astype(np.int64)).to(dev)
    eb = w.enc_bytes
    blob = base.repeat(tiles)
    off = torch.cat([off1[:-1] + t * eb for t in range(tiles)] + [off1[-1:] + (tiles - 1) * eb])
    off32 = off.to(torch.int32) if int(off[-1].item()) < 2**31 else off.to(torch.uint32)
    doff = decode_offsets_torch(off32)
    out = torch.empty(int(doff[-1].item()) + 16, dtype=torch.uint8, device=dev)
    n = w.n * tiles
    ol = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    t = cuda_time(lambda: codec.decode_into(blob, off32, out, doff, ol, st, device=True), 5, stream)
    ok = (not st.any().item()) and bool(torch.equal(ol[: w.n].to(torch.int64).cpu(),
                                                     torch.from_numpy(np.diff(w.dec_off.astype(np.int64)))))
    emit({"config": "config5", "literals_this_gpu": n, "encoded_bytes": eb * tiles,
          "decode_us": round(t * 1e6, 1), "decode_GiB_s": round(eb * tiles / t / 2**30, 2),
          "lengths_ok": ok, "note": "one GPU's share of 256M literals over 8 GPUs (weak-scaled shard)"})


def main():
    which = sys.argv[1:] or ["config1", "config3", "config4", "config5"]
    stream = torch.cuda.current_stream()
    with HuffmanCodec(0, stream=stream) as c:
        for cfg in which:
            if cfg == "config1":
                config1()
            elif cfg == "config3":
                config3(c, stream)
            elif cfg == "config4":
                config4(c)
            elif cfg == "config5":
                config5(c, stream)


if __name__ == "__main__":
    main()
