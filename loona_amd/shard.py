"""Sharding a literal batch across GPUs.

Every literal is independent (Huffman results do not depend on HPACK dynamic-table state,
decoder.rs:143-157), so a batch partitions into contiguous literal ranges balanced by encoded
bytes, with u32 offsets rebased per shard. Two ways to use it:

* weak scaling (bench.py): every rank generates / owns its own shard; no data-path collective;
* root-resident batch (`scatter_decode_gather`): rank 0 holds the whole batch (e.g. literals
  gathered from many connections on one host thread), sends each rank its shard, every rank
  decodes locally, results come back to rank 0. Unequal shard sizes go point-to-point
  (send/recv), which both RCCL ("nccl") and gloo support; sizes travel first.
"""

from __future__ import annotations

import numpy as np

U32 = np.uint32


def balanced_ranges(in_off, world: int):
    """Literal index boundaries b[0..world] (b[0]=0, b[world]=n): shard r = literals
    [b[r], b[r+1]), each holding ~1/world of the encoded bytes."""
    in_off = np.asarray(in_off, dtype=np.int64)
    n = len(in_off) - 1
    if world < 1:
        raise ValueError("world must be >= 1")
    total = int(in_off[-1])
    targets = (np.arange(1, world, dtype=np.int64) * total) // world
    cuts = np.searchsorted(in_off[1:], targets, side="left") + 1 if n else np.zeros(world - 1, np.int64)
    b = np.concatenate([[0], np.minimum(cuts, n), [n]]).astype(np.int64)
    return np.maximum.accumulate(b)


def shard(blob, in_off, lo: int, hi: int):
    """Literals [lo, hi) as (blob slice, rebased u32 offsets[hi-lo+1])."""
    in_off = np.asarray(in_off, dtype=np.int64)
    a, z = int(in_off[lo]), int(in_off[hi])
    return np.asarray(blob)[a:z], (in_off[lo : hi + 1] - a).astype(U32)


def local_shard(blob, in_off, rank: int, world: int):
    b = balanced_ranges(in_off, world)
    return shard(blob, in_off, int(b[rank]), int(b[rank + 1]))


def _send_array(dist, arr, dst, device, group):
    import torch

    t = torch.from_numpy(np.ascontiguousarray(arr)).to(device)
    dist.send(t, dst, group=group)


def _recv_array(dist, count, dtype, src, device, group):
    import torch

    t = torch.empty(count, dtype=dtype, device=device)
    dist.recv(t, src, group=group)
    return t


def scatter_decode_gather(decode_fn, blob=None, in_off=None, group=None, device="cpu", root=0):
    """Root-resident batch -> per-rank shards -> decode_fn on every rank -> results on root.

    decode_fn(blob_u8, off_u32) -> (out_blob u8, out_off u32[m+1], out_len u32[m], status u8[m])
    runs on each rank's shard (numpy in, numpy out). Returns on root the concatenated
    (out_blob, out_off, out_len, status) in the original literal order; None elsewhere."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    if rank == root:
        b = balanced_ranges(in_off, world)
        shards = [shard(blob, in_off, int(b[r]), int(b[r + 1])) for r in range(world)]
        for r in range(world):
            if r == root:
                continue
            sb, so = shards[r]
            _send_array(dist, np.array([len(so) - 1, len(sb)], dtype=np.int64), r, device, group)
            _send_array(dist, so.astype(np.int64), r, device, group)
            if len(sb):
                _send_array(dist, sb, r, device, group)
        my_blob, my_off = shards[root]
    else:
        hdr = _recv_array(dist, 2, torch.int64, root, device, group).cpu().numpy()
        m, nbytes = int(hdr[0]), int(hdr[1])
        my_off = _recv_array(dist, m + 1, torch.int64, root, device, group).cpu().numpy().astype(U32)
        my_blob = (_recv_array(dist, nbytes, torch.uint8, root, device, group).cpu().numpy()
                   if nbytes else np.zeros(0, np.uint8))

    ob, oo, ol, st = decode_fn(my_blob, my_off)
    m = len(my_off) - 1
    if rank != root:
        _send_array(dist, np.array([m, int(oo[-1])], dtype=np.int64), root, device, group)
        if m:
            _send_array(dist, np.asarray(oo, np.int64), root, device, group)
            _send_array(dist, np.asarray(ol, np.int64), root, device, group)
            _send_array(dist, np.asarray(st, np.uint8), root, device, group)
            if int(oo[-1]):
                _send_array(dist, np.asarray(ob[: int(oo[-1])], np.uint8), root, device, group)
        return None
    parts = []
    for r in range(world):
        if r == root:
            parts.append((ob[: int(oo[-1])], np.asarray(oo, np.int64), np.asarray(ol, np.int64), np.asarray(st)))
            continue
        hdr = _recv_array(dist, 2, torch.int64, r, device, group).cpu().numpy()
        mr, nb = int(hdr[0]), int(hdr[1])
        if mr == 0:
            parts.append((np.zeros(0, np.uint8), np.zeros(1, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint8)))
            continue
        roo = _recv_array(dist, mr + 1, torch.int64, r, device, group).cpu().numpy()
        rol = _recv_array(dist, mr, torch.int64, r, device, group).cpu().numpy()
        rst = _recv_array(dist, mr, torch.uint8, r, device, group).cpu().numpy()
        rob = _recv_array(dist, nb, torch.uint8, r, device, group).cpu().numpy() if nb else np.zeros(0, np.uint8)
        parts.append((rob, roo, rol, rst))
    # concatenate with rebased output offsets
    out_blob = np.concatenate([p[0] for p in parts]) if parts else np.zeros(0, np.uint8)
    base = 0
    offs = [np.zeros(1, np.int64)]
    for p in parts:
        offs.append(p[1][1:] + base)
        base += int(p[1][-1])
    out_off = np.concatenate(offs)
    if out_off[-1] >= 2**32:
        raise ValueError("gathered output exceeds u32 offsets")
    return (out_blob, out_off.astype(U32), np.concatenate([p[2] for p in parts]).astype(U32),
            np.concatenate([p[3] for p in parts]).astype(np.uint8))
