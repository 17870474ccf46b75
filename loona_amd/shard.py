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


def _wire(t):
    """A tensor as it travels: 4-byte offsets/lengths as int32 (uint32 bit-views included), bytes as
    uint8. RCCL and gloo both carry these; nothing is widened to int64."""
    import torch

    if t.dtype == torch.uint32:
        return t.view(torch.int32)
    return t


def _p2p(dist, ops, group):
    if not ops:
        return
    reqs = dist.batch_isend_irecv([dist.P2POp(op, t, peer, group) for op, t, peer in ops])
    for r in reqs:
        r.wait()


def owner(s: int, world: int) -> int:
    """Rank that decodes shard s (round-robin)."""
    return s % world


def scatter_decode_gather(shards, decode_fn, group=None, root=0, device=None):
    """Root-resident batch -> per-rank shards -> decode_fn on every rank -> results on root.

    shards (root only; ignored elsewhere): a list of (blob uint8, off int32/uint32 [m+1]) tensors
    on `device` — a batch already cut into shards of at most 4 GiB each (u32 offsets), e.g. by
    `balanced_ranges`. Shard s is decoded on rank owner(s, world); root keeps its own.
    decode_fn(blob, off) -> (out_blob, out_off, out_len, status) tensors on `device`.

    Everything stays in device memory when `device` is a GPU (RCCL point-to-point over xGMI: one
    grouped send/recv round out, one back; no host copy): the shard sizes go out with one broadcast,
    the offsets and blob of each shard with one grouped send/recv, the decoded blob, out_off,
    out_len and status come back the same way. With gloo and CPU tensors the same code runs on the
    host (tests/test_shard.py). Returns on root the list of (out_blob, out_off, out_len, status)
    in shard order; None elsewhere."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    # 1. shard sizes, from root to every rank: [S] then S x (literals, blob bytes)
    cnt = torch.tensor([len(shards) if rank == root else 0], dtype=torch.int64, device=dev)
    dist.broadcast(cnt, root, group=group)
    S = int(cnt.item())
    if rank == root:
        meta = torch.tensor([[int(o.numel()) - 1, int(b.numel())] for b, o in shards], dtype=torch.int64,
                            device=dev).reshape(S, 2)
    else:
        meta = torch.empty((S, 2), dtype=torch.int64, device=dev)
    if S:
        dist.broadcast(meta, root, group=group)
    sizes = meta.tolist()
    mine = [s for s in range(S) if owner(s, world) == rank]
    # 2. scatter: offsets + blob of each shard to its owner
    local, ops = {}, []
    for s in range(S):
        o = owner(s, world)
        m, nb = sizes[s]
        if rank == root and o != root:
            b, off = shards[s]
            ops.append((dist.isend, _wire(off), o))
            if nb:
                ops.append((dist.isend, b, o))
        elif rank == o and o != root:
            off = torch.empty(m + 1, dtype=torch.int32, device=dev)
            b = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
            ops.append((dist.irecv, off, root))
            if nb:
                ops.append((dist.irecv, b[:nb], root))
            local[s] = (b, off)
        elif rank == root:
            local[s] = shards[s]
    _p2p(dist, ops, group)
    # 3. decode the local shards
    res = {s: decode_fn(*local[s]) for s in mine}
    # 4. gather: output sizes first, then out_off, out_len, status and the decoded blob
    hdr, ops = {}, []
    for s in range(S):
        o = owner(s, world)
        if o == root:
            continue
        if rank == o:
            ob = res[s][1]
            hdr[s] = torch.tensor([int(ob[-1].item()) & 0xFFFFFFFF], dtype=torch.int64, device=dev)
            ops.append((dist.isend, hdr[s], root))
        elif rank == root:
            hdr[s] = torch.empty(1, dtype=torch.int64, device=dev)
            ops.append((dist.irecv, hdr[s], o))
    _p2p(dist, ops, group)
    out, ops = {}, []
    for s in range(S):
        o = owner(s, world)
        m = sizes[s][0]
        if o == root:
            continue
        if rank == o:
            ob, oo, ol, st = res[s]
            nbytes = int(hdr[s].item())
            ops += [(dist.isend, _wire(oo[: m + 1]), root), (dist.isend, _wire(ol[:m]), root),
                    (dist.isend, st[:m], root)]
            if nbytes:
                ops.append((dist.isend, ob[:nbytes], root))
        elif rank == root:
            nbytes = int(hdr[s].item())
            oo = torch.empty(m + 1, dtype=torch.int32, device=dev)
            ol = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
            st = torch.empty(max(m, 1), dtype=torch.uint8, device=dev)
            ob = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
            ops += [(dist.irecv, oo, o), (dist.irecv, ol[:m], o), (dist.irecv, st[:m], o)]
            if nbytes:
                ops.append((dist.irecv, ob[:nbytes], o))
            out[s] = (ob, oo, ol[:m], st[:m])
    ops = [x for x in ops if x[1].numel()]
    _p2p(dist, ops, group)
    if rank != root:
        return None
    for s in mine:
        ob, oo, ol, st = res[s]
        m = sizes[s][0]
        out[s] = (ob, oo, ol[:m], st[:m])
    return [out[s] for s in range(S)]
