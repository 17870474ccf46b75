"""Sharding a literal batch across GPUs.

Every literal is independent (Huffman results do not depend on HPACK dynamic-table state,
decoder.rs:143-157), so a batch partitions into contiguous literal ranges balanced by encoded
bytes, with u32 offsets rebased per shard. Two ways to use it:

* weak scaling (bench.py): every rank generates / owns its own shard; no data-path collective;
* root-resident batch (`scatter_decode_gather`): rank 0 holds the whole batch (e.g. literals
  gathered from many connections on one host thread), sends each rank its shard, every rank
  decodes locally, results come back to rank 0. Unequal shard sizes go point-to-point
  (send/recv); sizes travel first. The backend must carry the tensors' device: RCCL ("nccl") for
  GPU tensors, gloo for CPU tensors (gloo has no point-to-point for device tensors: posted anyway,
  the sends never complete). A mismatch is refused before the first collective.
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


def _check(t, name, kinds):
    """Refuse, before any message is posted, a tensor the receiving side would misread: the receiver
    allocates int32 / uint8 buffers from the sizes alone, so an int64 offset tensor or a strided view
    would be a size mismatch on the wire (an RCCL hang, or garbage), not an error."""
    dt = str(t.dtype).replace("torch.", "")
    if dt not in kinds:
        raise ValueError(f"{name}: dtype {dt} not in {kinds}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")


def _p2p(dist, ops, group):
    if not ops:
        return
    reqs = dist.batch_isend_irecv([dist.P2POp(op, t, peer, group) for op, t, peer in ops])
    for r in reqs:
        r.wait()


def owner(s: int, world: int) -> int:
    """Rank that decodes shard s (round-robin)."""
    return s % world


def compact_offsets(out_len, m):
    """int64 offsets [m + 1] of m literals' decoded bytes laid end to end (exclusive sum of out_len)."""
    import torch

    off = torch.zeros(m + 1, dtype=torch.int64, device=out_len.device)
    if m:
        torch.cumsum(out_len[:m].to(torch.int64), 0, out=off[1:])
    return off


def compact(out_blob, out_off, out_len, m, total, chunk=1 << 28):
    """The decoded bytes of m literals (literal i at out_off[i], out_len[i] bytes: the region layout a
    decode writes) laid end to end: a uint8 tensor of `total` bytes on the same device. Built in
    pieces of ~`chunk` bytes so the index tensor stays bounded; the pieces' literal and byte bounds
    come to the host in ONE read (total is known, so nothing else waits on the device)."""
    import torch

    dev = out_blob.device
    res = torch.empty(max(total, 1), dtype=torch.uint8, device=dev)
    if total == 0 or m == 0:
        return res[:0]
    ln = out_len[:m].to(torch.int64)
    src = out_off[:m].to(torch.int64) & 0xFFFFFFFF
    coff = compact_offsets(out_len, m)
    # literal ranges of about `chunk` output bytes each: cut indices and their byte offsets together
    cuts = torch.searchsorted(coff, torch.arange(0, total + chunk, chunk, device=dev, dtype=torch.int64))
    cuts = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), cuts.clamp_(max=m),
                      torch.full((1,), m, dtype=torch.int64, device=dev)])
    host = torch.stack([cuts, coff[cuts]]).tolist()  # the one host read
    bounds = sorted(set(zip(host[0], host[1])))
    for (a, x0), (b, x1) in zip(bounds[:-1], bounds[1:]):
        if a == b or x1 == x0:
            continue
        idx = torch.repeat_interleave(src[a:b] - (coff[a:b] - x0), ln[a:b], output_size=x1 - x0)
        idx += torch.arange(x1 - x0, device=dev, dtype=torch.int64)
        res[x0:x1] = out_blob[idx]
    return res


def check_backend(dist, group, dev):
    """Refuse a backend that cannot carry tensors on `dev` (every rank makes the same test, so all of
    them raise, before any message is posted): gloo has no device-tensor point-to-point (posted
    anyway, the sends never complete: gpurun_out/rehearse2/n2_e2e.json of round 3), RCCL no host
    tensors."""
    be = str(dist.get_backend(group)).lower()
    if dev.type == "cuda" and be == "gloo":
        raise ValueError("scatter_decode_gather: the gloo backend cannot send device tensors; use nccl (RCCL)")
    if dev.type == "cpu" and be == "nccl":
        raise ValueError("scatter_decode_gather: the nccl (RCCL) backend cannot send host tensors; use gloo")


def scatter_decode_gather(shards, decode_fn, group=None, root=0, device=None, compacted=False):
    """Root-resident batch -> per-rank shards -> decode_fn on every rank -> results on root.

    shards (root only; ignored elsewhere): a list of (blob uint8, off int32/uint32 [m+1]) tensors
    on `device` — a batch already cut into shards of at most 4 GiB each (u32 offsets), e.g. by
    `balanced_ranges`. Shard s is decoded on rank owner(s, world); root keeps its own.
    decode_fn(blob, off) -> (out_blob, out_off, out_len int32/uint32, status uint8) on `device`.
    compacted: decode_fn is the compacted form (HuffmanCodec.decode_compact, hpk_decode_batch_compact):
    literal i's bytes are at out_off[i] (starts, not regions: not monotone), and out_blob[:out_off[m]] is
    the span the decode wrote. With the wave-fill kernel (batches of >= 4M literals) that span holds
    unwritten gaps between its workgroups' shares (~1.3x the decoded bytes on a config-5 shard), so the
    owner gathers the decoded bytes end to end exactly as for the region form (`compact` takes any
    per-literal starts) and only decoded bytes travel; root's offsets are their exclusive sum either way.

    Everything stays in device memory when `device` is a GPU (RCCL point-to-point over xGMI; no host
    copy of the data): the shard sizes go out with one broadcast and the offsets and blob of each
    shard with one grouped send/recv round. Every owner then lays its shards' decoded bytes end to
    end (only out_len bytes per literal travel back, not the regions' slack), one all-reduce tells
    root every shard's decoded size, and the bytes, out_len and status come back in one more grouped
    round. Host synchronisation: the size broadcast, the all-reduce and one read of the piece bounds
    per owned shard in `compact`. Refusals (a backend that cannot carry the device, a bad shard on
    root, a failed decode on any rank) make EVERY rank raise, never a hang. With gloo and CPU tensors the same code runs on the host (tests/test_shard.py).
    Returns on root the list of (decoded bytes laid end to end, their int64 offsets [m+1], out_len,
    status) in shard order; None elsewhere."""
    import torch
    import torch.distributed as dist

    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    check_backend(dist, group, dev)
    # 1. shard sizes, from root to every rank: [S] then S x (literals, blob bytes). Root checks the
    # shards BEFORE the count goes out and sends S = -1 on a bad one, so every rank raises (a root
    # that raised after the broadcast would leave the others waiting in the next one)
    err = None
    if rank == root:
        try:
            for s, (b, off) in enumerate(shards):
                _check(off, f"shard {s} offsets", ("int32", "uint32"))
                _check(b, f"shard {s} blob", ("uint8",))
        except ValueError as e:
            err = e
    cnt = torch.tensor([(len(shards) if err is None else -1) if rank == root else 0], dtype=torch.int64, device=dev)
    dist.broadcast(cnt, root, group=group)
    S = int(cnt.item())
    if S < 0:
        raise err if err is not None else ValueError("scatter_decode_gather: root refused its shards")
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
    # 3. decode the local shards; every shard's decoded size, on the device
    # (an owner whose decode_fn fails or returns tensors the wire would misread does not raise here:
    # it flags the error in the all-reduce below, so every rank raises together instead of the
    # others waiting for it in the collective)
    res, err = {}, None
    tot = torch.zeros(S + 1, dtype=torch.int64, device=dev)  # [S] = ranks that failed
    try:
        for s in mine:
            res[s] = decode_fn(*local[s])
            ob, oo, ol, st = res[s]
            _check(ol, f"shard {s} out_len", ("int32", "uint32"))
            _check(st, f"shard {s} status", ("uint8",))
            m = sizes[s][0]
            if compacted:
                _check(oo, f"shard {s} out_off", ("int32", "uint32"))
            if m:
                tot[s] = ol[:m].to(torch.int64).sum()
    except Exception as e:  # noqa: BLE001 -- re-raised after the collective
        err = e
        tot.zero_()
        tot[S] = 1
    # 4. one all-reduce: every rank (root included) learns every shard's decoded size
    dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    totals = tot.tolist()
    if totals[S]:
        if err is not None:
            raise err
        raise RuntimeError(f"scatter_decode_gather: {totals[S]} rank(s) failed to decode their shards")
    # 5. the owners lay their shards' bytes end to end (region starts or compacted starts alike); bytes,
    # out_len and status go to root
    packed = {s: compact(*res[s][:3], sizes[s][0], int(totals[s])) for s in mine}
    out, ops = {}, []
    for s in range(S):
        o = owner(s, world)
        m, nbytes = sizes[s][0], int(totals[s])
        if o == root:
            continue
        if rank == o:
            ol, st = res[s][2], res[s][3]
            ops += [(dist.isend, _wire(ol[:m]), root), (dist.isend, st[:m], root)]
            if nbytes:
                ops.append((dist.isend, packed[s], root))
        elif rank == root:
            ol = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
            st = torch.empty(max(m, 1), dtype=torch.uint8, device=dev)
            cb = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
            ops += [(dist.irecv, ol[:m], o), (dist.irecv, st[:m], o)]
            if nbytes:
                ops.append((dist.irecv, cb[:nbytes], o))
            out[s] = (cb[:nbytes], ol[:m], st[:m])
    ops = [x for x in ops if x[1].numel()]
    _p2p(dist, ops, group)
    if rank != root:
        return None
    result = []
    for s in range(S):
        m = sizes[s][0]
        if s in mine:
            cb, ol, st = packed[s], res[s][2][:m], res[s][3][:m]
        else:
            cb, ol, st = out[s]
        result.append((cb, compact_offsets(ol, m), ol, st))
    return result
