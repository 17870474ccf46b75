"""Batched Huffman codec on the GPU (hpk_decode_batch / hpk_encode_batch of include/hpk.h).

Layout (one shard, u32 offsets): literal i is in_blob[in_off[i]:in_off[i+1]]; its output goes to
out_blob[out_off[i]:out_off[i+1]] (capacity), out_len[i] bytes are valid, status[i] is the
hpk_status (0 ok, 1 PaddingTooLarge, 2 InvalidPadding, 3 EOSInString, 4 output overflow).

Device tensors go straight to the kernels on the context's stream (by default torch's current
stream, so torch events and the kernels share one timeline). Host numpy arrays go through the
library's own H2D/D2H staging. There is no CPU fallback anywhere in this module.
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

U32 = np.uint32


def pack(literals):
    """list of bytes -> (blob u8, off u32[n+1])."""
    lens = np.fromiter((len(x) for x in literals), dtype=np.int64, count=len(literals))
    off = np.zeros(len(literals) + 1, dtype=np.int64)
    np.cumsum(lens, out=off[1:])
    if off[-1] >= 2**32:
        raise ValueError("a shard must stay below 4 GiB (u32 offsets)")
    blob = np.frombuffer(b"".join(bytes(x) for x in literals), dtype=np.uint8).copy()
    return blob, off.astype(U32)


def unpack(blob, off, lens=None):
    blob = np.asarray(blob)
    off = np.asarray(off, dtype=np.int64)
    if lens is None:
        return [blob[off[i] : off[i + 1]].tobytes() for i in range(len(off) - 1)]
    lens = np.asarray(lens, dtype=np.int64)
    return [blob[off[i] : off[i] + lens[i]].tobytes() for i in range(len(off) - 1)]


def _round4(b):
    return (b + 3) & ~3


def decode_offsets_np(in_off):
    """Output offsets from hpk_decoded_bound(len) = floor(8*len/5) per literal, each capacity
    rounded up to 4 bytes so every literal's output starts dword-aligned (the kernels' fast
    store path; unaligned offsets are still handled)."""
    in_off = np.asarray(in_off, dtype=np.int64)
    b = _round4((np.diff(in_off) * 8) // 5)
    out = np.zeros(len(in_off), dtype=np.int64)
    np.cumsum(b, out=out[1:])
    if out[-1] >= 2**32:
        raise ValueError("decoded bound of the shard exceeds 4 GiB")
    return out.astype(U32)


def encode_offsets_np(in_off):
    """Output offsets from hpk_encoded_bound(len) = ceil(30*len/8) per literal (rounded to 4)."""
    in_off = np.asarray(in_off, dtype=np.int64)
    b = _round4((np.diff(in_off) * 30 + 7) // 8)
    out = np.zeros(len(in_off), dtype=np.int64)
    np.cumsum(b, out=out[1:])
    if out[-1] >= 2**32:
        raise ValueError("encoded bound of the shard exceeds 4 GiB")
    return out.astype(U32)


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return x.ctypes.data_as(ctypes.c_void_p)
    return ctypes.c_void_p(x.data_ptr())  # torch tensor


class HuffmanCodec:
    """One device context (hpk_ctx): a HIP stream + LDS-staged decode tables on one GPU.

    loona is thread-per-core and !Send (crates/buffet/src/lib.rs:38-49): use one codec per
    host thread."""

    def __init__(self, device: int = 0, stream=None):
        self._L = _lib.lib()
        self.device = device
        h = self._L.hpk_ctx_create(device)
        if not h:
            raise RuntimeError(f"hpk_ctx_create({device}) failed: {_lib.last_error()}")
        self._h = h
        if stream is not None:
            self.set_stream(stream)

    def close(self):
        if getattr(self, "_h", None):
            self._L.hpk_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_stream(self, stream):
        """stream: a torch.cuda.Stream (its handle 0 = the legacy null stream), a raw hipStream_t
        int, or None (the ctx's own non-blocking stream)."""
        if stream is None:
            arg = None
        else:
            raw = int(getattr(stream, "cuda_stream", stream))
            arg = ctypes.c_void_p(raw) if raw else ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF)  # HPK_STREAM_LEGACY
        _lib.check(self._L.hpk_ctx_set_stream(self._h, arg), "hpk_ctx_set_stream")

    def sync(self):
        _lib.check(self._L.hpk_ctx_sync(self._h), "hpk_ctx_sync")

    # -- raw entry points --------------------------------------------------------------------
    def _call(self, fn, name, in_blob, in_off, n, out_blob, out_off, out_len, status, flags):
        rc = fn(self._h, _ptr(in_blob), _ptr(in_off), ctypes.c_uint32(n), _ptr(out_blob), _ptr(out_off),
                _ptr(out_len), _ptr(status), flags)
        _lib.check(rc, name)

    def decode_into(self, in_blob, in_off, out_blob, out_off, out_len, status, device=True, sync=False):
        n = int(in_off.shape[0]) - 1
        flags = _lib.HPK_PTR_DEVICE | (0 if sync else _lib.HPK_ASYNC) if device else _lib.HPK_PTR_HOST
        self._call(self._L.hpk_decode_batch, "hpk_decode_batch", in_blob, in_off, n, out_blob, out_off, out_len,
                   status, flags)

    def encode_into(self, in_blob, in_off, out_blob, out_off, out_len, status, device=True, sync=False):
        n = int(in_off.shape[0]) - 1
        flags = _lib.HPK_PTR_DEVICE | (0 if sync else _lib.HPK_ASYNC) if device else _lib.HPK_PTR_HOST
        self._call(self._L.hpk_encode_batch, "hpk_encode_batch", in_blob, in_off, n, out_blob, out_off, out_len,
                   status, flags)

    # -- host (numpy) convenience ------------------------------------------------------------
    def decode_host(self, in_blob, in_off, out_off=None):
        """numpy in -> (out_blob, out_off, out_len, status), staged through the ctx."""
        in_blob = np.ascontiguousarray(in_blob, dtype=np.uint8)
        in_off = np.ascontiguousarray(in_off, dtype=U32)
        out_off = decode_offsets_np(in_off) if out_off is None else np.ascontiguousarray(out_off, dtype=U32)
        n = len(in_off) - 1
        out_blob = np.zeros(max(int(out_off[-1]), 1), dtype=np.uint8)
        out_len = np.zeros(max(n, 1), dtype=U32)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        if in_blob.size == 0:
            in_blob = np.zeros(1, dtype=np.uint8)
        self.decode_into(in_blob, in_off, out_blob, out_off, out_len, status, device=False)
        return out_blob, out_off, out_len[:n], status[:n]

    def encode_host(self, in_blob, in_off, out_off=None):
        in_blob = np.ascontiguousarray(in_blob, dtype=np.uint8)
        in_off = np.ascontiguousarray(in_off, dtype=U32)
        out_off = encode_offsets_np(in_off) if out_off is None else np.ascontiguousarray(out_off, dtype=U32)
        n = len(in_off) - 1
        out_blob = np.zeros(max(int(out_off[-1]), 1), dtype=np.uint8)
        out_len = np.zeros(max(n, 1), dtype=U32)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        if in_blob.size == 0:
            in_blob = np.zeros(1, dtype=np.uint8)
        self.encode_into(in_blob, in_off, out_blob, out_off, out_len, status, device=False)
        return out_blob, out_off, out_len[:n], status[:n]

    # -- device (torch) convenience ----------------------------------------------------------
    def decode_device(self, in_blob, in_off, out_off=None, out_blob=None, out_len=None, status=None, sync=False):
        """torch cuda tensors (u8 blob, int32/uint32 offsets) -> (out_blob, out_off, out_len, status)."""
        import torch

        n = int(in_off.shape[0]) - 1
        if out_off is None:
            out_off = decode_offsets_torch(in_off)
        dev = in_blob.device
        if out_blob is None:
            out_blob = torch.empty(max(int(out_off[-1].item()), 1), dtype=torch.uint8, device=dev)
        if out_len is None:
            out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self.decode_into(in_blob, in_off, out_blob, out_off, out_len, status, device=True, sync=sync)
        return out_blob, out_off, out_len, status

    def encode_device(self, in_blob, in_off, out_off=None, out_blob=None, out_len=None, status=None, sync=False):
        import torch

        n = int(in_off.shape[0]) - 1
        if out_off is None:
            out_off = encode_offsets_torch(in_off)
        dev = in_blob.device
        if out_blob is None:
            out_blob = torch.empty(max(int(out_off[-1].item()), 1), dtype=torch.uint8, device=dev)
        if out_len is None:
            out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self.encode_into(in_blob, in_off, out_blob, out_off, out_len, status, device=True, sync=sync)
        return out_blob, out_off, out_len, status


def _bound_offsets_torch(in_off, num, den, add):
    import torch

    o = in_off.to(torch.int64)
    b = (((o[1:] - o[:-1]) * num + add) // den + 3) & ~3
    out = torch.zeros_like(o)
    torch.cumsum(b, 0, out=out[1:])
    if int(out[-1].item()) >= 2**32:
        raise ValueError("bound of the shard exceeds 4 GiB")
    return out.to(torch.int32) if int(out[-1].item()) < 2**31 else out.to(torch.uint32)


def decode_offsets_torch(in_off):
    return _bound_offsets_torch(in_off, 8, 5, 0)


def encode_offsets_torch(in_off):
    return _bound_offsets_torch(in_off, 30, 8, 7)


def _cpu_batch(fn_name, bound, in_blob, in_off, nthreads):
    L = _lib.lib()
    in_blob = np.ascontiguousarray(in_blob, dtype=np.uint8)
    in_off = np.ascontiguousarray(in_off, dtype=U32)
    out_off = bound(in_off)
    n = len(in_off) - 1
    out_blob = np.zeros(max(int(out_off[-1]), 1), dtype=np.uint8)
    out_len = np.zeros(max(n, 1), dtype=U32)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    src = in_blob if in_blob.size else np.zeros(1, dtype=np.uint8)
    rc = getattr(L, fn_name)(src.ctypes.data, in_off.ctypes.data, n, out_blob.ctypes.data, out_off.ctypes.data,
                             out_len.ctypes.data, status.ctypes.data, int(nthreads))
    _lib.check(rc, fn_name)
    return out_blob, out_off, out_len[:n], status[:n]


def decode_batch_cpu(in_blob, in_off, nthreads=0):
    """The library's table-driven CPU batch decode (hpk_decode_batch_cpu): same layout and
    results as the device path, host threads over byte-balanced shards."""
    return _cpu_batch("hpk_decode_batch_cpu", decode_offsets_np, in_blob, in_off, nthreads)


def encode_batch_cpu(in_blob, in_off, nthreads=0):
    return _cpu_batch("hpk_encode_batch_cpu", encode_offsets_np, in_blob, in_off, nthreads)
