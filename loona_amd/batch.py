"""Batched Huffman codec on the GPU (hpk_decode_batch / hpk_encode_batch of include/hpk.h).

Layout (one shard, u32 offsets): literal i is in_blob[in_off[i]:in_off[i+1]]; its output goes to
out_blob[out_off[i]:out_off[i+1]] (capacity), out_len[i] bytes are valid, status[i] is the
hpk_status (0 ok, 1 PaddingTooLarge, 2 InvalidPadding, 3 EOSInString, 4 output overflow).

Device tensors go straight to the kernels on the codec's stream: by default torch's current
stream on the codec's device at the time of each call, so torch ops that produced the inputs and
the caching allocator's reuse of the outputs are ordered with the kernels. Host numpy arrays go
through the library's own H2D/D2H staging. Every buffer is checked before it reaches the C ABI
(dtype, contiguity, device, room for n entries), and the C ABI gets each blob's capacity, so
offsets past a blob are rejected on the device (status HPK_BAD_OFFSETS) instead of read or written.
There is no CPU fallback anywhere in this module.
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


_OFF_DTYPES = ("int32", "uint32")


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _arg(x, name, kinds, min_len, device_index=None):
    """(pointer, byte size) of a contiguous numpy array or torch tensor, after checking its dtype
    (one of `kinds`), its length (>= min_len entries) and, for device calls, that it is a CUDA
    tensor on the codec's device. Raises ValueError / TypeError instead of handing the C ABI a
    buffer it would misread (an int64 offset tensor read as u32 halves, a view, a short array)."""
    if _is_torch(x):
        dt = str(x.dtype).replace("torch.", "")
        if device_index is not None:
            if not x.is_cuda or x.device.index != device_index:
                raise ValueError(f"{name}: expected a tensor on cuda:{device_index}, got {x.device}")
        elif x.is_cuda:
            raise ValueError(f"{name}: host-pointer call given a CUDA tensor")
        if not x.is_contiguous():
            raise ValueError(f"{name}: tensor must be contiguous")
        n, nbytes, ptr = x.numel(), x.numel() * x.element_size(), x.data_ptr()
    elif isinstance(x, np.ndarray):
        if device_index is not None:
            raise ValueError(f"{name}: device call given a host numpy array")
        dt = str(x.dtype)
        if not x.flags["C_CONTIGUOUS"]:
            raise ValueError(f"{name}: array must be C-contiguous")
        n, nbytes, ptr = x.size, x.nbytes, x.ctypes.data
    else:
        raise TypeError(f"{name}: expected a numpy array or torch tensor, got {type(x).__name__}")
    if dt not in kinds:
        raise TypeError(f"{name}: dtype {dt} not in {kinds}")
    if n < min_len:
        raise ValueError(f"{name}: {n} entries, need >= {min_len}")
    return ctypes.c_void_p(ptr), nbytes


class HuffmanCodec:
    """One device context (hpk_ctx): a HIP stream + LDS-staged decode tables on one GPU.

    loona is thread-per-core and !Send (crates/buffet/src/lib.rs:38-49): use one codec per
    host thread.

    stream: None (default) = torch's current stream on `device` at each call; a torch.cuda.Stream
    or raw hipStream_t int = that stream; "own" = the context's own non-blocking stream."""

    def __init__(self, device: int = 0, stream=None):
        self._L = _lib.lib()
        self.device = device
        h = self._L.hpk_ctx_create(device)
        if not h:
            raise RuntimeError(f"hpk_ctx_create({device}) failed: {_lib.last_error()}")
        self._h = h
        self._follow_torch = stream is None
        self._bound = None
        if stream is not None and stream != "own":
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
        int, or None (the ctx's own non-blocking stream). Fixes the stream for later calls."""
        self._follow_torch = False
        self._bind(stream)

    def _bind(self, stream):
        if stream is None:
            arg = None
        else:
            raw = int(getattr(stream, "cuda_stream", stream))
            arg = ctypes.c_void_p(raw) if raw else ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF)  # HPK_STREAM_LEGACY
        _lib.check(self._L.hpk_ctx_set_stream(self._h, arg), "hpk_ctx_set_stream")
        self._bound = None if arg is None else arg.value

    def _follow(self):
        """Bind torch's current stream on the codec's device (default mode)."""
        if not self._follow_torch:
            return
        import torch

        s = torch.cuda.current_stream(self.device)
        raw = int(s.cuda_stream) or (-1 & 0xFFFFFFFFFFFFFFFF)
        if raw != self._bound:
            self._bind(s)

    DECODE_KERNELS = {"auto": 0, "fill": 1, "wave": 2}

    def set_decode_kernel(self, kind: str):
        """'auto' (default: wave fills for every batch since round 6), 'fill' or 'wave'
        (hpk_ctx_set_decode_kernel): the same results, different speed."""
        if kind not in self.DECODE_KERNELS:
            raise ValueError(f"decode kernel {kind!r} not in {tuple(self.DECODE_KERNELS)}")
        _lib.check(self._L.hpk_ctx_set_decode_kernel(self._h, self.DECODE_KERNELS[kind]), "hpk_ctx_set_decode_kernel")

    def set_small_mode(self, max_literals: int, workgroups: int = 4, idle_ms: int = 50):
        """The small-call mode (hpk_ctx_set_small_mode): synchronous device-pointer decode calls of at
        most max_literals literals go to a persistent kernel of `workgroups` workgroups instead of a
        launch; it exits after idle_ms without a call. max_literals = 0 turns it off."""
        _lib.check(self._L.hpk_ctx_set_small_mode(self._h, int(max_literals), int(workgroups), int(idle_ms)),
                   "hpk_ctx_set_small_mode")

    def sync(self):
        _lib.check(self._L.hpk_ctx_sync(self._h), "hpk_ctx_sync")

    def check(self):
        """Sticky device error flag (bad offsets in an earlier HPK_ASYNC call): raises if set."""
        _lib.check(self._L.hpk_ctx_check(self._h), "hpk_ctx_check")

    # -- raw entry points --------------------------------------------------------------------
    def _call(self, fn, name, in_blob, in_off, out_blob, out_off, out_len, status, device, sync):
        dev = self.device if device else None
        n = (int(in_off.shape[0]) if hasattr(in_off, "shape") else len(in_off)) - 1
        if n < 0:
            raise ValueError("in_off needs n+1 >= 1 entries")
        if n >= 2**32:
            raise ValueError("a batch holds at most 2^32 - 1 literals")
        pi, in_cap = _arg(in_blob, "in_blob", ("uint8",), 0, dev)
        pio, _ = _arg(in_off, "in_off", _OFF_DTYPES, n + 1, dev)
        po, out_cap = _arg(out_blob, "out_blob", ("uint8",), 0, dev)
        poo, _ = _arg(out_off, "out_off", _OFF_DTYPES, n + 1, dev)
        pl, _ = _arg(out_len, "out_len", ("int32", "uint32"), n, dev)
        ps, _ = _arg(status, "status", ("uint8",), n, dev)
        if device:
            self._follow()
            flags = _lib.HPK_PTR_DEVICE | (0 if sync else _lib.HPK_ASYNC)
        else:
            flags = _lib.HPK_PTR_HOST
        rc = fn(self._h, pi, in_cap, pio, ctypes.c_uint32(n), po, out_cap, poo, pl, ps, flags)
        _lib.check(rc, name)

    def decode_into(self, in_blob, in_off, out_blob, out_off, out_len, status, device=True, sync=False):
        """hpk_decode_batch. device=True: CUDA tensors on the codec's device, enqueued (sync=False:
        HPK_ASYNC; bad offsets then show as status HPK_BAD_OFFSETS and in check()). device=False:
        host numpy arrays, staged and synchronous."""
        self._call(self._L.hpk_decode_batch, "hpk_decode_batch", in_blob, in_off, out_blob, out_off, out_len,
                   status, device, sync)

    def encode_into(self, in_blob, in_off, out_blob, out_off, out_len, status, device=True, sync=False):
        """hpk_encode_batch, same conventions as decode_into."""
        self._call(self._L.hpk_encode_batch, "hpk_encode_batch", in_blob, in_off, out_blob, out_off, out_len,
                   status, device, sync)

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

    def decode_compact(self, in_blob, in_off, out_blob=None, out_off=None, out_len=None, status=None, sync=False):
        """hpk_decode_batch_compact: torch cuda tensors -> (out_blob, out_off, out_len, status) with each
        literal's decoded bytes written exactly (the reference's exact-length outputs, huffman.rs:98, 160):
        literal i is out_blob[out_off[i] : out_off[i] + out_len[i]] and out_off[n] is the end of the span
        written to. out_off is an output (n + 1 entries; runs of literals in completion order, so not
        monotone). The span is not gap-free: listed (long / huge) literals keep their decoded bound, and
        the wave-fill kernel (>= 4M literals) packs per workgroup, each share ending in an unwritten tail
        (include/hpk.h); shard.compact gathers the bytes end to end."""
        import torch

        n = int(in_off.shape[0]) - 1
        dev = in_blob.device
        need = compact_capacity(int(in_blob.numel()), n)
        if out_blob is None:
            out_blob = torch.empty(max(need, 1), dtype=torch.uint8, device=dev)
        if out_off is None:
            out_off = torch.empty(n + 1, dtype=torch.int32 if need < 2**31 else torch.uint32, device=dev)
        if out_len is None:
            out_len = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        if status is None:
            status = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self._call(self._L.hpk_decode_batch_compact, "hpk_decode_batch_compact", in_blob, in_off, out_blob, out_off,
                   out_len, status, True, sync)
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


def compact_capacity(in_cap, n):
    """Output bytes hpk_decode_batch_compact needs: hpk_decoded_bound(in_cap) + 4 n."""
    return (8 * int(in_cap)) // 5 + 4 * int(n)


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
