"""ctypes binding of libhpk.so (the C ABI in include/hpk.h).

The library is built in-tree (loona_amd/libhpk.so, by __graft_entry__.build() or
`make -C loona_amd/csrc`). There is no fallback: if the library is missing or does not load,
every entry point raises, so a GPU run can never silently take a CPU path.
"""

from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HPK_LIB", os.path.join(HERE, "libhpk.so"))

# hpk_status (hpk.h) <-> HuffmanDecoderError (crates/loona-hpack/src/huffman.rs:28-41)
HPK_OK = 0
HPK_PADDING_TOO_LARGE = 1
HPK_INVALID_PADDING = 2
HPK_EOS_IN_STRING = 3
HPK_OUTPUT_OVERFLOW = 4
HPK_BAD_OFFSETS = 5  # device-pointer call with decreasing offsets / offsets past a capacity

HPK_E_OK = 0
HPK_E_INVAL = -1
HPK_E_NOSPACE = -2
HPK_E_DEVICE = -3
HPK_E_NODEVICE = -4

HPK_PTR_HOST = 0x0
HPK_PTR_DEVICE = 0x1
HPK_ASYNC = 0x2
HPK_MAX_OFFSET = 0xFFFFFFDF  # offsets of one shard stay at or below this (hpk.h)

# every symbol include/hpk.h declares (tests/test_host.py checks the .so exports all of them)
EXPORTS = (
    "hpk_decoded_bound",
    "hpk_encoded_bound",
    "hpk_huffman_encoded_len",
    "hpk_huffman_decode_one",
    "hpk_huffman_encode_one",
    "hpk_ctx_create",
    "hpk_ctx_destroy",
    "hpk_ctx_set_stream",
    "hpk_ctx_stream",
    "hpk_ctx_sync",
    "hpk_ctx_check",
    "hpk_last_error",
    "hpk_decode_batch",
    "hpk_decode_batch_compact",
    "hpk_encode_batch",
    "hpk_decode_batch_cpu",
    "hpk_encode_batch_cpu",
    "hpk_host_register",
    "hpk_host_unregister",
    "hpk_arena_create",
    "hpk_arena_base",
    "hpk_arena_len",
    "hpk_arena_destroy",
    "hpk_hdec_create",
    "hpk_hdec_destroy",
    "hpk_hdec_set_max_table_size",
    "hpk_hdec_set_max_allowed_table_size",
    "hpk_hdec_table_size",
    "hpk_hdec_decode_blocks",
    "hpk_blocks_out_free",
    "hpk_h2conn_create",
    "hpk_h2conn_destroy",
    "hpk_h2conn_decoder",
    "hpk_h2conn_set_max_frame_size",
    "hpk_h2conn_error",
    "hpk_h2_error_code",
    "hpk_h2_read_frames",
    "hpk_h2_out_free",
    "hpk_henc_create",
    "hpk_henc_destroy",
    "hpk_henc_set_max_table_size",
    "hpk_henc_encode",
    "hpk_henc_encode_blocks",
    "hpk_henc_out_free",
    "hpk_test_fail_batches",
    "hpk_test_bound_scan",
    "hpk_test_small_calls",
    "hpk_test_small_stamps",
    "hpk_ctx_set_decode_kernel",
    "hpk_ctx_set_small_mode",
    "hpk_version",
)

class Header(ctypes.Structure):
    _fields_ = [("name_off", ctypes.c_uint32), ("name_len", ctypes.c_uint32), ("value_off", ctypes.c_uint32),
                ("value_len", ctypes.c_uint32)]


class BlockResult(ctypes.Structure):
    _fields_ = [("first_header", ctypes.c_uint32), ("n_headers", ctypes.c_uint32), ("error", ctypes.c_int32),
                ("detail", ctypes.c_int32)]


class BlocksOut(ctypes.Structure):
    _fields_ = [("arena", ctypes.POINTER(ctypes.c_uint8)), ("arena_len", ctypes.c_size_t),
                ("headers", ctypes.POINTER(Header)), ("n_headers", ctypes.c_size_t),
                ("blocks", ctypes.POINTER(BlockResult)), ("n_blocks", ctypes.c_uint32)]


class HencOut(ctypes.Structure):
    _fields_ = [("bytes", ctypes.POINTER(ctypes.c_uint8)), ("len", ctypes.c_size_t),
                ("block_off", ctypes.POINTER(ctypes.c_uint32)), ("n_blocks", ctypes.c_uint32)]


class H2Block(ctypes.Structure):
    _fields_ = [("conn", ctypes.c_uint32), ("stream_id", ctypes.c_uint32), ("end_stream", ctypes.c_uint32),
                ("skipped", ctypes.c_uint32)]


class H2Out(ctypes.Structure):
    _fields_ = [("hb", BlocksOut), ("blocks", ctypes.POINTER(H2Block)), ("conn_error", ctypes.POINTER(ctypes.c_int32)),
                ("conn_consumed", ctypes.POINTER(ctypes.c_uint32)), ("n_conns", ctypes.c_uint32)]


_lock = threading.Lock()
_lib = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_sizep = ctypes.POINTER(ctypes.c_size_t)


def lib() -> ctypes.CDLL:
    """Load libhpk.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libhpk.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                " or `make -C loona_amd/csrc` (there is no CPU fallback)"
            )
        L = ctypes.CDLL(LIB_PATH)
        L.hpk_decoded_bound.argtypes = [ctypes.c_size_t]
        L.hpk_decoded_bound.restype = ctypes.c_size_t
        L.hpk_encoded_bound.argtypes = [ctypes.c_size_t]
        L.hpk_encoded_bound.restype = ctypes.c_size_t
        L.hpk_huffman_encoded_len.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.hpk_huffman_encoded_len.restype = ctypes.c_size_t
        for fn in (L.hpk_huffman_decode_one, L.hpk_huffman_encode_one):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, c_sizep]
            fn.restype = ctypes.c_int
        L.hpk_ctx_create.argtypes = [ctypes.c_int]
        L.hpk_ctx_create.restype = ctypes.c_void_p
        L.hpk_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.hpk_ctx_destroy.restype = None
        L.hpk_ctx_set_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.hpk_ctx_set_stream.restype = ctypes.c_int
        L.hpk_ctx_stream.argtypes = [ctypes.c_void_p]
        L.hpk_ctx_stream.restype = ctypes.c_void_p
        L.hpk_ctx_sync.argtypes = [ctypes.c_void_p]
        L.hpk_ctx_sync.restype = ctypes.c_int
        L.hpk_ctx_check.argtypes = [ctypes.c_void_p]
        L.hpk_ctx_check.restype = ctypes.c_int
        L.hpk_last_error.argtypes = [ctypes.c_void_p]
        L.hpk_last_error.restype = ctypes.c_char_p
        for fn in (L.hpk_decode_batch, L.hpk_encode_batch, L.hpk_decode_batch_compact):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint32,
                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_int]
            fn.restype = ctypes.c_int
        for fn in (L.hpk_decode_batch_cpu, L.hpk_encode_batch_cpu):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
            fn.restype = ctypes.c_int
        L.hpk_host_register.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.hpk_host_register.restype = ctypes.c_int
        L.hpk_host_unregister.argtypes = [ctypes.c_void_p]
        L.hpk_host_unregister.restype = ctypes.c_int
        L.hpk_arena_create.argtypes = [ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
        L.hpk_arena_create.restype = ctypes.c_void_p
        L.hpk_arena_base.argtypes = [ctypes.c_void_p]
        L.hpk_arena_base.restype = ctypes.c_void_p
        L.hpk_arena_len.argtypes = [ctypes.c_void_p]
        L.hpk_arena_len.restype = ctypes.c_size_t
        L.hpk_arena_destroy.argtypes = [ctypes.c_void_p]
        L.hpk_arena_destroy.restype = None
        L.hpk_hdec_create.argtypes = []
        L.hpk_hdec_create.restype = ctypes.c_void_p
        L.hpk_hdec_destroy.argtypes = [ctypes.c_void_p]
        L.hpk_hdec_destroy.restype = None
        for fn in (L.hpk_hdec_set_max_table_size, L.hpk_hdec_set_max_allowed_table_size):
            fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
            fn.restype = ctypes.c_int
        L.hpk_hdec_table_size.argtypes = [ctypes.c_void_p, c_sizep, c_sizep, c_sizep]
        L.hpk_hdec_table_size.restype = ctypes.c_int
        L.hpk_hdec_decode_blocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint32, ctypes.POINTER(BlocksOut)]
        L.hpk_hdec_decode_blocks.restype = ctypes.c_int
        L.hpk_blocks_out_free.argtypes = [ctypes.POINTER(BlocksOut)]
        L.hpk_blocks_out_free.restype = None
        L.hpk_h2conn_create.argtypes = []
        L.hpk_h2conn_create.restype = ctypes.c_void_p
        L.hpk_h2conn_destroy.argtypes = [ctypes.c_void_p]
        L.hpk_h2conn_destroy.restype = None
        L.hpk_h2conn_decoder.argtypes = [ctypes.c_void_p]
        L.hpk_h2conn_decoder.restype = ctypes.c_void_p
        L.hpk_h2conn_set_max_frame_size.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        L.hpk_h2conn_set_max_frame_size.restype = ctypes.c_int
        L.hpk_h2conn_error.argtypes = [ctypes.c_void_p]
        L.hpk_h2conn_error.restype = ctypes.c_int
        L.hpk_h2_error_code.argtypes = [ctypes.c_int]
        L.hpk_h2_error_code.restype = ctypes.c_int
        L.hpk_h2_read_frames.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint32, ctypes.POINTER(H2Out)]
        L.hpk_h2_read_frames.restype = ctypes.c_int
        L.hpk_h2_out_free.argtypes = [ctypes.POINTER(H2Out)]
        L.hpk_h2_out_free.restype = None
        L.hpk_henc_create.argtypes = [ctypes.c_int]
        L.hpk_henc_create.restype = ctypes.c_void_p
        L.hpk_henc_destroy.argtypes = [ctypes.c_void_p]
        L.hpk_henc_destroy.restype = None
        L.hpk_henc_set_max_table_size.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.hpk_henc_set_max_table_size.restype = ctypes.c_int
        L.hpk_henc_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p, ctypes.c_size_t, c_sizep]
        L.hpk_henc_encode.restype = ctypes.c_int
        L.hpk_henc_encode_blocks.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(HencOut)]
        L.hpk_henc_encode_blocks.restype = ctypes.c_int
        L.hpk_henc_out_free.argtypes = [ctypes.POINTER(HencOut)]
        L.hpk_henc_out_free.restype = None
        L.hpk_ctx_set_decode_kernel.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.hpk_ctx_set_decode_kernel.restype = ctypes.c_int
        L.hpk_ctx_set_small_mode.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32]
        L.hpk_ctx_set_small_mode.restype = ctypes.c_int
        # test-only entry points: bound when the library has them (an A/B build of another source may not)
        if hasattr(L, "hpk_test_fail_batches"):
            L.hpk_test_fail_batches.argtypes = [ctypes.c_int]
            L.hpk_test_fail_batches.restype = None
        if hasattr(L, "hpk_test_small_stamps"):
            L.hpk_test_small_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            L.hpk_test_small_stamps.restype = ctypes.c_int
        if hasattr(L, "hpk_test_small_calls"):
            L.hpk_test_small_calls.argtypes = [ctypes.c_void_p]
            L.hpk_test_small_calls.restype = ctypes.c_uint64
        if hasattr(L, "hpk_test_bound_scan"):
            L.hpk_test_bound_scan.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
            L.hpk_test_bound_scan.restype = ctypes.c_int
        L.hpk_version.argtypes = []
        L.hpk_version.restype = ctypes.c_char_p
        _lib = L
        return L


def last_error() -> str:
    msg = lib().hpk_last_error(None)
    return msg.decode(errors="replace") if msg else ""


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error()}")
    return rc
