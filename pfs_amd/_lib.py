"""ctypes binding of libpfscdc.so (the C ABI declared in include/pfscdc.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) and loaded from this
package directory.  There is no fallback: if the library is missing or a call fails, the
caller gets an exception.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PFSCDC_LIB") or os.path.join(_HERE, "libpfscdc.so")  # env: A/B builds

PFSCDC_OK = 0
PFSCDC_EINVAL = -1
PFSCDC_EHIP = -2
PFSCDC_ENOMEM = -3
PFSCDC_EUNSUPPORTED = -4
PFSCDC_ESTATE = -5
PFSCDC_ECALLBACK = -6

SEG_VALID = 1
SEG_CUT = 2
OPT_REF_IDS = 1
OPT_CUTS_ONLY = 2
OPT_CTEXT_IN_PLACE = 4
SCAN_SKIPPED_FIRST_MIN = 1
SCAN_SKIPPED_CUTS = 2

# Every exported symbol of include/pfscdc.h (checked by tests/test_abi.py).
EXPORTED = [
    "pfscdc_default_params", "pfscdc_table", "pfscdc_go_int63", "pfscdc_ctx_create",
    "pfscdc_ctx_destroy", "pfscdc_last_error", "pfscdc_set_stream", "pfscdc_stream_wait",
    "pfscdc_stream_handle",
    "pfscdc_scan",
    "pfscdc_scan_async", "pfscdc_wait", "pfscdc_num_segments", "pfscdc_segments",
    "pfscdc_file_segment_begin", "pfscdc_debug_candidates", "pfscdc_last_timings",
    "pfscdc_last_scan_bytes", "pfscdc_commit_refs",
    "pfscdc_set_options", "pfscdc_refs", "pfscdc_last_ref_ms", "pfscdc_get_chunks",
    "pfscdc_last_get_ms",
    "pfscdc_host_alloc", "pfscdc_host_free", "pfscdc_fill_synthetic", "pfscdc_fill_synthetic_ex", "pfscdc_writer_create",
    "pfscdc_writer_annotate", "pfscdc_writer_write", "pfscdc_writer_close",
    "pfscdc_writer_chunk_count", "pfscdc_writer_annotation_count", "pfscdc_writer_destroy",
    "pfscdc_create_refs", "pfscdc_last_create_ms", "pfscdc_form_chunks",
    "pfscdc_uw_create", "pfscdc_uw_put", "pfscdc_uw_delete", "pfscdc_uw_close",
    "pfscdc_uw_num_filesets", "pfscdc_uw_fileset", "pfscdc_uw_destroy", "pfscdc_uw_last_error", "pfscdc_uw_timings",
    "pfscdc_uw_trim_cache", "pfscdc_uw_cached_arena_bytes",
    "pfscdc_path_clean",
    "pfscdc_hash_data_refs", "pfscdc_store_create", "pfscdc_store_destroy", "pfscdc_store_put",
    "pfscdc_store_get", "pfscdc_store_count", "pfscdc_writer_set_store", "pfscdc_writer_copy",
    "pfscdc_merge_file_hash", "pfscdc_last_create_timings", "pfscdc_writer_prefetch",
    "pfscdc_candidates", "pfscdc_hash_ranges", "pfscdc_fill_synthetic_pieces",
    "pfscdc_last_kernel_spans", "pfscdc_last_kernel_clocks", "pfscdc_order_hash_after",
    "pfscdc_set_knob", "pfscdc_get_knob", "pfscdc_knob_info", "pfscdc_last_scan_mode",
    "pfscdc_deal", "pfscdc_group_create", "pfscdc_group_destroy", "pfscdc_group_size",
    "pfscdc_group_ctx", "pfscdc_group_last_error", "pfscdc_group_scan",
    "pfscdc_group_scan_resident", "pfscdc_group_num_segments", "pfscdc_group_segments",
    "pfscdc_group_file_segment_begin", "pfscdc_group_refs", "pfscdc_group_part_begin",
    "pfscdc_group_index_device", "pfscdc_group_last_timings", "pfscdc_uw_create_group",
    "pfscdc_group_scan_stream",
]


class Params(C.Structure):
    _fields_ = [("average_bits", C.c_uint32), ("reserved", C.c_uint32), ("seed", C.c_int64),
                ("min_chunk", C.c_int64), ("max_chunk", C.c_int64)]


class Segment(C.Structure):
    _fields_ = [("offset", C.c_uint64), ("size", C.c_uint64), ("file", C.c_uint32),
                ("flags", C.c_uint32), ("hash", C.c_uint8 * 32)]


class DataRef(C.Structure):
    _fields_ = [("hash", C.c_uint8 * 32), ("offset_bytes", C.c_int64), ("size_bytes", C.c_int64)]


class RefC(C.Structure):
    _fields_ = [("id", C.c_uint8 * 32), ("dek", C.c_uint8 * 32)]


class ChunkRef(C.Structure):
    _fields_ = [("chunk_index", C.c_uint64), ("size_bytes", C.c_int64), ("edge", C.c_int32),
                ("has_ref", C.c_int32), ("ref", RefC), ("copied", C.c_int32),
                ("reserved2", C.c_int32)]


class FullDataRef(C.Structure):
    _fields_ = [("ref", RefC), ("ref_size", C.c_int64), ("edge", C.c_int32),
                ("reserved", C.c_int32), ("data", DataRef)]


class AnnotationOut(C.Structure):
    _fields_ = [("user", C.c_uint64), ("has_data_ref", C.c_int32), ("reserved", C.c_int32),
                ("data_ref", DataRef)]


class UwEvent(C.Structure):
    _fields_ = [("kind", C.c_int32), ("index", C.c_int32), ("level", C.c_int32),
                ("fileset", C.c_uint32), ("chunk", ChunkRef), ("bytes", C.c_void_p),
                ("len", C.c_uint64)]


class FilesetInfo(C.Structure):
    _fields_ = [("size_bytes", C.c_int64), ("additive_root", C.c_void_p),
                ("additive_root_len", C.c_uint64), ("deletive_root", C.c_void_p),
                ("deletive_root_len", C.c_uint64), ("num_files", C.c_uint32),
                ("num_deletes", C.c_uint32)]


EV_CHUNK, EV_INDEX = 1, 2
UW_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(UwEvent))

assert C.sizeof(Segment) == 56 and C.sizeof(Params) == 32 and C.sizeof(ChunkRef) == 96 and C.sizeof(FullDataRef) == 128

WRITER_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(ChunkRef), C.POINTER(AnnotationOut),
                        C.c_uint32)

# numpy views of pfscdc_segment / pfscdc_ref
SEGMENT_DTYPE = None
REF_DTYPE = None


def ref_dtype():
    global REF_DTYPE
    if REF_DTYPE is None:
        import numpy as np
        REF_DTYPE = np.dtype([("id", "u1", (32,)), ("dek", "u1", (32,))])
        assert REF_DTYPE.itemsize == 64
    return REF_DTYPE


def segment_dtype():
    global SEGMENT_DTYPE
    if SEGMENT_DTYPE is None:
        import numpy as np
        SEGMENT_DTYPE = np.dtype([("offset", "<u8"), ("size", "<u8"), ("file", "<u4"),
                                  ("flags", "<u4"), ("hash", "u1", (32,))])
        assert SEGMENT_DTYPE.itemsize == 56
    return SEGMENT_DTYPE


_lib = None
_lock = threading.Lock()


class PfsCdcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pfscdc error {code}: {msg}")
        self.code = code


def load() -> C.CDLL:
    """Load libpfscdc.so (raises if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make` or "
                              "`python -c 'import __graft_entry__ as g; g.build()'`")
        # One HIP runtime per process: PyTorch wheels ship their own libamdhip64.so.7 (same
        # SONAME as /opt/rocm's).  Importing torch first makes the dynamic linker bind
        # libpfscdc.so to torch's copy, so device pointers, streams and the device context
        # are shared; loading ours first would leave torch unable to see the GPU.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = C.CDLL(LIB_PATH)
        u64, i64, u32, i32, vp = C.c_uint64, C.c_int64, C.c_uint32, C.c_int, C.c_void_p
        P = C.POINTER
        sig = {
            "pfscdc_default_params": (None, [P(Params)]),
            "pfscdc_table": (i32, [i64, P(u64)]),
            "pfscdc_go_int63": (i32, [i64, P(i64), i32]),
            "pfscdc_ctx_create": (i32, [P(Params), i32, P(vp)]),
            "pfscdc_ctx_destroy": (i32, [vp]),
            "pfscdc_last_error": (C.c_char_p, [vp]),
            "pfscdc_set_stream": (i32, [vp, vp]),
            "pfscdc_stream_wait": (i32, [vp, vp]),
            "pfscdc_stream_handle": (vp, [vp]),
            "pfscdc_order_hash_after": (i32, [vp, vp]),
            "pfscdc_scan": (i32, [vp, vp, u64, i32, P(u64), u32]),
            "pfscdc_scan_async": (i32, [vp, vp, u64, i32, P(u64), u32]),
            "pfscdc_wait": (i32, [vp]),
            "pfscdc_num_segments": (u64, [vp]),
            "pfscdc_segments": (P(Segment), [vp]),
            "pfscdc_file_segment_begin": (P(u64), [vp]),
            "pfscdc_debug_candidates": (u64, [vp, P(u64), u64]),
            "pfscdc_last_timings": (i32, [vp, P(C.c_float)]),
            "pfscdc_last_scan_bytes": (i32, [vp, P(u64)]),
            "pfscdc_last_scan_mode": (i32, [vp, P(u32)]),
            "pfscdc_set_knob": (i32, [C.c_char_p, i64]),
            "pfscdc_get_knob": (i32, [C.c_char_p, P(i64)]),
            "pfscdc_knob_info": (C.c_char_p, [i32, P(i64), P(i64), P(i64)]),
            "pfscdc_last_kernel_spans": (i32, [vp, P(C.c_float)]),
            "pfscdc_last_kernel_clocks": (i32, [vp, P(C.c_float)]),
            "pfscdc_set_options": (i32, [vp, u32]),
            "pfscdc_refs": (vp, [vp]),
            "pfscdc_last_ref_ms": (i32, [vp, P(C.c_float)]),
            "pfscdc_get_chunks": (i32, [vp, vp, u64, i32, P(u64), u32, vp, vp, i32, vp]),
            "pfscdc_last_get_ms": (i32, [vp, P(C.c_float)]),
            "pfscdc_host_alloc": (vp, [u64]),
            "pfscdc_host_free": (None, [vp]),
            "pfscdc_fill_synthetic": (i32, [vp, vp, P(u64), u32, u64]),
            "pfscdc_fill_synthetic_ex": (i32, [vp, vp, P(u64), u32, u64, u32]),
            "pfscdc_writer_create": (i32, [vp, WRITER_CB, vp, u64, P(vp)]),
            "pfscdc_writer_annotate": (i32, [vp, u64]),
            "pfscdc_writer_write": (i32, [vp, vp, u64]),
            "pfscdc_writer_close": (i32, [vp]),
            "pfscdc_writer_chunk_count": (i64, [vp]),
            "pfscdc_writer_annotation_count": (i64, [vp]),
            "pfscdc_writer_destroy": (i32, [vp]),
            "pfscdc_create_refs": (i32, [vp, vp, u64, i32, P(u64), u32, vp, vp, vp]),
            "pfscdc_commit_refs": (i32, [vp, vp, u64, i32, P(u64), u32, vp, vp, vp, vp]),
            "pfscdc_last_create_ms": (i32, [vp, P(C.c_float)]),
            "pfscdc_last_create_timings": (i32, [vp, P(C.c_float)]),
            "pfscdc_form_chunks": (i32, [vp, P(C.c_uint32), u32, P(u64), vp, vp, u64, P(u64)]),
            "pfscdc_uw_create": (i32, [vp, i64, P(Params), UW_CB, vp, P(vp)]),
            "pfscdc_uw_put": (i32, [vp, C.c_char_p, C.c_char_p, i32, vp, u64]),
            "pfscdc_uw_delete": (i32, [vp, C.c_char_p, C.c_char_p]),
            "pfscdc_uw_close": (i32, [vp]),
            "pfscdc_uw_num_filesets": (u32, [vp]),
            "pfscdc_uw_fileset": (i32, [vp, u32, P(FilesetInfo)]),
            "pfscdc_uw_destroy": (i32, [vp]),
            "pfscdc_uw_last_error": (C.c_char_p, [vp]),
            "pfscdc_uw_timings": (i32, [vp, P(C.c_double)]),
            "pfscdc_uw_trim_cache": (i32, [i32, P(u64), P(u32)]),
            "pfscdc_uw_cached_arena_bytes": (u64, []),
            "pfscdc_path_clean": (i32, [C.c_char_p, i32, C.c_char_p, u64]),
            "pfscdc_hash_data_refs": (i32, [vp, vp, u32, vp]),
            "pfscdc_store_create": (i32, [P(vp)]),
            "pfscdc_store_destroy": (i32, [vp]),
            "pfscdc_store_put": (i32, [vp, vp, vp, u64]),
            "pfscdc_store_get": (i32, [vp, vp, P(vp), P(u64)]),
            "pfscdc_store_count": (u64, [vp]),
            "pfscdc_writer_set_store": (i32, [vp, vp, i32]),
            "pfscdc_writer_copy": (i32, [vp, P(FullDataRef)]),
            "pfscdc_writer_prefetch": (i32, [vp, P(FullDataRef), u32]),
            "pfscdc_merge_file_hash": (i32, [vp, vp, P(FullDataRef), u32, vp]),
            "pfscdc_candidates": (i32, [vp, vp, u64, i32, u64, P(u64), u64, P(u64)]),
            "pfscdc_hash_ranges": (i32, [vp, vp, u64, i32, P(u64), P(u64), u32, vp]),
            "pfscdc_fill_synthetic_pieces": (i32, [vp, vp, P(u64), u32, P(C.c_uint32), P(u64),
                                                   u64, u32]),
            "pfscdc_deal": (i32, [P(u64), u32, u32, P(C.c_uint32)]),
            "pfscdc_group_create": (i32, [P(Params), P(C.c_int), u32, u32, P(vp)]),
            "pfscdc_group_destroy": (i32, [vp]),
            "pfscdc_group_size": (u32, [vp]),
            "pfscdc_group_ctx": (vp, [vp, u32]),
            "pfscdc_group_last_error": (C.c_char_p, [vp]),
            "pfscdc_group_scan": (i32, [vp, vp, u64, P(u64), u32]),
            "pfscdc_group_scan_resident": (i32, [vp, P(vp), P(u64), u32, P(C.c_uint32)]),
            "pfscdc_group_num_segments": (u64, [vp]),
            "pfscdc_group_segments": (vp, [vp]),
            "pfscdc_group_file_segment_begin": (P(u64), [vp]),
            "pfscdc_group_refs": (vp, [vp]),
            "pfscdc_group_part_begin": (P(C.c_uint32), [vp]),
            "pfscdc_group_index_device": (i32, [vp, P(vp), P(vp), P(C.c_int)]),
            "pfscdc_group_last_timings": (i32, [vp, P(C.c_float), P(C.c_float), P(u64)]),
            "pfscdc_uw_create_group": (i32, [vp, i64, P(Params), UW_CB, vp, P(vp)]),
            "pfscdc_group_scan_stream": (i32, [vp, vp, u64]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def default_params() -> Params:
    p = Params()
    load().pfscdc_default_params(C.byref(p))
    return p


def table(seed: int) -> list[int]:
    out = (C.c_uint64 * 256)()
    rc = load().pfscdc_table(seed, out)
    if rc:
        raise PfsCdcError(rc, "pfscdc_table")
    return list(out)


def go_int63(seed: int, n: int) -> list[int]:
    out = (C.c_int64 * n)()
    rc = load().pfscdc_go_int63(seed, out, n)
    if rc:
        raise PfsCdcError(rc, "pfscdc_go_int63")
    return list(out)


# ---- tuning knobs (pfscdc.h: process-wide integers named after their PFSCDC_* variables) ----

def knob_info() -> dict[str, tuple[int, int, int]]:
    """Every knob the library has: name -> (lo, hi, default)."""
    lib = load()
    out = {}
    i = 0
    while True:
        lo, hi, d = C.c_int64(), C.c_int64(), C.c_int64()
        name = lib.pfscdc_knob_info(i, C.byref(lo), C.byref(hi), C.byref(d))
        if name is None:
            return out
        out[name.decode()] = (lo.value, hi.value, d.value)
        i += 1


def get_knob(name: str) -> int:
    v = C.c_int64()
    rc = load().pfscdc_get_knob(name.encode(), C.byref(v))
    if rc:
        raise PfsCdcError(rc, f"unknown knob {name}")
    return v.value


def set_knob(name: str, value: int) -> None:
    rc = load().pfscdc_set_knob(name.encode(), int(value))
    if rc:
        raise PfsCdcError(rc, f"knob {name}={value}: unknown name or out of range")


class knobs:
    """Context manager: set knobs for the block, restore them after.
    ``with knobs(PFSCDC_SCAN_GRID=1): ...``"""

    def __init__(self, **kv):
        self.kv = kv
        self.old = {}

    def __enter__(self):
        info = knob_info()
        for k, v in self.kv.items():  # every name and range first: all or nothing
            if k not in info:
                raise PfsCdcError(PFSCDC_EINVAL, f"unknown knob {k}")
            lo, hi, _ = info[k]
            if not lo <= int(v) <= hi:
                raise PfsCdcError(PFSCDC_EINVAL, f"knob {k}={v} outside [{lo}, {hi}]")
        try:
            for k, v in self.kv.items():
                self.old[k] = get_knob(k)
                set_knob(k, v)
        except BaseException:
            self.__exit__()
            raise
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_knob(k, v)
        return False
