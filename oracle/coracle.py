"""ctypes wrapper of oracle/_build/liboracle.so (cdc_oracle.c) — TEST INFRASTRUCTURE ONLY.

Used by tests/ as the checker for large inputs and by bench.py's ``cpu_baseline`` leg as
the CPU column ("port": a C restatement of the reference Go chunker, not the Go code).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import chunker

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "_build", "liboracle.so")

SEG_DTYPE = np.dtype([("offset", "<u8"), ("size", "<u8"), ("file", "<u4"), ("flags", "<u4"),
                      ("hash", "u1", (32,))])


class _Params(C.Structure):
    _fields_ = [("average_bits", C.c_uint32), ("_pad", C.c_uint32), ("min_chunk", C.c_int64),
                ("max_chunk", C.c_int64)]


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        P, u64, u32, i32 = C.POINTER, C.c_uint64, C.c_uint32, C.c_int
        lib.oracle_blake2b256.argtypes = [C.c_void_p, u64, C.c_void_p]
        lib.oracle_blake2b256.restype = None
        lib.oracle_segment_files.argtypes = [C.c_void_p, P(u64), u32, P(u64), P(_Params), i32,
                                             i32, P(u64), C.c_void_p, P(u64)]
        lib.oracle_segment_files.restype = i32
        lib.oracle_candidates.argtypes = [C.c_void_p, u64, P(u64), u32, P(u64), u64]
        lib.oracle_candidates.restype = u64
        _lib = lib
    return _lib


def blake2b256(data: bytes) -> bytes:
    out = (C.c_uint8 * 32)()
    buf = bytes(data)
    load().oracle_blake2b256(buf, len(buf), out)
    return bytes(out)


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def segment_files(data: np.ndarray, file_offsets, params: chunker.Params = chunker.Params(),
                  nthreads: int = 1, do_hash: bool = True):
    """Per-file segments of a batch (each file = one fresh writer + one annotation).

    Returns (segments structured array ordered by (file, offset), file_begin[nfiles+1])."""
    lib = load()
    data = np.ascontiguousarray(data, dtype=np.uint8)
    offs = np.ascontiguousarray(np.asarray(file_offsets, dtype=np.uint64))
    nfiles = len(offs) - 1
    lens = np.diff(offs.astype(np.int64))
    caps = np.where(lens > 0, lens // params.min + 1, 0).astype(np.uint64)
    base = np.zeros(nfiles + 1, dtype=np.uint64)
    base[1:] = np.cumsum(caps)
    out = np.zeros(int(base[-1]) if nfiles else 0, dtype=SEG_DTYPE)
    nseg = np.zeros(max(nfiles, 1), dtype=np.uint64)
    table = np.asarray(chunker.table(params.seed), dtype=np.uint64)
    p = _Params(params.average_bits, 0, params.min, params.max)
    rc = lib.oracle_segment_files(data.ctypes.data if data.size else None, _u64p(offs), nfiles,
                                  _u64p(table), C.byref(p), nthreads, int(do_hash), _u64p(base),
                                  out.ctypes.data if out.size else None, _u64p(nseg))
    if rc:
        raise RuntimeError("oracle_segment_files failed")
    keep = np.concatenate([np.arange(int(base[f]), int(base[f] + nseg[f])) for f in range(nfiles)]) \
        if nfiles else np.zeros(0, dtype=np.int64)
    segs = out[keep.astype(np.int64)] if len(keep) else np.zeros(0, dtype=SEG_DTYPE)
    begin = np.zeros(nfiles + 1, dtype=np.uint64)
    begin[1:] = np.cumsum(nseg[:nfiles])
    return segs, begin


def candidates(data: np.ndarray, params: chunker.Params = chunker.Params(),
               cap: int = 1 << 20) -> np.ndarray:
    """All positions i >= 63 with h_i & mask == 0, rolling from one reset at offset 0."""
    lib = load()
    data = np.ascontiguousarray(data, dtype=np.uint8)
    table = np.asarray(chunker.table(params.seed), dtype=np.uint64)
    out = np.zeros(cap, dtype=np.uint64)
    n = lib.oracle_candidates(data.ctypes.data if data.size else None, data.size, _u64p(table),
                              params.average_bits, _u64p(out), cap)
    return out[:min(n, cap)]
