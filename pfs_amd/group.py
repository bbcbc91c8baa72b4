"""One process, several GPUs: a device group over the C ABI (pfscdc.h ``pfscdc_group_*``).

pachd is one process that owns one chunk storage
(/root/reference/src/server/pfs/server/driver.go:110-122), so a Go host reaches the GPUs of a
node through one caller.  A ``DeviceGroup`` holds one library context per member device and
deals each call's files across them (contiguous ranges balanced by bytes, ``deal``); every
file is its own chunk stream (chunk/writer.go:125-128 resets hash and seglen at Annotate), so
the results equal a single context's.  The chunk-ref index is gathered peer to peer onto the
first member's device and returned with global file ids.  ``fileset.Storage(devices=...)``
builds unordered writers over a group (serialized filesets dealt round robin).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .cdc import SYNTH_RANDOM, ChunkParams, ScanResult, _offsets_array


def deal(offsets: Sequence[int], nparts: int) -> np.ndarray:
    """pfscdc_deal: part r = items [b[r], b[r+1]), a greedy prefix split by bytes."""
    offs = _offsets_array(offsets)
    out = np.zeros(nparts + 1, dtype=np.uint32)
    rc = _lib.load().pfscdc_deal(offs.ctypes.data_as(C.POINTER(C.c_uint64)), len(offs) - 1,
                                 nparts, out.ctypes.data_as(C.POINTER(C.c_uint32)))
    if rc:
        raise _lib.PfsCdcError(rc, "pfscdc_deal")
    return out


class DeviceGroup:
    def __init__(self, devices: Sequence[int], params: ChunkParams = ChunkParams(),
                 ref_ids: bool = False):
        self.lib = _lib.load()
        self.devices = [int(d) for d in devices]
        self.params = params
        self.ref_ids = ref_ids
        devs = (C.c_int * len(self.devices))(*self.devices)
        g = C.c_void_p()
        p = params.to_c()
        rc = self.lib.pfscdc_group_create(C.byref(p), devs, len(self.devices),
                                          _lib.OPT_REF_IDS if ref_ids else 0, C.byref(g))
        if rc:
            raise _lib.PfsCdcError(rc, "pfscdc_group_create failed (no GPU or bad params)")
        self.g = g

    def __len__(self) -> int:
        return len(self.devices)

    def close(self) -> None:
        if getattr(self, "g", None):
            self.lib.pfscdc_group_destroy(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc:
            msg = self.lib.pfscdc_group_last_error(self.g)
            raise _lib.PfsCdcError(rc, f"{what}: {msg.decode() if msg else ''}")

    def member_ctx(self, k: int) -> int:
        return self.lib.pfscdc_group_ctx(self.g, k)

    def _result(self, nfiles: int) -> ScanResult:
        n = int(self.lib.pfscdc_group_num_segments(self.g))
        dt = _lib.segment_dtype()
        ptr = self.lib.pfscdc_group_segments(self.g)
        segs = np.frombuffer(C.string_at(ptr, n * dt.itemsize), dtype=dt).copy() if n else \
            np.zeros(0, dtype=dt)
        bp = self.lib.pfscdc_group_file_segment_begin(self.g)
        begin = np.ctypeslib.as_array(bp, shape=(nfiles + 1,)).copy()
        refs = None
        if self.ref_ids:
            rdt = _lib.ref_dtype()
            rp = self.lib.pfscdc_group_refs(self.g)
            refs = np.frombuffer(C.string_at(rp, n * rdt.itemsize), dtype=rdt).copy() \
                if (n and rp) else np.zeros(0, dtype=rdt)
        return ScanResult(segs, begin, refs=refs)

    def part_begin(self) -> Optional[np.ndarray]:
        """The dealing of the last scan (n + 1 entries; None after a stream scan)."""
        p = self.lib.pfscdc_group_part_begin(self.g)
        return np.ctypeslib.as_array(p, shape=(len(self) + 1,)).copy() if p else None

    def scan(self, data, file_offsets: Sequence[int]) -> ScanResult:
        """pfscdc_group_scan over host bytes (bytes/bytearray/np.uint8)."""
        offs = _offsets_array(file_offsets)
        arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
            else np.ascontiguousarray(data, dtype=np.uint8)
        rc = self.lib.pfscdc_group_scan(self.g, arr.ctypes.data if arr.size else None, arr.size,
                                        offs.ctypes.data_as(C.POINTER(C.c_uint64)), len(offs) - 1)
        self._check(rc, "group_scan")
        return self._result(len(offs) - 1)

    def scan_stream(self, data) -> ScanResult:
        """pfscdc_group_scan_stream: one stream (host bytes) split across the members."""
        arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
            else np.ascontiguousarray(data, dtype=np.uint8)
        rc = self.lib.pfscdc_group_scan_stream(self.g, arr.ctypes.data if arr.size else None,
                                               arr.size)
        self._check(rc, "group_scan_stream")
        return self._result(1)

    def scan_resident(self, member_bytes: Sequence, file_offsets: Sequence[int],
                      part_begin: Optional[Sequence[int]] = None) -> ScanResult:
        """pfscdc_group_scan_resident: member_bytes[k] a torch uint8 tensor on member k's
        device holding files [part_begin[k], part_begin[k+1]) (None: pfscdc_deal's split)."""
        import torch

        offs = _offsets_array(file_offsets)
        ptrs = (C.c_void_p * len(self))()
        for k, t in enumerate(member_bytes):
            if t is not None and t.numel():
                ptrs[k] = t.data_ptr()
        torch.cuda.synchronize()  # bytes written by torch work are visible to every member
        pb = None
        if part_begin is not None:
            pb = np.ascontiguousarray(np.asarray(part_begin, dtype=np.uint32))
        rc = self.lib.pfscdc_group_scan_resident(
            self.g, ptrs, offs.ctypes.data_as(C.POINTER(C.c_uint64)), len(offs) - 1,
            pb.ctypes.data_as(C.POINTER(C.c_uint32)) if pb is not None else None)
        self._check(rc, "group_scan_resident")
        return self._result(len(offs) - 1)

    def fill_synthetic_resident(self, file_offsets: Sequence[int], seed: int,
                                mode: int = SYNTH_RANDOM) -> list:
        """The synthetic files of file_offsets generated in place on the members, dealt as
        pfscdc_deal does: one torch tensor per member (its files, contiguous)."""
        import torch

        offs = _offsets_array(file_offsets)
        pb = deal(offs, len(self))
        torch.cuda.synchronize()  # recycled allocator blocks: torch's work on them is done
        out = []
        for k, dev in enumerate(self.devices):
            f0, f1 = int(pb[k]), int(pb[k + 1])
            nb = int(offs[f1] - offs[f0])
            t = torch.empty(max(nb, 1), dtype=torch.uint8, device=f"cuda:{dev}")
            if f1 > f0 and nb:
                local = np.ascontiguousarray(offs[f0:f1 + 1] - offs[f0])
                ids = np.arange(f0, f1, dtype=np.uint32)
                rc = self.lib.pfscdc_fill_synthetic_pieces(
                    self.member_ctx(k), t.data_ptr(), local.ctypes.data_as(C.POINTER(C.c_uint64)),
                    f1 - f0, ids.ctypes.data_as(C.POINTER(C.c_uint32)), None, seed, mode)
                self._check(rc, "fill_synthetic_pieces")
            out.append(t[:nb])
        return out

    def timings(self) -> dict:
        ms = (C.c_float * len(self))()
        g_ms, g_b = C.c_float(), C.c_uint64()
        self._check(self.lib.pfscdc_group_last_timings(self.g, ms, C.byref(g_ms), C.byref(g_b)),
                    "group_last_timings")
        return {"member_ms": list(ms), "gather_ms": g_ms.value, "gather_bytes": int(g_b.value)}

    def index_device(self) -> tuple[int, int, int]:
        """(device segments pointer, device refs pointer, index device) of the gathered index."""
        s, r, d = C.c_void_p(), C.c_void_p(), C.c_int()
        self._check(self.lib.pfscdc_group_index_device(self.g, C.byref(s), C.byref(r), C.byref(d)),
                    "group_index_device")
        return s.value or 0, r.value or 0, d.value
