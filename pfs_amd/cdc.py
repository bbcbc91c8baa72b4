"""Batch CDC + content-hash API over libpfscdc (one GPU per ``Chunker``).

``Chunker.scan`` is the batch form of the reference's per-file ``Writer.Annotate`` +
``Writer.Write`` + ``processChunk`` hashing (/root/reference/src/internal/storage/chunk/
writer.go:118-196,233-312): it returns, for every file of the batch, its segments (the
bytes of that file inside one chunk, i.e. one DataRef) with their BLAKE2b-256 digests.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib


SYNTH_RANDOM, SYNTH_DEDUP_BLOCKS, SYNTH_DEDUP_FILES = 0, 1, 2  # pfscdc.h PFSCDC_SYNTH_*


@dataclass(frozen=True)
class ChunkParams:
    """chunk.WithRollingHashConfig + WithMinMax (chunk/option.go:50-64); defaults writer.go:39-44."""
    average_bits: int = 23
    seed: int = 1
    min_chunk: int = 1_000_000
    max_chunk: int = 20_000_000

    def to_c(self) -> _lib.Params:
        return _lib.Params(self.average_bits, 0, self.seed, self.min_chunk, self.max_chunk)


@dataclass
class ScanResult:
    segments: np.ndarray        # structured SEGMENT_DTYPE, ordered by (file, offset)
    file_begin: np.ndarray      # uint64[nfiles+1]: file f owns segments[file_begin[f]:file_begin[f+1]]
    timings_ms: Optional[dict] = None
    refs: Optional[np.ndarray] = None  # REF_DTYPE (id, dek) per segment with ref_ids=True

    def file_segments(self, f: int) -> np.ndarray:
        return self.segments[int(self.file_begin[f]):int(self.file_begin[f + 1])]


def _offsets_array(file_offsets: Sequence[int]) -> np.ndarray:
    offs = np.ascontiguousarray(np.asarray(file_offsets, dtype=np.uint64))
    if offs.ndim != 1 or len(offs) < 1:
        raise ValueError("file_offsets must be a 1-D sequence of nfiles+1 offsets")
    return offs


class Chunker:
    """A GPU context bound to one device and one parameter set."""

    def __init__(self, params: ChunkParams = ChunkParams(), device: int = 0,
                 ref_ids: bool = False):
        self.lib = _lib.load()
        self.params = params
        self.device = device
        ctx = C.c_void_p()
        p = params.to_c()
        rc = self.lib.pfscdc_ctx_create(C.byref(p), device, C.byref(ctx))
        if rc:
            raise _lib.PfsCdcError(rc, "pfscdc_ctx_create failed (no GPU or bad params)")
        self.ctx = ctx
        self.ref_ids = False
        self.cuts_only = False
        self.ctext_in_place = False
        if ref_ids:
            self.set_ref_ids(True)

    def _set_options(self) -> None:
        o = (_lib.OPT_REF_IDS if self.ref_ids else 0) | (_lib.OPT_CUTS_ONLY if self.cuts_only else 0) \
            | (_lib.OPT_CTEXT_IN_PLACE if self.ctext_in_place else 0)
        self._check(self.lib.pfscdc_set_options(self.ctx, o), "set_options")

    def set_ref_ids(self, on: bool) -> None:
        """Also compute each segment's Ref (Id, Dek) of chunk.Create (pfscdc.h)."""
        self.ref_ids = on
        self._set_options()

    def set_ctext_in_place(self, on: bool) -> None:
        """commit_refs writes each chunk's ciphertext over its plaintext in the caller's
        device tensor (PFSCDC_OPT_CTEXT_IN_PLACE)."""
        self.ctext_in_place = on
        self._set_options()

    def set_cuts_only(self, on: bool) -> None:
        """Scans find the segments but leave their DataRef hashes to commit_refs
        (PFSCDC_OPT_CUTS_ONLY)."""
        self.cuts_only = on
        self._set_options()

    def close(self) -> None:
        if getattr(self, "ctx", None):
            self.lib.pfscdc_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc:
            msg = self.lib.pfscdc_last_error(self.ctx)
            raise _lib.PfsCdcError(rc, f"{what}: {msg.decode() if msg else ''}")

    def set_stream(self, stream_handle: Optional[int]) -> None:
        self._check(self.lib.pfscdc_set_stream(self.ctx, stream_handle or None), "set_stream")

    def order_hash_after(self, other: Optional["Chunker"]) -> None:
        """Start each later scan's BLAKE2b kernel after ``other``'s last enqueued one
        (pfscdc_order_hash_after): steps in flight overlap scans with hash tails only."""
        self._check(self.lib.pfscdc_order_hash_after(self.ctx, other.ctx if other else None),
                    "order_hash_after")

    def wait_for(self, other: "Chunker") -> None:
        """Order every later call of this ctx after the work ``other`` has enqueued so far
        (pfscdc_stream_wait on pfscdc_stream_handle(other))."""
        h = self.lib.pfscdc_stream_handle(other.ctx)
        self._check(self.lib.pfscdc_stream_wait(self.ctx, h), "stream_wait")

    def _after_torch(self, *tensors) -> None:
        """Order the ctx stream after torch's current stream (pfscdc_stream_wait) when a
        call reads or writes torch CUDA tensors, so bytes written by a torch kernel or a
        non-blocking copy have landed before the library's kernels read them."""
        for t in tensors:
            if t is not None and getattr(t, "is_cuda", False):
                import torch

                h = torch.cuda.current_stream(t.device).cuda_stream
                self._check(self.lib.pfscdc_stream_wait(self.ctx, h or None), "stream_wait")
                return

    def scan_async(self, data, file_offsets: Sequence[int]) -> None:
        """Enqueue a batch.  ``data``: bytes/bytearray/np.uint8 array (host) or a torch uint8
        CUDA tensor (device-resident, 16-byte aligned)."""
        offs = _offsets_array(file_offsets)
        self._offs_keep = offs
        nfiles = len(offs) - 1
        on_dev = 0
        if hasattr(data, "is_cuda") and data.is_cuda:
            if data.dtype.itemsize != 1 or not data.is_contiguous():
                raise ValueError("device data must be a contiguous uint8 tensor")
            ptr, nbytes, on_dev = data.data_ptr(), data.numel(), 1
            self._data_keep = data
            self._after_torch(data)
        else:
            arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray, memoryview)) \
                else np.ascontiguousarray(data, dtype=np.uint8)
            self._data_keep = arr
            ptr, nbytes = (arr.ctypes.data if arr.size else None), arr.size
        rc = self.lib.pfscdc_scan_async(self.ctx, ptr, nbytes, on_dev,
                                        offs.ctypes.data_as(C.POINTER(C.c_uint64)), nfiles)
        self._check(rc, "scan_async")
        self._nfiles = nfiles

    def wait(self) -> ScanResult:
        self._check(self.lib.pfscdc_wait(self.ctx), "wait")
        n = self.lib.pfscdc_num_segments(self.ctx)
        dt = _lib.segment_dtype()
        if n:
            ptr = self.lib.pfscdc_segments(self.ctx)
            buf = C.string_at(ptr, n * dt.itemsize)
            segs = np.frombuffer(buf, dtype=dt).copy()
        else:
            segs = np.zeros(0, dtype=dt)
        bp = self.lib.pfscdc_file_segment_begin(self.ctx)
        begin = np.ctypeslib.as_array(bp, shape=(self._nfiles + 1,)).copy() if bp else \
            np.zeros(self._nfiles + 1, dtype=np.uint64)
        refs = None
        if self.ref_ids:
            rdt = _lib.ref_dtype()
            rp = self.lib.pfscdc_refs(self.ctx)
            refs = np.frombuffer(C.string_at(rp, n * rdt.itemsize), dtype=rdt).copy() \
                if (n and rp) else np.zeros(0, dtype=rdt)
        return ScanResult(segs, begin, refs=refs)

    def scan(self, data, file_offsets: Sequence[int]) -> ScanResult:
        self.scan_async(data, file_offsets)
        return self.wait()

    def timings(self) -> dict:
        out = (C.c_float * 5)()
        self._check(self.lib.pfscdc_last_timings(self.ctx, out), "timings")
        t = dict(zip(["scan", "compact", "select", "hash", "total"], list(out)))
        sp = (C.c_float * 2)()
        self._check(self.lib.pfscdc_last_kernel_spans(self.ctx, sp), "kernel_spans")
        t["scan_span"], t["hash_span"] = sp[0], sp[1]
        ck = (C.c_float * 2)()
        self._check(self.lib.pfscdc_last_kernel_clocks(self.ctx, ck), "kernel_clocks")
        t["scan_mhz"], t["hash_mhz"] = ck[0], ck[1]
        if self.ref_ids:
            ms = C.c_float()
            self._check(self.lib.pfscdc_last_ref_ms(self.ctx, C.byref(ms)), "timings")
            t["ref_ids"] = ms.value
        return t

    def get_chunks(self, ctext, chunk_offsets: Sequence[int], refs: np.ndarray, out=None):
        """chunk.Get for a batch of stored chunks (pfscdc_get_chunks): returns
        (plaintext, ok[nchunks]).  ``ctext``: host bytes/array or a torch uint8 CUDA tensor;
        ``out``: optional torch CUDA tensor for device-resident plaintext."""
        offs = _offsets_array(chunk_offsets)
        n = len(offs) - 1
        refs = np.ascontiguousarray(refs, dtype=_lib.ref_dtype())
        if len(refs) != n:
            raise ValueError("one ref per chunk")
        self._after_torch(ctext, out)
        if hasattr(ctext, "is_cuda") and ctext.is_cuda:
            cptr, nbytes, con = ctext.data_ptr(), ctext.numel(), 1
        else:
            arr = np.ascontiguousarray(np.frombuffer(ctext, dtype=np.uint8)
                                       if isinstance(ctext, (bytes, bytearray)) else ctext,
                                       dtype=np.uint8)
            cptr, nbytes, con = (arr.ctypes.data if arr.size else None), arr.size, 0
            self._get_keep = arr
        if out is not None:
            optr, oon, res = out.data_ptr(), 1, out
        else:
            res = np.empty(nbytes, dtype=np.uint8)
            optr, oon = (res.ctypes.data if nbytes else None), 0
        ok = np.zeros(max(n, 1), dtype=np.uint8)
        rc = self.lib.pfscdc_get_chunks(self.ctx, cptr, nbytes, con,
                                        offs.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                                        refs.ctypes.data if n else None, optr, oon,
                                        ok.ctypes.data)
        self._check(rc, "get_chunks")
        return res, ok[:n].astype(bool)

    def form_chunks(self, stream_file_begin: Optional[Sequence[int]] = None):
        """Chunks chunk.Writer forms over the last scan's files (pfscdc_form_chunks), each
        stream (files [b[k], b[k+1])) one writer.  Returns (chunk_offsets uint64[n+1],
        content_hashes uint8[n,32], hash_known bool[n])."""
        if stream_file_begin is None:
            sb, ns, sbp = None, 0, None
        else:
            sb = np.ascontiguousarray(np.asarray(stream_file_begin, dtype=np.uint32))
            ns, sbp = len(sb) - 1, sb.ctypes.data_as(C.POINTER(C.c_uint32))
        cap = max(16, self._nfiles + 16)  # one chunk per 1 MB (min) plus one per stream
        cap += int(self._offs_keep[-1]) // 1_000_000 if self._nfiles else 0
        while True:
            offs = np.zeros(cap + 1, dtype=np.uint64)
            hashes = np.zeros((cap, 32), dtype=np.uint8)
            known = np.zeros(cap, dtype=np.uint8)
            n = C.c_uint64()
            rc = self.lib.pfscdc_form_chunks(self.ctx, sbp, ns,
                                             offs.ctypes.data_as(C.POINTER(C.c_uint64)),
                                             hashes.ctypes.data, known.ctypes.data, cap,
                                             C.byref(n))
            if rc == _lib.PFSCDC_ENOMEM and n.value > cap:
                cap = n.value
                continue
            self._check(rc, "form_chunks")
            k = n.value
            return offs[:k + 1].copy(), hashes[:k].copy(), known[:k].astype(bool)

    def commit_refs(self, data, chunk_offsets: Sequence[int], hash_known, create: bool = True):
        """After a cuts-only scan of ``data`` and form_chunks: the DataRef hashes of the
        scan's segments and the chunks' content hashes in one launch, then chunk.Create
        (pfscdc_commit_refs).  Returns (refs REF_DTYPE[n], content_hashes uint8[n,32],
        segment_hashes uint8[nsegs,32]); with create=False the hashes only (refs is None)."""
        offs = _offsets_array(chunk_offsets)
        n = len(offs) - 1
        nsegs = int(self.lib.pfscdc_num_segments(self.ctx))
        hashes = np.zeros((max(n, 1), 32), dtype=np.uint8)
        seg = np.zeros((max(nsegs, 1), 32), dtype=np.uint8)
        known = np.ascontiguousarray(np.asarray(hash_known, dtype=np.uint8))
        if hasattr(data, "is_cuda") and data.is_cuda:
            ptr, nbytes, on = data.data_ptr(), data.numel(), 1
        else:
            arr = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8)
                                       if isinstance(data, (bytes, bytearray)) else data,
                                       dtype=np.uint8)
            ptr, nbytes, on = (arr.ctypes.data if arr.size else None), arr.size, 0
        refs = np.zeros(max(n, 1), dtype=_lib.ref_dtype()) if create else None
        rc = self.lib.pfscdc_commit_refs(self.ctx, ptr, nbytes, on,
                                         offs.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                                         hashes.ctypes.data, known.ctypes.data if n else None,
                                         refs.ctypes.data if create else None, seg.ctypes.data)
        self._check(rc, "commit_refs")
        return (refs[:n] if create else None), hashes[:n], seg[:nsegs]

    def create_refs(self, data, chunk_offsets: Sequence[int], content_hashes=None,
                    hash_known=None):
        """chunk.Create(CreateOptions{}) per chunk (pfscdc_create_refs).  Returns (refs
        REF_DTYPE[n], content_hashes uint8[n,32]).  ``data``: host bytes/array or a torch
        uint8 CUDA tensor."""
        offs = _offsets_array(chunk_offsets)
        n = len(offs) - 1
        hashes = np.zeros((max(n, 1), 32), dtype=np.uint8)
        known = None
        if content_hashes is not None:
            hashes[:n] = np.asarray(content_hashes, dtype=np.uint8).reshape(n, 32)
            known = np.ascontiguousarray(np.asarray(hash_known, dtype=np.uint8)
                                         if hash_known is not None else np.ones(n, np.uint8))
        if hasattr(data, "is_cuda") and data.is_cuda:
            ptr, nbytes, on = data.data_ptr(), data.numel(), 1
            self._after_torch(data)
        else:
            arr = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8)
                                       if isinstance(data, (bytes, bytearray)) else data,
                                       dtype=np.uint8)
            ptr, nbytes, on = (arr.ctypes.data if arr.size else None), arr.size, 0
            self._create_keep = arr
        refs = np.zeros(max(n, 1), dtype=_lib.ref_dtype())
        rc = self.lib.pfscdc_create_refs(self.ctx, ptr, nbytes, on,
                                         offs.ctypes.data_as(C.POINTER(C.c_uint64)), n,
                                         hashes.ctypes.data,
                                         known.ctypes.data if known is not None and n else None,
                                         refs.ctypes.data)
        self._check(rc, "create_refs")
        return refs[:n], hashes[:n]

    def last_create_ms(self) -> float:
        ms = C.c_float()
        self._check(self.lib.pfscdc_last_create_ms(self.ctx, C.byref(ms)), "create_ms")
        return ms.value

    def last_create_timings(self) -> dict:
        out = (C.c_float * 2)()
        self._check(self.lib.pfscdc_last_create_timings(self.ctx, out), "create_timings")
        return {"content_hash": out[0], "ref_id": out[1]}

    def last_get_ms(self) -> float:
        ms = C.c_float()
        self._check(self.lib.pfscdc_last_get_ms(self.ctx, C.byref(ms)), "get_ms")
        return ms.value

    def candidates(self, data, halo: int = 0, cap: int = 1 << 16) -> np.ndarray:
        """Sorted candidate positions of one range of a split stream (pfscdc_candidates):
        offsets p >= halo into ``data`` (the range with ``halo`` bytes of the previous range
        in front) where the rolling hash of bytes [p-63, p] passes the mask test."""
        ptr, nbytes, on_dev = self._bytes_arg(data)
        while True:
            out = np.zeros(max(cap, 1), dtype=np.uint64)
            n = C.c_uint64()
            rc = self.lib.pfscdc_candidates(self.ctx, ptr, nbytes, on_dev, halo,
                                            out.ctypes.data_as(C.POINTER(C.c_uint64)), cap,
                                            C.byref(n))
            if rc == _lib.PFSCDC_ENOMEM and n.value > cap:
                cap = n.value
                continue
            self._check(rc, "candidates")
            return out[:n.value].copy()

    def hash_ranges(self, data, begins, sizes) -> np.ndarray:
        """BLAKE2b-256 of byte ranges of ``data`` (pfscdc_hash_ranges): uint8[n, 32]."""
        b = np.ascontiguousarray(np.asarray(begins, dtype=np.uint64))
        z = np.ascontiguousarray(np.asarray(sizes, dtype=np.uint64))
        if b.shape != z.shape:
            raise ValueError("begins and sizes differ in length")
        ptr, nbytes, on_dev = self._bytes_arg(data)
        out = np.zeros((max(len(b), 1), 32), dtype=np.uint8)
        rc = self.lib.pfscdc_hash_ranges(self.ctx, ptr, nbytes, on_dev,
                                         b.ctypes.data_as(C.POINTER(C.c_uint64)),
                                         z.ctypes.data_as(C.POINTER(C.c_uint64)), len(b),
                                         out.ctypes.data)
        self._check(rc, "hash_ranges")
        return out[:len(b)]

    def _bytes_arg(self, data):
        """(pointer, nbytes, on_device) of a torch CUDA tensor or host bytes; keeps the
        host array alive on self for the call."""
        if hasattr(data, "is_cuda") and data.is_cuda:
            if data.dtype.itemsize != 1 or not data.is_contiguous():
                raise ValueError("device data must be a contiguous uint8 tensor")
            self._after_torch(data)
            return data.data_ptr(), data.numel(), 1
        arr = np.frombuffer(data, dtype=np.uint8) \
            if isinstance(data, (bytes, bytearray, memoryview)) \
            else np.ascontiguousarray(data, dtype=np.uint8)
        self._arg_keep = arr
        return (arr.ctypes.data if arr.size else None), arr.size, 0

    def last_scan_bytes(self) -> int:
        """Bytes the last scan's candidate kernel rolled (the first min - 1 bytes of each file
        hold no cut point and are skipped; pfscdc_last_scan_bytes)."""
        v = C.c_uint64(0)
        self._check(self.lib.pfscdc_last_scan_bytes(self.ctx, C.byref(v)), "last_scan_bytes")
        return int(v.value)

    def last_scan_mode(self) -> int:
        """The skipping the last scan did (pfscdc_last_scan_mode): bit 1 the first min - 1
        bytes of each file, bit 2 past the cuts it settled (_lib.SCAN_SKIPPED_*)."""
        v = C.c_uint32(0)
        self._check(self.lib.pfscdc_last_scan_mode(self.ctx, C.byref(v)), "last_scan_mode")
        return int(v.value)

    def debug_candidates(self, cap: int = 1 << 20) -> np.ndarray:
        out = (C.c_uint64 * cap)()
        n = self.lib.pfscdc_debug_candidates(self.ctx, out, cap)
        return np.array(out[:min(n, cap)], dtype=np.uint64)

    def fill_synthetic_pieces(self, tensor, piece_offsets: Sequence[int], file_ids, file_starts,
                              seed: int, mode: int = SYNTH_RANDOM) -> None:
        """Fill a torch uint8 CUDA tensor with pieces of synthetic files: piece i = bytes
        [file_starts[i], ...) of file file_ids[i] (pfscdc_fill_synthetic_pieces)."""
        offs = _offsets_array(piece_offsets)
        ids = np.ascontiguousarray(np.asarray(file_ids, dtype=np.uint32))
        st = np.ascontiguousarray(np.asarray(file_starts, dtype=np.uint64))
        if len(ids) != len(offs) - 1 or len(st) != len(offs) - 1:
            raise ValueError("one file id and start per piece")
        self._after_torch(tensor)
        rc = self.lib.pfscdc_fill_synthetic_pieces(
            self.ctx, tensor.data_ptr(), offs.ctypes.data_as(C.POINTER(C.c_uint64)), len(ids),
            ids.ctypes.data_as(C.POINTER(C.c_uint32)) if len(ids) else None,
            st.ctypes.data_as(C.POINTER(C.c_uint64)) if len(st) else None, seed, mode)
        self._check(rc, "fill_synthetic_pieces")

    def fill_synthetic(self, tensor, file_offsets: Sequence[int], seed: int,
                       mode: int = SYNTH_RANDOM) -> None:
        """Fill a torch uint8 CUDA tensor with the synthetic byte stream (see pfscdc.h)."""
        offs = _offsets_array(file_offsets)
        self._after_torch(tensor)
        rc = self.lib.pfscdc_fill_synthetic_ex(self.ctx, tensor.data_ptr(),
                                               offs.ctypes.data_as(C.POINTER(C.c_uint64)),
                                               len(offs) - 1, seed, mode)
        self._check(rc, "fill_synthetic")


_POOL_FILE = 1 << 23
_M64 = (1 << 64) - 1


def _mix64(x: int) -> int:
    """murmur3 fmix64 (the dedup decision hash of pfscdc.h)."""
    x &= _M64
    x = ((x ^ (x >> 33)) * 0xFF51AFD7ED558CCD) & _M64
    x = ((x ^ (x >> 33)) * 0xC4CEB9FE1A85EC53) & _M64
    return x ^ (x >> 33)


def _synth_words(fid: int, w0: int, nw: int, seed: int) -> np.ndarray:
    gamma = np.uint64((seed + 1) * 0x9E3779B97F4A7C15 % (1 << 64))
    with np.errstate(over="ignore"):
        z = (np.uint64(fid) << np.uint64(40)) | np.arange(w0, w0 + nw, dtype=np.uint64)
        z = z + gamma
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)


def synthetic_piece_bytes(file_id: int, start: int, n: int, seed: int,
                          mode: int = SYNTH_RANDOM) -> np.ndarray:
    """Bytes [start, start + n) of synthetic file ``file_id`` (host mirror of
    pfscdc_fill_synthetic_pieces for one piece)."""
    if n == 0:
        return np.zeros(0, dtype=np.uint8)

    def words(fid, a, m):  # bytes [a, a + m) of the word sequence of synthetic file fid
        return _synth_words(fid, a >> 3, ((a & 7) + m + 7) >> 3, seed)[a & 7:(a & 7) + m]

    if mode == SYNTH_DEDUP_FILES:
        h = _mix64((seed << 48) ^ (file_id << 24) ^ 0x5EEDF11E)
        return words(_POOL_FILE + ((h >> 1) & 63) if h & 1 else file_id, start, n)
    if mode == SYNTH_DEDUP_BLOCKS:
        out = np.empty(n, dtype=np.uint8)
        for k in range(start >> 20, ((start + n - 1) >> 20) + 1):
            b0, b1 = max(start, k << 20), min(start + n, (k + 1) << 20)
            h = _mix64((seed << 48) ^ (file_id << 24) ^ k ^ 0xC5C5C5C5)
            out[b0 - start:b1 - start] = (words(_POOL_FILE + ((h >> 1) & 63), b0 - (k << 20),
                                                b1 - b0) if h & 1 else words(file_id, b0, b1 - b0))
        return out
    return words(file_id, start, n)


def synthetic_bytes(file_offsets: Sequence[int], seed: int, mode: int = SYNTH_RANDOM) -> np.ndarray:
    """Host copy of the synthetic stream (same definition as the device generator)."""
    offs = np.asarray(file_offsets, dtype=np.uint64)
    out = np.empty(int(offs[-1]), dtype=np.uint8)
    for f in range(len(offs) - 1):
        a, b = int(offs[f]), int(offs[f + 1])
        n = b - a
        if n == 0:
            continue
        if mode == SYNTH_DEDUP_FILES:
            h = _mix64((seed << 48) ^ (f << 24) ^ 0x5EEDF11E)
            fid = _POOL_FILE + ((h >> 1) & 63) if h & 1 else f
            out[a:b] = _synth_words(fid, 0, (n + 7) // 8, seed)[:n]
        elif mode == SYNTH_DEDUP_BLOCKS:
            for k in range((n + (1 << 20) - 1) >> 20):
                o0, o1 = k << 20, min(n, (k + 1) << 20)
                h = _mix64((seed << 48) ^ (f << 24) ^ k ^ 0xC5C5C5C5)
                if h & 1:
                    words = _synth_words(_POOL_FILE + ((h >> 1) & 63), 0, (o1 - o0 + 7) // 8, seed)
                else:
                    words = _synth_words(f, o0 >> 3, (o1 - o0 + 7) // 8, seed)
                out[a + o0:a + o1] = words[:o1 - o0]
        else:
            out[a:b] = _synth_words(f, 0, (n + 7) // 8, seed)[:n]
    return out
