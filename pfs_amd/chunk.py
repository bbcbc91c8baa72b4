"""Host-side mirror of the reference chunk layer API, backed by the GPU path.

Reference interface (paths under /root/reference/src/internal/storage/chunk):

* ``Storage.NewWriter(ctx, name, cb, ...WriterOption) *Writer``   storage.go:60-66
* ``Writer.Annotate / Write / Close / ChunkCount / AnnotationCount`` writer.go:105-143,423
* ``WriterCallback func([]*Annotation) error``                      writer.go:31
* ``WithRollingHashConfig(averageBits, seed)``, ``WithMinMax(min, max)``,
  ``WithNoUpload()``                                                option.go:50-71
* ``Annotation{RefDataRefs, NextDataRef, Data}``, ``DataRef{Ref, Hash, OffsetBytes,
  SizeBytes}``, ``Ref{Id, SizeBytes, Edge, ...}``                   writer.go:23-28, chunk.proto

Same names, argument meaning and error behaviour: errors are sticky (writer.go:145-161),
Write before Annotate is an error (Go panics), callbacks run serially in chunk order
(chain.go:55-68) and a raised exception inside the callback aborts the writer.
Every chunk's ``Ref.id``/``Ref.dek`` are those of ``chunk.Create(ctx, CreateOptions{}, ...)``
(writer.go:255-271, transform.go:26-46), computed on the GPU over the assembled chunk bytes
(multi-file chunks and chunks spanning flushes included); the upload itself is out of scope.
Differences: the callback receives fresh ``Annotation`` objects whose ``data`` is the
annotated object (Go passes the original for the first piece and ``copyAnnotation`` copies
after a split; both carry the same ``Data``); ``without_ref_ids()`` (no reference
counterpart) skips the Ref computation for callers that only need DataRef hashes.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Callable, Optional

from . import _lib
from .cdc import ChunkParams

DEFAULT_BATCH_BYTES = 1 << 30


@dataclass
class Ref:
    size_bytes: int
    edge: bool
    chunk_index: int
    id: bytes = b""
    dek: bytes = b""


@dataclass
class DataRef:
    ref: Ref
    hash: bytes
    offset_bytes: int
    size_bytes: int


@dataclass
class Annotation:
    data: object = None
    next_data_ref: Optional[DataRef] = None
    ref_data_refs: list = field(default_factory=list)


WriterOption = Callable[["_WriterConfig"], None]


@dataclass
class _WriterConfig:
    average_bits: int = 23
    seed: int = 1
    min_chunk: int = 1_000_000
    max_chunk: int = 20_000_000
    no_upload: bool = False
    ref_ids: bool = True


def with_rolling_hash_config(average_bits: int, seed: int) -> WriterOption:
    def opt(c: _WriterConfig) -> None:
        c.average_bits, c.seed = average_bits, seed
    return opt


def with_min_max(min_chunk: int, max_chunk: int) -> WriterOption:
    def opt(c: _WriterConfig) -> None:
        c.min_chunk, c.max_chunk = min_chunk, max_chunk
    return opt


def without_ref_ids() -> WriterOption:
    """Skip Ref.Id/Dek (not a reference option: the Go writer always runs chunk.Create)."""
    def opt(c: _WriterConfig) -> None:
        c.ref_ids = False
    return opt


def with_no_upload() -> WriterOption:
    def opt(c: _WriterConfig) -> None:
        c.no_upload = True
    return opt


class Storage:
    """``chunk.Storage`` restricted to the writer side, bound to one GPU."""

    def __init__(self, device: int = 0, batch_bytes: int = DEFAULT_BATCH_BYTES):
        self.device = device
        self.batch_bytes = batch_bytes

    def new_writer(self, name: str, cb: Optional[Callable[[list], None]],
                   *opts: WriterOption) -> "Writer":
        if not name:
            raise ValueError("name must not be empty")  # storage.go:61-63 panics
        cfg = _WriterConfig()
        for o in opts:
            o(cfg)
        return Writer(cfg, cb, self.device, self.batch_bytes)


class Writer:
    def __init__(self, cfg: _WriterConfig, cb, device: int, batch_bytes: int):
        from .cdc import Chunker

        self.lib = _lib.load()
        self._chunker = Chunker(ChunkParams(cfg.average_bits, cfg.seed, cfg.min_chunk,
                                            cfg.max_chunk), device, ref_ids=cfg.ref_ids)
        self._cb = cb
        self._objs: dict[int, object] = {}
        self._next_id = 0
        self._exc: Optional[BaseException] = None
        self._cfun = _lib.WRITER_CB(self._on_chunk)
        w = C.c_void_p()
        rc = self.lib.pfscdc_writer_create(self._chunker.ctx, self._cfun, None, batch_bytes,
                                           C.byref(w))
        if rc:
            raise _lib.PfsCdcError(rc, "pfscdc_writer_create")
        self._w = w

    def _on_chunk(self, _user, chunk_p, anns_p, n) -> int:
        try:
            ch = chunk_p.contents
            ref = Ref(size_bytes=ch.size_bytes, edge=bool(ch.edge), chunk_index=ch.chunk_index)
            if ch.has_ref:
                ref.id, ref.dek = bytes(ch.ref.id), bytes(ch.ref.dek)
            out = []
            for i in range(n):
                a = anns_p[i]
                ann = Annotation(data=self._objs[a.user])
                if a.has_data_ref:
                    d = a.data_ref
                    ann.next_data_ref = DataRef(ref=ref, hash=bytes(d.hash),
                                                offset_bytes=d.offset_bytes,
                                                size_bytes=d.size_bytes)
                out.append(ann)
            if self._cb is not None:
                self._cb(out)
            return 0
        except BaseException as e:  # surfaced by the Writer call that triggered the flush
            self._exc = e
            return 1

    def _check(self, rc: int, what: str) -> None:
        if self._exc is not None:
            exc, self._exc = self._exc, None
            raise exc
        if rc:
            raise _lib.PfsCdcError(rc, what)

    def annotate(self, a: Annotation) -> None:
        uid = self._next_id
        self._next_id += 1
        self._objs[uid] = a.data
        self._check(self.lib.pfscdc_writer_annotate(self._w, uid), "Annotate")

    def write(self, data) -> int:
        buf = bytes(data)
        self._check(self.lib.pfscdc_writer_write(self._w, buf, len(buf)), "Write")
        return len(buf)

    def close(self) -> None:
        self._check(self.lib.pfscdc_writer_close(self._w), "Close")

    def chunk_count(self) -> int:
        return self.lib.pfscdc_writer_chunk_count(self._w)

    def annotation_count(self) -> int:
        return self.lib.pfscdc_writer_annotation_count(self._w)

    def __del__(self):
        try:
            if getattr(self, "_w", None):
                self.lib.pfscdc_writer_destroy(self._w)
                self._w = None
            if getattr(self, "_chunker", None):
                self._chunker.close()
        except Exception:
            pass
