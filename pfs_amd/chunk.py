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


class ChunkStore:
    """The chunk client's object store (in memory, keyed by Ref.Id; pfscdc_store)."""

    def __init__(self):
        self.lib = _lib.load()
        s = C.c_void_p()
        rc = self.lib.pfscdc_store_create(C.byref(s))
        if rc:
            raise _lib.PfsCdcError(rc, "pfscdc_store_create")
        self._s = s

    def __len__(self) -> int:
        return self.lib.pfscdc_store_count(self._s)

    def get(self, ref_id: bytes) -> bytes:
        p, n = C.c_void_p(), C.c_uint64()
        rc = self.lib.pfscdc_store_get(self._s, ref_id, C.byref(p), C.byref(n))
        if rc:
            raise KeyError(ref_id.hex())
        return C.string_at(p, n.value) if n.value else b""

    def put(self, ref_id: bytes, ctext: bytes) -> None:
        rc = self.lib.pfscdc_store_put(self._s, ref_id, ctext, len(ctext))
        if rc:
            raise _lib.PfsCdcError(rc, "pfscdc_store_put")

    def __del__(self):
        try:
            if getattr(self, "_s", None):
                self.lib.pfscdc_store_destroy(self._s)
                self._s = None
        except Exception:
            pass


def _full(dr: DataRef) -> _lib.FullDataRef:
    f = _lib.FullDataRef()
    C.memmove(f.ref.id, dr.ref.id, 32)
    C.memmove(f.ref.dek, dr.ref.dek, 32)
    f.ref_size = dr.ref.size_bytes
    f.edge = int(dr.ref.edge)
    C.memmove(f.data.hash, dr.hash, 32)
    f.data.offset_bytes = dr.offset_bytes
    f.data.size_bytes = dr.size_bytes
    return f


class Storage:
    """``chunk.Storage`` bound to one GPU; ``store`` is its chunk client (Copy reads chunks
    back from it, writers without ``with_no_upload()`` upload into it)."""

    def __init__(self, device: int = 0, batch_bytes: int = DEFAULT_BATCH_BYTES,
                 store: Optional[ChunkStore] = None):
        self.device = device
        self.batch_bytes = batch_bytes
        self.store = store

    def new_writer(self, name: str, cb: Optional[Callable[[list], None]],
                   *opts: WriterOption) -> "Writer":
        if not name:
            raise ValueError("name must not be empty")  # storage.go:61-63 panics
        cfg = _WriterConfig()
        for o in opts:
            o(cfg)
        return Writer(cfg, cb, self.device, self.batch_bytes, self.store)


class Writer:
    def __init__(self, cfg: _WriterConfig, cb, device: int, batch_bytes: int,
                 store: Optional[ChunkStore] = None):
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
        self._store = store
        if store is not None:
            upload = cfg.ref_ids and not cfg.no_upload
            self._check(self.lib.pfscdc_writer_set_store(w, store._s, int(upload)), "set_store")

    def _on_chunk(self, _user, chunk_p, anns_p, n) -> int:
        try:
            ch = chunk_p.contents
            ref = Ref(size_bytes=ch.size_bytes, edge=bool(ch.edge),
                      chunk_index=-1 if ch.copied else ch.chunk_index)
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

    def prefetch(self, data_refs: list) -> None:
        """Batch chunk.Get of the chunks these DataRefs will certainly be re-rolled from."""
        arr = (_lib.FullDataRef * max(1, len(data_refs)))()
        for i, d in enumerate(data_refs):
            arr[i] = _full(d)
        self._check(self.lib.pfscdc_writer_prefetch(self._w, arr, len(data_refs)), "prefetch")

    def copy(self, data_ref: DataRef) -> None:
        """Writer.Copy (writer.go:315-420)."""
        f = _full(data_ref)
        self._check(self.lib.pfscdc_writer_copy(self._w, C.byref(f)), "Copy")

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


def hash_data_refs(hashes, device: int = 0, params: ChunkParams = ChunkParams()) -> bytes:
    """hashDataRefs (fileset/util.go:149-158) on the GPU: FileInfo.Hash of a file's DataRefs."""
    from .cdc import Chunker
    c = Chunker(params, device)
    buf = b"".join(bytes(h) for h in hashes)
    out = (C.c_uint8 * 32)()
    rc = c.lib.pfscdc_hash_data_refs(c.ctx, buf, len(buf) // 32, out)
    c.close()
    if rc:
        raise _lib.PfsCdcError(rc, "hash_data_refs")
    return bytes(out)


def merge_file_hash(store: ChunkStore, data_refs: list, device: int = 0,
                    params: ChunkParams = ChunkParams()) -> bytes:
    """MergeFileReader.Hash (fileset/merge.go:125-143): re-chunk a file's DataRefs through a
    fresh writer (cheap copies where whole chunks line up) and hash the resolved DataRefs.
    The Go writer there uses the default chunking; ``params`` is a test hook."""
    from .cdc import Chunker
    c = Chunker(params, device)
    arr = (_lib.FullDataRef * max(1, len(data_refs)))()
    for i, d in enumerate(data_refs):
        arr[i] = _full(d)
    out = (C.c_uint8 * 32)()
    rc = c.lib.pfscdc_merge_file_hash(c.ctx, store._s, arr, len(data_refs), out)
    msg = c.lib.pfscdc_last_error(c.ctx)
    c.close()
    if rc:
        raise _lib.PfsCdcError(rc, f"merge_file_hash: {msg.decode() if msg else ''}")
    return bytes(out)
