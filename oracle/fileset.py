"""pachd-level stream formation restated in Python — TEST INFRASTRUCTURE (oracle) ONLY.

Only ``tests/`` may use this module; the product path (``pfs_amd``) never imports it.

What it restates (paths relative to /root/reference/src/internal):

* ``storage/fileset/util.go:67-88``            Clean / IsDir (Go ``path.Clean`` restated below)
* ``storage/fileset/buffer.go:10-106``         Buffer: additive / deletive maps, sortFiles
* ``storage/fileset/unordered_writer.go:45-149,170-179``  Put (io.CopyN against memAvailable,
  serialize at 0, re-Add the same path), serialize / withWriter, Delete (files, and
  directories over the merged view of the filesets serialized so far), Close
* ``storage/fileset/merge.go:37-78,157-164``   merged (path, tag) view: a group is live iff its
  last stream (deletive before additive within a fileset, filesets in order) is additive
* ``storage/fileset/writer.go:36-182``         fileset.Writer: Add (Annotate + Write), Delete
  (deletive index), callback (per-file DataRefs), Close (Primitive{Additive, Deletive, SizeBytes})
* ``storage/fileset/index/writer.go:12-162``   multilevel index.Writer: level k chunked with
  WithRollingHashConfig(20, k), entries framed by pbutil (int64 LE length + proto,
  ``pbutil/pbutil.go:64-80``), Range{Offset, LastPath, ChunkRef} set by the level callback,
  root = the index of the last callback while closing
* ``storage/chunk/util.go:25-30``              Reference(dataRef)
* ``storage/chunk/chunk.proto``, ``storage/fileset/index/index.proto``  message layout; encoded
  here with the ``protobuf`` runtime from descriptors (an encoder independent of the product's)

Chunking and Ref ids come from ``oracle.chunker`` (chunk.Writer restated, with chunk.Create).
The upload and the Postgres metadata (fileset ids, composite) are out of scope.
Parity status: restated from the reference source; unpinned against a Go run.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from . import chunker as Ch

DEFAULT_FILE_TAG = "default"          # fileset/storage.go:39
DEFAULT_MEMORY_THRESHOLD = 10 ** 9    # fileset/storage.go:23 (units.GB, decimal)
INDEX_AVERAGE_BITS = 20               # index/writer.go:13
CHACHA20 = 1                          # chunk.proto EncryptionAlgo
MAX_INDEX_LEVELS = 32                 # guard: Go would add levels forever if entries >= avg


# ---------------------------------------------------------------- paths

def go_path_clean(p: str) -> str:
    """Go ``path.Clean`` (lexical: collapse //, drop ., resolve .. , no trailing /)."""
    if p == "":
        return "."
    rooted = p[0] == "/"
    n = len(p)
    out: list[str] = []
    r, dotdot = 0, 0
    if rooted:
        out.append("/")
        r, dotdot = 1, 1
    while r < n:
        if p[r] == "/":
            r += 1
        elif p[r] == "." and (r + 1 == n or p[r + 1] == "/"):
            r += 1
        elif p[r] == "." and r + 1 < n and p[r + 1] == "." and (r + 2 == n or p[r + 2] == "/"):
            r += 2
            if len(out) > dotdot:
                w = len(out) - 1
                while w > dotdot and out[w] != "/":
                    w -= 1
                del out[w:]
            elif not rooted:
                if out:
                    out.append("/")
                out += [".", "."]
                dotdot = len(out)
        else:
            if (rooted and len(out) != 1) or (not rooted and len(out) != 0):
                out.append("/")
            while r < n and p[r] != "/":
                out.append(p[r])
                r += 1
    return "".join(out) if out else "."


def is_dir(p: str) -> bool:
    return p.endswith("/")


def clean(p: str, isdir: bool) -> str:
    """fileset.Clean (util.go:67-77)."""
    p = go_path_clean(p)
    if p == ".":
        return "/"
    y = "/" + p.strip("/")
    if isdir and not is_dir(y):
        y += "/"
    return y


# ---------------------------------------------------------------- index messages

@dataclass
class Index:
    path: str
    tag: Optional[str] = None             # File.Tag (File is non-nil iff tag is not None)
    data_refs: list = field(default_factory=list)   # chunker.DataRef
    range: Optional[tuple] = None         # (offset, last_path, chunker.Ref)


def _pool():
    fdp = descriptor_pb2.FileDescriptorProto(name="pfs_oracle.proto", package="pfs", syntax="proto3")
    T = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields):
        m = fdp.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
    O, R = T.LABEL_OPTIONAL, T.LABEL_REPEATED
    msg("Ref", [("id", 1, T.TYPE_BYTES, O, None), ("size_bytes", 2, T.TYPE_INT64, O, None),
                ("edge", 3, T.TYPE_BOOL, O, None), ("dek", 4, T.TYPE_BYTES, O, None),
                ("encryption_algo", 5, T.TYPE_INT32, O, None),
                ("compression_algo", 6, T.TYPE_INT32, O, None)])
    msg("DataRef", [("ref", 1, T.TYPE_MESSAGE, O, ".pfs.Ref"), ("hash", 2, T.TYPE_BYTES, O, None),
                    ("offset_bytes", 3, T.TYPE_INT64, O, None),
                    ("size_bytes", 4, T.TYPE_INT64, O, None)])
    msg("Range", [("offset", 1, T.TYPE_INT64, O, None), ("last_path", 2, T.TYPE_STRING, O, None),
                  ("chunk_ref", 3, T.TYPE_MESSAGE, O, ".pfs.DataRef")])
    msg("File", [("tag", 1, T.TYPE_STRING, O, None),
                 ("data_refs", 2, T.TYPE_MESSAGE, R, ".pfs.DataRef")])
    msg("Index", [("path", 1, T.TYPE_STRING, O, None), ("range", 2, T.TYPE_MESSAGE, O, ".pfs.Range"),
                  ("file", 3, T.TYPE_MESSAGE, O, ".pfs.File")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return {n: message_factory.GetMessageClass(pool.FindMessageTypeByName("pfs." + n))
            for n in ("Ref", "DataRef", "Range", "File", "Index")}


_M = None


def _msgs():
    global _M
    if _M is None:
        _M = _pool()
    return _M


def _fill_ref(m, ref: Ch.Ref) -> None:
    # chunk.Create sets Id, SizeBytes, Dek, EncryptionAlgo=CHACHA20, CompressionAlgo=NONE;
    # processChunk sets Edge (writer.go:239)
    m.id = ref.id
    m.size_bytes = ref.size_bytes
    m.edge = ref.edge
    m.dek = ref.dek
    m.encryption_algo = CHACHA20
    m.compression_algo = 0


def _fill_dataref(m, d: Ch.DataRef) -> None:
    _fill_ref(m.ref, d.ref)
    m.hash = d.hash
    m.offset_bytes = d.offset_bytes
    m.size_bytes = d.size_bytes


def encode_index(idx: Index) -> bytes:
    M = _msgs()
    m = M["Index"]()
    m.path = idx.path
    if idx.range is not None:
        off, last_path, ref = idx.range
        m.range.SetInParent()
        m.range.offset = off
        m.range.last_path = last_path
        # chunk.Reference(dataRef): {Ref, SizeBytes = Ref.SizeBytes} (chunk/util.go:25-30)
        _fill_ref(m.range.chunk_ref.ref, ref)
        m.range.chunk_ref.size_bytes = ref.size_bytes
    if idx.tag is not None:
        m.file.SetInParent()
        m.file.tag = idx.tag
        for d in idx.data_refs:
            _fill_dataref(m.file.data_refs.add(), d)
    return m.SerializeToString(deterministic=True)


def frame(b: bytes) -> bytes:
    """pbutil WriteBytes: int64 little-endian length, then the bytes."""
    return len(b).to_bytes(8, "little", signed=True) + b


# ---------------------------------------------------------------- streaming chunk writer

class _ChunkWriter(Ch._SegmentReplayWriter):
    """chunk.Writer fed annotation by annotation (each annotation's bytes in one call), with
    chunk.Create refs; records every chunk for the event log."""

    def __init__(self, params: Ch.Params, cb, log: list, stream: tuple):
        super().__init__(cb=cb, params=params, with_ref_id=True)
        self.log, self.stream = log, stream

    def add(self, data, bytes_: bytes) -> None:
        self.annotate(Ch.Annotation(data=data))
        self.write_segments(bytes_, Ch.segments_numpy(bytes_, self.p) if bytes_ else [])

    def _process_chunk(self, chunk, edge, annotations):
        super()._process_chunk(chunk, edge, annotations)
        self.log.append(("chunk",) + self.stream + (len(chunk), edge, self.last_ref.id))
        self.chunks.clear()  # keep only the log (filesets may be large)


# ---------------------------------------------------------------- index.Writer

class IndexWriter:
    """index.Writer (index/writer.go:27-162)."""

    def __init__(self, which: int, log: list, index_params: Optional[Ch.Params] = None):
        self.which, self.log = which, log
        self.base = index_params or Ch.Params(average_bits=INDEX_AVERAGE_BITS, seed=0)
        self.levels: list = []      # [chunk writer, lastIdx]
        self.closed = False
        self.root: Optional[Index] = None

    def _new_level(self, level: int) -> None:
        p = Ch.Params(self.base.average_bits, self.base.seed + level, self.base.min, self.base.max)
        cw = _ChunkWriter(p, lambda anns, lv=level: self._callback(lv, anns), self.log,
                          (self.which, level))
        self.levels.append([cw, None])

    def write_index(self, idx: Index, level: int = 0) -> None:
        if not self.levels:
            self._new_level(0)
        b = frame(encode_index(idx))
        if level == 0:
            self.log.append(("index", self.which, b))
        self.levels[level][0].add(idx, b)

    def _callback(self, level: int, annotations: list) -> None:
        if not annotations:
            return
        lw = self.levels[level]
        idx, dref = annotations[0].data, annotations[0].next_data_ref
        if len(annotations) > 1 and lw[1] is not None and idx.path == lw[1].path:
            idx, dref = annotations[1].data, annotations[1].next_data_ref
        lw[1] = annotations[-1].data
        last_path = lw[1].range[1] if lw[1].range is not None else lw[1].path
        if dref is None:
            raise RuntimeError("index chunk without a data ref (Go: nil dereference)")
        idx.range = (dref.offset_bytes, last_path, dref.ref)
        if self.closed:
            self.root = idx
        if level == len(self.levels) - 1:
            if level + 1 >= MAX_INDEX_LEVELS:
                raise RuntimeError("index levels do not converge (an entry >= the index avg)")
            self._new_level(level + 1)
        self.write_index(idx, level + 1)

    def close(self) -> Optional[Index]:
        self.closed = True
        i = 0
        while i < len(self.levels):
            cw = self.levels[i][0]
            cw.close()
            if cw.annotation_count == 1 and cw.chunk_count == 1:
                break
            i += 1
        # A level above the one Close stopped at is never closed.  If it was cut while being
        # written (its one entry at or above the index min), the reference runs that chunk's
        # callback, which overwrites the root once closed is set, concurrently with Close's
        # return (index/writer.go:117-123, 148-161): the outcome is a race, so refuse it.
        # Unreachable with the reference's parameters (entries ~100 KB at most, index min 1 MB).
        for lw in self.levels[i + 1:]:
            if lw[0].chunk_count:
                raise RuntimeError("index level above the closed top was cut while written "
                                   "(the reference races its callback against Close)")
        return self.root


# ---------------------------------------------------------------- fileset.Writer

@dataclass
class Primitive:
    additive: Optional[bytes]   # encoded root Index (None: empty index)
    deletive: Optional[bytes]
    size_bytes: int
    files: list                 # (path, tag) additive, in order
    deletes: list               # (path, tag) deletive, in order


class FilesetWriter:
    """fileset.Writer (fileset/writer.go:36-182)."""

    def __init__(self, params: Ch.Params, log: list, index_params: Optional[Ch.Params] = None):
        self.log = log
        self.additive = IndexWriter(0, log, index_params)
        self.deletive = IndexWriter(1, log, index_params)
        self.cw = _ChunkWriter(params, self._callback, log, (-1, 0))
        self.idx = self.delete_idx = self.last_idx = None
        self.size_bytes = 0
        self.files, self.deletes = [], []

    @staticmethod
    def _check_path(prev: Optional[Index], idx: Index) -> None:
        if prev is None:
            return
        if prev.path == idx.path and prev.tag == idx.tag:
            raise ValueError(f"cannot write same path ({idx.path}) and tag ({idx.tag}) twice")
        if prev.path > idx.path:
            raise ValueError(f"cannot write path ({idx.path}) after ({prev.path})")

    def add(self, path: str, tag: str, data: bytes) -> None:
        idx = Index(path=path, tag=tag)
        self._check_path(self.idx, idx)
        self.idx = idx
        self.files.append((path, tag))
        self.cw.add(idx, data)
        self.size_bytes += len(data)

    def delete(self, path: str, tag: str) -> None:
        idx = Index(path=path, tag=tag)
        self._check_path(self.delete_idx, idx)
        self.delete_idx = idx
        self.deletes.append((path, tag))
        self.deletive.write_index(idx)

    def _callback(self, annotations: list) -> None:
        for a in annotations:
            idx = a.data
            if self.last_idx is None:
                self.last_idx = idx
            if idx.path != self.last_idx.path or idx.tag != self.last_idx.tag:
                self.additive.write_index(self.last_idx)
                self.last_idx = idx
            if a.next_data_ref is not None:
                self.last_idx.data_refs.append(a.next_data_ref)

    def close(self) -> Primitive:
        self.cw.close()
        if self.last_idx is not None:
            self.additive.write_index(self.last_idx)
        a = self.additive.close()
        d = self.deletive.close()
        return Primitive(encode_index(a) if a else None, encode_index(d) if d else None,
                         self.size_bytes, self.files, self.deletes)


# ---------------------------------------------------------------- Buffer + UnorderedWriter

class Buffer:
    """fileset.Buffer (buffer.go:10-106).  Inner dicts stay when emptied, as Go's maps do."""

    def __init__(self):
        self.additive: dict[str, dict[str, bytearray]] = {}
        self.deletive: dict[str, dict[str, None]] = {}

    def add(self, path: str, tag: str) -> bytearray:
        path = clean(path, False)
        return self.additive.setdefault(path, {}).setdefault(tag, bytearray())

    def delete(self, path: str, tag: str) -> None:
        path = clean(path, is_dir(path))
        if is_dir(path):
            for f in [f for f in self.additive if f.startswith(path)]:
                del self.additive[f]
            return
        if path in self.additive:
            self.additive[path].pop(tag, None)
        self.deletive.setdefault(path, {})[tag] = None

    def walk_additive(self):
        return sorted(((p, t, bytes(b)) for p, tags in self.additive.items() for t, b in tags.items()),
                      key=lambda x: (x[0].encode(), x[1].encode()))

    def walk_deletive(self):
        return sorted(((p, t) for p, tags in self.deletive.items() for t in tags),
                      key=lambda x: (x[0].encode(), x[1].encode()))

    def empty(self) -> bool:
        return not self.additive and not self.deletive


class UnorderedWriter:
    """fileset.UnorderedWriter (unordered_writer.go), storage = the list of Primitives."""

    def __init__(self, params: Ch.Params = Ch.Params(), mem_threshold: int = DEFAULT_MEMORY_THRESHOLD,
                 index_params: Optional[Ch.Params] = None):
        self.params, self.index_params = params, index_params
        self.mem_threshold = self.mem_available = mem_threshold
        self.buffer = Buffer()
        self.filesets: list[Primitive] = []
        self.log: list = []           # per fileset: chunk / index events

    def put(self, p: str, tag: str, append_file: bool, data: bytes) -> None:
        if tag == "":
            tag = DEFAULT_FILE_TAG
        if not append_file:
            self.buffer.delete(p, tag)
        w = self.buffer.add(p, tag)
        pos = 0
        while True:
            # io.CopyN(w, r, memAvailable): EOF iff fewer than memAvailable bytes were left
            n = min(self.mem_available, len(data) - pos)
            w += data[pos:pos + n]
            pos += n
            eof = n < self.mem_available
            self.mem_available -= n
            if eof:
                return
            if self.mem_available == 0:
                self.serialize()
                w = self.buffer.add(p, tag)

    def serialize(self) -> None:
        if self.buffer.empty():
            return
        log: list = []
        fw = FilesetWriter(self.params, log, self.index_params)
        for path, tag, data in self.buffer.walk_additive():
            fw.add(path, tag, data)
        for path, tag in self.buffer.walk_deletive():
            fw.delete(path, tag)
        self.filesets.append(fw.close())
        self.log.append(log)
        self.buffer = Buffer()
        self.mem_available = self.mem_threshold

    def _live(self, prefix: str):
        """(path, tag) groups of the merged view of the serialized filesets (merge.go)."""
        state: dict = {}
        for fs in self.filesets:
            for k in fs.deletes:
                state[k] = False
            for k in fs.files:
                state[k] = True
        return sorted((k for k, v in state.items() if v and k[0].startswith(prefix)),
                      key=lambda k: (k[0].encode(), k[1].encode()))

    def delete(self, p: str, tag: str = "") -> None:
        if tag == "":
            tag = DEFAULT_FILE_TAG
        p = clean(p, is_dir(p))
        if is_dir(p):
            self.buffer.delete(p, tag)
            for path, _ in self._live(p):
                self.delete(path, tag)
            return
        self.buffer.delete(p, tag)

    def close(self) -> list:
        self.serialize()
        return self.filesets
