"""Reference chunker restated in Python — TEST INFRASTRUCTURE (oracle) ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
this module; the product path (``pfs_amd``) never imports it.

What it restates (all paths relative to /root/reference):

* ``src/internal/storage/chunk/writer.go:12-44``   constants (window 64, avgBits 23, seed 1,
  min 1 MB, max 20 MB as decimal go-units sizes)
* ``writer.go:74-98,100-103``  newWriter / resetHash (Reset + Write(64 zero bytes))
* ``writer.go:118-130``        Annotate (cut before a file when buf.Len() >= avg)
* ``writer.go:132-143,163-196`` Write / roll / writeData (the cut rule)
* ``writer.go:198-231``        createChunk / splitAnnotations / copyAnnotation
* ``writer.go:233-253,288-312`` processChunk / processAnnotations / newDataRef
* ``writer.go:423-438``        Close (always emits a last chunk, possibly empty: E1)
* ``chunk/option.go:50-56``    WithRollingHashConfig (avg = 2^bits, mask = 2^bits-1, table)
* ``chunk/metadata.go:16-20`` + ``pachhash/hash.go:27-30`` Hash = BLAKE2b-256 (hashlib)
* ``chunk/transform.go:26-46,152-188`` Create with ``CreateOptions{}`` (writer.go:271 passes
  an EMPTY options struct: no compression, empty secret) -> Ref.Id = BLAKE2b(ChaCha20_k(chunk)),
  k = BLAKE2b(BLAKE2b(chunk)), zero nonce (optional, ``with_ref_id=True``)
* ``fileset/util.go:149-158``  hashDataRefs (FileInfo.Hash)

Two interchangeable segmenters are provided and cross-checked in tests: ``literal`` rolls a
``Buzhash64`` object byte by byte exactly like ``Writer.roll`` (small inputs only), and
``numpy`` evaluates the closed form ``h_i = XOR_k rotl(T[x_{i-k}], k)`` by doubling and then
applies the same cut rule.

Parity status: components pinned by known answers (Go seed-1 Int63 stream, rngCooked[0..1],
BLAKE2b RFC 7693 vectors); the composed boundary lists are "parity unpinned" against a Go
run (no Go toolchain here) — see DESIGN.md §Parity.
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np

from . import buzhash64

WINDOW_SIZE = 64
DEFAULT_AVERAGE_BITS = 23
DEFAULT_SEED = 1
DEFAULT_MIN = 1_000_000      # 1 * units.MB (docker/go-units v0.4.0: decimal)
DEFAULT_MAX = 20_000_000     # 20 * units.MB


def blake2b256(data) -> bytes:
    return hashlib.blake2b(bytes(data), digest_size=32).digest()


@dataclass(frozen=True)
class Params:
    average_bits: int = DEFAULT_AVERAGE_BITS
    seed: int = DEFAULT_SEED
    min: int = DEFAULT_MIN
    max: int = DEFAULT_MAX

    @property
    def avg(self) -> int:
        return 1 << self.average_bits

    @property
    def mask(self) -> int:
        return (1 << self.average_bits) - 1


_TABLES: dict[tuple, list[int]] = {}
TABLE_DRAW = "int63"  # assumption A1 (buzhash64.generate_hashes); "uint64" only for go_probe


def table(seed: int) -> list[int]:
    key = (TABLE_DRAW, seed)
    if key not in _TABLES:
        _TABLES[key] = buzhash64.generate_hashes(seed, TABLE_DRAW)
    return _TABLES[key]


class table_draw:
    """``with table_draw("uint64"): ...`` runs the oracle under the other A1 variant."""

    def __init__(self, draw: str):
        if draw not in ("int63", "uint64"):
            raise ValueError(draw)
        self.draw = draw

    def __enter__(self):
        global TABLE_DRAW
        self.old, TABLE_DRAW = TABLE_DRAW, self.draw
        return self

    def __exit__(self, *exc):
        global TABLE_DRAW
        TABLE_DRAW = self.old
        return False


@dataclass
class Ref:
    size_bytes: int
    edge: bool
    id: bytes = b""
    dek: bytes = b""
    chunk_index: int = 0


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
    size: int = 0


@dataclass
class Chunk:
    index: int
    data: bytes
    edge: bool
    annotations: list = field(default_factory=list)


# --------------------------------------------------------------------------------------
# Literal restatement of chunk.Writer
# --------------------------------------------------------------------------------------

def _merge_data_ref(dr1: Optional[DataRef], dr2: DataRef) -> DataRef:   # writer.go:354-363
    if dr1 is None:
        return dr2
    dr1.size_bytes += dr2.size_bytes
    if dr1.size_bytes == dr1.ref.size_bytes:
        dr1.hash = dr1.ref.id
    return dr1


def get_chunk(store: dict, ref: Ref) -> bytes:
    """chunk.Get (transform.go:50-78) with CreateOptions{}: verify Hash(ctext) == Ref.Id
    (verifyData), ChaCha20-decrypt with Ref.Dek."""
    ctext = store[ref.id]
    if blake2b256(ctext) != ref.id:
        raise ValueError("bad chunk")
    return chacha20_xor(ref.dek, ctext)


def read_data_ref(store: dict, dr: DataRef) -> bytes:
    """DataReader.Get (reader.go): the referenced slice of the chunk."""
    return get_chunk(store, dr.ref)[dr.offset_bytes:dr.offset_bytes + dr.size_bytes]


def merge_file_hash(store: dict, data_refs: list, params: Params = Params()) -> bytes:
    """MergeFileReader.Hash (fileset/merge.go:125-143): Copy the file's DataRefs into a fresh
    writer under one annotation and hash the DataRefs it resolves to (hashDataRefs).  The Go
    writer there uses the default chunking; ``params`` is a test hook."""
    resolved = []

    def cb(annotations):
        if annotations[0].next_data_ref is not None:
            resolved.append(annotations[0].next_data_ref)
    w = Writer(cb=cb, params=params, store=store, no_upload=True)
    w.annotate(Annotation())
    for dr in data_refs:
        w.copy(dr)
    w.close()
    return file_hash([d.hash for d in resolved])


class Writer:
    """``chunk.Writer`` (writer.go:52-438), upload replaced by an in-memory chunk list."""

    def __init__(self, cb: Optional[Callable[[list], None]] = None, params: Params = Params(),
                 with_ref_id: bool = False, store: Optional[dict] = None, no_upload: bool = False):
        self.p = params
        self.cb = cb
        self.with_ref_id = with_ref_id or store is not None
        self.store = store            # the chunk client: Ref.Id -> ciphertext (Copy reads it)
        self.no_upload = no_upload    # WithNoUpload: Id = Hash(ctext), nothing stored
        self.buffering = False
        self.hash = buzhash64.Buzhash64(table(params.seed))
        self.annotations: list[Annotation] = []
        self.num_chunk_bytes_annotation = 0
        self.buf = bytearray()
        self.first, self.last = True, False
        self.chunk_count = 0
        self.annotation_count = 0
        self.chunks: list[Chunk] = []
        self._reset_hash()

    def _reset_hash(self) -> None:                           # writer.go:100-103
        self.hash.reset()
        self.hash.write(bytes(WINDOW_SIZE))

    def annotate(self, a: Annotation) -> None:               # writer.go:118-130
        if len(self.buf) >= self.p.avg:
            self._create_chunk()
        self.annotations.append(a)
        self.num_chunk_bytes_annotation = 0
        self.annotation_count += 1
        self._reset_hash()

    def write(self, data: bytes) -> int:                     # writer.go:132-143
        self._flush_buffer()
        self._roll(memoryview(bytes(data)))
        return len(data)

    def _roll(self, data) -> None:                           # writer.go:163-189
        p = self.p
        offset = 0
        h = self.hash
        for i, b in enumerate(data):
            h.roll(b)
            if h.sum64() & p.mask == 0:
                if self.num_chunk_bytes_annotation + (i + 1 - offset) < p.min:
                    continue
                self._write_data(data[offset:i + 1])
                self._create_chunk()
                offset = i + 1
                continue
            if self.num_chunk_bytes_annotation + (i + 1 - offset) >= p.max:
                self._write_data(data[offset:i + 1])
                self._create_chunk()
                offset = i + 1
        self._write_data(data[offset:])

    def _write_data(self, data) -> None:                     # writer.go:191-196
        if not self.annotations:
            raise RuntimeError("write before annotate (Go: index out of range)")
        last = self.annotations[-1]
        last.size += len(data)
        self.num_chunk_bytes_annotation += len(data)
        self.buf += data

    def _create_chunk(self) -> None:                         # writer.go:198-213
        chunk = bytes(self.buf)
        edge = self.first or self.last
        annotations = self._split_annotations()
        self._process_chunk(chunk, edge, annotations)
        self.first = False
        self.num_chunk_bytes_annotation = 0
        self.buf = bytearray()
        self.chunk_count += 1
        self._reset_hash()

    def _split_annotations(self) -> list:                    # writer.go:215-231
        annotations = self.annotations
        last = annotations[-1]
        self.annotations = [Annotation(data=last.data)]
        return annotations

    def _process_chunk(self, chunk: bytes, edge: bool, annotations: list) -> None:
        ref = Ref(size_bytes=len(chunk), edge=edge, chunk_index=self.chunk_count)
        if self.with_ref_id:
            ref.id, ref.dek = create_ref_id(chunk)
            if self.store is not None and not self.no_upload and ref.id not in self.store:
                self.store[ref.id] = chacha20_xor(ref.dek, chunk)
        self.last_ref = ref
        content_hash = blake2b256(chunk)                     # writer.go:240
        offset = 0
        for a in annotations:                                # writer.go:288-299
            if a.size == 0:
                continue
            h = content_hash if a.size == len(chunk) else blake2b256(chunk[offset:offset + a.size])
            a.next_data_ref = DataRef(ref=ref, hash=h, offset_bytes=offset, size_bytes=a.size)
            offset += a.size
        self.chunks.append(Chunk(index=self.chunk_count, data=chunk, edge=edge,
                                 annotations=annotations))
        if self.cb is not None:
            self.cb(annotations)

    def close(self) -> None:                                 # writer.go:423-438
        self._flush_buffer()
        if self.annotations:
            self.last = True
            self._create_chunk()

    # ---- Copy (writer.go:315-420): buffer whole-chunk data refs, else re-roll their bytes

    def copy(self, dr: DataRef) -> None:
        self._maybe_buffer_data_ref(dr)
        self._maybe_cheap_copy()

    def _maybe_buffer_data_ref(self, dr: DataRef) -> None:  # writer.go:325-352
        last_a = self.annotations[-1]
        if last_a.next_data_ref is not None and last_a.next_data_ref.offset_bytes != 0:
            self._flush_buffer()
        if not self.buffering:
            # only at a chunk split point, for a non-edge chunk, from its first byte
            if len(self.buf) != 0 or dr.ref.edge or dr.offset_bytes != 0:
                self._flush_data_ref(dr)
                return
        else:
            prev = self._prev_data_ref()
            if prev.ref.id != dr.ref.id or prev.offset_bytes + prev.size_bytes != dr.offset_bytes:
                self._flush_buffer()
                self._flush_data_ref(dr)
                return
        last_a.next_data_ref = _merge_data_ref(last_a.next_data_ref, dr)
        self.buffering = True

    def _prev_data_ref(self) -> DataRef:                     # writer.go:365-372
        for a in reversed(self.annotations):
            if a.next_data_ref is not None:
                return a.next_data_ref
        raise RuntimeError("no previous data ref")

    def _flush_buffer(self) -> None:                         # writer.go:374-392
        if not self.buffering:
            return
        annotations, self.annotations = self.annotations, []
        for a in annotations:
            self.annotate(Annotation(data=a.data))
            self.annotation_count -= 1
            if a.next_data_ref is not None:
                self._flush_data_ref(a.next_data_ref)
        self.buffering = False

    def _flush_data_ref(self, dr: DataRef) -> None:          # writer.go:394-401 (DataReader.Get)
        self._roll(memoryview(read_data_ref(self.store, dr)))

    def _maybe_cheap_copy(self) -> None:                     # writer.go:403-420
        if not self.buffering:
            return
        last = self.annotations[-1].next_data_ref
        if last.offset_bytes + last.size_bytes == last.ref.size_bytes:
            annotations = self._split_annotations()
            if self.cb is not None:
                self.cb(annotations)
            self.buffering = False


# --------------------------------------------------------------------------------------
# Closed-form candidate scan + cut selection (fast oracle path)
# --------------------------------------------------------------------------------------

def _rotl_np(x: np.ndarray, k: int) -> np.ndarray:
    k %= 64
    if k == 0:
        return x
    return (x << np.uint64(k)) | (x >> np.uint64(64 - k))


def hashes_numpy(data: np.ndarray, seed: int) -> np.ndarray:
    """h_i for every byte of ONE annotation as ``Writer.roll`` sees it right after a reset.

    Pads 63 zero bytes in front (the reset window) and doubles: H_{2w}[i] = H_w[i] ^
    rotl(H_w[i-w], w), so H_64[i] = XOR_{k<64} rotl(T[x_{i-k}], k).
    """
    t = np.asarray(table(seed), dtype=np.uint64)
    x = np.concatenate([np.zeros(WINDOW_SIZE - 1, dtype=np.uint8), np.asarray(data, dtype=np.uint8)])
    h = t[x]
    w = 1
    while w < WINDOW_SIZE:
        nh = h.copy()
        nh[w:] ^= _rotl_np(h[:-w], w)   # H_w[j] is exact for j >= w-1; only i >= 63 is kept
        h = nh
        w *= 2
    return h[WINDOW_SIZE - 1:]


def candidates_numpy(data, params: Params) -> np.ndarray:
    """Offsets i (within the annotation) where (h_i & mask) == 0 and i >= 63."""
    h = hashes_numpy(np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data,
                     params.seed)
    c = np.nonzero((h & np.uint64(params.mask)) == 0)[0]
    return c[c >= WINDOW_SIZE - 1]


def select_cuts(length: int, cands, params: Params) -> list[int]:
    """Cut positions (inclusive last byte of each segment) inside one annotation.

    Same decision as writer.go:163-189 with seglen = i - segstart + 1: the cut is the first
    candidate >= segstart + min - 1, unless segstart + max - 1 comes first.  Requires
    min >= 64 so that every eligible hash is a pure function of the preceding 64 bytes.
    """
    assert params.min >= WINDOW_SIZE
    cands = np.asarray(cands, dtype=np.int64)
    cuts = []
    s = 0
    while True:
        lo = s + params.min - 1
        hi = s + params.max - 1
        if lo >= length:
            break
        j = int(np.searchsorted(cands, lo))
        c = int(cands[j]) if j < len(cands) else None
        cut = c if c is not None and c <= hi else hi
        if cut >= length:
            break
        cuts.append(cut)
        s = cut + 1
    return cuts


def segments_numpy(data, params: Params) -> list[tuple[int, int, bool]]:
    """(offset, size, ends_at_cut) of every segment of one annotation (empty for size 0).

    ``ends_at_cut`` is False only for a trailing segment that runs to the end of the file
    without the cut rule firing on its last byte (its bytes stay in the open chunk)."""
    n = len(data)
    if n == 0:
        return []
    cuts = select_cuts(n, candidates_numpy(data, params), params)
    segs, s = [], 0
    for c in cuts:
        segs.append((s, c + 1 - s, True))
        s = c + 1
    if s < n:
        segs.append((s, n - s, False))
    return segs


def segments_literal(data, params: Params) -> list[tuple[int, int]]:
    """Same as segments_numpy but by running the literal Writer over a single annotation."""
    w = Writer(params=params)
    a = Annotation(data=0)
    w.annotate(a)
    w.write(bytes(data))
    w.close()
    segs, pos = [], 0
    for ch in w.chunks:
        for ann in ch.annotations:
            if ann.next_data_ref is not None:
                segs.append((pos, ann.next_data_ref.size_bytes, True))
                pos += ann.next_data_ref.size_bytes
    # Close() emits the last chunk; it is empty (E1) iff the final segment ended on a cut.
    if segs and w.chunks[-1].data:
        segs[-1] = (segs[-1][0], segs[-1][1], False)
    return segs


def chunk_stream(files: list, params: Params = Params(), segmenter: str = "numpy",
                 with_ref_id: bool = False) -> list[Chunk]:
    """Run a whole annotation stream (one fileset serialization) through the chunker.

    ``files`` is a list of byte strings, one annotation each, in path order (fileset/writer.go:
    52-75 annotates once per file then copies the bytes).  ``segmenter='literal'`` uses the
    byte-by-byte Writer; ``'numpy'`` replays the same Writer with per-file segments from the
    closed form (valid because hash and seglen reset at every Annotate, writer.go:125-128).
    """
    if segmenter == "literal":
        w = Writer(params=params, with_ref_id=with_ref_id)
        for i, f in enumerate(files):
            w.annotate(Annotation(data=i))
            w.write(bytes(f))
        w.close()
        return w.chunks
    w = _SegmentReplayWriter(params=params, with_ref_id=with_ref_id)
    for i, f in enumerate(files):
        w.annotate(Annotation(data=i))
        w.write_segments(bytes(f), segments_numpy(f, params))
    w.close()
    return w.chunks


class _SegmentReplayWriter(Writer):
    """Writer whose roll() is replaced by precomputed per-annotation segments."""

    def write_segments(self, data: bytes, segs: list) -> None:
        for off, size, cut in segs:
            self._write_data(data[off:off + size])
            if cut:
                self._create_chunk()


def candidates_at(data: bytes, i: int, params: Params) -> bool:
    """Whether byte i of an annotation is a candidate (closed form over its 64-byte window)."""
    t = table(params.seed)
    h = 0
    for k in range(WINDOW_SIZE):
        j = i - k
        x = data[j] if j >= 0 else 0
        h ^= buzhash64.rotl(t[x], k)
    return (h & params.mask) == 0


def file_segments_from_chunks(chunks: list[Chunk], nfiles: int) -> list[list]:
    """Per file: list of (offset_in_file, size, hash) from the Writer's DataRefs."""
    out = [[] for _ in range(nfiles)]
    pos = [0] * nfiles
    for ch in chunks:
        for a in ch.annotations:
            if a.next_data_ref is not None:
                f = a.data
                d = a.next_data_ref
                out[f].append((pos[f], d.size_bytes, d.hash))
                pos[f] += d.size_bytes
    return out


def file_hash(segment_hashes: list) -> bytes:
    """FileInfo.Hash = BLAKE2b(concat DataRef.Hash) (fileset/util.go:149-158)."""
    h = hashlib.blake2b(digest_size=32)
    for d in segment_hashes:
        h.update(d)
    return h.digest()


# --------------------------------------------------------------------------------------
# Ref.Id (Create with CreateOptions{}): ChaCha20 (RFC 8439) in numpy
# --------------------------------------------------------------------------------------

def _chacha20_keystream(key: bytes, nbytes: int, counter0: int = 0) -> bytes:
    nblocks = (nbytes + 63) // 64
    if nblocks == 0:
        return b""
    k = np.frombuffer(key, dtype="<u4").astype(np.uint32)
    const = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)
    st = np.zeros((16, nblocks), dtype=np.uint32)
    st[0:4] = const[:, None]
    st[4:12] = k[:, None]
    st[12] = (np.arange(nblocks, dtype=np.uint64) + counter0).astype(np.uint32)
    # nonce words 13..15 are zero (transform.go:164,182: [12]byte{} nonce)
    x = st.copy()

    def rotl32(v, c):
        return (v << np.uint32(c)) | (v >> np.uint32(32 - c))

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl32(x[d], 16)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl32(x[b], 12)
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl32(x[d], 8)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl32(x[b], 7)

    for _ in range(10):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    x += st
    return x.T.astype("<u4").tobytes()[:nbytes]


def chacha20_xor(key: bytes, data: bytes) -> bytes:
    ks = np.frombuffer(_chacha20_keystream(key, len(data)), dtype=np.uint8)
    return (np.frombuffer(data, dtype=np.uint8) ^ ks).tobytes()


def create_ref_id(chunk: bytes, secret: bytes = b"") -> tuple[bytes, bytes]:
    """(Ref.Id, Ref.Dek) of ``chunk.Create(ctx, CreateOptions{}, chunk, ...)`` with no upload
    de-dup side effects: dek = Hash(secret || Hash(ptext))[:32]; Id = Hash(ChaCha20_dek(ptext))."""
    dek = blake2b256(secret + blake2b256(chunk))[:32]
    ctext = chacha20_xor(dek, chunk)
    return blake2b256(ctext), dek
