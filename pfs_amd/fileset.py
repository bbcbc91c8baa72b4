"""Host-side mirror of the reference's pachd write path above chunk.Writer, over the C ABI.

Reference interface (paths under /root/reference/src/internal/storage/fileset):

* ``Storage.NewUnorderedWriter(ctx, ...)``                         storage.go:84-92
* ``UnorderedWriter.Put(p, tag, appendFile, r) / Delete(p, tag) / Close()``
                                                                   unordered_writer.go:45-179
* ``fileset.Writer`` (Add / Delete / callback / Close) and the multilevel ``index.Writer``
  run inside the library per serialized fileset (writer.go:36-182, index/writer.go:27-162)
* ``Clean(p, isDir)``                                              util.go:67-77

Same names, argument meaning and error behaviour (errors are sticky; an out-of-order or
duplicate path inside a fileset is an error).  ``close()`` returns one ``Primitive`` per
serialized fileset (SizeBytes and the encoded root ``index.Index`` of the additive and
deletive indexes); the fileset ids and the composite of the Postgres metadata store, and the
chunk upload, are out of scope.  ``events`` records, per fileset, every formed chunk (data and
index streams, with its Ref.Id) and every level-0 index entry (pbutil frame).
"""
from __future__ import annotations

import ctypes as C
import weakref
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .cdc import ChunkParams, Chunker

DEFAULT_FILE_TAG = "default"
DEFAULT_MEMORY_THRESHOLD = 10 ** 9


@dataclass
class Primitive:
    additive: Optional[bytes]
    deletive: Optional[bytes]
    size_bytes: int
    num_files: int
    num_deletes: int


def clean(p: str, is_dir: bool) -> str:
    out = C.create_string_buffer(len(p.encode()) + 4)
    rc = _lib.load().pfscdc_path_clean(p.encode(), int(is_dir), out, len(out))
    if rc:
        raise _lib.PfsCdcError(rc, "path_clean")
    return out.value.decode()


class Storage:
    """``fileset.Storage`` restricted to the write path, bound to one GPU, or with
    ``devices`` to a device group (one process, several GPUs: pfscdc_uw_create_group deals
    the serialized filesets over them; the filesets and events equal one GPU's)."""

    def __init__(self, device: int = 0, params: ChunkParams = ChunkParams(),
                 mem_threshold: int = DEFAULT_MEMORY_THRESHOLD,
                 index_params: Optional[ChunkParams] = None,
                 devices: Optional[Sequence[int]] = None):
        self.device, self.params = device, params
        self.devices = list(devices) if devices is not None else None
        self.mem_threshold, self.index_params = mem_threshold, index_params
        self._idle: list = []  # data-stream contexts (or groups) of closed writers, for the next

    def new_unordered_writer(self) -> "UnorderedWriter":
        return UnorderedWriter(self)

    def _take_chunker(self):
        # a context (stream, events, device staging) per GPU, reused writer after writer, as
        # a pachd process would hold it; a writer still open gets a context of its own
        if self._idle:
            return self._idle.pop()
        if self.devices is not None:
            from .group import DeviceGroup
            return DeviceGroup(self.devices, self.params, ref_ids=True)
        return Chunker(self.params, self.device, ref_ids=True)

    def _give_chunker(self, c) -> None:
        if getattr(c, "ctx", None) or getattr(c, "g", None):  # (not closed by a finalizer)
            self._idle.append(c)

    def trim(self) -> dict:
        """Free what closed writers left for the next one: this Storage's idle data contexts
        (stream, events, grow-only device staging) and, process-wide for this device, the
        pooled page-locked fileset arenas with their device mirrors and the cached index
        contexts (pfscdc_uw_trim_cache).  Call it with no writer open on this device."""
        lib = _lib.load()
        n_idle = len(self._idle)
        while self._idle:
            self._idle.pop().close()
        freed, ctxs = C.c_uint64(0), C.c_uint32(0)
        rc = lib.pfscdc_uw_trim_cache(self.device, C.byref(freed), C.byref(ctxs))
        if rc != 0:
            raise _lib.PfsCdcError(rc, "pfscdc_uw_trim_cache")
        return {"data_contexts": n_idle, "arena_bytes": int(freed.value),
                "cached_contexts": int(ctxs.value)}


class UnorderedWriter:
    def __init__(self, storage: Storage):
        self.lib = _lib.load()
        self._storage = storage
        self._chunker = storage._take_chunker()
        self.events: list = []  # per serialized fileset, its events in arrival order
        self.log: list = []  # every event as (fileset, ...) in arrival order
        self._exc: Optional[BaseException] = None
        # the callback reaches the writer through a weak reference: a bound method here would
        # make a reference cycle, which the cyclic GC frees in arbitrary order, closing the
        # data context before this writer could hand it back to the Storage
        ref = weakref.ref(self)

        def on_event(user, ev_p, _ref=ref):
            o = _ref()
            return o._on_event(user, ev_p) if o is not None else 1

        self._cfun = _lib.UW_CB(on_event)
        ip = storage.index_params.to_c() if storage.index_params else None
        w = C.c_void_p()
        if storage.devices is not None:
            rc = self.lib.pfscdc_uw_create_group(self._chunker.g, storage.mem_threshold,
                                                 C.byref(ip) if ip is not None else None,
                                                 self._cfun, None, C.byref(w))
        else:
            rc = self.lib.pfscdc_uw_create(self._chunker.ctx, storage.mem_threshold,
                                           C.byref(ip) if ip is not None else None, self._cfun,
                                           None, C.byref(w))
        if rc:
            raise _lib.PfsCdcError(rc, "pfscdc_uw_create")
        self._w = w

    def _on_event(self, _user, ev_p) -> int:
        try:
            ev = ev_p.contents
            while len(self.events) <= ev.fileset:
                self.events.append([])
            if ev.kind == _lib.EV_CHUNK:
                ch = ev.chunk
                e = ("chunk", ev.index, ev.level if ev.index >= 0 else 0, ch.size_bytes,
                     bool(ch.edge), bytes(ch.ref.id))
            else:
                e = ("index", ev.index, C.string_at(ev.bytes, ev.len))
            self.events[ev.fileset].append(e)
            self.log.append((ev.fileset,) + e)
            return 0
        except BaseException as e:
            self._exc = e
            return 1

    def _check(self, rc: int, what: str) -> None:
        if self._exc is not None:
            exc, self._exc = self._exc, None
            raise exc
        if rc:
            msg = self.lib.pfscdc_uw_last_error(self._w) if getattr(self, "_w", None) else None
            raise _lib.PfsCdcError(rc, f"{what}: {msg.decode() if msg else ''}")

    def put(self, p: str, tag: str, append_file: bool, data) -> None:
        arr = np.frombuffer(data, dtype=np.uint8)  # no copy: the library copies once
        self._check(self.lib.pfscdc_uw_put(self._w, p.encode(), tag.encode(), int(append_file),
                                           arr.ctypes.data if arr.size else None, arr.size),
                    "Put")

    def delete(self, p: str, tag: str = "") -> None:
        self._check(self.lib.pfscdc_uw_delete(self._w, p.encode(), tag.encode()), "Delete")

    def timings(self) -> dict:
        """Stage times (ms) of this writer (pfscdc_uw_timings)."""
        out = (C.c_double * 9)()
        self._check(self.lib.pfscdc_uw_timings(self._w, out), "timings")
        return dict(zip(["put_copy", "upload", "scan", "replay", "hashes", "create",
                         "callbacks", "index", "group_wall"], [round(x, 3) for x in out]))

    def close(self) -> list:
        self._check(self.lib.pfscdc_uw_close(self._w), "Close")
        out = []
        for i in range(self.lib.pfscdc_uw_num_filesets(self._w)):
            info = _lib.FilesetInfo()
            self._check(self.lib.pfscdc_uw_fileset(self._w, i, C.byref(info)), "fileset")
            a = C.string_at(info.additive_root, info.additive_root_len) if info.additive_root else None
            d = C.string_at(info.deletive_root, info.deletive_root_len) if info.deletive_root else None
            out.append(Primitive(a, d, info.size_bytes, info.num_files, info.num_deletes))
        return out

    def release(self) -> None:
        """Destroy the writer and hand its data context back to the Storage."""
        if getattr(self, "_w", None):
            self.lib.pfscdc_uw_destroy(self._w)
            self._w = None
        if getattr(self, "_chunker", None):
            self._storage._give_chunker(self._chunker)
            self._chunker = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass
