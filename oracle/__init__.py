"""CPU oracle for the PFS chunk-ingest path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import, call, link or execute anything under ``oracle/``, and only as the checker (or the
CPU baseline column), never as the thing measured or shipped.  The product path
(``pfs_amd``) does not import this package and fails loudly without its HIP library.

Contents: ``gorand`` (Go 1.16 math/rand restated), ``buzhash64`` (rollinghash v4.0.0
restated), ``chunker`` (chunk.Writer restated: literal + numpy closed form), ``coracle``
(ctypes wrapper of ``cdc_oracle.c``: literal C restatement, multi-threaded, BLAKE2b).

Parity status (details in DESIGN.md §Parity): the reference has no Go toolchain here and its
tests pin no bits.  The oracle is pinned component-wise by known answers —
Go's seed-1 Int63 stream and rngCooked[0..1], BLAKE2b RFC 7693 vectors (hashlib), ChaCha20
RFC 8439 vectors — and by the reference's own property tests restated in tests/.  The
composed boundary lists are not pinned by a Go run ("parity unpinned" end to end).
"""
