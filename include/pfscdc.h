/*
 * pfscdc.h — C ABI of the MI355X PFS chunk-ingest path (libpfscdc.so).
 *
 * Drop-in boundary for the reference's chunk layer.  The reference has no FFI on this path
 * (pure Go, no cgo); its seam is the Go type chunk.Writer.  Each entry point below names
 * the reference interface it replaces (paths under /root/reference).  Plain pointers and
 * sizes only; no torch or HIP types cross this boundary except the opaque stream handle.
 *
 * Status codes: 0 = ok, negative = error (PFSCDC_E*).  Errors are sticky on a writer, like
 * chunk.Writer.err (src/internal/storage/chunk/writer.go:145-161).
 * Threading: a ctx (and its writers) is owned by one thread at a time; one ctx per GPU;
 * distinct ctxs may run concurrently (independent chunk.Writers, chunk/storage.go:60-66).
 */
#ifndef PFSCDC_H
#define PFSCDC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PFSCDC_OK 0
#define PFSCDC_EINVAL -1      /* bad argument */
#define PFSCDC_EHIP -2        /* HIP runtime error (see pfscdc_last_error) */
#define PFSCDC_ENOMEM -3      /* device or host allocation failed */
#define PFSCDC_EUNSUPPORTED -4 /* configuration the GPU path does not implement */
#define PFSCDC_ESTATE -5      /* call order violated (e.g. Write before Annotate) */
#define PFSCDC_ECALLBACK -6   /* the writer callback returned non-zero */
#define PFSCDC_ECORRUPT -7    /* a stored chunk failed verification (chunk.Get verifyData) */
#define PFSCDC_ENOTFOUND -8   /* a chunk id is not in the store */

/* chunk.WithRollingHashConfig(averageBits, seed) + chunk.WithMinMax(min, max)
 * (chunk/option.go:50-64); defaults writer.go:39-44: 23, 1, 1 MB, 20 MB (decimal). */
typedef struct pfscdc_params {
  uint32_t average_bits; /* split mask = 2^bits - 1, avg = 2^bits (1..32) */
  uint32_t reserved;
  int64_t seed;          /* buzhash64.GenerateHashes seed */
  int64_t min_chunk;     /* must be >= 64 (the window) on the GPU path */
  int64_t max_chunk;
} pfscdc_params;

/* One segment = the bytes of one file (annotation) inside one chunk = one DataRef
 * (writer.go:288-312: DataRef.Hash = BLAKE2b-256 of exactly these bytes). */
typedef struct pfscdc_segment {
  uint64_t offset;  /* offset of the segment inside its file */
  uint64_t size;    /* bytes */
  uint32_t file;    /* index of the file in the batch */
  uint32_t flags;   /* PFSCDC_SEG_* */
  uint8_t hash[32]; /* BLAKE2b-256 (pachhash.Sum, pachhash/hash.go:27-30) */
} pfscdc_segment;   /* 56 bytes */

/* Ref of the chunk a segment forms when each file is its own writer (the batch form): what
 * chunk.Create(ctx, CreateOptions{}, chunk, ...) stores (transform.go:26-46, client.go:57).
 * CreateOptions{} means no compression and an empty secret, so
 *   dek = BLAKE2b-256(BLAKE2b-256(chunk))      (deriveKey, transform.go:173-178)
 *   id  = BLAKE2b-256(ChaCha20_dek,nonce0(chunk)) (cryptoXOR :181-188, then Hash) */
typedef struct pfscdc_ref {
  uint8_t id[32];  /* Ref.Id */
  uint8_t dek[32]; /* Ref.Dek */
} pfscdc_ref;

#define PFSCDC_SEG_VALID 1u
#define PFSCDC_SEG_CUT 2u /* the segment ends on a CDC cut (else: at end of file) */

typedef struct pfscdc_ctx pfscdc_ctx;

/* Fills params with the reference defaults (writer.go:39-44). */
void pfscdc_default_params(pfscdc_params* p);

/* buzhash64.GenerateHashes(seed) (called at chunk/option.go:54). */
int pfscdc_table(int64_t seed, uint64_t out[256]);

/* First n values of Go's rand.NewSource(seed).Int63() (known-answer hook for tests). */
int pfscdc_go_int63(int64_t seed, int64_t* out, int n);

/* Replaces chunk.Storage.NewWriter's per-writer config (chunk/storage.go:60-66,
 * writer.go:74-98): binds params and a GPU.  device = HIP ordinal. */
int pfscdc_ctx_create(const pfscdc_params* params, int device, pfscdc_ctx** out);
int pfscdc_ctx_destroy(pfscdc_ctx* ctx);
const char* pfscdc_last_error(const pfscdc_ctx* ctx);

/* Run every following GPU call of ctx on this hipStream_t (NULL = the ctx's own stream). */
int pfscdc_set_stream(pfscdc_ctx* ctx, void* hip_stream);

/* Ordering rule for device-resident inputs: the ctx's stream is a non-blocking stream of its
 * own, so a device buffer written by work on another stream (a kernel, a non-blocking copy)
 * must be ordered before a call that reads it.  pfscdc_stream_wait makes every following GPU
 * call of ctx wait for the work already enqueued on hip_stream (NULL = the legacy default
 * stream); it does not block the host.  The Python binding calls it with torch's current
 * stream before each call on a torch tensor. */
int pfscdc_stream_wait(pfscdc_ctx* ctx, void* hip_stream);
/* The hipStream_t the ctx enqueues on (its own, or the one given to pfscdc_set_stream), e.g.
 * for pfscdc_stream_wait(other_ctx, pfscdc_stream_handle(ctx)): every later call of other_ctx
 * runs after the work ctx has enqueued so far. */
void* pfscdc_stream_handle(const pfscdc_ctx* ctx);

/* Steps in flight on two ctxs of one GPU: every later scan of ctx starts its BLAKE2b kernel
 * only after the BLAKE2b kernel last enqueued by other (NULL: no ordering).  The next step's
 * candidate scan still fills the CUs the current hash frees as its queue drains, but two
 * hashes never share the SIMDs, so each hash launch runs for its own duration.  other must
 * outlive the ordering (set NULL before destroying it). */
int pfscdc_order_hash_after(pfscdc_ctx* ctx, pfscdc_ctx* other);

/* CDC + content hash of a batch of files (one annotation each, concatenated).
 * Replaces, for every file of the batch, Writer.Annotate + Writer.Write + the hash part of
 * processChunk (writer.go:118-143,163-196,233-253,288-312): per-file cut positions and
 * per-segment BLAKE2b-256.  bytes: nbytes bytes, device pointer (16-B aligned) if
 * bytes_on_device else host memory (copied with hipMemcpyAsync).  file_offsets: host array
 * of nfiles+1 nondecreasing offsets, file_offsets[0] == 0, file_offsets[nfiles] == nbytes.
 * Blocks until the segment records are on the host; read them with pfscdc_segments. */
int pfscdc_scan(pfscdc_ctx* ctx, const void* bytes, uint64_t nbytes, int bytes_on_device,
                const uint64_t* file_offsets, uint32_t nfiles);

/* Asynchronous form: enqueue on the ctx stream; pfscdc_wait() completes it. */
int pfscdc_scan_async(pfscdc_ctx* ctx, const void* bytes, uint64_t nbytes,
                      int bytes_on_device, const uint64_t* file_offsets, uint32_t nfiles);
int pfscdc_wait(pfscdc_ctx* ctx);

/* Results of the last completed scan, ordered by (file, offset).  Valid until the next
 * scan on ctx.  seg_begin[f]..seg_begin[f+1] index file f's segments (nfiles+1 entries). */
uint64_t pfscdc_num_segments(const pfscdc_ctx* ctx);
const pfscdc_segment* pfscdc_segments(const pfscdc_ctx* ctx);
const uint64_t* pfscdc_file_segment_begin(const pfscdc_ctx* ctx);

/* Options of every following scan on ctx (bit set).  PFSCDC_OPT_REF_IDS: also compute each
 * segment's pfscdc_ref (a second BLAKE2b pass over the ChaCha20 ciphertext, fused). */
#define PFSCDC_OPT_REF_IDS 1u
/* PFSCDC_OPT_CUTS_ONLY: the scan finds the segments (cut positions) but leaves their DataRef
 * hashes to a following pfscdc_commit_refs, which computes them in one launch together with
 * the formed chunks' content hashes. */
#define PFSCDC_OPT_CUTS_ONLY 2u
/* PFSCDC_OPT_CTEXT_IN_PLACE: pfscdc_commit_refs writes every chunk's ciphertext (the object
 * chunk.Create uploads, ChaCha20_dek(chunk)) over the chunk's plaintext in the caller's device
 * buffer, which then holds the upload stream.  The commit needs no second buffer of its size
 * (a 200 GiB commit on one 288 GB GPU), and the Ref.Id pass can always take the split form.
 * Needs the scan over caller-owned device bytes. */
#define PFSCDC_OPT_CTEXT_IN_PLACE 4u
int pfscdc_set_options(pfscdc_ctx* ctx, uint32_t options);
/* Refs of the last completed scan, aligned with pfscdc_segments (NULL unless the scan ran
 * with PFSCDC_OPT_REF_IDS). */
const pfscdc_ref* pfscdc_refs(const pfscdc_ctx* ctx);
/* Device time (ms) of the last scan's Ref.Id kernels (0 without PFSCDC_OPT_REF_IDS). */
int pfscdc_last_ref_ms(pfscdc_ctx* ctx, float* ms);

/* chunk.Get (transform.go:50-78) for a batch of stored chunks, the GetFile read path: for
 * chunk i (bytes [chunk_offsets[i], chunk_offsets[i+1]) of ctext) compute BLAKE2b-256 of the
 * stored bytes, set ok[i] = 1 iff it equals refs[i].id (verifyData), and write the ChaCha20
 * decryption with refs[i].dek to the same range of ptext (CreateOptions{} never compresses).
 * ctext/ptext: device pointers if *_on_device (16-B aligned ctext), else host memory.
 * Returns PFSCDC_OK even when some chunk fails verification (see ok[]). */
int pfscdc_get_chunks(pfscdc_ctx* ctx, const void* ctext, uint64_t nbytes, int ctext_on_device,
                      const uint64_t* chunk_offsets, uint32_t nchunks, const pfscdc_ref* refs,
                      void* ptext, int ptext_on_device, uint8_t* ok);
/* Device time (ms) of the last pfscdc_get_chunks kernels (after the input copy). */
int pfscdc_last_get_ms(pfscdc_ctx* ctx, float* ms);

/* chunk.Create(ctx, CreateOptions{}, chunk, createFunc) (transform.go:26-46) for a batch of
 * formed chunks, the upload half of processChunk (writer.go:233-271): chunk i is bytes
 * [chunk_offsets[i], chunk_offsets[i+1]) (offsets as for pfscdc_get_chunks).  refs[i] gets
 * Ref.Dek = Hash(Hash(chunk)) and Ref.Id = Hash(ChaCha20_dek(chunk)).  content_hashes
 * (NULL or 32 B per chunk) is Hash(chunk) (chunkDataRef.Hash, writer.go:240): taken as
 * given where hash_known[i] != 0 (e.g. a single-DataRef chunk, whose hash the scan already
 * has), computed and written back otherwise.  Blocks until refs are on the host.
 * The Ref.Id pass runs fused (keystream on the BLAKE2b chain) or split (a parallel ChaCha20
 * pass into a ctx-owned ciphertext copy, then BLAKE2b of it) when nchunks cannot fill the
 * GPU and 8 GiB of device memory stay free; the environment variable PFSCDC_REFID_SPLIT=0/1
 * forces either.  Same results either way. */
int pfscdc_create_refs(pfscdc_ctx* ctx, const void* bytes, uint64_t nbytes, int bytes_on_device,
                       const uint64_t* chunk_offsets, uint32_t nchunks, uint8_t* content_hashes,
                       const uint8_t* hash_known, pfscdc_ref* refs);
/* The commit data plane's hashing in one pass, after a scan made with PFSCDC_OPT_CUTS_ONLY
 * over the same bytes and pfscdc_form_chunks: every segment's DataRef hash (writer.go:301-312,
 * into segment_hashes, 32 B each in pfscdc_segments order) and every chunk's content hash
 * (content_hashes out; a chunk with hash_known[i] != 0 is one segment, and its hash is that
 * segment's) run as one BLAKE2b launch in longest-first order, so the two independent sets of
 * serial chains share the GPU instead of running one pass after the other; then
 * chunk.Create's dek and Ref.Id as pfscdc_create_refs.  refs as pfscdc_create_refs, or NULL:
 * then only the hashes (every BLAKE2b Writer.processChunk computes, writer.go:240,301-312)
 * and no chunk.Create.  With refs and more chunks than the quads of one wave per SIMD, the
 * long chunks (and their Ref.Ids) run on the ctx stream beside the rest on a second one, so
 * their Ref.Id chains start as soon as their own content hashes are done (same results;
 * PFSCDC_COMMIT_TWO_SETS=0/1 forces either form).
 * Synchronous; the scan's segment list is consumed (pfscdc_segments is empty afterwards). */
int pfscdc_commit_refs(pfscdc_ctx* ctx, const void* bytes, uint64_t nbytes, int bytes_on_device,
                       const uint64_t* chunk_offsets, uint32_t nchunks, uint8_t* content_hashes,
                       const uint8_t* hash_known, pfscdc_ref* refs, uint8_t* segment_hashes);
/* hashDataRefs (fileset/util.go:149-158): FileInfo.Hash = BLAKE2b-256 over the n concatenated
 * 32-byte DataRef hashes (host array), computed by the hash kernel. */
int pfscdc_hash_data_refs(pfscdc_ctx* ctx, const uint8_t* hashes, uint32_t n, uint8_t out[32]);
/* Device time (ms) of the last chunk.Create batch (pfscdc_create_refs or a writer flush). */
int pfscdc_last_create_ms(pfscdc_ctx* ctx, float* ms);
/* Its split: out[0] content-hash pass, out[1] Ref.Id pass (dek, ChaCha20, BLAKE2b). */
int pfscdc_last_create_timings(pfscdc_ctx* ctx, float out[2]);

/* ---- one stream split across GPUs (writer.go:163-189 block-parallel) --------
 * A stream of N bytes is cut into equal byte ranges, one per GPU.  The rolling hash at a
 * position is a pure function of the 64 bytes ending there, so each GPU finds the candidate
 * positions of its range from its bytes plus the 64 bytes in front (the halo); the serial
 * min/max selection then runs once over the gathered, sorted candidates (cheap: ~1 per 8 MiB),
 * and each segment is hashed by the GPU whose range holds its first byte, after the bytes of a
 * segment that straddles the border are copied over from the next range. */

/* Candidates of one range: every position p of bytes (halo <= p < nbytes, p >= 63) where the
 * buzhash64 of bytes [p-63, p] has (h & mask) == 0, sorted ascending, as offsets into bytes.
 * halo (<= 64) = the bytes in front of the range copied from the previous one (0 at the
 * stream start, where positions < 63 are never candidates: min >= 64 puts them before the
 * first eligible cut).  out: cap entries; *n = the count (PFSCDC_ENOMEM if > cap, out holds
 * the first cap).  Tiles with more than 15 candidates are re-rolled exactly on the host.
 * Timings: pfscdc_last_timings out[0] (scan, compaction included). */
int pfscdc_candidates(pfscdc_ctx* ctx, const void* bytes, uint64_t nbytes, int bytes_on_device,
                      uint64_t halo, uint64_t* out, uint64_t cap, uint64_t* n);

/* BLAKE2b-256 of n byte ranges [begins[i], begins[i] + sizes[i]) of bytes (device pointer,
 * 16-B aligned, if bytes_on_device), into out (32 B each): the DataRef hashes of segments
 * whose cuts were selected elsewhere (writer.go:240,301-312).  Synchronous. */
int pfscdc_hash_ranges(pfscdc_ctx* ctx, const void* bytes, uint64_t nbytes, int bytes_on_device,
                       const uint64_t* begins, const uint64_t* sizes, uint32_t n, uint8_t* out);

/* Candidate positions (h & mask == 0, absolute offset >= 63) found by the last scan, sorted;
 * positions inside dense tiles are reported through the tile marker instead.  Positions the
 * scan skipped (see pfscdc_last_scan_bytes) are never listed.  Debug/test hook for the
 * candidate-scan kernel. */
uint64_t pfscdc_debug_candidates(pfscdc_ctx* ctx, uint64_t* out, uint64_t cap);

/* Bytes the last pfscdc_scan's candidate kernel actually rolled.  Writer.roll never cuts in
 * the first min - 1 bytes after an Annotate (writer.go:125-128,167-170), so the scan skips
 * that part of every file (in 8 KiB steps of its work units) and the count is below nbytes
 * when files are longer than min; results are unchanged.  With min - 1 >= 256 KiB it also
 * skips the min - 1 positions after every cut of a file that the scan has already settled
 * (its work units go out in rank order and report per file), so the count then also depends
 * on timing.  The knob PFSCDC_SCAN_CUTSKIP=0 keeps only the first skip; PFSCDC_SCAN_SKIP=0
 * rolls every byte (pfscdc_last_scan_mode tells which skipping the last scan did). */
int pfscdc_last_scan_bytes(pfscdc_ctx* ctx, uint64_t* out);

/* Device timing of the last scan's kernels (ms, HIP events on the ctx stream):
 * out[0] candidate scan (its last workgroup also compacts the candidates), out[1] 0 (the
 * compaction used to be a launch of its own), out[2] selection (its last workgroup also
 * compacts the segment list and builds the hash queue's LPT order), out[3] BLAKE2b,
 * out[4] total.  An interval between two events includes any time the kernel waited for
 * free CUs behind work of another stream. */
int pfscdc_last_timings(pfscdc_ctx* ctx, float out[5]);
/* Execution spans of the last scan's two main kernels (ms): out[0] the candidate scan, out[1]
 * the BLAKE2b kernel, each from its first wavefront's start to its last wavefront's end
 * (s_memrealtime in the kernels), so a kernel queued behind another stream's work is not
 * charged for the wait — the per-launch duration a kernel-trace profiler reports. */
int pfscdc_last_kernel_spans(pfscdc_ctx* ctx, float out[2]);
/* Shader clock (MHz) the last scan's two main kernels ran at: out[0] the candidate scan,
 * out[1] the BLAKE2b kernel; each the sum over its waves of their lifetimes in shader cycles
 * (s_memtime) divided by the same in wall-clock ticks (s_memrealtime).  The chip lowers its
 * clock under load, so an instruction-issue ceiling is priced at this clock. */
int pfscdc_last_kernel_clocks(pfscdc_ctx* ctx, float out[2]);

/* Pinned host memory for staging (PCIe-inclusive end-to-end path). */
void* pfscdc_host_alloc(uint64_t nbytes);
void pfscdc_host_free(void* p);

/* Synthetic data generator used by bench/tests (device-side): word k of file f is
 * splitmix64-finalize((f << 40 | k) + (seed + 1) * 0x9E3779B97F4A7C15), little endian.
 * Writes every file of file_offsets into dev_bytes on the ctx stream. */
int pfscdc_fill_synthetic(pfscdc_ctx* ctx, void* dev_bytes, const uint64_t* file_offsets,
                          uint32_t nfiles, uint64_t seed);

/* Dedup-heavy variants (BASELINE configs[4]).  With m(x) the murmur3 64-bit finalizer:
 *  PFSCDC_SYNTH_DEDUP_BLOCKS: the 1 MiB block k of file f is, when
 *    h = m((seed << 48) ^ (f << 24) ^ k ^ 0xC5C5C5C5) is odd, a copy of pooled block
 *    (h >> 1) & 63, whose word w is splitmix64-finalize(((2^23 + id) << 40 | w) + gamma);
 *  PFSCDC_SYNTH_DEDUP_FILES: the same decision per whole file with
 *    h = m((seed << 48) ^ (f << 24) ^ 0x5EEDF11E), the pooled file's words indexed from 0. */
#define PFSCDC_SYNTH_RANDOM 0u
#define PFSCDC_SYNTH_DEDUP_BLOCKS 1u
#define PFSCDC_SYNTH_DEDUP_FILES 2u
int pfscdc_fill_synthetic_ex(pfscdc_ctx* ctx, void* dev_bytes, const uint64_t* file_offsets,
                             uint32_t nfiles, uint64_t seed, uint32_t mode);
/* The same bytes for pieces of files: piece i (bytes [piece_offsets[i], piece_offsets[i+1])
 * of dev_bytes) holds bytes [file_starts[i], ...) of file file_ids[i] (NULL ids: file i;
 * NULL starts: from byte 0).  A rank generates just its pieces of a commit whose files are
 * cut across serialized filesets or ranks. */
int pfscdc_fill_synthetic_pieces(pfscdc_ctx* ctx, void* dev_bytes, const uint64_t* piece_offsets,
                                 uint32_t npieces, const uint32_t* file_ids,
                                 const uint64_t* file_starts, uint64_t seed, uint32_t mode);

/* ---- chunk.Writer mirror (writer.go:52-438) ------------------------------------------
 * A writer buffers annotated bytes in host memory, runs them through pfscdc_scan in
 * batches of whole files, assembles chunks exactly as createChunk/Annotate do (including
 * multi-file chunks, the buf.Len() >= avg cut before a file, edge flags and the empty last
 * chunk of Close) and invokes the callback serially in chunk order, like TaskChain
 * (chunk/chain.go:55-68). */

typedef struct pfscdc_dataref {
  uint8_t hash[32];      /* DataRef.Hash */
  int64_t offset_bytes;  /* DataRef.OffsetBytes (offset inside the chunk) */
  int64_t size_bytes;    /* DataRef.SizeBytes */
} pfscdc_dataref;

typedef struct pfscdc_chunk_ref {
  uint64_t chunk_index;  /* 0-based order of createChunk calls */
  int64_t size_bytes;    /* Ref.SizeBytes (== plaintext size: CreateOptions{} => no gzip) */
  int32_t edge;          /* Ref.Edge = first || last (writer.go:200) */
  int32_t has_ref;       /* ref below is set (the writer was created with PFSCDC_OPT_REF_IDS) */
  pfscdc_ref ref;        /* Ref.Id / Ref.Dek of the whole chunk (maybeUpload, writer.go:255-271) */
  int32_t copied;        /* 1: a cheap copy (maybeCheapCopy, writer.go:403-420): no new chunk;
                            the annotations' DataRefs point into the existing chunk whose
                            Ref this is (has_ref = 1, chunk_index = -1) */
  int32_t reserved2;
} pfscdc_chunk_ref;

typedef struct pfscdc_annotation_out {
  uint64_t user;         /* Annotation.Data: the id passed to pfscdc_writer_annotate */
  int32_t has_data_ref;  /* 0 => NextDataRef == nil (size-0 piece) */
  int32_t reserved;
  pfscdc_dataref data_ref;
} pfscdc_annotation_out;

/* WriterCallback (writer.go:31): annotations of one chunk, in order.  Non-zero aborts. */
typedef int (*pfscdc_writer_cb)(void* user, const pfscdc_chunk_ref* chunk,
                                const pfscdc_annotation_out* annotations, uint32_t n);

typedef struct pfscdc_writer pfscdc_writer;

/* A DataRef with its chunk's Ref (what fileset indexes store, chunk.proto DataRef). */
typedef struct pfscdc_full_dataref {
  pfscdc_ref ref;       /* Ref.Id, Ref.Dek */
  int64_t ref_size;     /* Ref.SizeBytes */
  int32_t edge;         /* Ref.Edge */
  int32_t reserved;
  pfscdc_dataref data;  /* Hash, OffsetBytes, SizeBytes */
} pfscdc_full_dataref;

/* In-memory chunk store (the chunk client's object store, keyed by Ref.Id: client.go
 * Create/Get).  Writers with a store upload the ciphertext of every new chunk (deduplicated
 * by id) and read chunks back for Copy. */
typedef struct pfscdc_store pfscdc_store;
int pfscdc_store_create(pfscdc_store** out);
int pfscdc_store_destroy(pfscdc_store* s);
int pfscdc_store_put(pfscdc_store* s, const uint8_t id[32], const void* ctext, uint64_t n);
int pfscdc_store_get(const pfscdc_store* s, const uint8_t id[32], const void** ctext,
                     uint64_t* n);
uint64_t pfscdc_store_count(const pfscdc_store* s);

/* batch_bytes: flush threshold for buffered file bytes (0 = 1 GiB).  If ctx has
 * PFSCDC_OPT_REF_IDS set when the writer is created, every chunk also gets its Ref
 * (pfscdc_create_refs over the assembled chunk bytes, multi-file chunks and chunks that span
 * flushes included); the writer's own scans never compute per-segment refs. */
int pfscdc_writer_create(pfscdc_ctx* ctx, pfscdc_writer_cb cb, void* user,
                         uint64_t batch_bytes, pfscdc_writer** out);
int pfscdc_writer_annotate(pfscdc_writer* w, uint64_t user);            /* writer.go:118 */
int pfscdc_writer_write(pfscdc_writer* w, const void* data, uint64_t n); /* writer.go:132 */
int pfscdc_writer_close(pfscdc_writer* w);                               /* writer.go:423 */
int64_t pfscdc_writer_chunk_count(const pfscdc_writer* w);               /* writer.go:113 */
int64_t pfscdc_writer_annotation_count(const pfscdc_writer* w);          /* writer.go:107 */
int pfscdc_writer_destroy(pfscdc_writer* w);

/* The writer's chunk client: Copy reads chunks from store (chunk.Get: verify + decrypt on
 * the GPU); with upload != 0 every new chunk's ciphertext is stored (needs Ref ids, i.e.
 * PFSCDC_OPT_REF_IDS on the ctx; WithNoUpload = upload 0). */
int pfscdc_writer_set_store(pfscdc_writer* w, pfscdc_store* store, int upload);
/* Writer.Copy(dataRef) (writer.go:315-420): consecutive whole-chunk DataRefs at a chunk
 * boundary are buffered and passed through by reference (cheap copy, a callback with
 * chunk.copied = 1); anything else is read back and re-rolled like written bytes. */
int pfscdc_writer_copy(pfscdc_writer* w, const pfscdc_full_dataref* dr);
/* Optional hint before a run of Copies: verifies and decrypts, in one batch, every chunk
 * those DataRefs will certainly be re-rolled from (edge chunks, DataRefs not starting at
 * offset 0), so their BLAKE2b chains run in parallel instead of one per Copy. */
int pfscdc_writer_prefetch(pfscdc_writer* w, const pfscdc_full_dataref* drs, uint32_t n);
/* MergeFileReader.Hash (fileset/merge.go:125-143): a fresh writer on ctx (no upload), one
 * annotation, Copy of every DataRef, Close; out = BLAKE2b-256 over the resolved DataRefs'
 * hashes (hashDataRefs, fileset/util.go:149-158). */
int pfscdc_merge_file_hash(pfscdc_ctx* ctx, pfscdc_store* store, const pfscdc_full_dataref* drs,
                           uint32_t n, uint8_t out[32]);

/* Chunk formation over a device-resident batch: the chunks chunk.Writer would create
 * (Annotate cut, CDC cuts, Close's last chunk: writer.go:118-130,198-231,423-438) for the
 * files of the last pfscdc_scan, each stream k = files [stream_file_begin[k],
 * stream_file_begin[k+1]) being one writer (one serialized fileset: a fresh chunk.Writer per
 * fileset.Writer, fileset/writer.go:36-50) that annotates its files in order and closes.
 * stream_file_begin: nstreams+1 entries from 0 to nfiles (NULL = one stream of all files).
 * Out: chunk_offsets (cap+1 entries; chunk i = scanned bytes [off[i], off[i+1]), so the
 * chunks tile the batch), per chunk hash_known/content_hashes as pfscdc_create_refs takes
 * them (known iff the chunk is one DataRef).  *nchunks = number of chunks; PFSCDC_ENOMEM if
 * it exceeds cap (outputs truncated).  Must follow the scan directly (PFSCDC_ESTATE after
 * a pfscdc_create_refs / pfscdc_get_chunks). */
int pfscdc_form_chunks(pfscdc_ctx* ctx, const uint32_t* stream_file_begin, uint32_t nstreams,
                       uint64_t* chunk_offsets, uint8_t* content_hashes, uint8_t* hash_known,
                       uint64_t cap, uint64_t* nchunks);

/* ---- pachd-level stream formation (fileset/unordered_writer.go, fileset/writer.go,
 * fileset/index/writer.go) --------------------------------------------------------------
 * An unordered writer buffers Put bytes (host memory) until memThreshold bytes are buffered,
 * then serializes the buffer as one fileset: files sorted by (path, tag) go through a fresh
 * chunk writer (pfscdc_writer on data_ctx, Ref ids on), per-file DataRefs are collected by
 * the fileset.Writer callback, and the additive and deletive index entries go through the
 * multilevel index writer (level k: its own pfscdc_writer with WithRollingHashConfig(20, k)).
 * Chunk bytes are not returned (the upload is out of scope); every chunk and every level-0
 * index entry is reported through the event callback, and each fileset's root indexes are
 * kept as encoded index.Index protos. */

#define PFSCDC_EV_CHUNK 1 /* a chunk was formed (data or index stream) */
#define PFSCDC_EV_INDEX 2 /* a level-0 index entry was written (additive or deletive) */

typedef struct pfscdc_uw_event {
  int32_t kind;           /* PFSCDC_EV_* */
  int32_t index;          /* -1: the data stream; 0: additive index; 1: deletive index */
  int32_t level;          /* CHUNK of an index stream: index level */
  uint32_t fileset;       /* serialized fileset number (UnorderedWriter.subFileSet) */
  pfscdc_chunk_ref chunk; /* CHUNK: chunk index, size, edge, Ref */
  const uint8_t* bytes;   /* INDEX: the pbutil frame (int64 LE length + index.Index proto) */
  uint64_t len;
} pfscdc_uw_event;

typedef int (*pfscdc_uw_cb)(void* user, const pfscdc_uw_event* ev); /* non-zero aborts */

typedef struct pfscdc_fileset_info {
  int64_t size_bytes;            /* Primitive.SizeBytes */
  const uint8_t* additive_root;  /* encoded index.Index (NULL: no additive entries) */
  uint64_t additive_root_len;
  const uint8_t* deletive_root;  /* encoded index.Index (NULL: no deletive entries) */
  uint64_t deletive_root_len;
  uint32_t num_files;            /* additive entries */
  uint32_t num_deletes;          /* deletive entries */
} pfscdc_fileset_info;

typedef struct pfscdc_uwriter pfscdc_uwriter;

/* fileset.Storage.NewUnorderedWriter (fileset/storage.go:84-92).  data_ctx must have
 * PFSCDC_OPT_REF_IDS set.  mem_threshold: 0 = DefaultMemoryThreshold (1e9 bytes).
 * index_params: NULL = the reference's index chunking (avgBits 20, seed 0 + level,
 * 1 MB / 20 MB); other values are a test hook. */
int pfscdc_uw_create(pfscdc_ctx* data_ctx, int64_t mem_threshold,
                     const pfscdc_params* index_params, pfscdc_uw_cb cb, void* user,
                     pfscdc_uwriter** out);
/* UnorderedWriter.Put(p, tag, appendFile, r) with r = the n bytes at data (tag NULL/"" =
 * "default"). */
int pfscdc_uw_put(pfscdc_uwriter* w, const char* path, const char* tag, int append_file,
                  const void* data, uint64_t n);
/* UnorderedWriter.Delete(p, tag); a path ending in "/" deletes a directory (buffered files
 * and the live files of the filesets this writer serialized; no parent fileset). */
int pfscdc_uw_delete(pfscdc_uwriter* w, const char* path, const char* tag);
int pfscdc_uw_close(pfscdc_uwriter* w); /* serializes the rest (Close, :171-179) */
/* Serialized filesets are written in groups of up to PFSCDC_UW_INFLIGHT bytes (knob, default
 * 32 GiB) on a background thread while Puts continue; the event callback may run on that
 * thread, never on two threads at once.  Order: groups in order (with several group writers,
 * PFSCDC_UW_WORKERS > 1 or a device group, each group's events are held until the groups
 * before it have emitted theirs); within a group, within one (fileset, index, level) stream
 * and within each fileset's data stream, events come in stream order; a group's data-stream
 * events come fileset by fileset, but its index streams are closed level by level across the
 * group's filesets, so index events of different filesets (and additive and deletive ones)
 * interleave.  Filesets are readable after Close. */
uint32_t pfscdc_uw_num_filesets(const pfscdc_uwriter* w);
/* Fileset i's Primitive (pointers valid until pfscdc_uw_destroy). */
int pfscdc_uw_fileset(const pfscdc_uwriter* w, uint32_t i, pfscdc_fileset_info* out);
int pfscdc_uw_destroy(pfscdc_uwriter* w);
/* Message of the writer's sticky error (Put/Delete/Close or the background fileset write,
 * with the data ctx's last error appended); "" while there is none. */
const char* pfscdc_uw_last_error(const pfscdc_uwriter* w);
/* Where the writer's time went (ms, summed over its Puts and its group writes; a group
 * write runs on a background thread while Puts continue (PFSCDC_UW_WORKERS > 1: several
 * groups in flight, each on a ctx of its own), so the stages overlap the Puts: out[0] the
 * Puts' host copies into the fileset arenas; per grouped close of the data streams out[1] the
 * upload (until the Puts' uploads into the arena mirrors have landed, then the gathers
 * queued; without mirrors the H2D copies queued), out[2] the cuts-only scan (without mirrors
 * it waits for the H2D copies), out[3] the chunk replay, out[4] the one BLAKE2b
 * launch over every piece and multi-piece chunk, out[5] chunk.Create (dek, ChaCha20, Ref.Id),
 * out[6] the data chunks' callbacks; out[7] the index writers; out[8] the group writes'
 * wall time. */
int pfscdc_uw_timings(const pfscdc_uwriter* w, double out[9]);

/* Memory the writers keep for the next writer (no reference counterpart: a GPU-side cache).
 * Each fileset's page-locked host arena (memThreshold bytes) and its device mirror (as many
 * bytes of HBM) go to a process-wide pool when the writer is destroyed, up to
 * PFSCDC_UW_ARENA_POOL_BYTES (env, default 40e9 host bytes + as many device bytes); the
 * contexts a writer made for itself (index levels, extra group writers), with their grow-only
 * device staging, go to a cache of up to PFSCDC_CTX_CACHE (default 32) contexts.  Both count
 * against the device memory other calls see (pfscdc_commit_refs takes its ciphertext copy only
 * with 8 GiB to spare).  pfscdc_uw_trim_cache frees the pooled arenas and destroys the cached
 * contexts of one device (-1: all devices); call it when no writer is being created or
 * destroyed.  pfscdc_uw_cached_arena_bytes: host bytes of the pooled arenas now. */
int pfscdc_uw_trim_cache(int device, uint64_t* arena_bytes_freed, uint32_t* ctxs_destroyed);
uint64_t pfscdc_uw_cached_arena_bytes(void);

/* ---- device groups: one process, several GPUs ------------------------------
 * pachd is one process owning one chunk storage (src/server/pfs/server/driver.go:110-122),
 * so the GPUs of a node are reached through one caller.  A group holds one ctx per member
 * device (a device may appear more than once: several ctxs on one GPU) and deals one call's
 * work across them; results never depend on the dealing or on the number of members.
 *   Files of a batch: each file is its own chunk stream (writer.go:125-128 resets hash and
 *     seglen at Annotate), dealt as contiguous file ranges balanced by bytes (pfscdc_deal).
 *   Unordered writer: serialized filesets (independent chunk streams, fileset/
 *     unordered_writer.go:83-122, fileset/writer.go:36-50) dealt in groups, round robin.
 * The chunk-ref index is gathered over xGMI: each member's segment records and Refs stay on
 * its device and are copied peer to peer (hipMemcpyPeerAsync, direct peer access enabled at
 * create) into one index on the first member's device (the index device), where their file ids
 * are rebased, then copied to the host once.  A group is owned by one thread at a time; its
 * member ctxs belong to it (do not destroy them; do not scan on the group while an unordered
 * writer made from it is open). */

typedef struct pfscdc_group pfscdc_group;

/* Byte-balanced contiguous split of nitems items (item i = [offsets[i], offsets[i+1]),
 * nondecreasing) into nparts parts: part r = items [part_begin[r], part_begin[r+1]), starting
 * at the first item whose prefix reaches ceil(r * total / nparts) bytes (greedy prefix split,
 * items whole and in order; parts may be empty).  part_begin: nparts + 1 entries.  Host only. */
int pfscdc_deal(const uint64_t* offsets, uint32_t nitems, uint32_t nparts, uint32_t* part_begin);

/* One ctx per devices[k] (k < n) with params and options (0 or PFSCDC_OPT_REF_IDS).  The
 * index device is devices[0]. */
int pfscdc_group_create(const pfscdc_params* params, const int* devices, uint32_t n,
                        uint32_t options, pfscdc_group** out);
int pfscdc_group_destroy(pfscdc_group* g);
uint32_t pfscdc_group_size(const pfscdc_group* g);
/* Member i's ctx (owned by the group), e.g. for pfscdc_fill_synthetic on its device. */
pfscdc_ctx* pfscdc_group_ctx(pfscdc_group* g, uint32_t i);
const char* pfscdc_group_last_error(const pfscdc_group* g);

/* pfscdc_scan of a batch of files in host memory over the group: member k scans the files
 * [part_begin[k], part_begin[k+1]) of pfscdc_deal(file_offsets, nfiles, n), copying its own
 * byte range to its device, all members at once.  Blocks until the gathered index is on the
 * host.  Results as pfscdc_scan's, file ids global. */
int pfscdc_group_scan(pfscdc_group* g, const void* bytes, uint64_t nbytes,
                      const uint64_t* file_offsets, uint32_t nfiles);
/* The same over device-resident bytes: member_bytes[k] (device pointer on member k's device,
 * 16-B aligned) holds files [part_begin[k], part_begin[k+1]) contiguously, i.e. bytes
 * [file_offsets[part_begin[k]], file_offsets[part_begin[k+1]]) of the batch.  part_begin:
 * n + 1 entries (NULL = pfscdc_deal's split). */
int pfscdc_group_scan_resident(pfscdc_group* g, const void* const* member_bytes,
                               const uint64_t* file_offsets, uint32_t nfiles,
                               const uint32_t* part_begin);
/* One stream (a single file of nbytes in host memory, e.g. configs[2]'s 10 GiB) split across
 * the members, block-parallel with window-overlap stitching: member k holds an equal byte range
 * (borders on 64-byte boundaries) plus the 64 bytes in front (the window) and up to
 * max_chunk - 1 bytes after (for the segment that straddles its end), finds its range's
 * candidate positions (pfscdc_candidates); the serial min/max selection (writer.go:163-189)
 * then runs once over the gathered candidates on the host, and each segment is hashed by the
 * member holding its first byte.  Results as for one file through the accessors below (file 0;
 * no Refs, no dealing, no device index); equal to pfscdc_scan of the stream on one ctx. */
int pfscdc_group_scan_stream(pfscdc_group* g, const void* bytes, uint64_t nbytes);
/* Results of the last group scan (valid until the next one): the gathered index ordered by
 * (file, offset) with global file ids, per-file ranges (nfiles + 1), Refs (NULL unless the
 * group has PFSCDC_OPT_REF_IDS), and the dealing used (n + 1). */
uint64_t pfscdc_group_num_segments(const pfscdc_group* g);
const pfscdc_segment* pfscdc_group_segments(const pfscdc_group* g);
const uint64_t* pfscdc_group_file_segment_begin(const pfscdc_group* g);
const pfscdc_ref* pfscdc_group_refs(const pfscdc_group* g);
const uint32_t* pfscdc_group_part_begin(const pfscdc_group* g);
/* The gathered index as it lies on the index device (device pointers; nullable outputs). */
int pfscdc_group_index_device(const pfscdc_group* g, const pfscdc_segment** segs,
                              const pfscdc_ref** refs, int* device);
/* Device time of the last group scan: member_ms[k] (n entries) member k's scan-to-hash
 * (pfscdc_last_timings out[4]); gather_ms the peer copies and rebase on the index device;
 * gather_bytes the bytes they moved. */
int pfscdc_group_last_timings(const pfscdc_group* g, float* member_ms, float* gather_ms,
                              uint64_t* gather_bytes);

/* fileset.Storage.NewUnorderedWriter over a device group (the group needs PFSCDC_OPT_REF_IDS):
 * as pfscdc_uw_create, with one group writer per member, each writing on its member's ctx and
 * device (index levels too).  Serialized filesets go out in groups of max(mem_threshold,
 * PFSCDC_UW_INFLIGHT / n) bytes, round robin over the members, and each Put's bytes are
 * uploaded to the device of the member that will write them.  Events reach cb in group order,
 * each group's events as one writer would emit them, so the event stream equals that of
 * pfscdc_uw_create on one ctx with PFSCDC_UW_INFLIGHT set to the same group bytes; roots
 * are identical whatever the grouping. */
int pfscdc_uw_create_group(pfscdc_group* g, int64_t mem_threshold,
                           const pfscdc_params* index_params, pfscdc_uw_cb cb, void* user,
                           pfscdc_uwriter** out);

/* fileset.Clean(p, isDir) (fileset/util.go:67-77) into out (cap bytes incl. NUL). */
int pfscdc_path_clean(const char* path, int is_directory, char* out, uint64_t cap);

/* ---- tuning knobs (no reference counterpart; INTEGRATION.md lists each with its range) ----
 * Every knob is one process-wide integer named after its environment variable (PFSCDC_*).
 * The library reads the environment once, the first time any knob is used; an unset, empty,
 * non-numeric or out-of-range variable leaves the default (a bad value is reported on stderr).
 * No knob changes any result: they select between exact forms of the same computation or size
 * the host-fed writer's pools.  pfscdc_set_knob changes a knob for the whole process (atomic:
 * a launch already enqueued keeps the value it read).  When a knob takes effect:
 *   PFSCDC_UW_* (and PFSCDC_CTX_CACHE for the contexts it makes): when an unordered writer
 *     is created, for that writer's lifetime;
 *   PFSCDC_COPY_THREADS: once, when the first large Put builds the process-wide copy pool;
 *     from then on setting it to another value returns PFSCDC_ESTATE;
 *   every other knob: at the next call that launches the kernels it selects.
 * PFSCDC_EINVAL for an unknown name or a value outside the knob's range.  A PFSCDC_* variable
 * in the environment that is not a knob is reported on stderr and ignored. */
int pfscdc_set_knob(const char* name, int64_t value);
int pfscdc_get_knob(const char* name, int64_t* value);
/* The i-th knob's name (0-based), NULL past the last; lo/hi (nullable) its range and def
 * (nullable) its built-in default. */
const char* pfscdc_knob_info(int i, int64_t* lo, int64_t* hi, int64_t* def);

/* How the last pfscdc_scan on ctx skipped bytes (bit set): PFSCDC_SCAN_SKIPPED_FIRST_MIN =
 * the first min - 1 bytes of each file were not rolled; PFSCDC_SCAN_SKIPPED_CUTS = the scan
 * also skipped past the cuts it had settled (rank-ordered units; needs min - 1 >= 256 KiB and
 * at most one file per 16 KiB of the batch).  0: every byte was rolled. */
#define PFSCDC_SCAN_SKIPPED_FIRST_MIN 1u
#define PFSCDC_SCAN_SKIPPED_CUTS 2u
int pfscdc_last_scan_mode(pfscdc_ctx* ctx, uint32_t* mode);

#ifdef __cplusplus
}
#endif
#endif /* PFSCDC_H */
