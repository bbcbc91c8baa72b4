// writer.cpp — chunk.Writer mirror over the GPU batch pipeline (host logic).
//
// Reference: /root/reference/src/internal/storage/chunk/writer.go
//   Annotate          :118-130  cut before a file when the open chunk holds >= avg bytes
//   Write / roll      :132-189  per-file cut positions          -> GPU (pfscdc_scan)
//   writeData         :191-196
//   createChunk       :198-213  edge = first || last, split annotations, chunkCount++
//   splitAnnotations  :215-231  the next chunk starts with a size-0 copy of the last one
//   processChunk      :233-253  hashing -> GPU; callbacks serially in chunk order
//   maybeUpload       :255-271  chunk.Create(CreateOptions{}) -> Ref.Id/Dek on the GPU
//                               (pfscdc::create_refs_device) when the ctx asks for refs
//   processAnnotations:288-312  DataRef{Hash, OffsetBytes, SizeBytes} per piece with size > 0
//   Close             :423-438  always emits a last chunk (possibly empty, E1)
// Hash and seglen reset at every Annotate (writer.go:125-128), so each file's cut positions
// depend only on its own bytes and whole files can be batched to the GPU; only the
// cross-file state (open-chunk length, annotation list, first/last) is replayed here, by
// ChunkFormer, which pfscdc_form_chunks also runs over a device-resident batch.
#include <cstring>
#include <string>
#include <vector>

#include "pfscdc_internal.h"

namespace {

struct PendingFile {
  uint64_t user;
  uint64_t begin;
};

struct OpenAnnotation {
  uint64_t user;
  int64_t size;
  uint8_t hash[32];  // hash of the (single) piece this annotation has in the open chunk
};

// One createChunk: the chunk's Ref fields, its annotations (outs[ann_begin, ann_end)) and
// its byte range [begin, end) in the buffer the pieces were replayed over.
struct ChunkEvent {
  pfscdc_chunk_ref ref;
  size_t ann_begin, ann_end;
  uint64_t begin, end;
  uint8_t known;     // the chunk is exactly one DataRef: Hash(chunk) == that DataRef's hash
  uint8_t hash[32];
};

// The cross-file state machine of chunk.Writer, fed with the GPU's per-file segments.
struct ChunkFormer {
  int64_t avg = 0;
  std::vector<OpenAnnotation> annotations;
  int64_t open_len = 0;  // w.buf.Len()
  bool first = true;
  int64_t chunk_count = 0;
  uint64_t pos = 0, open_start = 0;  // byte positions in the current buffer
  std::vector<ChunkEvent> events;
  std::vector<pfscdc_annotation_out> outs;

  void reset_stream() {  // a fresh chunk.Writer
    annotations.clear();
    open_len = 0;
    first = true;
    chunk_count = 0;
  }

  void create(bool last) {  // createChunk + splitAnnotations + processAnnotations
    ChunkEvent ev{};
    ev.ref.chunk_index = (uint64_t)chunk_count;
    ev.ref.size_bytes = open_len;
    ev.ref.edge = first || last ? 1 : 0;
    ev.ann_begin = outs.size();
    ev.begin = open_start;
    ev.end = pos;
    int64_t offset = 0;
    int pieces = 0;
    for (const OpenAnnotation& a : annotations) {
      pfscdc_annotation_out o{};
      o.user = a.user;
      if (a.size > 0) {
        o.has_data_ref = 1;
        std::memcpy(o.data_ref.hash, a.hash, 32);
        o.data_ref.offset_bytes = offset;
        o.data_ref.size_bytes = a.size;
        offset += a.size;
        pieces++;
        if (a.size == open_len) {  // newDataRef: chunkRef.SizeBytes == size -> same hash
          ev.known = 1;
          std::memcpy(ev.hash, a.hash, 32);
        }
      }
      outs.push_back(o);
    }
    if (pieces != 1) ev.known = 0;
    ev.ann_end = outs.size();
    events.push_back(ev);
    const uint64_t last_user = annotations.back().user;
    annotations.clear();
    annotations.push_back(OpenAnnotation{last_user, 0, {}});
    first = false;
    open_len = 0;
    open_start = pos;
    chunk_count++;
  }

  void annotate(uint64_t user) {  // writer.go:118-130
    if (open_len >= avg && !annotations.empty()) create(false);
    annotations.push_back(OpenAnnotation{user, 0, {}});
  }

  void piece(const pfscdc_segment& s) {  // writeData (+ createChunk at a cut)
    OpenAnnotation& a = annotations.back();
    a.size += (int64_t)s.size;
    std::memcpy(a.hash, s.hash, 32);
    open_len += (int64_t)s.size;
    pos += s.size;
    if (s.flags & PFSCDC_SEG_CUT) create(false);
  }

  void close() {  // writer.go:423-438
    if (!annotations.empty()) create(true);
  }
};

}  // namespace

struct pfscdc_writer {
  pfscdc_ctx* ctx = nullptr;
  pfscdc_writer_cb cb = nullptr;
  void* user = nullptr;
  uint64_t batch_bytes = 1ULL << 30;
  bool ref_ids = false;
  std::vector<uint8_t> buf;           // pending file bytes
  std::vector<uint8_t> carry;         // ref_ids: bytes of the open chunk from earlier flushes
  std::vector<PendingFile> files;     // pending annotations, in order
  std::vector<uint64_t> offsets;      // scratch
  std::vector<uint64_t> chunk_offs;   // scratch
  std::vector<uint8_t> hashes, known;
  std::vector<pfscdc_ref> refs;
  uint8_t* d_buf = nullptr;           // ref_ids: carry ++ pending files on the device
  uint64_t d_cap = 0;
  ChunkFormer cf;
  bool closed = false;
  int64_t annotation_count = 0;
  int err = 0;                        // sticky (writer.go:145-161)
};

namespace {

int set_err(pfscdc_writer* w, int code) {
  if (!w->err) w->err = code;
  return w->err;
}

// Refs for the chunks formed in this flush (contiguous ranges of d_buf), then the
// callbacks, serially in chunk order.
int dispatch(pfscdc_writer* w, uint64_t valid) {
  ChunkFormer& cf = w->cf;
  const size_t n = cf.events.size();
  int rc = PFSCDC_OK;
  if (w->ref_ids && n) {
    w->chunk_offs.resize(n + 1);
    w->hashes.resize(32 * n);
    w->known.resize(n);
    w->refs.resize(n);
    for (size_t i = 0; i < n; i++) {
      const ChunkEvent& ev = cf.events[i];
      w->chunk_offs[i] = ev.begin;
      w->known[i] = ev.known;
      std::memcpy(&w->hashes[32 * i], ev.hash, 32);
    }
    w->chunk_offs[n] = cf.events[n - 1].end;
    rc = pfscdc::create_refs_device(w->ctx, w->d_buf, valid, w->chunk_offs.data(), (uint32_t)n,
                                    w->hashes.data(), w->known.data(), w->refs.data());
    if (rc) {
      cf.events.clear();
      cf.outs.clear();
      return set_err(w, rc);
    }
  }
  for (size_t i = 0; i < n && !rc; i++) {
    ChunkEvent& ev = cf.events[i];
    if (w->ref_ids) {
      ev.ref.has_ref = 1;
      ev.ref.ref = w->refs[i];
    }
    if (w->cb && w->cb(w->user, &ev.ref, cf.outs.data() + ev.ann_begin,
                       (uint32_t)(ev.ann_end - ev.ann_begin)) != 0)
      rc = set_err(w, PFSCDC_ECALLBACK);
  }
  cf.events.clear();
  cf.outs.clear();
  return rc;
}

// Runs the pending files through the GPU, replays the chunk state machine over their
// segments (and Close's last chunk if final), then creates refs and calls back.
int flush(pfscdc_writer* w, bool final) {
  const uint32_t nfiles = (uint32_t)w->files.size();
  if (nfiles == 0 && !final) return PFSCDC_OK;
  ChunkFormer& cf = w->cf;
  const uint64_t nbytes = w->buf.size();
  uint64_t base = 0;  // device position of the first pending file byte
  if (w->ref_ids) {
    // [carry | files] contiguous on the device, files 16-byte aligned for the scan
    const uint64_t cl = w->carry.size();
    base = (cl + 15) & ~15ULL;
    const uint64_t need = base + nbytes + 64;
    if (need > w->d_cap) {
      if (w->d_buf) (void)hipFree(w->d_buf);
      w->d_buf = nullptr;
      w->d_cap = 0;
      const uint64_t want = need + need / 4;
      if (hipSetDevice(pfscdc::ctx_device(w->ctx)) != hipSuccess ||
          hipMalloc((void**)&w->d_buf, want) != hipSuccess)
        return set_err(w, PFSCDC_ENOMEM);
      w->d_cap = want;
    }
    if ((cl && hipMemcpy(w->d_buf + base - cl, w->carry.data(), cl, hipMemcpyHostToDevice) != hipSuccess) ||
        (nbytes && hipMemcpy(w->d_buf + base, w->buf.data(), nbytes, hipMemcpyHostToDevice) != hipSuccess))
      return set_err(w, PFSCDC_EHIP);
    cf.open_start = base - cl;
  } else {
    cf.open_start = 0;
  }
  cf.pos = base;
  if (nfiles) {
    w->offsets.resize(nfiles + 1);
    for (uint32_t f = 0; f < nfiles; f++) w->offsets[f] = w->files[f].begin;
    w->offsets[nfiles] = nbytes;
    int rc = w->ref_ids
                 ? pfscdc::scan_sync(w->ctx, w->d_buf + base, nbytes, 1, w->offsets.data(), nfiles, 0)
                 : pfscdc::scan_sync(w->ctx, w->buf.data(), nbytes, 0, w->offsets.data(), nfiles, 0);
    if (rc) return set_err(w, rc);
    const pfscdc_segment* segs = pfscdc_segments(w->ctx);
    const uint64_t* begin = pfscdc_file_segment_begin(w->ctx);
    for (uint32_t f = 0; f < nfiles; f++) {
      cf.annotate(w->files[f].user);
      for (uint64_t s = begin[f]; s < begin[f + 1]; s++) cf.piece(segs[s]);
    }
  }
  if (final) cf.close();
  int rc = dispatch(w, base + nbytes);
  if (rc) return rc;
  if (w->ref_ids) {  // the open chunk's bytes move to the front of the next flush
    const uint64_t cl = w->carry.size();
    const uint64_t keep_from = cf.open_start;  // >= base - cl
    std::vector<uint8_t> next;
    if (keep_from < base) next.assign(w->carry.begin() + (keep_from - (base - cl)), w->carry.end());
    const uint64_t from_buf = keep_from > base ? keep_from - base : 0;
    next.insert(next.end(), w->buf.begin() + from_buf, w->buf.end());
    w->carry.swap(next);
  }
  w->files.clear();
  w->buf.clear();
  return PFSCDC_OK;
}

}  // namespace

extern "C" {

int pfscdc_writer_create(pfscdc_ctx* ctx, pfscdc_writer_cb cb, void* user, uint64_t batch_bytes,
                         pfscdc_writer** out) {
  if (!ctx || !out) return PFSCDC_EINVAL;
  pfscdc_writer* w = new pfscdc_writer();
  w->ctx = ctx;
  w->cb = cb;
  w->user = user;
  if (batch_bytes) w->batch_bytes = batch_bytes;
  w->ref_ids = (pfscdc::ctx_options(ctx) & PFSCDC_OPT_REF_IDS) != 0;
  w->cf.avg = (int64_t)1 << pfscdc::ctx_params(ctx).average_bits;  // chunkSize.avg, option.go:52
  *out = w;
  return PFSCDC_OK;
}

int pfscdc_writer_annotate(pfscdc_writer* w, uint64_t user) {
  if (!w) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return set_err(w, PFSCDC_ESTATE);
  if (w->buf.size() >= w->batch_bytes) {
    int rc = flush(w, false);
    if (rc) return rc;
  }
  w->files.push_back(PendingFile{user, (uint64_t)w->buf.size()});
  w->annotation_count++;
  return PFSCDC_OK;
}

int pfscdc_writer_write(pfscdc_writer* w, const void* data, uint64_t n) {
  if (!w) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed || w->files.empty()) return set_err(w, PFSCDC_ESTATE);  // Go: panics
  if (n) {
    if (!data) return set_err(w, PFSCDC_EINVAL);
    const uint8_t* p = (const uint8_t*)data;
    w->buf.insert(w->buf.end(), p, p + n);
  }
  return PFSCDC_OK;
}

int pfscdc_writer_close(pfscdc_writer* w) {
  if (!w) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return PFSCDC_OK;
  w->closed = true;
  return flush(w, true);
}

int64_t pfscdc_writer_chunk_count(const pfscdc_writer* w) { return w ? w->cf.chunk_count : 0; }
int64_t pfscdc_writer_annotation_count(const pfscdc_writer* w) {
  return w ? w->annotation_count : 0;
}

int pfscdc_writer_destroy(pfscdc_writer* w) {
  if (!w) return PFSCDC_EINVAL;
  if (w->d_buf) (void)hipFree(w->d_buf);
  delete w;
  return PFSCDC_OK;
}

int pfscdc_form_chunks(pfscdc_ctx* ctx, const uint32_t* stream_file_begin, uint32_t nstreams,
                       uint64_t* chunk_offsets, uint8_t* content_hashes, uint8_t* hash_known,
                       uint64_t cap, uint64_t* nchunks) {
  if (!ctx || !nchunks || (cap && (!chunk_offsets || !content_hashes || !hash_known)))
    return PFSCDC_EINVAL;
  const uint64_t* begin = pfscdc_file_segment_begin(ctx);
  const pfscdc_segment* segs = pfscdc_segments(ctx);
  if (!pfscdc::ctx_scan_valid(ctx)) return PFSCDC_ESTATE;
  const uint32_t nfiles = pfscdc::ctx_nfiles(ctx);
  if (!begin || (nfiles && !segs)) return PFSCDC_ESTATE;
  const uint32_t one[2] = {0, nfiles};
  if (!stream_file_begin) {
    stream_file_begin = one;
    nstreams = 1;
  }
  if (stream_file_begin[0] != 0 || stream_file_begin[nstreams] != nfiles) return PFSCDC_EINVAL;
  ChunkFormer cf;
  cf.avg = (int64_t)1 << pfscdc::ctx_params(ctx).average_bits;
  uint64_t n = 0;
  int rc = PFSCDC_OK;
  for (uint32_t k = 0; k < nstreams; k++) {
    const uint32_t f0 = stream_file_begin[k], f1 = stream_file_begin[k + 1];
    if (f1 < f0) return PFSCDC_EINVAL;
    if (f1 == f0) continue;  // a stream with no annotation writes no chunk
    cf.reset_stream();
    cf.open_start = cf.pos = pfscdc::ctx_file_offset(ctx, f0);
    for (uint32_t f = f0; f < f1; f++) {
      cf.annotate(f);
      for (uint64_t s = begin[f]; s < begin[f + 1]; s++) cf.piece(segs[s]);
    }
    cf.close();
    for (const ChunkEvent& ev : cf.events) {
      if (n < cap) {
        chunk_offsets[n] = ev.begin;
        chunk_offsets[n + 1] = ev.end;
        hash_known[n] = ev.known;
        std::memcpy(content_hashes + 32 * n, ev.hash, 32);
      } else {
        rc = PFSCDC_ENOMEM;
      }
      n++;
    }
    cf.events.clear();
    cf.outs.clear();
  }
  *nchunks = n;
  return rc;
}

}  // extern "C"
