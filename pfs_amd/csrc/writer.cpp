// writer.cpp — chunk.Writer mirror over the GPU batch pipeline (host logic).
//
// Reference: /root/reference/src/internal/storage/chunk/writer.go
//   Annotate          :118-130  cut before a file when the open chunk holds >= avg bytes
//   Write / roll      :132-189  per-file cut positions          -> GPU (pfscdc_scan)
//   writeData         :191-196
//   createChunk       :198-213  edge = first || last, split annotations, chunkCount++
//   splitAnnotations  :215-231  the next chunk starts with a size-0 copy of the last one
//   processChunk      :233-253  hashing -> GPU; callbacks serially in chunk order
//   processAnnotations:288-312  DataRef{Hash, OffsetBytes, SizeBytes} per piece with size > 0
//   Close             :423-438  always emits a last chunk (possibly empty, E1)
// Hash and seglen reset at every Annotate (writer.go:125-128), so each file's cut positions
// depend only on its own bytes and whole files can be batched to the GPU; only the
// cross-file state (open-chunk length, annotation list, first/last) is replayed here.
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
  pfscdc_dataref ref;  // hash of the (single) piece this annotation has in the open chunk
};

}  // namespace

struct pfscdc_writer {
  pfscdc_ctx* ctx = nullptr;
  pfscdc_writer_cb cb = nullptr;
  void* user = nullptr;
  uint64_t batch_bytes = 1ULL << 30;
  std::vector<uint8_t> buf;           // pending file bytes
  std::vector<PendingFile> files;     // pending annotations, in order
  std::vector<uint64_t> offsets;      // scratch
  std::vector<OpenAnnotation> annotations;
  std::vector<pfscdc_annotation_out> out;  // scratch for callbacks
  int64_t open_len = 0;               // w.buf.Len()
  int64_t avg = 0;
  bool first = true;
  bool last = false;
  bool closed = false;
  int64_t chunk_count = 0;
  int64_t annotation_count = 0;
  int err = 0;                        // sticky (writer.go:145-161)
  std::string err_msg;
};

namespace {

int set_err(pfscdc_writer* w, int code) {
  if (!w->err) w->err = code;
  return w->err;
}

int create_chunk(pfscdc_writer* w) {
  const bool edge = w->first || w->last;
  pfscdc_chunk_ref ref{};
  ref.chunk_index = (uint64_t)w->chunk_count;
  ref.size_bytes = w->open_len;
  ref.edge = edge ? 1 : 0;
  w->out.clear();
  int64_t offset = 0;
  for (const OpenAnnotation& a : w->annotations) {
    pfscdc_annotation_out o{};
    o.user = a.user;
    if (a.size > 0) {
      o.has_data_ref = 1;
      o.data_ref = a.ref;
      o.data_ref.offset_bytes = offset;
      o.data_ref.size_bytes = a.size;
      offset += a.size;
    }
    w->out.push_back(o);
  }
  const uint64_t last_user = w->annotations.back().user;
  w->annotations.clear();
  w->annotations.push_back(OpenAnnotation{last_user, 0, {}});
  w->first = false;
  w->open_len = 0;
  w->chunk_count++;
  if (w->cb && w->cb(w->user, &ref, w->out.data(), (uint32_t)w->out.size()) != 0)
    return set_err(w, PFSCDC_ECALLBACK);
  return PFSCDC_OK;
}

int annotate_replay(pfscdc_writer* w, uint64_t user) {
  if (w->open_len >= w->avg && !w->annotations.empty()) {
    int rc = create_chunk(w);
    if (rc) return rc;
  }
  w->annotations.push_back(OpenAnnotation{user, 0, {}});
  return PFSCDC_OK;
}

// Runs the pending files through the GPU and replays the chunk state machine.
int flush(pfscdc_writer* w) {
  if (w->files.empty()) return PFSCDC_OK;
  const uint32_t nfiles = (uint32_t)w->files.size();
  w->offsets.resize(nfiles + 1);
  for (uint32_t f = 0; f < nfiles; f++) w->offsets[f] = w->files[f].begin;
  w->offsets[nfiles] = w->buf.size();
  int rc = pfscdc_scan(w->ctx, w->buf.data(), w->buf.size(), 0, w->offsets.data(), nfiles);
  if (rc) {
    w->err_msg = pfscdc_last_error(w->ctx);
    return set_err(w, rc);
  }
  const pfscdc_segment* segs = pfscdc_segments(w->ctx);
  const uint64_t* begin = pfscdc_file_segment_begin(w->ctx);
  for (uint32_t f = 0; f < nfiles; f++) {
    rc = annotate_replay(w, w->files[f].user);
    if (rc) return rc;
    for (uint64_t s = begin[f]; s < begin[f + 1]; s++) {
      OpenAnnotation& a = w->annotations.back();
      a.size += (int64_t)segs[s].size;
      std::memcpy(a.ref.hash, segs[s].hash, 32);
      w->open_len += (int64_t)segs[s].size;
      if (segs[s].flags & PFSCDC_SEG_CUT) {
        rc = create_chunk(w);
        if (rc) return rc;
      }
    }
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
  w->avg = (int64_t)1 << pfscdc::ctx_params(ctx).average_bits;  // chunkSize.avg, option.go:52
  *out = w;
  return PFSCDC_OK;
}

int pfscdc_writer_annotate(pfscdc_writer* w, uint64_t user) {
  if (!w) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return set_err(w, PFSCDC_ESTATE);
  if (w->buf.size() >= w->batch_bytes) {
    int rc = flush(w);
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
  int rc = flush(w);
  if (rc) return rc;
  w->closed = true;
  if (!w->annotations.empty()) {
    w->last = true;
    rc = create_chunk(w);
    if (rc) return rc;
  }
  return PFSCDC_OK;
}

int64_t pfscdc_writer_chunk_count(const pfscdc_writer* w) { return w ? w->chunk_count : 0; }
int64_t pfscdc_writer_annotation_count(const pfscdc_writer* w) {
  return w ? w->annotation_count : 0;
}

int pfscdc_writer_destroy(pfscdc_writer* w) {
  delete w;
  return PFSCDC_OK;
}

}  // extern "C"
