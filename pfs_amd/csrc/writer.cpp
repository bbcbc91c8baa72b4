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
//   Copy              :315-420  buffer whole-chunk DataRefs (cheap copy) or re-roll them
//   Close             :423-438  always emits a last chunk (possibly empty, E1)
// The hash and seglen reset at every Annotate and every cut (writer.go:125-128,211), so the
// bytes after a reset point are scanned as an independent "file" on the GPU; only the
// cross-file state (open-chunk length, annotation list, first/last) is replayed here, by
// ChunkFormer, which pfscdc_form_chunks also runs over a device-resident batch.
//
// Pending bytes are a list of pending files: a fresh annotation, or a continuation of the
// last open annotation (bytes written after a flush that stopped at a cut).  A flush scans
// them and replays the segments; a PARTIAL flush (Copy needs buf.Len()) withholds the last
// annotation's bytes after its last cut, which stay pending as a continuation.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "pfscdc_internal.h"

namespace {

struct PendingFile {
  uint64_t user;
  uint64_t begin;
  bool cont;  // continues the last open annotation (no Annotate to replay)
};

struct OpenAnnotation {
  uint64_t user;
  int64_t size;      // bytes in the open chunk
  uint8_t hash[32];  // hash of the (single) piece this annotation has in the open chunk
  bool has_next;     // a buffered (Copy) DataRef: Annotation.NextDataRef while buffering
  pfscdc_full_dataref next;
  uint64_t pbegin = 0;    // buffer position of the piece
  bool hpending = false;  // the piece's hash is still to be computed (deferred flush)
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
  std::vector<uint64_t> out_begin;   // per out: buffer position of its piece
  std::vector<uint8_t> out_pending;  // per out: piece hash still to be computed

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
      out_begin.push_back(a.pbegin);
      out_pending.push_back(a.size > 0 && a.hpending);
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
    annotations.push_back(OpenAnnotation{last_user, 0, {}, false, {}, pos, false});
    first = false;
    open_len = 0;
    open_start = pos;
    chunk_count++;
  }

  void annotate(uint64_t user) {  // writer.go:118-130
    if (open_len >= avg && !annotations.empty()) create(false);
    annotations.push_back(OpenAnnotation{user, 0, {}, false, {}, pos, false});
  }

  // writeData (+ createChunk at a cut); pending: the segment's hash was not computed yet
  void piece(const pfscdc_segment& s, bool pending = false) {
    OpenAnnotation& a = annotations.back();
    if (a.size == 0) a.pbegin = pos;
    a.size += (int64_t)s.size;
    if (!pending) std::memcpy(a.hash, s.hash, 32);
    a.hpending = pending;
    open_len += (int64_t)s.size;
    pos += s.size;
    if (s.flags & PFSCDC_SEG_CUT) create(false);
  }

  void close() {  // writer.go:423-438
    if (!annotations.empty()) create(true);
  }
};

}  // namespace

struct pfscdc_store {
  std::map<std::string, std::string> objects;  // Ref.Id -> ciphertext
};

struct pfscdc_writer {
  pfscdc_ctx* ctx = nullptr;
  pfscdc_writer_cb cb = nullptr;
  void* user = nullptr;
  uint64_t batch_bytes = 1ULL << 30;
  bool ref_ids = false;
  pfscdc_store* store = nullptr;      // the chunk client (Copy reads it)
  bool upload = false;                // Create stores each new chunk's ciphertext
  std::vector<uint8_t> buf;           // pending file bytes
  // pending bytes held by the caller instead (writer_write_span: a fileset's Put arena);
  // their concatenation replaces buf, which stays empty while spans are pending
  std::vector<std::pair<const uint8_t*, uint64_t>> spans;
  std::vector<const uint8_t*> span_dev;  // per span: the same bytes already on the device, or null
  uint64_t span_bytes = 0;
  std::vector<uint8_t> carry;         // ref_ids: bytes of the open chunk from earlier flushes
  std::vector<PendingFile> files;     // pending annotations, in order
  std::vector<uint64_t> offsets;      // scratch
  std::vector<uint64_t> chunk_offs;   // scratch
  std::vector<uint8_t> hashes, known;
  std::vector<pfscdc_ref> refs;
  std::vector<uint8_t> fetched;       // scratch: a chunk read back for Copy
  std::map<std::string, std::string> plain;  // chunks verified + decrypted ahead (prefetch)
  uint8_t* d_buf = nullptr;           // ref_ids: carry ++ pending files on the device
  uint8_t* d_ctext = nullptr;         // upload: ciphertexts, same layout as d_buf
  uint64_t d_cap = 0;
  ChunkFormer cf;
  // deferred flushes (Copy's buf.Len() probes): buf[0, replayed) was replayed without its
  // BLAKE2b; buf, carry and the formed chunks stay until a dispatching flush hashes them
  uint64_t replayed = 0;
  // a deferred flush ran and nothing has dispatched since (replayed alone cannot say: a
  // deferred flush may replay 0 bytes of buf, e.g. only the carry forming a chunk at an
  // Annotate, and the next flush must not re-base the open chunk onto the carry again)
  bool deferred = false;
  uint64_t dev_upto = 0;              // while deferring: buf[0, dev_upto) is already on the device
  bool buffering = false;             // Writer.buffering (Copy)
  bool closed = false;
  int64_t annotation_count = 0;
  int err = 0;                        // sticky (writer.go:145-161)
};

namespace {

enum FlushMode { kBatch, kPartial, kFinal };

int set_err(pfscdc_writer* w, int code) {
  if (!w->err) w->err = code;
  return w->err;
}

// Grows the device buffer to need bytes, keeping its first keep bytes.
int ensure_device(pfscdc_writer* w, uint64_t need, uint64_t keep = 0) {
  if (need <= w->d_cap) return PFSCDC_OK;
  const uint64_t want = need + need / 4;
  uint8_t *nb = nullptr, *nc = nullptr;
  if (hipSetDevice(pfscdc::ctx_device(w->ctx)) != hipSuccess ||
      hipMalloc((void**)&nb, want) != hipSuccess)
    return PFSCDC_ENOMEM;
  if (w->upload && w->store && hipMalloc((void**)&nc, want) != hipSuccess) {
    (void)hipFree(nb);
    return PFSCDC_ENOMEM;
  }
  if (keep && w->d_buf && hipMemcpy(nb, w->d_buf, keep, hipMemcpyDeviceToDevice) != hipSuccess) {
    (void)hipFree(nb);
    if (nc) (void)hipFree(nc);
    return PFSCDC_EHIP;
  }
  if (w->d_buf) (void)hipFree(w->d_buf);
  if (w->d_ctext) (void)hipFree(w->d_ctext);
  w->d_buf = nb;
  w->d_ctext = nc;
  w->d_cap = want;
  return PFSCDC_OK;
}

void clear_events(ChunkFormer& cf) {
  cf.events.clear();
  cf.outs.clear();
  cf.out_begin.clear();
  cf.out_pending.clear();
}

// The callbacks of the chunks formed in this flush, serially in chunk order (refs in w->refs).
int callbacks(pfscdc_writer* w) {
  ChunkFormer& cf = w->cf;
  int rc = PFSCDC_OK;
  for (size_t i = 0; i < cf.events.size() && !rc; i++) {
    ChunkEvent& ev = cf.events[i];
    if (w->ref_ids && !ev.ref.copied) {
      ev.ref.has_ref = 1;
      ev.ref.ref = w->refs[i];
    }
    if (w->cb && w->cb(w->user, &ev.ref, cf.outs.data() + ev.ann_begin,
                       (uint32_t)(ev.ann_end - ev.ann_begin)) != 0)
      rc = set_err(w, PFSCDC_ECALLBACK);
  }
  clear_events(cf);
  return rc;
}

// client.Create's upload of chunk i's ciphertext (device ct + [begin, end)) unless present.
int upload(pfscdc_store* st, const pfscdc_ref& ref, const uint8_t* ct, uint64_t begin,
           uint64_t end) {
  std::string id((const char*)ref.id, 32);
  if (st->objects.count(id)) return PFSCDC_OK;
  std::string obj(end - begin, '\0');
  if (!obj.empty() && hipMemcpy(&obj[0], ct + begin, obj.size(), hipMemcpyDeviceToHost) != hipSuccess)
    return PFSCDC_EHIP;
  st->objects.emplace(std::move(id), std::move(obj));
  return PFSCDC_OK;
}

// Refs (and the upload) for the chunks formed in this flush (contiguous ranges of d_buf),
// then the callbacks, serially in chunk order.
int dispatch(pfscdc_writer* w, uint64_t valid) {
  ChunkFormer& cf = w->cf;
  const size_t n = cf.events.size();
  int rc = PFSCDC_OK;
  w->refs.resize(n);
  if (w->ref_ids && n) {
    std::vector<size_t> which;  // new chunks (cheap copies reference existing ones)
    for (size_t i = 0; i < n; i++)
      if (!cf.events[i].ref.copied) which.push_back(i);
    const size_t m = which.size();
    w->hashes.resize(32 * m);
    w->known.resize(m);
    std::vector<pfscdc_ref> refs(m);
    for (size_t k = 0; k < m; k++) {
      const ChunkEvent& ev = cf.events[which[k]];
      w->known[k] = ev.known;
      std::memcpy(&w->hashes[32 * k], ev.hash, 32);
    }
    uint8_t* ct = w->upload && w->store ? w->d_ctext : nullptr;
    // one create_refs call per run of new chunks that are contiguous in the device buffer (a
    // chunk's bytes are [offs[k], offs[k + 1]) there, so the offsets of one call must tile);
    // the chunks of one flush normally form a single run
    for (size_t r0 = 0; r0 < m && !rc;) {
      size_t r1 = r0 + 1;
      while (r1 < m && cf.events[which[r1]].begin == cf.events[which[r1 - 1]].end) r1++;
      w->chunk_offs.resize(r1 - r0 + 1);
      for (size_t k = r0; k < r1; k++) w->chunk_offs[k - r0] = cf.events[which[k]].begin;
      w->chunk_offs[r1 - r0] = cf.events[which[r1 - 1]].end;
      rc = pfscdc::create_refs_device(w->ctx, w->d_buf, valid, w->chunk_offs.data(),
                                      (uint32_t)(r1 - r0), w->hashes.data() + 32 * r0,
                                      w->known.data() + r0, refs.data() + r0, ct);
      for (size_t k = r0; k < r1 && !rc; k++) {
        w->refs[which[k]] = refs[k];
        if (ct) rc = upload(w->store, refs[k], ct, cf.events[which[k]].begin,
                            cf.events[which[k]].end);
      }
      r0 = r1;
    }
    if (rc) {
      clear_events(cf);
      return set_err(w, rc);
    }
  }
  return callbacks(w);
}

// The piece hashes deferred by kPartial flushes (formed chunks' pieces and the open
// chunk's), in one launch over the device buffer: the re-rolled chains run in parallel.
int resolve_pending(pfscdc_writer* w, uint64_t valid) {
  ChunkFormer& cf = w->cf;
  std::vector<uint64_t> begins, sizes;
  std::vector<std::pair<int, size_t>> who;  // (0: out, 1: open annotation), index
  for (size_t i = 0; i < cf.outs.size(); i++)
    if (cf.out_pending[i]) {
      begins.push_back(cf.out_begin[i]);
      sizes.push_back((uint64_t)cf.outs[i].data_ref.size_bytes);
      who.emplace_back(0, i);
    }
  for (size_t i = 0; i < cf.annotations.size(); i++)
    if (cf.annotations[i].hpending && cf.annotations[i].size > 0) {
      begins.push_back(cf.annotations[i].pbegin);
      sizes.push_back((uint64_t)cf.annotations[i].size);
      who.emplace_back(1, i);
    }
  if (who.empty()) return PFSCDC_OK;
  std::vector<uint8_t> h(32 * who.size());
  int rc = pfscdc::hash_records_device(w->ctx, w->d_buf, valid, begins.data(), sizes.data(),
                                       (uint32_t)who.size(), h.data());
  if (rc) return set_err(w, rc);
  for (size_t k = 0; k < who.size(); k++) {
    const uint8_t* hk = h.data() + 32 * k;
    if (who[k].first == 0) {
      std::memcpy(cf.outs[who[k].second].data_ref.hash, hk, 32);
      cf.out_pending[who[k].second] = 0;
    } else {
      OpenAnnotation& a = cf.annotations[who[k].second];
      std::memcpy(a.hash, hk, 32);
      a.hpending = false;
    }
  }
  for (ChunkEvent& ev : cf.events)  // a one-DataRef chunk's hash is its piece's
    if (!ev.ref.copied && ev.known)
      for (size_t i = ev.ann_begin; i < ev.ann_end; i++)
        if (cf.outs[i].has_data_ref) std::memcpy(ev.hash, cf.outs[i].data_ref.hash, 32);
  return PFSCDC_OK;
}

// Runs the pending files through the GPU and replays the chunk state machine over their
// segments (all of them, or for kPartial up to the last cut of the last annotation), plus
// Close's last chunk for kFinal; then creates refs and calls back.
// Copies pending caller spans into buf (every path but the grouped close reads buf).
void materialize(pfscdc_writer* w) {
  if (w->spans.empty()) return;
  w->buf.reserve(w->buf.size() + w->span_bytes);
  for (auto& sp : w->spans) w->buf.insert(w->buf.end(), sp.first, sp.first + sp.second);
  w->spans.clear();
  w->span_dev.clear();
  w->span_bytes = 0;
}

int flush(pfscdc_writer* w, FlushMode mode) {
  materialize(w);
  const uint32_t nfiles = (uint32_t)w->files.size();
  if (nfiles == 0 && mode != kFinal) return PFSCDC_OK;
  ChunkFormer& cf = w->cf;
  const uint64_t nbytes = w->buf.size();
  const uint64_t R = w->replayed;
  // a kPartial flush defers the hashing unless the kept bytes have grown to a batch
  const bool defer = mode == kPartial && nbytes < w->batch_bytes;
  // [carry | buf] contiguous on the device (carry: the open chunk's bytes of earlier
  // dispatched flushes, kept for chunk.Create)
  const uint64_t cl = w->carry.size();
  const uint64_t base = (cl + 15) & ~15ULL;
  // while deferring, carry and buf[0, dev_upto) are already on the device: send the rest
  const uint64_t have = w->deferred ? w->dev_upto : 0;
  int rc = ensure_device(w, base + nbytes + 64, have ? base + have : 0);
  if (rc) return set_err(w, rc);
  if ((!have && cl && hipMemcpy(w->d_buf + base - cl, w->carry.data(), cl, hipMemcpyHostToDevice) != hipSuccess) ||
      (nbytes > have && hipMemcpy(w->d_buf + base + have, w->buf.data() + have, nbytes - have,
                                  hipMemcpyHostToDevice) != hipSuccess))
    return set_err(w, PFSCDC_EHIP);
  w->dev_upto = nbytes;
  if (!w->deferred) cf.open_start = base - cl;  // else unchanged since the deferred flush
  cf.pos = base + R;
  uint64_t consumed = nbytes;  // bytes of buf replayed
  bool keep_tail = false;
  uint64_t tail_user = 0;
  if (nfiles) {
    // scan from a 16-byte aligned start; the few replayed bytes before base + R form a
    // dummy file whose segments are ignored
    const uint64_t start = (base + R) & ~15ULL;
    const uint32_t dummy = start < base + w->files[0].begin ? 1 : 0;
    w->offsets.clear();
    if (dummy) w->offsets.push_back(0);
    for (uint32_t f = 0; f < nfiles; f++) w->offsets.push_back(base + w->files[f].begin - start);
    w->offsets.push_back(base + nbytes - start);
    rc = pfscdc::scan_sync(w->ctx, w->d_buf + start, base + nbytes - start, 1, w->offsets.data(),
                           nfiles + dummy, defer ? pfscdc::kScanNoHash : 0);
    if (rc) return set_err(w, rc);
    const pfscdc_segment* segs = pfscdc_segments(w->ctx);
    const uint64_t* begin = pfscdc_file_segment_begin(w->ctx);
    for (uint32_t f = 0; f < nfiles; f++) {
      const uint32_t g = f + dummy;
      if (!w->files[f].cont) cf.annotate(w->files[f].user);
      uint64_t end = begin[g + 1];
      if (mode == kPartial && f + 1 == nfiles) {
        // withhold the bytes after the last cut: the annotation is still being written
        uint64_t s_end = begin[g];
        for (uint64_t s = begin[g]; s < end; s++)
          if (segs[s].flags & PFSCDC_SEG_CUT) s_end = s + 1;
        consumed = w->files[f].begin +
                   (s_end > begin[g] ? segs[s_end - 1].offset + segs[s_end - 1].size : 0);
        keep_tail = consumed < nbytes;
        tail_user = w->files[f].user;
        end = s_end;
      }
      for (uint64_t s = begin[g]; s < end; s++) cf.piece(segs[s], defer);
    }
  }
  if (mode == kFinal) cf.close();
  w->files.clear();
  if (defer) {  // everything stays: buf, carry, the formed chunks; only the tail is pending
    w->replayed = consumed;
    w->deferred = true;
    if (keep_tail) w->files.push_back(PendingFile{tail_user, consumed, true});
    return PFSCDC_OK;
  }
  rc = resolve_pending(w, base + nbytes);
  if (!rc) rc = dispatch(w, base + nbytes);
  if (rc) return rc;
  {  // the open chunk's replayed bytes move to the front of the next flush
    const uint64_t keep_from = cf.open_start;  // >= base - cl
    const uint64_t keep_to = base + consumed;
    std::vector<uint8_t> next;
    if (w->ref_ids) {
      if (keep_from < base) next.assign(w->carry.begin() + (keep_from - (base - cl)), w->carry.end());
      const uint64_t from_buf = keep_from > base ? keep_from - base : 0;
      if (keep_to > base + from_buf)
        next.insert(next.end(), w->buf.begin() + from_buf, w->buf.begin() + (keep_to - base));
    }
    w->carry.swap(next);
  }
  w->replayed = 0;
  w->deferred = false;
  if (keep_tail) {
    w->buf.erase(w->buf.begin(), w->buf.begin() + consumed);
    w->files.push_back(PendingFile{tail_user, 0, true});
  } else {
    w->buf.clear();
  }
  return PFSCDC_OK;
}

// Bytes for the current annotation: into the last pending file, or a continuation of the
// last open annotation.
int append_bytes(pfscdc_writer* w, const uint8_t* p, uint64_t n) {
  materialize(w);
  if (w->files.empty()) {
    if (w->cf.annotations.empty()) return set_err(w, PFSCDC_ESTATE);  // Go: index out of range
    w->files.push_back(PendingFile{w->cf.annotations.back().user, (uint64_t)w->buf.size(), true});
  }
  if (n) w->buf.insert(w->buf.end(), p, p + n);
  return PFSCDC_OK;
}

// DataReader.Get (reader.go) via chunk.Get on the GPU, then roll (flushDataRef, :394-401).
int flush_data_ref(pfscdc_writer* w, const pfscdc_full_dataref& dr) {
  if (!w->store) return set_err(w, PFSCDC_ESTATE);
  auto pc = w->plain.find(std::string((const char*)dr.ref.id, 32));
  if (pc != w->plain.end()) {
    if (dr.data.offset_bytes < 0 || dr.data.size_bytes < 0 ||
        (uint64_t)(dr.data.offset_bytes + dr.data.size_bytes) > pc->second.size())
      return set_err(w, PFSCDC_EINVAL);
    return append_bytes(w, (const uint8_t*)pc->second.data() + dr.data.offset_bytes,
                        (uint64_t)dr.data.size_bytes);
  }
  auto it = w->store->objects.find(std::string((const char*)dr.ref.id, 32));
  if (it == w->store->objects.end()) return set_err(w, PFSCDC_ENOTFOUND);
  const std::string& ct = it->second;
  if (dr.data.offset_bytes < 0 || dr.data.size_bytes < 0 ||
      (uint64_t)(dr.data.offset_bytes + dr.data.size_bytes) > ct.size())
    return set_err(w, PFSCDC_EINVAL);
  w->fetched.resize(ct.size() + 1);
  const uint64_t offs[2] = {0, (uint64_t)ct.size()};
  uint8_t ok = 0;
  int rc = pfscdc_get_chunks(w->ctx, ct.data(), ct.size(), 0, offs, 1, &dr.ref, w->fetched.data(),
                             0, &ok);
  if (rc) return set_err(w, rc);
  if (!ok) return set_err(w, PFSCDC_ECORRUPT);
  return append_bytes(w, w->fetched.data() + dr.data.offset_bytes, (uint64_t)dr.data.size_bytes);
}

int pending_annotate(pfscdc_writer* w, uint64_t user) {
  if (w->spans.empty() && w->buf.size() >= w->batch_bytes) {
    int rc = flush(w, kBatch);
    if (rc) return rc;
  }
  w->files.push_back(PendingFile{user, (uint64_t)(w->buf.size() + w->span_bytes), false});
  return PFSCDC_OK;
}

int flush_buffer(pfscdc_writer* w) {  // writer.go:374-392
  if (!w->buffering) return PFSCDC_OK;
  std::vector<OpenAnnotation> anns;
  anns.swap(w->cf.annotations);
  for (const OpenAnnotation& a : anns) {
    int rc = pending_annotate(w, a.user);  // Annotate(copyAnnotation(a)), not counted
    if (!rc && a.has_next) rc = flush_data_ref(w, a.next);
    if (rc) return rc;
  }
  w->buffering = false;
  return PFSCDC_OK;
}

pfscdc_full_dataref merge_data_ref(const pfscdc_full_dataref* dr1, const pfscdc_full_dataref& dr2) {
  if (!dr1) return dr2;  // writer.go:354-363
  pfscdc_full_dataref m = *dr1;
  m.data.size_bytes += dr2.data.size_bytes;
  if (m.data.size_bytes == m.ref_size) std::memcpy(m.data.hash, m.ref.id, 32);
  return m;
}

int maybe_cheap_copy(pfscdc_writer* w) {  // writer.go:403-420
  if (!w->buffering) return PFSCDC_OK;
  ChunkFormer& cf = w->cf;
  const OpenAnnotation& la = cf.annotations.back();
  if (!la.has_next) return set_err(w, PFSCDC_ESTATE);  // Go: nil NextDataRef dereference
  const pfscdc_full_dataref& last = la.next;
  if (last.data.offset_bytes + last.data.size_bytes != last.ref_size) return PFSCDC_OK;
  // the callback of a chunk that already exists: queued behind the chunks formed before it
  const bool now = cf.events.empty();
  ChunkEvent ev{};
  ev.ref.chunk_index = ~0ULL;
  ev.ref.size_bytes = last.ref_size;
  ev.ref.edge = last.edge;
  ev.ref.has_ref = 1;
  ev.ref.ref = last.ref;
  ev.ref.copied = 1;
  ev.ann_begin = cf.outs.size();
  for (const OpenAnnotation& a : cf.annotations) {
    pfscdc_annotation_out o{};
    o.user = a.user;
    if (a.has_next) {
      o.has_data_ref = 1;
      o.data_ref = a.next.data;
    }
    cf.outs.push_back(o);
    cf.out_begin.push_back(0);
    cf.out_pending.push_back(0);
  }
  ev.ann_end = cf.outs.size();
  cf.events.push_back(ev);
  const uint64_t last_user = la.user;
  cf.annotations.clear();  // splitAnnotations
  cf.annotations.push_back(OpenAnnotation{last_user, 0, {}, false, {}, cf.pos, false});
  w->buffering = false;
  return now ? callbacks(w) : PFSCDC_OK;
}

int copy_ref(pfscdc_writer* w, const pfscdc_full_dataref& dr) {  // writer.go:315-352
  ChunkFormer& cf = w->cf;
  if (cf.annotations.empty() && w->files.empty()) return set_err(w, PFSCDC_ESTATE);
  bool stale = false;  // Go merges into the pre-flush lastA, then dereferences nil
  if (w->buffering) {
    const OpenAnnotation& la = cf.annotations.back();
    if (la.has_next && la.next.data.offset_bytes != 0) {
      int rc = flush_buffer(w);
      if (rc) return rc;
      stale = true;
    }
  }
  if (!w->buffering) {
    if (dr.edge || dr.data.offset_bytes != 0) return flush_data_ref(w, dr);
    if (!w->files.empty()) {  // buf.Len() needs the pending bytes scanned
      int rc = flush(w, kPartial);
      if (rc) return rc;
    }
    if (cf.open_len != 0 || w->buf.size() > w->replayed) return flush_data_ref(w, dr);
  } else {
    const pfscdc_full_dataref* prev = nullptr;  // getPrevDataRef
    for (auto it = cf.annotations.rbegin(); it != cf.annotations.rend() && !prev; ++it)
      if (it->has_next) prev = &it->next;
    if (!prev) return set_err(w, PFSCDC_ESTATE);
    if (std::memcmp(prev->ref.id, dr.ref.id, 32) != 0 ||
        prev->data.offset_bytes + prev->data.size_bytes != dr.data.offset_bytes) {
      int rc = flush_buffer(w);
      if (rc) return rc;
      return flush_data_ref(w, dr);
    }
  }
  if (stale || cf.annotations.empty()) return set_err(w, PFSCDC_ESTATE);
  OpenAnnotation& la = cf.annotations.back();
  la.next = merge_data_ref(la.has_next ? &la.next : nullptr, dr);
  la.has_next = true;
  w->buffering = true;
  return maybe_cheap_copy(w);
}

pfscdc_writer* new_writer(pfscdc_ctx* ctx, pfscdc_writer_cb cb, void* user, uint64_t batch_bytes,
                          bool ref_ids) {
  pfscdc_writer* w = new pfscdc_writer();
  w->ctx = ctx;
  w->cb = cb;
  w->user = user;
  if (batch_bytes) w->batch_bytes = batch_bytes;
  w->ref_ids = ref_ids;
  w->cf.avg = (int64_t)1 << pfscdc::ctx_params(ctx).average_bits;  // chunkSize.avg, option.go:52
  return w;
}

}  // namespace

namespace pfscdc {

// Close several writers of one ctx with one scan and one chunk.Create pass, equivalent to
// pfscdc_writer_close on each in order (their chunk streams are independent).  Only for
// writers that never flushed and buffer no Copy (each fileset's data writer at Close);
// anything else closes one by one.  Batching keeps enough BLAKE2b chains in flight: one
// 1e9-byte fileset of ~10 MB files has ~100 chains, far below the ~32K the GPU holds.
int writers_close_group(pfscdc_writer* const* ws, size_t n, double* stage_ms,
                        const hipEvent_t* wait_events, size_t n_wait) {
  if (n == 0) return PFSCDC_OK;
  pfscdc_ctx* ctx = ws[0]->ctx;
  // a lone writer takes the grouped path too: its pieces and multi-piece chunks still share
  // one hash launch (pfscdc_writer_close runs them as two passes)
  bool group = true;
  for (size_t i = 0; i < n && group; i++) {
    const pfscdc_writer* w = ws[i];
    group = !w->err && !w->closed && w->ctx == ctx && !w->buffering && w->carry.empty() &&
            w->d_cap == 0 && w->replayed == 0 && !w->deferred && w->cf.events.empty() &&
            w->ref_ids == ws[0]->ref_ids &&
            (w->upload && w->store) == (ws[0]->upload && ws[0]->store);
  }
  if (!group) {
    for (size_t i = 0; i < n; i++) {
      int rc = pfscdc_writer_close(ws[i]);
      if (rc) return rc;
    }
    return PFSCDC_OK;
  }
  const bool trace = knob(Knob::Trace) != 0;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  const auto t0 = now();
  // layout: writer i's pending bytes at base[i] (16-B aligned); the alignment gaps are
  // dummy files whose segments are ignored
  std::vector<uint64_t> base(n), offsets;
  std::vector<size_t> first(n);
  uint64_t pos = 0;
  for (size_t i = 0; i < n; i++) {
    const uint64_t b = (pos + 15) & ~15ULL;
    if (b > pos) offsets.push_back(pos);
    base[i] = b;
    first[i] = offsets.size();
    for (const PendingFile& f : ws[i]->files) offsets.push_back(b + f.begin);
    pos = b + ws[i]->buf.size() + ws[i]->span_bytes;
  }
  const uint64_t total = pos;
  const uint32_t nfiles = (uint32_t)offsets.size();
  offsets.push_back(total);
  uint8_t *d = nullptr, *dct = nullptr;
  const bool up = ws[0]->upload && ws[0]->store;
  int rc = PFSCDC_OK;
  // the ctx's grow-only staging: a commit closes many groups, and a fresh hipMalloc/hipFree
  // of up to the group's size per close would dominate small groups
  if (hipSetDevice(ctx_device(ctx)) != hipSuccess ||
      ctx_group_buffers(ctx, total + 64, up, &d, &dct) != hipSuccess)
    rc = PFSCDC_ENOMEM;
  // the upload: every writer's bytes (the spans straight from the page-locked Put arenas)
  // queued on the ctx stream, which the scan then follows; no host wait in between
  hipStream_t st = (hipStream_t)pfscdc_stream_handle(ctx);
  // spans whose bytes were uploaded during the Puts (the caller's events mark them landed)
  // are gathered device to device; the rest come from host memory
  for (size_t e = 0; e < n_wait && !rc; e++)
    if (hipStreamWaitEvent(st, wait_events[e], 0) != hipSuccess) rc = PFSCDC_EHIP;
  for (size_t i = 0; i < n && !rc; i++) {
    const pfscdc_writer* w = ws[i];
    uint64_t at = base[i];
    if (!w->buf.empty() &&
        hipMemcpyAsync(d + at, w->buf.data(), w->buf.size(), hipMemcpyHostToDevice, st) != hipSuccess)
      rc = PFSCDC_EHIP;
    at += w->buf.size();
    for (size_t k = 0; k < w->spans.size() && !rc; k++) {
      const auto& sp = w->spans[k];
      const uint8_t* dv = k < w->span_dev.size() ? w->span_dev[k] : nullptr;
      if (sp.second &&
          hipMemcpyAsync(d + at, dv ? dv : sp.first, sp.second,
                         dv ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, st) != hipSuccess)
        rc = PFSCDC_EHIP;
      at += sp.second;
    }
  }
  if (!rc && trace && hipStreamSynchronize(st) != hipSuccess) rc = PFSCDC_EHIP;  // exact stages
  // the Puts' uploads into the arena mirrors landed: the upload stage ends there, so the scan
  // stage is the scan's own (the scan would wait for them on the stream anyway)
  for (size_t e = 0; e < n_wait && !rc; e++)
    if (hipEventSynchronize(wait_events[e]) != hipSuccess) rc = PFSCDC_EHIP;
  const auto t1 = now();
  // cut positions only: the DataRef hashes join the chunk content hashes in one launch below
  // (the commit data plane's pfscdc_commit_refs order), so their two sets of serial BLAKE2b
  // chains share the GPU instead of running one pass after the other
  const bool ids = ws[0]->ref_ids;
  if (!rc && nfiles) rc = scan_sync(ctx, d, total, 1, offsets.data(), nfiles, ids ? kScanNoHash : 0);
  const auto t2 = now();
  // replay every writer over its own files (piece hashes pending when the scan had none)
  if (!rc) {
    const pfscdc_segment* segs = pfscdc_segments(ctx);
    const uint64_t* begin = pfscdc_file_segment_begin(ctx);
    for (size_t i = 0; i < n; i++) {
      pfscdc_writer* w = ws[i];
      ChunkFormer& cf = w->cf;
      cf.open_start = cf.pos = base[i];
      for (size_t k = 0; k < w->files.size(); k++) {
        const size_t g = first[i] + k;
        if (!w->files[k].cont) cf.annotate(w->files[k].user);
        for (uint64_t s = begin[g]; s < begin[g + 1]; s++) cf.piece(segs[s], ids);
      }
      cf.close();
    }
  }
  const auto t3 = now();
  // every piece (DataRef.Hash, writer.go:301-312) and every multi-DataRef chunk (the content
  // hash, writer.go:240) in one LPT-ordered launch; a one-piece chunk's hash is its piece's
  if (!rc && ids) {
    std::vector<uint64_t> begins, sizes;
    std::vector<std::pair<size_t, size_t>> who;  // (writer, out) or (writer, ~event)
    for (size_t i = 0; i < n; i++) {
      const ChunkFormer& cf = ws[i]->cf;
      for (size_t o = 0; o < cf.outs.size(); o++)
        if (cf.out_pending[o]) {
          begins.push_back(cf.out_begin[o]);
          sizes.push_back((uint64_t)cf.outs[o].data_ref.size_bytes);
          who.emplace_back(i, o);
        }
      for (size_t e = 0; e < cf.events.size(); e++)
        if (!cf.events[e].known) {
          begins.push_back(cf.events[e].begin);
          sizes.push_back(cf.events[e].end - cf.events[e].begin);
          who.emplace_back(i, ~e);
        }
    }
    std::vector<uint8_t> h(32 * who.size());
    if (!who.empty())
      rc = hash_records_device(ctx, d, total, begins.data(), sizes.data(), (uint32_t)who.size(),
                               h.data());
    for (size_t k = 0; k < who.size() && !rc; k++) {
      ChunkFormer& cf = ws[who[k].first]->cf;
      const size_t x = who[k].second;
      if ((intptr_t)x >= 0) {
        std::memcpy(cf.outs[x].data_ref.hash, h.data() + 32 * k, 32);
        cf.out_pending[x] = 0;
      } else {
        std::memcpy(cf.events[~x].hash, h.data() + 32 * k, 32);
      }
    }
    for (size_t i = 0; i < n && !rc; i++) {
      ChunkFormer& cf = ws[i]->cf;
      for (ChunkEvent& ev : cf.events) {
        if (ev.known)  // one piece: its hash (the unknown ones were hashed above)
          for (size_t o = ev.ann_begin; o < ev.ann_end; o++)
            if (cf.outs[o].has_data_ref) std::memcpy(ev.hash, cf.outs[o].data_ref.hash, 32);
        ev.known = 1;  // every chunk's content hash is now known
      }
    }
  }
  const auto t4 = now();
  // one chunk.Create (dek + Ref.Id) over every writer's chunks (gaps between writers are dummy
  // records)
  if (!rc && ids) {
    std::vector<uint64_t> coffs;
    std::vector<uint8_t> hashes, known;
    std::vector<std::pair<size_t, size_t>> who;  // record -> (writer, event), or gap
    uint64_t at = 0;
    for (size_t i = 0; i < n; i++) {
      for (size_t e = 0; e < ws[i]->cf.events.size(); e++) {
        const ChunkEvent& ev = ws[i]->cf.events[e];
        if (ev.begin > at) {  // gap
          coffs.push_back(at);
          known.push_back(1);
          hashes.resize(hashes.size() + 32, 0);
          who.emplace_back(SIZE_MAX, 0);
        }
        coffs.push_back(ev.begin);
        known.push_back(ev.known);
        hashes.insert(hashes.end(), ev.hash, ev.hash + 32);
        who.emplace_back(i, e);
        at = ev.end;
      }
      ws[i]->refs.resize(ws[i]->cf.events.size());
    }
    coffs.push_back(at);
    const uint32_t nrec = (uint32_t)who.size();
    std::vector<pfscdc_ref> refs(nrec);
    if (nrec)
      rc = create_refs_device(ctx, d, total, coffs.data(), nrec, hashes.data(), known.data(),
                              refs.data(), dct);
    for (uint32_t r = 0; r < nrec && !rc; r++) {
      if (who[r].first == SIZE_MAX) continue;
      pfscdc_writer* w = ws[who[r].first];
      w->refs[who[r].second] = refs[r];
      if (up) rc = upload(w->store, refs[r], dct, coffs[r], coffs[r + 1]);
    }
  }
  const auto t5 = now();
  for (size_t i = 0; i < n; i++) {
    pfscdc_writer* w = ws[i];
    w->closed = true;
    w->files.clear();
    w->buf.clear();
    w->buf.shrink_to_fit();
    w->spans.clear();
    w->span_dev.clear();
    w->span_bytes = 0;
    if (rc) {
      clear_events(w->cf);
      set_err(w, rc);
      continue;
    }
    int r2 = callbacks(w);
    if (r2 && !rc) rc = r2;
  }
  const auto t6 = now();
  // stages (ms): upload queued (with PFSCDC_TRACE: landed), scan (incl. the upload when not
  // traced), replay, hashes, chunk.Create, callbacks
  const double stages[6] = {ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, t5), ms(t5, t6)};
  if (stage_ms)
    for (int k = 0; k < 6; k++) stage_ms[k] += stages[k];
  if (trace)
    fprintf(stderr, "[pfscdc] close_group n=%zu bytes=%lu upload %.1f ms scan %.1f replay %.1f "
            "hashes %.1f create %.1f callbacks %.1f\n", n, (unsigned long)total, stages[0],
            stages[1], stages[2], stages[3], stages[4], stages[5]);
  return rc;
}

// Write of n caller-owned bytes kept until the writer flushes (no copy).
int writer_write_span(pfscdc_writer* w, const uint8_t* p, uint64_t n, const uint8_t* dev) {
  if (w->err) return w->err;
  if (w->closed || w->buffering || w->files.empty())
    return pfscdc_writer_write(w, p, n);  // anything unusual: the copying path
  if (n) {
    w->spans.emplace_back(p, n);
    w->span_dev.resize(w->spans.size() - 1, nullptr);
    w->span_dev.push_back(dev);
    w->span_bytes += n;
  }
  return PFSCDC_OK;
}

}  // namespace pfscdc

extern "C" {

int pfscdc_writer_create(pfscdc_ctx* ctx, pfscdc_writer_cb cb, void* user, uint64_t batch_bytes,
                         pfscdc_writer** out) {
  if (!ctx || !out) return PFSCDC_EINVAL;
  *out = new_writer(ctx, cb, user, batch_bytes,
                    (pfscdc::ctx_options(ctx) & PFSCDC_OPT_REF_IDS) != 0);
  return PFSCDC_OK;
}

int pfscdc_writer_set_store(pfscdc_writer* w, pfscdc_store* store, int upload) {
  if (!w || (upload && !w->ref_ids)) return PFSCDC_EINVAL;
  if (w->d_cap) return PFSCDC_ESTATE;  // before the first flush
  w->store = store;
  w->upload = upload != 0 && store;
  return PFSCDC_OK;
}

int pfscdc_writer_annotate(pfscdc_writer* w, uint64_t user) {
  if (!w) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return set_err(w, PFSCDC_ESTATE);
  w->annotation_count++;
  if (w->buffering) {  // Annotate does not flush the buffer; the open chunk is empty
    w->cf.annotations.push_back(OpenAnnotation{user, 0, {}, false, {}});
    return PFSCDC_OK;
  }
  return pending_annotate(w, user);
}

int pfscdc_writer_write(pfscdc_writer* w, const void* data, uint64_t n) {
  if (!w) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed || (w->files.empty() && w->cf.annotations.empty()))
    return set_err(w, PFSCDC_ESTATE);  // Go: panics
  if (n && !data) return set_err(w, PFSCDC_EINVAL);
  int rc = flush_buffer(w);
  if (rc) return rc;
  return append_bytes(w, (const uint8_t*)data, n);
}

int pfscdc_writer_prefetch(pfscdc_writer* w, const pfscdc_full_dataref* drs, uint32_t n) {
  // chunk.Get of every chunk these DataRefs will certainly be re-rolled from (edge chunks and
  // DataRefs not starting at a chunk's first byte: maybeBufferDataRef never buffers them), in
  // one batch: their BLAKE2b verifications run as parallel chains instead of one by one
  if (!w || (n && !drs)) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (!w->store) return PFSCDC_OK;
  std::vector<std::string> ids;
  std::vector<pfscdc_ref> refs;
  std::vector<uint64_t> offs{0};
  std::string ct;
  for (uint32_t i = 0; i < n; i++) {
    const pfscdc_full_dataref& d = drs[i];
    if (!d.edge && d.data.offset_bytes == 0) continue;
    std::string id((const char*)d.ref.id, 32);
    if (w->plain.count(id) || std::find(ids.begin(), ids.end(), id) != ids.end()) continue;
    auto it = w->store->objects.find(id);
    if (it == w->store->objects.end()) continue;  // reported by the Copy that needs it
    ids.push_back(id);
    refs.push_back(d.ref);
    ct += it->second;
    offs.push_back(ct.size());
  }
  if (ids.empty()) return PFSCDC_OK;
  std::vector<uint8_t> pt(ct.size() + 1), ok(ids.size());
  int rc = pfscdc_get_chunks(w->ctx, ct.data(), ct.size(), 0, offs.data(), (uint32_t)ids.size(),
                             refs.data(), pt.data(), 0, ok.data());
  if (rc) return set_err(w, rc);
  for (size_t i = 0; i < ids.size(); i++)  // a chunk failing verification stays uncached
    if (ok[i]) w->plain.emplace(ids[i], std::string((const char*)pt.data() + offs[i], offs[i + 1] - offs[i]));
  return PFSCDC_OK;
}

int pfscdc_writer_copy(pfscdc_writer* w, const pfscdc_full_dataref* dr) {
  if (!w || !dr) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return set_err(w, PFSCDC_ESTATE);
  return copy_ref(w, *dr);
}

int pfscdc_writer_close(pfscdc_writer* w) {
  if (!w) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return PFSCDC_OK;
  int rc = flush_buffer(w);
  if (rc) return rc;
  w->closed = true;
  return flush(w, kFinal);
}

int64_t pfscdc_writer_chunk_count(const pfscdc_writer* w) { return w ? w->cf.chunk_count : 0; }
int64_t pfscdc_writer_annotation_count(const pfscdc_writer* w) {
  return w ? w->annotation_count : 0;
}

int pfscdc_writer_destroy(pfscdc_writer* w) {
  if (!w) return PFSCDC_EINVAL;
  if (w->d_buf) (void)hipFree(w->d_buf);
  if (w->d_ctext) (void)hipFree(w->d_ctext);
  delete w;
  return PFSCDC_OK;
}

int pfscdc_store_create(pfscdc_store** out) {
  if (!out) return PFSCDC_EINVAL;
  *out = new pfscdc_store();
  return PFSCDC_OK;
}

int pfscdc_store_destroy(pfscdc_store* s) {
  delete s;
  return PFSCDC_OK;
}

int pfscdc_store_put(pfscdc_store* s, const uint8_t id[32], const void* ctext, uint64_t n) {
  if (!s || !id || (n && !ctext)) return PFSCDC_EINVAL;
  s->objects.emplace(std::string((const char*)id, 32), std::string((const char*)ctext, n));
  return PFSCDC_OK;
}

int pfscdc_store_get(const pfscdc_store* s, const uint8_t id[32], const void** ctext,
                     uint64_t* n) {
  if (!s || !id || !ctext || !n) return PFSCDC_EINVAL;
  auto it = s->objects.find(std::string((const char*)id, 32));
  if (it == s->objects.end()) return PFSCDC_ENOTFOUND;
  *ctext = it->second.data();
  *n = it->second.size();
  return PFSCDC_OK;
}

uint64_t pfscdc_store_count(const pfscdc_store* s) { return s ? s->objects.size() : 0; }

int pfscdc_merge_file_hash(pfscdc_ctx* ctx, pfscdc_store* store, const pfscdc_full_dataref* drs,
                           uint32_t n, uint8_t out[32]) {
  if (!ctx || !store || !out || (n && !drs)) return PFSCDC_EINVAL;
  std::vector<uint8_t> resolved;  // the hashes of annotations[0].NextDataRef per callback
  auto cb = [](void* user, const pfscdc_chunk_ref*, const pfscdc_annotation_out* a,
               uint32_t na) -> int {
    if (na && a[0].has_data_ref) {
      auto* r = (std::vector<uint8_t>*)user;
      r->insert(r->end(), a[0].data_ref.hash, a[0].data_ref.hash + 32);
    }
    return 0;
  };
  // WithNoUpload: the new chunks' ids never reach the result, so no Ref pass is run
  pfscdc_writer* w = new_writer(ctx, cb, &resolved, 0, false);
  w->store = store;
  int rc = pfscdc_writer_prefetch(w, drs, n);
  if (!rc) rc = pfscdc_writer_annotate(w, 0);
  for (uint32_t i = 0; i < n && !rc; i++) rc = pfscdc_writer_copy(w, &drs[i]);
  if (!rc) rc = pfscdc_writer_close(w);
  pfscdc_writer_destroy(w);
  if (rc) return rc;
  return pfscdc_hash_data_refs(ctx, resolved.data(), (uint32_t)(resolved.size() / 32), out);
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
