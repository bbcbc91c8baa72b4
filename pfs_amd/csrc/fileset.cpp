// fileset.cpp — pachd-level stream formation over the GPU chunk writer (host logic).
//
// Reference (paths under /root/reference/src/internal/storage):
//   fileset/unordered_writer.go:45-179  UnorderedWriter: Put (io.CopyN against memAvailable,
//                                        serialize at 0), Delete (files; directories over the
//                                        merged view of what was serialized), Close
//   fileset/buffer.go:10-106            Buffer (additive/deletive, sorted by path then tag)
//   fileset/merge.go:37-78,157-164      merged (path, tag) view used by directory deletes
//   fileset/writer.go:36-182            fileset.Writer: Add, Delete, callback, Close
//   fileset/index/writer.go:12-162      multilevel index.Writer (level k: avgBits 20, seed k)
//   fileset/util.go:67-88               Clean / IsDir (Go path.Clean)
//   pbutil/pbutil.go:64-80              int64 LE length-prefixed protos
//   chunk/chunk.proto, fileset/index/index.proto, chunk/util.go:25-30 (Reference)
// Every chunk stream (the data writer of a serialized fileset and each index level) is a
// pfscdc_writer: CDC, BLAKE2b and chunk.Create run on the GPU; this file is the bookkeeping.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "pfscdc_internal.h"

namespace {

// ---------------------------------------------------------------- protobuf (proto3) encoder

struct RefT {
  uint8_t id[32];
  int64_t size;
  bool edge;
  uint8_t dek[32];
};

struct DataRefT {
  RefT ref;
  uint8_t hash[32];
  int64_t offset, size;
};

struct IndexT {
  std::string path;
  bool has_range = false;
  int64_t range_offset = 0;
  std::string range_last_path;
  RefT range_ref{};
  std::string tag;  // File is always set on this path (fileset.Writer.Add / Delete)
  std::vector<DataRefT> data_refs;
};

void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
void put_key(std::string& o, int field, int wire) { put_varint(o, (uint64_t)(field << 3 | wire)); }
void put_bytes(std::string& o, int field, const void* p, size_t n) {
  if (!n) return;  // proto3: empty bytes/strings are not emitted
  put_key(o, field, 2);
  put_varint(o, n);
  o.append((const char*)p, n);
}
void put_int(std::string& o, int field, int64_t v) {
  if (!v) return;
  put_key(o, field, 0);
  put_varint(o, (uint64_t)v);
}
void put_msg(std::string& o, int field, const std::string& m) {  // set messages: always emitted
  put_key(o, field, 2);
  put_varint(o, m.size());
  o += m;
}

// chunk.Ref as chunk.Create + processChunk leave it: EncryptionAlgo CHACHA20 (1),
// CompressionAlgo NONE (0, not emitted)
std::string enc_ref(const RefT& r) {
  std::string o;
  put_bytes(o, 1, r.id, 32);
  put_int(o, 2, r.size);
  put_int(o, 3, r.edge ? 1 : 0);
  put_bytes(o, 4, r.dek, 32);
  put_int(o, 5, 1);
  return o;
}

std::string enc_dataref(const RefT& r, const uint8_t* hash, int64_t offset, int64_t size) {
  std::string o;
  put_msg(o, 1, enc_ref(r));
  if (hash) put_bytes(o, 2, hash, 32);
  put_int(o, 3, offset);
  put_int(o, 4, size);
  return o;
}

std::string enc_index(const IndexT& x) {
  std::string o;
  put_bytes(o, 1, x.path.data(), x.path.size());
  if (x.has_range) {
    std::string r;
    put_int(r, 1, x.range_offset);
    put_bytes(r, 2, x.range_last_path.data(), x.range_last_path.size());
    // chunk.Reference(dataRef) = {Ref, SizeBytes: Ref.SizeBytes}
    put_msg(r, 3, enc_dataref(x.range_ref, nullptr, 0, x.range_ref.size));
    put_msg(o, 2, r);
  }
  std::string f;
  put_bytes(f, 1, x.tag.data(), x.tag.size());
  for (const DataRefT& d : x.data_refs) put_msg(f, 2, enc_dataref(d.ref, d.hash, d.offset, d.size));
  put_msg(o, 3, f);
  return o;
}

std::string frame(const std::string& m) {  // pbutil WriteBytes
  std::string o(8, '\0');
  const uint64_t n = m.size();
  for (int i = 0; i < 8; i++) o[i] = (char)(n >> (8 * i));
  return o + m;
}

RefT ref_of(const pfscdc_chunk_ref* c) {
  RefT r{};
  std::memcpy(r.id, c->ref.id, 32);
  std::memcpy(r.dek, c->ref.dek, 32);
  r.size = c->size_bytes;
  r.edge = c->edge != 0;
  return r;
}

// ---------------------------------------------------------------- paths (Go path.Clean)

std::string go_path_clean(const std::string& p) {
  if (p.empty()) return ".";
  const bool rooted = p[0] == '/';
  const size_t n = p.size();
  std::string out;
  size_t r = 0, dotdot = 0;
  if (rooted) {
    out.push_back('/');
    r = dotdot = 1;
  }
  while (r < n) {
    if (p[r] == '/') {
      r++;
    } else if (p[r] == '.' && (r + 1 == n || p[r + 1] == '/')) {
      r++;
    } else if (p[r] == '.' && r + 1 < n && p[r + 1] == '.' && (r + 2 == n || p[r + 2] == '/')) {
      r += 2;
      if (out.size() > dotdot) {
        size_t w = out.size() - 1;
        while (w > dotdot && out[w] != '/') w--;
        out.resize(w);
      } else if (!rooted) {
        if (!out.empty()) out.push_back('/');
        out += "..";
        dotdot = out.size();
      }
    } else {
      if ((rooted && out.size() != 1) || (!rooted && !out.empty())) out.push_back('/');
      for (; r < n && p[r] != '/'; r++) out.push_back(p[r]);
    }
  }
  return out.empty() ? "." : out;
}

bool is_dir(const std::string& p) { return !p.empty() && p.back() == '/'; }

std::string clean(const std::string& p0, bool dir) {  // fileset/util.go:67-77
  std::string p = go_path_clean(p0);
  if (p == ".") return "/";
  size_t a = 0, b = p.size();
  while (a < b && p[a] == '/') a++;
  while (b > a && p[b - 1] == '/') b--;
  std::string y = "/" + p.substr(a, b - a);
  if (dir && !is_dir(y)) y += "/";
  return y;
}

}  // namespace

// ---------------------------------------------------------------- writers

struct pfscdc_uwriter;

namespace {

// Contexts the writers make for themselves (a second group writer's data ctx, one ctx per
// index level) are kept for the next writer: a ctx owns its stream, events and grow-only
// device staging (a group write's whole input), so making them per commit costs more than
// the commit's small index streams.  Keyed by (device, params, options); at most the
// PFSCDC_CTX_CACHE knob's count of them (default 32; 0 turns the cache off).
struct CtxCache {
  std::mutex mu;
  std::vector<std::pair<std::string, pfscdc_ctx*>> free;
  static std::string key(const pfscdc_params& p, int device, uint32_t options) {
    char b[160];
    snprintf(b, sizeof b, "%d/%u/%lld/%lld/%lld/%u", device, p.average_bits, (long long)p.seed,
             (long long)p.min_chunk, (long long)p.max_chunk, options);
    return b;
  }
  pfscdc_ctx* take(const pfscdc_params& p, int device, uint32_t options) {
    const std::string k = key(p, device, options);
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = free.size(); i-- > 0;)
        if (free[i].first == k) {
          pfscdc_ctx* c = free[i].second;
          free.erase(free.begin() + (ptrdiff_t)i);
          return c;
        }
    }
    pfscdc_ctx* c = nullptr;
    if (pfscdc_ctx_create(&p, device, &c) != PFSCDC_OK) return nullptr;
    if (pfscdc_set_options(c, options) != PFSCDC_OK) {
      pfscdc_ctx_destroy(c);
      return nullptr;
    }
    return c;
  }
  // Destroy the cached contexts of one device (-1: all): their streams, events and grow-only
  // device staging (a group write's whole input and ciphertext).
  uint32_t trim(int device) {
    std::vector<pfscdc_ctx*> out;
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = free.size(); i-- > 0;)
        if (device < 0 || pfscdc::ctx_device(free[i].second) == device) {
          out.push_back(free[i].second);
          free.erase(free.begin() + (ptrdiff_t)i);
        }
    }
    for (pfscdc_ctx* c : out) pfscdc_ctx_destroy(c);
    return (uint32_t)out.size();
  }
  void give(pfscdc_ctx* c) {
    if (!c) return;
    std::unique_lock<std::mutex> lk(mu);
    if (free.size() < (size_t)pfscdc::knob(pfscdc::Knob::CtxCache)) {
      free.emplace_back(key(pfscdc::ctx_params(c), pfscdc::ctx_device(c), pfscdc::ctx_options(c)), c);
      return;
    }
    lk.unlock();
    pfscdc_ctx_destroy(c);
  }
};
CtxCache& ctx_cache() {
  static CtxCache* p = new CtxCache();  // never destroyed: no HIP calls in static dtors
  return *p;
}

struct Streams {  // the ctxs of every chunk stream kind; events out
  pfscdc_ctx* data_ctx = nullptr;
  bool own_data_ctx = false;  // a second group writer's ctx (same params, options, device)
  pfscdc_params index_params{};
  std::map<int64_t, pfscdc_ctx*> index_ctx;  // by seed (= level)
  pfscdc_uw_cb cb = nullptr;
  void* user = nullptr;
  std::mutex* emit_mu = nullptr;  // events of concurrent group writers reach cb one at a time
  // several group writers: a group's events are held here (the index frames copied) and
  // released in group order once the groups before it have emitted theirs
  std::vector<std::pair<pfscdc_uw_event, std::string>>* hold = nullptr;
  int err = 0;

  int emit(pfscdc_uw_event& ev, uint32_t fileset) {
    ev.fileset = fileset;
    if (!cb) return PFSCDC_OK;
    if (hold) {
      hold->emplace_back(ev, ev.kind == PFSCDC_EV_INDEX
                                 ? std::string((const char*)ev.bytes, (size_t)ev.len)
                                 : std::string());
      return PFSCDC_OK;
    }
    std::unique_lock<std::mutex> lk;
    if (emit_mu) lk = std::unique_lock<std::mutex>(*emit_mu);
    return cb(user, &ev) != 0 ? PFSCDC_ECALLBACK : PFSCDC_OK;
  }
  pfscdc_ctx* level_ctx(int level) {
    auto it = index_ctx.find(level);
    if (it != index_ctx.end()) return it->second;
    pfscdc_params p = index_params;
    p.seed = index_params.seed + level;
    pfscdc_ctx* c = ctx_cache().take(p, pfscdc::ctx_device(data_ctx), PFSCDC_OPT_REF_IDS);
    if (!c) return nullptr;
    index_ctx[level] = c;
    return c;
  }
  ~Streams() {
    for (auto& kv : index_ctx) ctx_cache().give(kv.second);
    if (own_data_ctx) ctx_cache().give(data_ctx);
  }
};

struct IndexWriter;
constexpr int kMaxIndexLevels = 32;

struct Span {  // bytes [off, off + len) of a fileset's Put arena
  uint64_t off, len;
};

struct Level {
  IndexWriter* iw;
  int level;
  pfscdc_writer* cw = nullptr;
  IndexT* last = nullptr;
};

struct IndexWriter {  // index/writer.go:27-162
  Streams* st;
  int which;  // 0 additive, 1 deletive
  std::vector<std::unique_ptr<Level>> levels;
  bool closed = false;
  IndexT* root = nullptr;
  std::vector<std::unique_ptr<IndexT>>* pool;
  uint32_t fs = 0;  // serialized fileset number (events)

  ~IndexWriter() {
    for (auto& l : levels)
      if (l->cw) pfscdc_writer_destroy(l->cw);
  }

  int new_level() {
    const int k = (int)levels.size();
    pfscdc_ctx* c = st->level_ctx(k);
    if (!c) return PFSCDC_EHIP;
    auto l = std::make_unique<Level>();
    l->iw = this;
    l->level = k;
    int rc = pfscdc_writer_create(c, &IndexWriter::callback, l.get(), 0, &l->cw);
    if (rc) return rc;
    levels.push_back(std::move(l));
    return PFSCDC_OK;
  }

  int write_index(IndexT* idx, int level) {
    if (levels.empty()) {
      int rc = new_level();
      if (rc) return rc;
    }
    const std::string b = frame(enc_index(*idx));
    if (level == 0) {
      pfscdc_uw_event ev{};
      ev.kind = PFSCDC_EV_INDEX;
      ev.index = which;
      ev.bytes = (const uint8_t*)b.data();
      ev.len = b.size();
      int rc = st->emit(ev, fs);
      if (rc) return rc;
    }
    pfscdc_writer* cw = levels[level]->cw;
    int rc = pfscdc_writer_annotate(cw, (uint64_t)(uintptr_t)idx);
    if (!rc) rc = pfscdc_writer_write(cw, b.data(), b.size());
    return rc;
  }

  static int callback(void* user, const pfscdc_chunk_ref* chunk, const pfscdc_annotation_out* a,
                      uint32_t n) {
    Level* lw = (Level*)user;
    IndexWriter* w = lw->iw;
    pfscdc_uw_event ev{};
    ev.kind = PFSCDC_EV_CHUNK;
    ev.index = w->which;
    ev.level = lw->level;
    ev.chunk = *chunk;
    int rc = w->st->emit(ev, w->fs);
    if (rc || n == 0) return rc;
    IndexT* idx = (IndexT*)(uintptr_t)a[0].user;
    const pfscdc_annotation_out* dr = &a[0];
    if (n > 1 && lw->last && idx->path == lw->last->path) {  // started in the previous chunk
      idx = (IndexT*)(uintptr_t)a[1].user;
      dr = &a[1];
    }
    lw->last = (IndexT*)(uintptr_t)a[n - 1].user;
    const std::string last_path = lw->last->has_range ? lw->last->range_last_path : lw->last->path;
    if (!dr->has_data_ref) return PFSCDC_ESTATE;  // Go dereferences a nil NextDataRef here
    idx->has_range = true;
    idx->range_offset = dr->data_ref.offset_bytes;
    idx->range_last_path = last_path;
    idx->range_ref = ref_of(chunk);
    if (w->closed) w->root = idx;
    const int level = lw->level;  // lw stays valid: levels hold unique_ptrs
    if (level == (int)w->levels.size() - 1) {
      // an entry >= the index avg is cut before at every level and the levels never
      // converge (Go keeps adding levels); the reference's 1 MiB avg rules that out
      if (level + 1 >= kMaxIndexLevels) return PFSCDC_EUNSUPPORTED;
      rc = w->new_level();
      if (rc) return rc;
    }
    return w->write_index(idx, level + 1);
  }

  int close(IndexT** out) {
    closed = true;
    for (size_t i = 0; i < levels.size(); i++) {
      pfscdc_writer* cw = levels[i]->cw;
      int rc = pfscdc_writer_close(cw);
      if (rc) return rc;
      if (pfscdc_writer_annotation_count(cw) == 1 && pfscdc_writer_chunk_count(cw) == 1) break;
    }
    *out = root;
    return PFSCDC_OK;
  }
};

struct FilesetInfo {
  int64_t size_bytes = 0;
  std::string additive, deletive;  // encoded root Index
  bool has_additive = false, has_deletive = false;
  std::vector<std::pair<std::string, std::string>> files, deletes;  // (path, tag) in order
};

struct FilesetWriter {  // fileset/writer.go:21-182
  Streams* st;
  std::vector<std::unique_ptr<IndexT>> pool;
  IndexWriter additive, deletive;
  pfscdc_writer* cw = nullptr;
  IndexT *idx = nullptr, *delete_idx = nullptr, *last_idx = nullptr;
  FilesetInfo info;
  uint32_t fs;
  int err = 0;

  FilesetWriter(Streams* s, uint32_t fileset) : st(s), additive{s, 0, {}, false, nullptr, &pool},
                                                deletive{s, 1, {}, false, nullptr, &pool},
                                                fs(fileset) {
    additive.fs = deletive.fs = fileset;
  }
  ~FilesetWriter() {
    if (cw) pfscdc_writer_destroy(cw);
  }

  int open() { return pfscdc_writer_create(st->data_ctx, &FilesetWriter::callback, this, 0, &cw); }

  static int check_path(const IndexT* prev, const IndexT* idx) {
    if (!prev) return PFSCDC_OK;
    if (prev->path == idx->path && prev->tag == idx->tag) return PFSCDC_EINVAL;  // same path twice
    if (prev->path > idx->path) return PFSCDC_EINVAL;                            // out of order
    return PFSCDC_OK;
  }

  IndexT* make(const std::string& path, const std::string& tag) {
    pool.push_back(std::make_unique<IndexT>());
    pool.back()->path = path;
    pool.back()->tag = tag;
    return pool.back().get();
  }

  // Add(path, tag, r) with r = the concatenation of spans of base (kept alive by the caller
  // until the data writer closes)
  int add(const std::string& path, const std::string& tag, const uint8_t* base,
          const std::vector<Span>& spans, const uint8_t* dev_base = nullptr) {
    IndexT* x = make(path, tag);
    int rc = check_path(idx, x);
    if (rc) return rc;
    idx = x;
    info.files.emplace_back(path, tag);
    rc = pfscdc_writer_annotate(cw, (uint64_t)(uintptr_t)x);
    for (const Span& sp : spans) {
      if (!rc) rc = pfscdc::writer_write_span(cw, base + sp.off, sp.len,
                                              dev_base ? dev_base + sp.off : nullptr);
      info.size_bytes += (int64_t)sp.len;
    }
    return rc;
  }

  int del(const std::string& path, const std::string& tag) {
    IndexT* x = make(path, tag);
    int rc = check_path(delete_idx, x);
    if (rc) return rc;
    delete_idx = x;
    info.deletes.emplace_back(path, tag);
    return deletive.write_index(x, 0);
  }

  static int callback(void* user, const pfscdc_chunk_ref* chunk, const pfscdc_annotation_out* a,
                      uint32_t n) {
    FilesetWriter* w = (FilesetWriter*)user;
    pfscdc_uw_event ev{};
    ev.kind = PFSCDC_EV_CHUNK;
    ev.index = -1;
    ev.chunk = *chunk;
    int rc = w->st->emit(ev, w->fs);
    if (rc) return rc;
    const RefT ref = ref_of(chunk);
    for (uint32_t i = 0; i < n; i++) {
      IndexT* x = (IndexT*)(uintptr_t)a[i].user;
      if (!w->last_idx) w->last_idx = x;
      if (x->path != w->last_idx->path || x->tag != w->last_idx->tag) {
        rc = w->additive.write_index(w->last_idx, 0);
        if (rc) return rc;
        w->last_idx = x;
      }
      if (a[i].has_data_ref) {
        DataRefT d{};
        d.ref = ref;
        std::memcpy(d.hash, a[i].data_ref.hash, 32);
        d.offset = a[i].data_ref.offset_bytes;
        d.size = a[i].data_ref.size_bytes;
        w->last_idx->data_refs.push_back(d);
      }
    }
    return PFSCDC_OK;
  }

  int close() {
    int rc = pfscdc_writer_close(cw);
    return rc ? rc : finish();
  }

  int finish() {  // Close after the data writer closed: the last entry, then the indexes
    int rc = finish_last_entry();
    IndexT *a = nullptr, *d = nullptr;
    if (!rc) rc = additive.close(&a);
    if (!rc) rc = deletive.close(&d);
    if (rc) return rc;
    finish_info(a, d);
    return PFSCDC_OK;
  }
  int finish_last_entry() {  // the additive index entry of the last file (writer.go:151-167)
    return last_idx ? additive.write_index(last_idx, 0) : PFSCDC_OK;
  }
  void finish_info(IndexT* a, IndexT* d) {  // the roots of the closed indexes
    if (a) {
      info.has_additive = true;
      info.additive = enc_index(*a);
    }
    if (d) {
      info.has_deletive = true;
      info.deletive = enc_index(*d);
    }
  }
};

// IndexWriter::close of many index writers (the additive and deletive indexes of every
// fileset of a group), level by level: level k of every writer still open is closed in one
// grouped close on the level's ctx (one scan, one hash launch and one chunk.Create instead of
// one of each per writer), which runs their callbacks and so fills level k + 1.  Each index
// stream is independent, so the roots and events equal closing the writers one by one; a
// writer stops at the level that closed with one annotation in one chunk, as close() does.
int close_indexes_grouped(const std::vector<IndexWriter*>& iws) {
  std::vector<size_t> next(iws.size(), 0);
  std::vector<char> done(iws.size(), 0);
  for (IndexWriter* w : iws) w->closed = true;
  for (;;) {
    int lvl = -1;
    for (size_t i = 0; i < iws.size(); i++) {
      if (done[i]) continue;
      if (next[i] >= iws[i]->levels.size()) {
        done[i] = 1;
        continue;
      }
      if (lvl < 0 || (int)next[i] < lvl) lvl = (int)next[i];
    }
    if (lvl < 0) break;
    std::vector<size_t> ids;
    std::vector<pfscdc_writer*> cws;
    for (size_t i = 0; i < iws.size(); i++)
      if (!done[i] && (int)next[i] == lvl) {
        ids.push_back(i);
        cws.push_back(iws[i]->levels[lvl]->cw);
      }
    int rc = pfscdc::writers_close_group(cws.data(), cws.size(), nullptr, nullptr, 0);
    if (rc) return rc;
    for (size_t i : ids) {
      pfscdc_writer* cw = iws[i]->levels[lvl]->cw;
      if (pfscdc_writer_annotation_count(cw) == 1 && pfscdc_writer_chunk_count(cw) == 1) done[i] = 1;
      else next[i]++;
    }
  }
  return PFSCDC_OK;
}

// Host bytes of one fileset's Puts, appended in arrival order (a Put copies into it once);
// the Buffer keeps each file as spans of it and the fileset's chunk writer uploads the spans
// straight from here in path order.  Recycled through the writer's pool.
struct Arena {
  uint8_t* p = nullptr;
  uint64_t cap = 0, used = 0;
  bool pinned = false;  // page-locked: the H2D upload runs at full PCIe rate
  // The device mirror: each Put's bytes go up (async, on the writer's upload stream) right
  // after their host copy, so a group write finds its input on the device and gathers it
  // device to device instead of waiting for a PCIe upload of the whole group.
  uint8_t* dev = nullptr;
  int device = -1;
  hipEvent_t ev = nullptr;  // the last upload into the mirror
  ~Arena() {
    if (pinned) (void)hipHostFree(p);
    else delete[] p;
    if (dev) (void)hipFree(dev);
    if (ev) (void)hipEventDestroy(ev);
  }
};

// memcpy split over threads for large Puts (one core copies ~10 GB/s).  The threads are
// persistent: a Put is typically one file of ~10 MB, and spawning 15 threads per Put cost
// more than the copy (c4: 30-40 GB/s with spawned threads).
// The PFSCDC_COPY_THREADS knob (read when the first large Put copies), else up to 16 hardware
// threads (the job's share on the MI355X pool: 16 per GPU, whose nproc shows the whole machine).
class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool* p = new CopyPool();  // never destroyed: its threads run until exit
    return *p;
  }
  unsigned threads() const { return (unsigned)workers_.size() + 1; }
  // dst[0, n) = src[0, n), split in parts of at least kPart over the pool and the caller.  A
  // c4 Put of 10.7 MB takes 5 threads: all 16 (256 KiB parts) copied at 77 GB/s on 8 GiB but
  // 43 GB/s on 32 GiB, against 69-72 GB/s with 2 MiB parts (the copies share the host's
  // memory bandwidth with the mirrors' uploads; profiles/r3/uw/uw_final_*.json)
  void copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
    constexpr uint64_t kMin = 4ull << 20, kPart = 2ull << 20;
    const unsigned t = n < kMin || workers_.empty()
                           ? 1u
                           : (unsigned)std::min<uint64_t>(threads(), n / kPart);
    if (t <= 1) {
      std::memcpy(dst, src, n);
      return;
    }
    std::unique_lock<std::mutex> one(call_mu_);  // one multi-part copy at a time
    const uint64_t part = (n / t + 4095) & ~4095ULL;
    {
      std::lock_guard<std::mutex> lk(mu_);
      dst_ = dst;
      src_ = src;
      n_ = n;
      part_ = part;
      parts_ = t;
      next_ = 1;  // part 0 is the caller's
      left_ = t - 1;
      gen_++;
    }
    cv_.notify_all();
    std::memcpy(dst, src, std::min<uint64_t>(n, part));
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return left_ == 0; });
  }

 private:
  CopyPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    unsigned t = std::min(16u, hw ? hw : 1u);
    if (const int64_t k = pfscdc::knob_freeze(pfscdc::Knob::CopyThreads)) t = (unsigned)k;
    for (unsigned i = 1; i < t; i++) workers_.emplace_back([this] { run(); });
    for (auto& w : workers_) w.detach();
  }
  void run() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [&] { return gen_ != seen && next_ < parts_; });
      while (next_ < parts_) {
        const unsigned i = next_++;
        const uint64_t a = std::min<uint64_t>(n_, part_ * i), b = std::min<uint64_t>(n_, part_ * (i + 1));
        uint8_t* d = dst_;
        const uint8_t* s = src_;
        lk.unlock();
        if (b > a) std::memcpy(d + a, s + a, b - a);
        lk.lock();
        if (--left_ == 0) done_cv_.notify_all();
      }
      seen = gen_;
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_cv_;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  uint64_t n_ = 0, part_ = 0, gen_ = 0;
  unsigned parts_ = 0, next_ = 0, left_ = 0;
};

void copy_parallel(uint8_t* dst, const uint8_t* src, uint64_t n) { CopyPool::get().copy(dst, src, n); }

// Page-locked arenas outlive their writer: a commit creates a fresh UnorderedWriter, and
// page-locking 1 GB for every fileset of every commit (hipHostMalloc) costs more than the Put
// copies themselves.  Process-wide pool, capped by BYTES (each pooled arena holds its host
// bytes page-locked and, with the device mirror, as many bytes of HBM):
// the PFSCDC_UW_ARENA_POOL_BYTES knob, default 40e9 (one 32 GiB group's worth of 1e9-byte
// arenas, so a group never page-locks fresh ones; a 16-arena pool re-allocated 18 of them every
// commit, 11.7 vs 27.8 GiB/s, profiles/r3/uw_groups/).  pfscdc_uw_trim_cache() frees the pool.
struct ArenaPool {
  std::mutex mu;
  std::vector<std::unique_ptr<Arena>> free;
  uint64_t held = 0;  // bytes of the pooled arenas (host; the mirrors hold as many on devices)
  std::unique_ptr<Arena> take(uint64_t bytes, int device) {
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = free.size(); i-- > 0;)
      if (free[i]->cap == bytes && free[i]->device == device) {
        std::unique_ptr<Arena> a = std::move(free[i]);
        free.erase(free.begin() + (ptrdiff_t)i);
        held -= a->cap;
        a->used = 0;
        return a;
      }
    return nullptr;
  }
  void give(std::unique_ptr<Arena> a) {
    std::unique_lock<std::mutex> lk(mu);
    if (held + a->cap <= (uint64_t)pfscdc::knob(pfscdc::Knob::UwArenaPoolBytes)) {
      held += a->cap;
      free.push_back(std::move(a));
      return;
    }
    lk.unlock();
    a.reset();  // over the cap: page-locked host bytes and the mirror freed now
  }
  // Free the pooled arenas of one device (their mirrors live there; -1: every arena).
  uint64_t trim(int device) {
    std::vector<std::unique_ptr<Arena>> out;
    {
      std::lock_guard<std::mutex> lk(mu);
      for (size_t i = free.size(); i-- > 0;)
        if (device < 0 || free[i]->device == device || free[i]->device < 0) {
          held -= free[i]->cap;
          out.push_back(std::move(free[i]));
          free.erase(free.begin() + (ptrdiff_t)i);
        }
    }
    uint64_t n = 0;
    for (auto& a : out) n += a->cap;
    out.clear();  // hipHostFree / hipFree outside the lock
    return n;
  }
};
ArenaPool& arena_pool() {
  static ArenaPool* p = new ArenaPool();  // never destroyed: arenas may outlive static dtors
  return *p;
}

struct Buffer {  // buffer.go:10-106; std::map orders keys bytewise, as sortFiles does
  std::map<std::string, std::map<std::string, std::vector<Span>>> additive;
  std::map<std::string, std::set<std::string>> deletive;
  std::unique_ptr<Arena> arena;

  std::vector<Span>& add(const std::string& path0, const std::string& tag) {
    return additive[clean(path0, false)][tag];
  }
  void del(const std::string& path0, const std::string& tag) {
    const std::string path = clean(path0, is_dir(path0));
    if (is_dir(path)) {
      for (auto it = additive.lower_bound(path); it != additive.end() &&
                                                 it->first.compare(0, path.size(), path) == 0;)
        it = additive.erase(it);
      return;
    }
    auto it = additive.find(path);
    if (it != additive.end()) it->second.erase(tag);  // the (now maybe empty) path entry stays
    deletive[path].insert(tag);
  }
  bool empty() const { return additive.empty() && deletive.empty(); }
};

}  // namespace

// One background group writer: its own data ctx (so groups overlap on the GPU, each on its
// ctx's stream) and index ctxs; the group it writes; its stage times.
struct GroupWorker {
  Streams st;
  std::thread th;
  std::atomic<int> rc{PFSCDC_OK};
  std::vector<Buffer> group;
  std::vector<std::pair<pfscdc_uw_event, std::string>> held;  // this group's events (ordered)
  int device = 0;
  double stage_ms[8] = {};  // close_group's 6 stages, [6] the index writers, [7] group wall
};

struct pfscdc_uwriter {  // unordered_writer.go:15-26
  int64_t mem_threshold = 1000000000;
  int64_t mem_available = 1000000000;
  Buffer buffer;
  std::vector<FilesetInfo> filesets;  // by serialized fileset number (groups finish in any order)
  std::mutex fs_mu, emit_mu;
  // Serialized buffers waiting for the GPU: up to inflight_bytes of them are written
  // together (one scan, one hash launch and one chunk.Create for all their data streams) by
  // one of the group writers, round robin, while Puts continue.  The output equals
  // serializing one at a time; each fileset's chunk stream is independent.  A group's GPU
  // time is bound by its longest chunks' two serial chains (~340 ms on c4) whatever its size,
  // so groups are large: 32 GiB (the PFSCDC_UW_INFLIGHT knob; c4, 32 GiB Put: 8 GiB groups 18.8, 16
  // GiB 25.1, 32 GiB 27.8 GiB/s, profiles/r3/uw_groups/).
  std::vector<Buffer> pending;
  std::vector<std::unique_ptr<Arena>> pool;  // arenas of written filesets, for reuse
  std::mutex pool_mu;
  std::vector<std::unique_ptr<GroupWorker>> workers;
  size_t next_worker = 0;
  ~pfscdc_uwriter() {  // the written filesets' arenas serve the next writer
    for (auto& kv : up_streams) {
      (void)hipSetDevice(kv.first);
      (void)hipStreamSynchronize(kv.second);
      (void)hipStreamDestroy(kv.second);
    }
    for (auto& a : pool)
      if (a->pinned) arena_pool().give(std::move(a));
  }
  double put_copy_ms = 0;  // host copies of the Puts into the arenas
  bool mirror = true;  // the PFSCDC_UW_MIRROR knob (0: upload at group write time instead)
  bool index_grouped = true;  // the PFSCDC_UW_INDEX_GROUPED knob (0: one fileset at a time)
  std::map<int, hipStream_t> up_streams;  // the Puts' uploads into the arena mirrors, per device
  // several group writers: events go out group by group (emit_seq = the next group to emit)
  bool ordered = false;
  std::mutex seq_mu;
  std::condition_variable seq_cv;
  uint64_t emit_seq = 0, next_seq = 0;
  bool emit_failed = false;
  uint64_t pending_bytes = 0, inflight_bytes = 32ull << 30;
  std::vector<std::pair<std::vector<std::pair<std::string, std::string>>,
                        std::vector<std::pair<std::string, std::string>>>> keys;  // files, deletes
  uint32_t next_fileset = 0;
  bool closed = false;
  int err = 0;
  std::string errmsg;  // pfscdc_uw_last_error

  int fail(int rc, const char* what = nullptr) {
    join();  // the background group writes use the data ctxs (and their error strings) too
    if (!err) {
      err = rc;
      errmsg = std::string(what ? what : "unordered writer") + " failed (status " +
               std::to_string(rc) + ")";
      for (auto& w : workers) {
        const char* ce = pfscdc_last_error(w->st.data_ctx);
        if (ce && *ce) {
          errmsg += std::string(": ") + ce;
          break;
        }
      }
    }
    return err;
  }

  std::unique_ptr<Arena> new_arena() {
    // the mirror lives on the device of the group writer the next flush goes to (all of a
    // group's filesets are written by one writer)
    const int device = workers[next_worker]->device;
    {
      std::lock_guard<std::mutex> lk(pool_mu);
      if (!pool.empty()) {  // a written fileset's arena, preferably one mirrored on device
        size_t pick = pool.size() - 1;
        for (size_t i = pool.size(); i-- > 0;)
          if (pool[i]->device == device) {
            pick = i;
            break;
          }
        std::unique_ptr<Arena> a = std::move(pool[pick]);
        pool.erase(pool.begin() + (ptrdiff_t)pick);
        a->used = 0;
        return a;
      }
    }
    if (auto a = arena_pool().take((uint64_t)mem_threshold, mirror ? device : -1)) return a;
    auto a = std::make_unique<Arena>();
    a->cap = (uint64_t)mem_threshold;  // a Buffer never holds more than memThreshold bytes
    if (hipHostMalloc((void**)&a->p, a->cap, hipHostMallocDefault) == hipSuccess) {
      a->pinned = true;
    } else {
      a->p = new (std::nothrow) uint8_t[a->cap];
      if (!a->p) return nullptr;
    }
    // a mirror only for a page-locked arena (async uploads) and while device memory lasts
    if (mirror && a->pinned && hipSetDevice(device) == hipSuccess &&
        hipMalloc((void**)&a->dev, a->cap) == hipSuccess) {
      if (hipEventCreateWithFlags(&a->ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipFree(a->dev);
        a->dev = nullptr;
      } else {
        a->device = device;
      }
    }
    return a;
  }

  int serialize() {  // unordered_writer.go:83-122
    if (buffer.empty()) return PFSCDC_OK;
    std::vector<std::pair<std::string, std::string>> files, deletes;
    for (auto& p : buffer.additive)
      for (auto& t : p.second) files.emplace_back(p.first, t.first);
    for (auto& p : buffer.deletive)
      for (auto& t : p.second) deletes.emplace_back(p.first, t);
    keys.emplace_back(std::move(files), std::move(deletes));
    pending_bytes += buffer.arena ? buffer.arena->used : 0;
    pending.push_back(std::move(buffer));
    buffer = Buffer();
    mem_available = mem_threshold;
    next_fileset++;
    return pending_bytes >= inflight_bytes ? flush_pending(true) : PFSCDC_OK;
  }

  // Writes one group of serialized buffers: a fileset.Writer each, their data streams
  // through one grouped close, then their indexes; the arenas go back to the pool.
  // Group seq's held events, once groups < seq have emitted theirs (several group writers).
  // A group that failed, or follows a failed emission, emits nothing but still takes its turn.
  int release_events(GroupWorker& gw, uint64_t seq, int rc) {
    std::unique_lock<std::mutex> lk(seq_mu);
    seq_cv.wait(lk, [&] { return emit_seq == seq; });
    if (!rc && !emit_failed) {
      std::lock_guard<std::mutex> ek(emit_mu);
      for (auto& e : gw.held) {
        if (e.first.kind == PFSCDC_EV_INDEX) e.first.bytes = (const uint8_t*)e.second.data();
        if (gw.st.cb(gw.st.user, &e.first) != 0) {
          rc = PFSCDC_ECALLBACK;
          break;
        }
      }
    }
    if (rc) emit_failed = true;
    gw.held.clear();
    emit_seq++;
    seq_cv.notify_all();
    return rc;
  }

  int write_group(GroupWorker& gw, std::vector<Buffer>& group, uint32_t fs0, uint64_t seq) {
    int rc = write_group_body(gw, group, fs0);
    return ordered && gw.st.cb ? release_events(gw, seq, rc) : rc;
  }

  int write_group_body(GroupWorker& gw, std::vector<Buffer>& group, uint32_t fs0) {
    using clk = std::chrono::steady_clock;
    const auto g0 = clk::now();
    Streams& st = gw.st;
    st.hold = ordered ? &gw.held : nullptr;
    std::vector<std::unique_ptr<FilesetWriter>> fws;
    std::vector<pfscdc_writer*> cws;
    std::vector<hipEvent_t> evs;  // the group's arena uploads
    int rc = PFSCDC_OK;
    for (size_t i = 0; i < group.size() && !rc; i++) {
      fws.push_back(std::make_unique<FilesetWriter>(&st, fs0 + (uint32_t)i));
      FilesetWriter& fw = *fws.back();
      rc = fw.open();
      const uint8_t* base = group[i].arena ? group[i].arena->p : nullptr;
      const uint8_t* dev = group[i].arena && group[i].arena->device == pfscdc::ctx_device(st.data_ctx)
                               ? group[i].arena->dev : nullptr;
      if (dev) evs.push_back(group[i].arena->ev);
      for (auto& p : group[i].additive)
        for (auto& t : p.second)
          if (!rc) rc = fw.add(p.first, t.first, base, t.second, dev);
      for (auto& p : group[i].deletive)
        for (auto& t : p.second)
          if (!rc) rc = fw.del(p.first, t);
      cws.push_back(fw.cw);
    }
    if (!rc)
      rc = pfscdc::writers_close_group(cws.data(), cws.size(), gw.stage_ms, evs.data(), evs.size());
    const auto g1 = clk::now();
    // the indexes of every fileset of the group, closed level by level in grouped closes
    // (the PFSCDC_UW_INDEX_GROUPED knob at 0: one fileset at a time)
    if (index_grouped) {
      std::vector<IndexWriter*> iws;
      for (size_t i = 0; i < fws.size() && !rc; i++) {
        rc = fws[i]->finish_last_entry();
        iws.push_back(&fws[i]->additive);
        iws.push_back(&fws[i]->deletive);
      }
      if (!rc) rc = close_indexes_grouped(iws);
      for (size_t i = 0; i < fws.size() && !rc; i++)
        fws[i]->finish_info(fws[i]->additive.root, fws[i]->deletive.root);
    } else {
      for (size_t i = 0; i < fws.size() && !rc; i++) rc = fws[i]->finish();
    }
    for (size_t i = 0; i < fws.size() && !rc; i++) {
      std::lock_guard<std::mutex> lk(fs_mu);
      const size_t k = fs0 + i;
      if (filesets.size() <= k) filesets.resize(k + 1);
      filesets[k] = std::move(fws[i]->info);
    }
    fws.clear();
    const auto g2 = clk::now();
    gw.stage_ms[6] += std::chrono::duration<double, std::milli>(g2 - g1).count();
    gw.stage_ms[7] += std::chrono::duration<double, std::milli>(g2 - g0).count();
    std::lock_guard<std::mutex> lk(pool_mu);
    for (Buffer& b : group)
      if (b.arena) pool.push_back(std::move(b.arena));
    return rc;
  }

  int join() {  // waits for every group being written in the background
    int rc = PFSCDC_OK;
    for (auto& w : workers) {
      if (w->th.joinable()) w->th.join();
      if (!rc) rc = w->rc;
    }
    return rc;
  }

  int worker_failed() const {
    for (const auto& w : workers)
      if (int rc = w->rc.load()) return rc;
    return PFSCDC_OK;
  }

  // Hands the pending buffers to the next group writer's thread (async) or writes them here;
  // one group per writer is in flight, so Puts keep filling arenas while the GPU writes the
  // last groups, and consecutive groups overlap on the GPU (one ctx stream each).
  int flush_pending(bool async) {
    if (int rc = worker_failed()) return rc;
    if (pending.empty()) return PFSCDC_OK;
    GroupWorker& gw = *workers[next_worker];
    next_worker = (next_worker + 1) % workers.size();
    if (gw.th.joinable()) gw.th.join();
    if (int rc = gw.rc.load()) return rc;
    const uint32_t fs0 = next_fileset - (uint32_t)pending.size();
    const uint64_t seq = next_seq++;
    gw.group.clear();
    gw.group.swap(pending);
    pending_bytes = 0;
    if (!async) return write_group(gw, gw.group, fs0, seq);
    gw.th = std::thread([this, &gw, fs0, seq] { gw.rc = write_group(gw, gw.group, fs0, seq); });
    return PFSCDC_OK;
  }

  int put(const std::string& p, std::string tag, bool append, const uint8_t* data, uint64_t n) {
    if (int rc = worker_failed()) return rc;  // a background group write already failed
    if (tag.empty()) tag = "default";
    if (!append) buffer.del(p, tag);
    std::vector<Span>* w = &buffer.add(p, tag);
    uint64_t pos = 0;
    for (;;) {  // io.CopyN(w, r, memAvailable): EOF iff fewer than memAvailable bytes were left
      const uint64_t want = (uint64_t)mem_available;
      const uint64_t got = std::min<uint64_t>(want, n - pos);
      if (got) {
        if (!buffer.arena && !(buffer.arena = new_arena())) return PFSCDC_ENOMEM;
        Arena& a = *buffer.arena;
        const auto c0 = std::chrono::steady_clock::now();
        copy_parallel(a.p + a.used, data + pos, got);
        put_copy_ms += std::chrono::duration<double, std::milli>(
                           std::chrono::steady_clock::now() - c0).count();
        if (a.dev) {  // on to the device while the next Puts copy
          hipStream_t& up = up_streams[a.device];
          if (hipSetDevice(a.device) != hipSuccess ||
              (!up && hipStreamCreateWithFlags(&up, hipStreamNonBlocking) != hipSuccess))
            return PFSCDC_EHIP;
          if (hipMemcpyAsync(a.dev + a.used, a.p + a.used, got, hipMemcpyHostToDevice, up) !=
                  hipSuccess ||
              hipEventRecord(a.ev, up) != hipSuccess)
            return PFSCDC_EHIP;
        }
        if (!w->empty() && w->back().off + w->back().len == a.used) w->back().len += got;
        else w->push_back(Span{a.used, got});
        a.used += got;
      }
      pos += got;
      mem_available -= (int64_t)got;
      if (got < want) return PFSCDC_OK;
      if (mem_available == 0) {
        int rc = serialize();
        if (rc) return rc;
        w = &buffer.add(p, tag);
      }
    }
  }

  int del(const std::string& p0, std::string tag) {  // unordered_writer.go:125-149
    if (tag.empty()) tag = "default";
    const std::string p = clean(p0, is_dir(p0));
    if (!is_dir(p)) {
      buffer.del(p, tag);
      return PFSCDC_OK;
    }
    buffer.del(p, tag);
    // merged view of the serialized filesets (merge.go: a (path, tag) group is live iff its
    // last stream, deletive before additive within a fileset, is additive)
    std::map<std::pair<std::string, std::string>, bool> live;
    for (const auto& fs : keys) {  // serialized filesets, written or pending
      for (auto& k : fs.second) live[k] = false;
      for (auto& k : fs.first) live[k] = true;
    }
    for (auto& kv : live)
      if (kv.second && kv.first.first.compare(0, p.size(), p) == 0) buffer.del(kv.first.first, tag);
    return PFSCDC_OK;
  }
};

extern "C" {

}  // extern "C"

namespace {

pfscdc_params index_params_or_default(const pfscdc_params* index_params) {
  pfscdc_params ip;
  if (index_params) {
    ip = *index_params;
  } else {  // index/writer.go:13,60: WithRollingHashConfig(20, level), default min/max
    pfscdc_default_params(&ip);
    ip.average_bits = 20;
    ip.seed = 0;
  }
  return ip;
}

void finish_create(pfscdc_uwriter* w, int64_t mem_threshold) {
  if (mem_threshold) w->mem_threshold = w->mem_available = mem_threshold;
  w->inflight_bytes = (uint64_t)pfscdc::knob(pfscdc::Knob::UwInflight);
  w->mirror = pfscdc::knob(pfscdc::Knob::UwMirror) != 0;
  w->index_grouped = pfscdc::knob(pfscdc::Knob::UwIndexGrouped) != 0;
  w->ordered = w->workers.size() > 1;
}

}  // namespace

extern "C" {

int pfscdc_uw_create_group(pfscdc_group* g, int64_t mem_threshold,
                           const pfscdc_params* index_params, pfscdc_uw_cb cb, void* user,
                           pfscdc_uwriter** out) {
  const uint32_t n = pfscdc_group_size(g);
  if (!g || !out || mem_threshold < 0 || n == 0) return PFSCDC_EINVAL;
  if (!(pfscdc::ctx_options(pfscdc_group_ctx(g, 0)) & PFSCDC_OPT_REF_IDS)) return PFSCDC_EINVAL;
  pfscdc_uwriter* w = new pfscdc_uwriter();
  const pfscdc_params ip = index_params_or_default(index_params);
  for (uint32_t k = 0; k < n; k++) {  // one group writer per member, on the member's ctx
    auto gw = std::make_unique<GroupWorker>();
    gw->st.cb = cb;
    gw->st.user = user;
    gw->st.emit_mu = &w->emit_mu;
    gw->st.index_params = ip;
    gw->st.data_ctx = pfscdc_group_ctx(g, k);
    gw->device = pfscdc::ctx_device(gw->st.data_ctx);
    w->workers.push_back(std::move(gw));
  }
  finish_create(w, mem_threshold);
  // n groups in flight hold what one writer's group would
  w->inflight_bytes = std::max<uint64_t>(w->inflight_bytes / n, (uint64_t)w->mem_threshold);
  *out = w;
  return PFSCDC_OK;
}

int pfscdc_uw_create(pfscdc_ctx* data_ctx, int64_t mem_threshold,
                     const pfscdc_params* index_params, pfscdc_uw_cb cb, void* user,
                     pfscdc_uwriter** out) {
  if (!data_ctx || !out || mem_threshold < 0) return PFSCDC_EINVAL;
  if (!(pfscdc::ctx_options(data_ctx) & PFSCDC_OPT_REF_IDS)) return PFSCDC_EINVAL;
  pfscdc_uwriter* w = new pfscdc_uwriter();
  const pfscdc_params ip = index_params_or_default(index_params);
  // group writers: the first on the caller's data ctx, the others on ctxs of their own
  // (the PFSCDC_UW_WORKERS knob, default 1: two groups in flight contend for the CUs, and each
  // group's chunk.Create chains then run longer; c4, 8 GiB: 15.2 GiB/s with one, 8.9 with two)
  const int nworkers = (int)pfscdc::knob(pfscdc::Knob::UwWorkers);
  for (int k = 0; k < nworkers; k++) {
    auto gw = std::make_unique<GroupWorker>();
    gw->st.cb = cb;
    gw->st.user = user;
    gw->st.emit_mu = &w->emit_mu;
    gw->st.index_params = ip;
    if (k == 0) {
      gw->st.data_ctx = data_ctx;
    } else {
      pfscdc_ctx* c = ctx_cache().take(pfscdc::ctx_params(data_ctx), pfscdc::ctx_device(data_ctx),
                                       pfscdc::ctx_options(data_ctx));
      if (!c) {
        delete w;
        return PFSCDC_EHIP;
      }
      gw->st.data_ctx = c;
      gw->st.own_data_ctx = true;
    }
    gw->device = pfscdc::ctx_device(gw->st.data_ctx);
    w->workers.push_back(std::move(gw));
  }
  finish_create(w, mem_threshold);
  *out = w;
  return PFSCDC_OK;
}

int pfscdc_uw_put(pfscdc_uwriter* w, const char* path, const char* tag, int append_file,
                  const void* data, uint64_t n) {
  if (!w || !path || (n && !data)) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return w->fail(PFSCDC_ESTATE, "Put after Close");
  int rc = w->put(path, tag ? tag : "", append_file != 0, (const uint8_t*)data, n);
  return rc ? w->fail(rc, "Put") : PFSCDC_OK;
}

int pfscdc_uw_delete(pfscdc_uwriter* w, const char* path, const char* tag) {
  if (!w || !path) return PFSCDC_EINVAL;
  if (w->err) return w->err;
  if (w->closed) return w->fail(PFSCDC_ESTATE, "Delete after Close");
  int rc = w->del(path, tag ? tag : "");
  return rc ? w->fail(rc, "Delete") : PFSCDC_OK;
}

int pfscdc_uw_close(pfscdc_uwriter* w) {
  if (!w) return PFSCDC_EINVAL;
  // the background group write may still be appending to filesets: join it on every path
  const int wrc = w->join();
  if (w->err) return w->err;
  if (wrc) return w->fail(wrc, "Close (background fileset write)");
  if (w->closed) return PFSCDC_OK;
  w->closed = true;
  int rc = w->serialize();
  if (!rc) rc = w->flush_pending(false);
  const int jr = w->join();  // the groups still in flight on the other writers
  if (!rc) rc = jr;
  return rc ? w->fail(rc, "Close") : PFSCDC_OK;
}

int pfscdc_uw_timings(const pfscdc_uwriter* w, double out[9]) {
  if (!w || !out) return PFSCDC_EINVAL;
  out[0] = w->put_copy_ms;
  for (int k = 1; k < 9; k++) out[k] = 0;
  for (const auto& g : w->workers)
    for (int k = 0; k < 8; k++) out[1 + k] += g->stage_ms[k];
  return PFSCDC_OK;
}

int pfscdc_uw_trim_cache(int device, uint64_t* arena_bytes_freed, uint32_t* ctxs_destroyed) {
  const uint64_t b = arena_pool().trim(device);
  const uint32_t n = ctx_cache().trim(device);
  if (arena_bytes_freed) *arena_bytes_freed = b;
  if (ctxs_destroyed) *ctxs_destroyed = n;
  return PFSCDC_OK;
}

uint64_t pfscdc_uw_cached_arena_bytes(void) {
  ArenaPool& p = arena_pool();
  std::lock_guard<std::mutex> lk(p.mu);
  return p.held;
}

const char* pfscdc_uw_last_error(const pfscdc_uwriter* w) {
  return w ? w->errmsg.c_str() : "null unordered writer";
}

uint32_t pfscdc_uw_num_filesets(const pfscdc_uwriter* w) {
  return w ? (uint32_t)w->filesets.size() : 0;
}

int pfscdc_uw_fileset(const pfscdc_uwriter* w, uint32_t i, pfscdc_fileset_info* out) {
  if (!w || !out || i >= w->filesets.size()) return PFSCDC_EINVAL;
  const FilesetInfo& f = w->filesets[i];
  out->size_bytes = f.size_bytes;
  out->additive_root = f.has_additive ? (const uint8_t*)f.additive.data() : nullptr;
  out->additive_root_len = f.has_additive ? f.additive.size() : 0;
  out->deletive_root = f.has_deletive ? (const uint8_t*)f.deletive.data() : nullptr;
  out->deletive_root_len = f.has_deletive ? f.deletive.size() : 0;
  out->num_files = (uint32_t)f.files.size();
  out->num_deletes = (uint32_t)f.deletes.size();
  return PFSCDC_OK;
}

int pfscdc_uw_destroy(pfscdc_uwriter* w) {
  if (w) w->join();
  delete w;
  return PFSCDC_OK;
}

int pfscdc_path_clean(const char* path, int is_directory, char* out, uint64_t cap) {
  if (!path || !out) return PFSCDC_EINVAL;
  const std::string y = clean(path, is_directory != 0);
  if (y.size() + 1 > cap) return PFSCDC_ENOMEM;
  std::memcpy(out, y.c_str(), y.size() + 1);
  return PFSCDC_OK;
}

}  // extern "C"
