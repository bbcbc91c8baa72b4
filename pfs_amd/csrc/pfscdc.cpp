// pfscdc.cpp — host side of libpfscdc.so: context, batch pipeline, C ABI.
//
// Replaces, per batch of files, the byte loop of chunk.Writer (reference
// src/internal/storage/chunk/writer.go:118-196) and the hashing half of processChunk
// (writer.go:233-253,288-312).  Chunk assembly and callbacks live in writer.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include <unistd.h>

#include "pfscdc_internal.h"

using namespace pfscdc;

namespace {

template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;  // elements
  hipError_t ensure(size_t n, bool exact = false) {
    if (n <= cap && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 1);
    if (!exact) want = want + want / 4;  // amortize growth
    hipError_t e = hipMalloc((void**)&p, want * sizeof(T));
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

template <typename T>
struct PinnedBuf {
  T* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap && p) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 1);
    want = want + want / 4;
    hipError_t e = hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

// create_refs_device(finish = false) -> create_refs_finish: what the second half unpacks
struct CreatePending {
  bool active = false, split = false;
  uint32_t k = 0, nr = 0;
  uint8_t* hashes = nullptr;
  pfscdc_ref* refs = nullptr;
};

}  // namespace

struct pfscdc_ctx {
  pfscdc_params params{};
  int device = 0;
  int num_cus = 256;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  uint64_t table[256];
  uint64_t* d_table = nullptr;
  DevBuf<uint8_t> d_data, d_tail;
  DevBuf<TileRec> d_recs;
  DevBuf<uint32_t> d_unit_ctr;  // the scan's work-unit counter
  DevBuf<uint32_t> d_skip;      // per scan work unit: leading strip steps with no cut point
  // the cut-skipping scan (ScanPlan): per unit {file, skip | rank}, the rank-ordered
  // dispatch slots, the plan words, per file its rank slots
  DevBuf<uint32_t> d_uinfo, d_plan;
  DevBuf<uint4> d_uslots;
  DevBuf<uint32_t> d_rslots;
  DevBuf<ScanPlan> d_planhdr;  // the scan kernel's view of the plan (scan_slots_kernel stores it)
  bool scan_skipped = false;    // the last scan ran with d_skip (d_counts[3] = bytes scanned,
                                // less d_counts[6] the settled cuts removed)
  uint32_t scan_mode = 0;       // the last scan's PFSCDC_SCAN_SKIPPED_* bits
  uint64_t scanned_bytes = 0;   // bytes the last waited-for scan rolled (copied in pfscdc_wait)
  bool cuts_only = false;       // the last pfscdc_scan left the DataRef hashes to commit_refs
  DevBuf<uint64_t> d_entries, d_counts;  // d_counts: [0] n_entries
  DevBuf<uint64_t> d_offs, d_seg_base, d_nseg, d_seg_begin;
  DevBuf<pfscdc_segment> d_slots, d_segs;
  DevBuf<uint32_t> d_order, d_qctr;  // LPT segment order + hash queue counter
  DevBuf<uint32_t> d_next;            // hash bins: each segment's successor in its bin
  DevBuf<pfscdc_ref> d_refs;
  DevBuf<uint8_t> d_out;  // get_chunks: plaintext when the caller's output is on the host
  // kernel execution spans: [0,1] scan begin/end, [2,3] hash begin/end; shader-clock sums
  // [4,5] scan (cycles, 100 MHz ticks), [6,7] hash
  DevBuf<uint64_t> d_span;
  PinnedBuf<uint64_t> h_span;
  double wall_khz = 100000.0;  // s_memrealtime ticks per ms
  DevBuf<uint32_t> d_ids;  // fill_synthetic_pieces
  DevBuf<uint64_t> d_starts;
  DevBuf<uint8_t> d_group, d_group_ct;  // writers_close_group: staged bytes, ciphertexts
  DevBuf<pfscdc_segment> d_segs2;       // create_refs (split Ref.Id): records of the id pass
  DevBuf<uint64_t> d_blk;               // create_refs (split): 64-B block prefix per record
  DevBuf<uint8_t> d_ctext;              // create_refs (split): ciphertext when not asked for
  PinnedBuf<uint64_t> h_blk;
  PinnedBuf<pfscdc_segment> h_segs2;
  PinnedBuf<pfscdc_ref> h_refs;
  uint32_t options = 0;
  float get_ms = 0.f;
  float create_ms = 0.f, create_hash_ms = 0.f;
  hipEvent_t cev = nullptr;  // create_refs: between the content-hash and the Ref.Id passes
  hipEvent_t wev = nullptr;  // pfscdc_stream_wait: the caller's stream position
  hipStream_t aux_stream = nullptr;      // create_refs: the second Ref.Id stream (lazy)
  hipEvent_t xev[2] = {nullptr, nullptr};  // its fork / join events
  std::vector<uint32_t> perm;  // create_refs: record -> chunk
  CreatePending cr;            // create_refs enqueued, not yet finished
  // create_refs launch shape for this call (commit_refs' two chunk sets): waves per SIMD cap
  // (0: none; also caps the ChaCha20 grid at one wave per SIMD), issue priority of every hash
  // launch (0: the launch's own), ChaCha20 waves at issue priority 2
  int cr_wave_cap = 0;
  uint32_t cr_hash_prio = 0;
  bool cr_chacha_prio = false;
  bool cr_one_stream = false;  // no second-stream split of the Ref.Id pass
  pfscdc_ctx* helper = nullptr;  // commit_refs: the short chunk set's context (lazy)
  hipEvent_t pev[3] = {nullptr, nullptr, nullptr};  // commit_refs: start, long / short unions
  bool have_refs = false;
  bool scan_valid = false;  // h_offs/h_segs/h_seg_begin hold the last scan's results
  bool host_records = true;  // h_segs / h_refs were fetched (not by a device group's member)
  PinnedBuf<uint64_t> h_offs, h_seg_base, h_seg_begin;
  PinnedBuf<pfscdc_segment> h_segs;
  hipEvent_t ev[8] = {};
  bool pending = false;
  uint32_t nfiles = 0;
  uint64_t nbytes = 0;
  uint64_t ntiles = 0;
  uint64_t slot_cap = 0;
  uint64_t nsegs = 0;
  const uint8_t* dev_data = nullptr;  // data pointer of the last scan
  pfscdc_ctx* hash_after = nullptr;   // pfscdc_order_hash_after
};

namespace pfscdc {
const pfscdc_params& ctx_params(const pfscdc_ctx* ctx) { return ctx->params; }
}  // namespace pfscdc

namespace {

// Scan workgroups: one per CU (each takes a whole CU's LDS), at most the tiles.  A workgroup
// that finds no CU free waits for one, and the launch ends only after every workgroup has run:
// with other streams' chain-bound hash launches resident on some CUs (c3's streams in flight,
// which reserve their CUs), a full-width scan waits for them.  The PFSCDC_SCAN_GRID knob caps
// the workgroups (the work queue spreads the units over however many run).
static int scan_grid(uint64_t ntiles, int num_cus) {
  uint64_t g = std::min<uint64_t>(ntiles, (uint64_t)num_cus);
  const int64_t cap = knob(Knob::ScanGrid);
  if (cap > 0 && (uint64_t)cap < g) g = (uint64_t)cap;
  return (int)g;
}

// Waves per SIMD of a hash launch (the PFSCDC_HASH_WAVES knob forces a count)
static int knob_waves(uint64_t longest, uint64_t sum, int num_cus) {
  return hash_waves(longest, sum, num_cus, (int)knob(Knob::HashWaves));
}

// The scan also skips the min - 1 positions after each file's cuts once they are settled
// (ScanPlan).  Exact for min - 1 >= one work unit (pfscdc_internal.h); the PFSCDC_SCAN_CUTSKIP
// knob turns it off.
bool cut_skip_exact(const pfscdc_params& p) {
  return knob(Knob::ScanCutSkip) != 0 && (uint64_t)p.min_chunk >= kScanUnit + 1 &&
         p.max_chunk > p.min_chunk;
}

int fail(pfscdc_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIP_OK(ctx, expr)                                                           \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess)                                                           \
      return fail((ctx), e_ == hipErrorOutOfMemory ? PFSCDC_ENOMEM : PFSCDC_EHIP,   \
                  std::string(#expr) + ": " + hipGetErrorString(e_));               \
  } while (0)

int validate_params(const pfscdc_params* p, std::string* why) {
  if (!p) {
    *why = "params is NULL";
    return PFSCDC_EINVAL;
  }
  if (p->average_bits < 1 || p->average_bits > 63) {
    *why = "average_bits must be in [1, 63]";
    return PFSCDC_EINVAL;
  }
  if (p->max_chunk < p->min_chunk || p->min_chunk < 1) {
    *why = "need 1 <= min_chunk <= max_chunk";
    return PFSCDC_EINVAL;
  }
  if (p->min_chunk < 64) {
    // A cut position < 64 bytes after a reset would hash part of the zero reset window;
    // the block-parallel scan assumes every eligible hash sees 64 real bytes.
    *why = "min_chunk < 64 (the rolling window) is not supported on the GPU path";
    return PFSCDC_EUNSUPPORTED;
  }
  return PFSCDC_OK;
}

constexpr int kSpanSlots = 8;
// Kernel spans start as (begin = ~0, end = 0): the kernels lower begin and raise end.
hipError_t reset_spans(pfscdc_ctx* c, hipStream_t st) {
  hipError_t e = hipMemsetAsync(c->d_span.p, 0, kSpanSlots * sizeof(uint64_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(c->d_span.p, 0xFF, sizeof(uint64_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(c->d_span.p + 2, 0xFF, sizeof(uint64_t), st);
  return e;
}

}  // namespace

extern "C" {

void pfscdc_default_params(pfscdc_params* p) {
  p->average_bits = 23;
  p->reserved = 0;
  p->seed = 1;
  p->min_chunk = 1000000;
  p->max_chunk = 20000000;
}

int pfscdc_table(int64_t seed, uint64_t out[256]) {
  if (!out) return PFSCDC_EINVAL;
  generate_hashes(seed, out);
  return PFSCDC_OK;
}

int pfscdc_go_int63(int64_t seed, int64_t* out, int n) {
  if (!out || n < 0) return PFSCDC_EINVAL;
  go_int63(seed, out, n);
  return PFSCDC_OK;
}

int pfscdc_ctx_create(const pfscdc_params* params, int device, pfscdc_ctx** out) {
  return pfscdc::ctx_create_on(params, device, nullptr, out);
}

}  // extern "C"

// A context on the caller's stream (shared != nullptr: no stream of its own; commit_refs'
// helper runs on its owner's second stream, so the commit uses two hardware queues, not
// four: streams beyond GPU_MAX_HW_QUEUES share a queue and serialize).
int pfscdc::ctx_create_on(const pfscdc_params* params, int device, hipStream_t shared,
                          pfscdc_ctx** out) {
  if (!out) return PFSCDC_EINVAL;
  *out = nullptr;
  std::string why;
  int rc = validate_params(params, &why);
  if (rc) {
    std::fprintf(stderr, "pfscdc_ctx_create: %s\n", why.c_str());
    return rc;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    std::fprintf(stderr, "pfscdc_ctx_create: no HIP device visible\n");
    return PFSCDC_EHIP;
  }
  if (device < 0 || device >= ndev) return PFSCDC_EINVAL;
  pfscdc_ctx* c = new pfscdc_ctx();
  c->params = *params;
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return PFSCDC_EHIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->num_cus = prop.multiProcessorCount;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
    c->wall_khz = khz;
  if (hipError_t e = prepare_kernels(); e != hipSuccess) {
    std::fprintf(stderr, "pfscdc_ctx_create: kernel attributes: %s\n", hipGetErrorString(e));
    delete c;
    return PFSCDC_EHIP;
  }
  generate_hashes(params->seed, c->table);
  if ((!shared && hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) ||
      hipMalloc((void**)&c->d_table, sizeof c->table) != hipSuccess ||
      hipMemcpy(c->d_table, c->table, sizeof c->table, hipMemcpyHostToDevice) != hipSuccess) {
    delete c;
    return PFSCDC_EHIP;
  }
  for (auto& e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) {
      delete c;
      return PFSCDC_EHIP;
    }
  if (hipEventCreate(&c->cev) != hipSuccess ||
      hipEventCreateWithFlags(&c->wev, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return PFSCDC_EHIP;
  }
  c->stream = shared ? shared : c->own_stream;
  *out = c;
  return PFSCDC_OK;
}

extern "C" {

int pfscdc_ctx_destroy(pfscdc_ctx* c) {
  if (!c) return PFSCDC_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->pending) (void)hipStreamSynchronize(c->stream);
  if (c->helper) pfscdc_ctx_destroy(c->helper);  // it runs on c->aux_stream
  c->d_data.release();
  c->d_tail.release();
  c->d_recs.release();
  c->d_unit_ctr.release();
  c->d_entries.release();
  c->d_skip.release();
  c->d_uinfo.release();
  c->d_plan.release();
  c->d_uslots.release();
  c->d_rslots.release();
  c->d_planhdr.release();
  c->d_counts.release();
  c->d_offs.release();
  c->d_seg_base.release();
  c->d_nseg.release();
  c->d_seg_begin.release();
  c->d_slots.release();
  c->d_segs.release();
  c->d_next.release();
  c->d_order.release();
  c->d_qctr.release();
  c->d_refs.release();
  c->h_refs.release();
  c->d_out.release();
  c->d_ids.release();
  c->d_span.release();
  c->h_span.release();
  c->d_starts.release();
  c->d_group.release();
  c->d_group_ct.release();
  c->d_segs2.release();
  c->d_blk.release();
  c->d_ctext.release();
  c->h_blk.release();
  c->h_segs2.release();
  c->h_offs.release();
  c->h_seg_base.release();
  c->h_seg_begin.release();
  c->h_segs.release();
  if (c->d_table) (void)hipFree(c->d_table);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->cev) (void)hipEventDestroy(c->cev);
  if (c->wev) (void)hipEventDestroy(c->wev);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  if (c->aux_stream) (void)hipStreamDestroy(c->aux_stream);
  for (auto& e : c->pev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : c->xev)
    if (e) (void)hipEventDestroy(e);
  delete c;
  return PFSCDC_OK;
}

const char* pfscdc_last_error(const pfscdc_ctx* c) { return c ? c->err.c_str() : "null ctx"; }

int pfscdc_set_stream(pfscdc_ctx* c, void* hip_stream) {
  if (!c) return PFSCDC_EINVAL;
  c->stream = hip_stream ? (hipStream_t)hip_stream : c->own_stream;
  return PFSCDC_OK;
}

int pfscdc_order_hash_after(pfscdc_ctx* c, pfscdc_ctx* other) {
  if (!c || other == c) return PFSCDC_EINVAL;
  c->hash_after = other;
  return PFSCDC_OK;
}

void* pfscdc_stream_handle(const pfscdc_ctx* c) { return c ? (void*)c->stream : nullptr; }

int pfscdc_stream_wait(pfscdc_ctx* c, void* hip_stream) {
  if (!c) return PFSCDC_EINVAL;
  hipStream_t s = (hipStream_t)hip_stream;
  if (s == c->stream) return PFSCDC_OK;
  HIP_OK(c, hipSetDevice(c->device));
  HIP_OK(c, hipEventRecord(c->wev, s));
  HIP_OK(c, hipStreamWaitEvent(c->stream, c->wev, 0));
  return PFSCDC_OK;
}

}  // extern "C"

namespace {

int scan_async_impl(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
                    const uint64_t* file_offsets, uint32_t nfiles, uint32_t options) {
  if (!c) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "previous scan not waited for");
  c->cuts_only = false;
  if (!file_offsets) return fail(c, PFSCDC_EINVAL, "file_offsets is NULL");
  if (nbytes && !bytes) return fail(c, PFSCDC_EINVAL, "bytes is NULL");
  if (file_offsets[0] != 0 || file_offsets[nfiles] != nbytes)
    return fail(c, PFSCDC_EINVAL, "file_offsets must start at 0 and end at nbytes");
  for (uint32_t f = 0; f < nfiles; f++)
    if (file_offsets[f + 1] < file_offsets[f])
      return fail(c, PFSCDC_EINVAL, "file_offsets must be nondecreasing");
  if (bytes_on_device && ((uintptr_t)bytes & 15))
    return fail(c, PFSCDC_EINVAL, "device bytes must be 16-byte aligned");
  c->ntiles = (nbytes + kTile - 1) / kTile;
  if (c->ntiles * (uint64_t)kScanWaves >= (1ull << 32))  // the scan's 32-bit work-unit counter
    return fail(c, PFSCDC_EUNSUPPORTED, "batch too large for one scan (split it)");
  c->scan_valid = false;
  HIP_OK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  const pfscdc_params& p = c->params;

  // per-file segment slot ranges: every segment but a file's last is >= min bytes
  HIP_OK(c, c->h_offs.ensure(nfiles + 1));
  HIP_OK(c, c->h_seg_base.ensure(nfiles + 1));
  std::memcpy(c->h_offs.p, file_offsets, sizeof(uint64_t) * (nfiles + 1));
  uint64_t cap = 0, longest_file = 0;
  for (uint32_t f = 0; f < nfiles; f++) {
    c->h_seg_base.p[f] = cap;
    const uint64_t len = file_offsets[f + 1] - file_offsets[f];
    cap += len ? len / (uint64_t)p.min_chunk + 1 : 0;
    longest_file = std::max(longest_file, len);
  }
  // the hash's longest chain is at most the largest file and at most max_chunk
  const int waves = knob_waves(std::min<uint64_t>(longest_file, (uint64_t)p.max_chunk), nbytes,
                              c->num_cus);
  // hash bins: the files of at most one quad's share of the bytes are hashed whole by one
  // quad each (lpt_order_block); the PFSCDC_HASH_BIN_BYTES knob fixes the bin size (0: every
  // segment its own queue entry)
  const uint64_t quads = (uint64_t)c->num_cus * 4 * (uint64_t)waves * 16;
  const int64_t kb = knob(Knob::HashBinBytes);
  const uint64_t bin_bytes = kb >= 0 ? (uint64_t)kb : (nbytes + quads - 1) / quads;
  c->h_seg_base.p[nfiles] = cap;
  c->slot_cap = cap;
  c->nfiles = nfiles;
  c->nbytes = nbytes;

  HIP_OK(c, c->d_offs.ensure(nfiles + 1));
  HIP_OK(c, c->d_seg_base.ensure(nfiles + 1));
  HIP_OK(c, c->d_nseg.ensure(nfiles + 1));
  HIP_OK(c, c->d_seg_begin.ensure(nfiles + 1));
  HIP_OK(c, c->d_slots.ensure(cap));
  HIP_OK(c, c->d_segs.ensure(cap));
  HIP_OK(c, c->d_order.ensure(cap));
  if (bin_bytes) HIP_OK(c, c->d_next.ensure(cap));
  HIP_OK(c, c->d_qctr.ensure(2));
  if (options & PFSCDC_OPT_REF_IDS) HIP_OK(c, c->d_refs.ensure(cap));
  HIP_OK(c, c->d_recs.ensure(c->ntiles));
  HIP_OK(c, c->d_unit_ctr.ensure(3));
  HIP_OK(c, c->d_entries.ensure(c->ntiles * kTileK + 1));
  // [3] bytes scanned, [4] the hash queue's length (select), [5] fair share, [6] bytes the
  // settled cuts took off [3]
  HIP_OK(c, c->d_counts.ensure(7));
  HIP_OK(c, c->d_tail.ensure(kTailBytes));
  HIP_OK(c, c->d_span.ensure(kSpanSlots));
  HIP_OK(c, c->h_span.ensure(kSpanSlots + 4));

  const uint8_t* data;
  if (bytes_on_device) {
    data = (const uint8_t*)bytes;
  } else {
    HIP_OK(c, c->d_data.ensure(nbytes + 64));
    if (nbytes) HIP_OK(c, hipMemcpyAsync(c->d_data.p, bytes, nbytes, hipMemcpyHostToDevice, st));
    data = c->d_data.p;
  }
  c->dev_data = data;
  HIP_OK(c, hipMemcpyAsync(c->d_offs.p, c->h_offs.p, sizeof(uint64_t) * (nfiles + 1),
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_seg_base.p, c->h_seg_base.p, sizeof(uint64_t) * (nfiles + 1),
                           hipMemcpyHostToDevice, st));
  // zero-padded copy of the final partial 64-byte block (so the scan never reads past n)
  const uint64_t n_main = nbytes & ~63ULL;
  HIP_OK(c, hipMemsetAsync(c->d_tail.p, 0, kTailBytes, st));
  if (nbytes > n_main)
    HIP_OK(c, hipMemcpyAsync(c->d_tail.p, data + n_main, nbytes - n_main,
                             hipMemcpyDeviceToDevice, st));
  HIP_OK(c, hipMemsetAsync(c->d_counts.p, 0, 7 * sizeof(uint64_t), st));
  // the scan adds candidates to the tile records with atomics
  if (c->ntiles) HIP_OK(c, hipMemsetAsync(c->d_recs.p, 0, sizeof(TileRec) * c->ntiles, st));
  HIP_OK(c, hipMemsetAsync(c->d_unit_ctr.p, 0, 3 * sizeof(uint32_t), st));  // + done counters
  HIP_OK(c, reset_spans(c, st));

  HIP_OK(c, hipEventRecord(c->ev[0], st));
  c->scan_skipped = false;
  c->scan_mode = 0;
  if (c->ntiles) {  // scan + (last workgroup) compaction into the sorted entry list
    // the first min - 1 bytes of every file hold no cut point: those strip steps are skipped
    const uint32_t* skip = nullptr;
    c->scan_skipped = knob(Knob::ScanSkip) != 0;
    c->scan_mode = c->scan_skipped ? PFSCDC_SCAN_SKIPPED_FIRST_MIN : 0u;
    const ScanPlan* d_plan = nullptr;
    const uint64_t nunits = c->ntiles * kScanWaves;
    if (c->scan_skipped) {
      HIP_OK(c, c->d_skip.ensure(nunits));
      // (the rank slots cost 256 B per file: batches of mostly tiny files, where it gains
      // nothing, keep the plain form)
      const bool cs_room = nfiles < kPlanMaxFiles &&
                           (uint64_t)nfiles * kRankSlots * sizeof(uint32_t) * 64 <= nbytes;
      if (cs_room && cut_skip_exact(p)) {
        c->scan_mode |= PFSCDC_SCAN_SKIPPED_CUTS;
        // and past every cut the scan has settled (ScanPlan: rank order, per-file rank slots)
        HIP_OK(c, c->d_uinfo.ensure(2 * nunits));
        HIP_OK(c, c->d_uslots.ensure(nunits));
        HIP_OK(c, c->d_plan.ensure(kPlanWords));
        HIP_OK(c, c->d_rslots.ensure((size_t)nfiles * kRankSlots));
        HIP_OK(c, hipMemsetAsync(c->d_plan.p, 0, kPlanWords * sizeof(uint32_t), st));
        HIP_OK(c, hipMemsetAsync(c->d_rslots.p, 0, (size_t)nfiles * kRankSlots * sizeof(uint32_t), st));
        HIP_OK(c, c->d_planhdr.ensure(1));
        const ScanPlan hdr{c->d_uslots.p, c->d_plan.p, c->d_uinfo.p, c->d_rslots.p, c->d_offs.p,
                           (uint64_t)p.min_chunk, (uint64_t)p.max_chunk,
                           (unsigned long long*)(c->d_counts.p + 6)};
        HIP_OK(c, launch_scan_plan(c->d_offs.p, nfiles, nbytes, (uint64_t)p.min_chunk, c->ntiles,
                                   c->d_skip.p, c->d_counts.p + 3, c->d_uinfo.p, c->d_uslots.p,
                                   c->d_plan.p, hdr, c->d_planhdr.p, st));
        d_plan = c->d_planhdr.p;
      } else {
        HIP_OK(c, launch_scan_skip(c->d_offs.p, nfiles, nbytes, (uint64_t)p.min_chunk, c->ntiles,
                                   c->d_skip.p, c->d_counts.p + 3, st));
      }
      skip = c->d_skip.p;
    }
    const int grid = scan_grid(c->ntiles, c->num_cus);  // 1 WG per CU (LDS)
    HIP_OK(c, launch_scan(data, c->d_tail.p, nbytes, c->d_table, p.average_bits, c->ntiles,
                          c->d_recs.p, grid, c->d_unit_ctr.p, c->d_unit_ctr.p + 1,
                          c->d_entries.p, c->d_counts.p, c->d_span.p, st, skip, d_plan));
  }
  HIP_OK(c, hipEventRecord(c->ev[1], st));
  HIP_OK(c, hipEventRecord(c->ev[2], st));
  if (nfiles)  // selection + (last workgroup) segment compaction and LPT order
    HIP_OK(c, launch_select(data, c->d_table, c->d_entries.p, c->d_counts.p, c->d_offs.p,
                            c->d_seg_base.p, nfiles, p.average_bits, (uint64_t)p.min_chunk,
                            (uint64_t)p.max_chunk, c->d_slots.p, c->d_nseg.p,
                            c->d_unit_ctr.p + 2, c->d_segs.p, c->d_seg_begin.p, c->d_order.p,
                            c->d_qctr.p, st, bin_bytes, bin_bytes ? c->d_next.p : nullptr,
                            c->d_counts.p + 4));
  // the queue: its length from the selection (bins count once), the bins' successor links
  const uint64_t* qlen = c->d_counts.p + 4;
  const uint32_t* next = bin_bytes ? c->d_next.p : nullptr;
  HIP_OK(c, hipEventRecord(c->ev[3], st));
  // steps in flight on several ctxs: this step's hash starts after the other ctx's last
  // enqueued hash (the scans still overlap the hash tails; two hashes never share the CUs)
  if (c->hash_after && c->hash_after->device == c->device)
    HIP_OK(c, hipStreamWaitEvent(st, c->hash_after->ev[4], 0));
  // a chain-bound launch (one wave per SIMD) keeps its CUs to itself (launch_blake2b); with
  // hash bins the waves of a SIMD share the issue fairly (the PFSCDC_HASH_FAIR knob)
  if (nfiles && !(options & kScanNoHash))
    HIP_OK(c, launch_blake2b(data, c->d_offs.p, c->d_segs.p, qlen, cap,
                             c->d_order.p, c->d_qctr.p, c->num_cus, nbytes, st, true,
                             c->d_span.p + 2, waves, 0u, waves == 1, next,
                             knob(Knob::HashFair) && waves > 1 && next ? c->d_counts.p + 5
                                                                      : nullptr,
                             (uint32_t)knob(Knob::HashFairEvery)));
  HIP_OK(c, hipEventRecord(c->ev[4], st));
  c->have_refs = (options & PFSCDC_OPT_REF_IDS) != 0 && !(options & kScanNoHash);
  if (c->have_refs && nfiles)
    HIP_OK(c, launch_ref_ids(data, c->d_offs.p, c->d_segs.p, qlen, cap,
                             c->d_order.p, c->d_qctr.p + 1, c->num_cus, nbytes, c->d_refs.p,
                             nullptr, st, waves, 0u, next, c->d_seg_begin.p + nfiles));
  HIP_OK(c, hipEventRecord(c->ev[6], st));
  HIP_OK(c, c->h_seg_begin.ensure(nfiles + 1));
  if (nfiles)
    HIP_OK(c, hipMemcpyAsync(c->h_seg_begin.p, c->d_seg_begin.p, sizeof(uint64_t) * (nfiles + 1),
                             hipMemcpyDeviceToHost, st));
  else
    c->h_seg_begin.p[0] = 0;
  c->pending = true;
  return PFSCDC_OK;
}

}  // namespace

extern "C" {

int pfscdc_scan_async(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
                      const uint64_t* file_offsets, uint32_t nfiles) {
  if (!c) return PFSCDC_EINVAL;
  const uint32_t o = c->options;
  const bool cuts = (o & PFSCDC_OPT_CUTS_ONLY) != 0;
  const int rc = scan_async_impl(c, bytes, nbytes, bytes_on_device, file_offsets, nfiles,
                                 (o & ~PFSCDC_OPT_CUTS_ONLY) | (cuts ? kScanNoHash : 0u));
  if (rc == PFSCDC_OK) c->cuts_only = cuts;
  return rc;
}

int pfscdc_wait(pfscdc_ctx* c) { return pfscdc::wait_impl(c, true); }

}  // extern "C"

// fetch = false (a device group's member): the segment records and refs stay on the device
// for the group's gather; only the per-file segment counts come back.
int pfscdc::wait_impl(pfscdc_ctx* c, bool fetch) {
  if (!c) return PFSCDC_EINVAL;
  if (!c->pending) return PFSCDC_OK;
  c->pending = false;
  HIP_OK(c, hipSetDevice(c->device));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  const uint64_t total = c->nfiles ? c->h_seg_begin.p[c->nfiles] : 0;
  if (total > c->slot_cap) return fail(c, PFSCDC_EHIP, "segment count exceeds slot capacity");
  HIP_OK(c, c->h_segs.ensure(total));
  if (total && fetch)
    HIP_OK(c, hipMemcpyAsync(c->h_segs.p, c->d_segs.p, total * sizeof(pfscdc_segment),
                             hipMemcpyDeviceToHost, c->stream));
  if (c->have_refs && fetch) {
    HIP_OK(c, c->h_refs.ensure(total));
    if (total)
      HIP_OK(c, hipMemcpyAsync(c->h_refs.p, c->d_refs.p, total * sizeof(pfscdc_ref),
                               hipMemcpyDeviceToHost, c->stream));
  }
  HIP_OK(c, hipMemcpyAsync(c->h_span.p, c->d_span.p, kSpanSlots * sizeof(uint64_t),
                           hipMemcpyDeviceToHost, c->stream));
  // the rolled-byte count now: later calls on this ctx reuse d_counts
  const bool skipped = c->scan_skipped && c->ntiles;
  if (skipped)  // [3] scanned after the first-min skip, [6] what the settled cuts took off
    HIP_OK(c, hipMemcpyAsync(c->h_span.p + kSpanSlots, c->d_counts.p + 3, 4 * sizeof(uint64_t),
                             hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipEventRecord(c->ev[5], c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  c->scanned_bytes = skipped ? c->h_span.p[kSpanSlots] - c->h_span.p[kSpanSlots + 3] : c->nbytes;
  c->nsegs = total;
  c->scan_valid = fetch;
  c->host_records = fetch;
  return PFSCDC_OK;
}

extern "C" {

int pfscdc_last_kernel_spans(pfscdc_ctx* c, float out[2]) {
  if (!c || !out) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "scan pending");
  if (!c->h_span.p) {  // no scan yet (spans are recorded by pfscdc_scan only)
    out[0] = out[1] = 0.f;
    return PFSCDC_OK;
  }
  const double ticks_per_ms = c->wall_khz;  // kHz = ticks per ms
  for (int k = 0; k < 2; k++) {
    const uint64_t a = c->h_span.p[2 * k], b = c->h_span.p[2 * k + 1];
    out[k] = (b > a && a != ~0ULL) ? (float)((double)(b - a) / ticks_per_ms) : 0.f;
  }
  return PFSCDC_OK;
}

int pfscdc_last_kernel_clocks(pfscdc_ctx* c, float out[2]) {
  if (!c || !out) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "scan pending");
  out[0] = out[1] = 0.f;
  if (!c->h_span.p) return PFSCDC_OK;
  for (int k = 0; k < 2; k++) {  // sum of wave lifetimes: shader cycles / 100 MHz ticks
    const uint64_t cyc = c->h_span.p[4 + 2 * k], ticks = c->h_span.p[5 + 2 * k];
    out[k] = ticks ? (float)((double)cyc / (double)ticks * (c->wall_khz / 1000.0)) : 0.f;
  }
  return PFSCDC_OK;
}

int pfscdc_scan(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
                const uint64_t* file_offsets, uint32_t nfiles) {
  int rc = pfscdc_scan_async(c, bytes, nbytes, bytes_on_device, file_offsets, nfiles);
  if (rc) return rc;
  return pfscdc_wait(c);
}

uint64_t pfscdc_num_segments(const pfscdc_ctx* c) { return c ? c->nsegs : 0; }

int pfscdc_set_options(pfscdc_ctx* c, uint32_t options) {
  if (!c || (options & ~(PFSCDC_OPT_REF_IDS | PFSCDC_OPT_CUTS_ONLY | PFSCDC_OPT_CTEXT_IN_PLACE)))
    return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "set_options during a pending scan");
  c->options = options;
  return PFSCDC_OK;
}

const pfscdc_ref* pfscdc_refs(const pfscdc_ctx* c) {
  return c && c->have_refs && !c->pending && c->host_records ? c->h_refs.p : nullptr;
}

int pfscdc_last_ref_ms(pfscdc_ctx* c, float* ms) {
  if (!c || !ms) return PFSCDC_EINVAL;
  *ms = 0.f;
  if (c->have_refs) HIP_OK(c, hipEventElapsedTime(ms, c->ev[4], c->ev[6]));
  return PFSCDC_OK;
}
const pfscdc_segment* pfscdc_segments(const pfscdc_ctx* c) {
  return c && c->host_records ? c->h_segs.p : nullptr;
}
const uint64_t* pfscdc_file_segment_begin(const pfscdc_ctx* c) {
  return c ? c->h_seg_begin.p : nullptr;
}

uint64_t pfscdc_debug_candidates(pfscdc_ctx* c, uint64_t* out, uint64_t cap) {
  if (!c || c->pending || !c->ntiles) return 0;
  uint64_t ne = 0;
  if (hipMemcpy(&ne, c->d_counts.p, sizeof ne, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  if (out && cap) {
    const uint64_t k = std::min(ne, cap);
    if (hipMemcpy(out, c->d_entries.p, k * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess)
      return 0;
  }
  return ne;
}

int pfscdc_last_scan_bytes(pfscdc_ctx* c, uint64_t* out) {
  if (!c || !out) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "scan pending");
  *out = c->scanned_bytes;
  return PFSCDC_OK;
}

int pfscdc_last_scan_mode(pfscdc_ctx* c, uint32_t* mode) {
  if (!c || !mode) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "scan pending");
  *mode = c->scan_mode;
  return PFSCDC_OK;
}

int pfscdc_last_timings(pfscdc_ctx* c, float out[5]) {
  if (!c || !out) return PFSCDC_EINVAL;
  HIP_OK(c, hipEventElapsedTime(&out[0], c->ev[0], c->ev[1]));
  HIP_OK(c, hipEventElapsedTime(&out[1], c->ev[1], c->ev[2]));
  HIP_OK(c, hipEventElapsedTime(&out[2], c->ev[2], c->ev[3]));
  HIP_OK(c, hipEventElapsedTime(&out[3], c->ev[3], c->ev[4]));
  HIP_OK(c, hipEventElapsedTime(&out[4], c->ev[0], c->ev[4]));
  return PFSCDC_OK;
}

int pfscdc_get_chunks(pfscdc_ctx* c, const void* ctext, uint64_t nbytes, int ctext_on_device,
                      const uint64_t* chunk_offsets, uint32_t nchunks, const pfscdc_ref* refs,
                      void* ptext, int ptext_on_device, uint8_t* ok) {
  if (!c) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "get_chunks during a pending scan");
  if (!chunk_offsets || (nchunks && (!refs || !ok)) || (nbytes && (!ctext || !ptext)))
    return fail(c, PFSCDC_EINVAL, "NULL argument");
  if (chunk_offsets[0] != 0 || chunk_offsets[nchunks] != nbytes)
    return fail(c, PFSCDC_EINVAL, "chunk_offsets must start at 0 and end at nbytes");
  for (uint32_t i = 0; i < nchunks; i++)
    if (chunk_offsets[i + 1] < chunk_offsets[i])
      return fail(c, PFSCDC_EINVAL, "chunk_offsets must be nondecreasing");
  if (ctext_on_device && ((uintptr_t)ctext & 15))
    return fail(c, PFSCDC_EINVAL, "device ctext must be 16-byte aligned");
  if (nchunks == 0) return PFSCDC_OK;
  c->scan_valid = false;
  HIP_OK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  // one segment record per chunk: file i, offset 0 (the kernels address offs[file] + offset)
  HIP_OK(c, c->h_offs.ensure(nchunks + 1));
  std::memcpy(c->h_offs.p, chunk_offsets, sizeof(uint64_t) * (nchunks + 1));
  HIP_OK(c, c->h_segs.ensure(nchunks));
  for (uint32_t i = 0; i < nchunks; i++) {
    pfscdc_segment& sg = c->h_segs.p[i];
    std::memset(&sg, 0, sizeof sg);
    sg.size = chunk_offsets[i + 1] - chunk_offsets[i];
    sg.file = i;
    sg.flags = PFSCDC_SEG_VALID;
  }
  HIP_OK(c, c->h_refs.ensure(nchunks));
  std::memcpy(c->h_refs.p, refs, sizeof(pfscdc_ref) * nchunks);
  HIP_OK(c, c->d_offs.ensure(nchunks + 1));
  HIP_OK(c, c->d_segs.ensure(nchunks));
  HIP_OK(c, c->d_refs.ensure(nchunks));
  HIP_OK(c, c->d_order.ensure(nchunks));
  HIP_OK(c, c->d_qctr.ensure(2));
  HIP_OK(c, c->d_counts.ensure(4));
  const uint8_t* in;
  if (ctext_on_device) {
    in = (const uint8_t*)ctext;
  } else {
    HIP_OK(c, c->d_data.ensure(nbytes + 64));
    HIP_OK(c, hipMemcpyAsync(c->d_data.p, ctext, nbytes, hipMemcpyHostToDevice, st));
    in = c->d_data.p;
  }
  uint8_t* outp;
  if (ptext_on_device) {
    outp = (uint8_t*)ptext;
  } else {
    HIP_OK(c, c->d_out.ensure(nbytes + 64));
    outp = c->d_out.p;
  }
  HIP_OK(c, c->h_seg_begin.ensure(1));
  c->h_seg_begin.p[0] = nchunks;  // pinned source for the device segment count
  HIP_OK(c, hipMemcpyAsync(c->d_offs.p, c->h_offs.p, sizeof(uint64_t) * (nchunks + 1),
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_segs.p, c->h_segs.p, sizeof(pfscdc_segment) * nchunks,
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_refs.p, c->h_refs.p, sizeof(pfscdc_ref) * nchunks,
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_counts.p + 1, c->h_seg_begin.p, sizeof(uint64_t),
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipEventRecord(c->ev[7], st));
  uint64_t longest = 0;
  for (uint32_t i = 0; i < nchunks; i++) longest = std::max(longest, c->h_segs.p[i].size);
  HIP_OK(c, launch_get(in, c->d_offs.p, c->d_segs.p, c->d_counts.p + 1, nchunks, c->d_order.p,
                       c->d_qctr.p, c->num_cus, nbytes, c->d_refs.p, outp, st,
                       knob_waves(longest, nbytes, c->num_cus)));
  HIP_OK(c, hipEventRecord(c->ev[6], st));
  HIP_OK(c, hipMemcpyAsync(c->h_segs.p, c->d_segs.p, sizeof(pfscdc_segment) * nchunks,
                           hipMemcpyDeviceToHost, st));
  if (!ptext_on_device && nbytes)
    HIP_OK(c, hipMemcpyAsync(ptext, outp, nbytes, hipMemcpyDeviceToHost, st));
  HIP_OK(c, hipStreamSynchronize(st));
  for (uint32_t i = 0; i < nchunks; i++)
    ok[i] = std::memcmp(c->h_segs.p[i].hash, refs[i].id, 32) == 0 ? 1 : 0;
  c->nsegs = 0;  // the scan results were overwritten
  c->have_refs = false;
  c->scan_valid = false;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, c->ev[7], c->ev[6]) == hipSuccess) c->get_ms = ms;
  return PFSCDC_OK;
}

int pfscdc_create_refs(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
                       const uint64_t* chunk_offsets, uint32_t nchunks, uint8_t* content_hashes,
                       const uint8_t* hash_known, pfscdc_ref* refs) {
  if (!c) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "create_refs during a pending scan");
  if (!chunk_offsets || (nchunks && !refs) || (nbytes && !bytes) || (hash_known && !content_hashes))
    return fail(c, PFSCDC_EINVAL, "NULL argument");
  if (chunk_offsets[0] != 0 || chunk_offsets[nchunks] != nbytes)
    return fail(c, PFSCDC_EINVAL, "chunk_offsets must start at 0 and end at nbytes");
  for (uint32_t i = 0; i < nchunks; i++)
    if (chunk_offsets[i + 1] < chunk_offsets[i])
      return fail(c, PFSCDC_EINVAL, "chunk_offsets must be nondecreasing");
  if (bytes_on_device && ((uintptr_t)bytes & 15))
    return fail(c, PFSCDC_EINVAL, "device bytes must be 16-byte aligned");
  if (nchunks == 0) return PFSCDC_OK;
  const uint8_t* data;
  if (bytes_on_device) {
    data = (const uint8_t*)bytes;
  } else {
    HIP_OK(c, hipSetDevice(c->device));
    HIP_OK(c, c->d_data.ensure(nbytes + 64));
    HIP_OK(c, hipMemcpyAsync(c->d_data.p, bytes, nbytes, hipMemcpyHostToDevice, c->stream));
    data = c->d_data.p;
  }
  return create_refs_device(c, data, nbytes, chunk_offsets, nchunks, content_hashes, hash_known,
                            refs);
}

// pfscdc_commit_refs in two chunk sets (PFSCDC_COMMIT_TWO_SETS=0: one union pass over every
// record, then one Ref.Id pass, A/B).  A chunk's Ref.Id needs only its own content hash, and
// the commit's critical path is the longest chunks' two serial chains (content hash, then the
// BLAKE2b of its ciphertext, writer.go:240 + client.go:57).  So the chunks longer than
// PFSCDC_COMMIT_LONG_PCT (default 30) percent of the longest, with every segment inside them,
// form the long set on this ctx's stream: their hashes, then at once their deks, ChaCha20 and
// Ref.Id chains, at issue priority 2.  The rest (segments, content hashes and chunk.Create of
// the shorter chunks) runs on a helper ctx's stream beside them, at one wave per SIMD so the
// long set's launches always find room on every SIMD.  The two sets read and (in place)
// write disjoint bytes.  Returns kOnePass when the chunk list does not allow it.
constexpr int kOnePass = 1;

// PFSCDC_COMMIT_TWO_SETS knob: 0 off, 1 on, -1 (default) auto: on when the commit's chunks
// outnumber the quads of one wave per SIMD (the chunk chains alone then keep the GPU busy past
// the longest chunk's two chains: c4 at two commits per step, 28K chunks, 342 -> 362 GiB/s; at
// one commit, 14K chunks, the one-pass form is faster: 248 vs 230-233 GiB/s,
// profiles/r3/two_sets/)
static bool commit_two_sets(uint32_t nchunks, int num_cus) {
  const int64_t k = knob(Knob::CommitTwoSets);
  if (k >= 0) return k != 0;
  return (uint64_t)nchunks > (uint64_t)num_cus * 4 * 16;
}
// The long set: chunks longer than the PFSCDC_COMMIT_LONG_PCT knob's percentage of the longest
// (c4 G = 2: 10% 335, 20% 305, 30% 362, 35% 356, 40% 338, 50% 305 GiB/s).  Its hash launches
// and its ChaCha20 pass raise their issue priority; the short set runs at one wave per SIMD.
// Measured and rejected (round 3-4, no longer built): the long set hashing only its chunks'
// content chains (331 vs 362 GiB/s), other wave counts for either set, and no priority.

static int commit_refs_two_sets(pfscdc_ctx* c, const uint8_t* data, uint64_t nbytes,
                                const std::vector<uint64_t>& sbeg, const std::vector<uint64_t>& ssz,
                                const uint64_t* co, uint32_t nchunks, uint8_t* content_hashes,
                                const uint8_t* hash_known, pfscdc_ref* refs,
                                uint8_t* segment_hashes, uint8_t* ct) {
  if (!commit_two_sets(nchunks, c->num_cus) || nchunks < 2) return kOnePass;
  const uint64_t m = sbeg.size();
  // the chunk holding each segment; the segment a one-segment chunk's content hash is
  std::vector<uint32_t> seg_chunk(m);
  std::vector<int64_t> known_seg(nchunks, -1);
  for (uint64_t s = 0; s < m; s++) {
    const uint64_t a = sbeg[s], z = ssz[s];
    uint32_t i = (uint32_t)(std::upper_bound(co, co + nchunks, a) - co);
    i = i ? i - 1 : 0;
    while (z > 0 && i > 0 && co[i + 1] <= a) i--;
    if (co[i] > a || a + z > co[i + 1]) return kOnePass;  // not inside one chunk
    seg_chunk[s] = i;
    if (hash_known[i] && known_seg[i] < 0 && a == co[i] && z == co[i + 1] - co[i])
      known_seg[i] = (int64_t)s;
  }
  uint64_t longest = 0;
  for (uint32_t i = 0; i < nchunks; i++) {
    if (hash_known[i] && known_seg[i] < 0) return kOnePass;  // the one-pass form reports it
    longest = std::max(longest, co[i + 1] - co[i]);
  }
  const uint64_t thr = longest * (uint64_t)knob(Knob::CommitLongPct) / 100;
  std::vector<uint8_t> set_of(nchunks);  // 0: long, 1: short
  uint32_t nlong = 0;
  for (uint32_t i = 0; i < nchunks; i++) {
    set_of[i] = co[i + 1] - co[i] > thr ? 0 : 1;
    nlong += set_of[i] == 0;
  }
  if (nlong == 0 || nlong == nchunks) return kOnePass;
  if (!c->aux_stream) {
    HIP_OK(c, hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking));
    for (auto& e : c->xev) HIP_OK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  if (!c->helper && ctx_create_on(&c->params, c->device, c->aux_stream, &c->helper) != PFSCDC_OK) {
    c->helper = nullptr;
    return kOnePass;
  }
  for (auto& e : c->pev)
    if (!e) HIP_OK(c, hipEventCreate(&e));
  pfscdc_ctx* const X[2] = {c, c->helper};
  // any early return below (a HIP error) first drains both streams, so no launch of this call
  // still reads the caller's bytes or the ctxs' buffers after it returns
  struct DrainOnReturn {
    hipStream_t a, b;
    bool armed = true;
    ~DrainOnReturn() {
      if (armed) {
        (void)hipStreamSynchronize(a);
        (void)hipStreamSynchronize(b);
      }
    }
  } drain{c->stream, X[1]->stream};
  // per set: its chunks; its union records (content hashes of its multi-DataRef chunks, then
  // every segment inside its chunks)
  std::vector<uint32_t> sel[2], rec_chunk[2];
  std::vector<uint64_t> rec_seg[2];
  for (uint32_t i = 0; i < nchunks; i++) {
    sel[set_of[i]].push_back(i);
    if (!hash_known[i]) rec_chunk[set_of[i]].push_back(i);
  }
  for (uint64_t s = 0; s < m; s++) rec_seg[set_of[seg_chunk[s]]].push_back(s);
  HIP_OK(c, hipEventRecord(c->pev[0], c->stream));  // the scan and the bytes are ready
  HIP_OK(c, hipStreamWaitEvent(X[1]->stream, c->pev[0], 0));
  for (int x = 0; x < 2; x++) {
    pfscdc_ctx* u = X[x];
    hipStream_t st = u->stream;
    const uint64_t kc = rec_chunk[x].size(), R = kc + rec_seg[x].size();
    HIP_OK(c, u->h_segs.ensure(R ? R : 1));
    HIP_OK(c, u->h_offs.ensure(1));
    HIP_OK(c, u->h_seg_begin.ensure(1));
    HIP_OK(c, u->d_offs.ensure(1));
    HIP_OK(c, u->d_segs.ensure(R ? R : 1));
    HIP_OK(c, u->d_order.ensure(R ? R : 1));
    HIP_OK(c, u->d_qctr.ensure(2));
    HIP_OK(c, u->d_counts.ensure(4));
    u->h_offs.p[0] = 0;
    u->h_seg_begin.p[0] = R;
    uint64_t lg = 0, sum = 0;
    for (uint64_t r = 0; r < R; r++) {
      pfscdc_segment& g = u->h_segs.p[r];
      std::memset(&g, 0, sizeof g);
      if (r < kc) {
        const uint32_t i = rec_chunk[x][r];
        g.offset = co[i];
        g.size = co[i + 1] - co[i];
      } else {
        const uint64_t s = rec_seg[x][r - kc];
        g.offset = sbeg[s];
        g.size = ssz[s];
      }
      g.flags = PFSCDC_SEG_VALID;
      lg = std::max(lg, g.size);
      sum += g.size;
    }
    HIP_OK(c, hipMemcpyAsync(u->d_offs.p, u->h_offs.p, sizeof(uint64_t), hipMemcpyHostToDevice, st));
    if (R)
      HIP_OK(c, hipMemcpyAsync(u->d_segs.p, u->h_segs.p, sizeof(pfscdc_segment) * R,
                               hipMemcpyHostToDevice, st));
    HIP_OK(c, hipMemcpyAsync(u->d_counts.p + 1, u->h_seg_begin.p, sizeof(uint64_t),
                             hipMemcpyHostToDevice, st));
    const int w = knob_waves(lg, sum, u->num_cus);
    if (R)
      HIP_OK(c, launch_blake2b(data, u->d_offs.p, u->d_segs.p, u->d_counts.p + 1, R, u->d_order.p,
                               u->d_qctr.p, u->num_cus, nbytes, st, false, nullptr,
                               x ? std::min(w, 1) : w, x ? kHashPrioNone : 1u));
    if (R)
      HIP_OK(c, hipMemcpyAsync(u->h_segs.p, u->d_segs.p, sizeof(pfscdc_segment) * R,
                               hipMemcpyDeviceToHost, st));
    HIP_OK(c, hipEventRecord(c->pev[1 + x], st));
  }
  // as each set's hashes land: its content hashes, then its chunk.Create on its own stream
  std::vector<uint8_t> all(nchunks, 1);
  bool done[2] = {false, false};
  while (!done[0] || !done[1]) {
    bool progressed = false;
    for (int x = 0; x < 2; x++) {
      if (done[x]) continue;
      const hipError_t q = hipEventQuery(c->pev[1 + x]);
      if (q == hipErrorNotReady) continue;
      HIP_OK(c, q);
      pfscdc_ctx* u = X[x];
      const uint64_t kc = rec_chunk[x].size();
      for (uint64_t r = 0; r < kc; r++)
        std::memcpy(content_hashes + 32ull * rec_chunk[x][r], u->h_segs.p[r].hash, 32);
      for (uint64_t r = 0; r < rec_seg[x].size(); r++)
        std::memcpy(segment_hashes + 32 * rec_seg[x][r], u->h_segs.p[kc + r].hash, 32);
      for (uint32_t i : sel[x])
        if (hash_known[i])
          std::memcpy(content_hashes + 32ull * i, segment_hashes + 32 * known_seg[i], 32);
      u->cr_wave_cap = x ? 1 : 0;
      u->cr_hash_prio = x ? kHashPrioNone : 1u;
      u->cr_chacha_prio = x == 0;
      u->cr_one_stream = true;  // each set has one stream (two in all)
      const int rc = create_refs_device(u, data, nbytes, co, nchunks, content_hashes, all.data(),
                                        refs, ct, sel[x].data(), (uint32_t)sel[x].size(), false);
      u->cr_wave_cap = 0;
      u->cr_hash_prio = 0;
      u->cr_chacha_prio = false;
      u->cr_one_stream = false;
      if (rc) {
        if (x) c->err = X[1]->err;
        return rc;  // drain waits for both streams
      }
      done[x] = progressed = true;
    }
    if (!progressed && !(done[0] && done[1])) usleep(50);
  }
  const int r1 = create_refs_finish(X[1]);
  const int r0 = create_refs_finish(c);
  if (r1) {
    c->err = X[1]->err;
    return r1;
  }
  if (r0) return r0;
  float ms = 0.f, a = 0.f, b = 0.f;
  for (int x = 0; x < 2; x++)
    if (hipEventElapsedTime(&ms, c->pev[0], c->pev[1 + x]) == hipSuccess) a = std::max(a, ms);
  for (int x = 0; x < 2; x++)
    if (hipEventElapsedTime(&ms, c->pev[0], X[x]->ev[6]) == hipSuccess) b = std::max(b, ms);
  drain.armed = false;  // create_refs_finish waited for both streams
  if (knob(Knob::Trace)) {  // each set's timeline (ms after the scan): hashes, chunk.Create
    float t[4] = {0, 0, 0, 0};
    for (int x = 0; x < 2; x++) {
      (void)hipEventElapsedTime(&t[x], c->pev[0], c->pev[1 + x]);
      (void)hipEventElapsedTime(&t[2 + x], c->pev[0], X[x]->ev[6]);
    }
    fprintf(stderr, "[pfscdc] commit two sets: long %zu chunks %zu segs: hashes %.1f create %.1f | "
            "short %zu chunks %zu segs: hashes %.1f create %.1f ms\n", sel[0].size(),
            rec_seg[0].size(), t[0], t[2], sel[1].size(), rec_seg[1].size(), t[1], t[3]);
  }
  c->create_hash_ms = a;  // both sets' hashes (they overlap the long set's Ref.Id pass)
  c->create_ms = b;
  c->scan_valid = false;
  c->nsegs = 0;
  c->have_refs = false;
  return PFSCDC_OK;
}

int pfscdc_commit_refs(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
                       const uint64_t* chunk_offsets, uint32_t nchunks, uint8_t* content_hashes,
                       const uint8_t* hash_known, pfscdc_ref* refs, uint8_t* segment_hashes) {
  if (!c) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "commit_refs during a pending scan");
  if (!c->scan_valid || !c->cuts_only || !c->dev_data)
    return fail(c, PFSCDC_ESTATE, "commit_refs needs the last scan made with PFSCDC_OPT_CUTS_ONLY");
  // refs == NULL: the content-hash half only (every BLAKE2b of writer.go:240,301-312, no
  // chunk.Create)
  if (!chunk_offsets || (nchunks && (!content_hashes || !hash_known)) ||
      (c->nsegs && !segment_hashes))
    return fail(c, PFSCDC_EINVAL, "NULL argument");
  if (nbytes != c->nbytes || (bytes_on_device && (const uint8_t*)bytes != c->dev_data))
    return fail(c, PFSCDC_EINVAL, "commit_refs must get the bytes of the last scan");
  const bool in_place = (c->options & PFSCDC_OPT_CTEXT_IN_PLACE) != 0;
  if (in_place && !bytes_on_device)
    return fail(c, PFSCDC_EINVAL, "PFSCDC_OPT_CTEXT_IN_PLACE needs the caller's device bytes");
  if (chunk_offsets[0] != 0 || chunk_offsets[nchunks] != nbytes)
    return fail(c, PFSCDC_EINVAL, "chunk_offsets must start at 0 and end at nbytes");
  for (uint32_t i = 0; i < nchunks; i++)
    if (chunk_offsets[i + 1] < chunk_offsets[i])
      return fail(c, PFSCDC_EINVAL, "chunk_offsets must be nondecreasing");
  HIP_OK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  const uint8_t* data = c->dev_data;  // the scan's device copy (or the caller's device bytes)
  // the scan's segments as absolute ranges (the ctx buffers are reused below)
  const uint64_t m = c->nsegs;
  std::vector<uint64_t> sbeg(m), ssz(m);
  for (uint64_t s = 0; s < m; s++) {
    const pfscdc_segment& g = c->h_segs.p[s];
    sbeg[s] = c->h_offs.p[g.file] + g.offset;
    ssz[s] = g.size;
  }
  // the record set-up below overwrites h_segs/h_offs (and in place, the caller's bytes): a
  // retry after any error from here on must be refused, not run on the overwritten arrays
  c->scan_valid = false;
  c->nsegs = 0;
  if (refs) {
    // a ciphertext buffer both chunk sets write (in place: the plaintext itself)
    uint8_t* ct = in_place ? const_cast<uint8_t*>(data) : nullptr;
    size_t free_b = 0, total_b = 0;
    if (!ct && (c->d_ctext.cap >= nbytes ||
                (hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
                 free_b + c->d_ctext.cap >= nbytes + (8ull << 30))) &&
        c->d_ctext.ensure(nbytes ? nbytes : 1, true) == hipSuccess)
      ct = c->d_ctext.p;
    if (ct) {
      const int rc = commit_refs_two_sets(c, data, nbytes, sbeg, ssz, chunk_offsets, nchunks,
                                          content_hashes, hash_known, refs, segment_hashes, ct);
      if (rc != kOnePass) return rc;
    }
  }
  // one record list: the chunks whose content hash is unknown, then every segment; all
  // absolute (file 0, offs = {0}), hashed in one LPT-ordered launch
  uint32_t k = 0;
  for (uint32_t i = 0; i < nchunks; i++) k += hash_known[i] ? 0 : 1;
  const uint64_t R = k + m;
  if (R > 0xffffffffull) return fail(c, PFSCDC_EUNSUPPORTED, "too many records");
  HIP_OK(c, c->h_segs.ensure(R ? R : 1));
  HIP_OK(c, c->h_offs.ensure(1));
  c->h_offs.p[0] = 0;
  uint64_t longest = 0, sum = 0;
  {
    uint64_t r = 0;
    auto put = [&](uint64_t start, uint64_t size, uint32_t tag) {
      pfscdc_segment& g = c->h_segs.p[r++];
      std::memset(&g, 0, sizeof g);
      g.offset = start;
      g.size = size;
      g.file = 0;
      g.flags = PFSCDC_SEG_VALID;
      (void)tag;
      longest = std::max(longest, size);
      sum += size;
    };
    for (uint32_t i = 0; i < nchunks; i++)
      if (!hash_known[i]) put(chunk_offsets[i], chunk_offsets[i + 1] - chunk_offsets[i], i);
    for (uint64_t s = 0; s < m; s++) put(sbeg[s], ssz[s], 0);
  }
  HIP_OK(c, c->d_offs.ensure(1));
  HIP_OK(c, c->d_segs.ensure(R ? R : 1));
  HIP_OK(c, c->d_order.ensure(R ? R : 1));
  HIP_OK(c, c->d_qctr.ensure(2));
  HIP_OK(c, c->d_counts.ensure(4));
  HIP_OK(c, c->h_seg_begin.ensure(1));
  c->h_seg_begin.p[0] = R;
  HIP_OK(c, hipMemcpyAsync(c->d_offs.p, c->h_offs.p, sizeof(uint64_t), hipMemcpyHostToDevice, st));
  if (R)
    HIP_OK(c, hipMemcpyAsync(c->d_segs.p, c->h_segs.p, sizeof(pfscdc_segment) * R,
                             hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_counts.p + 1, c->h_seg_begin.p, sizeof(uint64_t),
                           hipMemcpyHostToDevice, st));
  hipEvent_t e0 = c->ev[7], e1 = c->cev;  // create_refs_device records them again below
  HIP_OK(c, hipEventRecord(e0, st));
  if (R)
    HIP_OK(c, launch_blake2b(data, c->d_offs.p, c->d_segs.p, c->d_counts.p + 1, R, c->d_order.p,
                             c->d_qctr.p, c->num_cus, nbytes, st, false, nullptr,
                             knob_waves(longest, sum, c->num_cus)));
  HIP_OK(c, hipEventRecord(e1, st));
  if (R)
    HIP_OK(c, hipMemcpyAsync(c->h_segs.p, c->d_segs.p, sizeof(pfscdc_segment) * R,
                             hipMemcpyDeviceToHost, st));
  HIP_OK(c, hipStreamSynchronize(st));
  float pass_ms = 0.f;
  HIP_OK(c, hipEventElapsedTime(&pass_ms, e0, e1));
  for (uint64_t s = 0; s < m; s++) std::memcpy(segment_hashes + 32 * s, c->h_segs.p[k + s].hash, 32);
  // content hashes: computed, or (one-segment chunks) the segment's, matched by range
  {
    uint32_t r = 0;
    uint64_t s = 0;
    for (uint32_t i = 0; i < nchunks; i++) {
      const uint64_t a = chunk_offsets[i], z = chunk_offsets[i + 1] - a;
      if (!hash_known[i]) {
        std::memcpy(content_hashes + 32ull * i, c->h_segs.p[r++].hash, 32);
        continue;
      }
      while (s < m && (sbeg[s] < a || (sbeg[s] == a && ssz[s] != z))) s++;
      if (s == m || sbeg[s] != a || ssz[s] != z)
        return fail(c, PFSCDC_EINVAL, "a hash_known chunk is not one segment of the scan");
      std::memcpy(content_hashes + 32ull * i, segment_hashes + 32 * s, 32);
    }
  }
  c->scan_valid = false;
  c->nsegs = 0;
  if (!refs) {  // content hashes only
    c->have_refs = false;
    c->create_hash_ms = pass_ms;
    c->create_ms = pass_ms;
    return PFSCDC_OK;
  }
  std::vector<uint8_t> all(nchunks, 1);
  // in place: the ciphertext goes over the plaintext (every hash that reads it is done)
  const int rc = create_refs_device(c, data, nbytes, chunk_offsets, nchunks, content_hashes,
                                    all.data(), refs,
                                    in_place ? const_cast<uint8_t*>(data) : nullptr);
  c->create_hash_ms = pass_ms;  // the union pass (DataRef + content hashes)
  c->create_ms += pass_ms;
  return rc;
}

int pfscdc_hash_data_refs(pfscdc_ctx* c, const uint8_t* hashes, uint32_t n, uint8_t out[32]) {
  // hashDataRefs (fileset/util.go:149-158): BLAKE2b-256 of the concatenated DataRef hashes,
  // one record through the hash kernel
  if (!c || !out || (n && !hashes)) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "hash_data_refs during a pending scan");
  const uint64_t nb = 32ull * n;
  c->scan_valid = false;
  HIP_OK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  HIP_OK(c, c->d_data.ensure(nb + 64));
  HIP_OK(c, c->h_offs.ensure(2));
  HIP_OK(c, c->h_segs.ensure(1));
  HIP_OK(c, c->h_seg_begin.ensure(1));
  HIP_OK(c, c->d_offs.ensure(2));
  HIP_OK(c, c->d_segs.ensure(1));
  HIP_OK(c, c->d_order.ensure(1));
  HIP_OK(c, c->d_qctr.ensure(2));
  HIP_OK(c, c->d_counts.ensure(4));
  c->h_offs.p[0] = 0;
  c->h_offs.p[1] = nb;
  std::memset(c->h_segs.p, 0, sizeof(pfscdc_segment));
  c->h_segs.p[0].size = nb;
  c->h_segs.p[0].flags = PFSCDC_SEG_VALID;
  c->h_seg_begin.p[0] = 1;
  if (nb) HIP_OK(c, hipMemcpyAsync(c->d_data.p, hashes, nb, hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_offs.p, c->h_offs.p, 2 * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_segs.p, c->h_segs.p, sizeof(pfscdc_segment), hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_counts.p + 1, c->h_seg_begin.p, sizeof(uint64_t),
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, launch_blake2b(c->d_data.p, c->d_offs.p, c->d_segs.p, c->d_counts.p + 1, 1,
                           c->d_order.p, c->d_qctr.p, c->num_cus, nb, st, false, nullptr, 1));
  HIP_OK(c, hipMemcpyAsync(c->h_segs.p, c->d_segs.p, sizeof(pfscdc_segment), hipMemcpyDeviceToHost, st));
  HIP_OK(c, hipStreamSynchronize(st));
  std::memcpy(out, c->h_segs.p[0].hash, 32);
  c->nsegs = 0;
  c->have_refs = false;
  return PFSCDC_OK;
}

int pfscdc_candidates(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
                      uint64_t halo, uint64_t* out, uint64_t cap, uint64_t* n) {
  // The block-parallel half of Writer.roll (writer.go:163-189) for one range of a stream split
  // across GPUs: the scan and compaction kernels, then the rare dense tiles (more than kTileK
  // candidates in 3 MiB) re-rolled here on the host from the 64-byte windows, exactly.
  if (!c || !n || (cap && !out) || (nbytes && !bytes)) return PFSCDC_EINVAL;
  *n = 0;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "candidates during a pending scan");
  if (bytes_on_device && ((uintptr_t)bytes & 15))
    return fail(c, PFSCDC_EINVAL, "device bytes must be 16-byte aligned");
  if (halo > 64) return fail(c, PFSCDC_EINVAL, "halo must be at most 64 bytes");
  const uint64_t ntiles = (nbytes + kTile - 1) / kTile;
  if (ntiles * (uint64_t)kScanWaves >= (1ull << 32))
    return fail(c, PFSCDC_EUNSUPPORTED, "range too large for one scan (split it)");
  if (nbytes <= halo) return PFSCDC_OK;
  c->scan_valid = false;
  c->nsegs = 0;
  c->have_refs = false;
  HIP_OK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  HIP_OK(c, c->d_recs.ensure(ntiles));
  HIP_OK(c, c->d_unit_ctr.ensure(3));
  HIP_OK(c, c->d_entries.ensure(ntiles * kTileK + 1));
  HIP_OK(c, c->d_counts.ensure(4));
  HIP_OK(c, c->d_tail.ensure(kTailBytes));
  HIP_OK(c, c->d_span.ensure(kSpanSlots));
  const uint8_t* data;
  if (bytes_on_device) {
    data = (const uint8_t*)bytes;
  } else {
    HIP_OK(c, c->d_data.ensure(nbytes + 64));
    HIP_OK(c, hipMemcpyAsync(c->d_data.p, bytes, nbytes, hipMemcpyHostToDevice, st));
    data = c->d_data.p;
  }
  const uint64_t n_main = nbytes & ~63ULL;
  HIP_OK(c, hipMemsetAsync(c->d_tail.p, 0, kTailBytes, st));
  if (nbytes > n_main)
    HIP_OK(c, hipMemcpyAsync(c->d_tail.p, data + n_main, nbytes - n_main, hipMemcpyDeviceToDevice, st));
  HIP_OK(c, hipMemsetAsync(c->d_counts.p, 0, 4 * sizeof(uint64_t), st));
  HIP_OK(c, hipMemsetAsync(c->d_recs.p, 0, sizeof(TileRec) * ntiles, st));
  HIP_OK(c, hipMemsetAsync(c->d_unit_ctr.p, 0, 3 * sizeof(uint32_t), st));
  HIP_OK(c, reset_spans(c, st));
  HIP_OK(c, hipEventRecord(c->ev[0], st));
  const int grid = scan_grid(ntiles, c->num_cus);
  HIP_OK(c, launch_scan(data, c->d_tail.p, nbytes, c->d_table, c->params.average_bits, ntiles,
                        c->d_recs.p, grid, c->d_unit_ctr.p, c->d_unit_ctr.p + 1, c->d_entries.p,
                        c->d_counts.p, c->d_span.p, st));
  HIP_OK(c, hipEventRecord(c->ev[1], st));
  HIP_OK(c, hipEventRecord(c->ev[2], st));
  uint64_t ne = 0;
  HIP_OK(c, hipMemcpyAsync(&ne, c->d_counts.p, sizeof ne, hipMemcpyDeviceToHost, st));
  HIP_OK(c, hipStreamSynchronize(st));
  std::vector<uint64_t> ent(ne);
  if (ne)
    HIP_OK(c, hipMemcpy(ent.data(), c->d_entries.p, ne * sizeof(uint64_t), hipMemcpyDeviceToHost));
  const uint64_t mask = c->params.average_bits >= 64 ? ~0ULL
                                                     : ((1ULL << c->params.average_bits) - 1);
  std::vector<uint8_t> win;
  uint64_t k = 0;
  auto emit = [&](uint64_t p) {
    if (p < halo) return;  // the previous range's bytes
    if (k < cap) out[k] = p;
    k++;
  };
  for (uint64_t e : ent) {
    if (!(e & kDenseBit)) {
      emit(e);
      continue;
    }
    // dense tile: every position of [ts, te] re-rolled from its 64-byte window
    const uint64_t te = e & ~kDenseBit, ts = (te / kTile) * kTile;
    const uint64_t a = ts >= 64 ? ts - 64 : 0;
    win.resize(te + 1 - a);
    HIP_OK(c, hipMemcpy(win.data(), data + a, win.size(), hipMemcpyDeviceToHost));
    auto byte = [&](uint64_t p) -> uint64_t { return p >= a ? win[p - a] : 0; };
    // h_{ts-1} = XOR_k rotl(T[x_{ts-1-k}], k): roll the 64 bytes before ts from a zero state
    // (x_j = 0 before the range start, the reset window)
    uint64_t h = 0;
    for (int64_t i = 0; i < 64; i++) {
      const int64_t p = (int64_t)ts - 64 + i;
      h = ((h << 1) | (h >> 63)) ^ c->table[p >= 0 ? byte((uint64_t)p) : 0];
    }
    for (uint64_t p = ts; p <= te; p++) {
      const uint64_t in = byte(p), outb = p >= 64 ? byte(p - 64) : 0;
      h = ((h << 1) | (h >> 63)) ^ c->table[in] ^ c->table[outb];
      if (p >= 63 && (h & mask) == 0) emit(p);
    }
  }
  *n = k;
  return k > cap ? fail(c, PFSCDC_ENOMEM, "candidate count exceeds cap") : PFSCDC_OK;
}

int pfscdc_hash_ranges(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
                       const uint64_t* begins, const uint64_t* sizes, uint32_t n, uint8_t* out) {
  if (!c || (n && (!begins || !sizes || !out)) || (nbytes && !bytes)) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "hash_ranges during a pending scan");
  for (uint32_t i = 0; i < n; i++)
    if (begins[i] > nbytes || sizes[i] > nbytes - begins[i])
      return fail(c, PFSCDC_EINVAL, "range outside the buffer");
  if (bytes_on_device && ((uintptr_t)bytes & 15))
    return fail(c, PFSCDC_EINVAL, "device bytes must be 16-byte aligned");
  if (n == 0) return PFSCDC_OK;
  const uint8_t* data;
  if (bytes_on_device) {
    data = (const uint8_t*)bytes;
  } else {
    HIP_OK(c, hipSetDevice(c->device));
    HIP_OK(c, c->d_data.ensure(nbytes + 64));
    HIP_OK(c, hipMemcpyAsync(c->d_data.p, bytes, nbytes, hipMemcpyHostToDevice, c->stream));
    data = c->d_data.p;
  }
  HIP_OK(c, hipEventRecord(c->ev[3], c->stream));
  int rc = hash_records_device(c, data, nbytes, begins, sizes, n, out);
  if (rc) return rc;
  HIP_OK(c, hipEventRecord(c->ev[4], c->stream));
  return PFSCDC_OK;
}

int pfscdc_last_create_ms(pfscdc_ctx* c, float* ms) {
  if (!c || !ms) return PFSCDC_EINVAL;
  *ms = c->create_ms;
  return PFSCDC_OK;
}

int pfscdc_last_create_timings(pfscdc_ctx* c, float out[2]) {
  if (!c || !out) return PFSCDC_EINVAL;
  out[0] = c->create_hash_ms;                  // content hashes of multi-DataRef chunks
  out[1] = c->create_ms - c->create_hash_ms;   // order + dek + ChaCha20/BLAKE2b of ctext
  return PFSCDC_OK;
}

int pfscdc_last_get_ms(pfscdc_ctx* c, float* ms) {
  if (!c || !ms) return PFSCDC_EINVAL;
  *ms = c->get_ms;
  return PFSCDC_OK;
}

void* pfscdc_host_alloc(uint64_t nbytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, nbytes ? nbytes : 1, hipHostMallocDefault) != hipSuccess) return nullptr;
  return p;
}

void pfscdc_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int pfscdc_fill_synthetic_pieces(pfscdc_ctx* c, void* dev_bytes, const uint64_t* piece_offsets,
                                 uint32_t npieces, const uint32_t* file_ids,
                                 const uint64_t* file_starts, uint64_t seed, uint32_t mode) {
  if (!c || !piece_offsets || (!dev_bytes && npieces && piece_offsets[npieces]))
    return PFSCDC_EINVAL;
  if (mode > PFSCDC_SYNTH_DEDUP_FILES) return PFSCDC_EINVAL;
  if (c->pending) return fail(c, PFSCDC_ESTATE, "fill during a pending scan");
  if (npieces == 0 || piece_offsets[npieces] == 0) return PFSCDC_OK;
  c->scan_valid = false;
  HIP_OK(c, hipSetDevice(c->device));
  HIP_OK(c, c->h_offs.ensure(npieces + 1));
  HIP_OK(c, c->d_offs.ensure(npieces + 1));
  std::memcpy(c->h_offs.p, piece_offsets, sizeof(uint64_t) * (npieces + 1));
  HIP_OK(c, hipMemcpyAsync(c->d_offs.p, c->h_offs.p, sizeof(uint64_t) * (npieces + 1),
                           hipMemcpyHostToDevice, c->stream));
  const uint32_t* ids = nullptr;
  const uint64_t* starts = nullptr;
  if (file_ids) {
    HIP_OK(c, c->d_ids.ensure(npieces));
    HIP_OK(c, hipMemcpy(c->d_ids.p, file_ids, sizeof(uint32_t) * npieces, hipMemcpyHostToDevice));
    ids = c->d_ids.p;
  }
  if (file_starts) {
    HIP_OK(c, c->d_starts.ensure(npieces));
    HIP_OK(c, hipMemcpy(c->d_starts.p, file_starts, sizeof(uint64_t) * npieces,
                        hipMemcpyHostToDevice));
    starts = c->d_starts.p;
  }
  HIP_OK(c, launch_synth((uint8_t*)dev_bytes, c->d_offs.p, npieces, ids, starts, seed, mode,
                         c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  return PFSCDC_OK;
}

int pfscdc_fill_synthetic_ex(pfscdc_ctx* c, void* dev_bytes, const uint64_t* file_offsets,
                             uint32_t nfiles, uint64_t seed, uint32_t mode) {
  return pfscdc_fill_synthetic_pieces(c, dev_bytes, file_offsets, nfiles, nullptr, nullptr, seed,
                                      mode);
}

int pfscdc_fill_synthetic(pfscdc_ctx* c, void* dev_bytes, const uint64_t* file_offsets,
                          uint32_t nfiles, uint64_t seed) {
  return pfscdc_fill_synthetic_ex(c, dev_bytes, file_offsets, nfiles, seed, PFSCDC_SYNTH_RANDOM);
}

}  // extern "C"

namespace pfscdc {

int ctx_device(const pfscdc_ctx* c) { return c->device; }
hipError_t ctx_group_buffers(pfscdc_ctx* c, uint64_t bytes, bool ctext, uint8_t** d,
                             uint8_t** dct) {
  hipError_t e = c->d_group.ensure(bytes);
  if (e == hipSuccess && ctext) e = c->d_group_ct.ensure(bytes);
  *d = e == hipSuccess ? c->d_group.p : nullptr;
  *dct = e == hipSuccess && ctext ? c->d_group_ct.p : nullptr;
  return e;
}
uint32_t ctx_options(const pfscdc_ctx* c) { return c->options; }
bool ctx_scan_valid(const pfscdc_ctx* c) { return c->scan_valid && !c->pending; }
uint32_t ctx_nfiles(const pfscdc_ctx* c) { return c->nfiles; }
uint64_t ctx_file_offset(const pfscdc_ctx* c, uint32_t f) { return c->h_offs.p[f]; }
void ctx_device_results(const pfscdc_ctx* c, pfscdc_segment** segs, pfscdc_ref** refs,
                        uint64_t* n) {
  *segs = c->d_segs.p;
  *refs = c->have_refs ? c->d_refs.p : nullptr;
  *n = c->nsegs;
}
hipStream_t ctx_stream(const pfscdc_ctx* c) { return c->stream; }

int scan_sync(pfscdc_ctx* c, const void* bytes, uint64_t nbytes, int bytes_on_device,
              const uint64_t* file_offsets, uint32_t nfiles, uint32_t options) {
  int rc = scan_async_impl(c, bytes, nbytes, bytes_on_device, file_offsets, nfiles, options);
  if (rc) return rc;
  return pfscdc_wait(c);
}

// BLAKE2b-256 of n byte ranges [begins[i], begins[i] + sizes[i]) of a device buffer (one
// record each, LPT order), into out (32 B per range).  Synchronous.
int hash_records_device(pfscdc_ctx* c, const uint8_t* data, uint64_t nbytes,
                        const uint64_t* begins, const uint64_t* sizes, uint32_t n, uint8_t* out) {
  if (c->pending) return fail(c, PFSCDC_ESTATE, "hash during a pending scan");
  if (n == 0) return PFSCDC_OK;
  c->scan_valid = false;
  HIP_OK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  HIP_OK(c, c->h_offs.ensure(n + 1));
  HIP_OK(c, c->h_segs.ensure(n));
  HIP_OK(c, c->h_seg_begin.ensure(1));
  for (uint32_t i = 0; i < n; i++) {
    c->h_offs.p[i] = begins[i];
    pfscdc_segment& sg = c->h_segs.p[i];
    std::memset(&sg, 0, sizeof sg);
    sg.size = sizes[i];
    sg.file = i;
    sg.flags = PFSCDC_SEG_VALID;
  }
  c->h_offs.p[n] = nbytes;
  c->h_seg_begin.p[0] = n;
  HIP_OK(c, c->d_offs.ensure(n + 1));
  HIP_OK(c, c->d_segs.ensure(n));
  HIP_OK(c, c->d_order.ensure(n));
  HIP_OK(c, c->d_qctr.ensure(2));
  HIP_OK(c, c->d_counts.ensure(4));
  HIP_OK(c, hipMemcpyAsync(c->d_offs.p, c->h_offs.p, sizeof(uint64_t) * (n + 1),
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_segs.p, c->h_segs.p, sizeof(pfscdc_segment) * n,
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_counts.p + 1, c->h_seg_begin.p, sizeof(uint64_t),
                           hipMemcpyHostToDevice, st));
  uint64_t longest = 0, sum = 0;
  for (uint32_t i = 0; i < n; i++) {
    longest = std::max(longest, sizes[i]);
    sum += sizes[i];
  }
  HIP_OK(c, launch_blake2b(data, c->d_offs.p, c->d_segs.p, c->d_counts.p + 1, n, c->d_order.p,
                           c->d_qctr.p, c->num_cus, nbytes, st, false, nullptr,
                           knob_waves(longest, sum, c->num_cus)));
  HIP_OK(c, hipMemcpyAsync(c->h_segs.p, c->d_segs.p, sizeof(pfscdc_segment) * n,
                           hipMemcpyDeviceToHost, st));
  HIP_OK(c, hipStreamSynchronize(st));
  for (uint32_t i = 0; i < n; i++) std::memcpy(out + 32ull * i, c->h_segs.p[i].hash, 32);
  c->nsegs = 0;
  c->have_refs = false;
  return PFSCDC_OK;
}

// Split Ref.Id pass (ChaCha20 in parallel, then BLAKE2b of the ciphertext) when the chunk list
// cannot fill the hash grid's quads, i.e. the pass is bound by its longest chains.  The
// PFSCDC_REFID_SPLIT knob forces either form (0 fused, 1 split).
static bool refid_split(uint32_t n, int num_cus) {
  const int64_t k = knob(Knob::RefIdSplit);
  if (k >= 0) return k != 0;
  const uint64_t quads = (uint64_t)num_cus * 4 * kHashWavesPerSimd * 16;
  return n <= quads;
}

// the long subset of a two-stream Ref.Id pass: chunks longer than 65% of the longest
constexpr uint64_t kRefIdLongPct = 65;

// chunk.Create(ctx, CreateOptions{}, chunk, createFunc) for n chunks of a device buffer
// (transform.go:26-46): dek = Hash(Hash(chunk)) (deriveKey :173-178), id = Hash(ChaCha20_dek
// (chunk)) (cryptoXOR :181-188; the id the chunk client stores it under, client.go:57).
// One record per chunk (file = chunk index, offset 0, over offs).  Chunks whose content hash
// is not known come first so that one hash pass over records [0, k) computes them; the
// Ref.Id pass then runs over all records in its own LPT order.  sel (nullable): only the
// chunks sel[0..nsel) (indices into offs / hashes / known / refs).  finish = false: enqueue
// only; create_refs_finish() waits and fills hashes / refs.
int create_refs_device(pfscdc_ctx* c, const uint8_t* data, uint64_t nbytes, const uint64_t* offs,
                       uint32_t n, uint8_t* hashes, const uint8_t* known, pfscdc_ref* refs,
                       uint8_t* ctext_out, const uint32_t* sel, uint32_t nsel, bool finish) {
  if (c->pending) return fail(c, PFSCDC_ESTATE, "create_refs during a pending scan");
  const uint32_t nr = sel ? nsel : n;  // records
  c->cr = CreatePending{};
  if (nr == 0) return PFSCDC_OK;
  c->scan_valid = false;
  HIP_OK(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  auto chunk_of = [&](uint32_t t) { return sel ? sel[t] : t; };
  c->perm.resize(nr);
  uint32_t k = 0;
  for (uint32_t t = 0; t < nr; t++)
    if (!(known && known[chunk_of(t)])) c->perm[k++] = chunk_of(t);
  for (uint32_t t = 0, r = k; t < nr; t++)
    if (known && known[chunk_of(t)]) c->perm[r++] = chunk_of(t);
  auto size_of = [&](uint32_t i) { return offs[i + 1] - offs[i]; };
  // waves per SIMD and issue priority of this call's launches (commit_refs' two chunk sets on
  // two contexts: one wave per SIMD and no priority for the short set, so the long set's
  // launches always find room and issue first)
  auto waves_for = [&](uint64_t longest, uint64_t sum) {
    const int w = knob_waves(longest, sum, c->num_cus);
    return c->cr_wave_cap > 0 && w > c->cr_wave_cap ? c->cr_wave_cap : w;
  };
  // With every content hash known (pfscdc_commit_refs), a split Ref.Id pass runs on two
  // streams: the chunks longer than half the longest first on the ctx stream (their ChaCha20
  // pass is short, so the serial BLAKE2b chains that bound the pass start right away), the
  // rest on a second stream beside them (its ChaCha20 pass and shorter chains fit in the long
  // chains' shadow).
  // The split point: the long set is the chunks longer than 65% of the longest
  // (kRefIdLongPct).  c4 commit, Ref.Id pass: 50% 230, 65% 208-211, 80% 227,
  // 90% 246 ms, one stream 240 ms: a larger long set lengthens its own ChaCha20 pass, a
  // smaller one leaves rest chains that outlast the longest one (they run at two waves per
  // SIMD, slower than a lone chain).
  uint32_t nl = 0;
  if (k == 0 && nr > 1 && !c->cr_one_stream) {
    uint64_t longest = 0;
    for (uint32_t t = 0; t < nr; t++) longest = std::max(longest, size_of(chunk_of(t)));
    const uint64_t thr = longest * kRefIdLongPct / 100;
    auto is_long = [&](uint32_t i) { return size_of(i) > thr; };
    std::stable_partition(c->perm.begin(), c->perm.end(), is_long);
    for (uint32_t t = 0; t < nr; t++) nl += is_long(chunk_of(t)) ? 1 : 0;
    if (nl == nr) nl = 0;
  }
  HIP_OK(c, c->h_offs.ensure(n + 1));
  std::memcpy(c->h_offs.p, offs, sizeof(uint64_t) * (n + 1));
  HIP_OK(c, c->h_segs.ensure(nr));
  for (uint32_t r = 0; r < nr; r++) {
    const uint32_t i = c->perm[r];
    pfscdc_segment& sg = c->h_segs.p[r];
    std::memset(&sg, 0, sizeof sg);
    sg.size = size_of(i);
    sg.file = i;
    sg.flags = PFSCDC_SEG_VALID;
    if (r >= k) std::memcpy(sg.hash, hashes + 32ull * i, 32);
  }
  HIP_OK(c, c->d_offs.ensure(n + 1));
  HIP_OK(c, c->d_segs.ensure(nr));
  HIP_OK(c, c->d_refs.ensure(nr));
  HIP_OK(c, c->d_order.ensure(nr));
  HIP_OK(c, c->d_qctr.ensure(3));
  HIP_OK(c, c->d_counts.ensure(6));
  HIP_OK(c, c->h_refs.ensure(nr));
  HIP_OK(c, c->h_seg_begin.ensure(4));
  c->h_seg_begin.p[0] = k;  // pinned sources of the device record counts
  c->h_seg_begin.p[1] = nr;
  c->h_seg_begin.p[2] = nl;
  c->h_seg_begin.p[3] = nr - nl;
  HIP_OK(c, hipMemcpyAsync(c->d_offs.p, c->h_offs.p, sizeof(uint64_t) * (n + 1),
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_segs.p, c->h_segs.p, sizeof(pfscdc_segment) * nr,
                           hipMemcpyHostToDevice, st));
  HIP_OK(c, hipMemcpyAsync(c->d_counts.p + 1, c->h_seg_begin.p, 4 * sizeof(uint64_t),
                           hipMemcpyHostToDevice, st));
  uint64_t longest_k = 0, sum_k = 0, longest_n = 0, sum_n = 0;
  for (uint32_t r = 0; r < nr; r++) {
    const uint64_t z = c->h_segs.p[r].size;
    if (r < k) {
      longest_k = std::max(longest_k, z);
      sum_k += z;
    }
    longest_n = std::max(longest_n, z);
    sum_n += z;
  }
  HIP_OK(c, hipEventRecord(c->ev[7], st));
  if (k)
    HIP_OK(c, launch_blake2b(data, c->d_offs.p, c->d_segs.p, c->d_counts.p + 1, k, c->d_order.p,
                             c->d_qctr.p, c->num_cus, nbytes, st, false, nullptr,
                             waves_for(longest_k, sum_k), c->cr_hash_prio));
  HIP_OK(c, hipEventRecord(c->cev, st));
  // Ref.Id = Hash(ChaCha20_dek(chunk)).  Fused (the quad computes each block's keystream on
  // its BLAKE2b chain) when the chunks fill the GPU; split into a parallel ChaCha20 pass and
  // a plain BLAKE2b pass over the ciphertext when they do not, so the serial chain of the
  // longest chunk carries only BLAKE2b (about half the per-block latency).
  uint8_t* ct = ctext_out;
  // the ciphertext over the plaintext (PFSCDC_OPT_CTEXT_IN_PLACE) always takes the split form:
  // the fused kernel reads its plaintext and writes its ciphertext through two __restrict__
  // pointers, which must not alias (the PFSCDC_REFID_SPLIT knob cannot force it here)
  const bool in_place = ct != nullptr && ct == data;
  bool split = in_place || refid_split(nr, c->num_cus);
  if (split && !ct) {
    // a ciphertext copy of the whole input, only with room to spare (the fused pass needs
    // none, and other contexts on the device need theirs)
    size_t free_b = 0, total_b = 0;
    if (c->d_ctext.cap < nbytes &&
        (hipMemGetInfo(&free_b, &total_b) != hipSuccess ||
         free_b + c->d_ctext.cap < nbytes + (8ull << 30)))
      split = false;
    else if (c->d_ctext.ensure(nbytes ? nbytes : 1, true) == hipSuccess)
      ct = c->d_ctext.p;
    else
      split = false;
  }
  if (split) {
    // 64-B block prefix per record subset: [0, nl) from h_blk[0], [nl, nr) from h_blk[nl + 1]
    HIP_OK(c, c->h_blk.ensure(nr + 2));
    HIP_OK(c, c->d_blk.ensure(nr + 2));
    HIP_OK(c, c->d_segs2.ensure(nr));
    HIP_OK(c, c->h_segs2.ensure(nr));
    uint64_t longest_a = 0, sum_a = 0, longest_b = 0, sum_b = 0;
    c->h_blk.p[0] = 0;
    for (uint32_t r = 0; r < nl; r++) {
      const uint64_t z = c->h_segs.p[r].size;
      c->h_blk.p[r + 1] = c->h_blk.p[r] + (z + 63) / 64;
      longest_a = std::max(longest_a, z);
      sum_a += z;
    }
    c->h_blk.p[nl + 1] = 0;
    for (uint32_t r = nl; r < nr; r++) {
      const uint64_t z = c->h_segs.p[r].size;
      c->h_blk.p[r + 2] = c->h_blk.p[r + 1] + (z + 63) / 64;
      longest_b = std::max(longest_b, z);
      sum_b += z;
    }
    HIP_OK(c, hipMemcpyAsync(c->d_blk.p, c->h_blk.p, sizeof(uint64_t) * (nr + 2),
                             hipMemcpyHostToDevice, st));
    HIP_OK(c, launch_deks(c->d_segs.p, c->d_counts.p + 2, nr, c->d_refs.p, c->d_qctr.p + 1, st));
    // subset [r0, r0 + m) on stream s: ChaCha20 into ct, then BLAKE2b of the ciphertext
    // (pb: where the subset's block prefix starts in h_blk / d_blk)
    auto chacha_pass = [&](uint32_t r0, uint32_t m, uint32_t pb, hipStream_t s) {
      return launch_chacha_xor(data, c->d_offs.p, c->d_segs.p + r0, c->d_blk.p + pb, m,
                               c->h_blk.p[pb + m], c->d_refs.p + r0, ct, c->num_cus, s,
                               c->cr_chacha_prio, c->cr_wave_cap > 0);
    };
    auto refid_pass = [&](uint32_t r0, uint32_t m, uint32_t pb, const uint64_t* d_count,
                          uint32_t* ctr, uint64_t longest, uint64_t sum, hipStream_t s,
                          uint32_t prio, bool chacha) -> hipError_t {
      hipError_t e = chacha ? chacha_pass(r0, m, pb, s) : hipSuccess;
      if (e == hipSuccess)
        e = hipMemcpyAsync(c->d_segs2.p + r0, c->d_segs.p + r0, sizeof(pfscdc_segment) * m,
                           hipMemcpyDeviceToDevice, s);
      if (e == hipSuccess)
        e = launch_blake2b(ct, c->d_offs.p, c->d_segs2.p + r0, d_count, m, c->d_order.p + r0,
                           ctr, c->num_cus, nbytes, s, false, nullptr, waves_for(longest, sum),
                           c->cr_hash_prio ? c->cr_hash_prio : prio);
      return e;
    };
    if (nl) {
      if (!c->aux_stream) {
        HIP_OK(c, hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking));
        for (auto& e : c->xev) HIP_OK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      }
      // the long chunks' ChaCha20 pass has the GPU to itself; then their BLAKE2b chains start
      // while the rest's ChaCha20 pass and chains run beside them on the second stream, the
      // long chains' waves issuing first on every SIMD they share (s_setprio 2 while a quad
      // has more than one block left)
      HIP_OK(c, chacha_pass(0, nl, 0, st));
      HIP_OK(c, hipEventRecord(c->xev[0], st));
      HIP_OK(c, hipStreamWaitEvent(c->aux_stream, c->xev[0], 0));
      HIP_OK(c, refid_pass(0, nl, 0, c->d_counts.p + 3, c->d_qctr.p + 1, longest_a, sum_a, st,
                           1u, false));
      HIP_OK(c, refid_pass(nl, nr - nl, nl + 1, c->d_counts.p + 4, c->d_qctr.p + 2, longest_b,
                           sum_b, c->aux_stream, 0u, true));
      HIP_OK(c, hipEventRecord(c->xev[1], c->aux_stream));
      HIP_OK(c, hipStreamWaitEvent(st, c->xev[1], 0));
    } else {
      HIP_OK(c, refid_pass(0, nr, 1, c->d_counts.p + 2, c->d_qctr.p + 1, longest_n, sum_n, st,
                           0u, true));
    }
  } else {
    HIP_OK(c, launch_order(c->d_segs.p, c->d_counts.p + 2, c->d_order.p, c->d_qctr.p + 1, st));
    HIP_OK(c, launch_ref_ids(data, c->d_offs.p, c->d_segs.p, c->d_counts.p + 2, nr, c->d_order.p,
                             c->d_qctr.p + 1, c->num_cus, nbytes, c->d_refs.p, ctext_out, st,
                             waves_for(longest_n, sum_n), c->cr_hash_prio));
  }
  HIP_OK(c, hipEventRecord(c->ev[6], st));
  if (hashes && k)
    HIP_OK(c, hipMemcpyAsync(c->h_segs.p, c->d_segs.p, sizeof(pfscdc_segment) * k,
                             hipMemcpyDeviceToHost, st));
  HIP_OK(c, hipMemcpyAsync(c->h_refs.p, c->d_refs.p, sizeof(pfscdc_ref) * nr,
                           hipMemcpyDeviceToHost, st));
  if (split)
    HIP_OK(c, hipMemcpyAsync(c->h_segs2.p, c->d_segs2.p, sizeof(pfscdc_segment) * nr,
                             hipMemcpyDeviceToHost, st));
  c->cr.active = true;
  c->cr.split = split;
  c->cr.k = k;
  c->cr.nr = nr;
  c->cr.hashes = hashes;
  c->cr.refs = refs;
  c->nsegs = 0;  // the scan results are being overwritten
  c->have_refs = false;
  c->scan_valid = false;
  return finish ? create_refs_finish(c) : PFSCDC_OK;
}

// The second half of create_refs_device(finish = false): wait for the ctx stream, then the
// refs (and computed content hashes) of every record into the caller's arrays.
int create_refs_finish(pfscdc_ctx* c) {
  if (!c->cr.active) return PFSCDC_OK;
  const CreatePending p = c->cr;
  c->cr = CreatePending{};
  HIP_OK(c, hipSetDevice(c->device));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  for (uint32_t r = 0; r < p.nr; r++) {
    const uint32_t i = c->perm[r];
    p.refs[i] = c->h_refs.p[r];
    if (p.split) std::memcpy(p.refs[i].id, c->h_segs2.p[r].hash, 32);
    if (p.hashes && r < p.k) std::memcpy(p.hashes + 32ull * i, c->h_segs.p[r].hash, 32);
  }
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, c->ev[7], c->ev[6]) == hipSuccess) c->create_ms = ms;
  if (hipEventElapsedTime(&ms, c->ev[7], c->cev) == hipSuccess) c->create_hash_ms = ms;
  return PFSCDC_OK;
}

}  // namespace pfscdc
