// group.cpp — one process, several GPUs: a device group of contexts (C ABI pfscdc_group_*).
//
// pachd is one process that owns one chunk storage (reference
// src/server/pfs/server/driver.go:110-122), so a commit reaches the GPUs of a node through one
// caller, not one process per GPU.  A group holds one pfscdc_ctx per member device and deals
// the work of one call across them:
//   * a batch of independent files (configs[1], and any Put batch): contiguous file ranges
//     balanced by bytes (pfscdc_deal), each scanned on its member's stream; the per-file
//     results depend on the file's bytes alone (writer.go:125-128 resets hash and seglen at
//     every Annotate), so the dealing never changes a result;
//   * an unordered writer (fileset.cpp, pfscdc_uw_create_group): serialized filesets, each an
//     independent chunk stream (unordered_writer.go:83-122), in groups round robin.
// The gather of the chunk-ref index: every member's segment records (and Refs) stay on its
// device and are copied peer to peer (hipMemcpyPeerAsync: xGMI between MI355X devices, a
// device-local copy when members share a GPU) into one index on the first member's device,
// their member-local file ids rebased there, then brought to the host in one copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include "pfscdc_internal.h"

using namespace pfscdc;

struct pfscdc_group {
  std::vector<pfscdc_ctx*> members;
  std::vector<int> devices;
  int index_device = 0;
  hipStream_t stream = nullptr;  // the gather (index device)
  hipEvent_t ev[2] = {nullptr, nullptr};
  std::string err;
  // the last scan
  std::vector<uint32_t> part_begin;
  std::vector<uint64_t> seg_begin;
  std::vector<float> member_ms;
  float gather_ms = 0.f;
  uint64_t nsegs = 0;
  bool have_refs = false;
  pfscdc_segment* d_index = nullptr;  // on index_device
  pfscdc_ref* d_refs = nullptr;
  uint64_t d_cap = 0;
  pfscdc_segment* h_index = nullptr;  // page-locked
  pfscdc_ref* h_refs = nullptr;
  uint64_t h_cap = 0;
  uint64_t bytes_copied = 0;  // bytes the gather moved (records + refs)
  // pfscdc_group_scan_stream: each member's range of the stream (plus the 64-byte halo in
  // front and up to max_chunk - 1 bytes after, for the segment that straddles its end)
  std::vector<uint8_t*> d_stream;
  std::vector<uint64_t> d_stream_cap;
  std::vector<pfscdc_segment> h_stream_segs;  // the stream form's records (host)
  bool stream_form = false;                    // the last scan was pfscdc_group_scan_stream

  int fail(int code, const std::string& msg) {
    err = msg;
    return code;
  }
  void release_buffers() {
    for (size_t k = 0; k < d_stream.size(); k++)
      if (d_stream[k]) {
        (void)hipSetDevice(devices[k]);
        (void)hipFree(d_stream[k]);
        d_stream[k] = nullptr;
      }
    if (d_index || d_refs) (void)hipSetDevice(index_device);
    if (d_index) (void)hipFree(d_index);
    if (d_refs) (void)hipFree(d_refs);
    if (h_index) (void)hipHostFree(h_index);
    if (h_refs) (void)hipHostFree(h_refs);
    d_index = nullptr;
    d_refs = nullptr;
    h_index = nullptr;
    h_refs = nullptr;
    d_cap = h_cap = 0;
  }
};

namespace {

#define GROUP_HIP(g, expr)                                                                  \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return (g)->fail(e_ == hipErrorOutOfMemory ? PFSCDC_ENOMEM : PFSCDC_EHIP,             \
                       std::string(#expr) + ": " + hipGetErrorString(e_));                  \
  } while (0)

int check_offsets(pfscdc_group* g, const uint64_t* offs, uint32_t nfiles, uint64_t nbytes) {
  if (!offs) return g->fail(PFSCDC_EINVAL, "file_offsets is NULL");
  if (offs[0] != 0 || offs[nfiles] != nbytes)
    return g->fail(PFSCDC_EINVAL, "file_offsets must start at 0 and end at nbytes");
  for (uint32_t f = 0; f < nfiles; f++)
    if (offs[f + 1] < offs[f]) return g->fail(PFSCDC_EINVAL, "file_offsets must be nondecreasing");
  return PFSCDC_OK;
}

// Member k scans files [pb[k], pb[k+1]) from src (its bytes, host or device), keeping the
// records on its device.
int member_scan(pfscdc_ctx* c, const uint8_t* src, int on_device, const uint64_t* offs,
                uint32_t f0, uint32_t f1, float* ms) {
  std::vector<uint64_t> local(f1 - f0 + 1);
  for (uint32_t f = f0; f <= f1; f++) local[f - f0] = offs[f] - offs[f0];
  int rc = pfscdc_scan_async(c, src, local.back(), on_device, local.data(), f1 - f0);
  if (!rc) rc = wait_impl(c, false);
  float t[5] = {0, 0, 0, 0, 0};
  if (!rc && pfscdc_last_timings(c, t) == PFSCDC_OK) *ms = t[4];
  return rc;
}

int ensure_index(pfscdc_group* g, uint64_t n, bool refs) {
  if (n > g->d_cap || (refs && !g->d_refs && n)) {
    GROUP_HIP(g, hipSetDevice(g->index_device));
    const uint64_t want = n + n / 4 + 1;
    if (g->d_index) (void)hipFree(g->d_index);
    if (g->d_refs) (void)hipFree(g->d_refs);
    g->d_index = nullptr;
    g->d_refs = nullptr;
    g->d_cap = 0;
    GROUP_HIP(g, hipMalloc((void**)&g->d_index, want * sizeof(pfscdc_segment)));
    if (refs) GROUP_HIP(g, hipMalloc((void**)&g->d_refs, want * sizeof(pfscdc_ref)));
    g->d_cap = want;
  }
  if (n > g->h_cap || (refs && !g->h_refs && n)) {
    const uint64_t want = n + n / 4 + 1;
    if (g->h_index) (void)hipHostFree(g->h_index);
    if (g->h_refs) (void)hipHostFree(g->h_refs);
    g->h_index = nullptr;
    g->h_refs = nullptr;
    g->h_cap = 0;
    GROUP_HIP(g, hipHostMalloc((void**)&g->h_index, want * sizeof(pfscdc_segment),
                               hipHostMallocDefault));
    if (refs)
      GROUP_HIP(g, hipHostMalloc((void**)&g->h_refs, want * sizeof(pfscdc_ref), hipHostMallocDefault));
    g->h_cap = want;
  }
  return PFSCDC_OK;
}

// The scan of every member (one host thread each: a member's H2D copy from pageable memory
// blocks its thread only), then the gather.
int group_scan(pfscdc_group* g, const uint8_t* host, const void* const* member_bytes,
               const uint64_t* offs, uint32_t nfiles) {
  const uint32_t n = (uint32_t)g->members.size();
  g->stream_form = false;
  const uint32_t* pb = g->part_begin.data();
  g->member_ms.assign(n, 0.f);
  std::vector<int> rcs(n, PFSCDC_OK);
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < n; k++) {
    if (pb[k + 1] == pb[k]) continue;
    const uint8_t* src = host ? host + offs[pb[k]] : (const uint8_t*)member_bytes[k];
    const int on_dev = host ? 0 : 1;
    auto job = [g, k, src, on_dev, offs, pb, &rcs] {
      rcs[k] = member_scan(g->members[k], src, on_dev, offs, pb[k], pb[k + 1], &g->member_ms[k]);
    };
    if (k + 1 == n) {
      job();  // the caller's thread takes the last member
      continue;
    }
    try {
      th.emplace_back(job);
    } catch (const std::system_error&) {
      job();  // no thread to be had: this member runs here, before the next one starts
    }
  }
  for (auto& t : th) t.join();
  for (uint32_t k = 0; k < n; k++)
    if (rcs[k])
      return g->fail(rcs[k], "member " + std::to_string(k) + " (device " +
                                 std::to_string(g->devices[k]) + "): " +
                                 pfscdc_last_error(g->members[k]));
  // the global per-file segment ranges, then the records of every member peer to peer
  g->seg_begin.assign((size_t)nfiles + 1, 0);
  std::vector<uint64_t> base(n + 1, 0);
  g->have_refs = (pfscdc::ctx_options(g->members[0]) & PFSCDC_OPT_REF_IDS) != 0;
  for (uint32_t k = 0; k < n; k++) {
    uint64_t cnt = 0;
    if (pb[k + 1] > pb[k]) {
      const uint64_t* lb = pfscdc_file_segment_begin(g->members[k]);
      for (uint32_t f = pb[k]; f < pb[k + 1]; f++) g->seg_begin[f] = base[k] + lb[f - pb[k]];
      cnt = lb[pb[k + 1] - pb[k]];
    }
    base[k + 1] = base[k] + cnt;
  }
  const uint64_t total = base[n];
  g->seg_begin[nfiles] = total;
  g->nsegs = total;
  int rc = ensure_index(g, total, g->have_refs);
  if (rc) return rc;
  GROUP_HIP(g, hipSetDevice(g->index_device));
  GROUP_HIP(g, hipEventRecord(g->ev[0], g->stream));
  g->bytes_copied = 0;
  for (uint32_t k = 0; k < n; k++) {
    const uint64_t cnt = base[k + 1] - base[k];
    if (!cnt) continue;
    pfscdc_segment* ds = nullptr;
    pfscdc_ref* dr = nullptr;
    uint64_t got = 0;
    ctx_device_results(g->members[k], &ds, &dr, &got);
    if (got != cnt) return g->fail(PFSCDC_EHIP, "member segment count changed");
    GROUP_HIP(g, hipMemcpyPeerAsync(g->d_index + base[k], g->index_device, ds, g->devices[k],
                                    cnt * sizeof(pfscdc_segment), g->stream));
    g->bytes_copied += cnt * sizeof(pfscdc_segment);
    if (g->have_refs && dr) {
      GROUP_HIP(g, hipMemcpyPeerAsync(g->d_refs + base[k], g->index_device, dr, g->devices[k],
                                      cnt * sizeof(pfscdc_ref), g->stream));
      g->bytes_copied += cnt * sizeof(pfscdc_ref);
    }
    GROUP_HIP(g, launch_rebase_files(g->d_index + base[k], cnt, pb[k], g->stream));
  }
  GROUP_HIP(g, hipEventRecord(g->ev[1], g->stream));
  if (total) {
    GROUP_HIP(g, hipMemcpyAsync(g->h_index, g->d_index, total * sizeof(pfscdc_segment),
                                hipMemcpyDeviceToHost, g->stream));
    if (g->have_refs)
      GROUP_HIP(g, hipMemcpyAsync(g->h_refs, g->d_refs, total * sizeof(pfscdc_ref),
                                  hipMemcpyDeviceToHost, g->stream));
  }
  GROUP_HIP(g, hipStreamSynchronize(g->stream));
  GROUP_HIP(g, hipEventElapsedTime(&g->gather_ms, g->ev[0], g->ev[1]));
  return PFSCDC_OK;
}

// Writer.roll's serial cut rule (writer.go:163-189) for one annotation of n bytes over its
// sorted candidate positions: a segment starting at s ends at the first candidate at or past
// s + min - 1 unless s + max - 1 comes first (a forced cut); the rest is the open tail.
void select_stream_cuts(const std::vector<uint64_t>& cands, uint64_t n, uint64_t mn, uint64_t mx,
                        std::vector<pfscdc_segment>* out) {
  uint64_t s = 0;
  for (;;) {
    const uint64_t lo = s + mn - 1, hi = s + mx - 1;
    if (lo >= n) break;
    const auto it = std::lower_bound(cands.begin(), cands.end(), lo);
    const uint64_t cut = (it != cands.end() && *it <= hi) ? *it : hi;
    if (cut >= n) break;
    pfscdc_segment seg{};
    seg.offset = s;
    seg.size = cut + 1 - s;
    seg.flags = PFSCDC_SEG_VALID | PFSCDC_SEG_CUT;
    out->push_back(seg);
    s = cut + 1;
  }
  if (s < n) {
    pfscdc_segment seg{};
    seg.offset = s;
    seg.size = n - s;
    seg.flags = PFSCDC_SEG_VALID;
    out->push_back(seg);
  }
}

// Runs job(k) for every member k with work, one host thread each (the caller's thread takes
// the last), and returns the first member's failure.
template <class F>
int for_members(pfscdc_group* g, const std::vector<char>& busy, F job) {
  const uint32_t n = (uint32_t)g->members.size();
  std::vector<int> rcs(n, PFSCDC_OK);
  std::vector<std::thread> th;
  uint32_t last = n;
  for (uint32_t k = 0; k < n; k++)
    if (busy[k]) last = k;
  for (uint32_t k = 0; k < n; k++) {
    if (!busy[k]) continue;
    auto run = [&, k] { rcs[k] = job(k); };
    if (k == last) {
      run();
      continue;
    }
    try {
      th.emplace_back(run);
    } catch (const std::system_error&) {
      run();
    }
  }
  for (auto& t : th) t.join();
  for (uint32_t k = 0; k < n; k++)
    if (rcs[k])
      return g->fail(rcs[k], "member " + std::to_string(k) + " (device " +
                                 std::to_string(g->devices[k]) + "): " +
                                 pfscdc_last_error(g->members[k]));
  return PFSCDC_OK;
}

}  // namespace

extern "C" {

int pfscdc_group_scan_stream(pfscdc_group* g, const void* bytes, uint64_t nbytes) {
  if (!g) return PFSCDC_EINVAL;
  g->err.clear();
  g->nsegs = 0;
  g->have_refs = false;
  if (nbytes && !bytes) return g->fail(PFSCDC_EINVAL, "bytes is NULL");
  const uint32_t n = (uint32_t)g->members.size();
  const pfscdc_params& p = pfscdc::ctx_params(g->members[0]);
  const uint64_t mx = (uint64_t)p.max_chunk;
  // equal byte ranges, borders on 64-byte boundaries (pfs_amd.distributed.split_stream)
  std::vector<uint64_t> bound(n + 1, 0);
  for (uint32_t r = 1; r < n; r++) {
    const uint64_t b = (uint64_t)(((unsigned __int128)nbytes * r / n) / 64 * 64);
    bound[r] = std::max(bound[r - 1], std::min(b, nbytes));
  }
  bound[n] = nbytes;
  g->part_begin.clear();  // one file split by bytes: no file dealing to report
  g->d_stream.resize(n, nullptr);
  g->d_stream_cap.resize(n, 0);
  std::vector<char> busy(n, 0);
  for (uint32_t k = 0; k < n; k++) busy[k] = bound[k + 1] > bound[k];
  const uint8_t* src = (const uint8_t*)bytes;
  g->member_ms.assign(n, 0.f);
  using clk = std::chrono::steady_clock;
  // 1. every member's candidates, from its bytes plus the halo in front (the bytes after its
  // range, up to max - 1, come along for the hash of the segment that straddles its end)
  std::vector<std::vector<uint64_t>> cands(n);
  std::vector<clk::time_point> t0(n);
  int rc = for_members(g, busy, [&](uint32_t k) -> int {
    t0[k] = clk::now();
    const uint64_t a = bound[k], b = bound[k + 1], h = std::min<uint64_t>(64, a);
    const uint64_t end = std::min<uint64_t>(nbytes, b + mx), len = end - (a - h);
    if (hipSetDevice(g->devices[k]) != hipSuccess) return PFSCDC_EHIP;
    if (len > g->d_stream_cap[k]) {
      if (g->d_stream[k]) (void)hipFree(g->d_stream[k]);
      g->d_stream[k] = nullptr;
      g->d_stream_cap[k] = 0;
      if (hipMalloc((void**)&g->d_stream[k], len) != hipSuccess) return PFSCDC_ENOMEM;
      g->d_stream_cap[k] = len;
    }
    if (hipMemcpy(g->d_stream[k], src + (a - h), len, hipMemcpyHostToDevice) != hipSuccess)
      return PFSCDC_EHIP;
    uint64_t cap = (b - a) / 4096 + 64, got = 0;
    for (;;) {
      cands[k].resize(cap);
      const int r = pfscdc_candidates(g->members[k], g->d_stream[k], (b - a) + h, 1, h,
                                      cands[k].data(), cap, &got);
      if (r == PFSCDC_ENOMEM && got > cap) {
        cap = got;
        continue;
      }
      if (r) return r;
      break;
    }
    cands[k].resize(got);
    for (uint64_t& c : cands[k]) c += a - h;  // stream offsets
    return PFSCDC_OK;
  });
  if (rc) return rc;
  // 2. the serial selection over the gathered, sorted candidates (ranges are in stream order)
  std::vector<uint64_t> all;
  for (const auto& v : cands) all.insert(all.end(), v.begin(), v.end());
  std::vector<pfscdc_segment> segs;
  select_stream_cuts(all, nbytes, (uint64_t)p.min_chunk, mx, &segs);
  // 3. each segment hashed by the member holding its first byte
  std::vector<uint64_t> first(n + 1, 0);
  for (uint32_t k = 0, i = 0; k <= n; k++) {
    while (k < n && i < segs.size() && segs[i].offset < bound[k]) i++;
    first[k] = k < n ? i : segs.size();
  }
  rc = for_members(g, busy, [&](uint32_t k) -> int {
    const uint64_t a = bound[k], h = std::min<uint64_t>(64, a);
    const uint64_t i0 = first[k], i1 = first[k + 1];
    if (i1 > i0) {
      std::vector<uint64_t> begins(i1 - i0), sizes(i1 - i0);
      for (uint64_t i = i0; i < i1; i++) {
        begins[i - i0] = segs[i].offset - (a - h);
        sizes[i - i0] = segs[i].size;
      }
      std::vector<uint8_t> out(32 * (i1 - i0));
      const uint64_t len = std::min<uint64_t>(nbytes, bound[k + 1] + mx) - (a - h);
      const int r = pfscdc_hash_ranges(g->members[k], g->d_stream[k], len, 1, begins.data(),
                                       sizes.data(), (uint32_t)(i1 - i0), out.data());
      if (r) return r;
      for (uint64_t i = i0; i < i1; i++) std::memcpy(segs[i].hash, &out[32 * (i - i0)], 32);
    }
    g->member_ms[k] = std::chrono::duration<float, std::milli>(clk::now() - t0[k]).count();
    return PFSCDC_OK;
  });
  if (rc) return rc;
  g->h_stream_segs.swap(segs);
  g->stream_form = true;
  g->nsegs = g->h_stream_segs.size();
  g->seg_begin.assign({0, g->nsegs});
  g->gather_ms = 0.f;
  g->bytes_copied = 0;
  return PFSCDC_OK;
}

int pfscdc_deal(const uint64_t* offsets, uint32_t nitems, uint32_t nparts, uint32_t* part_begin) {
  if (!offsets || !part_begin || nparts == 0) return PFSCDC_EINVAL;
  for (uint32_t i = 0; i < nitems; i++)
    if (offsets[i + 1] < offsets[i]) return PFSCDC_EINVAL;
  // part r starts at the first item whose prefix reaches r/nparts of the bytes (greedy prefix
  // split; items stay whole and in order)
  const uint64_t o0 = offsets[0], total = offsets[nitems] - o0;
  part_begin[0] = 0;
  for (uint32_t r = 1; r < nparts; r++) {
    const unsigned __int128 t = (unsigned __int128)total * r;
    const uint64_t target = (uint64_t)((t + nparts - 1) / nparts);  // ceil
    uint32_t lo = 0, hi = nitems;  // first i in [0, nitems] with prefix(i) >= target
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (offsets[mid] - o0 >= target) hi = mid;
      else lo = mid + 1;
    }
    part_begin[r] = lo < part_begin[r - 1] ? part_begin[r - 1] : lo;
  }
  part_begin[nparts] = nitems;
  return PFSCDC_OK;
}

int pfscdc_group_create(const pfscdc_params* params, const int* devices, uint32_t n,
                        uint32_t options, pfscdc_group** out) {
  if (!out || !devices || n == 0 || !params) return PFSCDC_EINVAL;
  *out = nullptr;
  if (options & ~PFSCDC_OPT_REF_IDS) return PFSCDC_EINVAL;  // no cuts-only / in-place groups
  pfscdc_group* g = new pfscdc_group();
  for (uint32_t k = 0; k < n; k++) {
    pfscdc_ctx* c = nullptr;
    int rc = pfscdc_ctx_create(params, devices[k], &c);
    if (!rc) rc = pfscdc_set_options(c, options);
    if (rc) {
      if (c) pfscdc_ctx_destroy(c);
      pfscdc_group_destroy(g);
      return rc;
    }
    g->members.push_back(c);
    g->devices.push_back(devices[k]);
  }
  g->index_device = devices[0];
  // direct peer access from the index device to every other member device (xGMI); without it
  // hipMemcpyPeerAsync still works, staged through host memory
  for (uint32_t k = 1; k < n; k++) {
    if (devices[k] == g->index_device) continue;
    int can = 0;
    if (hipDeviceCanAccessPeer(&can, g->index_device, devices[k]) == hipSuccess && can) {
      (void)hipSetDevice(g->index_device);
      const hipError_t e = hipDeviceEnablePeerAccess(devices[k], 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        pfscdc_group_destroy(g);
        return PFSCDC_EHIP;
      }
      (void)hipGetLastError();  // "already enabled" is not an error here
    }
  }
  if (hipSetDevice(g->index_device) != hipSuccess ||
      hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&g->ev[0]) != hipSuccess || hipEventCreate(&g->ev[1]) != hipSuccess) {
    pfscdc_group_destroy(g);
    return PFSCDC_EHIP;
  }
  *out = g;
  return PFSCDC_OK;
}

int pfscdc_group_destroy(pfscdc_group* g) {
  if (!g) return PFSCDC_EINVAL;
  if (g->stream) {
    (void)hipSetDevice(g->index_device);
    (void)hipStreamSynchronize(g->stream);
  }
  g->release_buffers();
  for (auto& e : g->ev)
    if (e) (void)hipEventDestroy(e);
  if (g->stream) (void)hipStreamDestroy(g->stream);
  for (pfscdc_ctx* c : g->members) pfscdc_ctx_destroy(c);
  delete g;
  return PFSCDC_OK;
}

uint32_t pfscdc_group_size(const pfscdc_group* g) { return g ? (uint32_t)g->members.size() : 0; }

pfscdc_ctx* pfscdc_group_ctx(pfscdc_group* g, uint32_t i) {
  return g && i < g->members.size() ? g->members[i] : nullptr;
}

const char* pfscdc_group_last_error(const pfscdc_group* g) { return g ? g->err.c_str() : "null group"; }

int pfscdc_group_scan(pfscdc_group* g, const void* bytes, uint64_t nbytes,
                      const uint64_t* file_offsets, uint32_t nfiles) {
  if (!g) return PFSCDC_EINVAL;
  g->err.clear();
  g->nsegs = 0;
  if (nbytes && !bytes) return g->fail(PFSCDC_EINVAL, "bytes is NULL");
  int rc = check_offsets(g, file_offsets, nfiles, nbytes);
  if (rc) return rc;
  const uint32_t n = (uint32_t)g->members.size();
  g->part_begin.assign(n + 1, 0);
  rc = pfscdc_deal(file_offsets, nfiles, n, g->part_begin.data());
  if (rc) return g->fail(rc, "deal");
  return group_scan(g, (const uint8_t*)bytes, nullptr, file_offsets, nfiles);
}

int pfscdc_group_scan_resident(pfscdc_group* g, const void* const* member_bytes,
                               const uint64_t* file_offsets, uint32_t nfiles,
                               const uint32_t* part_begin) {
  if (!g || !member_bytes) return PFSCDC_EINVAL;
  g->err.clear();
  g->nsegs = 0;
  if (!file_offsets) return g->fail(PFSCDC_EINVAL, "file_offsets is NULL");
  int rc = check_offsets(g, file_offsets, nfiles, file_offsets[nfiles]);
  if (rc) return rc;
  const uint32_t n = (uint32_t)g->members.size();
  g->part_begin.assign(n + 1, 0);
  if (part_begin) {
    if (part_begin[0] != 0 || part_begin[n] != nfiles)
      return g->fail(PFSCDC_EINVAL, "part_begin must run from 0 to nfiles");
    for (uint32_t k = 0; k < n; k++)
      if (part_begin[k + 1] < part_begin[k])
        return g->fail(PFSCDC_EINVAL, "part_begin must be nondecreasing");
    std::memcpy(g->part_begin.data(), part_begin, sizeof(uint32_t) * (n + 1));
  } else {
    rc = pfscdc_deal(file_offsets, nfiles, n, g->part_begin.data());
    if (rc) return g->fail(rc, "deal");
  }
  for (uint32_t k = 0; k < n; k++)
    if (g->part_begin[k + 1] > g->part_begin[k] &&
        file_offsets[g->part_begin[k + 1]] > file_offsets[g->part_begin[k]] && !member_bytes[k])
      return g->fail(PFSCDC_EINVAL, "member " + std::to_string(k) + " has bytes but no buffer");
  return group_scan(g, nullptr, member_bytes, file_offsets, nfiles);
}

uint64_t pfscdc_group_num_segments(const pfscdc_group* g) { return g ? g->nsegs : 0; }

const pfscdc_segment* pfscdc_group_segments(const pfscdc_group* g) {
  if (!g || !g->nsegs) return nullptr;
  return g->stream_form ? g->h_stream_segs.data() : g->h_index;
}

const uint64_t* pfscdc_group_file_segment_begin(const pfscdc_group* g) {
  return g && !g->seg_begin.empty() ? g->seg_begin.data() : nullptr;
}

const pfscdc_ref* pfscdc_group_refs(const pfscdc_group* g) {
  return g && g->have_refs && g->nsegs ? g->h_refs : nullptr;
}

const uint32_t* pfscdc_group_part_begin(const pfscdc_group* g) {
  return g && !g->part_begin.empty() ? g->part_begin.data() : nullptr;
}

int pfscdc_group_index_device(const pfscdc_group* g, const pfscdc_segment** segs,
                              const pfscdc_ref** refs, int* device) {
  if (!g) return PFSCDC_EINVAL;
  if (segs) *segs = g->nsegs && !g->stream_form ? g->d_index : nullptr;
  if (refs) *refs = g->nsegs && g->have_refs && !g->stream_form ? g->d_refs : nullptr;
  if (device) *device = g->index_device;
  return PFSCDC_OK;
}

int pfscdc_group_last_timings(const pfscdc_group* g, float* member_ms, float* gather_ms,
                              uint64_t* gather_bytes) {
  if (!g) return PFSCDC_EINVAL;
  if (member_ms)
    for (size_t k = 0; k < g->members.size(); k++)
      member_ms[k] = k < g->member_ms.size() ? g->member_ms[k] : 0.f;
  if (gather_ms) *gather_ms = g->gather_ms;
  if (gather_bytes) *gather_bytes = g->bytes_copied;
  return PFSCDC_OK;
}

}  // extern "C"
