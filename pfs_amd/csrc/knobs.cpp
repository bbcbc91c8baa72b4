// knobs.cpp — the library's tuning knobs: one table, read from the environment once.
//
// No knob changes a result (chunk boundaries, digests, Refs, indexes): each selects between
// exact forms of the same computation or sizes a host-side pool.  The library reads the
// environment here and nowhere else (tests/test_abi.py checks the sources and the strings of
// the built library against INTEGRATION.md's list), once, the first time a knob is used; from
// then on a knob is a process-wide atomic integer, so pfscdc_set_knob never races with the
// background group writers that read knobs while they launch kernels.
#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <unistd.h>  // environ

#include "pfscdc_internal.h"

namespace pfscdc {
namespace {

struct KnobDef {
  const char* name;
  int64_t def, lo, hi;
};

// Indexed by Knob (pfscdc_internal.h); the order is the enumeration order of pfscdc_knob_info.
constexpr int64_t kMax = (int64_t)1 << 62;
constexpr KnobDef kDefs[(int)Knob::kCount] = {
    {"PFSCDC_SCAN_SKIP", 1, 0, 1},          // skip the first min - 1 bytes of every file
    {"PFSCDC_SCAN_CUTSKIP", 1, 0, 1},       // ... and min - 1 past every settled cut
    {"PFSCDC_SCAN_GRID", 0, 0, 1 << 20},    // scan workgroups cap (0: one per CU)
    {"PFSCDC_HASH_BIN_BYTES", -1, -1, kMax},  // hash bins: -1 auto, 0 none, else bin bytes
    {"PFSCDC_HASH_WAVES", 0, 0, 8},         // hash waves per SIMD (0: by chain length)
    {"PFSCDC_HASH_FAIR", 1, 0, 1},          // fair-share issue priority with hash bins
    {"PFSCDC_HASH_FAIR_EVERY", 256, 8, 65536},  // blocks between fair-share updates
    {"PFSCDC_REFID_SPLIT", -1, -1, 1},      // Ref.Id pass: -1 auto, 0 fused, 1 split
    {"PFSCDC_COMMIT_TWO_SETS", -1, -1, 1},  // commit_refs chunk sets: -1 auto, 0 one, 1 two
    {"PFSCDC_COMMIT_LONG_PCT", 30, 1, 99},  // long set: chunks above this % of the longest
    {"PFSCDC_UW_WORKERS", 1, 1, 8},         // unordered writer: group writers
    {"PFSCDC_UW_INFLIGHT", (int64_t)32 << 30, 0, kMax},  // unordered writer: group bytes
    {"PFSCDC_UW_MIRROR", 1, 0, 1},          // unordered writer: upload during the Puts
    {"PFSCDC_UW_INDEX_GROUPED", 1, 0, 1},   // unordered writer: index levels closed grouped
    {"PFSCDC_UW_ARENA_POOL_BYTES", 40000000000ll, 0, kMax},  // pooled page-locked arenas
    {"PFSCDC_CTX_CACHE", 32, 0, 4096},      // cached writer contexts
    {"PFSCDC_COPY_THREADS", 0, 0, 256},     // Put copy threads (0: up to 16 hardware threads)
    {"PFSCDC_TRACE", 0, 0, 1},              // stage timelines on stderr
};

static_assert(kDefs[(int)Knob::kCount - 1].name != nullptr, "one entry per Knob");

struct Table {
  std::atomic<int64_t> v[(int)Knob::kCount];
  std::atomic<bool> frozen[(int)Knob::kCount];  // read once by a process-wide pool, now fixed
  Table() {
    for (auto& f : frozen) f.store(false, std::memory_order_relaxed);
    for (int i = 0; i < (int)Knob::kCount; i++) {
      const KnobDef& d = kDefs[i];
      int64_t x = d.def;
      const char* e = std::getenv(d.name);
      if (e && *e) {
        char* end = nullptr;
        errno = 0;
        const long long y = std::strtoll(e, &end, 10);
        if (errno || !end || *end || y < d.lo || y > d.hi)
          std::fprintf(stderr, "pfscdc: ignoring %s=%s (want an integer in [%lld, %lld])\n",
                       d.name, e, (long long)d.lo, (long long)d.hi);
        else
          x = y;
      }
      v[i].store(x, std::memory_order_relaxed);
    }
    // a PFSCDC_* variable the table does not hold (a misspelling, or the knob of a removed
    // form) would otherwise be ignored without a word
    for (char** e = environ; e && *e; e++) {
      if (std::strncmp(*e, "PFSCDC_", 7) != 0) continue;
      const char* eq = std::strchr(*e, '=');
      const size_t len = eq ? (size_t)(eq - *e) : std::strlen(*e);
      bool known = false;
      for (int i = 0; i < (int)Knob::kCount && !known; i++)
        known = std::strlen(kDefs[i].name) == len && std::strncmp(kDefs[i].name, *e, len) == 0;
      if (!known)
        std::fprintf(stderr, "pfscdc: ignoring %.*s (not a knob of this library; "
                     "INTEGRATION.md lists them)\n", (int)len, *e);
    }
  }
};

Table& table() {
  static Table* t = new Table();  // magic static: one reader of the environment, ever
  return *t;
}

int find(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < (int)Knob::kCount; i++)
    if (std::strcmp(kDefs[i].name, name) == 0) return i;
  return -1;
}

}  // namespace

int64_t knob(Knob k) { return table().v[(int)k].load(std::memory_order_relaxed); }

int64_t knob_freeze(Knob k) {
  table().frozen[(int)k].store(true, std::memory_order_relaxed);
  return knob(k);
}

}  // namespace pfscdc

extern "C" {

int pfscdc_set_knob(const char* name, int64_t value) {
  const int i = pfscdc::find(name);
  if (i < 0) return PFSCDC_EINVAL;
  const pfscdc::KnobDef& d = pfscdc::kDefs[i];
  if (value < d.lo || value > d.hi) return PFSCDC_EINVAL;
  auto& t = pfscdc::table();
  // a knob a process-wide pool has already read (PFSCDC_COPY_THREADS) can no longer change
  if (t.frozen[i].load(std::memory_order_relaxed) &&
      value != t.v[i].load(std::memory_order_relaxed))
    return PFSCDC_ESTATE;
  t.v[i].store(value, std::memory_order_relaxed);
  return PFSCDC_OK;
}

int pfscdc_get_knob(const char* name, int64_t* value) {
  const int i = pfscdc::find(name);
  if (i < 0 || !value) return PFSCDC_EINVAL;
  *value = pfscdc::table().v[i].load(std::memory_order_relaxed);
  return PFSCDC_OK;
}

const char* pfscdc_knob_info(int i, int64_t* lo, int64_t* hi, int64_t* def) {
  if (i < 0 || i >= (int)pfscdc::Knob::kCount) return nullptr;
  const pfscdc::KnobDef& d = pfscdc::kDefs[i];
  if (lo) *lo = d.lo;
  if (hi) *hi = d.hi;
  if (def) *def = d.def;
  return d.name;
}

}  // extern "C"
