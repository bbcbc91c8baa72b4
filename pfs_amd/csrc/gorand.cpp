// gorand.cpp — rolling-hash table generation for the chunker (product code, host side).
//
// Replaces buzhash64.GenerateHashes(seed) as called by chunk.WithRollingHashConfig
// (/root/reference/src/internal/storage/chunk/option.go:54; data writers seed 1,
// writer.go:41,92; index writers seeds 0,1,2,... fileset/index/writer.go:60,129).
// GenerateHashes draws uint64(rand.Int63()) from Go 1.16 math/rand, skipping duplicates
// (third-party github.com/chmduquesne/rollinghash v4.0.0, assumption A1 in SURVEY.md §8c).
//
// Go's rngSource: additive lagged Fibonacci, lags 607/273 over Z/2^64, seeded by a
// Park-Miller LCG XOR the "cooked" state rngCooked = ALFG state after 7.8e12 steps from
// srand(1).  We regenerate rngCooked by a polynomial jump-ahead x^N mod (x^607 - x^334 - 1)
// rather than embedding Go's table.  ~30 ms once per process, then cached.
#include <array>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <vector>

namespace pfscdc {
namespace {

constexpr int kLen = 607;
constexpr int kTap = 273;
constexpr int32_t kInt32Max = 2147483647;
constexpr uint64_t kCookedSteps = 7800000000000ULL;

int32_t seedrand(int32_t x) {
  // x <- 48271 x mod (2^31 - 1), Schrage's method as in Go.
  const int32_t A = 48271, Q = 44488, R = 3399;
  int32_t hi = x / Q, lo = x % Q;
  x = A * lo - R * hi;
  if (x < 0) x += kInt32Max;
  return x;
}

void lcg_fill(int64_t seed, int sh0, int sh1, uint64_t* vec) {
  seed = seed % kInt32Max;  // C++ and Go both truncate toward zero
  if (seed < 0) seed += kInt32Max;
  if (seed == 0) seed = 89482311;
  int32_t x = (int32_t)seed;
  for (int i = -20; i < kLen; i++) {
    x = seedrand(x);
    if (i >= 0) {
      uint64_t u = (uint64_t)(int64_t)x << sh0;
      x = seedrand(x);
      u ^= (uint64_t)(int64_t)x << sh1;
      x = seedrand(x);
      u ^= (uint64_t)(int64_t)x;
      vec[i] = u;
    }
  }
}

using Poly = std::array<uint64_t, kLen>;

Poly mulmod(const Poly& a, const Poly& b) {
  std::vector<uint64_t> c(2 * kLen - 1, 0);
  for (int i = 0; i < kLen; i++) {
    uint64_t ai = a[i];
    if (!ai) continue;
    uint64_t* ci = c.data() + i;
    for (int j = 0; j < kLen; j++) ci[j] += ai * b[j];  // wraps mod 2^64
  }
  for (int k = 2 * kLen - 2; k >= kLen; k--) {  // x^607 = x^334 + 1
    uint64_t ck = c[k];
    if (ck) {
      c[k - kLen] += ck;
      c[k - kTap] += ck;
    }
  }
  Poly r;
  std::memcpy(r.data(), c.data(), sizeof(uint64_t) * kLen);
  return r;
}

Poly xpow(uint64_t n) {
  Poly result{}, base{};
  result[0] = 1;
  base[1] = 1;
  while (n) {
    if (n & 1) result = mulmod(result, base);
    n >>= 1;
    if (n) base = mulmod(base, base);
  }
  return result;
}

const uint64_t* rng_cooked() {
  static uint64_t cooked[kLen];
  static std::once_flag once;
  std::call_once(once, [] {
    uint64_t vec0[kLen];
    lcg_fill(1, 20, 10, vec0);  // gen_cooked.go srand(1)
    // vec[i] of a fresh source holds y_t, t in [-606, 0], t == 334 - i (mod 607)
    uint64_t y0[kLen];
    for (int i = 0; i < kLen; i++) {
      int t = ((kLen - kTap - i) % kLen + kLen) % kLen;
      if (t > 0) t -= kLen;
      y0[t + kLen - 1] = vec0[i];
    }
    const uint64_t n = kCookedSteps;
    Poly c = xpow(n);  // coefficients of y_{n-606}
    uint64_t window[kLen];
    for (int j = 0; j < kLen; j++) {
      uint64_t s = 0;
      for (int k = 0; k < kLen; k++) s += c[k] * y0[k];
      window[j] = s;
      uint64_t top = c[kLen - 1];  // c <- c * x mod P
      for (int k = kLen - 1; k > 0; k--) c[k] = c[k - 1];
      c[0] = top;
      c[kLen - kTap] += top;
    }
    for (int i = 0; i < kLen; i++) {
      // latest step t <= n whose feed index was i: t = n - ((n - (334 - i)) mod 607)
      int64_t d = kLen - kTap - i;
      uint64_t nd = d >= 0 ? n - (uint64_t)d : n + (uint64_t)(-d);
      uint64_t t = n - nd % kLen;
      cooked[i] = window[t - (n - (kLen - 1))];
    }
  });
  return cooked;
}

struct Source {
  int tap, feed;
  uint64_t vec[kLen];
  explicit Source(int64_t seed) {
    tap = 0;
    feed = kLen - kTap;
    uint64_t fill[kLen];
    lcg_fill(seed, 40, 20, fill);
    const uint64_t* ck = rng_cooked();
    for (int i = 0; i < kLen; i++) vec[i] = fill[i] ^ ck[i];
  }
  uint64_t uint64() {
    if (--tap < 0) tap += kLen;
    if (--feed < 0) feed += kLen;
    uint64_t x = vec[feed] + vec[tap];
    vec[feed] = x;
    return x;
  }
  int64_t int63() { return (int64_t)(uint64() & 0x7fffffffffffffffULL); }
};

}  // namespace

// buzhash64.GenerateHashes(seed): 256 distinct uint64(Int63()) values (assumption A1).
void generate_hashes(int64_t seed, uint64_t out[256]) {
  static std::mutex mu;
  static std::map<int64_t, std::array<uint64_t, 256>> cache;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(seed);
    if (it != cache.end()) {
      std::memcpy(out, it->second.data(), 256 * sizeof(uint64_t));
      return;
    }
  }
  Source r(seed);
  std::set<uint64_t> used;
  std::array<uint64_t, 256> t{};
  for (int i = 0; i < 256; i++) {
    uint64_t x = (uint64_t)r.int63();
    while (used.count(x)) x = (uint64_t)r.int63();
    used.insert(x);
    t[i] = x;
  }
  std::memcpy(out, t.data(), sizeof t);
  std::lock_guard<std::mutex> g(mu);
  cache[seed] = t;
}

// First n Int63 values of rand.NewSource(seed) (exported for known-answer tests).
void go_int63(int64_t seed, int64_t* out, int n) {
  Source r(seed);
  for (int i = 0; i < n; i++) out[i] = r.int63();
}

}  // namespace pfscdc
