// cdc_kernels.hip — gfx950 kernels of the PFS chunk-ingest path.
//
// Reference path replaced (paths under /root/reference):
//   chunk.Writer.roll            src/internal/storage/chunk/writer.go:163-189  (CDC)
//   buzhash64 Roll/Sum64         third-party rollinghash v4.0.0, writer.go:166-167
//   chunk.Hash / pachhash.Sum    chunk/metadata.go:16-20, pachhash/hash.go:27-30 (BLAKE2b-256)
//   newDataRef hashing           writer.go:240,301-312
//
// Pipeline for one batch (files concatenated in HBM):
//   1. cdc_scan_kernel     every byte: h_i = XOR_{k<64} rotl64(T[x_{i-k}], k), candidate iff
//                          h_i & mask == 0.  Lane = 4 KiB strip, 64-byte halo re-read;
//                          rolling recurrence; T replicated 32x in LDS so ds_read_b64 is
//                          bank-conflict free; per 3 MiB tile (12 waves) <= 15 candidates
//                          appended to a global tile record, or a DENSE count.  Reads 1
//                          byte per file byte; VALU-issue bound in practice.
//   2. compact_kernel      one workgroup: prefix sum over tiles, each tile's offsets sorted
//                          by rank -> sorted candidate list.
//   3. select_kernel       one wave per file: serial cut selection over the sparse list
//                          (writer.go:168,179 min/max rule), dense tiles re-rolled in-wave.
//   4. segcompact_kernel   one workgroup: per-file segment counts -> dense segment list.
//   5. hash_order_kernel   one workgroup: segments sorted longest-first (LPT queue order).
//      blake2b_kernel      resident waves, 4 lanes (a quad) per segment, one BLAKE2b column
//                          each (DPP quad rotations for the diagonal step), message words
//                          through double-buffered LDS; quads pull the next segment from
//                          the queue when one finishes.  VALU-issue bound.
// Why the hash of a cut only needs the last 64 bytes: min >= 64 and hash+seglen reset at
// every Annotate/cut (writer.go:125-128,211), so no eligible position sees the reset window.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "pfscdc_internal.h"

#define PFS_DEV __device__ __forceinline__

namespace pfscdc {

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------

PFS_DEV uint64_t rotl1_64(uint64_t x) { return (x << 1) | (x >> 63); }

// LDS byte address of T[byte j of w] in this lane's copy: (idx << 8) | (lane & 31) * 8.
PFS_DEV uint32_t tab_addr(uint32_t w, uint32_t lane_off, int j) {
  return __builtin_amdgcn_perm(w, lane_off, 0x0c0c0000u | ((4u + (uint32_t)j) << 8));
}

template <typename T>
PFS_DEV T lds_load(const uint8_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const T*>(lds + byte_addr);
}

// LDS read at an absolute LDS byte address (the scan kernel's dynamic LDS starts at 0: it
// declares no static __shared__), so no base add is emitted.
typedef __attribute__((address_space(3))) const uint64_t lds_u64_t;
PFS_DEV uint64_t lds_abs_u64(uint32_t a) { return *(lds_u64_t*)(uintptr_t)a; }

// gfx950 has no v_xor3_b32; v_bitop3_b32 with truth table 0x96 is a 3-input XOR.
PFS_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

PFS_DEV void load64(uint32_t (&w)[16], const uint8_t* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const u32x4 v = __builtin_nontemporal_load(q + i);  // file bytes are read exactly once
    w[4 * i + 0] = v.x;
    w[4 * i + 1] = v.y;
    w[4 * i + 2] = v.z;
    w[4 * i + 3] = v.w;
  }
}

// Wave-uniform min / max of a 32-bit lane value (every lane active).
PFS_DEV uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
    v = u < v ? u : v;
  }
  return __builtin_amdgcn_readfirstlane(v);
}
PFS_DEV uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t u = (uint32_t)__shfl_xor((int)v, o, 64);
    v = u > v ? u : v;
  }
  return __builtin_amdgcn_readfirstlane(v);
}

PFS_DEV uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t lo = __shfl_xor((uint32_t)v, o, 64);
    uint32_t hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    uint64_t u = ((uint64_t)hi << 32) | lo;
    v = u < v ? u : v;
  }
  return v;
}

// ------------------------------------------------------------------------------------------
// 1. candidate scan
// ------------------------------------------------------------------------------------------

// One rolling step: h = rotl(h,1) ^ T[in] ^ T[out]   (buzhash64 Roll with window 64)
#define PFS_ROLL(WIN, WOUT, J)                                                   \
  do {                                                                           \
    const uint64_t ti_ = lds_abs_u64(tab_addr((WIN), lane_off, (J)));            \
    const uint64_t to_ = lds_abs_u64(tab_addr((WOUT), lane_off, (J)));           \
    const uint32_t nl_ = __builtin_amdgcn_alignbit(hl, hh, 31);                  \
    const uint32_t nh_ = __builtin_amdgcn_alignbit(hh, hl, 31);                  \
    hl = xor3(nl_, (uint32_t)ti_, (uint32_t)to_);                                \
    hh = xor3(nh_, (uint32_t)(ti_ >> 32), (uint32_t)(to_ >> 32));                \
  } while (0)

template <bool WIDE>
PFS_DEV uint32_t cand_key(uint32_t hl, uint32_t hh, uint32_t kshift) {
  // zero iff (h & mask) == 0; narrow: bits <= 32, key = hl << (32 - bits)
  if (WIDE) return hl | (hh << kshift);
  return hl << kshift;
}

// Source of the 64-byte block at absolute offset p: the file bytes below n_main (n rounded
// down to 64), else the zero-padded tail copy (so the loop never needs guarded loads).
PFS_DEV const uint8_t* block_src(const uint8_t* data, const uint8_t* tail, uint64_t n_main,
                                 uint64_t p) {
  return p < n_main ? data + p : tail + (p - n_main);
}

// Rare path: a block had a candidate; re-roll it byte by byte from its entry state and
// record exact in-tile offsets (writer.go:167 test, positions >= 63 and < n only).  Bytes
// are re-read from memory so the hot loop's register blocks are never indexed dynamically.
// With a plan, the unit's lowest candidate also goes to its file's rank slot (an agent-scope
// atomic max of kScanUnit - offset, waited for here, so the done bit the unit sets when it
// ends can never be seen without it); the unit's file and rank come from the plan's per-unit
// words, so nothing more is live across the hot loop for this than the plan pointer.
PFS_DEV void record_block(const uint8_t* __restrict__ data,
                                          const uint8_t* __restrict__ tail, uint64_t n_main,
                                          uint64_t h, uint64_t pos, uint64_t n,
                                          uint64_t tile_base, uint64_t mask64,
                                          const uint64_t* __restrict__ table,
                                          TileRec* __restrict__ rec,
                                          const ScanPlan* __restrict__ plan) {
  const uint8_t* in = block_src(data, tail, n_main, pos);
  const uint8_t* out = pos >= 64 ? block_src(data, tail, n_main, pos - 64) : nullptr;
  uint32_t* rslot = nullptr;
  uint64_t unit = pos;
  asm volatile("" : "+v"(unit));  // computed here on the rare path, not hoisted into the hot one
  unit /= kScanUnit;
  if (plan) {
    const uint32_t f = plan->uinfo[2 * unit], rank = plan->uinfo[2 * unit + 1] >> 8;
    if (f != ~0u && rank < kRankSlots) rslot = plan->rslots + (uint64_t)f * kRankSlots + rank;
  }
  for (int t = 0; t < 64; t++) {
    const uint64_t i = pos + t;
    const uint32_t bi = in[t];
    const uint32_t bo = out ? out[t] : 0u;
    h = rotl1_64(h) ^ table[bi] ^ table[bo];
    if ((h & mask64) == 0 && i >= 63 && i < n) {
      // unordered; compact_kernel sorts the tile's offsets (count > kTileK marks it dense)
      const uint32_t k = atomicAdd(&rec->count, 1u);
      if (k < (uint32_t)kTileK) rec->off[k] = (uint32_t)(i - tile_base);
      if (rslot) {
        const uint32_t old = __hip_atomic_fetch_max(
            rslot, (uint32_t)(kScanUnit - (i - unit * kScanUnit)), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(old));  // performed before this wave goes on
      }
    }
  }
}

// Roll 64 positions: IN = this block's 16 dwords, OUT = the block 64 bytes earlier; test all
// 64 positions with one min-reduce and fall into the exact re-roll only if one hit.
// Compile-time loop: f(std::integral_constant<int, I>) for I in [I0, I1).
template <int I, int I1>
struct StaticFor {
  template <class F>
  static PFS_DEV void run(F&& f) {
    if constexpr (I < I1) {
      f(std::integral_constant<int, I>{});
      StaticFor<I + 1, I1>::run(f);
    }
  }
};

// T lookup issued by hand so the waits can be counted exactly (the compiler falls back to
// lgkmcnt(0) around LDS-DMA); consumers sit behind an explicit s_waitcnt + sched_barrier.
PFS_DEV uint64_t lds_read_async(uint32_t a) {
  uint64_t v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

constexpr int kRollAhead = 6;  // bytes of T lookups in flight (2 ds_read_b64 each)
static_assert(kRollAhead >= 1 && 2 * (kRollAhead - 1) <= 15, "lgkmcnt is 4 bits");
#define PFS_ROT1(NL, NH)                                   \
  const uint32_t NL = __builtin_amdgcn_alignbit(hl, hh, 31); \
  const uint32_t NH = __builtin_amdgcn_alignbit(hh, hl, 31);

// Roll 64 positions: IN = this block's 16 dwords, OUT = the block 64 bytes earlier; test all
// 64 positions with one min-reduce and fall into the exact re-roll only if one hit.
#define PFS_ROLL64(IN, OUT, POS)                                                          \
  {                                                                                       \
    const uint32_t hl0 = hl, hh0 = hh;                                                    \
    uint32_t acc = 0xffffffffu;                                                           \
    uint64_t ti_[kRollAhead], to_[kRollAhead];                                            \
    StaticFor<0, kRollAhead>::run([&](auto tc) {                                          \
      constexpr int t = decltype(tc)::value;                                              \
      ti_[t] = lds_read_async(tab_addr(IN[t >> 2], lane_off, t & 3));                     \
      to_[t] = lds_read_async(tab_addr(OUT[t >> 2], lane_off, t & 3));                    \
    });                                                                                   \
    StaticFor<0, 64>::run([&](auto tc) {                                                  \
      constexpr int t = decltype(tc)::value;                                              \
      /* pairs in flight: t .. min(t+K-1, 63); wait until only the younger ones remain */  \
      constexpr int inflight = (64 - t < kRollAhead) ? 64 - t : kRollAhead;               \
      __builtin_amdgcn_s_waitcnt(0xC07F | ((2 * (inflight - 1)) << 8));                   \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      const uint64_t a_ = ti_[t % kRollAhead], b_ = to_[t % kRollAhead];                  \
      PFS_ROT1(nl_, nh_)                                                                  \
      hl = xor3(nl_, (uint32_t)a_, (uint32_t)b_);                                         \
      hh = xor3(nh_, (uint32_t)(a_ >> 32), (uint32_t)(b_ >> 32));                         \
      const uint32_t key = cand_key<WIDE>(hl, hh, kshift);                                \
      acc = acc < key ? acc : key;                                                        \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr (t + kRollAhead < 64) {                                                \
        constexpr int u = t + kRollAhead;                                                 \
        ti_[t % kRollAhead] = lds_read_async(tab_addr(IN[u >> 2], lane_off, u & 3));      \
        to_[t % kRollAhead] = lds_read_async(tab_addr(OUT[u >> 2], lane_off, u & 3));     \
      }                                                                                   \
    });                                                                                   \
    if (__builtin_expect(acc == 0, 0))                                                    \
      record_block(data, tail, n_main, ((uint64_t)hh0 << 32) | hl0, (POS), n, tile_base,  \
                   mask64, table, rec, plan);                                             \
  }

// --- narrow masks (average_bits <= 32): the rolling hash without the outgoing byte -----------
// With g_i = rotl(g_{i-1}, 1) ^ T[x_i] (the hash of everything since a start point), and the
// rotation taken mod 64, h_i = g_i ^ rotl(g_{i-64}, 64) = g_i ^ g_{i-64}: bytes older than the
// window cancel.  So the scan needs one table lookup per byte (T[in]) instead of two, and
// the cut test (h_i & mask) == 0 only needs the low word of g_{i-64}: a 64-entry register
// ring, indexed statically inside the unrolled 64-byte block.  The whole recurrence runs in
// a frame rotated left by kshift = 32 - bits (table entries pre-rotated in LDS; rotation
// commutes with the XORs), which moves the tested bits to the top of the low word: the
// key is then just G_lo ^ ring (one v_bitop3_b32 3-way XOR with the new byte's T_lo),
// min-reduced and compared with 2^kshift, and the new G_lo is written straight into the
// ring slot it replaces (no copy).

// Rare path for the g-form: rebuild h_{pos-1} from the 64 bytes before pos (zeros before the
// stream start = the reset window), then re-roll the block exactly like record_block.
PFS_DEV void record_block_g(const uint8_t* __restrict__ data, const uint8_t* __restrict__ tail,
                            uint64_t n_main, uint64_t pos, uint64_t n, uint64_t tile_base,
                            uint64_t mask64, const uint64_t* __restrict__ table,
                            TileRec* __restrict__ rec, const ScanPlan* __restrict__ plan) {
  uint64_t h = 0;
  if (pos >= 64) {
    const uint8_t* w = block_src(data, tail, n_main, pos - 64);
    for (int k = 0; k < 64; k++) h = rotl1_64(h) ^ table[w[k]];
  } else {
    for (int k = 0; k < 64; k++) h = rotl1_64(h) ^ table[0];
  }
  record_block(data, tail, n_main, h, pos, n, tile_base, mask64, table, rec, plan);
}

constexpr int kGAhead = 10;  // T[in] lookups in flight (one ds_read_b64 each)
static_assert(kGAhead >= 1 && kGAhead - 1 <= 15, "lgkmcnt is 4 bits");
constexpr int kGWait = 2;  // positions per s_waitcnt
static_assert(64 % kGWait == 0 && kGWait <= kGAhead, "wait groups tile the block");

#define PFS_ROLL64G(IN, POS)                                                              \
  {                                                                                       \
    uint32_t acc = 0xffffffffu;                                                           \
    uint64_t ti_[kGAhead];                                                                \
    StaticFor<0, kGAhead>::run([&](auto tc) {                                             \
      constexpr int t = decltype(tc)::value;                                              \
      ti_[t] = lds_read_async(tab_addr(IN[t >> 2], lane_off, t & 3));                     \
    });                                                                                   \
    StaticFor<0, 64>::run([&](auto tc) {                                                  \
      constexpr int t = decltype(tc)::value;                                              \
      /* one wait per kGWait positions: lookups t .. t+kGWait-1 have landed */             \
      if constexpr (t % kGWait == 0) {                                                    \
        constexpr int inflight = (64 - t < kGAhead) ? 64 - t : kGAhead;                   \
        constexpr int keep = inflight > kGWait ? inflight - kGWait : 0;                   \
        __builtin_amdgcn_s_waitcnt(0xC07F | (keep << 8));                                 \
      }                                                                                   \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      const uint64_t a_ = ti_[t % kGAhead];                                               \
      PFS_ROT1(nl_, nh_)                                                                  \
      const uint32_t key = xor3(nl_, (uint32_t)a_, ring[t]);                              \
      ring[t] = nl_ ^ (uint32_t)a_;                                                       \
      hl = ring[t];                                                                       \
      hh = nh_ ^ (uint32_t)(a_ >> 32);                                                    \
      acc = acc < key ? acc : key;                                                        \
      __builtin_amdgcn_sched_barrier(0);                                                  \
      if constexpr (t + kGAhead < 64) {                                                   \
        constexpr int u = t + kGAhead;                                                    \
        ti_[t % kGAhead] = lds_read_async(tab_addr(IN[u >> 2], lane_off, u & 3));         \
      }                                                                                   \
    });                                                                                   \
    if (__builtin_expect(acc < cand_thr, 0))                                              \
      record_block_g(data, tail, n_main, (POS), n, tile_base, mask64, table, rec, plan);  \
  }

// Data staging: a wave owns 64 strips (lane l <-> strip l, kStrip bytes each) and walks
// them 128 bytes at a time.  Per step, 8 LDS-DMA instructions (global_load_lds_dwordx4)
// each fetch one full 128-byte line from 8 strips (8 lines per instruction: the coalesced
// rate; per-lane strip loads touch 64 lines per instruction and run at ~2.1 TB/s), into a
// per-wave 8 KiB LDS image of 64 rows x 128 B.  Chunk c of row r sits in slot c ^ swz(r),
// swz(r) = (r >> 1) & 7, so the row reads (ds_read_b128) are bank-conflict free.
PFS_DEV uint32_t stage_swz(uint32_t r) { return (r >> 1) & 7u; }

template <int BLOCK>
PFS_DEV void compact_tiles(const TileRec* __restrict__ recs, uint64_t ntiles, uint64_t n,
                           uint64_t* __restrict__ entries, uint64_t* __restrict__ n_entries,
                           uint64_t* s_wave);
PFS_DEV bool last_block_done(uint32_t* done_ctr, uint32_t* s_flag);

// Exact kernel execution span for timing (bench roofline): the first wavefront to start
// lowers span[0], the last to finish raises span[1] (s_memrealtime, the constant wall clock;
// vector atomics).  The shader clock the kernel ran at: every wave adds its lifetime in
// shader cycles (s_memtime) to span[4] and in 100 MHz ticks (s_memrealtime) to span[5], so
// clock = span[4] / span[5] x 100 MHz over all waves (DVFS lowers it under load: the VALU
// issue ceiling is priced at this clock, not the nominal one).  span == nullptr: not recorded.
struct SpanClock {
  uint64_t t0, r0;
};
PFS_DEV SpanClock span_begin(uint64_t* span) {
  const SpanClock c{__builtin_amdgcn_s_memtime(), __builtin_amdgcn_s_memrealtime()};
  if (span && threadIdx.x == 0) atomicMin((unsigned long long*)span, (unsigned long long)c.r0);
  return c;
}
PFS_DEV void span_end(uint64_t* span, SpanClock c) {
  if (span && (threadIdx.x & 63) == 0) {
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    atomicMax((unsigned long long*)span + 1, (unsigned long long)r1);
    atomicAdd((unsigned long long*)span + 4, (unsigned long long)(t1 - c.t0));
    atomicAdd((unsigned long long*)span + 5, (unsigned long long)(r1 - c.r0));
  }
}

PFS_DEV uint64_t readlane_u64(uint64_t v, uint32_t lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)lane);
  return ((uint64_t)hi << 32) | lo;
}

// Cut skipping (ScanPlan), at the start of a unit: the unit behind dispatch slot `slot`
// belongs to file f, `rank` units past the unit holding the file's first eligible position
// E = fs + min - 1.  One returning agent-scope atomic per lane reads the file's 64 rank slots
// (a unit's slot holds its done bit and its lowest candidate, set in that order), then the
// wave replays the selection (select_file, writer.go:163-189) over the ranks before this
// one: from a segment's first eligible position lo, its cut is the first candidate at or past
// lo within max - 1 bytes of the segment start, else the forced cut at start + max - 1;
// settled when every rank from lo's up to the cut's has reported.  Each settled cut makes
// the next min - 1 positions dead (the count restarts at the cut, writer.go:167-170, 211).
// The unit skips its strip steps below the first eligible position after the last settled
// cut.  The replay stops at the first unreported rank, at a rank past this unit's, or where a
// rank's lowest candidate lies below lo in lo's own unit (another may follow in that unit);
// every slot value is self-consistent, so a stale read only settles fewer cuts.
PFS_DEV void scan_unit_plan(const ScanPlan* __restrict__ plan, uint64_t slot, uint32_t lane,
                            uint64_t n, uint64_t& unit, uint32_t& skip, uint32_t& fr) {
  const uint4 sl = plan->slots[slot];
  unit = sl.x;
  const uint32_t f = sl.y, rank = sl.z >> 8;
  skip = sl.z & 0xffu;
  fr = f | (rank < 255 ? rank : 255u) << 24;
  if (rank == 0) return;  // nothing of the file before this unit
  const uint32_t v = __hip_atomic_fetch_or(plan->rslots + (uint64_t)f * kRankSlots + lane, 0u,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t fs = plan->offs[f], fe = plan->offs[f + 1];
  const uint64_t mn = plan->min_chunk, mx = plan->max_chunk;
  const uint64_t e = fs + mn - 1, u0 = e / kScanUnit;  // u0: the unit of rank 0
  const uint64_t done_m = __ballot((v & kSlotDone) != 0);
  const uint32_t inv = v & ~kSlotDone;  // kScanUnit - the lowest candidate's offset, 0: none
  const uint64_t cand_m = __ballot(inv != 0);
  const uint64_t cpos = (u0 + lane + 1) * kScanUnit - inv;  // lane q: rank q's lowest candidate
  const uint64_t rlim = rank < kRankSlots ? rank : kRankSlots;
  uint64_t lo = e, hi = fs + mx - 1, d = 0;
  for (uint32_t it = 0; it < kRankSlots; it++) {
    const uint64_t qlo = lo / kScanUnit - u0;  // the rank holding lo
    if (qlo >= rlim) break;
    const uint64_t from = cand_m & (~0ull << qlo);
    const uint32_t qc = from ? (uint32_t)__builtin_ctzll(from) : 64u;
    const uint64_t c = qc < 64 ? readlane_u64(cpos, qc) : ~0ull;
    if (qc == qlo && c < lo) break;  // lo's own unit: a later candidate may follow its lowest
    uint64_t cut, qneed;
    if (c <= hi && c < fe) {
      cut = c;
      qneed = qc;
    } else {
      if (hi >= fe) break;  // the file ends first: no more cuts
      cut = hi;             // forced (writer.go:179)
      qneed = hi / kScanUnit - u0;
    }
    if (qneed >= rlim) break;
    const uint64_t need = (qneed >= 63 ? ~0ull : (2ull << qneed) - 1) & (~0ull << qlo);
    if ((done_m & need) != need) break;
    d = cut + mn;  // the next eligible position
    lo = d;
    hi = cut + mx;
  }
  if (d == 0) return;
  const uint64_t ub = unit * kScanUnit;
  if (d <= ub) return;
  const uint64_t s2 = (d - ub) / kUnitStep;
  const uint32_t ns = s2 < kUnitSteps ? (uint32_t)s2 : kUnitSteps;
  if (ns <= skip) return;
  if (lane == 0) {
    const uint64_t ue = ub + kScanUnit < n ? ub + kScanUnit : n;
    const uint64_t a = ub + skip * kUnitStep, b = ub + ns * kUnitStep;
    atomicAdd(plan->dyn_skipped, (unsigned long long)((b < ue ? b : ue) - a));
  }
  skip = ns;
}

// Cut skipping, at the end of a unit: its done bit into its rank slot (its lowest candidate
// is there already: record_block waited for each update).  No reply is needed.
PFS_DEV void scan_unit_report(const ScanPlan* __restrict__ plan, uint32_t fr, uint32_t lane) {
  const uint32_t f = fr & (kPlanMaxFiles - 1), rank = fr >> 24;
  if (rank >= kRankSlots || lane != 0) return;
  asm volatile("" ::: "memory");
  __hip_atomic_fetch_or(plan->rslots + (uint64_t)f * kRankSlots + rank, kSlotDone,
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool WIDE>
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(kScanWaves / 4, kScanWaves / 4))) void cdc_scan_kernel(
    const uint8_t* __restrict__ data, const uint8_t* __restrict__ tail, uint64_t n,
    const uint64_t* __restrict__ table, uint32_t kshift, uint64_t mask64, uint64_t ntiles,
    TileRec* __restrict__ recs, uint32_t* __restrict__ unit_ctr, uint32_t* __restrict__ done_ctr,
    uint64_t* __restrict__ entries, uint64_t* __restrict__ n_entries,
    const uint32_t* __restrict__ unit_skip, uint64_t* span,
    const ScanPlan* __restrict__ plan) {
  const SpanClock span_clk = span_begin(span);
  // Dynamic LDS only (base address 0): [0, 64 KiB) table copies, then the per-wave staging
  // images.  recs[] is zeroed before the launch; candidates are added to it directly.
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint64_t n_main = n & ~63ULL;

  // T replicated: entry idx of copy c at byte idx*256 + c*8 -> banks {2c, 2c+1}.
  for (int i = threadIdx.x; i < 256 * 32; i += kScanBlock) {
    const int idx = i >> 5, c = i & 31;
    // narrow masks roll in a frame rotated left by kshift = 32 - bits (see PFS_ROLL64G)
    const uint64_t v = table[idx];
    reinterpret_cast<uint64_t*>(smem)[idx * 32 + c] =
        WIDE || kshift == 0 ? v : (v << kshift) | (v >> (64 - kshift));
  }
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const uint32_t lane_off = (lane & 31u) * 8u;
  uint8_t* wbuf = smem + kTableLdsBytes + wave * kStageBytes;
  const uint32_t rd_base = lane * 128u;
  const uint32_t swz_l = stage_swz(lane);
  __syncthreads();  // table copies written; from here on every wave runs on its own

  // Work unit = one wave's 64 strips of a tile.  Each wave takes the next unit from a
  // launch-wide counter (zeroed before the launch), so CUs that start late (another step's
  // hash still draining there) simply take fewer units instead of finishing last.
  // With a plan (cut skipping, ScanPlan in device memory) the counter runs over its
  // rank-ordered slots instead of the units.  The next slot is taken at the end of a unit,
  // before that unit reports to its file, so the two round trips overlap.
  const uint64_t nunits = plan ? (uint64_t)plan->plan[0] : ntiles * (uint64_t)kScanWaves;
  uint32_t u0 = 0;
  if (lane == 0) u0 = atomicAdd(unit_ctr, 1u);
  for (;;) {
    const uint64_t slot = (uint32_t)__builtin_amdgcn_readfirstlane(u0);
    if (slot >= nunits) break;
    uint64_t unit = slot;
    uint32_t skip = 0;
    uint32_t fr = ~0u;  // the file this unit reports to | its rank << 24 (~0u: none)
    if (plan) scan_unit_plan(plan, slot, lane, n, unit, skip, fr);
    const uint64_t tile = unit / kScanWaves;
    const uint64_t wslot = unit % kScanWaves;
    TileRec* const rec = recs + tile;
    const uint64_t tile_base = tile * kTile;
    // Leading 128-byte steps of this unit's strips that hold no eligible position (inside
    // the first min - 1 bytes of a file: scan_skip_kernel); the strips then shrink to cover
    // the rest of the unit.  kStrip / 128 = the whole unit is skipped.
    if (unit_skip && !plan)
      skip = (uint32_t)__builtin_amdgcn_readfirstlane((int)unit_skip[tile * kScanWaves + wslot]);
    const uint32_t nsteps = kStrip / 128 - skip, strip = nsteps * 128u;
    const uint64_t wave_base = tile_base + wslot * 64 * kStrip + (uint64_t)skip * (64 * 128);
    if (nsteps && wave_base < n) {  // wave-uniform
      // this lane's DMA piece in instruction i: row r_i = 8i + lane/8, chunk (lane%8) ^ swz(r_i)
      uint32_t dma_off[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint32_t r = 8u * i + (lane >> 3);
        dma_off[i] = r * strip + 16u * ((lane & 7u) ^ stage_swz(r));
      }
      const bool fast = wave_base + 64 * (uint64_t)strip <= n_main;
      // the unit's bytes as a raw buffer (SGPR descriptor: base = the unit's first byte; every
      // offset is below 256 KiB): the fast path's DMA is buffer_load ... lds with the lane's
      // 32-bit offset and the step in soffset, no 64-bit address add per instruction (8 VALU
      // per 128-B step with global_load_lds)
      const __amdgpu_buffer_rsrc_t unit_rsrc = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(data + wave_base), (short)0, 0x7fffffff, 0x00020000);
      auto dma_step = [&](uint32_t step) {
        if (fast) {  // wave-uniform: descriptor + soffset in SGPRs, LDS dst in M0
#pragma unroll
          for (int i = 0; i < 8; i++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                unit_rsrc, (__attribute__((address_space(3))) void*)(wbuf + i * 1024), 16,
                dma_off[i], step * 128u, 0, 0);
          return;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const uint64_t p = wave_base + dma_off[i] + step * 128u;
          const uint8_t* src = (fast || p < n_main) ? data + p
                               : tail + (p - n_main < 64 ? p - n_main : 64);
          __builtin_amdgcn_global_load_lds((const void*)src,
              (__attribute__((address_space(3))) void*)(wbuf + i * 1024), 16, 0, 0);
        }
      };
      const uint64_t s0 = wave_base + (uint64_t)lane * strip;
      dma_step(0);
      uint32_t prv[16], cur[32];
      if (s0 >= 64 && s0 - 64 < n) {
        load64(prv, block_src(data, tail, n_main, s0 - 64));
      } else {
#pragma unroll
        for (int i = 0; i < 16; i++) prv[i] = 0;  // reset window (writer.go:17-19)
      }
      // Write(window): h = XOR rotl(T[b_j], 63 - j) == h_{s0-1}.  For the g-form the same
      // roll from a zero start point gives g over the halo, and its low words seed the ring.
      uint32_t hl = 0, hh = 0;
      uint32_t ring[64];
#pragma unroll
      for (int t = 0; t < 64; t++) {
        const uint64_t ti = lds_abs_u64(tab_addr(prv[t >> 2], lane_off, t & 3));
        const uint32_t nl = __builtin_amdgcn_alignbit(hl, hh, 31);
        const uint32_t nh = __builtin_amdgcn_alignbit(hh, hl, 31);
        hl = nl ^ (uint32_t)ti;
        hh = nh ^ (uint32_t)(ti >> 32);
        ring[t] = hl;
      }
      // rotated frame: the tested low `bits` bits of h sit at the top of the low word, so a
      // position is a candidate iff (G_lo ^ ring) < 2^kshift, and the block test is a min
      const uint32_t cand_thr = 1u << kshift;
      const bool active = s0 < n;
      for (uint32_t step = 0; step < nsteps; step++) {
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this step's DMA has landed
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = 0; c < 8; c++) {
          const uint4 v = *reinterpret_cast<const uint4*>(wbuf + rd_base + 16u * (c ^ swz_l));
          cur[4 * c + 0] = v.x;
          cur[4 * c + 1] = v.y;
          cur[4 * c + 2] = v.z;
          cur[4 * c + 3] = v.w;
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): row is in registers (WAR vs DMA)
        __builtin_amdgcn_wave_barrier();
        if (step + 1 < nsteps) dma_step(step + 1);    // refill while we compute
        const uint64_t pos = s0 + step * 128u;
        if (active && pos < n) {
          uint32_t* c0 = cur;
          uint32_t* c1 = cur + 16;
          if constexpr (WIDE) {
            PFS_ROLL64(c0, prv, pos)
            if (pos + 64 < n) PFS_ROLL64(c1, c0, pos + 64)
          } else {
            PFS_ROLL64G(c0, pos)
            if (pos + 64 < n) PFS_ROLL64G(c1, pos + 64)
          }
        }
        if constexpr (WIDE) {
#pragma unroll
          for (int i = 0; i < 16; i++) prv[i] = cur[16 + i];
        }
      }
    }
    if (lane == 0) u0 = atomicAdd(unit_ctr, 1u);  // the next unit, in flight during the report
    if (fr != ~0u) scan_unit_report(plan, fr, lane);
  }
  // the last workgroup compacts the tile records into the sorted entry list (the table and
  // staging LDS are free once every wave of the workgroup is past its last unit)
  if (done_ctr) {
    uint32_t* s_flag = reinterpret_cast<uint32_t*>(smem);
    uint64_t* s_wave = reinterpret_cast<uint64_t*>(smem + 64);
    if (last_block_done(done_ctr, s_flag))
      compact_tiles<kScanBlock>(recs, ntiles, n, entries, n_entries, s_wave);
  }
  span_end(span, span_clk);
}

// Which leading part of each scan work unit (a wave's 64 strips, 64 * kStrip bytes) can hold
// no cut.  Writer.roll cuts at position i only when the bytes since the last reset reach min
// (writer.go:167-170: numChunkBytesAnnotation + len(data[offset:i+1]) < min -> continue), and
// the count resets at every Annotate (writer.go:125-128), i.e. at every file start of a batch.
// So the first min - 1 positions of a file are never cut points, whatever the hash says there,
// and select_file never looks at candidates below fs + min - 1.  Per unit, skip[u] = the number
// of leading 128-byte strip steps (8 KiB of the unit each) below the unit's first eligible
// position; kStrip / 128 when the unit has none.  The positions the scan still covers see
// their full 64-byte window (the halo load in front of each strip), so every candidate at an
// eligible position is found exactly as before.  *scanned += the bytes left to scan.
// One thread per unit; a unit spanning more than 64 files is scanned whole.
//
// With uinfo/plan (the cut-skipping scan, ScanPlan; min - 1 >= one unit, so a unit's
// eligible positions all belong to the file holding its first one): uinfo[2u] = that file
// (~0u: the unit is not scanned), uinfo[2u + 1] = skip | rank << 8, rank = the unit's index
// past the unit holding the file's first eligible position; plan[2 + min(rank, 63)] counts
// the units of each rank, and the last workgroup turns the counts into each rank's first
// dispatch slot (plan[0] = the slots used).
__global__ __launch_bounds__(256) void scan_skip_kernel(
    const uint64_t* __restrict__ offs, uint32_t nfiles, uint64_t n, uint64_t min_chunk,
    uint64_t nunits, uint32_t* __restrict__ skip, unsigned long long* __restrict__ scanned,
    uint32_t* __restrict__ uinfo, uint32_t* __restrict__ plan) {
  constexpr uint64_t U = kScanUnit, kStep = kUnitStep;
  constexpr uint32_t kAll = kUnitSteps;
  __shared__ uint32_t s_flag;
  __shared__ uint32_t s_hist[kPlanBuckets];  // this block's units per rank (one global add each)
  if (uinfo && threadIdx.x < kPlanBuckets) s_hist[threadIdx.x] = 0;
  if (uinfo) __syncthreads();
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long live = 0;
  if (u < nunits) {
    const uint64_t ub = u * U, ue = ub + U < n ? ub + U : n;
    uint32_t s = kAll, tf = ~0u, rank = 0;
    if (ub < n) {
      // the file holding ub: the last f < nfiles with offs[f] <= ub (offs[nfiles] = n > ub)
      uint32_t lo = 0, hi = nfiles;
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (offs[mid] <= ub) lo = mid;
        else hi = mid;
      }
      uint32_t f = lo;
      s = 0;  // a unit crowded with files is scanned whole
      for (int k = 0; k < 64; k++, f++) {
        if (f >= nfiles || offs[f] >= ue) {
          s = kAll;
          break;
        }
        const uint64_t ls = offs[f] + min_chunk - 1, fe = offs[f + 1];
        if (ls < fe) {  // the file's first eligible position; later files start beyond it
          const uint64_t first = ls > ub ? ls : ub;
          s = first < ue ? (uint32_t)((first - ub) / kStep) : kAll;
          tf = f;
          rank = (uint32_t)(ub / U - ls / U);  // ls <= first < ue: ls's unit is at most u
          break;
        }
      }
      // A unit crowded with more than 64 file starts and no tracked file: with a plan
      // (min - 1 >= one unit) it has no eligible position at all -- every file past the first
      // starts after ub, so its first eligible position lies past ue -- and it must not take a
      // dispatch slot scan_slots_kernel would never fill.
      if (uinfo && tf == ~0u) s = kAll;
      if (s < kAll && ub + s * kStep >= ue) s = kAll;
      if (s < kAll) live = ue - (ub + s * kStep);
    }
    skip[u] = s;
    if (uinfo) {
      const bool scanned_unit = s < kAll;  // implies tf != ~0u
      uinfo[2 * u] = scanned_unit ? tf : ~0u;
      uinfo[2 * u + 1] = s | (rank < 255 ? rank : 255u) << 8;
      if (scanned_unit) atomicAdd(&s_hist[rank < kPlanBuckets - 1 ? rank : kPlanBuckets - 1], 1u);
    }
  }
  // one atomic per wave
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) live += __shfl_xor(live, o, 64);
  if ((threadIdx.x & 63) == 0 && live) atomicAdd(scanned, live);
  if (!uinfo) return;
  __syncthreads();
  if (threadIdx.x < kPlanBuckets && s_hist[threadIdx.x])
    atomicAdd(&plan[2 + threadIdx.x], s_hist[threadIdx.x]);
  static_assert(kPlanBuckets == 64, "one wave turns the rank counts into first slots");
  if (last_block_done(&plan[1], &s_flag) && threadIdx.x < 64) {
    // each rank's count -> its first slot (a wave-wide exclusive scan)
    const uint32_t c = __hip_atomic_load(&plan[2 + threadIdx.x], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    uint32_t x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
      if ((int)threadIdx.x >= o) x += y;
    }
    plan[2 + threadIdx.x] = x - c;
    if (threadIdx.x == 63) plan[0] = x;
  }
}

// The cut-skipping scan's dispatch slots: every scanned unit at the next slot of its rank, a
// block's units of one rank together (one global add per block and rank, then LDS).
// Thread 0 also stores the plan header the scan kernel reads (its arguments by value here: no
// host copy into device memory, which from pageable memory would block the host).
__global__ __launch_bounds__(256) void scan_slots_kernel(uint64_t nunits,
                                                         const uint32_t* __restrict__ uinfo,
                                                         uint32_t* __restrict__ plan,
                                                         uint4* __restrict__ slots,
                                                         ScanPlan hdr, ScanPlan* __restrict__ d_hdr) {
  __shared__ uint32_t s_cnt[kPlanBuckets], s_base[kPlanBuckets];
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u == 0) *d_hdr = hdr;
  if (threadIdx.x < kPlanBuckets) s_cnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t f = ~0u, sr = 0, b = 0, local = 0;
  if (u < nunits) {
    f = uinfo[2 * u];
    sr = uinfo[2 * u + 1];
    const uint32_t rank = sr >> 8;
    b = rank < kPlanBuckets - 1 ? rank : kPlanBuckets - 1;
    if (f != ~0u) local = atomicAdd(&s_cnt[b], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kPlanBuckets && s_cnt[threadIdx.x])
    s_base[threadIdx.x] = atomicAdd(&plan[2 + threadIdx.x], s_cnt[threadIdx.x]);
  __syncthreads();
  if (f != ~0u) slots[s_base[b] + local] = make_uint4((uint32_t)u, f, sr, 0u);
}

// ------------------------------------------------------------------------------------------
// 2. compaction: tile records -> sorted entry list
// ------------------------------------------------------------------------------------------

// Block-wide exclusive scan (BLOCK threads, BLOCK/64 waves, s_wave[BLOCK/64 + 1] of LDS);
// returns the exclusive prefix and sets *total.
template <int BLOCK>
PFS_DEV uint64_t block_exscan(uint64_t v, uint64_t* s_wave, uint64_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t lo = __shfl_up((uint32_t)x, o, 64);
    const uint32_t hi = __shfl_up((uint32_t)(x >> 32), o, 64);
    if (lane >= o) x += ((uint64_t)hi << 32) | lo;
  }
  if (lane == 63) s_wave[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t run = 0;
    for (int w = 0; w < BLOCK / 64; w++) {
      const uint64_t t = s_wave[w];
      s_wave[w] = run;
      run += t;
    }
    s_wave[BLOCK / 64] = run;
  }
  __syncthreads();
  const uint64_t r = s_wave[wave] + x - v;
  *total = s_wave[BLOCK / 64];
  __syncthreads();
  return r;
}

// "Last workgroup" hand-off for the small serial steps of the pipeline (compaction after
// the scan; segment compaction and the LPT order after the selection): every workgroup
// writes back its stores (device-scope release: buffer_wbl2 on each XCD's L2) and counts
// itself done; the one that counts last acquires (buffer_inv) and runs the step itself.  A
// separate one-workgroup launch would instead wait for a whole free CU behind the other
// step's resident hash waves (15 ms instead of 0.2 ms with two steps in flight).
PFS_DEV bool last_block_done(uint32_t* done_ctr, uint32_t* s_flag) {
  // Every wave waits until its stores have reached its XCD's L2 (vmcnt(0)); after the
  // barrier one thread writes that L2 back and counts the workgroup done (device-scope
  // release: a buffer_wbl2 per workgroup, not one per wave as a __threadfence in every
  // thread would issue); the last workgroup then acquires (invalidates its L2).
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    *s_flag = atomicAdd(done_ctr, 1u) == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  const bool last = *s_flag != 0;
  if (last) __threadfence();
  return last;
}

// Tile records -> sorted entry list (the scan's candidates in stream order).
template <int BLOCK>
PFS_DEV void compact_tiles(const TileRec* __restrict__ recs, uint64_t ntiles, uint64_t n,
                           uint64_t* __restrict__ entries, uint64_t* __restrict__ n_entries,
                           uint64_t* s_wave) {
  uint64_t carry = 0;
  for (uint64_t base = 0; base < ntiles; base += BLOCK) {
    const uint64_t t = base + threadIdx.x;
    uint32_t c = 0;
    uint64_t e = 0;
    if (t < ntiles) {
      c = recs[t].count;
      e = c <= (uint32_t)kTileK ? c : 1;
    }
    uint64_t total;
    const uint64_t ex = block_exscan<BLOCK>(e, s_wave, &total) + carry;
    if (t < ntiles) {
      const uint64_t ts = t * kTile;
      if (c <= (uint32_t)kTileK) {
        // the scan records a tile's offsets in arrival order; place each by its rank
        uint32_t o[kTileK];
#pragma unroll
        for (int i = 0; i < kTileK; i++) o[i] = i < (int)c ? recs[t].off[i] : ~0u;
#pragma unroll
        for (int i = 0; i < kTileK; i++) {
          uint32_t rank = 0;
#pragma unroll
          for (int j = 0; j < kTileK; j++) rank += o[j] < o[i];
          if (i < (int)c) entries[ex + rank] = ts + o[i];
        }
      } else {
        const uint64_t te = (ts + kTile < n) ? ts + kTile : n;
        entries[ex] = kDenseBit | (te - 1);  // sorts as the tile's last byte
      }
    }
    carry += total;
  }
  if (threadIdx.x == 0) *n_entries = carry;
}

__global__ __launch_bounds__(kCompactBlock) void compact_kernel(
    const TileRec* __restrict__ recs, uint64_t ntiles, uint64_t n,
    uint64_t* __restrict__ entries, uint64_t* __restrict__ n_entries) {
  __shared__ uint64_t s_wave[kCompactBlock / 64 + 1];
  compact_tiles<kCompactBlock>(recs, ntiles, n, entries, n_entries, s_wave);
}

// Per-file segment counts -> dense segment list in (file, offset) order; returns the total.
template <int BLOCK>
PFS_DEV uint64_t segcompact_block(const pfscdc_segment* __restrict__ slots,
                                  const uint64_t* __restrict__ seg_base,
                                  const uint64_t* __restrict__ nseg, uint32_t nfiles,
                                  pfscdc_segment* __restrict__ segs,
                                  uint64_t* __restrict__ seg_begin, uint64_t* s_wave) {
  uint64_t carry = 0;
  for (uint64_t base = 0; base < nfiles; base += BLOCK) {
    const uint64_t f = base + threadIdx.x;
    const uint64_t c = f < nfiles ? nseg[f] : 0;
    uint64_t total;
    const uint64_t ex = block_exscan<BLOCK>(c, s_wave, &total) + carry;
    if (f < nfiles) {
      seg_begin[f] = ex;
      const pfscdc_segment* src = slots + seg_base[f];
      for (uint64_t i = 0; i < c; i++) segs[ex + i] = src[i];
    }
    carry += total;
  }
  if (threadIdx.x == 0) seg_begin[nfiles] = carry;
  return carry;
}

// LPT order: segment indices sorted by block count, longest first (counting sort on a 10-bit
// key).  The hash kernel's quads pull segments in this order, so the longest serial chains
// start first and the short ones fill in behind them.
PFS_DEV uint32_t lpt_key(uint64_t size) {
  const uint64_t nblk = (size + 127) / 128;
  const uint64_t k = nblk >> 6;  // 8 KiB granularity
  return 1023u - (uint32_t)(k < 1023 ? k : 1023);  // ascending key = descending length
}

// Hash bins (bin_bytes > 0, next != nullptr): every file of at most bin_bytes is one queue
// entry, its segments hashed back to back by the quad that takes it (next[i] = the file's
// following segment, kNoNext after its last); a larger file's segments are entries of their
// own.  bin_bytes is the launch's bytes per quad, so on many equal files (configs[1]'s
// aggregated steps: 4 MiB files, 4 MiB per quad) every quad gets the same work and the launch
// drains with no quad-level imbalance; where segments outweigh a quad's share nothing changes.
// qlen (nullable): the number of queue entries.
template <int BLOCK>
PFS_DEV void lpt_order_block(const pfscdc_segment* __restrict__ segs, uint64_t n,
                             uint32_t* __restrict__ order, uint32_t* __restrict__ counter,
                             uint32_t* hist, uint64_t* s_wave,
                             const uint64_t* __restrict__ offs = nullptr, uint64_t bin_bytes = 0,
                             uint32_t* __restrict__ next = nullptr, uint64_t* qlen = nullptr) {
  const bool bins = next && offs && bin_bytes;
  auto binned = [&](uint64_t i) {
    const uint32_t f = segs[i].file;
    return bins && offs[f + 1] - offs[f] <= bin_bytes;
  };
  // is segment i a queue entry (a bin's first segment, or a segment alone); its sort key
  auto entry = [&](uint64_t i, uint32_t& key) {
    if (binned(i)) {
      const uint32_t f = segs[i].file;
      key = lpt_key(offs[f + 1] - offs[f]);
      return i == 0 || segs[i - 1].file != f;
    }
    key = lpt_key(segs[i].size);
    return true;
  };
  constexpr int kPer = 1024 / BLOCK;  // histogram bins per thread
  static_assert(1024 % BLOCK == 0, "bins split evenly over the block");
  for (int b = 0; b < kPer; b++) hist[threadIdx.x * kPer + b] = 0;
  __syncthreads();
  for (uint64_t i = threadIdx.x; i < n; i += BLOCK) {
    uint32_t key;
    if (entry(i, key)) atomicAdd(&hist[key], 1u);
    if (bins) next[i] = binned(i) && i + 1 < n && segs[i + 1].file == segs[i].file
                            ? (uint32_t)(i + 1) : kNoNext;
  }
  __syncthreads();
  uint32_t local[kPer];
  uint64_t sum = 0;
  for (int b = 0; b < kPer; b++) {
    local[b] = hist[threadIdx.x * kPer + b];
    sum += local[b];
  }
  uint64_t total;
  uint64_t start = block_exscan<BLOCK>(sum, s_wave, &total);
  for (int b = 0; b < kPer; b++) {
    hist[threadIdx.x * kPer + b] = (uint32_t)start;
    start += local[b];
  }
  __syncthreads();
  for (uint64_t i = threadIdx.x; i < n; i += BLOCK) {
    uint32_t key;
    if (entry(i, key)) order[atomicAdd(&hist[key], 1u)] = (uint32_t)i;
  }
  if (threadIdx.x == 0) {
    *counter = 0;
    if (qlen) *qlen = total;
  }
}

// ------------------------------------------------------------------------------------------
// 3. selection: one wave per file
// ------------------------------------------------------------------------------------------

// First candidate in [a, b] (absolute offsets, a >= 63), by re-rolling in 64 lanes.
PFS_DEV uint64_t rescan_first(const uint8_t* __restrict__ data, const uint64_t* __restrict__ T,
                              uint64_t a, uint64_t b, uint64_t mask) {
  const uint32_t lane = threadIdx.x & 63u;
  constexpr uint64_t W = 256;
  for (uint64_t base = a; base <= b; base += 64 * W) {
    const uint64_t st = base + lane * W;
    const uint64_t en = (st + W - 1 < b) ? st + W - 1 : b;
    uint64_t found = kNone;
    if (st <= en) {
      uint64_t h = 0;
      for (int k = 0; k < 64; k++) h = rotl1_64(h) ^ T[data[st - 63 + k]];  // h_st
      if ((h & mask) == 0) found = st;
      for (uint64_t i = st + 1; found == kNone && i <= en; i++) {
        h = rotl1_64(h) ^ T[data[i - 64]] ^ T[data[i]];
        if ((h & mask) == 0) found = i;
      }
    }
    found = wave_min_u64(found);
    if (found != kNone) return found;
  }
  return kNone;
}

PFS_DEV void select_file(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ T,
    const uint64_t* __restrict__ entries, const uint64_t* __restrict__ n_entries,
    const uint64_t* __restrict__ offs, const uint64_t* __restrict__ seg_base, uint64_t f,
    uint64_t mask, uint64_t min_chunk, uint64_t max_chunk,
    pfscdc_segment* __restrict__ slots, uint64_t* __restrict__ nseg) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t fs = offs[f], fe = offs[f + 1];
  const uint64_t sb = seg_base[f], cap = seg_base[f + 1] - sb;
  const uint64_t ne = *n_entries;
  pfscdc_segment* out = slots + sb;
  uint64_t count = 0;
  auto emit = [&](uint64_t s, uint64_t size, uint32_t flags) {
    if (lane == 0 && count < cap) {
      out[count].offset = s - fs;
      out[count].size = size;
      out[count].file = (uint32_t)f;
      out[count].flags = flags;
    }
    count++;
  };
  // lower_bound(entries, fs + min - 1) on the entry value (dense markers = tile end), a
  // 64-way search: each pass the wave's lanes test 64 evenly spaced entries and keep the
  // stretch holding the boundary (~3 dependent loads for 10^4 entries instead of ~14)
  uint64_t k = 0;
  {
    const uint64_t key = fs + min_chunk - 1;
    uint64_t lo = 0, hi = ne;  // the answer lies in [lo, hi]
    while (hi - lo > 64) {
      const uint64_t step = (hi - lo + 63) / 64;
      const uint64_t i = lo + lane * step;
      const bool below = i < hi && (entries[i] & ~kDenseBit) < key;
      const uint32_t cnt = (uint32_t)__popcll(__ballot(below));  // a prefix of the lanes
      if (cnt == 0) {
        hi = lo;
      } else {
        const uint64_t top = lo + (uint64_t)cnt * step;
        lo = lo + (uint64_t)(cnt - 1) * step + 1;
        hi = top < hi ? top : hi;
      }
    }
    const uint64_t i = lo + lane;
    const bool below = i < hi && (entries[i] & ~kDenseBit) < key;
    k = lo + (uint64_t)__popcll(__ballot(below));
  }
  uint64_t s = fs;
  while (true) {
    const uint64_t lo = s + min_chunk - 1;
    if (lo >= fe) break;
    const uint64_t hi = s + max_chunk - 1;
    const uint64_t limit = hi < fe - 1 ? hi : fe - 1;
    while (k < ne && (entries[k] & ~kDenseBit) < lo) k++;
    uint64_t c = kNone;
    for (uint64_t kk = k; kk < ne; kk++) {
      const uint64_t e = entries[kk];
      const uint64_t v = e & ~kDenseBit;
      if (!(e & kDenseBit)) {
        if (v <= limit) c = v;
        break;
      }
      const uint64_t ts = (v / kTile) * kTile;
      const uint64_t a = lo > ts ? lo : ts;
      const uint64_t bnd = v < limit ? v : limit;
      if (a <= bnd) {
        c = rescan_first(data, T, a, bnd, mask);
        if (c != kNone) break;
      }
      if (v >= limit) break;
    }
    uint64_t cut;
    if (c != kNone) cut = c;
    else if (hi <= fe - 1) cut = hi;  // forced at max (writer.go:179)
    else break;
    emit(s, cut + 1 - s, PFSCDC_SEG_VALID | PFSCDC_SEG_CUT);
    s = cut + 1;
  }
  if (s < fe) emit(s, fe - s, PFSCDC_SEG_VALID);
  if (lane == 0) {
    for (uint64_t i = count; i < cap; i++) out[i].flags = 0;
    nseg[f] = count;
  }
}

// One wave per file; the last workgroup to finish then compacts the per-file segment slots
// into the dense (file, offset)-ordered list and builds the hash queue's LPT order (both
// once per batch, see last_block_done).
__global__ __launch_bounds__(kSelectBlock) void select_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ T,
    const uint64_t* __restrict__ entries, const uint64_t* __restrict__ n_entries,
    const uint64_t* __restrict__ offs, const uint64_t* __restrict__ seg_base, uint32_t nfiles,
    uint64_t mask, uint64_t min_chunk, uint64_t max_chunk,
    pfscdc_segment* __restrict__ slots, uint64_t* __restrict__ nseg, uint32_t* done_ctr,
    pfscdc_segment* __restrict__ segs, uint64_t* __restrict__ seg_begin,
    uint32_t* __restrict__ order, uint32_t* __restrict__ counter, uint64_t bin_bytes,
    uint32_t* __restrict__ next, uint64_t* __restrict__ qlen) {
  __shared__ uint32_t hist[1024];
  __shared__ uint64_t s_wave[kSelectBlock / 64 + 1];
  __shared__ uint32_t s_flag;
  const uint64_t f = ((uint64_t)blockIdx.x * kSelectBlock + threadIdx.x) >> 6;
  if (f < nfiles)  // wave-uniform
    select_file(data, T, entries, n_entries, offs, seg_base, f, mask, min_chunk, max_chunk,
                slots, nseg);
  if (!last_block_done(done_ctr, &s_flag)) return;
  const uint64_t total = segcompact_block<kSelectBlock>(slots, seg_base, nseg, nfiles, segs,
                                                        seg_begin, s_wave);
  __threadfence_block();
  __syncthreads();
  if (order)
    lpt_order_block<kSelectBlock>(segs, total, order, counter, hist, s_wave, offs, bin_bytes,
                                  next, qlen);
}

// ------------------------------------------------------------------------------------------
// 4. segment compaction (per-file counts -> dense list in (file, offset) order) and the LPT
//    order of the hash queue
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(kCompactBlock) void segcompact_kernel(
    const pfscdc_segment* __restrict__ slots, const uint64_t* __restrict__ seg_base,
    const uint64_t* __restrict__ nseg, uint32_t nfiles, pfscdc_segment* __restrict__ segs,
    uint64_t* __restrict__ seg_begin) {
  __shared__ uint64_t s_wave[kCompactBlock / 64 + 1];
  segcompact_block<kCompactBlock>(slots, seg_base, nseg, nfiles, segs, seg_begin, s_wave);
}

__global__ __launch_bounds__(kCompactBlock) void hash_order_kernel(
    const pfscdc_segment* __restrict__ segs, const uint64_t* __restrict__ seg_count,
    uint32_t* __restrict__ order, uint32_t* __restrict__ counter) {
  __shared__ uint32_t hist[1024];
  __shared__ uint64_t s_wave[kCompactBlock / 64 + 1];
  lpt_order_block<kCompactBlock>(segs, *seg_count, order, counter, hist, s_wave);
}

// ------------------------------------------------------------------------------------------
// 5. BLAKE2b-256 per segment, 4 lanes per segment
// ------------------------------------------------------------------------------------------

constexpr uint64_t kB2IV[8] = {
    0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
    0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
    0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

template <typename T>
PFS_DEV T pick4(uint32_t j, T v0, T v1, T v2, T v3) {
  return j == 0 ? v0 : j == 1 ? v1 : j == 2 ? v2 : v3;
}

// Per (round, lane): byte offsets (word*8) of the 4 message words the lane consumes:
// column G_j uses sigma[r][2j], sigma[r][2j+1]; the diagonal step runs G_{4+i}, i = (j+3)%4,
// on sigma[r][8+2i], [9+2i] (see PFS_ROUND: row b never leaves its lane).
constexpr uint32_t kSigmaPack[12][4] = {
#define PK(a, b, c, d) ((uint32_t)(a) * 8u | (uint32_t)(b) * 8u << 8 | (uint32_t)(c) * 8u << 16 | (uint32_t)(d) * 8u << 24)
// b stays in its lane; lane j computes the diagonal through b_j, G_{4+(j+3)%4}
#define ROW(s0, s1, s2, s3, s4, s5, s6, s7, s8, s9, s10, s11, s12, s13, s14, s15) \
  {PK(s0, s1, s14, s15), PK(s2, s3, s8, s9), PK(s4, s5, s10, s11), PK(s6, s7, s12, s13)}
    ROW(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15),
    ROW(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3),
    ROW(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4),
    ROW(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8),
    ROW(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13),
    ROW(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9),
    ROW(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11),
    ROW(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10),
    ROW(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5),
    ROW(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0),
    ROW(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15),
    ROW(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3),
#undef ROW
#undef PK
};

// 64-bit rotations on register halves (v_alignbit_b32 x2; rotr 32 is a register swap).
PFS_DEV uint64_t mk64(uint32_t lo, uint32_t hi) { return ((uint64_t)hi << 32) | lo; }
PFS_DEV uint64_t xor_rotr32(uint64_t x, uint64_t y) {
  return mk64((uint32_t)(x >> 32) ^ (uint32_t)(y >> 32), (uint32_t)x ^ (uint32_t)y);
}
template <int N>
PFS_DEV uint64_t xor_rotr(uint64_t x, uint64_t y) {  // rotr64(x ^ y, N), 0 < N < 32
  const uint32_t lo = (uint32_t)x ^ (uint32_t)y, hi = (uint32_t)(x >> 32) ^ (uint32_t)(y >> 32);
  return mk64(__builtin_amdgcn_alignbit(hi, lo, N), __builtin_amdgcn_alignbit(lo, hi, N));
}
PFS_DEV uint64_t xor_rotr63(uint64_t x, uint64_t y) {  // rotr64(x ^ y, 63) = rotl 1
  const uint32_t lo = (uint32_t)x ^ (uint32_t)y, hi = (uint32_t)(x >> 32) ^ (uint32_t)(y >> 32);
  return mk64(__builtin_amdgcn_alignbit(lo, hi, 31), __builtin_amdgcn_alignbit(hi, lo, 31));
}

template <int CTRL>
PFS_DEV uint64_t quad_perm64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, true);
  return mk64(lo, hi);
}

// BLAKE2b G (RFC 7693 §3.1) on one column held by this lane: 6 v_lshl_add_u64,
// 8 v_xor_b32, 6 v_alignbit_b32.
#define PFS_G(a, b, c, d, x, y)  \
  do {                           \
    a = a + b + (x);             \
    d = xor_rotr32(d, a);        \
    c = c + d;                   \
    b = xor_rotr<24>(b, c);      \
    a = a + b + (y);             \
    d = xor_rotr<16>(d, a);      \
    c = c + d;                   \
    b = xor_rotr63(b, c);        \
  } while (0)

// Lane q of the quad loads bytes [32q, 32q+32) of a 128-byte message block.
PFS_DEV void msg_load_full(uint4& m0, uint4& m1, const uint8_t* p) {
  __builtin_memcpy(&m0, p, 16);
  __builtin_memcpy(&m1, p + 16, 16);
}

// Last block of a segment: bytes at or past `avail` are zero (BLAKE2b pads with zeros).
// Two 16-byte loads and a byte mask when the 32-byte window lies inside the batch buffer
// (bytes past the segment belong to the next segment or file); byte loads only for the
// final block of the buffer.
PFS_DEV uint32_t keep_bytes(int64_t k) {  // mask of the low k bytes of a dword (k may be <0, >4)
  return k >= 4 ? 0xffffffffu : k <= 0 ? 0u : (1u << (8 * (uint32_t)k)) - 1u;
}

PFS_DEV void msg_load_tail(uint4& m0, uint4& m1, const uint8_t* p, int64_t avail,
                           const uint8_t* end) {
  if (p + 32 <= end) {
    msg_load_full(m0, m1, p);
    m0.x &= keep_bytes(avail - 0);
    m0.y &= keep_bytes(avail - 4);
    m0.z &= keep_bytes(avail - 8);
    m0.w &= keep_bytes(avail - 12);
    m1.x &= keep_bytes(avail - 16);
    m1.y &= keep_bytes(avail - 20);
    m1.z &= keep_bytes(avail - 24);
    m1.w &= keep_bytes(avail - 28);
    return;
  }
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint32_t v = 0;
    for (int b = 0; b < 4; b++)
      if (4 * i + b < avail) v |= (uint32_t)p[4 * i + b] << (8 * b);
    w[i] = v;
  }
  m0 = make_uint4(w[0], w[1], w[2], w[3]);
  m1 = make_uint4(w[4], w[5], w[6], w[7]);
}

// 5a. LPT order: see lpt_order_block (run by the last selection workgroup, or alone by
// hash_order_kernel for the chunk.Create / chunk.Get passes).

// 5b. BLAKE2b-256 per segment: 4 lanes (a quad) hash one segment, lane j owning column j of
// the 4x4 state; waves stay resident and each quad pulls its next segment from the LPT
// queue when it finishes one (one wave-aggregated atomic per refill).  The compression runs
// with every lane enabled (a finished quad computes on stale registers and discards it), so
// the DPP quad rotations never see a disabled lane.
// perm(c) + d, the permutation folded into the add as a DPP source operand (v_add_co_u32_dpp
// + v_addc_co_u32_dpp) instead of two v_mov_b32_dpp and a v_lshl_add_u64.
template <int CTRL>
PFS_DEV uint64_t perm_add(uint64_t c, uint64_t d) {
  const uint32_t cl = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)c, CTRL, 0xF, 0xF, true);
  const uint32_t ch = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(c >> 32), CTRL, 0xF, 0xF, true);
  const uint32_t lo = cl + (uint32_t)d;
  const uint32_t hi = ch + (uint32_t)(d >> 32) + (lo < cl ? 1u : 0u);
  return mk64(lo, hi);
}

// G with the incoming diagonal rotation of c folded into its first use.
#define PFS_G_PC(a, b, c, d, x, y, CC) \
  do {                                 \
    a = a + b + (x);                   \
    d = xor_rotr32(d, a);              \
    c = perm_add<CC>(c, d);            \
    b = xor_rotr<24>(b, c);            \
    a = a + b + (y);                   \
    d = xor_rotr<16>(d, a);            \
    c = c + d;                         \
    b = xor_rotr63(b, c);              \
  } while (0)

// ChaCha20 block (RFC 8439 §2.3; x/crypto chacha20 with a zero 12-byte nonce) computed by a
// quad: lane j holds column j (a = const[j], b = key[j], c = key[4+j], d = counter or 0),
// the diagonal round rotates b, c, d across the quad.  ks[w] = keystream word j + 4w.
PFS_DEV uint32_t rotl32(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
template <int CTRL>
PFS_DEV uint32_t qp32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
}
#define PFS_QR(a, b, c, d)                 \
  do {                                     \
    a += b; d ^= a; d = rotl32(d, 16);     \
    c += d; b ^= c; b = rotl32(b, 12);     \
    a += b; d ^= a; d = rotl32(d, 8);      \
    c += d; b ^= c; b = rotl32(b, 7);      \
  } while (0)
PFS_DEV void chacha20_column(uint32_t (&ks)[4], uint32_t a0, uint32_t b0, uint32_t c0,
                             uint32_t d0) {
  uint32_t a = a0, b = b0, c = c0, d = d0;
#pragma unroll
  for (int r = 0; r < 10; r++) {
    PFS_QR(a, b, c, d);  // column round
    b = qp32<0x39>(b);   // b <- column j+1, c <- j+2, d <- j+3
    c = qp32<0x4E>(c);
    d = qp32<0x93>(d);
    PFS_QR(a, b, c, d);  // diagonal round
    b = qp32<0x93>(b);
    c = qp32<0x4E>(c);
    d = qp32<0x39>(d);
  }
  ks[0] = a + a0;
  ks[1] = b + b0;
  ks[2] = c + c0;
  ks[3] = d + d0;
}

// One BLAKE2b-256 compression in one lane (message m[16], counter t, last-block flag).
PFS_DEV void b2_compress_lane(uint64_t (&h)[8], const uint64_t (&m)[16], uint64_t t, bool last);

// Ref.Dek per segment: BLAKE2b-256(secret || DataRef.Hash) with the empty secret of
// CreateOptions{} (transform.go:173-178): a single 32-byte block.  One lane per segment.
__global__ void dek_kernel(const pfscdc_segment* __restrict__ segs,
                           const uint64_t* __restrict__ seg_count, pfscdc_ref* __restrict__ refs,
                           uint32_t* __restrict__ counter) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *counter = 0;  // the Ref.Id launch's queue (same LPT order as the hash)
  if (i >= *seg_count) return;
  uint64_t m[16];
  const uint64_t* hs = reinterpret_cast<const uint64_t*>(segs[i].hash);
#pragma unroll
  for (int k = 0; k < 16; k++) m[k] = k < 4 ? hs[k] : 0;
  uint64_t h[8] = {kB2IV[0] ^ 0x01010020ULL, kB2IV[1], kB2IV[2], kB2IV[3],
                   kB2IV[4], kB2IV[5], kB2IV[6], kB2IV[7]};
  b2_compress_lane(h, m, 32, true);
  uint64_t* out = reinterpret_cast<uint64_t*>(refs[i].dek);
#pragma unroll
  for (int k = 0; k < 4; k++) out[k] = h[k];
}

// One BLAKE2b round of the quad kernel in hand-scheduled gfx950 assembly.  The state lives
// in fixed registers a = v[100:101], b = v[102:103], c = v[104:105], d = v[106:107] (temps
// v108-v111) so 64-bit ops (v_lshl_add_u64) and their 32-bit halves (DPP, alignbit) can be
// named; the compiler-scheduled form spends ~26 VALU per G on register-pair copies and
// separate DPP moves.  Here each G is 22 VALU and nothing is moved between lanes on its own:
// row b never leaves its lane (lane j runs the diagonal through b_j, G_{4+(j+3)%4}), and the
// quad rotation of rows a, c and d, into the diagonal layout and back, is a DPP source
// operand of their first uses: a' + x and c' + d (v_add_co_u32_dpp / v_addc_co_u32_dpp),
// d' ^ a (v_xor_b32_dpp).  Keeping b in place rather than a (the textbook choice) leaves
// b ^ c in the 2-cycle plain v_xor_b32 form: 16 four-cycle + 6 two-cycle ops per G instead
// of 18 + 4 (issue-rate table).
// Hazards: a DPP read needs 2 wait states after the VALU write of its source; the DPP sources
// here (a, c, d) were last written 6+ instructions earlier, inside the previous round's asm
// (the first G of a block has no DPP operand).  No s_nop guards the compiler's code between
// rounds (it writes none of v100-v107 there): tests/test_dpp_hazards.py checks every DPP
// instruction of the compiled library (an s_nop 1 per round cost 2% of a lone chain).
#define PFS_DPP(P) " quad_perm:" P " row_mask:0xf bank_mask:0xf\n"
#define PFS_G_ASM(PA, PC, PD, XL, XH, Y)                               \
  "v_add_co_u32_dpp v100, vcc, v100, " XL PFS_DPP(PA)                  \
  "v_addc_co_u32_dpp v101, vcc, v101, " XH ", vcc" PFS_DPP(PA)         \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"             \
  "v_xor_b32_dpp v108, v107, v101" PFS_DPP(PD)                         \
  "v_xor_b32_dpp v109, v106, v100" PFS_DPP(PD)                         \
  "v_add_co_u32_dpp v104, vcc, v104, v108" PFS_DPP(PC)                 \
  "v_addc_co_u32_dpp v105, vcc, v105, v109, vcc" PFS_DPP(PC)           \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v111, v110, 24\n"                              \
  "v_alignbit_b32 v103, v110, v111, 24\n"                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " Y "\n"                  \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"             \
  "v_xor_b32 v110, v108, v100\n"                                       \
  "v_xor_b32 v111, v109, v101\n"                                       \
  "v_alignbit_b32 v106, v111, v110, 16\n"                              \
  "v_alignbit_b32 v107, v110, v111, 16\n"                              \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[106:107]\n"             \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v110, v111, 31\n"                              \
  "v_alignbit_b32 v103, v111, v110, 31\n"
// The first G of a block: a, c, d are already in the column layout, so no DPP operands (an
// identity quad_perm still costs the DPP issue rate): a + x and c + d are one v_lshl_add_u64
// each, and d ^ a is the 2-cycle VOP2 form (20 VALU instead of 22).
#define PFS_G_ASM_PLAIN(X, Y)                                          \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " X "\n"                  \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"             \
  "v_xor_b32 v108, v107, v101\n"                                       \
  "v_xor_b32 v109, v106, v100\n"                                       \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[108:109]\n"             \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v111, v110, 24\n"                              \
  "v_alignbit_b32 v103, v110, v111, 24\n"                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " Y "\n"                  \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"             \
  "v_xor_b32 v110, v108, v100\n"                                       \
  "v_xor_b32 v111, v109, v101\n"                                       \
  "v_alignbit_b32 v106, v111, v110, 16\n"                              \
  "v_alignbit_b32 v107, v110, v111, 16\n"                              \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[106:107]\n"             \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v110, v111, 31\n"                              \
  "v_alignbit_b32 v103, v111, v110, 31\n"
// The first G of a block reading the block's initial state where it lives: a0 = h[j] and
// b0 = h[4+j] (the chaining value, kept for the feed-forward), c0 = IV, and d0 ^ dt (IV with
// the byte counter t in lane 0) as a 3-way XOR with a; the results land in the fixed
// registers, so the block's set-up costs no moves (3 v_mov_b64 and 2 v_xor_b32 per block
// before).  Outputs are early-clobber: no input may share v100-v107.
#define PFS_G_ASM_FIRST(X, Y)                                          \
  "v_lshl_add_u64 v[100:101], %[a0], 0, " X "\n"                      \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, %[b0]\n"                 \
  "v_bitop3_b32 v108, %[d0h], %[dth], v101 bitop3:0x96\n"             \
  "v_bitop3_b32 v109, %[d0l], %[dtl], v100 bitop3:0x96\n"             \
  "v_lshl_add_u64 v[104:105], %[c0], 0, v[108:109]\n"                 \
  "v_xor_b32 v110, %[b0l], v104\n"                                    \
  "v_xor_b32 v111, %[b0h], v105\n"                                    \
  "v_alignbit_b32 v102, v111, v110, 24\n"                             \
  "v_alignbit_b32 v103, v110, v111, 24\n"                             \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " Y "\n"                 \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"            \
  "v_xor_b32 v110, v108, v100\n"                                      \
  "v_xor_b32 v111, v109, v101\n"                                      \
  "v_alignbit_b32 v106, v111, v110, 16\n"                             \
  "v_alignbit_b32 v107, v110, v111, 16\n"                             \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[106:107]\n"            \
  "v_xor_b32 v110, v102, v104\n"                                      \
  "v_xor_b32 v111, v103, v105\n"                                      \
  "v_alignbit_b32 v102, v110, v111, 31\n"                             \
  "v_alignbit_b32 v103, v111, v110, 31\n"
#define PFS_QP_ID "[0,1,2,3]"
#define PFS_QP_R1 "[1,2,3,0]"  // 0x39: lane j reads lane j+1
#define PFS_QP_R2 "[2,3,0,1]"  // 0x4E
#define PFS_QP_R3 "[3,0,1,2]"  // 0x93: lane j reads lane j-1
// Diagonal step on lane j: a_{j-1}, b_j, c_{j+1}, d_{j+2} (R3, -, R1, R2); the next column
// step takes a, c, d back from the diagonal layout (R1, -, R3, R2).
#define PFS_DIAG_G PFS_G_ASM(PFS_QP_R3, PFS_QP_R1, PFS_QP_R2, "%[x2l]", "%[x2h]", "%[x3]")
#define PFS_ROUND_OPS(x0_, x1_, x2_, x3_)                                                \
  : "+{v[100:101]}"(a), "+{v[102:103]}"(b), "+{v[104:105]}"(c), "+{v[106:107]}"(d)      \
  : [x0] "v"(x0_), [x0l] "v"((uint32_t)(x0_)), [x0h] "v"((uint32_t)((x0_) >> 32)),      \
    [x1] "v"(x1_), [x2l] "v"((uint32_t)(x2_)), [x2h] "v"((uint32_t)((x2_) >> 32)),       \
    [x3] "v"(x3_)                                                                        \
  : "vcc", "v108", "v109", "v110", "v111"
#define PFS_ROUND_FIRST(a0_, b0_, c0_, d0_, dt_, x0_, x1_, x2_, x3_)                          \
  asm volatile(PFS_G_ASM_FIRST("%[x0]", "%[x1]") PFS_DIAG_G                                    \
               : "=&{v[100:101]}"(a), "=&{v[102:103]}"(b), "=&{v[104:105]}"(c),                  \
                 "=&{v[106:107]}"(d)                                                           \
               : [a0] "v"(a0_), [b0] "v"(b0_), [b0l] "v"((uint32_t)(b0_)),                     \
                 [b0h] "v"((uint32_t)((b0_) >> 32)), [c0] "v"(c0_),                            \
                 [d0l] "v"((uint32_t)(d0_)), [d0h] "v"((uint32_t)((d0_) >> 32)),               \
                 [dtl] "v"((uint32_t)(dt_)), [dth] "v"((uint32_t)((dt_) >> 32)),               \
                 [x0] "v"(x0_), [x1] "v"(x1_), [x2l] "v"((uint32_t)(x2_)),                      \
                 [x2h] "v"((uint32_t)((x2_) >> 32)), [x3] "v"(x3_)                              \
               : "vcc", "v108", "v109", "v110", "v111")
#define PFS_ROUND(FIRST, x0_, x1_, x2_, x3_)                                                  \
  do {                                                                                        \
    if (FIRST)                                                                                \
      asm volatile(PFS_G_ASM_PLAIN("%[x0]", "%[x1]") PFS_DIAG_G                    \
                 PFS_ROUND_OPS(x0_, x1_, x2_, x3_));                                          \
    else                                                                                      \
      asm volatile(PFS_G_ASM(PFS_QP_R1, PFS_QP_R3, PFS_QP_R2, "%[x0l]", "%[x0h]", \
                                         "%[x1]") PFS_DIAG_G                                   \
                 PFS_ROUND_OPS(x0_, x1_, x2_, x3_));                                          \
  } while (0)

// MODE kModeHash:  DataRef.Hash = BLAKE2b-256(segment) into segs[].hash.
// MODE kModeRefId: Ref.Id = BLAKE2b-256(ChaCha20_dek(segment)) into refs[].id, dek read from
//   refs[].dek (chunk.Create with CreateOptions{}: transform.go:26-46,173-188, client.go:57);
//   with out != nullptr the ciphertext (the object chunk.Create uploads) is stored there too.
//   The keystream for the two 64-byte ChaCha20 blocks of each 128-byte message block is
//   computed by the same quad (lane j = state column j, DPP diagonals, as for BLAKE2b) and
//   XORed into the LDS message buffer (ds_xor_b32) before the BLAKE2b rounds read it.
// MODE kModeGet:   chunk.Get (transform.go:50-78): the segments are stored chunks; their
//   BLAKE2b (the id to verify) goes to segs[].hash, and after each block's rounds the
//   keystream is XORed into the LDS buffer and the plaintext stored to out.
// The feed-forward h ^= v[0..7] ^ v[8..15] straight from the diagonal layout the last round
// leaves (a, c, d rotated as DPP operands of the XORs, 8 VALU instead of 6 DPP moves back to
// the column layout and 4 three-way XORs).  a, c, d were last written inside the round's asm,
// 5+ instructions earlier (checked with the rest by tests/test_dpp_hazards.py).
PFS_DEV void fold_diag(uint64_t& ha, uint64_t& hb, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
  uint32_t hal = (uint32_t)ha, hah = (uint32_t)(ha >> 32), hbl = (uint32_t)hb,
           hbh = (uint32_t)(hb >> 32);
  asm volatile(
      "v_xor_b32_dpp %0, %4, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32_dpp %1, %5, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32_dpp %0, %6, %0 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32_dpp %1, %7, %1 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32 %2, %8, %2\n"
      "v_xor_b32 %3, %9, %3\n"
      "v_xor_b32_dpp %2, %10, %2 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      "v_xor_b32_dpp %3, %11, %3 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n"
      : "+v"(hal), "+v"(hah), "+v"(hbl), "+v"(hbh)
      : "v"((uint32_t)a), "v"((uint32_t)(a >> 32)), "v"((uint32_t)c), "v"((uint32_t)(c >> 32)),
        "v"((uint32_t)b), "v"((uint32_t)(b >> 32)), "v"((uint32_t)d), "v"((uint32_t)(d >> 32)));
  ha = ((uint64_t)hah << 32) | hal;
  hb = ((uint64_t)hbh << 32) | hbl;
}

constexpr int kModeHash = 0, kModeRefId = 1, kModeGet = 2;
template <int MODE>
__global__ __launch_bounds__(kHashBlock) __attribute__((amdgpu_waves_per_eu(1, 2))) void blake2b_kernel(
    const uint8_t* __restrict__ data, const uint64_t* __restrict__ offs,
    pfscdc_segment* __restrict__ segs, const uint64_t* __restrict__ seg_count,
    const uint32_t* __restrict__ order, uint32_t* __restrict__ counter, uint64_t nbytes,
    pfscdc_ref* __restrict__ refs, uint8_t* __restrict__ out, uint32_t prio_blocks,
    uint64_t* span, const uint32_t* __restrict__ next, uint64_t* __restrict__ fair,
    uint32_t fair_every) {
  constexpr bool CIPHER = MODE != kModeHash;
  const SpanClock span_clk = span_begin(span);
  // Per quad two 128-byte message buffers.  Iteration i of the wave compresses from buffer
  // i&1 while the quad's next block (loaded into registers one iteration earlier) is written
  // to the other buffer halfway through; the wave-uniform parity makes every ds_read offset
  // an immediate (the loop body is unrolled twice).  Quad slots are kMsgStride = 160 bytes
  // apart: at a 128- or 256-byte stride the 8 quads of a ds_read_b64 lane group (which all
  // read the same message word) hit the same bank pair (8-way conflict, 16 LDS cycles per
  // read); 160 bytes (40 dwords) spreads them to ~2-way on the 48 reads of a block
  // (tools/lds_msg_layout.py).
  constexpr uint32_t kMsgStride = 160, kMsgBuf = kHashBlock / 4 * kMsgStride;
  __shared__ __attribute__((aligned(16))) uint8_t s_msg[2 * kMsgBuf];
  const uint8_t* const end = data + nbytes;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t j = lane & 3u;
  const uint64_t nseg = *seg_count;
  const uint32_t slot = (threadIdx.x >> 2) * kMsgStride;
  uint8_t* my = s_msg + slot + 32u * j;

  // Absolute LDS addresses (buffer 0) of the 4 message words this lane consumes in each
  // of rounds 0-9 (10 and 11 reuse the words of 0 and 1), 40 registers held for the whole
  // kernel (the buffer parity is the ds_read offset immediate).  Left to itself the compiler keeps the sigma bytes packed and rebuilds each
  // address with a v_add per read (48 VALU per block, ~8% of the hash); the empty asm makes
  // the values opaque so they stay in registers (budget: amdgpu_waves_per_eu(1, 2)).
  const uint32_t lds_base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t*)s_msg;
  uint32_t ma[10][4];
#pragma unroll
  for (int r = 0; r < 10; r++) {
    const uint32_t pk = pick4(j, kSigmaPack[r][0], kSigmaPack[r][1], kSigmaPack[r][2], kSigmaPack[r][3]);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      ma[r][k] = lds_base + slot + ((pk >> (8 * k)) & 0xFFu);
      asm volatile("" : "+v"(ma[r][k]));
    }
  }
  // lane constants from immediates (v_cndmask), not loads: a load here would leave the
  // compiler unable to count vmcnt across the loop and it waits for vmcnt(0) every block
  const uint64_t iv_c = pick4(j, kB2IV[0], kB2IV[1], kB2IV[2], kB2IV[3]);
  const uint64_t iv_d = pick4(j, kB2IV[4], kB2IV[5], kB2IV[6], kB2IV[7]);
  const uint64_t h0a = j == 0 ? (kB2IV[0] ^ 0x01010020ULL) : iv_c;  // digest 32, fanout/depth 1
  const uint64_t t_mask = j == 0 ? ~0ULL : 0ULL;  // the byte counter t goes into v[12] (lane 0)
  const uint64_t h0b = iv_d;

  if (prio_blocks == kHashPrioAuto)  // only when quads refill
    prio_blocks = nseg > (uint64_t)gridDim.x * (kHashBlock / 4) ? 8192u : 0u;
  bool active = false;   // this quad holds a segment
  uint32_t bin_next = kNoNext;  // hash bins: the quad's next segment (its file's following one)
  bool drained = false;  // wave-uniform: the queue is exhausted
  // wave-uniform: blocks to come in which no quad can finish and the priority cannot change,
  // so the refill ballot, the exit test and the priority ballot are skipped (they cost ~20
  // VALU per block when evaluated every block)
  uint32_t quiet = 0;
  uint64_t L = 0, nblk = 0, blk = 0;
  const uint8_t* src = data;
  pfscdc_segment* seg = segs;
  uint32_t sidx = 0;
  uint64_t ha = 0, hb = 0;
  uint4 m0 = make_uint4(0, 0, 0, 0), m1 = m0;  // the quad's block blk+1 (lane j: bytes 32j..)
  uint32_t key_b = 0, key_c = 0;  // CIPHER: ChaCha20 key words j and 4+j (state b, c of column j)
  uint8_t* dst_base = out;         // kModeGet: plaintext of the quad's segment
  const uint32_t cc_a = pick4(j, 0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u);

  auto lds_put = [&](uint32_t buf) {
    reinterpret_cast<uint4*>(my + buf)[0] = m0;
    reinterpret_cast<uint4*>(my + buf)[1] = m1;
  };
  auto load_block = [&](uint64_t b) {  // block b of the quad's segment -> m0, m1
    const uint8_t* p = src + b * 128 + 32 * j;
    if (b + 1 == nblk) msg_load_tail(m0, m1, p, (int64_t)(L - b * 128) - 32 * (int64_t)j, end);
    else msg_load_full(m0, m1, p);
  };

  auto store_block = [&](uint32_t buf) {  // this lane's 32 bytes of the LDS block -> out
    const int64_t avail = (int64_t)(L - blk * 128) - 32 * (int64_t)j;
    if (active && avail > 0) {
      const uint4 p0 = reinterpret_cast<const uint4*>(my + buf)[0];
      const uint4 p1 = reinterpret_cast<const uint4*>(my + buf)[1];
      uint8_t* o = dst_base + blk * 128 + 32 * j;
      if (avail >= 32) {
        __builtin_memcpy(o, &p0, 16);
        __builtin_memcpy(o + 16, &p1, 16);
      } else {
        uint8_t tmp[32];
        __builtin_memcpy(tmp, &p0, 16);
        __builtin_memcpy(tmp + 16, &p1, 16);
        for (int64_t k = 0; k < avail; k++) o[k] = tmp[k];
      }
    }
  };

  // The 12 rounds of one block from LDS buffer `par` (state in a, b, c, d, column layout in
  // and out); at round 5, put_next() stages the quad's next block in the other buffer.
  // pre (optional): round 0's message words, already read (the quiet-run loop reads the next
  // block's at round 11 into pre, from the buffer round 5 staged it in).
  auto rounds = [&](auto par, uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d,
                    auto&& put_next, uint64_t* pre = nullptr, bool back = true,
                    uint64_t dt = 0) {  // the first G takes d ^ dt
    constexpr uint32_t cur = decltype(par)::value * kMsgBuf, nxt = kMsgBuf - cur;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint64_t x0, x1, x2, x3;
    if (pre) {
      x0 = pre[0]; x1 = pre[1]; x2 = pre[2]; x3 = pre[3];
    } else {
      x0 = lds_abs_u64(ma[0][0] + cur); x1 = lds_abs_u64(ma[0][1] + cur);
      x2 = lds_abs_u64(ma[0][2] + cur); x3 = lds_abs_u64(ma[0][3] + cur);
    }
    // rounds 10 and 11 use sigma 0 and 1 again: their words are kept from rounds 0 and 1
    // (16 VGPRs) instead of read from LDS a second time (8 of the block's 48 reads)
    uint64_t sv[2][4];
#pragma unroll
    for (int r = 0; r < 12; r++) {
      if (r < 2) {
        sv[r][0] = x0; sv[r][1] = x1; sv[r][2] = x2; sv[r][3] = x3;
      }
      uint64_t y0 = 0, y1 = 0, y2 = 0, y3 = 0;
      if (r == 9 || r == 10) {
        y0 = sv[r - 9][0]; y1 = sv[r - 9][1]; y2 = sv[r - 9][2]; y3 = sv[r - 9][3];
      } else if (r < 11) {
        y0 = lds_abs_u64(ma[r + 1][0] + cur);
        y1 = lds_abs_u64(ma[r + 1][1] + cur);
        y2 = lds_abs_u64(ma[r + 1][2] + cur);
        y3 = lds_abs_u64(ma[r + 1][3] + cur);
      } else if (pre) {  // the next block's round 0, staged at round 5 in the other buffer
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pre[0] = lds_abs_u64(ma[0][0] + nxt);
        pre[1] = lds_abs_u64(ma[0][1] + nxt);
        pre[2] = lds_abs_u64(ma[0][2] + nxt);
        pre[3] = lds_abs_u64(ma[0][3] + nxt);
      }
      if (r == 0) {  // leaves a, c, d in the diagonal layout
        const uint64_t a0 = a, b0 = b, c0 = c, d0 = d;
        PFS_ROUND_FIRST(a0, b0, c0, d0, dt, x0, x1, x2, x3);
      } else {
        PFS_ROUND(false, x0, x1, x2, x3);
      }
      x0 = y0; x1 = y1; x2 = y2; x3 = y3;
      if (r == 5) put_next();
    }
    if (back) {
      a = quad_perm64<0x39>(a);  // back to the column layout
      c = quad_perm64<0x93>(c);
      d = quad_perm64<0x4E>(d);
    }
  };

  // A block in a run of quiet blocks (content hash only): every active quad is at least 4
  // blocks from its end, so nothing in it depends on a lane's position in its chain.  Runs
  // of these execute in their own loop, straight-line code between the round blocks.
  // Fair share (fair != nullptr): with hash bins the two waves of a SIMD hold equal work, but
  // the SIMD's arbiter lets one run ahead (oldest first), which then ends early and leaves the
  // other alone at the lone-wave rate.  At least every fair_every blocks each wave adds the
  // blocks it ran to a launch-wide counter and raises its issue priority while it is behind
  // the launch's average, so the waves of a SIMD advance together.
  const uint32_t kFairEvery = fair_every ? fair_every : 256;
  uint32_t wave_steps = 0;  // blocks this wave ran (wave-uniform; fair share, the trace)
  uint32_t reported = 0;
  const uint64_t nwaves = (uint64_t)gridDim.x * (kHashBlock / 64);
  // the fast loop's byte counter t (lane 0 only: ((blk + 1) << 7) & t_mask), advanced by one
  // 64-bit add per block instead of rebuilt from blk (shift, add, two selects)
  uint64_t tm = 0;
  const uint64_t tinc = 128 & t_mask;
  auto fast_step = [&](auto par, uint64_t* pre) {
    constexpr uint32_t cur = decltype(par)::value * kMsgBuf, nxt = kMsgBuf - cur;
    uint64_t a = ha, b = hb, c = iv_c, d = iv_d;  // d ^ tm in the first G
    rounds(par, a, b, c, d, [&] {
      if (active) {
        lds_put(nxt);
        msg_load_full(m0, m1, src + (blk + 2) * 128 + 32 * j);
      }
    }, pre, false, tm);
    fold_diag(ha, hb, a, b, c, d);
    tm += tinc;
    blk++;  // inactive quads too: a refill resets blk
  };

  auto step = [&](auto par) -> bool {
    constexpr uint32_t cur = decltype(par)::value * kMsgBuf, nxt = kMsgBuf - cur;
    // fast (wave-uniform): a quiet block in which every active quad is at least 4 blocks from
    // its end (after the decrement, the shortest active chain has quiet + 1 blocks left), so
    // no block is the last, and the block fetched at round 5 is a full one: the per-block
    // bookkeeping reduces to straight-line code (no per-lane last/tail selects or branches).
    bool fast = false;
    if (quiet) {
      quiet--;
      fast = quiet >= 3;
    } else {
      auto begin = [&](uint32_t s) {  // start segment s on this quad
        sidx = s;
        seg = segs + sidx;
        L = seg->size;
        if (CIPHER) {
          const uint32_t* dk = reinterpret_cast<const uint32_t*>(refs[sidx].dek);
          key_b = dk[j];
          key_c = dk[4 + j];
        }
        src = data + offs[seg->file] + seg->offset;
        if (MODE != kModeHash && out) dst_base = out + offs[seg->file] + seg->offset;
        nblk = L == 0 ? 1 : (L + 127) / 128;
        blk = 0;
        ha = h0a;
        hb = h0b;
        active = true;
        load_block(0);
        lds_put(cur);
        if (nblk > 1) load_block(1);
      };
      if (!active && bin_next != kNoNext) {  // the rest of the quad's bin, no queue access
        begin(bin_next);
        bin_next = kNoNext;
      }
      if (!drained) {
        const bool need = !active;
        const uint64_t want = __ballot(need && j == 0);  // one bit per idle quad (its lane 0)
        if (want) {
          const uint32_t cnt = (uint32_t)__popcll(want);
          const uint32_t leader = (uint32_t)__builtin_ctzll(want);
          uint32_t base = 0;
          if (lane == leader) base = atomicAdd(counter, cnt);
          base = (uint32_t)__shfl((int)base, (int)leader, 64);
          if (need) {
            const uint64_t below = want & ((1ULL << (lane & ~3u)) - 1);
            const uint64_t idx = (uint64_t)base + (uint64_t)__popcll(below);
            if (idx < nseg) begin(order[idx]);
          }
          if ((uint64_t)base + cnt >= nseg) drained = true;
        }
      }
      if (__ballot(active) == 0) return false;  // every quad idle and the queue empty
      if (fair) {
        const uint32_t d = wave_steps - reported;
        uint64_t tot = 0;
        if (lane == 0) tot = atomicAdd((unsigned long long*)fair, (unsigned long long)d);
        tot = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tot >> 32)) << 32) |
              (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tot);
        reported = wave_steps;
        const uint64_t mine = (uint64_t)wave_steps * nwaves, all = tot + d;
        if (mine < all) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      } else if (prio_blocks) {  // waves holding a long chain issue first
        const uint64_t T = prio_blocks, rem = active ? nblk - blk : 0;
        if (__ballot(rem > T)) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(0);
      }

      // next event: the step after the first active quad's last block, or the step at which
      // the longest remaining chain drops to the priority threshold
      const uint64_t rem64 = active ? nblk - blk : 0;
      const uint32_t rem = rem64 > 0xffffffffULL ? 0xffffffffu : (uint32_t)rem64;
      uint32_t q = wave_min_u32(active ? rem : 0xffffffffu) - 1;
      if (fair && q > kFairEvery - 1) q = kFairEvery - 1;
      if (!fair && prio_blocks) {
        // the next block at which the longest chain left crosses the priority threshold
        const uint32_t T = prio_blocks, rmax = wave_max_u32(rem);
        if (rmax > T && rmax - T - 1 < q) q = rmax - T - 1;
      }
      quiet = q;
    }
    const bool last = !fast && blk + 1 == nblk;
    if (MODE == kModeRefId) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // keystream blocks 2*blk and 2*blk+1, XORed into the plaintext already in LDS; in the
      // last block only the bytes before the segment end (BLAKE2b zero-pads the rest)
      const int64_t avail = (int64_t)(L - blk * 128);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        uint32_t ks[4];
        chacha20_column(ks, cc_a, key_b, key_c, j == 0 ? (uint32_t)(2 * blk + h) : 0u);
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_msg + cur + slot + 64 * h) + j;
#pragma unroll
        for (int w = 0; w < 4; w++) {
          const uint32_t v = last ? ks[w] & keep_bytes(avail - 64 * h - 16 * w - 4 * (int64_t)j) : ks[w];
          __hip_atomic_fetch_xor(dst + 4 * w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      if (out) {  // the ciphertext as uploaded (chunk.Create's buf) -> out
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        store_block(cur);
      }
    }
    uint64_t a = ha, b = hb, c = iv_c, d;
    if (fast) {
      d = iv_d ^ (((blk + 1) << 7) & t_mask);
    } else {
      const uint64_t t = last ? L : (blk + 1) * 128;
      d = iv_d ^ (j == 0 ? t : 0) ^ ((j == 2 && last) ? ~0ULL : 0);
    }
    rounds(par, a, b, c, d, [&] {
      if (active && !last) {  // block blk+1 -> the other buffer; fetch blk+2
        lds_put(nxt);
        if (blk + 2 < nblk) load_block(blk + 2);
      }
    });
    ha ^= a ^ c;
    hb ^= b ^ d;
    if (MODE == kModeGet) {  // decrypt the hashed ciphertext block in place, store plaintext
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int h = 0; h < 2; h++) {
        uint32_t ks[4];
        chacha20_column(ks, cc_a, key_b, key_c, j == 0 ? (uint32_t)(2 * blk + h) : 0u);
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_msg + cur + slot + 64 * h) + j;
#pragma unroll
        for (int w = 0; w < 4; w++)
          __hip_atomic_fetch_xor(dst + 4 * w, ks[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      store_block(cur);
    }
    if (fast) {
      blk++;  // inactive quads too: a refill resets blk
    } else if (active) {
      blk++;
      if (last) {  // digest = h[0..3] little endian; lane j owns h[j]
        if (MODE == kModeRefId) reinterpret_cast<uint64_t*>(refs[sidx].id)[j] = ha;
        else reinterpret_cast<uint64_t*>(seg->hash)[j] = ha;
        active = false;
        if (next) bin_next = next[sidx];
      }
    }
    return true;
  };
  constexpr std::integral_constant<uint32_t, 0> P0{};
  constexpr std::integral_constant<uint32_t, 1> P1{};
  // quiet counts blocks still free of bookkeeping; a block with quiet = Q before it has every
  // active quad at least Q blocks from its end, so pairs of fast blocks need Q >= 5
  // (one copy of the fast loop, entered after a parity-1 step: one hot loop body in the
  // instruction cache)
  while (true) {
    if (!step(P0)) break;
    if (!step(P1)) break;
    wave_steps += 2;
    if constexpr (MODE == kModeHash) {
      if (quiet >= 5) {
        uint64_t pre[4] = {lds_abs_u64(ma[0][0]), lds_abs_u64(ma[0][1]), lds_abs_u64(ma[0][2]),
                           lds_abs_u64(ma[0][3])};  // buffer 0 (P0): the next block
        tm = ((blk + 1) << 7) & t_mask;
        do {
          fast_step(P0, pre);
          fast_step(P1, pre);
          quiet -= 2;
          wave_steps += 2;
        } while (quiet >= 5);
      }
    }
  }
  span_end(span, span_clk);
}

// 5d. ChaCha20 ciphertext of whole chunks, one lane per 64-byte keystream block (the Ref.Id
// pass split in two for chunk lists that cannot fill the GPU, see create_refs_device).  Every
// block is independent (RFC 8439 §2.4: counter = block index within the chunk, zero nonce,
// key = the chunk's dek), so this pass runs at the VALU rate however long the chunks are,
// and the serial BLAKE2b chain that follows no longer carries the keystream.  Record r
// covers blocks [blk_base[r], blk_base[r+1]); consecutive lanes take consecutive blocks.
PFS_DEV uint32_t rotl32v(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
#define PFS_CQR(a, b, c, d)                         \
  do {                                              \
    x[a] += x[b]; x[d] = rotl32v(x[d] ^ x[a], 16);  \
    x[c] += x[d]; x[b] = rotl32v(x[b] ^ x[c], 12);  \
    x[a] += x[b]; x[d] = rotl32v(x[d] ^ x[a], 8);   \
    x[c] += x[d]; x[b] = rotl32v(x[b] ^ x[c], 7);   \
  } while (0)
// Memory traffic is coalesced.  Were lane l to XOR its own 64-byte block, one 16-byte load or
// store instruction would span 64 blocks (4 KiB, 32 lines); instead each lane computes its
// block's keystream, parks it in LDS (64 B per lane, 16-byte slots
// XOR-rotated by (block >> 1) & 3 so the 8-lane groups of ds_write_b128 and the 16-lane
// groups of ds_read_b128 are conflict-free), and the wave then walks its 64-block window as
// 256 consecutive 16-byte pieces: lane l takes pieces l, l + 64, l + 128, l + 192, so one
// instruction covers 1 KiB of one chunk (8 lines).  A chunk's last, partial block is written
// byte by byte up to the chunk's end (in place, the next chunk's first block is another
// lane's).  c4 commit data plane at G = 2, same box, alternating: 369.5-369.9 -> 378.3-378.8
// GiB/s against the per-lane form (profiles/r4/chacha/; that form is no longer built).
// data and out are not __restrict__: in place (PFSCDC_OPT_CTEXT_IN_PLACE) they are the same
// buffer; every byte is read before the same lane writes it.
constexpr int kChachaBlock = 256;
__global__ __launch_bounds__(kChachaBlock) void chacha_xor_coalesced_kernel(
    const uint8_t* data, const uint64_t* __restrict__ offs,
    const pfscdc_segment* __restrict__ segs, const uint64_t* __restrict__ blk_base, uint32_t n,
    const pfscdc_ref* __restrict__ refs, uint8_t* out, uint32_t prio) {
  if (prio) __builtin_amdgcn_s_setprio(2);
  __shared__ __attribute__((aligned(16))) uint32_t s_ks[kChachaBlock / 64][64 * 16];
  __shared__ uint64_t s_at[kChachaBlock / 64][64];
  __shared__ int64_t s_avail[kChachaBlock / 64][64];
  const uint64_t nblocks = blk_base[n];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t* const ks = s_ks[wv];
  const uint64_t w0 = (uint64_t)blockIdx.x * blockDim.x +
                      (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
  for (uint64_t g0 = w0; g0 < nblocks; g0 += stride) {
    uint32_t lo = 0, hi = n;  // the last r with blk_base[r] <= g0
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (blk_base[mid] <= g0) lo = mid;
      else hi = mid;
    }
    const uint64_t g = g0 + lane;
    uint32_t x[16];
    uint64_t at = 0;
    int64_t avail = 0;  // <= 0: no block here (past the pass's last block)
    if (g < nblocks) {
      while (blk_base[lo + 1] <= g) lo++;
      const pfscdc_segment& sg = segs[lo];
      const uint64_t b = g - blk_base[lo];
      at = offs[sg.file] + sg.offset + 64 * b;
      avail = (int64_t)(sg.size - 64 * b);
      const uint4 k0 = reinterpret_cast<const uint4*>(refs[lo].dek)[0];
      const uint4 k1 = reinterpret_cast<const uint4*>(refs[lo].dek)[1];
      const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                              k0.x, k0.y, k0.z, k0.w, k1.x, k1.y, k1.z, k1.w,
                              (uint32_t)b, 0u, 0u, 0u};
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = s[i];
#pragma unroll
      for (int r = 0; r < 10; r++) {
        PFS_CQR(0, 4, 8, 12);
        PFS_CQR(1, 5, 9, 13);
        PFS_CQR(2, 6, 10, 14);
        PFS_CQR(3, 7, 11, 15);
        PFS_CQR(0, 5, 10, 15);
        PFS_CQR(1, 6, 11, 12);
        PFS_CQR(2, 7, 8, 13);
        PFS_CQR(3, 4, 9, 14);
      }
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] += s[i];
    } else {
#pragma unroll
      for (int i = 0; i < 16; i++) x[i] = 0;
    }
    // park the keystream: slot q of block `lane` at lane * 64 + 16 * ((q + (lane >> 1)) & 3)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t slot = ((uint32_t)q + (lane >> 1)) & 3u;
      *reinterpret_cast<uint4*>(ks + lane * 16 + 4 * slot) =
          make_uint4(x[4 * q], x[4 * q + 1], x[4 * q + 2], x[4 * q + 3]);
    }
    s_at[wv][lane] = at;
    s_avail[wv][lane] = avail;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // 256 pieces of 16 bytes: piece p = lane + 64 i is slot p & 3 of block p >> 2
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t p = lane + 64u * (uint32_t)i, j = p >> 2, q = p & 3u;
      const int64_t av = s_avail[wv][j] - 16 * (int64_t)q;
      if (av <= 0) continue;
      const uint32_t slot = (q + (j >> 1)) & 3u;
      const uint4 k = *reinterpret_cast<const uint4*>(ks + j * 16 + 4 * slot);
      const uint64_t a = s_at[wv][j] + 16 * q;
      if (av >= 16) {
        uint4 v;
        __builtin_memcpy(&v, data + a, 16);
        v.x ^= k.x;
        v.y ^= k.y;
        v.z ^= k.z;
        v.w ^= k.w;
        __builtin_memcpy(out + a, &v, 16);
      } else {  // the chunk's last bytes: only its own (the next chunk's follow)
        const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
        for (int64_t t = 0; t < av; t++)
          out[a + t] = data[a + t] ^ (uint8_t)(kw[t >> 2] >> (8 * (t & 3)));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();  // the window's keystream is read before the next one lands
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}
#undef PFS_CQR

// 5c. BLAKE2b-256, one lane per segment.  No cross-lane traffic at all: the 16-word state,
// the chaining value and the message block live in the lane's registers, and the sigma
// schedule is resolved at compile time (every round fully unrolled), so a block costs the
// bare 96 G functions (6 v_lshl_add_u64 + 8 v_xor_b32 + 6 v_alignbit_b32 each) and its
// loads.  The 4-lane kernel above spends ~30% more VALU per block on DPP quad rotations
// and LDS message gathers; on gfx950 nearly every VALU op holds the SIMD-32 for 4 cycles
// (v_xor_b32 for 2), so instructions per chain-block, not latency, set the throughput once
// enough segments are in flight.  Lanes pull segments from the same LPT queue.
constexpr uint8_t kSigma[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
};
constexpr uint64_t kIV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                             0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                             0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

PFS_DEV void b2_compress_lane(uint64_t (&h)[8], const uint64_t (&x)[16], uint64_t t, bool last) {
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[8 + i] = kIV[i];
  }
  v[12] ^= t;
  v[14] ^= last ? ~0ULL : 0ULL;
#pragma unroll
  for (int r = 0; r < 12; r++) {
    PFS_G(v[0], v[4], v[8], v[12], x[kSigma[r][0]], x[kSigma[r][1]]);
    PFS_G(v[1], v[5], v[9], v[13], x[kSigma[r][2]], x[kSigma[r][3]]);
    PFS_G(v[2], v[6], v[10], v[14], x[kSigma[r][4]], x[kSigma[r][5]]);
    PFS_G(v[3], v[7], v[11], v[15], x[kSigma[r][6]], x[kSigma[r][7]]);
    PFS_G(v[0], v[5], v[10], v[15], x[kSigma[r][8]], x[kSigma[r][9]]);
    PFS_G(v[1], v[6], v[11], v[12], x[kSigma[r][10]], x[kSigma[r][11]]);
    PFS_G(v[2], v[7], v[8], v[13], x[kSigma[r][12]], x[kSigma[r][13]]);
    PFS_G(v[3], v[4], v[9], v[14], x[kSigma[r][14]], x[kSigma[r][15]]);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[8 + i];
}

// ------------------------------------------------------------------------------------------
// synthetic data (bench/tests): splitmix64 finalizer of (file << 40 | word) + gamma*(seed+1)
// ------------------------------------------------------------------------------------------

PFS_DEV uint64_t synth_word(uint64_t f, uint64_t k, uint64_t seed) {
  uint64_t z = ((f << 40) | k) + (seed + 1) * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

// Dedup-heavy layouts (BASELINE configs[4]): source (file, word) of the byte at offset o of
// file f.  mode 1: each 1 MiB block of a file is, with p = 1/2, a copy of one of 64 pooled
// blocks (pool "file" kPoolFile + id), else fresh bytes; mode 2: the same per whole file.
constexpr uint64_t kPoolFile = 1ULL << 23;
PFS_DEV uint64_t synth_mix(uint64_t x) {
  x = (x ^ (x >> 33)) * 0xFF51AFD7ED558CCDULL;
  x = (x ^ (x >> 33)) * 0xC4CEB9FE1A85EC53ULL;
  return x ^ (x >> 33);
}
PFS_DEV uint64_t synth_byte_word(uint64_t f, uint64_t o, uint64_t seed, uint32_t mode) {
  if (mode == 1) {
    const uint64_t h = synth_mix((seed << 48) ^ (f << 24) ^ (o >> 20) ^ 0xC5C5C5C5ULL);
    if (h & 1) return synth_word(kPoolFile + ((h >> 1) & 63), (o & 0xFFFFF) >> 3, seed);
  } else if (mode == 2) {
    const uint64_t h = synth_mix((seed << 48) ^ (f << 24) ^ 0x5EEDF11EULL);
    if (h & 1) return synth_word(kPoolFile + ((h >> 1) & 63), o >> 3, seed);
  }
  return synth_word(f, o >> 3, seed);
}

// Local file f of the launch is bytes [starts[f], ...) of file ids[f] of the synthetic
// commit (ids/starts NULL: file f from its first byte), so a rank can generate just its
// pieces of files that are cut across serialized filesets or ranks.
__global__ void synth_kernel(uint8_t* __restrict__ out, const uint64_t* __restrict__ offs,
                             uint32_t nfiles, const uint32_t* __restrict__ ids,
                             const uint64_t* __restrict__ starts, uint64_t seed, uint32_t mode) {
  const uint64_t n = offs[nfiles];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 8;
  for (uint64_t g = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; g < n; g += stride) {
    // file of byte g (upper_bound - 1)
    uint32_t lo = 0, hi = nfiles;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (offs[mid] <= g) lo = mid;
      else hi = mid;
    }
    uint32_t f = lo;
    uint8_t bytes[8];
    for (int b = 0; b < 8; b++) {
      const uint64_t p = g + b;
      if (p >= n) break;
      while (f + 1 < nfiles && offs[f + 1] <= p) f++;
      const uint64_t o = p - offs[f] + (starts ? starts[f] : 0);
      const uint64_t fid = ids ? ids[f] : f;
      bytes[b] = (uint8_t)(synth_byte_word(fid, o, seed, mode) >> (8 * (o & 7)));
    }
    if (g + 8 <= n) {
      uint64_t w;
      __builtin_memcpy(&w, bytes, 8);
      *reinterpret_cast<uint64_t*>(out + g) = w;
    } else {
      for (uint64_t p = g; p < n; p++) out[p] = bytes[p - g];
    }
  }
}

// ------------------------------------------------------------------------------------------
// launchers (host)
// ------------------------------------------------------------------------------------------

// Per-device kernel attributes (the scan's 154 KB of dynamic LDS), set by pfscdc_ctx_create
// on the ctx's device before any launch; idempotent, so every ctx sets them on its device.
hipError_t prepare_kernels() {
  const int lds = (int)kScanLdsBytes;
  hipError_t e = hipFuncSetAttribute((const void*)cdc_scan_kernel<false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)cdc_scan_kernel<true>,
                             hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

hipError_t launch_scan_skip(const uint64_t* offs, uint32_t nfiles, uint64_t n, uint64_t min_chunk,
                            uint64_t ntiles, uint32_t* skip, uint64_t* scanned, hipStream_t st) {
  const uint64_t nunits = ntiles * kScanWaves;
  if (nunits == 0) return hipSuccess;
  scan_skip_kernel<<<(unsigned)((nunits + 255) / 256), 256, 0, st>>>(
      offs, nfiles, n, min_chunk, nunits, skip, (unsigned long long*)scanned, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_scan_plan(const uint64_t* offs, uint32_t nfiles, uint64_t n, uint64_t min_chunk,
                            uint64_t ntiles, uint32_t* skip, uint64_t* scanned, uint32_t* uinfo,
                            uint4* slots, uint32_t* plan, const ScanPlan& hdr, ScanPlan* d_hdr,
                            hipStream_t st) {
  const uint64_t nunits = ntiles * kScanWaves;
  if (nunits == 0) return hipSuccess;
  const unsigned grid = (unsigned)((nunits + 255) / 256);
  scan_skip_kernel<<<grid, 256, 0, st>>>(offs, nfiles, n, min_chunk, nunits, skip,
                                         (unsigned long long*)scanned, uinfo, plan);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  scan_slots_kernel<<<grid, 256, 0, st>>>(nunits, uinfo, plan, slots, hdr, d_hdr);
  return hipGetLastError();
}

hipError_t launch_scan(const uint8_t* data, const uint8_t* tail, uint64_t n, const uint64_t* d_table,
                       uint32_t average_bits, uint64_t ntiles, TileRec* recs, int grid,
                       uint32_t* unit_ctr, uint32_t* done_ctr, uint64_t* entries,
                       uint64_t* n_entries, uint64_t* span, hipStream_t st, const uint32_t* skip,
                       const ScanPlan* d_plan) {
  const size_t lds = kScanLdsBytes;
  const uint64_t mask64 = average_bits >= 64 ? ~0ULL : ((1ULL << average_bits) - 1);
  const ScanPlan* const pl = d_plan;
  if (average_bits <= 32)
    cdc_scan_kernel<false><<<grid, kScanBlock, lds, st>>>(
        data, tail, n, d_table, 32 - average_bits, mask64, ntiles, recs, unit_ctr, done_ctr,
        entries, n_entries, skip, span, pl);
  else
    cdc_scan_kernel<true><<<grid, kScanBlock, lds, st>>>(
        data, tail, n, d_table, 64 - average_bits, mask64, ntiles, recs, unit_ctr, done_ctr,
        entries, n_entries, skip, span, pl);
  return hipGetLastError();
}

hipError_t launch_compact(const TileRec* recs, uint64_t ntiles, uint64_t n, uint64_t* entries,
                          uint64_t* n_entries, hipStream_t st) {
  compact_kernel<<<1, kCompactBlock, 0, st>>>(recs, ntiles, n, entries, n_entries);
  return hipGetLastError();
}

hipError_t launch_select(const uint8_t* data, const uint64_t* d_table, const uint64_t* entries,
                         const uint64_t* n_entries, const uint64_t* offs,
                         const uint64_t* seg_base, uint32_t nfiles, uint32_t average_bits,
                         uint64_t min_chunk, uint64_t max_chunk, pfscdc_segment* slots,
                         uint64_t* nseg, uint32_t* done_ctr, pfscdc_segment* segs,
                         uint64_t* seg_begin, uint32_t* order, uint32_t* counter,
                         hipStream_t st, uint64_t bin_bytes, uint32_t* next, uint64_t* qlen) {
  const uint64_t mask64 = average_bits >= 64 ? ~0ULL : ((1ULL << average_bits) - 1);
  const uint64_t waves_per_block = kSelectBlock / 64;
  const uint64_t grid = (nfiles + waves_per_block - 1) / waves_per_block;
  select_kernel<<<(unsigned)grid, kSelectBlock, 0, st>>>(data, d_table, entries, n_entries,
                                                         offs, seg_base, nfiles, mask64,
                                                         min_chunk, max_chunk, slots, nseg,
                                                         done_ctr, segs, seg_begin, order,
                                                         counter, bin_bytes, next, qlen);
  return hipGetLastError();
}

hipError_t launch_segcompact(const pfscdc_segment* slots, const uint64_t* seg_base,
                             const uint64_t* nseg, uint32_t nfiles, pfscdc_segment* segs,
                             uint64_t* seg_begin, hipStream_t st) {
  segcompact_kernel<<<1, kCompactBlock, 0, st>>>(slots, seg_base, nseg, nfiles, segs, seg_begin);
  return hipGetLastError();
}

// Wave issue priority in the hash kernels: a wave raises its priority (s_setprio 2) while
// one of its quads has more than this many 128-B blocks left, so the long chains of the LPT
// queue are issued ahead of the short fill-in work.  It pays when the queue holds more
// segments than the grid has quads (c2: 44K segments, 32K quads: hash 79 ms vs 96 ms per
// 128 GiB at 8192 blocks = 1 MiB; 6000-10000 within 1%, graded levels and a static
// block-parity priority worse, no longer built) and costs ~4% when every segment starts at
// once (c4: 132 vs 127 ms), so the default (kHashPrioAuto) enables it at 8192 only when quads
// will refill (profiles/r1_prio/).
static uint32_t prio_arg(uint32_t prio) {
  return prio == kHashPrioNone ? 0u : prio ? prio : kHashPrioAuto;
}

// Waves per SIMD for a hash launch.  One quad runs a chain's 128-B blocks strictly in order,
// so no launch ends before its longest chain; a second wave on a SIMD only slows that chain
// down (the two share the issue slots).  One wave per SIMD when the launch is bound by its
// longest chain even then (longest blocks >= total blocks / the quads of one wave per SIMD:
// c3, c4, a single configs[1] batch, most chunk.Create passes), two otherwise (c2's 128 GiB
// steps: 72 vs 80 ms; c4: 100 vs 104-110 ms).  forced (the PFSCDC_HASH_WAVES knob) in 1..8
// overrides it.
int hash_waves(uint64_t longest_bytes, uint64_t total_bytes, int num_cus, int forced) {
  if (forced >= 1 && forced <= 8) return forced;
  const uint64_t quads1 = (uint64_t)num_cus * 4 * (64 / 4);
  const uint64_t longest = (longest_bytes + 127) / 128, total = total_bytes / 128;
  return longest * quads1 >= total ? 1 : kHashWavesPerSimd;
}

static unsigned hash_grid(uint64_t max_segments, int num_cus, int waves) {
  const uint64_t quads_per_block = kHashBlock / 4;
  const uint64_t need = (max_segments + quads_per_block - 1) / quads_per_block;
  const uint64_t full = (uint64_t)num_cus * 4 * (waves > 0 ? waves : kHashWavesPerSimd) /
                        (kHashBlock / 64);
  return (unsigned)(need < full ? need : full);
}

hipError_t launch_blake2b(const uint8_t* data, const uint64_t* offs, pfscdc_segment* segs,
                          const uint64_t* seg_count, uint64_t max_segments, uint32_t* order,
                          uint32_t* counter, int num_cus, uint64_t nbytes, hipStream_t st,
                          bool ordered, uint64_t* span, int waves, uint32_t prio,
                          bool cu_exclusive, const uint32_t* next, uint64_t* fair,
                          uint32_t fair_every) {
  if (max_segments == 0) return hipSuccess;
  if (!ordered) hash_order_kernel<<<1, kCompactBlock, 0, st>>>(segs, seg_count, order, counter);
  // cu_exclusive: 64 KiB of unused dynamic LDS on top of the 20 KiB message buffers, so no
  // two workgroups (of this or of another launch) share a CU.  A chain-bound launch at one
  // wave per SIMD has one workgroup per CU anyway; the reservation keeps a second such launch
  // in flight (configs[2]'s two streams) off its CUs, where the two launches' chains would
  // share SIMDs (hash 215 instead of 180 ms when the dispatcher put them together).
  const size_t dyn = cu_exclusive ? 64u * 1024u : 0u;
  blake2b_kernel<kModeHash><<<hash_grid(max_segments, num_cus, waves), kHashBlock, dyn, st>>>(
      data, offs, segs, seg_count, order, counter, nbytes, nullptr, nullptr,
      prio_arg(prio), span, ordered ? next : nullptr, ordered ? fair : nullptr, fair_every);
  return hipGetLastError();
}

hipError_t launch_order(const pfscdc_segment* segs, const uint64_t* seg_count, uint32_t* order,
                        uint32_t* counter, hipStream_t st) {
  hash_order_kernel<<<1, kCompactBlock, 0, st>>>(segs, seg_count, order, counter);
  return hipGetLastError();
}

hipError_t launch_ref_ids(const uint8_t* data, const uint64_t* offs, pfscdc_segment* segs,
                          const uint64_t* seg_count, uint64_t max_segments, const uint32_t* order,
                          uint32_t* counter, int num_cus, uint64_t nbytes, pfscdc_ref* refs,
                          uint8_t* ctext_out, hipStream_t st, int waves, uint32_t prio,
                          const uint32_t* next, const uint64_t* nsegs) {
  if (max_segments == 0) return hipSuccess;
  // a dek for every segment (nsegs; with hash bins seg_count is the queue's length)
  dek_kernel<<<(unsigned)((max_segments + 255) / 256), 256, 0, st>>>(
      segs, nsegs ? nsegs : seg_count, refs, counter);
  blake2b_kernel<kModeRefId><<<hash_grid(max_segments, num_cus, waves), kHashBlock, 0, st>>>(
      data, offs, segs, seg_count, order, counter, nbytes, refs, ctext_out,
      prio_arg(prio), nullptr, next, nullptr, 0u);
  return hipGetLastError();
}

hipError_t launch_deks(pfscdc_segment* segs, const uint64_t* seg_count, uint64_t max_segments,
                       pfscdc_ref* refs, uint32_t* counter, hipStream_t st) {
  if (max_segments == 0) return hipSuccess;
  dek_kernel<<<(unsigned)((max_segments + 255) / 256), 256, 0, st>>>(segs, seg_count, refs, counter);
  return hipGetLastError();
}

hipError_t launch_chacha_xor(const uint8_t* data, const uint64_t* offs, const pfscdc_segment* segs,
                             const uint64_t* blk_base, uint32_t n, uint64_t nblocks,
                             const pfscdc_ref* refs, uint8_t* out, int num_cus, hipStream_t st,
                             bool prio, bool one_wave_per_simd) {
  if (nblocks == 0) return hipSuccess;
  // one_wave_per_simd: num_cus workgroups of 4 waves (room left on every SIMD for another
  // context's launches)
  const uint64_t need = (nblocks + 255) / 256,
                 full = (uint64_t)num_cus * (one_wave_per_simd ? 1 : 32);
  const unsigned grid = (unsigned)(need < full ? need : full);
  chacha_xor_coalesced_kernel<<<grid, kChachaBlock, 0, st>>>(data, offs, segs, blk_base, n,
                                                            refs, out, prio ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_get(const uint8_t* ctext, const uint64_t* offs, pfscdc_segment* segs,
                      const uint64_t* seg_count, uint64_t nsegs, uint32_t* order, uint32_t* counter,
                      int num_cus, uint64_t nbytes, pfscdc_ref* refs, uint8_t* ptext, hipStream_t st,
                      int waves) {
  if (nsegs == 0) return hipSuccess;
  hash_order_kernel<<<1, kCompactBlock, 0, st>>>(segs, seg_count, order, counter);
  blake2b_kernel<kModeGet><<<hash_grid(nsegs, num_cus, waves), kHashBlock, 0, st>>>(
      ctext, offs, segs, seg_count, order, counter, nbytes, refs, ptext, prio_arg(0), nullptr,
      nullptr, nullptr, 0u);
  return hipGetLastError();
}

hipError_t launch_synth(uint8_t* out, const uint64_t* offs, uint32_t nfiles, const uint32_t* ids,
                        const uint64_t* starts, uint64_t seed, uint32_t mode, hipStream_t st) {
  synth_kernel<<<2048, 256, 0, st>>>(out, offs, nfiles, ids, starts, seed, mode);
  return hipGetLastError();
}

// A device group's gathered chunk-ref index: member-local file ids + the member's first file.
__global__ void rebase_files_kernel(pfscdc_segment* __restrict__ segs, uint64_t n, uint32_t base) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    segs[i].file += base;
}

hipError_t launch_rebase_files(pfscdc_segment* segs, uint64_t n, uint32_t base, hipStream_t st) {
  if (n == 0 || base == 0) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 1024);
  rebase_files_kernel<<<(unsigned)blocks, 256, 0, st>>>(segs, n, base);
  return hipGetLastError();
}

}  // namespace pfscdc
