// pfscdc_internal.h — shared constants and launcher declarations (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pfscdc.h"

namespace pfscdc {

// candidate scan geometry: waves x 64 lanes x 4 KiB strips per tile.  Candidates go
// straight to the tile's record in global memory (zeroed before the scan), so waves never
// synchronise per tile and all LDS beyond the table is staging.
constexpr int kScanWaves = 12;  // 12 = 3 per SIMD: LDS exactly full (8: 2 per SIMD, 3.5% slower)
constexpr int kScanBlock = 64 * kScanWaves;
constexpr int kStrip = 4096;  // bytes per lane per tile (plus a 64-byte halo)
constexpr uint64_t kTile = (uint64_t)kScanBlock * kStrip;
constexpr int kTileK = 15;          // candidates kept per tile before it is marked dense
constexpr uint32_t kTableLdsBytes = 256u * 256u;  // T x 32 bank-disjoint copies
constexpr uint32_t kStageBytes = 64u * 128u;       // per-wave LDS-DMA image: 64 rows x 128 B
constexpr uint32_t kScanLdsBytes = kTableLdsBytes + kScanWaves * kStageBytes;
static_assert(kScanLdsBytes <= 160 * 1024, "scan kernel LDS budget");
constexpr int kCompactBlock = 1024;
constexpr int kSelectBlock = 1024;  // 16 files (waves) per block; the last block's tail (segment
                                    // compaction, LPT order) runs on all 1024 threads
constexpr int kHashBlock = 256;     // 64 quads (one segment each at a time) per block
constexpr int kHashWavesPerSimd = 2;  // 2 saturate VALU issue (SIMD-32)
constexpr uint64_t kDenseBit = 1ULL << 63;
constexpr uint64_t kNone = ~0ULL;
constexpr uint32_t kNoNext = 0xffffffffu;  // hash bins: no following segment
constexpr uint64_t kTailBytes = 256;  // zero-padded copy of the final partial 64-byte block

struct TileRec {
  uint32_t count;
  uint32_t off[kTileK];
};
static_assert(sizeof(TileRec) == 64, "tile record is one 64-byte line");
static_assert(sizeof(pfscdc_segment) == 56, "segment record layout");
static_assert(sizeof(pfscdc_ref) == 64, "ref record layout");

// Tuning knobs (knobs.cpp): process-wide integers, read from the environment once.
enum class Knob : int {
  ScanSkip, ScanCutSkip, ScanGrid,
  HashBinBytes, HashWaves, HashFair, HashFairEvery,
  RefIdSplit, CommitTwoSets, CommitLongPct,
  UwWorkers, UwInflight, UwMirror, UwIndexGrouped, UwArenaPoolBytes, CtxCache, CopyThreads,
  Trace,
  kCount
};
int64_t knob(Knob k);
// the knob's value, fixed from now on (pfscdc_set_knob to another value: PFSCDC_ESTATE)
int64_t knob_freeze(Knob k);

void generate_hashes(int64_t seed, uint64_t out[256]);
const pfscdc_params& ctx_params(const pfscdc_ctx* ctx);
void go_int63(int64_t seed, int64_t* out, int n);

// internal scan option: cut positions only (segment records without their BLAKE2b)
constexpr uint32_t kScanNoHash = 0x100;
// BLAKE2b-256 of n ranges [begins[i], begins[i] + sizes[i]) of device data, into out
int hash_records_device(pfscdc_ctx* ctx, const uint8_t* data, uint64_t nbytes,
                        const uint64_t* begins, const uint64_t* sizes, uint32_t n, uint8_t* out);
// pfscdc_scan with explicit options (the writer scans without per-segment refs).
int scan_sync(pfscdc_ctx* ctx, const void* bytes, uint64_t nbytes, int bytes_on_device,
              const uint64_t* file_offsets, uint32_t nfiles, uint32_t options);
// chunk.Create for chunks i = [offs[i], offs[i+1]) of the device buffer data (nbytes valid
// bytes; offs absolute, offs[0] may be > 0).  hashes (32 B per chunk, may be NULL): in where
// known[i], else out (Hash(chunk)).  refs: out.  Synchronous.
// ctext_out (device, nullable): the ciphertexts at the same offsets as data.
// sel (nullable): only chunks sel[0..nsel).  finish = false: enqueue only, then
// create_refs_finish(ctx) waits and writes hashes / refs.
int create_refs_device(pfscdc_ctx* ctx, const uint8_t* data, uint64_t nbytes,
                       const uint64_t* offs, uint32_t n, uint8_t* hashes, const uint8_t* known,
                       pfscdc_ref* refs, uint8_t* ctext_out = nullptr,
                       const uint32_t* sel = nullptr, uint32_t nsel = 0, bool finish = true);
int create_refs_finish(pfscdc_ctx* ctx);
// pfscdc_ctx_create on a given stream (shared: the ctx creates none and never destroys it)
int ctx_create_on(const pfscdc_params* params, int device, hipStream_t shared, pfscdc_ctx** out);
int ctx_device(const pfscdc_ctx* ctx);
// grow-only device staging owned by the ctx (writers_close_group): bytes, and the
// ciphertexts when ctext; both stay valid until the next call or pfscdc_ctx_destroy
hipError_t ctx_group_buffers(pfscdc_ctx* ctx, uint64_t bytes, bool ctext, uint8_t** d,
                             uint8_t** dct);
// pfscdc_writer_close of n writers on one ctx with one scan, one hash launch (every piece and
// multi-piece chunk) and one chunk.Create pass; stage_ms (nullable, 6 doubles) accumulates
// upload, scan, replay, hashes, create, callbacks
// wait_events: the group's input is on the device once these have fired (uploads made
// during the Puts); spans with a device copy are then gathered device to device
int writers_close_group(pfscdc_writer* const* ws, size_t n, double* stage_ms = nullptr,
                        const hipEvent_t* wait_events = nullptr, size_t n_wait = 0);
// a write whose bytes stay owned by the caller until the writer flushes or closes; dev
// (nullable): the same bytes already on the writer's device
int writer_write_span(pfscdc_writer* w, const uint8_t* p, uint64_t n,
                      const uint8_t* dev = nullptr);
uint32_t ctx_options(const pfscdc_ctx* ctx);
// the last completed scan: still readable (no create_refs / get_chunks since), its files
bool ctx_scan_valid(const pfscdc_ctx* ctx);
uint32_t ctx_nfiles(const pfscdc_ctx* ctx);
uint64_t ctx_file_offset(const pfscdc_ctx* ctx, uint32_t f);
// pfscdc_wait; fetch = false leaves the segment records and refs on the device (the host
// gets the per-file segment counts only): a device group gathers them over xGMI
int wait_impl(pfscdc_ctx* ctx, bool fetch);
// the last waited-for scan's device records: segments, refs (nullptr without Ref ids), count
void ctx_device_results(const pfscdc_ctx* ctx, pfscdc_segment** segs, pfscdc_ref** refs,
                        uint64_t* n);
hipStream_t ctx_stream(const pfscdc_ctx* ctx);

hipError_t prepare_kernels();  // per-device kernel attributes; call after hipSetDevice

// Scan work unit = one wave's 64 strips of a tile; kUnitSteps 128-byte strip steps of
// kUnitStep bytes each.
constexpr uint64_t kScanUnit = 64ull * kStrip;
constexpr uint64_t kUnitStep = 64ull * 128;
constexpr uint32_t kUnitSteps = kStrip / 128;
// Cut skipping past settled cuts (scan_skip_kernel + scan_slots_kernel): the
// work units go out in rank order (rank = the unit's index past the unit holding its file's
// first eligible position; every file's rank-k unit before any file's rank-(k+1) unit); each
// unit of rank < kRankSlots leaves one 32-bit word in its file's rank slots -- done bit, and
// kScanUnit - (its lowest candidate's offset in the unit) -- and a unit that finds the file's
// cuts before it settled by those slots skips the min - 1 positions after the last of them.
// Needs min - 1 >= kScanUnit: a unit's eligible positions then belong to one file.
constexpr uint32_t kPlanBuckets = 64;  // ranks >= 63 share the last bucket
constexpr uint32_t kPlanWords = 2 + kPlanBuckets;  // [0] slots used, [1] done ctr, cursors
constexpr uint32_t kPlanMaxFiles = 1u << 24;       // a slot's file | rank << 24 in one word
constexpr uint32_t kRankSlots = 64;                // per file: one wave reads them all
constexpr uint32_t kSlotDone = 1u << 31;
// in device memory (the scan kernel takes its address: one pointer live across the scan)
struct ScanPlan {
  const uint4* slots;     // per dispatch slot {unit, file, skip | rank << 8, 0}
  const uint32_t* plan;   // plan words ([0] = slots used)
  const uint32_t* uinfo;  // per unit {file (~0u: not scanned), skip | rank << 8}
  uint32_t* rslots;       // per file kRankSlots words (zeroed before the scan)
  const uint64_t* offs;   // file offsets (nfiles + 1)
  uint64_t min_chunk, max_chunk;
  unsigned long long* dyn_skipped;  // bytes the settled cuts removed from the scan
};
hipError_t launch_scan(const uint8_t* data, const uint8_t* tail, uint64_t n, const uint64_t* d_table,
                       uint32_t average_bits, uint64_t ntiles, TileRec* recs, int grid,
                       uint32_t* unit_ctr, uint32_t* done_ctr, uint64_t* entries,
                       uint64_t* n_entries, uint64_t* span, hipStream_t st,
                       const uint32_t* skip = nullptr, const ScanPlan* d_plan = nullptr);
// per scan work unit, the leading 128-B strip steps below its first eligible cut position
// (file start + min - 1); *scanned += the bytes the scan still covers
hipError_t launch_scan_skip(const uint64_t* offs, uint32_t nfiles, uint64_t n, uint64_t min_chunk,
                            uint64_t ntiles, uint32_t* skip, uint64_t* scanned, hipStream_t st);
// the same, plus the rank-ordered dispatch slots of the cut-skipping scan: uinfo (2 words
// per unit), slots (one per unit), plan (kPlanWords, zeroed); hdr
// is stored at d_hdr for the scan kernel
hipError_t launch_scan_plan(const uint64_t* offs, uint32_t nfiles, uint64_t n, uint64_t min_chunk,
                            uint64_t ntiles, uint32_t* skip, uint64_t* scanned, uint32_t* uinfo,
                            uint4* slots, uint32_t* plan, const ScanPlan& hdr, ScanPlan* d_hdr,
                            hipStream_t st);
hipError_t launch_compact(const TileRec* recs, uint64_t ntiles, uint64_t n, uint64_t* entries,
                          uint64_t* n_entries, hipStream_t st);
hipError_t launch_select(const uint8_t* data, const uint64_t* d_table, const uint64_t* entries,
                         const uint64_t* n_entries, const uint64_t* offs,
                         const uint64_t* seg_base, uint32_t nfiles, uint32_t average_bits,
                         uint64_t min_chunk, uint64_t max_chunk, pfscdc_segment* slots,
                         uint64_t* nseg, uint32_t* done_ctr, pfscdc_segment* segs,
                         uint64_t* seg_begin, uint32_t* order, uint32_t* counter,
                         hipStream_t st, uint64_t bin_bytes = 0, uint32_t* next = nullptr,
                         uint64_t* qlen = nullptr);
hipError_t launch_segcompact(const pfscdc_segment* slots, const uint64_t* seg_base,
                             const uint64_t* nseg, uint32_t nfiles, pfscdc_segment* segs,
                             uint64_t* seg_begin, hipStream_t st);
// Hash issue priority (launcher argument prio): 0 = the default (kHashPrioAuto: raise it for
// chains of more than 8192 blocks when quads refill), kHashPrioNone = never, else a threshold
// in 128-B blocks.
constexpr uint32_t kHashPrioAuto = 0x3fffffffu;
constexpr uint32_t kHashPrioNone = 0x80000000u;
hipError_t launch_blake2b(const uint8_t* data, const uint64_t* offs, pfscdc_segment* segs,
                          const uint64_t* seg_count, uint64_t max_segments, uint32_t* order,
                          uint32_t* counter, int num_cus, uint64_t nbytes, hipStream_t st,
                          bool ordered = false, uint64_t* span = nullptr, int waves = 0,
                          uint32_t prio = 0,  // issue priority (see kHashPrioNone)
                          bool cu_exclusive = false,  // one workgroup per CU (see launcher)
                          const uint32_t* next = nullptr,  // hash bins (lpt_order_block)
                          uint64_t* fair = nullptr,  // bins: fair-share counter (zeroed)
                          uint32_t fair_every = 256);  // blocks between fair-share updates
// waves per SIMD for a hash launch over chains of at most longest_bytes, total_bytes in all;
// forced in 1..8 (the PFSCDC_HASH_WAVES knob) overrides
int hash_waves(uint64_t longest_bytes, uint64_t total_bytes, int num_cus, int forced);
hipError_t launch_order(const pfscdc_segment* segs, const uint64_t* seg_count, uint32_t* order,
                        uint32_t* counter, hipStream_t st);
hipError_t launch_ref_ids(const uint8_t* data, const uint64_t* offs, pfscdc_segment* segs,
                          const uint64_t* seg_count, uint64_t max_segments, const uint32_t* order,
                          uint32_t* counter, int num_cus, uint64_t nbytes, pfscdc_ref* refs,
                          uint8_t* ctext_out, hipStream_t st, int waves = 0, uint32_t prio = 0,
                          const uint32_t* next = nullptr,  // hash bins: seg_count = queue length
                          const uint64_t* nsegs = nullptr);  // then: the segment count (deks)
// dek per record (refs[].dek from segs[].hash); zeroes *counter
hipError_t launch_deks(pfscdc_segment* segs, const uint64_t* seg_count, uint64_t max_segments,
                       pfscdc_ref* refs, uint32_t* counter, hipStream_t st);
// out[range of record r] = ChaCha20_{refs[r].dek}(data[range]); blk_base: prefix of 64-B blocks
hipError_t launch_chacha_xor(const uint8_t* data, const uint64_t* offs, const pfscdc_segment* segs,
                             const uint64_t* blk_base, uint32_t n, uint64_t nblocks,
                             const pfscdc_ref* refs, uint8_t* out, int num_cus, hipStream_t st,
                             bool prio = false, bool one_wave_per_simd = false);
hipError_t launch_get(const uint8_t* ctext, const uint64_t* offs, pfscdc_segment* segs,
                      const uint64_t* seg_count, uint64_t nsegs, uint32_t* order, uint32_t* counter,
                      int num_cus, uint64_t nbytes, pfscdc_ref* refs, uint8_t* ptext, hipStream_t st,
                      int waves = 0);
// segs[i].file += base for i < n (a device group's gathered index: member-local file ids
// become the commit's)
hipError_t launch_rebase_files(pfscdc_segment* segs, uint64_t n, uint32_t base, hipStream_t st);
hipError_t launch_synth(uint8_t* out, const uint64_t* offs, uint32_t nfiles, const uint32_t* ids,
                        const uint64_t* starts, uint64_t seed, uint32_t mode, hipStream_t st);

}  // namespace pfscdc
