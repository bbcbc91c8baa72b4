// g_probe.hip — SIMD throughput of the hand-scheduled BLAKE2b G (development tool).
// Every wave runs `iters` x 8 G functions on registers only; reports cycles per G per SIMD
// (wall time x clock / (G's per SIMD)) for 1, 2 and 4 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define DPP(P) " quad_perm:" P " row_mask:0xf bank_mask:0xf\n"
#define G_DPP(PB, PC, PD)                                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[112:113]\n"             \
  "v_add_co_u32_dpp v100, vcc, v102, v100" DPP(PB)                     \
  "v_addc_co_u32_dpp v101, vcc, v103, v101, vcc" DPP(PB)               \
  "v_xor_b32_dpp v108, v107, v101" DPP(PD)                             \
  "v_xor_b32_dpp v109, v106, v100" DPP(PD)                             \
  "v_add_co_u32_dpp v104, vcc, v104, v108" DPP(PC)                     \
  "v_addc_co_u32_dpp v105, vcc, v105, v109, vcc" DPP(PC)               \
  "v_xor_b32_dpp v110, v102, v104" DPP(PB)                             \
  "v_xor_b32_dpp v111, v103, v105" DPP(PB)                             \
  "v_alignbit_b32 v102, v111, v110, 24\n"                              \
  "v_alignbit_b32 v103, v110, v111, 24\n"                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[114:115]\n"             \
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
// same instruction count, no DPP (plain VOP2 adds/xors)
#define G_PLAIN                                                        \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[112:113]\n"             \
  "v_add_co_u32 v100, vcc, v102, v100\n"                               \
  "v_addc_co_u32 v101, vcc, v103, v101, vcc\n"                         \
  "v_xor_b32 v108, v107, v101\n"                                       \
  "v_xor_b32 v109, v106, v100\n"                                       \
  "v_add_co_u32 v104, vcc, v104, v108\n"                               \
  "v_addc_co_u32 v105, vcc, v105, v109, vcc\n"                         \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v111, v110, 24\n"                              \
  "v_alignbit_b32 v103, v110, v111, 24\n"                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[114:115]\n"             \
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
// the G's 64-bit adds as v_lshl_add_u64 only (20 instrs; b and c not permuted)
#define G_LSHL                                                         \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[112:113]\n"             \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"             \
  "v_xor_b32 v108, v107, v101\n"                                       \
  "v_xor_b32 v109, v106, v100\n"                                       \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[108:109]\n"             \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v111, v110, 24\n"                              \
  "v_alignbit_b32 v103, v110, v111, 24\n"                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[114:115]\n"             \
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
// latency form: 64-bit adds as v_lshl_add_u64, the quad rotations as separate DPP moves
// (b moved first behind an s_nop, so a + b' is not delayed)
#define G_LAT1(PB, PC, PD)                                             \
  "s_nop 1\n"                                                          \
  "v_mov_b32_dpp v102, v102" DPP(PB)                                   \
  "v_mov_b32_dpp v103, v103" DPP(PB)                                   \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[112:113]\n"             \
  "v_mov_b32_dpp v106, v106" DPP(PD)                                   \
  "v_mov_b32_dpp v107, v107" DPP(PD)                                   \
  "v_mov_b32_dpp v104, v104" DPP(PC)                                   \
  "v_mov_b32_dpp v105, v105" DPP(PC)                                   \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"             \
  "v_xor_b32 v108, v107, v101\n"                                       \
  "v_xor_b32 v109, v106, v100\n"                                       \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[108:109]\n"             \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v111, v110, 24\n"                              \
  "v_alignbit_b32 v103, v110, v111, 24\n"                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[114:115]\n"             \
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
// b moved last (no s_nop)
#define G_LAT2(PB, PC, PD)                                             \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[112:113]\n"             \
  "v_mov_b32_dpp v106, v106" DPP(PD)                                   \
  "v_mov_b32_dpp v107, v107" DPP(PD)                                   \
  "v_mov_b32_dpp v104, v104" DPP(PC)                                   \
  "v_mov_b32_dpp v105, v105" DPP(PC)                                   \
  "v_mov_b32_dpp v102, v102" DPP(PB)                                   \
  "v_mov_b32_dpp v103, v103" DPP(PB)                                   \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"             \
  "v_xor_b32 v108, v107, v101\n"                                       \
  "v_xor_b32 v109, v106, v100\n"                                       \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[108:109]\n"             \
  "v_xor_b32 v110, v102, v104\n"                                       \
  "v_xor_b32 v111, v103, v105\n"                                       \
  "v_alignbit_b32 v102, v111, v110, 24\n"                              \
  "v_alignbit_b32 v103, v110, v111, 24\n"                              \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[114:115]\n"             \
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
template <int V>
__global__ void gk(uint64_t* out, uint32_t iters, uint64_t seed) {
  uint64_t a = seed + threadIdx.x, b = a * 3, c = a ^ 5, d = a + 7, x = a * 11, y = a * 13;
  for (uint32_t i = 0; i < iters; i++) {
    if (V == 0) asm volatile("s_nop 1\n" G_DPP("[3,0,1,2]", "[2,3,0,1]", "[1,2,3,0]") G_DPP("[1,2,3,0]", "[2,3,0,1]", "[3,0,1,2]")
                             G_DPP("[3,0,1,2]", "[2,3,0,1]", "[1,2,3,0]") G_DPP("[1,2,3,0]", "[2,3,0,1]", "[3,0,1,2]")
                 : "+{v[100:101]}"(a), "+{v[102:103]}"(b), "+{v[104:105]}"(c), "+{v[106:107]}"(d)
                 : "{v[112:113]}"(x), "{v[114:115]}"(y) : "vcc", "v108", "v109", "v110", "v111");
    if (V == 1) asm volatile(G_PLAIN G_PLAIN G_PLAIN G_PLAIN
                 : "+{v[100:101]}"(a), "+{v[102:103]}"(b), "+{v[104:105]}"(c), "+{v[106:107]}"(d)
                 : "{v[112:113]}"(x), "{v[114:115]}"(y) : "vcc", "v108", "v109", "v110", "v111");
    if (V == 3) asm volatile(G_LAT1("[3,0,1,2]", "[2,3,0,1]", "[1,2,3,0]") G_LAT1("[1,2,3,0]", "[2,3,0,1]", "[3,0,1,2]")
                             G_LAT1("[3,0,1,2]", "[2,3,0,1]", "[1,2,3,0]") G_LAT1("[1,2,3,0]", "[2,3,0,1]", "[3,0,1,2]")
                 : "+{v[100:101]}"(a), "+{v[102:103]}"(b), "+{v[104:105]}"(c), "+{v[106:107]}"(d)
                 : "{v[112:113]}"(x), "{v[114:115]}"(y) : "vcc", "v108", "v109", "v110", "v111");
    if (V == 4) asm volatile(G_LAT2("[3,0,1,2]", "[2,3,0,1]", "[1,2,3,0]") G_LAT2("[1,2,3,0]", "[2,3,0,1]", "[3,0,1,2]")
                             G_LAT2("[3,0,1,2]", "[2,3,0,1]", "[1,2,3,0]") G_LAT2("[1,2,3,0]", "[2,3,0,1]", "[3,0,1,2]")
                 : "+{v[100:101]}"(a), "+{v[102:103]}"(b), "+{v[104:105]}"(c), "+{v[106:107]}"(d)
                 : "{v[112:113]}"(x), "{v[114:115]}"(y) : "vcc", "v108", "v109", "v110", "v111");
    if (V == 2) asm volatile(G_LSHL G_LSHL G_LSHL G_LSHL
                 : "+{v[100:101]}"(a), "+{v[102:103]}"(b), "+{v[104:105]}"(c), "+{v[106:107]}"(d)
                 : "{v[112:113]}"(x), "{v[114:115]}"(y) : "vcc", "v108", "v109", "v110", "v111");
  }
  if (threadIdx.x == 0) out[blockIdx.x] = a ^ b ^ c ^ d;
}
int main() {
  uint64_t* d; (void)hipMalloc(&d, 8 * 4096);
  void (*ks[])(uint64_t*, uint32_t, uint64_t) = {gk<0>, gk<1>, gk<2>, gk<3>, gk<4>};
  const char* nm[] = {"G dpp (22 instr)", "G plain (22)", "G lshl-only (20)", "G lat b-first (26)",
                      "G lat b-last (26)"};
  int ncu = 256; const uint32_t it = 4000;
  for (int V = 0; V < 5; V++) for (int w : {1, 2, 4}) {
    ks[V]<<<ncu, 256 * w>>>(d, 10, 1); (void)hipDeviceSynchronize();
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0); ks[V]<<<ncu, 256 * w>>>(d, it, 2); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double gs_per_simd = (double)w * it * 4;  // G functions per SIMD
    printf("%-18s %d wave/SIMD: %.2f ms, %.1f cycles per G per SIMD (@2.38 GHz)\n", nm[V], w, ms,
           ms * 1e-3 * 2.38e9 / gs_per_simd);
  }
  return 0;
}
