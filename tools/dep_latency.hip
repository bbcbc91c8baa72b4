// dep_latency.hip — dependent-issue latency of the instruction pairs in the BLAKE2b G, one
// wave alone on its SIMD (development tool, not product).  Each probe is a chain in which
// every instruction reads the previous one's result; cycles per instruction from s_memtime.
// Also: the hand-scheduled G (22 VALU) as in the kernel and reordered forms, one wave.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define REPS 256
#define R16(x) ".rept 16\n" x ".endr\n"
#define DPP(P) " quad_perm:" P " row_mask:0xf bank_mask:0xf\n"

// chains over v[100:111]; every probe body is a repeated group whose instructions each depend
// on the one before (pairs noted in the names)
#define P_XOR_XOR "v_xor_b32 v100, v100, v101\n"
#define P_ALB_ALB "v_alignbit_b32 v100, v100, v101, 24\n"
#define P_L64_L64 "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"
#define P_XOR_ALB "v_xor_b32 v100, v100, v101\nv_alignbit_b32 v100, v100, v102, 24\n"
#define P_ALB_L64 "v_alignbit_b32 v100, v100, v101, 24\nv_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"
#define P_L64_XOR "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\nv_xor_b32 v100, v100, v104\n"
#define P_L64_XORHI "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\nv_xor_b32 v101, v101, v104\n"
#define P_XOR_L64 "v_xor_b32 v100, v100, v104\nv_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"
#define P_ADDC_PAIR "v_add_co_u32 v100, vcc, v100, v102\nv_addc_co_u32 v101, vcc, v101, v103, vcc\n"
#define P_ADDCDPP_PAIR "v_add_co_u32_dpp v100, vcc, v102, v100" DPP("[1,2,3,0]") "v_addc_co_u32_dpp v101, vcc, v103, v101, vcc" DPP("[1,2,3,0]")
#define P_ADDC_XOR "v_add_co_u32 v100, vcc, v100, v102\nv_addc_co_u32 v101, vcc, v101, v103, vcc\nv_xor_b32 v100, v101, v100\n"
#define P_XDPP_ADDCDPP "v_xor_b32_dpp v100, v101, v100" DPP("[1,2,3,0]") "v_add_co_u32_dpp v100, vcc, v102, v100" DPP("[1,2,3,0]")
#define P_ALB_XOR "v_alignbit_b32 v100, v100, v101, 24\nv_xor_b32 v100, v100, v102\n"
#define P_ALB_XDPP "v_alignbit_b32 v100, v100, v101, 24\ns_nop 1\nv_xor_b32_dpp v100, v100, v102" DPP("[1,2,3,0]")

// the kernel's G (column layout after a diagonal step: DPP operands on first uses)
#define G_ASM(X, Y)                                                     \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " X "\n"                   \
  "v_add_co_u32_dpp v100, vcc, v102, v100" DPP("[3,0,1,2]")             \
  "v_addc_co_u32_dpp v101, vcc, v103, v101, vcc" DPP("[3,0,1,2]")       \
  "v_xor_b32_dpp v108, v107, v101" DPP("[1,2,3,0]")                     \
  "v_xor_b32_dpp v109, v106, v100" DPP("[1,2,3,0]")                     \
  "v_add_co_u32_dpp v104, vcc, v104, v108" DPP("[2,3,0,1]")             \
  "v_addc_co_u32_dpp v105, vcc, v105, v109, vcc" DPP("[2,3,0,1]")       \
  "v_xor_b32_dpp v110, v102, v104" DPP("[3,0,1,2]")                     \
  "v_xor_b32_dpp v111, v103, v105" DPP("[3,0,1,2]")                     \
  "v_alignbit_b32 v102, v111, v110, 24\n"                               \
  "v_alignbit_b32 v103, v110, v111, 24\n"                               \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " Y "\n"                   \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"              \
  "v_xor_b32 v110, v108, v100\n"                                        \
  "v_xor_b32 v111, v109, v101\n"                                        \
  "v_alignbit_b32 v106, v111, v110, 16\n"                               \
  "v_alignbit_b32 v107, v110, v111, 16\n"                               \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[106:107]\n"              \
  "v_xor_b32 v110, v102, v104\n"                                        \
  "v_xor_b32 v111, v103, v105\n"                                        \
  "v_alignbit_b32 v102, v110, v111, 31\n"                               \
  "v_alignbit_b32 v103, v111, v110, 31\n"
// the same G with a + y hoisted next to the first half (a + b' + x + y = (a + b' + x) + y,
// and d' ^ a has already read a), filling the c + d carry chain's wait
#define G_HOIST(X, Y)                                                   \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " X "\n"                   \
  "v_add_co_u32_dpp v100, vcc, v102, v100" DPP("[3,0,1,2]")             \
  "v_addc_co_u32_dpp v101, vcc, v103, v101, vcc" DPP("[3,0,1,2]")       \
  "v_xor_b32_dpp v108, v107, v101" DPP("[1,2,3,0]")                     \
  "v_xor_b32_dpp v109, v106, v100" DPP("[1,2,3,0]")                     \
  "v_add_co_u32_dpp v104, vcc, v104, v108" DPP("[2,3,0,1]")             \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, " Y "\n"                   \
  "v_addc_co_u32_dpp v105, vcc, v105, v109, vcc" DPP("[2,3,0,1]")       \
  "v_xor_b32_dpp v110, v102, v104" DPP("[3,0,1,2]")                     \
  "v_xor_b32_dpp v111, v103, v105" DPP("[3,0,1,2]")                     \
  "v_alignbit_b32 v102, v111, v110, 24\n"                               \
  "v_alignbit_b32 v103, v110, v111, 24\n"                               \
  "v_lshl_add_u64 v[100:101], v[100:101], 0, v[102:103]\n"              \
  "v_xor_b32 v110, v108, v100\n"                                        \
  "v_xor_b32 v111, v109, v101\n"                                        \
  "v_alignbit_b32 v106, v111, v110, 16\n"                               \
  "v_alignbit_b32 v107, v110, v111, 16\n"                               \
  "v_lshl_add_u64 v[104:105], v[104:105], 0, v[106:107]\n"              \
  "v_xor_b32 v110, v102, v104\n"                                        \
  "v_xor_b32 v111, v103, v105\n"                                        \
  "v_alignbit_b32 v102, v110, v111, 31\n"                               \
  "v_alignbit_b32 v103, v111, v110, 31\n"

// a long G chain (one wave): s_memtime cycles vs wall time = the shader clock a lone wave
// runs at
__global__ void g_long(uint64_t* out, uint32_t seed, int iters) {
  uint64_t x = seed, y = seed * 7ull;
  asm volatile("v_mov_b32 v100, %0\nv_mov_b32 v101, %0\nv_mov_b32 v102, %0\nv_mov_b32 v103, %0\n"
               "v_mov_b32 v104, %0\nv_mov_b32 v105, %0\nv_mov_b32 v106, %0\nv_mov_b32 v107, %0\n"
               "s_nop 4\n" ::"v"(seed)
               : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < iters; r++)
    asm volatile(".rept 4\n" G_ASM("%0", "%1") ".endr\n" ::"v"(x), "v"(y)
                 : "vcc", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                   "v108", "v109", "v110", "v111");
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
}

template <int K>
__global__ void probe(uint64_t* out, uint32_t seed) {
  uint64_t t0 = 0, t1 = 0;
  uint64_t x = seed, y = seed * 7ull;
  asm volatile("v_mov_b32 v100, %0\nv_mov_b32 v101, %0\nv_mov_b32 v102, %0\nv_mov_b32 v103, %0\n"
               "v_mov_b32 v104, %0\nv_mov_b32 v105, %0\nv_mov_b32 v106, %0\nv_mov_b32 v107, %0\n"
               "v_mov_b32 v108, %0\nv_mov_b32 v109, %0\nv_mov_b32 v110, %0\nv_mov_b32 v111, %0\n"
               "s_nop 4\n" ::"v"(seed)
               : "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109",
                 "v110", "v111");
  t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) {
#define RUN(BODY) asm volatile(R16(BODY) ::: "vcc", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111")
    if constexpr (K == 0) RUN(P_XOR_XOR);
    if constexpr (K == 1) RUN(P_ALB_ALB);
    if constexpr (K == 2) RUN(P_L64_L64);
    if constexpr (K == 3) RUN(P_XOR_ALB);
    if constexpr (K == 4) RUN(P_ALB_L64);
    if constexpr (K == 5) RUN(P_L64_XOR);
    if constexpr (K == 6) RUN(P_L64_XORHI);
    if constexpr (K == 7) RUN(P_XOR_L64);
    if constexpr (K == 8) RUN(P_ADDC_PAIR);
    if constexpr (K == 9) RUN(P_ADDCDPP_PAIR);
    if constexpr (K == 10) RUN(P_ADDC_XOR);
    if constexpr (K == 11) RUN(P_XDPP_ADDCDPP);
    if constexpr (K == 12) RUN(P_ALB_XOR);
    if constexpr (K == 13) RUN(P_ALB_XDPP);
    if constexpr (K == 20)
      asm volatile(".rept 4\n" G_ASM("%0", "%1") ".endr\n" ::"v"(x), "v"(y)
                   : "vcc", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                     "v108", "v109", "v110", "v111");
    if constexpr (K == 21)
      asm volatile(".rept 4\n" G_HOIST("%0", "%1") ".endr\n" ::"v"(x), "v"(y)
                   : "vcc", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107",
                     "v108", "v109", "v110", "v111");
  }
  t1 = __builtin_amdgcn_s_memtime();
  uint32_t v;
  asm volatile("v_mov_b32 %0, v100" : "=v"(v));
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (v == 0x12345678u) out[1000] = v;
}

int main() {
  uint64_t* d = nullptr;
  if (hipMalloc(&d, 8 * 1024) != hipSuccess) return 1;
  struct P {
    const char* name;
    void (*k)(uint64_t*, uint32_t);
    double per_rep;  // instructions (or G's) per repetition of the asm body
  } ps[] = {
      {"xor->xor", probe<0>, 16}, {"alignbit->alignbit", probe<1>, 16},
      {"lshl_add_u64->lshl_add_u64", probe<2>, 16}, {"xor->alignbit (pair)", probe<3>, 32},
      {"alignbit->lshl_add_u64 (pair)", probe<4>, 32}, {"lshl_add_u64->xor lo (pair)", probe<5>, 32},
      {"lshl_add_u64->xor hi (pair)", probe<6>, 32}, {"xor->lshl_add_u64 (pair)", probe<7>, 32},
      {"add_co->addc (pair)", probe<8>, 32}, {"add_co_dpp->addc_dpp (pair)", probe<9>, 32},
      {"add_co->addc->xor (triple)", probe<10>, 48}, {"xor_dpp->add_co_dpp (pair)", probe<11>, 32},
      {"alignbit->xor (pair)", probe<12>, 32}, {"alignbit->nop1->xor_dpp", probe<13>, 32},
  };
  uint64_t h;
  printf("dependent chains, one wave alone on its SIMD: cycles per instruction\n");
  for (auto& p : ps) {
    p.k<<<1, 64>>>(d, 1);
    (void)hipDeviceSynchronize();
    p.k<<<1, 64>>>(d, 1);
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("%-34s %.2f\n", p.name, (double)h / (REPS * p.per_rep));
  }
  const struct {
    const char* name;
    void (*k)(uint64_t*, uint32_t);
  } gs[] = {{"G as in the kernel (22 VALU)", probe<20>}, {"G with a+y hoisted (22 VALU)", probe<21>}};
  for (auto& g : gs) {
    for (int w : {1, 2}) {
      g.k<<<256 * w, 64 * 4>>>(d, 1);  // w waves per SIMD on every CU
      (void)hipDeviceSynchronize();
      g.k<<<1, 64 * w>>>(d, 1);  // 1 or 2 waves in one CU (waves spread over SIMDs: w=1 lone)
      (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
      printf("%-34s 1 block of %d wave(s): %.1f cycles per G\n", g.name, w, (double)h / (REPS * 4));
    }
  }
  {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 20000;
    g_long<<<1, 64>>>(d, 1, 100);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    g_long<<<1, 64>>>(d, 1, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    printf("lone wave, %d G: %.1f cycles per G, %.3f ms -> shader clock %.2f GHz, %.1f ns per G\n",
           iters * 4, (double)h / (iters * 4.0), ms, (double)h / (ms * 1e6),
           ms * 1e6 / (iters * 4.0));
  }
  return 0;
}
