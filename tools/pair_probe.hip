// pair_probe.hip — does gfx950 co-issue the simple VALU ops of two waves that share a SIMD
// when the waves run in phase?  (development tool, not product)
// One workgroup of 8 waves per CU (2 per SIMD); the waves meet at a barrier, then run 12
// independent chains of a pattern.  Reported: SIMD cycles per pattern step (wall clock x
// measured shader clock / steps per SIMD).  Variants start the two waves of a SIMD in phase
// (barrier) or half a run apart (the odd waves first run 12 extra 4-cycle ops).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define REPS 1024
#define XOR(R) "v_xor_b32 " R ", " R ", %12\n"
#define ALB(R) "v_alignbit_b32 " R ", " R ", %12, 24\n"
#define ALL12(M) M("%0") M("%1") M("%2") M("%3") M("%4") M("%5") M("%6") M("%7") M("%8") M("%9") M("%10") M("%11")
#define OPS                                                                                  \
  : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),       \
    "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11])                              \
  : "v"(b)
#define XA(R) XOR(R) ALB(R)

template <int K, bool SKEW>
__global__ __launch_bounds__(512) void probe(uint64_t* out, uint32_t seed) {
  uint32_t a[12];
#pragma unroll
  for (int i = 0; i < 12; i++) a[i] = seed * (i + 3) + threadIdx.x;
  const uint32_t b = seed * 17 + 1;
  __syncthreads();
  if (SKEW && ((threadIdx.x >> 6) & 4)) asm volatile(ALL12(ALB) OPS);  // waves 4-7: half a run late
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) {
    if constexpr (K == 0) asm volatile(ALL12(XOR) ALL12(XOR) OPS);           // 24 simple
    if constexpr (K == 1) asm volatile(ALL12(XA) OPS);                       // alternate
    if constexpr (K == 2) asm volatile(ALL12(XOR) ALL12(ALB) OPS);           // runs of 12
    if constexpr (K == 3) asm volatile(ALL12(ALB) ALL12(ALB) OPS);           // 24 complex
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s ^= a[i];
  if (s == 0x12345678u) out[1 << 20] = s;
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  struct P { const char* name; void (*k)(uint64_t*, uint32_t); } ps[] = {
      {"24 x v_xor_b32            in phase", probe<0, false>},
      {"24 x v_alignbit_b32       in phase", probe<3, false>},
      {"xor,alignbit alternating  in phase", probe<1, false>},
      {"12 xor then 12 alignbit   in phase", probe<2, false>},
      {"xor,alignbit alternating  skewed  ", probe<1, true>},
      {"12 xor then 12 alignbit   skewed  ", probe<2, true>},
  };
  int ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) ncu = prop.multiProcessorCount;
  uint64_t* d = nullptr;
  if (hipMalloc(&d, 8 * ((1 << 20) + 1)) != hipSuccess) return 1;
  static uint64_t h[256 * 8 * 4];
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  printf("%d CUs, 2 waves per SIMD (one 512-thread workgroup per CU), 24 VALU x %d per wave\n", ncu, REPS);
  printf("pattern                               SIMD cycles per VALU instruction (wall x clock)\n");
  for (auto& p : ps) {
    p.k<<<ncu, 512>>>(d, 1);  // warm
    hipEventRecord(e0);
    p.k<<<ncu, 512>>>(d, 2);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipMemcpy(h, d, 8 * ncu * 8, hipMemcpyDeviceToHost);
    uint64_t mx = 0;
    for (int i = 0; i < ncu * 8; i++) mx = h[i] > mx ? h[i] : mx;
    const double clk = (double)mx / (ms * 1e6);         // s_memtime cycles per ns (upper bound)
    const double instr = 2.0 * 24.0 * REPS;             // per SIMD: 2 waves x 24 x REPS
    printf("%s   %6.2f   (s_memtime span %6.2f, clock %.2f GHz)\n", p.name,
           ms * 1e6 * clk / instr, (double)mx / instr, clk);
  }
  return 0;
}
