// valu_issue.hip — VALU issue rate of independent instruction streams on gfx950 at 1, 2, 4
// and 8 waves per SIMD (development tool, not product).  Settles which integer ops issue a
// wave64 instruction in ~2 cycles (the guide's SIMD-32 figure) and which take ~4: the
// ceiling that bounds the BLAKE2b and CDC kernels.
//
// Every wave runs 12 independent chains of one instruction (no dependency stalls even at one
// wave per SIMD).  The grid is 256 CUs x 4 SIMDs x W waves (blocks of 256 threads = one wave
// per SIMD each, W blocks per CU).  Reported: SIMD cycles per wave-instruction =
// (wall time x shader clock x 1024 SIMDs) / (wave-instructions issued), with the clock taken
// from s_memtime (shader cycles) over the slowest wave, and the same from wall time at the
// measured clock.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define REPS 2048
#define CH12(OP)                                                                              \
  asm volatile(".rept 4\n" OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6")     \
                   OP("%7") OP("%8") OP("%9") OP("%10") OP("%11") ".endr\n"                   \
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]),      \
                 "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11])     \
               : "v"(b), "v"(c)                                                               \
               : "vcc")
#define CH12_64(OP)                                                                           \
  asm volatile(".rept 4\n" OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6")     \
                   OP("%7") OP("%8") OP("%9") OP("%10") OP("%11") ".endr\n"                   \
               : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),      \
                 "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11])     \
               : "v"(y))

#define XOR(R) "v_xor_b32 " R ", " R ", %12\n"
#define AND(R) "v_and_b32 " R ", " R ", %12\n"
#define OR(R) "v_or_b32 " R ", " R ", %12\n"
#define ADDU(R) "v_add_u32 " R ", " R ", %12\n"
#define SUBU(R) "v_sub_u32 " R ", " R ", %12\n"
#define ADDCO(R) "v_add_co_u32 " R ", vcc, " R ", %12\n"
#define MOV(R) "v_mov_b32 " R ", %12\n"
#define ALB(R) "v_alignbit_b32 " R ", " R ", %12, 24\n"
#define ALBY(R) "v_alignbyte_b32 " R ", " R ", %12, 3\n"
#define PERM(R) "v_perm_b32 " R ", " R ", %12, %13\n"
#define B3(R) "v_bitop3_b32 " R ", " R ", %12, %13 bitop3:0x96\n"
#define ADD3(R) "v_add3_u32 " R ", " R ", %12, %13\n"
#define LSHLOR(R) "v_lshl_or_b32 " R ", " R ", 1, %13\n"
#define LSHR(R) "v_lshrrev_b32 " R ", 3, " R "\n"
#define XDPP(R) "v_xor_b32_dpp " R ", %12, " R " quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
#define MDPP(R) "v_mov_b32_dpp " R ", %12 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
#define CND(R) "v_cndmask_b32 " R ", " R ", %12, vcc\n"
#define ADDF(R) "v_add_f32 " R ", " R ", %12\n"
#define FMAF(R) "v_fma_f32 " R ", " R ", %12, %13\n"
#define PKADD16(R) "v_pk_add_u16 " R ", " R ", %12\n"
#define LSHL_ADD64(R) "v_lshl_add_u64 " R ", " R ", 0, %12\n"
#define LSHL64(R) "v_lshlrev_b64 " R ", 3, " R "\n"
#define PKFMA(R) "v_pk_fma_f32 " R ", " R ", %12, " R "\n"
#define PKADDF(R) "v_pk_add_f32 " R ", " R ", %12\n"
#define PKMOV(R) "v_pk_mov_b32 " R ", %12, " R " op_sel:[0,1]\n"
#define XSDWA(R) "v_xor_b32_sdwa " R ", " R ", %12 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1\n"
#define XSDWAP(R) "v_xor_b32_sdwa " R ", " R ", %12 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_0\n"
#define MIXXA(R) XOR(R) ALB(R)  /* one VOP2 + one VOP3 per chain step (counted as 2) */
// runs of k simple ops then k 4-cycle ops over k chains (each chain: one of each per step)
#define RUNS(K, OPS_X, OPS_A) asm volatile(".rept 4\n" OPS_X OPS_A ".endr\n" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), \
    "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]) : "v"(b), "v"(c))
#define X2(a0, a1) XOR(a0) XOR(a1)
#define A2(a0, a1) ALB(a0) ALB(a1)
#define RUN2 RUNS(2, X2("%0", "%1") A2("%0", "%1") X2("%2", "%3") A2("%2", "%3") X2("%4", "%5") A2("%4", "%5") \
    X2("%6", "%7") A2("%6", "%7") X2("%8", "%9") A2("%8", "%9") X2("%10", "%11") A2("%10", "%11"), "")
#define RUN3 RUNS(3, X2("%0", "%1") XOR("%2") A2("%0", "%1") ALB("%2") X2("%3", "%4") XOR("%5") A2("%3", "%4") ALB("%5") \
    X2("%6", "%7") XOR("%8") A2("%6", "%7") ALB("%8") X2("%9", "%10") XOR("%11") A2("%9", "%10") ALB("%11"), "")
#define RUN6 RUNS(6, X2("%0", "%1") X2("%2", "%3") X2("%4", "%5") A2("%0", "%1") A2("%2", "%3") A2("%4", "%5") \
    X2("%6", "%7") X2("%8", "%9") X2("%10", "%11") A2("%6", "%7") A2("%8", "%9") A2("%10", "%11"), "")
#define RUN12 RUNS(12, X2("%0", "%1") X2("%2", "%3") X2("%4", "%5") X2("%6", "%7") X2("%8", "%9") X2("%10", "%11"), \
    A2("%0", "%1") A2("%2", "%3") A2("%4", "%5") A2("%6", "%7") A2("%8", "%9") A2("%10", "%11"))

template <int K>
__global__ __launch_bounds__(256) void thr(uint64_t* out, uint32_t seed) {
  uint64_t t0, t1;
  if constexpr (K >= 100) {  // 64-bit operand instructions
    uint64_t x[12];
#pragma unroll
    for (int i = 0; i < 12; i++) x[i] = seed * (i + 3) + threadIdx.x;
    const uint64_t y = seed * 17ull + 1;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REPS; r++) {
      if constexpr (K == 100) CH12_64(LSHL_ADD64);
      if constexpr (K == 101) CH12_64(LSHL64);
      if constexpr (K == 102) CH12_64(PKFMA);
      if constexpr (K == 103) CH12_64(PKADDF);
      if constexpr (K == 104) CH12_64(PKMOV);
    }
    t1 = __builtin_amdgcn_s_memtime();
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) s ^= x[i];
    if (s == 0x123456789ull) out[1 << 20] = s;
  } else {
    uint32_t a[12];
#pragma unroll
    for (int i = 0; i < 12; i++) a[i] = seed * (i + 3) + threadIdx.x;
    const uint32_t b = seed * 17 + 1, c = seed ^ 0x99;
    t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REPS; r++) {
      if constexpr (K == 0) CH12(XOR);
      if constexpr (K == 1) CH12(AND);
      if constexpr (K == 2) CH12(OR);
      if constexpr (K == 3) CH12(ADDU);
      if constexpr (K == 4) CH12(SUBU);
      if constexpr (K == 5) CH12(ADDCO);
      if constexpr (K == 6) CH12(MOV);
      if constexpr (K == 7) CH12(ALB);
      if constexpr (K == 8) CH12(ALBY);
      if constexpr (K == 9) CH12(PERM);
      if constexpr (K == 10) CH12(B3);
      if constexpr (K == 11) CH12(ADD3);
      if constexpr (K == 12) CH12(LSHLOR);
      if constexpr (K == 13) CH12(LSHR);
      if constexpr (K == 14) CH12(XDPP);
      if constexpr (K == 15) CH12(MDPP);
      if constexpr (K == 16) CH12(CND);
      if constexpr (K == 17) CH12(ADDF);
      if constexpr (K == 18) CH12(FMAF);
      if constexpr (K == 19) CH12(PKADD16);
      if constexpr (K == 20) CH12(XSDWA);
      if constexpr (K == 21) CH12(XSDWAP);
      if constexpr (K == 22) CH12(MIXXA);
      if constexpr (K == 23) RUN2;
      if constexpr (K == 24) RUN3;
      if constexpr (K == 25) RUN6;
      if constexpr (K == 26) RUN12;
    }
    t1 = __builtin_amdgcn_s_memtime();
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) s ^= a[i];
    if (s == 0x12345678u) out[1 << 20] = s;
  }
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

struct Probe {
  const char* name;
  void (*k)(uint64_t*, uint32_t);
};

int main() {
  const Probe probes[] = {
      {"v_xor_b32", thr<0>},        {"v_and_b32", thr<1>},         {"v_or_b32", thr<2>},
      {"v_add_u32", thr<3>},        {"v_sub_u32", thr<4>},         {"v_add_co_u32", thr<5>},
      {"v_mov_b32", thr<6>},        {"v_alignbit_b32", thr<7>},    {"v_alignbyte_b32", thr<8>},
      {"v_perm_b32", thr<9>},       {"v_bitop3_b32", thr<10>},     {"v_add3_u32", thr<11>},
      {"v_lshl_or_b32", thr<12>},   {"v_lshrrev_b32", thr<13>},    {"v_xor_b32_dpp", thr<14>},
      {"v_mov_b32_dpp", thr<15>},   {"v_cndmask_b32", thr<16>},    {"v_add_f32", thr<17>},
      {"v_fma_f32", thr<18>},       {"v_pk_add_u16", thr<19>},     {"v_lshl_add_u64", thr<100>},
      {"v_lshlrev_b64", thr<101>},  {"v_pk_fma_f32", thr<102>},    {"v_pk_add_f32", thr<103>},
      {"v_pk_mov_b32", thr<104>},   {"v_xor_b32_sdwa (word, preserve)", thr<20>},
      {"v_xor_b32_sdwa (word, pad)", thr<21>}, {"v_xor_b32 + v_alignbit_b32 (per pair)", thr<22>},
      {"runs of 2 xor / 2 alignbit (per pair)", thr<23>}, {"runs of 3 / 3 (per pair)", thr<24>},
      {"runs of 6 / 6 (per pair)", thr<25>},  {"runs of 12 / 12 (per pair)", thr<26>},
  };
  int ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) ncu = prop.multiProcessorCount;
  const int nsimd = ncu * 4;
  uint64_t* d = nullptr;
  if (hipMalloc(&d, 8 * ((1 << 20) + 1)) != hipSuccess) return 1;
  static uint64_t h[8 * 256 * 4 * 8];
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double instr_per_wave = (double)REPS * 48.0;
  printf("%d CUs; 12 independent chains per wave, %d instructions per wave\n", ncu,
         (int)instr_per_wave);
  printf("%-16s %s\n", "instruction", "SIMD cycles per wave64 instruction at 1/2/4/8 waves per SIMD "
                                      "(s_memtime span of the slowest wave | wall x clock)");
  double clk = 2.4;
  for (const Probe& p : probes) {
    printf("%-16s", p.name);
    for (int w : {1, 2, 4, 8}) {
      const int blocks = ncu * w;
      p.k<<<blocks, 256>>>(d, 1);  // warm
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0);
      p.k<<<blocks, 256>>>(d, 1);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      (void)hipMemcpy(h, d, 8ull * blocks * 4, hipMemcpyDeviceToHost);
      uint64_t mx = 0;
      for (int i = 0; i < blocks * 4; i++) mx = h[i] > mx ? h[i] : mx;
      const double waves_per_simd = (double)blocks * 4 / nsimd;
      const double cyc = (double)mx / (waves_per_simd * instr_per_wave);
      const double clock_ghz = (double)mx / (ms * 1e6);  // shader cycles per ns over the launch
      const double cyc_wall = ms * 1e6 * clk / (waves_per_simd * instr_per_wave);
      printf("  %5.2f|%5.2f", cyc, cyc_wall);
      if (w == 1) clk = clock_ghz;  // one wave per SIMD: every wave resident for the whole launch
    }
    printf("   (clock %.2f GHz)\n", clk);
  }
  return 0;
}
