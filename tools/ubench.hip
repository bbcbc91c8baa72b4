// ubench.hip — instruction latency/throughput probes on gfx950 (development tool, not product).
// Each probe: one workgroup; s_memtime around REPS x 64 instructions in a dependent chain
// (or 4 interleaved chains).  Prints cycles per instruction.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define REPS 200
#define R64(x) ".rept 64\n" x "\n.endr\n"

template <int K> __global__ void probe(uint64_t* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3 + 1, c = seed ^ 0x55, d = seed + 7, e = 9;
  uint64_t x = seed, y = seed * 5, z = 3, w = 11;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < REPS; r++) {
    if (K == 0) asm volatile(R64("v_xor_b32 %0, %0, %1") : "+v"(a) : "v"(b));
    if (K == 1) asm volatile(R64("v_alignbit_b32 %0, %0, %1, 24") : "+v"(a) : "v"(b));
    if (K == 2) asm volatile(R64("v_lshl_add_u64 %0, %0, 0, %1") : "+v"(x) : "v"(y));
    if (K == 3) asm volatile(R64("v_add_co_u32 %0, vcc, %0, %2\nv_addc_co_u32 %1, vcc, %1, %3, vcc") : "+v"(a), "+v"(c) : "v"(b), "v"(d) : "vcc");
    if (K == 4) asm volatile(R64("s_nop 1\nv_mov_b32_dpp %0, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf") : "+v"(a));
    if (K == 5) asm volatile(R64("v_perm_b32 %0, %0, %1, %2") : "+v"(a) : "v"(b), "v"(c));
    if (K == 6) asm volatile(R64("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96") : "+v"(a) : "v"(b), "v"(c));
    // 4 independent chains interleaved
    if (K == 7) asm volatile(".rept 16\nv_xor_b32 %0, %0, %4\nv_xor_b32 %1, %1, %4\nv_xor_b32 %2, %2, %4\nv_xor_b32 %3, %3, %4\n.endr" : "+v"(a), "+v"(c), "+v"(d), "+v"(e) : "v"(b));
    if (K == 8) asm volatile(".rept 16\nv_lshl_add_u64 %0, %0, 0, %4\nv_lshl_add_u64 %1, %1, 0, %4\nv_lshl_add_u64 %2, %2, 0, %4\nv_lshl_add_u64 %3, %3, 0, %4\n.endr" : "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(y));
    if (K == 9) asm volatile(R64("v_mov_b32_dpp %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf") : "=v"(a) : "v"(b));
    if (K == 10) asm volatile(R64("v_xor_b32_dpp %0, %1, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf") : "+v"(a) : "v"(b));
    if (K == 11) asm volatile(R64("v_lshlrev_b64 %0, 3, %0") : "+v"(x));
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (a == 0x12345 && x == 7 && c == 3 && y == 1 && z == 2 && w == 3 && d == 4 && e == 5) out[1000] = 1;
}

// LDS pointer chase: ds_read_b32 latency
__global__ void lds_chase(uint64_t* out) {
  __shared__ uint32_t s[1024];
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) s[i] = ((i + 1) & 1023) * 4;
  __syncthreads();
  uint32_t p = threadIdx.x * 4 % 4096;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < 2000; r++) p = *(volatile uint32_t*)((char*)s + p);
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (p == 0xffffffff) out[1] = 1;
}

// memory access pattern probes over a 4 GiB buffer: fully coalesced vs per-lane strips
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void rd_coalesced(const u32x4* __restrict__ p, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    u32x4 v = __builtin_nontemporal_load(p + i); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x1234567) out[0] = acc;
}
template <int S>  // each lane walks a 4 KiB strip, strips S bytes apart (S >= 4096)
__global__ void rd_stride(const uint8_t* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  const uint64_t tile = (uint64_t)blockDim.x * S;
  for (uint64_t t = blockIdx.x; (t + 1) * tile <= n; t += gridDim.x) {
    const uint8_t* s = p + t * tile + threadIdx.x * (uint64_t)S;
    for (int o = 0; o < 4096; o += 64) {
#pragma unroll
      for (int k = 0; k < 4; k++) { u32x4 v = __builtin_nontemporal_load((const u32x4*)(s + o) + k); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}
// 4 lanes per strip per instruction: instruction i covers strips 16i..16i+15, 64 B each
__global__ void rd_strip4(const uint8_t* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  const uint64_t tile = (uint64_t)blockDim.x * 4096;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (uint64_t t = blockIdx.x; t * tile < n; t += gridDim.x) {
    const uint8_t* w = p + t * tile + (uint64_t)wave * 64 * 4096;
    for (int o = 0; o < 4096; o += 64) {
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint8_t* q = w + (uint64_t)(16 * i + (lane >> 2)) * 4096 + o + (lane & 3) * 16;
        u32x4 v = __builtin_nontemporal_load((const u32x4*)q); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}
// lane l owns the 64-byte block l of each 4 KiB wave chunk (4 instructions, lane stride 64 B)
__global__ void rd_block64(const uint8_t* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  const int lane = threadIdx.x & 63;
  const uint64_t nchunk = n / 4096, wid = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
  const uint64_t nw = (uint64_t)gridDim.x * blockDim.x / 64;
  for (uint64_t c = wid; c < nchunk; c += nw) {
    const uint8_t* q = p + c * 4096 + lane * 64;
#pragma unroll
    for (int k = 0; k < 4; k++) { u32x4 v = __builtin_nontemporal_load((const u32x4*)q + k); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  }
  if (acc == 0x1234567) out[0] = acc;
}
template <int BLK>  // each lane walks a 4 KiB strip in BLK-byte steps
__global__ void rd_strip(const uint8_t* __restrict__ p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  const uint64_t tile = (uint64_t)blockDim.x * 4096;
  for (uint64_t t = blockIdx.x; t * tile < n; t += gridDim.x) {
    const uint8_t* s = p + t * tile + threadIdx.x * 4096ull;
    for (int o = 0; o < 4096; o += BLK) {
#pragma unroll
      for (int k = 0; k < BLK / 16; k++) { u32x4 v = __builtin_nontemporal_load((const u32x4*)(s + o) + k); acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
  }
  if (acc == 0x1234567) out[0] = acc;
}

// Does a pending LDS-DMA (global_load_lds) count in lgkmcnt?  t[0]: ds_read + lgkmcnt(0);
// t[1]: DMA then ds_read + lgkmcnt(0); t[2]: DMA then vmcnt(0).
__global__ void dma_lgkm(const uint8_t* __restrict__ src, uint64_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[4096];
  const int lane = threadIdx.x & 63;
  buf[lane] = lane; __syncthreads();
  uint32_t v = 0;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t0 = __builtin_amdgcn_s_memtime();
  asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lane * 4) : "memory");
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  uint64_t t2 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_global_load_lds((const void*)(src + lane * 16), (__attribute__((address_space(3))) void*)(buf + 1024), 16, 0, 0);
  asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lane * 4) : "memory");
  uint64_t t3 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  uint64_t t4 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_global_load_lds((const void*)(src + 65536 + lane * 16), (__attribute__((address_space(3))) void*)(buf + 2048), 16, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint64_t t5 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = t3 - t2; out[2] = t5 - t4; out[3] = v; }
}

// Aggregate VALU throughput: every wave runs 8 independent chains; result = instructions
// issued per SIMD per cycle (all waves) using the slowest wave's s_memtime span.
template <int K> __global__ void thr(uint64_t* out, uint32_t seed) {
  if constexpr (K == 16) {  // 64-bit ops
    uint64_t x0 = seed + threadIdx.x, x1 = x0 * 3, x2 = x0 ^ 5, x3 = x0 + 9, y = seed * 17ull + 1;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < 256; r++)
      asm volatile(".rept 8\nv_lshl_add_u64 %0, %0, 1, %4\nv_lshl_add_u64 %1, %1, 1, %4\nv_lshl_add_u64 %2, %2, 1, %4\nv_lshl_add_u64 %3, %3, 1, %4\n.endr" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3) : "v"(y));
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 32 + (threadIdx.x >> 6)] = t1 - t0;
    if ((x0 ^ x1 ^ x2 ^ x3) == 0x1234567) out[100000] = 1;
    return;
  }
  uint32_t a0 = seed + threadIdx.x, a1 = a0 * 3, a2 = a0 ^ 5, a3 = a0 + 9, a4 = a0 * 7, a5 = a0 ^ 77, a6 = a0 + 1234, a7 = a0 * 13;
  uint32_t b = seed * 17 + 1, c = seed ^ 0x99;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 0; r < 256; r++) {
#define CH8(OP) asm volatile(".rept 4\n" OP("%0") OP("%1") OP("%2") OP("%3") OP("%4") OP("%5") OP("%6") OP("%7") ".endr\n" \
      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
#define XOR(R) "v_xor_b32 " R ", " R ", %8\n"
#define ALB(R) "v_alignbit_b32 " R ", " R ", %8, 31\n"
#define B3(R) "v_bitop3_b32 " R ", " R ", %8, %9 bitop3:0x96\n"
#define PRM(R) "v_perm_b32 " R ", " R ", %8, %9\n"
#define ANDOR(R) "v_and_or_b32 " R ", " R ", %8, %9\n"
#define LSHLOR(R) "v_lshl_or_b32 " R ", " R ", 1, %9\n"
#define OR3(R) "v_or3_b32 " R ", " R ", %8, %9\n"
#define BFE(R) "v_bfe_u32 " R ", " R ", 8, 8\n"
#define LSHL(R) "v_lshlrev_b32 " R ", 1, " R "\n"
#define SDWA(R) "v_lshlrev_b32_sdwa " R ", 8, " R " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1\n"
#define MIN3(R) "v_min3_u32 " R ", " R ", %8, %9\n"
#define MIN(R) "v_min_u32 " R ", " R ", %8\n"
#define MAD24(R) "v_mad_u32_u24 " R ", " R ", %8, %9\n"
#define ADD3(R) "v_add3_u32 " R ", " R ", %8, %9\n"
#define XDPP(R) "v_xor_b32_dpp " R ", %8, " R " quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
#define MDPP(R) "v_mov_b32_dpp " R ", %8 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
#define ADDC(R) "v_add_co_u32 " R ", vcc, " R ", %8\nv_addc_co_u32 %9, vcc, %9, %8, vcc\n"
#define ADDDPP(R) "v_add_co_u32_dpp " R ", vcc, %8, " R " quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n"
#define LSHLORDPP(R) "v_or_b32_sdwa " R ", %8, " R " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD\n"
    if (K == 0) CH8(XOR)
    if (K == 1) CH8(ALB)
    if (K == 2) CH8(B3)
    if (K == 3) CH8(PRM)
    if (K == 4) CH8(ANDOR)
    if (K == 5) CH8(LSHLOR)
    if (K == 6) CH8(OR3)
    if (K == 7) CH8(BFE)
    if (K == 8) CH8(LSHL)
    if (K == 9) CH8(SDWA)
    if (K == 10) CH8(MIN3)
    if (K == 11) CH8(MIN)
    if (K == 12) CH8(MAD24)
    if (K == 13) CH8(ADD3)
    if (K == 14) CH8(XDPP)
    if (K == 15) CH8(LSHLORDPP)
    if (K == 17) CH8(MDPP)
    if (K == 18) asm volatile(".rept 4\n" ADDC("%0") ADDC("%1") ADDC("%2") ADDC("%3") ADDC("%4") ADDC("%5") ADDC("%6") ADDC("%7") ".endr\n"
      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c) : "vcc");
    if (K == 19) asm volatile(".rept 4\n" ADDDPP("%0") ADDDPP("%1") ADDDPP("%2") ADDDPP("%3") ADDDPP("%4") ADDDPP("%5") ADDDPP("%6") ADDDPP("%7") ".endr\n"
      : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c) : "vcc");
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[blockIdx.x * 32 + (threadIdx.x >> 6)] = t1 - t0;
  if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x1234567) out[100000] = 1;
}

int main() {
  uint64_t* d; hipMalloc(&d, 8 * 2048);
  const char* names[] = {"xor dep", "alignbit dep", "lshl_add_u64 dep", "add_co+addc dep (pair)",
                         "nop1+mov_dpp dep (pair)", "perm dep", "bitop3 dep", "xor 4-chain",
                         "lshl_add_u64 4-chain", "mov_dpp indep", "xor_dpp dep", "lshlrev_b64 dep"};
  uint64_t h[2048];
  for (int waves : {1, 2, 4, 8}) {
    printf("--- %d wave(s) per SIMD (block %d threads) ---\n", waves, 256 * waves);
#define RUN(K) { probe<K><<<1, 256 * waves>>>(d, 1); hipDeviceSynchronize(); probe<K><<<1, 256 * waves>>>(d, 1); hipMemcpy(h, d, 8, hipMemcpyDeviceToHost); \
      printf("%-26s %.2f cycles/instr-slot\n", names[K], (double)h[0] / (REPS * 64.0)); }
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11)
  }
  {
    uint64_t n = 4ull << 30; uint8_t* buf; hipMalloc(&buf, n); hipMemset(buf, 1, n);
    uint32_t* o; hipMalloc(&o, 64);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms;
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0); rd_coalesced<<<2048, 256>>>((const u32x4*)buf, n / 16, o); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("rd_coalesced   %.1f GB/s\n", n / ms / 1e6);
      hipEventRecord(e0); rd_strip<64><<<512, 512>>>(buf, n, o); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("rd_strip<64>   %.1f GB/s\n", n / ms / 1e6);
      hipEventRecord(e0); rd_strip<128><<<512, 512>>>(buf, n, o); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("rd_strip<128>  %.1f GB/s\n", n / ms / 1e6);
#define STRIDE(S) { hipEventRecord(e0); rd_stride<S><<<512, 512>>>(buf, n, o); hipEventRecord(e1); hipEventSynchronize(e1); \
        hipEventElapsedTime(&ms, e0, e1); uint64_t tiles = n / (512ull * S); printf("rd_stride<%d>  %.1f GB/s\n", S, tiles * 512ull * 4096 / ms / 1e6); }
      hipEventRecord(e0); rd_strip4<<<512, 512>>>(buf, n, o); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("rd_strip4      %.1f GB/s\n", n / ms / 1e6);
      hipEventRecord(e0); rd_block64<<<2048, 256>>>(buf, n, o); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("rd_block64     %.1f GB/s\n", n / ms / 1e6);
      hipEventRecord(e0); rd_strip<256><<<512, 512>>>(buf, n, o); hipEventRecord(e1); hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1); printf("rd_strip<256>  %.1f GB/s\n", n / ms / 1e6);
    }
    hipFree(buf);
  }
  {
    uint8_t* src; hipMalloc(&src, 1 << 24); hipMemset(src, 3, 1 << 24);
    for (int rep = 0; rep < 3; rep++) {
      dma_lgkm<<<1, 64>>>(src + rep * (1 << 20), d); hipDeviceSynchronize(); hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
      printf("ds_read+lgkm0 %llu | DMA,ds_read+lgkm0 %llu | DMA+vmcnt0 %llu (s_memtime ticks)\n",
             (unsigned long long)h[0], (unsigned long long)h[1], (unsigned long long)h[2]);
    }
  }
  {
    uint64_t* tb; hipMalloc(&tb, 8 * 256 * 32 + 8 * 100001);
    const char* nm[] = {"xor", "alignbit", "bitop3", "perm", "and_or", "lshl_or", "or3", "bfe", "lshlrev", "lshl_sdwa", "min3", "min", "mad_u24", "add3", "xor_dpp", "or_sdwa", "lshl_add64", "mov_dpp", "addco+addc", "addco_dpp"};
    void (*ks[])(uint64_t*, uint32_t) = {thr<0>, thr<1>, thr<2>, thr<3>, thr<4>, thr<5>, thr<6>, thr<7>, thr<8>, thr<9>, thr<10>, thr<11>, thr<12>, thr<13>, thr<14>, thr<15>, thr<16>, thr<17>, thr<18>, thr<19>};
    for (int w : {1, 2, 4}) {
      for (int K = 0; K < 20; K++) {
        void (*kern)(uint64_t*, uint32_t) = ks[K];
        kern<<<256, 256 * w>>>(tb, 1); hipDeviceSynchronize(); kern<<<256, 256 * w>>>(tb, 1); hipDeviceSynchronize();
        static uint64_t hb[256 * 32]; hipMemcpy(hb, tb, 8 * 256 * 32, hipMemcpyDeviceToHost);
        uint64_t mx = 0; for (int b = 0; b < 256; b++) for (int k = 0; k < 4 * w; k++) mx = hb[b * 32 + k] > mx ? hb[b * 32 + k] : mx;
        double instr_per_simd = (double)w * 256 * 32;  // waves per SIMD x instructions per wave
        printf("thr %-9s %d waves/SIMD: %.3f instr/cycle/SIMD (%.2f cycles per wave-instr)\n", nm[K], w, instr_per_simd / mx, mx / instr_per_simd);
      }
    }
  }
  lds_chase<<<1, 64>>>(d); hipDeviceSynchronize(); lds_chase<<<1, 64>>>(d); hipMemcpy(h, d, 8, hipMemcpyDeviceToHost);
  printf("ds_read_b32 chase: %.1f cycles\n", h[0] / 2000.0);
  return 0;
}
