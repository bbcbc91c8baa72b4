// clock_probe.hip — effective shader clock under sustained VALU load (development tool).
// Every wave runs a dependent 64-bit add/xor/alignbit mix (the BLAKE2b G instruction mix)
// for `iters` loops; wave 0 of each block records s_memtime (shader cycles) and
// s_memrealtime (100 MHz) so clock = d(memtime) / d(realtime) * 100 MHz.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int V>
__global__ void mix(uint64_t* out, uint32_t iters, uint32_t seed) {
  __shared__ uint64_t s[1024];
  s[threadIdx.x & 1023] = threadIdx.x * 77;
  __syncthreads();
  uint64_t a = seed + threadIdx.x, b = a * 3, c = a ^ 0x55, d = a + 7;
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      a = a + b + d;
      d ^= a; d = (d >> 32) | (d << 32);
      c = c + d;
      b ^= c; b = (b >> 24) | (b << 40);
      if (V == 1) {  // a 64-bit quad rotation (2 DPP movs) per step
        const uint32_t lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)c, 0x39, 0xF, 0xF, true);
        const uint32_t hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(c >> 32), 0x39, 0xF, 0xF, true);
        c = ((uint64_t)hi << 32) | lo;
      }
      if (V == 2) a += s[(threadIdx.x + (uint32_t)b) & 1023];  // a dependent LDS read per step
      if (V == 3) a += s[(threadIdx.x * 20 + k) & 1023];       // independent LDS read per step
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
  if ((a ^ b ^ c ^ d) == 0x1234567) out[100000] = 1;
}
int main() {
  uint64_t* d; (void)hipMalloc(&d, 8 * 200000);
  static uint64_t h[8192];
  void (*ks[])(uint64_t*, uint32_t, uint32_t) = {mix<0>, mix<1>, mix<2>, mix<3>};
  for (int V = 0; V < 4; V++) for (int blocks : {256, 512}) for (int thr : {256, 512}) for (uint32_t it : {5000u}) {
    printf("V%d ", V);
    ks[V]<<<blocks, thr>>>(d, it, 1); (void)hipDeviceSynchronize();
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0); ks[V]<<<blocks, thr>>>(d, it, 2); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(h, d, 16 * blocks, hipMemcpyDeviceToHost);
    double sc = 0, sr = 0; for (int b = 0; b < blocks; b++) { sc += h[2 * b]; sr += h[2 * b + 1]; }
    const double instr = (double)it * 16 * 8;  // ~8 VALU per inner step (approx)
    printf("blocks %4d x %4d thr, iters %6u: %.2f ms, clock %.0f MHz, %.2f cycles/step-instr (per wave)\n",
           blocks, thr, it, ms, sc / sr * 100.0, sc / blocks / instr);
  }
  return 0;
}
