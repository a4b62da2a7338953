#include <hip/hip_runtime.h>
#include <cstdio>
// cycles per instruction for one wave per SIMD: 8 independent chains, 64 iterations x 8 ops
#define BODY(OP) \
  for (int it = 0; it < 64; it++) { _Pragma("unroll") for (int c = 0; c < 8; c++) { OP; } }
template <int K>
__global__ void __launch_bounds__(64) k(uint32_t *out, uint32_t seed, unsigned long long *cyc) {
  uint32_t a[8];
  uint64_t w[8];
  for (int c = 0; c < 8; c++) { a[c] = seed * (threadIdx.x + c + 1); w[c] = a[c]; }
  const uint32_t m = seed | 0x10001u;
  unsigned long long t0 = __builtin_readcyclecounter();
  if (K == 0) BODY(asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[c]) : "v"(m)))
  if (K == 1) BODY(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[c]) : "v"(m)))
  if (K == 2) BODY(asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[c]) : "v"(m)))
  if (K == 3) BODY(asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[c]) : "v"(a[c]), "v"(m) : "vcc"))
  if (K == 4) BODY(asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[c]) : "v"(m)))
  if (K == 5) BODY(asm volatile("v_lshl_add_u64 %0, %0, 1, %0" : "+v"(w[c])))
  if (K == 6) BODY(asm volatile("v_readlane_b32 s0, %0, 5\n s_nop 0" : : "v"(a[c]) : "s0"))
  if (K == 7) BODY(asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[8:9]" : "+v"(a[c]) : "v"(m) : "s8", "s9"))
  if (K == 8) BODY(asm volatile("v_cmp_eq_u32_e64 s[8:9], %0, %1\n s_nop 1\n v_cndmask_b32_e64 %0, %0, %1, s[8:9]" : "+v"(a[c]) : "v"(m) : "s8", "s9"))
  if (K == 9) BODY(asm volatile("v_cmp_eq_u32_e64 s[8:9], %0, %1\n v_cndmask_b32_e64 %0, %0, %1, s[8:9]" : "+v"(a[c]) : "v"(m) : "s8", "s9"))
  if (K == 10) BODY(asm volatile("s_nop 1" ::: ))
  unsigned long long t1 = __builtin_readcyclecounter();
  uint32_t x = 0;
  for (int c = 0; c < 8; c++) x ^= a[c] ^ (uint32_t)w[c];
  out[blockIdx.x * 64 + threadIdx.x] = x;
  if (threadIdx.x == 0 && blockIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  uint32_t *o; unsigned long long *c;
  hipMalloc(&o, 1024 * 64 * 4); hipMalloc(&c, 8);
  const char *nm[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_mul_u32_u24", "v_lshl_add_u64", "v_readlane+nop", "v_cndmask_e64", "cmp+nop1+cndmask", "cmp+cndmask", "s_nop 1"};
  for (int r = 0; r < 2; r++)
  for (int K = 0; K < 11; K++) {
    switch (K) {
      case 0: hipLaunchKernelGGL(k<0>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 1: hipLaunchKernelGGL(k<1>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 2: hipLaunchKernelGGL(k<2>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 3: hipLaunchKernelGGL(k<3>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 4: hipLaunchKernelGGL(k<4>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 5: hipLaunchKernelGGL(k<5>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 6: hipLaunchKernelGGL(k<6>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 7: hipLaunchKernelGGL(k<7>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 8: hipLaunchKernelGGL(k<8>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 9: hipLaunchKernelGGL(k<9>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
      case 10: hipLaunchKernelGGL(k<10>, dim3(1024), dim3(64), 0, 0, o, 7u, c); break;
    }
    unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    if (r) printf("%-16s %6.2f cycles / instruction (one wave per SIMD, 8 independent chains)\n", nm[K], h / 512.0);
  }
  return 0;
}
