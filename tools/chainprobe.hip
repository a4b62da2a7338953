// Diagnostic: the cost of one instruction in a DEPENDENT chain on a lone wave (one workgroup of one
// wave on the whole chip), in s_memtime ticks (the unit of the trio's phase stamps,
// cog_engine.hip stamp_clock) -- the denominator-side constant of bench.py's
// roofline.limiter.issue_frac: the stepping wave's per-step instructions x this cost / its
// measured ticks per step.  tools/rateprobe.hip measured the independent-chain issue rate (8
// chains); here every instruction waits for the previous one's result.
//   hipcc --offload-arch=gfx950 -O3 tools/chainprobe.hip -o tools/bin/chainprobe
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHAIN(OP) for (int it = 0; it < 512; it++) { OP; }
template <int K>
__global__ void __launch_bounds__(64) k(uint32_t *out, uint32_t seed, unsigned long long *cyc) {
  __shared__ uint32_t lds[64];
  uint32_t a = seed * (threadIdx.x + 1), b = seed | 0x10001u;
  lds[threadIdx.x] = threadIdx.x * 4u;                     // (K 6: the chain's next LDS address)
  if (K == 6) a = threadIdx.x * 4u;
  __syncthreads();
  unsigned long long t0 = __builtin_readcyclecounter();
  if (K == 0) CHAIN(asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b)))
  if (K == 1) CHAIN(asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a) : "v"(b)))
  if (K == 2) CHAIN(asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(a)))
  if (K == 3) CHAIN(asm volatile("v_cmp_gt_u32_e64 s[8:9], %0, %1\n s_nop 1\n v_cndmask_b32_e64 %0, %1, %0, s[8:9]"
                                 : "+v"(a) : "v"(b) : "s8", "s9"))
  if (K == 4) CHAIN(asm volatile("s_add_u32 s10, s10, s11" ::: "s10", "scc"))
  if (K == 5) CHAIN(asm volatile("v_readfirstlane_b32 s10, %0\n s_add_u32 s10, s10, 1\n v_mov_b32 %0, s10"
                                 : "+v"(a) :: "s10", "scc"))
  if (K == 6) CHAIN(asm volatile("ds_read_b32 %0, %0\n s_waitcnt lgkmcnt(0)\n v_and_b32 %0, 0xfc, %0"
                                 : "+v"(a) :: "memory"))
  if (K == 7) CHAIN(asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(b)))
  // independent (issue-bound) forms: 4 chains interleaved, the cost of one instruction when the
  // wave has independent work to issue
  uint32_t c1 = a + 1u, c2 = a + 2u, c3 = a + 3u;
  if (K == 8) CHAIN(asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4"
                                 : "+v"(a), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(b)))
  if (K == 9) CHAIN(asm volatile("s_add_u32 s10, s10, 1\n s_add_u32 s11, s11, 1\n s_add_u32 s12, s12, 1\n s_add_u32 s13, s13, 1"
                                 ::: "s10", "s11", "s12", "s13", "scc"))
  if (K == 10) CHAIN(asm volatile("ds_read_b32 %0, %4\n ds_read_b32 %1, %4 offset:4\n ds_read_b32 %2, %4 offset:8\n"
                                  " ds_read_b32 %3, %4 offset:12\n s_waitcnt lgkmcnt(0)"
                                  : "=v"(a), "=v"(c1), "=v"(c2), "=v"(c3) : "v"(0u) : "memory"))
  a ^= c1 ^ c2 ^ c3;
  unsigned long long t1 = __builtin_readcyclecounter();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  uint32_t *o;
  unsigned long long *c;
  if (hipMalloc(&o, 64 * 4) != hipSuccess || hipMalloc(&c, 8) != hipSuccess) return 1;
  const char *nm[] = {"v_add_u32", "v_and_or_b32", "v_bfe_u32", "v_cmp+nop1+v_cndmask", "s_add_u32",
                      "readfirstlane+s_add+v_mov", "ds_read_b32+wait+v_and", "v_mul_hi_u32",
                      "ISSUE 4 x v_add_u32", "ISSUE 4 x s_add_u32", "ISSUE 4 x ds_read_b32 + wait"};
  const int per[] = {1, 1, 1, 2, 1, 3, 2, 1, 4, 4, 5};   // instructions per link (s_nop excluded)
  for (int r = 0; r < 2; r++)
    for (int K = 0; K < 11; K++) {
      switch (K) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 6: hipLaunchKernelGGL(k<6>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 7: hipLaunchKernelGGL(k<7>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 8: hipLaunchKernelGGL(k<8>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 9: hipLaunchKernelGGL(k<9>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
        case 10: hipLaunchKernelGGL(k<10>, dim3(1), dim3(64), 0, 0, o, 0x3u, c); break;
      }
      unsigned long long h = 0;
      if (hipDeviceSynchronize() != hipSuccess || hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      if (r)
        printf("CHAIN %-28s %6.2f ticks per link, %5.2f per instruction (lone wave, %s)\n", nm[K], h / 512.0,
               h / 512.0 / per[K], K < 8 ? "dependent" : "independent");
    }
  return 0;
}
