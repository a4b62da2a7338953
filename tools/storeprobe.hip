// Diagnostic only: the cost of the rollout's scattered record stores on MI355X.
// Each wave owns 64 env records of 17,216 B (the ObsData stride) and, per "step", stores G
// granules of 16 B into each env's 1,088-B record tail.  LPE = lanes per env in one store
// instruction: 1 (each lane its own env: 64 distinct lines per instruction, the rollout's store
// phase), 4 (a 64-B line per env: 16 lines per instruction) or 8 (128 B: 8 lines).  The same
// number of instructions and granule writes in each case; only the lines per instruction differ.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/storeprobe.hip -o tools/storeprobe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

constexpr size_t kObs = 17216, kTail = 16128;

// MODE: 0 plain, 1 non-temporal (nt), 2 write-through to memory (sc0 sc1), 3 nt sc1
template <int MODE>
__device__ __forceinline__ void st16(uint4 *p, uint4 v) {
  if (MODE == 0) *p = v;
  else if (MODE == 1) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4 *>(p));
  }
  else {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w = {v.x, v.y, v.z, v.w};
    if (MODE == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(w) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(p), "v"(w) : "memory");
  }
}
template <int LPE, int MODE = 0, bool SPREAD = false>
__global__ void __launch_bounds__(256) k_store(uint8_t *obs, size_t n, int steps, int g_per_step) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const size_t e0 = wave * 64;
  if (e0 >= n) return;
  const int sub = lane % LPE, grp = lane / LPE;             // lane sub of env group grp
  uint4 v = make_uint4(lane, (uint32_t)wave, 1u, 2u);
  for (int t = 0; t < steps; t++) {
    for (int k = 0; k < g_per_step; k++) {
      // instruction k of step t: envs e0 + grp + j * (64 / LPE) for the k-th slice
      const int slice = k % LPE;                             // which block of 64/LPE envs
      const size_t e = e0 + (size_t)slice * (64 / LPE) + grp;
      // SPREAD: each granule of a step in its own 128-B line of the tail, the set of lines
      // shifting every 8 steps (a new acting player): a per-XCD footprint beyond the 4 MiB L2
      const int g = SPREAD ? (((k / LPE) * 3 + ((t >> 3) & 3) * 2) % 8) * 8 + (t & 1) * 4 + sub
                           : ((k / LPE) * LPE + sub) % 68;  // granule in the tail (68 x 16 B)
      st16<MODE>(reinterpret_cast<uint4 *>(obs + e * kObs + kTail + 16 * g), v);
      v.z += 1u;
    }
  }
}

// The rollout's per-step output stores without the step (one env per work-item): per env-step
// the phase granule, two granules of the acting player's deck, every other step a granule of its
// stored mask or of the selected mask, the acting agent's Info steps byte and the 8-B action; the
// acting player changes every 8 steps.  6 requests per env-step over ~4.7 lines, like the rollout.
__global__ void __launch_bounds__(256) k_mimic(uint8_t *obs, uint8_t *sel, uint8_t *info, uint8_t *act, size_t n,
                                               int steps) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  uint8_t *ob = obs + e * kObs;
  uint4 v = make_uint4((uint32_t)e, 1u, 2u, 3u);
  for (int t = 0; t < steps; t++) {
    const int p = (t >> 3) & 3;
    uint8_t *pr = ob + 16192 + 256 * p;
    *reinterpret_cast<uint4 *>(ob + 16128) = v;
    *reinterpret_cast<uint4 *>(pr + 16 * (t % 7)) = v;
    *reinterpret_cast<uint4 *>(pr + 16 * ((t + 3) % 7)) = v;
    if (t & 1) *reinterpret_cast<uint4 *>(pr + 128 + 16 * (t % 6)) = v;
    else *reinterpret_cast<uint4 *>(sel + e * 128 + 16 * ((t >> 1) % 6)) = v;
    info[e * 192 + 4 + 32 * p] = (uint8_t)t;
    *reinterpret_cast<uint2 *>(act + e * 64) = make_uint2(v.x, (uint32_t)t);
    v.y += 1u;
  }
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 65536;
  const int wpg = argc > 2 ? atoi(argv[2]) : 4;              // waves per workgroup
  const int steps = 200, G = 16;
  uint8_t *obs;
  if (hipMalloc(&obs, n * kObs) != hipSuccess) return 1;
  if (hipMemset(obs, 0, n * kObs) != hipSuccess) return 1;
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
  const dim3 grid((unsigned)((n / 64 + wpg - 1) / wpg)), blk(64 * wpg);
  if (argc > 3 && !strcmp(argv[3], "coeff")) {             // the two store costs of bench.py's roofline
    const int g = 6;
    double us[2];
    for (int sp = 0; sp < 2; sp++) {
      float best = 1e30f;
      for (int r = 0; r < 3; r++) {
        if (hipEventRecord(a, 0) != hipSuccess) return 1;
        if (sp) hipLaunchKernelGGL((k_store<1, 0, true>), grid, blk, 0, 0, obs, n, steps, g);
        else hipLaunchKernelGGL((k_store<1, 0, false>), grid, blk, 0, 0, obs, n, steps, g);
        if (hipEventRecord(b, 0) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return 1;
        float ms;
        if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 1;
        best = ms < best ? ms : best;
      }
      us[sp] = best * 1e3;
    }
    printf("{\"envs\": %zu, \"steps\": %d, \"stores_per_env_step\": %d, \"packed_us\": %.3f, \"spread_us\": %.3f}\n",
           n, steps, g, us[0], us[1]);
    return 0;
  }
  if (argc > 3 && !strcmp(argv[3], "mimic")) {
    uint8_t *sel, *info, *act;
    if (hipMalloc(&sel, n * 128) != hipSuccess || hipMalloc(&info, n * 192) != hipSuccess ||
        hipMalloc(&act, n * 64) != hipSuccess)
      return 1;
    for (int ksteps : {20, 200, 1000}) {
      float best = 1e30f;
      for (int r = 0; r < 3; r++) {
        if (hipEventRecord(a, 0) != hipSuccess) return 1;
        hipLaunchKernelGGL(k_mimic, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, obs, sel, info, act, n, ksteps);
        if (hipEventRecord(b, 0) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return 1;
        float ms;
        if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 1;
        best = ms < best ? ms : best;
      }
      printf("n=%zu mimic (the rollout's output stores, no step): %d steps per launch: %.3f us per step\n", n, ksteps,
             best * 1e3 / ksteps);
    }
    return 0;
  }
  if (argc > 3) {                                            // G granules per env-step, spread vs packed
    const int g = atoi(argv[3]);
    for (int sp = 0; sp < 4; sp++) {                       // packed, spread, spread 2 and 4 lanes per env
      float best = 1e30f;
      for (int r = 0; r < 3; r++) {
        if (hipEventRecord(a, 0) != hipSuccess) return 1;
        if (sp == 1) hipLaunchKernelGGL((k_store<1, 0, true>), grid, blk, 0, 0, obs, n, steps, g);
        else if (sp == 2) hipLaunchKernelGGL((k_store<2, 0, true>), grid, blk, 0, 0, obs, n, steps, 2 * g);
        else if (sp == 3) hipLaunchKernelGGL((k_store<4, 0, true>), grid, blk, 0, 0, obs, n, steps, 4 * g);
        else hipLaunchKernelGGL((k_store<1, 0, false>), grid, blk, 0, 0, obs, n, steps, g);
        if (hipEventRecord(b, 0) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return 1;
        float ms;
        if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 1;
        best = ms < best ? ms : best;
      }
      const char *what[4] = {"packed (2 lines/env), 16 B per line", "spread (footprint > L2), 16 B per line",
                             "spread, 32 B per line (2 lanes)", "spread, 64 B per line (4 lanes)"};
      printf("n=%zu wpg=%d %s: %d lines per env-step: %.3f us per step, %.0f G line-requests/s\n", n, wpg, what[sp], g,
             best * 1e3 / steps, (double)n * g * steps / (best * 1e-3) / 1e9);
    }
    return 0;
  }
  for (int lpe : {1, 2, 4, 8, 11, 12, 13, 14, 21, 24}) {   // 11..14: LPE 1, modes 1..3 (+4: LPE 4 nt)
    float best = 1e30f;
    for (int r = 0; r < 3; r++) {
      if (hipEventRecord(a, 0) != hipSuccess) return 1;
      switch (lpe) {
        case 1: hipLaunchKernelGGL(k_store<1>, grid, blk, 0, 0, obs, n, steps, G); break;
        case 2: hipLaunchKernelGGL(k_store<2>, grid, blk, 0, 0, obs, n, steps, G); break;
        case 4: hipLaunchKernelGGL(k_store<4>, grid, blk, 0, 0, obs, n, steps, G); break;
        case 8: hipLaunchKernelGGL(k_store<8>, grid, blk, 0, 0, obs, n, steps, G); break;
        case 11: hipLaunchKernelGGL((k_store<1, 1>), grid, blk, 0, 0, obs, n, steps, G); break;
        case 12: hipLaunchKernelGGL((k_store<1, 2>), grid, blk, 0, 0, obs, n, steps, G); break;
        case 13: hipLaunchKernelGGL((k_store<1, 3>), grid, blk, 0, 0, obs, n, steps, G); break;
        case 14: hipLaunchKernelGGL((k_store<1, 0>), grid, blk, 0, 0, obs, n, steps, G); break;
        case 21: hipLaunchKernelGGL((k_store<2, 1>), grid, blk, 0, 0, obs, n, steps, G); break;
        default: hipLaunchKernelGGL((k_store<4, 1>), grid, blk, 0, 0, obs, n, steps, G); break;
      }
      if (hipEventRecord(b, 0) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return 1;
      float ms;
      if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 1;
      best = ms < best ? ms : best;
    }
    const double instr = (double)(n / 64) * steps * G;      // wave store instructions
    const int mode = lpe > 10 ? (lpe % 10 == 4 && lpe < 20 ? 0 : lpe < 20 ? lpe % 10 : 1) : 0;
    const int lp = lpe > 20 ? lpe % 10 : lpe > 10 ? 1 : lpe;
    printf("mode %d ", mode);
    lpe = lp;
    const double us_step = best * 1e3 / steps;
    printf("n=%zu wpg=%d LPE=%d: %.3f us per step of %d store instr/wave (%.1f ns per wave-instr per CU, "
           "%.0f G granules/s, %.0f G lines/s)\n", n, wpg, lpe, us_step, G,
           best * 1e6 / (instr / 256.0), instr * 64 / (best * 1e-3) / 1e9, instr * 64 / lpe / (best * 1e-3) / 1e9);
  }
  return 0;
}
