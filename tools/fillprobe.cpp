// Diagnostic only: the rollout prologue's player-record fill in isolation.  65,536 envs laid out
// as the engine's records (ObsData 17,216 B with the 4 DeckObs at 16,176 + 240 p, EnvPriv 160 B
// with granules 4..9, 5 mask-bit heads of 16 B); each 64-lane workgroup moves its 64 envs' 38
// granules (608 B) into LDS and the kernel ends.  Variants:
//   lane     one env per lane, register loads + ds_write        (the engine's lds_fill_players)
//   dma      one env per lane, global_load_lds_dwordx4
//   tdma     transposed: lane j of instruction q moves flat granule 64 q + j of the wave's
//            [env][39] layout (38 + 1 pad), so lanes share cache lines; global_load_lds
//   treg     transposed register loads + ds_write into the same layout
//   empty    the launch alone
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kObs = 17216, kDeck0 = 16176, kDeckStride = 240, kPriv = 160;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(const void *src, void *lds) {
  __builtin_amdgcn_global_load_lds(src, (lds_void *)lds, 16, 0, 0);
}
__device__ __forceinline__ const uint4 *gsrc(const uint8_t *obs, const uint8_t *priv, const uint4 *heads, size_t e, int c) {
  if (c < 28) return reinterpret_cast<const uint4 *>(obs + e * kObs + kDeck0 + kDeckStride * (c / 7)) + c % 7;
  if (c < 34) return reinterpret_cast<const uint4 *>(priv + e * kPriv) + 4 + (c - 28);
  if (c < 38) return heads + 5 * e + 1 + (c - 34);
  return heads + 5 * e + 4;   // pad slot: a harmless repeat
}

template <int V>
__global__ void __launch_bounds__(64) k_fill(const uint8_t *obs, const uint8_t *priv, const uint4 *heads, uint32_t *sink) {
  __shared__ uint4 L[64 * 39];
  const int l = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * 64;
  if (V == 0) {                 // lane
    const size_t e = base + l;
#pragma unroll
    for (int c = 0; c < 38; c++) L[c * 64 + l] = *gsrc(obs, priv, heads, e, c);
  } else if (V == 1) {          // dma, per lane
    const size_t e = base + l;
#pragma unroll
    for (int c = 0; c < 38; c++) dma16(gsrc(obs, priv, heads, e, c), &L[c * 64]);
  } else if (V == 2 || V == 3) {   // transposed
    int e = l / 39, c = l % 39;
#pragma unroll
    for (int q = 0; q < 39; q++) {
      if (V == 2) dma16(gsrc(obs, priv, heads, base + e, c), &L[q * 64]);
      else L[q * 64 + l] = *gsrc(obs, priv, heads, base + e, c);
      c += 25; e += 1;           // 64 = 39 + 25
      if (c >= 39) { c -= 39; e += 1; }
    }
  }
  if (V == 4) return;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < 39; c++) acc ^= L[(l * 39 + c) % (64 * 39)].x;
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;
}

int main() {
  const size_t n = 65536;
  uint8_t *obs, *priv;
  uint4 *heads;
  uint32_t *sink;
  if (hipMalloc(&obs, n * kObs) || hipMalloc(&priv, n * kPriv) || hipMalloc(&heads, n * 80) || hipMalloc(&sink, 4096 * 4)) return 1;
  hipMemset(obs, 1, n * kObs);
  hipMemset(priv, 2, n * kPriv);
  hipMemset(heads, 3, n * 80);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  void *flush;
  if (hipMalloc(&flush, 1ull << 30)) return 1;
  const char *names[] = {"lane", "dma", "tdma", "treg", "empty"};
  for (int cold = 0; cold < 2; cold++)
    for (int v = 0; v < 5; v++) {
      std::vector<double> t;
      for (int r = 0; r < 25; r++) {
        if (cold) hipMemsetAsync(flush, r, 1ull << 30);    // evict the records from L2 / MALL
        hipEventRecord(a);
        switch (v) {
          case 0: hipLaunchKernelGGL(k_fill<0>, dim3(n / 64), dim3(64), 0, 0, obs, priv, heads, sink); break;
          case 1: hipLaunchKernelGGL(k_fill<1>, dim3(n / 64), dim3(64), 0, 0, obs, priv, heads, sink); break;
          case 2: hipLaunchKernelGGL(k_fill<2>, dim3(n / 64), dim3(64), 0, 0, obs, priv, heads, sink); break;
          case 3: hipLaunchKernelGGL(k_fill<3>, dim3(n / 64), dim3(64), 0, 0, obs, priv, heads, sink); break;
          default: hipLaunchKernelGGL(k_fill<4>, dim3(n / 64), dim3(64), 0, 0, obs, priv, heads, sink);
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        t.push_back(ms * 1e3);
      }
      std::sort(t.begin(), t.end());
      printf("%-5s %-5s median %7.2f us  min %7.2f us   (%.1f MB useful -> %.2f TB/s)\n", cold ? "cold" : "warm", names[v],
             t[t.size() / 2], t[0], n * 608 / 1e6, n * 608 / (t[t.size() / 2] * 1e-6) / 1e12);
    }
  return 0;
}
