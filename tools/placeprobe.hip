// Diagnostic only: which SIMD of which CU each wave of a multi-wave workgroup lands on.
// Every wave reads HW_REG_HW_ID (SIMD, CU, SH, SE) and HW_REG_XCC_ID, then waits ~30 us so that
// the whole grid is resident at once, and lane 0 stores the ids.  The host counts, per CU, how
// the roles (wave index in the workgroup) spread over the CU's four SIMDs.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/placeprobe.hip -o tools/placeprobe
//   tools/placeprobe <waves per workgroup> <workgroups> <LDS bytes per workgroup>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ void k_place(uint32_t *out, long long spin) {
  extern __shared__ uint32_t lds[];
  const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));     // HW_REG_HW_ID
  const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // HW_REG_XCC_ID
  if (threadIdx.x == 0) lds[0] = 0;
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(10);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    const size_t k = (size_t)blockIdx.x * (blockDim.x >> 6) + w;
    out[2 * k] = hw;
    out[2 * k + 1] = xcc + lds[0];
  }
}

int main(int argc, char **argv) {
  const int wpg = argc > 1 ? atoi(argv[1]) : 2;
  const int wgs = argc > 2 ? atoi(argv[2]) : 1024;
  const int lds = argc > 3 ? atoi(argv[3]) : 39936;
  const size_t nw = (size_t)wpg * wgs;
  uint32_t *d;
  if (hipMalloc(&d, nw * 8) != hipSuccess) return 1;
  if (lds > 65536 && hipFuncSetAttribute((const void *)k_place, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_place, dim3(wgs), dim3(64 * wpg), lds, 0, d, 100LL * 30);   // wall clock: 100 MHz
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
  std::vector<uint32_t> h(nw * 2);
  if (hipMemcpy(h.data(), d, nw * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  // per CU (xcc, se, sh, cu): count of waves per (simd, role)
  std::map<uint32_t, std::vector<int>> cu;
  std::map<uint32_t, int> wgs_per_cu;
  for (size_t k = 0; k < nw; k++) {
    const uint32_t hw = h[2 * k], xcc = h[2 * k + 1];
    const uint32_t simd = (hw >> 4) & 3, cuid = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    const uint32_t key = xcc << 16 | se << 8 | sh << 4 | cuid;
    auto &v = cu[key];
    if (v.empty()) v.assign(4 * wpg, 0);
    const int role = (int)(k % wpg);
    v[simd * wpg + role]++;
    if (role == 0) wgs_per_cu[key]++;
  }
  // histogram of per-CU patterns
  std::map<std::vector<int>, int> pat;
  for (auto &kv : cu) pat[kv.second]++;
  printf("waves/WG %d, WGs %d, LDS %d B: %zu CUs used\n", wpg, wgs, lds, cu.size());
  for (auto &kv : pat) {
    printf("%5d CUs:", kv.second);
    for (int s = 0; s < 4; s++) {
      printf("  SIMD%d[", s);
      for (int r = 0; r < wpg; r++) printf("%s%d", r ? " " : "", kv.first[s * wpg + r]);
      printf("]");
    }
    printf("\n");
  }
  // first few workgroups: simd of each wave
  printf("first WGs (simd per wave, cu key):");
  for (int b = 0; b < 8 && b < wgs; b++) {
    printf(" {");
    for (int r = 0; r < wpg; r++) printf("%s%u", r ? "," : "", (h[2 * ((size_t)b * wpg + r)] >> 4) & 3);
    printf("}");
  }
  printf("\n");
  return 0;
}
