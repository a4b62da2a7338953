// Diagnostic only: the reference's host loop (sample(masks); step(actions)) through the C ABI,
// timed per call, with the HIP pieces it is made of timed alone (a small H2D copy, a D2H copy of
// the refresh size, a 2D D2H of the ObsData tails, an empty-stream sync).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Igym-eldorado_amd/csrc tools/hostloop.cpp \
//         gym-eldorado_amd/csrc/cog_engine.hip gym-eldorado_amd/csrc/cog_abi.cpp -o tools/hostloop
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#include "../include/cog.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(const std::function<void()> &f, int reps = 200) {
  std::vector<double> v;
  for (int r = 0; r < 20; r++) f();
  for (int r = 0; r < reps; r++) {
    const double t0 = now_us();
    f();
    v.push_back(now_us() - t0);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

// zero-copy probes: a kernel storing the ObsData tails (rows of 1,088 B at the record stride)
// straight into pinned host memory, and one reading the masks from it
__global__ void k_put_tails(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t row = t / 68, g = t - 68 * row;
  // the tail is granules 1008..1075 of the 1,076-granule record
  if (row < n) dst[row * (17216 / 16) + 16128 / 16 + g] = src[row * (17216 / 16) + 16128 / 16 + g];
}
__global__ void k_get(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t m) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < m) dst[t] = src[t];
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 256;
  cog_env *env;
  cog_sampler *smp;
  if (cog_env_create(n, 0, &env) || cog_sampler_create(n, 12345, 0, &smp) ||
      cog_env_reset(env, 12345, 4, 3, 0, 100000, 0)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  cog_env_views v;
  cog_env_get_views(env, &v);
  const cog_action_mask_t *masks = v.selected_action_masks;
  cog_action_t *acts = cog_sampler_actions(smp);
  const double t_sample = med([&] { cog_sampler_sample(smp, masks, n); });
  const double t_step = med([&] { cog_env_step(env, acts, n); });
  const double t_loop = med([&] {
    cog_sampler_sample(smp, masks, n);
    cog_env_step(env, acts, n);
  });
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  void *d, *h;
  const size_t big = n * 1600;
  if (hipMalloc(&d, n * 17216) != hipSuccess || hipHostMalloc(&h, n * 17216) != hipSuccess) return 1;
  const double t_sync = med([&] { (void)hipStreamSynchronize(st); });
  const double t_h2d = med([&] {
    (void)hipMemcpyAsync(d, h, n * 128, hipMemcpyHostToDevice, st);
    (void)hipStreamSynchronize(st);
  });
  const double t_d2h = med([&] {
    (void)hipMemcpyAsync(h, d, big, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
  });
  const double t_2d = med([&] {
    (void)hipMemcpy2DAsync(h, 17216, d, 17216, 1088, n, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
  });
  const double t_3 = med([&] {
    (void)hipMemcpyAsync(d, h, n * 5, hipMemcpyHostToDevice, st);
    (void)hipMemcpy2DAsync(h, 17216, d, 17216, 1088, n, hipMemcpyDeviceToHost, st);
    (void)hipMemcpyAsync(h, d, n * 340, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
  });
  void *hd;
  if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess) return 1;
  const double t_kput = med([&] {
    hipLaunchKernelGGL(k_put_tails, dim3((unsigned)((n * 68 + 255) / 256)), dim3(256), 0, st, (const uint4 *)d, (uint4 *)hd, n);
    (void)hipStreamSynchronize(st);
  });
  const double t_kget = med([&] {
    hipLaunchKernelGGL(k_get, dim3((unsigned)((n * 8 + 255) / 256)), dim3(256), 0, st, (const uint4 *)hd, (uint4 *)d, n * 8);
    (void)hipStreamSynchronize(st);
  });
  const double t_kempty = med([&] {
    hipLaunchKernelGGL(k_get, dim3(1), dim3(64), 0, st, (const uint4 *)d, (uint4 *)d + 64, (size_t)0);
    (void)hipStreamSynchronize(st);
  });
  hipLaunchKernelGGL(k_put_tails, dim3((unsigned)((n * 68 + 255) / 256)), dim3(256), 0, st, (const uint4 *)d, (uint4 *)hd, n);
  printf("launch: %s; sync: %s\n", hipGetErrorString(hipGetLastError()), hipGetErrorString(hipStreamSynchronize(st)));
  printf("zero-copy: kernel put tails %.1f us, kernel get masks %.1f us, empty kernel+sync %.1f us\n", t_kput, t_kget, t_kempty);
  printf("n=%zu  sample %.1f us  step %.1f us  loop %.1f us (%.2f M env-steps/s) | idle sync %.1f  H2D %zu B %.1f  "
         "D2H %zu B %.1f  2D D2H %zu x 1088 B %.1f  H2D+2D+D2H %.1f us\n",
         n, t_sample, t_step, t_loop, n / t_loop, t_sync, n * 128, t_h2d, big, t_d2h, n, t_2d, t_3);
  return 0;
}
