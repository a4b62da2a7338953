// Diagnostic only: host-side completion latency of short launches -- hipStreamSynchronize against
// a host spin on a completion word the kernel stores into pinned, device-mapped memory.  Shapes:
// an empty 1-WG kernel, the C2 sampler/step shape (256 envs: 4 WGs reading 32 KB of host masks
// and storing 2 KB into host memory), two kernels back to back, and the rollout's 1,024-WG shape.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/latprobe.hip -o tools/latprobe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double med(const std::function<void()> &f, int reps = 300) {
  std::vector<double> v;
  for (int r = 0; r < 30; r++) f();
  for (int r = 0; r < reps; r++) {
    const double t0 = now_us();
    f();
    v.push_back(now_us() - t0);
  }
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

// the last workgroup to finish stores `seq` into the host word (system scope, after a
// system-scope release by every workgroup), so the host sees the kernel's host stores first
__device__ void signal_done(unsigned *ctr, unsigned *hword, unsigned seq) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    const unsigned prev = atomicAdd(ctr, 1u);
    if (prev == gridDim.x - 1) {
      *ctr = 0u;
      __hip_atomic_store(hword, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// the same with an agent-scope fence per workgroup (waits for the workgroup's stores to be acked)
__device__ void signal_done_agent(unsigned *ctr, unsigned *hword, unsigned seq) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(ctr, 1u);
    if (prev == gridDim.x - 1) {
      *ctr = 0u;
      __hip_atomic_store(hword, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
__global__ void __launch_bounds__(64) k_lds_agent(int n, unsigned *ctr, unsigned *hword, unsigned seq) {
  __shared__ uint4 big[2400];
  if (n < 0) big[threadIdx.x] = make_uint4(n, n, n, n);
  if (n < 0) hword[0] = big[threadIdx.x + 1].x;
  signal_done_agent(ctr, hword, seq);
}
__global__ void __launch_bounds__(256) k_put(uint4 *__restrict__ h, int n, unsigned *ctr, unsigned *hword, unsigned seq,
                                             int sys) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
    h[i] = make_uint4(i, seq, i ^ seq, 7u);
  if (sys) signal_done(ctr, hword, seq);
  else signal_done_agent(ctr, hword, seq);
}
__global__ void k_empty() {}
__global__ void k_sig(unsigned *ctr, unsigned *hword, unsigned seq) { signal_done(ctr, hword, seq); }
// C2 shape: each work-item reads a 128-B mask from host memory and writes 8 B to host memory
__global__ void k_c2(const uint4 *__restrict__ hmask, uint2 *__restrict__ hact, int n, unsigned *ctr, unsigned *hword,
                     unsigned seq) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint4 a = make_uint4(0, 0, 0, 0);
    for (int k = 0; k < 8; k++) {
      const uint4 v = hmask[i * 8 + k];
      a.x ^= v.x; a.y += v.y; a.z |= v.z; a.w ^= v.w;
    }
    hact[i] = make_uint2(a.x ^ a.z, a.y ^ a.w ^ seq);
  }
  if (ctr) signal_done(ctr, hword, seq);
}
__global__ void __launch_bounds__(64) k_lds(int n, unsigned *ctr, unsigned *hword, unsigned seq) {
  __shared__ uint4 big[2400];   // 38,400 B: the rollout's LDS per workgroup
  if (n < 0) big[threadIdx.x] = make_uint4(n, n, n, n);
  if (n < 0) hword[0] = big[threadIdx.x + 1].x;
  if (ctr) signal_done(ctr, hword, seq);
}

static inline void spin(volatile unsigned *w, unsigned seq) {
  while (*w != seq) __builtin_ia32_pause();
}

int main(int argc, char **argv) {
  // argv[1]: "spin" / "yield" / "block" -- hipSetDeviceFlags before the device is used (the host
  // thread's wait in hipStreamSynchronize / hipDeviceSynchronize); default: the runtime's choice
  if (argc > 1) {
    const unsigned f = !strcmp(argv[1], "spin") ? hipDeviceScheduleSpin
                       : !strcmp(argv[1], "yield") ? hipDeviceScheduleYield : hipDeviceScheduleBlockingSync;
    printf("hipSetDeviceFlags(%s): %s\n", argv[1], hipGetErrorString(hipSetDeviceFlags(f)));
  }
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  unsigned *hword, *ctr;
  uint4 *hmask;
  uint2 *hact;
  const unsigned zc = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
  if (hipHostMalloc(&hword, 256, zc) || hipMalloc(&ctr, 256) || hipHostMalloc(&hmask, 256 * 128, zc) ||
      hipHostMalloc(&hact, 256 * 8, zc))
    return 1;
  (void)hipMemset(ctr, 0, 256);
  *hword = 0;
  void *dword_v, *dmask_v, *dact_v;
  (void)hipHostGetDevicePointer(&dword_v, hword, 0);
  (void)hipHostGetDevicePointer(&dmask_v, hmask, 0);
  (void)hipHostGetDevicePointer(&dact_v, hact, 0);
  unsigned *dword = (unsigned *)dword_v;
  const uint4 *dmask = (const uint4 *)dmask_v;
  uint2 *dact = (uint2 *)dact_v;
  unsigned seq = 0;
  (void)hipDeviceSynchronize();

  const double a = med([&] {
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
    (void)hipStreamSynchronize(st);
  });
  const double b = med([&] {
    ++seq;
    hipLaunchKernelGGL(k_sig, dim3(1), dim3(64), 0, st, ctr, dword, seq);
    spin(hword, seq);
  });
  const double b2 = med([&] {
    ++seq;
    hipLaunchKernelGGL(k_sig, dim3(1), dim3(64), 0, st, ctr, dword, seq);
    spin(hword, seq);
    (void)hipStreamSynchronize(st);
  });
  const double b3 = med([&] { (void)hipStreamSynchronize(st); });
  const double c_sync = med([&] {
    hipLaunchKernelGGL(k_c2, dim3(4), dim3(64), 0, st, dmask, dact, 256, (unsigned *)nullptr, dword, 0u);
    (void)hipStreamSynchronize(st);
  });
  const double c_spin = med([&] {
    ++seq;
    hipLaunchKernelGGL(k_c2, dim3(4), dim3(64), 0, st, dmask, dact, 256, ctr, dword, seq);
    spin(hword, seq);
  });
  const double e_sync = med([&] {
    hipLaunchKernelGGL(k_c2, dim3(4), dim3(64), 0, st, dmask, dact, 256, (unsigned *)nullptr, dword, 0u);
    hipLaunchKernelGGL(k_c2, dim3(4), dim3(64), 0, st, dmask, dact, 256, (unsigned *)nullptr, dword, 0u);
    (void)hipStreamSynchronize(st);
  });
  const double e_spin = med([&] {
    ++seq;
    hipLaunchKernelGGL(k_c2, dim3(4), dim3(64), 0, st, dmask, dact, 256, (unsigned *)nullptr, dword, 0u);
    hipLaunchKernelGGL(k_c2, dim3(4), dim3(64), 0, st, dmask, dact, 256, ctr, dword, seq);
    spin(hword, seq);
  });
  const double e_sigk = med([&] {
    ++seq;
    hipLaunchKernelGGL(k_c2, dim3(4), dim3(64), 0, st, dmask, dact, 256, (unsigned *)nullptr, dword, 0u);
    hipLaunchKernelGGL(k_sig, dim3(1), dim3(64), 0, st, ctr, dword, seq);
    spin(hword, seq);
  });
  const double h_sync = med([&] {
    hipLaunchKernelGGL(k_lds, dim3(1024), dim3(64), 0, st, 1, (unsigned *)nullptr, dword, 0u);
    (void)hipStreamSynchronize(st);
  });
  const double h_spin = med([&] {
    ++seq;
    hipLaunchKernelGGL(k_lds, dim3(1024), dim3(64), 0, st, 1, ctr, dword, seq);
    spin(hword, seq);
  });
  const double h_dev = med([&] {
    hipLaunchKernelGGL(k_lds, dim3(1024), dim3(64), 0, st, 1, (unsigned *)nullptr, dword, 0u);
    (void)hipDeviceSynchronize();
  });
  const double h_agent = med([&] {
    ++seq;
    hipLaunchKernelGGL(k_lds_agent, dim3(1024), dim3(64), 0, st, 1, ctr, dword, seq);
    spin(hword, seq);
  });
  uint4 *hput;
  void *dput_v;
  if (hipHostMalloc(&hput, 23552 * 16, zc) || hipHostGetDevicePointer(&dput_v, hput, 0)) return 1;
  uint4 *dput = (uint4 *)dput_v;
  double put[4][2];
  const int grids[4] = {1, 12, 92, 256};
  unsigned bad = 0;
  for (int g = 0; g < 4; g++)
    for (int sys = 0; sys < 2; sys++)
      put[g][sys] = med([&] {
        ++seq;
        hipLaunchKernelGGL(k_put, dim3(grids[g]), dim3(256), 0, st, dput, 23552, ctr, dword, seq, sys);
        spin(hword, seq);
        for (int i = 0; i < 23552; i += 97) bad += ((volatile unsigned *)hput)[4 * i + 1] != seq;   // stores visible before the word?
      });
  const double launch_only = med([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st); }, 100);
  (void)hipStreamSynchronize(st);
  printf("latprobe (medians, us):\n");
  printf("  empty kernel + hipStreamSynchronize            %6.2f\n", a);
  printf("  signalling kernel + host spin                  %6.2f\n", b);
  printf("  signalling kernel + spin + hipStreamSynchronize %6.2f\n", b2);
  printf("  idle hipStreamSynchronize                      %6.2f\n", b3);
  printf("  C2 kernel (256 masks from host) + stream sync  %6.2f\n", c_sync);
  printf("  C2 kernel + host spin                          %6.2f\n", c_spin);
  printf("  2 x C2 kernel + stream sync                    %6.2f\n", e_sync);
  printf("  2 x C2 kernel, the second signalling + spin    %6.2f\n", e_spin);
  printf("  C2 kernel + 1-WG signal kernel + spin          %6.2f\n", e_sigk);
  printf("  1,024 x 38 KB-LDS WGs + stream sync            %6.2f\n", h_sync);
  printf("  1,024 x 38 KB-LDS WGs, last signalling + spin  %6.2f\n", h_spin);
  printf("  1,024 x 38 KB-LDS WGs + hipDeviceSynchronize   %6.2f\n", h_dev);
  printf("  1,024 WGs, agent-scope fence per WG + spin     %6.2f\n", h_agent);
  for (int g = 0; g < 4; g++)
    printf("  put 23,552 granules to host, %3d WGs: agent fence %6.2f  system fence %6.2f\n", grids[g], put[g][0], put[g][1]);
  printf("  host stores seen stale after the word: %u (of %d sampled)\n", bad, 8 * 330 * 243);
  printf("  hipLaunchKernelGGL call alone (queued)         %6.2f\n", launch_only);
  printf("  last error: %s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
