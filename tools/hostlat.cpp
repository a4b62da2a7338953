// Diagnostic only: host-side cost of one short rollout call (the driver's --steps 20 shape):
// wall time of rollout(K) + sync against the device time of the launch, and the pieces of the
// sync (stream sync alone, the status read-back).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Igym-eldorado_amd/csrc tools/hostlat.cpp \
//         gym-eldorado_amd/csrc/cog_engine.hip gym-eldorado_amd/csrc/cog_abi.cpp -o tools/hostlat
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/cog.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 65536;
  const int K = argc > 2 ? atoi(argv[2]) : 20;
  cog_env *env;
  cog_sampler *smp;
  cog_runner *run;
  if (cog_env_create(n, 0, &env) || cog_sampler_create(n, 12345, 0, &smp) ||
      cog_env_reset(env, 12345, 4, 3, 2, 100000, 0) || cog_runner_create(env, smp, 1, COG_RUNNER_DEVICE_VIEWS, &run)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  cog_runner_set_chunk(run, 1000);
  cog_runner_rollout(run, 200);
  cog_runner_sync(run);
  hipStream_t st = (hipStream_t)cog_env_stream(env);
  std::vector<double> wall, dev, ssync, rsync;
  for (int r = 0; r < 30; r++) {
    double ms;
    uint64_t k;
    cog_runner_set_timing(run, 1);
    const double t0 = now_us();
    cog_runner_rollout(run, K);
    cog_runner_sync(run);
    const double t1 = now_us();
    cog_runner_kernel_time(run, &ms, &k);
    cog_runner_set_timing(run, 0);
    wall.push_back(t1 - t0);
    dev.push_back(ms * 1e3);
    const double t2 = now_us();
    (void)hipStreamSynchronize(st);
    ssync.push_back(now_us() - t2);
    const double t3 = now_us();
    cog_runner_sync(run);
    rsync.push_back(now_us() - t3);
  }
  // rollout + plain stream sync (no status read-back)
  std::vector<double> wall2;
  for (int r = 0; r < 30; r++) {
    const double t0 = now_us();
    cog_runner_rollout(run, K);
    (void)hipStreamSynchronize(st);
    wall2.push_back(now_us() - t0);
  }
  cog_runner_sync(run);
  printf("n=%zu K=%d: wall(rollout+sync) %.1f us, device(events) %.1f us, wall(rollout+streamsync) %.1f us, "
         "idle streamsync %.1f us, idle runner sync %.1f us\n",
         n, K, median(wall), median(dev), median(wall2), median(ssync), median(rsync));
  // device time of one launch against its step count: the intercept is the fixed per-launch cost
  for (int k : {1, 2, 5, 20, 100}) {
    std::vector<double> d, w;
    cog_runner_set_chunk(run, k);
    for (int r = 0; r < 20; r++) {
      double ms;
      uint64_t kk;
      cog_runner_set_timing(run, 1);
      const double t0 = now_us();
      cog_runner_rollout(run, k);
      cog_runner_sync(run);
      w.push_back(now_us() - t0);
      cog_runner_kernel_time(run, &ms, &kk);
      cog_runner_set_timing(run, 0);
      d.push_back(ms * 1e3);
    }
    printf("  K=%4d  device %.1f us  wall %.1f us\n", k, median(d), median(w));
  }
  return 0;
}
