// Diagnostic only: A/B timing probe.  Built twice from two engine source trees (tools/ab.sh) so
// that two engine versions are timed on the same box in the same call (box-to-box spread is a
// few per cent, as large as the effects measured).  Prints, per env count: the rollout's device
// us/step in 1,000-step launches, the device time of a 20-step launch, and the per-launch step
// kernel (k_env_step<selected>), each the median of repeated HIP-event timings.
#include "cog_engine.hip"
#include "cog_abi.cpp"
#include <algorithm>
#include <cstdio>
#include <vector>

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const char *tag = argc > 1 ? argv[1] : "?";
  for (size_t n : {65536ul, 8192ul}) {
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
    const cog::DevState &s = env->sh[0].s;
    uint32_t *rng = smp->sh[0].d_rng;
    uint8_t *act = smp->sh[0].d_actions;
    hipStream_t st = env->sh[0].stream;
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
    auto timed = [&](auto launch, int reps) {
      std::vector<double> v;
      for (int r = 0; r < reps; r++) {
        if (hipEventRecord(a, st) != hipSuccess) return -1.0;
        launch();
        if (hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return -1.0;
        float ms;
        if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.0;
        v.push_back(ms * 1e3);
      }
      return med(v);
    };
    const unsigned g = (unsigned)((n + 63) / 64);
    const double r1000 = timed([&] { hipLaunchKernelGGL((cog::k_env_rollout<cog::MASK_SELECTED, 64>), dim3(g), dim3(64), 0, st, s, 1000, rng, act); }, 5);
    const double r20 = timed([&] { hipLaunchKernelGGL((cog::k_env_rollout<cog::MASK_SELECTED, 64>), dim3(g), dim3(64), 0, st, s, 20, rng, act); }, 25);
    const double k1 = timed([&] { hipLaunchKernelGGL(cog::k_env_step<cog::MASK_SELECTED>, dim3(g), dim3(64), 0, st, s, nullptr, rng, act); }, 50);
    printf("%s n=%6zu  rollout %6.3f us/step (1000)  20-step launch %7.2f us  k_env_step %6.2f us\n", tag, n, r1000 / 1000,
           r20, k1);
    fflush(stdout);
    cog_runner_destroy(run);
    cog_sampler_destroy(smp);
    cog_env_destroy(env);
  }
  return 0;
}
