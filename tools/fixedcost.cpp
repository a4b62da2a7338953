// Diagnostic only: the rollout kernel's fixed per-launch cost.  Launches k_env_rollout directly
// with 0, 1, 2, 5, 20 steps (0: prologue + epilogue only) and prints the median device time
// (hipEvents).  Built with -DCOG_ABLATE_FILL / -DCOG_ABLATE_EPI by tools/fixedcost.sh to price
// the prologue's player-record loads and the epilogue's private-state stores (timing only).
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <algorithm>
#include <cstdio>
#include <vector>

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 65536;
  cog_env *env;
  cog_sampler *smp;
  cog_runner *run;
  if (cog_env_create(n, 0, &env) || cog_sampler_create(n, 12345, 0, &smp) ||
      cog_env_reset(env, 12345, 4, 3, 2, 100000, 0) || cog_runner_create(env, smp, 1, COG_RUNNER_DEVICE_VIEWS, &run)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  cog_runner_set_chunk(run, 100);
  cog_runner_rollout(run, 100);
  cog_runner_sync(run);
  const cog::DevState &s = env->sh[0].s;
  uint32_t *rng = smp->sh[0].d_rng;
  uint8_t *act = smp->sh[0].d_actions;
  hipStream_t st = env->sh[0].stream;
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
  for (int k : {0, 1, 2, 5, 20}) {
    std::vector<double> v;
    for (int r = 0; r < 25; r++) {
      if (hipEventRecord(a, st) != hipSuccess) return 1;
      hipLaunchKernelGGL((cog::k_env_rollout<cog::MASK_SELECTED, 64>), dim3((unsigned)((n + 63) / 64)), dim3(64), 0,
                         st, s, k, rng, act);
      if (hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return 1;
      float ms;
      if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 1;
      v.push_back(ms * 1e3);
    }
    std::sort(v.begin(), v.end());
    printf("  steps %3d  device %7.1f us\n", k, v[v.size() / 2]);
  }
  return 0;
}
