// Diagnostic only: rollout time per step of the bench workload (65,536 envs, 4p HARD, selected
// masks, 1,000 steps per launch) for builds with parts of the step compiled out
// (-DCOG_ABLATE_STORES / -DCOG_ABLATE_UPDOBS: neither changes selected-mode dynamics), to
// attribute the step's cost.   tools/ablate.sh builds and runs the variants.
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <cstdio>

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 65536;
  const int steps = argc > 2 ? atoi(argv[2]) : 3000;
  cog_env *env;
  cog_sampler *smp;
  cog_runner *run;
  if (cog_env_create(n, 0, &env) || cog_sampler_create(n, 12345, 0, &smp) ||
      cog_env_reset(env, 12345, 4, 3, 2, 100000, 0) || cog_runner_create(env, smp, 1, COG_RUNNER_DEVICE_VIEWS, &run)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  cog_runner_set_chunk(run, 1000);
  cog_runner_rollout(run, 1000);
  cog_runner_sync(run);
  cog_runner_set_timing(run, 1);
  cog_runner_rollout(run, steps);
  double ms;
  uint64_t k;
  cog_runner_kernel_time(run, &ms, &k);
  printf("%.3f us/step\n", ms * 1e3 / (double)k);
  return 0;
}
