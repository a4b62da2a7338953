// Diagnostic only: the fused step kernel built with -DCOG_STAMPS (per-wave s_memtime at phase
// boundaries of staged_step) on the bench workload; prints mean cycles per phase.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DCOG_STAMPS -Iinclude \
//         -Igym-eldorado_amd/csrc tools/stamp_step.cpp -o tools/stamp_step
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <cstdio>
#include <algorithm>
#include <vector>

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 65536;
  const int steps = argc > 2 ? atoi(argv[2]) : 50;
  cog_env *env;
  cog_sampler *smp;
  cog_runner *run;
  if (cog_env_create(n, 0, &env) || cog_sampler_create(n, 12345, 0, &smp) ||
      cog_env_reset(env, 12345, 4, 3, 2, 100000, 0) || cog_runner_create(env, smp, 1, COG_RUNNER_DEVICE_VIEWS, &run)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  cog_runner_rollout(run, 100);
  cog_runner_sync(run);
  const size_t waves = (n + 63) / 64;
  unsigned long long *d;
  hipMalloc(&d, waves * 8 * sizeof(unsigned long long));
  env->s.stamps = d;
  std::vector<unsigned long long> h(waves * 8);
  std::vector<double> ph[6];
  for (int t = 0; t < steps; t++) {
    hipMemset(d, 0, waves * 8 * sizeof(unsigned long long));
    cog_runner_rollout(run, 1);
    cog_runner_sync(run);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    for (size_t w = 0; w < waves; w++) {
      for (int k = 1; k < 6; k++) ph[k].push_back((double)(long long)(h[w * 8 + k] - h[w * 8 + k - 1]));
      ph[0].push_back((double)(long long)(h[w * 8 + 5] - h[w * 8 + 0]));
    }
  }
  const char *names[] = {"total", "stage-in (2 dependent rounds of 16-B loads)", "sample (5 masked picks)",
                         "env_step", "auto-reset + outputs", "stage-out (stores issued)"};
  printf("s_memtime ticks per wave, median / p90 (n=%zu, %d steps):\n", n, steps);
  for (int k = 1; k < 7; k++) {
    const int j = k % 6;
    std::vector<double> &v = ph[j];
    std::sort(v.begin(), v.end());
    printf("  %-48s %10.0f %10.0f\n", names[j], v[v.size() / 2], v[v.size() * 9 / 10]);
  }
  return 0;
}
