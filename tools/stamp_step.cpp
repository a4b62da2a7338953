// Diagnostic only: the fused step kernel built with -DCOG_STAMPS (per-wave s_memtime at phase
// boundaries of env_step_lane) on the bench workload; prints mean cycles per phase.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DCOG_STAMPS -Iinclude \
//         -Igym-eldorado_amd/csrc tools/stamp_step.cpp -o tools/stamp_step
//   tools/stamp_step N STEPS CHUNK [STORED]   (STORED=1: the full-dynamics driver, stored masks)
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <cstdio>
#include <algorithm>
#include <vector>

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 65536;
  const int steps = argc > 2 ? atoi(argv[2]) : 50;
  const int chunk = argc > 3 ? atoi(argv[3]) : 1;   // > 1: the persistent rollout, per-phase totals
  const bool stored = argc > 4 && atoi(argv[4]) != 0;  // 1: full dynamics (stored masks, the wave kernel)
  cog_env *env;
  cog_sampler *smp;
  cog_runner *run;
  if (cog_env_create(n, 0, &env) || cog_sampler_create(n, 12345, 0, &smp) ||
      cog_env_reset(env, 12345, 4, 3, 2, 100000, 0) || cog_runner_create(env, smp, 1, COG_RUNNER_DEVICE_VIEWS | (stored ? COG_RUNNER_STORED_MASKS : 0u), &run)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  cog_runner_rollout(run, 100);
  cog_runner_sync(run);
  const size_t waves = (n + 63) / 64;
  if (chunk > 1) {
    unsigned long long *d;
    constexpr int K = 16;
    if (hipMalloc(&d, waves * K * sizeof(unsigned long long)) != hipSuccess) return 1;
    if (hipMemset(d, 0, waves * K * sizeof(unsigned long long)) != hipSuccess) return 1;
    env->sh[0].s.stamps = d;
    cog_runner_set_chunk(run, chunk);
    cog_runner_rollout(run, chunk);
    cog_runner_sync(run);
    std::vector<unsigned long long> h(waves * K);
    if (hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char *pn[16] = {"LDS players + unpack", "sample + action/rng stores", "game logic: rest",
                          "compare + stores", "LDS write-back", "finish / done / reset", "wave encode", "",
                          "  logic: info, phase, action branch", "  logic: mip + end_turn discard",
                          "  logic: draw", "  logic: mask swap, sh, moved cells", "  logic: update_observation",
                          "", "", ""};
    printf("rollout: s_memtime ticks per step per wave, median over waves (n=%zu, %d steps):\n", n, chunk);
    double tot = 0;
    for (int k = 0; k < 13; k++) {
      if (!pn[k][0]) continue;
      std::vector<double> v;
      for (size_t w = 0; w < waves; w++) v.push_back((double)h[w * K + k] / chunk);
      std::sort(v.begin(), v.end());
      printf("  %-40s %9.0f\n", pn[k], v[v.size() / 2]);
      tot += v[v.size() / 2];
    }
    printf("  %-40s %9.0f\n", "sum", tot);
    return 0;
  }
  constexpr int K = 16;
  unsigned long long *d;
  if (hipMalloc(&d, waves * K * sizeof(unsigned long long)) != hipSuccess) return 1;
  env->sh[0].s.stamps = d;
  std::vector<unsigned long long> h(waves * K);
  // phase j = ticks from the previous stamp that was reached to stamp j
  const char *names[K] = {"", "loads (2 rounds) + sample + unpack", "repack registers",
                          "game logic (registers)", "compare + stores issued", "finish / done / reset",
                          "wave encode", "", "", "", "", "", "", "", "", ""};
  std::vector<double> ph[K], tot;
  for (int t = 0; t < steps; t++) {
    if (hipMemset(d, 0, waves * K * sizeof(unsigned long long)) != hipSuccess) return 1;
    cog_runner_rollout(run, 1);
    cog_runner_sync(run);
    if (hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (size_t w = 0; w < waves; w++) {
      const unsigned long long *r = &h[w * K];
      int prev = 0;
      for (int k = 1; k < K; k++) {
        if (!r[k]) continue;
        ph[k].push_back((double)(long long)(r[k] - r[prev]));
        prev = k;
      }
      tot.push_back((double)(long long)(r[prev] - r[0]));
    }
  }
  printf("s_memtime ticks per wave, median / p90 / max (n=%zu, %d steps):\n", n, steps);
  for (int k = 1; k < K; k++) {
    std::vector<double> &v = ph[k];
    if (v.empty()) continue;
    std::sort(v.begin(), v.end());
    printf("  %-46s %9.0f %9.0f %9.0f  (%zu)\n", names[k], v[v.size() / 2], v[v.size() * 9 / 10], v.back(), v.size());
  }
  std::sort(tot.begin(), tot.end());
  printf("  %-46s %9.0f %9.0f %9.0f\n", "total", tot[tot.size() / 2], tot[tot.size() * 9 / 10], tot.back());
  return 0;
}
