// Diagnostic only: the one-step-per-launch kernel (k_env_step<selected>, the runner at
// set_chunk(1): what env.step() / runner.step() launch) on the bench workload.  Prints the
// device us per launch (median of 200 launches, HIP events on the env's stream) per env count.
// With tools/stepprobe_priv.patch applied to the engine (git apply; revert after the build) and
// -DPROBE_PRIV_MODE=1 / 2 / 3: no state stores / the private stores as issued (AoS) / the same in a
// structure-of-arrays layout, both into scratch (profiles/r06_step_store_probe.txt).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp \
//         -Iinclude -Igym-eldorado_amd/csrc tools/stepprobe.cpp -o tools/bin/stepprobe
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <algorithm>
#include <cstdio>
#include <vector>

int main(int argc, char **argv) {
  const char *tag = argc > 1 ? argv[1] : "step";
  std::vector<size_t> sizes;
  for (int a = 2; a < argc; a++) sizes.push_back(strtoul(argv[a], nullptr, 10));
  if (sizes.empty()) sizes = {65536, 32768, 16384, 8192, 1024};
  for (size_t n : sizes) {
    cog_env *env;
    cog_sampler *smp;
    cog_runner *run;
    if (cog_env_create(n, 0, &env) || cog_sampler_create(n, 12345, 0, &smp) ||
        cog_env_reset(env, 12345, 4, 3, 2, 100000, 0) || cog_runner_create(env, smp, 1, COG_RUNNER_DEVICE_VIEWS, &run)) {
      printf("setup failed: %s\n", cog_last_error());
      return 1;
    }
    cog_runner_set_chunk(run, 1);
    cog_runner_rollout(run, 50);
    cog_runner_sync(run);
    hipStream_t st = env->sh[0].stream;
    std::vector<hipEvent_t> ev(201);
    for (auto &e : ev)
      if (hipEventCreate(&e) != hipSuccess) return 1;
    if (hipEventRecord(ev[0], st) != hipSuccess) return 1;
    for (int r = 0; r < 200; r++) {
      cog_runner_rollout(run, 1);
      if (hipEventRecord(ev[r + 1], st) != hipSuccess) return 1;
    }
    if (hipEventSynchronize(ev[200]) != hipSuccess) return 1;
    std::vector<double> v;
    for (int r = 0; r < 200; r++) {
      float ms;
      if (hipEventElapsedTime(&ms, ev[r], ev[r + 1]) != hipSuccess) return 1;
      v.push_back(ms * 1e3);
    }
    std::sort(v.begin(), v.end());
    const int rc = cog_runner_sync(run);
    printf("%s n=%6zu  launch %7.2f us median (p10 %7.2f, p90 %7.2f)  %.3f G env-steps/s  sync %d\n", tag, n, v[100],
           v[20], v[180], n / v[100] * 1e-3, rc);
    fflush(stdout);
    for (auto &e : ev) (void)hipEventDestroy(e);
    cog_runner_destroy(run);
    cog_sampler_destroy(smp);
    cog_env_destroy(env);
  }
  return 0;
}
