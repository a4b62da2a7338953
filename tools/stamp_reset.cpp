// Diagnostic only: where a batch reset's time goes.  k_reset built with -DCOG_STAMPS (per-wave
// s_memtime at the phase boundaries of env_reset); prints the median ticks per phase over waves
// and the kernel's device time.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DCOG_STAMPS -Iinclude \
//         -Igym-eldorado_amd/csrc tools/stamp_reset.cpp -o tools/stamp_reset
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <algorithm>
#include <cstdio>
#include <vector>

int main(int argc, char **argv) {
  const size_t n = argc > 1 ? strtoul(argv[1], nullptr, 10) : 65536;
  const int diff = argc > 2 ? atoi(argv[2]) : 2;
  cog_env *env;
  if (cog_env_create(n, 0, &env)) {
    printf("setup failed: %s\n", cog_last_error());
    return 1;
  }
  const size_t waves = (n + 63) / 64;
  constexpr int K = 16;
  unsigned long long *d;
  if (hipMalloc(&d, waves * K * 8) != hipSuccess || hipMemset(d, 0, waves * K * 8) != hipSuccess) return 1;
  if (cog_env_reset(env, 12345, 4, 3, diff, 100000, 0)) return 1;   // warm
  env->sh[0].s.stamps = d;
  hipEvent_t a, b;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
  if (hipEventRecord(a, env->sh[0].stream) != hipSuccess) return 1;
  cog::ResetParams p{};
  p.use_params = 1; p.seed = 777; p.n_players = 4; p.n_pieces = 3; p.difficulty = diff; p.max_steps = 100000;
  if (cog::launch_reset(env->sh[0].s, p, env->sh[0].stream)) return 1;
  if (hipEventRecord(b, env->sh[0].stream) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return 1;
  float ms;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return 1;
  std::vector<unsigned long long> h(waves * K);
  if (hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  const char *pn[6] = {"generate", "build_cgrid", "player_reset x4", "add_players + shop", "update_observation + sel",
                       "load_cells"};
  printf("k_reset + k_sync_heads: %.3f ms for %zu envs (difficulty %d)\n", ms, n, diff);
  printf("median s_memtime ticks per wave (100 MHz? see guide: shader cycles) by phase:\n");
  for (int k = 0; k < 6; k++) {
    std::vector<double> v;
    for (size_t w = 0; w < waves; w++)
      if (h[w * K + k] && h[w * K + k + 1]) v.push_back((double)(h[w * K + k + 1] - h[w * K + k]));
    std::sort(v.begin(), v.end());
    if (v.empty()) continue;
    printf("  %-28s %12.0f  (waves %zu)\n", pn[k], v[v.size() / 2], v.size());
  }
  return 0;
}
