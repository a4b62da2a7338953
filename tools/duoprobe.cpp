// Diagnostic only: the duo rollout (k_env_rollout_duo + k_env_fixup) on the bench workload.
// Prints the device us/step of 1,000-step and 20-step launches per env count; built with
// -DCOG_STAMPS it also prints the per-phase s_memtime ticks per step of the stepping and the
// storing waves (median over waves).  Variants: -DDUO_* ablations in the engine source.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -amdgpu-sched-strategy=max-ilp \
//         -Iinclude -Igym-eldorado_amd/csrc [-DCOG_STAMPS] tools/duoprobe.cpp -o tools/duoprobe
#include "../gym-eldorado_amd/csrc/cog_engine.hip"
#include "../gym-eldorado_amd/csrc/cog_abi.cpp"
#include <algorithm>
#include <cstdio>
#include <vector>

static double med(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char **argv) {
  const char *tag = argc > 1 ? argv[1] : "duo";
  std::vector<size_t> sizes;
  for (int a = 2; a < argc; a++) sizes.push_back(strtoul(argv[a], nullptr, 10));
  if (sizes.empty()) sizes = {65536, 32768, 16384, 8192};
  for (size_t n : sizes) {
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
    hipStream_t st = env->sh[0].stream;
    hipEvent_t a, b;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return 1;
    auto timed = [&](int k, int reps) {
      std::vector<double> v;
      cog_runner_set_chunk(run, k);
      for (int r = 0; r < reps; r++) {
        if (hipEventRecord(a, st) != hipSuccess) return -1.0;
        cog_runner_rollout(run, k);
        if (hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess) return -1.0;
        float ms;
        if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.0;
        v.push_back(ms * 1e3);
      }
      return med(v);
    };
    const double r1000 = timed(1000, 5), r20 = timed(20, 25);
    printf("%s n=%6zu  %6.3f us/step (1000-step launches)  20-step launch %7.2f us (%5.3f us/step)\n", tag, n,
           r1000 / 1000, r20, r20 / 20);
    if (getenv("PROBE_SHORT")) {                           // the fixed cost: 1-, 2- and 5-step launches
      const double r1 = timed(1, 25), r2 = timed(2, 25), r5 = timed(5, 25);
      printf("%s n=%6zu  launch of 1 / 2 / 5 steps: %7.2f %7.2f %7.2f us  (fixed ~ %.2f us)\n", tag, n, r1, r2, r5,
             r1 - (r5 - r1) / 4);
    }
    fflush(stdout);
#ifdef COG_STAMPS
    {
      // the duo: 2 waves per workgroup (stepping, storing); the trio ($COG_TRIO unset): 4 (stepping,
      // drawing, storing A, storing B).  Each wave's PH slots (cog_engine.hip): its phase names below.
      const char *trio_env = getenv("COG_TRIO");
      const int wpg = (trio_env && *trio_env == '0') ? 2 : 4;
      const size_t epw = wpg == 4 ? (size_t)cog::trio_epw(n) : 64;
      const size_t waves = (size_t)wpg * ((n + epw - 1) / epw);
      constexpr int K = 16;
      unsigned long long *d;
      if (hipMalloc(&d, waves * K * sizeof(unsigned long long)) != hipSuccess) return 1;
      if (hipMemset(d, 0, waves * K * sizeof(unsigned long long)) != hipSuccess) return 1;
      env->sh[0].s.stamps = d;
      const int chunk = getenv("PROBE_CHUNK") ? atoi(getenv("PROBE_CHUNK")) : 200;
      cog_runner_set_chunk(run, chunk);
      cog_runner_rollout(run, chunk);
      cog_runner_sync(run);
      env->sh[0].s.stamps = nullptr;
      std::vector<unsigned long long> h(waves * K);
      if (hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      const char *step_names[16] = {"step tail (done check)", "LDS player writes", "wait X", "ring write + turn change",
                                    "wait Y", "", "", "", "sample + action branch", "mip + end_turn discard",
                                    "draw", "mask swap, sh, cells", "update_observation", "", "", ""};
      const char *store_names[16] = {"", "", "", "", "", "wait Y / B: wait record", "A: wait drawn / B: wait drawn",
                                     "wait X / B: front cursor work", "", "", "", "", "", "stores (the drawn record's)",
                                     "", ""};
      const char *draw_names[16] = {"", "", "", "", "", "", "", "plays", "wait: records", "turn-end pass + ring words", "", "", "",
                                    "", "", ""};
      // the trio's stepping wave (trio_stepper): 2 = the loop top's waits (ring slot, presampled
      // draws), 5 = the turn change's wait for the drawing wave; the rest is its own work
      const char *trio_step_names[16] = {"sample + lean step", "record + turn-change reads", "wait: presampled draws",
                                         "turn change", "turn-change distance", "wait: drawing wave",
                                         "prologue (per launch)", "drain (per launch)", "epilogue (per launch)", "wait: ring slot",
                                         "", "", "", "", "", ""};
      const char *role_name[4] = {"stepping", wpg == 4 ? "drawing" : "storing", "storing A", "storing B"};
      if (getenv("PROBE_JSON") && wpg == 4) {              // one line for tools/stamps_profile.py
        double ph[16];
        for (int k = 0; k < 16; k++) {
          std::vector<double> v;
          for (size_t w = 0; w < waves; w += wpg) v.push_back((double)h[w * K + k] / chunk);
          ph[k] = med(v);
        }
        const double wait = ph[2] + ph[5] + ph[9], busy = ph[0] + ph[1] + ph[3] + ph[4];
        printf("STAMPS_JSON {\"envs\": %zu, \"steps_per_launch\": %d, \"busy_ticks_per_step\": %.1f, "
               "\"wait_ticks_per_step\": %.1f, \"ticks_per_step\": %.1f, \"busy_frac\": %.4f, \"phases\": {",
               n, chunk, busy, wait, busy + wait, busy / (busy + wait));
        for (int k = 0; k < 10; k++) printf("%s\"%s\": %.1f", k ? ", " : "", trio_step_names[k], ph[k]);
        printf("}}\n");
      }
      if (wpg == 4) {                                      // the launch timeline (stepping waves, 100 MHz)
        unsigned long long t0 = ~0ull;
        for (size_t w = 0; w < waves; w += wpg) t0 = std::min(t0, h[w * K + 10]);
        // per round of blocks ($PROBE_ROUND blocks each, default 512 = two workgroups per CU): the
        // hardware's rounds of workgroups, or a multi-block launch's k-th block of each workgroup
        const size_t rb = getenv("PROBE_ROUND") ? strtoul(getenv("PROBE_ROUND"), nullptr, 10) : 512;
        const size_t nblk = waves / wpg;
        for (size_t r0 = 0; nblk > rb && r0 < nblk; r0 += rb) {
          printf("  round of blocks %zu..%zu (us after the first stepper start; median / max):\n", r0,
                 std::min(nblk, r0 + rb) - 1);
          const char *nm[6] = {"block start", "prologue done", "last step done", "other waves done (FIN)",
                               "epilogue stores issued", "prologue loads done"};
          for (int k = 10; k < 16; k++) {
            std::vector<double> v;
            for (size_t b = r0; b < std::min(nblk, r0 + rb); b++) v.push_back((double)(h[b * wpg * K + k] - t0) * 0.01);
            printf("    stepping   %-31s %8.2f %8.2f\n", nm[k - 10], med(v), *std::max_element(v.begin(), v.end()));
          }
          const char *rn2[4] = {"stepping", "drawing", "storing A", "storing B"};
          for (int role = 1; role < 4; role++) {
            const int ks[4] = {14, 15, 11, 12};
            const char *kn[4] = {"block start", "prologue done", "last record's wait returned", "loop done"};
            for (int j = 0; j < 4; j++) {
              std::vector<double> v;
              for (size_t b = r0; b < std::min(nblk, r0 + rb); b++)
                v.push_back((double)(h[(b * wpg + role) * K + ks[j]] - t0) * 0.01);
              printf("    %-10s %-31s %8.2f %8.2f\n", rn2[role], kn[j], med(v), *std::max_element(v.begin(), v.end()));
            }
          }
        }
        const char *tl_names[5] = {"stepper start (after the table barrier)", "prologue done (barrier B)",
                                   "last step done", "other waves done (FIN)", "epilogue stores issued"};
        printf("  launch timeline of a %d-step launch (us after the first stepper start; median / max over workgroups):\n", chunk);
        for (int k = 10; k < 15; k++) {
          std::vector<double> v;
          for (size_t w = 0; w < waves; w += wpg) v.push_back((double)(h[w * K + k] - t0) * 0.01);
          const double mx = *std::max_element(v.begin(), v.end());
          printf("    %-42s %8.2f %8.2f\n", tl_names[k - 10], med(v), mx);
        }
        const char *rn[4] = {"stepping", "drawing", "storing A", "storing B"};
        for (int role = 0; role < 4; role++) {
          std::vector<double> v;
          for (size_t w = role; w < waves; w += wpg) v.push_back((double)(h[w * K + 15] - t0) * 0.01);
          printf("    %-10s %-31s %8.2f %8.2f\n", rn[role], "prologue loads done", med(v),
                 *std::max_element(v.begin(), v.end()));
        }
        for (int role = 1; role < 4; role++)
          for (int k = 11; k < 13; k++) {
            std::vector<double> v;
            for (size_t w = role; w < waves; w += wpg) v.push_back((double)(h[w * K + k] - t0) * 0.01);
            printf("    %-10s %-31s %8.2f %8.2f\n", rn[role], k == 11 ? "last record's wait returned" : "loop done",
                   med(v), *std::max_element(v.begin(), v.end()));
          }
        printf("TIMELINE_JSON {\"envs\": %zu, \"steps\": %d", n, chunk);
        for (int k = 10; k < 15; k++) {
          std::vector<double> v;
          for (size_t w = 0; w < waves; w += wpg) v.push_back((double)(h[w * K + k] - t0) * 0.01);
          printf(", \"t%d_med\": %.2f, \"t%d_max\": %.2f", k - 10, med(v), k - 10, *std::max_element(v.begin(), v.end()));
        }
        printf("}\n");
      }
      for (int role = 0; role < wpg; role++) {
        const char **pn = role == 0 ? (wpg == 4 ? trio_step_names : step_names)
                                    : (wpg == 4 && role == 1) ? draw_names : store_names;
        double tot = 0;
        printf("  %s wave:\n", role_name[role]);
        for (int k = 0; k < 16; k++) {
          if (!pn[k][0]) continue;
          std::vector<double> v;
          for (size_t w = role; w < waves; w += wpg) v.push_back((double)h[w * K + k] / chunk);
          const double m = med(v);
          tot += m;
          printf("    %-34s %8.0f\n", pn[k], m);
        }
        printf("    %-34s %8.0f  (ticks per step)\n", "sum", tot);
      }
      (void)hipFree(d);
    }
#endif
    cog_runner_destroy(run);
    cog_sampler_destroy(smp);
    cog_env_destroy(env);
  }
  return 0;
}
