/* asan_harness.c -- TEST INFRASTRUCTURE ONLY: the C oracle (cog_oracle.c) driven over the golden
 * trace scenarios in a plain executable, so that it can be built with
 * -fsanitize=address,undefined -- the equivalent of the reference's Debug build, which compiles
 * its core with -fsanitize=address,undefined (reference CMakeLists.txt:97-105).  The oracle
 * reproduces the reference's u8 wrap-around and its flat-DeckObs scans on
 * purpose; this run shows that none of it is undefined behaviour or an out-of-bounds access in
 * the restatement.
 *
 *   make -C oracle asan      -> oracle/_asan/harness_asan (sanitized) and oracle/_asan/harness (plain)
 *   oracle/_asan/harness_asan              one line per scenario: name, steps, resets, FNV-1a hash, flags
 *   oracle/_asan/harness_asan --selftest   a deliberate heap overread (the sanitizer must stop it)
 *
 * Scenarios: the reference trace sets of tests/golden/ref_traces (oracle/gen_golden.py traces():
 * the stored-mask driver with auto-resets, B-start seeds, 2 and 3 players, the selected-mask
 * loop), run as batches of n envs with seeds seed + i, every output record hashed after every step.
 * tests/test_oracle_asan.py checks that the sanitized build reports nothing and that its hashes
 * equal the plain build's.  Not used by the product, bench or smoke. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/cog_types.h"
#include "cog_oracle.h"

typedef struct {
  const char *name;
  uint32_t seed;
  uint8_t n_players, n_pieces;
  int difficulty;
  uint32_t max_steps, sampler_seed;
  int stored; /* 1: the current agent's stored mask (test_environment.cpp:97-98); 0: selected masks */
  int steps;
  size_t n;
} scenario;

static const scenario kScen[] = {
    {"C2shape_sel_medium", 12345, 4, 3, 1, 100000, 12345, 0, 1000, 16},
    {"C3shape_sel_hard", 12345, 4, 3, 2, 100000, 12345, 0, 1000, 16},
    {"stored_hard_ms30", 7, 4, 3, 2, 30, 7, 1, 1500, 16},
    {"stored_medium_ms40_bstart", 70000, 4, 3, 1, 40, 70000, 1, 1500, 16},
    {"c1like_2p_medium_sel", 0, 2, 3, 1, 100000, 0, 0, 20000, 1},
    {"c1like_2p_medium_sto", 0, 2, 3, 1, 100000, 0, 1, 5000, 1},
    {"p3_hard_sto_ms60", 300, 3, 3, 2, 60, 300, 1, 1500, 8},
};

static uint64_t fnv(uint64_t h, const void *p, size_t b) {
  const uint8_t *c = (const uint8_t *)p;
  for (size_t k = 0; k < b; k++) h = (h ^ c[k]) * 0x100000001b3ull;
  return h;
}

int main(int argc, char **argv) {
  if (argc > 1 && !strcmp(argv[1], "--selftest")) {        /* the sanitizer is live: one heap overread */
    volatile uint8_t *p = (volatile uint8_t *)malloc(16);
    volatile int past = 16;
    const int v = p[past];
    free((void *)p);
    return v == 0x5a ? 3 : 4;
  }
  int bad = 0;
  for (size_t q = 0; q < sizeof(kScen) / sizeof(kScen[0]); q++) {
    const scenario *sc = &kScen[q];
    orc_vec *v = orc_create(sc->n);
    orc_sampler *s = orc_sampler_create(sc->n, sc->sampler_seed);
    uint8_t *masks = (uint8_t *)calloc(sc->n, COG_MASK_BYTES);
    if (!v || !s || !masks) return 2;
    if (orc_reset(v, sc->seed, sc->n_players, sc->n_pieces, sc->difficulty, sc->max_steps)) {
      printf("%s reset-failed\n", sc->name);
      bad = 1;
      continue;
    }
    uint64_t h = 0xcbf29ce484222325ull;
    long resets = 0;
    for (int t = 0; t < sc->steps; t++) {
      const uint8_t *obs = (const uint8_t *)orc_obs(v);
      const uint8_t *agent = orc_agent_sel(v);
      if (sc->stored) {
        for (size_t i = 0; i < sc->n; i++)
          memcpy(masks + i * COG_MASK_BYTES,
                 obs + i * COG_OBS_BYTES + COG_OBS_PLAYER0 + (size_t)COG_OBS_PLAYER_STRIDE * agent[i] + COG_PD_MASK,
                 COG_MASK_BYTES);
        orc_sample(s, masks);
      } else {
        orc_sample(s, orc_sel(v));
      }
      orc_step(v, orc_sampler_actions(s));
      h = fnv(h, orc_obs(v), sc->n * COG_OBS_BYTES);
      h = fnv(h, orc_sel(v), sc->n * COG_MASK_BYTES);
      h = fnv(h, orc_rewards(v), sc->n * 4 * sizeof(float));
      h = fnv(h, orc_dones(v), sc->n);
      h = fnv(h, orc_agent_sel(v), sc->n);
      h = fnv(h, orc_infos(v), sc->n * COG_INFO_BYTES);
      h = fnv(h, orc_sampler_actions(s), sc->n * COG_ACTION_BYTES);
      for (size_t i = 0; i < sc->n; i++) resets += orc_dones(v)[i] ? 1 : 0;
    }
    uint32_t flags = 0;
    for (size_t i = 0; i < sc->n; i++) flags |= orc_flags(v, i);
    printf("%s %d %ld %016llx %02x\n", sc->name, sc->steps, resets, (unsigned long long)h, flags);
    fflush(stdout);
    free(masks);
    orc_sampler_destroy(s);
    orc_destroy(v);
  }
  return bad;
}
