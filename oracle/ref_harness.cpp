// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY.  Links the UNMODIFIED reference core
// (/root/reference/src/{environment,map,player,cards,geometry}.cpp + its headers) and exposes a
// tiny C API so tests/golden generation can drive the reference's own vec_cog_env<1> and
// vec_action_sampler<1> (include/vec_environment.h, include/vec_sampler.h).
//
// Built by oracle/Makefile into oracle/_ref/libref.so with the image's clang++ against the
// image's libstdc++ 11; no shims, stand-in headers or patched libraries.  Consequence: the
// reference ABORTS on seeds whose map generation erases past the end of valid_indices
// (map.cpp:727, behaviour that needs GCC>=13 libstdc++) and on 2/3-player B-start maps
// (map.cpp:347-352).  Callers must screen seeds with the C oracle's hazard flags first.
#include "vec_environment.h"
#include "vec_sampler.h"
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

using env1 = vec_cog_env<1>;
using smp1 = vec_action_sampler<1>;

// Constructed in zero-filled memory: the reference leaves Player::has_won of players >=
// n_players uninitialised (player.cpp:45) and sums it into every reward (environment.cpp:
// 283-285).  Zeroed storage is the state of fresh pages and the behaviour the
// engine defines; heap reuse would otherwise make 2/3-player rewards depend on process history.
extern "C" {
void *ref_create() {
  const size_t bytes = (sizeof(env1) + 63) / 64 * 64;
  void *mem = std::aligned_alloc(64, bytes);
  std::memset(mem, 0, bytes);
  return new (mem) env1();
}
void ref_destroy(void *h) {
  static_cast<env1 *>(h)->~env1();
  std::free(h);
}
int ref_reset(void *h, uint32_t seed, uint8_t np, uint8_t npieces, int diff, uint32_t max_steps) {
  try {
    static_cast<env1 *>(h)->reset(seed, np, npieces, static_cast<Difficulty>(diff), max_steps, false);
  } catch (const generate_map_failure &) {
    return -1;
  }
  return 0;
}
int ref_reset_default(void *h) {
  try {
    static_cast<env1 *>(h)->reset();
  } catch (const generate_map_failure &) {
    return -1;
  }
  return 0;
}
int ref_step(void *h, const void *action) {
  try {
    static_cast<env1 *>(h)->step(*reinterpret_cast<const std::array<ActionData, 1> *>(action));
  } catch (const generate_map_failure &) {
    return -1;
  }
  return 0;
}
const void *ref_obs(void *h) { return static_cast<env1 *>(h)->get_observations().data(); }
const void *ref_sel(void *h) { return static_cast<env1 *>(h)->get_selected_action_masks().data(); }
const void *ref_rewards(void *h) { return static_cast<env1 *>(h)->get_rewards().data(); }
const void *ref_dones(void *h) { return static_cast<env1 *>(h)->get_dones().data(); }
const void *ref_agent(void *h) { return static_cast<env1 *>(h)->get_agent_selections().data(); }
const void *ref_infos(void *h) { return static_cast<env1 *>(h)->get_infos().data(); }
size_t ref_sizeof(int which) {
  switch (which) {
  case 0: return sizeof(ObsData);
  case 1: return sizeof(ActionMask);
  case 2: return sizeof(ActionData);
  case 3: return sizeof(Info);
  default: return 0;
  }
}
// Field offsets of the reference's records (api.h:67-161), by dotted numpy field path, so the
// layout test pins every named field against the reference build rather than a restatement.
// (Address differences inside one object: offsetof cannot index a std::array.)
struct RefField {
  const char *name;
  size_t off;
};
static std::vector<RefField> ref_layout() {
  static ObsData o;
  static ActionMask m;
  static ActionData a;
  static Info f;
#define D(obj, T, path) RefField{#T "." #path, (size_t)((const char *)&obj.path - (const char *)&obj)}
  return {
      D(o, ObsData, shared), D(o, ObsData, shared.map), D(o, ObsData, shared.phase),
      D(o, ObsData, shared.current_resources), D(o, ObsData, shared.shop), D(o, ObsData, player_data),
      D(o, ObsData, player_data[1]), D(o, ObsData, player_data[3]), D(o, ObsData, player_data[0].obs.draw),
      D(o, ObsData, player_data[0].obs.hand), D(o, ObsData, player_data[0].obs.active),
      D(o, ObsData, player_data[0].obs.played), D(o, ObsData, player_data[0].obs.discard),
      D(o, ObsData, player_data[0].action_mask), D(o, ObsData, player_data[0].action_mask.play),
      D(o, ObsData, player_data[0].action_mask.play_special), D(o, ObsData, player_data[0].action_mask.remove),
      D(o, ObsData, player_data[0].action_mask.move), D(o, ObsData, player_data[0].action_mask.get_from_shop),
      D(m, ActionMask, play), D(m, ActionMask, play_special), D(m, ActionMask, remove), D(m, ActionMask, move),
      D(m, ActionMask, get_from_shop), D(a, ActionData, play), D(a, ActionData, play_special),
      D(a, ActionData, remove), D(a, ActionData, move), D(a, ActionData, get_from_shop), D(f, Info, total_length),
      D(f, Info, agent_infos), D(f, Info, agent_infos[1]), D(f, Info, agent_infos[0].steps_taken),
      D(f, Info, agent_infos[0].returns), D(f, Info, agent_infos[0].travelled_hexes),
      D(f, Info, agent_infos[0].cards_added), D(f, Info, agent_infos[0].cards_removed),
      D(f, Info, agent_infos[0].n_machete_uses), D(f, Info, agent_infos[0].n_paddle_uses),
      D(f, Info, agent_infos[0].n_coin_uses), D(f, Info, agent_infos[0].n_card_uses),
  };
#undef D
}
int ref_layout_count() { return (int)ref_layout().size(); }
const char *ref_layout_name(int k) { return ref_layout()[k].name; }
size_t ref_layout_offset(int k) { return ref_layout()[k].off; }
void *ref_sampler_create(uint32_t seed) { return new smp1(seed); }
void ref_sampler_destroy(void *s) { delete static_cast<smp1 *>(s); }
void ref_sample(void *s, const void *mask) {
  static_cast<smp1 *>(s)->sample(*reinterpret_cast<const std::array<ActionMask, 1> *>(mask));
}
const void *ref_sampler_actions(void *s) { return static_cast<smp1 *>(s)->get_actions().data(); }
}

// The reference's own loop for one env (benchmarks/benchmarks.py:47-51 with the runner's
// mask source, include/runner.h:46-55): `steps` x (sample(selected_action_masks); step(actions)),
// in C so that fixtures of whole timed workloads (tens of thousands of envs x ~1,000 steps) are
// cheap to generate.  0, or -1 when a reset inside the loop failed.
extern "C" int ref_run_selected(void *h, void *s, int steps) {
  env1 *e = static_cast<env1 *>(h);
  smp1 *q = static_cast<smp1 *>(s);
  try {
    for (int t = 0; t < steps; t++) {
      q->sample(e->get_selected_action_masks());
      e->step(q->get_actions());
    }
  } catch (const generate_map_failure &) {
    return -1;
  }
  return 0;
}

// Calibration only: the reference's own sequential loop (vec_cog_env<1>::step + action_sampler)
// over n envs with the given (hazard-free) seeds, `steps` x (sample(selected mask); step).
#include <chrono>
#include <vector>
extern "C" double ref_bench_seq(const uint32_t *seeds, int n, int steps, uint8_t np, uint8_t npieces, int diff) {
  std::vector<env1 *> envs(n);
  std::vector<smp1 *> smps(n);
  for (int i = 0; i < n; i++) {
    envs[i] = static_cast<env1 *>(ref_create());
    envs[i]->reset(seeds[i], np, npieces, static_cast<Difficulty>(diff), 100000, false);
    smps[i] = new smp1(seeds[i]);
  }
  auto t0 = std::chrono::steady_clock::now();
  for (int t = 0; t < steps; t++)
    for (int i = 0; i < n; i++) {
      smps[i]->sample(envs[i]->get_selected_action_masks());
      envs[i]->step(smps[i]->get_actions());
    }
  auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; i++) {
    ref_destroy(envs[i]);
    delete smps[i];
  }
  return std::chrono::duration<double>(t1 - t0).count();
}
