/* cog_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference City-of-Gold vectorized environment
 * (reference include/vec_environment.h, include/sampler.h, include/vec_sampler.h,
 *  src/{environment,player,cards,map,geometry}.cpp), written in plain C.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline.  The product (gym-eldorado_amd/) never
 * links or calls it.
 *
 * Pinning: see oracle/README.md -- checked against the reference core compiled in this
 * container (oracle/_ref, hazard-free seeds) and the committed fixtures in tests/golden/.
 */
#ifndef COG_ORACLE_H
#define COG_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* hazard flags (reference UB / toolchain-dependent behaviour) */
#define ORC_F_MAPGEN_FAIL 0x01u   /* generate_map_failure thrown (map.cpp:699-702) */
#define ORC_F_ERASE_PAST 0x02u    /* vector::erase past the end (map.cpp:727, Q5; GCC>=13 semantics) */
#define ORC_F_Q9_OOB 0x04u        /* add_players wrote past player_locations (map.cpp:347-352, Q9) */
#define ORC_F_Q24_CLAMP 0x08u     /* discard_cards n > n_active (player.cpp:92, Q24) */
#define ORC_F_GRID_OVER 0x10u     /* map wider than 49 cells: finalize would overflow (Q27) */
#define ORC_F_OOB_LOOKUP 0x20u    /* hex lookup outside hex_array */
#define ORC_F_SCAN_OVER 0x40u     /* card scan ran past the 105-byte DeckObs */
#define ORC_F_B_START_LT4 0x80u   /* start piece B with < 4 players (Q9 trigger) */

typedef struct orc_vec orc_vec;
typedef struct orc_sampler orc_sampler;

orc_vec *orc_create(size_t n);
void orc_destroy(orc_vec *v);
size_t orc_num_envs(const orc_vec *v);
/* vec_cog_env::reset(seed, ...) : env i reset with seed + i (u32).  Returns 0 or -1 on
 * generate_map_failure (envs before the failing one are reset, like the reference loop). */
int orc_reset(orc_vec *v, uint32_t seed, uint8_t n_players, uint8_t n_pieces,
              int difficulty, uint32_t max_steps);
int orc_reset_default(orc_vec *v);
int orc_reset_threaded(orc_vec *v, uint32_t seed, uint8_t n_players, uint8_t n_pieces,
                       int difficulty, uint32_t max_steps, int n_threads);
/* vec_cog_env::step: actions = n ActionData records (64 B stride) */
int orc_step(orc_vec *v, const void *actions);
/* step only envs [lo, hi) */
int orc_step_range(orc_vec *v, const void *actions, size_t lo, size_t hi);
void *orc_obs(orc_vec *v);            /* ObsData[n] */
void *orc_sel(orc_vec *v);            /* ActionMask[n] */
float *orc_rewards(orc_vec *v);       /* f32[n][4] */
uint8_t *orc_dones(orc_vec *v);       /* bool[n] */
uint8_t *orc_agent_sel(orc_vec *v);   /* u8[n] */
void *orc_infos(orc_vec *v);          /* Info[n] */
uint32_t orc_flags(const orc_vec *v, size_t i);   /* per-env sticky hazard flags */
void orc_clear_flags(orc_vec *v);
/* private state for debugging: 16 bytes per player + env scalars */
int orc_debug_state(const orc_vec *v, size_t i, uint32_t *out, size_t n_out);

orc_sampler *orc_sampler_create(size_t n, uint32_t seed);
orc_sampler *orc_sampler_create_at(size_t n, uint32_t seed, uint64_t first);   /* seeds seed + first + i */
void orc_sampler_destroy(orc_sampler *s);
void orc_sample(orc_sampler *s, const void *masks);   /* ActionMask[n] -> actions */
void orc_sample_range(orc_sampler *s, const void *masks, size_t lo, size_t hi);
void *orc_sampler_actions(orc_sampler *s);            /* ActionData[n] */

/* reference ThreadedRunner shape (runner.h:21-64): contiguous env blocks, one pinned worker
 * per block, per step "sample(selected masks); step(actions)" then a barrier.
 * Returns wall seconds for `steps` steps. */
double orc_run_threaded(orc_vec *v, orc_sampler *s, int steps, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
