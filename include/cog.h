/* cog.h -- C ABI of the MI355X-native City-of-Gold batched step engine (libcog_hip.so).
 *
 * This is the boundary a reference-side binding calls (see INTEGRATION.md for the pybind11 /
 * ctypes stubs).  Plain pointers and sizes only: no torch, numpy or HIP types.  Every entry
 * point returns an int status (COG_OK == 0) and never throws; cog_last_error() gives the
 * message of the last failing call on the calling thread.  A handle is single-threaded: calls
 * on one handle must not overlap.  Work is ordered on one HIP stream per handle.
 *
 * Record layouts (ObsData, ActionMask, ActionData, Info) are in cog_types.h and are
 * byte-identical to the reference's numpy structured views (reference include/api.h:67-161).
 *
 * Reference interface replaced by each group (reference file:line):
 *   cog_env_*      vec_cog_env<N> + py_vec_env<N>   include/vec_environment.h:10-81,
 *                                                   include/pybind/vectorized.h:25-105,185-214
 *   cog_sampler_*  vec_action_sampler<N> + py_vec_action_sampler<N>
 *                                                   include/vec_sampler.h:7-28,
 *                                                   include/pybind/vectorized.h:107-127,217-230
 *   cog_runner_*   ThreadedRunner<N> + py_threaded_runner<N>
 *                                                   include/runner.h:21-115,
 *                                                   include/pybind/vectorized.h:129-161,232-256
 */
#ifndef COG_H
#define COG_H

#include <stddef.h>
#include <stdint.h>

#include "cog_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__)
#define COG_API __attribute__((visibility("default")))
#else
#define COG_API
#endif

#define COG_ABI_VERSION 1

/* status codes */
#define COG_OK 0
#define COG_ERR_INVALID (-1)   /* bad argument: NULL handle, wrong batch length, ... */
#define COG_ERR_HIP (-2)       /* HIP runtime failure (message in cog_last_error) */
#define COG_ERR_MAPGEN (-3)    /* generate_map_failure (reference map.cpp:699-702) */
#define COG_ERR_NODEVICE (-4)  /* no usable gfx950 device: the engine never falls back to CPU */
#define COG_ERR_OOM (-5)       /* device or pinned-host allocation failed */

/* difficulty (reference include/constants.h:11) */
#define COG_EASY 0
#define COG_MEDIUM 1
#define COG_HARD 2

/* hazard flags reported per env by cog_env_hazards: reference UB or toolchain-dependent
 * behaviour that this engine defines */
#define COG_HAZ_MAPGEN_FAIL 0x01u
#define COG_HAZ_ERASE_PAST 0x02u   /* map.cpp:727 erase past the end: GCC>=13 semantics used */
#define COG_HAZ_Q9_OOB 0x04u       /* map.cpp:347-352 write past player_locations: dropped */
#define COG_HAZ_Q24_CLAMP 0x08u    /* player.cpp:92 discard more than active: clamped */
#define COG_HAZ_GRID_OVER 0x10u    /* map wider than the 48x48 observation: rejected */
#define COG_HAZ_OOB_LOOKUP 0x20u   /* hex lookup outside the map: reads as mountain */
#define COG_HAZ_SCAN_OVER 0x40u    /* card scan past the DeckObs record */
#define COG_HAZ_B_START_LT4 0x80u  /* start piece B with < 4 players */
#define COG_HAZ_BAD_ACTION 0x100u  /* host action index past its head (reference: OOB access): clamped */

/* runner flags */
#define COG_RUNNER_DEVICE_VIEWS 0x1u  /* sync() does not refresh the host views (C5: outputs stay in HBM) */
#define COG_RUNNER_STORED_MASKS 0x2u  /* sample from the current agent's stored mask (full dynamics) */

typedef struct cog_env cog_env;
typedef struct cog_sampler cog_sampler;
typedef struct cog_runner cog_runner;

/* Persistent views.  Host views are pinned host memory updated in place by every synchronous
 * call (reference common.h:97-101 semantics: non-owning, persistent).  Device views are the
 * engine state itself, in HBM, same layouts. */
typedef struct cog_env_views {
  size_t n_envs;
  cog_obs_t *observations;                 /* [n] ObsData          */
  cog_action_mask_t *selected_action_masks;/* [n] ActionMask       */
  float *rewards;                          /* [n][4]               */
  uint8_t *dones;                          /* [n] bool             */
  uint8_t *agent_selection;                /* [n]                  */
  cog_info_t *infos;                       /* [n] Info             */
  void *d_observations;
  void *d_selected_action_masks;
  void *d_rewards;
  void *d_dones;
  void *d_agent_selection;
  void *d_infos;
} cog_env_views;

COG_API const char *cog_last_error(void);
COG_API int cog_abi_version(void);
COG_API int cog_device_count(int *out);
/* which persistent rollout kernel cog_runner_rollout launches for a shard of n envs with
 * n_players players, sampling the selected (stored_masks 0) or stored masks (measurement labels
 * only): 0 duo (k_env_rollout_duo + k_env_fixup), 1 wave (k_env_rollout), 2 pipe
 * (k_env_rollout_pipe), 3 trio (k_env_rollout_trio + k_env_fixup); $COG_ROLLOUT / $COG_TRIO
 * force one (cog_engine.hip rollout_kind) */
COG_API int cog_rollout_kind(size_t n_envs, int n_players, int stored_masks);

/* ---- vectorized environment ------------------------------------------------------------ */
/* vec_cog_env<N>() (vec_environment.h:23-30): N default-constructed envs on `device`;
 * default params seed=std::random_device, 4 players, 3 pieces, EASY, 100000 max steps. */
COG_API int cog_env_create(size_t n_envs, int device, cog_env **out);
/* the same batch split over several GPUs of this process: shard k holds the contiguous envs
 * [first_k, first_k + count_k), the reference ThreadedRunner's block split (runner.h:33-38:
 * n / n_devices each, the last shard takes the remainder), with its own HIP stream.  A device
 * may be listed more than once (two shards, two streams, one GPU).  Seeds are seed + global
 * index, so every result is independent of the shard layout. */
COG_API int cog_env_create_multi(size_t n_envs, const int *devices, int n_devices, cog_env **out);
COG_API int cog_env_num_shards(const cog_env *env, int *out);
COG_API int cog_env_shard_info(const cog_env *env, int shard, size_t *first, size_t *count, int *device);
COG_API void cog_env_destroy(cog_env *env);
COG_API int cog_env_num_envs(const cog_env *env, size_t *out);
/* vec_cog_env::reset(seed, n_players, n_pieces, difficulty, max_steps, render)
 * (vec_environment.h:38-44): env i gets seed + i (u32).  Synchronous. */
COG_API int cog_env_reset(cog_env *env, uint32_t seed, uint8_t n_players, uint8_t n_pieces,
                          int32_t difficulty, uint32_t max_steps, int32_t render);
/* vec_cog_env::reset() (vec_environment.h:32-36): keep params, continue each env's rng. */
COG_API int cog_env_reset_default(cog_env *env);
/* vec_cog_env::step(actions) (vec_environment.h:46-61) with n == num_envs host ActionData
 * records; auto-resets finished envs; host views refreshed before return. */
COG_API int cog_env_step(cog_env *env, const cog_action_t *actions, size_t n);
/* same, actions already in device memory (e.g. a sampler's device actions); single-shard envs */
COG_API int cog_env_step_device(cog_env *env, const void *d_actions, size_t n);
/* same, the actions produced by work queued on `stream` (a hipStream_t of the env's device, e.g.
 * torch.cuda.current_stream(); NULL is the null stream): the step is ordered after that work
 * (event + stream wait).  COG_NO_STREAM: no ordering (cog_env_step_device). */
#define COG_NO_STREAM ((void *)(intptr_t)-1)
COG_API int cog_env_step_device_stream(cog_env *env, const void *d_actions, size_t n, void *stream);
/* views (allocates + fills the pinned host views on first use).  Device pointers are set for
 * single-shard envs only; cog_env_shard_views gives shard k's device records and its slice of
 * the host views. */
COG_API int cog_env_get_views(cog_env *env, cog_env_views *out);
COG_API int cog_env_shard_views(cog_env *env, int shard, cog_env_views *out);
COG_API int cog_env_sync_host(cog_env *env);
/* OR of hazard flags over envs; per_env (n entries) may be NULL */
COG_API int cog_env_hazards(cog_env *env, uint32_t *flags_or, uint32_t *per_env);
COG_API int cog_env_clear_hazards(cog_env *env);
COG_API void *cog_env_stream(cog_env *env);     /* hipStream_t of shard 0 */
COG_API void *cog_env_shard_stream(cog_env *env, int shard);
/* ordering against a caller's stream on shard k's device (e.g. torch.cuda.current_stream();
 * NULL is the null stream):
 * wait_stream: engine work queued later on shard k runs after the work queued on `stream` so far;
 * signal_stream: work queued later on `stream` runs after the engine work queued on shard k */
COG_API int cog_env_wait_stream(cog_env *env, int shard, void *stream);
COG_API int cog_env_signal_stream(cog_env *env, int shard, void *stream);
/* after the caller wrote the env's device records (DLPack views / d_* pointers), ordered after
 * the work queued on `stream` so far (COG_NO_STREAM: none): the engine takes the records as they
 * now are, as the reference's views alias its live state (include/pybind/common.h:97-101) -- the
 * decks, phase, resources and shop are read from the records anyway; the selected and stored
 * ActionMask records (0/1 bytes) and Info steps_taken also feed the engine's private mirrors, which
 * this rebuilds.  Host views are refreshed when the env has them.  Without this call, writes to
 * those records are not seen by the next step (see INTEGRATION.md "Device views"). */
COG_API int cog_env_invalidate_device(cog_env *env, void *stream);
/* diagnostics: re-run the map-observation encode (map.cpp:389-405) over all envs `iters`
 * times back to back; average device time per launch (HIP events).  Output is unchanged.
 * variant: 0 = production kernel, >0 = alternative implementations kept for A/B timing. */
COG_API int cog_env_time_encode(cog_env *env, int iters, int variant, double *ms_per_launch);
/* measurement: read + write bytes per second of the engine's device copy kernel (16-B loads and
 * stores, plain or non-temporal, 8 or 32 waves per CU: the fastest) over two `bytes` buffers on
 * `device`: the copy peak beside which the encode's HBM fraction is reported (BASELINE.md "a
 * measured copy-kernel peak") */
COG_API int cog_time_copy(int device, size_t bytes, int iters, double *gb_per_s);
/* measurement: read + write bytes per second of a stream with the encode's read:write mix (reads
 * `bytes`, writes 7 x `bytes`, coalesced, plain or non-temporal stores: the faster) on `device`:
 * the bandwidth peak of a kernel shaped like the map-observation encode */
COG_API int cog_time_stream_mix(int device, size_t bytes, int iters, double *gb_per_s);
COG_API int cog_env_device(const cog_env *env); /* device ordinal */
/* on (default): a finished env is reset inside the same step call, as vec_cog_env<N>::step does
 * (vec_environment.h:56-59).  off: cog_env::step semantics (environment.cpp:91-95) -- the env
 * stays done and later steps are dead steps until reset() */
COG_API int cog_env_set_autoreset(cog_env *env, int on);

/* ---- masked uniform random sampler ------------------------------------------------------- */
/* vec_action_sampler<N>(seed) (vec_sampler.h:9-13): sampler i seeded seed + i (seed a u32, the
 * sum not wrapped). */
COG_API int cog_sampler_create(size_t n_envs, uint64_t seed, int device, cog_sampler **out);
/* sharded like cog_env_create_multi (a runner needs the env's and the sampler's shards equal) */
COG_API int cog_sampler_create_multi(size_t n_envs, uint64_t seed, const int *devices, int n_devices,
                                     cog_sampler **out);
/* the batch is the block [first_index, first_index + n_envs) of a larger one (a rank's shard,
 * city_of_gold/shard.py): sampler i seeded seed + first_index + i, the sum in 64 bits as the
 * unsharded batch computes it (vec_sampler.h:9-13), so a sharded run samples the same actions for
 * every seed -- a u32 base of seed + first_index would wrap where the reference does not */
COG_API int cog_sampler_create_at(size_t n_envs, uint64_t seed, uint64_t first_index, const int *devices,
                                  int n_devices, cog_sampler **out);
COG_API int cog_sampler_num_shards(const cog_sampler *s, int *out);
COG_API void cog_sampler_destroy(cog_sampler *s);
/* vec_action_sampler::sample(masks) (vec_sampler.h:14-21): n == num_envs host ActionMask
 * records; host actions view refreshed before return. */
COG_API int cog_sampler_sample(cog_sampler *s, const cog_action_mask_t *masks, size_t n);
/* same, masks in device memory (e.g. an env's d_selected_action_masks); single-shard samplers */
COG_API int cog_sampler_sample_device(cog_sampler *s, const void *d_masks, size_t n);
COG_API cog_action_t *cog_sampler_actions(cog_sampler *s);   /* persistent host view */
COG_API void *cog_sampler_device_actions(cog_sampler *s);    /* device view (shard 0) */
COG_API void *cog_sampler_shard_device_actions(cog_sampler *s, int shard);
COG_API int cog_sampler_device(const cog_sampler *s);       /* device ordinal */
/* samples so far, and how many of them took the speculative sample of the env step before them
 * (env.step(actions) with this sampler's actions view samples the next actions from the masks it
 * leaves; sample() of that env's own mask view then needs no launch).  Diagnostics. */
COG_API int cog_sampler_spec_stats(const cog_sampler *s, uint64_t *samples, uint64_t *hits);

/* ---- runner: asynchronous sample/step on the env's streams (runner.h:81-100) ---------------- */
COG_API int cog_runner_create(cog_env *env, cog_sampler *s, size_t n_threads, uint32_t flags,
                              cog_runner **out);
COG_API void cog_runner_destroy(cog_runner *r);
COG_API size_t cog_runner_n_threads(const cog_runner *r);
COG_API int cog_runner_sample(cog_runner *r);    /* enqueue sample(selected masks) */
COG_API int cog_runner_step(cog_runner *r);      /* enqueue step(sampler actions); fuses a pending sample */
COG_API int cog_runner_sync(cog_runner *r);      /* wait; refresh host views unless DEVICE_VIEWS */
COG_API int cog_runner_rollout(cog_runner *r, int steps);   /* enqueue steps x (sample; step) */
/* rollout() steps per kernel launch: 1 = one launch per step; K > 1 = a persistent kernel runs
   K x (sample; step) per launch, storing every step's outputs as a single step does */
COG_API int cog_runner_set_chunk(cog_runner *r, int steps_per_launch);
COG_API int cog_runner_set_timing(cog_runner *r, int enable);
/* device time of the fused launches since enabled: HIP events bracket each step() launch and each
   rollout() batch on every shard's stream; the slowest shard's total; *launches = fused launches
   covered */
COG_API int cog_runner_kernel_time(cog_runner *r, double *total_ms, uint64_t *launches);

#ifdef __cplusplus
}
#endif
#endif /* COG_H */
