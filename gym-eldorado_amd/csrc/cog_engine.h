// cog_engine.h -- internal interface between the C-ABI layer (cog_abi.cpp) and the CDNA4 kernels
// (cog_engine.hip).  Not part of the public ABI.
//
// Device data layout per environment i (all buffers allocated once per handle, in HBM):
//   obs   [N] x 17216 B   ObsData records, byte-identical to reference api.h:126-129 -- THE
//                         engine state for everything the reference keeps in ObsData (decks,
//                         stored masks, phase, resources, shop) and the map encode target.
//   sel   [N] x 128 B     selected ActionMask (the deck's mask, player.cpp:16-27)
//   info  [N] x 192 B     Info records
//   rew   [N] x 4 f32, done [N] u8, agent [N] u8
//   priv  [N] x 160 B     EnvPriv: everything the reference keeps in private members
//                         (rng, turn counter, Player/Deck/Shop counters, player locations,
//                         map bounds) + a cache of each player's 7 neighbourhood hex codes
//   grid  [N] x 16384 B   absolute-coordinate hex-code grid, 128 x 128 cells, cell (x, y) at
//                         (x + 64) * 128 + (y + 64); 0 = no hex.  Built by map generation,
//                         read by movement masks, done checks and the map-observation encode.
//   cgrid [N] x 2304 B    compact 48x48 hex-code grid of the final map in observation cell order
//                         (the lookup table of movement masks / done checks, and the source of
//                         the map-observation encode)
//   gen   [N] x 256 B     map-generation scratch (pieces list, per-env piece transforms)
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/cog_types.h"

namespace cog {

constexpr int kGridDim = 128;
constexpr int kGridOff = 64;
constexpr int kGridBytes = kGridDim * kGridDim;
#define COG_CELLS 2304                // 48 * 48
constexpr int kMaxCoord = 62;        // |x|,|y| of any placed hex; beyond -> hazard GRID_OVER
constexpr int kMaxPlaced = 96;       // pieces placed in one generation (incl. recursion)

// hazard / status flags (same bit meaning as the oracle's ORC_F_*)
constexpr uint32_t F_MAPGEN_FAIL = 0x01u;
constexpr uint32_t F_ERASE_PAST = 0x02u;
constexpr uint32_t F_Q9_OOB = 0x04u;
constexpr uint32_t F_Q24_CLAMP = 0x08u;
constexpr uint32_t F_GRID_OVER = 0x10u;
constexpr uint32_t F_OOB_LOOKUP = 0x20u;
constexpr uint32_t F_SCAN_OVER = 0x40u;
constexpr uint32_t F_B_START_LT4 = 0x80u;
constexpr uint32_t F_BAD_ACTION = 0x100u;
constexpr uint32_t F_SYNC_TIMEOUT = 0x200u;  // (device status only) a trio wave's progress wait timed out
constexpr uint32_t F_PARK_NOFIX = 0x400u;    // (device status only) an env parked in a launch without a fix-up
constexpr uint32_t F_ERROR_MASK = F_MAPGEN_FAIL | F_GRID_OVER;

struct PlayerPriv {                  // Player + Deck private members (player.h:60-75, cards.h:137-145)
  uint8_t has_won, mip, n_removes, next_card_free;
  uint8_t next_move_free, n_in_hand, n_active, n_in_draw;
  uint8_t idx_last, steps_taken, n_added_cards, pad;
  uint32_t n_movements;
};

struct EnvPriv {                    // cog_env private members (environment.h:12-33) + Map/Shop state
                                     // (4-byte aligned: also lives in LDS step slots)
  uint32_t rng;                      // env minstd_rand0 state
  uint32_t seed;
  uint32_t max_steps;
  uint32_t turn_counter;
  uint8_t n_players, n_pieces, difficulty, done;
  uint8_t agent, n_in_market, loc_size, render;
  uint32_t in_market;                // Shop::in_market bits
  uint32_t flags;                    // sticky hazard flags
  int8_t minx, miny, maxx, maxy;     // Map::min_xy / max_xy (integer hex coords)
  uint8_t dimx, dimy, pad0, pad1b;
  int8_t locx[4], locy[4];           // Map::player_locations
  uint8_t info_steps[4];             // mirror of Info.agent_infos[p].steps_taken (never read back)
  uint32_t pad1[3];
  PlayerPriv pl[4];
  uint8_t cells[4][8];               // per player: hex codes of its cell [0] and neighbours [1..6]
                                     // as Map::get_from_array returns them, [7] = out-of-map bits
};
static_assert(sizeof(EnvPriv) == 160, "EnvPriv is ten 16-B granules");

struct alignas(64) GenScratch {
  uint8_t pieces[kMaxPlaced];
  int16_t pcx[20], pcy[20];          // piece centres (doubled coords)
  uint8_t prot[20];                  // piece rotations mod 6
  uint8_t npieces, pad[11];
};
static_assert(sizeof(GenScratch) <= 256, "GenScratch");

struct DevState {
  size_t n;
  uint8_t *obs;
  uint8_t *sel;
  uint8_t *info;
  float *rew;
  uint8_t *done;
  uint8_t *agent;
  EnvPriv *priv;
  uint8_t *grid;
  uint8_t *cgrid;                    // [n] x 2304 B compact 48x48 hex codes (lookups + encode)
  uint4 *heads;                      // [n][5] mask bit-vectors: selected, stored of players 0..3
  // the trio drawing wave's compact deck image as of the end of the last trio launch (+ its
  // fix-up): [n][10] granules = players 0..3 x the five DeckObs piles of types 0-7 (8 B each,
  // deck_expand / compact_of), and [n] a word that is 1 when an env's deck held a type >= 8 (not
  // representable: that env parks at step 0).  cdeck_ok (the host's EnvShard::cdeck_ok): no launch
  // since wrote a deck without writing them, so a trio launch loads these 164 B instead of the
  // four 112-B DeckObs records (about a third of its prologue's HBM bytes at the line granularity)
  uint4 *cdeck;
  uint32_t *cwide;
  GenScratch *gen;
  uint32_t *status;                  // [0] OR of error flags, [1] error count, [2] dirty count
  uint32_t *dirty;                   // [cap] local indices of envs whose map was re-generated
  uint32_t *err;                     // host-mapped word (pinned): set to 1 on any error, so a sync
                                     // learns "no error" without a device-to-host copy
  size_t first;                      // global index of env 0 of this shard (seeds are seed + global index)
  size_t cap;                        // capacity of the dirty list; 0: no list (outputs stay on the device)
  uint32_t autoreset;                // 1: vec_cog_env (reset a finished env in the same call,
                                     // vec_environment.h:56-59); 0: cog_env (stays done)
  unsigned long long *stamps;        // diagnostic builds (COG_STAMPS) only: per-wave phase clocks
  uint32_t *park;                    // [n] rollout park codes: the step at which an env's episode
                                     // ended inside a launch (~0u: none), read by the fix-up kernel
  // the parked workgroups of a duo / trio launch, for k_env_fixup: [0], [1] two counters used by
  // alternate launches (park_par, the host's count of such launches mod 2: a launch appends to
  // counter park_par and zeroes the other one, which the previous launch's fix-up has read), then
  // the list of workgroup indices with a parked env (park_list_bytes(n))
  uint32_t *parkq;
  uint32_t park_par;
  uint32_t no_fixup;                 // 1: no k_env_fixup follows this launch (a park is an error)
  uint32_t trio_jt;                  // 1: the trio launch of at most one workgroup per CU (its LAT form)
  uint32_t cdeck_ok;                 // 1: cdeck / cwide hold every env's decks (see above)
  // direct publish (launch_step_pub only; null otherwise): device addresses of the shard's pinned
  // ObsData view and outs block, and the publish mirror (k_publish's `mir`)
  uint8_t *pub_obs, *pub_outs, *pub_mir;
  // test hooks (launch_rollout): the trio parks every env (redo_env -1: $COG_DEBUG_REDO_STEP) or
  // the env of local index redo_env ($COG_DEBUG_PARK_NOFIX=t:i, with no_fixup kept) at step
  // redo_at of each launch as if its action left the lean step (kParkRedo), so the tests exercise
  // the fix-up's redo path and the no-fix-up guard (F_PARK_NOFIX); redo_at -1 (default): off
  int32_t redo_at;
  int32_t redo_env;
};

struct ResetParams {
  uint32_t seed;
  uint8_t n_players, n_pieces, difficulty, use_params;   // use_params=0: cog_env::reset()
  uint32_t max_steps;
};

enum MaskSource : int { MASK_SELECTED = 0, MASK_STORED = 1, MASK_EXTERNAL = 2 };

// host-side launchers (stream = hipStream_t passed as void*)
int launch_init(const DevState &s, const uint32_t *seeds_host_unused, uint32_t default_seed,
                void *stream);
int launch_reset(const DevState &s, const ResetParams &p, void *stream);
int launch_encode_all(const DevState &s, void *stream, int variant = 0);
// the mask bit vectors and the Info steps mirror rebuilt from the device records (k_resync)
int launch_resync(const DevState &s, void *stream);
int launch_step(const DevState &s, const uint8_t *d_actions, void *stream);
// a host-visible step whose pinned views equal the records in HBM (after a publish, no device-only
// work since): every changed granule of a host-visible record is stored into the view and the
// publish mirror by the step itself (s.pub_* set), envs whose episode ended are published by
// comparison, and the last workgroup copies the status granules and stores the completion word
// (sig_ctr: a zeroed device counter).  Returns -1 when the batch is too large for it
// (step_pub_ok).
// The speculative next sample of a host step (launch_step_pub): env.step(actions) whose actions
// are a sampler's view samples that sampler's next actions from the step's new selected masks into
// spare buffers, so that the sampler's next sample of the env's own masks is a host copy
// (cog_abi.cpp SamplerSpec).  rng_in null: none.
struct SampleSpec {
  const uint32_t *rng_in;            // the sampler's state
  uint32_t *rng_out;                 // its state after the speculative sample
  uint8_t *act_dev;                  // ActionData records (device)
  uint8_t *act_host;                 // 8 B per env: device address of pinned staging
  uint32_t *invalid;                 // device address of a pinned word: 1 when an env's episode ended
};
int launch_step_pub(const DevState &s, const uint8_t *d_actions, void *stream, uint32_t *sig_ctr, uint32_t *sig_word,
                    uint32_t seq, const SampleSpec *spec = nullptr);
bool step_pub_ok(size_t n);
// the runner's fused sample + step in the same form; the sampled actions also go to the sampler's
// pinned view (h_actions, device address)
int launch_sample_step_pub(const DevState &s, int mask_source, uint32_t *d_rng, uint8_t *d_actions, uint8_t *h_actions,
                           void *stream, uint32_t *sig_ctr, uint32_t *sig_word, uint32_t seq);
// h_actions: device-mapped host view (or null); sig_ctr (or null), sig_word, seq: the in-kernel
// completion word (the last workgroup stores seq into *sig_word; sig_ctr a zeroed device counter)
int launch_sample(size_t n, const uint8_t *d_masks, uint32_t *d_rng, uint8_t *d_actions,
                  void *stream, uint8_t *h_actions = nullptr, uint32_t *sig_ctr = nullptr,
                  uint32_t *sig_word = nullptr, uint32_t seq = 0);
// the host views' dynamic records from HBM: granules that differ from `mir` (an HBM copy of the
// host views) are stored into the device-mapped pinned views h_obs / h_outs (and into mir);
// outs_bytes a multiple of 16; force = 1 stores every granule; d_actions / h_actions optional
int launch_publish(const DevState &s, const uint8_t *outs, uint8_t *mir, uint8_t *h_obs, uint8_t *h_outs,
                   size_t outs_bytes, int force, const uint8_t *d_actions, uint8_t *h_actions, void *stream,
                   uint32_t *sig_ctr = nullptr, uint32_t *sig_word = nullptr, uint32_t seq = 0);
size_t publish_mirror_bytes(size_t n, size_t outs_bytes);
// whether launch_publish may store a completion word itself (its grid is small enough)
bool publish_can_signal(size_t n, size_t outs_bytes, bool actions);
int launch_sample_step(const DevState &s, int mask_source, uint32_t *d_rng, uint8_t *d_actions,
                       void *stream);
// persistent K-step runner loop; defer_ok: every env of the shard has >= 3 players (the trio
// rollout's deferred turn end then runs the selected-mask loop at every shard size)
// park_seq: the shard's count of launches with a fix-up (counts them; alternate launches use
// alternate counters of DevState::parkq)
// no_fixup: the caller has shown that no env can park in this launch (cog_abi.cpp EnvShard::
// lean_clock): the trio launches alone, and a park it meets all the same is an error (F_PARK_NOFIX)
int launch_rollout(const DevState &s, int mask_source, int steps, uint32_t *d_rng, uint8_t *d_actions,
                   void *stream, bool defer_ok, uint32_t *park_seq, bool no_fixup = false);
inline size_t park_list_bytes(size_t n) { return (2 + (n + 31) / 32) * sizeof(uint32_t); }
int rollout_kind_of(size_t n, int mask_source, bool defer_ok);   // 0 duo, 1 wave, 2 pipe, 3 trio
int trio_epw(size_t n);                                          // envs per trio workgroup (32 or 64)
int launch_seed_sampler(size_t n, uint64_t seed, size_t first, uint32_t *d_rng, void *stream);
// completion word: stores seq into *d_word (device address of a pinned host word) once every
// earlier packet of the stream has completed
int launch_signal(uint32_t *d_word, uint32_t seq, void *stream);
// variant bit 0: non-temporal loads/stores; bit 4: one granule per work-item (bits 1-3 ignored);
// bit 1: 32 waves per CU instead of 8 (grid stride);
// bit 2: one pass, 32 KiB per workgroup (bit 1 ignored); bit 3: the encode's 1:7 read:write mix
// (reads `bytes`, writes 7 x `bytes` into dst; bit 0 = non-temporal stores); bytes: a multiple of 16
int launch_copy_peak(const void *src, void *dst, size_t bytes, void *stream, int variant);

}  // namespace cog
