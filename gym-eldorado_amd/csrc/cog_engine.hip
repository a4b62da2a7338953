// cog_engine.hip -- CDNA4 (gfx950) kernels of the batched City-of-Gold engine.
//
// One work-item owns one environment for the whole step (the per-env work is a short,
// branchy integer state machine over ~1 KB of state; there is no GEMM and no MFMA use).
// State lives in HBM in the layout documented in cog_engine.h: the reference's own ObsData /
// ActionMask / Info records (so host and device views are the engine state, no write-back
// pass) plus one 128-B private line per env and a 128x128 hex-code grid per env.
//
// Semantics follow the reference line by line (citations per function); the representation
// does not: hex geometry is exact integer arithmetic on a doubled lattice
// (rot+1: (x, y) -> (-y, x + y), the exact value of geometry.cpp:3-17 + map.cpp:17-37 on this
// lattice) and overlap tests use the occupancy grid instead of sort+merge (map.cpp:53-74).
//
// Kernels:
//   k_init           default-construct N envs (vec_environment.h:23-30)
//   k_reset          cog_env::reset(params) incl. procedural map generation (map.cpp:697-742)
//   k_encode         48x48x7 map-observation encode (map.cpp:389-405): streaming, 16 cells / item
//   k_sample         masked uniform sampler (sampler.h:14-79)
//   k_env_step<SRC>  vec_cog_env::step with auto-reset (vec_environment.h:46-61); SRC: host
//                    actions, or the runner-fused sample(selected | stored masks) + step
//                    (runner.h:46-55)
//   k_sync_heads     mask bit-vectors of every env from its byte records (init / reset)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "cog_engine.h"
#include "cog_tables.h"
#include "cog_rng.h"

#define DEV __device__ __forceinline__

// Diagnostic phase clocks (tools/stamp_step.cpp builds with -DCOG_STAMPS; never in the library)
#ifdef COG_STAMPS
DEV unsigned long long stamp_clock() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define STAMP(s, k)                                                                          \
  do {                                                                                       \
    const unsigned long long t_ = stamp_clock();                                             \
    if ((s).stamps && (threadIdx.x & 63) == 0)                                               \
      (s).stamps[((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 16 + (k)] = t_; \
  } while (0)
#else
#define STAMP(s, k) do { } while (0)
#endif
#define STAMP_AT(k) STAMP(e, k)     // inside step functions: Ctx carries the stamp buffer
// per-phase tick accumulators (diagnostic builds): PH(k) charges the ticks since the previous
// PH to phase k; PH_FLUSH writes this wave's totals to the stamp buffer.  step_regs takes the
// accumulator as an extra parameter (PH_PARAM / PH_PASS) in those builds only.
#ifdef COG_STAMPS
struct PhAcc {
  unsigned long long acc[16];
  unsigned long long last;
};
#define PH_DECL PhAcc ph_ = {}; ph_.last = stamp_clock()
#define PH(k) do { const unsigned long long t_ = stamp_clock(); ph_.acc[k] += t_ - ph_.last; ph_.last = t_; } while (0)
#define PH_PARAM , PhAcc &ph_
#define PH_PASS , ph_
// TL(k): slot k holds the chip-wide 100 MHz clock at this point (the launch timeline)
#define TL(k) do { ph_.acc[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define PH_RESET do { ph_.last = stamp_clock(); } while (0)
#define PH_FLUSH(s)                                                                         \
  do {                                                                                      \
    if ((s).stamps && (threadIdx.x & 63) == 0)                                              \
      for (int k_ = 0; k_ < 16; k_++)                                                       \
        (s).stamps[((size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 16 + k_] = ph_.acc[k_]; \
  } while (0)
#else
#define PH_DECL do { } while (0)
#define PH(k) do { } while (0)
#define PH_PARAM
#define PH_PASS
#define PH_FLUSH(s) do { } while (0)
#define TL(k) do { } while (0)
#define PH_RESET do { } while (0)
#endif

namespace cog {

__constant__ cog_card_t c_cards[COG_N_CARDTYPES] = COG_CARD_TABLE;
__constant__ uint8_t c_shop_types[COG_N_SHOP] = COG_SHOP_TYPES;
__constant__ cog_piece_meta_t c_pmeta[COG_N_PIECES] = COG_PIECE_META;
__constant__ uint8_t c_phex[COG_N_PIECES][37] = COG_PIECE_HEX;
__constant__ int8_t c_large[37][2] = COG_LARGE_XY2;
__constant__ int8_t c_small[16][2] = COG_SMALL_XY2;
__constant__ int8_t c_end[3][2] = COG_END_XY2;
__constant__ int8_t c_dirs[7][2] = COG_DIRS_XY2;
__constant__ int8_t c_conn_ll[2][2] = COG_CONN_LL_XY2;
__constant__ int8_t c_conn_ls[3][2] = COG_CONN_LS_XY2;
__constant__ int8_t c_conn_lt[1][2] = COG_CONN_LT_XY2;
__constant__ int8_t c_conn_sl[6][2] = COG_CONN_SL_XY2;
__constant__ int8_t c_opts_range[6] = {-2, -1, 0, 1, 2, 3};
__constant__ int8_t c_opts_ls[2] = {-1, 2};
__constant__ int8_t c_opts_lt[1] = {-3};

// the uniform's division table (cog_rng.h uid_entry): constant memory, copied to LDS by each
// kernel that draws (a per-lane k indexes it)
struct UidTab {
  UidEntry e[kUidTab];
};
constexpr UidTab make_uid_tab() {
  UidTab t{};
  for (int k = 0; k < kUidTab; k++) t.e[k] = uid_entry((uint32_t)k);
  return t;
}
__constant__ UidTab c_uid_tab = make_uid_tab();
DEV void uid_tab_fill(UidEntry *lds) {                    // the first 32 work-items; then a barrier
  if (threadIdx.x < (unsigned)kUidTab) lds[threadIdx.x] = c_uid_tab.e[threadIdx.x];
  __syncthreads();
}
DEV uint32_t uid_tab(const UidEntry *tab, uint32_t r, uint32_t k) {   // k in [1, 31], r accepted
  const UidEntry e = tab[k];
  return uid_tab_accepted(r, e.s, e.m);
}

// shop slots that start in the market (cards.cpp:85-92 / 94-100): slots 0,1,5,7,9,12
constexpr uint32_t kInMarket0 = (1u << 0) | (1u << 1) | (1u << 5) | (1u << 7) | (1u << 9) | (1u << 12);

// RNG (minstd_rand0 + libstdc++ uniform_int_distribution): cog_rng.h

// ------------------------------------------------------------------------------------------
// per-env context
// ------------------------------------------------------------------------------------------
struct Ctx {
  unsigned long long *stamps;   // diagnostic builds only (STAMP_AT)
  uint8_t *ob;        // ObsData record (global): map, decks / stored masks of other players
  uint8_t *sh;        // shared block = ObsData bytes 16128..16175 (phase @0, resources @4, shop @16)
  uint8_t *dka;       // DeckObs of player a0 (staged copy in LDS, or global)
  uint8_t *sta;       // stored ActionMask of player a0 (staged copy in LDS, or global)
  int a0;             // player whose deck / stored mask dka / sta point at (-1: none)
  uint8_t *sel;       // selected ActionMask
  uint8_t *info;      // Info record
  float *rew;         // rewards[4]
  EnvPriv *pv;        // private state
  uint8_t *grid;      // 128x128 absolute hex codes (map-generation scratch)
  uint8_t *cgrid;     // 48x48 compact hex codes of the final map
  GenScratch *gs;
};

// all-global context (reset / init paths)
DEV Ctx make_ctx(const DevState &s, size_t i) {
  Ctx e;
  e.ob = s.obs + i * COG_OBS_BYTES;
  e.sh = e.ob + COG_OBS_PHASE;
  e.dka = nullptr;
  e.sta = nullptr;
  e.a0 = -1;
  e.sel = s.sel + i * COG_MASK_BYTES;
  e.info = s.info + i * COG_INFO_BYTES;
  e.rew = s.rew + i * 4;
  e.pv = s.priv + i;
  e.grid = s.grid + i * (size_t)kGridBytes;
  e.cgrid = s.cgrid + i * COG_CELLS;
  e.gs = s.gen + i;
  e.stamps = nullptr;
  return e;
}

DEV void build_cgrid(const Ctx &e);

DEV uint8_t *deck(const Ctx &e, int p) {
  return p == e.a0 ? e.dka : e.ob + COG_OBS_PLAYER0 + COG_OBS_PLAYER_STRIDE * p;
}
DEV uint8_t *stm(const Ctx &e, int p) {
  return p == e.a0 ? e.sta : e.ob + COG_OBS_PLAYER0 + COG_OBS_PLAYER_STRIDE * p + COG_PD_MASK;
}
constexpr int SH_RES = COG_OBS_RES - COG_OBS_PHASE;    // 4
constexpr int SH_SHOP = COG_OBS_SHOP - COG_OBS_PHASE;  // 16
DEV float *res(const Ctx &e) { return reinterpret_cast<float *>(e.sh + SH_RES); }
DEV bool is_special(int c) { return c >= 15 && c <= 20; }

DEV uint8_t grid_at(const uint8_t *g, int x, int y) { return g[(x + kGridOff) * kGridDim + (y + kGridOff)]; }

// Map::get_from_array (map.cpp:273-275) on absolute integer coords
DEV uint8_t lookup(const Ctx &e, int x, int y) {
  EnvPriv *pv = e.pv;
  const int ix = x - pv->minx + 1, iy = y - pv->miny + 1;
  if (ix < 0 || iy < 0 || ix >= pv->dimx || iy >= pv->dimy) {
    pv->flags |= F_OOB_LOOKUP;
    return COG_HEX_MOUNTAIN;
  }
  if (ix >= COG_GRID || iy >= COG_GRID) return COG_HEX_MOUNTAIN;   // ring cell of a 49-wide map
  const uint8_t c = e.cgrid[ix * COG_GRID + iy];
  return c ? c : (uint8_t)COG_HEX_MOUNTAIN;
}

// the neighbourhood cache of one player (EnvPriv::cells): the codes lookup() returns for its
// cell and its six neighbours, and which of those seven lookups fall outside the map (the
// OOB_LOOKUP flag is raised when a cached cell is USED, as the reference's lookups would be)
DEV void load_cells(const Ctx &e, int player) {
  const EnvPriv *pv = e.pv;
  uint8_t *out = e.pv->cells[player];
  const int lx = pv->locx[player], ly = pv->locy[player];
  uint32_t oob = 0;
#pragma unroll
  for (int d = 0; d < 7; d++) {
    const int ix = lx + c_dirs[d][0] / 2 - pv->minx + 1, iy = ly + c_dirs[d][1] / 2 - pv->miny + 1;
    const bool out_ = ix < 0 || iy < 0 || ix >= pv->dimx || iy >= pv->dimy;
    const bool ring = ix >= COG_GRID || iy >= COG_GRID;
    const int cx = min(max(ix, 0), COG_GRID - 1), cy = min(max(iy, 0), COG_GRID - 1);
    const uint8_t v = e.cgrid[cx * COG_GRID + cy];
    out[d] = (out_ || ring || !v) ? (uint8_t)COG_HEX_MOUNTAIN : v;
    oob |= (out_ ? 1u : 0u) << d;
  }
  out[7] = (uint8_t)oob;
}

// ------------------------------------------------------------------------------------------
// Deck / Player / Shop (cards.cpp:94-294, player.cpp:29-206)
// ------------------------------------------------------------------------------------------
DEV int scan(const Ctx &e, const uint8_t *d, int base, uint32_t t) {
  int c = 0;
  while (t >= d[base + c]) {
    t -= d[base + c];
    ++c;
    if (base + c >= 105) {
      e.pv->flags |= F_SCAN_OVER;
      return c;
    }
  }
  return c;
}

DEV void move_discard_to_draw(const Ctx &e, int p) {      // cards.cpp:234-240
  uint8_t *d = deck(e, p);
  PlayerPriv &P = e.pv->pl[p];
  uint8_t nd = P.n_in_draw;
  for (int i = 0; i < COG_N_CARDTYPES; i++) {
    const uint8_t x = d[COG_DECK_DISCARD + i];
    d[COG_DECK_DRAW + i] = (uint8_t)(d[COG_DECK_DRAW + i] + x);
    nd = (uint8_t)(nd + x);
    d[COG_DECK_DISCARD + i] = 0;
  }
  P.n_in_draw = nd;
}

DEV void deck_draw(const Ctx &e, int p, uint8_t n) {        // cards.cpp:183-211
  PlayerPriv &P = e.pv->pl[p];
  uint8_t *d = deck(e, p);
  if (P.n_in_draw < n) move_discard_to_draw(e, p);
  if (n > P.n_in_draw) n = P.n_in_draw;
  uint32_t rng = e.pv->rng;
  for (int i = 0; i < n; i++) {
    const uint32_t t = uid(rng, P.n_in_draw);
    const int c = scan(e, d, COG_DECK_DRAW, t);
    d[COG_DECK_DRAW + c]--;
    P.n_in_draw--;
    d[COG_DECK_HAND + c]++;
    e.sel[COG_MASK_PLAY + 1 + c] = 1;
    e.sel[COG_MASK_SPECIAL + 1 + c] = is_special(c);
  }
  e.pv->rng = rng;
  P.n_in_hand = (uint8_t)(P.n_in_hand + n);
}

DEV void copy_mask(uint8_t *dst, const uint8_t *src) {     // ActionMask copy (named fields)
  const uint32_t *s = reinterpret_cast<const uint32_t *>(src);   // 4-byte aligned (LDS slots)
  uint32_t *d = reinterpret_cast<uint32_t *>(dst);
#pragma unroll
  for (int k = 0; k < 23; k++) d[k] = s[k];                // bytes 0..91: the named fields
}

DEV void shop_mask(const Ctx &e, float coins, uint8_t *mask) {  // cards.cpp:109-121
  const uint8_t *avail = e.sh + SH_SHOP;
  const uint32_t im = e.pv->in_market;
  const bool few = e.pv->n_in_market < COG_MKT_SLOTS;
  for (int i = 0; i < COG_N_SHOP; i++) {
    const float cost = (float)c_cards[c_shop_types[i]].cost;
    const bool ok = few ? avail[i] > 0 : ((im >> i) & 1u);
    mask[i + 1] = ok && (coins > cost);
  }
}

DEV void movement_mask(const Ctx &e, uint8_t *move, int player, const float *r, uint8_t n_active) {
  // map.cpp:369-387
  const int lx = e.pv->locx[player], ly = e.pv->locy[player];
#pragma unroll
  for (int i = 1; i < 7; i++) {
    const uint8_t c = lookup(e, lx + c_dirs[i][0] / 2, ly + c_dirs[i][1] / 2);
    const int req = COG_HEX_REQ(c);
    bool filled;
    if (req >= COG_REQ_DISCARD) filled = n_active > COG_HEX_N(c);
    else filled = r[req] >= (float)COG_HEX_N(c);
    move[i] = (req != COG_REQ_NULL) && filled;
  }
}

DEV void update_observation(const Ctx &e, int agent) {     // environment.cpp:252-279
  uint8_t *am = stm(e, agent);
  am[COG_MASK_MOVE] = 1;
  for (int k = 1; k < 7; k++) am[COG_MASK_MOVE + k] = 0;
  am[COG_MASK_SHOP] = 1;
  for (int k = 1; k < 19; k++) am[COG_MASK_SHOP + k] = 0;
  const uint8_t ph = e.sh[0];
  if (ph == COG_PHASE_MOVEMENT) {
    float r[3] = {res(e)[0], res(e)[1], res(e)[2]};
    movement_mask(e, am + COG_MASK_MOVE, agent, r, e.pv->pl[agent].n_active);
  } else if (ph == COG_PHASE_BUYING) {
    shop_mask(e, res(e)[2], am + COG_MASK_SHOP);
  }
}

DEV void player_reset(const Ctx &e, int p) {               // player.cpp:29-43
  PlayerPriv &P = e.pv->pl[p];
  uint8_t *d = deck(e, p);
  P.has_won = 0; P.mip = 0; P.next_card_free = 0; P.next_move_free = 0;
  P.n_removes = 0; P.steps_taken = 0; P.n_movements = 0; P.n_added_cards = 0;
  for (int k = 0; k < COG_N_CARDTYPES; k++) {              // DeckObs::reset keeps `played` (Q10)
    d[COG_DECK_DRAW + k] = 0; d[COG_DECK_HAND + k] = 0;
    d[COG_DECK_ACTIVE + k] = 0; d[COG_DECK_DISCARD + k] = 0;
  }
  for (int k = 0; k < 22; k++) {                           // ActionMask::reset (api.h:104-118)
    e.sel[COG_MASK_PLAY + k] = k == 0;
    e.sel[COG_MASK_REMOVE + k] = k == 0;
    e.sel[COG_MASK_SPECIAL + k] = k == 0;
  }
  e.sel[COG_MASK_MOVE] = 1;
  e.sel[COG_MASK_SHOP] = 1;
  d[COG_DECK_DISCARD + 0] = 3;                             // Deck::reset (cards.cpp:163-171)
  d[COG_DECK_DISCARD + 7] = 4;
  d[COG_DECK_DISCARD + 5] = 1;
  P.n_in_draw = 0; P.n_in_hand = 0; P.n_active = 0;
  deck_draw(e, p, COG_HAND_SIZE);
  copy_mask(stm(e, p), e.sel);
}

// ------------------------------------------------------------------------------------------
// Procedural map generation (map.cpp:17-74, 154-341, 697-752) on the doubled integer lattice
// ------------------------------------------------------------------------------------------
DEV void rot_pt(int t, int X, int Y, int &ox, int &oy) {   // rotate by t*60 degrees, t in [0,6)
  switch (t) {
    case 0: ox = X; oy = Y; break;
    case 1: ox = -Y; oy = X + Y; break;
    case 2: ox = -X - Y; oy = X; break;
    case 3: ox = -X; oy = -Y; break;
    case 4: ox = Y; oy = -X - Y; break;
    default: ox = X + Y; oy = -X; break;
  }
}
DEV int norm6(int t) {
  t %= 6;
  return t < 0 ? t + 6 : t;
}
DEV void piece_xy2(int piece, int k, int &X, int &Y) {
  const int sz = c_pmeta[piece].size;
  if (sz == COG_PS_LARGE) { X = c_large[k][0]; Y = c_large[k][1]; }
  else if (sz == COG_PS_SMALL) { X = c_small[k][0]; Y = c_small[k][1]; }
  else { X = c_end[k][0]; Y = c_end[k][1]; }
}

DEV void map_reset(const Ctx &e) {                         // map.cpp:744-752
  EnvPriv *pv = e.pv;
  for (int x = pv->minx; x <= pv->maxx; x++)
    for (int y = pv->miny; y <= pv->maxy; y++) e.grid[(x + kGridOff) * kGridDim + (y + kGridOff)] = 0;
  pv->minx = pv->miny = pv->maxx = pv->maxy = 0;
  pv->dimx = pv->dimy = 0;
  e.gs->npieces = 0;
}

// MapPiece::rotate + translate, then Map::add_piece bookkeeping (map.cpp:179-191, 309-341)
DEV bool add_piece(const Ctx &e, int p, int cx2, int cy2, int rot) {
  GenScratch *gs = e.gs;
  EnvPriv *pv = e.pv;
  const int r = norm6(gs->prot[p] + rot);
  gs->prot[p] = (uint8_t)r;
  const int pcx = gs->pcx[p] + cx2, pcy = gs->pcy[p] + cy2;
  gs->pcx[p] = (int16_t)pcx;
  gs->pcy[p] = (int16_t)pcy;
  if (gs->npieces >= kMaxPlaced) {
    pv->flags |= F_GRID_OVER;
    return false;
  }
  gs->pieces[gs->npieces++] = (uint8_t)p;
  int mnx = pv->minx, mny = pv->miny, mxx = pv->maxx, mxy = pv->maxy;
  const int nh = c_pmeta[p].n_hex;
  for (int k = 0; k < nh; k++) {
    int X, Y, rx, ry;
    piece_xy2(p, k, X, Y);
    rot_pt(r, X, Y, rx, ry);
    rx += pcx;
    ry += pcy;
    if ((rx | ry) & 1) {                                   // never on valid lattices
      pv->flags |= F_GRID_OVER;
      return false;
    }
    const int x = rx / 2, y = ry / 2;
    if (x < -kMaxCoord || x > kMaxCoord || y < -kMaxCoord || y > kMaxCoord) {
      pv->flags |= F_GRID_OVER;
      return false;
    }
    e.grid[(x + kGridOff) * kGridDim + (y + kGridOff)] = c_phex[p][k];
    mxx = max(mxx, x); mxy = max(mxy, y);
    mnx = min(mnx, x); mny = min(mny, y);
  }
  pv->minx = (int8_t)mnx; pv->miny = (int8_t)mny;
  pv->maxx = (int8_t)mxx; pv->maxy = (int8_t)mxy;
  return true;
}

// footprint of piece p (reset state) rotated by t and centred at (cx2, cy2) hits no placed hex?
DEV bool footprint_free(const Ctx &e, int p, int t, int cx2, int cy2) {
  const int nh = c_pmeta[p].n_hex;
  for (int k = 0; k < nh; k++) {
    int X, Y, rx, ry;
    piece_xy2(p, k, X, Y);
    rot_pt(t, X, Y, rx, ry);
    rx += cx2;
    ry += cy2;
    if ((rx | ry) & 1) continue;                           // off-lattice point: cannot coincide
    const int x = rx / 2, y = ry / 2;
    if (x < -kGridOff || x >= kGridOff || y < -kGridOff || y >= kGridOff) continue;
    if (grid_at(e.grid, x, y)) return false;
  }
  return true;
}

struct ConnSet {
  const int8_t (*base)[2];
  const int8_t *opts;
  int nbase, nopt, copies;
};

// MapPiece::get_ref_connection_points (map.cpp:203-263): what placed piece q offers to `psize`
DEV bool conn_set(int q, int psize, ConnSet &cs) {
  const int qs = c_pmeta[q].size, qk = c_pmeta[q].kind;
  if (qs == COG_PS_LARGE) {
    if (psize == COG_PS_LARGE) { cs.base = c_conn_ll; cs.nbase = 2; cs.opts = c_opts_range; cs.nopt = 6; cs.copies = 7; return true; }
    if (psize == COG_PS_SMALL) { cs.base = c_conn_ls; cs.nbase = 3; cs.opts = c_opts_ls; cs.nopt = 2; cs.copies = 7; return true; }
    if (psize == COG_PS_TRIPLE && qk != COG_PT_START) { cs.base = c_conn_lt; cs.nbase = 1; cs.opts = c_opts_lt; cs.nopt = 1; cs.copies = 7; return true; }
    return false;
  }
  if (qs == COG_PS_SMALL && psize == COG_PS_LARGE) {
    cs.base = c_conn_sl; cs.nbase = 6; cs.opts = c_opts_range; cs.nopt = 6; cs.copies = 1;
    return true;
  }
  return false;
}

// Map::add_random_piece (map.cpp:277-307): two passes over the candidate list instead of
// materialising it (count the valid ones, draw, find the chosen one again)
DEV bool add_random_piece(const Ctx &e, int p, uint32_t &rng) {
  GenScratch *gs = e.gs;
  gs->pcx[p] = 0; gs->pcy[p] = 0; gs->prot[p] = 0;         // MapPiece::reset
  const int psize = c_pmeta[p].size;
  const int npl = gs->npieces;
  uint32_t chosen = 0xffffffffu;
  uint32_t nvalid = 0;
  for (int pass = 0; pass < 2; pass++) {
    uint32_t count = 0;
    for (int qi = 0; qi < npl; qi++) {
      const int q = gs->pieces[qi];
      ConnSet cs;
      if (!conn_set(q, psize, cs)) continue;
      const int qcx = gs->pcx[q], qcy = gs->pcy[q], qrot = gs->prot[q];
      for (int ci = 0; ci < cs.copies; ci++) {
        for (int j = 0; j < cs.nbase; j++) {
          int cx, cy;
          rot_pt(norm6(ci + qrot), cs.base[j][0], cs.base[j][1], cx, cy);
          cx += qcx;
          cy += qcy;
          const int opt0 = cs.opts[0] + ci + qrot;
          if (!footprint_free(e, p, norm6(opt0), cx, cy)) continue;
          if (pass == 1 && count == chosen) {
            const uint32_t ri = uid(rng, (uint32_t)cs.nopt);
            const int rot = cs.opts[ri] + ci + qrot;
            return add_piece(e, p, cx, cy, rot);
          }
          count++;
        }
      }
    }
    if (pass == 0) {
      nvalid = count;
      if (!nvalid) return false;
      chosen = uid(rng, nvalid);
    }
  }
  return false;  // unreachable
}

DEV bool finalize_ok(const Ctx &e) {                       // map.cpp:389-405 (dims check, Q27)
  EnvPriv *pv = e.pv;
  const int dx = 3 + pv->maxx - pv->minx, dy = 3 + pv->maxy - pv->miny;
  if (dx > 49 || dy > 49) {
    pv->flags |= F_GRID_OVER;
    return false;
  }
  pv->dimx = (uint8_t)dx;
  pv->dimy = (uint8_t)dy;
  return true;
}

struct GenFrame {
  uint32_t rng;
  uint8_t i, nvalid, stage, pad;
  uint8_t valid[16];
};

// Map::generate (map.cpp:697-742) as an explicit-stack state machine.  A frame's rng is its own
// copy (the reference passes the engine by value), recursion depth == failures.
DEV bool generate(const Ctx &e) {
  enum { ENTER = 0, LOOP = 1, END = 2, FIN = 3 };
  EnvPriv *pv = e.pv;
  GenFrame fr[COG_MAX_FAILURES];
  int depth = 0;
  fr[0].rng = pv->rng;
  fr[0].stage = ENTER;
  const int n_pieces = pv->n_pieces, diff = pv->difficulty;
  while (depth >= 0) {
    GenFrame &F = fr[depth];
    if (F.stage == ENTER) {
      const uint32_t s = uid(F.rng, 2);
      if (!add_piece(e, COG_PIECE_START0 + (int)s, 0, 0, 0)) return false;
      F.nvalid = 0;
      for (int i = 0; i < COG_N_TRAVEL; i++)
        if (c_pmeta[COG_PIECE_TRAVEL0 + i].difficulty <= diff) F.valid[F.nvalid++] = (uint8_t)i;
      F.i = 0;
      F.stage = LOOP;
    } else if (F.stage == LOOP) {
      if (F.i < n_pieces) {
        bool ok = false;
        int next = 0;
        if (F.nvalid) {
          next = F.valid[uid(F.rng, F.nvalid)];
          ok = add_random_piece(e, COG_PIECE_TRAVEL0 + next, F.rng);
          if (pv->flags & F_GRID_OVER) return false;
        }
        F.i++;
        if (ok) {
          // vector::erase(begin() + next) with GCC>=13 libstdc++ semantics (Q5)
          const int num = (int)F.nvalid - (next + 1);
          for (int k = 0; k < num; k++) F.valid[next + k] = F.valid[next + 1 + k];
          if (next >= F.nvalid) pv->flags |= F_ERASE_PAST;
          F.nvalid--;
        } else {
          if (depth + 1 >= COG_MAX_FAILURES) return false;
          fr[depth + 1].rng = F.rng;
          fr[depth + 1].stage = ENTER;
          depth++;
        }
      } else {
        F.stage = END;
      }
    } else if (F.stage == END) {
      const uint32_t en = uid(F.rng, 2);
      F.stage = FIN;
      const bool ok = add_random_piece(e, COG_PIECE_END0 + (int)en, F.rng);
      if (pv->flags & F_GRID_OVER) return false;
      if (!ok) {
        map_reset(e);
        if (depth + 1 >= COG_MAX_FAILURES) return false;
        fr[depth + 1].rng = F.rng;
        fr[depth + 1].stage = ENTER;
        depth++;
      }
    } else {
      if (!finalize_ok(e)) return false;
      depth--;
    }
  }
  return true;
}

DEV void add_players(const Ctx &e) {                       // map.cpp:343-354 (Q9 defined)
  EnvPriv *pv = e.pv;
  const int n = pv->n_players;
  if (n < pv->loc_size) {
    pv->loc_size = (uint8_t)n;
  } else {
    for (int k = pv->loc_size; k < n && k < 4; k++) { pv->locx[k] = 0; pv->locy[k] = 0; }
    pv->loc_size = (uint8_t)n;
  }
  const int start = e.gs->pieces[0];
  for (int i = 0; i < 37; i++) {
    const uint8_t c = c_phex[start][i];
    const int ps = COG_HEX_REQ(c) == COG_REQ_NULL ? COG_HEX_N(c) : 0;
    if (ps > 0 && ps < n + 1) {
      if (i < pv->loc_size && i < 4) {
        pv->locx[i] = (int8_t)(c_large[i][0] / 2);
        pv->locy[i] = (int8_t)(c_large[i][1] / 2);
      } else {
        pv->flags |= F_Q9_OOB;
      }
    }
  }
  if (start == COG_PIECE_START0 + 1 && n < 4) pv->flags |= F_B_START_LT4;
}

// done: Info + rewards (environment.cpp:187-207, get_reward :281-288)
DEV void finish_episode(const Ctx &e) {
  EnvPriv *pv = e.pv;
  pv->done = 1;
  *reinterpret_cast<uint32_t *>(e.info) = pv->turn_counter;
  float n_winners = 0.f;
  for (int q = 0; q < 4; q++) n_winners += (float)pv->pl[q].has_won;
  for (int q = 0; q < pv->n_players; q++) {
    const PlayerPriv &Q = pv->pl[q];
    uint8_t *ai = e.info + COG_AGENT_INFO0 + COG_AGENT_INFO_STRIDE * q;
    const float rw = (float)(pv->n_players * Q.has_won) - n_winners;
    ai[0] = Q.steps_taken;
    pv->info_steps[q] = Q.steps_taken;
    *reinterpret_cast<float *>(ai + 4) = rw;
    *reinterpret_cast<uint32_t *>(ai + 8) = Q.n_movements;
    ai[12] = Q.n_added_cards;
    ai[13] = Q.n_added_cards;                          // get_n_removed (player.cpp:223-224)
    *reinterpret_cast<uint32_t *>(ai + 16) = 0u;       // n_spent never incremented (Q14)
    *reinterpret_cast<uint32_t *>(ai + 20) = 0u;
    *reinterpret_cast<uint32_t *>(ai + 24) = 0u;
    *reinterpret_cast<uint32_t *>(ai + 28) = Q.n_added_cards;
    e.rew[q] = rw;
  }
}

// ------------------------------------------------------------------------------------------
// map-observation encode (map.cpp:389-405): feature 0 stays 0 (Q2), f[req+1] = n, f[6] = is_end
// ------------------------------------------------------------------------------------------
// Feature f of a hex code, f known at compile time after unrolling.  Code 0 (no hex) and NULL
// hexes (mountain / start, requirement 5) give all-zero features, like finalize's zero fill.
DEV uint32_t feat(uint32_t code, int f) {
  if (f == 0) return 0u;                                   // occupying player: never written (Q2)
  if (f == 6) return (code >> 6) & 1u;                     // is_end
  return (((code >> 3) & 7u) == (uint32_t)(f - 1)) ? (code & 7u) : 0u;
}

// One 16-cell block k (cells 16k..16k+15 of the 48x48 grid, row-major [ix][iy] like the
// observation) -> output bytes [112k, 112k+112) of the 16,128-byte map: one aligned 16-byte
// load of hex codes, seven aligned 16-byte stores.  The byte -> (cell, feature) map is static.
DEV void encode_block(const uint8_t *__restrict__ cgrid, uint8_t *__restrict__ map, int k) {
  const uint4 c4 = reinterpret_cast<const uint4 *>(cgrid)[k];
  const uint32_t cw[4] = {c4.x, c4.y, c4.z, c4.w};
  uint32_t w[28];
#pragma unroll
  for (int q = 0; q < 28; q++) w[q] = 0u;
#pragma unroll
  for (int b = 0; b < 112; b++) {
    const int c = b / 7, f = b % 7;
    const uint32_t code = (cw[c >> 2] >> (8 * (c & 3))) & 0xffu;
    w[b >> 2] |= feat(code, f) << (8 * (b & 3));
  }
  uint4 *out = reinterpret_cast<uint4 *>(map + 112 * k);
#pragma unroll
  for (int q = 0; q < 7; q++) out[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

constexpr int kEncBlocks = COG_GRID * COG_GRID / 16;     // 144 blocks per env

// finalize's index mapping (map.cpp:335-340, 389-405): compact 48x48 code grid of the final
// map, cell (ix, iy) = hex at (ix - 1 + min_x, iy - 1 + min_y) or 0.  Also the lookup table of
// every movement mask / done check (hex_array, map.cpp:273-275).
DEV void build_cgrid(const Ctx &e) {
  const EnvPriv *pv = e.pv;
  const int minx = pv->minx, miny = pv->miny, dx = pv->dimx, dy = pv->dimy;
  uint4 *out = reinterpret_cast<uint4 *>(e.cgrid);
  for (int k = 0; k < kEncBlocks; k++) {
    const int ix = k / 3, iy0 = (k % 3) * 16;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (ix < dx) {
      const uint8_t *row = e.grid + (ix - 1 + minx + kGridOff) * kGridDim + kGridOff + miny - 1;
#pragma unroll
      for (int j = 0; j < 16; j++)
        if (iy0 + j < dy) w[j >> 2] |= (uint32_t)row[iy0 + j] << (8 * (j & 3));
    }
    out[k] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// the wave encodes, one after another, every env of its 64 that was (re)generated
DEV void wave_encode(const DevState &s, size_t i, bool enc) {
  uint64_t m = __ballot(enc);
  const int lane = threadIdx.x & 63;
  const int nl = blockDim.x < 64 ? (int)blockDim.x : 64;  // active lanes (narrow workgroups)
  while (m) {
    const int l = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const size_t env = (size_t)__shfl((int)i, l);
    const uint8_t *cg = s.cgrid + env * COG_CELLS;
    uint8_t *map = s.obs + env * COG_OBS_BYTES;
    for (int k = lane; k < kEncBlocks; k += nl) encode_block(cg, map, k);
  }
}

// ------------------------------------------------------------------------------------------
// Wave-cooperative map generation.  generate() above is the reference's algorithm one env per
// work-item: a long divergent chain of dependent grid loads (k_reset: 9.4 ms for 65,536 maps,
// 96 % of it in generate; one auto-reset inside a rollout stalls its wave for ~180 us).  Here the
// whole wave generates ONE env's map at a time: the generation state is wave-uniform (every lane
// holds the same value), the placed-piece list and the piece transforms are spread over lanes,
// and Map::add_random_piece's candidate placements are tested lane-parallel -- lane c checks
// candidate c's footprint with all its grid loads in flight at once -- and counted / selected
// by ballot + popcount, so the reference's two passes over the candidate list (count, draw, find
// the chosen one) cost one round of loads.  Same algorithm, same RNG draws, same candidate order
// (map.cpp:277-307), same hazards; the owner lane then finishes the reset (players, shop, masks).
// ------------------------------------------------------------------------------------------
DEV uint32_t nth_set_bit(uint32_t m, uint32_t j);
// Lanes of the wave read what other lanes stored: wait until the wave's stores have completed
// (a workgroup fence compiles to nothing for one-wave workgroups), then invalidate the CU's vector
// L1 (an agent-scope acquire: buffer_inv sc1), which may still hold a line loaded before those
// stores -- measured: without it, candidate footprints read hexes placed earlier in the same
// generation as empty
DEV void wg_fence() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}
DEV int lane_id() { return (int)(threadIdx.x & 63u); }
DEV int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }   // l wave-uniform
DEV int wave_min(int v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
DEV int wave_max(int v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
// rot_pt as a linear map: rotation t sends (X, Y) to X*u + Y*v; u, v components + 1 packed in
// 2-bit fields (ux, uy, vx, vy) per t
constexpr uint32_t rot_uv_code(int ux, int uy, int vx, int vy) {
  return (uint32_t)(ux + 1) | (uint32_t)(uy + 1) << 2 | (uint32_t)(vx + 1) << 4 | (uint32_t)(vy + 1) << 6;
}
constexpr uint32_t kRotUV[6] = {rot_uv_code(1, 0, 0, 1), rot_uv_code(0, 1, -1, 1), rot_uv_code(-1, 1, -1, 0),
                                rot_uv_code(-1, 0, 0, -1), rot_uv_code(0, -1, 1, -1), rot_uv_code(1, -1, 1, 0)};
constexpr uint64_t kRotUVPack = (uint64_t)kRotUV[0] | (uint64_t)kRotUV[1] << 8 | (uint64_t)kRotUV[2] << 16 |
                                (uint64_t)kRotUV[3] << 24 | (uint64_t)kRotUV[4] << 32 | (uint64_t)kRotUV[5] << 40;
struct RotUV {
  int ux, uy, vx, vy;
};
DEV RotUV rot_uv(int t) {                                   // t in [0, 6)
  const uint32_t f = (uint32_t)(kRotUVPack >> (8 * t)) & 0xffu;
  return RotUV{(int)(f & 3u) - 1, (int)((f >> 2) & 3u) - 1, (int)((f >> 4) & 3u) - 1, (int)(f >> 6) - 1};
}
constexpr bool rot_uv_ok() {                                // against rot_pt's six cases
  for (int t = 0; t < 6; t++) {
    const uint32_t f = kRotUV[t];
    const int ux = (int)(f & 3u) - 1, uy = (int)((f >> 2) & 3u) - 1, vx = (int)((f >> 4) & 3u) - 1, vy = (int)(f >> 6) - 1;
    const int X = 3, Y = 5;                                 // any point: the maps are linear
    const int ex[6] = {X, -Y, -X - Y, -X, Y, X + Y}, ey[6] = {Y, X + Y, X, -Y, -X - Y, -X};
    if (X * ux + Y * vx != ex[t] || X * uy + Y * vy != ey[t]) return false;
  }
  return true;
}
static_assert(rot_uv_ok(), "rotation table");
DEV int norm6_small(int v) {                                // v in [-6, 12)
  v = v < 0 ? v + 6 : v;
  return v >= 6 ? v - 6 : v;
}

constexpr int8_t kLargeXY[37][2] = COG_LARGE_XY2;
constexpr int8_t kSmallXY[16][2] = COG_SMALL_XY2;
constexpr int8_t kEndXY[3][2] = COG_END_XY2;
// connection sets (conn_set): 0 LARGE->LARGE, 1 LARGE->SMALL, 2 LARGE->TRIPLE, 3 SMALL->LARGE;
// their base points flattened (set s starts at kConnOff[s]), packed as bytes
constexpr int8_t kConnX[12] = {8, 6, 3, 5, 7, 0, -7, -5, -3, 7, 5, 3};
constexpr int8_t kConnY[12] = {6, 8, 7, 5, 3, 8, 10, 10, 10, -10, -10, -10};
constexpr bool conn_tables_ok() {
  const int8_t ll[2][2] = COG_CONN_LL_XY2, ls[3][2] = COG_CONN_LS_XY2, lt[1][2] = COG_CONN_LT_XY2,
               sl[6][2] = COG_CONN_SL_XY2;
  for (int j = 0; j < 2; j++) if (kConnX[j] != ll[j][0] || kConnY[j] != ll[j][1]) return false;
  for (int j = 0; j < 3; j++) if (kConnX[2 + j] != ls[j][0] || kConnY[2 + j] != ls[j][1]) return false;
  if (kConnX[5] != lt[0][0] || kConnY[5] != lt[0][1]) return false;
  for (int j = 0; j < 6; j++) if (kConnX[6 + j] != sl[j][0] || kConnY[6 + j] != sl[j][1]) return false;
  return true;
}
static_assert(conn_tables_ok(), "connection tables");
constexpr uint64_t pack8lo(const int8_t *v) {
  uint64_t r = 0;
  for (int k = 0; k < 8; k++) r |= (uint64_t)(uint8_t)v[k] << (8 * k);
  return r;
}
constexpr uint32_t pack8hi(const int8_t *v) {
  uint32_t r = 0;
  for (int k = 0; k < 4; k++) r |= (uint32_t)(uint8_t)v[8 + k] << (8 * k);
  return r;
}
constexpr uint64_t kConnXLo = pack8lo(kConnX), kConnYLo = pack8lo(kConnY);
constexpr uint32_t kConnXHi = pack8hi(kConnX), kConnYHi = pack8hi(kConnY);
DEV int conn_coord(uint64_t lo, uint32_t hi, int k) {      // signed byte k of the packed table
  const uint32_t b = k < 8 ? (uint32_t)(lo >> (8 * k)) : (hi >> (8 * (k - 8)));
  return (int)(int8_t)(b & 0xffu);
}
DEV int conn_off(int set) { return set == 0 ? 0 : set == 1 ? 2 : set == 2 ? 5 : 6; }
DEV int conn_nbase(int set) { return set == 0 ? 2 : set == 1 ? 3 : set == 2 ? 1 : 6; }
DEV int conn_copies(int set) { return set == 3 ? 1 : 7; }
DEV int conn_opt0(int set) { return set == 1 ? -1 : set == 2 ? -3 : -2; }
DEV int conn_nopt(int set) { return set == 1 ? 2 : set == 2 ? 1 : 6; }
DEV int conn_opt(int set, uint32_t ri) { return set == 1 ? (ri ? 2 : -1) : set == 2 ? -3 : (int)ri - 2; }
// conn_set(q, psize) as a set id, -1: q offers nothing to a piece of size psize
DEV int conn_set_id(int q, int psize) {
  const int qs = c_pmeta[q].size, qk = c_pmeta[q].kind;
  if (qs == COG_PS_LARGE) {
    if (psize == COG_PS_LARGE) return 0;
    if (psize == COG_PS_SMALL) return 1;
    if (psize == COG_PS_TRIPLE && qk != COG_PT_START) return 2;
    return -1;
  }
  return (qs == COG_PS_SMALL && psize == COG_PS_LARGE) ? 3 : -1;
}

struct GenW {                         // wave-uniform generation state of one env
  uint8_t *grid;
  int minx, miny, maxx, maxy, dimx, dimy;
  uint32_t flags;                     // EnvPriv::flags (sticky: read at entry, written back)
  int np;                             // pieces placed
  int pl0, pl1;                       // lane k: pieces[k], pieces[64 + k]
  int tx, ty, tr;                     // lane q < COG_N_PIECES: pcx[q], pcy[q], prot[q]
};
DEV int placed(const GenW &W, int qi) { return qi < 64 ? rdl(W.pl0, qi) : rdl(W.pl1, qi - 64); }

DEV void coop_map_reset(GenW &W) {                         // map.cpp:744-752
  for (int x = W.minx; x <= W.maxx; x++)
    for (int y = W.miny + lane_id(); y <= W.maxy; y += 64) W.grid[(x + kGridOff) * kGridDim + (y + kGridOff)] = 0;
  W.minx = W.miny = W.maxx = W.maxy = 0;
  W.dimx = W.dimy = 0;
  W.np = 0;
  wg_fence();
}

// add_piece (map.cpp:179-191, 309-341): lane k places hex k; the first failing hex (off the
// lattice / past kMaxCoord) stops the placement with the hexes before it written, as in order
DEV bool coop_add_piece(GenW &W, int p, int cx2, int cy2, int rot) {
  const int lane = lane_id();
  int r = rdl(W.tr, p) + rot;
  r %= 6;
  r = r < 0 ? r + 6 : r;
  const int pcx = rdl(W.tx, p) + cx2, pcy = rdl(W.ty, p) + cy2;
  if (lane == p) {
    W.tr = r;
    W.tx = pcx;
    W.ty = pcy;
  }
  if (W.np >= kMaxPlaced) {
    W.flags |= F_GRID_OVER;
    return false;
  }
  if (W.np < 64) {
    if (lane == W.np) W.pl0 = p;
  } else if (lane == W.np - 64) {
    W.pl1 = p;
  }
  W.np++;
  const int nh = c_pmeta[p].n_hex;
  const bool in = lane < nh;
  int X, Y;
  piece_xy2(p, in ? lane : 0, X, Y);
  const RotUV R = rot_uv(r);
  const int rx = X * R.ux + Y * R.vx + pcx, ry = X * R.uy + Y * R.vy + pcy;
  const int x = rx >> 1, y = ry >> 1;                      // exact: only used when both are even
  const bool bad = ((rx | ry) & 1) || x < -kMaxCoord || x > kMaxCoord || y < -kMaxCoord || y > kMaxCoord;
  const uint64_t bm = __builtin_amdgcn_ballot_w64(in && bad);
  const int f = bm ? __ffsll((unsigned long long)bm) - 1 : nh;
  if (lane < f) W.grid[(x + kGridOff) * kGridDim + (y + kGridOff)] = c_phex[p][lane];
  wg_fence();
  if (bm) {
    W.flags |= F_GRID_OVER;
    return false;
  }
  W.minx = min(W.minx, wave_min(in ? x : W.minx));
  W.miny = min(W.miny, wave_min(in ? y : W.miny));
  W.maxx = max(W.maxx, wave_max(in ? x : W.maxx));
  W.maxy = max(W.maxy, wave_max(in ? y : W.maxy));
  return true;
}

// footprint_free for this lane's candidate: every hex's grid load issued before any is used
template <int NH>
DEV bool footprint_hit(const uint8_t *grid, const int8_t (*xy)[2], int t, int cx2, int cy2) {
  const RotUV R = rot_uv(t);
  uint32_t v[NH];
  bool on[NH];
#pragma unroll
  for (int k = 0; k < NH; k++) {
    const int X = xy[k][0], Y = xy[k][1];
    const int rx = X * R.ux + Y * R.vx + cx2, ry = X * R.uy + Y * R.vy + cy2;
    const int x = rx >> 1, y = ry >> 1;
    on[k] = !((rx | ry) & 1) && x >= -kGridOff && x < kGridOff && y >= -kGridOff && y < kGridOff;
    v[k] = grid[on[k] ? (x + kGridOff) * kGridDim + (y + kGridOff) : 0];
  }
  bool hit = false;
#pragma unroll
  for (int k = 0; k < NH; k++) hit |= on[k] && v[k] != 0u;
  return hit;
}

struct Cand {                         // candidate c of add_random_piece's enumeration order
  int set, q, ci, j;
};
// candidate c (c < total) -> (placed piece, copy, base point), in map.cpp:282-300's loop order
DEV Cand cand_of(const GenW &W, int psize, int c) {
  Cand k{-1, 0, 0, 0};
  int acc = 0, local = 0;
  for (int qi = 0; qi < W.np; qi++) {
    const int q = placed(W, qi);
    const int set = conn_set_id(q, psize);
    const int n = set < 0 ? 0 : conn_copies(set) * conn_nbase(set);
    if (c >= acc && c < acc + n) {
      k.set = set;
      k.q = q;
      local = c - acc;
    }
    acc += n;
  }
  const int nb = conn_nbase(k.set);
  k.ci = k.set == 0 ? local >> 1 : k.set == 1 ? (local * 171) >> 9 : k.set == 2 ? local : 0;   // local / nb (< 21)
  k.j = local - k.ci * nb;
  return k;
}
// the candidate's centre and the rotation its footprint is tested at
DEV void cand_place(const GenW &W, const Cand &k, bool uniform_q, int &cx, int &cy, int &t, int &qrot) {
  int qcx, qcy;
  if (uniform_q) {
    qrot = rdl(W.tr, k.q); qcx = rdl(W.tx, k.q); qcy = rdl(W.ty, k.q);
  } else {
    qrot = __shfl(W.tr, k.q); qcx = __shfl(W.tx, k.q); qcy = __shfl(W.ty, k.q);
  }
  const int b = conn_off(k.set) + k.j;
  const int bx = conn_coord(kConnXLo, kConnXHi, b), by = conn_coord(kConnYLo, kConnYHi, b);
  const RotUV R = rot_uv(norm6_small(k.ci + qrot));
  cx = bx * R.ux + by * R.vx + qcx;
  cy = bx * R.uy + by * R.vy + qcy;
  t = norm6_small(conn_opt0(k.set) + k.ci + qrot);
}
// this lane's candidate (c = batch * 64 + lane) is a valid placement of piece p.  Every lane
// runs it (a lane past the end evaluates candidate 0): the transforms are read from other lanes
// (ds_bpermute), and an inactive source lane would read as 0
DEV bool cand_free(const GenW &W, int p, int psize, int c, int total) {
  const Cand k = cand_of(W, psize, c < total ? c : 0);
  int cx, cy, t, qrot;
  cand_place(W, k, false, cx, cy, t, qrot);
  bool hit;
  if (psize == COG_PS_LARGE) hit = footprint_hit<37>(W.grid, kLargeXY, t, cx, cy);
  else if (psize == COG_PS_SMALL) hit = footprint_hit<16>(W.grid, kSmallXY, t, cx, cy);
  else hit = footprint_hit<3>(W.grid, kEndXY, t, cx, cy);
  if (c >= total) return false;
  return !hit;
}
DEV int nth_set_bit64(uint64_t m, uint32_t j) {
  const uint32_t lo = (uint32_t)m, c = __popc(lo);
  return j < c ? (int)nth_set_bit(lo, j) : 32 + (int)nth_set_bit((uint32_t)(m >> 32), j - c);
}

// Map::add_random_piece (map.cpp:277-307)
DEV bool coop_add_random_piece(GenW &W, int p, uint32_t &rng) {
  const int lane = lane_id();
  if (lane == p) {                                         // MapPiece::reset
    W.tx = 0;
    W.ty = 0;
    W.tr = 0;
  }
  const int psize = c_pmeta[p].size;
  int total = 0;
  for (int qi = 0; qi < W.np; qi++) {
    const int set = conn_set_id(placed(W, qi), psize);
    total += set < 0 ? 0 : conn_copies(set) * conn_nbase(set);
  }
  uint64_t bal0 = 0, bal1 = 0;                             // the first two batches' ballots
  uint32_t nvalid = 0;
  for (int b = 0; b * 64 < total; b++) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(cand_free(W, p, psize, b * 64 + lane, total));
    if (b == 0) bal0 = m;
    if (b == 1) bal1 = m;
    nvalid += (uint32_t)__popcll(m);
  }
  if (!nvalid) return false;
  const uint32_t chosen = uid(rng, nvalid);
  int c = 0;
  uint32_t acc = 0;
  for (int b = 0; b * 64 < total; b++) {
    const uint64_t m = b == 0 ? bal0 : b == 1 ? bal1 : __builtin_amdgcn_ballot_w64(cand_free(W, p, psize, b * 64 + lane, total));
    const uint32_t pc = (uint32_t)__popcll(m);
    if (chosen < acc + pc) {
      c = b * 64 + nth_set_bit64(m, chosen - acc);
      break;
    }
    acc += pc;
  }
  const Cand k = cand_of(W, psize, c);
  int cx, cy, t, qrot;
  cand_place(W, k, true, cx, cy, t, qrot);
  const uint32_t ri = uid(rng, (uint32_t)conn_nopt(k.set));
  return coop_add_piece(W, p, cx, cy, conn_opt(k.set, ri) + k.ci + qrot);
}

DEV bool coop_finalize_ok(GenW &W) {                       // map.cpp:389-405 (dims check, Q27)
  const int dx = 3 + W.maxx - W.minx, dy = 3 + W.maxy - W.miny;
  if (dx > 49 || dy > 49) {
    W.flags |= F_GRID_OVER;
    return false;
  }
  W.dimx = dx;
  W.dimy = dy;
  return true;
}

constexpr uint32_t travel_mask(int diff) {                 // travel pieces of difficulty <= diff
  const uint8_t d[COG_N_TRAVEL] = {0, 1, 2, 0, 2, 1, 1, 0, 1, 1, 2, 1, 2, 1, 1, 1};
  uint32_t m = 0;
  for (int i = 0; i < COG_N_TRAVEL; i++) m |= (d[i] <= diff ? 1u : 0u) << i;
  return m;
}
constexpr bool travel_mask_ok() {
  const cog_piece_meta_t meta[COG_N_PIECES] = COG_PIECE_META;
  for (int diff = 0; diff < 4; diff++)
    for (int i = 0; i < COG_N_TRAVEL; i++)
      if ((((travel_mask(diff) >> i) & 1u) != 0u) != (meta[COG_PIECE_TRAVEL0 + i].difficulty <= diff)) return false;
  return true;
}
static_assert(travel_mask_ok(), "travel piece difficulties");

// generate() on wave-uniform frames: a frame is (rng, next travel index i, the valid list as a
// bit set -- it starts sorted and erasing keeps it sorted, so valid[k] is the k-th set bit --,
// stage), held in registers selected by depth
DEV bool coop_generate_frames(GenW &W, uint32_t rng0, int n_pieces, int diff) {
  enum { ENTER = 0, LOOP = 1, END = 2, FIN = 3 };
  uint32_t f_rng[COG_MAX_FAILURES], f_mask[COG_MAX_FAILURES];
  int f_i[COG_MAX_FAILURES], f_stage[COG_MAX_FAILURES];
#pragma unroll
  for (int d = 0; d < COG_MAX_FAILURES; d++) { f_rng[d] = 0; f_mask[d] = 0; f_i[d] = 0; f_stage[d] = ENTER; }
  f_rng[0] = rng0;
  int depth = 0;
  while (depth >= 0) {
    uint32_t rng = 0, mask = 0;
    int fi = 0, stage = 0;
#pragma unroll
    for (int d = 0; d < COG_MAX_FAILURES; d++)
      if (d == depth) { rng = f_rng[d]; mask = f_mask[d]; fi = f_i[d]; stage = f_stage[d]; }
    bool push = false, pop = false;
    if (stage == ENTER) {
      const uint32_t s = uid(rng, 2);
      if (!coop_add_piece(W, COG_PIECE_START0 + (int)s, 0, 0, 0)) return false;
      mask = travel_mask(diff);
      fi = 0;
      stage = LOOP;
    } else if (stage == LOOP) {
      if (fi < n_pieces) {
        bool ok = false;
        int next = 0;
        const uint32_t nv = (uint32_t)__popc(mask);
        if (nv) {
          next = (int)nth_set_bit(mask, uid(rng, nv));
          ok = coop_add_random_piece(W, COG_PIECE_TRAVEL0 + next, rng);
          if (W.flags & F_GRID_OVER) return false;
        }
        fi++;
        if (ok) {                                          // vector::erase(begin() + next), Q5
          if ((uint32_t)next >= nv) W.flags |= F_ERASE_PAST;   // past the end: the last one goes
          mask &= ~(1u << nth_set_bit(mask, (uint32_t)next < nv ? (uint32_t)next : nv - 1u));
        } else {
          if (depth + 1 >= COG_MAX_FAILURES) return false;
          push = true;
        }
      } else {
        stage = END;
      }
    } else if (stage == END) {
      const uint32_t en = uid(rng, 2);
      stage = FIN;
      const bool ok = coop_add_random_piece(W, COG_PIECE_END0 + (int)en, rng);
      if (W.flags & F_GRID_OVER) return false;
      if (!ok) {
        coop_map_reset(W);
        if (depth + 1 >= COG_MAX_FAILURES) return false;
        push = true;
      }
    } else {                                               // FIN: finalize, then return
      if (!coop_finalize_ok(W)) return false;
      pop = true;
    }
#pragma unroll
    for (int d = 0; d < COG_MAX_FAILURES; d++)
      if (d == depth) { f_rng[d] = rng; f_mask[d] = mask; f_i[d] = fi; f_stage[d] = stage; }
    if (push) {                                            // recursion with the frame's rng copy
#pragma unroll
      for (int d = 0; d < COG_MAX_FAILURES; d++)
        if (d == depth + 1) { f_rng[d] = rng; f_stage[d] = ENTER; }
      depth++;
    } else if (pop) {
      depth--;
    }
  }
  return true;
}

DEV void coop_build_cgrid(const GenW &W, uint8_t *cgrid) {  // build_cgrid, lane k: block k
  uint4 *out = reinterpret_cast<uint4 *>(cgrid);
  for (int k = lane_id(); k < kEncBlocks; k += 64) {
    const int ix = k / 3, iy0 = (k % 3) * 16;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    if (ix < W.dimx) {
      const uint8_t *row = W.grid + (ix - 1 + W.minx + kGridOff) * kGridDim + kGridOff + W.miny - 1;
#pragma unroll
      for (int j = 0; j < 16; j++)
        if (iy0 + j < W.dimy) w[j >> 2] |= (uint32_t)row[iy0 + j] << (8 * (j & 3));
    }
    out[k] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// map_reset + the piece transforms' reset (environment.cpp:46-49), Map::generate and, when it
// succeeds, the compact code grid, for env `env`, by the whole wave; returns whether generation
// succeeded.  The EnvPriv / GenScratch fields generation owns are written back at the end.
// The env's EnvPriv fields generation reads, as the owner lane holds them (it read them itself:
// program order covers its own earlier stores) and broadcasts them
struct GenIn {
  uint32_t rng, flags, bounds, npd;   // bounds: minx, miny, maxx, maxy bytes; npd: n_pieces | difficulty << 8
};
DEV GenIn gen_in_of(const EnvPriv *pv) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(pv);
  return GenIn{pv->rng, pv->flags, w[offsetof(EnvPriv, minx) / 4], (uint32_t)pv->n_pieces | (uint32_t)pv->difficulty << 8};
}
DEV bool coop_generate(const DevState &s, uint32_t env, int owner, const GenIn &own) {
  const int lane = lane_id();
  EnvPriv *pv = s.priv + env;
  GenScratch *gs = s.gen + env;
  GenW W;
  W.grid = s.grid + (size_t)env * kGridBytes;
  const uint32_t bounds = (uint32_t)rdl((int)own.bounds, owner);
  W.minx = (int8_t)(bounds & 0xffu); W.miny = (int8_t)((bounds >> 8) & 0xffu);
  W.maxx = (int8_t)((bounds >> 16) & 0xffu); W.maxy = (int8_t)(bounds >> 24);
  W.dimx = W.dimy = 0;
  W.flags = (uint32_t)rdl((int)own.flags, owner);
  const uint32_t rng0 = (uint32_t)rdl((int)own.rng, owner);
  const uint32_t npd = (uint32_t)rdl((int)own.npd, owner);
  const int n_pieces = (int)(npd & 0xffu), diff = (int)(npd >> 8);
  coop_map_reset(W);
  W.tx = W.ty = W.tr = 0;
  W.pl0 = W.pl1 = 0;
  const bool ok = coop_generate_frames(W, rng0, n_pieces, diff);
  if (ok) coop_build_cgrid(W, s.cgrid + (size_t)env * COG_CELLS);
  if (lane == owner) {                                     // what the owner lane reads back later
    pv->minx = (int8_t)W.minx; pv->miny = (int8_t)W.miny; pv->maxx = (int8_t)W.maxx; pv->maxy = (int8_t)W.maxy;
    pv->dimx = (uint8_t)W.dimx; pv->dimy = (uint8_t)W.dimy;
    pv->flags = W.flags;
    gs->npieces = (uint8_t)W.np;
    gs->pieces[0] = (uint8_t)rdl(W.pl0, 0);                // (add_players' start piece)
  }
  if (lane < COG_N_PIECES) {
    gs->pcx[lane] = (int16_t)W.tx;
    gs->pcy[lane] = (int16_t)W.ty;
    gs->prot[lane] = (uint8_t)W.tr;
  }
  if (lane > 0 && lane < W.np) gs->pieces[lane] = (uint8_t)W.pl0;
  if (64 + lane < W.np) gs->pieces[64 + lane] = (uint8_t)W.pl1;
  return ok;
}

// The wave generates, one env after another, the map of every lane whose `want` is set, and
// returns this lane's result.  Called by every lane of the wave in converged control flow (a
// wave-uniform no-op when no lane wants a map).  The owner lane reads the EnvPriv fields
// generation needs and writes back what it reads later itself; the grid and cgrid, which lanes
// write for each other, are ordered by waits for the wave's stores (wg_fence).
DEV bool wave_generate(const DevState &s, size_t i, bool want) {
  uint64_t m = __builtin_amdgcn_ballot_w64(want);
  if (!m) return false;
  GenIn own{};
  if (want) own = gen_in_of(s.priv + i);
  bool mine = false;
  while (m) {
    const int l = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const uint32_t env = (uint32_t)rdl((int)(uint32_t)i, l);
    const bool ok = coop_generate(s, env, l, own);
    if (lane_id() == l) mine = ok;
  }
  wg_fence();
  return mine;
}

// cog_env::reset() (environment.cpp:42-64) around the wave's generation: before it ...
DEV void env_reset_pre(const Ctx &e) {
  e.pv->agent = 0;
  e.sh[0] = COG_PHASE_INACTIVE;
}
// ... and after it, on the owner lane: players, shop, masks, neighbourhood caches
DEV bool env_reset_post(const Ctx &e, bool gen_ok) {
  EnvPriv *pv = e.pv;
  if (!gen_ok) {
    pv->flags |= F_MAPGEN_FAIL;
    return false;
  }
  for (int i = 0; i < pv->n_players; i++) player_reset(e, i);
  add_players(e);
  for (int k = 0; k < COG_N_SHOP; k++) e.sh[SH_SHOP + k] = COG_CARDS_PER_TYPE;
  pv->in_market = kInMarket0;                              // n_in_market NOT reset (Q12)
  pv->done = 0;
  pv->turn_counter = 0;
  for (int i = 0; i < pv->n_players; i++) update_observation(e, i);
  copy_mask(e.sel, stm(e, 0));
  for (int i = 0; i < pv->n_players; i++) load_cells(e, i);
  return true;
}

// ------------------------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------------------------
__global__ void k_init(DevState s, uint32_t default_seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= s.n) return;
  EnvPriv *pv = s.priv + i;
  EnvPriv z;
  memset(&z, 0, sizeof(z));
  z.seed = default_seed + (uint32_t)(s.first + i);
  z.rng = mr_seed(z.seed);
  z.n_players = 4; z.n_pieces = 3; z.difficulty = 0; z.max_steps = 100000;
  z.n_in_market = COG_MKT_SLOTS;
  z.in_market = kInMarket0;
  for (int p = 0; p < 4; p++) {                            // no map yet: every lookup is outside
    for (int d = 0; d < 7; d++) z.cells[p][d] = COG_HEX_MOUNTAIN;
    z.cells[p][7] = 0x7f;
  }
  *pv = z;
  uint8_t *ob = s.obs + i * COG_OBS_BYTES;
  for (int k = 0; k < COG_N_SHOP; k++) ob[COG_OBS_SHOP + k] = COG_CARDS_PER_TYPE;
  uint8_t *sel = s.sel + i * COG_MASK_BYTES;
  for (int m = 0; m < 5; m++) {                            // ActionMask() defaults (Q26)
    uint8_t *am = m == 4 ? sel : ob + COG_OBS_PLAYER0 + COG_OBS_PLAYER_STRIDE * m + COG_PD_MASK;
    am[COG_MASK_PLAY] = am[COG_MASK_SPECIAL] = am[COG_MASK_REMOVE] = 1;
    am[COG_MASK_MOVE] = am[COG_MASK_SHOP] = 1;
  }
}

// blocks of one wave; lanes 0 .. epw - 1 own envs, the others only help the wave's cooperative
// map generation (which runs one env at a time): a small batch spreads over many waves
__global__ void k_reset(DevState s, ResetParams p, int epw) {
  const size_t i0 = (size_t)blockIdx.x * epw + threadIdx.x;
  const bool live = (int)threadIdx.x < epw && i0 < s.n;
  const size_t i = live ? i0 : (size_t)blockIdx.x * epw;
  Ctx e = make_ctx(s, i);
  EnvPriv *pv = e.pv;
  if (live) {
    if (p.use_params) {                                    // cog_env::reset(params) :66-77
      pv->n_players = p.n_players;
      pv->n_pieces = p.n_pieces;
      pv->difficulty = p.difficulty;
      pv->max_steps = p.max_steps;
      pv->seed = p.seed + (uint32_t)(s.first + i);         // vec_environment.h:41, u32 wrap (Q33)
      pv->rng = mr_seed(pv->seed);
    }
    env_reset_pre(e);
  }
  const bool ok = wave_generate(s, i, live);               // converged: the whole wave
  if (live && !env_reset_post(e, ok)) {
    atomicOr(&s.status[0], pv->flags);
    atomicAdd(&s.status[1], 1u);
    *s.err = 1u;                                           // host-visible error flag
  }
}

// streaming map-observation encode over all envs: one work-item per 16-cell block
__global__ void __launch_bounds__(256) k_encode_direct(const uint8_t *__restrict__ cgrid, uint8_t *__restrict__ obs,
                                                       size_t n_blocks) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_blocks) return;
  const size_t env = t / kEncBlocks;
  const int k = (int)(t - env * kEncBlocks);
  encode_block(cgrid + env * COG_CELLS, obs + env * COG_OBS_BYTES, k);
}

// Same work, transposed through LDS so every store wave-instruction writes 1 KiB contiguous:
// item t builds its 112 bytes into LDS at 112*t (ds_write_b128, conflict-free at this stride),
// then the workgroup streams the 256*112 bytes out as 16-byte chunks in address order.
template <bool NT>
__global__ void __launch_bounds__(256) k_encode_lds(const uint8_t *__restrict__ cgrid, uint8_t *__restrict__ obs,
                                                    size_t n_blocks) {
  __shared__ uint4 stage[256 * 7];
  const size_t g0 = (size_t)blockIdx.x * 256;
  const size_t t = g0 + threadIdx.x;
  if (t < n_blocks) {
    const size_t env = t / kEncBlocks;
    const int k = (int)(t - env * kEncBlocks);
    const uint4 c4 = reinterpret_cast<const uint4 *>(cgrid + env * COG_CELLS)[k];
    const uint32_t cw[4] = {c4.x, c4.y, c4.z, c4.w};
    uint32_t w[28];
#pragma unroll
    for (int q = 0; q < 28; q++) w[q] = 0u;
#pragma unroll
    for (int b = 0; b < 112; b++) {
      const int c = b / 7, f = b % 7;
      const uint32_t code = (cw[c >> 2] >> (8 * (c & 3))) & 0xffu;
      w[b >> 2] |= feat(code, f) << (8 * (b & 3));
    }
#pragma unroll
    for (int q = 0; q < 7; q++) stage[threadIdx.x * 7 + q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
  __syncthreads();
  const size_t nb = n_blocks - g0 < 256 ? n_blocks - g0 : 256;
  for (int j = threadIdx.x; j < (int)nb * 7; j += 256) {
    const size_t gb = g0 + (size_t)(j / 7);
    const size_t env = gb / kEncBlocks;
    const int k = (int)(gb - env * kEncBlocks);
    uint4 *dst = reinterpret_cast<uint4 *>(obs + env * COG_OBS_BYTES + 112 * k) + (j % 7);
    if (NT) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const uint4 v = stage[j];
      u32x4 x = {v.x, v.y, v.z, v.w};
      __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(dst));
    } else {
      *dst = stage[j];
    }
  }
}

// ------------------------------------------------------------------------------------------
// Mask bit-vectors.  The step keeps every ActionMask as its 92 named bytes packed into bits
// (bit k == byte k != 0): w0 = bytes 0..31, w1 = 32..63, w2 = 64..91.  One 16-B record per mask
// in DevState::heads: [5 i] the selected mask, [5 i + 1 + p] the stored mask of player p.  The
// byte records (ObsData / selected_action_masks) are the outputs; the step never reads them.
// ------------------------------------------------------------------------------------------
struct Heads {                        // the five heads of one mask (sampler.h:14-79)
  uint32_t play, spec, rem, move, shop;
};
struct MBits {
  uint32_t w0, w1, w2;
};

DEV Heads heads_of(const MBits &b) {
  Heads h;
  h.play = b.w0 & 0x3fffffu;
  h.spec = ((b.w0 >> 22) | (b.w1 << 10)) & 0x3fffffu;
  h.rem = ((b.w1 >> 12) | (b.w2 << 20)) & 0x3fffffu;
  h.move = (b.w2 >> 2) & 0x7fu;
  h.shop = (b.w2 >> 9) & 0x7ffffu;
  return h;
}
DEV MBits bits_of(const Heads &h) {
  MBits b;
  b.w0 = h.play | (h.spec << 22);
  b.w1 = (h.spec >> 10) | (h.rem << 12);
  b.w2 = (h.rem >> 20) | (h.move << 2) | (h.shop << 9);
  return b;
}
DEV MBits mbits_of(const uint4 &v) { return MBits{v.x, v.y, v.z}; }
DEV uint4 mbits_u4(const MBits &b) { return make_uint4(b.w0, b.w1, b.w2, 0u); }

DEV uint32_t bools4(uint32_t w) {                          // 4 bool bytes -> 4 bits (nonzero = set)
  const uint32_t nz = (((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u;
  return ((nz >> 7) * 0x01020408u) >> 24 & 0xfu;
}
DEV uint32_t expand4(uint32_t x) { return (x * 0x00204081u) & 0x01010101u; }   // 4 bits -> 4 bool bytes

DEV MBits mbits_from_bytes(const uint8_t *mask) {          // ActionMask bytes -> bits (4-B aligned)
  const uint32_t *m32 = reinterpret_cast<const uint32_t *>(mask);
  MBits b{0u, 0u, 0u};
#pragma unroll
  for (int w = 0; w < 23; w++) {
    const uint32_t v = bools4(m32[w]) << (4 * (w & 7));
    if (w < 8) b.w0 |= v;
    else if (w < 16) b.w1 |= v;
    else b.w2 |= v;
  }
  return b;
}
DEV uint32_t mask_dword(const MBits &b, int q) {           // named dword q (bytes 4q..4q+3), q < 24
  const uint32_t w = q < 8 ? b.w0 : (q < 16 ? b.w1 : b.w2);
  return q < 23 ? expand4((w >> (4 * (q & 7))) & 0xfu) : 0u;
}
DEV uint4 mask_granule(const MBits &b, int g) {            // 16-B granule g (0..5) of the record
  return make_uint4(mask_dword(b, 4 * g), mask_dword(b, 4 * g + 1), mask_dword(b, 4 * g + 2), mask_dword(b, 4 * g + 3));
}
DEV uint32_t mask_diff_granules(const MBits &a, const MBits &b) {   // granules whose bytes differ
  const uint32_t x0 = a.w0 ^ b.w0, x1 = a.w1 ^ b.w1, x2 = a.w2 ^ b.w2;
  return ((x0 & 0xffffu) ? 1u : 0u) | ((x0 >> 16) ? 2u : 0u) | ((x1 & 0xffffu) ? 4u : 0u) | ((x1 >> 16) ? 8u : 0u) |
         ((x2 & 0xffffu) ? 16u : 0u) | ((x2 >> 16) ? 32u : 0u);
}

// heads of every mask of env i from its byte records (after init / reset / auto-reset)
DEV void sync_heads(const DevState &s, size_t i) {
  uint4 *h = s.heads + 5 * i;
  h[0] = mbits_u4(mbits_from_bytes(s.sel + i * COG_MASK_BYTES));
  const uint8_t *ob = s.obs + i * COG_OBS_BYTES + COG_OBS_PLAYER0 + COG_PD_MASK;
#pragma unroll
  for (int p = 0; p < 4; p++) h[1 + p] = mbits_u4(mbits_from_bytes(ob + COG_OBS_PLAYER_STRIDE * p));
}

// ------------------------------------------------------------------------------------------
// sampler (sampler.h:14-79): 5 independent uniform picks over the set bits of each head
// ------------------------------------------------------------------------------------------
DEV uint32_t nth_set_bit(uint32_t m, uint32_t j) {        // index of the j-th (0-based) set bit
  uint32_t base = 0;
  uint32_t c = __popc(m & 0xffffu);
  if (j >= c) { j -= c; base += 16; m >>= 16; }
  c = __popc(m & 0xffu);
  if (j >= c) { j -= c; base += 8; m >>= 8; }
  c = __popc(m & 0xfu);
  if (j >= c) { j -= c; base += 4; m >>= 4; }
  c = __popc(m & 0x3u);
  if (j >= c) { j -= c; base += 2; m >>= 2; }
  c = m & 1u;
  if (j >= c) { base += 1; }
  return base;
}
DEV uint8_t pick(uint32_t &rng, uint32_t m) {
  const uint32_t k = __popc(m);
  if (!k) return 0;
  if (k == 1) {                                            // one candidate: a single accepted draw
    uint32_t r = mr_next(rng) - 1u;                        // (past = range: only r == range rejects)
    while (r >= kUrngRange) r = mr_next(rng) - 1u;
    return (uint8_t)(__ffs(m) - 1);
  }
  return (uint8_t)nth_set_bit(m, uid_small(rng, k));      // k <= 22: division-free
}
// The five heads draw in order, one accepted draw per non-empty head.  Every head has <= 22
// candidates, so a draw below kSmallSafe is accepted whatever k is: the draws are taken
// branch-free first (the state advances past a head only if it has candidates), and only the
// heads with two or more candidates do arithmetic.  A lane holding a draw that might be rejected
// (probability < 2^-25 per head) redoes the sampling the sequential way, rejections included.
DEV void sample_heads(const Heads &h, uint32_t &rng, uint8_t out[5], const UidEntry *tab) {
  const uint32_t m[5] = {h.play, h.spec, h.rem, h.move, h.shop};
  uint32_t x = rng, r[5], k[5], riskv = 0;
  const UidEntry e0 = tab[__popc(m[0])];                  // head 0's entry, read before the draws
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 5; j++) {
    k[j] = __popc(m[j]);
    uint32_t xn = x;
    r[j] = mr_next(xn) - 1u;
    x = k[j] ? xn : x;
    // r >= kSmallSafe  <=>  bit 31 of r + 34 (r < 2^31 - 2); m | -m has bit 31 set iff m != 0:
    // the flag stays in a vector register (no compare into a scalar mask per head)
    riskv |= (r[j] + (0x80000000u - kSmallSafe)) & (m[j] | (0u - m[j]));
  }
  __builtin_amdgcn_sched_barrier(0);
  if (riskv >> 31) {
    uint32_t y = rng;
#pragma unroll
    for (int j = 0; j < 5; j++) out[j] = pick(y, m[j]);
    rng = y;
    return;
  }
  rng = x;
#pragma unroll
  for (int j = 0; j < 5; j++) out[j] = (uint8_t)(k[j] ? (uint32_t)(__ffs(m[j]) - 1) : 0u);
  if (k[0] >= 2u) out[0] = (uint8_t)nth_set_bit(m[0], uid_tab_accepted(r[0], e0.s, e0.m));
  // heads 1-4 rarely hold two candidates (the selected mask's special / remove / move / shop
  // heads): one uniform branch skips them all when no lane of the wave needs arithmetic there
  if (__builtin_amdgcn_ballot_w64(max(max(k[1], k[2]), max(k[3], k[4])) >= 2u)) {
#pragma unroll
    for (int j = 1; j < 5; j++)
      if (k[j] >= 2u) out[j] = (uint8_t)nth_set_bit(m[j], uid_tab(tab, r[j], k[j]));
  }
}
// The trio's presampled draws.  With every head non-empty a sample takes exactly five accepted
// draws, so the sampler's state two steps on is known before those steps run: the storing wave
// computes, from the state a step record carries, the five draws of the step after next
// (presample: the state they start from, head 0's draw, the state after the five, and whether any
// draw could be rejected) and the stepping wave samples from them (sample_lean) when its state is
// the one they start from and heads 1-4 are {0} -- else it draws the sequential way (sample_heads).  The values
// are the same either way (cog_rng.h jump-ahead: x * 16807^j mod (2^31 - 1)).
constexpr uint32_t kPow15 = mr_pow(15);
DEV uint4 presample(uint32_t x) {                          // x: the state the step starts from
  uint32_t y = x, r0 = 0, risk = 0;
#pragma unroll
  for (int j = 0; j < 5; j++) {
    const uint32_t r = mr_next(y) - 1u;
    if (j == 0) r0 = r;
    risk |= r >= kSmallSafe ? 1u : 0u;
  }
  return make_uint4(x, r0, y, risk);
}
DEV void sample_mask(const uint8_t *mask, uint32_t &rng, uint8_t out[5], const UidEntry *tab) {
  sample_heads(heads_of(mbits_from_bytes(mask)), rng, out, tab);
}
DEV void store_action(uint8_t *dst, const uint8_t a[5]) {
  const uint32_t lo = (uint32_t)a[0] | (uint32_t)a[1] << 8 | (uint32_t)a[2] << 16 | (uint32_t)a[3] << 24;
  reinterpret_cast<uint2 *>(dst)[0] = make_uint2(lo, (uint32_t)a[4]);
}

// ------------------------------------------------------------------------------------------
// Register-resident step (cog_env::step, environment.cpp:91-288).  Each work-item loads its
// env's working set (~300 B) straight into VGPRs in two rounds (fixed-address records, then the
// acting player's records), runs the game logic on registers only, and stores back the 16-B
// granules that changed.  Card / shop tables are compile-time bit-packed constants, so no
// divergent table loads sit on the critical path.
// ------------------------------------------------------------------------------------------
constexpr cog_card_t kCards[COG_N_CARDTYPES] = COG_CARD_TABLE;
constexpr uint8_t kShopTypes[COG_N_SHOP] = COG_SHOP_TYPES;
constexpr uint32_t kSpecialBits = 0x1f8000u;              // card types 15..20

enum CardField { CF_RES0, CF_RES1, CF_RES2, CF_COST, CF_SPECIAL, CF_SINGLE };
constexpr uint32_t card_field(int c, int f) {
  return f == CF_COST ? kCards[c].cost : f == CF_SPECIAL ? kCards[c].special : f == CF_SINGLE ? kCards[c].single_use
                                                                                             : kCards[c].res[f];
}
constexpr uint64_t pack3(int f) {                          // 21 cards x 3 bits
  uint64_t v = 0;
  for (int c = 0; c < COG_N_CARDTYPES; c++) v |= (uint64_t)(card_field(c, f) & 7u) << (3 * c);
  return v;
}
constexpr uint64_t kRes0 = pack3(CF_RES0), kRes1 = pack3(CF_RES1), kRes2 = pack3(CF_RES2);
constexpr uint64_t kCost = pack3(CF_COST), kSpecial = pack3(CF_SPECIAL), kSingle = pack3(CF_SINGLE);
constexpr uint32_t shop_cost_mask(int v) {                 // shop slots whose card costs v
  uint32_t m = 0;
  for (int i = 0; i < COG_N_SHOP; i++) m |= (kCards[kShopTypes[i]].cost == v ? 1u : 0u) << i;
  return m;
}
static_assert(pack3(CF_RES0) >> 63 == 0, "3-bit card fields");

constexpr uint32_t kCostMask1 = shop_cost_mask(1), kCostMask2 = shop_cost_mask(2), kCostMask3 = shop_cost_mask(3),
                   kCostMask4 = shop_cost_mask(4), kCostMask5 = shop_cost_mask(5);
constexpr int shop_type(int k) { return k < 4 ? k + 1 : (k == 4 ? 6 : k + 3); }   // COG_SHOP_TYPES
constexpr bool shop_types_ok() {
  for (int k = 0; k < COG_N_SHOP; k++)
    if (shop_type(k) != kShopTypes[k]) return false;
  return (kCostMask1 | kCostMask2 | kCostMask3 | kCostMask4 | kCostMask5) == 0x3ffffu;
}
static_assert(shop_types_ok(), "shop slot -> card type formula / cost masks");

DEV uint32_t cardf(uint64_t table, int c) { return (uint32_t)(table >> (3 * c)) & 7u; }
DEV uint32_t set_bit(uint32_t m, int k, bool v) { return v ? (m | (1u << k)) : (m & ~(1u << k)); }

// DeckObs bytes 0..111 in 28 dwords: constant-position accessors, and dynamic-index accessors
// that select over the dwords a 21-byte pile can touch (u8 wrap-around, like the reference)
DEV uint32_t dk_get(const uint32_t *d, int b) { return (d[b >> 2] >> (8 * (b & 3))) & 0xffu; }
DEV void dk_put(uint32_t *d, int b, uint32_t v) {
  const int sh = 8 * (b & 3);
  d[b >> 2] = (d[b >> 2] & ~(0xffu << sh)) | ((v & 0xffu) << sh);
}
DEV uint32_t add8(uint32_t x, uint32_t y) {                // byte-wise x + y, each byte mod 256
  return ((x & 0x7f7f7f7fu) + (y & 0x7f7f7f7fu)) ^ ((x ^ y) & 0x80808080u);
}
DEV uint32_t fsh8(uint32_t hi, uint32_t lo, int nb) {      // bytes nb .. nb+3 of the pair lo:hi
  return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)nb);
}
DEV uint32_t bcast8(uint32_t v) { return __builtin_amdgcn_perm(0u, v, 0u); }   // byte 0 x 4
DEV uint32_t sum8(uint32_t x, uint32_t acc) { return __builtin_amdgcn_sad_u8(x, 0u, acc); }

template <int LO, int HI>                                  // byte index in [LO, HI]
DEV uint32_t dk_getv(const uint32_t *d, int b) {
  const int q = b >> 2;
  uint32_t w = 0;
#pragma unroll
  for (int k = LO >> 2; k <= (HI >> 2); k++) w = k == q ? d[k] : w;
  return (w >> (8 * (b & 3))) & 0xffu;
}
template <int LO, int HI>
DEV void dk_addv(uint32_t *d, int b, uint32_t delta) {
  const int q = b >> 2;
  const uint32_t sh = 8 * (b & 3), m = 0xffu << sh;
#pragma unroll
  for (int k = LO >> 2; k <= (HI >> 2); k++) {
    const uint32_t t = ((d[k] + (delta << sh)) & m) | (d[k] & ~m);
    d[k] = k == q ? t : d[k];
  }
}
template <int BASE>
DEV uint32_t pile_get(const uint32_t *d, int c) { return dk_getv<BASE, BASE + 20>(d, BASE + c); }
template <int BASE>
DEV void pile_add(uint32_t *d, int c, uint32_t delta) { dk_addv<BASE, BASE + 20>(d, BASE + c, delta); }

// c = number of k in [0, 21) whose prefix sum pile[0] + .. + pile[k] <= t: the index the
// reference's draw-pile scan stops at (cards.cpp:196-201) while the pile holds more than t
template <int BASE>
DEV uint32_t pile_scan(const uint32_t *d, uint32_t t) {
  uint32_t s = 0, c = 0;
#pragma unroll
  for (int k = 0; k < COG_N_CARDTYPES; k++) {
    s += dk_get(d, BASE + k);
    c += s <= t ? 1u : 0u;
  }
  return c;
}

struct PState {                       // PlayerPriv unpacked (player.h:60-75, cards.h:137-145)
  uint32_t has_won, mip, n_removes, next_card_free, next_move_free, n_in_hand, n_active, n_in_draw;
  uint32_t idx_last, steps_taken, n_added_cards, pad, n_movements;
};
DEV PState unpack_player(const uint4 &v) {
  PState P;
  P.has_won = v.x & 0xffu; P.mip = (v.x >> 8) & 0xffu; P.n_removes = (v.x >> 16) & 0xffu; P.next_card_free = v.x >> 24;
  P.next_move_free = v.y & 0xffu; P.n_in_hand = (v.y >> 8) & 0xffu; P.n_active = (v.y >> 16) & 0xffu; P.n_in_draw = v.y >> 24;
  P.idx_last = v.z & 0xffu; P.steps_taken = (v.z >> 8) & 0xffu; P.n_added_cards = (v.z >> 16) & 0xffu; P.pad = v.z >> 24;
  P.n_movements = v.w;
  return P;
}
DEV uint32_t b4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return (a & 0xffu) | (b & 0xffu) << 8 | (c & 0xffu) << 16 | (d & 0xffu) << 24;
}
DEV uint4 pack_player(const PState &P) {
  return make_uint4(b4(P.has_won, P.mip, P.n_removes, P.next_card_free),
                    b4(P.next_move_free, P.n_in_hand, P.n_active, P.n_in_draw),
                    b4(P.idx_last, P.steps_taken, P.n_added_cards, P.pad), P.n_movements);
}
// The difference of two granules folded into one register (xor / or: 3-input bitop3 on gfx950)
// before the one compare: left to itself the compiler turns it into four compares into scalar
// masks and three scalar ors, 7 issue slots per granule of the store phase instead of 5.
DEV bool ne4(const uint4 &a, const uint4 &b) {
  uint32_t d = (a.x ^ b.x) | (a.y ^ b.y) | (a.z ^ b.z) | (a.w ^ b.w);
  asm volatile("" : "+v"(d));
  return d != 0u;
}

// shop slots with cards left (or, with the market full, the slots in the market): the shop
// mask's availability half (cards.cpp:109-121); sh4 = ObsData dwords 4..8 (the 18 shop bytes)
DEV uint32_t shop_avail_of(const uint32_t *sh4, uint32_t n_in_market, uint32_t in_market) {
  uint32_t nz = 0;
#pragma unroll
  for (int q = 0; q < 5; q++) nz |= bools4(sh4[q]) << (4 * q);
  return n_in_market < COG_MKT_SLOTS ? (nz & 0x3ffffu) : (in_market & 0x3ffffu);
}

struct RegEnv {
  // EnvPriv granules 0/1 (unpacked fields) and the Info mirror (granule 3, dword 0)
  uint32_t rng, seed, max_steps, turn_counter;
  uint32_t g1x, g1y, in_market, flags;                    // g1x: n_players n_pieces difficulty done
  uint32_t info_steps;
  PState P;                                                // acting player ag
  uint32_t na_active;                                      // n_active of the next player na
  uint2 cells_a, cells_n;                                  // neighbourhood caches of ag / na
  uint32_t sh[12];                                         // ObsData 16128..16175: phase, res, shop
  uint32_t d[28];                                          // DeckObs of ag
  Heads sel, sta, stn;                                     // selected / stored(ag) / stored(na)
  bool moved;
  uint4 g2;                                                // map bounds + locations
  uint32_t avail;                                          // shop_avail(), kept across steps
  const UidEntry *tab;                                     // the uniform's table (LDS)

  DEV uint32_t n_players() const { return g1x & 0xffu; }
  DEV uint32_t done() const { return g1x >> 24; }
  DEV uint32_t agent() const { return g1y & 0xffu; }
  DEV uint32_t n_in_market() const { return (g1y >> 8) & 0xffu; }
  DEV void set_done(uint32_t v) { g1x = (g1x & 0x00ffffffu) | (v << 24); }
  DEV void set_agent(uint32_t v) { g1y = (g1y & ~0xffu) | (v & 0xffu); }
  DEV void set_n_in_market(uint32_t v) { g1y = (g1y & ~0xff00u) | ((v & 0xffu) << 8); }
  DEV uint32_t shop_byte(int k) const {                   // dynamic k: select, no indexed registers
    const int q = 4 + (k >> 2);
    uint32_t w = 0;
#pragma unroll
    for (int x = 4; x < 9; x++) w = x == q ? sh[x] : w;
    return (w >> (8 * (k & 3))) & 0xffu;
  }

  DEV uint8_t use_cell(const uint2 &cc, int dir) {        // cached lookup (map.cpp:273-275)
    const uint32_t oob = cc.y >> 24;
    if ((oob >> dir) & 1u) flags |= F_OOB_LOOKUP;
    return (uint8_t)(dir < 4 ? (cc.x >> (8 * dir)) : (cc.y >> (8 * (dir - 4))));
  }
  DEV uint8_t use_cell_dyn(const uint2 &cc, int dir) {
    const uint32_t oob = cc.y >> 24;
    if ((oob >> dir) & 1u) flags |= F_OOB_LOOKUP;
    const uint64_t v = (uint64_t)cc.x | (uint64_t)cc.y << 32;
    return (uint8_t)(v >> (8 * dir));
  }

  // Deck::discard_all_active + discard_all_played (cards.cpp:219-232): discard += active + played,
  // four types per dword (active and played re-aligned to the discard pile's dword grid).
  // NQ = 2: the deck holds no card of type >= 8 (only dwords 0-1 of each pile's grid can change)
  template <int NQ>
  DEV void discard_all() {
    uint32_t D[6];
#pragma unroll
    for (int q = 0; q < NQ; q++)
      D[q] = add8(add8(d[21 + q], fsh8(d[11 + q], d[10 + q], 2)), fsh8(d[16 + q], d[15 + q], 3));
#pragma unroll
    for (int q = 0; q < NQ && q < 5; q++) d[21 + q] = D[q];
    if (NQ == 6) d[26] = (d[26] & 0xffffff00u) | (D[5] & 0xffu);   // discard[20]; bytes 105.. are padding
    d[10] &= 0x0000ffffu;                                  // active[0..1] ..
#pragma unroll
    for (int q = 11; q < 21; q++)                          // .. played[20]: bytes 42..83 = 0
      if (NQ == 6 || q == 11 || q == 12 || q == 15 || q == 16 || q == 17) d[q] = 0u;
  }
  // Deck::move_discard_to_draw (cards.cpp:234-240): both piles start on a dword
  template <int NQ>
  DEV void move_discard_to_draw() {
    uint32_t n = P.n_in_draw;
#pragma unroll
    for (int q = 0; q < NQ && q < 5; q++) {
      n = sum8(d[21 + q], n);
      d[q] = add8(d[q], d[21 + q]);
      d[21 + q] = 0u;
    }
    if (NQ == 6) {
      const uint32_t last = d[26] & 0xffu;                 // discard[20] -> draw[20]
      d[5] = (d[5] & 0xffffff00u) | ((d[5] + last) & 0xffu);
      d[26] &= 0xffffff00u;
      n += last;
    }
    P.n_in_draw = n & 0xffu;
  }
  DEV uint32_t hand_bits() const {                         // hand[k] > 0 for k < 21
    uint32_t h = 0;
#pragma unroll
    for (int q = 0; q < 6; q++) h |= bools4(fsh8(d[6 + q], d[5 + q], 1)) << (4 * q);
    return h & 0x1fffffu;
  }
  DEV void enable_playing() {                              // player.cpp:198-206
    const uint32_t h = hand_bits();
    sel.rem = 1u;
    sel.play = 1u | (h << 1);
    sel.spec = 1u | ((h & kSpecialBits) << 1);
  }
  // the pile back from its prefix sums (nondecreasing bytes < 128: no borrows), and the drawn
  // counts (old pile - new pile, no borrows either) added to the hand: byte k of the draw
  // pile's dword grid is hand byte 21 + k.  The selected mask gains the drawn types (its
  // play_special bits only ever hold special types, so setting is all the reference's
  // per-card assignment does).  Only the first NQ dwords of the pile can hold cards.
  template <int NQ>
  DEV void draw_rebuild(const uint32_t pre[6], uint32_t dm) {
    uint32_t h[6] = {0u, 0u, 0u, 0u, 0u, 0u}, prevp = 0;
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const uint32_t nd = pre[q] - fsh8(pre[q], prevp, 3);   // p[k] - p[k-1]
      prevp = pre[q];
      if (q < 5) {
        h[q] = d[q] - nd;
        d[q] = nd;
      } else {
        h[5] = (d[5] - nd) & 0xffu;
        d[5] = (d[5] & 0xffffff00u) | (nd & 0xffu);
      }
    }
#pragma unroll
    for (int q = 0; q < 6 && q <= NQ; q++) d[5 + q] = add8(d[5 + q], fsh8(h[q], q ? h[q - 1] : 0u, 3));
    sel.play |= dm << 1;
    sel.spec |= (dm & kSpecialBits) << 1;
  }
  // Deck::draw (cards.cpp:183-211).  n_in_draw == sum(draw[]) mod 256 (every Deck operation keeps
  // it), so the scan for the t-th card ends inside the pile.  While the pile holds < 128 cards
  // (always in valid play) the scan runs on byte-wise prefix sums, four types per dword: the card
  // is the number of types whose prefix sum is <= t.  Otherwise -- stale-mask driving can wrap a
  // count to 255 (Q23) -- card by card, as the reference scans (the guard only raises the flag).
  //
  // NQ = 2: the deck holds no card of type >= 8 (the wave's `wide` ballot at the end of the turn,
  // from the per-player flag a purchase of such a card sets): only dwords 0-1 of the pile grid
  // are scanned -- the types above hold prefix sums equal to the pile total, never drawn and never
  // changed.  Results are the same either way.
  template <int NQ>
  DEV void draw(uint32_t n) {
    if (P.n_in_draw < n) move_discard_to_draw<NQ>();
    if (n > P.n_in_draw) n = P.n_in_draw;
    draw_n<NQ>(n);
    P.n_in_hand = (P.n_in_hand + n) & 0xffu;
  }
  template <int NQ>
  DEV void draw_fast(uint32_t pre[6], uint32_t n, uint32_t K0, const uint32_t xs[COG_HAND_SIZE],
                     const UidEntry ue[COG_HAND_SIZE]) {
    constexpr uint32_t NT = NQ < 6 ? 4 * NQ : COG_N_CARDTYPES;   // types covered
    uint32_t dm = 0;                                     // types drawn
#pragma unroll
    for (int j = 0; j < COG_HAND_SIZE; j++) {
      const uint32_t live = (uint32_t)j < n ? 0x80808080u : 0u;
      const uint32_t T = bcast8(uid_tab_accepted(xs[j] - 1u, ue[j].s, ue[j].m) + 1u);
      uint32_t above = 0;                                // as below
#pragma unroll
      for (int q = 0; q < NQ; q++) {
        const uint32_t g = ((pre[q] | 0x80808080u) - T) & (q < 5 ? live : (live & 0x80u));
        above += __popc(g);
        pre[q] -= g >> 7;
      }
      dm |= live ? 1u << (NT - above) : 0u;
    }
    uint32_t x = rng;                                      // the state after the n-th draw: selects,
    x = n >= 1u ? xs[0] : x;                               // no branches
    x = n >= 2u ? xs[1] : x;
    x = n >= 3u ? xs[2] : x;
    rng = n >= 4u ? xs[3] : x;
    P.n_in_draw = (K0 - n) & 0xffu;
    draw_rebuild<NQ>(pre, dm);
  }
  template <int NQ>
  DEV void draw_n(uint32_t n) {
    constexpr uint32_t NT = NQ < 6 ? 4 * NQ : COG_N_CARDTYPES;   // types covered
    // pre[q] byte j: draw[0] + .. + draw[4q+j].  The in-dword prefix sums take byte shifts
    // (alignbyte: kept from being fused into quarter-rate multiplies by 0x01010101); the running
    // total before dword q (exact, no u8 wrap) is a separate chain of byte-sum adds.
    uint32_t pre[6], carry = 0;
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const uint32_t x = q < 5 ? d[q] : (d[5] & 0xffu);
      const uint32_t p1 = x + fsh8(x, 0u, 3);              // x + (x << 8)
      pre[q] = p1 + fsh8(p1, 0u, 2) + bcast8(carry);       // + (p1 << 16)
      carry = sum8(x, carry);
    }
    const uint32_t total = carry;                          // pile total
    // The draws' generator states are jumped to independently (x 16807^j): with every draw's
    // value below kSmallSafe (no rejection for any pile of <= 31) they are the states the
    // sequential draws reach, and the n uniforms need no serial chain.  n <= COG_HAND_SIZE.
    const uint32_t K0 = P.n_in_draw;
    UidEntry ue[COG_HAND_SIZE];                            // the draws' table entries, read first:
#pragma unroll                                             // the LDS reads overlap the jumps below
    for (int j = 0; j < COG_HAND_SIZE; j++) ue[j] = tab[min(max(K0 - (uint32_t)j, 1u), 31u)];
    __builtin_amdgcn_sched_barrier(0);                     // (kept ahead of the jumps: the
    uint32_t xs[COG_HAND_SIZE];                            // scheduler sinks loads to their use)
    bool seq = K0 > 31u || n > (uint32_t)COG_HAND_SIZE;
#pragma unroll
    for (int j = 0; j < COG_HAND_SIZE; j++) {
      xs[j] = mr_jump(rng, mr_pow(j + 1));
      seq |= (uint32_t)j < n && xs[j] - 1u >= kSmallSafe;
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool fast = total == P.n_in_draw && total < 128u && !seq;
    if (fast) {
      draw_fast<NQ>(pre, n, K0, xs, ue);
    } else if (total == P.n_in_draw && total < 128u) {     // every prefix sum fits in 7 bits
      uint32_t dm = 0;                                     // types drawn
      for (uint32_t i = 0; i < n; i++) {
        const uint32_t k = P.n_in_draw;                    // piles of <= 31: division-free draw
        const uint32_t T = bcast8((k <= 31u ? uid_small(rng, k) : uid_fast(rng, k)) + 1u);
        uint32_t above = 0;                                // types whose prefix sum is > t: bit 7
#pragma unroll                                             // of (0x80 + p) - (t + 1), no borrows;
        for (int q = 0; q < NQ; q++) {                     // they are the types >= the drawn card
          const uint32_t g = ((pre[q] | 0x80808080u) - T) & (q < 5 ? 0x80808080u : 0x80u);
          above += __popc(g);
          pre[q] -= g >> 7;                                // (>= 1 there: no borrow)
        }
        P.n_in_draw = (k - 1u) & 0xffu;
        dm |= 1u << (NT - above);
      }
      draw_rebuild<NQ>(pre, dm);
    } else {
      P.pad = 1u;                                          // the deck's "wide" flag (see draw)
      for (uint32_t i = 0; i < n; i++) {
        const uint32_t t = uid_fast(rng, P.n_in_draw);
        uint32_t c = pile_scan<COG_DECK_DRAW>(d, t);
        if (c >= COG_N_CARDTYPES) {
          flags |= F_SCAN_OVER;
          c = COG_N_CARDTYPES - 1;
        }
        pile_add<COG_DECK_DRAW>(d, (int)c, 0xffu);
        P.n_in_draw = (P.n_in_draw - 1) & 0xffu;
        pile_add<COG_DECK_HAND>(d, (int)c, 1u);
        sel.play |= 1u << (c + 1);
        sel.spec = set_bit(sel.spec, (int)c + 1, is_special((int)c));
      }
    }
  }
  // card c leaves the hand (Deck::activate / play_immediate / remove_immediate, cards.cpp:242-290)
  DEV void leave_hand(int c, bool rem_rule) {
    const uint32_t prev = pile_get<COG_DECK_HAND>(d, c);
    pile_add<COG_DECK_HAND>(d, c, 0xffu);
    P.n_in_hand = (P.n_in_hand - 1) & 0xffu;
    const uint32_t b = 1u << (c + 1);
    bool pl = prev > 1;
    if (rem_rule) {
      if (!pl) sel.rem &= ~b;
      pl = pl && (sel.play & b);
    }
    sel.play = pl ? (sel.play | b) : (sel.play & ~b);
    sel.spec = (pl && is_special(c)) ? (sel.spec | b) : (sel.spec & ~b);
  }
  // Player::cards_from_active (player.cpp:85-131): n random cards leave the active pile; the
  // reference's scan (cards.cpp:196-201) may run past the pile on an inconsistent deck
  DEV void take_from_active(uint32_t n, bool discard) {
    const uint32_t avail = P.n_active;
    P.pad = 1u;                                            // the deck's "wide" flag (see draw)
    if (n > avail) {
      if (discard) flags |= F_Q24_CLAMP;
      n = avail;
    }
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t t = uid_fast(rng, avail - i);
      uint32_t s = 0, c = 0;
#pragma unroll
      for (int k = COG_DECK_ACTIVE; k < 105; k++) {
        s += dk_get(d, k);
        c += s <= t ? 1u : 0u;
      }
      if (COG_DECK_ACTIVE + c >= 105) flags |= F_SCAN_OVER;
      P.n_active = (P.n_active - 1) & 0xffu;
      dk_addv<COG_DECK_ACTIVE, 105>(d, COG_DECK_ACTIVE + (int)c, 0xffu);
      if (discard) dk_addv<COG_DECK_DISCARD, COG_DECK_DISCARD + 20>(d, COG_DECK_DISCARD + (int)c, 1u);
    }
  }
  // movement mask bits 1..6 (map.cpp:369-387) + bit 0, from a player's cached neighbourhood.
  // A hex code's low 6 bits are req * 8 + n.  The largest n each requirement meets is
  // floor(resource) for machete / paddle / coin (r >= n, n integer) and n_active - 1 for discard
  // / remove (n_active > n; codes 6 and 7 compare like them), none for NULL; so the hexes that
  // can be entered form one 64-bit set over (req, n), tested once per neighbour.
  DEV uint32_t move_bits(const uint2 &cc, float r0, float r1, float r2, uint32_t n_active) {
    if ((cc.y >> 24) & 0x7eu) flags |= F_OOB_LOOKUP;      // the lookups of cells 1..6
    auto width = [](float r) {                             // n in [0, width) is met by r >= n
      return (uint32_t)__builtin_amdgcn_fmed3f(floorf(r) + 1.f, 0.f, 8.f);
    };
    const uint32_t wa = min(n_active, 8u);
    const uint32_t lo = __builtin_amdgcn_ubfe(0xffu, 0, width(r0)) | __builtin_amdgcn_ubfe(0xffu, 0, width(r1)) << 8 |
                        __builtin_amdgcn_ubfe(0xffu, 0, width(r2)) << 16 | __builtin_amdgcn_ubfe(0xffu, 0, wa) << 24;
    const uint32_t ha = __builtin_amdgcn_ubfe(0xffu, 0, wa);
    const uint64_t ok = (uint64_t)lo | (uint64_t)(ha | ha << 16 | ha << 24) << 32;   // req 4, 6, 7
    uint32_t m = 1u;
#pragma unroll
    for (int dir = 1; dir < 7; dir++) {
      const uint32_t idx = (dir < 4 ? cc.x >> (8 * dir) : cc.y >> (8 * (dir - 4))) & 0x3fu;
      m |= (uint32_t)((ok >> idx) & 1u) << dir;
    }
    return m;
  }
  // shop mask bits 1..18 (cards.cpp:109-121) + bit 0
  DEV uint32_t shop_avail() const { return shop_avail_of(sh + 4, n_in_market(), in_market); }
  // shop mask bits from `avail`, the cached shop_avail() (it changes only with a purchase)
  DEV uint32_t shop_bits(float coins) const {
    const uint32_t afford = (coins > 1.f ? kCostMask1 : 0u) | (coins > 2.f ? kCostMask2 : 0u) |
                            (coins > 3.f ? kCostMask3 : 0u) | (coins > 4.f ? kCostMask4 : 0u) |
                            (coins > 5.f ? kCostMask5 : 0u);
    return 1u | ((avail & afford) << 1);
  }
  // Player::end_turn's deck part (player.cpp:170-180, cards.cpp:219-232,183-211): discard the
  // active and played piles, draw up to the hand size.  NQ by the wave's `wide` ballot (see draw).
  DEV void end_turn_deck() {
    const int n_draw = COG_HAND_SIZE - (int)P.n_in_hand;
    if (__builtin_amdgcn_ballot_w64(P.pad != 0u)) {        // a deck of the wave holds a type >= 8
      discard_all<6>();
      if (n_draw > 0) draw<6>((uint32_t)n_draw);
    } else {
      discard_all<2>();
      if (n_draw > 0) draw<2>((uint32_t)n_draw);
    }
  }
  // special actions (cards.cpp:8-36, the remove lambda environment.cpp:156-158) on the stored
  // mask `m` of the current agent and the selected mask, for the acting player (:183-186)
  DEV void apply_special(int special, Heads &m) {
    switch (special) {
      case COG_SPECIAL_DRAW2:
      case COG_SPECIAL_DRAW3: draw<6>(special == COG_SPECIAL_DRAW2 ? 2u : 3u); break;
      case COG_SPECIAL_DRAW1_REMOVE1:
      case COG_SPECIAL_DRAW2_REMOVE2: {
        const uint32_t k = special == COG_SPECIAL_DRAW1_REMOVE1 ? 1u : 2u;
        draw<6>(k);
        P.n_removes = k;
        m.rem = m.play;                                    // mask.remove = mask.play
        sel.play = 1u;                                     // disable_playing
        sel.spec = 1u;
        m.shop &= 1u;                                      // shop_mask(0): nothing affordable
      } break;
      case COG_SPECIAL_TRANSMIT: {
        m.move = 1u;
        sel.play = 1u;
        sel.spec = 1u;
        uint32_t nz = 0;
#pragma unroll
        for (int q = 0; q < 5; q++) nz |= bools4(sh[4 + q]) << (4 * q);
        m.shop = (m.shop & 1u) | ((nz & 0x3ffffu) << 1);
        P.next_card_free = 1;
      } break;
      case COG_SPECIAL_NATIVE: {
        uint32_t mb = m.move & 1u;
#pragma unroll
        for (int dir = 1; dir < 7; dir++)                  // movement_mask with 100 of everything
          if (COG_HEX_REQ(use_cell(cells_a, dir)) != COG_REQ_NULL) mb |= 1u << dir;
        m.move = mb;
        P.next_move_free = 1;
        sel.play = 1u;
        sel.spec = 1u;
        m.shop &= 1u;
      } break;
      case COG_SPECIAL_SHOP_OFF: m.shop &= 1u; break;
      default: break;
    }
  }
};

// the mover's new neighbourhood (load_cells on registers + the compact code grid)
// COG_DIRS_XY2 / 2 + 1 as 2-bit fields (direction d at bits 2d): no constant-memory load
constexpr uint32_t dir_pack(int axis) {
  const int8_t v[7][2] = COG_DIRS_XY2;
  uint32_t r = 0;
  for (int d = 0; d < 7; d++) r |= (uint32_t)(v[d][axis] / 2 + 1) << (2 * d);
  return r;
}
DEV int dir_dx(int d) { return (int)((dir_pack(0) >> (2 * d)) & 3u) - 1; }
DEV int dir_dy(int d) { return (int)((dir_pack(1) >> (2 * d)) & 3u) - 1; }

// The 7 cells lie on 3 grid rows (x - 1 .. x + 1), 3 consecutive bytes each from column y - 1:
// one 8-byte load per row from a dword-aligned start (48 is a multiple of 4, so every row has
// the same alignment offset, <= 3, and the 3 bytes fit in the 8).  A start is clamped into the
// env's grid, which only moves the windows of cells that are masked below anyway.
// cell_rows issues the three loads; rows_ready takes all three windows at once through an empty
// asm, so the loads stay back to back and in flight until the cells are needed (under register
// pressure the scheduler otherwise serialises per-cell loads).  rows_ready runs in converged
// control flow: the wait for the loads then sits on every path, and no later write of those
// registers (the store phase reuses them) needs a conservative vmcnt(0) behind the stores.
DEV int row_start(int ix, int iy0) { return min(max((ix * COG_GRID + iy0 - 1) & ~3, 0), COG_CELLS - 8); }
struct CellRows {
  uint32_t w[6];
  int ix0, iy0;                                            // the centre in grid indices
};
DEV CellRows cell_rows(const uint8_t *cgrid, const uint4 &g2, int lx, int ly) {
  CellRows c;
  c.ix0 = lx - (int8_t)(g2.x & 0xffu) + 1;
  c.iy0 = ly - (int8_t)((g2.x >> 8) & 0xffu) + 1;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(cgrid + row_start(c.ix0 + r - 1, c.iy0));
    c.w[2 * r] = p[0];
    c.w[2 * r + 1] = p[1];
  }
  return c;
}
DEV void rows_ready(CellRows &c) {
  asm volatile("" : "+v"(c.w[0]), "+v"(c.w[1]), "+v"(c.w[2]), "+v"(c.w[3]), "+v"(c.w[4]), "+v"(c.w[5]));
}
DEV uint2 cells_from_rows(const CellRows &c, const uint4 &g2) {
  const int dimx = g2.y & 0xffu, dimy = (g2.y >> 8) & 0xffu;
  const int ix0 = c.ix0, iy0 = c.iy0;
  const uint32_t *w = c.w;
  uint32_t v[7], oob = 0;
#pragma unroll
  for (int dir = 0; dir < 7; dir++) {
    const int dx = dir_dx(dir), ix = ix0 + dx, iy = iy0 + dir_dy(dir);
    const bool out_ = ix < 0 || iy < 0 || ix >= dimx || iy >= dimy;
    const bool ring = ix >= COG_GRID || iy >= COG_GRID;
    const uint64_t row = (uint64_t)w[2 * (dx + 1) + 1] << 32 | w[2 * (dx + 1)];
    const int pos = ix * COG_GRID + iy - row_start(ix, iy0);   // 0..7 for every unmasked cell
    const uint32_t c = (uint32_t)(row >> (8 * (pos & 7))) & 0xffu;
    v[dir] = (out_ || ring || !c) ? (uint32_t)COG_HEX_MOUNTAIN : c;
    oob |= (out_ ? 1u : 0u) << dir;
  }
  return make_uint2(v[0] | v[1] << 8 | v[2] << 16 | v[3] << 24, v[4] | v[5] << 8 | v[6] << 16 | oob << 24);
}

// cog_env::step (environment.cpp:91-224) for the acting player ag == agent, every action kind.
// Returns true when the episode ends (finish_episode runs on the stored state afterwards).
#if defined(COG_ABLATE_DUPENDTURN) || defined(COG_ABLATE_DUPPLAY) || defined(COG_ABLATE_DUPUPDOBS) || \
    defined(COG_ABLATE_DUPDISCARD) || defined(COG_ABLATE_DUPDRAW)
// diagnostic timing builds only: a part of the step run a second time on a laundered copy of the
// registers (results discarded), to measure its marginal cost without changing the dynamics
DEV void dup_launder(RegEnv &R2) {
#pragma unroll
  for (int k = 0; k < 28; k++) asm volatile("" : "+v"(R2.d[k]));
  asm volatile("" : "+v"(R2.rng), "+v"(R2.P.n_in_hand), "+v"(R2.P.n_in_draw), "+v"(R2.sel.play), "+v"(R2.sel.spec));
}
DEV void dup_sink(const RegEnv &R2) {
  uint32_t x = R2.rng ^ R2.P.n_in_hand ^ R2.P.n_in_draw ^ R2.sel.play ^ R2.sel.spec ^ R2.P.n_active;
#pragma unroll
  for (int k = 0; k < 28; k++) x ^= R2.d[k];
  asm volatile("" ::"v"(x));
}
#endif

DEV bool step_regs(RegEnv &R, const uint8_t act[5], const DevState &s, size_t i, int na PH_PARAM) {
  const int ag = (int)R.agent();
  PState &P = R.P;
  const uint32_t info = ((R.info_steps >> (8 * ag)) + 1u) & 0xffu;   // Info steps_taken (u8):
  R.info_steps = (R.info_steps & ~(0xffu << (8 * ag))) | (info << (8 * ag));   // stored with the outputs
  uint32_t phase = R.sh[0] & 0xffu;
  if (phase == COG_PHASE_INACTIVE) phase = COG_PHASE_MOVEMENT;
  P.steps_taken = (P.steps_taken + 1) & 0xffu;
  float r0 = __uint_as_float(R.sh[1]), r1 = __uint_as_float(R.sh[2]), r2 = __uint_as_float(R.sh[3]);
  const int a_play = act[0], a_special = act[1], a_remove = act[2], a_move = act[3], a_shop = act[4];
  // the deck's "wide" flag (sticky): set by any action naming a card type >= 8 (a valid one names a
  // card the deck holds; an invalid one -- stale masks, host actions -- may create the type by u8
  // wrap-around), by a purchase of such a type, and by the scans that can run past a pile
  if (max(max(a_play, a_special), a_remove) > 8) P.pad = 1u;
  int special = COG_SPECIAL_NONE;
  // A wave whose lanes only play cards or pass, with no free move / free card / pending removes
  // / move in progress (all of the canonical selected-mask loop), takes the short
  // path: one uniform branch instead of one divergent skip per action kind.
  const bool rare = (a_special | a_remove | a_move | a_shop) != 0 ||
                    (P.next_move_free | P.next_card_free | P.n_removes | P.mip) != 0u;
  const bool wave_simple = !__builtin_amdgcn_ballot_w64(rare);
  auto play_card = [&](int c) {                            // Player::play_card (player.cpp:45-60)
#ifdef COG_ABLATE_DUPPLAY
    { RegEnv R2 = R; dup_launder(R2); R2.leave_hand(c, false); pile_add<COG_DECK_ACTIVE>(R2.d, c, 1u); dup_sink(R2); }
#endif
    if (phase == COG_PHASE_MOVEMENT) {
      r0 = (float)cardf(kRes0, c); r1 = (float)cardf(kRes1, c); r2 = (float)cardf(kRes2, c);
    } else if (phase == COG_PHASE_BUYING) {
      const uint32_t coin = cardf(kRes2, c);
      r2 = r2 + (coin > 0 ? (float)coin : 0.5f);
    }
    R.leave_hand(c, false);                                // Deck::activate
    pile_add<COG_DECK_ACTIVE>(R.d, c, 1u);
    P.n_active = (P.n_active + 1) & 0xffu;
    P.idx_last = (uint32_t)c;
  };
  CellRows moved_rows = {};
  if (wave_simple) {
    if (a_play) play_card(a_play - 1);
    else phase = (phase + 1) % 3;                          // pass: next phase
  } else {
    if (a_move && !a_play && !a_special) {                   // the destination's neighbourhood: its
      const int lx = (int8_t)((R.g2.z >> (8 * ag)) & 0xffu) + dir_dx(a_move);   // loads are issued
      const int ly = (int8_t)((R.g2.w >> (8 * ag)) & 0xffu) + dir_dy(a_move);   // first, used last
      R.g2.z = (R.g2.z & ~(0xffu << (8 * ag))) | (((uint32_t)lx & 0xffu) << (8 * ag));
      R.g2.w = (R.g2.w & ~(0xffu << (8 * ag))) | (((uint32_t)ly & 0xffu) << (8 * ag));
      moved_rows = cell_rows(s.cgrid + i * COG_CELLS, R.g2, lx, ly);
    }
    if (a_play) {
      play_card(a_play - 1);
    } else if (a_special) {                                  // play_special (environment.cpp:108-114)
      const int c = a_special - 1;
      const bool single = cardf(kSingle, c) != 0u;
      R.leave_hand(c, single);                               // remove_immediate / play_immediate
      if (!single) pile_add<COG_DECK_PLAYED>(R.d, c, 1u);
      special = (int)cardf(kSpecial, c);
    } else if (a_move) {                                     // move (environment.cpp:115-127)
      const uint32_t c = R.use_cell_dyn(R.cells_a, a_move);
      if (!P.next_move_free) {                               // Player::handle_requirement (:141-162)
        const uint32_t req = COG_HEX_REQ(c), n = COG_HEX_N(c);
        if (req < 3) {
          const float left = (req == 0 ? r0 : req == 1 ? r1 : r2) - (float)n;
          r0 = req == 0 ? left : 0.f;
          r1 = req == 1 ? left : 0.f;
          r2 = req == 2 ? left : 0.f;
          if (!P.mip) {                                      // Deck::play_last_activated
            const int l = (int)P.idx_last;
            P.n_active = (P.n_active - 1) & 0xffu;
            dk_addv<COG_DECK_ACTIVE, 105>(R.d, COG_DECK_ACTIVE + l, 0xffu);
            if (!cardf(kSingle, l)) dk_addv<COG_DECK_PLAYED, 105>(R.d, COG_DECK_PLAYED + l, 1u);
            P.mip = 1;
          }
        } else if (req == COG_REQ_REMOVE || req == COG_REQ_DISCARD) {
          R.take_from_active(n, req == COG_REQ_DISCARD);
          r0 = r1 = r2 = 0.f;
          P.mip = 0;
        }
      } else {
        P.next_move_free = 0;
        R.enable_playing();
      }
      P.n_movements++;
      P.has_won = COG_HEX_END(c);
      R.moved = true;
    } else {
      P.next_move_free = 0;
      if (a_shop) {                                          // Shop::get_card (cards.cpp:123-142)
        const int k = a_shop - 1;
        const int ty = shop_type(k);
        const uint32_t bit = 1u << k;
        uint32_t nim = R.n_in_market();
        if (!P.next_card_free) {
          nim = (nim + ((R.in_market & bit) ? 0u : 1u)) & 0xffu;
          R.in_market |= bit;
        }
        const uint32_t left = (R.shop_byte(k) - 1u) & 0xffu;
        const int q = 4 + (k >> 2), sh8 = 8 * (k & 3);
  #pragma unroll
        for (int w = 4; w < 9; w++)
          if (w == q) R.sh[w] = (R.sh[w] & ~(0xffu << sh8)) | (left << sh8);
        if (!left && (R.in_market & bit)) {
          R.in_market &= ~bit;
          nim = (nim - 1u) & 0xffu;
        }
        R.set_n_in_market(nim);
        R.avail = R.shop_avail();                            // (after the market bookkeeping)
        if (!P.next_card_free) {
          r2 = r2 - (float)cardf(kCost, ty);
          phase = (phase + 1) % 3;
        }
        pile_add<COG_DECK_DISCARD>(R.d, ty, 1u);
        if (ty >= 8) P.pad = 1u;                             // the deck's "wide" flag (see draw)
        P.n_added_cards = (P.n_added_cards + 1) & 0xffu;
      } else if (a_remove) {
        const int c = a_remove - 1;
        R.leave_hand(c, true);                               // Deck::remove_immediate
        P.n_removes = (P.n_removes - 1) & 0xffu;
        if (!P.n_removes) R.enable_playing();
        else special = COG_SPECIAL_SHOP_OFF;
      } else {                                               // pass: next phase
        phase = (phase + 1) % 3;
        if (P.n_removes > 0) {
          P.n_removes = 0;
          R.enable_playing();
        }
      }
      if (P.next_card_free) {
        P.next_card_free = 0;
        R.enable_playing();
      }
    }
  }
  PH(8);
  if (!wave_simple && P.mip && !a_move) {                  // the move HEAD, whatever was taken
    P.mip = 0;
    r0 = r1 = r2 = 0.f;
  }
  bool cur_is_ag = true;
  if (P.has_won || phase == COG_PHASE_INACTIVE) {          // maybe_end_turn -> next_agent
#if defined(COG_ABLATE_DUPENDTURN) || defined(COG_ABLATE_DUPDISCARD) || defined(COG_ABLATE_DUPDRAW)
    {
      RegEnv R2 = R;
      dup_launder(R2);
      const int nd2 = COG_HAND_SIZE - (int)R2.P.n_in_hand;
      if (__builtin_amdgcn_ballot_w64(R2.P.pad != 0u)) {
#ifndef COG_ABLATE_DUPDRAW
        R2.discard_all<6>();
#endif
#ifndef COG_ABLATE_DUPDISCARD
        if (nd2 > 0) R2.draw<6>((uint32_t)nd2);
#endif
      } else {
#ifndef COG_ABLATE_DUPDRAW
        R2.discard_all<2>();
#endif
#ifndef COG_ABLATE_DUPDISCARD
        if (nd2 > 0) R2.draw<2>((uint32_t)nd2);
#endif
      }
      dup_sink(R2);
    }
#endif
    P.n_active = 0;                                        // Player::end_turn (player.cpp:170-180)
    PH(9);
    R.end_turn_deck();
    PH(10);
    R.sta = R.sel;                                         // save_actionmask
    R.set_agent((uint32_t)na);
    if (na == ag) R.sel = R.sta;                           // load_actionmask
    else {
      R.sel = R.stn;
      cur_is_ag = false;
    }
    r0 = r1 = r2 = 0.f;
    R.turn_counter++;
  }
  R.sh[0] = (R.sh[0] & ~0xffu) | phase;
  R.sh[1] = __float_as_uint(r0); R.sh[2] = __float_as_uint(r1); R.sh[3] = __float_as_uint(r2);
#ifndef COG_ABLATE_ROWS                                    // diagnostic timing builds only
  // on every path, converged: the wait for the rows then sits where no store of this step is
  // outstanding yet (the step's stores all come after it), and no later reuse of the row
  // registers needs a conservative vmcnt wait -- which would wait for this step's stores
  rows_ready(moved_rows);
#endif
  if (!wave_simple && R.moved) {                           // the mover's new neighbourhood
    R.cells_a = cells_from_rows(moved_rows, R.g2);
    if (na == ag) R.cells_n = R.cells_a;
  }
  PH(11);
  const uint2 cc = cur_is_ag ? R.cells_a : R.cells_n;
  Heads &stc = cur_is_ag ? R.sta : R.stn;
  uint32_t mv = 1u, sp = 1u;                               // update_observation (:252-279)
#ifndef COG_ABLATE_UPDOBS                                  // diagnostic timing builds only
  if (phase == COG_PHASE_MOVEMENT) mv = R.move_bits(cc, r0, r1, r2, cur_is_ag ? P.n_active : R.na_active);
  else if (phase == COG_PHASE_BUYING) sp = R.shop_bits(r2);
#endif
#ifdef COG_ABLATE_DUPUPDOBS
  { RegEnv R2 = R; float q0 = r0, q1 = r1, q2 = r2; uint2 c2 = cc; uint32_t na2 = cur_is_ag ? P.n_active : R.na_active;
    asm volatile("" : "+v"(q0), "+v"(q1), "+v"(q2), "+v"(c2.x), "+v"(c2.y), "+v"(na2), "+v"(R2.avail));
    uint32_t m2 = 1u, s2 = 1u;
    if (phase == COG_PHASE_MOVEMENT) m2 = R2.move_bits(c2, q0, q1, q2, na2);
    else if (phase == COG_PHASE_BUYING) s2 = R2.shop_bits(q2);
    asm volatile("" ::"v"(m2 ^ s2 ^ R2.flags)); }
#endif
  stc.move = mv;
  stc.shop = sp;
  PH(12);
  if (!wave_simple && special != COG_SPECIAL_NONE) {
    R.apply_special(special, stc);
    return false;
  }
  const uint32_t c0 = R.use_cell(cc, 0);                   // done check (:187)
  return COG_HEX_END(c0) || R.turn_counter >= R.max_steps;
}

// The trio's step (k_env_rollout_trio, trio_stepper's loop): cog_env::step (environment.cpp:91-224)
// for an action that plays a card or passes, by a player with no move, free card, free move or
// pending removes in progress and who has not won (lean_player) -- every step of the canonical
// selected-mask loop; any other env is parked before its step (kParkRedo) and run by
// the full step.  Three parts of the reference's step are left to the other waves: the deck's piles
// other than the hand (the drawing wave replays the play on its copy of the deck, trio_drawer), the
// turn end's discard + draws (the drawing wave too) and update_observation's movement / shop heads
// of the acting player's stored mask when the turn goes on -- with the selected masks nothing reads
// those heads but the output record (save_actionmask replaces them at the turn end), so the storing
// wave computes them from the step record (trio_storer).  At a turn end the new agent's stored
// mask gets update_observation's values for the INACTIVE phase (move = shop = {0}) in the stepper.

// ---- lane drivers ---------------------------------------------------------------------------
// Snap: the step-start image of everything a step may modify; the store phase writes back the
// 16-B granules that differ from it (and nothing else).
struct Snap {
  uint4 g0, g1, g2;                   // EnvPriv granules 0, 1, 2
  uint32_t avail;                     // shop_avail_of(sh, g1): refreshed by a purchase
  uint32_t info_steps;                // EnvPriv granule 3, dword 0
  uint4 sh[3];                        // ObsData 16128..16175: phase, resources, shop
  MBits sel;                          // selected mask
  uint4 pla, pln;                     // pl[ag], pl[na]
  uint2 ca, cn;                       // cells[ag], cells[na]
  MBits sta, stn;                     // stored masks of ag, na
  uint4 dk[7];                        // DeckObs of ag
};

DEV void load_env(const DevState &s, size_t i, Snap &S) {          // records at fixed addresses
  const uint4 *pv4 = reinterpret_cast<const uint4 *>(s.priv + i);
  const uint4 *sh4 = reinterpret_cast<const uint4 *>(s.obs + i * COG_OBS_BYTES + COG_OBS_PHASE);
  S.g0 = pv4[0];
  S.g1 = pv4[1];
  S.g2 = pv4[2];
  S.info_steps = reinterpret_cast<const uint32_t *>(pv4 + 3)[0];
  S.sel = mbits_of(s.heads[5 * i]);
  S.sh[0] = sh4[0];
  S.sh[1] = sh4[1];
  S.sh[2] = sh4[2];
  const uint32_t w[5] = {S.sh[1].x, S.sh[1].y, S.sh[1].z, S.sh[1].w, S.sh[2].x};
  S.avail = shop_avail_of(w, (S.g1.y >> 8) & 0xffu, S.g1.z);
}
DEV uint8_t *deck_ptr(const DevState &s, size_t i, int p) {
  return s.obs + i * COG_OBS_BYTES + COG_OBS_PLAYER0 + COG_OBS_PLAYER_STRIDE * p;
}
DEV void load_players(const DevState &s, size_t i, int ag, int na, Snap &S) {   // acting / next
  const uint4 *pv4 = reinterpret_cast<const uint4 *>(s.priv + i);
  S.pla = pv4[4 + ag];
  S.pln = pv4[4 + na];
  S.ca = reinterpret_cast<const uint2 *>(pv4 + 8)[ag];
  S.cn = reinterpret_cast<const uint2 *>(pv4 + 8)[na];
  S.sta = mbits_of(s.heads[5 * i + 1 + ag]);
  S.stn = mbits_of(s.heads[5 * i + 1 + na]);
  const uint4 *dk = reinterpret_cast<const uint4 *>(deck_ptr(s, i, ag));
#pragma unroll
  for (int k = 0; k < 7; k++) S.dk[k] = dk[k];
}
DEV void regs_env(RegEnv &R, const Snap &S) {
  R.rng = S.g0.x; R.seed = S.g0.y; R.max_steps = S.g0.z; R.turn_counter = S.g0.w;
  R.g1x = S.g1.x; R.g1y = S.g1.y; R.in_market = S.g1.z; R.flags = S.g1.w;
  R.info_steps = S.info_steps;
  R.g2 = S.g2;
  R.avail = S.avail;
  R.moved = false;
  R.sel = heads_of(S.sel);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    R.sh[4 * k] = S.sh[k].x; R.sh[4 * k + 1] = S.sh[k].y; R.sh[4 * k + 2] = S.sh[k].z; R.sh[4 * k + 3] = S.sh[k].w;
  }
}
DEV void regs_players(RegEnv &R, const Snap &S) {
  R.P = unpack_player(S.pla);
  R.na_active = (S.pln.y >> 16) & 0xffu;
  R.cells_a = S.ca;
  R.cells_n = S.cn;
  R.sta = heads_of(S.sta);
  R.stn = heads_of(S.stn);
#pragma unroll
  for (int k = 0; k < 7; k++) {
    R.d[4 * k] = S.dk[k].x; R.d[4 * k + 1] = S.dk[k].y; R.d[4 * k + 2] = S.dk[k].z; R.d[4 * k + 3] = S.dk[k].w;
  }
}
// ObsData record granules, and the dynamic tail (phase, resources, shop, decks, stored masks) the
// host views refresh: granules kTail0 .. kRecG - 1
constexpr size_t kRecG = COG_OBS_BYTES / 16, kTail0 = COG_OBS_MAP_BYTES / 16, kTailG = kRecG - kTail0;

// Direct publish (k_env_step_pub): a store of a host-visible record also goes to the pinned view
// and to the publish mirror (k_publish's `mir`: [n][kTailG] tail granules, then the outs block),
// which keeps both equal to HBM without a compare pass.  PUB: 0 off, 1 an ObsData tail record of
// env i, 2 a record of the outs block (status | selected masks | infos | rewards | dones | agents).
template <int PUB, class T>
DEV void pub_store(const DevState &s, size_t i, T *dev, const T &v) {
  *dev = v;
  if (PUB == 1) {
    const size_t off = (size_t)(reinterpret_cast<const uint8_t *>(dev) - s.obs);
    *reinterpret_cast<T *>(s.pub_obs + off) = v;
    *reinterpret_cast<T *>(s.pub_mir + i * (kTailG * 16) + (off - i * COG_OBS_BYTES - COG_OBS_MAP_BYTES)) = v;
  } else if (PUB == 2) {
    const size_t off = (size_t)(reinterpret_cast<const uint8_t *>(dev) - reinterpret_cast<const uint8_t *>(s.status));
    *reinterpret_cast<T *>(s.pub_outs + off) = v;
    *reinterpret_cast<T *>(s.pub_mir + s.n * (kTailG * 16) + off) = v;
  }
}
template <int PUB = 0>
DEV void store_mask_record(const DevState &s, size_t i, uint4 *rec, const MBits &b, uint32_t gm) {
#pragma unroll
  for (int g = 0; g < 6; g++)
    if ((gm >> g) & 1u) pub_store<PUB>(s, i, rec + g, mask_granule(b, g));
}
DEV void store_mask_record(uint4 *rec, const MBits &b, uint32_t gm) {
#pragma unroll
  for (int g = 0; g < 6; g++)
    if ((gm >> g) & 1u) rec[g] = mask_granule(b, g);
}
// The store phase.  Outputs -- the ObsData tail (phase / resources / shop, the acting player's
// deck, the stored masks) and the selected_action_masks record -- are stored granule by granule
// where they differ from the step-start image S, on every step.  Private state (EnvPriv, the
// mask bit vectors) is stored by the single-step kernel on every step; the rollout keeps it
// on-chip and stores it before anything reads it back (episode end, reset, end of launch).
// A move stores the new locations at once: the next move re-reads them.
template <bool PUB = false>
DEV void store_outputs(const DevState &s, size_t i, int ag, int na, const Snap &S, const RegEnv &R) {
  constexpr int PT = PUB ? 1 : 0, PO = PUB ? 2 : 0;        // (direct publish: tail / outs records)
  uint8_t *ob = s.obs + i * COG_OBS_BYTES;
  pub_store<PO>(s, i, s.info + i * COG_INFO_BYTES + COG_AGENT_INFO0 + COG_AGENT_INFO_STRIDE * ag,
                (uint8_t)(R.info_steps >> (8 * ag)));
  if (R.moved) reinterpret_cast<uint4 *>(s.priv + i)[2] = R.g2;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint4 v = make_uint4(R.sh[4 * k], R.sh[4 * k + 1], R.sh[4 * k + 2], R.sh[4 * k + 3]);
    if (ne4(v, S.sh[k])) pub_store<PT>(s, i, reinterpret_cast<uint4 *>(ob + COG_OBS_PHASE) + k, v);
  }
  uint8_t *deck = deck_ptr(s, i, ag);
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const uint4 v = make_uint4(R.d[4 * k], R.d[4 * k + 1], R.d[4 * k + 2], R.d[4 * k + 3]);
    if (ne4(v, S.dk[k])) pub_store<PT>(s, i, reinterpret_cast<uint4 *>(deck) + k, v);
  }
  const MBits bs = bits_of(R.sel), ba = bits_of(R.sta), bn = bits_of(R.stn);
  store_mask_record<PO>(s, i, reinterpret_cast<uint4 *>(s.sel + i * COG_MASK_BYTES), bs, mask_diff_granules(bs, S.sel));
  store_mask_record<PT>(s, i, reinterpret_cast<uint4 *>(deck + COG_PD_MASK), ba, mask_diff_granules(ba, S.sta));
  if (na != ag)
    store_mask_record<PT>(s, i, reinterpret_cast<uint4 *>(deck_ptr(s, i, na) + COG_PD_MASK), bn,
                          mask_diff_granules(bn, S.stn));
}
DEV void store_private(const DevState &s, size_t i, int ag, int na, const Snap &S, const RegEnv &R) {
  uint4 *pw = reinterpret_cast<uint4 *>(s.priv + i);
  const uint4 g0n = make_uint4(R.rng, R.seed, R.max_steps, R.turn_counter);
  const uint4 g1n = make_uint4(R.g1x, R.g1y, R.in_market, R.flags);
  if (ne4(g0n, S.g0)) pw[0] = g0n;
  if (ne4(g1n, S.g1)) pw[1] = g1n;
  reinterpret_cast<uint32_t *>(pw + 3)[0] = R.info_steps;  // both change on every step
  pw[4 + ag] = pack_player(R.P);
  if (R.moved) reinterpret_cast<uint2 *>(pw + 8)[ag] = R.cells_a;
  const MBits bs = bits_of(R.sel), ba = bits_of(R.sta), bn = bits_of(R.stn);
  if (mask_diff_granules(bs, S.sel)) s.heads[5 * i] = mbits_u4(bs);
  if (mask_diff_granules(ba, S.sta)) s.heads[5 * i + 1 + ag] = mbits_u4(ba);
  if (na != ag && mask_diff_granules(bn, S.stn)) s.heads[5 * i + 1 + na] = mbits_u4(bn);
}
template <bool PUB = false>
DEV void store_changes(const DevState &s, size_t i, int ag, int na, const Snap &S, const RegEnv &R) {
  store_outputs<PUB>(s, i, ag, na, S, R);
  store_private(s, i, ag, na, S, R);
}

// the action of this step: sampled (runner) or the host's (indices past a head are the
// reference's out-of-range accesses: clamped and flagged)
// (ext: MASK_EXTERNAL's ActionData bytes 0..7, loaded by the caller at the start of the step)
template <int SRC>
DEV void step_action(RegEnv &R, const uint2 &ext, uint32_t &srng, uint8_t act[5]) {
  if (SRC == MASK_SELECTED) sample_heads(R.sel, srng, act, R.tab);
  else if (SRC == MASK_STORED) sample_heads(R.sta, srng, act, R.tab);
  else {
    const uint8_t top[5] = {COG_N_CARDTYPES, COG_N_CARDTYPES, COG_N_CARDTYPES, 6, COG_N_SHOP};
#pragma unroll
    for (int k = 0; k < 5; k++) {
      act[k] = (uint8_t)((k < 4 ? ext.x >> (8 * k) : ext.y) & 0xffu);
      if (act[k] > top[k]) {
        act[k] = top[k];
        R.flags |= F_BAD_ACTION;
      }
    }
  }
}

// episode end + dones[i] + auto-reset (environment.cpp:187-207, vec_environment.h:56-59) on the
// stored state, in two halves around the wave's map generation (wave_generate, converged):
// end_of_step_a finishes the episode and stores dones[i]; it returns true when the env
// auto-resets, and end_of_step_b then completes the reset (true: the map was regenerated, the
// wave encodes it).  `out` caches (dones[i] | agent_selection[i] << 8) as last stored (~0u:
// unknown), so bytes that already hold the value are not stored again.
template <bool PUB = false>
DEV bool end_of_step_a(const DevState &s, size_t i, bool was_done, bool finish, uint32_t &agent, uint32_t &out) {
  constexpr int PO = PUB ? 2 : 0;                          // (an ended episode: pub_env_compare)
  if (finish) finish_episode(make_ctx(s, i));
  const bool done = was_done || finish;
  if ((out & 0xffu) != (done ? 1u : 0u)) pub_store<PO>(s, i, s.done + i, (uint8_t)(done ? 1 : 0));   // dones[i]
  if (done && s.autoreset) {                                                                        // before the reset
    env_reset_pre(make_ctx(s, i));
    out = (out & ~0xffu) | 1u;
    return true;
  }
  if (((out >> 8) & 0xffu) != (agent & 0xffu)) pub_store<PO>(s, i, s.agent + i, (uint8_t)agent);
  out = (done ? 1u : 0u) | (agent & 0xffu) << 8;
  return false;
}
DEV bool end_of_step_b(const DevState &s, size_t i, bool gen_ok, uint32_t &agent, uint32_t &out) {
  Ctx e = make_ctx(s, i);
  bool enc = false;
  if (!env_reset_post(e, gen_ok)) {
    atomicOr(&s.status[0], e.pv->flags);
    atomicAdd(&s.status[1], 1u);
    *s.err = 1u;                                           // host-visible error flag
  } else {
    enc = true;
    if (s.cap) {                                           // host views: list the regenerated maps
      const uint32_t k = atomicAdd(&s.status[2], 1u);
      if (k < s.cap) s.dirty[k] = (uint32_t)i;
    }
  }
  sync_heads(s, i);
  agent = e.pv->agent;
  if (((out >> 8) & 0xffu) != (agent & 0xffu)) s.agent[i] = (uint8_t)agent;
  out = 1u | (agent & 0xffu) << 8;
  return enc;
}

// One step of env i: load (two rounds; the sampler runs on round 1 while round 2 is in
// flight), step on registers, store what changed, [finish / auto-reset].
template <int SRC, bool PUB = false>
DEV bool env_step_lane(const DevState &s, size_t i, const uint8_t *act_in, uint32_t *rngs, uint8_t *actions_out,
                       const UidEntry *tab, uint32_t &agent, uint32_t &out, bool *ended = nullptr,
                       uint8_t *h_actions_out = nullptr) {
  STAMP(s, 0);
  PH_DECL;
  Snap S;
  RegEnv R;
  // the host's action first: often pinned host memory read over PCIe, its latency then overlaps
  // the state loads' instead of adding a round after them
  uint2 ext = make_uint2(0u, 0u);
  if (SRC == MASK_EXTERNAL) ext = *reinterpret_cast<const uint2 *>(act_in + i * COG_ACTION_BYTES);
  load_env(s, i, S);
  uint32_t srng = SRC == MASK_EXTERNAL ? 0u : rngs[i];
  regs_env(R, S);
  R.tab = tab;
  const int ag = (int)R.agent();
  const int na = ag + 1 >= (int)R.n_players() ? 0 : ag + 1;
  load_players(s, i, ag, na, S);
  uint8_t act[5];
  if (SRC == MASK_SELECTED) step_action<SRC>(R, ext, srng, act);
  regs_players(R, S);
  if (SRC != MASK_SELECTED) step_action<SRC>(R, ext, srng, act);
  STAMP(s, 1);
  const bool was_done = R.done() != 0u;
  const bool finish = !was_done && step_regs(R, act, s, i, na PH_PASS);
  if (finish) R.set_done(1u);
  STAMP(s, 2);
  store_changes<PUB>(s, i, ag, na, S, R);
  if (ended) *ended = was_done || finish;
  if (SRC != MASK_EXTERNAL) {                              // (every store after the step's loads)
    rngs[i] = srng;
    store_action(actions_out + i * COG_ACTION_BYTES, act);
    if (PUB && h_actions_out) store_action(h_actions_out + i * COG_ACTION_BYTES, act);   // the sampler's view
  }
  STAMP(s, 3);
  agent = R.agent();
  out = ~0u;
  const bool rs = end_of_step_a<PUB>(s, i, was_done, finish, agent, out);
  STAMP(s, 4);
  return rs;                                               // the env auto-resets (end_of_step_b)
}

template <int SRC>
__global__ void __launch_bounds__(64) k_env_step(DevState s, const uint8_t *__restrict__ act_in, uint32_t *__restrict__ rngs,
                                                 uint8_t *__restrict__ actions_out) {
  __shared__ UidEntry tab[kUidTab];
  uid_tab_fill(tab);
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i = i0 < s.n ? i0 : 0;
  bool rs = false, enc = false;
  uint32_t agent = 0, out = ~0u;
  if (i0 < s.n) rs = env_step_lane<SRC>(s, i, act_in, rngs, actions_out, tab, agent, out);
  const bool ok = wave_generate(s, i, rs);                 // converged: the whole wave generates
  if (rs) enc = end_of_step_b(s, i, ok, agent, out);
  wave_encode(s, i, enc);                                  // converged: the whole wave encodes
  STAMP(s, 5);
}

// In-kernel completion word of a host call (the host spins on it, cog_abi.cpp Signal): the last
// workgroup to finish stores `seq` into the pinned word, after every workgroup's stores (device
// records and the host views) have been acknowledged.  A counter in device memory finds the last
// workgroup (about 14 ns per arriving workgroup on one address, tools/latprobe.hip), so kernels
// that signal keep their grids small; the last workgroup re-arms the counter.
struct GridSignal {
  uint32_t *ctr;                      // device counter (0 between calls); null: no signal
  uint32_t *word;                     // device address of the pinned host word
  uint32_t seq;
};
DEV void grid_signal(const GridSignal &g) {
  if (!g.ctr) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();                                       // this workgroup's stores performed
    // acq_rel arrival + acquire fence in the last workgroup (as k_env_step_pub): every other
    // workgroup's stores happen-before the release store of the word
    if (__hip_atomic_fetch_add(g.ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(g.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(g.word, g.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Direct publish of an env whose episode ended in this step (finish_episode, dones, reset and
// encode rewrote records the step's own stores do not cover): its ObsData tail and its records in
// the outs block compared granule by granule with the mirror, as k_publish does, by the env's lane.
DEV void pub_compare(const DevState &s, const uint4 *src, uint4 *mir, uint4 *dst, int ng) {
  for (int g0 = 0; g0 < ng; g0 += 8) {                     // 8 granules in flight per round
    uint4 c[8], m[8];
#pragma unroll
    for (int g = 0; g < 8; g++)
      if (g0 + g < ng) {
        c[g] = src[g0 + g];
        m[g] = mir[g0 + g];
      }
#pragma unroll
    for (int g = 0; g < 8; g++)
      if (g0 + g < ng && ne4(c[g], m[g])) {
        dst[g0 + g] = c[g];
        mir[g0 + g] = c[g];
      }
  }
}
DEV void pub_env_compare(const DevState &s, size_t i) {
  const size_t mo = s.n * kTailG;                          // the outs block in the mirror (granules)
  uint4 *mir = reinterpret_cast<uint4 *>(s.pub_mir);
  const uint4 *obs = reinterpret_cast<const uint4 *>(s.obs) + i * kRecG + kTail0;
  pub_compare(s, obs, mir + i * kTailG, reinterpret_cast<uint4 *>(s.pub_obs) + i * kRecG + kTail0, (int)kTailG);
  const uint4 *outs = reinterpret_cast<const uint4 *>(s.status);
  uint4 *hout = reinterpret_cast<uint4 *>(s.pub_outs);
  const size_t sel = (size_t)(s.sel - reinterpret_cast<const uint8_t *>(s.status)) / 16 + i * (COG_MASK_BYTES / 16);
  const size_t inf = (size_t)(s.info - reinterpret_cast<const uint8_t *>(s.status)) / 16 + i * (COG_INFO_BYTES / 16);
  const size_t rew = (size_t)(reinterpret_cast<const uint8_t *>(s.rew) - reinterpret_cast<const uint8_t *>(s.status)) / 16 + i;
  pub_compare(s, outs + sel, mir + mo + sel, hout + sel, COG_MASK_BYTES / 16);
  pub_compare(s, outs + inf, mir + mo + inf, hout + inf, COG_INFO_BYTES / 16);
  pub_compare(s, outs + rew, mir + mo + rew, hout + rew, 1);
  pub_store<2>(s, i, s.done + i, s.done[i]);               // (bytes: stored as they are)
  pub_store<2>(s, i, s.agent + i, s.agent[i]);
}
// k_env_step for a host-visible step whose pinned views equal HBM (launch_step_pub): the step's
// stores go to the views and the mirror as well, ended episodes are published by comparison, and
// the last workgroup copies the status granules (error flags, dirty-map count) and stores the
// completion word -- one kernel instead of k_env_step + k_publish.
// SRC = MASK_EXTERNAL: env.step(actions); MASK_SELECTED / MASK_STORED: the runner's fused
// sample + step, whose sampled actions also go to the sampler's pinned view (h_actions).
template <int SRC>
__global__ void __launch_bounds__(64) k_env_step_pub(DevState s, const uint8_t *__restrict__ act_in, uint32_t *__restrict__ rngs,
                                                     uint8_t *__restrict__ actions_out, uint8_t *__restrict__ h_actions,
                                                     GridSignal sig, SampleSpec spec) {
  __shared__ UidEntry tab[kUidTab];
  uid_tab_fill(tab);
  const size_t i0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t i = i0 < s.n ? i0 : 0;
  bool rs = false, enc = false, ended = false;
  uint32_t agent = 0, out = ~0u;
  if (i0 < s.n)
    rs = env_step_lane<SRC, true>(s, i, act_in, rngs, actions_out, tab, agent, out, &ended, h_actions);
  const bool ok = wave_generate(s, i, rs);                 // converged: the whole wave generates
  if (rs) enc = end_of_step_b(s, i, ok, agent, out);
  wave_encode(s, i, enc);                                  // converged: the whole wave encodes
  if (__builtin_amdgcn_ballot_w64(ended)) {                // (wave-uniform) the wave's records as
    __builtin_amdgcn_s_waitcnt(0);                         // stored, including other lanes' encode
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    if (ended) pub_env_compare(s, i);
  }
  if (SRC == MASK_EXTERNAL && spec.rng_in && i0 < s.n) {   // the sampler's next sample, speculative:
    if (ended) {                                           // from the selected mask this step left (an
      *spec.invalid = 1u;                                  // ended episode's reset: no speculation)
    } else {
      uint32_t rng = spec.rng_in[i];
      uint8_t a[5];
      sample_heads(heads_of(mbits_of(s.heads[5 * i])), rng, a, tab);   // (this lane's own store)
      spec.rng_out[i] = rng;
      store_action(spec.act_dev + i * COG_ACTION_BYTES, a);
      store_action(spec.act_host + i * 8, a);
    }
  }
  // completion: the last workgroup to arrive publishes the status granules, then the word
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    if (__hip_atomic_fetch_add(sig.ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store(sig.ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const uint4 *st = reinterpret_cast<const uint4 *>(s.status);
      uint4 *mo = reinterpret_cast<uint4 *>(s.pub_mir) + s.n * kTailG;
#pragma unroll
      for (int g = 0; g < 4; g++) {
        const uint4 v = st[g];
        reinterpret_cast<uint4 *>(s.pub_outs)[g] = v;
        mo[g] = v;
      }
      __threadfence();
      __hip_atomic_store(sig.word, sig.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Persistent rollout: K x (sample; step) per launch (the runner's device loop, runner.h:46-55).
// Every step stores its outputs exactly as a single-step launch does (the HBM state after each
// step is the reference's); what changes is where the next step reads its inputs from: the
// env-level records stay in VGPRs and every player's records (deck, counters, neighbourhood
// cache, stored mask) in this wave's LDS, so a step issues no global loads unless it resets.
template <int NL>                     // NL: envs (lanes) per workgroup
struct LaneLds {
  uint4 deck[4][7][NL];               // [player][granule][lane]: lane-contiguous, conflict-free
  uint4 pl[4][NL];
  uint2 cells[4][NL];
  uint4 heads[4][NL];                 // stored masks (MBits + pad)
  UidEntry tab[kUidTab];              // the uniform's division table
};
template <class LaneLds>
DEV void lds_fill_players(LaneLds &L, const DevState &s, size_t i, int l) {
  const uint4 *pv4 = reinterpret_cast<const uint4 *>(s.priv + i);
#pragma unroll
  for (int p = 0; p < 4; p++) {
    const uint4 *dk = reinterpret_cast<const uint4 *>(deck_ptr(s, i, p));
#pragma unroll
    for (int k = 0; k < 7; k++) L.deck[p][k][l] = dk[k];
    L.pl[p][l] = pv4[4 + p];
    L.cells[p][l] = reinterpret_cast<const uint2 *>(pv4 + 8)[p];
    L.heads[p][l] = s.heads[5 * i + 1 + p];
  }
}
// The wave's player records are stored cooperatively at the end of a launch: consecutive
// work-items take consecutive 16-B granules of one env's records (its counters and neighbourhood
// caches are EnvPriv granules 4..9, its stored-mask bit vectors 4 consecutive heads), so one
// store instruction covers a few contiguous runs instead of 64 envs' scattered granules.
// Measured (tools/fixedcost.sh): the per-work-item store cost 6.2 us per launch at 65,536 envs,
// this one about 1 us.  The same transposition for the launch's loads was slower (19.7 against
// 9.5 us): those stay one env per work-item (lds_fill_players).  ne = the wave's envs; a
// work-item past the end of a ragged last wave stores env ne - 1's records again.
template <class LaneLds, int NL>
DEV void lds_store_wave(const LaneLds &L, const DevState &s, size_t base, int ne) {
  const int l = threadIdx.x;                               // (past the end: env ne - 1's records again)
#pragma unroll
  for (int j = 0; j < 4 * NL / 64; j++) {
    const int f = j * 64 + l, e = min(f >> 2, ne - 1), q = f & 3;
    reinterpret_cast<uint4 *>(s.priv + base + e)[4 + q] = L.pl[q][e];
  }
#pragma unroll
  for (int j = 0; j < 2 * NL / 64; j++) {
    const int f = j * 64 + l, e = min(f >> 1, ne - 1), q = f & 1;
    const uint2 a = L.cells[2 * q][e], b = L.cells[2 * q + 1][e];
    reinterpret_cast<uint4 *>(s.priv + base + e)[8 + q] = make_uint4(a.x, a.y, b.x, b.y);
  }
#pragma unroll
  for (int j = 0; j < 4 * NL / 64; j++) {
    const int f = j * 64 + l, e = min(f >> 2, ne - 1), p = f & 3;
    s.heads[5 * (base + e) + 1 + p] = L.heads[p][e];
  }
}
// the env-level private records of env i (EnvPriv granules 0, 1, 3, the selected mask's bits)
DEV void store_env_private(const DevState &s, size_t i, const Snap &S) {
  uint4 *pw = reinterpret_cast<uint4 *>(s.priv + i);
  pw[0] = S.g0;
  pw[1] = S.g1;
  reinterpret_cast<uint32_t *>(pw + 3)[0] = S.info_steps;
  s.heads[5 * i] = mbits_u4(S.sel);
}
// every private record of env i (EnvPriv granules 0, 1, 3, all players, all mask bit vectors)
// from the rollout's on-chip copies
template <class LaneLds>
DEV void store_private_all(const DevState &s, size_t i, const Snap &S, const LaneLds &L, int l) {
  uint4 *pw = reinterpret_cast<uint4 *>(s.priv + i);
  pw[0] = S.g0;
  pw[1] = S.g1;
  reinterpret_cast<uint32_t *>(pw + 3)[0] = S.info_steps;
  s.heads[5 * i] = mbits_u4(S.sel);
#pragma unroll
  for (int p = 0; p < 4; p++) {
    pw[4 + p] = L.pl[p][l];
    reinterpret_cast<uint2 *>(pw + 8)[p] = L.cells[p][l];
    s.heads[5 * i + 1 + p] = L.heads[p][l];
  }
}
template <class LaneLds>
DEV void lds_players(const LaneLds &L, int l, int ag, int na, Snap &S) {
  S.pla = L.pl[ag][l];
  S.pln = L.pl[na][l];
  S.ca = L.cells[ag][l];
  S.cn = L.cells[na][l];
  S.sta = mbits_of(L.heads[ag][l]);
  S.stn = mbits_of(L.heads[na][l]);
#pragma unroll
  for (int k = 0; k < 7; k++) S.dk[k] = L.deck[ag][k][l];
}

// The rollout is one kernel in two passes.  The lean pass (FIX = false) carries no episode-end
// code: a lane whose env finishes (or starts done) at step t stores its state, keeps t (its
// "park" code) and leaves the loop; the other lanes go on.  After the loop, a wave with a parked
// lane runs the fix-up pass (FIX = true, a wave-uniform branch) for exactly those lanes: it
// completes step t's episode end (finish_episode, dones, auto-reset, encode) and runs the env's
// remaining steps with the full step (resets included).  Nothing reads the env in between and
// envs are independent (no barrier between the reference's workers either, runner.h:39-62), so
// the outputs are those of one full-step loop; the lean loop keeps the reset path's registers
// out of its allocation.  A wave with nothing parked ends after the lean pass (round 1 launched
// the fix-up as a second kernel: 4.8 us per launch even when it had nothing to do).
// park codes: bits 0..29 the step t; kParkFinish: step t finished the episode (else the env
// started step t done); kParkRedo: step t was not run (the trio's stepping wave met an action
// outside its lean step, lean_player in trio_stepper) -- the fix-up runs it with the full step
constexpr uint32_t kParkNone = ~0u, kParkFinish = 1u << 31, kParkRedo = 1u << 30;
constexpr uint32_t kParkStep = kParkRedo - 1u;
// The records of a wave's envs seen from the wave's first env: a per-wave (scalar) base and a
// per-lane index below 64, so that record addresses are a scalar base plus a 32-bit lane offset
// (the saddr form of global loads and stores) instead of 64-bit products of a global index,
// which the compiler rematerialises at every store under the kernel's register pressure.
DEV DevState wave_view(const DevState &s, size_t base) {
  DevState v = s;
  v.obs += base * COG_OBS_BYTES;
  v.sel += base * COG_MASK_BYTES;
  v.info += base * COG_INFO_BYTES;
  v.rew += base * 4;
  v.done += base;
  v.agent += base;
  v.priv += base;
  v.grid += base * (size_t)kGridBytes;
  v.cgrid += base * COG_CELLS;
  v.heads += 5 * base;
  v.cdeck += 10 * base;
  v.cwide += base;
  v.gen += base;
  v.park += base;
  v.first += base;
  v.n = s.n > base ? s.n - base : 0;
  return v;
}
// a duo / trio workgroup with a parked env appends its index to the launch's parked list (one
// atomic per such wave), so that k_env_fixup visits only those (DevState::parkq)
DEV void park_list_push(const DevState &s_glob, bool parked) {
  if (__builtin_amdgcn_ballot_w64(parked) && (threadIdx.x & 63) == 0) {
    if (s_glob.no_fixup) {                                 // the host showed no park could happen
      atomicOr(&s_glob.status[0], F_PARK_NOFIX);
      atomicAdd(&s_glob.status[1], 1u);
      *s_glob.err = 1u;
    }
    const uint32_t j = atomicAdd(&s_glob.parkq[s_glob.park_par], 1u);
    s_glob.parkq[2 + j] = blockIdx.x;
  }
}
// the other counter back to 0 for the next launch (the previous launch's fix-up, which read it,
// has completed: same stream)
DEV void park_list_clear_other(const DevState &s_glob) {
  if (blockIdx.x == 0 && threadIdx.x == 0) s_glob.parkq[s_glob.park_par ^ 1u] = 0u;
}
// Two-wave rollout for small shards (k_env_rollout_pipe): the stepping wave hands each step's
// outputs to a second wave of its workgroup through a double-buffered LDS ring, and the second
// wave finds what changed and issues the store phase (mask expansions and the granule stores)
// while the first runs the next step.  One record per lane and step, [buffer][granule][lane]:
//   0-2   ObsData 16128.. (phase, resources, shop) after the step, 3-5 before it
//   6-12  the acting player's DeckObs after the step
//   13    selected-mask bits after, .w = flags: 28 valid, 29 moved, 30 next player != acting
//         player (the storing wave keeps every player's deck as last stored, DeckImage)
//   14    acting player's stored-mask bits after, .w = ag | na << 8 | Info steps byte << 16
//   15    next player's stored-mask bits after
//   16-18 the three mask bit vectors before the step (9 dwords), then the action (8 bytes)
//   19    EnvPriv granule 2 (locations) when moved
constexpr int kOutG = 20;
struct OutRing {
  uint4 g[2][kOutG][64];
};
DEV void out_record_write(OutRing &O, int b, int l, int ag, int na, const Snap &S, const RegEnv &R,
                          const uint8_t act[5]) {
  const uint32_t gm = 1u << 28 | (R.moved ? 1u << 29 : 0u) | (na != ag ? 1u << 30 : 0u);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    O.g[b][k][l] = make_uint4(R.sh[4 * k], R.sh[4 * k + 1], R.sh[4 * k + 2], R.sh[4 * k + 3]);
    O.g[b][3 + k][l] = S.sh[k];
  }
#pragma unroll
  for (int k = 0; k < 7; k++) O.g[b][6 + k][l] = make_uint4(R.d[4 * k], R.d[4 * k + 1], R.d[4 * k + 2], R.d[4 * k + 3]);
  const MBits bs = bits_of(R.sel), ba = bits_of(R.sta), bn = bits_of(R.stn);
  O.g[b][13][l] = make_uint4(bs.w0, bs.w1, bs.w2, gm);
  O.g[b][14][l] = make_uint4(ba.w0, ba.w1, ba.w2,
                             (uint32_t)ag | (uint32_t)na << 8 | ((R.info_steps >> (8 * ag)) & 0xffu) << 16);
  O.g[b][15][l] = make_uint4(bn.w0, bn.w1, bn.w2, 0u);
  O.g[b][16][l] = make_uint4(S.sel.w0, S.sel.w1, S.sel.w2, S.sta.w0);
  O.g[b][17][l] = make_uint4(S.sta.w1, S.sta.w2, S.stn.w0, S.stn.w1);
  O.g[b][18][l] = make_uint4(S.stn.w2,
                             (uint32_t)act[0] | (uint32_t)act[1] << 8 | (uint32_t)act[2] << 16 | (uint32_t)act[3] << 24,
                             (uint32_t)act[4], 0u);
  O.g[b][19][l] = R.g2;
}
DEV uint4 sel4(bool c, const uint4 &a, const uint4 &b) {
  return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}
// the storing wave's copy of every player's DeckObs as it stands in HBM (loaded at the start of
// the launch, then updated by its own stores): the previous value of the acting player's deck
struct DeckImage {
  uint4 d[4][7];
};
DEV void deck_image_load(DeckImage &I, const DevState &s, size_t i) {
#pragma unroll
  for (int p = 0; p < 4; p++) {
    const uint4 *dk = reinterpret_cast<const uint4 *>(deck_ptr(s, i, p));
#pragma unroll
    for (int k = 0; k < 7; k++) I.d[p][k] = dk[k];
  }
}
// the storing wave: exactly the stores store_outputs + store_action issue, in the same order
DEV void out_record_store(const OutRing &O, int b, int l, const DevState &s, size_t i, uint8_t *actions_out,
                          DeckImage &I) {
  const uint4 m = O.g[b][13][l];
  const uint32_t gm = m.w;
  if (!((gm >> 28) & 1u)) return;
  const uint4 x = O.g[b][14][l], o0 = O.g[b][16][l], o1 = O.g[b][17][l], o2 = O.g[b][18][l];
  const int ag = (int)(x.w & 0xffu), na = (int)((x.w >> 8) & 0xffu);
  uint8_t *ob = s.obs + i * COG_OBS_BYTES;
  s.info[i * COG_INFO_BYTES + COG_AGENT_INFO0 + COG_AGENT_INFO_STRIDE * ag] = (uint8_t)(x.w >> 16);
  if ((gm >> 29) & 1u) reinterpret_cast<uint4 *>(s.priv + i)[2] = O.g[b][19][l];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const uint4 v = O.g[b][k][l];
    if (ne4(v, O.g[b][3 + k][l])) reinterpret_cast<uint4 *>(ob + COG_OBS_PHASE)[k] = v;
  }
  uint8_t *deck = deck_ptr(s, i, ag);
#pragma unroll
  for (int k = 0; k < 7; k++) {
    const uint4 v = O.g[b][6 + k][l];
    uint4 old = I.d[3][k];                                 // (selects: a register array indexed
#pragma unroll                                             // by a lane value would go to scratch)
    for (int p = 2; p >= 0; p--) old = sel4(ag == p, I.d[p][k], old);
    if (ne4(v, old)) reinterpret_cast<uint4 *>(deck)[k] = v;
#pragma unroll
    for (int p = 0; p < 4; p++) I.d[p][k] = sel4(ag == p, v, I.d[p][k]);
  }
  const MBits bs{m.x, m.y, m.z}, ba{x.x, x.y, x.z};
  store_mask_record(reinterpret_cast<uint4 *>(s.sel + i * COG_MASK_BYTES), bs,
                    mask_diff_granules(bs, MBits{o0.x, o0.y, o0.z}));
  store_mask_record(reinterpret_cast<uint4 *>(deck + COG_PD_MASK), ba, mask_diff_granules(ba, MBits{o0.w, o1.x, o1.y}));
  if ((gm >> 30) & 1u) {
    const uint4 y = O.g[b][15][l];
    const MBits bn{y.x, y.y, y.z};
    store_mask_record(reinterpret_cast<uint4 *>(deck_ptr(s, i, na) + COG_PD_MASK), bn,
                      mask_diff_granules(bn, MBits{o1.z, o1.w, o2.x}));
  }
  reinterpret_cast<uint2 *>(actions_out + i * COG_ACTION_BYTES)[0] = make_uint2(o2.y, o2.z);
}

// wbase_in: the wave's first env (k_env_fixup: a parked workgroup's); default blockIdx.x * NL
template <int SRC, bool FIX, int NL, bool PIPE = false>
DEV uint32_t rollout_pass(LaneLds<NL> &L, const DevState &s_glob, int steps, uint32_t *__restrict__ rngs_glob,
                          uint8_t *__restrict__ actions_glob, uint32_t park, OutRing *O = nullptr,
                          size_t wbase_in = ~(size_t)0) {
  const int l = threadIdx.x;                               // (the stepping wave: threads 0..NL-1)
  const size_t wbase = wbase_in != ~(size_t)0 ? wbase_in : (size_t)blockIdx.x * NL;
  const size_t i0 = wbase + l;
  // (s, i): the wave's view and the lane's index in it, for every record access; the wave's
  // generation, its encode and the regenerated-map list take the shard's (s_glob, i_glob)
  const DevState s = wave_view(s_glob, wbase);
  const size_t i = (size_t)l;
  const size_t i_glob = i0 < s_glob.n ? i0 : 0;
  uint32_t *__restrict__ rngs = rngs_glob + wbase;
  uint8_t *__restrict__ actions_out = actions_glob + wbase * COG_ACTION_BYTES;
  int t_first = 0;                                         // fix-up: this lane's first full step
  bool live = i0 < s_glob.n && (!FIX || park != kParkNone);
  Snap S;
  uint32_t srng = 0, out = ~0u;                           // out: end_of_step's output cache
  auto next_of = [&](int a) { return a + 1 >= (int)(S.g1.x & 0xffu) ? 0 : a + 1; };   // n_players
  if (live) {
    load_env(s, i, S);
#ifndef COG_ABLATE_FILL                                    // diagnostic timing builds only
    lds_fill_players(L, s, i, l);
#endif
    srng = rngs[i];
  }

  if (FIX) {                                               // step `park`'s episode end
    bool enc = false, rs = false;
    uint32_t agent = 0;
    if (live && (park & kParkRedo)) {                      // step `park` itself was not run
      t_first = (int)(park & kParkStep);
    } else if (live) {
      t_first = (int)(park & kParkStep) + 1;
      agent = S.g1.y & 0xffu;
      const bool finish = (park & kParkFinish) != 0u;
      rs = end_of_step_a(s, i, !finish, finish, agent, out);
    }
    const bool ok = wave_generate(s_glob, i_glob, rs);               // converged: the whole wave generates
    if (live) {
      if (rs) enc = end_of_step_b(s_glob, i_glob, ok, agent, out);
      load_env(s, i, S);                                   // reset: reload from the stored state
      lds_fill_players(L, s, i, l);
    }
    wave_encode(s_glob, i_glob, enc);                                // converged: the whole wave encodes
  }
  if (live) {
    const int ag = (int)(S.g1.y & 0xffu);
    lds_players(L, l, ag, next_of(ag), S);
  }
  // Every load above completes before the loop: the loop issues no load whose wait could be
  // merged with them, so the wait-count pass places no per-iteration vmcnt wait for registers
  // they wrote (such a wait, executed every step, would also wait for the step's stores).
  __builtin_amdgcn_s_waitcnt(0);
  if (PIPE && !FIX) __syncthreads();                       // the decks in LDS: the storing wave's image
  PH_DECL;
  for (int t = 0; t < steps; t++) {
    if (PIPE) {                                            // every lane, every step: the records
      if (t) __syncthreads();                              // of step t - 1 to the storing wave
      if (!live) O->g[t & 1][13][l] = make_uint4(0u, 0u, 0u, 0u);   // (no record)
    }
    if (!FIX && !PIPE && !live) break;                     // lean: a parked lane leaves the loop
    bool enc = false, ended = false, rs = false;
    uint32_t agent = 0;
    if (live && t >= t_first) {
      RegEnv R;
      regs_env(R, S);
      R.tab = L.tab;
      const int ag = (int)R.agent();                       // S holds ag's and na's records: read
      const int na = ag + 1 >= (int)R.n_players() ? 0 : ag + 1;   // at the end of the last step
      uint8_t act[5];
      PH(0);
      if (SRC == MASK_SELECTED) step_action<SRC>(R, make_uint2(0u, 0u), srng, act);
#ifdef COG_ABLATE_DUPSAMPLE                                // diagnostic timing builds only: the
      {                                                    // sampler's cost, measured by running
        uint32_t r2 = srng ^ 0x5555u;                      // it a second time on a discarded state
        uint8_t a2[5];
        sample_heads(R.sel, r2, a2, R.tab);
        asm volatile("" ::"v"((uint32_t)a2[0] | a2[1] << 8 | a2[2] << 16 | (uint32_t)a2[3] << 24), "v"(a2[4] ^ r2));
      }
#endif
      regs_players(R, S);
      if (SRC == MASK_STORED) step_action<SRC>(R, make_uint2(0u, 0u), srng, act);
      PH(1);
      const bool was_done = R.done() != 0u;
      const bool finish = !was_done && step_regs(R, act, s, i, na PH_PASS);
      if (finish) R.set_done(1u);
      PH(2);
      // the player records to this wave's LDS, and the next step's players back, before the
      // store phase: the LDS round trip overlaps the stores instead of stalling the loop's tail
      L.pl[ag][l] = pack_player(R.P);
      L.cells[ag][l] = R.cells_a;
      L.heads[ag][l] = mbits_u4(bits_of(R.sta));
      if (na != ag) L.heads[na][l] = mbits_u4(bits_of(R.stn));
#pragma unroll
      for (int k = 0; k < 7; k++) L.deck[ag][k][l] = make_uint4(R.d[4 * k], R.d[4 * k + 1], R.d[4 * k + 2], R.d[4 * k + 3]);
      agent = R.agent();
      Snap N;                                              // the next step's player records
      lds_players(L, l, (int)agent, next_of((int)agent), N);
      PH(3);
#ifndef COG_ABLATE_STORES                                  // diagnostic timing builds only
      if (PIPE) {
        out_record_write(*O, t & 1, l, ag, na, S, R, act);
      } else {
        store_outputs(s, i, ag, na, S, R);
        store_action(actions_out + i * COG_ACTION_BYTES, act);
      }
#endif
      PH(4);
      // the next step's image: registers (env level) and the player records just read
      S.g0 = make_uint4(R.rng, R.seed, R.max_steps, R.turn_counter);
      S.g1 = make_uint4(R.g1x, R.g1y, R.in_market, R.flags);
      S.g2 = R.g2;
      S.avail = R.avail;
      S.info_steps = R.info_steps;
#pragma unroll
      for (int k = 0; k < 3; k++) S.sh[k] = make_uint4(R.sh[4 * k], R.sh[4 * k + 1], R.sh[4 * k + 2], R.sh[4 * k + 3]);
      S.sel = bits_of(R.sel);
      S.pla = N.pla; S.pln = N.pln; S.ca = N.ca; S.cn = N.cn; S.sta = N.sta; S.stn = N.stn;
#pragma unroll
      for (int k = 0; k < 7; k++) S.dk[k] = N.dk[k];
      if (was_done || finish) {                            // episode end: state to HBM first
        store_private_all(s, i, S, L, l);
        if (!FIX) {                                        // hand the env to the fix-up pass
          rngs[i] = srng;
          park = (uint32_t)t | (finish ? kParkFinish : 0u);
          live = false;
          continue;
        }
        ended = true;
        rs = end_of_step_a(s, i, was_done, finish, agent, out);
      } else {
        end_of_step_a(s, i, false, false, agent, out);
      }
      PH(5);
    }
    if (FIX) {                                             // converged: the whole wave generates
      const bool ok = wave_generate(s_glob, i_glob, rs);
      if (ended) {
        if (rs) enc = end_of_step_b(s_glob, i_glob, ok, agent, out);
        load_env(s, i, S);                                 // reload from the stored state
        lds_fill_players(L, s, i, l);
        agent = S.g1.y & 0xffu;
        lds_players(L, l, (int)agent, next_of((int)agent), S);
      }
      wave_encode(s_glob, i_glob, enc);                              // converged: the whole wave encodes
    }
    PH(6);
  }
  if (PIPE && steps > 0) __syncthreads();                 // the last step's records
  if (live) {                                              // env-level private state back to HBM
    store_env_private(s, i, S);                            // (the player records: lds_store_wave)
    rngs[i] = srng;
  }
  if (!FIX) PH_FLUSH(s);
  return FIX ? kParkNone : park;
}

template <int SRC, int NL>
__global__ void __launch_bounds__(NL) k_env_rollout(DevState s, int steps, uint32_t *__restrict__ rngs,
                                                    uint8_t *__restrict__ actions_out) {
  __shared__ LaneLds<NL> L;
  const size_t base = (size_t)blockIdx.x * NL;
  const int ne = (int)min((size_t)NL, s.n - base);
  uid_tab_fill(L.tab);
  const uint32_t park = rollout_pass<SRC, false, NL>(L, s, steps, rngs, actions_out, kParkNone);
  if (__builtin_amdgcn_ballot_w64(park != kParkNone))    // (wave-uniform)
    rollout_pass<SRC, true, NL>(L, s, steps, rngs, actions_out, park);
  __syncthreads();
#ifndef COG_ABLATE_EPI                                     // diagnostic timing builds only
  lds_store_wave<LaneLds<NL>, NL>(L, s, base, ne);
#endif
}

// Shards of <= 32,768 envs leave SIMDs idle (one 64-env wave per SIMD at most): each workgroup
// gets a second wave for its store phase (OutRing above).  Barriers: one at the start, one per
// step (the stepping wave hands over step t - 1 at the top of step t, the last step after its
// loop), one when the storing wave's stores have completed, one before the epilogue.  The fix-up
// pass (episode ends, resets) then runs on the stepping wave alone with the plain store phase,
// after an L1 invalidate, since it reloads records the storing wave wrote.
template <int SRC>
__global__ void __launch_bounds__(128) k_env_rollout_pipe(DevState s, int steps, uint32_t *__restrict__ rngs,
                                                          uint8_t *__restrict__ actions_out) {
  __shared__ LaneLds<64> L;
  __shared__ OutRing O;
  const size_t base = (size_t)blockIdx.x * 64;
  const int ne = (int)min((size_t)64, s.n - base);
  // (roles rotated per workgroup, so that a CU's two workgroups could not put both stepping waves
  // on one SIMD, measured the same: profiles/r04y_trio_role_rotation.txt)
  const int role = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform
  uid_tab_fill(L.tab);
  uint32_t park = kParkNone;
  if (role == 0) {
    park = rollout_pass<SRC, false, 64, true>(L, s, steps, rngs, actions_out, kParkNone, &O);
    __syncthreads();                                       // the storing wave's stores are done
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");     // (drop L1 lines they replaced)
    if (__builtin_amdgcn_ballot_w64(park != kParkNone))    // (wave-uniform)
      rollout_pass<SRC, true, 64>(L, s, steps, rngs, actions_out, park);
  } else {
    const int l = (int)threadIdx.x - 64;
    const DevState v = wave_view(s, base);
    uint8_t *av = actions_out + base * COG_ACTION_BYTES;
    DeckImage I;
    __syncthreads();                                       // the stepping wave's fill is in LDS: the
    if (l < ne) {                                          // image from there, not a second read of
#pragma unroll                                             // every deck from memory
      for (int p = 0; p < 4; p++)
#pragma unroll
        for (int k = 0; k < 7; k++) I.d[p][k] = L.deck[p][k][l];
    }
    for (int t = 0; t < steps; t++) {
      __syncthreads();
      if (l < ne) out_record_store(O, t & 1, l, v, (size_t)l, av, I);
    }
    __builtin_amdgcn_s_waitcnt(0);                         // every store of this wave completed
    __syncthreads();
  }
  __syncthreads();
#ifndef COG_ABLATE_EPI                                     // diagnostic timing builds only
  if (role == 0) lds_store_wave<LaneLds<64>, 64>(L, s, base, ne);
#endif
}

// ------------------------------------------------------------------------------------------
// Duo rollout (round 3): two waves per 64-env workgroup -- a stepping wave and a storing wave --
// sized so that FOUR workgroups share a CU (32,000 B of LDS each, <= 256 VGPRs + AGPRs per
// work-item), i.e. two waves per SIMD at 65,536 envs.  A lone wave issues at most one
// instruction per quad-cycle; the SIMD's VALU takes one per two cycles, so the storing wave of
// one workgroup runs beside the stepping wave of another on the same SIMD, and the stepping wave
// runs only the game logic.
//
// Ownership.  The stepping wave keeps the env in registers (RegEnv, across steps: no per-step
// image repacking) and every player's counters, neighbourhood cache and stored-mask bits in LDS
// (`pl`, `cells`, `heads`).  The storing wave keeps every player's DeckObs as last stored
// (DeckImage, registers) and the "before" images the store phase compares with: the shared
// block (phase, resources, shop), the selected-mask bits and each player's stored-mask bits.
// Per step the stepping wave hands over only after-values through a single-buffered LDS ring
// (`ring`, 14 granules per env), and the storing wave hands back the deck of the player who
// acts after a turn change (`slot`: the next player's deck as of the step's start -- only the
// acting player's deck changes within a step).
//
// Before the loop, barrier B: the storing wave has loaded every player's deck (its image) and
// hands the acting player's to the stepping wave through the ring's deck buffer 1, so the stepping
// wave's prologue is one round of loads (no dependent read of the deck the agent selects).
// Per step t, two barriers (both waves execute them):
//   stepping wave: step t on registers; pl/cells/heads of the acting player to LDS;
//                  X_t; record t to the ring; on a turn change the next player's records from
//                  LDS and its deck from the slot; Y_t
//   storing wave:  (X_0 after its prologue) Y_t; record t from the ring into registers; update
//                  its images; the slot for step t + 1; X_{t+1}; the stores of record t
// The storing wave reaches X long before the stepping wave ends its step, and the stepping wave
// reaches Y long after the storing wave's stores were issued, so neither barrier stalls the
// stepping wave beyond its own issue.
//
// Episode ends (and envs that start a launch done) park as in k_env_rollout's lean pass: the
// lane stores its private state, records its park code in DevState::park and leaves the loop;
// k_env_fixup, launched right after on the same stream, completes them.  The fix-up's register
// appetite (map generation, the full step) therefore does not cap this kernel's occupancy.
constexpr int kRingG = 7, kSlotG = 7;
struct DuoLds {
  uint4 pl[4][64];                    // [player][lane]: PlayerPriv (packed)
  uint2 cells[4][64];                 // neighbourhood caches
  uint4 heads[4][64];                 // stored-mask bits (MBits + pad)
  uint4 ring[kRingG][64];             // step record, stepping wave -> storing wave
  uint4 deckr[2][7][64];              // the record's DeckObs, double-buffered (written before X)
  uint4 slot[kSlotG][64];             // next player's DeckObs, storing wave -> stepping wave
  UidEntry tab[kUidTab];
};
static_assert(sizeof(DuoLds) <= 40960, "four duo workgroups per CU");
// step record t: deckr[t & 1] = the acting player's DeckObs after the step, and ring granules
//   0-2   ObsData 16128..16175 (phase, resources, shop) after the step
//   3     selected-mask bits; .w = meta (below)
//   4     the acting player's stored-mask bits; .w = action bytes 0..3
//   5     the next player's stored-mask bits; .w = action byte 4
//   6     EnvPriv granule 2 (map bounds + locations), read when the acting player moved
// meta: bit 0 valid, 1 moved, 2-3 ag, 4-5 na, 6-7 na1 (the player after the next step's
// acting player), 8-15 Info steps byte of ag, 16 the episode ended (parked: dones / agent are
// left to the fix-up), 24-31 agent after the step
constexpr uint32_t kMetaValid = 1u, kMetaMoved = 2u, kMetaEnded = 1u << 16;
constexpr uint32_t kMetaStepped = 1u << 17;               // (trio) the step ran: the env was not done

DEV uint32_t next_player(uint32_t a, uint32_t np) { return a + 1u >= np ? 0u : a + 1u; }

// The env-level private records of env i from the stepping wave's registers (EnvPriv granules
// 0, 1, 3, the selected mask's bits).  The player records (counters, neighbourhood caches,
// stored-mask bits) are stored from the wave's LDS by the epilogue (lds_store_wave), parked envs'
// included, after the last update of them.  DEFER (the trio): the env rng is the drawing wave's
// (it stores it at its end), so granule 0's first dword is left alone.
template <bool DEFER>
DEV void duo_store_env_private(const DevState &s, size_t i, const RegEnv &R) {
  uint4 *pw = reinterpret_cast<uint4 *>(s.priv + i);
  if (DEFER) reinterpret_cast<uint3 *>(reinterpret_cast<uint32_t *>(pw) + 1)[0] = make_uint3(R.seed, R.max_steps, R.turn_counter);
  else pw[0] = make_uint4(R.rng, R.seed, R.max_steps, R.turn_counter);
  pw[1] = make_uint4(R.g1x, R.g1y, R.in_market, R.flags);
  reinterpret_cast<uint32_t *>(pw + 3)[0] = R.info_steps;
  s.heads[5 * i] = mbits_u4(bits_of(R.sel));
}

// The deferred turn end (the trio rollout: selected masks, >= 3 players).  The stepping wave ends
// a turn without touching the deck -- no discard, no draws -- and the drawing wave completes it
// from the step record (the acting player's deck after the step, its counters in `pl`, the saved
// mask) with the env rng, which it owns: Player::end_turn's discard + draw (player.cpp:170-180),
// then the saved mask gains the drawn cards (draw's mask updates, cards.cpp:183-211, precede
// save_actionmask).  Nothing the stepping wave reads before that player acts again depends on it:
// with >= 3 players the next two agents are other players, whose turn ends lie at least two steps
// back.  Any action outside the lean step (lean_player: never in the canonical loop) parks
// the env with kParkRedo, and k_env_fixup runs that step and the rest with the full step.

template <int SRC>
DEV void duo_stepper(DuoLds &D, const DevState &s_glob, int steps, uint32_t *__restrict__ rngs_glob) {
  const int l = threadIdx.x;
  const size_t wbase = (size_t)blockIdx.x * 64;
  const DevState s = wave_view(s_glob, wbase);
  const size_t i = (size_t)l;
  const int ne = (int)min((size_t)64, s_glob.n - wbase);
  uint32_t *__restrict__ rngs = rngs_glob + wbase;
  bool live = l < ne;
  uint32_t park = kParkNone, srng = 0;
  RegEnv R;
  int ag = 0, na = 0;
  if (live) {
    Snap S;
    load_env(s, i, S);
    regs_env(R, S);
    const uint4 *pv4 = reinterpret_cast<const uint4 *>(s.priv + i);
#pragma unroll
    for (int p = 0; p < 4; p++) {
      D.pl[p][l] = pv4[4 + p];
      D.cells[p][l] = reinterpret_cast<const uint2 *>(pv4 + 8)[p];
      D.heads[p][l] = s.heads[5 * i + 1 + p];
    }
    srng = rngs[i];
    ag = (int)R.agent();
    na = (int)next_player((uint32_t)ag, R.n_players());
    R.P = unpack_player(D.pl[ag][l]);
    R.na_active = (D.pl[na][l].y >> 16) & 0xffu;
    R.cells_a = D.cells[ag][l];
    R.cells_n = D.cells[na][l];
    R.sta = heads_of(mbits_of(D.heads[ag][l]));
    R.stn = heads_of(mbits_of(D.heads[na][l]));
  }
  R.tab = D.tab;
  // every load above completes before the loop (no per-iteration vmcnt wait covers them)
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();                                         // B: the storing wave loaded every deck;
  if (live) {                                              // the acting player's from its hand-over
#pragma unroll                                             // (no second, dependent read of memory)
    for (int k = 0; k < 7; k++) {
      const uint4 v = D.deckr[1][k][l];
      R.d[4 * k] = v.x; R.d[4 * k + 1] = v.y; R.d[4 * k + 2] = v.z; R.d[4 * k + 3] = v.w;
    }
  }
  PH_DECL;
  for (int t = 0; t < steps; t++) {
    bool ended = false, finish = false;
    uint8_t act[5];
    if (live) {
      step_action<SRC>(R, make_uint2(0u, 0u), srng, act);
      const bool was_done = R.done() != 0u;
      finish = !was_done && step_regs(R, act, s, i, na PH_PASS);
      if (finish) R.set_done(1u);
      ended = was_done || finish;
      PH(0);
      D.pl[ag][l] = pack_player(R.P);
      D.cells[ag][l] = R.cells_a;
      D.heads[ag][l] = mbits_u4(bits_of(R.sta));
      if (na != ag) D.heads[na][l] = mbits_u4(bits_of(R.stn));
#pragma unroll
      for (int k = 0; k < 7; k++)                          // (buffer t & 1: record t - 2's, taken)
        D.deckr[t & 1][k][l] = make_uint4(R.d[4 * k], R.d[4 * k + 1], R.d[4 * k + 2], R.d[4 * k + 3]);
      PH(1);
    }
    __syncthreads();                                       // X_t: record t - 1 taken, slot written
    PH(2);
    if (live) {
      const int ag1 = (int)R.agent();
      const int na1 = (int)next_player((uint32_t)ag1, R.n_players());
      const MBits bs = bits_of(R.sel), ba = bits_of(R.sta), bn = bits_of(R.stn);
      const uint32_t info = (R.info_steps >> (8 * ag)) & 0xffu;
      const uint32_t meta = kMetaValid | (R.moved ? kMetaMoved : 0u) | (uint32_t)ag << 2 | (uint32_t)na << 4 |
                            (uint32_t)na1 << 6 | info << 8 | (ended ? kMetaEnded : 0u) | (uint32_t)ag1 << 24;
#pragma unroll
      for (int k = 0; k < 3; k++) D.ring[k][l] = make_uint4(R.sh[4 * k], R.sh[4 * k + 1], R.sh[4 * k + 2], R.sh[4 * k + 3]);
      D.ring[3][l] = make_uint4(bs.w0, bs.w1, bs.w2, meta);
      D.ring[4][l] = make_uint4(ba.w0, ba.w1, ba.w2,
                                (uint32_t)act[0] | (uint32_t)act[1] << 8 | (uint32_t)act[2] << 16 | (uint32_t)act[3] << 24);
      D.ring[5][l] = make_uint4(bn.w0, bn.w1, bn.w2, (uint32_t)act[4]);
      D.ring[6][l] = R.g2;
      R.moved = false;
      if (ag1 != ag) {                                     // turn change: ag1 == na acts next
#pragma unroll
        for (int k = 0; k < 7; k++) {
          const uint4 v = D.slot[k][l];
          R.d[4 * k] = v.x; R.d[4 * k + 1] = v.y; R.d[4 * k + 2] = v.z; R.d[4 * k + 3] = v.w;
        }
        R.P = unpack_player(D.pl[ag1][l]);
        R.cells_a = R.cells_n;
        R.sta = R.stn;
        R.stn = heads_of(mbits_of(D.heads[na1][l]));
        R.cells_n = D.cells[na1][l];
        R.na_active = (D.pl[na1][l].y >> 16) & 0xffu;
      }
      if (ended) {                                         // hand the env to k_env_fixup
        duo_store_env_private<false>(s, i, R);
        rngs[i] = srng;
        park = (uint32_t)t | (finish ? kParkFinish : 0u);
        live = false;
      }
      ag = ag1;
      na = na1;
    } else {
      D.ring[3][l] = make_uint4(0u, 0u, 0u, 0u);           // no record
    }
    PH(3);
    __syncthreads();                                       // Y_t: record t in the ring
    PH(4);
  }
  __syncthreads();                                         // X_steps
  PH_FLUSH(s_glob);
  if (live) {                                              // env-level private state back to HBM
    duo_store_env_private<false>(s, i, R);
    rngs[i] = srng;
  }
  if (l < ne) s.park[i] = park;
  park_list_push(s_glob, park != kParkNone);
  lds_store_wave<DuoLds, 64>(D, s, 0, ne);                 // every player's records (cooperative)
}

DEV uint4 sel4_of(const DeckImage &I, int p, int k) {      // I.d[p][k] for a lane-varying p
  uint4 v = I.d[3][k];
#pragma unroll
  for (int q = 2; q >= 0; q--) v = sel4(p == q, I.d[q][k], v);
  return v;
}
DEV MBits selm(const MBits b[4], int p) {
  MBits v = b[3];
#pragma unroll
  for (int q = 2; q >= 0; q--) {
    v.w0 = p == q ? b[q].w0 : v.w0;
    v.w1 = p == q ? b[q].w1 : v.w1;
    v.w2 = p == q ? b[q].w2 : v.w2;
  }
  return v;
}
DEV void setm(MBits b[4], int p, const MBits &v) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    b[q].w0 = p == q ? v.w0 : b[q].w0;
    b[q].w1 = p == q ? v.w1 : b[q].w1;
    b[q].w2 = p == q ? v.w2 : b[q].w2;
  }
}

// DEFER: the turn end of record t's acting player ag (meta: ag1 != ag), on the drawing wave --
// Player::end_turn's discard + draw on the deck as the step left it, with the env rng; the saved
// mask gains the drawn cards; the player's counters and stored-mask bits go back to the LDS
// records the stepping wave reads when ag acts again.
template <class Lds>
DEV void duo_turn_end(Lds &D, int l, int ag, uint4 dk[7], MBits &ba, uint32_t &rng, uint32_t &flags) {
  RegEnv E;
#pragma unroll
  for (int k = 0; k < 7; k++) {
    E.d[4 * k] = dk[k].x; E.d[4 * k + 1] = dk[k].y; E.d[4 * k + 2] = dk[k].z; E.d[4 * k + 3] = dk[k].w;
  }
  E.P = unpack_player(D.pl[ag][l]);
  E.rng = rng;
  E.sel = heads_of(ba);
  E.flags = 0u;
  E.tab = D.tab;
  E.end_turn_deck();
#pragma unroll
  for (int k = 0; k < 7; k++) dk[k] = make_uint4(E.d[4 * k], E.d[4 * k + 1], E.d[4 * k + 2], E.d[4 * k + 3]);
  ba = bits_of(E.sel);
  rng = E.rng;
  D.pl[ag][l] = pack_player(E.P);
  D.heads[ag][l] = mbits_u4(ba);
  flags |= E.flags;
}

DEV void duo_storer(DuoLds &D, const DevState &s_glob, int steps, uint8_t *__restrict__ actions_glob) {
  const int l = (int)threadIdx.x - 64;
  const size_t wbase = (size_t)blockIdx.x * 64;
  const DevState s = wave_view(s_glob, wbase);
  const size_t i = (size_t)l;
  const bool live = wbase + (size_t)l < s_glob.n;
  uint8_t *__restrict__ av = actions_glob + wbase * COG_ACTION_BYTES;
  DeckImage I;
  uint4 shb[3];
  MBits selb = {0u, 0u, 0u}, stb[4];
  uint32_t out = ~0u;                                      // dones[i] | agent_selection[i] << 8 as stored
  if (live) {
    deck_image_load(I, s, i);
    const uint4 *sh4 = reinterpret_cast<const uint4 *>(s.obs + i * COG_OBS_BYTES + COG_OBS_PHASE);
#pragma unroll
    for (int k = 0; k < 3; k++) shb[k] = sh4[k];
    selb = mbits_of(s.heads[5 * i]);
#pragma unroll
    for (int p = 0; p < 4; p++) stb[p] = mbits_of(s.heads[5 * i + 1 + p]);
    const uint4 g1 = reinterpret_cast<const uint4 *>(s.priv + i)[1];
    const int ag0 = (int)(g1.y & 0xffu), na0 = (int)next_player(g1.y & 0xffu, g1.x & 0xffu);
#pragma unroll
    for (int k = 0; k < 7; k++) {
      D.slot[k][l] = sel4_of(I, na0, k);
      D.deckr[1][k][l] = sel4_of(I, ag0, k);               // (buffer 1 is first written at step 1)
    }
  }
  __syncthreads();                                         // B: the acting player's deck handed over
  __syncthreads();                                         // X_0
  PH_DECL;
  for (int t = 0; t < steps; t++) {
    __syncthreads();                                       // Y_t
    PH(5);
    uint4 g[kRingG], dk[7];
#pragma unroll
    for (int k = 0; k < kRingG; k++) g[k] = D.ring[k][l];
#pragma unroll
    for (int k = 0; k < 7; k++) dk[k] = D.deckr[t & 1][k][l];
    const uint32_t meta = g[3].w;
    const bool rec = live && (meta & kMetaValid);
    const int ag = (int)((meta >> 2) & 3u), na = (int)((meta >> 4) & 3u), na1 = (int)((meta >> 6) & 3u);
    if (rec) {
      uint32_t dm = 0;                                     // deck granules that changed
#pragma unroll
      for (int k = 0; k < 7; k++) {
        if (ne4(dk[k], sel4_of(I, ag, k))) dm |= 1u << k;
#pragma unroll
        for (int p = 0; p < 4; p++) I.d[p][k] = sel4(ag == p, dk[k], I.d[p][k]);
      }
#pragma unroll
      for (int k = 0; k < 7; k++) D.slot[k][l] = sel4_of(I, na1, k);
      PH(6);
#ifndef COG_ABLATE_DUOSTORES                               // diagnostic timing builds only
      uint8_t *ob = s.obs + i * COG_OBS_BYTES;
      s.info[i * COG_INFO_BYTES + COG_AGENT_INFO0 + COG_AGENT_INFO_STRIDE * ag] = (uint8_t)(meta >> 8);
      if (meta & kMetaMoved) reinterpret_cast<uint4 *>(s.priv + i)[2] = g[6];
#pragma unroll
      for (int k = 0; k < 3; k++) {
        if (ne4(g[k], shb[k])) reinterpret_cast<uint4 *>(ob + COG_OBS_PHASE)[k] = g[k];
        shb[k] = g[k];
      }
      uint8_t *deck = deck_ptr(s, i, ag);
#pragma unroll
      for (int k = 0; k < 7; k++)
        if ((dm >> k) & 1u) reinterpret_cast<uint4 *>(deck)[k] = dk[k];
      const MBits bs{g[3].x, g[3].y, g[3].z}, ba{g[4].x, g[4].y, g[4].z};
      store_mask_record(reinterpret_cast<uint4 *>(s.sel + i * COG_MASK_BYTES), bs, mask_diff_granules(bs, selb));
      selb = bs;
      store_mask_record(reinterpret_cast<uint4 *>(deck + COG_PD_MASK), ba, mask_diff_granules(ba, selm(stb, ag)));
      setm(stb, ag, ba);
      if (na != ag) {
        const MBits bn{g[5].x, g[5].y, g[5].z};
        store_mask_record(reinterpret_cast<uint4 *>(deck_ptr(s, i, na) + COG_PD_MASK), bn,
                          mask_diff_granules(bn, selm(stb, na)));
        setm(stb, na, bn);
      }
      reinterpret_cast<uint2 *>(av + i * COG_ACTION_BYTES)[0] = make_uint2(g[4].w, g[5].w);
#else
      asm volatile("" ::"v"(g[0].x ^ g[1].y ^ g[2].z ^ g[3].x ^ g[4].y ^ g[5].z ^ g[6].w ^ dm ^ dk[0].x ^ dk[6].w));
#endif
      if (!(meta & kMetaEnded)) {                          // dones[i] = 0, agent_selection[i]
        const uint32_t agent = meta >> 24;                 // (an ended episode: k_env_fixup)
        if (out & 0xffu) s.done[i] = 0;
        if (((out >> 8) & 0xffu) != agent) s.agent[i] = (uint8_t)agent;
        out = agent << 8;
      }
    }
    PH(13);
    __syncthreads();                                       // X_{t+1}
    PH(7);
  }
  PH_FLUSH(s_glob);
}

template <int SRC>
__global__ void __launch_bounds__(128) k_env_rollout_duo(DevState s, int steps, uint32_t *__restrict__ rngs,
                                                         uint8_t *__restrict__ actions_out) {
  __shared__ DuoLds D;
  // (roles rotated per workgroup, so that a CU's two workgroups could not put both stepping waves
  // on one SIMD, measured the same: profiles/r04y_trio_role_rotation.txt)
  const int role = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform
  park_list_clear_other(s);
  uid_tab_fill(D.tab);
  if (role == 0) {
#ifndef DUO_NOPRIO                                         // (diagnostic A/B builds only)
    __builtin_amdgcn_s_setprio(3);                         // the stepping wave wins VALU issue on
#endif                                                     // a SIMD it shares with a storing wave
    duo_stepper<SRC>(D, s, steps, rngs);
  } else {
    duo_storer(D, s, steps, actions_out);
  }
}

// ------------------------------------------------------------------------------------------
// Trio rollout (round 4): the selected-mask loop with >= 3 players at every shard size (cog_rollout_kind),
// one step's work spread over four waves per 64 envs.  The stepping wave runs the lean step
// (the lean step: sample, play or pass, turn change, done check) and nothing else; the drawing wave
// owns the decks (replays each play on its copy, runs the turn ends' discard + draws with the env
// rng); two storing waves issue the store phase, one of them also producing the sampler's
// presampled draws (presample).  History (8,192 envs, device us per step in 1,000-step launches,
// profiles/r04*_trio*.txt): the duo 2.45; its storing wave doing the draws 3.17 (it set the pace,
// profiles/r04d_duo_defer.txt); the draws on a third wave 1.96; lean step, hand-only stepping
// wave, presampled draws and two storing waves, in barrier lockstep 1.80 (the drawing wave's turn
// ends set the pace); turn ends batched over two records, still in lockstep, 1.86 (a two-record
// round is as long as the two it replaces); decoupled through progress counters (below).
//
// The waves run as a pipeline over LDS buffers, synchronised by progress counters in LDS (cnt[],
// stored after the records they publish -- in-order LDS, cnt_store; a waiting wave sleeps between
// polls) instead of barriers, so each runs at its own average rate:
//   stepping wave  step t: ring slot t % 8 free (record t - 8 stored by both storing waves), step
//                  t's presampled draws written (cnt[PRE] > t - 4); step; record t -> ring,
//                  cnt[REC] = t + 1; at a turn change, the drawing wave past the last turn ends of
//                  the new agent (its hand, counters) and of the player after it (its stored mask,
//                  hand nibbles) -- the later of the two is 1 (3 players) or 2 (4 players) turn
//                  ends back (te1, te2); with >= 3 players and turns of >= 2 steps those lie >= 2
//                  steps back.
//   drawing wave   records r, r + 1 (r even) once written: the plays replayed on the acting players'
//                  decks (img: two byte updates each), then ONE turn-end pass -- a lean turn lasts at least two steps (pass
//                  in MOVEMENT, pass in BUYING), so a player ends at most one turn in two records --
//                  and the deck granules each record changed (ring granule 2, bits 16..22);
//                  cnt[DRAW] = r + 2
//   storing wave B record r once written: step r + 4's presampled draws (cnt[PRE] = r + 1), the
//                  selected mask, Info, action, dones / agent_selection; on a second cursor
//                  kTrioBLag records behind, once drawn, the changed deck granules straight from img -- a granule a later record changed again may
//                  already hold that later value (or be read mid-update), but that record stores
//                  it again, in order, so the last store of every granule is its final value;
//                  cnt[STB] = r + 1
//   storing wave A record r once drawn: ObsData, the stored masks; cnt[STA] = r + 1
// The waits form no cycle: every wait of the stepping wave needs only records it has published.
// A wait that outlasts kTrioSpinLimit polls (a bug, never a slow wave) sets F_SYNC_TIMEOUT, the
// host error word and a sticky abort counter that ends every wait of the workgroup, so that no
// fault can hang the GPU.
//
// record t: 0 ObsData 16128.. (the phase dword from the stepping wave; the resources from the
// drawing wave; the lean step never changes the shop), 1 selected-mask bits + meta, 2 the acting
// player's stored-mask bits (saved mask at a turn end: the drawing wave adds the drawn cards) +
// action byte 0 + n_active of the acting player << 8 (the drawing wave's in the LAT form) + the deck
// granules the record changed << 16 (drawing wave).  The next player's stored mask changes only at a
// turn end, by fixed heads (the lean step), so storing wave A derives it from its own image.  The
// neighbourhood caches never change in the lean step (no moves): the stepping wave and storing wave
// A keep their own copies, and the epilogue does not store them.  The acting player's counters: the
// stepping wave's, written to LDS at a turn end (for the drawing wave) and at a park or the end (for
// the epilogue); in the LAT form the drawing wave's alone.
constexpr int kTrioRingG = 3;
#ifndef COG_TRIO_DEPTH                                     // (diagnostic builds)
#define COG_TRIO_DEPTH 8                                   // (16 measured the same: profiles/r05i_trio_depth16.txt, r05_trio_ab.txt r05z7)
#endif
constexpr int kTrioDepth = COG_TRIO_DEPTH;                 // ring slots (records in flight)
constexpr int kTrioLead = 4;                               // presampled draws: steps ahead of the record
#ifndef COG_TRIO_BLAG                                      // (diagnostic A/B builds)
#define COG_TRIO_BLAG 2
#endif
constexpr int kTrioBLag = COG_TRIO_BLAG;                   // storing wave B: deck cursor behind its front
// CNT_ABORT: set (sticky) by the first progress wait that times out; every later wait of every
// wave returns at once, so a broken invariant ends the launch promptly with the error set
// (instead of one ~0.2 s timeout per remaining wait)
enum TrioCnt : int { CNT_REC = 0, CNT_DRAW, CNT_STA, CNT_STB, CNT_PRE, CNT_FIN, CNT_ABORT, kTrioCnts };
constexpr uint32_t kTrioSpinLimit = 1u << 21;             // polls (~0.2 s)
struct TrioLds {
  uint2 img[4][5][64];                // every player's compact DeckObs (the drawing wave's): piles of types 0-7
  uint4 ring[kTrioDepth][kTrioRingG][64];   // record t (above), slot t % kTrioDepth
  uint32_t srng[kTrioDepth][64];      // the sampler state after step t, slot t % kTrioDepth
  uint3 pre[kTrioLead][64];           // step t's presampled draws, t % 4: state, head 0's draw | risk << 31, state after
  uint4 pl[4][64];
  uint4 heads[4][64];
  uint4 stbA[4][64];                  // storing wave A: every player's stored mask as last stored (bits)
  uint32_t wide[64];                  // the env's deck holds a type >= 8 (the drawing wave's prologue)
  uint32_t flg[64];                   // the other waves' hazard flags (the stepping wave's epilogue)
  uint32_t cnt[kTrioCnts];            // progress counters
  UidEntry tab[kUidTab];
};
static_assert(sizeof(TrioLds) <= 54613, "three trio workgroups per CU (trio_pad_lds keeps two)");
static_assert((kTrioDepth & (kTrioDepth - 1)) == 0 && kTrioDepth >= 4, "ring slots: a power of two");

// A wave keeps the counters it last read (wave-uniform, in SGPRs) and reads them again -- all six
// in one round trip -- only when the one it needs is short: the counters only grow, and what an
// acquire read once made visible stays so.  A waiting wave sleeps between reads.
struct TrioCnt6 {
  uint32_t rec = 0, draw = 0, sta = 0, stb = 0, pre = 0, fin = 0, abort = 0;
};
DEV void cnt_read(const TrioLds &D, TrioCnt6 &c) {
  uint32_t v[kTrioCnts];
#pragma unroll
  for (int k = 0; k < kTrioCnts; k++) v[k] = __hip_atomic_load(&D.cnt[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  c.rec = __builtin_amdgcn_readfirstlane(v[CNT_REC]);
  c.draw = __builtin_amdgcn_readfirstlane(v[CNT_DRAW]);
  c.sta = __builtin_amdgcn_readfirstlane(v[CNT_STA]);
  c.stb = __builtin_amdgcn_readfirstlane(v[CNT_STB]);
  c.pre = __builtin_amdgcn_readfirstlane(v[CNT_PRE]);
  c.fin = __builtin_amdgcn_readfirstlane(v[CNT_FIN]);
  c.abort = __builtin_amdgcn_readfirstlane(v[CNT_ABORT]);
}
// Publishes this wave's earlier LDS writes, all lanes' included, through lane 0's store of the
// counter.  The LDS executes one wave's DS instructions in issue order (their lgkmcnt returns are
// in order), so a wave that reads the counter's new value and then the records reads what was
// written before it: the ordering that matters is the compiler's, which a wavefront-scope fence
// keeps (no instruction).  A workgroup-scope release would add an s_waitcnt lgkmcnt(0) on the
// stepping wave's path every step, waiting also for its own reads in flight ($COG_TRIO_FENCE
// builds, -DCOG_TRIO_FENCE, keep that form for A/B).
DEV void cnt_store(TrioLds &D, int k, uint32_t v) {
#ifdef COG_TRIO_FENCE
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(&D.cnt[k], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(&D.cnt[k], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}
// wait (wave-uniform) until counter `field` of c (a member of c) >= v
#ifdef COG_ISSUE_COUNT
// (diagnostic ISA builds, tools/issue_frac.py: the no-wait path alone -- what a step issues when
// the counter it needs is already there; the waits are the stamps' own phases)
DEV void cnt_wait(TrioLds &, TrioCnt6 &, const uint32_t &field, uint32_t v, const DevState &) {
  if (field < v) asm volatile("s_nop 0");
}
#else
DEV void cnt_wait(TrioLds &D, TrioCnt6 &c, const uint32_t &field, uint32_t v, const DevState &s) {
  // (the common case first, alone: one scalar compare and branch -- the sticky abort matters only
  // to a wave that would wait)
  if (__builtin_expect(field >= v, 1)) return;
  if (c.abort) return;
  for (uint32_t spins = 0;; spins++) {
    cnt_read(D, c);
    if (field >= v || c.abort) return;
    if (spins >= kTrioSpinLimit) {
      if ((threadIdx.x & 63) == 0) {
        atomicOr(&s.status[0], F_SYNC_TIMEOUT);
        atomicAdd(&s.status[1], 1u);
        *s.err = 1u;
        __hip_atomic_store(&D.cnt[CNT_ABORT], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      c.abort = 1u;
      return;
    }
    __builtin_amdgcn_s_sleep(2);                           // (1 or 0: the same, r05y2)
  }
}
#endif
// the stepping wave's presampled record: {the state the step starts from, head 0's index for every
// play-head size k = 2..9 (4 bits each: uid_tab_accepted of the first draw, the narrow hand's play
// head holds at most the pass bit and types 0-7), the state after the five draws | any draw could be
// rejected << 31} -- the divisions off the stepping wave's chain (storing wave B has the slack)
DEV uint3 pre_pack(const uint4 p, bool jtab) {
  if (!jtab) return make_uint3(p.x, p.y, p.z | p.w << 31);   // head 0's draw itself
  uint32_t jt = 0u;
#pragma unroll
  for (int k = 2; k <= 9; k++) {
    const UidEntry e = uid_entry((uint32_t)k);
    jt |= uid_tab_accepted(p.y, e.s, e.m) << (4 * (k - 2));
  }
  return make_uint3(p.x, jt, p.z | p.w << 31);
}

// the epilogue's player records (lds_store_wave without the neighbourhood caches)
DEV void trio_store_players(const TrioLds &D, const DevState &s, int ne) {
  const int l = (int)(threadIdx.x & 63);
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const int f = j * 64 + l, e = min(f >> 2, ne - 1), q = f & 3;
    reinterpret_cast<uint4 *>(s.priv + e)[4 + q] = D.pl[q][e];
    s.heads[5 * e + 1 + q] = D.heads[q][e];
  }
}

// ---- the stepping wave's lean image and the compact deck (round 5) ----------------------------
// Decks in LDS hold types 0-7 only ("narrow": the canonical loop's decks never hold another type --
// no purchases, no specials -- DeckObs piles draw / hand / active / played / discard, 8 counts
// each, a uint2 per pile): 160 B per env instead of 448, so that four workgroups fit a CU's LDS and
// the metric's 65,536 envs step in one round.  An env whose deck holds a type >= 8 (compact_of
// says wide) is parked at step 0 and run by k_env_fixup's full step.  The acting player's hand is
// the stepping wave's copy of its compact hand pile (two dwords of u8 counts).
// DeckObs byte offset of pile p (api.h:67-82): 21 p
DEV void deck_expand(const uint2 pile[5], uint4 dk[7]) {   // compact -> the record's 7 granules
  uint32_t d[28];
#pragma unroll
  for (int k = 0; k < 28; k++) d[k] = 0u;
#pragma unroll
  for (int p = 0; p < 5; p++) {
    const int b = 21 * p, q = b >> 2, sh = b & 3;          // compile-time
    const uint32_t lo = pile[p].x, hi = pile[p].y;
    if (sh == 0) {
      d[q] |= lo;
      d[q + 1] |= hi;
    } else {
      d[q] |= lo << (8 * sh);
      d[q + 1] |= __builtin_amdgcn_alignbyte(hi, lo, 4 - sh);
      d[q + 2] |= hi >> (8 * (4 - sh));
    }
  }
#pragma unroll
  for (int k = 0; k < 7; k++) dk[k] = make_uint4(d[4 * k], d[4 * k + 1], d[4 * k + 2], d[4 * k + 3]);
}
// the record's granules -> compact piles; false: a count of a type >= 8 is non-zero (wide)
DEV bool compact_of(const uint4 dk[7], uint2 pile[5]) {
  uint32_t d[28];
#pragma unroll
  for (int k = 0; k < 7; k++) { d[4 * k] = dk[k].x; d[4 * k + 1] = dk[k].y; d[4 * k + 2] = dk[k].z; d[4 * k + 3] = dk[k].w; }
  uint32_t rest = 0u;                                      // every byte of types 8..20: one
#pragma unroll                                             // compile-time byte mask per dword
  for (int k = 0; k < 28; k++) {
    uint32_t m = 0u;
#pragma unroll
    for (int y = 4 * k; y < 4 * k + 4; y++)
      if (y < 105 && y % 21 >= 8) m |= 0xffu << (8 * (y & 3));
    if (m) rest |= d[k] & m;
  }
#pragma unroll
  for (int p = 0; p < 5; p++) {
    const int b = 21 * p, q = b >> 2, sh = b & 3;
    pile[p].x = sh ? __builtin_amdgcn_alignbyte(d[q + 1], d[q], sh) : d[q];
    pile[p].y = sh ? __builtin_amdgcn_alignbyte(d[q + 2], d[q + 1], sh) : d[q + 1];
  }
  return rest == 0u;
}
// card c (< 8) leaves the compact hand (Deck::activate's hand part, player.cpp:45-60,
// cards.cpp:242-253: hand[c] - 1, u8): the count before
DEV uint32_t hand_take(uint2 &h, int c) {
  const uint32_t sh = 8u * (uint32_t)(c & 3);
  const uint32_t w = c < 4 ? h.x : h.y;
  const uint32_t prev = (w >> sh) & 0xffu;
  const uint32_t nw = (w & ~(0xffu << sh)) | (((prev - 1u) & 0xffu) << sh);
  h.x = c < 4 ? nw : h.x;
  h.y = c < 4 ? h.y : nw;
  return prev;
}
// the selected mask's heads 1-4 are {0} (special, remove, move, shop: MBits bits 22.., w1, w2)
DEV bool heads14_zero(const MBits &b) { return (b.w0 >> 22) == 1u && b.w1 == (1u << 12) && b.w2 == 0x204u; }
constexpr uint32_t kMoveShopBits = (0x7fu << 2) | (0x7ffffu << 9);   // MBits w2: move and shop heads
// the j-th set bit of m (j < popc(m)): clear the lowest set bit j times, as many rounds as the
// wave's largest j (the play head holds the pass bit and the hand's types: j <= 3 in the canonical
// loop, where the binary search of nth_set_bit costs five full rounds)
DEV uint32_t nth_set_bit_iter(uint32_t m, uint32_t j) {
  while (__builtin_amdgcn_ballot_w64(j != 0u)) {
    m = j ? (m & (m - 1u)) : m;
    j = j ? j - 1u : 0u;
  }
  return (uint32_t)(__ffs(m) - 1);
}
// head 0's draw from the presampled record when the state is the one it starts from and heads
// 1-4 are {0} (then the five draws are the presampled ones: act 1-4 = 0); false: sample the
// sequential way
DEV bool sample_lean(const MBits &sel, const uint3 &pr, uint32_t &rng, uint32_t &a0, bool jtab, const UidEntry *tab) {
  const uint32_t m0 = sel.w0 & 0x3fffffu, k0 = __popc(m0);
  if (!(pr.x == rng && (pr.z >> 31) == 0u && heads14_zero(sel) && k0 >= 1u && k0 <= 9u)) return false;
  uint32_t j;
  if (jtab) {
    j = k0 >= 2u ? (pr.y >> (4u * (k0 - 2u))) & 15u : 0u;
  } else {
    const UidEntry e0 = tab[k0];
    j = k0 >= 2u ? uid_tab_accepted(pr.y, e0.s, e0.m) : 0u;
  }
  a0 = nth_set_bit_iter(m0, j);
  rng = pr.z;
  return true;
}
DEV uint4 pack_lean_player(uint4 pp, uint32_t n_in_hand, uint32_t n_active, uint32_t steps_taken) {
  pp.y = (pp.y & 0xff0000ffu) | (n_in_hand & 0xffu) << 8 | (n_active & 0xffu) << 16;
  pp.z = (pp.z & 0xffff00ffu) | (steps_taken & 0xffu) << 8;
  return pp;
}
// the lean step may run for this player: no move, free card, free move or pending removes in
// progress, has not won (PlayerPriv x: has_won, mip, n_removes, next_card_free; y byte 0:
// next_move_free)
DEV bool lean_player(const uint4 &pp) { return (pp.x | (pp.y & 0xffu)) == 0u; }
// the env-level private records from the stepping wave (duo_store_env_private<true> with the
// selected mask as bits)
DEV void trio_store_private(const DevState &s, size_t i, const RegEnv &R, const MBits &selb) {
  uint4 *pw = reinterpret_cast<uint4 *>(s.priv + i);
  reinterpret_cast<uint3 *>(reinterpret_cast<uint32_t *>(pw) + 1)[0] = make_uint3(R.seed, R.max_steps, R.turn_counter);
  pw[1] = make_uint4(R.g1x, R.g1y, R.in_market, R.flags);
  s.heads[5 * i] = mbits_u4(selb);                         // (Info steps: the drawing wave's)
}

template <int SRC, bool LAT>
DEV void trio_stepper(TrioLds &D, const DevState &s_glob, int steps, int epw, uint32_t *__restrict__ rngs_glob) {
  const int l = (int)(threadIdx.x & 63);
  const size_t wbase = (size_t)blockIdx.x * epw;
  const DevState s = wave_view(s_glob, wbase);
  const size_t i = (size_t)l;
  const int ne = (int)min((size_t)epw, s_glob.n - wbase);
  uint32_t *__restrict__ rngs = rngs_glob + wbase;
  bool live = l < ne;
  uint32_t park = kParkNone, srng = 0;
  PH_DECL;                                                 // (diagnostic builds: phase stamps)
  TL(10);                                                  // (and the launch timeline: slots 10..14)
  RegEnv R;                                                // env level (the lean image below)
  uint2 cells[4];                                          // every player's neighbourhood cache
  // the steps of the last two turn ends before the current step (-1: none in this launch); the
  // lean loop passes the turn strictly in order, so the last turn end of the player after the next
  // agent -- the later of the two records the turn change reads -- lies 1 (3 players) or 2 (4
  // players) turn ends back
  int te1 = -1, te2 = -1;
  int ag = 0, na = 0;
  MBits selb = {0u, 0u, 0u}, stab = selb, stnb = selb;     // selected, stored(ag), stored(na)
  // The acting player's counters (steps_taken, n_in_hand, n_active, idx_last) are kept by this
  // wave and handed to the drawing wave at turn changes when two workgroups share a CU (their
  // total work per CU counts), and by the drawing wave alone when a workgroup has its CU to
  // itself (LAT: the stepping wave's chain counts): profiles/r05_trio_ab.txt r05z3 / r05z5
  constexpr bool lat = LAT;
  uint4 pp = make_uint4(0u, 0u, 0u, 0u);                   // PlayerPriv of ag (packed)
  uint32_t n_in_hand = 0u, n_active = 0u, steps_taken = 0u;
  uint32_t own = 0u;                                       // each player's own hex code (a byte each)
  if (live) {
    Snap S;
    load_env(s, i, S);
    regs_env(R, S);
    const uint4 *pv4 = reinterpret_cast<const uint4 *>(s.priv + i);
#pragma unroll
    for (int p = 0; p < 4; p++) {
      D.pl[p][l] = pv4[4 + p];
      cells[p] = reinterpret_cast<const uint2 *>(pv4 + 8)[p];
      D.heads[p][l] = s.heads[5 * i + 1 + p];
    }
    srng = rngs[i];
    ag = (int)R.agent();
    na = (int)next_player((uint32_t)ag, R.n_players());
    pp = D.pl[ag][l];
    n_in_hand = (pp.y >> 8) & 0xffu;
    n_active = (pp.y >> 16) & 0xffu;
    steps_taken = (pp.z >> 8) & 0xffu;
#pragma unroll
    for (int p = 0; p < 4; p++) own |= (cells[p].x & 0xffu) << (8 * p);   // (neighbourhood cell 0)
    selb = S.sel;
    stab = mbits_of(D.heads[ag][l]);
    stnb = mbits_of(D.heads[na][l]);
  }
  R.tab = D.tab;
  __builtin_amdgcn_s_waitcnt(0);                           // (no per-iteration vmcnt wait covers them)
  TL(15);                                                  // (timeline: this wave's prologue done)
  __syncthreads();                                         // B: every wave's prologue is done
  uint2 H = make_uint2(0u, 0u);                            // ag's hand (compact: types 0-7)
  bool lean_p = false, narrow = false;
  if (live) {                                              // from the drawing wave's image
    H = D.img[ag][1][l];
    narrow = D.wide[l] == 0u;
    lean_p = narrow && lean_player(pp);
  }
  PH(6);                                                   // the prologue (to the barrier)
  TL(11);
  TrioCnt6 cc;
  // step t + 1's presampled record, read at the end of step t when storing wave B is known to be
  // past it (so that the read's latency overlaps the record's stores); else at step t + 1's start
  uint3 pr_next = D.pre[0][l];
  bool have_next = true;
  // the next turn change's records read ahead (pf_ok: valid)
  uint2 pf_hd = make_uint2(0u, 0u);
  uint4 pf_pla = make_uint4(0u, 0u, 0u, 0u), pf_hdn = pf_pla;
  bool pf_ok = false;
  for (int t = 0; t < steps; t++) {
    const int sl = t & (kTrioDepth - 1);
    if (t >= kTrioDepth) {                                 // slot t % kTrioDepth free
      cnt_wait(D, cc, cc.sta, (uint32_t)(t - kTrioDepth + 1), s_glob);
      cnt_wait(D, cc, cc.stb, (uint32_t)(t - kTrioDepth + 1), s_glob);
    }
    PH(9);
    if (!have_next) cnt_wait(D, cc, cc.pre, (uint32_t)(t - kTrioLead + 1), s_glob);   // (t >= kTrioLead)
    PH(2);
    bool ended = false, finish = false, turn_end = false, stepped = false;
    uint32_t a_play = 0u;
    // (round 6: the common path computed by every lane with selects -- no exec-mask branches, which
    // a 64-env wave would take on nearly every step anyway; the rare parts keep their branches)
    {
      const uint32_t srng0 = srng;
      uint3 pr = pr_next;                                  // (have_next is wave-uniform: a scalar
      if (!have_next) pr = D.pre[t & (kTrioLead - 1)][l];  // branch, not a select of addresses)
      // head 0's draw from the presampled record when the state is the one it starts from and heads
      // 1-4 are {0} (then the five draws are the presampled ones: act 1-4 = 0; sample_lean)
      const uint32_t m0 = selb.w0 & 0x3fffffu, k0 = __popc(m0);
      const bool fast = live && pr.x == srng && (pr.z >> 31) == 0u && heads14_zero(selb) && k0 - 1u < 9u;
      uint32_t j;
      if (LAT) {
        j = (pr.y >> (4u * ((k0 - 2u) & 7u))) & 15u;      // (head 0's index table, k0 = 2..9)
      } else {
        const UidEntry e0 = R.tab[k0 & (kUidTab - 1)];
        j = uid_tab_accepted(pr.y, e0.s, e0.m);
      }
      j = fast && k0 >= 2u ? j : 0u;
      const uint32_t a0 = nth_set_bit_iter(m0, j);
      a_play = fast ? a0 : 0u;
      srng = fast ? pr.z : srng;
      bool other = false;                                  // an action head other than play set
      if (__builtin_amdgcn_ballot_w64(live && !fast) && live && !fast) {   // (wave-uniform skip)
#ifdef COG_ISSUE_COUNT                                     // (diagnostic ISA builds, tools/issue_frac.py:
        other = true;                                      // the rare fallback's code out of the count)
#else
        uint8_t act[5];
        R.sel = heads_of(selb);
        step_action<SRC>(R, make_uint2(0u, 0u), srng, act);
        a_play = act[0];
        other = ((uint32_t)act[1] | act[2] | act[3] | act[4]) != 0u;
#endif
      }
      other = other || a_play > 8u;                        // (a type >= 8: not in a narrow deck's hand)
      const bool was_done = R.done() != 0u;
      // not the lean step's case (never in the canonical loop), or the test hooks: hand the env to
      // k_env_fixup before its step t
      bool hook = false;                                   // (test hooks: t uniform, so a scalar
      if (t == s.redo_at) hook = s.redo_env < 0 || (int)(wbase + i) == s.redo_env;   // branch in the loop)
      const bool parks = live && !was_done && (!lean_p || other || hook);
      stepped = live && !was_done && !parks;               // cog_env::step, the lean case (Info steps
      if (__builtin_amdgcn_ballot_w64(parks) && parks) {   // and the resources: the drawing wave's)
        srng = srng0;
#ifndef COG_ISSUE_COUNT                                    // (a rare lane's stores: out of the count)
        trio_store_private(s, i, R, selb);
        rngs[i] = srng;
#endif
        if (!lat) D.pl[ag][l] = pack_lean_player(pp, n_in_hand, n_active, steps_taken);   // (the epilogue's)
        park = (uint32_t)t | kParkRedo;
        live = false;
      }
      uint32_t phase = R.sh[0] & 0xffu;
      if (phase == COG_PHASE_INACTIVE) phase = COG_PHASE_MOVEMENT;
      if (!lat) steps_taken = stepped ? (steps_taken + 1u) & 0xffu : steps_taken;
      // Player::play_card (player.cpp:45-60): Deck::activate's hand part (the active pile and the
      // counters: the drawing wave); the play bit (its special bit stays clear: types 0-7 are not
      // special, is_special; a type >= 8 has parked above)
      const bool play = stepped && a_play != 0u;
      const int c = (int)((a_play - 1u) & 7u);
      uint2 Hp = H;
      const uint32_t prev = hand_take(Hp, c);
      H = play ? Hp : H;
      const uint32_t bp = 1u << (c + 1);
      selb.w0 = play ? (prev > 1u ? (selb.w0 | bp) : (selb.w0 & ~bp)) : selb.w0;
      if (!lat) {
        n_in_hand = play ? (n_in_hand - 1u) & 0xffu : n_in_hand;
        n_active = play ? (n_active + 1u) & 0xffu : n_active;
        pp.z = play ? (pp.z & ~0xffu) | (uint32_t)c : pp.z;   // idx_last
      }
      const uint32_t nph = phase == COG_PHASE_BUYING ? COG_PHASE_INACTIVE : phase + 1u;   // pass: next phase
      phase = stepped && !play ? nph : phase;
      turn_end = stepped && phase == COG_PHASE_INACTIVE;   // maybe_end_turn -> next_agent
      // (Player::end_turn: the drawing wave) save_actionmask, load_actionmask (na != ag: >= 3
      // players), update_observation's INACTIVE phase for the next player's stored mask
      n_active = turn_end ? 0u : n_active;
      const MBits sel0 = selb;
      selb.w0 = turn_end ? stnb.w0 : selb.w0;
      selb.w1 = turn_end ? stnb.w1 : selb.w1;
      selb.w2 = turn_end ? stnb.w2 : selb.w2;
      stab.w0 = turn_end ? sel0.w0 : stab.w0;
      stab.w1 = turn_end ? sel0.w1 : stab.w1;
      stab.w2 = turn_end ? sel0.w2 : stab.w2;
      stnb.w2 = turn_end ? (stnb.w2 & ~kMoveShopBits) | 0x204u : stnb.w2;
      R.g1y = turn_end ? (R.g1y & ~0xffu) | ((uint32_t)na & 0xffu) : R.g1y;   // R.set_agent(na)
      R.turn_counter += turn_end ? 1u : 0u;
      R.sh[0] = stepped ? (R.sh[0] & ~0xffu) | phase : R.sh[0];
      // done (environment.cpp:183-207): the (next) agent's cell or the turn counter.  Both change
      // only with the turn here (no move: the agent's cell is the one checked after its last step,
      // never an end; a player's own cell is never an out-of-bounds lookup)
      finish = turn_end && (COG_HEX_END((own >> (8 * na)) & 0xffu) || R.turn_counter >= R.max_steps);
      R.g1x = finish ? (R.g1x & 0x00ffffffu) | (1u << 24) : R.g1x;   // R.set_done(1)
      PH(0);
      ended = live && (was_done || finish);
    }
    uint4(*ring)[64] = D.ring[sl];
    int ag1 = ag, na1 = na;
    if (live) {
      ag1 = (int)R.agent();
      na1 = (int)next_player((uint32_t)ag1, R.n_players());
    }
    const bool tc = live && ag1 != ag;                     // turn change: ag1 == na acts next
    // the new agent's records (hand, counters) and the next player's (stored mask), once the
    // drawing wave is past their last turn ends; read ahead of the record's stores, so that their
    // latency overlaps them
    // (read ahead at an earlier step of the turn when the drawing wave was past them: pf_ok)
    // (the records land in pf_* themselves: the turn change below takes them from there, and
    // re-reads ahead after it -- no copies of ten dwords through every step)
    const bool slow = tc && !pf_ok;
    if (__builtin_amdgcn_ballot_w64(slow)) {
      const int need = R.n_players() == 3u ? te1 : te2;   // the later of ag1's and na1's last turn ends
      // the drawing wave past record max(need) over the wave: its distance from t by ballots (no
      // cross-lane shuffles, which go through LDS); >= 2 in play (>= 3 players, turns of >= 2
      // steps), and from 5 on it asks for a little more than it needs.  (needw folds the lane's
      // condition into the value, so that each ballot is one compare)
      const int needw = slow && need >= 0 ? need : INT32_MIN;
      if (__builtin_amdgcn_ballot_w64(needw >= 0)) {
        int dmin = 5;
#pragma unroll
        for (int d = 4; d >= 1; d--) dmin = __builtin_amdgcn_ballot_w64(needw >= t - d) ? d : dmin;
        PH(4);
        cnt_wait(D, cc, cc.draw, (uint32_t)(t - dmin + 1), s_glob);
        PH(5);
      }
      if (slow) {
        pf_hd = D.img[ag1][1][l];
        pf_pla = D.pl[ag1][l];
        pf_hdn = D.heads[na1][l];
      }
    }
    if (live) {
      if (!lat && (tc || ended)) D.pl[ag][l] = pack_lean_player(pp, n_in_hand, n_active, steps_taken);
      const uint32_t meta = kMetaValid | (uint32_t)ag << 2 | (uint32_t)na << 4 | (uint32_t)na1 << 6 |
                            (ended ? kMetaEnded : 0u) | (stepped ? kMetaStepped : 0u) | (uint32_t)ag1 << 24;
      ring[0][l].x = R.sh[0];                              // (the resources: the drawing wave's)
      ring[1][l] = make_uint4(selb.w0, selb.w1, selb.w2, meta);
      ring[2][l] = make_uint4(stab.w0, stab.w1, stab.w2, a_play | (lat ? 0u : (n_active & 0xffu) << 8));
      D.srng[sl][l] = srng;
    } else {
      ring[1][l] = make_uint4(0u, 0u, 0u, 0u);             // no record
    }
    cnt_store(D, CNT_REC, (uint32_t)(t + 1));
    // (B rewrites slot (t + 1) % 4 only after record t + 1: this read is issued before that)
    have_next = t + 1 < kTrioLead || cc.pre >= (uint32_t)(t + 2 - kTrioLead);
    if (have_next) pr_next = D.pre[(t + 1) & (kTrioLead - 1)][l];
    PH(1);
    if (tc) {
      te2 = te1;
      te1 = t;
      H = pf_hd;                                           // its hand from the drawing wave
      pp = pf_pla;
      n_in_hand = (pf_pla.y >> 8) & 0xffu;
      n_active = (pf_pla.y >> 16) & 0xffu;
      steps_taken = (pf_pla.z >> 8) & 0xffu;
      lean_p = narrow && lean_player(pf_pla);
      stab = stnb;
      stnb = mbits_of(pf_hdn);
      pf_ok = false;
    }
    // the next turn change's records (the agent after ag1 and the player after it), read ahead
    // once the drawing wave is past their last turn ends (the counter as last read: no wait)
    if (live && !pf_ok && !ended) {
      const int need = R.n_players() == 3u ? te1 : te2;   // (as the turn change itself will ask)
      if (need < 0 || cc.draw >= (uint32_t)(need + 1)) {
        const int nn = (int)next_player((uint32_t)na1, R.n_players());
        pf_hd = D.img[na1][1][l];
        pf_pla = D.pl[na1][l];
        pf_hdn = D.heads[nn][l];
        pf_ok = true;
      }
    }
    if (live && ended) {                                   // hand the env to k_env_fixup
#ifndef COG_ISSUE_COUNT
      trio_store_private(s, i, R, selb);
      rngs[i] = srng;
#endif
      park = (uint32_t)t | (finish ? kParkFinish : 0u);
      live = false;
    }
    ag = ag1;
    na = na1;
    PH(3);
  }
  TL(12);
  if (live && !lat) D.pl[ag][l] = pack_lean_player(pp, n_in_hand, n_active, steps_taken);   // (the epilogue's)
  cnt_store(D, CNT_REC, (uint32_t)steps + 1u);             // the loop is over (storing wave A's epilogue)
  // the env-level private state back to HBM (lat: while the other waves drain; the flags word after
  // them: it takes their hazard flags); no other wave reads these words in the launch
  uint4 *pw = reinterpret_cast<uint4 *>(s.priv + i);
  if (lat) {
    if (live) {
      reinterpret_cast<uint3 *>(reinterpret_cast<uint32_t *>(pw) + 1)[0] = make_uint3(R.seed, R.max_steps, R.turn_counter);
      s.heads[5 * i] = mbits_u4(selb);
      rngs[i] = srng;
    }
    if (l < ne) s.park[i] = park;
    park_list_push(s_glob, park != kParkNone);
  }
  cnt_wait(D, cc, cc.fin, 3u, s_glob);                     // the other waves are done
  PH(7);                                                   // the drain (the other waves' last records)
  TL(13);
  const uint32_t fl = D.flg[l];                            // their hazard flags
  if (lat) {
    if (live) pw[1] = make_uint4(R.g1x, R.g1y, R.in_market, R.flags | fl);
    else if (l < ne && fl) reinterpret_cast<uint32_t *>(pw)[7] = R.flags | fl;   // a parked env: its last records'
  } else {
    if (live) {
      R.flags |= fl;
      trio_store_private(s, i, R, selb);
      rngs[i] = srng;
    } else if (l < ne && fl) {
      reinterpret_cast<uint32_t *>(pw)[7] = R.flags | fl;
    }
    if (l < ne) s.park[i] = park;
    park_list_push(s_glob, park != kParkNone);
  }
  trio_store_players(D, s, ne);                            // every player's records (cooperative)
  PH(8);                                                   // the epilogue's stores (issued)
  TL(14);
  PH_FLUSH(s_glob);
}

// One record's play on the drawing wave (trio_drawer; round 6): the acting player's counters
// (LAT), the ObsData phase / resources granule, the Info steps byte and Deck::activate's hand /
// active piles, on the values the caller read (p4: D.pl[ag], h / a: D.img[ag][1 / 2]), which it
// updates and stores back; selects instead of exec-mask branches for the common path.
template <bool LAT>
DEV void trio_draw_play(TrioLds &D, const DevState &s, int l, bool live, int slot, uint32_t mt, uint32_t w2,
                        uint32_t gx, uint4 &p4, uint2 &h, uint2 &a, uint4 &shb0, uint32_t &infob, bool &te,
                        bool &rec_out, uint32_t &dm, uint32_t &nact) {
  const size_t i = (size_t)l;
  const int ag = (int)((mt >> 2) & 3u);
  const bool valid = live && (mt & kMetaValid);
  const bool rec = valid && (mt & kMetaStepped);
  rec_out = rec;
  te = rec && (int)(mt >> 24) != ag;
  const uint32_t a_play = w2 & 0xffu;
  const bool play = rec && a_play != 0u;
  const int c = (int)((a_play - 1u) & 7u);               // (c < 8: the stepping wave parks any other type)
  if (LAT) {                                             // the acting player's counters (PlayerPriv:
    uint4 q = p4;                                        // steps_taken, n_in_hand, n_active, idx_last;
    uint32_t na = (q.y >> 16) & 0xffu;                   // Player::play_card, player.cpp:45-60; u8)
    q.z = (q.z & 0xffff00ffu) | (((q.z >> 8) + 1u) & 0xffu) << 8;
    q.y = play ? (q.y & 0xffff00ffu) | ((((q.y >> 8) & 0xffu) - 1u) & 0xffu) << 8 : q.y;
    na = play ? (na + 1u) & 0xffu : na;
    q.z = play ? (q.z & ~0xffu) | (a_play - 1u) : q.z;
    na = te ? 0u : na;                                   // Player::end_turn
    q.y = (q.y & 0xff00ffffu) | na << 16;
    p4.x = rec ? q.x : p4.x;                             // (component selects: a select of two
    p4.y = rec ? q.y : p4.y;                             // vectors compiles to one of two addresses
    p4.z = rec ? q.z : p4.z;                             // in scratch)
    if (rec) D.pl[ag][l] = p4;
    nact = rec ? na : 0u;
  }
  // the ObsData phase / resources granule and the Info byte (the stepping wave leaves the resources
  // and the counts to this wave)
  infob = rec ? (infob & ~(0xffu << (8 * ag))) | ((((infob >> (8 * ag)) + 1u) & 0xffu) << (8 * ag)) : infob;
  uint32_t phase = shb0.x & 0xffu;
  phase = phase == COG_PHASE_INACTIVE ? (uint32_t)COG_PHASE_MOVEMENT : phase;
  const bool mv = play && phase == COG_PHASE_MOVEMENT, buy = play && phase == COG_PHASE_BUYING;
  const uint32_t coin = cardf(kRes2, c);                 // Player::play_card (player.cpp:45-60)
  uint4 g0 = shb0;
  g0.y = mv ? __float_as_uint((float)cardf(kRes0, c)) : g0.y;
  g0.z = mv ? __float_as_uint((float)cardf(kRes1, c)) : g0.z;
  const float bw = __uint_as_float(g0.w) + (coin > 0 ? (float)coin : 0.5f);
  g0.w = mv ? __float_as_uint((float)coin) : buy ? __float_as_uint(bw) : g0.w;
  g0.y = te ? 0u : g0.y;                                 // Player::end_turn (+0.f)
  g0.z = te ? 0u : g0.z;
  g0.w = te ? 0u : g0.w;
  g0.x = rec ? gx : g0.x;
  if (valid) {
    reinterpret_cast<uint3 *>(&D.ring[slot][0][l].y)[0] = make_uint3(g0.y, g0.z, g0.w);   // (storing wave A)
    s.info[i * COG_INFO_BYTES + COG_AGENT_INFO0 + COG_AGENT_INFO_STRIDE * ag] = (uint8_t)(infob >> (8 * ag));
    if (ne4(g0, shb0)) reinterpret_cast<uint4 *>(s.obs + i * COG_OBS_BYTES + COG_OBS_PHASE)[0] = g0;
  }
  shb0.x = valid ? g0.x : shb0.x;
  shb0.y = valid ? g0.y : shb0.y;
  shb0.z = valid ? g0.z : shb0.z;
  shb0.w = valid ? g0.w : shb0.w;
  // Deck::activate (cards.cpp:242-253): hand[c]--, active[c]++ (u8)
  const uint32_t sh = 8u * (uint32_t)(c & 3);
  uint32_t hw = c < 4 ? h.x : h.y, aw = c < 4 ? a.x : a.y;
  hw = (hw & ~(0xffu << sh)) | ((((hw >> sh) - 1u) & 0xffu) << sh);
  aw = (aw & ~(0xffu << sh)) | ((((aw >> sh) + 1u) & 0xffu) << sh);
  const bool lo = c < 4;
  h.x = play && lo ? hw : h.x;
  h.y = play && !lo ? hw : h.y;
  a.x = play && lo ? aw : a.x;
  a.y = play && !lo ? aw : a.y;
  if (play) {
    D.img[ag][1][l] = h;
    D.img[ag][2][l] = a;
  }
  const int bh = COG_DECK_HAND + c, ba = COG_DECK_ACTIVE + c;   // the record's granules
  dm = play ? 1u << (bh >> 4) | 1u << (ba >> 4) : 0u;
}

// The drawing wave keeps every player's deck (img).  It takes records in pairs r, r + 1 (r even):
// each record's play replayed on the acting player's deck (the hand and active piles, as
// Deck::activate does); then one pass over the turn ends of either record (discard + draws,
// duo_turn_end: the env rng is this wave's).  Which granules each record changed goes to storing
// wave B (ring granule 2, bits 16..22).  It also stores each record's ObsData phase/resources
// granule and Info steps byte (the resources for storing wave A in ring granule 0), and with LAT
// keeps the acting player's counters (PlayerPriv: steps_taken, n_in_hand, n_active, idx_last).
template <bool LAT>
DEV uint32_t trio_drawer(TrioLds &D, const DevState &s_glob, int steps, int epw) {
  PH_DECL;
  TL(14);                                                  // (timeline: this wave's start)
  const int l = (int)(threadIdx.x & 63);
  const size_t wbase = (size_t)blockIdx.x * epw;
  const DevState s = wave_view(s_glob, wbase);
  const size_t i = (size_t)l;
  const bool live = l < epw && wbase + (size_t)l < s_glob.n;
  uint32_t rng = 0u;                                       // the env rng
  bool narrow = true;
  constexpr bool lat = LAT;                                // (the acting player's counters: trio_stepper)
  uint4 shb0 = make_uint4(0u, 0u, 0u, 0u);                 // ObsData 16128.. as stored: the phase
  uint32_t infob = 0u;                                     // dword and the resources; Info steps
  if (live && !s_glob.cdeck_ok) {                          // the DeckObs records (else storing wave A
#pragma unroll                                             // loads the compact image the last launch left)
    for (int p = 0; p < 4; p++) {
      const uint4 *src = reinterpret_cast<const uint4 *>(deck_ptr(s, i, p));
      uint4 dk[7];
      uint2 pile[5];
#pragma unroll
      for (int k = 0; k < 7; k++) dk[k] = src[k];
      narrow = compact_of(dk, pile) && narrow;
#pragma unroll
      for (int q = 0; q < 5; q++) D.img[p][q][l] = pile[q];
    }
  }
  if (live) {
    rng = reinterpret_cast<const uint32_t *>(s.priv + i)[0];
    infob = reinterpret_cast<const uint32_t *>(s.priv + i)[12];   // EnvPriv granule 3, dword 0
    shb0 = reinterpret_cast<const uint4 *>(s.obs + i * COG_OBS_BYTES + COG_OBS_PHASE)[0];
  }
  if (!s_glob.cdeck_ok) D.wide[l] = narrow ? 0u : 1u;      // (a wide env: the stepper parks it at step 0)
  uint32_t flags = 0u;                                     // hazard flags of the draws
  __builtin_amdgcn_s_waitcnt(0);
  TL(15);                                                  // (timeline: this wave's prologue done)
  __syncthreads();                                         // B: the decks are in LDS
  PH_RESET;
  TrioCnt6 cc;
  for (int r = 0; r < steps; r += 2) {
    const int nrec = r + 1 < steps ? 2 : 1;
    cnt_wait(D, cc, cc.rec, (uint32_t)(r + nrec), s_glob);   // the records are written
    PH(8);
    if (r + nrec >= steps) TL(11);                         // (timeline: the last records written)
    const int slot[2] = {r & (kTrioDepth - 1), (r + 1) & (kTrioDepth - 1)};
    uint32_t dm[2] = {0u, 0u}, nact[2] = {0u, 0u};
    int agj[2] = {0, 0};
    bool te[2] = {false, false}, recj[2] = {false, false};
    // (round 6: both records' words, and both acting players' counters, hand and active piles, read
    // at once -- a second record of the same player continues from the first one's values in
    // registers -- and the common path computed with selects, not exec-mask branches)
    const uint32_t mt0 = D.ring[slot[0]][1][l].w, w20 = D.ring[slot[0]][2][l].w, gx0 = D.ring[slot[0]][0][l].x;
    uint32_t mt1 = D.ring[slot[1]][1][l].w;                // (a slot past nrec: read, not used)
    const uint32_t w21 = D.ring[slot[1]][2][l].w, gx1 = D.ring[slot[1]][0][l].x;
    if (nrec < 2) mt1 = 0u;                                // (uniform: no second record)
    const int ag0 = (int)((mt0 >> 2) & 3u), ag1 = (int)((mt1 >> 2) & 3u);
    uint4 p0 = make_uint4(0u, 0u, 0u, 0u), p1 = p0;
    if (lat) {
      p0 = D.pl[ag0][l];
      p1 = D.pl[ag1][l];
    }
    uint2 h0 = D.img[ag0][1][l], a0 = D.img[ag0][2][l], h1 = D.img[ag1][1][l], a1 = D.img[ag1][2][l];
    trio_draw_play<lat>(D, s, l, live, slot[0], mt0, w20, gx0, p0, h0, a0, shb0, infob, te[0], recj[0], dm[0], nact[0]);
    agj[0] = ag0;
    if (nrec > 1) {                                        // (uniform)
      if (ag1 == ag0) {                                    // the same player: record 0's values
        p1.x = p0.x; p1.y = p0.y; p1.z = p0.z; p1.w = p0.w;
        h1.x = h0.x; h1.y = h0.y;
        a1.x = a0.x; a1.y = a0.y;
      }
      trio_draw_play<lat>(D, s, l, live, slot[1], mt1, w21, gx1, p1, h1, a1, shb0, infob, te[1], recj[1], dm[1], nact[1]);
      agj[1] = ag1;
    }
    PH(7);                                                 // (stamps: the plays)
    const bool any = te[0] || te[1];                       // (at most one of them)
    if (__builtin_amdgcn_ballot_w64(any) && any) {         // the turn end's discard + draws
      const int j = te[1] ? 1 : 0, sl = te[1] ? slot[1] : slot[0], ag = te[1] ? agj[1] : agj[0];
      uint2 pile[5];
#pragma unroll
      for (int q = 0; q < 5; q++) pile[q] = D.img[ag][q][l];
      uint4 dk[7], old[7];
      deck_expand(pile, dk);
#pragma unroll
      for (int k = 0; k < 7; k++) old[k] = dk[k];
      const uint4 x = D.ring[sl][2][l];
      MBits ba{x.x, x.y, x.z};
      duo_turn_end(D, l, ag, dk, ba, rng, flags);          // (a narrow deck stays narrow)
      D.ring[sl][2][l] = make_uint4(ba.w0, ba.w1, ba.w2, x.w);
      uint32_t dd = 0;
#pragma unroll
      for (int k = 0; k < 7; k++) dd |= ne4(dk[k], old[k]) ? 1u << k : 0u;
      (void)compact_of(dk, pile);
#pragma unroll
      for (int q = 0; q < 5; q++) D.img[ag][q][l] = pile[q];
      dm[0] |= j == 0 ? dd : 0u;
      dm[1] |= j == 1 ? dd : 0u;
    }
#pragma unroll
    for (int j = 0; j < 2; j++)                            // granule 2's last dword: the action (the
      if (j < nrec) {                                      // stepping wave's), n_active, the changed deck
        uint32_t *w = &D.ring[slot[j]][2][l].w;            // granules (storing waves A and B)
        if (lat && recj[j]) *w = (*w & 0xffu) | nact[j] << 8 | dm[j] << 16;
        else reinterpret_cast<uint16_t *>(w)[1] = (uint16_t)dm[j];
      }
    cnt_store(D, CNT_DRAW, (uint32_t)(r + nrec));
    PH(9);
  }
  TL(12);
  if (live) {
    reinterpret_cast<uint32_t *>(s.priv + i)[0] = rng;     // the env rng after its last draws
    reinterpret_cast<uint32_t *>(s.priv + i)[12] = infob;  // Info steps (a parked env's: as of the park)
  }
  PH_FLUSH(s_glob);
  return flags;
}

// The store phase of the trio on two waves: wave A (PART 0) the stored masks --
// update_observation's heads of the acting player's when the turn goes on (the lean step leaves
// them) -- and wave B (PART 1) the presampled draws (presample; with LAT head 0's index table), the
// selected-mask record, the action, dones / agent_selection and the decks.  Each keeps its own
// images of what it stored last.
template <int PART, bool LAT>
DEV uint32_t trio_storer(TrioLds &D, const DevState &s_glob, int steps, int epw, const uint32_t *__restrict__ rngs_glob,
                         uint8_t *__restrict__ actions_glob) {
  PH_DECL;
  TL(14);                                                  // (timeline: this wave's start)
  const int l = (int)(threadIdx.x & 63);
  const size_t wbase = (size_t)blockIdx.x * epw;
  const DevState s = wave_view(s_glob, wbase);
  const size_t i = (size_t)l;
  const bool live = l < epw && wbase + (size_t)l < s_glob.n;
  uint8_t *__restrict__ av = actions_glob + wbase * COG_ACTION_BYTES;
  MBits selb = {0u, 0u, 0u};                               // B: the selected mask as stored
  uint2 cells[4];                                          // A: every player's neighbourhood cache
  uint32_t out = ~0u;                                      // B: dones[i] | agent_selection[i] << 8 as stored
  RegEnv E;                                                // A: update_observation's inputs and flags
  E.flags = 0u;
  E.avail = 0u;
  uint32_t x = 1u;                                         // B: the sampler state at step 0
  if (live) {
    if (PART == 0) {
      const uint4 *sh4 = reinterpret_cast<const uint4 *>(s.obs + i * COG_OBS_BYTES + COG_OBS_PHASE);
      const uint4 sh1 = sh4[1], sh2 = sh4[2];
      const uint4 *pv4 = reinterpret_cast<const uint4 *>(s.priv + i);
#pragma unroll
      for (int p = 0; p < 4; p++) {
        D.stbA[p][l] = s.heads[5 * i + 1 + p];
        cells[p] = reinterpret_cast<const uint2 *>(pv4 + 8)[p];
      }
      const uint4 g1 = pv4[1];
      const uint32_t w[5] = {sh1.x, sh1.y, sh1.z, sh1.w, sh2.x};
      E.avail = shop_avail_of(w, (g1.y >> 8) & 0xffu, g1.z);   // (no purchase in the lean step: fixed)
      if (s_glob.cdeck_ok) {                               // the drawing wave's compact decks as the
        const uint4 *src = s.cdeck + 10 * i;               // last launch left them (DevState::cdeck)
        uint4 c[10];
#pragma unroll
        for (int g = 0; g < 10; g++) c[g] = src[g];
#pragma unroll
        for (int g = 0; g < 10; g++) {                     // entries 2g, 2g + 1 of [player][pile]
          D.img[(2 * g) / 5][(2 * g) % 5][l] = make_uint2(c[g].x, c[g].y);
          D.img[(2 * g + 1) / 5][(2 * g + 1) % 5][l] = make_uint2(c[g].z, c[g].w);
        }
      }
    } else {
      selb = mbits_of(s.heads[5 * i]);
      x = rngs_glob[wbase + (size_t)l];
    }
  }
  if (PART == 0 && s_glob.cdeck_ok) D.wide[l] = live ? s.cwide[i] : 0u;   // (else the drawing wave's)
  if (PART == 1) {                                         // steps 0..3 from the state at step 0
#pragma unroll
    for (int k = 0; k < kTrioLead; k++) {
      const uint4 p = presample(x);
      D.pre[k][l] = pre_pack(p, LAT);
      x = p.z;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  TL(15);                                                  // (timeline: this wave's prologue done)
  __syncthreads();                                         // B
  PH_RESET;
  // B runs two cursors: record r's part that needs no draws (the presampled draws first: the
  // stepping wave waits for them), and record r - kTrioBLag's deck granules once drawn, so that
  // the presampled draws never wait for the drawing wave.  A: record r once drawn.
  constexpr int LAG = PART == 1 ? kTrioBLag : 0;
  auto deck_rec = [&](int q) {                             // B: the deck granules record q changed
    const int sl = q & (kTrioDepth - 1);
    const uint32_t meta = D.ring[sl][1][l].w;
    const int ag = (int)((meta >> 2) & 3u);
    if (live && (meta & kMetaValid)) {                     // (from img)
      const uint32_t dm = D.ring[sl][2][l].w >> 16;
      uint2 pile[5];
#pragma unroll
      for (int k = 0; k < 5; k++) pile[k] = D.img[ag][k][l];
      uint4 dk[7];
      deck_expand(pile, dk);
      uint4 *deck = reinterpret_cast<uint4 *>(deck_ptr(s, i, ag));
#pragma unroll
      for (int k = 0; k < 7; k++)
        if ((dm >> k) & 1u) deck[k] = dk[k];
    }
    cnt_store(D, CNT_STB, (uint32_t)(q + 1));
  };
  TrioCnt6 cc;
  for (int r = 0; r < steps + LAG; r++) {
    if (PART == 1 && r < steps) {                          // record r written
      const int sl = r & (kTrioDepth - 1);
      cnt_wait(D, cc, cc.rec, (uint32_t)(r + 1), s_glob);
      PH(5);
      const uint4 m = D.ring[sl][1][l];
      const uint32_t meta = m.w;
      const bool rec = live && (meta & kMetaValid);
      if (rec && r + kTrioLead < steps)                    // step r + 4's draws: the state after step r,
        D.pre[(r + kTrioLead) & (kTrioLead - 1)][l] = pre_pack(presample(mr_jump(D.srng[sl][l], kPow15)), LAT);
      cnt_store(D, CNT_PRE, (uint32_t)(r + 1));            // + 15 draws (steps r + 1 .. r + 3)
      const uint32_t a_play = D.ring[sl][2][l].w & 0xffu;
      if (rec) {
        const MBits bs{m.x, m.y, m.z};
        store_mask_record(reinterpret_cast<uint4 *>(s.sel + i * COG_MASK_BYTES), bs, mask_diff_granules(bs, selb));
        selb = bs;
        reinterpret_cast<uint2 *>(av + i * COG_ACTION_BYTES)[0] = make_uint2(a_play, 0u);   // (lean: heads 1-4 are 0)
        if (!(meta & kMetaEnded)) {                        // dones[i] = 0, agent_selection[i]
          const uint32_t agent = meta >> 24;               // (an ended episode: k_env_fixup)
          if (out & 0xffu) s.done[i] = 0;
          if (((out >> 8) & 0xffu) != agent) s.agent[i] = (uint8_t)agent;
          out = agent << 8;
        }
      }
    }
    PH(7);
    const int q = r - LAG;                                 // record q drawn
    if (q < 0) continue;                                   // (uniform)
    const int sl = q & (kTrioDepth - 1);
    cnt_wait(D, cc, cc.draw, (uint32_t)(q + 1), s_glob);
    PH(6);
    if (q == steps - 1) TL(11);                            // (timeline: the last record drawn)
    const uint32_t meta = D.ring[sl][1][l].w;
    const bool rec = live && (meta & kMetaValid);
    const int ag = (int)((meta >> 2) & 3u), na = (int)((meta >> 4) & 3u);
    if (rec && PART == 0) {
      const uint4 g0 = D.ring[sl][0][l], xa = D.ring[sl][2][l], oa = D.stbA[ag][l];
      MBits ba{xa.x, xa.y, xa.z};
      if ((int)(meta >> 24) == ag && (meta & kMetaStepped)) {   // the turn goes on: update_observation's
        const uint32_t phase = g0.x & 0xffu;               // heads of ag's stored mask
        const float r0 = __uint_as_float(g0.y), r1 = __uint_as_float(g0.z), r2 = __uint_as_float(g0.w);
        const uint32_t n_active = (xa.w >> 8) & 0xffu;     // (environment.cpp:252-279)
        uint2 ca = cells[3];                               // (selects: no indexed registers)
#pragma unroll
        for (int p = 2; p >= 0; p--) ca = ag == p ? cells[p] : ca;
        const uint32_t mv = phase == COG_PHASE_MOVEMENT ? E.move_bits(ca, r0, r1, r2, n_active) : 1u;
        const uint32_t sp = phase == COG_PHASE_BUYING ? E.shop_bits(r2) : 1u;
        ba.w2 = (ba.w2 & ~kMoveShopBits) | mv << 2 | sp << 9;
      }
      uint8_t *deck = deck_ptr(s, i, ag);
      store_mask_record(reinterpret_cast<uint4 *>(deck + COG_PD_MASK), ba, mask_diff_granules(ba, mbits_of(oa)));
      D.stbA[ag][l] = mbits_u4(ba);
      if ((int)(meta >> 24) != ag && (meta & kMetaStepped)) {   // a turn end: the new agent's stored mask
        const uint4 on = D.stbA[na][l];                    // gets update_observation's INACTIVE-phase
        const MBits bn{on.x, on.y, (on.z & ~kMoveShopBits) | 0x204u};   // heads (the lean step)
        store_mask_record(reinterpret_cast<uint4 *>(deck_ptr(s, i, na) + COG_PD_MASK), bn,
                          mask_diff_granules(bn, mbits_of(on)));
        D.stbA[na][l] = mbits_u4(bn);
      }
    }
    if (PART == 1) {
      deck_rec(q);
    } else {
      cnt_store(D, CNT_STA, (uint32_t)(q + 1));
    }
    PH(13);
  }
  TL(12);
  // A: the stored-mask bit vectors as stored (the epilogue's; the drawing wave's turn ends
  // included), once the stepping wave no longer reads them
  if (PART == 0) {
    cnt_wait(D, cc, cc.rec, (uint32_t)steps + 1u, s_glob);
    if (live) {
#pragma unroll
      for (int p = 0; p < 4; p++) D.heads[p][l] = D.stbA[p][l];
      uint4 *dst = s.cdeck + 10 * i;                       // the drawing wave's final decks (it is past
#pragma unroll                                             // the last record) for the next launch; a
      for (int g = 0; g < 10; g++) {                       // parked env's: k_env_fixup rewrites them
        const uint2 a = D.img[(2 * g) / 5][(2 * g) % 5][l], b = D.img[(2 * g + 1) / 5][(2 * g + 1) % 5][l];
        dst[g] = make_uint4(a.x, a.y, b.x, b.y);
      }
      s.cwide[i] = D.wide[l];
    }
  }
  PH_FLUSH(s_glob);
  return E.flags;                                          // (A: update_observation's lookups)
}

// four waves per workgroup: stepping, drawing and two storing waves, for epw (32 or 64) envs: lanes
// epw.. idle (trio_epw: half-empty waves fill all 256 CUs at 8,192 envs).  The drawing and storing
// waves leave their hazard flags in flg[] and count themselves done in cnt[FIN]; the stepping wave
// waits for all three before its epilogue.
// LAT (a launch of at most one workgroup per CU, DevState::trio_jt): head 0's index table in the
// presampled records and the acting player's counters on the drawing wave -- the stepping wave's
// chain is the launch's time; otherwise (two workgroups share a CU) the total work per CU counts
template <int SRC, bool LAT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_env_rollout_trio(DevState s, int steps, int epw, uint32_t *__restrict__ rngs,
                                                          uint8_t *__restrict__ actions_out) {
  __shared__ TrioLds D;
  // (roles rotated per workgroup, so that a CU's two workgroups could not put both stepping waves
  // on one SIMD, measured the same: profiles/r04y_trio_role_rotation.txt, r05_trio_ab.txt r05s)
  const int role = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));   // wave-uniform
  if (threadIdx.x < 64) D.flg[threadIdx.x] = 0u;
  if (threadIdx.x < kTrioCnts) D.cnt[threadIdx.x] = 0u;
  park_list_clear_other(s);
  uid_tab_fill(D.tab);                                     // (ends on a barrier)
  if (role == 0) {
    __builtin_amdgcn_s_setprio(3);
    trio_stepper<SRC, LAT>(D, s, steps, epw, rngs);
    return;
  }
  uint32_t flags;
  if (role == 1) flags = trio_drawer<LAT>(D, s, steps, epw);
  else if (role == 2) flags = trio_storer<0, LAT>(D, s, steps, epw, rngs, actions_out);
  else flags = trio_storer<1, LAT>(D, s, steps, epw, rngs, actions_out);
  const int l = (int)(threadIdx.x & 63);
  if (flags) __hip_atomic_fetch_or(&D.flg[l], flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  if (l == 0) __hip_atomic_fetch_add(&D.cnt[CNT_FIN], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The envs a duo / trio launch parked (episode ends; the trio's actions outside its lean step):
// for each workgroup on the launch's parked list (park_list_push), one wave runs k_env_rollout's
// fix-up pass for exactly the parked lanes (finish_episode, dones, auto-reset with the wave's map
// generation and encode, then the env's remaining steps with the full step).  A small grid strides
// over the list; with nothing parked every wave returns after one scalar load (round 4 dispatched
// one wave per 64 envs, each reading its envs' park codes: 4.1-4.7 us per launch at 65,536 envs).
// Same stream, right after the rollout launch: nothing reads the envs in between.  epw: envs per
// workgroup of the launch (64, or the trio's 32); lanes epw.. idle.
template <int SRC>
__global__ void __launch_bounds__(64) k_env_fixup(DevState s, int steps, uint32_t *__restrict__ rngs,
                                                  uint8_t *__restrict__ actions_out, int epw) {
  __shared__ LaneLds<64> L;
  const uint32_t cnt = s.parkq[s.park_par];                // (uniform: a scalar load)
  if (blockIdx.x >= cnt) return;
  uid_tab_fill(L.tab);
  for (uint32_t w = blockIdx.x; w < cnt; w += gridDim.x) {
    const size_t base = (size_t)s.parkq[2 + w] * (size_t)epw;
    const size_t i0 = base + threadIdx.x;
    const uint32_t park = (int)threadIdx.x < epw && i0 < s.n ? s.park[i0] : kParkNone;
    rollout_pass<SRC, true, 64>(L, s, steps, rngs, actions_out, park, nullptr, base);
    if (park != kParkNone) {                               // the parked envs' player records
      const int l = (int)threadIdx.x;
      uint4 *pw = reinterpret_cast<uint4 *>(s.priv + i0);
#pragma unroll
      for (int p = 0; p < 4; p++) {
        pw[4 + p] = L.pl[p][l];
        reinterpret_cast<uint2 *>(pw + 8)[p] = L.cells[p][l];
        s.heads[5 * i0 + 1 + p] = L.heads[p][l];
      }
      bool narrow = true;                                  // the trio's compact decks (DevState::cdeck)
#pragma unroll                                             // from the records this lane just stored
      for (int p = 0; p < 4; p++) {
        const uint4 *src = reinterpret_cast<const uint4 *>(deck_ptr(s, i0, p));
        uint4 dk[7];
        uint2 pile[5];
#pragma unroll
        for (int k = 0; k < 7; k++) dk[k] = src[k];
        narrow = compact_of(dk, pile) && narrow;
        uint2 *dst = reinterpret_cast<uint2 *>(s.cdeck + 10 * i0) + 5 * p;
#pragma unroll
        for (int q = 0; q < 5; q++) dst[q] = pile[q];
      }
      s.cwide[i0] = narrow ? 0u : 1u;
      s.park[i0] = kParkNone;
    }
  }
}

// masks may be device memory or pinned host memory (zero-copy); h_actions (may be null) is the
// host view of the actions, written straight over PCIe beside the device copy
__global__ void __launch_bounds__(256) k_sample(size_t n, const uint8_t *__restrict__ masks,
                                                uint32_t *__restrict__ rngs, uint8_t *__restrict__ actions,
                                                uint8_t *__restrict__ h_actions, GridSignal sig) {
  __shared__ UidEntry tab[kUidTab];
  uid_tab_fill(tab);
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    uint32_t rng = rngs[i];
    uint8_t a[5];
    sample_mask(masks + i * COG_MASK_BYTES, rng, a, tab);
    rngs[i] = rng;
    store_action(actions + i * COG_ACTION_BYTES, a);
    if (h_actions) store_action(h_actions + i * COG_ACTION_BYTES, a);
  }
  grid_signal(sig);
}

// Host views without copy commands: the dynamic part of every host-visible record -- the ObsData
// tail (phase, resources, shop, decks, stored masks: granules 1008..1075 of each 1,076-granule
// record) and the shard's outs block (status, selected masks, info, rewards, dones, agents) -- is
// compared granule by granule with `mir`, an HBM copy of what the host views hold, and only the
// granules that differ are stored over PCIe into the pinned host views (and into `mir`).  The
// status granules always go.  A step changes about 200 of the 1,490 bytes per env, so PCIe
// carries the changes instead of a full refresh, and one kernel replaces the D2H copy commands
// (each costs 10-15 us of latency; a 2-D copy of the tails measured 15.7-140 us for 256 envs,
// depending on the box).  force = 1 stores everything (the host views' state is unknown).  The
// sampler's actions (the 8 bytes store_action writes at the head of each 64-B record) ride along
// when act is given.
// Two granules per work-item, both loaded before either is compared (all loads in flight), so
// that a small batch's grid is small enough for the in-kernel completion word (<= 128 workgroups:
// 256 envs take 46); larger grids are signalled by k_signal after the kernel.
constexpr unsigned kPublishPerItem = 2, kPublishSignalBlocks = 128;
__global__ void __launch_bounds__(256) k_publish(const uint4 *__restrict__ obs, const uint4 *__restrict__ outs,
                                                 uint4 *__restrict__ mir, uint4 *__restrict__ h_obs,
                                                 uint4 *__restrict__ h_outs, size_t n, size_t outs_g, int force,
                                                 const uint2 *__restrict__ act, uint2 *__restrict__ h_act,
                                                 GridSignal sig) {
  const size_t tail = n * kTailG, ng = tail + outs_g;
  const size_t t0 = ((size_t)blockIdx.x * blockDim.x) * kPublishPerItem + threadIdx.x;
  const uint4 *src[kPublishPerItem];
  uint4 *dst[kPublishPerItem];
  uint4 c[kPublishPerItem], m[kPublishPerItem];
  bool cmp[kPublishPerItem];
#pragma unroll
  for (unsigned j = 0; j < kPublishPerItem; j++) {         // granule t of the views: a tail or outs granule
    const size_t t = t0 + (size_t)j * blockDim.x;
    src[j] = nullptr;
    if (t < tail) {
      const size_t row = t / kTailG, a = row * kRecG + kTail0 + (t - kTailG * row);
      src[j] = obs + a;
      dst[j] = h_obs + a;
      cmp[j] = !force;
    } else if (t < ng) {
      const size_t u = t - tail;
      src[j] = outs + u;
      dst[j] = h_outs + u;
      cmp[j] = !force && u >= 4;                           // (the status granules always go)
    }
    if (src[j]) {
      c[j] = *src[j];
      if (cmp[j]) m[j] = mir[t];
    }
  }
#pragma unroll
  for (unsigned j = 0; j < kPublishPerItem; j++) {
    const size_t t = t0 + (size_t)j * blockDim.x;
    if (src[j] && (!cmp[j] || ne4(c[j], m[j]))) {
      *dst[j] = c[j];
      mir[t] = c[j];
    }
  }
  // the sampler's actions: one work-item per env after the granules
  const size_t ia = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t g_items = (ng + kPublishPerItem - 1) / kPublishPerItem;
  if (act && ia >= g_items && ia - g_items < n) {
    const size_t i = ia - g_items;
    h_act[(COG_ACTION_BYTES / 8) * i] = act[(COG_ACTION_BYTES / 8) * i];
  }
  grid_signal(sig);
}

__global__ void k_sync_heads(DevState s) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < s.n) sync_heads(s, i);
}
// cog_env_invalidate_device: after a caller wrote device records, the engine's private mirrors of
// records the reference reads back are rebuilt from them -- the mask bit vectors from the selected
// and stored ActionMask records (player.cpp:16-27 reads the mask bools), and the Info steps_taken
// mirror from the Info records (environment.cpp:97: steps_taken += 1 reads the record)
__global__ void k_resync(DevState s) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= s.n) return;
  sync_heads(s, i);
  const uint8_t *inf = s.info + i * COG_INFO_BYTES + COG_AGENT_INFO0;
  uint32_t v = 0u;
#pragma unroll
  for (int p = 0; p < 4; p++) v |= (uint32_t)inf[COG_AGENT_INFO_STRIDE * p] << (8 * p);
  reinterpret_cast<uint32_t *>(s.priv + i)[12] = v;        // EnvPriv::info_steps (granule 3, dword 0)
}

// Completion word of a host call: queued behind the call's work on its stream, it stores `seq`
// into a pinned, device-mapped word that the host spins on (a system-scope release store, after
// every earlier packet of the stream has completed).  The host learns completion about 2.5 us
// sooner than through hipStreamSynchronize (tools/latprobe.hip, profiles/r03_latprobe.txt).
__global__ void __launch_bounds__(64) k_signal(uint32_t *word, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void k_seed_sampler(size_t n, uint64_t seed, size_t first, uint32_t *rngs) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) rngs[i] = mr_seed(seed + (uint64_t)(first + i));   // vec_sampler.h:9-13 (no u32 wrap)
}

// The measured device copy peak beside which the encode's HBM fraction is reported (BASELINE.md
// "plus a measured copy-kernel peak"): 16-B loads and stores (plain or non-temporal), 4 granules
// in flight per work-item, a grid striding over the buffer; cog_time_copy reports the faster.
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
template <bool NT>
DEV u32x4_t cp_ld(const u32x4_t *p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
DEV void cp_st(u32x4_t v, u32x4_t *p) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT>
__global__ void __launch_bounds__(256) k_copy_peak(const u32x4_t *__restrict__ src, u32x4_t *__restrict__ dst, size_t n16) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const u32x4_t a = cp_ld<NT>(src + i), b = cp_ld<NT>(src + i + stride);
    const u32x4_t c = cp_ld<NT>(src + i + 2 * stride), d = cp_ld<NT>(src + i + 3 * stride);
    cp_st<NT>(a, dst + i);
    cp_st<NT>(b, dst + i + stride);
    cp_st<NT>(c, dst + i + 2 * stride);
    cp_st<NT>(d, dst + i + 3 * stride);
  }
  for (; i < n16; i += stride) cp_st<NT>(cp_ld<NT>(src + i), dst + i);
}
// one pass, no grid stride: a workgroup copies one contiguous 32 KiB block (8 granules in flight
// per work-item, all loads issued before the first store); a grid of n16 / 2048 workgroups
template <bool NT>
__global__ void __launch_bounds__(256) k_copy_block(const u32x4_t *__restrict__ src, u32x4_t *__restrict__ dst, size_t n16) {
  const size_t base = (size_t)blockIdx.x * 2048 + threadIdx.x;
  if (base + 7 * 256 < n16) {
    u32x4_t v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = cp_ld<NT>(src + base + k * 256);
#pragma unroll
    for (int k = 0; k < 8; k++) cp_st<NT>(v[k], dst + base + k * 256);
  } else {
    for (size_t i = base; i < n16; i += 256) cp_st<NT>(cp_ld<NT>(src + i), dst + i);
  }
}
// one granule per work-item, a grid covering the buffer (the plain float4 copy of
// MI355X_MICROARCH.md's measured 6.29 TB/s)
template <bool NT>
__global__ void __launch_bounds__(256) k_copy_one(const u32x4_t *__restrict__ src, u32x4_t *__restrict__ dst, size_t n16) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n16) cp_st<NT>(cp_ld<NT>(src + i), dst + i);
}

// The encode's own read:write mix as a stream (1 granule read, 7 written, all coalesced): the
// bandwidth an HBM-bound kernel of that mix can reach on this chip, the peak k_encode (16 B of
// cells read, 112 B of observation written per work-item) is compared with.
template <bool NT>
__global__ void __launch_bounds__(256) k_stream_mix(const u32x4_t *__restrict__ src, u32x4_t *__restrict__ dst, size_t n_rd) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_rd) return;
  const u32x4_t v = cp_ld<false>(src + i);
#pragma unroll
  for (int k = 0; k < 7; k++) cp_st<NT>(v + (unsigned)k, dst + i + (size_t)k * n_rd);
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
static inline unsigned blocks_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

int launch_init(const DevState &s, const uint32_t *, uint32_t default_seed, void *stream) {
  if (!s.n) return 0;
  hipLaunchKernelGGL(k_init, dim3(blocks_for(s.n, 256)), dim3(256), 0, (hipStream_t)stream, s, default_seed);
  hipLaunchKernelGGL(k_sync_heads, dim3(blocks_for(s.n, 256)), dim3(256), 0, (hipStream_t)stream, s);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_reset(const DevState &s, const ResetParams &p, void *stream) {
  if (!s.n) return 0;
  // envs per wave: enough waves to keep every SIMD generating (about 4,096 waves), at most 64
  static const int epw_env = [] {
    const char *e = getenv("COG_RESET_EPW");
    return e ? atoi(e) : 0;
  }();
  const size_t auto_epw = (s.n + 4095) / 4096;
  const int epw = epw_env > 0 ? (epw_env < 64 ? epw_env : 64) : (int)(auto_epw < 1 ? 1 : auto_epw > 64 ? 64 : auto_epw);
  hipLaunchKernelGGL(k_reset, dim3(blocks_for(s.n, (unsigned)epw)), dim3(64), 0, (hipStream_t)stream, s, p, epw);
  hipLaunchKernelGGL(k_sync_heads, dim3(blocks_for(s.n, 256)), dim3(256), 0, (hipStream_t)stream, s);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_resync(const DevState &s, void *stream) {
  if (!s.n) return 0;
  hipLaunchKernelGGL(k_resync, dim3(blocks_for(s.n, 256)), dim3(256), 0, (hipStream_t)stream, s);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_encode_all(const DevState &s, void *stream, int variant) {
  if (!s.n) return 0;
  const size_t nb = s.n * kEncBlocks;
  const dim3 g(blocks_for(nb, 256)), b(256);
  // production (0): LDS-transposed + non-temporal stores (88 % of HBM peak measured);
  // 1: LDS-transposed, plain stores; 2: direct per-item 112-B stores (A/B references)
  if (variant == 1) hipLaunchKernelGGL(k_encode_lds<false>, g, b, 0, (hipStream_t)stream, s.cgrid, s.obs, nb);
  else if (variant == 2) hipLaunchKernelGGL(k_encode_direct, g, b, 0, (hipStream_t)stream, s.cgrid, s.obs, nb);
  else hipLaunchKernelGGL(k_encode_lds<true>, g, b, 0, (hipStream_t)stream, s.cgrid, s.obs, nb);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_step(const DevState &s, const uint8_t *d_actions, void *stream) {
  if (!s.n) return 0;
  hipLaunchKernelGGL(k_env_step<MASK_EXTERNAL>, dim3(blocks_for(s.n, 64)), dim3(64), 0, (hipStream_t)stream, s,
                     d_actions, nullptr, nullptr);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
constexpr unsigned kStepPubMaxBlocks = 128;              // (completion counter arrivals)
bool step_pub_ok(size_t n) { return n && blocks_for(n, 64) <= kStepPubMaxBlocks; }
int launch_step_pub(const DevState &s, const uint8_t *d_actions, void *stream, uint32_t *sig_ctr, uint32_t *sig_word,
                    uint32_t seq, const SampleSpec *spec) {
  if (!step_pub_ok(s.n) || !sig_ctr || !s.pub_obs || !s.pub_outs || !s.pub_mir) return -1;
  const SampleSpec none{nullptr, nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(k_env_step_pub<MASK_EXTERNAL>, dim3(blocks_for(s.n, 64)), dim3(64), 0, (hipStream_t)stream, s,
                     d_actions, nullptr, nullptr, nullptr, GridSignal{sig_ctr, sig_word, seq}, spec ? *spec : none);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_sample_step_pub(const DevState &s, int mask_source, uint32_t *d_rng, uint8_t *d_actions, uint8_t *h_actions,
                           void *stream, uint32_t *sig_ctr, uint32_t *sig_word, uint32_t seq) {
  if (!step_pub_ok(s.n) || !sig_ctr || !s.pub_obs || !s.pub_outs || !s.pub_mir || !h_actions) return -1;
  const dim3 g(blocks_for(s.n, 64)), b(64);
  const SampleSpec none{nullptr, nullptr, nullptr, nullptr, nullptr};
  if (mask_source == MASK_STORED)
    hipLaunchKernelGGL(k_env_step_pub<MASK_STORED>, g, b, 0, (hipStream_t)stream, s, nullptr, d_rng, d_actions, h_actions,
                       GridSignal{sig_ctr, sig_word, seq}, none);
  else
    hipLaunchKernelGGL(k_env_step_pub<MASK_SELECTED>, g, b, 0, (hipStream_t)stream, s, nullptr, d_rng, d_actions,
                       h_actions, GridSignal{sig_ctr, sig_word, seq}, none);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_sample(size_t n, const uint8_t *d_masks, uint32_t *d_rng, uint8_t *d_actions, void *stream,
                  uint8_t *h_actions, uint32_t *sig_ctr, uint32_t *sig_word, uint32_t seq) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_sample, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, d_masks, d_rng, d_actions,
                     h_actions, GridSignal{sig_ctr, sig_word, seq});
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_sample_step(const DevState &s, int mask_source, uint32_t *d_rng, uint8_t *d_actions, void *stream) {
  if (!s.n) return 0;
  if (mask_source == MASK_STORED)
    hipLaunchKernelGGL(k_env_step<MASK_STORED>, dim3(blocks_for(s.n, 64)), dim3(64), 0, (hipStream_t)stream, s,
                       nullptr, d_rng, d_actions);
  else
    hipLaunchKernelGGL(k_env_step<MASK_SELECTED>, dim3(blocks_for(s.n, 64)), dim3(64), 0, (hipStream_t)stream, s,
                       nullptr, d_rng, d_actions);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
template <int NL>
static void rollout_launch(const DevState &s, int mask_source, int steps, uint32_t *d_rng, uint8_t *d_actions,
                           hipStream_t st) {
  const dim3 g(blocks_for(s.n, NL)), b(NL);
  if (mask_source == MASK_STORED)
    hipLaunchKernelGGL((k_env_rollout<MASK_STORED, NL>), g, b, 0, st, s, steps, d_rng, d_actions);
  else
    hipLaunchKernelGGL((k_env_rollout<MASK_SELECTED, NL>), g, b, 0, st, s, steps, d_rng, d_actions);
}
// Which rollout kernels run a shard of n envs (measured on MI355X, device us/step in 1,000-step
// launches, profiles/r03_rollout_kinds.txt, profiles/r04e_trio_ab.txt):
//   selected masks, >= 3 players: trio at every size (k_env_rollout_trio + k_env_fixup,
//                profiles/r04p_trio_sweep.txt: 1.48 at 8,192-24,576, 1.93 at 32,768, 2.97 at 65,536
//                against duo 2.46 at 8,192, pipe 2.75 at 32,768 and wave 3.52 / 4.12 at 32,768 /
//                65,536; 20-step launches at 65,536: 84.7 against 104.0 us)
//   otherwise    n <= 16,384 duo (k_env_rollout_duo + k_env_fixup: 2.47-2.49 against pipe 2.65-2.68),
//                n <= 32,768 pipe (k_env_rollout_pipe: 2.75-2.76 against duo 2.96), larger wave
//                (k_env_rollout: 3.91-3.96 against duo 4.0-4.7)
// Above 16,384 envs the chip's shader clock drops (2.34 -> 2.08 GHz measured by s_memtime at the
// same cycles per step), and the duo's storing wave costs more work per env-step than its
// hand-off saves, so the leaner kernels win there.  $COG_ROLLOUT = duo | pipe | wave forces one
// (duo: the trio where it applies; $COG_TRIO=0 keeps the duo).
enum RolloutKind : int { RK_AUTO = -1, RK_DUO = 0, RK_WAVE = 1, RK_PIPE = 2, RK_TRIO = 3 };
static bool trio_on() {                                    // $COG_TRIO=0: no trio (A/B)
  static const bool on = [] {
    const char *e = getenv("COG_TRIO");
    return !(e && *e == '0');
  }();
  return on;
}
static int rollout_kind(size_t n, int mask_source, bool defer_ok) {
  static const int forced = [] {
    const char *e = getenv("COG_ROLLOUT");
    if (!e || !*e || !strcmp(e, "auto")) return (int)RK_AUTO;
    return !strcmp(e, "duo") ? (int)RK_DUO : !strcmp(e, "wave") ? (int)RK_WAVE : (int)RK_PIPE;
  }();
  const bool trio = defer_ok && mask_source == MASK_SELECTED && trio_on();
  if (forced != RK_AUTO) return forced == RK_DUO && trio ? (int)RK_TRIO : forced;
  if (trio) return RK_TRIO;
  return n <= 16384 ? RK_DUO : n <= 32768 ? RK_PIPE : RK_WAVE;
}
int rollout_kind_of(size_t n, int mask_source, bool defer_ok) { return rollout_kind(n, mask_source, defer_ok); }
// envs per trio workgroup ($COG_TRIO_EPW = 32 | 64 forces it)
int trio_epw(size_t n) {
  static const int forced = [] {
    const char *e = getenv("COG_TRIO_EPW");
    return e && *e ? atoi(e) : 0;
  }();
  if (forced == 32 || forced == 64) return forced;
  (void)n;
  return 64;
}
// Trio workgroups per CU.  The compact decks (TrioLds, 53 KB) admit three per CU, but the output
// stores are bound by each XCD's L2: at 65,536 envs, 32,768 stepping at once keep an XCD's written
// lines (~4.7 per env-step) within its 4 MiB L2, 49,152 or all 65,536 do not (measured: four per
// CU, all 65,536 at once, 3.94 us per step; three per CU 4.01; two per CU, in two rounds, 2.75;
// one per CU 5.43: profiles/r05f_trio_wpc.txt).  So a launch of more than one workgroup per CU
// pads each workgroup's LDS to half a CU's (the dispatcher would otherwise pack three on some CUs);
// $COG_TRIO_WPC = 1..4 overrides (A/B).
// The current device's CU count and LDS bytes per CU (hipGetDeviceProperties once per device: a
// partitioned MI355X exposes fewer CUs than the whole chip's 256; 160 KiB of LDS per CU on gfx950)
struct CuShape {
  unsigned cus;
  size_t lds;
};
static CuShape cu_shape() {
  static CuShape cache[64] = {};
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return {256u, 163840};
  if (!cache[d].cus) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess && p.multiProcessorCount > 0)
      cache[d] = {(unsigned)p.multiProcessorCount,
                  p.maxSharedMemoryPerMultiProcessor ? (size_t)p.maxSharedMemoryPerMultiProcessor : (size_t)163840};
    else
      cache[d] = {256u, 163840};
  }
  return cache[d];
}
static size_t trio_pad_lds(unsigned nblocks) {
  static const int forced = [] {
    const char *e = getenv("COG_TRIO_WPC");
    return e && *e ? atoi(e) : 0;
  }();
  const CuShape c = cu_shape();
  const int wpc = forced >= 1 && forced <= 4 ? forced : (nblocks > c.cus ? 2 : 0);
  if (!wpc) return 0;
  const size_t per = c.lds / (size_t)wpc - 2048;           // (a margin for the allocation granule)
  return per > sizeof(TrioLds) ? per - sizeof(TrioLds) : 0;
}
// k_env_fixup's grid: at most this many one-wave workgroups stride over the parked list
// ($COG_FIXUP_GRID overrides; A/B only).  A wave per CU keeps a launch with every workgroup parked
// (short episodes) running in parallel, and a launch with none parked cheap.
static unsigned fixup_grid(unsigned nblocks) {
  static const unsigned forced = [] {
    const char *e = getenv("COG_FIXUP_GRID");
    const int v = e && *e ? atoi(e) : 0;
    return v > 0 ? (unsigned)v : 0u;
  }();
  return std::max(1u, std::min(nblocks, forced ? forced : cu_shape().cus));
}
int launch_rollout(const DevState &s, int mask_source, int steps, uint32_t *d_rng, uint8_t *d_actions, void *stream,
                   bool defer_ok, uint32_t *park_seq, bool no_fixup) {
  if (!s.n || steps <= 0) return 0;
  const int kind = rollout_kind(s.n, mask_source, defer_ok);
  if (kind == RK_DUO || kind == RK_TRIO) {
    if (!park_seq || !s.parkq) return -1;
    const hipStream_t st = (hipStream_t)stream;
    static const int redo_at = [] {                        // test hook (DevState::redo_at)
      const char *e = getenv("COG_DEBUG_REDO_STEP");
      return e && *e ? atoi(e) : -1;
    }();
    // test hook: "t:i" parks env i (local index) at step t of each launch and keeps a no-fix-up
    // launch so (the guard's test: the park must surface as F_PARK_NOFIX)
    static const std::pair<int, long long> park_nofix = [] {
      const char *e = getenv("COG_DEBUG_PARK_NOFIX");
      if (!e || !*e) return std::make_pair(-1, -1LL);
      const char *c = strchr(e, ':');
      return std::make_pair(atoi(e), c ? atoll(c + 1) : 0LL);
    }();
    DevState sd = s;
    sd.redo_at = park_nofix.first >= 0 ? park_nofix.first : redo_at;
    sd.redo_env = park_nofix.first >= 0 ? (int32_t)park_nofix.second : -1;
    sd.park_par = (*park_seq)++ & 1u;
    // (the redo hook parks every env: never without the fix-up; $COG_ALWAYS_FIXUP for A/B)
    static const bool always_fixup = getenv("COG_ALWAYS_FIXUP") != nullptr;
    sd.no_fixup = no_fixup && kind == RK_TRIO && (redo_at < 0 || park_nofix.first >= 0) && !always_fixup ? 1u : 0u;
    const int epw = kind == RK_TRIO ? trio_epw(s.n) : 64;
    const unsigned nb = blocks_for(s.n, epw);
    const dim3 g(nb), gf(fixup_grid(nb));
    static const int jt_env = [] {                         // $COG_TRIO_JT = 0 / 1 overrides (A/B)
      const char *e = getenv("COG_TRIO_JT");
      return e && *e ? atoi(e) : -1;
    }();
    sd.trio_jt = jt_env >= 0 ? (uint32_t)(jt_env != 0) : (nb <= cu_shape().cus ? 1u : 0u);
    if (mask_source == MASK_STORED) {
      hipLaunchKernelGGL((k_env_rollout_duo<MASK_STORED>), g, dim3(128), 0, st, sd, steps, d_rng, d_actions);
      hipLaunchKernelGGL((k_env_fixup<MASK_STORED>), gf, dim3(64), 0, st, sd, steps, d_rng, d_actions, epw);
    } else if (kind == RK_TRIO) {                          // selected masks, >= 3 players
      // (k_env_fixup inside the trio launch, for shards of one workgroup per CU -- inlined, or as a
      // never-inlined call -- was slower: 20-step launch at 8,192 44.2 / 42.0 against 41.3 us,
      // profiles/r04t_trio_fused.txt)
      if (sd.trio_jt)
        hipLaunchKernelGGL((k_env_rollout_trio<MASK_SELECTED, true>), g, dim3(256), trio_pad_lds(nb), st, sd, steps, epw,
                           d_rng, d_actions);
      else
        hipLaunchKernelGGL((k_env_rollout_trio<MASK_SELECTED, false>), g, dim3(256), trio_pad_lds(nb), st, sd, steps, epw,
                           d_rng, d_actions);
      if (!sd.no_fixup)
        hipLaunchKernelGGL((k_env_fixup<MASK_SELECTED>), gf, dim3(64), 0, st, sd, steps, d_rng, d_actions, epw);
    } else {
      hipLaunchKernelGGL((k_env_rollout_duo<MASK_SELECTED>), g, dim3(128), 0, st, sd, steps, d_rng, d_actions);
      hipLaunchKernelGGL((k_env_fixup<MASK_SELECTED>), gf, dim3(64), 0, st, sd, steps, d_rng, d_actions, epw);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  // one 64-env wave per workgroup: 32-env workgroups measured 7.3 us/step against 3.8 at 65,536
  // envs (round 2).  The kernel's register allocation (about 490 VGPRs + AGPRs per work-item)
  // admits one wave per SIMD, so 2,048 half-empty waves ran in two rounds on 1,024 SIMDs
  const hipStream_t st = (hipStream_t)stream;
  if (kind == RK_PIPE) {                                   // SIMDs to spare: the two-wave form
    const dim3 g(blocks_for(s.n, 64)), b(128);
    if (mask_source == MASK_STORED)
      hipLaunchKernelGGL((k_env_rollout_pipe<MASK_STORED>), g, b, 0, st, s, steps, d_rng, d_actions);
    else
      hipLaunchKernelGGL((k_env_rollout_pipe<MASK_SELECTED>), g, b, 0, st, s, steps, d_rng, d_actions);
  } else {
    rollout_launch<64>(s, mask_source, steps, d_rng, d_actions, st);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
// work-items: granule pairs (a workgroup covers 512 consecutive granules), then one per action
static unsigned publish_blocks(size_t n, size_t outs_bytes, bool actions) {
  const size_t ng = n * kTailG + outs_bytes / 16;
  return blocks_for((ng + kPublishPerItem - 1) / kPublishPerItem + (actions ? n : 0), 256);
}
int launch_publish(const DevState &s, const uint8_t *outs, uint8_t *mir, uint8_t *h_obs, uint8_t *h_outs, size_t outs_bytes,
                   int force, const uint8_t *d_actions, uint8_t *h_actions, void *stream, uint32_t *sig_ctr,
                   uint32_t *sig_word, uint32_t seq) {
  if (!s.n) return 0;
  const unsigned blocks = publish_blocks(s.n, outs_bytes, d_actions != nullptr);
  if (sig_ctr && blocks > kPublishSignalBlocks) return -1; // (publish_can_signal says no)
  const size_t outs_g = outs_bytes / 16;
  hipLaunchKernelGGL(k_publish, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const uint4 *>(s.obs), reinterpret_cast<const uint4 *>(outs),
                     reinterpret_cast<uint4 *>(mir), reinterpret_cast<uint4 *>(h_obs), reinterpret_cast<uint4 *>(h_outs),
                     s.n, outs_g, force, reinterpret_cast<const uint2 *>(d_actions), reinterpret_cast<uint2 *>(h_actions),
                     GridSignal{sig_ctr, sig_word, seq});
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
bool publish_can_signal(size_t n, size_t outs_bytes, bool actions) {
  return publish_blocks(n, outs_bytes, actions) <= kPublishSignalBlocks;
}
size_t publish_mirror_bytes(size_t n, size_t outs_bytes) { return n * kTailG * 16 + outs_bytes; }
int launch_copy_peak(const void *src, void *dst, size_t bytes, void *stream, int variant) {
  const u32x4_t *a = static_cast<const u32x4_t *>(src);
  u32x4_t *b = static_cast<u32x4_t *>(dst);
  const size_t n16 = bytes / 16;
  if (variant & 8) {                                  // the encode's mix: bytes / 16 granules read, 7x written
    const dim3 g(blocks_for(n16, 256)), t(256);
    if (variant & 1) hipLaunchKernelGGL(k_stream_mix<true>, g, t, 0, (hipStream_t)stream, a, b, n16);
    else hipLaunchKernelGGL(k_stream_mix<false>, g, t, 0, (hipStream_t)stream, a, b, n16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (variant & 16) {                                 // one granule per work-item
    const dim3 g(blocks_for(n16, 256)), t(256);
    if (variant & 1) hipLaunchKernelGGL(k_copy_one<true>, g, t, 0, (hipStream_t)stream, a, b, n16);
    else hipLaunchKernelGGL(k_copy_one<false>, g, t, 0, (hipStream_t)stream, a, b, n16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (variant & 4) {                                  // one pass, 32 KiB per workgroup
    const dim3 g(blocks_for(n16, 2048)), t(256);
    if (variant & 1) hipLaunchKernelGGL(k_copy_block<true>, g, t, 0, (hipStream_t)stream, a, b, n16);
    else hipLaunchKernelGGL(k_copy_block<false>, g, t, 0, (hipStream_t)stream, a, b, n16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  const dim3 g(variant & 2 ? 8192 : 2048), t(256);   // grid stride: 8 or 32 waves per CU
  if (variant & 1) hipLaunchKernelGGL(k_copy_peak<true>, g, t, 0, (hipStream_t)stream, a, b, n16);
  else hipLaunchKernelGGL(k_copy_peak<false>, g, t, 0, (hipStream_t)stream, a, b, n16);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_signal(uint32_t *d_word, uint32_t seq, void *stream) {
  hipLaunchKernelGGL(k_signal, dim3(1), dim3(64), 0, (hipStream_t)stream, d_word, seq);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_seed_sampler(size_t n, uint64_t seed, size_t first, uint32_t *d_rng, void *stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_seed_sampler, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, seed, first,
                     d_rng);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cog
