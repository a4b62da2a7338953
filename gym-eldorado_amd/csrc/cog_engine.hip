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
//   k_step           vec_cog_env::step with auto-reset (vec_environment.h:46-61)
//   k_sample_step    runner-fused sample(selected|stored masks) + step (runner.h:46-55)
#include <hip/hip_runtime.h>

#include "cog_engine.h"
#include "cog_tables.h"

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

// shop slots that start in the market (cards.cpp:85-92 / 94-100): slots 0,1,5,7,9,12
constexpr uint32_t kInMarket0 = (1u << 0) | (1u << 1) | (1u << 5) | (1u << 7) | (1u << 9) | (1u << 12);

// ------------------------------------------------------------------------------------------
// RNG: minstd_rand0 and libstdc++ uniform_int_distribution<size_t> downscaling
// ------------------------------------------------------------------------------------------
DEV uint32_t mr_seed(uint64_t s) {
  uint32_t x = (uint32_t)(s % 2147483647ull);
  return x == 0 ? 1u : x;
}
DEV uint32_t mr_next(uint32_t &x) {
  const uint64_t p = (uint64_t)x * 16807u;                 // < 2^46
  uint32_t r = (uint32_t)(p & 0x7fffffffu) + (uint32_t)(p >> 31);
  r = r >= 0x7fffffffu ? r - 0x7fffffffu : r;
  x = r;
  return r;
}
// uniform integer in [0, k-1], k >= 1 (uniform_int_distribution<size_t>(0, k-1))
DEV uint32_t uid(uint32_t &x, uint32_t k) {
  const uint32_t scaling = 2147483645u / k;
  const uint32_t past = k * scaling;
  uint32_t r;
  do {
    r = mr_next(x) - 1u;
  } while (r >= past);
  return r / scaling;
}

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

// cog_env::reset() (environment.cpp:42-64)
DEV bool env_reset(const Ctx &e) {
  EnvPriv *pv = e.pv;
  pv->agent = 0;
  e.sh[0] = COG_PHASE_INACTIVE;
  map_reset(e);
  GenScratch *gs = e.gs;
  for (int p = 0; p < COG_N_PIECES; p++) { gs->pcx[p] = 0; gs->pcy[p] = 0; gs->prot[p] = 0; }
  if (!generate(e)) {
    pv->flags |= F_MAPGEN_FAIL;
    return false;
  }
  build_cgrid(e);
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
  while (m) {
    const int l = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const size_t env = (size_t)__shfl((int)i, l);
    const uint8_t *cg = s.cgrid + env * COG_CELLS;
    uint8_t *map = s.obs + env * COG_OBS_BYTES;
    for (int k = lane; k < kEncBlocks; k += 64) encode_block(cg, map, k);
  }
}

// ------------------------------------------------------------------------------------------
// sampler (sampler.h:14-79): 5 independent uniform picks over the set bits of each head
// ------------------------------------------------------------------------------------------
DEV uint32_t bools4(uint32_t w) {                          // 4 bool bytes -> 4 bits (nonzero = set)
  const uint32_t nz = (((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u;
  return ((nz >> 7) * 0x01020408u) >> 24 & 0xfu;
}
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
  return (uint8_t)nth_set_bit(m, uid(rng, k));
}
DEV void sample_mask(const uint8_t *mask, uint32_t &rng, uint8_t out[5]) {
  const uint32_t *m32 = reinterpret_cast<const uint32_t *>(mask);   // 4-byte aligned (LDS slot or record)
  uint64_t lo = 0, hi = 0;
#pragma unroll
  for (int word = 0; word < 23; word++) {                  // bytes 4*word .. 4*word+3
    const uint64_t b = bools4(m32[word]);
    const int bit = 4 * word;
    if (bit < 64) lo |= b << bit;
    else hi |= b << (bit - 64);
  }
  const uint32_t play = (uint32_t)(lo & 0x3fffffu);
  const uint32_t spec = (uint32_t)((lo >> 22) & 0x3fffffu);
  const uint32_t rem = (uint32_t)(((lo >> 44) | (hi << 20)) & 0x3fffffu);
  const uint32_t mov = (uint32_t)((hi >> 2) & 0x7fu);
  const uint32_t shop = (uint32_t)((hi >> 9) & 0x7ffffu);
  out[0] = pick(rng, play);
  out[1] = pick(rng, spec);
  out[2] = pick(rng, rem);
  out[3] = pick(rng, mov);
  out[4] = pick(rng, shop);
}
DEV void store_action(uint8_t *dst, const uint8_t a[5]) {
  const uint32_t lo = (uint32_t)a[0] | (uint32_t)a[1] << 8 | (uint32_t)a[2] << 16 | (uint32_t)a[3] << 24;
  reinterpret_cast<uint2 *>(dst)[0] = make_uint2(lo, (uint32_t)a[4]);
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
  z.seed = default_seed + (uint32_t)i;
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

__global__ void k_reset(DevState s, ResetParams p) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= s.n) return;
  Ctx e = make_ctx(s, i);
  EnvPriv *pv = e.pv;
  if (p.use_params) {                                      // cog_env::reset(params) :66-77
    pv->n_players = p.n_players;
    pv->n_pieces = p.n_pieces;
    pv->difficulty = p.difficulty;
    pv->max_steps = p.max_steps;
    pv->seed = p.seed + (uint32_t)i;                       // vec_environment.h:41, u32 wrap (Q33)
    pv->rng = mr_seed(pv->seed);
  }
  if (!env_reset(e)) {
    atomicOr(&s.status[0], pv->flags);
    atomicAdd(&s.status[1], 1u);
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

// ---- per-env LDS slots of a step's working set, staged by the whole wave ------------------
// slot = 155 dwords (odd stride: same-offset dword accesses of a wave are bank-conflict free)
//   [  0,160) EnvPriv                 [160,256) selected ActionMask (96 B)
//   [256,304) ObsData 16128..16175 (phase, resources, shop)
//   [304,416) DeckObs of the acting player a0 (112 B)   [416,512) stored ActionMask of a0
//   [512,608) stored ActionMask of the next player na (the turn change reads it)
//   [608,616) store plan: dirty 16-B granules of each staged record
// Loads and stores are cooperative: item (env e, granule g) of a record goes to lane
// (e * G + g) mod 64, so one instruction covers 64 / G whole records instead of 64 scattered
// 16-B pieces; the game logic then runs one env per lane on its slot.
constexpr int kSlotWords = 155;
constexpr int SLOT_PV = 0, SLOT_SEL = 160, SLOT_SH = 256, SLOT_DK = 304, SLOT_ST = 416, SLOT_STN = 512,
              SLOT_PLAN = 608;
constexpr int kPvG = (int)sizeof(EnvPriv) / 16;          // 10 granules
constexpr int kWaveEnvs = 64;

DEV void lds_put4(uint32_t *d, const uint4 &v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w; }
DEV uint4 lds_get4(const uint32_t *d) { return make_uint4(d[0], d[1], d[2], d[3]); }

// ---- fast path: play / pass / turn change on registers (environment.cpp:91-250) -------------
// Selected and stored masks are held as five head bitsets (bit k == index k of the head); the
// deck's bulk operations run on dwords with compile-time byte positions.  Move / shop / remove /
// special actions and resets take the byte-level path above (env_step / env_reset).
struct Heads {
  uint32_t play, spec, rem, move, shop;
};

DEV Heads heads_from(const uint8_t *mask) {               // ActionMask bytes -> bitsets
  const uint32_t *m32 = reinterpret_cast<const uint32_t *>(mask);
  uint64_t lo = 0, hi = 0;
#pragma unroll
  for (int w = 0; w < 23; w++) {
    const uint64_t b = bools4(m32[w]);
    if (4 * w < 64) lo |= b << (4 * w);
    else hi |= b << (4 * w - 64);
  }
  Heads h;
  h.play = (uint32_t)(lo & 0x3fffffu);
  h.spec = (uint32_t)((lo >> 22) & 0x3fffffu);
  h.rem = (uint32_t)(((lo >> 44) | (hi << 20)) & 0x3fffffu);
  h.move = (uint32_t)((hi >> 2) & 0x7fu);
  h.shop = (uint32_t)((hi >> 9) & 0x7ffffu);
  return h;
}
DEV uint32_t expand4(uint32_t x) { return (x * 0x00204081u) & 0x01010101u; }   // 4 bits -> 4 bool bytes
DEV void heads_to(const Heads &h, uint32_t *m32) {        // bitsets -> the 23 named dwords
  const uint64_t lo = (uint64_t)h.play | ((uint64_t)h.spec << 22) | ((uint64_t)h.rem << 44);
  const uint64_t hi = ((uint64_t)h.rem >> 20) | ((uint64_t)h.move << 2) | ((uint64_t)h.shop << 9);
#pragma unroll
  for (int w = 0; w < 23; w++)
    m32[w] = expand4((uint32_t)((4 * w < 64 ? lo >> (4 * w) : hi >> (4 * w - 64)) & 0xfu));
}
DEV void sample_heads(const Heads &h, uint32_t &rng, uint8_t out[5]) {      // sampler.h:14-79
  out[0] = pick(rng, h.play);
  out[1] = pick(rng, h.spec);
  out[2] = pick(rng, h.rem);
  out[3] = pick(rng, h.move);
  out[4] = pick(rng, h.shop);
}
DEV uint32_t set_bit(uint32_t m, int k, bool v) { return v ? (m | (1u << k)) : (m & ~(1u << k)); }

constexpr cog_card_t kCards[COG_N_CARDTYPES] = COG_CARD_TABLE;
constexpr uint8_t kShopTypes[COG_N_SHOP] = COG_SHOP_TYPES;
constexpr uint32_t kSpecialBits = 0x1f8000u;              // card types 15..20

DEV uint32_t byte_of(const uint32_t *w, int idx) { return (w[idx >> 2] >> (8 * (idx & 3))) & 0xffu; }
DEV void put_byte(uint32_t *w, int idx, uint32_t v) {
  const int sh = 8 * (idx & 3);
  w[idx >> 2] = (w[idx >> 2] & ~(0xffu << sh)) | ((v & 0xffu) << sh);
}

// Deck::discard_all_active + discard_all_played (cards.cpp:219-232) on dwords 10..26
DEV void fast_discard_all(uint32_t *dk32) {
  uint32_t w[17];
#pragma unroll
  for (int q = 0; q < 17; q++) w[q] = dk32[10 + q];
#pragma unroll
  for (int k = 0; k < COG_N_CARDTYPES; k++) {
    const uint32_t a = byte_of(w, COG_DECK_ACTIVE + k - 40), p = byte_of(w, COG_DECK_PLAYED + k - 40);
    put_byte(w, COG_DECK_DISCARD + k - 40, byte_of(w, COG_DECK_DISCARD + k - 40) + a + p);
    put_byte(w, COG_DECK_ACTIVE + k - 40, 0u);
    put_byte(w, COG_DECK_PLAYED + k - 40, 0u);
  }
#pragma unroll
  for (int q = 0; q < 17; q++) dk32[10 + q] = w[q];
}

// Deck::move_discard_to_draw (cards.cpp:234-240): draw dwords 0..5, discard dwords 21..26
DEV void fast_move_discard_to_draw(uint32_t *dk32, PlayerPriv &P) {
  uint32_t d[6], x[6];
#pragma unroll
  for (int q = 0; q < 6; q++) { d[q] = dk32[q]; x[q] = dk32[21 + q]; }
  uint32_t nd = P.n_in_draw;
#pragma unroll
  for (int k = 0; k < COG_N_CARDTYPES; k++) {
    const uint32_t v = byte_of(x, k);                      // discard byte 84+k == x byte k
    put_byte(d, k, byte_of(d, k) + v);
    nd += v;
    put_byte(x, k, 0u);
  }
  P.n_in_draw = (uint8_t)nd;
#pragma unroll
  for (int q = 0; q < 6; q++) { dk32[q] = d[q]; dk32[21 + q] = x[q]; }
}

// hand[k] > 0 for k < 21 as a bitset (hand = bytes 21..41 = dwords 5..10)
DEV uint32_t hand_bits(const uint32_t *dk32) {
  uint32_t w[6];
#pragma unroll
  for (int q = 0; q < 6; q++) w[q] = dk32[5 + q];
  uint32_t h = 0;
#pragma unroll
  for (int k = 0; k < COG_N_CARDTYPES; k++) h |= (byte_of(w, COG_DECK_HAND + k - 20) != 0u ? 1u : 0u) << k;
  return h;
}
DEV void fast_enable_playing(const uint32_t *dk32, Heads &sel) {   // player.cpp:198-206
  const uint32_t h = hand_bits(dk32);
  sel.rem = 1u;
  sel.play = 1u | (h << 1);
  sel.spec = 1u | ((h & kSpecialBits) << 1);
}

// Deck::draw (cards.cpp:183-211); the draw-pile scan runs on registers.  n_in_draw equals the
// sum of draw[] mod 256 (every Deck operation keeps it), so t < n_in_draw always ends inside
// draw[0..20]; the guard only raises the hazard flag.
DEV void fast_draw(const Ctx &e, PlayerPriv &P, uint32_t *dk32, Heads &sel, uint32_t &rng, uint8_t n) {
  if (P.n_in_draw < n) fast_move_discard_to_draw(dk32, P);
  if (n > P.n_in_draw) n = P.n_in_draw;
  if (!n) return;
  uint32_t d[6];
#pragma unroll
  for (int q = 0; q < 6; q++) d[q] = dk32[q];
  for (int i = 0; i < n; i++) {
    uint32_t t = uid(rng, P.n_in_draw);
    int c = COG_N_CARDTYPES;
#pragma unroll
    for (int k = 0; k < COG_N_CARDTYPES; k++) {
      const uint32_t v = byte_of(d, k);
      if (c == COG_N_CARDTYPES) {
        if (t >= v) t -= v;
        else c = k;
      }
    }
    if (c == COG_N_CARDTYPES) {                            // unreachable (see above)
      e.pv->flags |= F_SCAN_OVER;
      c = COG_N_CARDTYPES - 1;
    }
#pragma unroll
    for (int q = 0; q < 6; q++)
      if (q == (c >> 2)) d[q] -= 1u << (8 * (c & 3));      // draw[c] >= 1: no borrow
    P.n_in_draw--;
    e.dka[COG_DECK_HAND + c]++;
    sel.play |= 1u << (c + 1);
    sel.spec = set_bit(sel.spec, c + 1, is_special(c));
  }
#pragma unroll
  for (int q = 0; q < 5; q++) dk32[q] = d[q];
  e.dka[20] = (uint8_t)byte_of(d, 20);                     // bytes 21..23 are hand[0..2]
  P.n_in_hand = (uint8_t)(P.n_in_hand + n);
}

// bytes 66..91 (move[0..6], get_from_shop[0..18]) of a stored mask from two bitsets
DEV void put_move_shop(uint32_t *st32, uint32_t move, uint32_t shop) {
  const uint32_t v = move | (shop << 7);
  st32[16] = (st32[16] & 0xffffu) | ((v & 1u) << 16) | (((v >> 1) & 1u) << 24);
#pragma unroll
  for (int q = 0; q < 6; q++) st32[17 + q] = expand4((v >> (2 + 4 * q)) & 0xfu);
}

DEV uint8_t use_cell(const Ctx &e, const uint8_t *cc, int d) {   // a lookup of the cached cell d
  if ((cc[7] >> d) & 1u) e.pv->flags |= F_OOB_LOOKUP;
  return cc[d];
}
// movement mask bits 1..6 (map.cpp:369-387) + bit 0, from a player's cached neighbourhood
DEV uint32_t move_bits(const Ctx &e, const uint8_t *cc, float r0, float r1, float r2, uint8_t n_active) {
  uint32_t m = 1u;
#pragma unroll
  for (int d = 1; d < 7; d++) {
    const uint8_t c = use_cell(e, cc, d);
    const int req = COG_HEX_REQ(c);
    const uint32_t n = COG_HEX_N(c);
    const float r = req == 0 ? r0 : (req == 1 ? r1 : r2);
    const bool filled = req >= COG_REQ_DISCARD ? n_active > n : r >= (float)n;
    if (req != COG_REQ_NULL && filled) m |= 1u << d;
  }
  return m;
}
// shop mask bits 1..18 (cards.cpp:109-121) + bit 0
DEV uint32_t shop_bits(const Ctx &e, float coins) {
  const bool few = e.pv->n_in_market < COG_MKT_SLOTS;
  const uint32_t im = e.pv->in_market;
  uint32_t m = 1u;
#pragma unroll
  for (int i = 0; i < COG_N_SHOP; i++) {
    const bool ok = few ? e.sh[SH_SHOP + i] > 0 : ((im >> i) & 1u);
    if (ok && coins > (float)kCards[kShopTypes[i]].cost) m |= 1u << (i + 1);
  }
  return m;
}
DEV uint32_t gran(int byte) { return 1u << (byte >> 4); }   // 16-B granule bit of a record byte

// Player::cards_from_active (player.cpp:85-131): n random cards leave the active pile
DEV void take_from_active(const Ctx &e, PlayerPriv &P, uint8_t n, bool discard) {
  uint8_t *d = e.dka;
  const uint8_t avail = P.n_active;
  if (n > avail) {
    if (discard) e.pv->flags |= F_Q24_CLAMP;
    n = avail;
  }
  uint32_t rng = e.pv->rng;
  for (uint8_t i = 0; i < n; i++) {
    const uint32_t t = uid(rng, (uint32_t)(avail - i));
    const int c = scan(e, d, COG_DECK_ACTIVE, t);
    P.n_active--;
    d[COG_DECK_ACTIVE + c]--;
    if (discard) d[COG_DECK_DISCARD + c]++;
  }
  e.pv->rng = rng;
}

// card c leaves the hand (Deck::activate / play_immediate / remove_immediate, cards.cpp:242-290)
// and the selected mask's play / special / remove bits of c follow (rem_rule: remove_immediate)
DEV void leave_hand(const Ctx &e, PlayerPriv &P, Heads &sel, int c, bool rem_rule) {
  const uint8_t prev = e.dka[COG_DECK_HAND + c];
  e.dka[COG_DECK_HAND + c] = (uint8_t)(prev - 1);
  P.n_in_hand--;
  const uint32_t b = 1u << (c + 1);
  bool pl = prev > 1;
  if (rem_rule) {
    if (!pl) sel.rem &= ~b;
    pl = pl && (sel.play & b);
  }
  sel.play = pl ? (sel.play | b) : (sel.play & ~b);
  sel.spec = (pl && is_special(c)) ? (sel.spec | b) : (sel.spec & ~b);
}

struct Plan {                         // 16-B granules to store back, per staged record
  uint32_t pv, sh, dk, st, stn;
};

// special actions (cards.cpp:8-36, the remove lambda environment.cpp:156-158) on the stored mask
// `stc` of the CURRENT agent and the selected mask, for the ACTING player P (:183-186)
DEV void apply_special(const Ctx &e, int special, int ag, PlayerPriv &P, Heads &sel, uint8_t *stc) {
  Heads m = heads_from(stc);
  switch (special) {
    case COG_SPECIAL_DRAW2:
    case COG_SPECIAL_DRAW3: {
      uint32_t rng = e.pv->rng;
      fast_draw(e, P, reinterpret_cast<uint32_t *>(e.dka), sel, rng, special == COG_SPECIAL_DRAW2 ? 2 : 3);
      e.pv->rng = rng;
    } break;
    case COG_SPECIAL_DRAW1_REMOVE1:
    case COG_SPECIAL_DRAW2_REMOVE2: {
      const uint8_t k = special == COG_SPECIAL_DRAW1_REMOVE1 ? 1 : 2;
      uint32_t rng = e.pv->rng;
      fast_draw(e, P, reinterpret_cast<uint32_t *>(e.dka), sel, rng, k);
      e.pv->rng = rng;
      P.n_removes = k;
      m.rem = m.play;                                      // mask.remove = mask.play
      sel.play = 1u;                                       // disable_playing
      sel.spec = 1u;
      m.shop &= 1u;                                        // shop_mask(0): nothing affordable
    } break;
    case COG_SPECIAL_TRANSMIT: {
      m.move = 1u;
      sel.play = 1u;
      sel.spec = 1u;
      uint32_t sb = m.shop & 1u;
#pragma unroll
      for (int i = 0; i < COG_N_SHOP; i++)
        if (e.sh[SH_SHOP + i] > 0) sb |= 1u << (i + 1);
      m.shop = sb;
      P.next_card_free = 1;
    } break;
    case COG_SPECIAL_NATIVE: {
      const uint8_t *cc = e.pv->cells[ag];
      uint32_t mb = m.move & 1u;
#pragma unroll
      for (int d = 1; d < 7; d++)                          // movement_mask with 100 of everything
        if (COG_HEX_REQ(use_cell(e, cc, d)) != COG_REQ_NULL) mb |= 1u << d;
      m.move = mb;
      P.next_move_free = 1;
      sel.play = 1u;
      sel.spec = 1u;
      m.shop &= 1u;
    } break;
    case COG_SPECIAL_SHOP_OFF: m.shop &= 1u; break;
    default: break;
  }
  heads_to(m, reinterpret_cast<uint32_t *>(stc));
}

// cog_env::step (environment.cpp:91-224) for the acting player a0 == agent, every action kind.
// State: deck / stored mask of a0, stored mask of na, phase / resources / shop and EnvPriv in
// the LDS slot; selected mask in `sel` (bitsets).  Returns the granules it modified.
DEV Plan step_env(const Ctx &e, const uint8_t act[5], Heads &sel, uint8_t *stn, int na) {
  EnvPriv *pv = e.pv;
  const int ag = pv->agent;
  Plan o{0xbu | (1u << (4 + ag)), 0x1u, 0u, 0u, 0u};       // rng/counters, agent/flags, info mirror
  e.info[COG_AGENT_INFO0 + COG_AGENT_INFO_STRIDE * ag] = ++pv->info_steps[ag];   // steps_taken (u8)
  uint8_t phase = e.sh[0];
  if (phase == COG_PHASE_INACTIVE) phase = COG_PHASE_MOVEMENT;
  PlayerPriv &P = pv->pl[ag];
  P.steps_taken++;
  float *res3 = res(e);
  float r0 = res3[0], r1 = res3[1], r2 = res3[2];
  uint8_t *d = e.dka;
  uint32_t *dk32 = reinterpret_cast<uint32_t *>(d);
  const uint8_t a_play = act[0], a_special = act[1], a_remove = act[2], a_move = act[3], a_shop = act[4];
  int special = COG_SPECIAL_NONE;
  bool moved = false;
  if (a_play) {                                            // Player::play_card (player.cpp:45-60)
    const int c = a_play - 1;
    if (phase == COG_PHASE_MOVEMENT) {
      r0 = (float)c_cards[c].res[0]; r1 = (float)c_cards[c].res[1]; r2 = (float)c_cards[c].res[2];
    } else if (phase == COG_PHASE_BUYING) {
      const uint8_t coin = c_cards[c].res[2];
      r2 = r2 + (coin > 0 ? (float)coin : 0.5f);
    }
    leave_hand(e, P, sel, c, false);                       // Deck::activate
    d[COG_DECK_ACTIVE + c]++;
    P.n_active++;
    P.idx_last = (uint8_t)c;
    o.dk |= gran(COG_DECK_HAND + c) | gran(COG_DECK_ACTIVE + c);
  } else if (a_special) {                                  // play_special (environment.cpp:108-114)
    const int c = a_special - 1;
    const bool single = c_cards[c].single_use;
    leave_hand(e, P, sel, c, single);                      // remove_immediate / play_immediate
    if (!single) {
      d[COG_DECK_PLAYED + c]++;
      o.dk |= gran(COG_DECK_PLAYED + c);
    }
    o.dk |= gran(COG_DECK_HAND + c);
    special = c_cards[c].special;
  } else if (a_move) {                                     // move (environment.cpp:115-127)
    const uint8_t c = use_cell(e, pv->cells[ag], a_move);
    pv->locx[ag] = (int8_t)(pv->locx[ag] + c_dirs[a_move][0] / 2);
    pv->locy[ag] = (int8_t)(pv->locy[ag] + c_dirs[a_move][1] / 2);
    if (!P.next_move_free) {                               // Player::handle_requirement (:141-162)
      const int req = COG_HEX_REQ(c);
      const uint8_t n = COG_HEX_N(c);
      if (req < 3) {
        const float left = (req == 0 ? r0 : req == 1 ? r1 : r2) - (float)n;
        r0 = req == 0 ? left : 0.f;
        r1 = req == 1 ? left : 0.f;
        r2 = req == 2 ? left : 0.f;
        if (!P.mip) {                                      // Deck::play_last_activated
          const int l = P.idx_last;
          P.n_active--;
          d[COG_DECK_ACTIVE + l]--;
          o.dk |= gran(COG_DECK_ACTIVE + l);
          if (!c_cards[l].single_use) {
            d[COG_DECK_PLAYED + l]++;
            o.dk |= gran(COG_DECK_PLAYED + l);
          }
          P.mip = 1;
        }
      } else if (req == COG_REQ_REMOVE || req == COG_REQ_DISCARD) {
        take_from_active(e, P, n, req == COG_REQ_DISCARD);
        r0 = r1 = r2 = 0.f;
        P.mip = 0;
        o.dk = 0x7fu;
      }
    } else {
      P.next_move_free = 0;
      fast_enable_playing(dk32, sel);
    }
    P.n_movements++;
    P.has_won = COG_HEX_END(c);
    moved = true;
    o.pv |= 0x4u;                                          // player locations
  } else {
    P.next_move_free = 0;
    if (a_shop) {                                          // Shop::get_card (cards.cpp:123-142)
      const int k = a_shop - 1;
      const int type = kShopTypes[k];
      const uint32_t bit = 1u << k;
      if (!P.next_card_free) {
        pv->n_in_market = (uint8_t)(pv->n_in_market + ((pv->in_market & bit) ? 0 : 1));
        pv->in_market |= bit;
      }
      const uint8_t left = (uint8_t)(e.sh[SH_SHOP + k] - 1);
      e.sh[SH_SHOP + k] = left;
      if (!left && (pv->in_market & bit)) {
        pv->in_market &= ~bit;
        pv->n_in_market--;
      }
      if (!P.next_card_free) {
        r2 = r2 - (float)c_cards[type].cost;
        phase = (uint8_t)((phase + 1) % 3);
      }
      d[COG_DECK_DISCARD + type]++;
      P.n_added_cards++;
      o.dk |= gran(COG_DECK_DISCARD + type);
      o.sh |= gran(SH_SHOP + k);
    } else if (a_remove) {
      const int c = a_remove - 1;
      leave_hand(e, P, sel, c, true);                      // Deck::remove_immediate
      o.dk |= gran(COG_DECK_HAND + c);
      P.n_removes--;
      if (!P.n_removes) fast_enable_playing(dk32, sel);
      else special = COG_SPECIAL_SHOP_OFF;
    } else {                                               // pass: next phase
      phase = (uint8_t)((phase + 1) % 3);
      if (P.n_removes > 0) {
        P.n_removes = 0;
        fast_enable_playing(dk32, sel);
      }
    }
    if (P.next_card_free) {
      P.next_card_free = 0;
      fast_enable_playing(dk32, sel);
    }
  }
  STAMP_AT(3);
  if (P.mip && !a_move) {                                  // the move HEAD, whatever was taken
    P.mip = 0;
    r0 = r1 = r2 = 0.f;
  }
  int cur = ag;
  if (P.has_won || phase == COG_PHASE_INACTIVE) {          // maybe_end_turn -> next_agent
    P.n_active = 0;                                        // Player::end_turn (player.cpp:170-180)
    fast_discard_all(dk32);
    const int n_draw = COG_HAND_SIZE - (int)P.n_in_hand;
    if (n_draw > 0) {
      uint32_t rng = pv->rng;
      fast_draw(e, P, dk32, sel, rng, (uint8_t)n_draw);
      pv->rng = rng;
    }
    heads_to(sel, reinterpret_cast<uint32_t *>(e.sta));  // save_actionmask
    o.dk = 0x7fu;
    o.st = 0x3fu;
    pv->agent = (uint8_t)na;
    sel = heads_from(na == ag ? e.sta : stn);             // load_actionmask
    r0 = r1 = r2 = 0.f;
    pv->turn_counter++;
    cur = na;
  }
  STAMP_AT(4);
  e.sh[0] = phase;
  res3[0] = r0; res3[1] = r1; res3[2] = r2;
  if (moved) {                                             // the mover's new neighbourhood
    load_cells(e, ag);
    o.pv |= 1u << (8 + ag / 2);
  }
  STAMP_AT(5);
  const uint8_t *cc = pv->cells[cur];
  uint8_t *stc = cur == ag ? e.sta : stn;
  uint32_t mv = 1u, sp = 1u;                               // update_observation (:252-279)
  if (phase == COG_PHASE_MOVEMENT) mv = move_bits(e, cc, r0, r1, r2, pv->pl[cur].n_active);
  else if (phase == COG_PHASE_BUYING) sp = shop_bits(e, r2);
  put_move_shop(reinterpret_cast<uint32_t *>(stc), mv, sp);
  STAMP_AT(6);
  uint32_t st_dirty = 0x30u;
  if (special != COG_SPECIAL_NONE) {
    apply_special(e, special, ag, P, sel, stc);
    st_dirty = 0x3fu;
    o.dk = 0x7fu;
  } else {
    const uint8_t c = use_cell(e, cc, 0);                  // done check (:187)
    if (COG_HEX_END(c) || pv->turn_counter >= pv->max_steps) finish_episode(e);
  }
  STAMP_AT(7);
  if (cur == ag) o.st |= st_dirty;
  else o.stn |= st_dirty;
  return o;
}

// Cooperative staging helpers.  Item it = k * 64 + lane of a record of G granules belongs to env
// it / G, granule it % G.  Loads clamp the env to the block's last valid one (duplicate reads,
// no branches); stores are predicated on the store plan.
template <int G>
DEV int item_env(int k, int lane) { return (k * 64 + lane) / G; }
template <int G>
DEV int item_gran(int k, int lane) { return (k * 64 + lane) % G; }
template <int G>
constexpr int n_items() { return (G * kWaveEnvs + 63) / 64; }

// One step of the wave's 64 envs (each optionally preceded by sampling its action).
// act_in: actions of the host API path (nullptr in the fused runner path).
// Latency plan (one wave per SIMD at the benchmark's size, so nothing hides a stall):
//   round 1 loads (state at fixed addresses) -> LDS -> round 2 loads (agent-dependent records)
//   issued -> sampling on the round-1 state while they fly -> LDS -> game logic -> all LDS
//   reads of the store phase batched -> predicated 16-B stores.
DEV void wave_step(const DevState &s, uint32_t *slots, const uint8_t *act_in, int mask_source,
                   uint32_t *rngs, uint8_t *actions_out) {
  const int lane = threadIdx.x;
  const size_t base = (size_t)blockIdx.x * kWaveEnvs;
  const int nv = s.n - base < (size_t)kWaveEnvs ? (int)(s.n - base) : kWaveEnvs;
  auto slot_of = [&](int e) { return slots + e * kSlotWords; };
  auto cl = [&](int e) { return e < nv ? e : nv - 1; };
  auto obs_of = [&](int e) { return s.obs + (base + e) * COG_OBS_BYTES; };
  auto player_of = [&](int e, int p) { return obs_of(e) + COG_OBS_PLAYER0 + COG_OBS_PLAYER_STRIDE * p; };
  STAMP(s, 0);
  const size_t i = base + (size_t)cl(lane);
  const bool live = lane < nv;

  // round 1: EnvPriv (10 granules), selected mask (6), phase/resources/shop (3), sampler rng
  {
    constexpr int KA = n_items<kPvG>(), KB = n_items<6>(), KC = n_items<3>();
    uint4 a[KA], b[KB], c[KC];
#pragma unroll
    for (int k = 0; k < KA; k++)
      a[k] = reinterpret_cast<const uint4 *>(s.priv + base + cl(item_env<kPvG>(k, lane)))[item_gran<kPvG>(k, lane)];
#pragma unroll
    for (int k = 0; k < KB; k++)
      b[k] = reinterpret_cast<const uint4 *>(s.sel + (base + cl(item_env<6>(k, lane))) * COG_MASK_BYTES)[item_gran<6>(k, lane)];
#pragma unroll
    for (int k = 0; k < KC; k++)
      c[k] = reinterpret_cast<const uint4 *>(obs_of(cl(item_env<3>(k, lane))) + COG_OBS_PHASE)[item_gran<3>(k, lane)];
#pragma unroll
    for (int k = 0; k < KA; k++) lds_put4(slot_of(item_env<kPvG>(k, lane)) + SLOT_PV / 4 + 4 * item_gran<kPvG>(k, lane), a[k]);
#pragma unroll
    for (int k = 0; k < KB; k++) lds_put4(slot_of(item_env<6>(k, lane)) + SLOT_SEL / 4 + 4 * item_gran<6>(k, lane), b[k]);
#pragma unroll
    for (int k = 0; k < KC; k++) lds_put4(slot_of(item_env<3>(k, lane)) + SLOT_SH / 4 + 4 * item_gran<3>(k, lane), c[k]);
  }
  uint32_t rng = act_in ? 0u : rngs[i];
  __syncthreads();

  // round 2 (addresses depend on the agent): deck + stored mask of a0 (13 granules, skipping the
  // DeckObs padding granule), stored mask of na (6).  Issued, then the sampler runs on the
  // round-1 state while they are in flight.
  uint32_t *slot = slot_of(lane);
  uint8_t *lds = reinterpret_cast<uint8_t *>(slot);
  EnvPriv *pv = reinterpret_cast<EnvPriv *>(lds + SLOT_PV);
  const int a0 = pv->agent;
  const int na = a0 + 1 >= pv->n_players ? 0 : a0 + 1;
  const int players = a0 | na << 2;                        // this lane's env: a0, na
  constexpr int KD = n_items<13>(), KE = n_items<6>();
  uint4 dk[KD], sn[KE];
#pragma unroll
  for (int k = 0; k < KD; k++) {
    const int e = item_env<13>(k, lane), g = item_gran<13>(k, lane);
    const int pa = __shfl(players, cl(e)) & 3;
    dk[k] = reinterpret_cast<const uint4 *>(player_of(cl(e), pa))[g < 7 ? g : g + 1];
  }
#pragma unroll
  for (int k = 0; k < KE; k++) {
    const int e = item_env<6>(k, lane), g = item_gran<6>(k, lane);
    const int pn = __shfl(players, cl(e)) >> 2;
    sn[k] = reinterpret_cast<const uint4 *>(player_of(cl(e), pn) + COG_PD_MASK)[g];
  }
  Heads sel = heads_from(lds + SLOT_SEL);
  uint8_t act[5] = {0, 0, 0, 0, 0};
  if (act_in) {                                            // host actions: indices past a head
    const uint8_t *ai = act_in + i * COG_ACTION_BYTES;     // are the reference's OOB accesses
    const uint8_t top[5] = {COG_N_CARDTYPES, COG_N_CARDTYPES, COG_N_CARDTYPES, 6, COG_N_SHOP};
#pragma unroll
    for (int k = 0; k < 5; k++) {
      act[k] = ai[k];
      if (act[k] > top[k]) {
        act[k] = top[k];
        if (live) pv->flags |= F_BAD_ACTION;
      }
    }
  } else if (mask_source != MASK_STORED) {                 // runner: sample(selected masks)
    sample_heads(sel, rng, act);
  }
#pragma unroll
  for (int k = 0; k < KD; k++) lds_put4(slot_of(item_env<13>(k, lane)) + SLOT_DK / 4 + 4 * item_gran<13>(k, lane), dk[k]);
#pragma unroll
  for (int k = 0; k < KE; k++) lds_put4(slot_of(item_env<6>(k, lane)) + SLOT_STN / 4 + 4 * item_gran<6>(k, lane), sn[k]);
  __syncthreads();
  STAMP(s, 1);

  // per-lane game logic on the slot of env `lane`
  bool enc = false;
  if (live) {
    Ctx e;
    e.ob = s.obs + i * COG_OBS_BYTES;
    e.sh = lds + SLOT_SH;
    e.dka = lds + SLOT_DK;
    e.sta = lds + SLOT_ST;
    e.a0 = a0;
    e.sel = lds + SLOT_SEL;
    e.info = s.info + i * COG_INFO_BYTES;
    e.rew = s.rew + i * 4;
    e.pv = pv;
    e.grid = s.grid + i * (size_t)kGridBytes;
    e.cgrid = s.cgrid + i * COG_CELLS;
    e.gs = s.gen + i;
    e.stamps = s.stamps;

    if (!act_in) {
      if (mask_source == MASK_STORED) sample_heads(heads_from(e.sta), rng, act);   // runner, stored masks
      rngs[i] = rng;
      store_action(actions_out + i * COG_ACTION_BYTES, act);
    }
    STAMP(s, 2);
    Plan o{0x3u, 0u, 0u, 0u, 0u};                          // flags may change (bad action)
    if (!pv->done) o = step_env(e, act, sel, lds + SLOT_STN, na);
    STAMP(s, 10);
    const uint8_t done = pv->done;
    s.done[i] = done;                                      // dones[i] before the auto-reset
    if (done) {                                            // vec_environment.h:56-59
      heads_to(sel, reinterpret_cast<uint32_t *>(e.sel));
      o = Plan{(1u << kPvG) - 1u, 0x7u, 0x7fu, 0x3fu, 0u}; // na's staged mask is stale now
      if (!env_reset(e)) {
        atomicOr(&s.status[0], pv->flags);
        atomicAdd(&s.status[1], 1u);
      } else {
        enc = true;
        const uint32_t k = atomicAdd(&s.status[2], 1u);
        if (k < s.n) s.dirty[k] = (uint32_t)i;
      }
      sel = heads_from(e.sel);
    }
    s.agent[i] = pv->agent;
    heads_to(sel, slot + SLOT_SEL / 4);
    slot[SLOT_PLAN / 4] = o.pv | o.sh << 10 | o.dk << 13 | o.st << 20 | o.stn << 26;
    slot[SLOT_PLAN / 4 + 1] = (uint32_t)a0 | (uint32_t)na << 2;   // records of the ORIGINAL agent
    STAMP(s, 11);
  } else {
    slot[SLOT_PLAN / 4] = 0u;                              // lanes past the batch store nothing
  }
  __syncthreads();

  // cooperative stores of the dirty granules: every LDS read first (one wait), then the stores
  {
    constexpr int KA = n_items<kPvG>(), KB = n_items<6>(), KC = n_items<3>();
    uint4 va[KA], vb[KB], vc[KC], vd[KD], ve[KE];
    uint32_t pa[KA], pc[KC], pd[KD], pe[KE], wd[KD], we[KE];
#pragma unroll
    for (int k = 0; k < KA; k++) {
      const int e = item_env<kPvG>(k, lane), g = item_gran<kPvG>(k, lane);
      pa[k] = (slot_of(e)[SLOT_PLAN / 4] >> g) & 1u;
      va[k] = lds_get4(slot_of(e) + SLOT_PV / 4 + 4 * g);
    }
#pragma unroll
    for (int k = 0; k < KB; k++) {
      const int e = item_env<6>(k, lane), g = item_gran<6>(k, lane);
      vb[k] = lds_get4(slot_of(e) + SLOT_SEL / 4 + 4 * g);
    }
#pragma unroll
    for (int k = 0; k < KC; k++) {
      const int e = item_env<3>(k, lane), g = item_gran<3>(k, lane);
      pc[k] = (slot_of(e)[SLOT_PLAN / 4] >> (10 + g)) & 1u;
      vc[k] = lds_get4(slot_of(e) + SLOT_SH / 4 + 4 * g);
    }
#pragma unroll
    for (int k = 0; k < KD; k++) {                         // deck granules = plan bits 13..19,
      const int e = item_env<13>(k, lane), g = item_gran<13>(k, lane);   // stored mask = bits 20..25
      pd[k] = (slot_of(e)[SLOT_PLAN / 4] >> (13 + g)) & 1u;
      wd[k] = slot_of(e)[SLOT_PLAN / 4 + 1] & 3u;
      vd[k] = lds_get4(slot_of(e) + SLOT_DK / 4 + 4 * g);
    }
#pragma unroll
    for (int k = 0; k < KE; k++) {                         // na's stored mask = bits 26..31
      const int e = item_env<6>(k, lane), g = item_gran<6>(k, lane);
      pe[k] = (slot_of(e)[SLOT_PLAN / 4] >> (26 + g)) & 1u;
      we[k] = (slot_of(e)[SLOT_PLAN / 4 + 1] >> 2) & 3u;
      ve[k] = lds_get4(slot_of(e) + SLOT_STN / 4 + 4 * g);
    }
#pragma unroll
    for (int k = 0; k < KA; k++) {
      const int e = item_env<kPvG>(k, lane), g = item_gran<kPvG>(k, lane);
      if (pa[k]) reinterpret_cast<uint4 *>(s.priv + base + e)[g] = va[k];
    }
#pragma unroll
    for (int k = 0; k < KB; k++) {
      const int e = item_env<6>(k, lane), g = item_gran<6>(k, lane);
      if (e < nv) reinterpret_cast<uint4 *>(s.sel + (base + e) * COG_MASK_BYTES)[g] = vb[k];
    }
#pragma unroll
    for (int k = 0; k < KC; k++) {
      const int e = item_env<3>(k, lane), g = item_gran<3>(k, lane);
      if (pc[k]) reinterpret_cast<uint4 *>(obs_of(e) + COG_OBS_PHASE)[g] = vc[k];
    }
#pragma unroll
    for (int k = 0; k < KD; k++) {
      const int e = item_env<13>(k, lane), g = item_gran<13>(k, lane);
      if (pd[k]) reinterpret_cast<uint4 *>(player_of(e, wd[k]))[g < 7 ? g : g + 1] = vd[k];
    }
#pragma unroll
    for (int k = 0; k < KE; k++) {
      const int e = item_env<6>(k, lane), g = item_gran<6>(k, lane);
      if (pe[k]) reinterpret_cast<uint4 *>(player_of(e, we[k]) + COG_PD_MASK)[g] = ve[k];
    }
  }
  STAMP(s, 12);
  wave_encode(s, base + lane, enc);
}

__global__ void __launch_bounds__(64) k_step(DevState s, const uint8_t *__restrict__ actions) {
  __shared__ uint32_t slots[kWaveEnvs * kSlotWords];
  wave_step(s, slots, actions, 0, nullptr, nullptr);
}

__global__ void __launch_bounds__(256) k_sample(size_t n, const uint8_t *__restrict__ masks,
                                                uint32_t *__restrict__ rngs, uint8_t *__restrict__ actions) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t rng = rngs[i];
  uint8_t a[5];
  sample_mask(masks + i * COG_MASK_BYTES, rng, a);
  rngs[i] = rng;
  store_action(actions + i * COG_ACTION_BYTES, a);
}

__global__ void __launch_bounds__(64) k_sample_step(DevState s, int mask_source, uint32_t *__restrict__ rngs,
                                                    uint8_t *__restrict__ actions) {
  __shared__ uint32_t slots[kWaveEnvs * kSlotWords];
  wave_step(s, slots, nullptr, mask_source, rngs, actions);
}

__global__ void k_seed_sampler(size_t n, uint32_t seed, uint32_t *rngs) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) rngs[i] = mr_seed((uint64_t)seed + (uint64_t)i);   // vec_sampler.h:9-13 (no u32 wrap)
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
static inline unsigned blocks_for(size_t n, unsigned t) { return (unsigned)((n + t - 1) / t); }

int launch_init(const DevState &s, const uint32_t *, uint32_t default_seed, void *stream) {
  if (!s.n) return 0;
  hipLaunchKernelGGL(k_init, dim3(blocks_for(s.n, 256)), dim3(256), 0, (hipStream_t)stream, s, default_seed);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_reset(const DevState &s, const ResetParams &p, void *stream) {
  if (!s.n) return 0;
  hipLaunchKernelGGL(k_reset, dim3(blocks_for(s.n, 64)), dim3(64), 0, (hipStream_t)stream, s, p);
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
  hipLaunchKernelGGL(k_step, dim3(blocks_for(s.n, kWaveEnvs)), dim3(kWaveEnvs), 0, (hipStream_t)stream, s, d_actions);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_sample(size_t n, const uint8_t *d_masks, uint32_t *d_rng, uint8_t *d_actions, void *stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_sample, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, d_masks, d_rng, d_actions);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_sample_step(const DevState &s, int mask_source, uint32_t *d_rng, uint8_t *d_actions, void *stream) {
  if (!s.n) return 0;
  hipLaunchKernelGGL(k_sample_step, dim3(blocks_for(s.n, kWaveEnvs)), dim3(kWaveEnvs), 0, (hipStream_t)stream, s,
                     mask_source, d_rng, d_actions);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
int launch_seed_sampler(size_t n, uint32_t seed, uint32_t *d_rng, void *stream) {
  if (!n) return 0;
  hipLaunchKernelGGL(k_seed_sampler, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, n, seed, d_rng);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace cog
