/* cog_oracle.c -- TEST INFRASTRUCTURE ONLY (see cog_oracle.h).
 *
 * Plain-C restatement of the reference City-of-Gold engine.  It deliberately follows the
 * reference's data representation where that representation decides results:
 *   - float32 hex geometry exactly as geometry.cpp:3-17 / map.cpp:17-51 (not integer maths),
 *   - sort + merge overlap test (map.cpp:53-74),
 *   - hex_array rebuilt after every piece (map.cpp:309-341),
 *   - libstdc++ minstd_rand0 + uniform_int_distribution<size_t>,
 *   - u8 wrap-around everywhere the reference uses u_char.
 * The HIP engine uses a different representation (doubled-integer lattice + occupancy
 * bitmap), so agreement between the two is evidence, not tautology.
 *
 * Compile: gcc -std=c11 -O2 -ffp-contract=off -fPIC -shared -pthread
 */
#define _GNU_SOURCE
#include "cog_oracle.h"

#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/cog_types.h"
#include "../gym-eldorado_amd/csrc/cog_tables.h"

static const cog_card_t CARDS[COG_N_CARDTYPES] = COG_CARD_TABLE;
static const uint8_t SHOP_TYPES[COG_N_SHOP] = COG_SHOP_TYPES;
static const cog_piece_meta_t PMETA[COG_N_PIECES] = COG_PIECE_META;
static const uint8_t PHEX[COG_N_PIECES][37] = COG_PIECE_HEX;
static const int8_t LARGE_XY2[37][2] = COG_LARGE_XY2;
static const int8_t SMALL_XY2[16][2] = COG_SMALL_XY2;
static const int8_t END_XY2[3][2] = COG_END_XY2;
static const int8_t DIR_XY2[7][2] = COG_DIRS_XY2;

/* ------------------------------------------------------------------------------------ */
/* RNG: libstdc++ std::default_random_engine == minstd_rand0 (a=16807, m=2^31-1)          */
/* ------------------------------------------------------------------------------------ */
static inline uint32_t mr_seed(uint64_t s) {          /* linear_congruential_engine::seed */
  uint64_t x = s % 2147483647ull;
  return x == 0 ? 1u : (uint32_t)x;
}
static inline uint32_t mr_next(uint32_t *x) {
  *x = (uint32_t)(((uint64_t)*x * 16807ull) % 2147483647ull);
  return *x;
}
/* uniform_int_distribution<size_t>(a, b) with the "downscaling" branch
 * (urng range 2147483645 > b - a).  Every call consumes >= 1 draw. */
static uint64_t uid(uint32_t *x, uint64_t a, uint64_t b) {
  const uint64_t urngrange = 2147483645ull;
  const uint64_t urange = b - a;
  uint64_t ret;
  if (urngrange > urange) {
    const uint64_t uerange = urange + 1;
    const uint64_t scaling = urngrange / uerange;
    const uint64_t past = uerange * scaling;
    do {
      ret = (uint64_t)mr_next(x) - 1u;
    } while (ret >= past);
    ret /= scaling;
  } else {
    /* never reached by valid play (Q24 is clamped before calling) */
    ret = (uint64_t)mr_next(x) - 1u;
  }
  return ret + a;
}

/* ------------------------------------------------------------------------------------ */
/* float geometry (geometry.cpp:3-17, map.cpp:17-51)                                     */
/* ------------------------------------------------------------------------------------ */
typedef struct { float x, y; } pt;
typedef struct { float u, v, w; } cube;

static pt cube_to_xy(cube c) {
  pt r;
  r.x = -4.0f / 3.0f * (c.v + 0.5f * c.u);
  r.y = 4.0f / 3.0f * (c.u + 0.5f * c.v);
  return r;
}
static cube xy_to_cube(pt p) {
  float hx = p.x / 2, hy = p.y / 2;
  cube c;
  c.u = hx + p.y;
  c.v = -p.x - hy;
  c.w = hx - hy;
  return c;
}
static cube cube_rotate(cube c, int times) {
  float u = -c.u, v = -c.v, w = -c.w;
  if (times == 1) { cube r = {v, w, u}; return r; }
  if (times == -1) { cube r = {w, u, v}; return r; }
  int single = (times < 0) ? -1 : 1;       /* 1 - 2*signbit(times) */
  return cube_rotate(cube_rotate(c, single), times - single);
}
static pt point_rotate(pt p, int times) {
  times = times % 6;
  return cube_to_xy(cube_rotate(xy_to_cube(p), times));
}
static inline int pt_less(pt a, pt b) { return (a.x < b.x) || (a.x == b.x && a.y < b.y); }
static inline int pt_eq(pt a, pt b) { return a.x == b.x && a.y == b.y; }
static int pt_cmp(const void *pa, const void *pb) {
  pt a = *(const pt *)pa, b = *(const pt *)pb;
  return pt_less(a, b) ? -1 : (pt_less(b, a) ? 1 : 0);
}

/* ------------------------------------------------------------------------------------ */
/* per-env map state                                                                     */
/* ------------------------------------------------------------------------------------ */
typedef struct {               /* one "global" MapPiece object (map.cpp:154-191); per env (Q8) */
  pt center;
  int rotation;
  int n;
  pt xy[37];
} piece_t;

typedef struct {
  piece_t pc[COG_N_PIECES];
  int *pieces; int npieces, cap_pieces;
  pt *xy; uint8_t *hex; int32_t *hidx; int nhex, cap_hex;
  pt mn, mx;
  long dimx, dimy;
  uint8_t *arr;                /* hex_array (dimx x dimy codes) */
  pt loc[4];
  int loc_size;
} omap;

/* ------------------------------------------------------------------------------------ */
/* per-env engine state                                                                  */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  uint8_t has_won, mip, n_removes, next_card_free, next_move_free;
  uint8_t n_in_hand, n_active, n_in_draw, idx_last;
  uint8_t steps_taken, n_added_cards;
  uint32_t n_movements;
} oplayer;

typedef struct {
  uint32_t seed;
  uint8_t n_players, n_pieces, difficulty;
  uint32_t max_steps;
  uint32_t rng;
  uint8_t agent, done;
  uint32_t turn_counter;
  oplayer pl[4];
  uint8_t n_in_market;
  uint8_t in_market[COG_N_SHOP];
  uint32_t flags;
  omap m;
  /* views into the vec buffers */
  cog_obs_t *obs;
  cog_action_mask_t *sel;
  float *rew;
  cog_info_t *info;
} oenv;

struct orc_vec {
  size_t n;
  cog_obs_t *obs;
  cog_action_mask_t *sel;
  float *rew;
  uint8_t *dones;
  uint8_t *agent_sel;
  cog_info_t *infos;
  oenv *env;
};

/* ---- map primitives ---------------------------------------------------------------- */
static void piece_init(piece_t *p, int id) {
  const cog_piece_meta_t *mt = &PMETA[id];
  p->center.x = 0; p->center.y = 0; p->rotation = 0; p->n = mt->n_hex;
  for (int k = 0; k < mt->n_hex; k++) {
    const int8_t *c = mt->size == COG_PS_LARGE ? LARGE_XY2[k]
                    : (mt->size == COG_PS_SMALL ? SMALL_XY2[k] : END_XY2[k]);
    p->xy[k].x = (float)c[0] / 2.0f;
    p->xy[k].y = (float)c[1] / 2.0f;
  }
}
static void piece_translate(piece_t *p, pt d) {            /* map.cpp:186-191 */
  for (int k = 0; k < p->n; k++) { p->xy[k].x = p->xy[k].x + d.x; p->xy[k].y = p->xy[k].y + d.y; }
  p->center.x = p->center.x + d.x; p->center.y = p->center.y + d.y;
}
static void piece_rotate(piece_t *p, int times) {          /* map.cpp:179-184 */
  times = times % 6;
  for (int k = 0; k < p->n; k++) p->xy[k] = point_rotate(p->xy[k], times);
  p->rotation = p->rotation + times;
}
static void piece_reset(piece_t *p) {                      /* map.cpp:174-177 */
  pt d = {-p->center.x, -p->center.y};
  piece_translate(p, d);
  piece_rotate(p, -p->rotation);
}

static void map_reset(omap *m) {                           /* map.cpp:744-752 */
  m->npieces = 0; m->nhex = 0;
  m->mn.x = m->mn.y = 0; m->mx.x = m->mx.y = 0;
  free(m->arr); m->arr = NULL; m->dimx = m->dimy = 0;
}

static void *grow(void *p, int *cap, int need, size_t elem) {
  if (need <= *cap) return p;
  int nc = *cap ? *cap : 64;
  while (nc < need) nc *= 2;
  p = realloc(p, (size_t)nc * elem);
  *cap = nc;
  return p;
}

static void add_piece(omap *m, int id, pt at, int rotation) {   /* map.cpp:309-341 */
  piece_t *p = &m->pc[id];
  piece_rotate(p, rotation);
  piece_translate(p, at);
  int cp = m->cap_pieces;
  m->pieces = (int *)grow(m->pieces, &cp, m->npieces + 1, sizeof(int));
  m->cap_pieces = cp;
  m->pieces[m->npieces++] = id;
  int need = m->nhex + p->n, ch = m->cap_hex;
  m->xy = (pt *)grow(m->xy, &ch, need, sizeof(pt));
  ch = m->cap_hex;
  m->hex = (uint8_t *)grow(m->hex, &ch, need, 1);
  ch = m->cap_hex;
  m->hidx = (int32_t *)grow(m->hidx, &ch, need, 2 * sizeof(int32_t));
  m->cap_hex = ch;
  for (int k = 0; k < p->n; k++) {
    m->xy[m->nhex + k] = p->xy[k];
    m->hex[m->nhex + k] = PHEX[id][k];
  }
  m->nhex = need;
  float b0 = m->mx.x, b1 = m->mx.y, b2 = m->mn.x, b3 = m->mn.y;
  for (int k = 0; k < p->n; k++) {
    pt a = p->xy[k];
    float n0 = a.x > b0 ? a.x : b0, n1 = a.y > b1 ? a.y : b1;
    float n2 = a.x < b2 ? a.x : b2, n3 = a.y < b3 ? a.y : b3;
    b0 = n0; b1 = n1; b2 = n2; b3 = n3;
  }
  m->dimx = (long)(3 + b0 - b2);
  m->dimy = (long)(3 + b1 - b3);
  m->mx.x = b0; m->mx.y = b1; m->mn.x = b2; m->mn.y = b3;
  free(m->arr);
  m->arr = (uint8_t *)malloc((size_t)(m->dimx * m->dimy));
  memset(m->arr, COG_HEX_MOUNTAIN, (size_t)(m->dimx * m->dimy));
  for (int i = 0; i < m->nhex; i++) {
    long ix = (long)(m->xy[i].x - m->mn.x + 1);
    long iy = (long)(m->xy[i].y - m->mn.y + 1);
    m->arr[ix * m->dimy + iy] = m->hex[i];
    m->hidx[2 * i] = (int32_t)ix;
    m->hidx[2 * i + 1] = (int32_t)iy;
  }
}

/* hex_array lookup, map.cpp:273-275: p = target - min; index (size_t)p + 1 */
static uint8_t map_lookup(oenv *e, pt target) {
  omap *m = &e->m;
  float px = target.x - m->mn.x, py = target.y - m->mn.y;
  long ix = (long)px + 1, iy = (long)py + 1;
  if (ix < 0 || iy < 0 || ix >= m->dimx || iy >= m->dimy || m->arr == NULL) {
    e->flags |= ORC_F_OOB_LOOKUP;
    return COG_HEX_MOUNTAIN;
  }
  return m->arr[ix * m->dimy + iy];
}

/* connection candidates of placed piece q for new piece p (map.cpp:192-263) */
typedef struct { pt c; int nopt; int opt[6]; } conn_t;

static int ref_connections(int qid, int new_size, conn_t *out) {
  const cog_piece_meta_t *q = &PMETA[qid];
  static const int8_t LL[2][2] = COG_CONN_LL_XY2, LS[3][2] = COG_CONN_LS_XY2;
  static const int8_t LT[1][2] = COG_CONN_LT_XY2, SL[6][2] = COG_CONN_SL_XY2;
  const int8_t (*base)[2] = NULL;
  int n = 0, nopt = 0, opt0[6];
  int can_rotate = 0;
  if (q->size == COG_PS_LARGE) {
    if (new_size == COG_PS_LARGE) {
      base = LL; n = 2; nopt = 6; can_rotate = 1;
      for (int k = 0; k < 6; k++) opt0[k] = -2 + k;
    } else if (new_size == COG_PS_SMALL) {
      base = LS; n = 3; nopt = 2; can_rotate = 1; opt0[0] = -1; opt0[1] = 2;
    } else if (new_size == COG_PS_TRIPLE && q->kind != COG_PT_START) {
      base = LT; n = 1; nopt = 1; can_rotate = 1; opt0[0] = -3;
    }
  } else if (q->size == COG_PS_SMALL && new_size == COG_PS_LARGE) {
    base = SL; n = 6; nopt = 6;
    for (int k = 0; k < 6; k++) opt0[k] = -2 + k;
  }
  if (n == 0) return 0;
  int total = 0;
  for (int j = 0; j < n; j++) {
    out[total].c.x = (float)base[j][0] / 2.0f;
    out[total].c.y = (float)base[j][1] / 2.0f;
    out[total].nopt = nopt;
    for (int k = 0; k < nopt; k++) out[total].opt[k] = opt0[k];
    total++;
  }
  if (can_rotate) {
    for (int i = 0; i < 6; i++)
      for (int j = 0; j < n; j++) {
        conn_t src = out[i * n + j];
        out[total].c = point_rotate(src.c, 1);
        out[total].nopt = src.nopt;
        for (int k = 0; k < src.nopt; k++) out[total].opt[k] = src.opt[k] + 1;
        total++;
      }
  }
  return total;
}

static int overlap(pt *p1, int n1, const pt *p2src, int n2, pt *scratch) {  /* map.cpp:53-74 */
  memcpy(scratch, p2src, sizeof(pt) * (size_t)n2);
  qsort(p1, (size_t)n1, sizeof(pt), pt_cmp);
  qsort(scratch, (size_t)n2, sizeof(pt), pt_cmp);
  int found = 0, done = (n1 == 0) || (n2 == 0);
  int i = 0, j = 0;
  while (!done) {
    pt a = p1[i], b = scratch[j];
    found = pt_eq(a, b);
    done = found;
    if (pt_less(a, b)) { i++; done |= i >= n1; }
    else { j++; done |= j >= n2; }
  }
  return found;
}

static int add_random_piece(omap *m, int id, uint32_t *rng) {   /* map.cpp:277-307 */
  piece_t *p = &m->pc[id];
  piece_reset(p);
  int ncand = 0;
  conn_t *cand = (conn_t *)malloc(sizeof(conn_t) * (size_t)(m->npieces * 42 + 1));
  conn_t tmp[42];
  for (int qi = 0; qi < m->npieces; qi++) {
    piece_t *q = &m->pc[m->pieces[qi]];
    int nc = ref_connections(m->pieces[qi], PMETA[id].size, tmp);
    for (int k = 0; k < nc; k++) {
      conn_t c = tmp[k];
      for (int o = 0; o < c.nopt; o++) c.opt[o] += q->rotation;
      pt r = point_rotate(c.c, q->rotation % 6);
      c.c.x = r.x + q->center.x;
      c.c.y = r.y + q->center.y;
      cand[ncand++] = c;
    }
  }
  int nvalid = 0;
  conn_t *valid = (conn_t *)malloc(sizeof(conn_t) * (size_t)(ncand + 1));
  pt fp[37];
  pt *scratch = (pt *)malloc(sizeof(pt) * (size_t)(m->nhex + 1));
  for (int i = 0; i < ncand; i++) {
    int t = cand[i].opt[0] % 6;
    for (int k = 0; k < p->n; k++) {
      pt r = point_rotate(p->xy[k], t);
      fp[k].x = r.x + cand[i].c.x;
      fp[k].y = r.y + cand[i].c.y;
    }
    if (!overlap(fp, p->n, m->xy, m->nhex, scratch)) valid[nvalid++] = cand[i];
  }
  free(scratch);
  int ok = 0;
  if (nvalid) {
    uint64_t idx = uid(rng, 0, (uint64_t)nvalid - 1);
    conn_t c = valid[idx];
    uint64_t ri = uid(rng, 0, (uint64_t)c.nopt - 1);
    add_piece(m, id, c.c, c.opt[ri]);
    ok = 1;
  }
  free(cand);
  free(valid);
  return ok;
}

static void finalize(oenv *e) {                            /* map.cpp:389-405 */
  omap *m = &e->m;
  if (m->dimx > 49 || m->dimy > 49) { e->flags |= ORC_F_GRID_OVER; return; }
  memset(e->obs->shared.map, 0, sizeof(e->obs->shared.map));
  for (int i = 0; i < m->nhex; i++) {
    uint8_t c = m->hex[i];
    uint8_t f[7] = {0, 0, 0, 0, 0, 0, 0};
    if (COG_HEX_REQ(c) != COG_REQ_NULL) f[COG_HEX_REQ(c) + 1] = COG_HEX_N(c);
    f[6] = COG_HEX_END(c);
    memcpy(e->obs->shared.map[m->hidx[2 * i]][m->hidx[2 * i + 1]], f, 7);
  }
}

/* libstdc++ >= 13 vector::erase(begin()+pos) on a trivially-copyable vector: move of
 * [pos+1, end) guarded by `_Num > 1` / `_Num == 1` (a no-op for negative counts), then
 * --finish.  A past-the-end position therefore drops the last element (Q5). */
static void erase_gcc13(uint64_t *v, int *n, uint64_t pos, uint32_t *flags) {
  long num = (long)*n - (long)(pos + 1);
  if (num >= 1) memmove(&v[pos], &v[pos + 1], sizeof(uint64_t) * (size_t)num);
  if ((long)pos >= (long)*n) *flags |= ORC_F_ERASE_PAST;
  *n -= 1;
}

static int generate(oenv *e, int failures, uint32_t rng) {  /* map.cpp:697-742; rng by value */
  if (failures >= COG_MAX_FAILURES) { e->flags |= ORC_F_MAPGEN_FAIL; return -1; }
  omap *m = &e->m;
  uint64_t s = uid(&rng, 0, 1);
  pt origin = {0, 0};
  add_piece(m, COG_PIECE_START0 + (int)s, origin, 0);
  uint64_t valid[COG_N_TRAVEL];
  int nvalid = 0;
  for (int i = 0; i < COG_N_TRAVEL; i++)
    if (PMETA[COG_PIECE_TRAVEL0 + i].difficulty <= e->difficulty) valid[nvalid++] = (uint64_t)i;
  for (int i = 0; i < e->n_pieces; i++) {
    int success;
    uint64_t next = 0;
    if (nvalid) {
      next = valid[uid(&rng, 0, (uint64_t)nvalid - 1)];
      success = add_random_piece(m, COG_PIECE_TRAVEL0 + (int)next, &rng);
    } else {
      success = 0;
    }
    if (success) erase_gcc13(valid, &nvalid, next, &e->flags);
    else if (generate(e, failures + 1, rng)) return -1;
  }
  uint64_t en = uid(&rng, 0, 1);
  if (!add_random_piece(m, COG_PIECE_END0 + (int)en, &rng)) {
    map_reset(m);
    if (generate(e, failures + 1, rng)) return -1;
  }
  finalize(e);
  return 0;
}

static void add_players(oenv *e) {                         /* map.cpp:343-354 */
  omap *m = &e->m;
  int n = e->n_players;
  if (n < m->loc_size) m->loc_size = n;
  else {
    for (int k = m->loc_size; k < n && k < 4; k++) { m->loc[k].x = 0; m->loc[k].y = 0; }
    m->loc_size = n;
  }
  int start = m->pieces[0];
  for (int i = 0; i < PMETA[start].n_hex; i++) {
    uint8_t c = PHEX[start][i];
    int ps = COG_HEX_REQ(c) == COG_REQ_NULL ? COG_HEX_N(c) : 0;
    if (ps > 0 && ps < n + 1) {
      if (i < m->loc_size) m->loc[i] = m->xy[i];
      else e->flags |= ORC_F_Q9_OOB;
    }
  }
  if (start == COG_PIECE_START0 + 1 && n < 4) e->flags |= ORC_F_B_START_LT4;
}

/* ------------------------------------------------------------------------------------ */
/* deck / player / shop (cards.cpp, player.cpp)                                          */
/* ------------------------------------------------------------------------------------ */
#define DK(e, p) ((uint8_t *)&(e)->obs->player_data[p].obs)
#define ST(e, p) (&(e)->obs->player_data[p].action_mask)

static inline int is_special(int c) { return c >= 15 && c <= 20; }

static size_t scan(oenv *e, const uint8_t *deck, int base, uint64_t target) {
  size_t c = 0;
  while (target >= deck[base + c]) {
    target -= deck[base + c];
    ++c;
    if ((size_t)base + c >= 105) { e->flags |= ORC_F_SCAN_OVER; return c; }
  }
  return c;
}

static void deck_move_discard_to_draw(oenv *e, int p) {    /* cards.cpp:234-240 */
  uint8_t *d = DK(e, p);
  oplayer *P = &e->pl[p];
  for (int i = 0; i < COG_N_CARDTYPES; i++) {
    d[COG_DECK_DRAW + i] = (uint8_t)(d[COG_DECK_DRAW + i] + d[COG_DECK_DISCARD + i]);
    P->n_in_draw = (uint8_t)(P->n_in_draw + d[COG_DECK_DISCARD + i]);
    d[COG_DECK_DISCARD + i] = 0;
  }
}

static void deck_draw(oenv *e, int p, uint8_t n) {         /* cards.cpp:183-211 */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  if (P->n_in_draw < n) deck_move_discard_to_draw(e, p);
  if (n > P->n_in_draw) n = P->n_in_draw;
  for (int i = 0; i < n; i++) {
    uint64_t t = uid(&e->rng, 0, (uint64_t)P->n_in_draw - 1);
    size_t c = scan(e, d, COG_DECK_DRAW, t);
    d[COG_DECK_DRAW + c]--;
    P->n_in_draw--;
    d[COG_DECK_HAND + c]++;
    e->sel->play[c + 1] = 1;
    e->sel->play_special[c + 1] = (uint8_t)is_special((int)c);
  }
  P->n_in_hand = (uint8_t)(P->n_in_hand + n);
}

static void deck_activate(oenv *e, int p, int c) {         /* cards.cpp:242-253 */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  P->n_in_hand--;
  P->n_active++;
  P->idx_last = (uint8_t)c;
  uint8_t prev = d[COG_DECK_HAND + c]--;
  d[COG_DECK_ACTIVE + c]++;
  e->sel->play[c + 1] = prev > 1;
  e->sel->play_special[c + 1] = e->sel->play[c + 1] && is_special(c);
}

static void deck_play_last_activated(oenv *e, int p) {     /* cards.cpp:255-261 */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  P->n_active--;
  d[COG_DECK_ACTIVE + P->idx_last]--;
  if (!CARDS[P->idx_last].single_use) d[COG_DECK_PLAYED + P->idx_last]++;
}

static void deck_play_immediate(oenv *e, int p, int c) {   /* cards.cpp:263-273 */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  P->n_in_hand--;
  uint8_t prev = d[COG_DECK_HAND + c]--;
  d[COG_DECK_PLAYED + c]++;
  e->sel->play[c + 1] = prev > 1;
  e->sel->play_special[c + 1] = e->sel->play[c + 1] && is_special(c);
}

static void deck_remove_immediate(oenv *e, int p, int c) { /* cards.cpp:281-290 */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  P->n_in_hand--;
  uint8_t prev = d[COG_DECK_HAND + c]--;
  e->sel->remove[c + 1] = e->sel->remove[c + 1] && prev > 1;
  e->sel->play[c + 1] = e->sel->play[c + 1] && prev > 1;
  e->sel->play_special[c + 1] = e->sel->play[c + 1] && is_special(c);
}

static void player_disable_playing(oenv *e) {              /* player.cpp:191-196 */
  memset(e->sel->play, 0, 22); e->sel->play[0] = 1;
  memset(e->sel->play_special, 0, 22); e->sel->play_special[0] = 1;
}
static void player_enable_playing(oenv *e, int p) {        /* player.cpp:198-206 */
  uint8_t *d = DK(e, p);
  memset(e->sel->remove, 0, 22); e->sel->remove[0] = 1;
  for (int k = 1; k < 22; k++) {
    e->sel->play[k] = d[COG_DECK_HAND + k - 1] > 0;
    e->sel->play_special[k] = e->sel->play[k] && is_special(k - 1);
  }
}

static void player_cards_from_active(oenv *e, int p, uint8_t n, int discard) {
  /* discard_cards / remove_cards (player.cpp:85-131) */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  uint8_t avail = P->n_active;
  if (n > avail) {
    if (discard) e->flags |= ORC_F_Q24_CLAMP;
    n = avail;
  }
  for (uint8_t i = 0; i < n; i++) {
    uint64_t t = uid(&e->rng, 0, (uint64_t)(avail - 1 - i));
    size_t c = scan(e, d, COG_DECK_ACTIVE, t);
    P->n_active--;
    d[COG_DECK_ACTIVE + c]--;
    if (discard) d[COG_DECK_DISCARD + c]++;
  }
}

static void player_handle_requirement(oenv *e, int p, int req, uint8_t n) {  /* player.cpp:141-162 */
  oplayer *P = &e->pl[p];
  float *res = e->obs->shared.current_resources;
  if (req < 3) {
    float left = res[req] - (float)n;
    res[0] = res[1] = res[2] = 0;
    res[req] = left;
    if (!P->mip) { deck_play_last_activated(e, p); P->mip = 1; }
  } else if (req == COG_REQ_REMOVE) {
    player_cards_from_active(e, p, n, 0);
    res[0] = res[1] = res[2] = 0;
    P->mip = 0;
  } else if (req == COG_REQ_DISCARD) {
    player_cards_from_active(e, p, n, 1);
    res[0] = res[1] = res[2] = 0;
    P->mip = 0;
  }
}

static void save_mask(oenv *e, int p) { memcpy(ST(e, p), e->sel, COG_MASK_USED); }
static void load_mask(oenv *e, int p) { memcpy(e->sel, ST(e, p), COG_MASK_USED); }

static void player_end_turn(oenv *e, int p) {              /* player.cpp:170-180 */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  P->n_active = 0;
  for (int i = 0; i < COG_N_CARDTYPES; i++) {
    d[COG_DECK_DISCARD + i] = (uint8_t)(d[COG_DECK_DISCARD + i] + d[COG_DECK_ACTIVE + i]);
    d[COG_DECK_ACTIVE + i] = 0;
  }
  for (int i = 0; i < COG_N_CARDTYPES; i++) {
    d[COG_DECK_DISCARD + i] = (uint8_t)(d[COG_DECK_DISCARD + i] + d[COG_DECK_PLAYED + i]);
    d[COG_DECK_PLAYED + i] = 0;
  }
  int n_draw = COG_HAND_SIZE - (int)P->n_in_hand;
  if (n_draw > 0) deck_draw(e, p, (uint8_t)n_draw);
  e->obs->shared.current_resources[0] = 0;
  e->obs->shared.current_resources[1] = 0;
  e->obs->shared.current_resources[2] = 0;
  save_mask(e, p);
}

static void player_reset(oenv *e, int p) {                 /* player.cpp:29-43 */
  oplayer *P = &e->pl[p];
  uint8_t *d = DK(e, p);
  P->has_won = P->mip = P->next_card_free = P->next_move_free = 0;
  P->n_removes = 0; P->steps_taken = 0; P->n_movements = 0; P->n_added_cards = 0;
  memset(d + COG_DECK_DRAW, 0, 21); memset(d + COG_DECK_HAND, 0, 21);
  memset(d + COG_DECK_ACTIVE, 0, 21); memset(d + COG_DECK_DISCARD, 0, 21);   /* played kept (Q10) */
  cog_action_mask_t *s = e->sel;                           /* ActionMask::reset, api.h:104-118 */
  s->play[0] = 1; memset(s->play + 1, 0, 21);
  s->remove[0] = 1; memset(s->remove + 1, 0, 21);
  s->play_special[0] = 1; memset(s->play_special + 1, 0, 21);
  s->move[0] = 1; s->get_from_shop[0] = 1;
  d[COG_DECK_DISCARD + 0] = 3; d[COG_DECK_DISCARD + 7] = 4; d[COG_DECK_DISCARD + 5] = 1;
  P->n_in_draw = 0; P->n_in_hand = 0; P->n_active = 0;
  deck_draw(e, p, COG_HAND_SIZE);
  save_mask(e, p);
}

static void shop_set_available_mask(oenv *e, float coins, uint8_t *mask) {  /* cards.cpp:109-121 */
  const uint8_t *avail = e->obs->shared.shop;
  for (int i = 0; i < COG_N_SHOP; i++) {
    float cost = (float)CARDS[SHOP_TYPES[i]].cost;
    if (e->n_in_market < COG_MKT_SLOTS) mask[i + 1] = (avail[i] > 0) && (coins > cost);
    else mask[i + 1] = e->in_market[i] && (coins > cost);
  }
}

static int shop_get(oenv *e, int k) {                      /* cards.cpp:136-142 */
  uint8_t *avail = e->obs->shared.shop;
  avail[k]--;
  if (!avail[k] && e->in_market[k]) { e->in_market[k] = 0; e->n_in_market--; }
  return SHOP_TYPES[k];
}

static void set_movement_mask(oenv *e, uint8_t *move, int player, const float *res, uint8_t n_active) {
  /* map.cpp:369-387 */
  pt loc = e->m.loc[player];
  for (int i = 1; i < 7; i++) {
    pt t = {loc.x + (float)DIR_XY2[i][0] / 2.0f, loc.y + (float)DIR_XY2[i][1] / 2.0f};
    uint8_t c = map_lookup(e, t);
    int req = COG_HEX_REQ(c), filled;
    if (req >= COG_REQ_DISCARD) filled = n_active > COG_HEX_N(c);
    else filled = res[req] >= (float)COG_HEX_N(c);
    move[i] = (req != COG_REQ_NULL) && filled;
  }
}

static void update_observation(oenv *e, int agent) {       /* environment.cpp:252-279 */
  cog_action_mask_t *am = ST(e, agent);
  memset(am->move, 0, 7); am->move[0] = 1;
  memset(am->get_from_shop, 0, 19); am->get_from_shop[0] = 1;
  uint8_t ph = e->obs->shared.phase;
  if (ph == COG_PHASE_MOVEMENT)
    set_movement_mask(e, am->move, agent, e->obs->shared.current_resources, e->pl[agent].n_active);
  else if (ph == COG_PHASE_BUYING)
    shop_set_available_mask(e, e->obs->shared.current_resources[2], am->get_from_shop);
}

static int env_reset(oenv *e) {                            /* environment.cpp:42-64 */
  e->agent = 0;
  e->obs->shared.phase = COG_PHASE_INACTIVE;
  map_reset(&e->m);
  if (generate(e, 0, e->rng)) return -1;
  for (int i = 0; i < e->n_players; i++) player_reset(e, i);
  add_players(e);
  for (int k = 0; k < COG_N_SHOP; k++) {                   /* Shop::reset, cards.cpp:94-100 */
    e->obs->shared.shop[k] = COG_CARDS_PER_TYPE;
    e->in_market[k] = CARDS[SHOP_TYPES[k]].in_market;
  }
  e->done = 0;
  e->turn_counter = 0;
  for (int i = 0; i < e->n_players; i++) update_observation(e, i);
  memcpy(e->sel, ST(e, 0), COG_MASK_USED);
  return 0;
}

static void apply_special(oenv *e, int special, int p) {   /* cards.cpp:8-36, environment.cpp:156-158 */
  cog_action_mask_t *mask = ST(e, e->agent);
  oplayer *P = &e->pl[p];
  switch (special) {
  case COG_SPECIAL_DRAW2: deck_draw(e, p, 2); break;
  case COG_SPECIAL_DRAW3: deck_draw(e, p, 3); break;
  case COG_SPECIAL_DRAW1_REMOVE1:
  case COG_SPECIAL_DRAW2_REMOVE2: {
    int k = special == COG_SPECIAL_DRAW1_REMOVE1 ? 1 : 2;
    deck_draw(e, p, (uint8_t)k);
    P->n_removes = (uint8_t)k;
    memcpy(mask->remove, mask->play, 22);
    player_disable_playing(e);
    shop_set_available_mask(e, 0.0f, mask->get_from_shop);
  } break;
  case COG_SPECIAL_TRANSMIT:
    memset(mask->move, 0, 7); mask->move[0] = 1;
    player_disable_playing(e);
    for (int i = 0; i < COG_N_SHOP; i++) mask->get_from_shop[i + 1] = e->obs->shared.shop[i] > 0;
    P->next_card_free = 1;
    break;
  case COG_SPECIAL_NATIVE: {
    float r100[3] = {100, 100, 100};
    set_movement_mask(e, mask->move, p, r100, 100);
    P->next_move_free = 1;
    player_disable_playing(e);
    shop_set_available_mask(e, 0.0f, mask->get_from_shop);
  } break;
  case COG_SPECIAL_SHOP_OFF: shop_set_available_mask(e, 0.0f, mask->get_from_shop); break;
  default: break;
  }
}

static void env_step(oenv *e, const cog_action_t *a) {     /* environment.cpp:91-224 */
  if (e->done) return;
  int ag = e->agent;
  e->info->agent_infos[ag].steps_taken++;
  if (e->obs->shared.phase == COG_PHASE_INACTIVE) e->obs->shared.phase = COG_PHASE_MOVEMENT;
  oplayer *P = &e->pl[ag];
  P->steps_taken++;
  float *res = e->obs->shared.current_resources;
  int special = COG_SPECIAL_NONE;
  if (a->play) {
    int c = (uint8_t)(a->play - 1);
    const cog_card_t *cd = &CARDS[c];
    uint8_t ph = e->obs->shared.phase;
    if (ph == COG_PHASE_MOVEMENT) {
      res[0] = cd->res[0]; res[1] = cd->res[1]; res[2] = cd->res[2];
    } else if (ph == COG_PHASE_BUYING) {
      if (cd->res[2] > 0) res[2] += cd->res[2];
      else res[2] += 0.5f;
    }
    deck_activate(e, ag, c);
  } else if (a->play_special) {
    int c = (uint8_t)(a->play_special - 1);
    if (CARDS[c].single_use) deck_remove_immediate(e, ag, c);
    else deck_play_immediate(e, ag, c);
    special = CARDS[c].special;
  } else if (a->move) {
    pt *loc = &e->m.loc[ag];
    loc->x = loc->x + (float)DIR_XY2[a->move][0] / 2.0f;
    loc->y = loc->y + (float)DIR_XY2[a->move][1] / 2.0f;
    uint8_t c = map_lookup(e, *loc);
    if (!P->next_move_free) player_handle_requirement(e, ag, COG_HEX_REQ(c), COG_HEX_N(c));
    else { P->next_move_free = 0; player_enable_playing(e, ag); }
    P->n_movements++;
    P->has_won = COG_HEX_END(c);
  } else {
    P->next_move_free = 0;
    if (a->get_from_shop) {
      int k = (uint8_t)(a->get_from_shop - 1);
      int type;
      if (P->next_card_free) {
        type = shop_get(e, k);
      } else {
        e->n_in_market = (uint8_t)(e->n_in_market + (uint8_t)(1 - e->in_market[k]));
        e->in_market[k] = 1;
        type = shop_get(e, k);
        res[2] -= (float)CARDS[type].cost;
        e->obs->shared.phase = (uint8_t)((e->obs->shared.phase + 1) % 3);
      }
      DK(e, ag)[COG_DECK_DISCARD + type]++;
      P->n_added_cards++;
    } else if (a->remove) {
      int c = (uint8_t)(a->remove - 1);
      deck_remove_immediate(e, ag, c);
      if (!--P->n_removes) player_enable_playing(e, ag);
      else special = COG_SPECIAL_SHOP_OFF;
    } else {
      e->obs->shared.phase = (uint8_t)((e->obs->shared.phase + 1) % 3);
      if (P->n_removes > 0) { P->n_removes = 0; player_enable_playing(e, ag); }
    }
    if (P->next_card_free) { P->next_card_free = 0; player_enable_playing(e, ag); }
  }
  if (P->mip && !a->move) { P->mip = 0; res[0] = res[1] = res[2] = 0; }
  /* maybe_end_turn / next_agent (environment.cpp:244-250, 79-89) */
  if (P->has_won || e->obs->shared.phase == COG_PHASE_INACTIVE) {
    player_end_turn(e, ag);
    e->agent = (uint8_t)(e->agent + 1);
    if (e->agent >= e->n_players) e->agent = 0;
    load_mask(e, e->agent);
    res[0] = res[1] = res[2] = 0;
    e->turn_counter++;
  }
  update_observation(e, e->agent);
  if (special != COG_SPECIAL_NONE) {
    apply_special(e, special, ag);
  } else {
    uint8_t c = map_lookup(e, e->m.loc[e->agent]);
    if (COG_HEX_END(c) || e->turn_counter >= e->max_steps) {
      e->done = 1;
      e->info->total_length = e->turn_counter;
      float n_winners = 0;
      for (int q = 0; q < 4; q++) n_winners += (float)e->pl[q].has_won;
      for (int q = 0; q < e->n_players; q++) {
        cog_agent_info_t *ai = &e->info->agent_infos[q];
        oplayer *Q = &e->pl[q];
        ai->steps_taken = Q->steps_taken;
        float r = (float)(e->n_players * Q->has_won) - n_winners;
        ai->returns = r;
        e->rew[q] = r;
        ai->travelled_hexes = Q->n_movements;
        ai->cards_added = Q->n_added_cards;
        ai->n_machete_uses = ai->n_paddle_uses = ai->n_coin_uses = 0;
        ai->n_card_uses = Q->n_added_cards;
        ai->cards_removed = Q->n_added_cards;
      }
    }
  }
}

/* ------------------------------------------------------------------------------------ */
/* vec layer (vec_environment.h)                                                          */
/* ------------------------------------------------------------------------------------ */
static void mask_default(cog_action_mask_t *m) {          /* ActionMask() ctor, tails zero (Q26) */
  memset(m, 0, sizeof(*m));
  m->play[0] = m->play_special[0] = m->remove[0] = m->move[0] = m->get_from_shop[0] = 1;
}

orc_vec *orc_create(size_t n) {
  orc_vec *v = (orc_vec *)calloc(1, sizeof(orc_vec));
  v->n = n;
  v->obs = (cog_obs_t *)aligned_alloc(64, n * sizeof(cog_obs_t) + 64);
  v->sel = (cog_action_mask_t *)aligned_alloc(64, n * sizeof(cog_action_mask_t) + 64);
  v->infos = (cog_info_t *)aligned_alloc(64, n * sizeof(cog_info_t) + 64);
  memset(v->obs, 0, n * sizeof(cog_obs_t));
  memset(v->infos, 0, n * sizeof(cog_info_t));
  v->rew = (float *)calloc(n * 4 + 1, sizeof(float));
  v->dones = (uint8_t *)calloc(n + 1, 1);
  v->agent_sel = (uint8_t *)calloc(n + 1, 1);
  v->env = (oenv *)calloc(n, sizeof(oenv));
  uint32_t rs = (uint32_t)time(NULL);
  for (size_t i = 0; i < n; i++) {
    oenv *e = &v->env[i];
    e->obs = &v->obs[i]; e->sel = &v->sel[i]; e->rew = &v->rew[4 * i]; e->info = &v->infos[i];
    mask_default(e->sel);
    for (int p = 0; p < 4; p++) mask_default(&v->obs[i].player_data[p].action_mask);
    e->seed = rs + (uint32_t)i;                 /* std::random_device in the reference */
    e->rng = mr_seed(e->seed);
    e->n_players = 4; e->n_pieces = 3; e->difficulty = 0; e->max_steps = 100000;
    e->n_in_market = COG_MKT_SLOTS;             /* Shop ctor, cards.cpp:85-92 */
    for (int k = 0; k < COG_N_SHOP; k++) {
      e->in_market[k] = CARDS[SHOP_TYPES[k]].in_market;
      v->obs[i].shared.shop[k] = COG_CARDS_PER_TYPE;   /* Shop::init */
    }
    for (int pid = 0; pid < COG_N_PIECES; pid++) piece_init(&e->m.pc[pid], pid);
  }
  return v;
}

void orc_destroy(orc_vec *v) {
  if (!v) return;
  for (size_t i = 0; i < v->n; i++) {
    omap *m = &v->env[i].m;
    free(m->pieces); free(m->xy); free(m->hex); free(m->hidx); free(m->arr);
  }
  free(v->env); free(v->obs); free(v->sel); free(v->infos); free(v->rew); free(v->dones);
  free(v->agent_sel); free(v);
}

size_t orc_num_envs(const orc_vec *v) { return v->n; }

int orc_reset(orc_vec *v, uint32_t seed, uint8_t n_players, uint8_t n_pieces, int difficulty,
              uint32_t max_steps) {
  for (size_t i = 0; i < v->n; i++) {
    oenv *e = &v->env[i];
    e->n_players = n_players; e->n_pieces = n_pieces; e->difficulty = (uint8_t)difficulty;
    e->max_steps = max_steps;
    e->seed = (uint32_t)(seed + (uint32_t)i);
    e->rng = mr_seed(e->seed);
    if (env_reset(e)) return -1;
  }
  return 0;
}

/* orc_reset over n_threads threads (envs are independent; each env's reset is the serial one) */
typedef struct { orc_vec *v; uint32_t seed; uint8_t np, npc; int diff; uint32_t ms; size_t lo, hi; int rc; } reset_arg;
static void *reset_worker(void *p) {
  reset_arg *a = (reset_arg *)p;
  for (size_t i = a->lo; i < a->hi; i++) {
    oenv *e = &a->v->env[i];
    e->n_players = a->np; e->n_pieces = a->npc; e->difficulty = (uint8_t)a->diff;
    e->max_steps = a->ms;
    e->seed = (uint32_t)(a->seed + (uint32_t)i);
    e->rng = mr_seed(e->seed);
    if (env_reset(e)) a->rc = -1;
  }
  return NULL;
}
int orc_reset_threaded(orc_vec *v, uint32_t seed, uint8_t n_players, uint8_t n_pieces, int difficulty,
                       uint32_t max_steps, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
  reset_arg *ra = (reset_arg *)calloc((size_t)n_threads, sizeof(reset_arg));
  const size_t b = v->n / (size_t)n_threads;
  int rc = 0;
  for (int i = 0; i < n_threads; i++) {
    ra[i] = (reset_arg){v, seed, n_players, n_pieces, difficulty, max_steps, (size_t)i * b,
                        i < n_threads - 1 ? (size_t)(i + 1) * b : v->n, 0};
    pthread_create(&th[i], NULL, reset_worker, &ra[i]);
  }
  for (int i = 0; i < n_threads; i++) {
    pthread_join(th[i], NULL);
    rc |= ra[i].rc;
  }
  free(th); free(ra);
  return rc;
}

int orc_reset_default(orc_vec *v) {
  for (size_t i = 0; i < v->n; i++)
    if (env_reset(&v->env[i])) return -1;
  return 0;
}

int orc_step_range(orc_vec *v, const void *actions, size_t lo, size_t hi) {
  const cog_action_t *a = (const cog_action_t *)actions;
  int rc = 0;
  for (size_t i = lo; i < hi; i++) {           /* vec_cog_env::step_single, :53-61 */
    oenv *e = &v->env[i];
    env_step(e, &a[i]);
    v->dones[i] = e->done;
    if (e->done && env_reset(e)) rc = -1;
    v->agent_sel[i] = e->agent;
  }
  return rc;
}
int orc_step(orc_vec *v, const void *actions) { return orc_step_range(v, actions, 0, v->n); }

void *orc_obs(orc_vec *v) { return v->obs; }
void *orc_sel(orc_vec *v) { return v->sel; }
float *orc_rewards(orc_vec *v) { return v->rew; }
uint8_t *orc_dones(orc_vec *v) { return v->dones; }
uint8_t *orc_agent_sel(orc_vec *v) { return v->agent_sel; }
void *orc_infos(orc_vec *v) { return v->infos; }
uint32_t orc_flags(const orc_vec *v, size_t i) { return v->env[i].flags; }
void orc_clear_flags(orc_vec *v) { for (size_t i = 0; i < v->n; i++) v->env[i].flags = 0; }

int orc_debug_state(const orc_vec *v, size_t i, uint32_t *out, size_t n_out) {
  const oenv *e = &v->env[i];
  uint32_t tmp[64];
  size_t k = 0;
  tmp[k++] = e->rng; tmp[k++] = e->turn_counter; tmp[k++] = e->agent; tmp[k++] = e->done;
  tmp[k++] = e->n_in_market;
  uint32_t im = 0;
  for (int s = 0; s < COG_N_SHOP; s++) im |= (uint32_t)e->in_market[s] << s;
  tmp[k++] = im;
  for (int p = 0; p < 4; p++) {
    const oplayer *P = &e->pl[p];
    tmp[k++] = (uint32_t)P->has_won | (uint32_t)P->mip << 8 | (uint32_t)P->n_removes << 16 |
               (uint32_t)P->next_card_free << 24;
    tmp[k++] = (uint32_t)P->next_move_free | (uint32_t)P->n_in_hand << 8 |
               (uint32_t)P->n_active << 16 | (uint32_t)P->n_in_draw << 24;
    tmp[k++] = (uint32_t)P->idx_last | (uint32_t)P->steps_taken << 8 |
               (uint32_t)P->n_added_cards << 16;
    tmp[k++] = P->n_movements;
    int lx = (int)lrintf(e->m.loc[p].x * 2), ly = (int)lrintf(e->m.loc[p].y * 2);
    tmp[k++] = (uint32_t)(lx & 0xffff) | (uint32_t)(ly & 0xffff) << 16;
  }
  int mnx = (int)lrintf(e->m.mn.x * 2), mny = (int)lrintf(e->m.mn.y * 2);
  tmp[k++] = (uint32_t)(mnx & 0xffff) | (uint32_t)(mny & 0xffff) << 16;
  tmp[k++] = (uint32_t)e->m.dimx | (uint32_t)e->m.dimy << 16;
  for (size_t j = 0; j < k && j < n_out; j++) out[j] = tmp[j];
  return (int)k;
}

/* ------------------------------------------------------------------------------------ */
/* sampler (sampler.h:14-79, vec_sampler.h:7-28)                                          */
/* ------------------------------------------------------------------------------------ */
struct orc_sampler {
  size_t n;
  uint32_t *rng;
  cog_action_t *actions;
};

/* sampler i seeded seed + first + i in size_t (vec_sampler.h:9-13: seed + i, seed a u32; first: the
   global index of env 0 when the batch is one rank's block of a larger one) */
orc_sampler *orc_sampler_create_at(size_t n, uint32_t seed, uint64_t first) {
  orc_sampler *s = (orc_sampler *)calloc(1, sizeof(orc_sampler));
  s->n = n;
  s->rng = (uint32_t *)calloc(n + 1, sizeof(uint32_t));
  s->actions = (cog_action_t *)aligned_alloc(64, n * sizeof(cog_action_t) + 64);
  memset(s->actions, 0, n * sizeof(cog_action_t));
  for (size_t i = 0; i < n; i++) s->rng[i] = mr_seed((uint64_t)seed + first + (uint64_t)i);
  return s;
}
orc_sampler *orc_sampler_create(size_t n, uint32_t seed) { return orc_sampler_create_at(n, seed, 0); }
void orc_sampler_destroy(orc_sampler *s) {
  if (!s) return;
  free(s->rng); free(s->actions); free(s);
}

static uint8_t sample_head(uint32_t *rng, const uint8_t *m, int len) {
  uint8_t valid[32];
  int k = 0;
  for (int i = 0; i < len; i++)
    if (m[i]) valid[k++] = (uint8_t)i;
  if (!k) return 0;
  return valid[uid(rng, 0, (uint64_t)k - 1)];
}

void orc_sample_range(orc_sampler *s, const void *masks, size_t lo, size_t hi) {
  const cog_action_mask_t *m = (const cog_action_mask_t *)masks;
  for (size_t i = lo; i < hi; i++) {
    cog_action_t *a = &s->actions[i];
    uint32_t *r = &s->rng[i];
    a->play = sample_head(r, m[i].play, 22);
    a->play_special = sample_head(r, m[i].play_special, 22);
    a->remove = sample_head(r, m[i].remove, 22);
    a->move = sample_head(r, m[i].move, 7);
    a->get_from_shop = sample_head(r, m[i].get_from_shop, 19);
  }
}
void orc_sample(orc_sampler *s, const void *masks) { orc_sample_range(s, masks, 0, s->n); }
void *orc_sampler_actions(orc_sampler *s) { return s->actions; }

/* ------------------------------------------------------------------------------------ */
/* threaded CPU baseline in the shape of ThreadedRunner (runner.h:21-64)                  */
/* ------------------------------------------------------------------------------------ */
typedef struct {
  orc_vec *v; orc_sampler *s; size_t lo, hi; int steps; int cpu;
  pthread_barrier_t *bar;
} worker_arg;

static void *worker(void *p) {
  worker_arg *w = (worker_arg *)p;
  if (w->cpu >= 0) {
    cpu_set_t cs; CPU_ZERO(&cs); CPU_SET(w->cpu, &cs);
    pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
  }
  pthread_barrier_wait(w->bar);
  for (int t = 0; t < w->steps; t++) {
    orc_sample_range(w->s, w->v->sel, w->lo, w->hi);        /* runner.h:46-50 */
    orc_step_range(w->v, w->s->actions, w->lo, w->hi);      /* runner.h:51-55 */
    pthread_barrier_wait(w->bar);                           /* step_sync per step */
  }
  return NULL;
}

double orc_run_threaded(orc_vec *v, orc_sampler *s, int steps, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  cpu_set_t allowed; CPU_ZERO(&allowed);
  sched_getaffinity(0, sizeof(allowed), &allowed);
  int cpus[1024], ncpu = 0;
  for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; c++) if (CPU_ISSET(c, &allowed)) cpus[ncpu++] = c;
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)n_threads + 1);
  pthread_t *th = (pthread_t *)calloc((size_t)n_threads, sizeof(pthread_t));
  worker_arg *wa = (worker_arg *)calloc((size_t)n_threads, sizeof(worker_arg));
  size_t batch = v->n / (size_t)n_threads;
  for (int i = 0; i < n_threads; i++) {
    wa[i].v = v; wa[i].s = s; wa[i].steps = steps; wa[i].bar = &bar;
    wa[i].lo = (size_t)i * batch;
    wa[i].hi = i < n_threads - 1 ? wa[i].lo + batch : v->n;
    wa[i].cpu = ncpu > 0 ? cpus[(i + 1) % ncpu] : -1;   /* leave cpus[0] to the main thread */
    pthread_create(&th[i], NULL, worker, &wa[i]);
  }
  struct timespec t0, t1;
  pthread_barrier_wait(&bar);
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < steps; t++) pthread_barrier_wait(&bar);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  for (int i = 0; i < n_threads; i++) pthread_join(th[i], NULL);
  pthread_barrier_destroy(&bar);
  free(th); free(wa);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
