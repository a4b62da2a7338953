/* cog_tables.h -- City-of-Gold game data, shared (as data only) by the HIP engine and the
 * CPU oracle.  Plain C so it compiles under gcc (oracle), g++ and hipcc (engine).
 *
 * Provenance (all values re-encoded, no reference code):
 *   cards           : reference src/cards.cpp:40-71   (cost, starts_in_market, single_use, m/p/c, special)
 *   shop slots      : reference src/cards.cpp:72-78
 *   hex catalogue   : reference src/map.cpp:113-152
 *   piece hexes     : reference src/map.cpp:464-695   (extracted by oracle/tools/extract_tables.py)
 *   piece coords    : reference src/map.cpp:446-462
 *   connections     : reference src/map.cpp:203-263
 *
 * Hex code byte:  bits 0-2 = n_required (for NULL hexes: player_start, unobservable),
 *                 bits 3-5 = requirement (MACHETE 0, PADDLE 1, COIN 2, DISCARD 3, REMOVE 4, NULL 5),
 *                 bit  6   = is_end.
 * Coordinates are stored DOUBLED (2x, 2y) so every lattice point is an integer.
 */
#ifndef COG_TABLES_H
#define COG_TABLES_H
#include <stdint.h>

#define COG_N_CARDTYPES 21
#define COG_N_SHOP 18
#define COG_GRID 48
#define COG_N_FEAT 7
#define COG_MAX_PLAYERS 4
#define COG_MAX_FAILURES 5
#define COG_HAND_SIZE 4
#define COG_MKT_SLOTS 6
#define COG_CARDS_PER_TYPE 3

enum { COG_REQ_MACHETE = 0, COG_REQ_PADDLE, COG_REQ_COIN, COG_REQ_DISCARD, COG_REQ_REMOVE, COG_REQ_NULL };
enum { COG_PHASE_INACTIVE = 0, COG_PHASE_MOVEMENT = 1, COG_PHASE_BUYING = 2 };
enum { COG_SPECIAL_NONE = 0, COG_SPECIAL_TRANSMIT, COG_SPECIAL_DRAW2, COG_SPECIAL_DRAW3,
       COG_SPECIAL_DRAW1_REMOVE1, COG_SPECIAL_DRAW2_REMOVE2, COG_SPECIAL_NATIVE,
       COG_SPECIAL_SHOP_OFF /* the remove-lambda of environment.cpp:156-158 */ };

#define COG_HEX_REQ(c) (((c) >> 3) & 7)
#define COG_HEX_N(c) ((c) & 7)
#define COG_HEX_END(c) (((c) >> 6) & 1)
#define COG_HEX_MOUNTAIN 40

/* card: cost, starts_in_market, single_use, machete, paddle, coin, special-kind */
typedef struct { uint8_t cost, in_market, single_use, res[3], special; } cog_card_t;
#define COG_CARD_TABLE { \
    {1, 0, 0, {1, 0, 0}, 0}, /* 0 Explorer        */ \
    {1, 1, 0, {2, 0, 0}, 0}, /* 1 Scout           */ \
    {3, 1, 0, {3, 0, 0}, 0}, /* 2 Trailblazer     */ \
    {5, 0, 0, {5, 0, 0}, 0}, /* 3 Pioneer         */ \
    {3, 0, 1, {6, 0, 0}, 0}, /* 4 Giant machete   */ \
    {1, 0, 0, {0, 1, 0}, 0}, /* 5 Sailor          */ \
    {2, 0, 0, {0, 3, 0}, 0}, /* 6 Captain         */ \
    {1, 0, 0, {0, 0, 1}, 0}, /* 7 Traveler        */ \
    {2, 1, 0, {0, 0, 2}, 0}, /* 8 Photographer    */ \
    {3, 0, 0, {0, 0, 3}, 0}, /* 9 Journalist      */ \
    {3, 1, 0, {0, 0, 4}, 0}, /* 10 Treasure chest */ \
    {5, 0, 0, {0, 0, 4}, 0}, /* 11 Millionaire    */ \
    {2, 1, 0, {1, 1, 1}, 0}, /* 12 Jack of all trades */ \
    {4, 0, 0, {2, 2, 2}, 0}, /* 13 Adventurer     */ \
    {4, 0, 1, {4, 4, 4}, 0}, /* 14 Prop plane     */ \
    {4, 1, 1, {0, 0, 0}, COG_SPECIAL_TRANSMIT},          /* 15 Transmitter  */ \
    {4, 0, 0, {0, 0, 0}, COG_SPECIAL_DRAW2},             /* 16 Cartographer */ \
    {2, 0, 1, {0, 0, 0}, COG_SPECIAL_DRAW3},             /* 17 Compass      */ \
    {4, 0, 0, {0, 0, 0}, COG_SPECIAL_DRAW1_REMOVE1},     /* 18 Scientist    */ \
    {3, 0, 1, {0, 0, 0}, COG_SPECIAL_DRAW2_REMOVE2},     /* 19 Travel log   */ \
    {5, 0, 0, {0, 0, 0}, COG_SPECIAL_NATIVE},            /* 20 Native       */ \
}
/* shop slot -> card type (cards.cpp:72-78) */
#define COG_SHOP_TYPES {1, 2, 3, 4, 6, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20}
/* starting deck: 3 Explorer, 4 Traveler, 1 Sailor (cards.cpp:163-166) */

/* ---- map pieces ---------------------------------------------------------------------- */
enum { COG_PT_START = 0, COG_PT_TRAVEL = 1, COG_PT_END = 2 };
enum { COG_PS_LARGE = 0, COG_PS_SMALL = 1, COG_PS_TRIPLE = 2 };
#define COG_N_PIECES 20      /* 0-1 start A/B, 2-17 travel C..R, 18-19 end 1/2 */
#define COG_PIECE_START0 0
#define COG_PIECE_TRAVEL0 2
#define COG_N_TRAVEL 16
#define COG_PIECE_END0 18

/* kind, size, difficulty, n_hexes */
typedef struct { uint8_t kind, size, difficulty, n_hex; } cog_piece_meta_t;
#define COG_PIECE_META { \
    {0, 0, 0, 37}, /* A */ \
    {0, 0, 0, 37}, /* B */ \
    {1, 0, 0, 37}, /* C */ \
    {1, 0, 1, 37}, /* D */ \
    {1, 0, 2, 37}, /* E */ \
    {1, 0, 0, 37}, /* F */ \
    {1, 0, 2, 37}, /* G */ \
    {1, 0, 1, 37}, /* H */ \
    {1, 0, 1, 37}, /* I */ \
    {1, 0, 0, 37}, /* J */ \
    {1, 0, 1, 37}, /* K */ \
    {1, 0, 1, 37}, /* L */ \
    {1, 0, 2, 37}, /* M */ \
    {1, 0, 1, 37}, /* N */ \
    {1, 1, 2, 16}, /* O */ \
    {1, 1, 1, 16}, /* P */ \
    {1, 1, 1, 16}, /* Q */ \
    {1, 1, 1, 16}, /* R */ \
    {2, 2, 0, 3}, /* END1 */ \
    {2, 2, 0, 3}, /* END2 */ \
}
#define COG_PIECE_HEX { \
    {41, 42, 43, 44, 1, 1, 1, 1, 1, 1, 1, 17, 1, 9, 1, 1, 17, 1, 9, 1, 17, 1, 1, 40, 17, 1, 1, 1, 9, 40, 1, 1, 17, 1, 33, 1, 1}, /* A */ \
    {44, 43, 42, 41, 1, 1, 1, 1, 1, 1, 1, 9, 1, 1, 1, 9, 1, 17, 1, 17, 1, 1, 1, 17, 1, 1, 1, 1, 1, 1, 17, 40, 1, 1, 9, 33, 9}, /* B */ \
    {1, 1, 9, 9, 17, 25, 1, 17, 9, 17, 25, 9, 9, 17, 17, 9, 17, 25, 40, 9, 25, 25, 9, 9, 17, 17, 25, 9, 1, 17, 25, 9, 9, 1, 1, 25, 25}, /* C */ \
    {2, 1, 1, 1, 1, 9, 9, 9, 1, 1, 9, 10, 9, 9, 1, 2, 1, 1, 40, 10, 9, 2, 1, 19, 40, 1, 9, 1, 40, 17, 19, 1, 1, 11, 40, 1, 2}, /* D */ \
    {1, 1, 1, 25, 25, 10, 40, 2, 1, 25, 2, 25, 1, 9, 17, 40, 40, 27, 9, 9, 40, 17, 25, 25, 3, 40, 1, 17, 1, 2, 1, 2, 17, 1, 25, 1, 33}, /* E */ \
    {25, 25, 1, 33, 25, 17, 17, 3, 2, 2, 1, 18, 26, 1, 25, 1, 1, 10, 40, 1, 10, 34, 40, 40, 11, 2, 1, 10, 40, 9, 9, 1, 25, 9, 9, 25, 25}, /* F */ \
    {1, 1, 1, 25, 25, 9, 40, 2, 1, 25, 1, 25, 1, 9, 17, 40, 40, 27, 9, 9, 40, 17, 25, 25, 3, 40, 1, 17, 1, 2, 1, 2, 17, 1, 25, 1, 33}, /* G */ \
    {2, 2, 2, 1, 2, 1, 1, 1, 10, 2, 1, 17, 17, 9, 10, 1, 1, 17, 18, 17, 9, 10, 17, 18, 18, 17, 9, 10, 18, 40, 18, 9, 10, 19, 18, 17, 9}, /* H */ \
    {2, 2, 2, 1, 2, 1, 1, 1, 10, 2, 1, 17, 17, 9, 10, 1, 1, 17, 18, 17, 9, 10, 17, 18, 18, 17, 9, 10, 18, 40, 18, 9, 10, 19, 18, 17, 9}, /* I */ \
    {17, 17, 17, 26, 17, 18, 18, 40, 25, 17, 18, 1, 1, 26, 25, 17, 17, 3, 33, 1, 26, 25, 9, 10, 1, 2, 26, 25, 9, 40, 10, 9, 26, 9, 9, 9, 9}, /* J */ \
    {2, 2, 2, 1, 1, 1, 1, 1, 2, 1, 2, 3, 3, 11, 2, 33, 1, 1, 1, 1, 1, 33, 2, 20, 3, 3, 2, 1, 2, 1, 1, 1, 1, 1, 2, 2, 2}, /* K */ \
    {2, 2, 1, 3, 1, 1, 1, 3, 33, 1, 2, 40, 3, 9, 33, 40, 1, 1, 1, 1, 9, 9, 1, 18, 2, 40, 1, 1, 2, 33, 2, 1, 2, 2, 18, 1, 2}, /* L */ \
    {33, 1, 1, 1, 12, 40, 40, 20, 1, 40, 9, 1, 1, 18, 1, 40, 1, 1, 26, 1, 1, 40, 1, 26, 40, 40, 40, 40, 1, 26, 1, 1, 1, 1, 1, 9, 9}, /* M */ \
    {17, 9, 9, 1, 17, 18, 9, 1, 1, 1, 18, 19, 9, 2, 1, 1, 1, 1, 20, 1, 1, 1, 1, 2, 9, 19, 18, 17, 1, 1, 9, 9, 17, 1, 1, 9, 9}, /* N */ \
    {18, 2, 17, 17, 18, 17, 40, 40, 12, 40, 17, 17, 1, 2, 1, 17, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, /* O */ \
    {11, 10, 9, 10, 11, 1, 9, 9, 9, 9, 25, 9, 26, 11, 2, 9, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, /* P */ \
    {1, 27, 1, 1, 10, 2, 25, 2, 19, 9, 2, 25, 17, 17, 9, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, /* Q */ \
    {1, 1, 40, 17, 17, 1, 3, 40, 17, 33, 17, 1, 1, 40, 17, 17, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, /* R */ \
    {73, 73, 73, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, /* END1 */ \
    {65, 65, 65, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, /* END2 */ \
}

/* doubled coordinates of the three piece footprints */
#define COG_LARGE_XY2 { \
    {0,-6},{2,-6},{4,-6},{6,-6},{-2,-4},{0,-4},{2,-4},{4,-4},{6,-4},{-4,-2},{-2,-2},{0,-2},{2,-2}, \
    {4,-2},{6,-2},{-6,0},{-4,0},{-2,0},{0,0},{2,0},{4,0},{6,0},{-6,2},{-4,2},{-2,2},{0,2},{2,2}, \
    {4,2},{-6,4},{-4,4},{-2,4},{0,4},{2,4},{-6,6},{-4,6},{-2,6},{0,6} }
#define COG_SMALL_XY2 { \
    {-3,-2},{-1,-2},{1,-2},{3,-2},{5,-2},{-5,0},{-3,0},{-1,0},{1,0},{3,0},{5,0},{-5,2},{-3,2}, \
    {-1,2},{1,2},{3,2} }
#define COG_END_XY2 { {0,0},{2,0},{-2,2} }

/* connection reference points (map.cpp:203-263), doubled coords.
 * LARGE->LARGE : 2 coords, rotation options -2..3   (+6 rotated copies)
 * LARGE->SMALL : 3 coords, options {-1, 2}         (+6 rotated copies)
 * LARGE(non-start)->TRIPLE : 1 coord, option {-3}  (+6 rotated copies)
 * SMALL->LARGE : 6 coords, options -2..3           (no copies)                           */
#define COG_CONN_LL_XY2 { {8,6},{6,8} }
#define COG_CONN_LS_XY2 { {3,7},{5,5},{7,3} }
#define COG_CONN_LT_XY2 { {0,8} }
#define COG_CONN_SL_XY2 { {-7,10},{-5,10},{-3,10},{7,-10},{5,-10},{3,-10} }

#define COG_DIRS_XY2 { {0,0},{2,0},{0,2},{-2,2},{-2,0},{0,-2},{2,-2} }  /* geometry.h:42-50 */

#endif
