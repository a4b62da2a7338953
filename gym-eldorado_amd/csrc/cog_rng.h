// cog_rng.h -- the reference's random numbers: std::default_random_engine (libstdc++ =
// minstd_rand0) and uniform_int_distribution<size_t>(0, k-1) downscaling (uses at
// sampler.h:25-75, cards.cpp:190-191, player.cpp:92-93,115-116, map.cpp:298-301,705-734).
//
// Plain integer code shared by the kernels and a host-side exhaustive test
// (tests/test_rng_cpu.py builds it with g++ after defining COG_HD).
#pragma once
#include <stdint.h>

#ifndef COG_HD
#define COG_HD __host__ __device__ __forceinline__
#endif

namespace cog {

// libstdc++'s uniform_int_distribution over minstd_rand0: __urngrange = max - min = 2^31 - 3
constexpr uint32_t kUrngRange = 2147483645u;

COG_HD uint32_t mr_seed(uint64_t s) {
  const uint32_t x = (uint32_t)(s % 2147483647ull);
  return x == 0 ? 1u : x;
}
COG_HD uint32_t mr_next(uint32_t &x) {                     // x <- 16807 x mod (2^31 - 1)
  const uint64_t p = (uint64_t)x * 16807u;                 // < 2^46
  uint32_t r = (uint32_t)(p & 0x7fffffffu) + (uint32_t)(p >> 31);
  r = r >= 0x7fffffffu ? r - 0x7fffffffu : r;
  x = r;
  return r;
}

// uniform integer in [0, k-1], k >= 1, exactly as libstdc++ computes it:
//   scaling = range / k; past = k * scaling; do r = urng() - 1 while r >= past; return r / scaling
COG_HD uint32_t uid(uint32_t &x, uint32_t k) {
  const uint32_t scaling = kUrngRange / k;
  const uint32_t past = k * scaling;
  uint32_t r;
  do {
    r = mr_next(x) - 1u;
  } while (r >= past);
  return r / scaling;
}

// The same value with one division instead of two.  With s = range / k (exact quotient
// s = (range - m) / k, m = range mod k) and an accepted r < k s:
//   r / s = r k / (range - m)  and  0 <= r k / (range - m) - r k / range < k^2 / range < 1
// for k < 2^15, so floor(r / s) is q = floor(r k / range) or q + 1, and it is q + 1 exactly
// when (q + 1) s <= r.  floor(x / range) for x < 2^47 is x >> 31 or one more: range = 2^31 - 3.
COG_HD uint32_t div_range(uint64_t x) {                    // floor(x / kUrngRange), x < 2^47
  const uint64_t y = x >> 31;
  return (uint32_t)y + (x + 3u * (y + 1u) >= ((y + 1u) << 31) ? 1u : 0u);
}
COG_HD uint32_t uid_fast(uint32_t &x, uint32_t k) {        // k in [1, 2^15)
  const uint32_t s = kUrngRange / k;
  const uint32_t past = k * s;
  uint32_t r = mr_next(x) - 1u;
  while (r >= past) r = mr_next(x) - 1u;                   // probability < k / 2^31 per draw
  const uint32_t q = div_range((uint64_t)r * k);
  return q + ((q + 1u) * s <= r ? 1u : 0u);
}

// Division-free for the sampler's heads (k <= 31): range mod k from a compile-time table of
// 5-bit residues, s = (range - m) / k never materialised:
//   reject  r >= k s = range - m;   q + 1 wins  <=>  (q + 1)(range - m) <= r k.
constexpr uint32_t range_mod(uint32_t k) { return kUrngRange % k; }
constexpr uint64_t residues5(uint32_t k0) {                // 12 residues of 5 bits: k0 .. k0 + 11
  uint64_t v = 0;
  for (uint32_t j = 0; j < 12; j++) v |= (uint64_t)(range_mod(k0 + j) & 31u) << (5 * j);
  return v;
}
constexpr uint64_t kRes5_1 = residues5(1), kRes5_13 = residues5(13), kRes5_25 = residues5(25);
COG_HD uint32_t small_past(uint32_t k) {                  // k * (range / k), k in [1, 31]
  const uint64_t tab = k < 13 ? kRes5_1 : (k < 25 ? kRes5_13 : kRes5_25);
  const uint32_t j = k < 13 ? k - 1u : (k < 25 ? k - 13u : k - 25u);
  return kUrngRange - ((uint32_t)(tab >> (5u * j)) & 31u);
}
COG_HD uint32_t small_mod(uint32_t k) {                    // range mod k, k in [1, 31]
  const uint64_t tab = k < 13 ? kRes5_1 : (k < 25 ? kRes5_13 : kRes5_25);
  const uint32_t j = k < 13 ? k - 1u : (k < 25 ? k - 13u : k - 25u);
  return (uint32_t)(tab >> (5u * j)) & 31u;
}
// r < small_past(k): the value, in 32-bit arithmetic after the one 64-bit product r k < 2^36.
// With r k = y 2^31 + l (l < 2^31) and range = 2^31 - 3: q0 = floor(r k / range) is y + c, where
// c = 1 exactly when l + 3 y + 3 >= 2^31, and the remainder is l + 3 y - 3 c (mod 2^31).  Then
// (q0 + 1)(range - m) <= r k  <=>  rem + (q0 + 1) m >= range  (m = range mod k <= 30).
COG_HD uint32_t uid_small_accepted(uint32_t r, uint32_t k) {
  const uint64_t rk = (uint64_t)r * k;
  const uint32_t lo = (uint32_t)rk, l = lo & 0x7fffffffu;
  const uint32_t y = (uint32_t)(rk >> 31);                 // <= 31
  const uint32_t S = l + 3u * y + 3u;                      // < 2^31 + 96
  const uint32_t c = S >> 31;
  const uint32_t q0 = y + c;
  const uint32_t rem = S - (c ? 0x80000000u : 3u);
  return q0 + (rem + (q0 + 1u) * small_mod(k) >= kUrngRange ? 1u : 0u);
}
COG_HD uint32_t uid_small(uint32_t &x, uint32_t k) {       // k in [1, 31]
  const uint32_t past = small_past(k);
  uint32_t r = mr_next(x) - 1u;
  while (r >= past) r = mr_next(x) - 1u;
  return uid_small_accepted(r, k);
}
// every draw a k in [1, 31] can reject has r >= range - 30 (range mod k <= 30)
constexpr uint32_t kSmallSafe = kUrngRange - 31u;

// Table form for k in [1, 31] (the kernels keep the table in LDS): entry k = {s, m} with
// s = range / k and m = floor(2^32 / s).  For an accepted r (< k s < 2^31) the quotient r / s is
// q' = mulhi(r, m) or q' + 1: r m / 2^32 > r / s - r / 2^32 > r / s - 1/2, so q' >= r / s - 1;
// and r - q' s < 2 s < 2^32, so the correction is one exact 32-bit compare.
struct UidEntry {
  uint32_t s, m;
};
constexpr UidEntry uid_entry(uint32_t k) {
  return k == 0 ? UidEntry{1u, 0u} : UidEntry{kUrngRange / k, (uint32_t)((1ull << 32) / (kUrngRange / k))};
}
constexpr int kUidTab = 32;                                // k = 0 .. 31
COG_HD uint32_t uid_tab_accepted(uint32_t r, uint32_t s, uint32_t m) {
  const uint32_t q = (uint32_t)(((uint64_t)r * m) >> 32);
  return q + (r - q * s >= s ? 1u : 0u);
}

// Jump-ahead: the state j steps on is x * 16807^j mod (2^31 - 1), so the states of several
// consecutive draws are independent products instead of a serial chain.
constexpr uint32_t kMinstdM = 0x7fffffffu;
constexpr uint32_t mr_pow(uint32_t j) {
  uint64_t v = 1;
  for (uint32_t i = 0; i < j; i++) v = v * 16807u % kMinstdM;
  return (uint32_t)v;
}
COG_HD uint32_t mr_jump(uint32_t x, uint32_t c) {          // x * c mod (2^31 - 1), x, c < 2^31
  const uint64_t p = (uint64_t)x * c;                      // < 2^62
  const uint32_t s = (uint32_t)(p & kMinstdM) + (uint32_t)(p >> 31);   // <= 2^32 - 2
  const uint32_t r = (s & kMinstdM) + (s >> 31);          // <= 2^31
  return r >= kMinstdM ? r - kMinstdM : r;
}

}  // namespace cog
