// pyrepr.h -- Python's float repr and round(x, 3), and int formatting, for
// the GPU response writer (responses.hip) and its host-side checks.
//
// json.dumps writes a float with float.__repr__: the shortest digit string
// that reads back to the same double, the closest such string to the exact
// value (David Gay's dtoa, mode 0), in fixed notation when the decimal point
// falls in (-4, 16] (reporter_service.py's response bodies, report.cpp
// json::put_float on the host).  Here: Burger & Dybvig's free-format digit
// generation with exact 128-bit integer state, for |d| in [2^-10, 2^52) and
// 0.0, which covers every float a /report body holds (epoch times, lengths in
// km); outside that range py_repr returns -1 and the caller leaves the body to
// the host writer.  tests/test_pyrepr.py pins it against Python's repr.
#pragma once
#include <cstdint>

#if defined(__HIPCC__)
#define OTM_HD __host__ __device__ __forceinline__
#else
#define OTM_HD inline
#endif

namespace otm {
namespace pyrepr {

typedef unsigned __int128 u128;

OTM_HD uint64_t dbits(double d) {
  union {
    double d;
    uint64_t u;
  } x;
  x.d = d;
  return x.u;
}

OTM_HD int put_u64(uint64_t v, char* o) {
  char t[20];
  int n = 0;
  do {
    t[n++] = (char)('0' + v % 10u);
    v /= 10u;
  } while (v);
  for (int k = 0; k < n; ++k) o[k] = t[n - 1 - k];
  return n;
}

OTM_HD int put_i64(int64_t v, char* o) {
  if (v < 0) {
    o[0] = '-';
    return 1 + put_u64((uint64_t)0 - (uint64_t)v, o + 1);
  }
  return put_u64((uint64_t)v, o);
}

OTM_HD u128 pow10u(int k) {
  u128 p = 1;
  for (int i = 0; i < k; ++i) p *= 10u;
  return p;
}

// repr(d) into o (at most 24 bytes); returns the length, or -1 (the host's)
OTM_HD int py_repr(double d, char* o) {
  const uint64_t b = dbits(d);
  const bool neg = (b >> 63) != 0;
  const int ef = (int)((b >> 52) & 0x7FF);
  const uint64_t fr = b & ((1ull << 52) - 1);
  int n = 0;
  if (neg) o[n++] = '-';
  if (ef == 0 && fr == 0) {
    o[n++] = '0';
    o[n++] = '.';
    o[n++] = '0';
    return n;
  }
  // d = M x 2^e2; supported: 2^-10 <= |d| < 2^52
  const int e2 = ef - 1075;
  if (ef == 0 || e2 >= 0 || e2 < -62) return -1;
  const uint64_t M = fr | (1ull << 52);
  // Burger & Dybvig: value r/s, neighbours' half-gaps mm/mp (all scaled)
  u128 r, s, mp, mm;
  if (fr != 0) {
    r = (u128)M << 1;
    s = (u128)1 << (1 - e2);
    mp = 1;
    mm = 1;
  } else {  // a power of two: the gap below is half the gap above
    r = (u128)M << 2;
    s = (u128)1 << (2 - e2);
    mp = 2;
    mm = 1;
  }
  const bool incl = (M & 1u) == 0;  // round-half-even reading: the ends belong when M is even
  // k = the decimal exponent: 10^(k-1) <= value < 10^k (value = r / s)
  int k = 0;
  {
    // estimate from the binary exponent, then correct exactly
    const int lg = (52 + e2);  // floor(log2 |d|)
    k = (int)((double)lg * 0.30102999566398120) + 1;  // close to ceil(log10)
    // scale to r/s in [0.1, 1) x 10^k: s x 10^k when k > 0, r x 10^-k when k < 0
    if (k >= 0) {
      s *= pow10u(k);
    } else {
      const u128 p = pow10u(-k);
      r *= p;
      mp *= p;
      mm *= p;
    }
    // fixups: r + mp >= s (or >) means the value reaches 10^k: one more digit place
    while (incl ? (r + mp >= s) : (r + mp > s)) {
      s *= 10u;
      ++k;
    }
    while (true) {
      const u128 r10 = r * 10u, mp10 = mp * 10u;
      if (incl ? (r10 + mp10 < s) : (r10 + mp10 <= s)) {
        r = r10;
        mp = mp10;
        mm *= 10u;
        --k;
      } else {
        break;
      }
    }
  }
  // digits: 0.D1 D2 ... x 10^k
  char dg[20];
  int nd = 0;
  while (true) {
    r *= 10u;
    mp *= 10u;
    mm *= 10u;
    int dig = 0;
    while (r >= s) {
      r -= s;
      ++dig;
    }
    const bool lo = incl ? (r <= mm) : (r < mm);
    const bool hi = incl ? (r + mp >= s) : (r + mp > s);
    if (!lo && !hi) {
      dg[nd++] = (char)('0' + dig);
      if (nd > 17) return -1;
      continue;
    }
    if (lo && hi) {
      const u128 r2 = r << 1;
      // closer of the two; exactly half-way: the even digit (dtoa's
      // round-half-even on the last digit)
      if (r2 > s || (r2 == s && (dig & 1))) ++dig;
    } else if (hi) {
      ++dig;
    }
    // (dig == 10 cannot happen: the high test stops a digit earlier)
    dg[nd++] = (char)('0' + dig);
    break;
  }
  if (nd > 17) return -1;
  // Python repr layout (fixed for -4 < k <= 16: always, in this range)
  const int decpt = k;
  if (decpt <= 0) {
    o[n++] = '0';
    o[n++] = '.';
    for (int i = 0; i < -decpt; ++i) o[n++] = '0';
    for (int i = 0; i < nd; ++i) o[n++] = dg[i];
  } else if (decpt >= nd) {
    for (int i = 0; i < nd; ++i) o[n++] = dg[i];
    for (int i = nd; i < decpt; ++i) o[n++] = '0';
    o[n++] = '.';
    o[n++] = '0';
  } else {
    for (int i = 0; i < decpt; ++i) o[n++] = dg[i];
    o[n++] = '.';
    for (int i = decpt; i < nd; ++i) o[n++] = dg[i];
  }
  return n;
}

// py_round3 (report.cpp / json.cpp): x rounded half-even to 3 decimals on its
// exact binary value (snprintf "%.3f"), read back correctly rounded: the
// integer R = round(x * 1000) over 1000.0 (exact operands: one IEEE division).
// Returns false where that needs more than 64-bit state (|x| >= 2^43).
OTM_HD bool py_round3(double x, double* out) {
  const uint64_t b = dbits(x);
  const bool neg = (b >> 63) != 0;
  const int ef = (int)((b >> 52) & 0x7FF);
  const uint64_t fr = b & ((1ull << 52) - 1);
  if (ef == 0x7FF) return false;
  if (ef == 0 && fr == 0) {
    *out = x;
    return true;
  }
  const uint64_t M = ef ? (fr | (1ull << 52)) : fr;
  const int e2 = (ef ? ef : 1) - 1075;
  if (e2 > -10) return false;  // |x| >= 2^43: not in a response
  const int sh = -e2;
  uint64_t R;
  if (sh >= 64 + 10) {
    R = 0;  // x * 1000 < 2^63 x 1024 / 2^74 < 0.5
  } else {
    const u128 t = (u128)M * 1000u;
    R = (uint64_t)(t >> sh);
    const u128 rem = t & (((u128)1 << sh) - 1u);
    const u128 half = (u128)1 << (sh - 1);
    if (rem > half || (rem == half && (R & 1u))) ++R;
  }
  const double v = (double)R / 1000.0;
  *out = neg ? -v : v;
  return true;
}

}  // namespace pyrepr
}  // namespace otm
