// pyrepr.h -- Python's float repr and round(x, 3), and int formatting, for
// the GPU response writer (responses.hip) and its host-side checks.
//
// json.dumps writes a float with float.__repr__: the shortest digit string
// that reads back to the same double, the closest such string to the exact
// value (David Gay's dtoa, mode 0), in fixed notation when the decimal point
// falls in (-4, 16] (reporter_service.py's response bodies, report.cpp
// json::put_float on the host).  Here: Burger & Dybvig's free-format digit
// generation in exact integers (64-bit when they fit, else 128-bit), for |d| in [2^-10, 2^52) and
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

// A byte sink is any type with put(char) and put8(w, m) (m <= 8 bytes of w,
// byte 0 first).  CharSink: a plain buffer.
struct CharSink {
  char* p;
  int n;
  OTM_HD void put(char c) { p[n++] = c; }
  OTM_HD void put8(uint64_t w, int m) {  // m <= 8 bytes of w, byte 0 first
    for (int j = 0; j < m; ++j) p[n++] = (char)(uint8_t)(w >> (8 * j));
  }
};

// up to 16 decimal digits of v (at least minw, zero-padded), most significant
// first: built in a 128-bit string register (each new, less significant...
// digit shifted in below: byte 0 ends up the first character), so no
// digit array is indexed at run time
template <class S>
OTM_HD void put_digits16(uint64_t v, int minw, S& o) {
  u128 str = 0;
  int n = 0;
  do {
    str = (str << 8) | (u128)('0' + (unsigned)(v % 10u));
    v /= 10u;
    ++n;
  } while (v || n < minw);
  // (a sink takes up to 8 bytes at once: put8)
  o.put8((uint64_t)str, n < 8 ? n : 8);
  if (n > 8) o.put8((uint64_t)(str >> 64), n - 8);
}

template <class S>
OTM_HD void put_u64(uint64_t v, S& o) {
  constexpr uint64_t P16 = 10000000000000000ull;
  if (v >= P16) {
    put_digits16(v / P16, 0, o);
    put_digits16(v % P16, 16, o);
  } else {
    put_digits16(v, 0, o);
  }
}

template <class S>
OTM_HD void put_i64(int64_t v, S& o) {
  if (v < 0) {
    o.put('-');
    put_u64((uint64_t)0 - (uint64_t)v, o);
  } else {
    put_u64((uint64_t)v, o);
  }
}

OTM_HD int put_i64(int64_t v, char* o) {
  CharSink s{o, 0};
  put_i64(v, s);
  return s.n;
}

OTM_HD uint64_t pow10_64(int k) {  // (k <= 19)
  uint64_t p = 1;
  for (int i = 0; i < k; ++i) p *= 10u;
  return p;
}

// Burger & Dybvig's digit generation from the scaled state (value r / s in
// [0.1, 1) x 10^decpt, half-gaps mp / mm): T = uint64_t when every quantity
// the loop forms stays below 2^64 (the caller checks s < 2^60: r < s, mp < 10 s
// and mm <= mp, so 10 r and r + mp stay below 11 s), else u128 -- the same
// exact arithmetic either way, so the same digits
template <class T, class S>
OTM_HD bool repr_digits(T r, T s, T mp, T mm, bool incl, int decpt, S& o) {
  // digits: 0.D1 D2 ... x 10^decpt, each written as it is fixed, in Python's
  // repr layout (fixed notation for -4 < decpt <= 16: always, in this range)
  if (decpt <= 0) {
    o.put('0');
    o.put('.');
    for (int i = 0; i < -decpt; ++i) o.put('0');
  }
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
    const bool last = lo || hi;
    if (lo && hi) {
      const T r2 = r << 1;
      // closer of the two; exactly half-way: the even digit (dtoa's
      // round-half-even on the last digit)
      if (r2 > s || (r2 == s && (dig & 1))) ++dig;
    } else if (hi) {
      ++dig;
    }
    // (dig == 10 cannot happen: the high test stops a digit earlier)
    if (nd == 17) return false;
    if (decpt > 0 && nd == decpt) o.put('.');
    o.put((char)('0' + dig));
    ++nd;
    if (last) break;
  }
  if (decpt > 0 && nd <= decpt) {
    for (int i = nd; i < decpt; ++i) o.put('0');
    o.put('.');
    o.put('0');
  }
  return true;
}

// repr(d) into the sink (at most 24 bytes); false: d is outside the range
// (the sink may hold part of it; the host writes that body)
template <class S>
OTM_HD bool py_repr(double d, S& o) {
  const uint64_t b = dbits(d);
  const bool neg = (b >> 63) != 0;
  const int ef = (int)((b >> 52) & 0x7FF);
  const uint64_t fr = b & ((1ull << 52) - 1);
  if (ef == 0 && fr == 0) {
    if (neg) o.put('-');
    o.put('0');
    o.put('.');
    o.put('0');
    return true;
  }
  // d = M x 2^e2; supported: 2^-10 <= |d| < 2^52
  const int e2 = ef - 1075;
  if (ef == 0 || e2 >= 0 || e2 < -62) return false;
  if (neg) o.put('-');
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
      s *= pow10_64(k);
    } else {
      const uint64_t p = pow10_64(-k);
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
  if ((s >> 60) == 0)
    return repr_digits<uint64_t>((uint64_t)r, (uint64_t)s, (uint64_t)mp, (uint64_t)mm, incl, k, o);
  return repr_digits<u128>(r, s, mp, mm, incl, k, o);
}

OTM_HD int py_repr(double d, char* o) {
  CharSink s{o, 0};
  return py_repr(d, s) ? s.n : -1;
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
