// formatter.cpp -- see formatter.h.
#include "formatter.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <thread>

#include "json.h"
#include "javastr.h"
#include "otmatch.h"

namespace otm {

namespace {

// ------------------------------------------------------------------ text
// One code point at s[i] (an invalid byte decodes as itself, length 1).
size_t decode_cp(std::string_view s, size_t i, uint32_t* cp) {
  const unsigned char c = (unsigned char)s[i];
  if (c < 0x80) {
    *cp = c;
    return 1;
  }
  int n = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 0;
  if (n == 0 || i + (size_t)n > s.size()) {
    *cp = c;
    return 1;
  }
  uint32_t v = c & (0x7Fu >> n);
  for (int k = 1; k < n; ++k) {
    const unsigned char d = (unsigned char)s[i + (size_t)k];
    if ((d & 0xC0) != 0x80) {
      *cp = c;
      return 1;
    }
    v = (v << 6) | (d & 0x3F);
  }
  *cp = v;
  return (size_t)n;
}

// Kafka's StringDeserializer: new String(bytes, UTF_8) of JDK 8, malformed
// input replaced by U+FFFD (javastr.h).  Returns false (and leaves *out
// alone) when the bytes are already well-formed, the common case.
bool utf8_sanitize(std::string_view s, std::string* out) {
  if (json::utf8_error(s).empty()) return false;
  *out = jstr::utf8_encode(jstr::utf8_decode(s));
  return true;
}

// String.trim(): strip code units <= ' ' at both ends
std::string_view java_trim(std::string_view s) {
  size_t a = 0, b = s.size();
  while (a < b && (unsigned char)s[a] <= ' ') ++a;
  while (b > a && (unsigned char)s[b - 1] <= ' ') --b;
  return s.substr(a, b - a);
}

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// Character.digit(ch, 10) of a UTF-16 unit (JDK 8, Unicode 6.2): the BMP's
// decimal-digit blocks; -1 for anything else (supplementary digits arrive as
// surrogate halves, which are not digits)
int java_digit(uint32_t cp) {
  static const uint32_t kZero[] = {0x30,   0x660,  0x6F0,  0x7C0,  0x966,  0x9E6,  0xA66,  0xAE6,  0xB66,
                                   0xBE6,  0xC66,  0xCE6,  0xD66,  0xE50,  0xED0,  0xF20,  0x1040, 0x1090,
                                   0x17E0, 0x1810, 0x1946, 0x19D0, 0x1A80, 0x1A90, 0x1B50, 0x1BB0, 0x1C40,
                                   0x1C50, 0xA620, 0xA8D0, 0xA900, 0xA9D0, 0xAA50, 0xABF0, 0xFF10};
  if (cp < 0x30) return -1;
  if (cp <= 0x39) return (int)(cp - 0x30);
  if (cp > 0xFFFF) return -1;
  for (uint32_t z : kZero)
    if (cp >= z && cp <= z + 9) return (int)(cp - z);
  return -1;
}
inline bool is_hex(char c) { return is_digit(c) || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }

// Java narrowing conversions of a double (JLS 5.1.3)
int32_t java_d2i(double d) {
  if (std::isnan(d)) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}
int64_t java_d2l(double d) {
  if (std::isnan(d)) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}

bool java_parse_int(std::string_view s, int32_t* out) {
  int64_t v;
  if (!java_parse_long(s, &v) || v < INT32_MIN || v > INT32_MAX) return false;
  *out = (int32_t)v;
  return true;
}

}  // namespace

// ------------------------------------------------------- java.lang numbers
// Long.parseLong: optional sign, one or more digits (Character.digit), in range.
bool java_parse_long(std::string_view s, int64_t* out) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    if (s.size() == 1) return false;
    i = 1;
  }
  uint64_t v = 0;
  const uint64_t lim = neg ? (uint64_t)INT64_MAX + 1u : (uint64_t)INT64_MAX;
  while (i < s.size()) {
    uint32_t cp;
    i += decode_cp(s, i, &cp);
    const int dg = java_digit(cp);  // Character.digit(c, 10)
    if (dg < 0) return false;
    const uint64_t d = (uint64_t)dg;
    if (v > (lim - d) / 10u) return false;
    v = v * 10u + d;
  }
  *out = neg ? (int64_t)(0u - v) : (int64_t)v;
  return true;
}

// Double.parseDouble (FloatingDecimal.readJavaFormatString): trimmed;
// optional sign; NaN | Infinity | hex (0x..p..) | decimal with at least one
// digit and an optional exponent; an optional f/F/d/D suffix.  The value is
// the correctly rounded double, which is what strtod returns for the same text.
bool java_parse_double(std::string_view in, double* out) {
  std::string_view s = java_trim(in);
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    ++i;
  }
  if (i >= s.size()) return false;
  if (s[i] == 'N') {
    if (s.substr(i) != "NaN") return false;
    *out = std::numeric_limits<double>::quiet_NaN();
    return true;
  }
  if (s[i] == 'I') {
    if (s.substr(i) != "Infinity") return false;
    *out = neg ? -INFINITY : INFINITY;
    return true;
  }
  std::string t(s.substr(0, i));
  if (s[i] == '0' && i + 1 < s.size() && (s[i + 1] == 'x' || s[i + 1] == 'X')) {
    // ([-+])?0[xX](((hex+)\.?)|((hex*)\.(hex+)))[pP]([-+])?(digit+)[fFdD]?
    size_t k = i + 2, nh = 0;
    while (k < s.size() && is_hex(s[k])) ++k, ++nh;
    size_t nf = 0;
    if (k < s.size() && s[k] == '.') {
      ++k;
      while (k < s.size() && is_hex(s[k])) ++k, ++nf;
    }
    if (nh + nf == 0) return false;
    if (k >= s.size() || (s[k] != 'p' && s[k] != 'P')) return false;
    ++k;
    if (k < s.size() && (s[k] == '+' || s[k] == '-')) ++k;
    size_t nd = 0;
    while (k < s.size() && is_digit(s[k])) ++k, ++nd;
    if (nd == 0) return false;
    const size_t body_end = k;
    if (k < s.size() && (s[k] == 'f' || s[k] == 'F' || s[k] == 'd' || s[k] == 'D')) ++k;
    if (k != s.size()) return false;
    t.append(s.substr(i, body_end - i));
    *out = std::strtod(t.c_str(), nullptr);
    return true;
  }
  size_t k = i, nd = 0;
  bool dot = false;
  while (k < s.size() && (is_digit(s[k]) || s[k] == '.')) {
    if (s[k] == '.') {
      if (dot) return false;  // multiple points
      dot = true;
    } else {
      ++nd;
    }
    ++k;
  }
  if (nd == 0) return false;
  if (k < s.size() && (s[k] == 'e' || s[k] == 'E')) {
    ++k;
    if (k < s.size() && (s[k] == '+' || s[k] == '-')) ++k;
    size_t ne = 0;
    while (k < s.size() && is_digit(s[k])) ++k, ++ne;
    if (ne == 0) return false;
  }
  const size_t body_end = k;
  if (k < s.size()) {
    if (k != s.size() - 1 || (s[k] != 'f' && s[k] != 'F' && s[k] != 'd' && s[k] != 'D')) return false;
  }
  t.append(s.substr(i, body_end - i));
  *out = std::strtod(t.c_str(), nullptr);
  return true;
}

// Double.toString: NaN / Infinity / -Infinity; 10^-3 <= |d| < 10^7 as plain
// decimal with at least one fraction digit, otherwise d.dddE<exp>.  Digits:
// the shortest that round-trip, nearest to the value, and at least two
// candidates' worth when one digit would do (the JDK >= 19 specification;
// JDK 8 occasionally printed one more digit).
void java_double_to_string(double d, std::string* out) {
  if (std::isnan(d)) {
    out->append("NaN");
    return;
  }
  if (std::isinf(d)) {
    out->append(d < 0 ? "-Infinity" : "Infinity");
    return;
  }
  if (d == 0.0) {
    out->append(std::signbit(d) ? "-0.0" : "0.0");
    return;
  }
  char buf[40];
  int prec = 1;
  for (; prec <= 17; ++prec) {
    std::snprintf(buf, sizeof buf, "%.*e", prec - 1, d);
    if (std::strtod(buf, nullptr) == d) break;
  }
  // a one-digit shortest form competes with the two-digit decimals: the
  // closest wins (4.9E-324, not 5E-324)
  if (prec == 1) std::snprintf(buf, sizeof buf, "%.1e", d);
  // buf = [-]D[.DDD]e[+-]XX
  std::string digits;
  const char* p = buf;
  const bool neg = *p == '-';
  if (neg) ++p;
  for (; *p && *p != 'e'; ++p)
    if (is_digit(*p)) digits.push_back(*p);
  const int x = std::atoi(p + 1);  // value = D.DDD x 10^x
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  if (neg) out->push_back('-');
  const double a = std::fabs(d);
  if (a >= 1e-3 && a < 1e7) {
    if (x >= 0) {
      const size_t ip = (size_t)x + 1;
      for (size_t k = 0; k < ip; ++k) out->push_back(k < digits.size() ? digits[k] : '0');
      out->push_back('.');
      if (digits.size() > ip) out->append(digits.substr(ip));
      else out->push_back('0');
    } else {
      out->append("0.");
      out->append((size_t)(-x - 1), '0');
      out->append(digits);
    }
  } else {
    out->push_back(digits[0]);
    out->push_back('.');
    if (digits.size() > 1) out->append(digits.substr(1));
    else out->push_back('0');
    out->push_back('E');
    out->append(std::to_string(x));
  }
}

// DecimalFormat("###.######", DecimalFormatSymbols(Locale.US)).parse(text)
// .floatValue(), JDK 8 (DecimalFormat.parse / subparse, DigitList):
//  * NaN symbol "�" first; then prefix "" or "-" (longest); the
//    infinity symbol "∞";
//  * digits (Character.digit: any BMP decimal digit; leading zeros skipped),
//    one '.', grouping ',' skipped
//    before the point (grouping stays enabled for this pattern), exponent
//    "E" with an optional '-' (no '+': then the number ends before the 'E');
//    parsing stops at the first other character -- a prefix parse;
//  * at least one digit, else ParseException;
//  * a value that fits a long (no fraction, |v| <= 2^63, negative zero
//    excepted) is a Long and floatValue() rounds the integer once; anything
//    else is Double.parseDouble(".DIGITS E decimalAt") narrowed to float.
bool decimal_format_parse(std::string_view t, float* out) {
  static const char kNaN[] = "\xEF\xBF\xBD", kInf[] = "\xE2\x88\x9E";
  if (t.substr(0, 3) == std::string_view(kNaN, 3)) {
    *out = std::numeric_limits<float>::quiet_NaN();
    return true;
  }
  size_t i = 0;
  bool neg = false;
  if (!t.empty() && t[0] == '-') {
    neg = true;
    i = 1;
  }
  if (t.substr(i, 3) == std::string_view(kInf, 3)) {
    *out = neg ? -INFINITY : INFINITY;
    return true;
  }
  std::string digits;  // significant digits
  int32_t decimal_at = 0, digit_count = 0, exponent = 0;
  bool saw_decimal = false, saw_digit = false;
  for (size_t step = 0; i < t.size(); i += step) {
    uint32_t cp;
    step = decode_cp(t, i, &cp);
    const int dg = java_digit(cp);
    const char ch = cp < 0x80 ? (char)cp : '\x7f';
    if (dg == 0) {
      saw_digit = true;
      if (digits.empty()) {
        if (saw_decimal) decimal_at = (int32_t)((uint32_t)decimal_at - 1u);
        continue;
      }
      ++digit_count;
      digits.push_back('0');
    } else if (dg > 0) {
      saw_digit = true;
      ++digit_count;
      digits.push_back((char)('0' + dg));
    } else if (ch == '.') {
      if (saw_decimal) break;
      decimal_at = digit_count;
      saw_decimal = true;
    } else if (ch == ',') {
      if (saw_decimal) break;
    } else if (ch == 'E') {
      // the exponent: prefix "" / "-", digits only; applied when it parses
      // and fits a long, (int)-narrowed
      size_t k = i + 1;
      bool eneg = false;
      if (k < t.size() && t[k] == '-') {
        eneg = true;
        ++k;
      }
      std::string ed;
      bool esaw = false;
      while (k < t.size()) {
        uint32_t ec;
        const size_t l = decode_cp(t, k, &ec);
        const int ev = java_digit(ec);
        if (ev < 0) break;
        k += l;
        esaw = true;
        if (ed.empty() && ev == 0) continue;
        ed.push_back((char)('0' + ev));
      }
      if (esaw) {
        // fitsIntoLong(positive, ignoreNegativeZero = true)
        bool fits = ed.size() < 19 || (ed.size() == 19 && (ed < "9223372036854775808" ||
                                                           (eneg && ed == "9223372036854775808")));
        if (fits) {
          uint64_t v = 0;
          for (char c : ed) v = v * 10u + (uint64_t)(c - '0');
          if (eneg) v = 0u - v;
          exponent = (int32_t)(uint32_t)v;
        }
      }
      break;
    } else {
      break;
    }
  }
  if (!saw_decimal) decimal_at = digit_count;
  decimal_at = (int32_t)((uint32_t)decimal_at + (uint32_t)exponent);
  if (!saw_digit && digit_count == 0) return false;
  while (!digits.empty() && digits.back() == '0') digits.pop_back();
  if (digits.empty()) {  // zero: Long 0, or Double -0.0 when negative
    *out = neg ? -0.0f : 0.0f;
    return true;
  }
  const int32_t count = (int32_t)digits.size();
  bool fits = false;
  if (!(decimal_at < count || decimal_at > 19)) {
    if (decimal_at < 19) {
      fits = true;
    } else {
      static const char kMin[] = "9223372036854775808";
      int cmp = 0;
      for (int32_t k = 0; k < count && cmp == 0; ++k) cmp = digits[(size_t)k] < kMin[k] ? -1 : digits[(size_t)k] > kMin[k] ? 1 : 0;
      fits = cmp < 0 || (cmp == 0 && (count < decimal_at || neg));
    }
  }
  if (fits) {
    uint64_t v = 0;
    for (int32_t k = 0; k < decimal_at; ++k) v = v * 10u + (uint64_t)(k < count ? digits[(size_t)k] - '0' : 0);
    const int64_t sv = neg ? (int64_t)(0u - v) : (int64_t)v;
    *out = (float)sv;
    return true;
  }
  std::string s = neg ? "-0." : "0.";
  s += digits;
  s += 'e';
  s += std::to_string(decimal_at);
  *out = (float)std::strtod(s.c_str(), nullptr);
  return true;
}

// ------------------------------------------------- java.util.regex subset
struct Formatter::Re {
  struct Item {
    bool cls = false;  // literal code point or class
    uint32_t cp = 0;
    bool neg = false;
    std::vector<std::pair<uint32_t, uint32_t>> ranges;
    int lo = 1, hi = 1;  // quantifier, hi < 0 = unbounded
    bool match(uint32_t c) const {
      if (!cls) return c == cp;
      bool in = false;
      for (const auto& r : ranges)
        if (c >= r.first && c <= r.second) {
          in = true;
          break;
        }
      return in != neg;
    }
  };
  std::vector<Item> items;

  static void predefined(char e, Item* it) {
    it->cls = true;
    switch (e) {
      case 'd': case 'D': it->ranges = {{'0', '9'}}; break;
      case 's': case 'S': it->ranges = {{' ', ' '}, {'\t', '\r'}}; break;  // [ \t\n\x0B\f\r]
      case 'w': case 'W': it->ranges = {{'a', 'z'}, {'A', 'Z'}, {'_', '_'}, {'0', '9'}}; break;
    }
    it->neg = e == 'D' || e == 'S' || e == 'W';
  }
  // an escaped character outside the predefined classes; false if unsupported
  static bool escape(std::string_view p, size_t* i, uint32_t* cp, std::string* err) {
    const char e = p[*i];
    ++*i;
    switch (e) {
      case 't': *cp = '\t'; return true;
      case 'n': *cp = '\n'; return true;
      case 'r': *cp = '\r'; return true;
      case 'f': *cp = '\f'; return true;
      case 'a': *cp = 7; return true;
      case 'e': *cp = 27; return true;
      case 'x':
      case 'u': {
        const size_t nd = e == 'x' ? 2 : 4;
        if (*i + nd > p.size()) break;
        uint32_t v = 0;
        for (size_t k = 0; k < nd; ++k) {
          const char h = p[*i + k];
          if (!is_hex(h)) {
            *err = "bad hex escape in separator regex";
            return false;
          }
          v = v * 16u + (uint32_t)(is_digit(h) ? h - '0' : (h | 0x20) - 'a' + 10);
        }
        *i += nd;
        *cp = v;
        return true;
      }
      default:
        if ((e >= 'a' && e <= 'z') || (e >= 'A' && e <= 'Z') || is_digit(e)) break;
        {
          size_t k = *i - 1;
          *i = k + decode_cp(p, k, cp);
        }
        return true;
    }
    *err = std::string("unsupported escape \\") + e + " in separator regex";
    return false;
  }

  bool compile(std::string_view p, std::string* err) {
    size_t i = 0;
    while (i < p.size()) {
      const char c = p[i];
      Item it;
      if (c == '\\') {
        if (i + 1 >= p.size()) {
          *err = "separator regex ends in a backslash";
          return false;
        }
        const char e = p[i + 1];
        if (e == 'd' || e == 'D' || e == 's' || e == 'S' || e == 'w' || e == 'W') {
          predefined(e, &it);
          i += 2;
        } else {
          ++i;
          if (!escape(p, &i, &it.cp, err)) return false;
        }
      } else if (c == '.') {
        it.cls = true;
        it.neg = true;
        it.ranges = {{'\n', '\n'}, {'\r', '\r'}, {0x85, 0x85}, {0x2028, 0x2029}};
        ++i;
      } else if (c == '[') {
        ++i;
        it.cls = true;
        if (i < p.size() && p[i] == '^') {
          it.neg = true;
          ++i;
        }
        bool first = true, closed = false;
        while (i < p.size()) {
          if (p[i] == ']' && !first) {
            closed = true;
            ++i;
            break;
          }
          if (p[i] == '[' || (p[i] == '&' && i + 1 < p.size() && p[i + 1] == '&') || (p[i] == ']' && first)) {
            *err = "unsupported character class in separator regex";
            return false;
          }
          first = false;
          uint32_t a;
          if (p[i] == '\\') {
            if (i + 1 >= p.size()) break;
            const char e = p[i + 1];
            if (e == 'd' || e == 's' || e == 'w') {
              Item tmp;
              predefined(e, &tmp);
              it.ranges.insert(it.ranges.end(), tmp.ranges.begin(), tmp.ranges.end());
              i += 2;
              continue;
            }
            ++i;
            if (!escape(p, &i, &a, err)) return false;
          } else {
            i += decode_cp(p, i, &a);
          }
          uint32_t b = a;
          if (i + 1 < p.size() && p[i] == '-' && p[i + 1] != ']') {
            ++i;
            if (p[i] == '\\') {
              ++i;
              if (i >= p.size() || !escape(p, &i, &b, err)) {
                if (err->empty()) *err = "bad class range in separator regex";
                return false;
              }
            } else {
              i += decode_cp(p, i, &b);
            }
            if (b < a) {
              *err = "illegal character range in separator regex";
              return false;
            }
          }
          it.ranges.push_back({a, b});
        }
        if (!closed) {
          *err = "unclosed character class in separator regex";
          return false;
        }
      } else if (c == '|' || c == '(' || c == ')' || c == '^' || c == '$' || c == '*' || c == '+' || c == '?' ||
                 c == '{') {
        *err = std::string("unsupported separator regex (metacharacter '") + c + "')";
        return false;
      } else {
        i += decode_cp(p, i, &it.cp);
      }
      // quantifier
      if (i < p.size()) {
        const char q = p[i];
        bool quantified = false;
        if (q == '*' || q == '+' || q == '?') {
          it.lo = q == '+' ? 1 : 0;
          it.hi = q == '?' ? 1 : -1;
          ++i;
          quantified = true;
        } else if (q == '{') {
          size_t k = i + 1;
          int lo = 0, hi;
          size_t nd = 0;
          while (k < p.size() && is_digit(p[k]) && nd < 6) lo = lo * 10 + (p[k++] - '0'), ++nd;
          if (nd == 0) {
            *err = "bad repetition in separator regex";
            return false;
          }
          hi = lo;
          if (k < p.size() && p[k] == ',') {
            ++k;
            if (k < p.size() && p[k] == '}') {
              hi = -1;
            } else {
              hi = 0;
              nd = 0;
              while (k < p.size() && is_digit(p[k]) && nd < 6) hi = hi * 10 + (p[k++] - '0'), ++nd;
              if (nd == 0 || hi < lo) {
                *err = "bad repetition in separator regex";
                return false;
              }
            }
          }
          if (k >= p.size() || p[k] != '}') {
            *err = "bad repetition in separator regex";
            return false;
          }
          it.lo = lo;
          it.hi = hi;
          i = k + 1;
          quantified = true;
        }
        if (quantified && i < p.size() && (p[i] == '?' || p[i] == '+')) {
          *err = "lazy / possessive quantifiers are not supported in the separator regex";
          return false;
        }
      }
      items.push_back(std::move(it));
    }
    bool empty_ok = true;
    for (const Item& it : items) empty_ok = empty_ok && it.lo == 0;
    if (empty_ok) {
      *err = "separator regex can match the empty string (zero-width splits are not supported)";
      return false;
    }
    return true;
  }

  // greedy with backtracking
  bool match_at(std::string_view t, size_t ii, size_t pos, size_t* end) const {
    if (ii == items.size()) {
      *end = pos;
      return true;
    }
    const Item& it = items[ii];
    size_t stack_ends[64];
    std::vector<size_t> heap_ends;
    size_t* ends = stack_ends;
    size_t cap = 64, k = 0;
    ends[k++] = pos;
    size_t p = pos;
    int n = 0;
    while ((it.hi < 0 || n < it.hi) && p < t.size()) {
      uint32_t c;
      const size_t l = decode_cp(t, p, &c);
      if (!it.match(c)) break;
      p += l;
      ++n;
      if (k == cap) {
        heap_ends.assign(ends, ends + k);
        heap_ends.resize(cap * 2);
        cap *= 2;
        ends = heap_ends.data();
      }
      ends[k++] = p;
    }
    for (int j = n; j >= it.lo; --j)
      if (match_at(t, ii + 1, ends[(size_t)j], end)) return true;
    return false;
  }
  bool find(std::string_view t, size_t from, size_t* s, size_t* e) const {
    for (size_t p = from; p <= t.size();) {
      if (match_at(t, 0, p, e)) {
        *s = p;
        return true;
      }
      if (p == t.size()) break;
      uint32_t c;
      p += decode_cp(t, p, &c);
    }
    return false;
  }
  // String.split(regex) = Pattern.split(input, 0)
  void split(std::string_view t, std::vector<std::string_view>* parts) const {
    parts->clear();
    if (items.size() == 1 && !items[0].cls && items[0].lo == 1 && items[0].hi == 1 && items[0].cp < 0x80) {
      // one ASCII literal: String.split's own fast path
      const char c = (char)items[0].cp;
      size_t index = 0;
      bool any = false;
      for (const char* p; (p = (const char*)std::memchr(t.data() + index, c, t.size() - index)) != nullptr;) {
        const size_t s = (size_t)(p - t.data());
        parts->push_back(t.substr(index, s - index));
        index = s + 1;
        any = true;
        if (index >= t.size()) break;
      }
      if (!any) {
        parts->assign(1, t);
        return;
      }
      parts->push_back(t.substr(index));
      while (!parts->empty() && parts->back().empty()) parts->pop_back();
      return;
    }
    size_t index = 0, s, e, from = 0;
    while (find(t, from, &s, &e)) {
      parts->push_back(t.substr(index, s - index));
      index = e;
      from = e;
    }
    if (index == 0) {
      parts->assign(1, t);
      return;
    }
    parts->push_back(t.substr(index));
    while (!parts->empty() && parts->back().empty()) parts->pop_back();
  }
};

bool java_split(std::string_view regex, std::string_view text, std::vector<std::string_view>* parts,
                std::string* err) {
  Formatter::Re re;
  if (!re.compile(regex, err)) return false;
  re.split(text, parts);
  return true;
}

// ------------------------------------------------------------ joda-time
namespace {

bool is_letter(char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }

bool numeric_token(const std::string& tok) {
  if (tok.empty() || !is_letter(tok[0])) return false;
  switch (tok[0]) {
    case 'c': case 'C': case 'x': case 'y': case 'Y': case 'd': case 'h': case 'H': case 'm': case 's': case 'S':
    case 'e': case 'D': case 'F': case 'w': case 'W': case 'k': case 'K':
      return true;
    case 'M':
      return tok.size() <= 2;
  }
  return false;
}

// DateTimeFormat.parsePatternTo / parseToken (joda-time 2.9.9)
bool compile_time_pattern(std::string_view pat, std::vector<Formatter::TimeTok>* out, std::string* err) {
  std::vector<std::string> toks;  // letter runs, or "'" + literal text
  size_t i = 0;
  while (i < pat.size()) {
    std::string buf;
    const char c = pat[i];
    if (is_letter(c)) {
      buf.push_back(c);
      while (i + 1 < pat.size() && pat[i + 1] == c) {
        buf.push_back(c);
        ++i;
      }
    } else {
      buf.push_back('\'');
      bool in_lit = false;
      for (; i < pat.size(); ++i) {
        const char d = pat[i];
        if (d == '\'') {
          if (i + 1 < pat.size() && pat[i + 1] == '\'') {
            ++i;
            buf.push_back(d);
          } else {
            in_lit = !in_lit;
          }
        } else if (!in_lit && is_letter(d)) {
          --i;
          break;
        } else {
          buf.push_back(d);
        }
      }
    }
    toks.push_back(buf);
    ++i;
  }
  for (size_t k = 0; k < toks.size(); ++k) {
    const std::string& tok = toks[k];
    Formatter::TimeTok t{};
    if (tok[0] == '\'') {
      t.field = 0;
      t.lit = tok.substr(1);
      if (!t.lit.empty()) out->push_back(t);
      continue;
    }
    const int n = (int)tok.size();
    const bool next_numeric = k + 1 < toks.size() && numeric_token(toks[k + 1]);
    t.len = n;
    switch (tok[0]) {
      case 'y':
        if (n == 2) {
          *err = "time pattern 'yy' (two-digit year, pivot on the current date) is not supported";
          return false;
        }
        t.field = 'y';
        t.max_digits = next_numeric ? n : 9;
        break;
      case 'M':
        if (n > 2) {
          *err = "time pattern: month names (MMM) are not supported";
          return false;
        }
        t.field = 'M';
        t.max_digits = 2;
        break;
      case 'd': case 'H': case 'm': case 's':
        t.field = tok[0];
        t.max_digits = 2;
        break;
      case 'S':
        t.field = 'S';
        t.max_digits = std::min(n, 18);
        break;
      default:
        *err = std::string("time pattern letter '") + tok[0] + "' is not supported";
        return false;
    }
    out->push_back(t);
  }
  return true;
}

int64_t days_from_civil(int64_t y, int m, int d) {  // proleptic Gregorian, ISO years
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const int64_t yoe = y - era * 400;
  const int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}
bool leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
int days_in_month(int64_t y, int m) {
  static const int dm[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  return m == 2 && leap(y) ? 29 : dm[m - 1];
}

char lower_ascii(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }

// DateTimeFormatter.parseDateTime(text).getMillis() / 1000 (withZoneUTC)
bool parse_time(const std::vector<Formatter::TimeTok>& fmt, std::string_view t, int64_t* secs) {
  struct Saved {
    int rank;
    int64_t v;
  };
  Saved saved[32];
  int ns = 0;
  size_t pos = 0;
  for (const Formatter::TimeTok& tk : fmt) {
    if (tk.field == 0) {  // literal, case-insensitive (CharacterLiteral / StringLiteral)
      if (pos + tk.lit.size() > t.size()) return false;
      for (size_t k = 0; k < tk.lit.size(); ++k)
        if (lower_ascii(t[pos + k]) != lower_ascii(tk.lit[k])) return false;
      pos += tk.lit.size();
      continue;
    }
    if (tk.field == 'S') {  // Fraction: millis of second, truncated
      const size_t limit = std::min((size_t)tk.max_digits, t.size() - pos);
      int64_t value = 0, n = 10000;
      size_t len = 0;
      while (len < limit && is_digit(t[pos + len])) {
        const int64_t nn = n / 10;
        value += (t[pos + len] - '0') * nn;
        n = nn;
        ++len;
      }
      value /= 10;
      if (len == 0) return false;
      pos += len;
      if (ns < 32) saved[ns++] = Saved{6, value};
      continue;
    }
    // NumberFormatter.parseInto (signed for the year)
    const bool is_signed = tk.field == 'y';
    size_t limit = std::min((size_t)tk.max_digits, t.size() - pos);
    size_t len = 0;
    bool negative = false, positive = false;
    while (len < limit) {
      const char c = t[pos + len];
      if (len == 0 && (c == '-' || c == '+') && is_signed) {
        if (len + 1 >= limit || !is_digit(t[pos + len + 1])) break;
        negative = c == '-';
        positive = c == '+';
        ++len;
        limit = std::min(limit + 1, t.size() - pos);
        continue;
      }
      if (!is_digit(c)) break;
      ++len;
    }
    if (len == 0) return false;
    int64_t v = 0;
    for (size_t k = (negative || positive) ? 1 : 0; k < len; ++k) v = v * 10 + (t[pos + k] - '0');
    if (v > INT32_MAX) return false;  // Integer.parseInt overflow
    if (negative) v = -v;
    pos += len;
    int rank = 0;
    switch (tk.field) {
      case 'y': rank = 0; break;
      case 'M': rank = 1; break;
      case 'd': rank = 2; break;
      case 'H': rank = 3; break;
      case 'm': rank = 4; break;
      case 's': rank = 5; break;
    }
    if (ns < 32) saved[ns++] = Saved{rank, v};
  }
  if (pos != t.size()) return false;
  // DateTimeParserBucket.computeMillis: fields largest first (stable), each
  // set with validation then floored; a month or day leading with no year
  // parses in the default year 2000
  std::stable_sort(saved, saved + ns, [](const Saved& a, const Saved& b) { return a.rank < b.rank; });
  int64_t y = 1970;
  int mo = 1, d = 1, H = 0, mi = 0, s = 0, ms = 0;
  if (ns > 0 && (saved[0].rank == 1 || saved[0].rank == 2)) y = 2000;
  for (int k = 0; k < ns; ++k) {
    const int64_t v = saved[k].v;
    switch (saved[k].rank) {
      case 0:
        if (v < -292275054 || v > 292278993) return false;
        y = v, mo = 1, d = 1, H = mi = s = ms = 0;
        break;
      case 1:
        if (v < 1 || v > 12) return false;
        mo = (int)v, d = 1, H = mi = s = ms = 0;
        break;
      case 2:
        if (v < 1 || v > days_in_month(y, mo)) return false;
        d = (int)v, H = mi = s = ms = 0;
        break;
      case 3:
        if (v < 0 || v > 23) return false;
        H = (int)v, mi = s = ms = 0;
        break;
      case 4:
        if (v < 0 || v > 59) return false;
        mi = (int)v, s = ms = 0;
        break;
      case 5:
        if (v < 0 || v > 59) return false;
        s = (int)v, ms = 0;
        break;
      case 6:
        if (v < 0 || v > 999) return false;
        ms = (int)v;
        break;
    }
  }
  const int64_t millis = days_from_civil(y, mo, d) * 86400000LL + (int64_t)H * 3600000 + (int64_t)mi * 60000 +
                         (int64_t)s * 1000 + ms;
  *secs = millis / 1000;  // Java long division truncates toward zero
  return true;
}

// ------------------------------------------------ Jackson JsonNode access
// DecimalFormat.parse(node.asText()).floatValue() without the text round
// trip for number nodes: Double.toString round-trips and DecimalFormat reads
// its "E" exponent, so a DoubleNode gives (float)d (Infinity's text does not
// parse); an IntNode's decimal fits a long, (float)(long); a BigIntegerNode's
// digits do not, so (float)Double.parseDouble(digits).  Other nodes go
// through their text.
bool node_float(const json::Value& v, float* out);
std::string as_text(const json::Value& v) {
  switch (v.kind) {
    case json::Kind::Str: return v.s;
    case json::Kind::Int: {
      if (v.bigint) return v.s;
      return std::to_string(v.i);
    }
    case json::Kind::Float: {
      std::string o;
      java_double_to_string(v.f, &o);
      return o;
    }
    case json::Kind::Bool: return v.b ? "true" : "false";
    case json::Kind::Null: return "null";
    default: return "";  // ContainerNode.asText()
  }
}

bool node_float(const json::Value& v, float* out) {
  if (v.kind == json::Kind::Float) {
    if (std::isinf(v.f) || std::isnan(v.f)) return false;
    *out = (float)v.f;
    return true;
  }
  if (v.kind == json::Kind::Int) {
    *out = v.bigint ? (float)v.f : (float)v.i;
    return true;
  }
  return decimal_format_parse(as_text(v), out);
}

// NumberInput.parseAsLong(text, 0) (Jackson 2.8)
int64_t text_as_long(std::string_view in) {
  std::string_view s = java_trim(in);
  if (s.empty()) return 0;
  size_t i = 0;
  if (s[0] == '+') s = s.substr(1);
  else if (s[0] == '-') i = 1;
  for (; i < s.size(); ++i)
    if (!is_digit(s[i])) {
      double d;
      return java_parse_double(s, &d) ? java_d2l(d) : 0;
    }
  int64_t v;
  return java_parse_long(s, &v) ? v : 0;
}

int64_t as_long(const json::Value& v) {
  switch (v.kind) {
    case json::Kind::Int: {
      if (!v.bigint) return v.i;
      // BigInteger.longValue(): the low 64 bits
      uint64_t u = 0;
      const bool neg = !v.s.empty() && v.s[0] == '-';
      for (char c : v.s)
        if (is_digit(c)) u = u * 10u + (uint64_t)(c - '0');
      return (int64_t)(neg ? 0u - u : u);
    }
    case json::Kind::Float: return java_d2l(v.f);
    case json::Kind::Bool: return v.b ? 1 : 0;
    case json::Kind::Str: return text_as_long(v.s);
    default: return 0;
  }
}

double as_double(const json::Value& v) {
  switch (v.kind) {
    case json::Kind::Int: return v.bigint ? v.f : (double)v.i;
    case json::Kind::Float: return v.f;
    case json::Kind::Bool: return v.b ? 1.0 : 0.0;
    case json::Kind::Str: {
      // NumberInput.parseAsDouble(text, 0.0)
      double d;
      const std::string_view s = java_trim(v.s);
      return !s.empty() && java_parse_double(s, &d) ? d : 0.0;
    }
    default: return 0.0;
  }
}

}  // namespace

// ------------------------------------------------------------ Formatter
bool Formatter::init(const std::string& spec, std::string* err) {
  if (spec.empty()) {
    *err = "formatter spec is empty";
    return false;
  }
  uint32_t cp;
  const size_t l = decode_cp(spec, 0, &cp);
  std::string_view split_on(spec.data(), l), rest(spec.data() + l, spec.size() - l);
  std::vector<std::string_view> args;
  if (!java_split(split_on, rest, &args, err)) return false;
  auto need = [&](size_t n) {
    if (args.size() < n) {
      *err = "formatter spec has too few arguments";
      return false;
    }
    return true;
  };
  if (args.empty()) {
    *err = "formatter spec has too few arguments";
    return false;
  }
  std::string_view time_pattern;
  bool has_pattern = false;
  if (args[0] == "sv") {
    if (!need(7)) return false;
    sv_ = true;
    auto re = std::make_shared<Re>();
    if (!re->compile(args[1], err)) return false;
    re_.push_back(re);
    int32_t* idx[5] = {&uuid_i_, &lat_i_, &lon_i_, &time_i_, &acc_i_};
    for (int k = 0; k < 5; ++k)
      if (!java_parse_int(args[(size_t)k + 2], idx[k])) {
        *err = "formatter spec: column index \"" + std::string(args[(size_t)k + 2]) + "\" is not an int";
        return false;
      }
    if (args.size() > 7) {
      time_pattern = args[7];
      has_pattern = true;
    }
  } else if (args[0] == "json") {
    if (!need(6)) return false;
    sv_ = false;
    uuid_k_ = args[1];
    lat_k_ = args[2];
    lon_k_ = args[3];
    time_k_ = args[4];
    acc_k_ = args[5];
    if (args.size() > 6) {
      time_pattern = args[6];
      has_pattern = true;
    }
  } else {
    *err = "Unsupported raw format parser";
    return false;
  }
  has_time_fmt_ = has_pattern;
  if (has_pattern && !compile_time_pattern(time_pattern, &time_fmt_, err)) return false;
  return true;
}

bool Formatter::format(std::string_view msg, std::string* key, FormattedPoint* pt) const {
  std::string clean;
  if (utf8_sanitize(msg, &clean)) msg = clean;
  return sv_ ? format_sv(msg, key, pt) : format_json(msg, key, pt);
}

bool Formatter::format_sv(std::string_view msg, std::string* key, FormattedPoint* pt) const {
  thread_local std::vector<std::string_view> parts;
  re_[0]->split(msg, &parts);
  const int32_t n = (int32_t)parts.size();
  auto ok = [n](int32_t i) { return i >= 0 && i < n; };
  if (!ok(lat_i_) || !ok(lon_i_) || !ok(time_i_) || !ok(acc_i_) || !ok(uuid_i_)) return false;
  float lat, lon, acc;
  if (!decimal_format_parse(parts[(size_t)lat_i_], &lat)) return false;
  if (!decimal_format_parse(parts[(size_t)lon_i_], &lon)) return false;
  int64_t time;
  if (has_time_fmt_) {
    if (!parse_time(time_fmt_, parts[(size_t)time_i_], &time)) return false;
  } else if (!java_parse_long(parts[(size_t)time_i_], &time)) {
    return false;
  }
  if (!decimal_format_parse(parts[(size_t)acc_i_], &acc)) return false;
  pt->lat = lat;
  pt->lon = lon;
  pt->time = time;
  pt->accuracy = java_d2i(std::ceil((double)acc));
  key->assign(parts[(size_t)uuid_i_]);
  return true;
}

bool Formatter::format_json(std::string_view msg, std::string* key, FormattedPoint* pt) const {
  json::Value root;
  if (!json::parse_jackson(msg, &root)) return false;
  if (root.kind != json::Kind::Obj) return false;  // get(key) is null -> NullPointerException
  const json::Value* la = root.get(lat_k_);
  const json::Value* lo = root.get(lon_k_);
  const json::Value* tv = root.get(time_k_);
  const json::Value* av = root.get(acc_k_);
  const json::Value* uv = root.get(uuid_k_);
  if (!la || !lo || !tv || !av || !uv) return false;
  float lat, lon;
  if (!node_float(*la, &lat)) return false;
  if (!node_float(*lo, &lon)) return false;
  int64_t time;
  if (has_time_fmt_) {
    if (!parse_time(time_fmt_, as_text(*tv), &time)) return false;
  } else {
    time = as_long(*tv);
  }
  pt->lat = lat;
  pt->lon = lon;
  pt->time = time;
  pt->accuracy = java_d2i(std::ceil(as_double(*av)));
  *key = as_text(*uv);
  // the key goes out through StringSerializer: an unpaired surrogate (a lone
  // \uD800 escape, which Jackson keeps) is written as '?'
  std::string k2;
  if (jstr::wtf8_key(*key, &k2)) key->swap(k2);
  return true;
}

}  // namespace otm

// ------------------------------------------------------------------- C ABI
struct otm_formatter {
  otm::Formatter f;
};

namespace {

struct Chunk {
  std::string keys;
  std::vector<int64_t> klen;
};

void format_range(const otm::Formatter& F, const char* msgs, const int64_t* off, int32_t a, int32_t b,
                  otm_formatted* out, Chunk* c) {
  std::string key;
  for (int32_t i = a; i < b; ++i) {
    otm::FormattedPoint pt;
    key.clear();
    const bool ok = F.format(std::string_view(msgs + off[i], (size_t)(off[i + 1] - off[i])), &key, &pt);
    out->ok[i] = ok ? 1 : 0;
    out->lat[i] = ok ? pt.lat : 0.0f;
    out->lon[i] = ok ? pt.lon : 0.0f;
    out->accuracy[i] = ok ? pt.accuracy : 0;
    out->time[i] = ok ? pt.time : 0;
    if (ok) c->keys.append(key);
    c->klen.push_back(ok ? (int64_t)key.size() : 0);
  }
}

}  // namespace

extern "C" {

int otm_formatter_create(const char* spec, otm_formatter** out, char* err, size_t err_len) {
  if (!spec || !out) return OTM_EINVAL;
  auto* F = new otm_formatter();
  std::string e;
  if (!F->f.init(spec, &e)) {
    delete F;
    if (err && err_len) {
      std::snprintf(err, err_len, "%s", e.c_str());
    }
    return OTM_EINVAL;
  }
  *out = F;
  return OTM_OK;
}

void otm_formatter_destroy(otm_formatter* f) { delete f; }

int otm_format(const otm_formatter* f, int32_t n, const char* msgs, const int64_t* off, int nthreads,
               otm_formatted* out) {
  if (!f || !out || n < 0 || (n > 0 && (!msgs || !off))) return OTM_EINVAL;
  for (int32_t i = 0; i < n; ++i)
    if (off[i + 1] < off[i]) return OTM_EINVAL;
  std::memset(out, 0, sizeof *out);
  out->n = n;
  const size_t m = (size_t)n + 1;
  out->ok = (uint8_t*)std::malloc(m);
  out->key_off = (int64_t*)std::malloc(m * 8);
  out->lat = (float*)std::malloc(m * 4);
  out->lon = (float*)std::malloc(m * 4);
  out->accuracy = (int32_t*)std::malloc(m * 4);
  out->time = (int64_t*)std::malloc(m * 8);
  if (!out->ok || !out->key_off || !out->lat || !out->lon || !out->accuracy || !out->time) {
    otm_formatted_free(out);
    return OTM_ENOMEM;
  }
  int nt = nthreads < 1 ? 1 : nthreads;
  if (n < 16384) nt = 1;
  nt = std::min(nt, 64);
  std::vector<Chunk> chunks((size_t)nt);
  std::vector<std::thread> th;
  const int32_t per = (n + nt - 1) / std::max(nt, 1);
  for (int t = 0; t < nt; ++t) {
    const int32_t a = std::min(n, t * per), b = std::min(n, a + per);
    if (t == nt - 1) format_range(f->f, msgs, off, a, b, out, &chunks[(size_t)t]);
    else th.emplace_back(format_range, std::cref(f->f), msgs, off, a, b, out, &chunks[(size_t)t]);
  }
  for (auto& x : th) x.join();
  size_t total = 0;
  for (const Chunk& c : chunks) total += c.keys.size();
  out->keys = (char*)std::malloc(total + 1);
  if (!out->keys) {
    otm_formatted_free(out);
    return OTM_ENOMEM;
  }
  int64_t pos = 0;
  int32_t i = 0, ok = 0;
  for (const Chunk& c : chunks) {
    std::memcpy(out->keys + pos, c.keys.data(), c.keys.size());
    for (int64_t l : c.klen) {
      out->key_off[i] = pos;
      pos += l;
      ok += out->ok[i];
      ++i;
    }
  }
  out->key_off[n] = pos;
  out->keys[pos] = 0;
  out->n_ok = ok;
  return OTM_OK;
}

void otm_formatted_free(otm_formatted* r) {
  if (!r) return;
  std::free(r->ok);
  std::free(r->key_off);
  std::free(r->keys);
  std::free(r->lat);
  std::free(r->lon);
  std::free(r->accuracy);
  std::free(r->time);
  std::memset(r, 0, sizeof *r);
}

}  // extern "C"
