// json.cpp -- see json.h.
#include "json.h"

#include <cctype>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace otm {
namespace json {

const Value* Value::get(std::string_view k) const {
  if (kind != Kind::Obj) return nullptr;
  for (size_t n = 0; n < keys.size(); ++n)
    if (keys[n] == k) return &items[n];
  return nullptr;
}
Value* Value::get(std::string_view k) { return const_cast<Value*>(static_cast<const Value*>(this)->get(k)); }
void Value::set(std::string_view k, Value v) {
  for (size_t n = 0; n < keys.size(); ++n)
    if (keys[n] == k) {
      items[n] = std::move(v);
      return;
    }
  keys.emplace_back(k);
  items.push_back(std::move(v));
}
void Value::erase(std::string_view k) {
  for (size_t n = 0; n < keys.size(); ++n)
    if (keys[n] == k) {
      keys.erase(keys.begin() + (long)n);
      items.erase(items.begin() + (long)n);
      return;
    }
}
const char* Value::type_name() const {
  switch (kind) {
    case Kind::Null: return "NoneType";
    case Kind::Bool: return "bool";
    case Kind::Int: return "int";
    case Kind::Float: return "float";
    case Kind::Str: return "str";
    case Kind::Arr: return "list";
    default: return "dict";
  }
}

// ------------------------------------------------------------------ parser
namespace {

struct Parser {
  std::string_view t;
  size_t i = 0;
  std::string err;
  bool jackson = false;  // no NaN / Infinity literals (Jackson's default)

  void fail(const char* msg, size_t at) {
    if (!err.empty()) return;
    // positions in code points (the service parses a decoded str)
    size_t cp = 0, line = 1, last_nl = std::string::npos;
    for (size_t k = 0; k < at && k < t.size(); ++k) {
      unsigned char c = (unsigned char)t[k];
      if ((c & 0xC0) == 0x80) continue;
      if (c == '\n') {
        ++line;
        last_nl = cp;
      }
      ++cp;
    }
    size_t col = last_nl == std::string::npos ? cp + 1 : cp - last_nl;
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s: line %zu column %zu (char %zu)", msg, line, col, cp);
    err = buf;
  }
  void ws() {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\t' || t[i] == '\n' || t[i] == '\r')) ++i;
  }
  bool starts(const char* w) const { return t.substr(i, std::strlen(w)) == w; }

  static int hex(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  }
  static void utf8(uint32_t cp, std::string* o) {
    if (cp < 0x80) {
      o->push_back((char)cp);
    } else if (cp < 0x800) {
      o->push_back((char)(0xC0 | (cp >> 6)));
      o->push_back((char)(0x80 | (cp & 63)));
    } else if (cp < 0x10000) {
      o->push_back((char)(0xE0 | (cp >> 12)));
      o->push_back((char)(0x80 | ((cp >> 6) & 63)));
      o->push_back((char)(0x80 | (cp & 63)));
    } else {
      o->push_back((char)(0xF0 | (cp >> 18)));
      o->push_back((char)(0x80 | ((cp >> 12) & 63)));
      o->push_back((char)(0x80 | ((cp >> 6) & 63)));
      o->push_back((char)(0x80 | (cp & 63)));
    }
  }
  bool hex4(size_t at, uint32_t* v) const {
    if (at + 4 > t.size()) return false;
    uint32_t x = 0;
    for (int k = 0; k < 4; ++k) {
      int h = hex(t[at + k]);
      if (h < 0) return false;
      x = x * 16 + (uint32_t)h;
    }
    *v = x;
    return true;
  }
  bool string(std::string* o) {
    const size_t start = i++;
    while (true) {
      if (i >= t.size()) {
        fail("Unterminated string starting at", start);
        return false;
      }
      const unsigned char c = (unsigned char)t[i];
      if (c == '"') {
        ++i;
        return true;
      }
      if (c < 0x20) {
        fail("Invalid control character at", i);
        return false;
      }
      if (c != '\\') {
        // copy a run of plain bytes
        size_t j = i + 1;
        while (j < t.size() && t[j] != '"' && t[j] != '\\' && (unsigned char)t[j] >= 0x20) ++j;
        o->append(t.data() + i, j - i);
        i = j;
        continue;
      }
      if (i + 1 >= t.size()) {
        fail("Unterminated string starting at", start);
        return false;
      }
      const char e = t[i + 1];
      char rep = 0;
      switch (e) {
        case '"': rep = '"'; break;
        case '\\': rep = '\\'; break;
        case '/': rep = '/'; break;
        case 'b': rep = '\b'; break;
        case 'f': rep = '\f'; break;
        case 'n': rep = '\n'; break;
        case 'r': rep = '\r'; break;
        case 't': rep = '\t'; break;
      }
      if (rep) {
        o->push_back(rep);
        i += 2;
        continue;
      }
      if (e != 'u') {
        fail("Invalid \\escape", i);
        return false;
      }
      uint32_t cp;
      if (!hex4(i + 2, &cp)) {
        fail("Invalid \\uXXXX escape", i + 1);
        return false;
      }
      i += 6;
      if (cp >= 0xD800 && cp <= 0xDBFF && i + 1 < t.size() && t[i] == '\\' && t[i + 1] == 'u') {
        uint32_t lo;
        if (!hex4(i + 2, &lo)) {
          fail("Invalid \\uXXXX escape", i + 1);
          return false;
        }
        if (lo >= 0xDC00 && lo <= 0xDFFF) {
          cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          i += 6;
        }
      }
      utf8(cp, o);
    }
  }
  bool number(Value* v) {
    const size_t a = i;
    size_t k = i;
    if (k < t.size() && t[k] == '-') ++k;
    if (k >= t.size() || !std::isdigit((unsigned char)t[k])) return false;
    if (t[k] == '0') ++k;
    else
      while (k < t.size() && std::isdigit((unsigned char)t[k])) ++k;
    bool flt = false;
    if (k + 1 < t.size() && t[k] == '.' && std::isdigit((unsigned char)t[k + 1])) {
      flt = true;
      ++k;
      while (k < t.size() && std::isdigit((unsigned char)t[k])) ++k;
    }
    if (k < t.size() && (t[k] == 'e' || t[k] == 'E')) {
      size_t m = k + 1;
      if (m < t.size() && (t[m] == '+' || t[m] == '-')) ++m;
      if (m < t.size() && std::isdigit((unsigned char)t[m])) {
        flt = true;
        k = m;
        while (k < t.size() && std::isdigit((unsigned char)t[k])) ++k;
      }
    }
    const char* b = t.data() + a;
    const char* e = t.data() + k;
    if (flt) {
      v->kind = Kind::Float;
      // correctly rounded like strtod (float('...')), without a temporary
      // string; overflow / underflow (inf, subnormal) go through strtod
      if (decimal_fast(b, e, &v->f)) {
        i = k;
        return true;
      }
      auto r = std::from_chars(b, e, v->f);
      if (r.ec != std::errc()) {
        std::string tmp(b, e);
        v->f = std::strtod(tmp.c_str(), nullptr);
      }
    } else {
      v->kind = Kind::Int;
      auto r = std::from_chars(b, e, v->i);
      if (r.ec == std::errc::result_out_of_range) {
        v->bigint = true;
        v->s.assign(b, e);
        v->f = std::strtod(v->s.c_str(), nullptr);
      }
    }
    i = k;
    return true;
  }
  bool value(Value* v, int depth) {
    if (depth > 900 || i >= t.size()) {
      fail("Expecting value", i);
      return false;
    }
    const char c = t[i];
    if (c == '"') {
      v->kind = Kind::Str;
      return string(&v->s);
    }
    if (c == '{') {
      v->kind = Kind::Obj;
      // a trace point has 3-4 keys: one allocation each for keys and values
      v->keys.reserve(4);
      v->items.reserve(4);
      ++i;
      ws();
      if (i < t.size() && t[i] == '}') {
        ++i;
        return true;
      }
      while (true) {
        if (i >= t.size() || t[i] != '"') {
          fail("Expecting property name enclosed in double quotes", i);
          return false;
        }
        std::string key;
        if (!string(&key)) return false;
        ws();
        if (i >= t.size() || t[i] != ':') {
          fail("Expecting ':' delimiter", i);
          return false;
        }
        ++i;
        ws();
        Value x;
        if (!value(&x, depth + 1)) return false;
        v->set(key, std::move(x));
        ws();
        if (i < t.size() && t[i] == '}') {
          ++i;
          return true;
        }
        if (i >= t.size() || t[i] != ',') {
          fail("Expecting ',' delimiter", i);
          return false;
        }
        ++i;
        ws();
      }
    }
    if (c == '[') {
      v->kind = Kind::Arr;
      ++i;
      ws();
      if (i < t.size() && t[i] == ']') {
        ++i;
        return true;
      }
      while (true) {
        v->items.emplace_back();
        if (!value(&v->items.back(), depth + 1)) return false;
        ws();
        if (i < t.size() && t[i] == ']') {
          ++i;
          return true;
        }
        if (i >= t.size() || t[i] != ',') {
          fail("Expecting ',' delimiter", i);
          return false;
        }
        ++i;
        ws();
      }
    }
    if (starts("null")) {
      i += 4;
      v->kind = Kind::Null;
      return true;
    }
    if (starts("true")) {
      i += 4;
      v->kind = Kind::Bool;
      v->b = true;
      return true;
    }
    if (starts("false")) {
      i += 5;
      v->kind = Kind::Bool;
      v->b = false;
      return true;
    }
    if (jackson) {
      if (number(v)) return true;
      fail("Expecting value", i);
      return false;
    }
    if (starts("NaN")) {
      i += 3;
      v->kind = Kind::Float;
      v->f = NAN;
      return true;
    }
    if (starts("Infinity")) {
      i += 8;
      v->kind = Kind::Float;
      v->f = INFINITY;
      return true;
    }
    if (starts("-Infinity")) {
      i += 9;
      v->kind = Kind::Float;
      v->f = -INFINITY;
      return true;
    }
    if (number(v)) return true;
    fail("Expecting value", i);
    return false;
  }
};

}  // namespace

bool decimal_fast(const char* s, const char* e, double* out) {
  static const double p10[16] = {1e0, 1e1, 1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
  const bool neg = s < e && *s == '-';
  if (neg) ++s;
  uint64_t m = 0;
  int digits = 0, frac = -1;
  for (; s < e; ++s) {
    const char c = *s;
    if (c >= '0' && c <= '9') {
      m = m * 10 + (uint64_t)(c - '0');
      if (++digits > 15) return false;
      if (frac >= 0) ++frac;
    } else if (c == '.' && frac < 0) {
      frac = 0;
    } else {
      return false;
    }
  }
  if (!digits || frac == 0) return false;
  double d = (double)m;
  if (frac > 0) d /= p10[frac];
  *out = neg ? -d : d;
  return true;
}

bool parse(std::string_view text, Value* out, std::string* err) {
  Parser p;
  p.t = text;
  p.ws();
  *out = Value();
  if (p.value(out, 0)) {
    p.ws();
    if (p.i == text.size()) return true;
    p.fail("Extra data", p.i);
  }
  *err = p.err.empty() ? std::string("Expecting value: line 1 column 1 (char 0)") : p.err;
  return false;
}

bool parse_jackson(std::string_view text, Value* out) {
  Parser p;
  p.t = text;
  p.jackson = true;
  p.ws();
  *out = Value();
  return p.value(out, 0);  // ObjectMapper.readTree: content after the first value is not read
}

std::string utf8_error(std::string_view s) {
  char buf[160];
  size_t i = 0, n = s.size();
  while (i < n) {
    const unsigned char c = (unsigned char)s[i];
    if (c < 0x80) {
      ++i;
      continue;
    }
    int need = 0;
    unsigned lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) need = 2, lo = 0xA0;
    else if ((c >= 0xE1 && c <= 0xEC) || c == 0xEE || c == 0xEF) need = 2;
    else if (c == 0xED) need = 2, hi = 0x9F;
    else if (c == 0xF0) need = 3, lo = 0x90;
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) need = 3, hi = 0x8F;
    else {
      std::snprintf(buf, sizeof buf, "'utf-8' codec can't decode byte 0x%02x in position %zu: invalid start byte", c, i);
      return buf;
    }
    for (int k = 1; k <= need; ++k) {
      if (i + (size_t)k >= n) {
        if (k == 1)
          std::snprintf(buf, sizeof buf, "'utf-8' codec can't decode byte 0x%02x in position %zu: unexpected end of data",
                        c, i);
        else
          std::snprintf(buf, sizeof buf, "'utf-8' codec can't decode bytes in position %zu-%zu: unexpected end of data",
                        i, i + (size_t)k - 1);
        return buf;
      }
      const unsigned char d = (unsigned char)s[i + (size_t)k];
      const unsigned l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
      if (d < l || d > h) {
        if (k == 1)
          std::snprintf(buf, sizeof buf,
                        "'utf-8' codec can't decode byte 0x%02x in position %zu: invalid continuation byte", c, i);
        else
          std::snprintf(buf, sizeof buf, "'utf-8' codec can't decode bytes in position %zu-%zu: invalid continuation byte",
                        i, i + (size_t)k - 1);
        return buf;
      }
    }
    i += (size_t)need + 1;
  }
  return std::string();
}

// ------------------------------------------------------------------ writer
void put_int(int64_t v, std::string* out) {
  char buf[24];
  auto r = std::to_chars(buf, buf + sizeof buf, v);
  out->append(buf, r.ptr);
}

void put_float(double d, std::string* out) {
  if (std::isnan(d)) {
    out->append("NaN");
    return;
  }
  if (std::isinf(d)) {
    out->append(d > 0 ? "Infinity" : "-Infinity");
    return;
  }
  if (d == 0.0) {
    out->append(std::signbit(d) ? "-0.0" : "0.0");
    return;
  }
  // shortest round-trip digits in scientific form: [-]D[.DDD]e[+-]X
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof buf, d, std::chars_format::scientific);
  const char* p = buf;
  bool neg = false;
  if (*p == '-') {
    neg = true;
    ++p;
  }
  char digits[32];
  int nd = 0;
  while (p < r.ptr && *p != 'e') {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  // the exponent to_chars wrote after the 'e': [+-]DD[D]
  int e10 = 0;
  const char* q = p + 1;
  const bool eneg = q < r.ptr && *q == '-';
  if (q < r.ptr && (*q == '-' || *q == '+')) ++q;
  for (; q < r.ptr; ++q) e10 = e10 * 10 + (*q - '0');
  if (eneg) e10 = -e10;
  const int decpt = e10 + 1;  // value = 0.DIGITS x 10^decpt
  if (neg) out->push_back('-');
  if (decpt > -4 && decpt <= 16) {  // float_repr_style 'short', repr rules
    if (decpt <= 0) {
      out->append("0.");
      out->append((size_t)(-decpt), '0');
      out->append(digits, (size_t)nd);
    } else if (decpt >= nd) {
      out->append(digits, (size_t)nd);
      out->append((size_t)(decpt - nd), '0');
      out->append(".0");
    } else {
      out->append(digits, (size_t)decpt);
      out->push_back('.');
      out->append(digits + decpt, (size_t)(nd - decpt));
    }
  } else {
    out->push_back(digits[0]);
    if (nd > 1) {
      out->push_back('.');
      out->append(digits + 1, (size_t)(nd - 1));
    }
    const int x = decpt - 1;
    char eb[16];
    std::snprintf(eb, sizeof eb, "e%c%02d", x < 0 ? '-' : '+', x < 0 ? -x : x);
    out->append(eb);
  }
}

double py_round3(double x) {
  if (!std::isfinite(x)) return x;
  char buf[400];
  std::snprintf(buf, sizeof buf, "%.3f", x);
  return std::strtod(buf, nullptr);
}

static void put_str(std::string_view s, std::string* out) {
  static const char* hexd = "0123456789abcdef";
  out->push_back('"');
  for (size_t i = 0; i < s.size();) {
    const unsigned char c = (unsigned char)s[i];
    if (c >= 0x20 && c < 0x7f && c != '"' && c != '\\') {
      out->push_back((char)c);
      ++i;
      continue;
    }
    switch (c) {
      case '"': out->append("\\\""); ++i; continue;
      case '\\': out->append("\\\\"); ++i; continue;
      case '\n': out->append("\\n"); ++i; continue;
      case '\r': out->append("\\r"); ++i; continue;
      case '\t': out->append("\\t"); ++i; continue;
      case '\b': out->append("\\b"); ++i; continue;
      case '\f': out->append("\\f"); ++i; continue;
    }
    uint32_t cp;
    int len;
    if (c < 0x80) cp = c, len = 1;
    else if ((c & 0xE0) == 0xC0) cp = c & 31u, len = 2;
    else if ((c & 0xF0) == 0xE0) cp = c & 15u, len = 3;
    else cp = c & 7u, len = 4;
    for (int k = 1; k < len && i + (size_t)k < s.size(); ++k) cp = (cp << 6) | ((unsigned char)s[i + (size_t)k] & 63u);
    i += (size_t)len;
    auto u4 = [&](uint32_t v) {
      out->append("\\u");
      for (int sh = 12; sh >= 0; sh -= 4) out->push_back(hexd[(v >> sh) & 15u]);
    };
    if (cp >= 0x10000) {
      cp -= 0x10000;
      u4(0xD800 + (cp >> 10));
      u4(0xDC00 + (cp & 0x3FF));
    } else {
      u4(cp);
    }
  }
  out->push_back('"');
}

void dump(const Value& v, std::string* out) {
  switch (v.kind) {
    case Kind::Null: out->append("null"); return;
    case Kind::Bool: out->append(v.b ? "true" : "false"); return;
    case Kind::Int:
      if (v.bigint) out->append(v.s);
      else put_int(v.i, out);
      return;
    case Kind::Float: put_float(v.f, out); return;
    case Kind::Str: put_str(v.s, out); return;
    case Kind::Arr:
      out->push_back('[');
      for (size_t k = 0; k < v.items.size(); ++k) {
        if (k) out->push_back(',');
        dump(v.items[k], out);
      }
      out->push_back(']');
      return;
    case Kind::Obj:
      out->push_back('{');
      for (size_t k = 0; k < v.items.size(); ++k) {
        if (k) out->push_back(',');
        put_str(v.keys[k], out);
        out->push_back(':');
        dump(v.items[k], out);
      }
      out->push_back('}');
      return;
  }
}

}  // namespace json
}  // namespace otm
