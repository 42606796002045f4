// json.h -- JSON with CPython 3 json-module semantics (host side of libotmatch).
//
// The /report contract is byte-level: reporter_service
// parses bodies with json.loads (py/reporter_service.py:100) and answers with
// json.dumps(..., separators=(',', ':')) (:215).  This module reproduces both:
// int-vs-float by spelling, dict order with in-place duplicate-key update,
// JSONDecodeError texts with line/column/char positions in code points, float
// repr (shortest round trip) and ensure_ascii escaping.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace otm {
namespace json {

enum class Kind : uint8_t { Null, Bool, Int, Float, Str, Arr, Obj };

struct Value {
  Kind kind = Kind::Null;
  bool b = false;
  bool bigint = false;  // Int beyond int64: digits kept in s, value in f
  int64_t i = 0;
  double f = 0.0;
  std::string s;
  std::vector<Value> items;        // Arr values / Obj values
  std::vector<std::string> keys;   // Obj keys (same order as items)

  bool is_num() const { return kind == Kind::Int || kind == Kind::Float || kind == Kind::Bool; }
  double num() const { return kind == Kind::Float ? f : (kind == Kind::Bool ? (b ? 1.0 : 0.0) : (bigint ? f : (double)i)); }
  const Value* get(std::string_view k) const;
  Value* get(std::string_view k);
  void set(std::string_view k, Value v);  // dict.__setitem__
  void erase(std::string_view k);
  const char* type_name() const;  // Python type name
};

// json.loads; on failure returns false and *err = str(JSONDecodeError)
bool parse(std::string_view text, Value* out, std::string* err);
// Jackson 2.8 ObjectMapper.readTree of a String: the first JSON value, no
// NaN / Infinity literals, trailing content ignored
bool parse_jackson(std::string_view text, Value* out);
// bytes.decode('utf-8') check: empty string when valid, else str(UnicodeDecodeError)
std::string utf8_error(std::string_view bytes);

// float('...') of a plain decimal [-]digits[.digits] with at most 15 digits in
// all: the digits are an exact double below 2^53 and 10^k (k <= 15) is exact,
// so one IEEE division is the correctly rounded value strtod returns (Clinger's
// fast path).  false for anything else (exponents, more digits): use strtod.
bool decimal_fast(const char* s, const char* e, double* out);

// json.dumps(v, separators=(',', ':'))
void dump(const Value& v, std::string* out);
// float.__repr__ as json.dumps writes it (NaN / Infinity / -Infinity for non-finite)
void put_float(double d, std::string* out);
void put_int(int64_t v, std::string* out);
// round(x, 3) of CPython for a finite float
double py_round3(double x);

}  // namespace json
}  // namespace otm
