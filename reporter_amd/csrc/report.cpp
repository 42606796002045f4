// report.cpp -- see report.h.
#include "report.h"

#include <charconv>

#include <cmath>
#include <cstdio>
#include <cstring>

namespace otm {

using json::Kind;
using json::Value;

// Java DecimalFormat("###.######", HALF_EVEN) of a float widened to double
// (Point.java:29,41-42).  "###" sets no minimum integer digit, so |x| < 1
// prints without its leading zero (".5", "-.5"); a value that rounds to zero
// prints "0" (with the sign of a negative input).  No JVM exists here to pin
// this against: the rules are DecimalFormat's documented behaviour.
void java_decimal6(float f, std::string* o) {
  // n = the value in millionths, HALF_EVEN on the exact binary value: f * 1e6
  // is exact in double (24 + 14 significant bits) and nearbyint rounds ties
  // to even; the text is then n's digits with the point six from the right.
  const double d = (double)f * 1e6;
  if (std::fabs(d) < 9.0e15) {
    const double r = std::nearbyint(d);
    uint64_t n = (uint64_t)std::fabs(r);
    char buf[32];
    int p = (int)sizeof buf;
    uint64_t ip = n / 1000000u;
    uint32_t fr = (uint32_t)(n % 1000000u);
    int fd = 6;
    while (fd > 0 && fr % 10u == 0) {
      fr /= 10u;
      --fd;
    }
    for (int k = 0; k < fd; ++k) {
      buf[--p] = (char)('0' + fr % 10u);
      fr /= 10u;
    }
    if (fd > 0) buf[--p] = '.';
    if (ip > 0 || fd == 0) {
      do {
        buf[--p] = (char)('0' + ip % 10u);
        ip /= 10u;
      } while (ip > 0);
    }
    if (std::signbit(r)) o->push_back('-');
    o->append(buf + p, sizeof buf - (size_t)p);
    return;
  }
  char buf[64];
  std::snprintf(buf, sizeof buf, "%.6f", (double)f);  // exact binary value, half-even
  std::string s(buf);
  const bool neg = s[0] == '-';
  std::string mag = neg ? s.substr(1) : s;
  size_t end = mag.size();
  while (end > 0 && mag[end - 1] == '0') --end;
  if (end > 0 && mag[end - 1] == '.') --end;
  mag.resize(end);
  if (mag.size() > 1 && mag[0] == '0' && mag[1] == '.') mag = mag.substr(1);
  if (neg) o->push_back('-');
  o->append(mag);
}

void encode_request(std::string_view wire_uuid, int n, const float* lat, const float* lon, const int64_t* time,
                    const int32_t* accuracy, std::string* out) {
  std::string& s = *out;
  s.clear();
  s.reserve(9 + wire_uuid.size() + 11 + (size_t)n * 72 + 2);
  s.append("{\"uuid\":\"");
  s.append(wire_uuid);  // unescaped, as sb.append(key) (Batch.java:55)
  s.append("\",\"trace\":[");
  for (int k = 0; k < n; ++k) {
    s.append("{\"lat\":");
    java_decimal6(lat[k], &s);
    s.append(",\"lon\":");
    java_decimal6(lon[k], &s);
    s.append(",\"time\":");
    json::put_int(time[k], &s);
    s.append(",\"accuracy\":");
    json::put_int(accuracy[k], &s);
    s.append("},");
  }
  // sb.replace(len-1, len+1, "]}"): the trailing ',' becomes "]}"; with no
  // points the '[' itself is replaced (Batch.java:60)
  s.pop_back();
  s.append("]}");
}

std::string error_body(const std::string& msg) { return "{\"error\":\"" + msg + "\"}"; }

const char* trace_error_text(int kind) {
  switch (kind) {
    case OTM_TERR_ZERODIV: return "float division by zero";
    case OTM_TERR_ZERODIV_INT: return "division by zero";
    case OTM_TERR_CAND_OVERFLOW: return "too many candidate edges within search radius";
    case OTM_TERR_SEARCH_OVERFLOW: return "route search exceeded node limit";
  }
  return "";
}

static size_t cp_len(const std::string& s) {
  size_t n = 0;
  for (unsigned char c : s)
    if ((c & 0xC0) != 0x80) ++n;
  return n;
}

int parse_request(const char* path, std::string_view body, Value* trace, std::string* resp) {
  // :88-96 -- the action is the last path component
  if (path) {
    std::string_view pv(path);
    pv = pv.substr(0, pv.find_first_of("?#"));
    const size_t slash = pv.rfind('/');
    const std::string_view last = slash == std::string_view::npos ? pv : pv.substr(slash + 1);
    if (last != "report") {
      *resp = error_body("Try a valid action: ['report']");
      return 400;
    }
  }
  // :99-100
  std::string uerr = json::utf8_error(body);
  if (!uerr.empty()) {
    *resp = error_body(uerr);
    return 400;
  }
  std::string perr;
  if (!json::parse(body, trace, &perr)) {
    *resp = error_body(perr);
    return 400;
  }
  // :226 trace.get('uuid') runs outside the try: do() answers 400 str(e)
  if (trace->kind != Kind::Obj) {
    *resp = std::string("'") + trace->type_name() + "' object has no attribute 'get'";
    return 400;
  }
  const Value* uuid = trace->get("uuid");
  if (!uuid || uuid->kind == Kind::Null) {
    *resp = error_body("uuid is required");
    return 400;
  }
  // :231-234 trace['trace'][1]
  const Value* tr = trace->get("trace");
  bool ok = false;
  if (tr) {
    if (tr->kind == Kind::Arr) ok = tr->items.size() >= 2;
    else if (tr->kind == Kind::Str) ok = cp_len(tr->s) >= 2;
  }
  if (!ok) {
    *resp = error_body(
        "trace must be a non zero length array of object each of which must have at least lat, lon and time");
    return 400;
  }
  return 0;
}

// ------------------------------------------------------------ python values
namespace {

struct PV {  // a borrowed Python value
  const Value* v;  // nullptr == None
  Kind kind() const { return v ? v->kind : Kind::Null; }
  bool num() const { return v && v->is_num(); }
  bool integral() const { return v && (v->kind == Kind::Int || v->kind == Kind::Bool); }
  bool big() const { return v && v->bigint; }
  double d() const { return v->num(); }
  int64_t i() const { return v->kind == Kind::Bool ? (v->b ? 1 : 0) : v->i; }
  const char* tn() const { return v ? v->type_name() : "NoneType"; }
};

// a computed number: int or float
struct Num {
  bool is_int;
  int64_t i;
  double f;
  double d() const { return is_int ? (double)i : f; }
};

const Value kTrue = [] {
  Value v;
  v.kind = Kind::Bool;
  v.b = true;
  return v;
}();
const Value kFalse = [] {
  Value v;
  v.kind = Kind::Bool;
  v.b = false;
  return v;
}();

std::string fmt2(const char* f, const char* a, const char* b) {
  char buf[256];
  std::snprintf(buf, sizeof buf, f, a, b);
  return buf;
}

bool to_num(PV a, Num* n) {
  if (!a.num()) return false;
  if (a.integral() && !a.big()) *n = Num{true, a.i(), 0.0};
  else *n = Num{false, 0, a.d()};
  return true;
}

bool py_sub(PV a, PV b, Num* r, std::string* exc) {
  Num x, y;
  if (!to_num(a, &x) || !to_num(b, &y)) {
    *exc = fmt2("unsupported operand type(s) for -: '%s' and '%s'", a.tn(), b.tn());
    return false;
  }
  if (x.is_int && y.is_int) *r = Num{true, x.i - y.i, 0.0};
  else *r = Num{false, 0, x.d() - y.d()};
  return true;
}

bool py_eq(PV a, PV b);
bool value_eq(const Value& a, const Value& b) {
  if (a.kind == Kind::Str) return a.s == b.s;
  if (a.kind == Kind::Arr) {
    if (a.items.size() != b.items.size()) return false;
    for (size_t k = 0; k < a.items.size(); ++k)
      if (!py_eq(PV{&a.items[k]}, PV{&b.items[k]})) return false;
    return true;
  }
  if (a.kind == Kind::Obj) {
    if (a.items.size() != b.items.size()) return false;
    for (size_t k = 0; k < a.items.size(); ++k) {
      const Value* o = b.get(a.keys[k]);
      if (!o || !py_eq(PV{&a.items[k]}, PV{o})) return false;
    }
    return true;
  }
  return false;
}
bool py_eq(PV a, PV b) {
  if (a.num() && b.num()) {
    Num x, y;
    to_num(a, &x);
    to_num(b, &y);
    if (x.is_int && y.is_int) return x.i == y.i;
    return x.d() == y.d();
  }
  if (a.kind() == Kind::Null || b.kind() == Kind::Null) return a.kind() == b.kind();
  if (a.kind() != b.kind()) return false;
  return value_eq(*a.v, *b.v);
}
bool py_eq_int(PV a, int64_t k) {
  if (!a.num()) return false;
  Num x;
  to_num(a, &x);
  return x.is_int ? x.i == k : x.f == (double)k;
}

// a < b / a > b for Num-or-PV left operands against an int or threshold
bool num_cmp(Num a, Num b, char op) {
  if (a.is_int && b.is_int) return op == '<' ? a.i < b.i : a.i > b.i;
  return op == '<' ? a.d() < b.d() : a.d() > b.d();
}
bool py_cmp_int(PV a, int64_t k, char op, bool* res, std::string* exc) {
  Num x;
  if (!to_num(a, &x)) {
    char buf[256];
    std::snprintf(buf, sizeof buf, "'%c' not supported between instances of '%s' and 'int'", op, a.tn());
    *exc = buf;
    return false;
  }
  *res = num_cmp(x, Num{true, k, 0.0}, op);
  return true;
}
bool truthy(PV a) {
  switch (a.kind()) {
    case Kind::Null: return false;
    case Kind::Bool: return a.v->b;
    case Kind::Int: return a.v->bigint ? true : a.v->i != 0;
    case Kind::Float: return a.v->f != 0.0;
    case Kind::Str: return !a.v->s.empty();
    default: return !a.v->items.empty();
  }
}
const Value* getitem(const Value* x, const char* key, std::string* exc) {
  if (!x || x->kind == Kind::Null) {
    *exc = "'NoneType' object is not subscriptable";
    return nullptr;
  }
  if (x->kind == Kind::Obj) {
    const Value* v = x->get(key);
    if (!v) *exc = std::string("'") + key + "'";
    return v;
  }
  if (x->kind == Kind::Arr) *exc = "list indices must be integers or slices, not str";
  else if (x->kind == Kind::Str) *exc = "string indices must be integers";
  else *exc = std::string("'") + x->type_name() + "' object is not subscriptable";
  return nullptr;
}
const Value* index(const Value& x, int64_t k, std::string* exc) {
  if (x.kind == Kind::Arr) return &x.items[(size_t)k];
  if (x.kind == Kind::Obj) *exc = std::to_string(k);
  else *exc = "string indices must be integers";
  return nullptr;
}
bool in_set(const std::vector<int64_t>& s, int64_t x) {
  for (auto v : s)
    if (v == x) return true;
  return false;
}

}  // namespace

bool report_dom(const ReportConfig& rc, const Value& trace, Value* segments, std::string* resp,
                std::string* stderr_text, std::string* exc) {
  // :116
  const Value* tr = trace.get("trace");
  if (tr->kind != Kind::Arr) {
    *exc = "string indices must be integers";
    return false;
  }
  const Value* et = getitem(&tr->items.back(), "time", exc);
  if (!et) return false;
  PV end_time{et};
  // :120
  const Value* segs = getitem(segments, "segments", exc);
  if (!segs) return false;
  int64_t nseg;
  if (segs->kind == Kind::Arr || segs->kind == Kind::Obj) nseg = (int64_t)segs->items.size();
  else if (segs->kind == Kind::Str) nseg = (int64_t)cp_len(segs->s);
  else {
    *exc = std::string("object of type '") + segs->type_name() + "' has no len()";
    return false;
  }
  int64_t last_idx = nseg - 1;
  // threshold: int 15, or the bool True / False strtobool produced
  const Value thr_v = [&] {
    Value v;
    if (rc.threshold_sec == 15.0) {
      v.kind = Kind::Int;
      v.i = 15;
    } else {
      v.kind = Kind::Bool;
      v.b = rc.threshold_sec != 0.0;
    }
    return v;
  }();
  Num thr;
  to_num(PV{&thr_v}, &thr);
  // :121-122
  while (last_idx >= 0) {
    const Value* s = index(*segs, last_idx, exc);
    if (!s) return false;
    const Value* st = getitem(s, "start_time", exc);
    if (!st) return false;
    Num diff;
    if (!py_sub(end_time, PV{st}, &diff, exc)) return false;
    if (!num_cmp(diff, thr, '<')) break;
    --last_idx;
  }
  // :125-127
  const Value* shape_used = nullptr;
  if (last_idx >= 0) {
    const Value* s = index(*segs, last_idx, exc);
    if (!s) return false;
    shape_used = getitem(s, "begin_shape_index", exc);
    if (!shape_used) return false;
  }
  // :131
  {
    Value mode;
    mode.kind = Kind::Str;
    mode.s = "auto";
    segments->set("mode", std::move(mode));
  }
  segs = segments->get("segments");
  // :132-196
  bool have = false, first_seg = true;
  PV prior_id{nullptr}, prior_start{nullptr}, prior_end{nullptr}, prior_len{nullptr}, prior_ql{nullptr};
  int64_t prior_level = -1;
  int64_t successful = 0, unreported = 0, disc = 0, invalid = 0, unassoc = 0;
  bool succ_set = false, unrep_set = false;
  double succ_len = 0, unrep_len = 0;
  std::string reps;
  int nreps = 0;
  for (int64_t idx = 0; idx <= last_idx; ++idx) {
    const Value* seg = index(*segs, idx, exc);
    if (!seg) return false;
    if (seg->kind != Kind::Obj) {
      *exc = std::string("'") + seg->type_name() + "' object has no attribute 'get'";
      return false;
    }
    PV segment_id{seg->get("segment_id")}, start_time{seg->get("start_time")}, end_time_s{seg->get("end_time")};
    const Value* iv = seg->get("internal");
    PV internal{iv ? iv : &kFalse}, queue_length{seg->get("queue_length")}, length{seg->get("length")};
    // :150
    if (idx != 0) {
      const Value* a = getitem(seg, "start_time", exc);
      if (!a) return false;
      if (py_eq_int(PV{a}, -1)) {
        const Value* prev = index(*segs, idx - 1, exc);
        if (!prev) return false;
        const Value* b = getitem(prev, "end_time", exc);
        if (!b) return false;
        if (py_eq_int(PV{b}, -1)) ++disc;
      }
    }
    // :154
    int64_t level = -1;
    if (segment_id.kind() != Kind::Null) {
      if (!segment_id.integral() || segment_id.big()) {
        *exc = fmt2("unsupported operand type(s) for &: '%s' and '%s'", segment_id.tn(), "int");
        return false;
      }
      level = segment_id.i() & 0x7;
    }
    // :157
    if (have && prior_id.kind() != Kind::Null) {
      bool gt;
      if (!py_cmp_int(prior_len, 0, '>', &gt, exc)) return false;
      if (gt && !py_eq(internal, PV{&kTrue})) {
        if (in_set(rc.report_levels, prior_level)) {
          const bool trans = in_set(rc.transition_levels, level);
          PV t1 = trans ? start_time : prior_end;
          Num diff;
          if (!py_sub(t1, prior_start, &diff, exc)) return false;
          Num len;
          to_num(prior_len, &len);
          if (diff.d() == 0.0) {
            *exc = (len.is_int && diff.is_int) ? "division by zero" : "float division by zero";
            return false;
          }
          const double speed = (len.d() / diff.d()) * 3.6;
          if (speed < 200.0) {
            reps.append(nreps ? ",{\"id\":" : "{\"id\":");
            json::dump(*prior_id.v, &reps);
            reps.append(",\"t0\":");
            if (prior_start.v) json::dump(*prior_start.v, &reps);
            else reps.append("null");
            reps.append(",\"t1\":");
            if (t1.v) json::dump(*t1.v, &reps);
            else reps.append("null");
            reps.append(",\"length\":");
            json::dump(*prior_len.v, &reps);
            reps.append(",\"queue_length\":");
            if (prior_ql.v) json::dump(*prior_ql.v, &reps);
            else reps.append("null");
            if (trans && segment_id.kind() != Kind::Null) {
              reps.append(",\"next_id\":");
              json::dump(*segment_id.v, &reps);
            }
            reps.push_back('}');
            ++nreps;
            ++successful;
            succ_len = json::py_round3(len.d() * 0.001);
            succ_set = true;
          } else {
            stderr_text->append("Speed exceeds 200kph\n");
            ++invalid;
          }
        } else {
          ++unreported;
          Num len;
          to_num(prior_len, &len);
          unrep_len = json::py_round3(len.d() * 0.001);
          unrep_set = true;
        }
      }
    }
    // :179-189
    if (!(py_eq(internal, PV{&kTrue}) && !first_seg)) {
      prior_id = segment_id;
      prior_start = start_time;
      prior_end = end_time_s;
      prior_len = length;
      prior_level = level;
      prior_ql = queue_length;
      have = true;
    }
    first_seg = false;
    // :195
    if (segment_id.kind() == Kind::Null && py_eq(internal, PV{&kFalse})) ++unassoc;
  }
  // :198-215
  std::string& o = *resp;
  o.clear();
  o.append("{\"stats\":{\"successful_matches\":{\"count\":");
  json::put_int(successful, &o);
  o.append(",\"length\":");
  if (succ_set) json::put_float(succ_len, &o);
  else o.push_back('0');
  o.append("},\"unreported_matches\":{\"count\":");
  json::put_int(unreported, &o);
  o.append(",\"length\":");
  if (unrep_set) json::put_float(unrep_len, &o);
  else o.push_back('0');
  o.append("},\"match_errors\":{\"discontinuities\":");
  json::put_int(disc, &o);
  o.append(",\"invalid_speeds\":");
  json::put_int(invalid, &o);
  o.append("},\"unassociated_segments\":");
  json::put_int(unassoc, &o);
  o.push_back('}');
  if (shape_used && truthy(PV{shape_used})) {
    o.append(",\"shape_used\":");
    json::dump(*shape_used, &o);
  }
  o.append(",\"segment_matcher\":");
  json::dump(*segments, &o);
  o.append(",\"datastore\":{\"mode\":\"auto\"");
  if (nreps) {
    o.append(",\"reports\":[");
    o.append(reps);
    o.push_back(']');
  }
  o.append("}}");
  return true;
}

bool extract_points(const Value& trace, TracePoints* out, std::string* err) {
  const Value* tr = trace.get("trace");
  if (!tr || tr->kind != Kind::Arr) {
    *err = "trace must be an array of points";
    return false;
  }
  const size_t n = tr->items.size();
  out->lat.resize(n);
  out->lon.resize(n);
  out->acc.resize(n);
  out->time.resize(n);
  auto num = [](const Value* v, double* d) {
    if (!v || (v->kind != Kind::Int && v->kind != Kind::Float)) return false;
    *d = v->kind == Kind::Int ? (v->bigint ? v->f : (double)v->i) : v->f;
    return true;
  };
  for (size_t k = 0; k < n; ++k) {
    const Value& pt = tr->items[k];
    double la, lo, ti, ac;
    if (pt.kind != Kind::Obj || !num(pt.get("lat"), &la) || !num(pt.get("lon"), &lo) || !num(pt.get("time"), &ti)) {
      *err = "trace point " + std::to_string(k) + " must have numeric lat, lon and time";
      return false;
    }
    out->lat[k] = (float)la;
    out->lon[k] = (float)lo;
    out->time[k] = ti;
    out->acc[k] = num(pt.get("accuracy"), &ac) ? (float)ac : 0.0f;
  }
  return true;
}

bool fast_request(std::string_view b, TracePoints* out, std::string* uuid) {
  const size_t n = b.size();
  const char* const p = b.data();
  size_t i = 0;
  auto lit = [&](std::string_view w) {
    if (i + w.size() > n || std::memcmp(p + i, w.data(), w.size()) != 0) return false;
    i += w.size();
    return true;
  };
  auto digit = [&](size_t k) { return k < n && (unsigned)(p[k] - '0') < 10u; };
  // a JSON number as json.loads + float() read it (int -> exact double,
  // float -> correctly rounded), in one pass: up to 15 significant digits the
  // digits are exact and one division by an exact power of ten is the correctly
  // rounded value (json::decimal_fast); longer floats go through from_chars
  static const double p10[16] = {1e0, 1e1, 1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                 1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};
  auto num = [&](double* d) {
    const size_t a = i;
    const bool neg = i < n && p[i] == '-';
    if (neg) ++i;
    if (!digit(i)) return false;
    uint64_t m = 0;
    int nd = 0;
    if (p[i] == '0') {
      ++i;
      nd = 1;
    } else {
      while (digit(i)) {
        m = m * 10 + (uint64_t)(p[i] - '0');
        ++nd;
        ++i;
      }
    }
    int frac = 0;
    if (i < n && p[i] == '.') {
      if (!digit(i + 1)) return false;
      ++i;
      while (digit(i)) {
        m = m * 10 + (uint64_t)(p[i] - '0');
        ++nd;
        ++frac;
        ++i;
      }
      if (i < n && (p[i] == 'e' || p[i] == 'E')) return false;
      if (nd <= 15) {
        const double v = (double)m / p10[frac];
        *d = neg ? -v : v;
        return true;
      }
      const auto r = std::from_chars(p + a, p + i, *d);
      return r.ec == std::errc() && r.ptr == p + i;
    }
    if (i < n && (p[i] == 'e' || p[i] == 'E')) return false;
    if (i - a > 18) return false;  // (m cannot have wrapped: at most 18 digits)
    const int64_t v = neg ? -(int64_t)m : (int64_t)m;
    *d = (double)v;
    return true;
  };
  out->lat.clear();
  out->lon.clear();
  out->time.clear();
  out->acc.clear();
  // a Java point is ~66 bytes: reserve once instead of growing four vectors
  const size_t guess = n / 48 + 2;
  out->lat.reserve(guess);
  out->lon.reserve(guess);
  out->time.reserve(guess);
  out->acc.reserve(guess);
  if (!lit("{")) return false;
  bool have_uuid = false, have_trace = false;
  while (true) {
    if (lit("\"uuid\":\"")) {
      if (have_uuid) return false;
      have_uuid = true;
      const size_t a = i;
      while (i < n && b[i] != '"') {
        const unsigned char c = (unsigned char)b[i];
        if (c < 0x20 || c > 0x7e || c == '\\') return false;
        ++i;
      }
      if (i >= n) return false;
      uuid->assign(b.data() + a, i - a);
      ++i;
    } else if (lit("\"trace\":[")) {
      if (have_trace) return false;
      have_trace = true;
      while (true) {
        if (!lit("{")) return false;
        bool hl = false, ho = false, ht = false, ha = false;
        double la = 0.0, lo = 0.0, ti = 0.0, ac = 0.0;
        while (true) {
          // the key by its first letters, then checked whole (trying each key's
          // literal in turn measured ~40% slower)
          const char k1 = i + 2 < n ? p[i + 1] : 0, k2 = i + 2 < n ? p[i + 2] : 0;
          if (k1 == 'l' && k2 == 'a' && lit("\"lat\":")) {
            if (hl || !num(&la)) return false;
            hl = true;
          } else if (k1 == 'l' && k2 == 'o' && lit("\"lon\":")) {
            if (ho || !num(&lo)) return false;
            ho = true;
          } else if (k1 == 't' && lit("\"time\":")) {
            if (ht || !num(&ti)) return false;
            ht = true;
          } else if (k1 == 'a' && lit("\"accuracy\":")) {
            if (ha || !num(&ac)) return false;
            ha = true;
          } else {
            return false;
          }
          if (lit(",")) continue;
          if (lit("}")) break;
          return false;
        }
        if (!hl || !ho || !ht) return false;
        // extract_points' conversions
        out->lat.push_back((float)la);
        out->lon.push_back((float)lo);
        out->time.push_back(ti);
        out->acc.push_back(ha ? (float)ac : 0.0f);
        if (lit(",")) continue;
        if (lit("]")) break;
        return false;
      }
      if (out->lat.size() < 2) return false;
    } else {
      return false;
    }
    if (lit(",")) continue;
    if (lit("}")) break;
    return false;
  }
  return have_uuid && have_trace && i == n;
}

// ------------------------------------------------------------ typed segments
namespace {
constexpr double kExactInt = 9007199254740992.0;  // 2^53: ints below it are exact doubles
bool int_in(const Value* v, int64_t lo, int64_t hi, int64_t* out) {
  if (!v || v->kind != Kind::Int || v->bigint || v->i < lo || v->i > hi) return false;
  *out = v->i;
  return true;
}
// a time: int literal (exact) or finite float; *is_int says which
bool time_of(const Value* v, double* out, bool* is_int) {
  if (!v) return false;
  if (v->kind == Kind::Int && !v->bigint && std::fabs((double)v->i) < kExactInt) {
    *out = (double)v->i;
    *is_int = true;
    return true;
  }
  if (v->kind == Kind::Float && std::isfinite(v->f)) {
    *out = v->f;
    *is_int = false;
    return true;
  }
  return false;
}
}  // namespace

bool typed_segments(const Value& trace, const Value& match, std::vector<otm_segment>* out, double* end_time,
                    std::string* why) {
  out->clear();
  const Value* tr = trace.get("trace");
  bool et_int;
  if (!tr || tr->kind != Kind::Arr || tr->items.empty() || tr->items.back().kind != Kind::Obj ||
      !time_of(tr->items.back().get("time"), end_time, &et_int)) {
    *why = "the trace's last time is not a number";
    return false;
  }
  const Value* segs = match.kind == Kind::Obj ? match.get("segments") : nullptr;
  if (!segs || segs->kind != Kind::Arr) {
    *why = "Match output has no segments array";
    return false;
  }
  for (size_t k = 0; k < segs->items.size(); ++k) {
    const Value& sv = segs->items[k];
    otm_segment s;
    std::memset(&s, 0, sizeof s);
    const std::string at = "segment " + std::to_string(k) + ": ";
    if (sv.kind != Kind::Obj) {
      *why = at + "not an object";
      return false;
    }
    const Value* id = sv.get("segment_id");
    if (!id || id->kind == Kind::Null) {
      s.segment_id = -1;
    } else if (!int_in(id, 0, INT64_MAX, &s.segment_id)) {
      *why = at + "segment_id is not a non-negative int";
      return false;
    }
    bool si, ei;
    if (!time_of(sv.get("start_time"), &s.start_time, &si) || !time_of(sv.get("end_time"), &s.end_time, &ei)) {
      *why = at + "start_time / end_time are not numbers";
      return false;
    }
    s.flags = OTM_SEG_START_VALID | OTM_SEG_END_VALID | (si ? OTM_SEG_START_INT : 0u) | (ei ? OTM_SEG_END_INT : 0u);
    const Value* in = sv.get("internal");
    if (in && in->kind != Kind::Bool) {
      *why = at + "internal is not a bool";
      return false;
    }
    if (in && in->b) s.flags |= OTM_SEG_INTERNAL;
    int64_t v;
    if (!int_in(sv.get("length"), INT32_MIN, INT32_MAX, &v)) {
      *why = at + "length is not an int";
      return false;
    }
    s.length = (int32_t)v;
    if (!int_in(sv.get("queue_length"), INT32_MIN, INT32_MAX, &v)) {
      *why = at + "queue_length is not an int";
      return false;
    }
    s.queue_length = (int32_t)v;
    if (!int_in(sv.get("begin_shape_index"), 0, INT32_MAX, &v)) {
      *why = at + "begin_shape_index is not a non-negative int";
      return false;
    }
    s.begin_shape_index = (int32_t)v;
    s.end_shape_index = -1;
    out->push_back(s);
  }
  return true;
}

// ------------------------------------------------------------ typed writers
static void put_time(bool valid, double t, std::string* o) {
  if (valid) json::put_float(t, o);
  else o->append("-1");
}

static void write_segments_array(const otm_results& r, const otm_trace_result& tr, std::string* o) {
  o->push_back('[');
  for (int32_t k = 0; k < tr.seg_cnt; ++k) {
    const otm_segment& s = r.segments[tr.seg_off + k];
    if (k) o->push_back(',');
    o->push_back('{');
    if (s.segment_id >= 0) {
      o->append("\"segment_id\":");
      json::put_int(s.segment_id, o);
      o->push_back(',');
    }
    o->append("\"way_ids\":[");
    for (int32_t w = 0; w < s.way_cnt; ++w) {
      if (w) o->push_back(',');
      json::put_int(r.way_ids[s.way_off + w], o);
    }
    o->append("],\"start_time\":");
    put_time(s.flags & OTM_SEG_START_VALID, s.start_time, o);
    o->append(",\"end_time\":");
    put_time(s.flags & OTM_SEG_END_VALID, s.end_time, o);
    o->append(",\"queue_length\":");
    json::put_int(s.queue_length, o);
    o->append(",\"length\":");
    json::put_int(s.length, o);
    o->append((s.flags & OTM_SEG_INTERNAL) ? ",\"internal\":true" : ",\"internal\":false");
    o->append(",\"begin_shape_index\":");
    json::put_int(s.begin_shape_index, o);
    o->append(",\"end_shape_index\":");
    json::put_int(s.end_shape_index, o);
    o->push_back('}');
  }
  o->push_back(']');
}

void write_match_json(const otm_results& r, int32_t t, std::string* o) {
  o->append("{\"segments\":");
  write_segments_array(r, r.traces[t], o);
  o->push_back('}');
}

int write_report_response(const otm_results& r, int32_t t, std::string* o, const std::string* matcher_json) {
  const otm_trace_result& tr = r.traces[t];
  if (tr.code != 200) {
    *o = error_body(trace_error_text(tr.error_kind));
    return 500;
  }
  o->append("{\"stats\":{\"successful_matches\":{\"count\":");
  json::put_int(tr.successful_count, o);
  o->append(",\"length\":");
  if (tr.successful_length >= 0) json::put_float(json::py_round3((double)tr.successful_length * 0.001), o);
  else o->push_back('0');
  o->append("},\"unreported_matches\":{\"count\":");
  json::put_int(tr.unreported_count, o);
  o->append(",\"length\":");
  if (tr.unreported_length >= 0) json::put_float(json::py_round3((double)tr.unreported_length * 0.001), o);
  else o->push_back('0');
  o->append("},\"match_errors\":{\"discontinuities\":");
  json::put_int(tr.discontinuities, o);
  o->append(",\"invalid_speeds\":");
  json::put_int(tr.invalid_speeds, o);
  o->append("},\"unassociated_segments\":");
  json::put_int(tr.unassociated, o);
  o->push_back('}');
  if (tr.shape_used > 0) {
    o->append(",\"shape_used\":");
    json::put_int(tr.shape_used, o);
  }
  if (matcher_json) {
    o->append(",\"segment_matcher\":");
    o->append(*matcher_json);
    o->append(",\"datastore\":{\"mode\":\"auto\"");
  } else {
    o->append(",\"segment_matcher\":{\"segments\":");
    write_segments_array(r, tr, o);
    o->append(",\"mode\":\"auto\"},\"datastore\":{\"mode\":\"auto\"");
  }
  if (tr.rep_cnt > 0) {
    o->append(",\"reports\":[");
    for (int32_t k = 0; k < tr.rep_cnt; ++k) {
      const otm_report_rec& p = r.reports[tr.rep_off + k];
      if (k) o->push_back(',');
      o->append("{\"id\":");
      json::put_int(p.id, o);
      o->append(",\"t0\":");
      if (p.flags & OTM_REP_T0_INT) json::put_int((int64_t)p.t0, o);
      else json::put_float(p.t0, o);
      o->append(",\"t1\":");
      if (p.flags & OTM_REP_T1_INT) json::put_int((int64_t)p.t1, o);
      else json::put_float(p.t1, o);
      o->append(",\"length\":");
      json::put_int(p.length, o);
      o->append(",\"queue_length\":");
      json::put_int(p.queue_length, o);
      if (p.next_id >= 0) {
        o->append(",\"next_id\":");
        json::put_int(p.next_id, o);
      }
      o->push_back('}');
    }
    o->push_back(']');
  }
  o->append("}}");
  return 200;
}

}  // namespace otm
