/*
 * orc_json.c -- oracle JSON layer: a DOM with Python json semantics.
 * TEST INFRASTRUCTURE (see otm_oracle.h).
 *
 * Restates, for the bytes that reach reporter_service.py:
 *   json.loads  (CPython 3.10 json.decoder / json.scanner): value grammar,
 *               int-vs-float by the number's spelling, duplicate keys keep the
 *               first position with the last value, and the exact
 *               JSONDecodeError texts ("Expecting value: line L column C
 *               (char N)" ...), positions counted in code points.
 *   json.dumps(x, separators=(',', ':')) with ensure_ascii: float repr
 *               (shortest round-trip; exponent when decpt < -3 or > 16),
 *               \uXXXX escapes.
 * A small value model (int / float / bool / None / str / list / dict) with
 * the Python 3 operator semantics report() relies on lives in orc_report.c.
 */
#include "orc_json.h"

#include <ctype.h>
#include <errno.h>
#include <limits.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ buffer */
void sb_init(sbuf* b) {
  b->cap = 256;
  b->len = 0;
  b->p = (char*)malloc(b->cap);
  b->p[0] = 0;
}
void sb_put(sbuf* b, const char* s, size_t n) {
  if (b->len + n + 1 > b->cap) {
    while (b->len + n + 1 > b->cap) b->cap *= 2;
    b->p = (char*)realloc(b->p, b->cap);
  }
  memcpy(b->p + b->len, s, n);
  b->len += n;
  b->p[b->len] = 0;
}
void sb_puts(sbuf* b, const char* s) { sb_put(b, s, strlen(s)); }
void sb_printf(sbuf* b, const char* fmt, ...) {
  char tmp[512];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(tmp, sizeof tmp, fmt, ap);
  va_end(ap);
  if (n < (int)sizeof tmp) {
    sb_put(b, tmp, (size_t)n);
    return;
  }
  char* big = (char*)malloc((size_t)n + 1);
  va_start(ap, fmt);
  vsnprintf(big, (size_t)n + 1, fmt, ap);
  va_end(ap);
  sb_put(b, big, (size_t)n);
  free(big);
}

/* ------------------------------------------------------------------ values */
jv* jv_new(int t) {
  jv* v = (jv*)calloc(1, sizeof(jv));
  v->t = t;
  return v;
}
jv* jv_int(int64_t i) {
  jv* v = jv_new(JV_INT);
  v->i = i;
  return v;
}
jv* jv_float(double d) {
  jv* v = jv_new(JV_FLOAT);
  v->d = d;
  return v;
}
jv* jv_bool(int b) {
  jv* v = jv_new(JV_BOOL);
  v->i = b ? 1 : 0;
  return v;
}
jv* jv_str(const char* s, size_t n) {
  jv* v = jv_new(JV_STR);
  v->s = (char*)malloc(n + 1);
  memcpy(v->s, s, n);
  v->s[n] = 0;
  v->slen = n;
  return v;
}
void jv_free(jv* v) {
  if (!v) return;
  if (v->t == JV_STR || v->bigint) free(v->s);
  for (size_t k = 0; k < v->n; ++k) {
    jv_free(v->items[k]);
    if (v->keys) free(v->keys[k]);
  }
  free(v->items);
  free(v->keys);
  free(v->klens);
  free(v);
}
static void jv_grow(jv* v) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 4;
    v->items = (jv**)realloc(v->items, v->cap * sizeof(jv*));
    if (v->t == JV_OBJ) {
      v->keys = (char**)realloc(v->keys, v->cap * sizeof(char*));
      v->klens = (size_t*)realloc(v->klens, v->cap * sizeof(size_t));
    }
  }
}
void jv_push(jv* arr, jv* x) {
  jv_grow(arr);
  arr->items[arr->n++] = x;
}
/* dict.__setitem__: replaces in place if the key exists */
void jv_set(jv* obj, const char* k, size_t kn, jv* x) {
  for (size_t i = 0; i < obj->n; ++i)
    if (obj->klens[i] == kn && memcmp(obj->keys[i], k, kn) == 0) {
      jv_free(obj->items[i]);
      obj->items[i] = x;
      return;
    }
  jv_grow(obj);
  obj->keys[obj->n] = (char*)malloc(kn + 1);
  memcpy(obj->keys[obj->n], k, kn);
  obj->keys[obj->n][kn] = 0;
  obj->klens[obj->n] = kn;
  obj->items[obj->n++] = x;
}
jv* jv_get(const jv* obj, const char* k) {
  if (!obj || obj->t != JV_OBJ) return NULL;
  size_t kn = strlen(k);
  for (size_t i = 0; i < obj->n; ++i)
    if (obj->klens[i] == kn && memcmp(obj->keys[i], k, kn) == 0) return obj->items[i];
  return NULL;
}
void jv_del(jv* obj, const char* k) {
  size_t kn = strlen(k);
  for (size_t i = 0; i < obj->n; ++i)
    if (obj->klens[i] == kn && memcmp(obj->keys[i], k, kn) == 0) {
      jv_free(obj->items[i]);
      free(obj->keys[i]);
      memmove(obj->items + i, obj->items + i + 1, (obj->n - i - 1) * sizeof(jv*));
      memmove(obj->keys + i, obj->keys + i + 1, (obj->n - i - 1) * sizeof(char*));
      memmove(obj->klens + i, obj->klens + i + 1, (obj->n - i - 1) * sizeof(size_t));
      obj->n--;
      return;
    }
}
const char* jv_typename(const jv* v) {
  if (!v) return "NoneType";
  switch (v->t) {
    case JV_NULL: return "NoneType";
    case JV_BOOL: return "bool";
    case JV_INT: return "int";
    case JV_FLOAT: return "float";
    case JV_STR: return "str";
    case JV_ARR: return "list";
    default: return "dict";
  }
}

/* ------------------------------------------------------------------ parser */
typedef struct {
  const unsigned char* s;
  size_t n, i;
  char* err; /* malloc'd message on failure */
} jp;

/* code-point index of byte offset b (UTF-8 already validated) */
static size_t cp_index(const jp* p, size_t b) {
  size_t c = 0;
  for (size_t k = 0; k < b && k < p->n; ++k)
    if ((p->s[k] & 0xC0) != 0x80) ++c;
  return c;
}
static void jp_fail(jp* p, const char* what, size_t at) {
  if (p->err) return;
  size_t pos = cp_index(p, at);
  size_t line = 1, last_nl_cp = (size_t)-1, cp = 0;
  for (size_t k = 0; k < at && k < p->n; ++k) {
    if ((p->s[k] & 0xC0) != 0x80) {
      if (p->s[k] == '\n') {
        ++line;
        last_nl_cp = cp;
      }
      ++cp;
    }
  }
  size_t col = last_nl_cp == (size_t)-1 ? pos + 1 : pos - last_nl_cp;
  char buf[256];
  snprintf(buf, sizeof buf, "%s: line %zu column %zu (char %zu)", what, line, col, pos);
  p->err = strdup(buf);
}
static void ws(jp* p) {
  while (p->i < p->n && (p->s[p->i] == ' ' || p->s[p->i] == '\t' || p->s[p->i] == '\n' || p->s[p->i] == '\r'))
    ++p->i;
}
static jv* parse_value(jp* p, int depth);

static int hexv(int c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}
static void put_utf8(sbuf* b, unsigned cp) {
  char t[4];
  if (cp < 0x80) {
    t[0] = (char)cp;
    sb_put(b, t, 1);
  } else if (cp < 0x800) {
    t[0] = (char)(0xC0 | (cp >> 6));
    t[1] = (char)(0x80 | (cp & 63));
    sb_put(b, t, 2);
  } else if (cp < 0x10000) {
    t[0] = (char)(0xE0 | (cp >> 12));
    t[1] = (char)(0x80 | ((cp >> 6) & 63));
    t[2] = (char)(0x80 | (cp & 63));
    sb_put(b, t, 3);
  } else {
    t[0] = (char)(0xF0 | (cp >> 18));
    t[1] = (char)(0x80 | ((cp >> 12) & 63));
    t[2] = (char)(0x80 | ((cp >> 6) & 63));
    t[3] = (char)(0x80 | (cp & 63));
    sb_put(b, t, 4);
  }
}
/* p->i at the opening quote */
static jv* parse_string(jp* p) {
  size_t start = p->i;
  ++p->i;
  sbuf b;
  sb_init(&b);
  while (1) {
    if (p->i >= p->n) {
      jp_fail(p, "Unterminated string starting at", start);
      free(b.p);
      return NULL;
    }
    unsigned char c = p->s[p->i];
    if (c == '"') {
      ++p->i;
      break;
    }
    if (c < 0x20) {
      jp_fail(p, "Invalid control character at", p->i);
      free(b.p);
      return NULL;
    }
    if (c != '\\') {
      sb_put(&b, (const char*)&p->s[p->i], 1);
      ++p->i;
      continue;
    }
    if (p->i + 1 >= p->n) {
      jp_fail(p, "Unterminated string starting at", start);
      free(b.p);
      return NULL;
    }
    unsigned char e = p->s[p->i + 1];
    const char* rep = NULL;
    switch (e) {
      case '"': rep = "\""; break;
      case '\\': rep = "\\"; break;
      case '/': rep = "/"; break;
      case 'b': rep = "\b"; break;
      case 'f': rep = "\f"; break;
      case 'n': rep = "\n"; break;
      case 'r': rep = "\r"; break;
      case 't': rep = "\t"; break;
    }
    if (rep) {
      sb_put(&b, rep, 1);
      p->i += 2;
      continue;
    }
    if (e != 'u') {
      jp_fail(p, "Invalid \\escape", p->i);
      free(b.p);
      return NULL;
    }
    /* \uXXXX (+ surrogate pair) */
    unsigned cp = 0;
    int ok = p->i + 6 <= p->n;
    for (int k = 0; ok && k < 4; ++k) {
      int h = hexv(p->s[p->i + 2 + k]);
      if (h < 0) ok = 0;
      else cp = cp * 16 + (unsigned)h;
    }
    if (!ok) {
      jp_fail(p, "Invalid \\uXXXX escape", p->i + 1);
      free(b.p);
      return NULL;
    }
    p->i += 6;
    if (cp >= 0xD800 && cp <= 0xDBFF && p->i + 6 <= p->n && p->s[p->i] == '\\' && p->s[p->i + 1] == 'u') {
      unsigned lo = 0;
      int ok2 = 1;
      for (int k = 0; k < 4; ++k) {
        int h = hexv(p->s[p->i + 2 + k]);
        if (h < 0) ok2 = 0;
        else lo = lo * 16 + (unsigned)h;
      }
      if (!ok2) {
        jp_fail(p, "Invalid \\uXXXX escape", p->i + 1);
        free(b.p);
        return NULL;
      }
      if (lo >= 0xDC00 && lo <= 0xDFFF) {
        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
        p->i += 6;
      }
    }
    put_utf8(&b, cp);
  }
  jv* v = jv_str(b.p, b.len);
  free(b.p);
  return v;
}

static jv* parse_number(jp* p) {
  size_t a = p->i, k = p->i;
  if (k < p->n && p->s[k] == '-') ++k;
  if (k >= p->n || !isdigit(p->s[k])) return NULL; /* caller reports */
  if (p->s[k] == '0') ++k;
  else
    while (k < p->n && isdigit(p->s[k])) ++k;
  int is_float = 0;
  if (k + 1 < p->n && p->s[k] == '.' && isdigit(p->s[k + 1])) {
    is_float = 1;
    k += 1;
    while (k < p->n && isdigit(p->s[k])) ++k;
  }
  if (k < p->n && (p->s[k] == 'e' || p->s[k] == 'E')) {
    size_t m = k + 1;
    if (m < p->n && (p->s[m] == '+' || p->s[m] == '-')) ++m;
    if (m < p->n && isdigit(p->s[m])) {
      is_float = 1;
      k = m;
      while (k < p->n && isdigit(p->s[k])) ++k;
    }
  }
  char tmp[400];
  size_t len = k - a;
  char* buf = len < sizeof tmp ? tmp : (char*)malloc(len + 1);
  memcpy(buf, p->s + a, len);
  buf[len] = 0;
  jv* v;
  if (is_float) {
    v = jv_float(strtod(buf, NULL));
  } else {
    /* Python ints are unbounded; int64 covers every id/time/length here.
       A longer int keeps its digits verbatim (dumps writes them back) and
       takes part in arithmetic as a float. */
    errno = 0;
    long long ll = strtoll(buf, NULL, 10);
    if (errno == ERANGE) {
      v = jv_float(strtod(buf, NULL));
      v->bigint = 1;
      v->s = strdup(buf[0] == '-' && 0 ? buf : buf);
      v->slen = strlen(buf);
    } else {
      v = jv_int(ll);
    }
  }
  if (buf != tmp) free(buf);
  p->i = k;
  return v;
}

static int lit(jp* p, const char* w) {
  size_t n = strlen(w);
  return p->i + n <= p->n && memcmp(p->s + p->i, w, n) == 0;
}

static jv* parse_value(jp* p, int depth) {
  if (depth > 900) {
    jp_fail(p, "Expecting value", p->i);
    return NULL;
  }
  if (p->i >= p->n) {
    jp_fail(p, "Expecting value", p->i);
    return NULL;
  }
  unsigned char c = p->s[p->i];
  if (c == '"') return parse_string(p);
  if (c == '{') {
    size_t start = p->i;
    (void)start;
    ++p->i;
    jv* o = jv_new(JV_OBJ);
    ws(p);
    if (p->i < p->n && p->s[p->i] == '}') {
      ++p->i;
      return o;
    }
    while (1) {
      if (p->i >= p->n || p->s[p->i] != '"') {
        jp_fail(p, "Expecting property name enclosed in double quotes", p->i);
        jv_free(o);
        return NULL;
      }
      jv* k = parse_string(p);
      if (!k) {
        jv_free(o);
        return NULL;
      }
      ws(p);
      if (p->i >= p->n || p->s[p->i] != ':') {
        jp_fail(p, "Expecting ':' delimiter", p->i);
        jv_free(k);
        jv_free(o);
        return NULL;
      }
      ++p->i;
      ws(p);
      jv* x = parse_value(p, depth + 1);
      if (!x) {
        jv_free(k);
        jv_free(o);
        return NULL;
      }
      jv_set(o, k->s, k->slen, x);
      jv_free(k);
      ws(p);
      if (p->i < p->n && p->s[p->i] == '}') {
        ++p->i;
        return o;
      }
      if (p->i >= p->n || p->s[p->i] != ',') {
        jp_fail(p, "Expecting ',' delimiter", p->i);
        jv_free(o);
        return NULL;
      }
      ++p->i;
      ws(p);
    }
  }
  if (c == '[') {
    ++p->i;
    jv* a = jv_new(JV_ARR);
    ws(p);
    if (p->i < p->n && p->s[p->i] == ']') {
      ++p->i;
      return a;
    }
    while (1) {
      jv* x = parse_value(p, depth + 1);
      if (!x) {
        jv_free(a);
        return NULL;
      }
      jv_push(a, x);
      ws(p);
      if (p->i < p->n && p->s[p->i] == ']') {
        ++p->i;
        return a;
      }
      if (p->i >= p->n || p->s[p->i] != ',') {
        jp_fail(p, "Expecting ',' delimiter", p->i);
        jv_free(a);
        return NULL;
      }
      ++p->i;
      ws(p);
    }
  }
  if (lit(p, "null")) {
    p->i += 4;
    return jv_new(JV_NULL);
  }
  if (lit(p, "true")) {
    p->i += 4;
    return jv_bool(1);
  }
  if (lit(p, "false")) {
    p->i += 5;
    return jv_bool(0);
  }
  if (lit(p, "NaN")) {
    p->i += 3;
    return jv_float(NAN);
  }
  if (lit(p, "Infinity")) {
    p->i += 8;
    return jv_float(INFINITY);
  }
  if (lit(p, "-Infinity")) {
    p->i += 9;
    return jv_float(-INFINITY);
  }
  jv* num = parse_number(p);
  if (num) return num;
  jp_fail(p, "Expecting value", p->i);
  return NULL;
}

/* bytes.decode('utf-8') error text, or NULL when valid */
char* utf8_check(const unsigned char* s, size_t n) {
  size_t i = 0;
  char buf[160];
  while (i < n) {
    unsigned char c = s[i];
    if (c < 0x80) {
      ++i;
      continue;
    }
    int need;
    unsigned lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) need = 2, lo = 0xA0;
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) need = 2, hi = 0x9F;
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) need = 3, lo = 0x90;
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) need = 3, hi = 0x8F;
    else {
      snprintf(buf, sizeof buf, "'utf-8' codec can't decode byte 0x%02x in position %zu: invalid start byte", c, i);
      return strdup(buf);
    }
    size_t k = 1;
    for (; k <= (size_t)need; ++k) {
      if (i + k >= n) {
        if (k == 1)
          snprintf(buf, sizeof buf, "'utf-8' codec can't decode byte 0x%02x in position %zu: unexpected end of data",
                   c, i);
        else
          snprintf(buf, sizeof buf, "'utf-8' codec can't decode bytes in position %zu-%zu: unexpected end of data", i,
                   i + k - 1);
        return strdup(buf);
      }
      unsigned char d = s[i + k];
      unsigned l = k == 1 ? lo : 0x80, h = k == 1 ? hi : 0xBF;
      if (d < l || d > h) {
        if (k == 1)
          snprintf(buf, sizeof buf,
                   "'utf-8' codec can't decode byte 0x%02x in position %zu: invalid continuation byte", c, i);
        else
          snprintf(buf, sizeof buf,
                   "'utf-8' codec can't decode bytes in position %zu-%zu: invalid continuation byte", i, i + k - 1);
        return strdup(buf);
      }
    }
    i += (size_t)need + 1;
  }
  return NULL;
}

jv* json_parse(const char* s, size_t n, char** err) {
  jp p = {(const unsigned char*)s, n, 0, NULL};
  *err = NULL;
  ws(&p);
  jv* v = parse_value(&p, 0);
  if (v) {
    ws(&p);
    if (p.i != p.n) {
      jp_fail(&p, "Extra data", p.i);
      jv_free(v);
      v = NULL;
    }
  }
  if (!v) *err = p.err ? p.err : strdup("Expecting value: line 1 column 1 (char 0)");
  return v;
}

/* ------------------------------------------------------------------ writer */
/* Python float repr: shortest round-trip digits (the correctly rounded
 * p-digit decimal for the smallest p that round-trips), then
 * float_repr_style 'short' layout. */
void py_float_repr(sbuf* b, double d) {
  if (isnan(d)) {
    sb_puts(b, "NaN");
    return;
  }
  if (isinf(d)) {
    sb_puts(b, d > 0 ? "Infinity" : "-Infinity");
    return;
  }
  if (d == 0.0) {
    sb_puts(b, signbit(d) ? "-0.0" : "0.0");
    return;
  }
  char tmp[64];
  int prec;
  for (prec = 1; prec <= 17; ++prec) {
    snprintf(tmp, sizeof tmp, "%.*e", prec - 1, d);
    if (strtod(tmp, NULL) == d) break;
  }
  /* tmp = [-]D.DDDDe[+-]XX */
  const char* q = tmp;
  int neg = 0;
  if (*q == '-') {
    neg = 1;
    ++q;
  }
  char digits[32];
  int nd = 0;
  while (*q && *q != 'e') {
    if (*q != '.') digits[nd++] = *q;
    ++q;
  }
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  int e10 = atoi(q + 1);
  int decpt = e10 + 1; /* value = 0.DIGITS * 10^decpt */
  if (neg) sb_put(b, "-", 1);
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      sb_puts(b, "0.");
      for (int k = 0; k < -decpt; ++k) sb_put(b, "0", 1);
      sb_put(b, digits, (size_t)nd);
    } else if (decpt >= nd) {
      sb_put(b, digits, (size_t)nd);
      for (int k = nd; k < decpt; ++k) sb_put(b, "0", 1);
      sb_puts(b, ".0");
    } else {
      sb_put(b, digits, (size_t)decpt);
      sb_put(b, ".", 1);
      sb_put(b, digits + decpt, (size_t)(nd - decpt));
    }
  } else {
    sb_put(b, digits, 1);
    if (nd > 1) {
      sb_put(b, ".", 1);
      sb_put(b, digits + 1, (size_t)(nd - 1));
    }
    int x = decpt - 1;
    sb_printf(b, "e%c%02d", x < 0 ? '-' : '+', x < 0 ? -x : x);
  }
}

static void write_str(sbuf* b, const char* s, size_t n) {
  sb_put(b, "\"", 1);
  const unsigned char* u = (const unsigned char*)s;
  for (size_t i = 0; i < n;) {
    unsigned c = u[i];
    if (c == '"') {
      sb_puts(b, "\\\"");
      ++i;
    } else if (c == '\\') {
      sb_puts(b, "\\\\");
      ++i;
    } else if (c == '\n') {
      sb_puts(b, "\\n");
      ++i;
    } else if (c == '\r') {
      sb_puts(b, "\\r");
      ++i;
    } else if (c == '\t') {
      sb_puts(b, "\\t");
      ++i;
    } else if (c == '\b') {
      sb_puts(b, "\\b");
      ++i;
    } else if (c == '\f') {
      sb_puts(b, "\\f");
      ++i;
    } else if (c >= 0x20 && c < 0x7f) {
      sb_put(b, (const char*)&u[i], 1);
      ++i;
    } else if (c < 0x80) {
      sb_printf(b, "\\u%04x", c);
      ++i;
    } else {
      unsigned cp;
      int len;
      if ((c & 0xE0) == 0xC0) cp = c & 31, len = 2;
      else if ((c & 0xF0) == 0xE0) cp = c & 15, len = 3;
      else cp = c & 7, len = 4;
      for (int k = 1; k < len && i + (size_t)k < n; ++k) cp = (cp << 6) | (u[i + k] & 63);
      i += (size_t)len;
      if (cp >= 0x10000) {
        cp -= 0x10000;
        sb_printf(b, "\\u%04x\\u%04x", 0xD800 + (cp >> 10), 0xDC00 + (cp & 0x3FF));
      } else {
        sb_printf(b, "\\u%04x", cp);
      }
    }
  }
  sb_put(b, "\"", 1);
}

void json_write(sbuf* b, const jv* v) {
  if (!v || v->t == JV_NULL) {
    sb_puts(b, "null");
    return;
  }
  switch (v->t) {
    case JV_BOOL: sb_puts(b, v->i ? "true" : "false"); break;
    case JV_INT: sb_printf(b, "%lld", (long long)v->i); break;
    case JV_FLOAT:
      if (v->bigint) {
        sb_put(b, v->s, v->slen);
      } else {
        py_float_repr(b, v->d);
      }
      break;
    case JV_STR: write_str(b, v->s, v->slen); break;
    case JV_ARR:
      sb_put(b, "[", 1);
      for (size_t k = 0; k < v->n; ++k) {
        if (k) sb_put(b, ",", 1);
        json_write(b, v->items[k]);
      }
      sb_put(b, "]", 1);
      break;
    case JV_OBJ:
      sb_put(b, "{", 1);
      for (size_t k = 0; k < v->n; ++k) {
        if (k) sb_put(b, ",", 1);
        write_str(b, v->keys[k], v->klens[k]);
        sb_put(b, ":", 1);
        json_write(b, v->items[k]);
      }
      sb_put(b, "}", 1);
      break;
  }
}
