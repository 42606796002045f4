/*
 * orc_report.c -- oracle restatement of reporter_service.py's request path.
 * TEST INFRASTRUCTURE (see otm_oracle.h).
 *
 *   dom_report()      py/reporter_service.py:110-215 (report), over the parsed
 *                     Match output, with Python 3 value semantics (int/float/
 *                     bool/None/str arithmetic, comparisons and the exception
 *                     texts they raise).
 *   orc_handle_*      :85-106 parse_trace, :218-240 handle_request,
 *                     :259-264 do(): status codes and bodies.
 * Pinned by tests/golden/{report,request}_cases.json (reference run).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orc_json.h"
#include "orc_internal.h"
#include "otm_oracle.h"

/* ------------------------------------------------------------ py values */
typedef struct {
  int t; /* JV_* ; numbers carry i/d */
  int64_t i;
  double d;
  const jv* ref; /* non-number values */
  int bigint;
} pv;

static pv pv_of(const jv* v) {
  pv r;
  memset(&r, 0, sizeof r);
  if (!v) {
    r.t = JV_NULL;
    return r;
  }
  r.t = v->t;
  r.i = v->i;
  r.d = v->d;
  r.ref = v;
  r.bigint = v->bigint;
  return r;
}
static pv pv_int(int64_t i) {
  pv r;
  memset(&r, 0, sizeof r);
  r.t = JV_INT;
  r.i = i;
  return r;
}
static pv pv_flt(double d) {
  pv r;
  memset(&r, 0, sizeof r);
  r.t = JV_FLOAT;
  r.d = d;
  return r;
}
static const char* pv_tn(pv a) {
  if (a.t == JV_FLOAT && a.bigint) return "int";
  switch (a.t) {
    case JV_NULL: return "NoneType";
    case JV_BOOL: return "bool";
    case JV_INT: return "int";
    case JV_FLOAT: return "float";
    case JV_STR: return "str";
    case JV_ARR: return "list";
    default: return "dict";
  }
}
static int pv_isnum(pv a) { return a.t == JV_INT || a.t == JV_BOOL || a.t == JV_FLOAT; }
static int pv_isint(pv a) { return a.t == JV_INT || a.t == JV_BOOL || (a.t == JV_FLOAT && a.bigint); }
static double pv_dbl(pv a) { return a.t == JV_FLOAT ? a.d : (double)a.i; }

static char* fmt_err(const char* fmt, const char* a, const char* b) {
  char buf[256];
  snprintf(buf, sizeof buf, fmt, a, b);
  return strdup(buf);
}
static int pv_sub(pv a, pv b, pv* r, char** exc) {
  if (!pv_isnum(a) || !pv_isnum(b)) {
    *exc = fmt_err("unsupported operand type(s) for -: '%s' and '%s'", pv_tn(a), pv_tn(b));
    return 0;
  }
  if (pv_isint(a) && pv_isint(b) && !a.bigint && !b.bigint) *r = pv_int(a.i - b.i);
  else *r = pv_flt(pv_dbl(a) - pv_dbl(b));
  return 1;
}
static int pv_div(pv a, pv b, pv* r, char** exc) {
  if (!pv_isnum(a) || !pv_isnum(b)) {
    *exc = fmt_err("unsupported operand type(s) for /: '%s' and '%s'", pv_tn(a), pv_tn(b));
    return 0;
  }
  if (pv_dbl(b) == 0.0) {
    *exc = strdup(pv_isint(a) && pv_isint(b) ? "division by zero" : "float division by zero");
    return 0;
  }
  *r = pv_flt(pv_dbl(a) / pv_dbl(b));
  return 1;
}
static int pv_mulf(pv a, double f, pv* r, char** exc) {
  if (!pv_isnum(a)) {
    if (a.t == JV_STR || a.t == JV_ARR)
      *exc = fmt_err("can't multiply sequence by non-int of type '%s'%s", "float", "");
    else
      *exc = fmt_err("unsupported operand type(s) for *: '%s' and '%s'", pv_tn(a), "float");
    return 0;
  }
  *r = pv_flt(pv_dbl(a) * f);
  return 1;
}
/* a < b (op='<') or a > b (op='>') */
static int pv_cmp(pv a, pv b, char op, int* res, char** exc) {
  if (pv_isnum(a) && pv_isnum(b)) {
    if (pv_isint(a) && pv_isint(b) && !a.bigint && !b.bigint) *res = op == '<' ? a.i < b.i : a.i > b.i;
    else *res = op == '<' ? pv_dbl(a) < pv_dbl(b) : pv_dbl(a) > pv_dbl(b);
    return 1;
  }
  if (a.t == JV_STR && b.t == JV_STR) {
    int c = strcmp(a.ref->s, b.ref->s);
    *res = op == '<' ? c < 0 : c > 0;
    return 1;
  }
  char o[2] = {op, 0};
  char buf[256];
  snprintf(buf, sizeof buf, "'%s' not supported between instances of '%s' and '%s'", o, pv_tn(a), pv_tn(b));
  *exc = strdup(buf);
  return 0;
}
static int jv_eq(const jv* a, const jv* b);
static int pv_eq(pv a, pv b) {
  if (pv_isnum(a) && pv_isnum(b)) {
    if (pv_isint(a) && pv_isint(b) && !a.bigint && !b.bigint) return a.i == b.i;
    return pv_dbl(a) == pv_dbl(b);
  }
  if (a.t == JV_NULL || b.t == JV_NULL) return a.t == b.t;
  if (a.t != b.t) return 0;
  return jv_eq(a.ref, b.ref);
}
static int jv_eq(const jv* a, const jv* b) {
  if (a->t == JV_STR) return a->slen == b->slen && memcmp(a->s, b->s, a->slen) == 0;
  if (a->t == JV_ARR) {
    if (a->n != b->n) return 0;
    for (size_t k = 0; k < a->n; ++k)
      if (!pv_eq(pv_of(a->items[k]), pv_of(b->items[k]))) return 0;
    return 1;
  }
  if (a->t == JV_OBJ) {
    if (a->n != b->n) return 0;
    for (size_t k = 0; k < a->n; ++k) {
      const jv* o = jv_get(b, a->keys[k]);
      if (!o || !pv_eq(pv_of(a->items[k]), pv_of(o))) return 0;
    }
    return 1;
  }
  return pv_eq(pv_of(a), pv_of(b));
}
static int pv_truthy(pv a) {
  switch (a.t) {
    case JV_NULL: return 0;
    case JV_BOOL:
    case JV_INT: return a.i != 0;
    case JV_FLOAT: return a.d != 0.0;
    case JV_STR: return a.ref->slen != 0;
    default: return a.ref->n != 0;
  }
}
static const pv PV_TRUE = {JV_BOOL, 1, 0.0, NULL, 0};
static const pv PV_FALSE = {JV_BOOL, 0, 0.0, NULL, 0};

/* x[key] for a str key: value, or exception text */
static const jv* py_getitem(const jv* x, const char* key, char** exc) {
  if (!x || x->t == JV_NULL) {
    *exc = strdup("'NoneType' object is not subscriptable");
    return NULL;
  }
  if (x->t == JV_OBJ) {
    const jv* v = jv_get(x, key);
    if (!v) {
      char buf[256];
      snprintf(buf, sizeof buf, "'%s'", key);
      *exc = strdup(buf);
    }
    return v;
  }
  if (x->t == JV_ARR) *exc = strdup("list indices must be integers or slices, not str");
  else if (x->t == JV_STR) *exc = strdup("string indices must be integers");
  else *exc = fmt_err("'%s' object is not subscriptable%s", jv_typename(x), "");
  return NULL;
}
/* x.get(key[, default]) -- AttributeError for non-dicts */
static int py_get(const jv* x, const char* key, const jv** out, char** exc) {
  if (!x || x->t != JV_OBJ) {
    *exc = fmt_err("'%s' object has no attribute '%s'", x ? jv_typename(x) : "NoneType", "get");
    return 0;
  }
  *out = jv_get(x, key);
  return 1;
}
/* round(x, 3) for a float: correctly rounded decimal, back to the nearest double */
static double py_round3(double x) {
  if (!isfinite(x)) return x;
  char buf[400];
  snprintf(buf, sizeof buf, "%.3f", x);
  return strtod(buf, NULL);
}
static int in_levels(const int64_t* lv, int n, int64_t x) {
  for (int k = 0; k < n; ++k)
    if (lv[k] == x) return 1;
  return 0;
}

/* element k of a list-like, with Python's errors for the other containers */
static const jv* py_index(const jv* x, int64_t k, char** exc) {
  if (x->t == JV_ARR) return x->items[k];
  if (x->t == JV_OBJ) {
    char buf[64];
    snprintf(buf, sizeof buf, "%lld", (long long)k);
    *exc = strdup(buf);
    return NULL;
  }
  *exc = strdup("string indices must be integers");
  return NULL;
}

/* reporter_service.py:110-215.  Consumes nothing; `segments` is mutated
 * (segments['mode'] = 'auto').  Returns 1 with *out = response JSON, or 0
 * with *exc = str(exception). */
int dom_report(const orc_report_cfg* rc, const jv* trace, jv* segments, sbuf* out, sbuf* errs, char** exc) {
  /* :116 end_time = trace['trace'][len(trace['trace']) - 1]['time'] */
  const jv* tr = jv_get(trace, "trace");
  const jv* last_pt;
  if (tr->t == JV_ARR) {
    last_pt = tr->items[tr->n - 1];
  } else {
    *exc = strdup("string indices must be integers");
    return 0;
  }
  const jv* end_time_v = py_getitem(last_pt, "time", exc);
  if (!end_time_v) return 0;
  pv end_time = pv_of(end_time_v);
  /* :120 last_idx = len(segments['segments'])-1 */
  const jv* segs = py_getitem(segments, "segments", exc);
  if (!segs) return 0;
  int64_t nseg;
  if (segs->t == JV_ARR || segs->t == JV_OBJ) nseg = (int64_t)segs->n;
  else if (segs->t == JV_STR) {
    nseg = 0;
    for (size_t k = 0; k < segs->slen; ++k)
      if ((segs->s[k] & 0xC0) != 0x80) ++nseg;
  } else {
    *exc = fmt_err("object of type '%s' has no len()%s", jv_typename(segs), "");
    return 0;
  }
  int64_t last_idx = nseg - 1;
  pv thr = rc->threshold_sec == 15.0 ? pv_int(15) : (rc->threshold_sec != 0.0 ? PV_TRUE : PV_FALSE);
  /* :121-122 */
  while (last_idx >= 0) {
    const jv* s = py_index(segs, last_idx, exc);
    if (!s) return 0;
    const jv* st = py_getitem(s, "start_time", exc);
    if (!st) return 0;
    pv diff;
    int lt;
    if (!pv_sub(end_time, pv_of(st), &diff, exc)) return 0;
    if (!pv_cmp(diff, thr, '<', &lt, exc)) return 0;
    if (!lt) break;
    --last_idx;
  }
  /* :125-127 */
  const jv* shape_used = NULL;
  if (last_idx >= 0) {
    const jv* s = py_index(segs, last_idx, exc);
    if (!s) return 0;
    shape_used = py_getitem(s, "begin_shape_index", exc);
    if (!shape_used) return 0;
  }
  /* :131 */
  jv_set(segments, "mode", 4, jv_str("auto", 4));
  segs = jv_get(segments, "segments");
  /* :132-196 */
  int have_prior = 0;
  pv prior_id = {JV_NULL, 0, 0.0, NULL, 0};
  pv prior_start = prior_id, prior_end = prior_id, prior_len = prior_id,
     prior_ql = prior_id;
  int64_t prior_level = -1;
  int first_seg = 1;
  int64_t successful = 0, unreported = 0, disc = 0, invalid = 0, unassoc = 0;
  int succ_len_set = 0, unrep_len_set = 0;
  double succ_len = 0, unrep_len = 0;
  sbuf reps;
  sb_init(&reps);
  int nreps = 0;
  for (int64_t idx = 0; idx <= last_idx; ++idx) {
    const jv* seg = py_index(segs, idx, exc);
    if (!seg) goto fail;
    const jv *sid_v = NULL, *st_v = NULL, *et_v = NULL, *int_v = NULL, *ql_v = NULL, *len_v = NULL, *ways_v = NULL;
    if (!py_get(seg, "segment_id", &sid_v, exc)) goto fail;
    py_get(seg, "way_ids", &ways_v, exc);
    py_get(seg, "start_time", &st_v, exc);
    py_get(seg, "end_time", &et_v, exc);
    py_get(seg, "internal", &int_v, exc);
    py_get(seg, "queue_length", &ql_v, exc);
    py_get(seg, "length", &len_v, exc);
    (void)ways_v;
    pv segment_id = pv_of(sid_v), start_time = pv_of(st_v), end_time_s = pv_of(et_v);
    pv internal = int_v ? pv_of(int_v) : PV_FALSE, queue_length = pv_of(ql_v), length = pv_of(len_v);
    /* :150 */
    if (idx != 0) {
      const jv* a = py_getitem(seg, "start_time", exc);
      if (!a) goto fail;
      if (pv_eq(pv_of(a), pv_int(-1))) {
        const jv* prev = py_index(segs, idx - 1, exc);
        if (!prev) goto fail;
        const jv* b = py_getitem(prev, "end_time", exc);
        if (!b) goto fail;
        if (pv_eq(pv_of(b), pv_int(-1))) ++disc;
      }
    }
    /* :154 */
    int64_t level = -1;
    if (segment_id.t != JV_NULL) {
      if (!pv_isint(segment_id) || segment_id.bigint) {
        *exc = fmt_err("unsupported operand type(s) for &: '%s' and '%s'", pv_tn(segment_id), "int");
        goto fail;
      }
      level = segment_id.i & 0x7;
    }
    /* :157 */
    if (have_prior && prior_id.t != JV_NULL) {
      int gt;
      if (!pv_cmp(prior_len, pv_int(0), '>', &gt, exc)) goto fail;
      if (gt && !pv_eq(internal, PV_TRUE)) {
        if (in_levels(rc->report_levels, rc->n_report, prior_level)) {
          int trans = in_levels(rc->transition_levels, rc->n_transition, level);
          pv t1 = trans ? start_time : prior_end;
          pv diff, q, speed;
          if (!pv_sub(t1, prior_start, &diff, exc)) goto fail;
          if (!pv_div(prior_len, diff, &q, exc)) goto fail;
          if (!pv_mulf(q, 3.6, &speed, exc)) goto fail;
          int lt;
          if (!pv_cmp(speed, pv_int(200), '<', &lt, exc)) goto fail;
          if (lt) {
            /* {'id','t0','t1','length','queue_length'[,'next_id']} */
            sb_puts(&reps, nreps ? ",{\"id\":" : "{\"id\":");
            json_write(&reps, prior_id.ref);
            sb_puts(&reps, ",\"t0\":");
            json_write(&reps, prior_start.ref);
            sb_puts(&reps, ",\"t1\":");
            json_write(&reps, t1.ref);
            sb_puts(&reps, ",\"length\":");
            json_write(&reps, prior_len.ref);
            sb_puts(&reps, ",\"queue_length\":");
            json_write(&reps, prior_ql.ref);
            if (trans && segment_id.t != JV_NULL) {
              sb_puts(&reps, ",\"next_id\":");
              json_write(&reps, segment_id.ref);
            }
            sb_puts(&reps, "}");
            ++nreps;
            ++successful;
            pv km;
            pv_mulf(prior_len, 0.001, &km, exc);
            succ_len = py_round3(km.d);
            succ_len_set = 1;
          } else {
            sb_puts(errs, "Speed exceeds 200kph\n");
            ++invalid;
          }
        } else {
          ++unreported;
          pv km;
          pv_mulf(prior_len, 0.001, &km, exc);
          unrep_len = py_round3(km.d);
          unrep_len_set = 1;
        }
      }
    }
    /* :179-189 */
    if (pv_eq(internal, PV_TRUE) && !first_seg) {
      /* keep the prior */
    } else {
      prior_id = segment_id;
      prior_start = start_time;
      prior_end = end_time_s;
      prior_len = length;
      prior_level = level;
      prior_ql = queue_length;
      have_prior = 1;
    }
    first_seg = 0;
    /* :195 */
    if (segment_id.t == JV_NULL && pv_eq(internal, PV_FALSE)) ++unassoc;
  }
  /* :198-215 */
  sb_puts(out, "{\"stats\":{\"successful_matches\":{\"count\":");
  sb_printf(out, "%lld,\"length\":", (long long)successful);
  if (succ_len_set) py_float_repr(out, succ_len);
  else sb_puts(out, "0");
  sb_printf(out, "},\"unreported_matches\":{\"count\":%lld,\"length\":", (long long)unreported);
  if (unrep_len_set) py_float_repr(out, unrep_len);
  else sb_puts(out, "0");
  sb_printf(out,
            "},\"match_errors\":{\"discontinuities\":%lld,\"invalid_speeds\":%lld},\"unassociated_segments\":%lld}",
            (long long)disc, (long long)invalid, (long long)unassoc);
  if (shape_used && pv_truthy(pv_of(shape_used))) {
    sb_puts(out, ",\"shape_used\":");
    json_write(out, shape_used);
  }
  sb_puts(out, ",\"segment_matcher\":");
  json_write(out, segments);
  sb_puts(out, ",\"datastore\":{\"mode\":\"auto\"");
  if (nreps) {
    sb_puts(out, ",\"reports\":[");
    sb_put(out, reps.p, reps.len);
    sb_puts(out, "]");
  }
  sb_puts(out, "}}");
  free(reps.p);
  return 1;
fail:
  free(reps.p);
  return 0;
}

/* ------------------------------------------------------------ handle_request */
static char* errbody(const char* msg, size_t* n) {
  sbuf b;
  sb_init(&b);
  sb_puts(&b, "{\"error\":\"");
  sb_puts(&b, msg);
  sb_puts(&b, "\"}");
  *n = b.len;
  return b.p;
}
static char* rawbody(const char* msg, size_t* n) {
  *n = strlen(msg);
  return strdup(msg);
}

/* parse_trace + the validation of handle_request.  Returns 0 and *trace on
 * success, else the HTTP code with *out set. */
static int parse_and_validate(const char* path, const char* body, size_t len, jv** trace, char** out,
                              size_t* out_len) {
  /* :88-96 action = last path component */
  if (path) {
    size_t pl = strcspn(path, "?#");
    size_t a = pl;
    while (a > 0 && path[a - 1] != '/') --a;
    if (!(pl - a == 6 && memcmp(path + a, "report", 6) == 0)) {
      *out = errbody("Try a valid action: ['report']", out_len);
      return 400;
    }
  }
  /* :99-100 body.decode('utf-8'); json.loads */
  char* uerr = utf8_check((const unsigned char*)body, len);
  if (uerr) {
    *out = errbody(uerr, out_len);
    free(uerr);
    return 400;
  }
  char* perr;
  jv* t = json_parse(body, len, &perr);
  if (!t) {
    *out = errbody(perr, out_len);
    free(perr);
    return 400;
  }
  /* :226 trace.get('uuid') -- outside the try: do() answers 400 str(e) */
  if (t->t != JV_OBJ) {
    char buf[128];
    snprintf(buf, sizeof buf, "'%s' object has no attribute 'get'", jv_typename(t));
    *out = rawbody(buf, out_len);
    jv_free(t);
    return 400;
  }
  const jv* uuid = jv_get(t, "uuid");
  if (!uuid || uuid->t == JV_NULL) {
    *out = errbody("uuid is required", out_len);
    jv_free(t);
    return 400;
  }
  /* :231-234 trace['trace'][1] */
  const jv* tr = jv_get(t, "trace");
  int ok = 0;
  if (tr) {
    if (tr->t == JV_ARR) ok = tr->n >= 2;
    else if (tr->t == JV_STR) {
      size_t cps = 0;
      for (size_t k = 0; k < tr->slen; ++k)
        if ((tr->s[k] & 0xC0) != 0x80) ++cps;
      ok = cps >= 2;
    }
  }
  if (!ok) {
    *out = errbody(
        "trace must be a non zero length array of object each of which must have at least lat, lon and time",
        out_len);
    jv_free(t);
    return 400;
  }
  *trace = t;
  return 0;
}

int orc_report_segments(const orc_report_cfg* rc, const char* req, size_t len, const char* match_json,
                        size_t match_len, char** out, size_t* out_len, char** stderr_out) {
  jv* trace = NULL;
  *stderr_out = strdup("");
  int code = parse_and_validate("/report", req, len, &trace, out, out_len);
  if (code) return code;
  char* perr;
  jv* segs = json_parse(match_json, match_len, &perr);
  if (!segs) {
    *out = errbody(perr, out_len);
    free(perr);
    jv_free(trace);
    return 500;
  }
  sbuf o, e;
  sb_init(&o);
  sb_init(&e);
  char* exc = NULL;
  int ok = dom_report(rc, trace, segs, &o, &e, &exc);
  jv_free(segs);
  jv_free(trace);
  free(*stderr_out);
  *stderr_out = e.p;
  if (!ok) {
    free(o.p);
    *out = errbody(exc, out_len);
    free(exc);
    return 500;
  }
  *out = o.p;
  *out_len = o.len;
  return 200;
}

int orc_handle_request(const orc_graph* g, const orc_params* p, const orc_report_cfg* rc, const char* path,
                       const char* body, size_t len, char** out, size_t* out_len) {
  jv* trace = NULL;
  int code = parse_and_validate(path ? path : "/report", body, len, &trace, out, out_len);
  if (code) return code;
  /* :112 Match(json.dumps(trace)) -- the trace DOM carries the same values */
  char* merr = NULL;
  sbuf m;
  sb_init(&m);
  if (!orc_match_dom(g, p, trace, &m, &merr)) {
    free(m.p);
    *out = errbody(merr, out_len);
    free(merr);
    jv_free(trace);
    return 500;
  }
  char* perr;
  jv* segs = json_parse(m.p, m.len, &perr);
  free(m.p);
  sbuf o, e;
  sb_init(&o);
  sb_init(&e);
  char* exc = NULL;
  int ok = dom_report(rc, trace, segs, &o, &e, &exc);
  if (e.len) fputs(e.p, stderr);
  free(e.p);
  jv_free(segs);
  jv_free(trace);
  if (!ok) {
    free(o.p);
    *out = errbody(exc, out_len);
    free(exc);
    return 500;
  }
  *out = o.p;
  *out_len = o.len;
  return 200;
}

int orc_match_json(const orc_graph* g, const orc_params* p, const char* req, size_t len, char** out,
                   size_t* out_len) {
  char* perr;
  jv* t = json_parse(req, len, &perr);
  if (!t) {
    *out = errbody(perr, out_len);
    free(perr);
    return 500;
  }
  sbuf m;
  sb_init(&m);
  char* merr = NULL;
  int ok = t->t == JV_OBJ && orc_match_dom(g, p, t, &m, &merr);
  jv_free(t);
  if (!ok) {
    free(m.p);
    *out = errbody(merr ? merr : "request must be a JSON object", out_len);
    free(merr);
    return 500;
  }
  *out = m.p;
  *out_len = m.len;
  return 200;
}

int orc_json_redump(const char* s, size_t len, char** out, size_t* out_len) {
  char* perr;
  jv* v = json_parse(s, len, &perr);
  if (!v) {
    *out = perr;
    *out_len = strlen(perr);
    return 0;
  }
  sbuf b;
  sb_init(&b);
  json_write(&b, v);
  jv_free(v);
  *out = b.p;
  *out_len = b.len;
  return 1;
}
