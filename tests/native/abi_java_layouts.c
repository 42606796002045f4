/*
 * The C ABI as the committed Java hosts bind it (integration/java: OtmMatcher.java and OtmBatcher.java through
 * FFM, OtmJni.java + integration/jni/otmatch_jni.c through JNI), exercised from C with no GPU:
 *
 *   layouts   every struct the Java MemoryLayouts describe, as {size, field offsets} -- tests/test_java_abi.py
 *             parses the Java layouts and compares them field by field;
 *   batcher   the raw-message topology the host drives (otm_formatter_create -> otm_batcher_create with a
 *             /report handler -> otm_batcher_process_raw per poll -> otm_batcher_take -> otm_batcher_close),
 *             with a C handler that answers every request {"shape_used":n-12}; the forwarded records are printed
 *             for the test to compare with the Python face of the same library calls;
 *   compact   an otm_batch_compact filled as OtmMatcher.matchCompact fills it, handed to otm_match_compact
 *             without an engine: the call must refuse it (OTM_EINVAL), touching nothing.
 *
 * Output: one JSON object on stdout.  Build: see tests/test_java_abi.py (gcc, -lotmatch).
 */
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "otmatch.h"

#define FIELD(s, f) printf("%s\"%s\":%zu", first++ ? "," : "", #f, offsetof(s, f))
#define BEGIN(s) \
  do {           \
    int first = 0; \
    printf("%s\"%s\":{\"size\":%zu,\"fields\":{", nstruct++ ? "," : "", #s, sizeof(s));
#define END() \
  printf("}}"); \
  } while (0)

static int nstruct = 0;

static void layouts(void) {
  printf("\"layouts\":{");
  BEGIN(otm_batch_compact);
  FIELD(otm_batch_compact, n_traces);
  FIELD(otm_batch_compact, n_points);
  FIELD(otm_batch_compact, trace_off);
  FIELD(otm_batch_compact, time_base);
  FIELD(otm_batch_compact, lat);
  FIELD(otm_batch_compact, lon);
  FIELD(otm_batch_compact, time_delta);
  FIELD(otm_batch_compact, accuracy);
  END();
  BEGIN(otm_results);
  FIELD(otm_results, n_traces);
  FIELD(otm_results, n_segments);
  FIELD(otm_results, n_reports);
  FIELD(otm_results, n_way_ids);
  FIELD(otm_results, traces);
  FIELD(otm_results, segments);
  FIELD(otm_results, reports);
  FIELD(otm_results, way_ids);
  END();
  BEGIN(otm_trace_result);
  FIELD(otm_trace_result, code);
  FIELD(otm_trace_result, error_kind);
  FIELD(otm_trace_result, seg_off);
  FIELD(otm_trace_result, seg_cnt);
  FIELD(otm_trace_result, rep_off);
  FIELD(otm_trace_result, rep_cnt);
  FIELD(otm_trace_result, shape_used);
  FIELD(otm_trace_result, successful_count);
  FIELD(otm_trace_result, unreported_count);
  FIELD(otm_trace_result, discontinuities);
  FIELD(otm_trace_result, invalid_speeds);
  FIELD(otm_trace_result, unassociated);
  FIELD(otm_trace_result, successful_length);
  FIELD(otm_trace_result, unreported_length);
  END();
  BEGIN(otm_segment);
  FIELD(otm_segment, segment_id);
  FIELD(otm_segment, start_time);
  FIELD(otm_segment, end_time);
  FIELD(otm_segment, length);
  FIELD(otm_segment, queue_length);
  FIELD(otm_segment, begin_shape_index);
  FIELD(otm_segment, end_shape_index);
  FIELD(otm_segment, way_off);
  FIELD(otm_segment, way_cnt);
  FIELD(otm_segment, flags);
  FIELD(otm_segment, pad);
  END();
  BEGIN(otm_report_rec);
  FIELD(otm_report_rec, id);
  FIELD(otm_report_rec, next_id);
  FIELD(otm_report_rec, t0);
  FIELD(otm_report_rec, t1);
  FIELD(otm_report_rec, length);
  FIELD(otm_report_rec, queue_length);
  FIELD(otm_report_rec, flags);
  FIELD(otm_report_rec, pad);
  END();
  BEGIN(otm_result);
  FIELD(otm_result, tag);
  FIELD(otm_result, code);
  FIELD(otm_result, body);
  FIELD(otm_result, body_len);
  END();
  BEGIN(otm_forward);
  FIELD(otm_forward, key);
  FIELD(otm_forward, key_len);
  FIELD(otm_forward, body);
  FIELD(otm_forward, body_len);
  FIELD(otm_forward, seq);
  END();
  BEGIN(otm_batcher_cfg);
  FIELD(otm_batcher_cfg, report_dist);
  FIELD(otm_batcher_cfg, report_count);
  FIELD(otm_batcher_cfg, report_time_s);
  FIELD(otm_batcher_cfg, session_gap_ms);
  FIELD(otm_batcher_cfg, max_batch);
  FIELD(otm_batcher_cfg, json_path);
  FIELD(otm_batcher_cfg, max_pending);
  FIELD(otm_batcher_cfg, threads);
  FIELD(otm_batcher_cfg, reserved);
  END();
  printf("}");
}

/* the /report handler: {"shape_used":max(0, n-12)} for a body of n points (n = occurrences of "lat"): batches
 * hover around 12 points, so the gated reports of process() pass and forward (clean() reports every record
 * older than the session gap, BatchingProcessor.java:88-104, and trims with the same rule) */
static int handler(void* ctx, int n, const char* const* reqs, const size_t* lens, char** resps, size_t* resp_lens,
                   int* codes) {
  int* calls = (int*)ctx;
  ++*calls;
  for (int i = 0; i < n; ++i) {
    int pts = 0;
    for (size_t k = 0; k + 5 <= lens[i]; ++k)
      if (memcmp(reqs[i] + k, "\"lat\"", 5) == 0) ++pts;
    char buf[64];
    const int len = snprintf(buf, sizeof buf, "{\"shape_used\":%d}", pts > 12 ? pts - 12 : 0);
    resps[i] = (char*)malloc((size_t)len + 1);
    if (!resps[i]) return 1;
    memcpy(resps[i], buf, (size_t)len + 1);
    resp_lens[i] = (size_t)len;
    codes[i] = 200;
  }
  return 0;
}

/* The messages: 6 vehicles x 48 points, 10 s apart, ~110 m per step, time-ordered, README's json layout, every
 * 37th message unparseable (dropped by the formatter); tests/test_java_abi.py rebuilds the same stream. */
#define NV 6
#define NP 48
static int make_stream(char* buf, size_t cap, int64_t* off, int64_t* ts) {
  size_t at = 0;
  int m = 0;
  for (int k = 0; k < NP; ++k)
    for (int v = 0; v < NV; ++v) {
      const long long t = 1500000000LL + 10LL * k + v;
      off[m] = (int64_t)at;
      int len;
      if (m % 37 == 36)
        len = snprintf(buf + at, cap - at, "not json %d", m);
      else
        len = snprintf(buf + at, cap - at,
                       "{\"timestamp\":%lld,\"id\":\"veh%d\",\"accuracy\":%d,\"latitude\":%.6f,\"longitude\":%.6f}", t,
                       v, 5 + v, 37.75 + 0.001 * k + 0.01 * v, -122.40 - 0.0005 * k);
      at += (size_t)len;
      ts[m] = t * 1000;
      ++m;
    }
  off[m] = (int64_t)at;
  return m;
}

static void batcher(void) {
  static char buf[1 << 16];
  int64_t off[NV * NP + 1], ts[NV * NP];
  const int n = make_stream(buf, sizeof buf, off, ts);
  char err[256] = {0};
  otm_formatter* f = NULL;
  if (otm_formatter_create(",json,id,latitude,longitude,timestamp,accuracy", &f, err, sizeof err) != OTM_OK) {
    printf(",\"batcher\":{\"error\":\"formatter: %s\"}", err);
    return;
  }
  otm_batcher_cfg cfg;
  otm_batcher_defaults(&cfg);
  cfg.threads = 3;
  int calls = 0;
  otm_batcher* b = NULL;
  if (otm_batcher_create(NULL, &cfg, handler, &calls, &b) != OTM_OK) {
    printf(",\"batcher\":{\"error\":\"create\"}");
    otm_formatter_destroy(f);
    return;
  }
  /* two polls, as the consumer loop delivers them */
  const int half = n / 2;
  int rc = otm_batcher_process_raw(b, f, half, buf, off, ts, 2);
  int64_t off2[NV * NP + 1];
  for (int i = half; i <= n; ++i) off2[i - half] = off[i] - off[half];
  if (rc == OTM_OK) rc = otm_batcher_process_raw(b, f, n - half, buf + off[half], off2, ts + half, 2);
  if (rc == OTM_OK) rc = otm_batcher_flush(b);
  printf(",\"batcher\":{\"rc\":%d,\"forwarded\":[", rc);
  otm_forward fw[64];
  int got, nf = 0;
  while ((got = otm_batcher_take(b, fw, 64)) > 0) {
    for (int i = 0; i < got; ++i) {
      printf("%s[%lld,\"%.*s\",\"", nf++ ? "," : "", (long long)fw[i].seq, (int)fw[i].key_len, fw[i].key);
      for (size_t k = 0; k < fw[i].body_len; ++k) {
        const char ch = fw[i].body[k];
        if (ch == '"' || ch == '\\') putchar('\\');
        putchar(ch);
      }
      printf("\"]");
      otm_free(fw[i].key);
      otm_free(fw[i].body);
    }
    if (got < 64) break;
  }
  const int crc = otm_batcher_close(b);
  otm_batcher_stats st;
  otm_batcher_get_stats(b, &st);
  printf("],\"close_rc\":%d,\"calls\":%d,\"stats\":{\"records\":%lld,\"requests\":%lld,\"raw_messages\":%lld,"
         "\"raw_dropped\":%lld,\"stored_batches\":%lld}}",
         crc, calls, (long long)st.records, (long long)st.requests, (long long)st.raw_messages,
         (long long)st.raw_dropped, (long long)st.stored_batches);
  otm_batcher_destroy(b);
  otm_formatter_destroy(f);
}

static void compact(void) {
  /* filled as OtmMatcher.matchCompact fills it: two traces of 3 and 2 points */
  int64_t trace_off[3] = {0, 3, 5}, time_base[2] = {1500000000, 1500000100};
  float lat[5] = {37.75f, 37.751f, 37.752f, 37.76f, 37.761f}, lon[5] = {-122.4f, -122.4f, -122.4f, -122.41f, -122.41f};
  int32_t dt[5] = {0, 5, 10, 0, 5};
  int16_t acc[5] = {5, 5, 5, 10, 10};
  otm_batch_compact in = {2, 5, trace_off, time_base, lat, lon, dt, acc};
  otm_results out;
  memset(&out, 0x5A, sizeof out);
  const int rc = otm_match_compact(NULL, &in, &out);
  printf(",\"compact\":{\"rc_without_engine\":%d}", rc);
}

int main(void) {
  printf("{");
  layouts();
  batcher();
  compact();
  printf("}\n");
  return 0;
}
