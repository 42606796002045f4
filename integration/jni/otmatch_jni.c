/*
 * otmatch_jni.c -- JNI shim for the reference's Java 8 target (pom.xml), which has no FFM.
 *
 * Binds org.opentraffic.reporter.OtmJni (integration/java/.../OtmJni.java) to libotmatch.so.  OtmJni.POST
 * replaces HttpClient.POST at Batch.java:63 with the same contract: the body reporter_service.py would
 * answer (any status), or null when the call itself fails (HttpClient.java:37-39).  The String <-> bytes
 * steps stay in Java (OtmJni.POST), in HttpClient's charsets: ISO-8859-1 out, UTF-8 back.
 *
 * Build (needs a JDK, absent from this image):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *       otmatch_jni.c -L../../reporter_amd/lib -lotmatch -o libotmatch_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "otmatch.h"

static otm_engine* g_eng;

JNIEXPORT void JNICALL Java_org_opentraffic_reporter_OtmJni_init(JNIEnv* env, jclass c, jstring cfg, jint dev) {
  (void)c;
  const char* p = (*env)->GetStringUTFChars(env, cfg, 0);
  int d = dev;
  /* valhalla.Configure (py/reporter_service.py:279) + SegmentMatcher() (:52) */
  if (otm_engine_create(p, &d, 1, &g_eng) != OTM_OK)
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/IllegalStateException"), otm_last_error(NULL));
  (*env)->ReleaseStringUTFChars(env, cfg, p);
}

/* OtmJni.report(byte[]): the request bytes as HttpClient would send them (OtmJni.POST encodes the String
 * with ISO-8859-1 first, as new StringEntity(body) does, HttpClient.java:26), the response bytes back; the
 * Java side decodes them as UTF-8 (HttpClient.java:33).  null when the call itself fails. */
JNIEXPORT jbyteArray JNICALL Java_org_opentraffic_reporter_OtmJni_report(JNIEnv* env, jclass c, jbyteArray body) {
  (void)c;
  if (!g_eng || !body) return NULL;
  jsize n = (*env)->GetArrayLength(env, body);
  jbyte* b = (*env)->GetByteArrayElements(env, body, NULL);
  if (!b) return NULL;
  char* resp = NULL;
  size_t rn = 0;
  otm_report(g_eng, (const char*)b, (size_t)n, &resp, &rn);
  (*env)->ReleaseByteArrayElements(env, body, b, JNI_ABORT);
  if (!resp) return NULL;
  jbyteArray out = (*env)->NewByteArray(env, (jsize)rn);
  if (out) (*env)->SetByteArrayRegion(env, out, 0, (jsize)rn, (const jbyte*)resp);
  otm_free(resp);
  return out;
}

/* OtmJni.arenaAlloc(long): a library-owned page-locked request arena (otm_request_arena_alloc) as a
 * direct ByteBuffer the Java side writes its request bytes into. */
JNIEXPORT jobject JNICALL Java_org_opentraffic_reporter_OtmJni_arenaAlloc(JNIEnv* env, jclass c, jlong bytes) {
  (void)c;
  void* p = otm_request_arena_alloc((size_t)(bytes > 0 ? bytes : 1));
  return p ? (*env)->NewDirectByteBuffer(env, p, bytes > 0 ? bytes : 1) : NULL;
}

JNIEXPORT void JNICALL Java_org_opentraffic_reporter_OtmJni_arenaRelease(JNIEnv* env, jclass c, jobject arena) {
  (void)c;
  if (arena) otm_request_arena_release((*env)->GetDirectBufferAddress(env, arena));
}

/* OtmJni.reportBatch(ByteBuffer arena, long[] off): body i = arena[off[i], off[i+1]), sent to HBM straight
 * from the arena by otm_report_batch; the response bytes back per body (null where the call failed).  The
 * offsets must be monotonic and inside the buffer (else null: nothing is read past it); the result array stops
 * at the first allocation that fails (its Java exception is left pending, as JNI requires). */
JNIEXPORT jobjectArray JNICALL Java_org_opentraffic_reporter_OtmJni_reportBatch(JNIEnv* env, jclass c,
                                                                              jobject arena, jlongArray off) {
  (void)c;
  if (!g_eng || !arena || !off) return NULL;
  const char* base = (const char*)(*env)->GetDirectBufferAddress(env, arena);
  const jlong cap = (*env)->GetDirectBufferCapacity(env, arena);
  const jsize n = (*env)->GetArrayLength(env, off) - 1;
  if (!base || cap < 0 || n < 0) return NULL;
  jlong* o = (*env)->GetLongArrayElements(env, off, NULL);
  if (!o) return NULL;
  for (jsize i = 0; i < n; ++i)
    if (o[i] < 0 || o[i] > o[i + 1] || o[i + 1] > cap) {
      (*env)->ReleaseLongArrayElements(env, off, o, JNI_ABORT);
      return NULL;
    }
  const char** reqs = (const char**)malloc(sizeof(char*) * (size_t)(n ? n : 1));
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)(n ? n : 1));
  char** resps = (char**)calloc((size_t)(n ? n : 1), sizeof(char*));
  size_t* rlens = (size_t*)calloc((size_t)(n ? n : 1), sizeof(size_t));
  int* codes = (int*)calloc((size_t)(n ? n : 1), sizeof(int));
  jobjectArray out = NULL;
  if (reqs && lens && resps && rlens && codes) {
    for (jsize i = 0; i < n; ++i) {
      reqs[i] = base + o[i];
      lens[i] = (size_t)(o[i + 1] - o[i]);
    }
    const int rc = otm_report_batch(g_eng, (int)n, reqs, lens, resps, rlens, codes);
    const jclass bytes = (*env)->FindClass(env, "[B");
    if (bytes) out = (*env)->NewObjectArray(env, n, bytes, NULL);
    int ok = out != NULL;
    for (jsize i = 0; i < n; ++i) {
      if (ok && rc == OTM_OK && resps[i]) {
        jbyteArray b = (*env)->NewByteArray(env, (jsize)rlens[i]);
        if (!b || (*env)->ExceptionCheck(env)) {
          ok = 0;  /* an OutOfMemoryError is pending: no further JNI calls but releases */
        } else {
          (*env)->SetByteArrayRegion(env, b, 0, (jsize)rlens[i], (const jbyte*)resps[i]);
          (*env)->SetObjectArrayElement(env, out, i, b);
          (*env)->DeleteLocalRef(env, b);
        }
      }
      otm_free(resps[i]);
    }
    if (!ok) out = NULL;
  }
  (*env)->ReleaseLongArrayElements(env, off, o, JNI_ABORT);
  free(reqs);
  free(lens);
  free(resps);
  free(rlens);
  free(codes);
  return out;
}

/* OtmJni.matchCompact(nTraces, nPoints, traceOff, timeBase, lat, lon, timeDelta, accuracy): otm_match_compact
 * over direct buffers in the host's native byte order (Point.java's float lat/lon, an int32 time delta from the
 * trace's int64 base, an int16 accuracy; include/otmatch.h otm_batch_compact).  Returns four direct buffers over
 * the engine's result arrays -- otm_trace_result[n_traces], otm_segment[], otm_report_rec[], int64 way ids[] --
 * valid until the engine's next call (copy what is kept), or null when the call fails. */
JNIEXPORT jobjectArray JNICALL Java_org_opentraffic_reporter_OtmJni_matchCompact(
    JNIEnv* env, jclass c, jint n_traces, jlong n_points, jobject trace_off, jobject time_base, jobject lat,
    jobject lon, jobject time_delta, jobject accuracy) {
  (void)c;
  if (!g_eng || n_traces < 0 || n_points < 0) return NULL;
  const jobject bufs[6] = {trace_off, time_base, lat, lon, time_delta, accuracy};
  const jlong need[6] = {8 * ((jlong)n_traces + 1), 8 * (jlong)n_traces, 4 * n_points, 4 * n_points, 4 * n_points,
                         2 * n_points};
  void* ptr[6];
  for (int k = 0; k < 6; ++k) {
    ptr[k] = bufs[k] ? (*env)->GetDirectBufferAddress(env, bufs[k]) : NULL;
    if (!ptr[k] || (*env)->GetDirectBufferCapacity(env, bufs[k]) < need[k]) return NULL;
  }
  otm_batch_compact in;
  in.n_traces = n_traces;
  in.n_points = n_points;
  in.trace_off = (const int64_t*)ptr[0];
  in.time_base = (const int64_t*)ptr[1];
  in.lat = (const float*)ptr[2];
  in.lon = (const float*)ptr[3];
  in.time_delta = (const int32_t*)ptr[4];
  in.accuracy = (const int16_t*)ptr[5];
  if (in.trace_off[0] != 0 || in.trace_off[n_traces] != n_points) return NULL;
  otm_results r;
  if (otm_match_compact(g_eng, &in, &r) != OTM_OK) return NULL;
  const jclass bb = (*env)->FindClass(env, "java/nio/ByteBuffer");
  jobjectArray out = bb ? (*env)->NewObjectArray(env, 4, bb, NULL) : NULL;
  if (!out) return NULL;
  void* const src[4] = {(void*)r.traces, (void*)r.segments, (void*)r.reports, (void*)r.way_ids};
  const jlong len[4] = {(jlong)r.n_traces * (jlong)sizeof(otm_trace_result),
                        (jlong)r.n_segments * (jlong)sizeof(otm_segment),
                        (jlong)r.n_reports * (jlong)sizeof(otm_report_rec), (jlong)r.n_way_ids * 8};
  for (int k = 0; k < 4; ++k) {
    jobject v = (*env)->NewDirectByteBuffer(env, src[k], len[k]);
    if (!v || (*env)->ExceptionCheck(env)) return NULL;
    (*env)->SetObjectArrayElement(env, out, k, v);
    (*env)->DeleteLocalRef(env, v);
  }
  return out;
}

/* ---- the native batcher (KeyedFormattingProcessor -> BatchingProcessor, Reporter.java:93-103) ---- */
typedef struct {
  otm_batcher* b;
  otm_formatter* f;
  int threads;
} jni_batcher;

/* OtmJni.batcherCreate(spec, threads): the --formatter spec (Reporter.java:33-43) and the batcher with
 * BatchingProcessor's default gates (:28-31) over this process's engine; a handle, or 0 with an
 * IllegalArgumentException pending where Formatter.GetFormatter throws. */
JNIEXPORT jlong JNICALL Java_org_opentraffic_reporter_OtmJni_batcherCreate(JNIEnv* env, jclass c, jstring spec,
                                                                         jint threads) {
  (void)c;
  if (!g_eng || !spec) return 0;
  jni_batcher* h = (jni_batcher*)calloc(1, sizeof *h);
  if (!h) return 0;
  const char* sp = (*env)->GetStringUTFChars(env, spec, 0);
  char err[512] = {0};
  const int frc = sp ? otm_formatter_create(sp, &h->f, err, sizeof err) : OTM_EINVAL;
  if (sp) (*env)->ReleaseStringUTFChars(env, spec, sp);
  if (frc != OTM_OK) {
    free(h);
    (*env)->ThrowNew(env, (*env)->FindClass(env, "java/lang/IllegalArgumentException"), err);
    return 0;
  }
  otm_batcher_cfg cfg;
  otm_batcher_defaults(&cfg);
  cfg.threads = threads;
  if (otm_batcher_create(g_eng, &cfg, NULL, NULL, &h->b) != OTM_OK) {
    otm_formatter_destroy(h->f);
    free(h);
    return 0;
  }
  h->threads = threads;
  return (jlong)(intptr_t)h;
}

/* OtmJni.batcherProcessRaw(h, values, off, ts): one poll's raw values back to back in a direct buffer, value i =
 * values[off[i], off[i+1]) with record timestamp ts[i] (ms); 0 or a negative engine error. */
JNIEXPORT jint JNICALL Java_org_opentraffic_reporter_OtmJni_batcherProcessRaw(JNIEnv* env, jclass c, jlong hh,
                                                                            jobject values, jlongArray off,
                                                                            jlongArray ts) {
  (void)c;
  jni_batcher* h = (jni_batcher*)(intptr_t)hh;
  if (!h || !values || !off || !ts) return OTM_EINVAL;
  const char* base = (const char*)(*env)->GetDirectBufferAddress(env, values);
  const jlong cap = (*env)->GetDirectBufferCapacity(env, values);
  const jsize n = (*env)->GetArrayLength(env, ts);
  if (!base || cap < 0 || (*env)->GetArrayLength(env, off) != n + 1) return OTM_EINVAL;
  jlong* o = (*env)->GetLongArrayElements(env, off, NULL);
  jlong* t = o ? (*env)->GetLongArrayElements(env, ts, NULL) : NULL;
  int rc = OTM_EINVAL;
  if (o && t) {
    int ok = o[0] >= 0;
    for (jsize i = 0; ok && i < n; ++i) ok = o[i] <= o[i + 1] && o[i + 1] <= cap;
    if (ok)
      rc = otm_batcher_process_raw(h->b, h->f, (int32_t)n, base, (const int64_t*)o, (const int64_t*)t, h->threads);
  }
  if (t) (*env)->ReleaseLongArrayElements(env, ts, t, JNI_ABORT);
  if (o) (*env)->ReleaseLongArrayElements(env, off, o, JNI_ABORT);
  return rc;
}

/* OtmJni.batcherTake(h, max): up to max forwarded records as {byte[][] keys, byte[][] bodies, long[] seqs}
 * (UTF-8 bytes), or null when none are ready / an allocation fails (its exception left pending). */
JNIEXPORT jobjectArray JNICALL Java_org_opentraffic_reporter_OtmJni_batcherTake(JNIEnv* env, jclass c, jlong hh,
                                                                              jint max) {
  (void)c;
  jni_batcher* h = (jni_batcher*)(intptr_t)hh;
  if (!h || max <= 0) return NULL;
  otm_forward* f = (otm_forward*)calloc((size_t)max, sizeof(otm_forward));
  if (!f) return NULL;
  const int n = otm_batcher_take(h->b, f, max);
  jobjectArray out = NULL;
  if (n > 0) {
    const jclass bytes = (*env)->FindClass(env, "[B");
    const jclass obj = (*env)->FindClass(env, "java/lang/Object");
    jobjectArray keys = bytes ? (*env)->NewObjectArray(env, n, bytes, NULL) : NULL;
    jobjectArray bodies = keys ? (*env)->NewObjectArray(env, n, bytes, NULL) : NULL;
    jlongArray seqs = bodies ? (*env)->NewLongArray(env, n) : NULL;
    out = seqs && obj ? (*env)->NewObjectArray(env, 3, obj, NULL) : NULL;
    int ok = out != NULL;
    for (int i = 0; i < n; ++i) {
      for (int w = 0; ok && w < 2; ++w) {
        const char* p = w ? f[i].body : f[i].key;
        const size_t len = w ? f[i].body_len : f[i].key_len;
        jbyteArray a = (*env)->NewByteArray(env, (jsize)len);
        if (!a || (*env)->ExceptionCheck(env)) {
          ok = 0;
          break;
        }
        (*env)->SetByteArrayRegion(env, a, 0, (jsize)len, (const jbyte*)p);
        (*env)->SetObjectArrayElement(env, w ? bodies : keys, i, a);
        (*env)->DeleteLocalRef(env, a);
      }
      if (ok) {
        const jlong sq = (jlong)f[i].seq;
        (*env)->SetLongArrayRegion(env, seqs, i, 1, &sq);
      }
      otm_free(f[i].key);
      otm_free(f[i].body);
    }
    if (ok) {
      (*env)->SetObjectArrayElement(env, out, 0, keys);
      (*env)->SetObjectArrayElement(env, out, 1, bodies);
      (*env)->SetObjectArrayElement(env, out, 2, seqs);
    } else {
      out = NULL;
    }
  }
  free(f);
  return out;
}

/* OtmJni.batcherFlush(h) / batcherClose(h) (BatchingProcessor.close, :120-130) / batcherDestroy(h). */
JNIEXPORT jint JNICALL Java_org_opentraffic_reporter_OtmJni_batcherFlush(JNIEnv* env, jclass c, jlong hh) {
  (void)env;
  (void)c;
  jni_batcher* h = (jni_batcher*)(intptr_t)hh;
  return h ? otm_batcher_flush(h->b) : OTM_EINVAL;
}

JNIEXPORT jint JNICALL Java_org_opentraffic_reporter_OtmJni_batcherClose(JNIEnv* env, jclass c, jlong hh) {
  (void)env;
  (void)c;
  jni_batcher* h = (jni_batcher*)(intptr_t)hh;
  return h ? otm_batcher_close(h->b) : OTM_EINVAL;
}

JNIEXPORT void JNICALL Java_org_opentraffic_reporter_OtmJni_batcherDestroy(JNIEnv* env, jclass c, jlong hh) {
  (void)env;
  (void)c;
  jni_batcher* h = (jni_batcher*)(intptr_t)hh;
  if (!h) return;
  otm_batcher_destroy(h->b);
  otm_formatter_destroy(h->f);
  free(h);
}

JNIEXPORT void JNICALL Java_org_opentraffic_reporter_OtmJni_destroy(JNIEnv* env, jclass c) {
  (void)env;
  (void)c;
  otm_engine_destroy(g_eng);
  g_eng = NULL;
}
