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
 * from the arena by otm_report_batch; the response bytes back per body (null where the call failed). */
JNIEXPORT jobjectArray JNICALL Java_org_opentraffic_reporter_OtmJni_reportBatch(JNIEnv* env, jclass c,
                                                                              jobject arena, jlongArray off) {
  (void)c;
  if (!g_eng || !arena || !off) return NULL;
  const char* base = (const char*)(*env)->GetDirectBufferAddress(env, arena);
  const jsize n = (*env)->GetArrayLength(env, off) - 1;
  if (!base || n < 0) return NULL;
  jlong* o = (*env)->GetLongArrayElements(env, off, NULL);
  const char** reqs = (const char**)malloc(sizeof(char*) * (size_t)(n ? n : 1));
  size_t* lens = (size_t*)malloc(sizeof(size_t) * (size_t)(n ? n : 1));
  char** resps = (char**)calloc((size_t)(n ? n : 1), sizeof(char*));
  size_t* rlens = (size_t*)calloc((size_t)(n ? n : 1), sizeof(size_t));
  int* codes = (int*)calloc((size_t)(n ? n : 1), sizeof(int));
  jobjectArray out = NULL;
  if (o && reqs && lens && resps && rlens && codes) {
    for (jsize i = 0; i < n; ++i) {
      reqs[i] = base + o[i];
      lens[i] = (size_t)(o[i + 1] - o[i]);
    }
    const int rc = otm_report_batch(g_eng, (int)n, reqs, lens, resps, rlens, codes);
    out = (*env)->NewObjectArray(env, n, (*env)->FindClass(env, "[B"), NULL);
    for (jsize i = 0; out && i < n; ++i) {
      if (rc == OTM_OK && resps[i]) {
        jbyteArray b = (*env)->NewByteArray(env, (jsize)rlens[i]);
        if (b) {
          (*env)->SetByteArrayRegion(env, b, 0, (jsize)rlens[i], (const jbyte*)resps[i]);
          (*env)->SetObjectArrayElement(env, out, i, b);
          (*env)->DeleteLocalRef(env, b);
        }
      }
      otm_free(resps[i]);
    }
  }
  if (o) (*env)->ReleaseLongArrayElements(env, off, o, JNI_ABORT);
  free(reqs);
  free(lens);
  free(resps);
  free(rlens);
  free(codes);
  return out;
}

JNIEXPORT void JNICALL Java_org_opentraffic_reporter_OtmJni_destroy(JNIEnv* env, jclass c) {
  (void)env;
  (void)c;
  otm_engine_destroy(g_eng);
  g_eng = NULL;
}
