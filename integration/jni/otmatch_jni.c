/*
 * otmatch_jni.c -- JNI shim for the reference's Java 8 target (pom.xml), which has no FFM.
 *
 * Binds org.opentraffic.reporter.OtmJni (integration/java/.../OtmJni.java) to libotmatch.so.  OtmJni.POST
 * replaces HttpClient.POST at Batch.java:63 with the same contract: the body reporter_service.py would
 * answer (any status), or null when the call itself fails (HttpClient.java:37-39).
 *
 * Build (needs a JDK, absent from this image):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I../../include \
 *       otmatch_jni.c -L../../reporter_amd/lib -lotmatch -o libotmatch_jni.so
 */
#include <jni.h>

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

JNIEXPORT jstring JNICALL Java_org_opentraffic_reporter_OtmJni_POST(JNIEnv* env, jclass c, jstring url,
                                                                    jstring body) {
  (void)c;
  (void)url; /* ignored: the matcher is in process */
  if (!g_eng || !body) return NULL;
  /* Batch.java builds pure-ASCII bodies (digits, keys, the uuid), so modified UTF-8 == UTF-8 here */
  const char* b = (*env)->GetStringUTFChars(env, body, 0);
  jsize n = (*env)->GetStringUTFLength(env, body);
  char* resp = NULL;
  size_t rn = 0;
  otm_report(g_eng, b, (size_t)n, &resp, &rn);
  (*env)->ReleaseStringUTFChars(env, body, b);
  if (!resp) return NULL;
  jstring out = (*env)->NewStringUTF(env, resp); /* bodies are NUL-terminated, ensure_ascii JSON */
  otm_free(resp);
  return out;
}

JNIEXPORT void JNICALL Java_org_opentraffic_reporter_OtmJni_destroy(JNIEnv* env, jclass c) {
  (void)env;
  (void)c;
  otm_engine_destroy(g_eng);
  g_eng = NULL;
}
