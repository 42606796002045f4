package org.opentraffic.reporter;

import java.nio.ByteBuffer;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.List;

/**
 * JNI form of OtmMatcher for the reference's Java 8 target (pom.xml): HttpClient.POST's replacement at
 * Batch.java:63 is `OtmJni.POST(url, post_body)`.  Native side: integration/jni/otmatch_jni.c.
 */
public final class OtmJni {
  static {
    System.loadLibrary("otmatch_jni");
    init(System.getProperty("otm.config", "/etc/otmatch.json"), Integer.getInteger("otm.device", 0));
    Runtime.getRuntime().addShutdownHook(new Thread(OtmJni::destroy));
  }

  private static native void init(String cfgPath, int device);

  private static native void destroy();

  /** The /report call on request bytes: the response bytes, or null when the call fails. */
  private static native byte[] report(byte[] body);

  /** A page-locked request arena of the library (otm_request_arena_alloc) as a direct buffer. */
  private static native ByteBuffer arenaAlloc(long bytes);

  private static native void arenaRelease(ByteBuffer arena);

  /** otm_report_batch over body i = arena[off[i], off[i+1]); response bytes per body (null: failed). */
  private static native byte[][] reportBatch(ByteBuffer arena, long[] off);

  /**
   * Many POSTs at once, one GPU batch: each body's ISO-8859-1 bytes (HttpClient.java:26) written into a
   * request arena, sent to HBM from there; the responses read as UTF-8 (:33), null where the call failed.
   */
  public static List<String> POST_BATCH(String url, List<String> bodies) {
    long total = 0;
    for (String b : bodies) total += b.length();  // ISO-8859-1: one byte per char
    List<String> out = new ArrayList<>(bodies.size());
    ByteBuffer arena = arenaAlloc(total);
    if (arena == null) {
      for (String b : bodies) out.add(POST(url, b));
      return out;
    }
    try {
      long[] off = new long[bodies.size() + 1];
      for (int i = 0; i < bodies.size(); ++i) {
        arena.put(bodies.get(i).getBytes(StandardCharsets.ISO_8859_1));
        off[i + 1] = arena.position();
      }
      byte[][] r = reportBatch(arena, off);
      for (int i = 0; i < bodies.size(); ++i)
        out.add(r == null || r[i] == null ? null : new String(r[i], StandardCharsets.UTF_8));
    } finally {
      arenaRelease(arena);
    }
    return out;
  }

  /**
   * HttpClient.POST replacement: the response body, or null when the call fails.  The charset steps are
   * HttpClient's own: new StringEntity(body) sends ISO-8859-1 bytes (httpcore's default text/plain charset;
   * a character above U+00FF becomes '?', HttpClient.java:26) and the response is read as UTF-8 (:33).
   */
  public static String POST(String url, String body) {
    byte[] r = report(body.getBytes(StandardCharsets.ISO_8859_1));
    return r == null ? null : new String(r, StandardCharsets.UTF_8);
  }
}
