package org.opentraffic.reporter;

import java.nio.charset.StandardCharsets;

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
