package org.opentraffic.reporter;

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

  /** HttpClient.POST replacement: the response body, or null when the call fails. */
  public static native String POST(String url, String body);
}
