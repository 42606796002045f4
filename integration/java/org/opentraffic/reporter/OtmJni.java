package org.opentraffic.reporter;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.nio.CharBuffer;
import java.nio.charset.CharsetEncoder;
import java.nio.charset.CoderResult;
import java.nio.charset.CodingErrorAction;
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

  /** otm_match_compact over direct buffers; four direct views of the engine's result arrays (or null). */
  private static native ByteBuffer[] matchCompact(int nTraces, long nPoints, ByteBuffer traceOff, ByteBuffer timeBase,
                                                  ByteBuffer lat, ByteBuffer lon, ByteBuffer timeDelta,
                                                  ByteBuffer accuracy);

  /** The native batcher + formatter over this process's engine (a handle; 0 on failure). */
  static native long batcherCreate(String formatterSpec, int threads);

  /** One poll's raw values (back to back in a direct buffer, value i = [off[i], off[i+1])) and timestamps. */
  static native int batcherProcessRaw(long h, ByteBuffer values, long[] off, long[] timestampsMs);

  /** Up to max forwarded records as {byte[][] keys, byte[][] bodies, long[] seqs}, or null when none. */
  static native Object[] batcherTake(long h, int max);

  static native int batcherFlush(long h);

  static native int batcherClose(long h);

  static native void batcherDestroy(long h);

  // new StringEntity(body)'s bytes (HttpClient.java:26): ISO-8859-1, one '?' per code point it cannot map (a
  // surrogate pair included), exactly as String.getBytes(ISO_8859_1)
  private static CharsetEncoder latin1() {
    return StandardCharsets.ISO_8859_1.newEncoder().onMalformedInput(CodingErrorAction.REPLACE)
        .onUnmappableCharacter(CodingErrorAction.REPLACE);
  }

  /**
   * Many POSTs at once, one GPU batch: each body's ISO-8859-1 bytes encoded straight into a request arena (no
   * heap byte[]), sent to HBM from there; the responses read as UTF-8 (:33), null where the call failed.
   */
  public static List<String> POST_BATCH(String url, List<String> bodies) {
    long total = 0;
    for (String b : bodies) total += b.length();  // ISO-8859-1: at most one byte per char
    List<String> out = new ArrayList<>(bodies.size());
    ByteBuffer arena = arenaAlloc(total);
    if (arena == null) {
      for (String b : bodies) out.add(POST(url, b));
      return out;
    }
    try {
      long[] off = new long[bodies.size() + 1];
      CharsetEncoder enc = latin1();
      for (int i = 0; i < bodies.size(); ++i) {
        enc.reset();
        CoderResult cr = enc.encode(CharBuffer.wrap(bodies.get(i)), arena, true);
        if (cr.isError() || cr.isOverflow() || enc.flush(arena).isOverflow())
          throw new IllegalStateException("request arena encoding");
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
   * The binary batch path in the host's own types (Point.java:16-25): per trace its shape_used (-1: None) for
   * Batch.report's trim (Batch.java:67-70) and status; the typed segments and reports are read from the returned
   * views (include/otmatch.h otm_segment / otm_report_rec layouts) before the engine's next call.  null when the
   * call fails, as HttpClient.POST returns null.  Traces whose times span 2^31 s or whose accuracies leave int16
   * go through POST instead.
   */
  public static int[][] matchCompactShapeUsed(List<List<Point>> traces) {
    int nt = traces.size();
    long np = 0;
    for (List<Point> t : traces) np += t.size();
    ByteBuffer off = ByteBuffer.allocateDirect(8 * (nt + 1)).order(ByteOrder.nativeOrder());
    ByteBuffer tb = ByteBuffer.allocateDirect(8 * Math.max(nt, 1)).order(ByteOrder.nativeOrder());
    ByteBuffer la = ByteBuffer.allocateDirect((int) (4 * Math.max(np, 1))).order(ByteOrder.nativeOrder());
    ByteBuffer lo = ByteBuffer.allocateDirect((int) (4 * Math.max(np, 1))).order(ByteOrder.nativeOrder());
    ByteBuffer dt = ByteBuffer.allocateDirect((int) (4 * Math.max(np, 1))).order(ByteOrder.nativeOrder());
    ByteBuffer ac = ByteBuffer.allocateDirect((int) (2 * Math.max(np, 1))).order(ByteOrder.nativeOrder());
    long at = 0;
    for (List<Point> t : traces) {
      off.putLong(at);
      long base = t.isEmpty() ? 0 : t.get(0).time;
      tb.putLong(base);
      for (Point p : t) {
        la.putFloat(p.lat);
        lo.putFloat(p.lon);
        dt.putInt(Math.toIntExact(p.time - base));
        if (p.accuracy < Short.MIN_VALUE || p.accuracy > Short.MAX_VALUE) return null;
        ac.putShort((short) p.accuracy);
        ++at;
      }
    }
    off.putLong(at);
    ByteBuffer[] r = matchCompact(nt, np, off, tb, la, lo, dt, ac);
    if (r == null) return null;
    ByteBuffer tr = r[0].order(ByteOrder.nativeOrder());
    int[][] out = new int[nt][];
    for (int t = 0; t < nt; ++t) {
      // otm_trace_result: 14 x int32 -- code, error_kind, ..., shape_used at word 6
      out[t] = new int[] {tr.getInt(56 * t), tr.getInt(56 * t + 24)};
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
