package org.opentraffic.reporter;

import java.lang.foreign.*;
import java.lang.invoke.MethodHandle;
import java.nio.ByteBuffer;
import java.nio.CharBuffer;
import java.nio.charset.CharsetEncoder;
import java.nio.charset.CoderResult;
import java.nio.charset.CodingErrorAction;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.List;
import org.apache.log4j.Logger;

/**
 * In-process replacement of HttpClient.POST (HttpClient.java:18-45) -> libotmatch.so, through Panama FFM
 * (JDK 22+, no native glue to build).
 *
 * The one-line change in the reference is Batch.java:63:
 *   String response = HttpClient.POST(url, post_body);
 * becomes
 *   String response = OtmMatcher.POST(url, post_body);
 * `url` is ignored; it stays in the signature so the call-site diff is one identifier.
 *
 * Contract (include/otmatch.h, otm_report): same request bytes in, the exact body reporter_service.py
 * would answer out (200 / 400 / 500 bodies alike), null only on a failure of the call itself -- as
 * HttpClient.POST returns null on a transport exception (HttpClient.java:37-39).
 *
 * The async pair (submit / poll) lets a host that can defer context.forward hand many records to one
 * GPU batch: results of one uuid come back in submit order.
 *
 * Not compiled in this repository (the build image has no JDK); the C side it binds is built and tested
 * (tests/test_host.py checks every symbol used here is exported).
 */
public final class OtmMatcher {
  private final static Logger logger = Logger.getLogger(OtmMatcher.class);
  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB =
      SymbolLookup.libraryLookup(System.getProperty("otm.lib", "libotmatch.so"), Arena.global());

  private static MethodHandle fn(String name, FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  // int otm_engine_create(const char* cfg, const int* devices, int ndev, otm_engine** out)
  private static final MethodHandle CREATE = fn("otm_engine_create",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.JAVA_INT,
                            ValueLayout.ADDRESS));
  // int otm_report(otm_engine*, const char* req, size_t len, char** resp, size_t* resp_len)
  private static final MethodHandle REPORT = fn("otm_report",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.JAVA_LONG,
                            ValueLayout.ADDRESS, ValueLayout.ADDRESS));
  // int otm_submit(otm_engine*, const char* req, size_t len, uint64_t tag)
  private static final MethodHandle SUBMIT = fn("otm_submit",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.JAVA_LONG,
                            ValueLayout.JAVA_LONG));
  // int otm_poll(otm_engine*, otm_result* out, int max, int timeout_us)
  private static final MethodHandle POLL = fn("otm_poll",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.JAVA_INT,
                            ValueLayout.JAVA_INT));
  // int otm_report_batch(otm_engine*, int n, const char* const* reqs, const size_t* lens, char** resps,
  //                      size_t* resp_lens, int* codes)
  private static final MethodHandle REPORT_BATCH = fn("otm_report_batch",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.JAVA_INT, ValueLayout.ADDRESS,
                            ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.ADDRESS));
  // int otm_submit_batch(otm_engine*, int n, const char* const* reqs, const size_t* lens, const uint64_t* tags)
  private static final MethodHandle SUBMIT_BATCH = fn("otm_submit_batch",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.JAVA_INT, ValueLayout.ADDRESS,
                            ValueLayout.ADDRESS, ValueLayout.ADDRESS));
  // void* otm_request_arena_alloc(size_t bytes); int otm_request_arena_release(void* arena)
  private static final MethodHandle ARENA_ALLOC = fn("otm_request_arena_alloc",
      FunctionDescriptor.of(ValueLayout.ADDRESS, ValueLayout.JAVA_LONG));
  private static final MethodHandle ARENA_RELEASE = fn("otm_request_arena_release",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS));
  // void otm_free(void*)
  private static final MethodHandle FREE = fn("otm_free", FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));
  // const char* otm_last_error(const otm_engine*)
  private static final MethodHandle LAST_ERROR = fn("otm_last_error",
      FunctionDescriptor.of(ValueLayout.ADDRESS, ValueLayout.ADDRESS));

  // otm_result: {uint64_t tag; int code; (4 bytes padding) char* body; size_t body_len} = 32 bytes
  private static final MemoryLayout RESULT = MemoryLayout.structLayout(ValueLayout.JAVA_LONG.withName("tag"),
      ValueLayout.JAVA_INT.withName("code"), MemoryLayout.paddingLayout(4), ValueLayout.ADDRESS.withName("body"),
      ValueLayout.JAVA_LONG.withName("body_len"));

  // ---------------------------------------------------------------- binary batches (otm_match_compact)
  // int otm_match_compact(otm_engine*, const otm_batch_compact* in, otm_results* out)
  private static final MethodHandle MATCH_COMPACT = fn("otm_match_compact",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.ADDRESS));
  // void* otm_host_alloc(size_t); void otm_host_free(void*): page-locked buffers the library DMAs from
  private static final MethodHandle HOST_ALLOC = fn("otm_host_alloc",
      FunctionDescriptor.of(ValueLayout.ADDRESS, ValueLayout.JAVA_LONG));
  private static final MethodHandle HOST_FREE = fn("otm_host_free", FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));

  // otm_batch_compact: {int32_t n_traces; (4) int64_t n_points; int64_t* trace_off; int64_t* time_base;
  //                     float* lat; float* lon; int32_t* time_delta; int16_t* accuracy} = 64 bytes
  static final MemoryLayout BATCH_COMPACT = MemoryLayout.structLayout(ValueLayout.JAVA_INT.withName("n_traces"),
      MemoryLayout.paddingLayout(4), ValueLayout.JAVA_LONG.withName("n_points"),
      ValueLayout.ADDRESS.withName("trace_off"), ValueLayout.ADDRESS.withName("time_base"),
      ValueLayout.ADDRESS.withName("lat"), ValueLayout.ADDRESS.withName("lon"),
      ValueLayout.ADDRESS.withName("time_delta"), ValueLayout.ADDRESS.withName("accuracy"));
  // otm_results: {int32_t n_traces, n_segments, n_reports, n_way_ids; otm_trace_result* traces;
  //               otm_segment* segments; otm_report_rec* reports; int64_t* way_ids} = 48 bytes
  static final MemoryLayout RESULTS = MemoryLayout.structLayout(ValueLayout.JAVA_INT.withName("n_traces"),
      ValueLayout.JAVA_INT.withName("n_segments"), ValueLayout.JAVA_INT.withName("n_reports"),
      ValueLayout.JAVA_INT.withName("n_way_ids"), ValueLayout.ADDRESS.withName("traces"),
      ValueLayout.ADDRESS.withName("segments"), ValueLayout.ADDRESS.withName("reports"),
      ValueLayout.ADDRESS.withName("way_ids"));
  // otm_trace_result: 14 x int32_t = 56 bytes (reporter_service.py:201-213's stats, :125-127's shape_used)
  static final MemoryLayout TRACE_RESULT = MemoryLayout.structLayout(ValueLayout.JAVA_INT.withName("code"),
      ValueLayout.JAVA_INT.withName("error_kind"), ValueLayout.JAVA_INT.withName("seg_off"),
      ValueLayout.JAVA_INT.withName("seg_cnt"), ValueLayout.JAVA_INT.withName("rep_off"),
      ValueLayout.JAVA_INT.withName("rep_cnt"), ValueLayout.JAVA_INT.withName("shape_used"),
      ValueLayout.JAVA_INT.withName("successful_count"), ValueLayout.JAVA_INT.withName("unreported_count"),
      ValueLayout.JAVA_INT.withName("discontinuities"), ValueLayout.JAVA_INT.withName("invalid_speeds"),
      ValueLayout.JAVA_INT.withName("unassociated"), ValueLayout.JAVA_INT.withName("successful_length"),
      ValueLayout.JAVA_INT.withName("unreported_length"));
  // otm_segment, the fields of README.md:152-165: 56 bytes
  static final MemoryLayout SEGMENT = MemoryLayout.structLayout(ValueLayout.JAVA_LONG.withName("segment_id"),
      ValueLayout.JAVA_DOUBLE.withName("start_time"), ValueLayout.JAVA_DOUBLE.withName("end_time"),
      ValueLayout.JAVA_INT.withName("length"), ValueLayout.JAVA_INT.withName("queue_length"),
      ValueLayout.JAVA_INT.withName("begin_shape_index"), ValueLayout.JAVA_INT.withName("end_shape_index"),
      ValueLayout.JAVA_INT.withName("way_off"), ValueLayout.JAVA_INT.withName("way_cnt"),
      ValueLayout.JAVA_INT.withName("flags"), ValueLayout.JAVA_INT.withName("pad"));
  // otm_report_rec, the datastore report of reporter_service.py:160-166: 48 bytes
  static final MemoryLayout REPORT_REC = MemoryLayout.structLayout(ValueLayout.JAVA_LONG.withName("id"),
      ValueLayout.JAVA_LONG.withName("next_id"), ValueLayout.JAVA_DOUBLE.withName("t0"),
      ValueLayout.JAVA_DOUBLE.withName("t1"), ValueLayout.JAVA_INT.withName("length"),
      ValueLayout.JAVA_INT.withName("queue_length"), ValueLayout.JAVA_INT.withName("flags"),
      ValueLayout.JAVA_INT.withName("pad"));

  private static final MemorySegment ENGINE = create();

  /** The process's engine handle (the native batcher binds to it, OtmBatcher). */
  static MemorySegment engine() {
    return ENGINE;
  }

  private static MemorySegment create() {
    // one engine per process.  -Dotm.devices=0,1,...,7 gives this one JVM every listed GPU behind the one
    // handle (traces go to murmur2(uuid) % ndev, INTEGRATION.md §5); default: the one GPU this process owns
    // (-Dotm.device, LOCAL_RANK / HIP_VISIBLE_DEVICES).
    // Replaces valhalla.Configure (py/reporter_service.py:279) + SegmentMatcher() per worker (:52).
    try (Arena a = Arena.ofConfined()) {
      MemorySegment cfg = a.allocateFrom(System.getProperty("otm.config", "/etc/otmatch.json"));
      String list = System.getProperty("otm.devices", Integer.toString(Integer.getInteger("otm.device", 0)));
      int[] ids = java.util.Arrays.stream(list.split(",")).map(String::trim).mapToInt(Integer::parseInt).toArray();
      MemorySegment dev = a.allocateFrom(ValueLayout.JAVA_INT, ids);
      MemorySegment out = a.allocate(ValueLayout.ADDRESS);
      int rc = (int) CREATE.invokeExact(cfg, dev, ids.length, out);
      if (rc != 0) {
        MemorySegment msg = (MemorySegment) LAST_ERROR.invokeExact(MemorySegment.NULL);
        throw new IllegalStateException("otm_engine_create: " + msg.reinterpret(4096).getString(0));
      }
      return out.get(ValueLayout.ADDRESS, 0);
    } catch (Throwable t) {
      throw new ExceptionInInitializerError(t);
    }
  }

  private static String takeBody(MemorySegment p, long n) throws Throwable {
    String v = new String(p.reinterpret(n).toArray(ValueLayout.JAVA_BYTE), StandardCharsets.UTF_8);
    FREE.invokeExact(p);
    return v;
  }

  /** Same contract as HttpClient.POST: the response body, or null on a failure of the call. */
  public static String POST(String url, String body) {
    try (Arena a = Arena.ofConfined()) {
      // new StringEntity(body) (HttpClient.java:26): ISO-8859-1, '?' for a character above U+00FF
      byte[] b = body.getBytes(StandardCharsets.ISO_8859_1);
      MemorySegment req = a.allocate(b.length);
      MemorySegment.copy(b, 0, req, ValueLayout.JAVA_BYTE, 0, b.length);
      MemorySegment resp = a.allocate(ValueLayout.ADDRESS);
      MemorySegment len = a.allocate(ValueLayout.JAVA_LONG);
      int code = (int) REPORT.invokeExact(ENGINE, req, (long) b.length, resp, len);
      // HttpClient.POST hands back the body whatever the status (the 4xx/5xx bodies are JSON too)
      return takeBody(resp.get(ValueLayout.ADDRESS, 0), len.get(ValueLayout.JAVA_LONG, 0));
    } catch (Throwable t) {
      logger.error("otm_report failed for body " + body);
      return null;  // as HttpClient.POST on an exception (HttpClient.java:37-39)
    }
  }

  /**
   * Request bodies written straight into a library-owned page-locked request arena
   * (otm_request_arena_alloc): the bytes new StringEntity(body) would send (ISO-8859-1, HttpClient.java:26)
   * are encoded into the arena back to back, and otm_report_batch / otm_submit_batch send them to HBM from
   * there -- no heap array, no staging copy in the library.
   */
  private static final class RequestArena implements AutoCloseable {
    final MemorySegment base;
    final MemorySegment ptrs, lens;
    final int n;

    RequestArena(List<String> bodies, Arena a) throws Throwable {
      n = bodies.size();
      long total = 0;
      for (String b : bodies) total += b.length();  // ISO-8859-1: at most one byte per char
      MemorySegment p = (MemorySegment) ARENA_ALLOC.invokeExact(Math.max(total, 1L));
      if (p.equals(MemorySegment.NULL)) throw new OutOfMemoryError("otm_request_arena_alloc");
      base = p.reinterpret(Math.max(total, 1L));
      try {
        ptrs = a.allocate(ValueLayout.ADDRESS, n);
        lens = a.allocate(ValueLayout.JAVA_LONG, n);
        // each body encoded straight into the arena, as new StringEntity(body) encodes it (HttpClient.java:26):
        // ISO-8859-1 with '?' for what it cannot map -- one '?' per unmappable code point, a surrogate pair
        // included, exactly as String.getBytes(ISO_8859_1) -- and no heap byte[] on the way
        CharsetEncoder enc = StandardCharsets.ISO_8859_1.newEncoder()
            .onMalformedInput(CodingErrorAction.REPLACE).onUnmappableCharacter(CodingErrorAction.REPLACE);
        ByteBuffer out = base.asByteBuffer();
        for (int i = 0; i < n; ++i) {
          int at = out.position();
          enc.reset();
          CoderResult cr = enc.encode(CharBuffer.wrap(bodies.get(i)), out, true);
          if (cr.isError() || cr.isOverflow() || enc.flush(out).isOverflow())
            throw new IllegalStateException("request arena encoding");
          ptrs.setAtIndex(ValueLayout.ADDRESS, i, base.asSlice(at, out.position() - at));
          lens.setAtIndex(ValueLayout.JAVA_LONG, i, out.position() - at);
        }
      } catch (Throwable t) {
        int rc = (int) ARENA_RELEASE.invokeExact(base);  // (the constructor failed: close() will not run)
        throw t;
      }
    }

    @Override
    public void close() throws Exception {
      try {
        int rc = (int) ARENA_RELEASE.invokeExact(base);
      } catch (Throwable t) {
        throw new Exception(t);
      }
    }
  }

  /**
   * Many POSTs at once (the requests of one Kafka poll): the same contract as POST per body, in order, one
   * GPU batch; the bodies go to the GPU from a request arena.  null entries where the call failed.
   */
  public static List<String> POST_BATCH(String url, List<String> bodies) {
    List<String> out = new ArrayList<>();
    try (Arena a = Arena.ofConfined(); RequestArena ra = new RequestArena(bodies, a)) {
      int n = ra.n;
      MemorySegment resps = a.allocate(ValueLayout.ADDRESS, n);
      MemorySegment rlens = a.allocate(ValueLayout.JAVA_LONG, n);
      MemorySegment codes = a.allocate(ValueLayout.JAVA_INT, n);
      int rc = (int) REPORT_BATCH.invokeExact(ENGINE, n, ra.ptrs, ra.lens, resps, rlens, codes);
      for (int i = 0; i < n; ++i)
        out.add(rc != 0 ? null : takeBody(resps.getAtIndex(ValueLayout.ADDRESS, i), rlens.getAtIndex(ValueLayout.JAVA_LONG, i)));
    } catch (Throwable t) {
      logger.error("otm_report_batch failed");
      while (out.size() < bodies.size()) out.add(null);
    }
    return out;
  }

  /**
   * Queue many /report requests (results from poll() with these tags), straight from a request arena; the
   * submission holds the arena until its results are back, so it is released here at once.
   */
  public static boolean submitBatch(List<String> bodies, long[] tags) {
    try (Arena a = Arena.ofConfined(); RequestArena ra = new RequestArena(bodies, a)) {
      MemorySegment tg = a.allocateFrom(ValueLayout.JAVA_LONG, tags);
      return (int) SUBMIT_BATCH.invokeExact(ENGINE, ra.n, ra.ptrs, ra.lens, tg) == 0;
    } catch (Throwable t) {
      logger.error("otm_submit_batch failed");
      return false;
    }
  }

  /** Queue one /report request; its result comes back from poll() with this tag. */
  public static boolean submit(String body, long tag) {
    try (Arena a = Arena.ofConfined()) {
      // new StringEntity(body) (HttpClient.java:26): ISO-8859-1, '?' for a character above U+00FF
      byte[] b = body.getBytes(StandardCharsets.ISO_8859_1);
      MemorySegment req = a.allocate(b.length);
      MemorySegment.copy(b, 0, req, ValueLayout.JAVA_BYTE, 0, b.length);
      return (int) SUBMIT.invokeExact(ENGINE, req, (long) b.length, tag) == 0;
    } catch (Throwable t) {
      logger.error("otm_submit failed");
      return false;
    }
  }

  // ------------------------------------------------------------------ otm_match_compact
  /** One matched OSMLR segment (include/otmatch.h otm_segment; README.md:152-165). */
  public record Segment(long segmentId, double startTime, double endTime, int length, int queueLength,
                        int beginShapeIndex, int endShapeIndex, long[] wayIds, int flags) {}

  /** One datastore report (include/otmatch.h otm_report_rec; reporter_service.py:160-166). */
  public record Report(long id, long nextId, double t0, double t1, int length, int queueLength, int flags) {}

  /** A trace's outcome: status, shape_used (-1: None) for Batch's trim, its segments and reports. */
  public record TraceResult(int code, int errorKind, int shapeUsed, List<Segment> segments, List<Report> reports) {}

  /**
   * The binary batch path in the host's own types (Point.java:16-25): the batches' points go to the GPU as
   * float lat/lon, an int32 time delta from each trace's first time and an int16 accuracy (14 bytes per point,
   * include/otmatch.h otm_batch_compact), written into page-locked buffers (otm_host_alloc) the library DMAs
   * from.  What Batch.report needs back (shape_used, Batch.java:67-70) and the typed segments / reports the
   * JSON response would carry.  null when the call fails, as HttpClient.POST returns null.  A trace whose times
   * span 2^31 s or whose accuracies leave the int16 range must go through POST (the header's contract).
   */
  public static List<TraceResult> matchCompact(List<List<Point>> traces) {
    final int nt = traces.size();
    long np = 0;
    for (List<Point> t : traces) np += t.size();
    MemorySegment[] bufs = new MemorySegment[6];
    try (Arena a = Arena.ofConfined()) {
      long[] bytes = {8L * (nt + 1), 8L * Math.max(nt, 1), 4L * Math.max(np, 1), 4L * Math.max(np, 1),
                      4L * Math.max(np, 1), 2L * Math.max(np, 1)};
      for (int k = 0; k < 6; ++k) {
        MemorySegment p = (MemorySegment) HOST_ALLOC.invokeExact(bytes[k]);
        if (p.equals(MemorySegment.NULL)) throw new OutOfMemoryError("otm_host_alloc");
        bufs[k] = p.reinterpret(bytes[k]);
      }
      long at = 0;
      for (int t = 0; t < nt; ++t) {
        List<Point> pts = traces.get(t);
        bufs[0].setAtIndex(ValueLayout.JAVA_LONG, t, at);
        long base = pts.isEmpty() ? 0 : pts.get(0).time;
        bufs[1].setAtIndex(ValueLayout.JAVA_LONG, t, base);
        for (Point p : pts) {
          bufs[2].setAtIndex(ValueLayout.JAVA_FLOAT, at, p.lat);
          bufs[3].setAtIndex(ValueLayout.JAVA_FLOAT, at, p.lon);
          bufs[4].setAtIndex(ValueLayout.JAVA_INT, at, Math.toIntExact(p.time - base));
          if (p.accuracy < Short.MIN_VALUE || p.accuracy > Short.MAX_VALUE)
            throw new ArithmeticException("accuracy outside int16: use POST");
          bufs[5].setAtIndex(ValueLayout.JAVA_SHORT, at, (short) p.accuracy);
          ++at;
        }
      }
      bufs[0].setAtIndex(ValueLayout.JAVA_LONG, nt, at);
      MemorySegment in = a.allocate(BATCH_COMPACT);
      in.set(ValueLayout.JAVA_INT, BATCH_COMPACT.byteOffset(MemoryLayout.PathElement.groupElement("n_traces")), nt);
      in.set(ValueLayout.JAVA_LONG, BATCH_COMPACT.byteOffset(MemoryLayout.PathElement.groupElement("n_points")), np);
      String[] names = {"trace_off", "time_base", "lat", "lon", "time_delta", "accuracy"};
      for (int k = 0; k < 6; ++k)
        in.set(ValueLayout.ADDRESS, BATCH_COMPACT.byteOffset(MemoryLayout.PathElement.groupElement(names[k])), bufs[k]);
      MemorySegment out = a.allocate(RESULTS);
      if ((int) MATCH_COMPACT.invokeExact(ENGINE, in, out) != 0) return null;
      return readResults(out);
    } catch (Throwable t) {
      logger.error("otm_match_compact failed");
      return null;
    } finally {
      for (MemorySegment b : bufs) {
        try {
          if (b != null) HOST_FREE.invokeExact(b);
        } catch (Throwable ignored) {
        }
      }
    }
  }

  private static long off(MemoryLayout l, String field) {
    return l.byteOffset(MemoryLayout.PathElement.groupElement(field));
  }

  /** The engine-owned result arrays (valid until the engine's next call) copied into Java records. */
  private static List<TraceResult> readResults(MemorySegment out) {
    int nt = out.get(ValueLayout.JAVA_INT, off(RESULTS, "n_traces"));
    int ns = out.get(ValueLayout.JAVA_INT, off(RESULTS, "n_segments"));
    int nr = out.get(ValueLayout.JAVA_INT, off(RESULTS, "n_reports"));
    int nw = out.get(ValueLayout.JAVA_INT, off(RESULTS, "n_way_ids"));
    MemorySegment tr = out.get(ValueLayout.ADDRESS, off(RESULTS, "traces")).reinterpret(TRACE_RESULT.byteSize() * nt);
    MemorySegment sg = out.get(ValueLayout.ADDRESS, off(RESULTS, "segments")).reinterpret(SEGMENT.byteSize() * ns);
    MemorySegment rp = out.get(ValueLayout.ADDRESS, off(RESULTS, "reports")).reinterpret(REPORT_REC.byteSize() * nr);
    MemorySegment wy = out.get(ValueLayout.ADDRESS, off(RESULTS, "way_ids")).reinterpret(8L * nw);
    List<TraceResult> res = new ArrayList<>(nt);
    for (int t = 0; t < nt; ++t) {
      MemorySegment r = tr.asSlice(t * TRACE_RESULT.byteSize(), TRACE_RESULT.byteSize());
      int so = r.get(ValueLayout.JAVA_INT, off(TRACE_RESULT, "seg_off"));
      int sc = r.get(ValueLayout.JAVA_INT, off(TRACE_RESULT, "seg_cnt"));
      int ro = r.get(ValueLayout.JAVA_INT, off(TRACE_RESULT, "rep_off"));
      int rc = r.get(ValueLayout.JAVA_INT, off(TRACE_RESULT, "rep_cnt"));
      List<Segment> segs = new ArrayList<>(sc);
      for (int k = so; k < so + sc; ++k) {
        MemorySegment s = sg.asSlice(k * SEGMENT.byteSize(), SEGMENT.byteSize());
        int wo = s.get(ValueLayout.JAVA_INT, off(SEGMENT, "way_off"));
        int wc = s.get(ValueLayout.JAVA_INT, off(SEGMENT, "way_cnt"));
        long[] ways = wy.asSlice(8L * wo, 8L * wc).toArray(ValueLayout.JAVA_LONG);
        segs.add(new Segment(s.get(ValueLayout.JAVA_LONG, off(SEGMENT, "segment_id")),
            s.get(ValueLayout.JAVA_DOUBLE, off(SEGMENT, "start_time")),
            s.get(ValueLayout.JAVA_DOUBLE, off(SEGMENT, "end_time")), s.get(ValueLayout.JAVA_INT, off(SEGMENT, "length")),
            s.get(ValueLayout.JAVA_INT, off(SEGMENT, "queue_length")),
            s.get(ValueLayout.JAVA_INT, off(SEGMENT, "begin_shape_index")),
            s.get(ValueLayout.JAVA_INT, off(SEGMENT, "end_shape_index")), ways,
            s.get(ValueLayout.JAVA_INT, off(SEGMENT, "flags"))));
      }
      List<Report> reps = new ArrayList<>(rc);
      for (int k = ro; k < ro + rc; ++k) {
        MemorySegment q = rp.asSlice(k * REPORT_REC.byteSize(), REPORT_REC.byteSize());
        reps.add(new Report(q.get(ValueLayout.JAVA_LONG, off(REPORT_REC, "id")),
            q.get(ValueLayout.JAVA_LONG, off(REPORT_REC, "next_id")), q.get(ValueLayout.JAVA_DOUBLE, off(REPORT_REC, "t0")),
            q.get(ValueLayout.JAVA_DOUBLE, off(REPORT_REC, "t1")), q.get(ValueLayout.JAVA_INT, off(REPORT_REC, "length")),
            q.get(ValueLayout.JAVA_INT, off(REPORT_REC, "queue_length")),
            q.get(ValueLayout.JAVA_INT, off(REPORT_REC, "flags"))));
      }
      res.add(new TraceResult(r.get(ValueLayout.JAVA_INT, off(TRACE_RESULT, "code")),
          r.get(ValueLayout.JAVA_INT, off(TRACE_RESULT, "error_kind")),
          r.get(ValueLayout.JAVA_INT, off(TRACE_RESULT, "shape_used")), segs, reps));
    }
    return res;
  }

  /** A finished request: the tag given to submit(), the HTTP status and body. */
  public record Result(long tag, int code, String body) {}

  /** Up to max finished requests, waiting at most timeoutUs for the first. */
  public static List<Result> poll(int max, int timeoutUs) {
    List<Result> out = new ArrayList<>();
    try (Arena a = Arena.ofConfined()) {
      MemorySegment res = a.allocate(RESULT, max);
      int n = (int) POLL.invokeExact(ENGINE, res, max, timeoutUs);
      for (int i = 0; i < n; ++i) {
        MemorySegment r = res.asSlice(i * RESULT.byteSize(), RESULT.byteSize());
        long tag = r.get(ValueLayout.JAVA_LONG, 0);
        int code = r.get(ValueLayout.JAVA_INT, 8);
        MemorySegment body = r.get(ValueLayout.ADDRESS, 16);
        long blen = r.get(ValueLayout.JAVA_LONG, 24);
        out.add(new Result(tag, code, takeBody(body, blen)));
      }
    } catch (Throwable t) {
      logger.error("otm_poll failed");
    }
    return out;
  }
}
