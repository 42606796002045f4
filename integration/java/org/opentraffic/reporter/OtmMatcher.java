package org.opentraffic.reporter;

import java.lang.foreign.*;
import java.lang.invoke.MethodHandle;
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

  private static final MemorySegment ENGINE = create();

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
      for (String b : bodies) total += b.length();  // ISO-8859-1: one byte per char ('?' above U+00FF)
      MemorySegment p = (MemorySegment) ARENA_ALLOC.invokeExact(Math.max(total, 1L));
      if (p.equals(MemorySegment.NULL)) throw new OutOfMemoryError("otm_request_arena_alloc");
      base = p.reinterpret(Math.max(total, 1L));
      ptrs = a.allocate(ValueLayout.ADDRESS, n);
      lens = a.allocate(ValueLayout.JAVA_LONG, n);
      long at = 0;
      for (int i = 0; i < n; ++i) {
        String b = bodies.get(i);
        MemorySegment dst = base.asSlice(at, b.length());
        for (int k = 0; k < b.length(); ++k) {
          char ch = b.charAt(k);
          dst.set(ValueLayout.JAVA_BYTE, k, (byte) (ch <= 0xFF ? ch : '?'));
        }
        ptrs.setAtIndex(ValueLayout.ADDRESS, i, dst);
        lens.setAtIndex(ValueLayout.JAVA_LONG, i, b.length());
        at += b.length();
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
