package org.opentraffic.reporter;

import java.lang.foreign.*;
import java.lang.invoke.MethodHandle;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.List;

/**
 * The reporter's two stream processors, native, through Panama FFM (JDK 22+): KeyedFormattingProcessor ->
 * BatchingProcessor (Reporter.java:93-103; KeyedFormattingProcessor.java:30-37, BatchingProcessor.java:56-130,
 * Batch.java:46-84) run inside libotmatch.so, with the GPU engine of OtmMatcher as the matcher.  The host's
 * consumer loop hands each poll's raw values and record timestamps over and publishes what comes back:
 *
 *   try (OtmBatcher b = new OtmBatcher(formatterSpec, 8)) {
 *     for (ConsumerRecords<...> poll : polls) {
 *       b.processRaw(values, timestamps);                    // formats, batches, matches ready keys on the GPU
 *       for (OtmBatcher.Forward f : b.take()) producer.send(new ProducerRecord<>(leafTopic, f.key(), f.body()));
 *     }
 *     b.close();                                             // BatchingProcessor.close: relaxed reports
 *   }
 *
 * What comes back matches the reference's processors record for record: the forwarded (key, response) pairs and
 * the stored batches (tests/test_batcher.py, tests/test_gpu_batcher.py).  One instance is one stream task: call it
 * from one thread at a time (include/otmatch.h).  Not compiled in this repository (no JDK in the image); every
 * symbol and struct it binds is checked against the library (tests/test_java_abi.py).
 */
public final class OtmBatcher implements AutoCloseable {
  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB =
      SymbolLookup.libraryLookup(System.getProperty("otm.lib", "libotmatch.so"), Arena.global());

  private static MethodHandle fn(String name, FunctionDescriptor d) {
    return LINKER.downcallHandle(LIB.find(name).orElseThrow(), d);
  }

  // otm_batcher_cfg: {int32_t report_dist, report_count; int64_t report_time_s, session_gap_ms;
  //                   int32_t max_batch, json_path; int64_t max_pending; int32_t threads, reserved} = 48 bytes
  static final MemoryLayout BATCHER_CFG = MemoryLayout.structLayout(ValueLayout.JAVA_INT.withName("report_dist"),
      ValueLayout.JAVA_INT.withName("report_count"), ValueLayout.JAVA_LONG.withName("report_time_s"),
      ValueLayout.JAVA_LONG.withName("session_gap_ms"), ValueLayout.JAVA_INT.withName("max_batch"),
      ValueLayout.JAVA_INT.withName("json_path"), ValueLayout.JAVA_LONG.withName("max_pending"),
      ValueLayout.JAVA_INT.withName("threads"), ValueLayout.JAVA_INT.withName("reserved"));
  // otm_forward: {char* key; size_t key_len; char* body; size_t body_len; int64_t seq} = 40 bytes
  static final MemoryLayout FORWARD = MemoryLayout.structLayout(ValueLayout.ADDRESS.withName("key"),
      ValueLayout.JAVA_LONG.withName("key_len"), ValueLayout.ADDRESS.withName("body"),
      ValueLayout.JAVA_LONG.withName("body_len"), ValueLayout.JAVA_LONG.withName("seq"));

  // void otm_batcher_defaults(otm_batcher_cfg*)
  private static final MethodHandle DEFAULTS = fn("otm_batcher_defaults", FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));
  // int otm_batcher_create(otm_engine*, const otm_batcher_cfg*, otm_report_fn, void* ctx, otm_batcher**)
  private static final MethodHandle CREATE = fn("otm_batcher_create",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.ADDRESS,
                            ValueLayout.ADDRESS, ValueLayout.ADDRESS));
  private static final MethodHandle DESTROY = fn("otm_batcher_destroy", FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));
  // int otm_batcher_process_raw(otm_batcher*, const otm_formatter*, int32_t n, const char* msgs,
  //                             const int64_t* off, const int64_t* ts_ms, int nthreads)
  private static final MethodHandle PROCESS_RAW = fn("otm_batcher_process_raw",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.JAVA_INT,
                            ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.JAVA_INT));
  // int otm_batcher_flush(otm_batcher*); int otm_batcher_close(otm_batcher*)
  private static final MethodHandle FLUSH = fn("otm_batcher_flush",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS));
  private static final MethodHandle CLOSE = fn("otm_batcher_close",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS));
  // int otm_batcher_take(otm_batcher*, otm_forward* out, int max)
  private static final MethodHandle TAKE = fn("otm_batcher_take",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.JAVA_INT));
  // int otm_formatter_create(const char* spec, otm_formatter**, char* err, size_t err_len)
  private static final MethodHandle FMT_CREATE = fn("otm_formatter_create",
      FunctionDescriptor.of(ValueLayout.JAVA_INT, ValueLayout.ADDRESS, ValueLayout.ADDRESS, ValueLayout.ADDRESS,
                            ValueLayout.JAVA_LONG));
  private static final MethodHandle FMT_DESTROY = fn("otm_formatter_destroy",
      FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));
  private static final MethodHandle FREE = fn("otm_free", FunctionDescriptor.ofVoid(ValueLayout.ADDRESS));

  /** context.forward(key, response) of BatchingProcessor.process (:70-71); seq = the record's stream position. */
  public record Forward(String key, String body, long seq) {}

  private final MemorySegment batcher, formatter;
  private final int formatThreads;
  private boolean closed;

  /**
   * spec: the --formatter string (Reporter.java:33-43, Formatter.GetFormatter); threads: the batcher's and the
   * formatter's host threads.  Gates, session gap and trim are BatchingProcessor's defaults (:28-31).
   */
  public OtmBatcher(String spec, int threads) {
    try (Arena a = Arena.ofConfined()) {
      MemorySegment fo = a.allocate(ValueLayout.ADDRESS);
      MemorySegment err = a.allocate(512);
      if ((int) FMT_CREATE.invokeExact(a.allocateFrom(spec), fo, err, 512L) != 0)
        throw new IllegalArgumentException("formatter: " + err.getString(0));  // Formatter.GetFormatter throws
      formatter = fo.get(ValueLayout.ADDRESS, 0);
      MemorySegment cfg = a.allocate(BATCHER_CFG);
      DEFAULTS.invokeExact(cfg);
      cfg.set(ValueLayout.JAVA_INT, BATCHER_CFG.byteOffset(MemoryLayout.PathElement.groupElement("threads")), threads);
      MemorySegment bo = a.allocate(ValueLayout.ADDRESS);
      if ((int) CREATE.invokeExact(OtmMatcher.engine(), cfg, MemorySegment.NULL, MemorySegment.NULL, bo) != 0) {
        FMT_DESTROY.invokeExact(formatter);
        throw new IllegalStateException("otm_batcher_create");
      }
      batcher = bo.get(ValueLayout.ADDRESS, 0);
      formatThreads = threads;
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new IllegalStateException(t);
    }
  }

  /**
   * One poll of the raw topic: the record values as they arrived (bytes, any encoding the formatter reads) and
   * their record timestamps (ms).  Messages the reference's formatter would throw on are dropped and counted,
   * as KeyedFormattingProcessor logs and drops them.  The values are written back to back into one native
   * segment (no per-record call).
   */
  public void processRaw(List<byte[]> values, long[] timestampsMs) {
    final int n = values.size();
    if (timestampsMs.length != n) throw new IllegalArgumentException("one timestamp per value");
    long total = 0;
    for (byte[] v : values) total += v.length;
    try (Arena a = Arena.ofConfined()) {
      MemorySegment msgs = a.allocate(Math.max(total, 1L));
      MemorySegment off = a.allocate(ValueLayout.JAVA_LONG, n + 1L);
      long at = 0;
      for (int i = 0; i < n; ++i) {
        byte[] v = values.get(i);
        off.setAtIndex(ValueLayout.JAVA_LONG, i, at);
        MemorySegment.copy(v, 0, msgs, ValueLayout.JAVA_BYTE, at, v.length);
        at += v.length;
      }
      off.setAtIndex(ValueLayout.JAVA_LONG, n, at);
      MemorySegment ts = a.allocateFrom(ValueLayout.JAVA_LONG, timestampsMs);
      if ((int) PROCESS_RAW.invokeExact(batcher, formatter, n, msgs, off, ts, formatThreads) != 0)
        throw new IllegalStateException("otm_batcher_process_raw");
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new IllegalStateException(t);
    }
  }

  /** Runs every queued operation (matcher calls included); take() then has their forwards. */
  public void flush() {
    try {
      if ((int) FLUSH.invokeExact(batcher) != 0) throw new IllegalStateException("otm_batcher_flush");
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new IllegalStateException(t);
    }
  }

  /** The records forwarded since the last call, in completion order (per key in stream order). */
  public List<Forward> take() {
    List<Forward> out = new ArrayList<>();
    final int max = 4096;
    try (Arena a = Arena.ofConfined()) {
      MemorySegment buf = a.allocate(FORWARD, max);
      while (true) {
        int n = (int) TAKE.invokeExact(batcher, buf, max);
        for (int i = 0; i < n; ++i) {
          MemorySegment f = buf.asSlice(i * FORWARD.byteSize(), FORWARD.byteSize());
          MemorySegment k = f.get(ValueLayout.ADDRESS, 0);
          MemorySegment b = f.get(ValueLayout.ADDRESS, 16);
          long kl = f.get(ValueLayout.JAVA_LONG, 8), bl = f.get(ValueLayout.JAVA_LONG, 24);
          // keys are the formatted topic's UTF-8 (StringSerializer); bodies as HttpClient reads them (UTF-8)
          out.add(new Forward(new String(k.reinterpret(kl).toArray(ValueLayout.JAVA_BYTE), StandardCharsets.UTF_8),
                              new String(b.reinterpret(bl).toArray(ValueLayout.JAVA_BYTE), StandardCharsets.UTF_8),
                              f.get(ValueLayout.JAVA_LONG, 32)));
          FREE.invokeExact(k);
          FREE.invokeExact(b);
        }
        if (n < max) return out;
      }
    } catch (RuntimeException e) {
      throw e;
    } catch (Throwable t) {
      throw new IllegalStateException(t);
    }
  }

  /** BatchingProcessor.close (:120-130): relaxed reports of every stored batch, then the handles released. */
  @Override
  public void close() {
    if (closed) return;
    closed = true;
    try {
      int rc = (int) CLOSE.invokeExact(batcher);
      DESTROY.invokeExact(batcher);
      FMT_DESTROY.invokeExact(formatter);
    } catch (Throwable t) {
      throw new IllegalStateException(t);
    }
  }
}
