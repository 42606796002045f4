/*
 * otmatch.h -- C ABI of libotmatch.so, the MI355X-native map matcher that
 * replaces the /report path of Open Traffic Reporter.
 *
 * What it replaces (reference = burritojustice/reporter):
 *   - the HTTP hop the Java batcher makes for every match request:
 *       String response = HttpClient.POST(url, post_body);
 *         src/main/java/org/opentraffic/reporter/Batch.java:63
 *         src/main/java/org/opentraffic/reporter/HttpClient.java:18-45
 *   - the Python service that answers it:
 *       SegmentMatcherHandler.handle_request / report
 *         py/reporter_service.py:218-240, :110-215
 *   - the Valhalla/meili matcher that service calls:
 *       valhalla.Configure(conf)          py/reporter_service.py:279
 *       valhalla.SegmentMatcher()          py/reporter_service.py:52
 *       SegmentMatcher.Match(json) -> json py/reporter_service.py:112
 *
 * Conventions: plain C types only; no exceptions cross this boundary; every
 * buffer the library returns is released with otm_free().  Status codes of
 * the request-level calls are the HTTP codes reporter_service.py would send
 * (200 / 400 / 500) and the body is byte-identical to what it would write.
 * Engine-level calls return 0 on success and a negative OTM_E* code on
 * failure, with a message available from otm_last_error().
 *
 * Thread safety: an engine handle may be used from many threads at once.
 */
#ifndef OTMATCH_H
#define OTMATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OTM_OK 0
#define OTM_EINVAL (-1)   /* bad argument / config                          */
#define OTM_EIO (-2)      /* graph file unreadable / malformed              */
#define OTM_EDEVICE (-3)  /* HIP runtime error (no device, OOM, fault)      */
#define OTM_ECONFIG (-4)  /* env config rejected (reporter_service.py:55-62) */
#define OTM_EAGAIN (-5)   /* async queue full                               */
#define OTM_ENOMEM (-6)   /* host allocation failed                         */

typedef struct otm_engine otm_engine;

/* ------------------------------------------------------------------ engine */

/* Create an engine: load the flattened graph named by the config file into
 * the HBM of devices[0] and read the matcher parameters.
 *   cfg_path: JSON file; {"otm":{"graph":"<.otmg path>"}, "meili":{"default":
 *             {sigma_z, beta, max_route_distance_factor, breakage_distance,
 *              interpolation_distance, search_radius, max_search_radius,
 *              max_candidates}}}.  Unknown keys are ignored.
 *   Env (read once, here): REPORT_LEVELS, TRANSITION_LEVELS, THRESHOLD_SEC
 *   with reporter_service.py's parsing (make_thread_locals, :51-62),
 *   including its quirk that THRESHOLD_SEC goes through strtobool: a value
 *   such as "15" is rejected with OTM_ECONFIG ("invalid truth value '15'"),
 *   where the reference's worker threads would die.
 * Replaces valhalla.Configure (py/reporter_service.py:279) + per-thread
 * SegmentMatcher() construction (:52).
 *   ndev == 1: one GPU.  ndev > 1: a multi-device engine for a host that
 *   drives several GPUs from one process (the Java host is one JVM): one
 *   member engine per entry of devices (a full graph + index replica each;
 *   a device may repeat).  Request-level calls (otm_report, otm_report_batch,
 *   otm_submit/otm_poll, otm_match_json) and the batcher send each trace to
 *   member (murmur2(uuid) & 0x7fffffff) % ndev -- Kafka's partition of the
 *   key, SURVEY.md §8(e) -- run the members concurrently and merge the
 *   results in request order; otm_match_soa splits its traces into
 *   point-balanced contiguous ranges (the binary batch carries no uuid).
 *   Device-side calls (otm_match_device, otm_hist_bind*) go to a member
 *   (otm_engine_member); info getters answer for member 0.  Multi-process
 *   runs (one engine per GPU process, RCCL reduce of the histograms) are
 *   DESIGN.md §8. */
int otm_engine_create(const char* cfg_path, const int* devices, int ndev,
                      otm_engine** out);
/* The matcher parameters a config file gives, without a device: meili's
 * "default" section with the mode's section ("meili.mode", default "auto")
 * on top, as valhalla.Configure (py/reporter_service.py:279) reads the meili
 * config.  otm_engine_create uses exactly these. */
typedef struct otm_meili_params {
  float sigma_z, beta, max_route_distance_factor, breakage_distance, interpolation_distance;
  float search_radius, max_search_radius, gps_accuracy, turn_penalty_factor;
  int32_t max_candidates;
} otm_meili_params;
int otm_config_meili(const char* cfg_path, otm_meili_params* out);
/* Members of an engine: ndev of a multi-device engine, 1 otherwise. */
int otm_engine_members(const otm_engine* eng);
/* Member i of a multi-device engine (NULL when out of range); a one-device
 * engine is its own member 0.  Owned by eng. */
otm_engine* otm_engine_member(otm_engine* eng, int i);
/* A second batch context on the same GPU (extension): its own HIP stream and
 * work buffers over the parent's HBM-resident graph, distance index and
 * configuration.  Batches on a parent and its clones run concurrently when
 * issued from different host threads (each handle serialises its own
 * calls), so one kernel's tail overlaps the next batch's head.  Destroy
 * clones before their parent. */
int otm_engine_clone(otm_engine* eng, otm_engine** out);
void otm_engine_destroy(otm_engine* eng);

/* Last error message for this thread (eng may be NULL). */
const char* otm_last_error(const otm_engine* eng);

/* Release any buffer returned by this library. */
void otm_free(void* p);

/* ---------------------------------------------------------- request level */

/* The /report endpoint, in process.  req = the POST body the Java batcher
 * builds (Batch.java:52-61).  Returns the HTTP status (200/400/500) and sets
 * *resp to the exact body reporter_service.py would send
 * (handle_request, py/reporter_service.py:218-240; do(), :259-264).
 * Replaces HttpClient.POST(url, body) at Batch.java:63. */
int otm_report(otm_engine* eng, const char* req, size_t len, char** resp,
               size_t* resp_len);

/* Many /report requests at once: one GPU batch.  codes[i], resps[i],
 * resp_lens[i] as for otm_report.  Returns 0 or a negative engine error. */
int otm_report_batch(otm_engine* eng, int n, const char* const* reqs,
                     const size_t* lens, char** resps, size_t* resp_lens,
                     int* codes);

/* Request arenas: page-locked host memory owned by the library that a host
 * writes its request bodies into -- the Java host's body.getBytes(ISO_8859_1)
 * (HttpClient.java:26 sends those bytes) into a MemorySegment over the arena
 * instead of a heap array (Batch.java:52-63).  otm_report_batch and
 * otm_submit_batch recognise bodies inside an arena and send them to HBM
 * straight from it, in pieces as large as the bodies lying back to back
 * allow: no staging copy and no submission copy.  The caller may reuse an
 * arena once otm_report_batch returns; bodies given to otm_submit_batch must
 * stay unchanged until their results are polled (the submission holds the
 * arena, so otm_request_arena_release only gives up the caller's hold).
 * NULL on failure (otm_last_error). */
void* otm_request_arena_alloc(size_t bytes);
int otm_request_arena_release(void* arena);

/* valhalla.SegmentMatcher().Match(json) (py/reporter_service.py:112):
 * request JSON (uuid + trace) in, {"segments":[...]} JSON out.  Returns 200
 * on success, 500 with {"error":...} otherwise. */
int otm_match_json(otm_engine* eng, const char* req, size_t len, char** resp,
                   size_t* resp_len);

/* report() of reporter_service.py:110-215 on the GPU (the k_report kernel)
 * over caller-supplied Match outputs: n requests and their
 * SegmentMatcher.Match JSON.  The segments are converted to typed records and
 * the kernel's stats, shape_used and reports are written around the Match
 * output passed through, as the reference does.  codes[i] / resps[i] as
 * otm_report_segments; codes[i] = 0 with an explanation in resps[i] where a
 * Match output does not fit the typed records (a field of another JSON type
 * than the matcher emits: the host otm_report_segments reproduces Python's
 * exception for those).  Returns 0 or a negative engine error. */
int otm_report_segments_device(otm_engine* eng, int n, const char* const* reqs,
                               const size_t* lens, const char* const* match_jsons,
                               const size_t* match_lens, char** resps,
                               size_t* resp_lens, int* codes);

/* report() with a caller-supplied matcher output: runs
 * reporter_service.py:110-215 over `match_json` (what SegmentMatcher.Match
 * returned) for the request `req`.  Lets a host keep any matcher and use the
 * native post-processing.  eng may be NULL (then the env is read now). */
int otm_report_segments(otm_engine* eng, const char* req, size_t len,
                        const char* match_json, size_t match_len, char** resp,
                        size_t* resp_len);

/* Async form of otm_report for hosts that cannot block per key (the Kafka
 * Streams processor issues one blocking POST per record today,
 * BatchingProcessor.java:69).  Requests submitted before a poll are matched
 * together in one GPU batch; results for one tag come back once, results of
 * one uuid in submit order. */
typedef struct otm_result {
  uint64_t tag;
  int code;
  char* body; /* release with otm_free */
  size_t body_len;
} otm_result;
int otm_submit(otm_engine* eng, const char* req, size_t len, uint64_t tag);
/* n requests at once (a Kafka poll's records): the same as n otm_submit
 * calls in order, the bodies copied over the library's host threads.  The
 * async path is a pipeline: each worker runs whole request batches on its
 * own batch context (OTM_ASYNC_WORKERS, default 3; OTM_ASYNC_BATCH requests
 * per batch, default 16384), so one batch's parse and response writing overlap
 * another's GPU work; results are published in submit order. */
int otm_submit_batch(otm_engine* eng, int n, const char* const* reqs, const size_t* lens, const uint64_t* tags);
/* Fills up to max results; waits at most timeout_us for the first one.
 * Returns the number filled (>=0) or a negative engine error. */
int otm_poll(otm_engine* eng, otm_result* out, int max, int timeout_us);

/* Java request encoder (Batch.report + Point.Serder.put_json,
 * Batch.java:52-61, Point.java:39-45): float32 lat/lon through
 * DecimalFormat("###.######") HALF_EVEN, long time, int accuracy, in the
 * bytes HttpClient.POST sends: new StringEntity(body) is ISO-8859-1
 * (HttpClient.java:26), so the uuid -- the Kafka record key, given here as
 * its UTF-8 bytes and read as StringDeserializer reads it (JDK 8, U+FFFD for
 * malformed input) -- goes out unescaped with U+0080..U+00FF as single bytes
 * and anything above U+00FF as '?'.  Such a body is what the reference
 * service answers 400 ('utf-8' codec ...) when a Latin-1 byte breaks its
 * body.decode('utf-8') (py/reporter_service.py:99); otm_report answers it
 * the same.  *out is allocated by the library. */
int otm_encode_request(const char* uuid, int n, const float* lat,
                       const float* lon, const int64_t* time,
                       const int32_t* accuracy, char** out, size_t* out_len);

/* The points of one /report request body, as the matcher reads them
 * (parse_trace + handle_request validation, py/reporter_service.py:85-106,
 * 218-234, then each point's lat, lon, time and accuracy).  fast = 1 takes
 * the DOM-free reader of the Java batcher's own bytes and returns -2 for a
 * body outside its grammar (a request batch then takes the DOM path); fast =
 * 0 always parses the DOM.  Returns the point count (at most max_points are
 * written) with the uuid copied when it is a JSON string (NUL-terminated,
 * truncated to uuid_cap), -1 for a request the DOM path rejects. */
int otm_request_points(const char* req, size_t len, int fast, float* lat, float* lon, double* time, float* acc,
                       int max_points, char* uuid, size_t uuid_cap);

/* ----------------------------------------------------------- binary level */

/* A batch of traces, structure of arrays.  Points of trace t are
 * [trace_off[t], trace_off[t+1]).  The same struct describes host buffers
 * (otm_match_soa) or device buffers (otm_match_device). */
typedef struct otm_batch {
  int32_t n_traces;
  int64_t n_points;
  const int64_t* trace_off; /* n_traces + 1 */
  const float* lat;
  const float* lon;
  const double* time;    /* epoch seconds */
  const float* accuracy; /* metres; <= 0 means "not given" (gps_accuracy) */
} otm_batch;

/* One matched OSMLR segment (the elements of "segments", README.md:152-165). */
typedef struct otm_segment {
  int64_t segment_id;   /* -1: no OSMLR association (key omitted in JSON) */
  double start_time;    /* valid only if (flags & OTM_SEG_START_VALID)     */
  double end_time;      /* valid only if (flags & OTM_SEG_END_VALID)       */
  int32_t length;       /* metres, -1 if partially traversed               */
  int32_t queue_length; /* always 0 in this era                           */
  int32_t begin_shape_index;
  int32_t end_shape_index;
  int32_t way_off; /* into otm_results.way_ids */
  int32_t way_cnt;
  uint32_t flags;
  uint32_t pad;
} otm_segment;
#define OTM_SEG_START_VALID 1u
#define OTM_SEG_END_VALID 2u
#define OTM_SEG_INTERNAL 4u
/* start_time / end_time came from a JSON int literal (segments handed to
 * otm_report_segments_device; the matcher itself emits floats, and the int -1
 * of an invalid time is "not VALID") */
#define OTM_SEG_START_INT 8u
#define OTM_SEG_END_INT 16u

/* One datastore report (reporter_service.py:160-166). */
typedef struct otm_report_rec {
  int64_t id;
  int64_t next_id; /* -1: key absent */
  double t0;
  double t1; /* the JSON value is an int when (flags & OTM_REP_T1_INT): for
                the matcher's own segments that is the -1 of a partial next
                segment (reporter_service.py:160) */
  int32_t length;
  int32_t queue_length;
  uint32_t flags;
  uint32_t pad;
} otm_report_rec;
#define OTM_REP_T1_INT 1u
#define OTM_REP_T1_INT_MINUS1 OTM_REP_T1_INT /* the name of round 1 */
#define OTM_REP_T0_INT 2u

/* Per-trace outcome: the stats block (reporter_service.py:201-213),
 * shape_used (:125-127) and where the trace's segments/reports live. */
typedef struct otm_trace_result {
  int32_t code; /* 200, or 500 (error_kind says why) */
  int32_t error_kind;
  int32_t seg_off, seg_cnt;
  int32_t rep_off, rep_cnt;
  int32_t shape_used; /* -1 == None */
  int32_t successful_count;
  int32_t unreported_count;
  int32_t discontinuities;
  int32_t invalid_speeds;
  int32_t unassociated;
  int32_t successful_length; /* metres of the LAST counted segment, -1 none */
  int32_t unreported_length; /* ditto */
} otm_trace_result;
#define OTM_TERR_NONE 0
#define OTM_TERR_ZERODIV 1         /* "float division by zero" */
/* 2 and 3 were the 256-edge and 98,304-label spec limits until round 3;
 * round 4 has no such limits (the batch's tables grow on demand), so they
 * only report what cannot happen on a consistent graph (a finite transition
 * whose route search misses its target) or a failed host allocation */
#define OTM_TERR_CAND_OVERFLOW 2   /* (oracle) candidate workspace allocation failed */
#define OTM_TERR_SEARCH_OVERFLOW 3 /* a route search could not reproduce its transition */
#define OTM_TERR_ZERODIV_INT 4     /* "division by zero" (int / int in report()) */

/* Host-side result arrays of one batch (owned by the engine until the next
 * call on the same thread's engine, or copy them). */
typedef struct otm_results {
  int32_t n_traces;
  int32_t n_segments;
  int32_t n_reports;
  int32_t n_way_ids;
  const otm_trace_result* traces;
  const otm_segment* segments;
  const otm_report_rec* reports;
  const int64_t* way_ids;
} otm_results;

/* Match a host-resident batch; results copied back to host.  Inputs in
 * pinned memory (otm_host_alloc) go to the device by DMA at full PCIe speed;
 * pageable inputs are staged by the HIP runtime. */
int otm_match_soa(otm_engine* eng, const otm_batch* in, otm_results* out);
/* The same batch in the Java host's own types, narrowed for the link (14 B
 * per point instead of 24): Point's float lat/lon, its long time as an int32
 * delta from a per-trace int64 base (epoch seconds), its int accuracy as an
 * int16 (Point.java:16-25; Batch.java:52-61 sends exactly these integers).
 * time[i] = (double)(time_base[t] + time_delta[i]), accuracy[i] =
 * (float)accuracy16[i] -- widened on the device, results identical to
 * otm_match_soa on the widened batch.  A trace whose times span more than
 * 2^31 s or whose accuracies leave [-32768, 32767] goes through
 * otm_match_soa instead. */
typedef struct otm_batch_compact {
  int32_t n_traces;
  int64_t n_points;
  const int64_t* trace_off;  /* n_traces + 1 */
  const int64_t* time_base;  /* n_traces: epoch seconds */
  const float* lat;
  const float* lon;
  const int32_t* time_delta; /* seconds after the trace's time_base */
  const int16_t* accuracy;   /* metres; <= 0 means "not given" */
} otm_batch_compact;
int otm_match_compact(otm_engine* eng, const otm_batch_compact* in, otm_results* out);
/* Page-locked host memory for a host's batch buffers (hipHostMalloc): a Java
 * host maps it as a MemorySegment and fills its SoA arrays in place.
 * NULL on failure; release with otm_host_free (not otm_free). */
void* otm_host_alloc(size_t bytes);
void otm_host_free(void* p);

/* Match a batch whose arrays are already in this engine's device memory.
 * Results stay on the device (fetch with otm_fetch_results).  `stream` is a
 * hipStream_t (NULL = the engine's own stream); the call returns after the
 * work is enqueued and the variable-size outputs are sized. */
int otm_match_device(otm_engine* eng, const otm_batch* in_dev, void* stream);
int otm_fetch_results(otm_engine* eng, otm_results* out);
/* A stream for otm_match_device on the engine's device: own_queue != 0 gives it
 * a hardware queue of its own (a full CU mask), apart from the runtime's pool
 * of GPU_MAX_HW_QUEUES queues that every other stream of the process shares.
 * NULL on failure; release with otm_stream_destroy. */
void* otm_stream_create(otm_engine* eng, int own_queue);
void otm_stream_destroy(void* stream);

/* Per-segment speed histogram, accumulated on the device by every match
 * call: counts u32[n_segments * nbins], bin = floor(kph / bin_kph) clamped to
 * nbins-1, one count per datastore report.  The buffer is CALLER-owned device
 * memory (e.g. a torch tensor) so the host can reduce it across GPUs with
 * RCCL.  Pass NULL to stop accumulating. */
int otm_hist_bind(otm_engine* eng, void* dev_counts, int nbins, float bin_kph);
/* The same, with a second channel beside the counts: the sum
 * of the reports' speeds per segment, u64[n_segments] in units of 1/1000
 * km/h (fixed point, so sums are exact and independent of the order the
 * GPU adds them in), also caller-owned device memory.  A binding reaches the
 * engine's clones at their next batch. */
int otm_hist_bind_ex(otm_engine* eng, void* dev_counts, int nbins, float bin_kph,
                     void* dev_speed_sum);
int otm_graph_info(const otm_engine* eng, int64_t* n_nodes, int64_t* n_edges,
                   int64_t* n_segments);

/* The bounded route index built at engine creation (config
 * "otm":{"index_radius_m": R}, 0 = none; absent: sized from the graph's node
 * density, ~140 nodes per row, capped at max_route_distance_factor x
 * breakage_distance, and shrunk to fit half the free HBM): for every search
 * source (an edge's end entered along it, or a node), every label within R
 * road metres with its cost, distance, turn units and predecessor.
 * Transition and route queries whose bound 5 x gc exceeds R, or whose row
 * overflowed the builder, run the online bounded search instead; the results
 * are identical either way. */
int otm_index_info(const otm_engine* eng, float* rmax, int64_t* entries,
                   int32_t* incomplete_rows, float* build_ms);

/* The near indexes: the same rows at smaller radii (config
 * "otm":{"index_near_m": [r, ...]}, [] = none; absent: one at 0.45 R when the
 * index's tables reach 16 GB).  A transition or route query probes the
 * smallest whose radius covers its bound, so its probes land in smaller
 * tables; results are identical.  Writes up to `cap` radii (smallest first)
 * and entry counts; returns the number of near indexes, or < 0 on error. */
int otm_index_levels(const otm_engine* eng, float* radii, int64_t* entries, int cap);

/* The route index's device tables, full and near indexes together: hash
 * slots and their bytes (16 B a slot, the label's predecessor inside), and
 * the full index's table load in percent -- 30 when the tables fit half the
 * free HBM (53 B per entry), else 40 (40 B per entry) before the radius is
 * cut. */
int otm_index_tables(const otm_engine* eng, int64_t* slots, int64_t* bytes, int32_t* load_pct);

/* The candidate search's grid index on the device: the graph file's cells
 * (meili's 500 per 0.25 deg tile) merged mult x mult (config
 * "otm":{"grid_mult": m} or env OTM_GRID_MULT; absent or 0: chosen from the
 * graph's entry density and the search radius).  Coarser cells change how
 * many cells and entries a probe visits, never the candidates. */
int otm_grid_info(const otm_engine* eng, double* cell_deg, int32_t* rows, int32_t* cols,
                  int64_t* entries, int32_t* mult);

/* Work counters of the last batch (for the roofline's algorithmic bytes). */
typedef struct otm_work_counters {
  int64_t points, columns, cells_visited, cell_entries_scanned, candidates;
  int64_t searches, nodes_settled, edges_relaxed, transitions; /* K4 */
  int64_t route_searches, route_nodes_settled, route_edges_relaxed, route_edges; /* K6 */
  int64_t segments_out, reports_out;
} otm_work_counters;
/* Enable (1) or disable (0) counting; counting runs extra atomics, so timed
 * runs keep it off. */
int otm_set_counting(otm_engine* eng, int on);
int otm_get_counters(otm_engine* eng, otm_work_counters* out);

/* Per-stage timings (ms) of the last otm_match_device call, from HIP events
 * on the engine stream: [columns, candidates, trans_size, transitions,
 * viterbi, route, segments, report].  Enabled with otm_set_timing. */
int otm_set_timing(otm_engine* eng, int on);
int otm_get_stage_ms(otm_engine* eng, float* ms, int n);

/* Per-kernel timings (ms) of the last otm_match_device call (same HIP events,
 * one pair around each launch; enabled with otm_set_timing).  Kernel k is
 * named by otm_kernel_name(k), 0 <= k < OTM_NUM_KERNELS; the stage timings
 * above are sums of these. */
#define OTM_NUM_KERNELS 18
int otm_get_kernel_ms(otm_engine* eng, float* ms, int n);
const char* otm_kernel_name(int k);

/* How much work of the last batch each fallback tier took:
 * probes the lane candidate tier handed to the wave tier; transition columns
 * the route index could not answer (trans_online), then those the LDS wave
 * search spilled to the global-memory search (trans_global); the same for the
 * route stage's steps.  trans_wave / route_wave are kept for the layout and
 * equal trans_online / route_online: every online search starts in the LDS
 * wave tier since round 3 (the lane-per-search tier is gone). */
typedef struct otm_spill_stats {
  int32_t cand_wave;
  int32_t trans_online, trans_wave, trans_global;
  int32_t route_online, route_wave, route_global;
  /* round 4, no spec limits: probes with more distinct edges in their radius
   * than the LDS tier holds (cand_big), searches past the global tier's
   * label limit (trans_huge / route_huge), and how many times the batch was
   * run to size its buffers and tables (attempts, 1 = no redo) */
  int32_t cand_big, trans_huge, route_huge, attempts;
  /* round 6: of those runs, how many resumed from the tier whose tables grew
   * (the stages before it kept their results) instead of redoing the batch */
  int32_t resumed;
} otm_spill_stats;
/* The stats (like otm_get_stage_ms / otm_get_kernel_ms / otm_get_counters)
 * describe the last batch run on this handle's own batch context.  An
 * otm_report_batch of 4,096 requests or more runs its two halves on the
 * engine's clones, and otm_submit / otm_submit_batch run on the async
 * pipeline's clones: those batches do not update the handle's figures (each
 * clone keeps its own, and grows its own on-demand tier tables). */
int otm_get_spill_stats(otm_engine* eng, otm_spill_stats* out);

/* Stage outputs of the last batch, for parity tests (device -> host copy).
 * what: 0 ncand i32[P], 1 cand_edge i32[P*KMAX], 2 cand_off f32[P*KMAX],
 * 3 cand_emis f32[P*KMAX], 4 trans_off i64[P+1], 5 trans f32[total],
 * 6 state i32[P], 7 col_prev i32[P], 8 route_dist f32[P], 9 gc f32[P],
 * 10 ipos f32[P]; the batch inputs as the GPU request reader decoded them
 * (otm_report_batch; also a host batch of more than 2^18 points): 11 trace_off
 * i64[T+1], 12 lat f32[P], 13 lon f32[P], 14 time f64[P], 15 accuracy f32[P]. */
int otm_debug_fetch(otm_engine* eng, int what, void* dst, size_t bytes,
                    size_t* needed);
int otm_kmax(void);
/* The GPU response writer's float formatting run on the host (test hooks):
 * Python's repr of d into out (>= 32 bytes), its length or -1 where the
 * writer leaves a body to the host writer; py_round3 as report() rounds
 * lengths, 1 or 0 (unsupported). */
int otm_debug_py_repr(double d, char* out);
int otm_debug_py_round3(double x, double* out);
/* Test hook: the response arenas' otm_free under contention from threads
 * (each round: every thread cuts bodies from an arena, then all free a
 * strided share of everyone's, with plain allocations through the same
 * scan).  Returns the arenas left live after (0 expected), -1 on bad args. */
int otm_debug_arena_stress(int threads, int rounds);
/* Test hook: the chunks eng's last otm_report_batch was split into (one per
 * batch context, run concurrently; 1: not split). */
int otm_debug_last_split(const otm_engine* eng);
/* Which HIP runtime this library is bound to ("<path> hip_runtime_version=N"):
 * a host that also runs torch must load torch first so both share one. */
const char* otm_runtime_info(void);

/* ------------------------------------------------------------- host batcher */
/* Native restatement of the reference's Kafka Streams batcher -- Batch
 * (Batch.java:16-84) and BatchingProcessor (BatchingProcessor.java:19-133):
 * per-uuid batches, the 500 m / 10 points / 60 s report gates, the trim at
 * shape_used, the session-gap clean() with its relaxed (0, 2, 0) reports and
 * close().  A key's operations run in the reference's serial order; the
 * requests of all keys that are ready go to the matcher as one GPU batch.
 * Used as the config-5 driver (sustained ingest) and as a native host. */
typedef struct otm_batcher otm_batcher;
typedef struct otm_batcher_cfg {
  int32_t report_dist;    /* REPORT_DIST, metres (BatchingProcessor.java:30)  */
  int32_t report_count;   /* REPORT_COUNT, points (:29)                      */
  int64_t report_time_s;  /* REPORT_TIME, seconds (:28)                      */
  int64_t session_gap_ms; /* SESSION_GAP, ms of record time (:31)            */
  int32_t max_batch;      /* requests per matcher call (0: all ready ones)   */
  int32_t json_path;      /* 1: engine requests go through the JSON /report
                             path (otm_report_batch) instead of the binary one */
  int64_t max_pending;    /* otm_batcher_process drains once this many
                             operations are queued (0: only on flush/close)  */
  int32_t threads;        /* host threads for running keys, building batches
                             and applying responses (0 or 1: the caller's) */
  int32_t reserved;
} otm_batcher_cfg;
void otm_batcher_defaults(otm_batcher_cfg* cfg);
/* A /report handler for n request bodies (the HttpClient.POST of
 * Batch.java:63): fills codes / bodies; bodies must be malloc'd (the batcher
 * frees or forwards them).  Returns 0. */
typedef int (*otm_report_fn)(void* ctx, int n, const char* const* reqs, const size_t* lens, char** resps,
                             size_t* resp_lens, int* codes);
/* eng: the matcher (fn == NULL); or fn/ctx: any /report handler (eng may be NULL).
 * A batcher is one stream task, like the processor it restates: call it from
 * one thread at a time (its own thread team, cfg.threads, is internal; the
 * handler fn is only ever called from the calling thread). */
int otm_batcher_create(otm_engine* eng, const otm_batcher_cfg* cfg, otm_report_fn fn, void* ctx,
                       otm_batcher** out);
void otm_batcher_destroy(otm_batcher* b);
/* Formatted records in stream order: (key, Point, record timestamp in ms)
 * (BatchingProcessor.process, :56-85, with context.timestamp() = ts_ms).
 * keys are the records' key bytes on the formatted topic, read as Kafka's
 * StringDeserializer reads them (JDK 8 UTF-8, U+FFFD for malformed input:
 * keys that decode to one Java String are one key; forwarded keys are that
 * String's UTF-8).  Each request body carries the key as HttpClient sends it
 * (otm_encode_request): in binary mode a key whose body the service would
 * reject or read differently (a Latin-1 byte, a quote, a backslash, a
 * control character) is answered through the byte-level /report path, so
 * it gets the reference's response (its 400 body included). */
int otm_batcher_process(otm_batcher* b, int n, const char* const* keys, const size_t* key_lens, const float* lat,
                        const float* lon, const int32_t* accuracy, const int64_t* time, const int64_t* ts_ms);
/* Run every queued operation to completion (matcher calls included). */
int otm_batcher_flush(otm_batcher* b);
/* BatchingProcessor.close (:120-130): flush, then a relaxed report of every
 * stored batch (responses discarded). */
int otm_batcher_close(otm_batcher* b);
/* context.forward(key, response) of process() (:70-71), in completion order;
 * seq = the record's position in the stream (per key increasing).  key and
 * body are released with otm_free. */
typedef struct otm_forward {
  char* key;
  size_t key_len;
  char* body;
  size_t body_len;
  int64_t seq;
} otm_forward;
int otm_batcher_take(otm_batcher* b, otm_forward* out, int max);
typedef struct otm_batcher_stats {
  int64_t records, clean_ops, close_ops, requests, request_points, match_batches, forwarded;
  int64_t null_batch_in_clean; /* clean() on a key with no stored batch: the reference throws */
  int64_t keys, stored_batches, stored_points;
  /* host time (us) in: queueing records, running keys' operations, building
   * the matcher batches, the matcher itself, applying responses */
  int64_t us_enqueue, us_run, us_prepare, us_match, us_apply;
  /* otm_batcher_process_raw: messages in, messages the formatter dropped,
   * host time (us) formatting */
  int64_t raw_messages, raw_dropped, us_format;
  /* requests answered null because the handler failed (HttpClient.POST's
   * transport failure: the batch is cleared, nothing forwarded) */
  int64_t null_responses;
} otm_batcher_stats;
int otm_batcher_get_stats(const otm_batcher* b, otm_batcher_stats* out);
/* A key's stored batch (points in order, max_separation); returns its size
 * (copies at most max points) or -1 when the store has no batch for it. */
int otm_batcher_batch(const otm_batcher* b, const char* key, size_t key_len, int max, float* lat, float* lon,
                      int32_t* accuracy, int64_t* time, float* max_separation);

/* ------------------------------------------------------- ingest formatter */
/* The reference's raw-message Formatter, native:
 * src/main/java/org/opentraffic/reporter/Formatter.java.  `spec` is the
 * --formatter string (Reporter.java:33-43, Formatter.GetFormatter :36-51):
 *   "<c>sv<c><separator regex><c>uuid<c>lat<c>lon<c>time<c>accuracy[<c>time pattern]"
 *   "<c>json<c>uuid key<c>lat key<c>lon key<c>time key<c>accuracy key[<c>time pattern]"
 * with <c> the spec's own first character.  Fails (OTM_EINVAL, message in
 * err) where GetFormatter throws, and for separator regexes / joda patterns
 * outside the supported subset (reporter_amd/csrc/formatter.h). */
typedef struct otm_formatter otm_formatter;
int otm_formatter_create(const char* spec, otm_formatter** out, char* err, size_t err_len);
void otm_formatter_destroy(otm_formatter* f);
/* Formatter.format (:86-124) of n raw messages, message i = msgs[off[i],
 * off[i+1]).  ok[i] = 0 where the reference throws and
 * KeyedFormattingProcessor (:30-37) logs and drops the message.  Key i (the
 * uuid) = keys[key_off[i], key_off[i+1]).  Arrays are library-owned: release
 * with otm_formatted_free.  nthreads > 1 splits large calls across threads. */
typedef struct otm_formatted {
  int32_t n, n_ok;
  uint8_t* ok;
  int64_t* key_off;
  char* keys;
  float* lat;
  float* lon;
  int32_t* accuracy;
  int64_t* time;
} otm_formatted;
int otm_format(const otm_formatter* f, int32_t n, const char* msgs, const int64_t* off, int nthreads,
               otm_formatted* out);
void otm_formatted_free(otm_formatted* r);
/* KeyedFormattingProcessor -> BatchingProcessor: format n raw messages and
 * feed every formatted one to the batcher (otm_batcher_process), message i
 * with record timestamp ts_ms[i]; dropped messages are counted (raw_dropped). */
int otm_batcher_process_raw(otm_batcher* b, const otm_formatter* f, int32_t n, const char* msgs,
                            const int64_t* off, const int64_t* ts_ms, int nthreads);

/* The coordinate a request body carries to the matcher: DecimalFormat
 * ("###.######", HALF_EVEN on the exact value; Point.java:29) parsed back to
 * float.  The batcher's binary path applies it so that it matches what the
 * JSON path (and the reference's HTTP hop) delivers. */
void otm_quantize_decimal6(const float* in, float* out, int64_t n);

/* --------------------------------------------------- synthetic inputs ---- */
/* Harness tooling, not the hot path: the seeded synthetic road network and
 * probe traces of SURVEY.md §8(d) (no real Valhalla tiles exist here). */
typedef struct otm_synth_graph_params {
  double center_lat, center_lon;
  double width_m, height_m;
  double block_m;  /* grid spacing (150 m city) */
  double jitter_m; /* node position jitter (+-) */
  int arterial_every;
  int highway_every;
  double unassoc_frac; /* local street blocks without OSMLR coverage */
  int complex_every;   /* >0: crossings of lines that are multiples of this
                          become 4-node squares of internal edges */
  double seg_max_m;    /* OSMLR segment max length */
  double cell_deg;     /* grid index cell (meili grid.size 500 / 0.25 deg) */
  uint64_t seed;
} otm_synth_graph_params;
void otm_synth_graph_defaults(otm_synth_graph_params* p);
int otm_synth_graph(const otm_synth_graph_params* p, const char* out_path);

typedef struct otm_synth_trace_params {
  int32_t n_vehicles;
  int32_t points_per_vehicle;
  double interval_s;
  double noise_sigma_m;
  float accuracy;
  double t0;
  uint64_t seed;
  int32_t vehicle_offset; /* global index of vehicle 0 (for sharding) */
  const int32_t* vehicle_ids; /* optional: global index of each vehicle */
} otm_synth_trace_params;
/* Fills caller-allocated arrays sized n_vehicles*points_per_vehicle (lat,
 * lon, time, accuracy, true_edge, true_off) and n_vehicles+1 (trace_off).
 * Graph is read from graph_path. */
int otm_synth_traces(const char* graph_path, const otm_synth_trace_params* p,
                     int64_t* trace_off, float* lat, float* lon, double* time,
                     float* accuracy, int32_t* true_edge, float* true_off);

/* Valhalla's tile hierarchy as py/get_tiles.py computes it (:30-172): levels
 * 0 / 1 / 2 = 4 / 1 / 0.25 degree tiles over the world bbox.  otm_tile_id:
 * Row(lat) * ncolumns + Col(lon), -1 outside.  otm_tile_file: GetFile
 * (:82-102), e.g. "2/000/603/124.gph"; returns 0, or the buffer size needed
 * when cap is too small.  otm_tile_files_bbox: the files the script lists for
 * a bbox (split at the antimeridian), newline-separated, levels ascending;
 * *out released with otm_free.  The real-tile flattener
 * names its inputs with these; the synthetic one its OSMLR tile bits. */
int64_t otm_tile_id(int level, double lat, double lon);
int otm_tile_file(int64_t tile_id, int level, const char* suffix, char* out, size_t cap);
int otm_tile_files_bbox(double minx, double miny, double maxx, double maxy, const char* suffix,
                        char** out, size_t* out_len);

/* The ground truth behind otm_synth_traces (same generator and seeds): the
 * edges each vehicle drives from its first probe to its last, in order.
 * path_off[n_vehicles + 1]; at most cap edges are written; returns the total
 * edge count (cap 0 sizes the call) or a negative error. */
int64_t otm_synth_true_paths(const char* graph_path, const otm_synth_trace_params* p,
                             int64_t* path_off, int32_t* path_edges, int64_t cap);
/* The same with the time (epoch seconds) the vehicle entered each path edge
 * (it drives each edge at constant speed; the first edge's entry precedes the
 * first probe): the true segment times behind the datastore-report accuracy
 * figure (reporter_amd/synth.py report_agreement). */
int64_t otm_synth_true_paths_timed(const char* graph_path, const otm_synth_trace_params* p,
                                   int64_t* path_off, int32_t* path_edges, double* enter_time, int64_t cap);

/* Kafka's default key partitioner (murmur2, seed 0x9747b28c) -- the shard of
 * a uuid: (murmur2(key) & 0x7fffffff) % n. */
int32_t otm_murmur2(const char* key, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* OTMATCH_H */
