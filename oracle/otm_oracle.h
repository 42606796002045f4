/*
 * otm_oracle.h -- CPU oracle for the /report hot path.  TEST INFRASTRUCTURE.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.  The
 * product (reporter_amd/, libotmatch.so) never links or calls it.
 *
 * What it restates:
 *   - py/reporter_service.py:110-215 (report) and :85-106/:218-264
 *     (parse_trace / handle_request / do) -- PINNED by tests/golden/ (JSON),
 *     generated from the reference itself (tests/golden/make_golden.py).
 *   - Valhalla 2.2.7 meili's SegmentMatcher.Match (called at
 *     py/reporter_service.py:112) -- a third-party C++ dependency absent from
 *     /root/reference and from this image (Dockerfile:7,25-28).  Restated as
 *     the written spec of DESIGN.md §3 (candidate search, emission,
 *     bounded-route transitions, Viterbi, route -> OSMLR segments), after
 *     meili's published algorithm.  PARITY UNPINNED against meili itself: no
 *     meili output exists anywhere this build can see.
 *   - py/generate_test_trace.py:9-29 (decode) -- pinned by
 *     tests/golden/decode_cases.json.
 */
#ifndef OTM_ORACLE_H
#define OTM_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#define ORC_KMAX 32

typedef struct orc_graph orc_graph;

typedef struct orc_params {
  float sigma_z, beta, max_route_distance_factor, breakage_distance;
  float interpolation_distance, search_radius, max_search_radius, gps_accuracy;
  int max_candidates;
  float turn_penalty_factor; /* meili auto costing: 200 (0 = no turn costs) */
} orc_params;

typedef struct orc_report_cfg {
  int n_report, n_transition;
  int64_t report_levels[32];
  int64_t transition_levels[32];
  double threshold_sec;
} orc_report_cfg;

/* record layouts identical to the product's C ABI records (include/otmatch.h)
 * so tests compare them field by field */
typedef struct orc_segment {
  int64_t segment_id;
  double start_time, end_time;
  int32_t length, queue_length, begin_shape_index, end_shape_index;
  int32_t way_off, way_cnt;
  uint32_t flags, pad;
} orc_segment;
typedef struct orc_report_rec {
  int64_t id, next_id;
  double t0, t1;
  int32_t length, queue_length;
  uint32_t flags, pad;
} orc_report_rec;
typedef struct orc_trace_result {
  int32_t code, error_kind, seg_off, seg_cnt, rep_off, rep_cnt, shape_used;
  int32_t successful_count, unreported_count, discontinuities, invalid_speeds, unassociated;
  int32_t successful_length, unreported_length;
} orc_trace_result;

typedef struct orc_counters {
  int64_t points, columns, cells_visited, cell_entries_scanned, candidates;
  int64_t searches, nodes_settled, edges_relaxed, transitions;
  int64_t route_searches, route_nodes_settled, route_edges_relaxed, route_edges;
  int64_t segments_out, reports_out;
  /* SURVEY §8(d)'s unique-edge term, per probe the distinct edges whose shape
     segments its scan projects and their shape points (counted only when the
     batch keeps its stages: the timed CPU baseline does not pay for it) */
  int64_t edges_projected, edge_shape_points;
} orc_counters;

typedef struct orc_results {
  int32_t n_traces, n_segments, n_reports, n_way_ids;
  orc_trace_result* traces;
  orc_segment* segments;
  orc_report_rec* reports;
  int64_t* way_ids;
  /* stage outputs (point-indexed; filled when keep_stages) */
  int64_t n_points;
  int32_t* ncand;      /* [P]        */
  int32_t* cand_edge;  /* [P*KMAX]   */
  float* cand_off;     /* [P*KMAX]   */
  float* cand_emis;    /* [P*KMAX]   */
  int64_t* trans_off;  /* [P+1]      */
  float* trans;        /* [trans_off[P]] */
  int32_t* state;      /* [P]        */
  int32_t* col_prev;   /* [P]        */
  float* route_dist;   /* [P]        */
  float* gc;           /* [P]        */
  orc_counters counters;
  float* ipos;         /* [P] interpolated points: route position in their step, -1 none */
} orc_results;

orc_graph* orc_graph_load(const char* path);
void orc_graph_free(orc_graph* g);
int64_t orc_graph_count(const orc_graph* g, int what); /* 0 nodes 1 edges 2 segments */
void orc_params_default(orc_params* p);
void orc_report_cfg_default(orc_report_cfg* c);
float orc_cos_deg(float deg);
/* turn-cost units (1/64 m) of a turn that deviates d degrees from straight
 * on, d = 0..180: round(factor * exp(-(180 - d) / 45) * 64) */
uint32_t orc_turn_units(float factor, int d);

/* Match a batch (host arrays).  nthreads >= 1 worker threads, one trace per
 * task.  keep_stages != 0 also fills the stage arrays. */
int orc_match_batch(const orc_graph* g, const orc_params* p, const orc_report_cfg* rc, int32_t n_traces,
                    const int64_t* trace_off, const float* lat, const float* lon, const double* time,
                    const float* accuracy, int nthreads, int keep_stages, orc_results* out);
void orc_results_free(orc_results* r);

/* JSON level.  Returns HTTP code; *body malloc'd (free with orc_free). */
int orc_handle_request(const orc_graph* g, const orc_params* p, const orc_report_cfg* rc, const char* path,
                       const char* body, size_t len, char** out, size_t* out_len);
int orc_match_json(const orc_graph* g, const orc_params* p, const char* req, size_t len, char** out,
                   size_t* out_len);
/* report() over a caller-supplied Match output (as the golden fixtures do).
 * Writes "Speed exceeds 200kph\n" lines into *stderr_out. */
int orc_report_segments(const orc_report_cfg* rc, const char* req, size_t len, const char* match_json,
                        size_t match_len, char** out, size_t* out_len, char** stderr_out);
/* JSON-path batch for the CPU baseline: n requests, nthreads workers. */
int orc_handle_batch(const orc_graph* g, const orc_params* p, const orc_report_cfg* rc, int n,
                     const char* const* bodies, const size_t* lens, int nthreads, int* codes, char** outs,
                     size_t* out_lens);
/* orc_handle_batch as a batcher matcher callback (otm_report_fn's shape,
 * include/otmatch.h): ctx points to an orc_handler_ctx.  The CPU baseline of
 * BASELINE config 5 hands it to otm_batcher_create, so the native batcher's
 * matcher calls reach the CPU oracle without leaving C. */
typedef struct {
  const orc_graph* g;
  const orc_params* p;
  const orc_report_cfg* rc;
  int nthreads;
} orc_handler_ctx;
int orc_batcher_handler(void* ctx, int n, const char* const* reqs, const size_t* lens, char** resps,
                        size_t* resp_lens, int* codes);
/* Python json.loads(s) then json.dumps(x, separators=(',',':')) */
int orc_json_redump(const char* s, size_t len, char** out, size_t* out_len);
/* py/generate_test_trace.py:9-29; out = [lon,lat]* pairs; returns count */
int64_t orc_decode_polyline6(const char* enc, size_t len, double* out, int64_t max_pairs);
void orc_free(void* p);

#endif
