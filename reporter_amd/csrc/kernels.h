// kernels.h -- device data views and launch wrappers of the matcher kernels.
//
// Pipeline of one batch, all on one HIP stream:
//   K1 k_columns      thread / trace   interpolation filter, gc to previous column
//   K2 k_candidates   wave / probe     grid cells -> projections -> LDS edge hash
//                                      -> bitonic sort -> top-K + emission
//   K3 k_links        thread / point   chain links + transition-matrix sizes, scan
//   K4 k_trans_sub    8/16 lanes / col route-index probes per (source, target)
//                                      pair; k_transitions: turn-aware search
//                                      per source for what the index cannot
//                                      answer (LDS, then global tier)
//   K5 k_viterbi      wave / trace     min-sum decode, lanes = states
//   K6 k_route_index  thread / step    the winning label's predecessor chain (k_route: search)
//   K7 k_segments     thread / trace   traversals -> OSMLR segments (count+write)
//   K8 k_report       thread / trace   reporter_service.py:110-215 + histogram
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "otmatch.h"

namespace otm {

constexpr int KMAX = 32;           // max candidates per column (== ORC_KMAX)
// inline candidate slots per point (DevWork::cand_eo / cand_em); 4 (a point's
// blocks half the size, slots 4.. in the overflow) measured slower on configs
// 2 and 4
constexpr int KIN = 8;
static_assert(KIN == 4 || KIN == 8, "inline blocks of 4 or 8 slots (whole 16-B emission pieces)");
constexpr int KX = KMAX - KIN;     // overflow candidate slots per point (DevWork::cand_xeo / cand_xem)
constexpr int MAX_HITS = 256;      // distinct edges within one radius in the LDS tiers (beyond: the global tier)
constexpr int SEARCH_LIMIT = 98304;  // labels (edges + nodes) of one global-tier search (beyond: the huge tier)
constexpr int LDS_TABLE_CAP = 256;   // K4/K6 LDS tier: table slots
constexpr int LDS_TABLE_LIMIT = 192; // ... labels before spilling to the global tier
constexpr int BIG_TABLE_LOG2 = 17;
constexpr int BIG_TABLE_CAP = 1 << BIG_TABLE_LOG2;  // global tier table slots (> SEARCH_LIMIT / 0.75)
#ifndef OTM_BIG_SLOTS
#define OTM_BIG_SLOTS 512
#endif
constexpr int BIG_SLOTS = OTM_BIG_SLOTS;  // concurrent global-tier searches
// The huge search tier (round 4): searches beyond SEARCH_LIMIT labels, in
// HUGE_SLOTS tables of 2^huge_log2 slots sized by the host (grown and the
// batch redone when a search does not fit: no label limit but memory)
constexpr int HUGE_SLOTS = 8;
// The candidate search's HBM tier (round 4): probes with more than MAX_HITS
// distinct edges within their radius, CAND_BIG_SLOTS at a time, in tables of
// 2^cand_log2 slots (half of them the sort keys) sized like the huge tier.
constexpr int CAND_BIG_SLOTS = 64;
// the largest tables the host grows the two on-demand tiers to (8 x 2^27 huge
// slots ~ 29 GB, 64 x 2^23 candidate slots ~ 8.6 GB; env OTM_HUGE_MAX_LOG2 /
// OTM_CAND_MAX_LOG2 lower them, test hooks): past them, or when HBM runs out,
// a search or probe that does not fit fails its own trace with a 500, not
// the batch
constexpr int HUGE_MAX_LOG2 = 27, CAND_MAX_LOG2 = 23;
__host__ __device__ inline int huge_limit(int log2) { return log2 > 2 ? 3 << (log2 - 2) : 0; }  // 0.75 x slots

struct DevGraph {
  const float *node_lat, *node_lon;
  const int32_t* out_off;
  const int32_t *e_from, *e_to;
  const float* e_len;
  const int32_t* e_shape_off;
  const int64_t* e_way;
  const int32_t *e_seg, *e_seg_pos;
  const uint8_t* e_flags;
  const float *s_lat, *s_lon, *s_cum;
  const uint64_t* g_id;
  const float* g_len;
  const uint32_t* cell_off;  // 32-bit in HBM (engine_init checks the entry count)
  const uint32_t* cell_ent;
  const float4* ent_geo;  // per cell entry: shape segment endpoints (lat_a, lon_a, lat_b, lon_b)
  const uint16_t *e_head_out, *e_head_in;  // edge bearing at start / end, whole degrees (turn costs)
  const uint32_t* e_len64;                 // L(e) = round(len(e) x 64): the route searches' edge costs (1/64 m)
  // K7's per-edge record {len bits, seg, seg_pos | flags << 24, way number}
  // and the way numbers' ids (engine.cpp)
  const uint4* e_rec;
  const int2* e_fl;  // {from node, length bits} per edge: a transition source's row and start in one load
  const int64_t* way_tab;
  int32_t n_nodes, n_edges, n_segments, grid_rows, grid_cols;
  double lat0, lon0, cell;
  // spatial work order tiles: the node bbox cut into ORDER_SIDE^2 tiles
  float bb_lat0, bb_lon0, bb_inv_h, bb_inv_w;  // tile row = (lat - bb_lat0) * bb_inv_h, ...
};

// Spatial work order of a batch's columns: column points
// bucketed by the Hilbert index of their tile, the tiles cut into 8
// equal-count groups.  Group g runs on the blocks with blockIdx % 8 == g,
// which the dispatcher deals to one XCD, so each XCD's L2 holds one region's
// grid cells and index rows; inside a group, neighbouring lanes and waves get
// neighbouring probes.
#ifndef OTM_ORDER_BITS
#define OTM_ORDER_BITS 6
#endif
constexpr int ORDER_BITS = OTM_ORDER_BITS;  // <= 8: tile ids are u16
constexpr int ORDER_SIDE = 1 << ORDER_BITS;  // 64 x 64 tiles
constexpr int ORDER_TILES = ORDER_SIDE * ORDER_SIDE;
constexpr int ORDER_GROUPS = 8;
struct DevOrder {
  int32_t* item;      // [n] column points, grouped
  int32_t* grp;       // [ORDER_GROUPS + 1] group starts in item space
  uint16_t* tile;     // [P] tile of each column (K1)
  int32_t* tile_cnt;  // [ORDER_TILES] columns per tile (K1); nullptr: no order this batch
  int32_t* cursor;    // [ORDER_TILES] scatter cursors
};

// Bounded route index (built once per engine): one row per
// source of the turn-aware route search -- row e < E: from edge e's end node,
// entered along e; row E + u: from node u, no heading (node candidates) --
// holding every label of that search within cost cmax (1/64 m): the departure
// label of each edge (key = edge id) and the arrival label of each node (key
// = NODE_KEY | node), as one open-addressing hash table per row (linear
// probing from 2-slot buckets at 30 or 40 % load).  A slot is 16 bytes, {key, cost,
// route distance bits, turn units} with the label's predecessor slot in the
// cost's and units' top bytes (kernels.hip idx_slot_*): the route to the
// edge's start turned into it (or to the node), so a transition reads its
// distance and turn cost from one slot, and a route walks slot to slot.  cnt
// < 0 marks a row whose search exceeded the build table (queries on it use
// the online tiers).
struct IdxRow {
  int64_t off;    // first slot of the row's table
  int32_t cnt;    // entries, -1 incomplete
  uint32_t cap;   // table slots (0 for an empty or incomplete row)
};
struct DevIndex {
  float rmax;     // 0: no index
  uint32_t cmax;  // its cost bound, floor(rmax x 64)
  const IdxRow* row;   // [E + N]
  const uint4* slot;    // 16 B per slot: 53 B per entry at 30 % load, 40 B at 40 %
  int load_pct;         // the tables' load
};
constexpr int IDX_SLOT_BYTES = 16;
// the index radius is capped so that every cost in a slot is below 2^24 (1/64 m)
constexpr float INDEX_RMAX_CAP = 200000.0f;
constexpr uint32_t NODE_KEY = 0x80000000u;  // key of a node's arrival label (edges: their id, < 2^27)
constexpr uint32_t NONE_PRED = 0xFFFFFFFFu; // label predecessor of a route's first edge / the source node
// near indexes: at most NEAR_LEVELS smaller radii of the same rows
// (engine.cpp build_index).  By default one, at OTM_INDEX_NEAR_FRACS x the
// index's radius, when the index's tables reach OTM_INDEX_NEAR_MIN_GB: a
// large index's probes miss the caches, and a column whose bound the near
// index covers then probes tables a fraction of the size (config 3: 137 GB,
// k_trans_sub 4.65 -> 3.31 ms at 600 m of 1,250; config 4: 62 GB, 2.17 ->
// 1.74 ms at 3.5 km of 10); a small one's probes hit the caches already and
// two tables split them (config 2: 5 GB, 0.210 -> 0.225 ms at 400 m).
constexpr int NEAR_LEVELS = 3;
#ifndef OTM_INDEX_NEAR_FRACS
#define OTM_INDEX_NEAR_FRACS {0.45f}
#endif
#ifndef OTM_INDEX_NEAR_MIN_GB
#define OTM_INDEX_NEAR_MIN_GB 16.0
#endif
constexpr int INDEX_BUILD_LOG2 = 11;
constexpr int INDEX_BUILD_CAP = 1 << INDEX_BUILD_LOG2;  // LDS table of the index builder
constexpr int INDEX_BUILD_LIMIT = 1536; // labels per row before the row is left incomplete
// cost bound (1/64 m) of a search bounded by B metres (oracle cost_bound)
__host__ __device__ inline uint32_t index_cost_bound(float B) { return (uint32_t)floor((double)B * 64.0); }

// which kernels walk the spatial work order (DevParams::order_mask: all three)
constexpr int ORDER_CAND = 1, ORDER_TRANS = 2, ORDER_ROUTE = 4;
constexpr int TURN_TABLE = 181;                 // turn units per deviation 0..180 degrees
constexpr uint32_t TURN_UNITS_MAX = 0xFFFFFFu;   // 2^24 - 1: a route's units sum exact in a float
constexpr uint32_t NO_TURNS = 0xFFFFFFFFu;       // index slot heads of the empty route (v == u)
struct DevParams {
  float sigma_z, beta, factor, breakage, interp, search_radius, max_search_radius, gps_accuracy;
  const uint32_t* turn_units;  // [TURN_TABLE] (device)
  int max_candidates;
  int order_mask;
  int cand_wave_all;  // small batch: every probe to the wave tier (latency, not throughput, bound)
};

struct DevReportCfg {
  int n_report, n_transition;
  int64_t report_levels[16];
  int64_t transition_levels[16];
  double threshold_sec;
};

struct DevBatch {
  int32_t n_traces;
  int64_t n_points;
  const int64_t* trace_off;
  const float *lat, *lon;
  const double* time;
  const float* acc;
};

// device counters, same order as otm_work_counters
struct DevCounters {
  unsigned long long points, columns, cells_visited, cell_entries_scanned, candidates;
  unsigned long long searches, nodes_settled, edges_relaxed, transitions;
  unsigned long long route_searches, route_nodes_settled, route_edges_relaxed, route_edges;
  unsigned long long segments_out, reports_out;
};

// per-point / per-trace work arrays of one batch (device pointers)
struct DevWork {
  int32_t* pt_trace;     // [P] trace of point
  uint8_t* is_col;       // [P]
  int32_t* prevc;        // [P] column: previous column (unlinked), -1; other points: the column before them
  int32_t* nextc;        // [P] column q: its next column p when interpolated points lie between (K3), else -1
  float* gc;             // [P]
  int32_t* ncand;        // [P]
  float4* probe;         // [P] {lat, lon, accuracy, 0}: a probe's inputs in one line (K1)
  // Candidates of point p, slot j: the first KIN slots
  // inline -- {edge, offset bits} at cand_eo[p * KIN + j] (two points per
  // 128-B line) and the emission at cand_em[p * KIN + j] (four points per
  // line); slots KIN.. of the rare wider points at cand_xeo / cand_xem[p * KX
  // + j - KIN] (untouched lines for every other point)
  int2* cand_eo;         // [P*KIN]
  float* cand_em;        // [P*KIN]
  int2* cand_xeo;        // [P*KX]
  float* cand_xem;       // [P*KX]
  int32_t* col_prev;     // [P] linked previous column, -1
  int32_t* kq_prev;      // [P] candidates of the linked previous column (K3), so K4 reads them with p's own words
  uint8_t* vmeta;        // [P] K5's byte per point (K3): candidates | column << 6 | linked << 7
  int64_t* trans_off;    // [P+1]
  float* trans;          // [total]
  uint8_t* bp;           // [P*KMAX]
  int32_t* state;        // [P]
  int2* chosen;          // [P] the chosen candidate {edge, offset bits} where state >= 0 (K5)
  uint8_t* chain_start;  // [P]
  float* route_dist;     // [P]
  float* ipos;           // [P] interpolated point: position along its step's route (K7a), -1 none
  int32_t* path_off;     // [P]
  int32_t* path_len;     // [P]
  int32_t* path_pool;    // [pool_cap]
  int32_t pool_cap;
  int32_t* trace_err;    // [T]
  int32_t* overflow_list0; // [P] columns/steps the index could not answer
  int32_t* overflow_list2; // [P] ... the LDS search tier spilled (and k_trans_sub's wide columns)
  int32_t* snap;           // [48] spill snapshots A (after K2), B (after K4), C (after K6)
  int32_t* counters_i32;   // [64]: [1] pool used, [2] pool overflow flag, [3] list 2 count, [4] list 0 count,
                           // [5] candidate wave-tier count, [6] wide list count (0-15: per stage, snapshot
                           // and reset); per batch: [20] Viterbi wide list, [21] / [22] huge-tier
                           // transition / route searches, [23] huge grow flag, [24] candidate HBM-tier
                           // probes, [25] its grow flag
  int32_t* abort;          // [1] set when a capacity (transition matrices, path pool) was exceeded:
                           // every later kernel returns at once and the host redoes the batch
  int64_t trans_cap;       // floats allocated for w.trans
  // K4's column records in spatial-order position, written by K3 at the
  // position the order scatter noted per column (colrec_pos): {p, col_prev,
  // kq_prev | ncand << 8, gc bits}; null: k_trans_sub reads the per-point arrays
  int4* colrec;
  int32_t* colrec_pos;
  DevIndex idx;
  DevIndex idxn[NEAR_LEVELS];  // near indexes, smallest radius first (rmax 0: none): a column
                               // probes the first whose cmax covers its cost bound
  DevOrder ord;
  // global-tier scratch
  uint32_t* big_key;
  unsigned long long* big_lab;
  uint32_t* big_inq;
  uint32_t* big_fr;
  uint32_t* big_ins;       // [BIG_SLOTS * SEARCH_LIMIT] slots each table's last search inserted
  int32_t* big_prev;       // [BIG_SLOTS] their count (-1: clear the whole table)
  // huge-tier scratch ([HUGE_SLOTS << huge_log2] slots; huge_log2 == 0: none yet)
  uint32_t* huge_key;
  unsigned long long* huge_lab;
  uint32_t* huge_inq;
  uint32_t* huge_fr;
  uint32_t* huge_ins;      // [HUGE_SLOTS * huge_limit(huge_log2)]
  int32_t* huge_prev;      // [HUGE_SLOTS]
  int32_t huge_log2;
  int32_t huge_final;      // the huge tables cannot grow: an overflowing search fails its trace (500)
  // candidate HBM tier ([CAND_BIG_SLOTS << cand_log2] slots; cand_log2 == 0: none yet)
  uint32_t* cbig_key;
  unsigned long long* cbig_val;
  unsigned long long* cbig_skey;  // [CAND_BIG_SLOTS << (cand_log2 - 1)]
  int32_t cand_log2;
  int32_t cand_final;      // the candidate tables cannot grow: an overflowing probe fails its trace (500)
  int32_t* overflow_list3; // [P] searches the global tier spilled (counts: [21] transitions, [22] route)
  DevCounters* ctr;        // nullptr when counting is off
};

// Outputs of one batch.  Segments, way ids and reports are written in one
// pass into per-trace regions sized by an upper bound (2 traversals per
// matched point + its route's path edges, summed per trace and scanned over
// traces: trace t's region starts at seg_base[t]); otm_fetch_results compacts
// them.
struct DevOut {
  // per trace
  void* traces;          // otm_trace_result[T] (seg_off / rep_off = region start)
  int32_t* seg_cnt;      // [T+1] segments per trace
  int32_t* way_cnt;      // [T+1] way ids per trace
  int32_t* rep_cnt;      // [T+1] reports per trace
  int64_t* seg_base;     // [T+1] exclusive scan of the per-trace bound
  // regions (capacity = bound total)
  void* segments;        // otm_segment[]
  int32_t* seg_gidx;     // [] segment index in graph (-1 none)
  int64_t* way_ids;      // []
  void* reports;         // otm_report_rec[]
  uint32_t* hist;        // [n_segments * nbins] or nullptr
  unsigned long long* speed_sum;  // [n_segments] sum of report speeds, 1/1000 km/h, or nullptr
  int nbins;
  float bin_kph;
};

// Per-kernel timing (otm_get_kernel_ms): when ev != nullptr the launchers
// record ev[2k] just before and ev[2k+1] just after kernel k, on the launch
// stream.  Order and names: kKernelNames in kernels.hip.
enum KernelId {
  KN_COLUMNS,
  KN_ORDER,
  KN_CAND_LANE,
  KN_CAND_WAVE,
  KN_LINKS,
  KN_SCAN_TRANS,
  KN_TRANS_INDEX,
  KN_TRANS_WIDE,
  KN_TRANS_WAVE,
  KN_TRANS_GLOBAL,
  KN_VITERBI,
  KN_ROUTE_INDEX,
  KN_ROUTE_WAVE,
  KN_ROUTE_GLOBAL,
  KN_SEG_BOUND,
  KN_SEG_SCAN,
  KN_SEG_WRITE,
  KN_REPORT,
  KN_COUNT
};
extern const char* const kKernelNames[KN_COUNT];
struct Marks {
  hipEvent_t* ev = nullptr;
  void begin(int k, hipStream_t s) const {
    if (ev) (void)hipEventRecord(ev[2 * k], s);
  }
  void end(int k, hipStream_t s) const {
    if (ev) (void)hipEventRecord(ev[2 * k + 1], s);
  }
};

// ---- launch wrappers (kernels.hip)
void launch_columns(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                    const Marks& mk);
// Where a batch resumes after a tier's tables grew (engine_match): the stages
// before the tier that overflowed kept their results, so only that tier and
// what follows it run again (RESUME_ALL: the whole batch).
enum Resume { RESUME_ALL = 0, RESUME_CAND_BIG = 1, RESUME_TRANS_HUGE = 2, RESUME_ROUTE_HUGE = 3 };
void launch_candidates(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                       const Marks& mk, int from = RESUME_ALL);
void launch_links(const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s, const Marks& mk);
// sets *w.abort when the scanned transition total exceeds w.trans_cap
void launch_cap_check(const DevBatch& b, DevWork& w, hipStream_t s);
// index tier -> LDS search tier -> global tier, spill lists on the device
// (counters_i32[3] / [4] / [6] must be zero on entry)
void launch_transitions(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                        const Marks& mk, int sub, int from = RESUME_ALL);
void launch_viterbi(const DevBatch& b, DevWork& w, hipStream_t s, const Marks& mk);
void launch_route(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                  const Marks& mk, int from = RESUME_ALL);
void launch_segments(const DevGraph& g, const DevBatch& b, DevWork& w, DevOut& o, bool write, hipStream_t s,
                     const Marks& mk);
void launch_report(const DevBatch& b, const DevReportCfg& rc, DevWork& w, DevOut& o, hipStream_t s, const Marks& mk);
// spatial work order: tile counts, plan (group cuts), scatter of the columns
void launch_order(const DevBatch& b, DevWork& w, hipStream_t s, const Marks& mk);
// K7a: each trace's segment bound added into tb[T] (zeroed by the caller;
// scanned into DevOut::seg_base) and the interpolated points placed
void launch_seg_bound(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, int64_t* tb, hipStream_t s,
                      const Marks& mk);
// fetch-time compaction of the per-trace regions into dense arrays; offsets
// are the exclusive scans of seg_cnt / way_cnt / rep_cnt
void launch_compact(int32_t n_traces, const DevOut& o, const int32_t* seg_off, const int32_t* way_off,
                    const int32_t* rep_off, void* segs_out, int64_t* ways_out, void* reps_out, void* traces_out,
                    hipStream_t s);
// index build: pass 0 counts rows (row_cnt), pass 1 inserts them into the
// row tables (slot array pre-filled with 0xFF)
void launch_index_build(const DevGraph& g, const uint32_t* turn_units, uint32_t cmax, int32_t* row_cnt,
                        const IdxRow* rows, uint4* slot, bool write, hipStream_t s);
// the route index's table loads (percent): the faster one, and the denser one
// an index falls back to when the faster does not fit its HBM budget
int index_load_fast();
int index_load_dense();
void launch_row_sizes(const int32_t* row_cnt, int64_t* row_sizes, int32_t n, int pct, hipStream_t s);
struct BatchStatus {
  int32_t abort, grow;  // grow bit 0: the huge search tier needs (larger) tables; bit 1: the candidate HBM tier
  int64_t ttotal;
  int32_t cnt[3];
  int32_t route_huge;   // counters_i32[22]: the route stage reached its huge tier (else the transition stage did)
};
void launch_batch_init(int32_t* counters, int32_t* abort, hipStream_t s);
// otm_match_compact's inputs widened on the device (time = base + delta, accuracy as float)
void launch_expand_compact(const int64_t* trace_off, const int64_t* tbase, const int32_t* dt, const int16_t* acc16,
                           double* time, float* acc, int32_t n_traces, hipStream_t s);
void launch_snap(int32_t* counters, int32_t* snap, bool reset, hipStream_t s);
// batch bookkeeping folded into the stage kernels (no launches of their own)
bool fold_bookkeeping();
void launch_status(const int32_t* abort, const int64_t* ttotal, const int32_t* counters, BatchStatus* out,
                   hipStream_t s);
void launch_row_pack(const int32_t* row_cnt, const int64_t* row_off, IdxRow* rows, int32_t n, hipStream_t s);
// the /report request bytes read on the GPU (requests.hip): per request r of
// [r0, r1) of the staged blob (bytes [off[r], off[r+1])), accepted << 40 |
// points in cnt[r] and ok[r], its points into the sparse arrays
// (req_sparse_slots entries; cnt[n] = 0 by the launch that ends at n); after
// an exclusive scan of cnt (n + 1 entries), the compaction moves the accepted
// requests' points into out's arrays and their offsets into trace_off
size_t req_sparse_slots(int32_t n, size_t bytes);
void launch_req_read(const unsigned char* blob, const int64_t* off, int32_t r0, int32_t r1, int32_t n, int64_t* cnt,
                     uint8_t* ok, const DevBatch& sparse, hipStream_t s);
void launch_req_compact(const int64_t* off, int32_t n, const int64_t* pre, const uint8_t* ok, const DevBatch& sparse,
                        const DevBatch& out, int64_t* trace_off, hipStream_t s);
// the /report response bodies written on the GPU (responses.hip) from a
// batch's dense results (engine_fetch's compaction, device side)
constexpr int RESP_HDR_SLOT = 512;  // bytes of a trace's header piece
constexpr int RESP_SEG_SLOT = 320;  // ... of a segment object, + 24 per way id (8-byte aligned)
constexpr int RESP_REP_SLOT = 192;  // ... of a datastore report object
struct RespIn {
  int32_t nt, ns, nr;
  const otm_trace_result* traces;
  const otm_segment* segs;
  const int64_t* ways;
  const otm_report_rec* reps;
};
struct RespWork {
  char *hdr, *seg, *rep;       // piece slots
  int32_t *hlen, *slen, *rlen;  // piece lengths (-1: a float the host formats)
  int64_t* blen;               // [nt + 1] body lengths, scanned in place into offsets
  uint8_t* host;               // [nt] 1: the host writes this body
};
size_t resp_seg_scratch(int32_t ns, int32_t nw);
void launch_resp_items(const RespIn& in, const RespWork& w, hipStream_t s);
void launch_resp_len(const RespIn& in, const RespWork& w, hipStream_t s);
void launch_resp_copy(const RespIn& in, const RespWork& w, const int64_t* boff, char* blob, hipStream_t s);
// exclusive scan helpers (in place over n+1 elements: out[n] = total)
void scan_i64(int64_t* d, int64_t n, void* tmp, size_t tmp_bytes, hipStream_t s);
// exclusive scans of three per-trace counts (n <= FETCH_SCAN_MAX) in one
// single-block launch, totals at o*[n]
constexpr int FETCH_SCAN_MAX = 1 << 16;
void launch_fetch_scan(int32_t n, const int32_t* c0, const int32_t* c1, const int32_t* c2, int32_t* o0, int32_t* o1,
                       int32_t* o2, hipStream_t s);
void scan_i32(int32_t* d, int64_t n, void* tmp, size_t tmp_bytes, hipStream_t s);
size_t scan_tmp_bytes(int64_t n);

}  // namespace otm
