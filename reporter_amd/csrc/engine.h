// engine.h -- the otm_engine: one GPU, its HBM-resident graph, batch buffers.
#pragma once
#include <atomic>
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kernels.h"
#include "otm_internal.h"
#include "otmatch.h"

// One submission's request bodies, copied into one allocation (abi.cpp
// slabs::acquire; released to a cache when its last request is done)
struct ReqSlab {
  char* base = nullptr;
  size_t cap = 0;
  bool pinned = false;
};

namespace otm {
// The order in which batch contexts copy request bytes to HBM (the async
// workers' batches): ticket t's copies
// queue behind ticket t-1's on the device (ev[(t - 1) & 1], recorded on t-1's
// copy stream), so the host-to-device link carries one batch at a time, in
// order, while the earlier batches run their kernels (abi.cpp H2DTurn).
struct H2DOrder {
  std::mutex m;
  std::condition_variable cv;
  uint64_t next = 0;
  hipEvent_t ev[2] = {nullptr, nullptr};
  // the pipeline's one request-copy stream (created by the first turn's
  // holder): every context's pieces go there, in ticket order; own_queue: on
  // a hardware queue of its own (the async pipeline's, engine.cpp create_stream)
  hipStream_t copy = nullptr;
  bool own_queue = false;
};
}  // namespace otm

struct otm_engine {
  const otm_engine* parent = nullptr;  // a clone shares its parent's graph and index (otm_engine_clone)
  // a multi-device engine (otm_engine_create with ndev > 1, group.cpp): one
  // member engine per device and no GPU state of its own; host batches are split
  // across the members by uuid and merged back (the g_* arrays hold the merged
  // results of its last batch)
  std::vector<otm_engine*> members;
  // one persistent host thread per member (group.cpp): a HIP host thread keeps
  // runtime state that a thread spawned per batch would leak
  struct MemberPool* member_pool = nullptr;
  std::vector<otm_trace_result> g_traces;
  std::vector<otm_segment> g_segs;
  std::vector<otm_report_rec> g_reps;
  std::vector<int64_t> g_ways;
  int device = 0;
  std::atomic<int> n_clones{0};  // clones made of this engine (their stream slots; clones race with the async start)
  hipStream_t stream = nullptr;
  hipEvent_t sync_ev = nullptr;  // blocking-sync event of large batches' host waits
  bool spin_waits = false;       // otm_match_device in progress: spin-wait (engine.cpp wait_batch)
  otm::HostGraph host;
  otm::DevGraph g{};
  std::vector<void*> graph_allocs;
  // bounded distance index (built at create time; rmax 0 disables)
  // 1250 m answers every transition with gc <= 250 m (bound 5 x gc): probes up to
  // 50 m/s at 5 s sampling; measured on config 2, 1000 m left one column in 1M to
  // the online tiers at a cost of 0.13 ms per batch
  float index_rmax = -1.0f;  // < 0: sized from the graph's node density (auto_index_radius)
  int64_t small_points = 0;  // batches below this many points: natural order, wave-tier candidates
  int trans_lanes = 8;      // k_trans_sub lanes per column: 8 (two passes, wide columns at 16) or 16 (one pass)
  int grid_mult = 0;         // candidate grid cells = grid_mult x grid_mult of the file's (0: auto_grid_mult)
  int32_t grid_rows = 0, grid_cols = 0;
  int64_t grid_entries = 0;
  otm::DevIndex idx{};
  // near indexes (DevWork::idxn, smallest radius first, rmax 0: none): the same
  // rows at the radii index_near_m (not set: OTM_INDEX_NEAR_FRACS x index_rmax
  // when the index reaches OTM_INDEX_NEAR_MIN_GB), each probed by the columns
  // whose bound it is the smallest to cover
  otm::DevIndex idxn[otm::NEAR_LEVELS]{};
  std::vector<float> index_near_m;
  bool index_near_set = false;
  int64_t index_near_level_entries[otm::NEAR_LEVELS]{};
  int64_t index_entries = 0;
  int64_t index_slots = 0;       // hash-table slots of the full index (16 B each, the predecessor inside)
  int64_t index_near_slots = 0;  // ... of its near indexes
  int32_t index_incomplete_rows = 0;
  float index_build_ms = 0.0f;
  otm::MatchConfig mc;
  otm::ReportConfig rc;
  otm::DevParams dp{};
  otm::DevReportCfg drc{};
  std::mutex mu;  // one batch at a time per engine

  struct Buf {
    void* p = nullptr;
    size_t cap = 0;
  };
  // batch inputs (host batches are staged here)
  Buf in_off, in_lat, in_lon, in_time, in_acc, in_blob;
  // work
  Buf pt_trace, is_col, prevc, nextc, gc, ncand, cand_eo, cand_em, cand_xeo, cand_xem, probe, col_prev, kq_prev, vmeta, colrec, colrec_pos, trans_off, trans, bp, state, chosen,
      chain_start, route_dist, ipos, path_off, path_len, path_pool, trace_err, overflow_list0, overflow_list2,
      counters_i32, scan_tmp, snap;
  Buf big_key, big_lab, big_inq, big_fr, big_ins, big_prev;
  Buf huge_key, huge_lab, huge_inq, huge_fr, huge_ins, huge_prev, overflow_list3;
  int32_t huge_log2 = 0;  // huge search tier: 2^huge_log2 slots per table (0: none yet; grown on demand)
  int32_t huge_ready_log2 = 0;  // the layout the huge tables were last cleared for
  Buf cbig_key, cbig_val, cbig_skey;
  int32_t cand_log2 = 0;  // candidate HBM tier: 2^cand_log2 slots per table (0: none yet; grown on demand)
  int32_t huge_final = 0, cand_final = 0;  // the tier's tables cannot grow: overflows fail their traces
  int32_t last_attempts = 0;  // runs of the last batch (otm_spill_stats::attempts)
  int32_t last_resumes = 0;   // ... of them resumed from a grown tier (otm_spill_stats::resumed)
  Buf ord_tile, ord_cnt, ord_cursor, ord_grp, ord_item;  // spatial work order
  Buf abort_flag;                                       // capacity overflow of the batch in flight
  Buf rs_blob;                                          // otm_report_segments_device in/out
  int64_t trans_cap = 0;                                // floats in `trans` (grown on overflow)
  bool caps_read = false, caps_pinned = false;          // OTM_TRANS_CAP / OTM_POOL_CAP
  // outputs
  Buf o_traces, o_seg_cnt, o_way_cnt, o_rep_cnt, seg_ub, o_segments, o_seg_gidx, o_way_ids, o_reports;
  // dense copies made by engine_fetch
  Buf f_seg_off, f_way_off, f_rep_off, f_segs, f_ways, f_reps, f_traces;
  otm::DevCounters* ctr = nullptr;
  otm::DevCounters* ctr_save = nullptr;
  bool counting = false;
  // histogram (caller-owned device memory).  Clones read their parent's
  // binding at each batch (under the parent's hist_mu), so a rebind reaches them.
  std::mutex hist_mu;
  uint32_t* hist = nullptr;
  unsigned long long* speed_sum = nullptr;
  int nbins = 0;
  float bin_kph = 5.0f;
  // last batch
  int32_t last_T = 0;
  int64_t last_P = 0;
  int32_t last_S = 0, last_W = 0;
  int64_t last_trans = 0;
  int32_t pool_cap = 0;
  // host copies of the last fetched results
  // (pinned: the D2H copies run at PCIe speed without a staging hop)
  Buf h_traces, h_segs, h_reps_dense, h_ways, h_tot, h_in, h_status;
  // request bodies read on the GPU (engine_match_requests): the pinned staging
  // blob (offsets, then bytes), its device copy, per-request counts and flags
  Buf h_req, d_req, req_cnt, req_ok, h_req_ok;
  Buf req_lat, req_lon, req_time, req_acc;  // the reader's sparse point slots (requests.hip)
  int32_t req_read = 0;                     // requests of the staged batch read so far
  hipStream_t req_copy = nullptr;           // the request pieces' H2D copies (created at first use)
  double t_read_done = 0.0;                 // (OTM_JSON_PROFILE) when the last request batch's read synced
  // the async workers' contexts: their request pieces go on the pipeline's
  // one copy stream (H2DOrder::copy) instead of req_copy, so three batch
  // streams and one copy stream fit the runtime's four hardware queues
  // (GPU_MAX_HW_QUEUES), and the copies run on a copy engine, not as blit
  // kernels on the batch stream beside the batch's kernels
  hipStream_t req_shared = nullptr;
  std::vector<hipEvent_t> req_ev;           // [0] the copies' fence, [1 + p]: piece p copied
  size_t req_piece = 0;                     // pieces of the staged batch pushed so far
  // response bodies written on the GPU (engine_write_responses): piece slots,
  // lengths, the dense blob, and its pinned host copy with offsets and flags
  Buf resp_hdr, resp_seg, resp_rep, resp_hlen, resp_slen, resp_rlen, resp_blen, resp_host, resp_blob;
  Buf h_resp, h_resp_meta;
  // timing
  bool timing = false;
  hipEvent_t kev[2 * otm::KN_COUNT] = {};
  float kernel_ms[otm::KN_COUNT] = {};
  float stage_ms[8] = {};
  // async submit/poll: a pipeline of workers, each running whole request
  // batches on its own batch context (clones this engine owns, awx, each
  // stream on a hardware queue of its own), so the batches' kernels and copies
  // run side by side; batches are taken and their results published in
  // submit order (abi.cpp worker_loop)
  // a submitted request: its body inside the slab its submission copied
  // every body into (page-locked when large: the worker's batch copies it to
  // HBM from there, with no staging copy)
  struct Pending {
    uint64_t tag;
    const char* p;
    size_t len;
    std::shared_ptr<ReqSlab> slab;
    size_t run_left;  // requests of its submission from this one on (itself included)
    uint64_t sub;     // its submission's number
  };
  uint64_t n_subs = 0;  // submissions so far (under qmu)
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<Pending> queue;
  std::deque<otm_result> done;
  std::vector<std::thread> workers;
  // a split otm_report_batch's batch contexts (its chunks run on these
  // clones, whose streams have hardware queues of their own; created under qmu)
  std::vector<otm_engine*> actx;
  // the async workers' batch contexts: clones whose streams have hardware
  // queues of their own (worker i on awx[i]; none: one worker, on this engine);
  // created under qmu when the workers start
  std::vector<otm_engine*> awx;
  otm::H2DOrder aorder;           // the workers' batches' copies, in take order
  uint64_t take_seq = 0, pub_seq = 0;
  bool stop = false;
  bool worker_started = false;
  // a split otm_report_batch call (abi.cpp report_many_split): its chunks'
  // copies in order, one call at a time
  std::mutex split_mu;
  otm::H2DOrder split_order;
  std::atomic<int> last_split{1};  // the chunks of the last otm_report_batch (otm_debug_last_split)
};

namespace otm {

int engine_init(otm_engine* E, const char* graph_path, int device, std::string* err);
// turn cost units (1/64 m) of a turn deviating d = 0..180 degrees from straight on
uint32_t turn_units(float factor, int d);
// a second batch context on the same GPU: own stream and buffers, the
// parent's HBM graph, index and configuration
// (own_queue: its stream on a hardware queue of its own, engine.cpp create_stream)
int engine_clone(const otm_engine* parent, otm_engine* C, std::string* err, bool own_queue = false);
// a batch context's (or a copy order's) stream; nonzero on failure
int create_stream(int slot, hipStream_t* s, bool own_queue);
void engine_free(otm_engine* E);
// match a device-resident batch; returns 0 or OTM_EDEVICE (message in *err)
int engine_match(otm_engine* E, const DevBatch& b, hipStream_t s, std::string* err);
// stage a host batch to the device and match it
int engine_match_host(otm_engine* E, const otm_batch* in, std::string* err);
// checks of a compact batch (both engine kinds); *np = its point count
int validate_compact(const otm_batch_compact* in, int64_t* np, std::string* err);
int engine_match_compact(otm_engine* E, const otm_batch_compact* in, std::string* err);
// The /report request bodies read on the GPU: engine_stage_requests returns a
// pinned host staging buffer for n requests of `bytes` body bytes in all:
// int64 offsets[n + 1] (into the bytes) and the bytes; the caller fills both
// and calls engine_match_requests, which copies it to HBM, decodes the
// bodies of the Java batcher's exact form (requests.hip) into a batch and
// matches it.  *ok[r] (valid until the next call) says which requests the
// batch holds, in request order; the others are the caller's to read.
// (bodies false: the caller pushes every body from its own page-locked
// memory; the staging buffer then holds the offsets alone, *body null)
int engine_stage_requests(otm_engine* E, int32_t n, size_t bytes, bool bodies, int64_t** off, char** body,
                          std::string* err);
// (engine_push_requests: a piece of the staged blob on its way to HBM, so
// staging and copying overlap; pushed = every piece went that way)
// (src: those bytes from page-locked host memory instead of the staging buffer;
// upto: the requests [0, upto) are then whole on the device, and those not yet
// read are read behind the copy, while the host stages the next piece)
int engine_push_requests(otm_engine* E, int32_t n, size_t bytes, size_t from, size_t to, const char* src,
                         int32_t upto, std::string* err);
int engine_match_requests(otm_engine* E, int32_t n, size_t bytes, bool pushed, const uint8_t** ok,
                          int32_t* n_traces, std::string* err);
// H2DOrder's two ends on E's request-copy stream: the copies E pushes next
// wait for ev; ev marks the copies E has pushed so far
int engine_push_after(otm_engine* E, hipEvent_t ev);
int engine_push_mark(otm_engine* E, hipEvent_t ev);
// The last batch's /report response bodies written on the GPU
// (responses.hip) into a device blob of *total bytes: trace t's body is
// blob[off[t], off[t + 1] - 1), NUL-terminated, unless host[t] (a 500, or a
// float the GPU does not format: the host writes those from engine_fetch's
// records; no bytes in the blob); traces[t] its result record.  The pointers
// stay valid until the next batch.  engine_copy_responses brings the blob to
// dst (page-locked, e.g. the caller's response arena) or, with dst null, to
// the engine's own pinned buffer.
int engine_write_responses(otm_engine* E, const int64_t** off, const uint8_t** host,
                           const otm_trace_result** traces, int64_t* total, std::string* err);
int engine_copy_responses(otm_engine* E, char* dst, int64_t total, const char** blob, std::string* err);
// copy results of the last batch to host vectors and describe them
int engine_fetch(otm_engine* E, otm_results* out, std::string* err);
int engine_debug_fetch(otm_engine* E, int what, void* dst, size_t bytes, size_t* needed, std::string* err);
int engine_counters(otm_engine* E, otm_work_counters* out);
// report() on the GPU over caller-supplied typed segments (otm_report_segments_device):
// per trace t its points' times [trace_off[t], trace_off[t+1]) and segments
// [seg_off[t], seg_off[t+1]); fills traces[T] and the reports (trace t's at
// reports + seg_off[t], traces[t].rep_cnt of them)
int engine_report_segments(otm_engine* E, int32_t T, const int64_t* trace_off, const double* time,
                           const int32_t* seg_off, const otm_segment* segs, otm_trace_result* traces,
                           otm_report_rec* reports, std::string* err);
int engine_spill_stats(otm_engine* E, otm_spill_stats* out);
// host batch -> host results on any engine (group.cpp): one device
// (engine_match_host + engine_fetch), or a multi-device engine, whose traces go
// to member shard[t] (point-balanced contiguous ranges when shard is NULL), run
// concurrently and are merged in trace order.  The caller holds E->mu.
int match_host_fetch(otm_engine* E, const otm_batch* b, const int32_t* shard, otm_results* out, std::string* err);
// a uuid's member among n: Kafka's partition of the key, (murmur2 & 0x7fffffff) % n
int shard_of(const char* key, size_t len, int n);
// stop and join a multi-device engine's member threads (before its members go)
void member_pool_free(otm_engine* G);

}  // namespace otm
