// group.cpp -- host batches on one engine or on a multi-device engine.
//
// A multi-device engine (otm_engine_create with ndev > 1) is what one host
// process -- the Java Kafka Streams host of Batch.java:63 is one JVM -- uses to
// drive several GPUs through a single handle.  It owns no GPU state: one member
// engine per device holds a full graph and index replica, and
// every batch is split across the members by uuid with Kafka's own partitioner,
// (murmur2(uuid) & 0x7fffffff) % ndev, as the reference's keyed `formatted`
// topic splits vehicles over batchers (Reporter.java:97,102).  Nothing is
// exchanged between members on the data path; each runs its part concurrently
// from its own host thread and the results are merged back in request order.
#include <algorithm>
#include <condition_variable>
#include <functional>
#include <thread>

#include "engine.h"

extern "C" int32_t otm_murmur2(const char* key, size_t len);

namespace otm {

int shard_of(const char* key, size_t len, int n) {
  if (n <= 1) return 0;
  return (int)((otm_murmur2(key, len) & 0x7fffffff) % n);
}

}  // namespace otm

// One persistent host thread per member: run(tasks) hands task i to thread i
// and returns when all are done.  (Threads spawned per batch measured ~0.3 MB
// of host memory each that the HIP runtime keeps after the thread exits.)
struct MemberPool {
  explicit MemberPool(size_t n) : slots_(n) {
    try {
      for (size_t i = 0; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
    } catch (...) {
      // a thread that failed to start: stop and join the ones that did, so
      // no joinable std::thread is destroyed (std::terminate), then report it
      stop_all();
      throw;
    }
  }
  ~MemberPool() { stop_all(); }
  void run(std::vector<std::function<void()>>& tasks) {
    std::unique_lock<std::mutex> lk(mu_);
    pending_ = 0;
    for (size_t i = 0; i < slots_.size() && i < tasks.size(); ++i)
      if (tasks[i]) {
        slots_[i] = &tasks[i];
        ++pending_;
      }
    ++gen_;
    cv_.notify_all();
    done_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  void stop_all() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_)
      if (t.joinable()) t.join();
  }
  void loop(size_t i) {
    uint64_t seen = 0;
    while (true) {
      std::function<void()>* task = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || (gen_ != seen && slots_[i]); });
        if (stop_) return;
        seen = gen_;
        task = slots_[i];
        slots_[i] = nullptr;
      }
      (*task)();
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_.notify_all();
      }
    }
  }
  std::vector<std::function<void()>*> slots_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
};

namespace otm {

void member_pool_free(otm_engine* G) {
  delete G->member_pool;
  G->member_pool = nullptr;
}

namespace {

struct MemberOut {
  std::vector<int32_t> traces;  // batch trace index of each member trace
  std::vector<int64_t> off;
  std::vector<float> lat, lon, acc;
  std::vector<double> time;
  std::vector<otm_trace_result> tr;
  std::vector<otm_segment> segs;
  std::vector<otm_report_rec> reps;
  std::vector<int64_t> ways;
  int rc = 0;
  std::string err;
};

void run_member(otm_engine* M, MemberOut& o) {
  otm_batch sb;
  sb.n_traces = (int32_t)o.traces.size();
  sb.n_points = o.off.back();
  sb.trace_off = o.off.data();
  sb.lat = o.lat.data();
  sb.lon = o.lon.data();
  sb.time = o.time.data();
  sb.accuracy = o.acc.data();
  std::lock_guard<std::mutex> lk(M->mu);
  (void)hipSetDevice(M->device);
  otm_results r;
  o.rc = engine_match_host(M, &sb, &o.err);
  if (!o.rc) o.rc = engine_fetch(M, &r, &o.err);
  if (o.rc) return;
  // the member's result arrays live until its next batch: copy them out
  o.tr.assign(r.traces, r.traces + r.n_traces);
  o.segs.assign(r.segments, r.segments + r.n_segments);
  o.reps.assign(r.reports, r.reports + r.n_reports);
  o.ways.assign(r.way_ids, r.way_ids + r.n_way_ids);
}

int group_match(otm_engine* G, const otm_batch* b, const int32_t* shard, otm_results* out, std::string* err) {
  const int nd = (int)G->members.size();
  const int32_t nt = b->n_traces;
  const int64_t p0 = nt > 0 ? b->trace_off[0] : 0;
  const int64_t np = nt > 0 ? b->trace_off[nt] - p0 : 0;
  std::vector<MemberOut> mo((size_t)nd);
  std::vector<int32_t> mem((size_t)nt), pos((size_t)nt);
  for (int32_t t = 0; t < nt; ++t) {
    int m;
    if (shard) {
      m = shard[t];
      if (m < 0 || m >= nd) {
        *err = "shard index out of range";
        return OTM_EINVAL;
      }
    } else {
      // contiguous ranges balanced by points (the binary path carries no uuid)
      const int64_t mid = b->trace_off[t] - p0;
      m = np > 0 ? (int)std::min<int64_t>(nd - 1, mid * nd / np) : (int)((int64_t)t * nd / nt);
    }
    mem[(size_t)t] = m;
    MemberOut& o = mo[(size_t)m];
    pos[(size_t)t] = (int32_t)o.traces.size();
    o.traces.push_back(t);
  }
  for (MemberOut& o : mo) {
    o.off.assign(1, 0);
    int64_t n = 0;
    for (int32_t t : o.traces) n += b->trace_off[t + 1] - b->trace_off[t];
    o.lat.reserve((size_t)n);
    o.lon.reserve((size_t)n);
    o.acc.reserve((size_t)n);
    o.time.reserve((size_t)n);
    for (int32_t t : o.traces) {
      const int64_t a = b->trace_off[t], e = b->trace_off[t + 1];
      o.lat.insert(o.lat.end(), b->lat + a, b->lat + e);
      o.lon.insert(o.lon.end(), b->lon + a, b->lon + e);
      o.acc.insert(o.acc.end(), b->accuracy + a, b->accuracy + e);
      o.time.insert(o.time.end(), b->time + a, b->time + e);
      o.off.push_back((int64_t)o.lat.size());
    }
  }
  // the members' parts, each on its member's persistent thread (the caller
  // holds G->mu, so one batch at a time uses the pool)
  if (!G->member_pool) G->member_pool = new MemberPool((size_t)nd);
  std::vector<std::function<void()>> tasks((size_t)nd);
  for (int m = 0; m < nd; ++m)
    if (!mo[(size_t)m].traces.empty()) {
      otm_engine* M = G->members[(size_t)m];
      MemberOut* o = &mo[(size_t)m];
      tasks[(size_t)m] = [M, o] {
        try {
          run_member(M, *o);
        } catch (...) {  // (a host allocation failure) -> the batch's error, not terminate()
          o->rc = OTM_ENOMEM;
          o->err = "out of host memory";
        }
      };
    }
  G->member_pool->run(tasks);
  for (const MemberOut& o : mo)
    if (o.rc) {
      *err = o.err;
      return o.rc;
    }
  // merge in batch trace order
  G->g_traces.resize((size_t)nt);
  G->g_segs.clear();
  G->g_reps.clear();
  G->g_ways.clear();
  for (int32_t t = 0; t < nt; ++t) {
    const MemberOut& o = mo[(size_t)mem[(size_t)t]];
    otm_trace_result tr = o.tr[(size_t)pos[(size_t)t]];
    const int32_t s0 = tr.seg_off, r0 = tr.rep_off;
    tr.seg_off = (int32_t)G->g_segs.size();
    tr.rep_off = (int32_t)G->g_reps.size();
    for (int32_t s = s0; s < s0 + tr.seg_cnt; ++s) {
      otm_segment sg = o.segs[(size_t)s];
      const int32_t w0 = sg.way_off;
      sg.way_off = (int32_t)G->g_ways.size();
      G->g_ways.insert(G->g_ways.end(), o.ways.begin() + w0, o.ways.begin() + w0 + sg.way_cnt);
      G->g_segs.push_back(sg);
    }
    G->g_reps.insert(G->g_reps.end(), o.reps.begin() + r0, o.reps.begin() + r0 + tr.rep_cnt);
    G->g_traces[(size_t)t] = tr;
  }
  out->n_traces = nt;
  out->n_segments = (int32_t)G->g_segs.size();
  out->n_reports = (int32_t)G->g_reps.size();
  out->n_way_ids = (int32_t)G->g_ways.size();
  out->traces = G->g_traces.data();
  out->segments = G->g_segs.data();
  out->reports = G->g_reps.data();
  out->way_ids = G->g_ways.data();
  return OTM_OK;
}

}  // namespace

int match_host_fetch(otm_engine* E, const otm_batch* b, const int32_t* shard, otm_results* out, std::string* err) {
  if (!E->members.empty()) return group_match(E, b, shard, out, err);
  (void)hipSetDevice(E->device);
  int rc = engine_match_host(E, b, err);
  if (!rc) rc = engine_fetch(E, out, err);
  return rc;
}

}  // namespace otm
