// abi.cpp -- the extern "C" surface of libotmatch.so (include/otmatch.h).
#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <sstream>
#include <thread>

#include "engine.h"
#include "javastr.h"
#include "json.h"
#include "pyrepr.h"
#include "report.h"

using otm::json::Kind;
using otm::json::Value;

namespace {

thread_local std::string t_err;

int fail(int code, const std::string& msg) {
  t_err = msg;
  otm::set_thread_error(msg);
  return code;
}

// Host threads for the per-request work of a large request batch (JSON
// parse, point extraction, response writing): the machine's cores, at most 16,
// and at least 256 requests per thread (OTM_HOST_THREADS / OTM_HOST_CHUNK
// override both, read per call).
size_t host_threads(size_t n) {
  size_t cap, chunk = 256;
  if (const char* v = std::getenv("OTM_HOST_THREADS")) {
    cap = (size_t)std::max(1, std::atoi(v));
  } else {
    const unsigned hw = std::thread::hardware_concurrency();
    cap = (size_t)std::min(16u, hw ? hw : 1u);
  }
  if (const char* v = std::getenv("OTM_HOST_CHUNK")) chunk = (size_t)std::max(1, std::atoi(v));
  return std::max<size_t>(1, std::min(cap, (n + chunk - 1) / chunk));
}
// Persistent host workers for par_for: threads spawned per call cost ~75 thread
// creations per 10k-request batch and dropped each thread's response scratch
// buffer (below) with the thread.  A par_for posts its chunks as one job; the
// workers and the caller take chunks until none is left, so a caller always
// finishes its own job even when every worker is busy with another caller's.
// The pool never calls HIP.  It is leaked at exit on purpose (its workers sit
// in a wait; nothing to join).
class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool();
    return *p;
  }
  void run(size_t n, size_t T, const std::function<void(size_t, size_t)>& fn) {
    auto job = std::make_shared<Job>();
    job->fn = &fn;
    job->n = n;
    job->per = (n + T - 1) / T;
    job->chunks = (n + job->per - 1) / job->per;
    job->errs.resize(job->chunks);
    {
      std::lock_guard<std::mutex> lk(mu_);
      grow(T - 1);
      jobs_.push_back(job);
    }
    cv_.notify_all();
    work(*job);
    {
      std::unique_lock<std::mutex> lk(job->m);
      job->cv.wait(lk, [&] { return job->done == job->chunks; });
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = std::find(jobs_.begin(), jobs_.end(), job);
      if (it != jobs_.end()) jobs_.erase(it);
    }
    for (auto& x : job->errs)
      if (x) std::rethrow_exception(x);  // to the entry point's guard
  }

 private:
  struct Job {
    const std::function<void(size_t, size_t)>* fn = nullptr;
    size_t n = 0, per = 0, chunks = 0;
    std::atomic<size_t> next{0};
    size_t done = 0;  // under m
    std::vector<std::exception_ptr> errs;
    std::mutex m;
    std::condition_variable cv;
  };
  // chunks of job until none is left to take
  static void work(Job& j) {
    while (true) {
      const size_t c = j.next.fetch_add(1);
      if (c >= j.chunks) return;
      const size_t a = c * j.per, e = std::min(j.n, a + j.per);
      try {
        (*j.fn)(a, e);
      } catch (...) {
        j.errs[c] = std::current_exception();
      }
      std::lock_guard<std::mutex> lk(j.m);
      if (++j.done == j.chunks) j.cv.notify_all();
    }
  }
  void grow(size_t want) {  // under mu_
    while (nthreads_ < want) {
      try {
        std::thread([this] { loop(); }).detach();
      } catch (...) {
        return;  // no thread to be had: the callers take the chunks
      }
      ++nthreads_;
    }
  }
  void loop() {
    while (true) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          while (!jobs_.empty() && jobs_.front()->next.load() >= jobs_.front()->chunks) jobs_.pop_front();
          return !jobs_.empty();
        });
        j = jobs_.front();
      }
      work(*j);
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<Job>> jobs_;
  size_t nthreads_ = 0;
};


// fn(a, e) over [0, n) in contiguous chunks, one per thread (the caller's the
// first); on the persistent pool
template <class F>
void par_for(size_t n, F fn) {
  const size_t T = host_threads(n);
  if (T <= 1) {
    fn((size_t)0, n);
    return;
  }
  const std::function<void(size_t, size_t)> f = std::ref(fn);
  HostPool::get().run(n, T, f);
}

// the Java request bytes read without a DOM (otm::fast_request); OTM_FAST_JSON=0
// sends every body through the DOM (A/B and the parity tests)
bool fast_requests() {
  const char* v = std::getenv("OTM_FAST_JSON");
  return !(v && *v == '0');
}


char* dup_out(const std::string& s, size_t* n) {
  char* p = (char*)std::malloc(s.size() + 1);
  if (!p) throw std::bad_alloc();
  std::memcpy(p, s.data(), s.size());
  p[s.size()] = 0;
  if (n) *n = s.size();
  return p;
}

bool read_file(const char* path, std::string* out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  *out = ss.str();
  return true;
}

// The level sets of make_thread_locals (py/reporter_service.py:55-56) for
// k_report: Python sets, so duplicates collapse.  A level tested against them
// is segment_id & 7 (:154) or -1 (no segment id), so only -1..7 can ever
// match: other values are dropped here (the reference accepts any int and
// they never match), leaving at most 9 distinct levels for the device config.
bool device_levels(const std::vector<int64_t>& in, int64_t* out, int* n, const char* name, std::string* err) {
  (void)name;
  (void)err;
  *n = 0;
  for (int64_t v : in) {
    if (v < -1 || v > 7) continue;
    bool dup = false;
    for (int k = 0; k < *n; ++k) dup = dup || out[k] == v;
    if (!dup) out[(*n)++] = v;
  }
  return true;
}

bool fill_device_params(otm_engine* E, std::string* err) {
  const otm::MatchConfig& m = E->mc;
  E->dp.sigma_z = m.sigma_z;
  E->dp.beta = m.beta;
  E->dp.factor = m.max_route_distance_factor;
  E->dp.breakage = m.breakage_distance;
  E->dp.interp = m.interpolation_distance;
  E->dp.search_radius = m.search_radius;
  E->dp.max_search_radius = m.max_search_radius;
  E->dp.gps_accuracy = m.gps_accuracy;
  E->dp.max_candidates = m.max_candidates;
  // the spatial work order in all three kernels that walk it (measured on
  // config 2: candidates 0.60 -> 0.44 ms, route 0.107 -> 0.089, transitions
  // 0.408 -> 0.388)
  E->dp.order_mask = otm::ORDER_CAND | otm::ORDER_TRANS | otm::ORDER_ROUTE;
  if (const char* om = std::getenv("OTM_ORDER_MASK")) E->dp.order_mask = std::atoi(om) & 7;  // A/B knob
  E->dp.cand_wave_all = 0;
  // batches under this many points take the small-batch (latency) path
  const char* sp = std::getenv("OTM_SMALL_POINTS");
  E->small_points = sp ? (int64_t)std::strtoll(sp, nullptr, 0) : 65536;
  const otm::ReportConfig& r = E->rc;
  std::memset(&E->drc, 0, sizeof E->drc);
  if (!device_levels(r.report_levels, E->drc.report_levels, &E->drc.n_report, "REPORT_LEVELS", err)) return false;
  if (!device_levels(r.transition_levels, E->drc.transition_levels, &E->drc.n_transition, "TRANSITION_LEVELS", err))
    return false;
  E->drc.threshold_sec = r.threshold_sec;
  return true;
}

// OTM_JSON_PROFILE=1: one stderr line per request batch with its phases (ms)
double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
bool json_profile() {
  const char* v = std::getenv("OTM_JSON_PROFILE");
  return v && *v == '1';
}
thread_local double t_gpu_ms = 0.0, t_pack_ms = 0.0, t_write_ms = 0.0, t_extract_ms = 0.0;

// The reference's stderr line per invalid speed (reporter_service.py); a
// split call's chunk threads (report_many_split) collect the counts in t_lines
// instead, for the caller to print in chunk order
thread_local std::vector<int>* t_lines = nullptr;
void speed_lines(int n) {
  if (t_lines) {
    t_lines->push_back(n);
    return;
  }
  for (int q = 0; q < n; ++q) std::fputs("Speed exceeds 200kph\n", stderr);
}

// A batch's turn in an H2DOrder (engine.h): the constructor waits until
// every earlier ticket has queued its request copies; after() queues E's
// copies behind them on the device; pass() marks E's copies for the next
// ticket and hands the turn on (the destructor does, on any early exit).
class H2DTurn {
 public:
  H2DTurn(otm::H2DOrder* o, uint64_t t) : o_(o), t_(t) {
    if (!o_) return;
    std::unique_lock<std::mutex> lk(o_->m);
    o_->cv.wait(lk, [&] { return o_->next == t_; });
  }
  void after(otm_engine* E) {
    if (o_ && t_ > 0 && o_->ev[(t_ - 1) & 1]) (void)otm::engine_push_after(E, o_->ev[(t_ - 1) & 1]);
  }
  void pass(otm_engine* E) {
    if (!o_ || passed_) return;
    passed_ = true;
    hipEvent_t& ev = o_->ev[t_ & 1];
    if (E && !ev) (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (E && ev) (void)otm::engine_push_mark(E, ev);
    {
      std::lock_guard<std::mutex> lk(o_->m);
      o_->next = t_ + 1;
    }
    o_->cv.notify_all();
  }
  ~H2DTurn() { pass(nullptr); }
  H2DTurn(const H2DTurn&) = delete;
  H2DTurn& operator=(const H2DTurn&) = delete;

 private:
  otm::H2DOrder* o_;
  uint64_t t_;
  bool passed_ = false;
};

// One request of a batch: its DOM (parse_request), or -- for the Java
// batcher's own bytes -- its points and uuid read directly (fast_request).
struct Req {
  Value dom;
  otm::TracePoints tp;
  std::string uuid;
  bool fast = false;
};

// One GPU batch over parsed requests: results[k] -> (code, body)
void run_requests(otm_engine* E, std::vector<Req>& rq, std::vector<int>& codes, std::vector<std::string>& bodies,
                  const std::vector<int>& todo, bool match_only) {
  // points of every request that passed validation (extracted in parallel,
  // then laid out in request order)
  const double te0 = now_ms();
  std::vector<uint8_t> ok(todo.size(), 0);
  par_for(todo.size(), [&](size_t a, size_t e) {
    for (size_t i = a; i < e; ++i) {
      const int k = todo[i];
      std::string perr;
      if (rq[(size_t)k].fast || otm::extract_points(rq[(size_t)k].dom, &rq[(size_t)k].tp, &perr)) {
        ok[i] = 1;
      } else {
        codes[(size_t)k] = 500;
        bodies[(size_t)k] = otm::error_body(perr);
      }
    }
  });
  const double tp0 = now_ms();
  t_extract_ms = tp0 - te0;
  t_gpu_ms = t_write_ms = t_pack_ms = 0.0;
  std::vector<int64_t> off(1, 0);
  std::vector<int> which;  // request index of each batch trace
  for (size_t i = 0; i < todo.size(); ++i)
    if (ok[i]) {
      off.push_back(off.back() + (int64_t)rq[(size_t)todo[i]].tp.lat.size());
      which.push_back(todo[i]);
    }
  if (which.empty()) return;
  const size_t np = (size_t)off.back();
  // the batch arrays: per calling thread, kept between calls (grown, never
  // shrunk) -- fresh ones cost ~3 ms of page faults to fill and ~2.5 ms to
  // unmap per 1M points
  thread_local std::vector<float> keep_lat, keep_lon, keep_acc;
  thread_local std::vector<double> keep_tm;
  std::vector<float> own_lat, own_lon, own_acc;
  std::vector<double> own_tm;
  constexpr bool reuse = true;
  std::vector<float>& lat = reuse ? keep_lat : own_lat;
  std::vector<float>& lon = reuse ? keep_lon : own_lon;
  std::vector<float>& acc = reuse ? keep_acc : own_acc;
  std::vector<double>& tm = reuse ? keep_tm : own_tm;
  if (lat.size() < np) {
    lat.resize(np);
    lon.resize(np);
    acc.resize(np);
    tm.resize(np);
  }
  par_for(which.size(), [&](size_t a, size_t e) {
    for (size_t n = a; n < e; ++n) {
      otm::TracePoints& tp = rq[(size_t)which[n]].tp;
      const size_t o = (size_t)off[n];
      std::copy(tp.lat.begin(), tp.lat.end(), lat.begin() + o);
      std::copy(tp.lon.begin(), tp.lon.end(), lon.begin() + o);
      std::copy(tp.acc.begin(), tp.acc.end(), acc.begin() + o);
      std::copy(tp.time.begin(), tp.time.end(), tm.begin() + o);
      tp = otm::TracePoints();
    }
  });
  otm_batch b;
  b.n_traces = (int32_t)which.size();
  b.n_points = off.back();
  b.trace_off = off.data();
  b.lat = lat.data();
  b.lon = lon.data();
  b.time = tm.data();
  b.accuracy = acc.data();
  std::string err;
  otm_results r;
  int rc;
  // a multi-device engine: each trace to its uuid's member (Kafka's partition);
  // a uuid that is not a string (the reference accepts any non-null) to member 0
  std::vector<int32_t> shard;
  if (!E->members.empty()) {
    shard.resize(which.size(), 0);
    for (size_t n = 0; n < which.size(); ++n) {
      const Req& q = rq[(size_t)which[n]];
      const Value* u = q.fast ? nullptr : q.dom.get("uuid");
      if (q.fast) shard[n] = otm::shard_of(q.uuid.data(), q.uuid.size(), (int)E->members.size());
      else if (u && u->kind == Kind::Str) shard[n] = otm::shard_of(u->s.data(), u->s.size(), (int)E->members.size());
    }
  }
  {
    std::lock_guard<std::mutex> lk(E->mu);
    const double tg0 = now_ms();
    t_pack_ms = tg0 - tp0;
    rc = otm::match_host_fetch(E, &b, shard.empty() ? nullptr : shard.data(), &r, &err);
    const double tg1 = now_ms();
    t_gpu_ms = tg1 - tg0;
    if (!rc) {
      // the responses in parallel (each writes its own slot), the reference's
      // stderr lines after, in request order
      par_for(which.size(), [&](size_t a, size_t e) {
        for (size_t n = a; n < e; ++n) {
          const int k = which[n];
          std::string out;
          if (match_only) {
            const otm_trace_result& tr = r.traces[n];
            if (tr.code != 200 && tr.error_kind != OTM_TERR_ZERODIV) {
              codes[(size_t)k] = 500;
              bodies[(size_t)k] = otm::error_body(otm::trace_error_text(tr.error_kind));
            } else {
              otm::write_match_json(r, (int32_t)n, &out);
              codes[(size_t)k] = 200;
              bodies[(size_t)k] = std::move(out);
            }
          } else {
            // written into a per-thread buffer that keeps its capacity, then
            // copied once at its final size (no growth reallocations per body)
            thread_local std::string scratch;
            scratch.clear();
            codes[(size_t)k] = otm::write_report_response(r, (int32_t)n, &scratch);
            bodies[(size_t)k].assign(scratch);
          }
        }
      });
      if (!match_only)
        for (size_t n = 0; n < which.size(); ++n) {
          const int inv = r.traces[n].code == 200 ? r.traces[n].invalid_speeds : 0;
          speed_lines(inv);
        }
      t_write_ms = now_ms() - tg1;
    }
  }
  if (rc) {
    // a device failure fails the batch, not the process (500 like :239-240)
    for (int k : which) {
      codes[(size_t)k] = 500;
      bodies[(size_t)k] = otm::error_body(err);
    }
  }
}

// Response arenas: the bodies of one request batch cut from one allocation
// instead of one malloc each (10k mallocs per batch from many threads, each
// first-touching fresh heap pages, measured 2-20 ms per batch inside the
// bench against 0.5 ms warm).  otm_free recognises a pointer inside a live
// arena by its address range and releases the arena with its last body; any
// other pointer is std::free'd as before.  A released arena is kept (up to
// ARENA_CACHE bytes in all) for the next batch, so its pages stay mapped.
// The GPU response writer's arenas are page-locked: the body blob is copied
// from HBM straight into them, NUL terminators included, so its bodies are
// never copied on the host (0.45 ms per 10k responses).
namespace arena {
constexpr int SLOTS = 64;
constexpr size_t ARENA_CACHE = (size_t)256 << 20;
enum : int { FREE = 0, LIVE = 1, CACHED = 2 };
struct Slot {
  // gen is a seqlock over (state, lo, hi): odd while acquire() or release()
  // rewrites them, so free_body's lock-free scan can tell a consistent
  // snapshot from one torn across a release and a re-acquire
  std::atomic<uint64_t> gen{0};
  std::atomic<int> state{FREE};
  std::atomic<uintptr_t> lo{0}, hi{0};
  std::atomic<int64_t> refs{0};
  char* base = nullptr;
  size_t cap = 0;
  bool pinned = false;  // page-locked (hipHostMalloc): a device copy's target
};
Slot g_slot[SLOTS];
std::atomic<int64_t> g_releases{0};  // arenas released by their last body (otm_debug_arena_stress)
std::mutex g_mu;
size_t g_cached = 0;  // under g_mu

void drop(Slot& S) {
  if (S.pinned) (void)hipHostFree(S.base);
  else std::free(S.base);
  S.base = nullptr;
  S.cap = 0;
}

// an arena of >= bytes for nbodies bodies (page-locked if pinned), or nullptr
// (the caller places the bodies some other way)
char* acquire(size_t bytes, int64_t nbodies, bool pinned = false) {
  if (nbodies <= 0) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  int best = -1, free_slot = -1;
  for (int i = 0; i < SLOTS; ++i) {
    const int st = g_slot[i].state.load();
    if (st == CACHED && g_slot[i].pinned == pinned && g_slot[i].cap >= bytes &&
        (best < 0 || g_slot[i].cap < g_slot[best].cap))
      best = i;
    if (st == FREE && free_slot < 0) free_slot = i;
  }
  if (best < 0 && free_slot < 0) {
    // every slot taken: give up the smallest cached arena of either kind
    for (int i = 0; i < SLOTS; ++i)
      if (g_slot[i].state.load() == CACHED && (free_slot < 0 || g_slot[i].cap < g_slot[free_slot].cap)) free_slot = i;
    if (free_slot >= 0) {
      g_cached -= g_slot[free_slot].cap;
      drop(g_slot[free_slot]);
      g_slot[free_slot].state.store(FREE);
    }
  }
  if (best < 0) {
    if (free_slot < 0) return nullptr;
    void* p = nullptr;
    if (pinned) {
      if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) p = nullptr;
    } else {
      p = std::malloc(bytes);
    }
    if (!p) return nullptr;
    best = free_slot;
    g_slot[best].base = (char*)p;
    g_slot[best].cap = bytes;
    g_slot[best].pinned = pinned;
  } else {
    g_cached -= g_slot[best].cap;
  }
  Slot& S = g_slot[best];
  S.gen.fetch_add(1);  // odd: being rewritten
  S.refs.store(nbodies);
  S.lo.store((uintptr_t)S.base);
  S.hi.store((uintptr_t)S.base + S.cap);
  S.state.store(LIVE);
  S.gen.fetch_add(1);
  return S.base;
}

void release(Slot& S) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_releases.fetch_add(1);
  // out of every address range, then out of LIVE, inside one odd generation,
  // before the memory can go back to the allocator: free_body's scan must
  // never match a pointer the allocator hands out again inside the old range
  S.gen.fetch_add(1);
  S.hi.store(0);
  S.lo.store(0);
  const bool keep = g_cached + S.cap <= ARENA_CACHE;
  if (keep) g_cached += S.cap;
  S.state.store(keep ? CACHED : FREE);
  S.gen.fetch_add(1);
  if (!keep) drop(S);
}

// otm_free: a body inside a live arena, or a plain allocation
void free_body(void* p) {
  if (!p) return;
  const uintptr_t a = (uintptr_t)p;
  for (int i = 0; i < SLOTS; ++i) {
    Slot& S = g_slot[i];
    // a consistent (gen, state, lo, hi) snapshot: the generation even and
    // unchanged across the reads.  A LIVE range holding p at that instant is
    // p's arena (a live body keeps its arena's refs above 0, so it cannot be
    // released under us); a torn snapshot is read again.
    while (true) {
      const uint64_t g0 = S.gen.load(std::memory_order_acquire);
      if (g0 & 1u) continue;
      const int st = S.state.load(std::memory_order_acquire);
      const uintptr_t lo = S.lo.load(std::memory_order_acquire), hi = S.hi.load(std::memory_order_acquire);
      std::atomic_thread_fence(std::memory_order_acquire);
      if (S.gen.load(std::memory_order_relaxed) != g0) continue;
      if (st == LIVE && a >= lo && a < hi) {
        if (S.refs.fetch_sub(1) == 1) release(S);
        return;
      }
      break;
    }
  }
  std::free(p);
}
}  // namespace arena

// Submission slabs: otm_submit_batch copies its bodies into one allocation,
// page-locked from SLAB_PINNED_MIN bytes up, so the worker's batch goes to HBM
// straight from it (report_many_device's direct pieces): one host copy per
// body instead of two (the submit copy and the staging copy), and no malloc
// per request.  Released page-locked slabs are kept (up to SLAB_CACHE bytes)
// for later submissions; the small ones are plain mallocs.
namespace slabs {
constexpr size_t SLAB_PINNED_MIN = (size_t)1 << 20;
constexpr size_t SLAB_MAX = (size_t)128 << 20;  // one slab per submission up to this
size_t pinned_min() {  // OTM_SLAB_PINNED_MIN overrides (tests: every slab page-locked)
  const char* e = std::getenv("OTM_SLAB_PINNED_MIN");
  return e ? (size_t)std::strtoull(e, nullptr, 10) : SLAB_PINNED_MIN;
}
constexpr size_t SLAB_CACHE = (size_t)512 << 20;
std::mutex g_mu;
std::vector<ReqSlab*> g_cache;  // under g_mu
size_t g_cached = 0;

void release(ReqSlab* s) {
  if (s->pinned) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_cached + s->cap <= SLAB_CACHE) {
      g_cache.push_back(s);
      g_cached += s->cap;
      return;
    }
  }
  if (s->pinned) (void)hipHostFree(s->base);
  else std::free(s->base);
  delete s;
}

// a slab of >= bytes, page-locked from pinned_min() up (always with
// must_pin, else nullptr when none is to be had) unless !may_pin (throws
// std::bad_alloc when there is no memory at all)
std::shared_ptr<ReqSlab> acquire(size_t bytes, bool may_pin = true, bool must_pin = false) {
  ReqSlab* s = nullptr;
  if (must_pin || (may_pin && bytes >= pinned_min())) {
    {
      std::lock_guard<std::mutex> lk(g_mu);
      size_t best = g_cache.size();
      for (size_t i = 0; i < g_cache.size(); ++i)
        if (g_cache[i]->cap >= bytes && (best == g_cache.size() || g_cache[i]->cap < g_cache[best]->cap)) best = i;
      if (best < g_cache.size()) {
        s = g_cache[best];
        g_cache[best] = g_cache.back();
        g_cache.pop_back();
        g_cached -= s->cap;
      }
    }
    if (!s) {
      const size_t cap = (bytes + SLAB_PINNED_MIN - 1) & ~(SLAB_PINNED_MIN - 1);
      void* p = nullptr;
      if (hipHostMalloc(&p, cap, hipHostMallocDefault) == hipSuccess && p) s = new ReqSlab{(char*)p, cap, true};
    }
    if (!s && must_pin) return nullptr;
  }
  if (!s) {
    char* p = (char*)std::malloc(bytes ? bytes : 1);
    if (!p) throw std::bad_alloc();
    s = new ReqSlab{p, bytes, false};
  }
  return std::shared_ptr<ReqSlab>(s, release);
}
}  // namespace slabs

// Request arenas (otm_request_arena_alloc): page-locked slabs the host writes
// its request bodies into, registered by address range.  otm_report_batch
// and otm_submit_batch find their bodies here and send them to HBM straight
// from the arena (report_many_device's direct pieces): no staging copy, no
// submission copy.  A submission holds its arena (the shared slab) until its
// batch has run, so release only gives up the caller's hold.
namespace reqarena {
struct Entry {
  uintptr_t lo, hi;
  std::shared_ptr<ReqSlab> slab;
};
std::mutex g_mu;
std::vector<Entry> g_live;  // under g_mu

void* alloc(size_t bytes) {
  std::shared_ptr<ReqSlab> s = slabs::acquire(bytes ? bytes : 1, true, true);
  if (!s) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  g_live.push_back(Entry{(uintptr_t)s->base, (uintptr_t)s->base + s->cap, s});
  return s->base;
}

bool release(void* p) {
  std::shared_ptr<ReqSlab> drop;  // (released after the lock)
  std::lock_guard<std::mutex> lk(g_mu);
  for (size_t i = 0; i < g_live.size(); ++i)
    if (g_live[i].lo == (uintptr_t)p) {
      drop = std::move(g_live[i].slab);
      g_live[i] = std::move(g_live.back());
      g_live.pop_back();
      return true;
    }
  return false;
}

// the arena holding each body [reqs[k], reqs[k] + lens[k]) (all of it), or
// null; returns whether every body lies in one
bool find(int n, const char* const* reqs, const size_t* lens, std::vector<std::shared_ptr<ReqSlab>>* out) {
  out->assign((size_t)n, nullptr);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_live.empty()) return false;
  bool all = true;
  size_t last = 0;
  for (int k = 0; k < n; ++k) {
    const uintptr_t a = (uintptr_t)reqs[k], e = a + lens[k];
    bool hit = false;
    for (size_t t = 0; t < g_live.size() && !hit; ++t) {
      const size_t i = (last + t) % g_live.size();  // (bodies of one call mostly share an arena)
      if (a >= g_live[i].lo && e <= g_live[i].hi) {
        (*out)[(size_t)k] = g_live[i].slab;
        last = i;
        hit = true;
      }
    }
    all = all && hit;
  }
  return all;
}
}  // namespace reqarena

// each response of a batch into its place in one arena (or its own malloc'd
// buffer when no arena is to be had): src(k) -> (pointer, length); returns
// false when out of host memory (nothing left allocated)
template <class Src>
bool place_bodies(int n, Src src, char** resps, size_t* resp_lens) {
  std::vector<size_t> off((size_t)n + 1, 0);
  for (int k = 0; k < n; ++k) off[(size_t)k + 1] = off[(size_t)k] + src(k).second + 1;
  char* base = arena::acquire(off[(size_t)n], n);
  std::atomic<bool> oom{false};
  par_for((size_t)n, [&](size_t a, size_t e) {
    for (size_t k = a; k < e; ++k) {
      const std::pair<const char*, size_t> b = src((int)k);
      char* p = base ? base + off[k] : (char*)std::malloc(b.second + 1);
      if (!p) {
        oom = true;
        resps[k] = nullptr;
        continue;
      }
      if (b.second) std::memcpy(p, b.first, b.second);
      p[b.second] = 0;
      resps[k] = p;
      resp_lens[k] = b.second;
    }
  });
  if (oom) {
    for (int k = 0; k < n; ++k) {
      arena::free_body(resps[k]);
      resps[k] = nullptr;
    }
    return false;
  }
  return true;
}

// every request's response placed for the caller (otm_free releases each):
// all of them or none -- a failed allocation frees the ones already made
// (the caller gets only the error, nothing to otm_free)
void copy_out(int n, const std::vector<int>& c, const std::vector<std::string>& bodies, int* codes, char** resps,
              size_t* resp_lens) {
  for (int k = 0; k < n; ++k) codes[k] = c[(size_t)k];
  if (!place_bodies(n, [&](int k) { return std::pair<const char*, size_t>(bodies[(size_t)k].data(), bodies[(size_t)k].size()); },
                    resps, resp_lens))
    throw std::bad_alloc();
}

// the host readers: every body parsed on the host threads (fast_request, or
// the json.loads-semantics DOM), one GPU batch, responses on the host threads
void report_many_host(otm_engine* E, int n, const char* const* reqs, const size_t* lens, int* codes, char** resps,
                      size_t* resp_lens) {
  const double t0 = now_ms();
  std::vector<Req> rq((size_t)n);
  std::vector<int> c((size_t)n, 0);
  std::vector<std::string> bodies((size_t)n);
  std::vector<int> todo;
  par_for((size_t)n, [&](size_t a, size_t e) {
    for (size_t k = a; k < e; ++k) {
      const std::string_view body(reqs[k], lens[k]);
      if (fast_requests() && otm::fast_request(body, &rq[k].tp, &rq[k].uuid)) {
        rq[k].fast = true;
        continue;
      }
      const int code = otm::parse_request("/report", body, &rq[k].dom, &bodies[k]);
      if (code) c[k] = code;
    }
  });
  for (int k = 0; k < n; ++k)
    if (!c[(size_t)k]) todo.push_back(k);
  const double t1 = now_ms();
  run_requests(E, rq, c, bodies, todo, false);
  const double t2 = now_ms();
  copy_out(n, c, bodies, codes, resps, resp_lens);
  const double t3 = now_ms();
  // the response strings released by the pool threads that wrote them (their
  // allocator arenas), the requests with them
  par_for((size_t)n, [&](size_t a, size_t e) {
    for (size_t k = a; k < e; ++k) {
      std::string().swap(bodies[k]);
      rq[k] = Req();
    }
  });
  std::vector<Req>().swap(rq);
  const double t4 = now_ms();
  if (json_profile())
    std::fprintf(stderr, "[otm json] %d requests: parse %.2f, extract %.2f, pack %.2f, gpu %.2f, write %.2f, "
                 "tail %.2f, copy out %.2f, free %.2f ms\n",
                 n, t1 - t0, t_extract_ms, t_pack_ms, t_gpu_ms, t_write_ms,
                 (t2 - t1) - t_extract_ms - t_pack_ms - t_gpu_ms - t_write_ms, t3 - t2, t4 - t3);
}

// The GPU request reader (requests.hip) for a batch of at least
// OTM_GPU_JSON_MIN requests (default 32) on a one-device engine; OTM_GPU_JSON=0
// keeps every body on the host readers (A/B and the parity tests)
bool gpu_reader(const otm_engine* E, int n) {
  if (!E->members.empty()) return false;
  const char* v = std::getenv("OTM_GPU_JSON");
  if (v && *v == '0') return false;
  const char* m = std::getenv("OTM_GPU_JSON_MIN");
  return n >= (m ? std::atoi(m) : 32);
}

// The GPU response writer (responses.hip) behind the GPU request reader;
// OTM_GPU_WRITE=0 writes the responses on the host threads instead
bool gpu_writer() {
  const char* v = std::getenv("OTM_GPU_WRITE");
  return !(v && *v == '0');
}

// otm_report_batch on the GPU: the bodies staged into one pinned blob by the
// host threads, copied to HBM once, decoded and matched there
// (engine_match_requests), the response bodies written there
// (engine_write_responses) and copied back as one blob, from which each
// response is cut into its own allocation.  Bodies outside the Java
// batcher's exact form are read by the host readers after, as one more batch
// (report_many_host: the same results and error contract); a body the GPU
// writer leaves (a 500, a float outside its range) is written on the host
// from the batch's typed records.
void report_many_device(otm_engine* E, int n, const char* const* reqs, const size_t* lens, int* codes,
                        char** resps, size_t* resp_lens, const void* const* pinned, otm::H2DOrder* ord,
                        uint64_t ticket) {
  H2DTurn turn(ord, ticket);  // (before the context's lock: a turn never waits holding one)
  const double t0 = now_ms();
  std::vector<int> rest;  // left to the host readers
  std::vector<int> inv;   // invalid speeds per GPU-read request (stderr lines)
  std::vector<int> which;
  double t1 = t0, t2 = t0, t3 = t0, tl = t0, tm = t0;
  int rc;
  std::string err;
  for (int k = 0; k < n; ++k) resps[k] = nullptr;
  std::atomic<bool> oom{false};
  {
    std::lock_guard<std::mutex> lk(E->mu);
    tl = now_ms();
    // an async worker's batch (ord): its copies on the pipeline's one copy
    // stream (engine.h req_shared; created by the turn's holder, so by one
    // thread at a time); a one-call batch: the context's own copy stream
    if (ord && !ord->copy) (void)otm::create_stream(-1, &ord->copy, ord->own_queue);
    E->req_shared = ord ? ord->copy : nullptr;
    size_t bytes = 0;
    for (int k = 0; k < n; ++k) bytes += lens[k];
    int64_t* off = nullptr;
    char* dst = nullptr;
    bool all_pinned = pinned != nullptr;
    for (int k = 0; all_pinned && k < n; ++k) all_pinned = pinned[k] != nullptr;
    rc = otm::engine_stage_requests(E, n, bytes, !all_pinned, &off, &dst, &err);
    turn.after(E);
    if (!rc) {
      off[0] = 0;
      for (int k = 0; k < n; ++k) off[k + 1] = off[k] + (int64_t)lens[k];
      // staged in pieces of ~16 MB, each on its way to HBM while the next is
      // copied (the host copy and the DMA overlap)
      constexpr size_t PIECE = (size_t)16 << 20;
      int k0 = 0;
      size_t from = 0;
      while (!rc && k0 < n) {
        int k1 = k0;
        while (k1 < n && (size_t)off[k1 + 1] - from <= PIECE) ++k1;
        if (k1 == k0) ++k1;  // one body larger than a piece
        const bool direct = pinned && pinned[k0];
        if (direct) {
          // a run of bodies adjacent in one page-locked submission slab:
          // copied to HBM from there, not staged (two slabs that happen to be
          // adjacent in memory are two allocations: two copies)
          // (cut at PIECE bytes too, so the reads of one piece overlap the
          // next piece's DMA)
          k1 = k0 + 1;
          while (k1 < n && pinned[k1] == pinned[k0] && reqs[k1] == reqs[k1 - 1] + lens[k1 - 1] &&
                 (size_t)off[k1 + 1] - from <= PIECE)
            ++k1;
        } else {
          while (k1 > k0 + 1 && pinned && pinned[k1 - 1] != nullptr) --k1;  // (the staged piece stops at a slab run)
          par_for((size_t)(k1 - k0), [&](size_t a, size_t e) {
            for (size_t m = a; m < e; ++m) {
              const size_t k = (size_t)k0 + m;
              if (lens[k]) std::memcpy(dst + off[k], reqs[k], lens[k]);
            }
          });
        }
        const size_t to = (size_t)off[k1];
        rc = otm::engine_push_requests(E, n, bytes, from, to, direct ? reqs[k0] : nullptr, k1, &err);
        from = to;
        k0 = k1;
      }
      if (!rc && n == 0) rc = otm::engine_push_requests(E, n, bytes, 0, 0, nullptr, 0, &err);
    }
    turn.pass(E);
    if (!rc) {
      t1 = now_ms();
      const uint8_t* ok = nullptr;
      int32_t nt = 0;
      otm_results r;
      bool typed = false;
      const bool gw = gpu_writer();
      const int64_t* boff = nullptr;
      const uint8_t* hostw = nullptr;
      const otm_trace_result* trs = nullptr;
      int64_t total = 0;
      rc = otm::engine_match_requests(E, n, bytes, true, &ok, &nt, &err);
      tm = now_ms();
      if (!rc) {
        if (gw) {
          rc = otm::engine_write_responses(E, &boff, &hostw, &trs, &total, &err);
          bool any = false;
          for (int32_t m = 0; !rc && m < nt && !any; ++m) any = hostw[m] != 0;
          if (!rc && any) {
            rc = otm::engine_fetch(E, &r, &err);  // the typed records for the host writer
            typed = true;
          }
        } else {
          rc = otm::engine_fetch(E, &r, &err);
          typed = true;
          trs = r.traces;
        }
      }
      t2 = now_ms();
      if (!rc) {
        which.reserve((size_t)nt);
        for (int k = 0; k < n; ++k) (ok[k] ? which : rest).push_back(k);
        inv.assign(which.size(), 0);
        // the bodies the GPU did not write (host writer, from the typed records)
        std::vector<std::string> hb(typed ? which.size() : 0);
        if (typed)
          par_for(which.size(), [&](size_t a, size_t e) {
            for (size_t m = a; m < e; ++m)
              if (!gw || hostw[m]) codes[which[m]] = otm::write_report_response(r, (int32_t)m, &hb[m]);
          });
        for (size_t m = 0; m < which.size(); ++m) {
          if (gw && !hostw[m]) codes[which[m]] = 200;
          inv[m] = trs[m].code == 200 ? trs[m].invalid_speeds : 0;
        }
        // The GPU-written bodies are copied from HBM straight into a pinned
        // response arena, each already NUL-terminated in place (no host copy
        // of them); the host-written ones go after them in the same arena.
        size_t hbytes = 0;
        for (size_t m = 0; m < hb.size(); ++m)
          if (!gw || hostw[m]) hbytes += hb[m].size() + 1;
        char* base = gw ? arena::acquire((size_t)total + hbytes, (int64_t)which.size(), true) : nullptr;
        if (base) {
          size_t at = (size_t)total;
          for (size_t m = 0; m < which.size(); ++m) {
            const int k = which[m];
            if (!hostw[m]) {
              resps[k] = base + boff[m];
              resp_lens[k] = (size_t)(boff[m + 1] - boff[m] - 1);
            } else {
              resps[k] = base + at;
              resp_lens[k] = hb[m].size();
              std::memcpy(base + at, hb[m].data(), hb[m].size());
              base[at + hb[m].size()] = 0;
              at += hb[m].size() + 1;
            }
          }
          const char* blob = nullptr;
          rc = otm::engine_copy_responses(E, base, total, &blob, &err);  // (rc: free_all below)
        } else {
          // no pinned arena to be had (or the host writer): the blob through
          // the engine's buffer, each response cut from a plain arena
          const char* blob = nullptr;
          if (gw) rc = otm::engine_copy_responses(E, nullptr, total, &blob, &err);
          std::vector<char*> wr(which.size(), nullptr);
          std::vector<size_t> wl(which.size(), 0);
          if (!rc && !place_bodies(
                         (int)which.size(),
                         [&](int m) {
                           if (gw && !hostw[m])
                             return std::pair<const char*, size_t>(blob + boff[m], (size_t)(boff[m + 1] - boff[m] - 1));
                           return std::pair<const char*, size_t>(hb[(size_t)m].data(), hb[(size_t)m].size());
                         },
                         wr.data(), wl.data()))
            oom = true;
          for (size_t m = 0; m < which.size(); ++m) {
            resps[which[m]] = wr[m];
            resp_lens[which[m]] = wl[m];
          }
        }
        t3 = now_ms();
      }
    }
  }
  auto free_all = [&] {
    for (int k = 0; k < n; ++k) {
      arena::free_body(resps[k]);
      resps[k] = nullptr;
    }
  };
  if (oom) {
    free_all();
    throw std::bad_alloc();
  }
  if (rc) {
    // a staging or device failure: the whole batch through the host readers
    // (their own 400s, and 500s for what reaches the device)
    free_all();
    report_many_host(E, n, reqs, lens, codes, resps, resp_lens);
    return;
  }
  // the reference's stderr lines of the GPU-read requests, in request order
  for (size_t m = 0; m < which.size(); ++m)
    speed_lines(inv[m]);
  if (!rest.empty()) {
    const size_t nr = rest.size();
    std::vector<const char*> rq(nr);
    std::vector<size_t> rl(nr), ol(nr, 0);
    std::vector<int> rcodes(nr, 500);
    std::vector<char*> rr(nr, nullptr);
    for (size_t m = 0; m < nr; ++m) {
      rq[m] = reqs[rest[m]];
      rl[m] = lens[rest[m]];
    }
    try {
      report_many_host(E, (int)nr, rq.data(), rl.data(), rcodes.data(), rr.data(), ol.data());
    } catch (...) {
      free_all();
      throw;
    }
    for (size_t m = 0; m < nr; ++m) {
      codes[rest[m]] = rcodes[m];
      resps[rest[m]] = rr[m];
      resp_lens[rest[m]] = ol[m];
    }
  }
  if (json_profile())
    std::fprintf(stderr, "[otm json gpu] %d requests (%zu on the host readers): stage %.2f, gpu %.2f, copy out %.2f, "
                 "host readers %.2f ms; at %.2f: lock %.2f, read+sync %.2f, match %.2f, write %.2f ms\n",
                 n, rest.size(), t1 - t0, t2 - t1, t3 - t2, now_ms() - t3, t0, tl - t0,
                 E->t_read_done - t1, tm - E->t_read_done, t2 - tm);
}

// (pinned[k]: the page-locked submission slab body k lies in, or null;
// ord / ticket: the batch's place in an H2DOrder, or null)
void report_many(otm_engine* E, int n, const char* const* reqs, const size_t* lens, int* codes, char** resps,
                 size_t* resp_lens, const void* const* pinned = nullptr, otm::H2DOrder* ord = nullptr,
                 uint64_t ticket = 0) {
  // the batch buffers, pinned staging and copy streams this thread creates
  // belong on the engine's device, whatever device the calling thread is on
  if (E->members.empty() && E->device >= 0) (void)hipSetDevice(E->device);
  if (gpu_reader(E, n)) {
    report_many_device(E, n, reqs, lens, codes, resps, resp_lens, pinned, ord, ticket);
  } else {
    H2DTurn(ord, ticket).pass(nullptr);  // (no copies of its own: the turn moves on)
    report_many_host(E, n, reqs, lens, codes, resps, resp_lens);
  }
}

// Requests per async batch (OTM_ASYNC_BATCH): small enough that a burst of
// submissions splits over the pipeline's workers, large enough to fill the GPU
// (profiles/r03_s2/async_ab.txt: 3 workers x 16384 the steadiest, ~250M points/s
// on 10k-request submissions; 2 x 8192 ~220M; 1 worker ~150M).
size_t async_batch() {
  const char* e = std::getenv("OTM_ASYNC_BATCH");  // (read per batch: tests switch it)
  return e ? (size_t)std::max(1, std::atoi(e)) : (size_t)16384;
}
// Pipeline depth (OTM_ASYNC_WORKERS, default 3): batch contexts working at
// once.  A multi-device engine or a clone runs one (its members / parent own
// the other contexts).
int async_workers(const otm_engine* E) {
  if (!E->members.empty() || E->parent) return 1;
  const char* e = std::getenv("OTM_ASYNC_WORKERS");
  return e ? std::max(1, std::min(8, std::atoi(e))) : 3;
}


// Worker wi of the async pipeline: take the next batch (in submit order, a
// ticket each), run it whole on its own context -- parse, GPU, responses --
// then publish its results once every earlier batch has published, so each
// uuid's results come back in submit order.
void worker_loop(otm_engine* E, int wi) {
  otm_engine* ctx = E->awx.empty() ? E : E->awx[(size_t)wi];
  // a new thread starts on device 0: everything it creates for ctx (its
  // streams' buffers, page-locked staging) goes on ctx's device
  if (ctx->members.empty() && ctx->device >= 0) (void)hipSetDevice(ctx->device);
  while (true) {
    std::vector<otm_engine::Pending> batch;
    uint64_t seq;
    {
      std::unique_lock<std::mutex> lk(E->qmu);
      E->qcv.wait(lk, [&] { return E->stop || !E->queue.empty(); });
      if (E->queue.empty()) return;  // stopping, nothing left
      // up to cap requests; a submission that does not fit whole waits for
      // the next batch (unless it alone exceeds cap), so batches keep the
      // submissions' sizes and each is one run of one slab
      const size_t cap = async_batch();
      while (!E->queue.empty() && batch.size() < cap) {
        const otm_engine::Pending& f = E->queue.front();
        if (!batch.empty() && f.sub != batch.back().sub && batch.size() + f.run_left > cap) break;
        batch.push_back(std::move(E->queue.front()));
        E->queue.pop_front();
      }
      seq = E->take_seq++;
    }
    const int n = (int)batch.size();
    std::vector<const char*> reqs((size_t)n);
    std::vector<size_t> lens((size_t)n), rl((size_t)n, 0);
    std::vector<int> codes((size_t)n, 500);
    std::vector<char*> resps((size_t)n, nullptr);
    std::vector<const void*> pin((size_t)n, nullptr);
    for (int k = 0; k < n; ++k) {
      reqs[(size_t)k] = batch[(size_t)k].p;
      lens[(size_t)k] = batch[(size_t)k].len;
      pin[(size_t)k] = batch[(size_t)k].slab->pinned ? batch[(size_t)k].slab.get() : nullptr;
    }
    const double tw0 = now_ms();
    try {
      report_many(ctx, n, reqs.data(), lens.data(), codes.data(), resps.data(), rl.data(), pin.data(),
                  &E->aorder, seq);  // (copies in take order, H2DOrder)
    } catch (...) {
      // out of host memory (report_many freed what it made): the batch's
      // requests complete with a null body and code 500
      for (int k = 0; k < n; ++k) {
        codes[(size_t)k] = 500;
        resps[(size_t)k] = nullptr;
        rl[(size_t)k] = 0;
      }
    }
    const double tw1 = now_ms();
    {
      std::unique_lock<std::mutex> lk(E->qmu);
      E->qcv.wait(lk, [&] { return E->pub_seq == seq; });
      if (json_profile())
        std::fprintf(stderr, "[otm async] worker %d batch %llu: %d requests, start %.2f, ran %.2f, published +%.2f ms\n", wi,
                     (unsigned long long)seq, n, tw0, tw1 - tw0, now_ms() - tw1);
      for (int k = 0; k < n; ++k)
        E->done.push_back(otm_result{batch[(size_t)k].tag, codes[(size_t)k], resps[(size_t)k], rl[(size_t)k]});
      ++E->pub_seq;
    }
    E->qcv.notify_all();
  }
}

// the pipeline's workers and their contexts, at the first submission (under E->qmu)
// a split call's batch contexts: up to n clones (under E->qmu) whose streams
// have hardware queues of their own, so the chunks' kernels never sit in a
// queue behind the copy stream's packets (the chunks' copies go on a pooled
// copy stream: SDMA at ~50 GB/s).  Measured (round 5, profiles/r05_ab/
// split_form/, split_ownq/): on two own-queue clones 349-351M points/s
// whatever other streams the process holds; on this engine and a pooled
// clone 231-354M depending on which of the runtime's pooled queues the copy
// stream shared (behind the first chunk's kernels: its match 0.70 -> 1.52 ms);
// with the copy stream on an own queue too, 238-293M (copies at 28-40 GB/s).
void make_contexts(otm_engine* E, int n) {
  if (!E->members.empty() || E->parent) return;
  while ((int)E->actx.size() < n) {
    auto* C = new otm_engine();
    std::string err;
    if (otm::engine_clone(E, C, &err, true) != OTM_OK) {  // fewer contexts, same results
      otm::engine_free(C);
      delete C;
      break;
    }
    E->actx.push_back(C);
  }
}

// the workers and their batch contexts, at the first submission (under
// E->qmu): clones on hardware queues of their own (engine.cpp create_stream),
// apart from the one-call path's contexts
void start_workers(otm_engine* E) {
  const int nw = async_workers(E);
  for (int i = 0; nw > 1 && i < nw; ++i) {
    auto* C = new otm_engine();
    std::string err;
    if (otm::engine_clone(E, C, &err, true) != OTM_OK) {  // fewer workers, same results
      otm::engine_free(C);
      delete C;
      break;
    }
    E->awx.push_back(C);
  }
  E->aorder.own_queue = true;  // (pooled: async 470-480M against 549-554M)
  const int n = E->awx.empty() ? 1 : (int)E->awx.size();
  for (int i = 0; i < n; ++i) E->workers.emplace_back(worker_loop, E, i);
  E->worker_started = true;
}

// One otm_report_batch call over two batch contexts: the bodies cut into two
// chunks (half the bytes each), each run whole on its context (report_many)
// in a thread of its own, the chunks' request copies in chunk order on one
// copy stream (E->split_order), so the first chunk's kernels run while the
// second crosses PCIe, and its responses come back while the second runs.  Each chunk is a batch of its own: the same per-request results
// (the matcher's results do not depend on a trace's batch).  The reference's
// stderr lines are printed after, in chunk order.  Not split: a multi-device
// engine or a clone (one context), an engine counting or timing its kernels
// (those figures are per context), or fewer than SPLIT_MIN requests a chunk.
// Measured (round 5, bench.py json_report on one box, profiles/r05_ab/json_split/):
// two chunks with the first 50-60 % of the bytes 334-343M points/s, 40 %
// 315-323M, 25 % 300-305M, one batch 286-292M; three chunks 268M (their
// kernels share the GPU at once: each small batch's fixed cost is paid three
// times over).
constexpr int SPLIT_CHUNKS = 2;
constexpr int SPLIT_FIRST_PCT = 50;
constexpr int SPLIT_MIN = 2048;
void report_many_split(otm_engine* E, int n, const char* const* reqs, const size_t* lens, int* codes, char** resps,
                       size_t* resp_lens, const void* const* pinned) {
  std::vector<otm_engine*> ctx{E};
  if (E->members.empty() && !E->parent && !E->counting && !E->timing && n >= 2 * SPLIT_MIN) {
    std::lock_guard<std::mutex> lk(E->qmu);
    make_contexts(E, SPLIT_CHUNKS);
    if ((int)E->actx.size() >= SPLIT_CHUNKS) ctx.clear();  // (the chunks on the own-queue clones)
    ctx.insert(ctx.end(), E->actx.begin(), E->actx.end());
  }
  const int chunks = std::min<int>(std::min<int>((int)ctx.size(), SPLIT_CHUNKS), n / SPLIT_MIN);
  std::vector<int> cut((size_t)std::max(chunks, 1) + 1, n);
  cut[0] = 0;
  if (chunks >= 2) {
    // the first chunk SPLIT_FIRST_PCT % of the bytes (its kernels run while the
    // rest is copied), the others equal shares of the rest
    size_t total = 0, acc = 0;
    for (int k = 0; k < n; ++k) total += lens[k];
    const size_t first = total * SPLIT_FIRST_PCT / 100;
    int c = 1;
    for (int k = 0; k < n && c < chunks; ++k) {
      acc += lens[k];
      const size_t want = first + (total - first) * (size_t)(c - 1) / (size_t)(chunks - 1);
      if (acc >= want) cut[(size_t)c++] = k + 1;
    }
  }
  bool even = chunks >= 2;
  for (int c = 0; even && c < chunks; ++c) even = cut[(size_t)c + 1] - cut[(size_t)c] >= SPLIT_MIN / 2;
  if (!even || !gpu_reader(E, n / chunks)) {
    E->last_split = 1;
    report_many(E, n, reqs, lens, codes, resps, resp_lens, pinned);
    return;
  }
  E->last_split = chunks;
  std::lock_guard<std::mutex> sl(E->split_mu);
  otm::H2DOrder& ord = E->split_order;
  {
    std::lock_guard<std::mutex> lk(ord.m);
    ord.next = 0;
  }
  std::vector<std::vector<int>> lines((size_t)chunks);
  std::vector<std::exception_ptr> errs((size_t)chunks);
  auto run = [&](int c) {
    const int a = cut[(size_t)c], m = cut[(size_t)c + 1] - a;
    t_lines = &lines[(size_t)c];
    try {
      report_many(ctx[(size_t)c], m, reqs + a, lens + a, codes + a, resps + a, resp_lens + a,
                  pinned ? pinned + a : nullptr, &ord, (uint64_t)c);
    } catch (...) {
      errs[(size_t)c] = std::current_exception();  // (its turn was passed on: H2DTurn's destructor)
    }
    t_lines = nullptr;
  };
  std::vector<std::thread> th;
  for (int c = 1; c < chunks; ++c) th.emplace_back(run, c);
  run(0);
  for (auto& t : th) t.join();
  for (int c = 0; c < chunks; ++c)
    if (errs[(size_t)c]) {
      // out of host memory in a chunk (it freed its own): the other chunks' bodies too
      for (int k = 0; k < n; ++k) {
        arena::free_body(resps[k]);
        resps[k] = nullptr;
      }
      std::rethrow_exception(errs[(size_t)c]);
    }
  for (const auto& l : lines)
    for (int v : l) speed_lines(v);
}

}  // namespace

extern "C" {

const char* otm_last_error(const otm_engine*) { return t_err.empty() ? otm::thread_error() : t_err.c_str(); }

void otm_free(void* p) { arena::free_body(p); }

void* otm_request_arena_alloc(size_t bytes) {
  try {
    void* p = reqarena::alloc(bytes);
    if (!p) fail(OTM_ENOMEM, "no page-locked memory for a request arena");
    return p;
  } catch (...) {
    fail(OTM_ENOMEM, "out of host memory");
    return nullptr;
  }
}

int otm_request_arena_release(void* arena) {
  if (!arena) return OTM_OK;
  return reqarena::release(arena) ? OTM_OK : fail(OTM_EINVAL, "not a request arena");
}

// the GPU response writer's number formatting, compiled for the host: the
// checks of tests/test_pyrepr.py against Python's own repr / round
int otm_debug_py_repr(double d, char* out) { return otm::pyrepr::py_repr(d, out); }
int otm_debug_py_round3(double x, double* out) { return otm::pyrepr::py_round3(x, out) ? 1 : 0; }

int otm_kmax(void) { return otm::KMAX; }

// The arenas' lock-free otm_free under contention (run by
// tests/test_host.py, and so under TSan by tests/test_sanitizers.py): per
// round every thread cuts bodies from an arena of its own, then all threads
// free a strided share of every thread's bodies, interleaved with plain
// malloc'd pointers (which must never match an arena).  Returns the number of
// arenas left LIVE afterwards plus the difference between the arenas cut and
// the arenas released (0 when every arena was released once, by its own last
// body: a body freed into the wrong arena releases one early, and the real
// arena never).
int otm_debug_last_split(const otm_engine* E) { return E ? E->last_split.load() : -1; }

int otm_debug_arena_stress(int threads, int rounds) {
  if (threads < 1 || threads > 64 || rounds < 0) return -1;
  constexpr int NB = 16;
  std::vector<std::vector<char*>> bodies((size_t)threads, std::vector<char*>(NB, nullptr));
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  auto barrier = [&] {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t g = gen;
    if (++arrived == threads) {
      arrived = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  };
  std::vector<std::thread> th;
  std::atomic<int64_t> cut{0};
  const int64_t rel0 = arena::g_releases.load();
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      for (int r = 0; r < rounds; ++r) {
        const size_t each = 64 + (size_t)((r * 7 + t * 13) % 200);
        char* base = arena::acquire(each * NB, NB);
        if (base) cut.fetch_add(1);
        for (int k = 0; k < NB; ++k) bodies[(size_t)t][(size_t)k] = base ? base + each * (size_t)k : (char*)std::malloc(each);
        barrier();
        for (int q = 0; q < threads; ++q)
          for (int k = t; k < NB; k += threads) {
            arena::free_body(bodies[(size_t)q][(size_t)k]);
            arena::free_body(std::malloc(each));  // a plain pointer through the same scan
          }
        barrier();
      }
    });
  for (auto& x : th) x.join();
  int live = 0;
  for (int i = 0; i < arena::SLOTS; ++i) live += arena::g_slot[i].state.load() == arena::LIVE ? 1 : 0;
  return live + (int)std::llabs(cut.load() - (arena::g_releases.load() - rel0));
}

void* otm_stream_create(otm_engine* E, int own_queue) {
  if (!E) return nullptr;
  otm_engine* D = E->members.empty() ? E : E->members[0];
  if (D->device >= 0 && hipSetDevice(D->device) != hipSuccess) return nullptr;
  hipStream_t s = nullptr;
  if (otm::create_stream(0, &s, own_queue != 0)) return nullptr;
  return s;
}

void otm_stream_destroy(void* s) {
  if (s) (void)hipStreamDestroy((hipStream_t)s);
}

const char* otm_runtime_info(void) {
  static thread_local std::string info;
  Dl_info di;
  int ver = 0;
  (void)hipRuntimeGetVersion(&ver);
  const char* path = dladdr((void*)&hipRuntimeGetVersion, &di) && di.dli_fname ? di.dli_fname : "?";
  info = std::string(path) + " hip_runtime_version=" + std::to_string(ver);
  return info.c_str();
}

// The matcher parameters of a config, as meili builds them: the
// "meili.default" section with the travel mode's own section on top
// ("meili.<mode>", mode = "meili.mode" or "auto", the mode reporter_service.py's
// matches run in: README.md:136).  A stock valhalla_build_config file has
// default.turn_penalty_factor 0 and auto.turn_penalty_factor 200 (SURVEY
// Appendix B), so an auto match runs with 200.
static bool read_meili(const Value& cfg, otm::MatchConfig* mc, std::string* err) {
  const Value* meili = cfg.get("meili");
  std::string mode = "auto";
  if (meili) {
    const Value* m = meili->get("mode");
    if (m && m->kind == Kind::Str) mode = m->s;
  }
  for (const char* sec : {"default", mode.c_str()}) {
    const Value* d = meili ? meili->get(sec) : nullptr;
    if (!d || d->kind != Kind::Obj) continue;
    auto getf = [&](const char* k, float* dst) {
      const Value* v = d->get(k);
      if (v && v->is_num()) *dst = (float)v->num();
    };
    getf("sigma_z", &mc->sigma_z);
    getf("beta", &mc->beta);
    getf("max_route_distance_factor", &mc->max_route_distance_factor);
    getf("breakage_distance", &mc->breakage_distance);
    getf("interpolation_distance", &mc->interpolation_distance);
    getf("search_radius", &mc->search_radius);
    getf("max_search_radius", &mc->max_search_radius);
    getf("gps_accuracy", &mc->gps_accuracy);
    getf("turn_penalty_factor", &mc->turn_penalty_factor);
    const Value* mk = d->get("max_candidates");
    if (mk && mk->kind == Kind::Int) mc->max_candidates = (int)mk->i;
  }
  if (!(mc->turn_penalty_factor >= 0.0f && mc->turn_penalty_factor <= 10000.0f)) {
    *err = "turn_penalty_factor must be in [0, 10000]";
    return false;
  }
  if (mc->max_candidates < 1 || mc->max_candidates > otm::KMAX) {
    *err = "max_candidates must be in [1, 32]";
    return false;
  }
  return true;
}

int otm_config_meili(const char* cfg_path, otm_meili_params* out) {
  if (!cfg_path || !out) return fail(OTM_EINVAL, "bad arguments");
  try {
    std::string text, perr;
    if (!read_file(cfg_path, &text)) return fail(OTM_EINVAL, std::string("cannot read config ") + cfg_path);
    Value cfg;
    if (!otm::json::parse(text, &cfg, &perr)) return fail(OTM_EINVAL, "config: " + perr);
    otm::MatchConfig mc;
    if (!read_meili(cfg, &mc, &perr)) return fail(OTM_EINVAL, perr);
    out->sigma_z = mc.sigma_z;
    out->beta = mc.beta;
    out->max_route_distance_factor = mc.max_route_distance_factor;
    out->breakage_distance = mc.breakage_distance;
    out->interpolation_distance = mc.interpolation_distance;
    out->search_radius = mc.search_radius;
    out->max_search_radius = mc.max_search_radius;
    out->gps_accuracy = mc.gps_accuracy;
    out->turn_penalty_factor = mc.turn_penalty_factor;
    out->max_candidates = mc.max_candidates;
    return OTM_OK;
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  }
}

static int otm_engine_create_impl(const char* cfg_path, const int* devices, int ndev, otm_engine** out) {
  if (!out) return fail(OTM_EINVAL, "out is NULL");
  *out = nullptr;
  if (ndev < 1 || !devices) return fail(OTM_EINVAL, "devices must name at least one device");
  if (ndev > 1) {
    // a multi-device engine: one member per device, each a full replica
    auto* G = new otm_engine();
    for (int i = 0; i < ndev; ++i) {
      otm_engine* M = nullptr;
      int rc = otm_engine_create(cfg_path, devices + i, 1, &M);
      if (rc) {
        const std::string msg = std::string("device ") + std::to_string(devices[i]) + ": " + otm_last_error(nullptr);
        for (otm_engine* m : G->members) otm_engine_destroy(m);
        delete G;
        return fail(rc, msg);
      }
      G->members.push_back(M);
    }
    const otm_engine* L = G->members[0];
    G->device = L->device;
    G->mc = L->mc;
    G->rc = L->rc;
    *out = G;
    return OTM_OK;
  }
  std::string text;
  if (!cfg_path || !read_file(cfg_path, &text)) return fail(OTM_EINVAL, std::string("cannot read config ") + (cfg_path ? cfg_path : "(null)"));
  Value cfg;
  std::string perr;
  if (!otm::json::parse(text, &cfg, &perr)) return fail(OTM_EINVAL, "config: " + perr);
  const Value* o = cfg.get("otm");
  const Value* gp = o ? o->get("graph") : nullptr;
  if (!gp || gp->kind != Kind::Str) return fail(OTM_EINVAL, "config: otm.graph (path) is required");
  std::string graph = gp->s;
  if (!graph.empty() && graph[0] != '/') {
    std::string c(cfg_path);
    const size_t sl = c.rfind('/');
    if (sl != std::string::npos) graph = c.substr(0, sl + 1) + graph;
  }
  auto* E = new otm_engine();
  const Value* ir = o->get("index_radius_m");
  if (ir && ir->is_num()) E->index_rmax = (float)ir->num();
  if (const char* er = std::getenv("OTM_INDEX_RADIUS")) E->index_rmax = (float)std::atof(er);  // A/B override
  // near index radii: a number or a list of numbers (0 or []: none)
  const Value* inr = o->get("index_near_m");
  if (inr && inr->is_num()) {
    E->index_near_set = true;
    E->index_near_m = {(float)inr->num()};
  } else if (inr && inr->kind == otm::json::Kind::Arr) {
    E->index_near_set = true;
    E->index_near_m.clear();
    for (const Value& v : inr->items)
      if (v.is_num()) E->index_near_m.push_back((float)v.num());
  }
  if (const char* en = std::getenv("OTM_INDEX_NEAR")) {  // A/B override: comma-separated metres (0: none)
    E->index_near_set = true;
    E->index_near_m.clear();
    for (const char* c = en; *c;) {
      char* end = nullptr;
      const float v = std::strtof(c, &end);
      if (end == c) break;
      E->index_near_m.push_back(v);
      c = *end == ',' ? end + 1 : end;
    }
  }
  const Value* gm = o->get("grid_mult");
  if (gm && gm->kind == Kind::Int) E->grid_mult = (int)gm->i;
  if (const char* v = std::getenv("OTM_GRID_MULT")) E->grid_mult = std::atoi(v);
  if (E->grid_mult < 0 || E->grid_mult > 64) {
    delete E;
    return fail(OTM_EINVAL, "grid_mult must be in [0 (auto), 64]");
  }
  const Value* tl = o->get("trans_lanes");
  if (tl && tl->kind == Kind::Int) E->trans_lanes = (int)tl->i;
  if (E->trans_lanes != 8 && E->trans_lanes != 16) {
    delete E;
    return fail(OTM_EINVAL, "trans_lanes must be 8 or 16");
  }
  std::string err;
  if (!read_meili(cfg, &E->mc, &err)) {
    delete E;
    return fail(OTM_EINVAL, err);
  }
  if (!otm::read_report_env(&E->rc, &err)) {
    delete E;
    return fail(OTM_ECONFIG, err);
  }
  if (!fill_device_params(E, &err)) {
    delete E;
    return fail(OTM_ECONFIG, err);
  }
  int rc = otm::engine_init(E, graph.c_str(), devices[0], &err);
  if (rc) {
    otm::engine_free(E);
    delete E;
    return fail(rc, err);
  }
  *out = E;
  return OTM_OK;
}

int otm_engine_clone(otm_engine* P, otm_engine** out) {
  if (!P || !out) return fail(OTM_EINVAL, "engine or out is NULL");
  *out = nullptr;
  if (P->parent) return fail(OTM_EINVAL, "clone the parent engine, not a clone");
  if (!P->members.empty()) return fail(OTM_EINVAL, "clone a member engine (otm_engine_member), not a multi-device engine");
  auto* C = new otm_engine();
  std::string err;
  int rc = otm::engine_clone(P, C, &err);
  if (rc) {
    otm::engine_free(C);
    delete C;
    return fail(rc, err);
  }
  *out = C;
  return OTM_OK;
}

void otm_engine_destroy(otm_engine* E) {
  if (!E) return;
  if (E->worker_started) {
    {
      std::lock_guard<std::mutex> lk(E->qmu);
      E->stop = true;
    }
    E->qcv.notify_all();
    for (auto& t : E->workers) t.join();  // (queued requests are finished first)
    for (auto& r : E->done) arena::free_body(r.body);
  }
  for (otm_engine* C : E->actx) otm_engine_destroy(C);
  for (otm_engine* C : E->awx) otm_engine_destroy(C);
  for (otm::H2DOrder* o : {&E->aorder, &E->split_order}) {
    for (hipEvent_t ev : o->ev)
      if (ev) (void)hipEventDestroy(ev);
    if (o->copy) (void)hipStreamDestroy(o->copy);
  }
  if (!E->members.empty()) {
    otm::member_pool_free(E);
    for (otm_engine* m : E->members) otm_engine_destroy(m);
    delete E;
    return;
  }
  otm::engine_free(E);
  delete E;
}

int otm_engine_members(const otm_engine* E) { return !E ? 0 : E->members.empty() ? 1 : (int)E->members.size(); }

otm_engine* otm_engine_member(otm_engine* E, int i) {
  if (!E || i < 0) return nullptr;
  if (E->members.empty()) return i == 0 ? E : nullptr;
  return i < (int)E->members.size() ? E->members[(size_t)i] : nullptr;
}

static int otm_report_impl(otm_engine* E, const char* req, size_t len, char** resp, size_t* resp_len) {
  if (!E || !resp || (!req && len)) return fail(OTM_EINVAL, "bad arguments");
  int code = 0;
  const char* reqs[1] = {req};
  report_many(E, 1, reqs, &len, &code, resp, resp_len);
  return code;
}

static int otm_report_batch_impl(otm_engine* E, int n, const char* const* reqs, const size_t* lens, char** resps,
                     size_t* resp_lens, int* codes) {
  if (!E || n < 0) return fail(OTM_EINVAL, "bad arguments");
  // bodies in a request arena go to HBM straight from it
  std::vector<std::shared_ptr<ReqSlab>> held;
  reqarena::find(n, reqs, lens, &held);
  std::vector<const void*> pin((size_t)n, nullptr);
  bool any = false;
  for (int k = 0; k < n; ++k) {
    pin[(size_t)k] = held[(size_t)k].get();
    any = any || pin[(size_t)k];
  }
  report_many_split(E, n, reqs, lens, codes, resps, resp_lens, any ? pin.data() : nullptr);
  return OTM_OK;
}

int otm_request_points(const char* req, size_t len, int fast, float* lat, float* lon, double* time, float* acc,
                       int max_points, char* uuid, size_t uuid_cap) {
  if (!req) return fail(OTM_EINVAL, "req is NULL");
  otm::TracePoints tp;
  std::string u;
  bool have_uuid = false;
  if (fast) {
    if (!otm::fast_request(std::string_view(req, len), &tp, &u)) return -2;
    have_uuid = true;
  } else {
    Value dom;
    std::string resp, err;
    if (otm::parse_request("/report", std::string_view(req, len), &dom, &resp)) return -1;
    if (!otm::extract_points(dom, &tp, &err)) return -1;
    const Value* uv = dom.get("uuid");
    if (uv && uv->kind == Kind::Str) {
      u = uv->s;
      have_uuid = true;
    }
  }
  const int n = (int)tp.lat.size();
  for (int k = 0; k < n && k < max_points; ++k) {
    if (lat) lat[k] = tp.lat[(size_t)k];
    if (lon) lon[k] = tp.lon[(size_t)k];
    if (time) time[k] = tp.time[(size_t)k];
    if (acc) acc[k] = tp.acc[(size_t)k];
  }
  if (uuid && uuid_cap) {
    const size_t m = have_uuid ? std::min(u.size(), uuid_cap - 1) : 0;
    std::memcpy(uuid, u.data(), m);
    uuid[m] = 0;
  }
  return n;
}

static int otm_match_json_impl(otm_engine* E, const char* req, size_t len, char** resp, size_t* resp_len) {
  if (!E || !resp || (!req && len)) return fail(OTM_EINVAL, "bad arguments");
  std::vector<Req> rq(1);
  std::vector<int> codes(1, 0);
  std::vector<std::string> bodies(1);
  std::string perr;
  if (!otm::json::parse(std::string_view(req, len), &rq[0].dom, &perr)) {
    *resp = dup_out(otm::error_body(perr), resp_len);
    return 500;
  }
  if (rq[0].dom.kind != Kind::Obj) {
    *resp = dup_out(otm::error_body("request must be a JSON object"), resp_len);
    return 500;
  }
  run_requests(E, rq, codes, bodies, {0}, true);
  *resp = dup_out(bodies[0], resp_len);
  return codes[0];
}

int otm_report_segments(otm_engine* E, const char* req, size_t len, const char* match_json, size_t match_len,
                        char** resp, size_t* resp_len) {
  otm::ReportConfig rc;
  if (E) {
    rc = E->rc;
  } else {
    std::string err;
    if (!otm::read_report_env(&rc, &err)) {
      *resp = dup_out(otm::error_body(err), resp_len);
      return 500;
    }
  }
  Value trace;
  std::string body;
  int code = otm::parse_request("/report", std::string_view(req, len), &trace, &body);
  if (code) {
    *resp = dup_out(body, resp_len);
    return code;
  }
  Value segs;
  std::string perr;
  if (!otm::json::parse(std::string_view(match_json, match_len), &segs, &perr)) {
    *resp = dup_out(otm::error_body(perr), resp_len);
    return 500;
  }
  std::string out, errtext, exc;
  if (!otm::report_dom(rc, trace, &segs, &out, &errtext, &exc)) {
    *resp = dup_out(otm::error_body(exc), resp_len);
    return 500;
  }
  if (!errtext.empty()) std::fputs(errtext.c_str(), stderr);
  *resp = dup_out(out, resp_len);
  return 200;
}

static int otm_report_segments_device_impl(otm_engine* E, int n, const char* const* reqs, const size_t* lens,
                               const char* const* match_jsons, const size_t* match_lens, char** resps,
                               size_t* resp_lens, int* codes) {
  if (!E || n < 0) return fail(OTM_EINVAL, "bad arguments");
  if (!E->members.empty()) E = E->members[0];  // no per-uuid state: the first member's GPU
  std::vector<std::string> bodies((size_t)n), matcher((size_t)n);
  std::vector<int> c((size_t)n, 0);
  // the typed traces: one point each (the request's last time), their segments
  std::vector<int64_t> toff(1, 0);
  std::vector<double> tend;
  std::vector<int32_t> soff(1, 0);
  std::vector<otm_segment> segs;
  std::vector<int> which;
  for (int k = 0; k < n; ++k) {
    Value trace;
    int code = otm::parse_request("/report", std::string_view(reqs[k], lens[k]), &trace, &bodies[(size_t)k]);
    if (code) {
      c[(size_t)k] = code;
      continue;
    }
    Value m;
    std::string perr;
    if (!otm::json::parse(std::string_view(match_jsons[k], match_lens[k]), &m, &perr)) {
      c[(size_t)k] = 500;
      bodies[(size_t)k] = otm::error_body(perr);
      continue;
    }
    std::vector<otm_segment> ts;
    double et = 0.0;
    std::string why;
    if (!otm::typed_segments(trace, m, &ts, &et, &why)) {
      bodies[(size_t)k] = "not typed: " + why;  // code 0
      continue;
    }
    if (m.kind == Kind::Obj) {
      Value mode;
      mode.kind = Kind::Str;
      mode.s = "auto";
      m.set("mode", std::move(mode));  // segments['mode'] = 'auto' (reporter_service.py:131)
    }
    otm::json::dump(m, &matcher[(size_t)k]);
    segs.insert(segs.end(), ts.begin(), ts.end());
    soff.push_back((int32_t)segs.size());
    tend.push_back(et);
    toff.push_back((int64_t)tend.size());
    which.push_back(k);
  }
  if (!which.empty()) {
    const int32_t T = (int32_t)which.size();
    std::vector<otm_trace_result> tr((size_t)T);
    std::vector<otm_report_rec> rep(segs.size() + 1);
    std::string err;
    int rc;
    {
      std::lock_guard<std::mutex> lk(E->mu);
      (void)hipSetDevice(E->device);
      rc = otm::engine_report_segments(E, T, toff.data(), tend.data(), soff.data(), segs.data(), tr.data(),
                                       rep.data(), &err);
    }
    if (rc) return fail(rc, err);
    otm_results r{};
    r.n_traces = T;
    r.n_segments = (int32_t)segs.size();
    r.traces = tr.data();
    r.segments = segs.data();
    r.reports = rep.data();
    for (int32_t t = 0; t < T; ++t) {
      const int k = which[(size_t)t];
      std::string out;
      c[(size_t)k] = otm::write_report_response(r, t, &out, &matcher[(size_t)k]);
      bodies[(size_t)k] = std::move(out);
      const int inv = tr[(size_t)t].code == 200 ? tr[(size_t)t].invalid_speeds : 0;
      speed_lines(inv);
    }
  }
  for (int k = 0; k < n; ++k) {
    codes[k] = c[(size_t)k];
    resps[k] = dup_out(bodies[(size_t)k], &resp_lens[k]);
  }
  return OTM_OK;
}

static int otm_submit_impl(otm_engine* E, const char* req, size_t len, uint64_t tag) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  std::lock_guard<std::mutex> lk(E->qmu);
  if (!E->worker_started) start_workers(E);
  if (E->queue.size() >= (1u << 22)) return fail(OTM_EAGAIN, "submit queue full");
  std::shared_ptr<ReqSlab> slab = slabs::acquire(len);
  if (len) std::memcpy(slab->base, req, len);
  E->queue.push_back(otm_engine::Pending{tag, slab->base, len, std::move(slab), 1, E->n_subs++});
  E->qcv.notify_all();
  return OTM_OK;
}

static int otm_submit_batch_impl(otm_engine* E, int n, const char* const* reqs, const size_t* lens,
                                 const uint64_t* tags) {
  if (!E || n < 0 || (n && (!reqs || !lens || !tags))) return fail(OTM_EINVAL, "bad arguments");
  // the bodies copied into one slab (page-locked when large), outside the
  // queue lock, over the host threads; a submission beyond SLAB_MAX bytes
  // gets an allocation per body instead (page-locking that much per
  // submission costs more than the staging copy it saves)
  std::vector<size_t> off((size_t)n + 1, 0);
  for (int k = 0; k < n; ++k) off[(size_t)k + 1] = off[(size_t)k] + lens[k];
  std::vector<std::shared_ptr<ReqSlab>> held;
  if (n && reqarena::find(n, reqs, lens, &held)) {
    // every body in a request arena: the submission holds the arenas (a
    // shared count per body, taken on this thread), nothing is copied
    std::vector<otm_engine::Pending> items((size_t)n);
    for (size_t k = 0; k < (size_t)n; ++k)
      items[k] = otm_engine::Pending{tags[k], reqs[k], lens[k], std::move(held[k]), (size_t)n - k, 0};
    {
      std::lock_guard<std::mutex> lk(E->qmu);
      if (!E->worker_started) start_workers(E);
      if (E->queue.size() + (size_t)n > (1u << 22)) return fail(OTM_EAGAIN, "submit queue full");
      const uint64_t sub = E->n_subs++;
      for (auto& it : items) {
        it.sub = sub;
        E->queue.push_back(std::move(it));
      }
    }
    E->qcv.notify_all();
    return OTM_OK;
  }
  const char* mx = std::getenv("OTM_SLAB_MAX");  // (tests lower it)
  const bool one = off[(size_t)n] <= (mx ? (size_t)std::strtoull(mx, nullptr, 10) : slabs::SLAB_MAX);
  std::shared_ptr<ReqSlab> slab = one ? slabs::acquire(off[(size_t)n]) : nullptr;
  std::vector<otm_engine::Pending> items((size_t)n);
  if (one) {
    // the copies over the host threads; the slab's references taken on this
    // thread after (one shared count: no cross-thread contention on it)
    par_for((size_t)n, [&](size_t a, size_t e) {
      for (size_t k = a; k < e; ++k)
        if (lens[k]) std::memcpy(slab->base + off[k], reqs[k], lens[k]);
    });
    for (size_t k = 0; k < (size_t)n; ++k)
      items[k] = otm_engine::Pending{tags[k], slab->base + off[k], lens[k], slab, (size_t)n - k, 0};
  } else {
    par_for((size_t)n, [&](size_t a, size_t e) {
      for (size_t k = a; k < e; ++k) {
        std::shared_ptr<ReqSlab> s = slabs::acquire(lens[k], false);
        char* p = s->base;
        if (lens[k]) std::memcpy(p, reqs[k], lens[k]);
        items[k] = otm_engine::Pending{tags[k], p, lens[k], std::move(s), (size_t)n - k, 0};
      }
    });
  }
  {
    std::lock_guard<std::mutex> lk(E->qmu);
    if (!E->worker_started) start_workers(E);
    if (E->queue.size() + (size_t)n > (1u << 22)) return fail(OTM_EAGAIN, "submit queue full");
    const uint64_t sub = E->n_subs++;
    for (auto& it : items) {
      it.sub = sub;
      E->queue.push_back(std::move(it));
    }
  }
  E->qcv.notify_all();
  return OTM_OK;
}

int otm_poll(otm_engine* E, otm_result* out, int max, int timeout_us) {
  if (!E || max < 0) return fail(OTM_EINVAL, "bad arguments");
  std::unique_lock<std::mutex> lk(E->qmu);
  if (E->done.empty() && timeout_us > 0)
    E->qcv.wait_for(lk, std::chrono::microseconds(timeout_us), [&] { return !E->done.empty(); });
  int n = 0;
  while (n < max && !E->done.empty()) {
    out[n++] = E->done.front();
    E->done.pop_front();
  }
  return n;
}

int otm_encode_request(const char* uuid, int n, const float* lat, const float* lon, const int64_t* time,
                       const int32_t* accuracy, char** out, size_t* out_len) {
  if (!uuid || n < 0 || !out || (n > 0 && (!lat || !lon || !time || !accuracy))) return fail(OTM_EINVAL, "bad arguments");
  // Batch.java:52-61 + Point.java:39-45, then StringEntity's ISO-8859-1
  // (HttpClient.java:26): the uuid is the record key, given here as UTF-8
  std::string s;
  otm::encode_request(otm::jstr::key_on_wire(uuid), n, lat, lon, time, accuracy, &s);
  *out = dup_out(s, out_len);
  return OTM_OK;
}

void* otm_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault) != hipSuccess) {
    fail(OTM_ENOMEM, "hipHostMalloc failed");
    return nullptr;
  }
  return p;
}

void otm_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

static int otm_match_soa_impl(otm_engine* E, const otm_batch* in, otm_results* out) {
  if (!E || !in || !out) return fail(OTM_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(E->mu);
  std::string err;
  int rc = otm::match_host_fetch(E, in, nullptr, out, &err);
  return rc ? fail(rc, err) : OTM_OK;
}

static int otm_match_compact_impl(otm_engine* E, const otm_batch_compact* in, otm_results* out) {
  if (!E || !in || !out) return fail(OTM_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(E->mu);
  std::string err;
  int rc;
  if (E->members.empty()) {
    (void)hipSetDevice(E->device);
    rc = otm::engine_match_compact(E, in, &err);
    if (!rc) rc = otm::engine_fetch(E, out, &err);
  } else {
    // a multi-device engine splits the batch on the host: widened there,
    // after the same checks as one engine's
    const int32_t nt = in->n_traces;
    int64_t np = 0;
    if ((rc = otm::validate_compact(in, &np, &err))) return fail(rc, err);
    std::vector<double> tm((size_t)np);
    std::vector<float> acc((size_t)np);
    for (int32_t t = 0; t < nt; ++t)
      for (int64_t i = in->trace_off[t]; i < in->trace_off[t + 1]; ++i)
        tm[(size_t)i] = (double)(in->time_base[t] + (int64_t)in->time_delta[i]);
    for (int64_t i = 0; i < np; ++i) acc[(size_t)i] = (float)in->accuracy[i];
    const otm_batch b{nt, np, in->trace_off, in->lat, in->lon, tm.data(), acc.data()};
    rc = otm::match_host_fetch(E, &b, nullptr, out, &err);
  }
  return rc ? fail(rc, err) : OTM_OK;
}

static int otm_match_device_impl(otm_engine* E, const otm_batch* in, void* stream) {
  if (!E || !in) return fail(OTM_EINVAL, "bad arguments");
  if (!E->members.empty()) return fail(OTM_EINVAL, "device batches go to a member engine (otm_engine_member)");
  std::lock_guard<std::mutex> lk(E->mu);
  (void)hipSetDevice(E->device);
  otm::DevBatch b;
  b.n_traces = in->n_traces;
  b.n_points = in->n_points;
  b.trace_off = in->trace_off;
  b.lat = in->lat;
  b.lon = in->lon;
  b.time = in->time;
  b.acc = in->accuracy;
  std::string err;
  E->spin_waits = true;  // (wait_batch: the caller's threads drive the GPU)
  int rc = otm::engine_match(E, b, (hipStream_t)stream, &err);
  E->spin_waits = false;
  return rc ? fail(rc, err) : OTM_OK;
}

static int otm_fetch_results_impl(otm_engine* E, otm_results* out) {
  if (!E || !out) return fail(OTM_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(E->mu);
  if (!E->members.empty()) {
    // the merged results of the group's last batch
    out->n_traces = (int32_t)E->g_traces.size();
    out->n_segments = (int32_t)E->g_segs.size();
    out->n_reports = (int32_t)E->g_reps.size();
    out->n_way_ids = (int32_t)E->g_ways.size();
    out->traces = E->g_traces.data();
    out->segments = E->g_segs.data();
    out->reports = E->g_reps.data();
    out->way_ids = E->g_ways.data();
    return OTM_OK;
  }
  std::string err;
  int rc = otm::engine_fetch(E, out, &err);
  return rc ? fail(rc, err) : OTM_OK;
}

int otm_hist_bind_ex(otm_engine* E, void* dev_counts, int nbins, float bin_kph, void* dev_speed_sum) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  if (E->parent) return fail(OTM_EINVAL, "bind the histogram on the parent engine (clones share it)");
  if (!E->members.empty()) return fail(OTM_EINVAL, "bind one histogram per member engine (otm_engine_member)");
  if (dev_counts && (nbins < 1 || !(bin_kph > 0.0f))) return fail(OTM_EINVAL, "nbins >= 1 and bin_kph > 0");
  if (dev_speed_sum && !dev_counts) return fail(OTM_EINVAL, "a speed-sum channel needs the counts");
  // a batch in flight on this engine or a clone keeps the binding it started with
  std::lock_guard<std::mutex> lk(E->hist_mu);
  E->hist = (uint32_t*)dev_counts;
  E->speed_sum = dev_counts ? (unsigned long long*)dev_speed_sum : nullptr;
  E->nbins = dev_counts ? nbins : 0;
  E->bin_kph = bin_kph;
  return OTM_OK;
}

int otm_hist_bind(otm_engine* E, void* dev_counts, int nbins, float bin_kph) {
  return otm_hist_bind_ex(E, dev_counts, nbins, bin_kph, nullptr);
}

int otm_graph_info(const otm_engine* E, int64_t* n_nodes, int64_t* n_edges, int64_t* n_segments) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  if (!E->members.empty()) E = E->members[0];  // every member holds the same graph
  if (n_nodes) *n_nodes = E->host.h.n_nodes;
  if (n_edges) *n_edges = E->host.h.n_edges;
  if (n_segments) *n_segments = E->host.h.n_segments;
  return OTM_OK;
}

int otm_index_info(const otm_engine* E, float* rmax, int64_t* entries, int32_t* incomplete_rows, float* build_ms) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  if (!E->members.empty()) E = E->members[0];  // every member holds the same graph
  if (rmax) *rmax = E->idx.rmax;
  if (entries) *entries = E->index_entries;
  if (incomplete_rows) *incomplete_rows = E->index_incomplete_rows;
  if (build_ms) *build_ms = E->index_build_ms;
  return OTM_OK;
}

int otm_index_tables(const otm_engine* E, int64_t* slots, int64_t* bytes, int32_t* load_pct) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  if (!E->members.empty()) E = E->members[0];
  const int64_t n = E->index_slots + E->index_near_slots;
  if (slots) *slots = n;
  if (bytes) *bytes = n * otm::IDX_SLOT_BYTES;
  if (load_pct) *load_pct = E->idx.rmax > 0.0f ? E->idx.load_pct : 0;
  return OTM_OK;
}

int otm_index_levels(const otm_engine* E, float* radii, int64_t* entries, int cap) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  if (!E->members.empty()) E = E->members[0];
  int n = 0;
  for (int l = 0; l < otm::NEAR_LEVELS; ++l) {
    if (!(E->idxn[l].rmax > 0.0f)) continue;
    if (n < cap) {
      if (radii) radii[n] = E->idxn[l].rmax;
      if (entries) entries[n] = E->index_near_level_entries[l];
    }
    ++n;
  }
  return n;
}

int otm_grid_info(const otm_engine* E, double* cell_deg, int32_t* rows, int32_t* cols, int64_t* entries,
                  int32_t* mult) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  if (!E->members.empty()) E = E->members[0];  // every member holds the same graph
  if (cell_deg) *cell_deg = E->g.cell;
  if (rows) *rows = E->grid_rows;
  if (cols) *cols = E->grid_cols;
  if (entries) *entries = E->grid_entries;
  if (mult) *mult = E->grid_mult;
  return OTM_OK;
}

int otm_set_counting(otm_engine* E, int on) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  for (otm_engine* m : E->members) m->counting = on != 0;
  E->counting = on != 0;
  return OTM_OK;
}

int otm_get_counters(otm_engine* E, otm_work_counters* out) {
  if (!E || !out) return fail(OTM_EINVAL, "bad arguments");
  if (!E->members.empty()) E = E->members[0];  // the first member (others: otm_engine_member)
  std::lock_guard<std::mutex> lk(E->mu);
  return otm::engine_counters(E, out) ? fail(OTM_EDEVICE, "counter copy failed") : OTM_OK;
}

int otm_set_timing(otm_engine* E, int on) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  for (otm_engine* m : E->members) m->timing = on != 0;
  E->timing = on != 0;
  return OTM_OK;
}

int otm_get_stage_ms(otm_engine* E, float* ms, int n) {
  if (!E || !ms) return fail(OTM_EINVAL, "bad arguments");
  if (!E->members.empty()) E = E->members[0];  // the first member (others: otm_engine_member)
  for (int k = 0; k < n && k < 8; ++k) ms[k] = E->stage_ms[k];
  return OTM_OK;
}

int otm_get_kernel_ms(otm_engine* E, float* ms, int n) {
  if (!E || !ms) return fail(OTM_EINVAL, "bad arguments");
  if (!E->members.empty()) E = E->members[0];  // the first member (others: otm_engine_member)
  for (int k = 0; k < n && k < otm::KN_COUNT; ++k) ms[k] = E->kernel_ms[k];
  return OTM_OK;
}

static_assert(OTM_NUM_KERNELS == otm::KN_COUNT, "kernel table");
const char* otm_kernel_name(int k) { return k >= 0 && k < otm::KN_COUNT ? otm::kKernelNames[k] : nullptr; }

int otm_get_spill_stats(otm_engine* E, otm_spill_stats* out) {
  if (!E || !out) return fail(OTM_EINVAL, "bad arguments");
  if (!E->members.empty()) E = E->members[0];  // the first member (others: otm_engine_member)
  std::lock_guard<std::mutex> lk(E->mu);
  return otm::engine_spill_stats(E, out) ? fail(OTM_EDEVICE, "spill stats copy failed") : OTM_OK;
}

int otm_debug_fetch(otm_engine* E, int what, void* dst, size_t bytes, size_t* needed) {
  if (!E) return fail(OTM_EINVAL, "engine is NULL");
  if (!E->members.empty()) E = E->members[0];  // the first member (others: otm_engine_member)
  std::lock_guard<std::mutex> lk(E->mu);
  std::string err;
  int rc = otm::engine_debug_fetch(E, what, dst, bytes, needed, &err);
  return rc ? fail(rc, err) : OTM_OK;
}

// Entry points: nothing throws across the C ABI (an allocation failure or an
// internal exception becomes an error code, or a 500 body).
int otm_engine_create(const char* cfg_path, const int* devices, int ndev, otm_engine** out) {
  try {
    return otm_engine_create_impl(cfg_path, devices, ndev, out);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_report_batch(otm_engine* E, int n, const char* const* reqs, const size_t* lens, char** resps,
                     size_t* resp_lens, int* codes) {
  try {
    return otm_report_batch_impl(E, n, reqs, lens, resps, resp_lens, codes);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_report_segments_device(otm_engine* E, int n, const char* const* reqs, const size_t* lens,
                               const char* const* match_jsons, const size_t* match_lens, char** resps,
                               size_t* resp_lens, int* codes) {
  try {
    return otm_report_segments_device_impl(E, n, reqs, lens, match_jsons, match_lens, resps, resp_lens, codes);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_submit(otm_engine* E, const char* req, size_t len, uint64_t tag) {
  try {
    return otm_submit_impl(E, req, len, tag);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_submit_batch(otm_engine* E, int n, const char* const* reqs, const size_t* lens, const uint64_t* tags) {
  try {
    return otm_submit_batch_impl(E, n, reqs, lens, tags);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_match_soa(otm_engine* E, const otm_batch* in, otm_results* out) {
  try {
    return otm_match_soa_impl(E, in, out);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_match_compact(otm_engine* E, const otm_batch_compact* in, otm_results* out) {
  try {
    return otm_match_compact_impl(E, in, out);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_match_device(otm_engine* E, const otm_batch* in, void* stream) {
  try {
    return otm_match_device_impl(E, in, stream);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_fetch_results(otm_engine* E, otm_results* out) {
  try {
    return otm_fetch_results_impl(E, out);
  } catch (const std::bad_alloc&) {
    return fail(OTM_ENOMEM, "out of host memory");
  } catch (const std::exception& e) {
    return fail(OTM_EINVAL, std::string("internal error: ") + e.what());
  }
}

int otm_report(otm_engine* E, const char* req, size_t len, char** resp, size_t* resp_len) {
  try {
    return otm_report_impl(E, req, len, resp, resp_len);
  } catch (...) {
    // a 500 like :239-240, its body allocated without anything that throws
    static const char kBody[] = "{\"error\":\"internal error\"}";
    char* b = (char*)std::malloc(sizeof kBody);
    if (b) std::memcpy(b, kBody, sizeof kBody);
    if (resp) *resp = b;
    if (resp_len) *resp_len = b ? sizeof kBody - 1 : 0;
    return 500;
  }
}

int otm_match_json(otm_engine* E, const char* req, size_t len, char** resp, size_t* resp_len) {
  try {
    return otm_match_json_impl(E, req, len, resp, resp_len);
  } catch (...) {
    // a 500 like :239-240, its body allocated without anything that throws
    static const char kBody[] = "{\"error\":\"internal error\"}";
    char* b = (char*)std::malloc(sizeof kBody);
    if (b) std::memcpy(b, kBody, sizeof kBody);
    if (resp) *resp = b;
    if (resp_len) *resp_len = b ? sizeof kBody - 1 : 0;
    return 500;
  }
}

}  // extern "C"
