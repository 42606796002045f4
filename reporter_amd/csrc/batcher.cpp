// batcher.cpp -- native restatement of the reference's Kafka Streams batcher
// (BASELINE config 5), driving the matcher in GPU batches.
//
// What it restates (reference = burritojustice/reporter):
//   Batch            src/main/java/org/opentraffic/reporter/Batch.java:16-84
//     distance       :31-38   equirectangular, float lat/lon, double math
//     update         :40-44   max_separation = (float)max(.., distance(p, first))
//     report         :46-84   gates, request bytes (Point.java:39-45), POST,
//                             trim by findValue("shape_used"), clear on error
//   BatchingProcessor src/main/java/org/opentraffic/reporter/BatchingProcessor.java
//     constants      :28-31   REPORT_TIME 60 s, REPORT_COUNT 10, REPORT_DIST 500 m, SESSION_GAP 60000 ms
//     process        :56-85   clean(key); store.delete; new Batch | update + report -> forward;
//                             put back if non-empty
//     clean          :87-112  pop keys idle > SESSION_GAP (by record timestamp), report(k, 0, 2, 0);
//                             time_to_key.remove(iter) removes nothing (a ListIterator is never equal
//                             to a Pair), so EVERY record's entry expires 60 s later and triggers a
//                             relaxed report of its key; a popped key with no stored batch makes
//                             store.get return null and the reference throws (NPE, stream thread
//                             dies) -- here it is counted (null_batch_in_clean) and skipped
//     close          :120-130 relaxed report of every stored batch, keys in TreeMap order
//
// Serial semantics, batched execution: a key's operations (its records'
// process() and the clean()/close() reports that name it) run in exactly the
// serial order, but a key waiting for a match does not hold up the others.
// Which keys clean() pops depends only on record timestamps (the time_to_key
// list never changes on a response), so the operation list of every key is
// known when its records arrive.  Requests of all runnable keys go to the
// matcher together: one GPU batch per round.
#include <algorithm>
#include <exception>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <memory>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "engine.h"
#include "javastr.h"
#include "json.h"
#include "report.h"

namespace {

using otm::json::Kind;
using otm::json::Value;

struct JPoint {  // Point.java:15-17
  float lat, lon;
  int32_t acc;
  int64_t time;
};

struct JBatch {  // Batch.java:18-19
  float max_sep = 0.0f;
  std::vector<JPoint> pts;
};

const double kRadPerDeg = 3.14159265358979323846 / 180.0;  // Math.PI / 180.0
const double kMetersPerDeg = 20037581.187 / 180.0;

// Batch.distance (Batch.java:34-38), Java evaluation order: float lon/lat
// differences and .5f * (lat_a + lat_b) in float, the rest in double.
double jdistance(const JPoint& a, const JPoint& b) {
  const float dlon = a.lon - b.lon;
  const float mlat = 0.5f * (a.lat + b.lat);
  const double x = (double)dlon * kMetersPerDeg * std::cos((double)mlat * kRadPerDeg);
  const double y = (double)(float)(a.lat - b.lat) * kMetersPerDeg;
  return std::sqrt(x * x + y * y);
}

void jupdate(JBatch& b, const JPoint& p) {  // Batch.update
  if (!b.pts.empty()) b.max_sep = (float)std::max((double)b.max_sep, jdistance(p, b.pts[0]));
  b.pts.push_back(p);
}

bool jgates(const JBatch& b, int min_dist, int min_size, int64_t min_elapsed) {  // Batch.java:48-50
  if (b.max_sep < (float)min_dist) return false;
  if ((int64_t)b.pts.size() < min_size) return false;
  return !(b.pts.back().time - b.pts.front().time < min_elapsed);
}

// Jackson JsonNode.findValue: depth-first, a node's own fields before their
// children, in field order.
const Value* find_value(const Value& v, const std::string& name) {
  if (v.kind == Kind::Obj) {
    for (size_t k = 0; k < v.keys.size(); ++k)
      if (v.keys[k] == name) return &v.items[k];
    for (const Value& c : v.items)
      if (const Value* r = find_value(c, name)) return r;
  } else if (v.kind == Kind::Arr) {
    for (const Value& c : v.items)
      if (const Value* r = find_value(c, name)) return r;
  }
  return nullptr;
}

// Batch.java:64-81 after the POST: trim_to = shape_used or everything; any
// exception (unparsable body, out-of-range trim) clears the batch.
void japply(JBatch& b, int trim_to_or_neg) {
  const int64_t n = (int64_t)b.pts.size();
  const int64_t trim = trim_to_or_neg < 0 ? n : trim_to_or_neg;
  if (trim > n) {  // subList IndexOutOfBoundsException -> catch
    b.max_sep = 0.0f;
    b.pts.clear();
    return;
  }
  b.pts.erase(b.pts.begin(), b.pts.begin() + trim);
  b.max_sep = 0.0f;
  for (size_t i = 1; i < b.pts.size(); ++i)
    b.max_sep = (float)std::max((double)b.max_sep, jdistance(b.pts[i], b.pts[0]));
}

// trim target of a response body, as Batch.report parses it: -1 = findValue
// returned null (trim all); -2 = the body did not parse (clear)
int parse_trim(const char* body, size_t len) {
  Value v;
  std::string err;
  if (!body || !otm::json::parse(std::string_view(body, len), &v, &err)) return -2;
  const Value* su = find_value(v, "shape_used");
  if (!su) return -1;
  if (su->kind == Kind::Int && !su->bigint) return su->i < 0 ? -2 : (int)std::min<int64_t>(su->i, INT32_MAX);
  if (su->kind == Kind::Float) return su->f < 0 ? -2 : (int)su->f;  // JsonNode.intValue truncates
  return 0;  // non-numeric node: intValue() is 0
}

enum OpKind : uint8_t { OP_PROCESS = 0, OP_CLEAN = 1, OP_CLOSE = 2 };
struct Op {
  uint32_t key;
  OpKind kind;
  JPoint pt;
  int64_t seq;  // stream position of the record (forward order)
};

struct KeyState {
  std::string key;   // the key as StringSerializer writes it (javastr.h kafka_key)
  std::string wire;  // the key inside the /report body as HttpClient sends it (ISO-8859-1)
  bool plain = true; // that body parses as the binary path reads it (javastr.h wire_key_plain)
  JBatch batch;
  bool in_store = false;
  uint32_t ob = 0, oe = 0;  // pending operations: otm_batcher::ops[ob, oe)
  bool waiting = false;
  bool queued = false;  // in the run queue
  Op wop{};             // the op whose request is outstanding
};

struct Request {
  uint32_t key;
  std::string body;  // filled on the JSON path
  int npts;
};

// A fixed team of host threads for the per-key phases of a round (the
// caller is member 0).  run(n, fn) calls fn(member, begin, end) over [0, n)
// in contiguous chunks, one per member, and returns when all are done.
class Pool {
 public:
  explicit Pool(int n) : n_(n < 1 ? 1 : n) {
    for (int t = 1; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }
  void run(size_t n, const std::function<void(int, size_t, size_t)>& fn) {
    if (n_ == 1 || n < 2) {
      fn(0, 0, n);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_items_ = n;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    try {
      chunk(0, n, fn);
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu_);
      if (!err_) err_ = std::current_exception();
    }
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
    if (err_) {  // a member's exception, to the entry point's guard
      std::exception_ptr e = err_;
      err_ = nullptr;
      lk.unlock();
      std::rethrow_exception(e);
    }
  }

 private:
  void chunk(int t, size_t n, const std::function<void(int, size_t, size_t)>& fn) const {
    const size_t per = (n + (size_t)n_ - 1) / (size_t)n_;
    const size_t a = std::min(n, (size_t)t * per), e = std::min(n, a + per);
    fn(t, a, e);
  }
  void loop(int t) {
    uint64_t seen = 0;
    while (true) {
      const std::function<void(int, size_t, size_t)>* fn;
      size_t n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
        n = n_items_;
      }
      try {
        chunk(t, n, *fn);
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err_) err_ = std::current_exception();
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (--pending_ == 0) done_.notify_one();
      }
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::exception_ptr err_;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  uint64_t gen_ = 0;
  bool stop_ = false;
  const std::function<void(int, size_t, size_t)>* fn_ = nullptr;
  size_t n_items_ = 0;
  int pending_ = 0;
};

// What one member of the pool produces while applying responses
struct Sink {
  std::vector<Request> reqs;
  std::vector<otm_forward> out;
  std::vector<uint32_t> runq;
  int64_t nulls = 0, forwarded = 0;
  void clear() {
    reqs.clear();
    out.clear();
    runq.clear();
    nulls = forwarded = 0;
  }
};

}  // namespace

struct otm_batcher {
  otm_engine* eng = nullptr;
  otm_batcher_cfg cfg{};
  otm_report_fn fn = nullptr;
  void* ctx = nullptr;
  std::deque<std::string> key_text;                    // stable storage behind the index's views
  std::unordered_map<std::string_view, uint32_t> index;  // record key -> keys[]
  std::vector<KeyState> keys;
  std::deque<std::pair<int64_t, uint32_t>> time_to_key;  // BatchingProcessor.time_to_key
  int64_t seq = 0;
  std::vector<Op> log;       // operations in stream order since the last drain
  std::vector<Op> ops;       // ... grouped by key (stable), each key's range in KeyState
  std::vector<uint32_t> cnt;
  std::vector<uint32_t> runq;
  std::vector<Request> reqs;
  std::deque<otm_forward> out;
  otm_batcher_stats st{};
  std::string err;
  std::unique_ptr<Pool> pool;  // cfg.threads > 1
  std::vector<Sink> sinks;     // one per pool member
};

namespace {

// k: a canonical key (kafka_key applied)
uint32_t key_id(otm_batcher* B, const char* k, size_t n) {
  auto it = B->index.find(std::string_view(k, n));
  if (it != B->index.end()) return it->second;
  const uint32_t id = (uint32_t)B->keys.size();
  B->key_text.emplace_back(k, n);
  B->keys.emplace_back();
  KeyState& ks = B->keys.back();
  ks.key = B->key_text.back();
  ks.wire = otm::jstr::key_on_wire(ks.key);
  ks.plain = otm::jstr::wire_key_plain(ks.wire);
  B->index.emplace(std::string_view(B->key_text.back()), id);
  return id;
}

void enqueue(otm_batcher* B, uint32_t k, const Op& op) {
  B->log.push_back(op);
  B->log.back().key = k;
}

// Group the log by key (a stable counting sort: each key's operations stay in
// stream order, after any it still had pending) and queue every key that can run.
void distribute(otm_batcher* B) {
  const size_t nk = B->keys.size();
  B->cnt.assign(nk + 1, 0);
  size_t total = B->log.size();
  for (size_t k = 0; k < nk; ++k) {
    const KeyState& ks = B->keys[k];
    B->cnt[k] = ks.oe - ks.ob;
    total += B->cnt[k];
  }
  for (const Op& op : B->log) B->cnt[op.key]++;
  std::vector<Op> ops(total);
  uint32_t run = 0;
  for (size_t k = 0; k < nk; ++k) {
    KeyState& ks = B->keys[k];
    const uint32_t c = B->cnt[k];
    std::copy(B->ops.begin() + ks.ob, B->ops.begin() + ks.oe, ops.begin() + run);
    B->cnt[k] = run + (ks.oe - ks.ob);  // write cursor for the new operations
    ks.ob = run;
    ks.oe = run + c;
    run += c;
  }
  for (const Op& op : B->log) ops[B->cnt[op.key]++] = op;
  B->ops.swap(ops);
  B->log.clear();
  for (uint32_t k = 0; k < (uint32_t)nk; ++k) {
    KeyState& ks = B->keys[k];
    if (ks.ob < ks.oe && !ks.waiting && !ks.queued) {
      ks.queued = true;
      B->runq.push_back(k);
    }
  }
}

// Run a key's operations until one needs the matcher (its request goes to
// the sink).
void run_key(otm_batcher* B, uint32_t k, Sink& sk) {
  KeyState& ks = B->keys[k];
  ks.queued = false;
  while (!ks.waiting && ks.ob < ks.oe) {
    const Op op = B->ops[ks.ob++];
    int min_dist, min_size;
    int64_t min_elapsed;
    if (op.kind == OP_PROCESS) {
      if (!ks.in_store) {  // store.delete -> null: a new batch, no report
        ks.batch = JBatch{};
        ks.batch.pts.push_back(op.pt);
        ks.in_store = true;
        continue;
      }
      jupdate(ks.batch, op.pt);
      min_dist = B->cfg.report_dist;
      min_size = B->cfg.report_count;
      min_elapsed = B->cfg.report_time_s;
    } else {
      if (!ks.in_store) {  // clean(): store.get -> null (the reference throws); close(): not iterated
        if (op.kind == OP_CLEAN) sk.nulls++;
        continue;
      }
      min_dist = 0;
      min_size = 2;
      min_elapsed = 0;
    }
    if (!jgates(ks.batch, min_dist, min_size, min_elapsed)) {
      // report() returned null: nothing forwarded; process() puts the batch back
      continue;
    }
    ks.waiting = true;
    ks.wop = op;
    Request r;
    r.key = k;
    r.npts = (int)ks.batch.pts.size();
    sk.reqs.push_back(std::move(r));
    return;
  }
}

// Apply one response to its key (Batch.java:64-83, BatchingProcessor.java:69-81)
void complete(otm_batcher* B, uint32_t k, int trim, int code, char* body, size_t body_len, Sink& sk) {
  KeyState& ks = B->keys[k];
  if (trim == -2) {
    ks.batch.max_sep = 0.0f;
    ks.batch.pts.clear();
  } else {
    japply(ks.batch, trim);
  }
  (void)code;
  if (ks.wop.kind == OP_PROCESS && body == nullptr) {
    // a null response (transport failure): nothing forwarded (:70-71), and the
    // cleared batch is not put back
    ks.in_store = !ks.batch.pts.empty();
  } else if (ks.wop.kind == OP_PROCESS) {
    // context.forward(key, response); store.put only if non-empty
    otm_forward f;
    f.key = (char*)std::malloc(ks.key.size() + 1);
    std::memcpy(f.key, ks.key.data(), ks.key.size());
    f.key[ks.key.size()] = 0;
    f.key_len = ks.key.size();
    f.body = body;
    f.body_len = body_len;
    f.seq = ks.wop.seq;
    sk.out.push_back(f);
    sk.forwarded++;
    ks.in_store = !ks.batch.pts.empty();
  } else {
    // clean()/close() discard the response; the batch object stays in the
    // store even when emptied (store.get returned it, nothing puts it back)
    otm_free(body);
  }
  ks.waiting = false;
  if (ks.ob < ks.oe && !ks.queued) {
    ks.queued = true;
    sk.runq.push_back(k);
  }
}

// the pool over [0, n) (or the caller alone), sinks cleared first
void par(otm_batcher* B, size_t n, const std::function<void(Sink&, size_t, size_t)>& fn) {
  for (Sink& sk : B->sinks) sk.clear();
  if (!B->pool) {
    fn(B->sinks[0], 0, n);
    return;
  }
  B->pool->run(n, [&](int t, size_t a, size_t e) { fn(B->sinks[(size_t)t], a, e); });
}

// fold the sinks' forwards, re-queued keys and counts into the batcher
void merge_sinks(otm_batcher* B) {
  for (Sink& sk : B->sinks) {
    for (const otm_forward& f : sk.out) B->out.push_back(f);
    B->runq.insert(B->runq.end(), sk.runq.begin(), sk.runq.end());
    B->st.forwarded += sk.forwarded;
    B->st.null_batch_in_clean += sk.nulls;
  }
}

int64_t now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

}  // namespace

namespace otm {
// The quantisation a point's coordinates go through on the JSON path:
// DecimalFormat("###.######") in Java, json.loads in Python, float in the
// matcher.  Without the string: a float has 24 significant bits and 1e6 =
// 2^6 * 15625 needs 14, so v * 1e6 is exact in double; nearbyint (round to
// nearest, ties to even) is HALF_EVEN on the exact value; n / 1e6 with both
// operands exact is the correctly rounded double of the decimal n * 10^-6,
// which is what strtod returns for its text.  The string form stays for
// values the shortcut does not cover (|v| * 1e6 >= 2^53, NaN, Inf).
float quantize_decimal6(float v) {
  const double d = (double)v * 1e6;
  if (std::fabs(d) < 9.0e15) return (float)(std::nearbyint(d) / 1e6);
  std::string s;
  java_decimal6(v, &s);
  return (float)std::strtod(s.c_str(), nullptr);
}
}  // namespace otm

namespace {

int issue_binary(otm_batcher* B, size_t r0, size_t r1) {
  otm_engine* E = B->eng;
  const int64_t t0 = now_us();
  const size_t n = r1 - r0;
  std::vector<int64_t> off(n + 1, 0);
  for (size_t i = 0; i < n; ++i) off[i + 1] = off[i] + (int64_t)B->keys[B->reqs[r0 + i].key].batch.pts.size();
  const size_t np = (size_t)off[n];
  std::vector<float> lat(np), lon(np), acc(np);
  std::vector<double> tm(np);
  par(B, n, [&](Sink&, size_t a, size_t e) {
    for (size_t i = a; i < e; ++i) {
      size_t o = (size_t)off[i];
      for (const JPoint& p : B->keys[B->reqs[r0 + i].key].batch.pts) {
        lat[o] = otm::quantize_decimal6(p.lat);
        lon[o] = otm::quantize_decimal6(p.lon);
        tm[o] = (double)p.time;
        acc[o] = (float)p.acc;
        ++o;
      }
    }
  });
  otm_batch b;
  b.n_traces = (int32_t)n;
  b.n_points = (int64_t)np;
  b.trace_off = off.data();
  b.lat = lat.data();
  b.lon = lon.data();
  b.time = tm.data();
  b.accuracy = acc.data();
  std::string err;
  otm_results res;
  int rc;
  // a multi-device engine: each request to its key's member (Kafka's partition)
  std::vector<int32_t> shard;
  if (!E->members.empty()) {
    shard.resize(n);
    for (size_t i = 0; i < n; ++i) {
      const std::string& key = B->keys[B->reqs[r0 + i].key].key;
      shard[i] = otm::shard_of(key.data(), key.size(), (int)E->members.size());
    }
  }
  {
    std::lock_guard<std::mutex> lk(E->mu);
    const int64_t t1 = now_us();
    B->st.us_prepare += t1 - t0;
    rc = otm::match_host_fetch(E, &b, shard.empty() ? nullptr : shard.data(), &res, &err);
    const int64_t t2 = now_us();
    B->st.us_match += t2 - t1;
    if (!rc) {
      // per request (each a different key): the trim, and the response body
      // where process() forwards it
      par(B, n, [&](Sink& sk, size_t a, size_t e) {
        std::string s;
        for (size_t i = a; i < e; ++i) {
          const uint32_t k = B->reqs[r0 + i].key;
          const otm_trace_result& tr = res.traces[i];
          // shape_used is written only when 200 and truthy (reporter_service.py:202)
          const int trim = tr.code == 200 && tr.shape_used > 0 ? tr.shape_used : -1;
          char* body = nullptr;
          size_t blen = 0;
          if (B->keys[k].wop.kind == OP_PROCESS) {
            s.clear();
            (void)otm::write_report_response(res, (int32_t)i, &s);
            body = (char*)std::malloc(s.size() + 1);
            std::memcpy(body, s.data(), s.size());
            body[s.size()] = 0;
            blen = s.size();
          }
          complete(B, k, trim, tr.code, body, blen, sk);
        }
      });
      merge_sinks(B);
    }
    B->st.us_apply += now_us() - t2;
  }
  if (rc) {
    // a device failure fails the batch like a 500 from the service: every
    // request gets {"error":...}, whose missing shape_used clears its batch
    const std::string s = otm::error_body(err);
    par(B, n, [&](Sink& sk, size_t a, size_t e) {
      for (size_t i = a; i < e; ++i) {
        const uint32_t k = B->reqs[r0 + i].key;
        char* body = nullptr;
        size_t blen = 0;
        if (B->keys[k].wop.kind == OP_PROCESS) {
          body = (char*)std::malloc(s.size() + 1);
          std::memcpy(body, s.data(), s.size() + 1);
          blen = s.size();
        }
        complete(B, k, -1, 500, body, blen, sk);
      }
    });
    merge_sinks(B);
  }
  return OTM_OK;
}

int issue_json(otm_batcher* B, size_t r0, size_t r1) {
  const int64_t t0 = now_us();
  const int n = (int)(r1 - r0);
  std::vector<const char*> rp((size_t)n);
  std::vector<size_t> rl((size_t)n), ol((size_t)n);
  std::vector<char*> outs((size_t)n, nullptr);
  std::vector<int> codes((size_t)n, 0), trims((size_t)n, 0);
  // request bodies (Batch.java:52-61), per request
  par(B, (size_t)n, [&](Sink&, size_t a, size_t e) {
    std::vector<float> la, lo;
    std::vector<int64_t> tm;
    std::vector<int32_t> ac;
    for (size_t i = r0 + a; i < r0 + e; ++i) {
      KeyState& ks = B->keys[B->reqs[i].key];
      la.clear();
      lo.clear();
      tm.clear();
      ac.clear();
      for (const JPoint& p : ks.batch.pts) {
        la.push_back(p.lat);
        lo.push_back(p.lon);
        tm.push_back(p.time);
        ac.push_back(p.acc);
      }
      otm::encode_request(ks.wire, (int)la.size(), la.data(), lo.data(), tm.data(), ac.data(), &B->reqs[i].body);
      rp[i - r0] = B->reqs[i].body.data();
      rl[i - r0] = B->reqs[i].body.size();
    }
  });
  const int64_t t1 = now_us();
  B->st.us_prepare += t1 - t0;
  int rc = B->fn ? B->fn(B->ctx, n, rp.data(), rl.data(), outs.data(), ol.data(), codes.data())
                 : otm_report_batch(B->eng, n, rp.data(), rl.data(), outs.data(), ol.data(), codes.data());
  const int64_t t2 = now_us();
  B->st.us_match += t2 - t1;
  if (rc != OTM_OK) {
    // The handler failed as a whole: HttpClient.POST's transport failure,
    // which returns null (HttpClient.java:37-39).  Batch.report then fails to
    // parse the null response and clears the batch (Batch.java:77-81), and
    // process() forwards nothing (BatchingProcessor.java:70-71).  Every key
    // of this chunk completes that way; the drain goes on with the next.
    B->err = "matcher callback failed";
    B->st.null_responses += n;
    for (int i = 0; i < n; ++i) otm_free(outs[(size_t)i]);
    par(B, (size_t)n, [&](Sink& sk, size_t a, size_t e) {
      for (size_t i = a; i < e; ++i) complete(B, B->reqs[r0 + i].key, -2, 0, nullptr, 0, sk);
    });
    merge_sinks(B);
    B->st.us_apply += now_us() - t2;
    return OTM_OK;
  }
  // a callback must hand back malloc'd bodies (otm_free releases them)
  par(B, (size_t)n, [&](Sink& sk, size_t a, size_t e) {
    for (size_t i = a; i < e; ++i)
      complete(B, B->reqs[r0 + i].key, parse_trim(outs[i], ol[i]), codes[i], outs[i], ol[i], sk);
  });
  merge_sinks(B);
  B->st.us_apply += now_us() - t2;
  return OTM_OK;
}

// One formatted record (BatchingProcessor.process, :56-85): the clean()
// pops its timestamp causes, then the record's own operation.
void ingest(otm_batcher* B, uint32_t k, const JPoint& pt, int64_t ts) {
  // clean(key): keys whose entry is older than the session gap, stalest
  // first (BatchingProcessor.java:96-103)
  while (!B->time_to_key.empty() && ts - B->time_to_key.front().first > B->cfg.session_gap_ms) {
    const uint32_t kk = B->time_to_key.front().second;
    B->time_to_key.pop_front();
    Op c{};
    c.kind = OP_CLEAN;
    c.seq = B->seq;
    enqueue(B, kk, c);
    B->st.clean_ops++;
  }
  B->time_to_key.emplace_back(ts, k);  // (:106-111; the remove(iter) before it is a no-op)
  Op p{};
  p.kind = OP_PROCESS;
  p.pt = pt;
  p.seq = B->seq++;
  enqueue(B, k, p);
  B->st.records++;
}

// Key ids of n records: known keys looked up by the pool (read-only on the
// index), new ones inserted in record order by the caller.
template <class KeyAt>
void key_ids(otm_batcher* B, size_t n, const KeyAt& key_at, std::vector<uint32_t>* ids) {
  ids->resize(n);
  constexpr uint32_t kNew = 0xFFFFFFFFu;
  if (B->pool && n >= 16384) {
    par(B, n, [&](Sink&, size_t a, size_t e) {
      for (size_t i = a; i < e; ++i) {
        auto it = B->index.find(key_at(i));
        (*ids)[i] = it != B->index.end() ? it->second : kNew;
      }
    });
    for (size_t i = 0; i < n; ++i)
      if ((*ids)[i] == kNew) {
        const std::string_view k = key_at(i);
        (*ids)[i] = key_id(B, k.data(), k.size());
      }
    return;
  }
  for (size_t i = 0; i < n; ++i) {
    const std::string_view k = key_at(i);
    (*ids)[i] = key_id(B, k.data(), k.size());
  }
}

int drain(otm_batcher* B) {
  distribute(B);
  while (true) {
    const int64_t t0 = now_us();
    while (!B->runq.empty()) {
      std::vector<uint32_t> q;
      q.swap(B->runq);
      par(B, q.size(), [&](Sink& sk, size_t a, size_t e) {
        for (size_t i = a; i < e; ++i) run_key(B, q[i], sk);
      });
      for (Sink& sk : B->sinks) {
        B->reqs.insert(B->reqs.end(), std::make_move_iterator(sk.reqs.begin()),
                       std::make_move_iterator(sk.reqs.end()));
        B->st.null_batch_in_clean += sk.nulls;
      }
    }
    B->st.us_run += now_us() - t0;
    if (B->reqs.empty()) return OTM_OK;
    std::vector<Request> reqs;
    reqs.swap(B->reqs);
    B->reqs = std::move(reqs);
    const size_t n = B->reqs.size();
    const size_t chunk = B->cfg.max_batch > 0 ? (size_t)B->cfg.max_batch : n;
    for (size_t r0 = 0; r0 < n; r0 += chunk) {
      const size_t r1 = std::min(n, r0 + chunk);
      for (size_t i = r0; i < r1; ++i) B->st.request_points += B->reqs[i].npts;
      B->st.requests += (int64_t)(r1 - r0);
      B->st.match_batches++;
      int rc;
      if (B->fn || B->cfg.json_path) {
        rc = issue_json(B, r0, r1);
      } else {
        // keys whose body the service would not read as the binary path does
        // (a Latin-1 byte that breaks body.decode('utf-8'), a quote, a
        // backslash, a control character) take the byte-level path, which
        // answers them exactly (their 400s included)
        auto mid = std::stable_partition(B->reqs.begin() + (ptrdiff_t)r0, B->reqs.begin() + (ptrdiff_t)r1,
                                         [&](const Request& q) { return B->keys[q.key].plain; });
        const size_t m = (size_t)(mid - B->reqs.begin());
        rc = m > r0 ? issue_binary(B, r0, m) : OTM_OK;
        if (!rc && r1 > m) rc = issue_json(B, m, r1);
      }
      if (rc) return rc;
    }
    B->reqs.clear();
  }
}

}  // namespace

extern "C" {

void otm_batcher_defaults(otm_batcher_cfg* c) {
  c->report_dist = 500;           // BatchingProcessor.java:30
  c->report_count = 10;           // :29
  c->report_time_s = 60;          // :28
  c->session_gap_ms = 60000;      // :31
  c->max_batch = 0;
  c->json_path = 0;
  c->max_pending = 0;
  c->threads = 0;
  c->reserved = 0;
}

static int otm_batcher_create_impl(otm_engine* eng, const otm_batcher_cfg* cfg, otm_report_fn fn, void* ctx,
                       otm_batcher** out) {
  if (!out || (!eng && !fn)) return OTM_EINVAL;
  auto* B = new otm_batcher();
  B->eng = eng;
  if (cfg) B->cfg = *cfg;
  else otm_batcher_defaults(&B->cfg);
  B->fn = fn;
  B->ctx = ctx;
  const int nt = B->cfg.threads > 1 ? std::min(B->cfg.threads, 256) : 1;
  if (nt > 1) B->pool.reset(new Pool(nt));
  B->sinks.resize((size_t)nt);
  *out = B;
  return OTM_OK;
}

void otm_batcher_destroy(otm_batcher* B) {
  if (!B) return;
  for (auto& f : B->out) {
    otm_free(f.key);
    otm_free(f.body);
  }
  delete B;
}

static int otm_batcher_process_impl(otm_batcher* B, int n, const char* const* keys, const size_t* key_lens, const float* lat,
                        const float* lon, const int32_t* accuracy, const int64_t* time, const int64_t* ts_ms) {
  if (!B || n < 0) return OTM_EINVAL;
  const int64_t t0 = now_us();
  // keys as the Java host holds them: StringDeserializer then StringSerializer
  // (javastr.h); only a key with a byte >= 0x80 can change
  std::vector<std::string> canon;
  std::vector<int32_t> canon_at;
  for (int i = 0; i < n; ++i) {
    std::string c;
    if (otm::jstr::kafka_key(std::string_view(keys[i], key_lens[i]), &c)) {
      if (canon_at.empty()) canon_at.assign((size_t)n, -1);
      canon_at[(size_t)i] = (int32_t)canon.size();
      canon.push_back(std::move(c));
    }
  }
  std::vector<uint32_t> ids;
  key_ids(B, (size_t)n,
          [&](size_t i) {
            if (!canon_at.empty() && canon_at[i] >= 0) return std::string_view(canon[(size_t)canon_at[i]]);
            return std::string_view(keys[i], key_lens[i]);
          },
          &ids);
  for (int i = 0; i < n; ++i) ingest(B, ids[(size_t)i], JPoint{lat[i], lon[i], accuracy[i], time[i]}, ts_ms[i]);
  B->st.us_enqueue += now_us() - t0;
  if (B->cfg.max_pending > 0 && (int64_t)B->log.size() > B->cfg.max_pending) return drain(B);
  return OTM_OK;
}

static int otm_batcher_process_raw_impl(otm_batcher* B, const otm_formatter* f, int32_t n, const char* msgs, const int64_t* off,
                            const int64_t* ts_ms, int nthreads) {
  if (!B || !f || n < 0 || (n > 0 && !ts_ms)) return OTM_EINVAL;
  const int64_t t0 = now_us();
  otm_formatted r;
  int rc = otm_format(f, n, msgs, off, nthreads, &r);
  if (rc) return rc;
  const int64_t t1 = now_us();
  B->st.us_format += t1 - t0;
  B->st.raw_messages += n;
  B->st.raw_dropped += n - r.n_ok;
  std::vector<int32_t> okm;  // the formatted messages, in stream order
  okm.reserve((size_t)r.n_ok);
  for (int32_t i = 0; i < n; ++i)
    if (r.ok[i]) okm.push_back(i);
  std::vector<uint32_t> ids;
  key_ids(B, okm.size(),
          [&](size_t j) {
            const int32_t i = okm[j];
            return std::string_view(r.keys + r.key_off[i], (size_t)(r.key_off[i + 1] - r.key_off[i]));
          },
          &ids);
  for (size_t j = 0; j < okm.size(); ++j) {
    const int32_t i = okm[j];
    ingest(B, ids[j], JPoint{r.lat[i], r.lon[i], r.accuracy[i], r.time[i]}, ts_ms[i]);
  }
  otm_formatted_free(&r);
  B->st.us_enqueue += now_us() - t1;
  if (B->cfg.max_pending > 0 && (int64_t)B->log.size() > B->cfg.max_pending) return drain(B);
  return OTM_OK;
}

static int otm_batcher_flush_impl(otm_batcher* B) {
  if (!B) return OTM_EINVAL;
  return drain(B);
}

static int otm_batcher_close_impl(otm_batcher* B) {
  if (!B) return OTM_EINVAL;
  int rc = drain(B);
  if (rc) return rc;
  // store.all() of the in-memory store: keys in TreeMap (String) order
  std::vector<uint32_t> ks;
  for (uint32_t k = 0; k < (uint32_t)B->keys.size(); ++k)
    if (B->keys[k].in_store) ks.push_back(k);
  std::sort(ks.begin(), ks.end(),
            [&](uint32_t a, uint32_t b) { return otm::jstr::compare(B->keys[a].key, B->keys[b].key) < 0; });
  for (uint32_t k : ks) {
    Op c{};
    c.kind = OP_CLOSE;
    c.seq = B->seq;
    enqueue(B, k, c);
    B->st.close_ops++;
  }
  return drain(B);
}

void otm_quantize_decimal6(const float* in, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = otm::quantize_decimal6(in[i]);
}

int otm_batcher_take(otm_batcher* B, otm_forward* out, int max) {
  if (!B || max < 0) return OTM_EINVAL;
  int n = 0;
  while (n < max && !B->out.empty()) {
    out[n++] = B->out.front();
    B->out.pop_front();
  }
  return n;
}

int otm_batcher_get_stats(const otm_batcher* B, otm_batcher_stats* s) {
  if (!B || !s) return OTM_EINVAL;
  *s = B->st;
  int64_t stored = 0, pts = 0;
  for (const KeyState& k : B->keys)
    if (k.in_store) {
      ++stored;
      pts += (int64_t)k.batch.pts.size();
    }
  s->stored_batches = stored;
  s->stored_points = pts;
  s->keys = (int64_t)B->keys.size();
  return OTM_OK;
}

int otm_batcher_batch(const otm_batcher* B, const char* key, size_t key_len, int max, float* lat, float* lon,
                      int32_t* accuracy, int64_t* time, float* max_separation) {
  if (!B || !key) return OTM_EINVAL;
  std::string canon;
  auto it = otm::jstr::kafka_key(std::string_view(key, key_len), &canon) ? B->index.find(canon)
                                                                          : B->index.find(std::string_view(key, key_len));
  if (it == B->index.end() || !B->keys[it->second].in_store) return -1;
  const JBatch& b = B->keys[it->second].batch;
  const int n = (int)b.pts.size();
  for (int i = 0; i < n && i < max; ++i) {
    lat[i] = b.pts[(size_t)i].lat;
    lon[i] = b.pts[(size_t)i].lon;
    accuracy[i] = b.pts[(size_t)i].acc;
    time[i] = b.pts[(size_t)i].time;
  }
  if (max_separation) *max_separation = b.max_sep;
  return n;
}

// nothing throws across the C ABI
int otm_batcher_create(otm_engine* eng, const otm_batcher_cfg* cfg, otm_report_fn fn, void* ctx,
                       otm_batcher** out) {
  try {
    return otm_batcher_create_impl(eng, cfg, fn, ctx, out);
  } catch (...) {
    return OTM_ENOMEM;  // (a host allocation failure; the batcher should then be destroyed)
  }
}

int otm_batcher_process(otm_batcher* B, int n, const char* const* keys, const size_t* key_lens, const float* lat,
                        const float* lon, const int32_t* accuracy, const int64_t* time, const int64_t* ts_ms) {
  try {
    return otm_batcher_process_impl(B, n, keys, key_lens, lat, lon, accuracy, time, ts_ms);
  } catch (...) {
    return OTM_ENOMEM;  // (a host allocation failure; the batcher should then be destroyed)
  }
}

int otm_batcher_process_raw(otm_batcher* B, const otm_formatter* f, int32_t n, const char* msgs, const int64_t* off,
                            const int64_t* ts_ms, int nthreads) {
  try {
    return otm_batcher_process_raw_impl(B, f, n, msgs, off, ts_ms, nthreads);
  } catch (...) {
    return OTM_ENOMEM;  // (a host allocation failure; the batcher should then be destroyed)
  }
}

int otm_batcher_flush(otm_batcher* B) {
  try {
    return otm_batcher_flush_impl(B);
  } catch (...) {
    return OTM_ENOMEM;  // (a host allocation failure; the batcher should then be destroyed)
  }
}

int otm_batcher_close(otm_batcher* B) {
  try {
    return otm_batcher_close_impl(B);
  } catch (...) {
    return OTM_ENOMEM;  // (a host allocation failure; the batcher should then be destroyed)
  }
}

}  // extern "C"
