// synth_traces.cpp -- seeded synthetic probe traces over a .otmg graph.
//
// Stand-in for py/generate_test_trace.py (routes via a live Valhalla, then
// synthesize_gps :31-73) at benchmark scale, per SURVEY.md §8(d) config 2:
// vehicles drive a random walk (no immediate U-turns, 70 % straight-on
// preference) at a per-level speed (level 0: 20-25 m/s, 1: 12-16, 2: 8-11),
// sampled every interval_s, with isotropic Gaussian noise of noise_sigma_m
// on each axis.  lat/lon are float32 and time integral, as the Java host
// would send them (Point.java:19-21).  Vehicle v's stream depends only on
// (seed, vehicle_offset + v), so uuid shards generate identical vehicles.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "otm_internal.h"

namespace otm {
namespace {
const double kMpd = 20037581.187 / 180.0;
const double kPi = 3.14159265358979323846;

double heading(const HostGraph& g, int e, bool at_end) {
  int a = g.e_shape_off[e], b = g.e_shape_off[e + 1] - 1;
  int i0 = at_end ? b - 1 : a, i1 = at_end ? b : a + 1;
  double dy = (double)g.s_lat[i1] - g.s_lat[i0];
  double dx = ((double)g.s_lon[i1] - g.s_lon[i0]) * std::cos(g.s_lat[i0] * kPi / 180.0);
  return std::atan2(dy, dx);
}
}  // namespace

// path (optional): the edges each vehicle drives from its first to its last
// probe, in order, appended per vehicle; path_off[v] = where vehicle v's
// start; enter (optional, with path): the time the vehicle entered each path
// edge (the first edge's before the first probe, at the vehicle's speed)
int synth_traces(const HostGraph& g, const otm_synth_trace_params* p, int64_t* trace_off, float* lat, float* lon,
                 double* time, float* accuracy, int32_t* true_edge, float* true_off,
                 std::vector<int32_t>* path = nullptr, int64_t* path_off = nullptr,
                 std::vector<double>* enter = nullptr) {
  const int NE = g.h.n_edges;
  std::vector<int> starts;
  for (int e = 0; e < NE; ++e)
    if (!(g.e_flags[e] & OTM_EDGE_INTERNAL)) starts.push_back(e);
  if (starts.empty()) return OTM_EINVAL;
  int64_t P = 0;
  for (int v = 0; v < p->n_vehicles; ++v) {
    trace_off[v] = P;
    uint64_t gv = (uint64_t)(p->vehicle_ids ? p->vehicle_ids[v] : p->vehicle_offset + v);
    Rng rng(p->seed * 0x9E3779B97F4A7C15ull ^ (gv + 1) * 0xD1B54A32D192ED03ull);
    rng.next();
    int e = starts[rng.next() % starts.size()];
    double off = rng.uni() * g.e_len[e];
    if (path) {
      path_off[v] = (int64_t)path->size();
      path->push_back(e);
    }
    double f = rng.uni();
    int internal_run = 0;
    auto speed_of = [&](int edge) {
      int lv = g.e_level[edge];
      double lo = lv == 0 ? 20.0 : (lv == 1 ? 12.0 : 8.0), hi = lv == 0 ? 25.0 : (lv == 1 ? 16.0 : 11.0);
      if (g.e_flags[edge] & OTM_EDGE_INTERNAL) lo = 6.0, hi = 9.0;
      return lo + f * (hi - lo);
    };
    if (path && enter) enter->push_back(p->t0 - off / speed_of(e));
    for (int s = 0; s < p->points_per_vehicle; ++s) {
      // position on (e, off)
      int a = g.e_shape_off[e], b = g.e_shape_off[e + 1] - 1;
      int k = a;
      while (k + 1 < b && (double)g.s_cum[k + 1] < off) ++k;
      double c0 = g.s_cum[k], c1 = g.s_cum[k + 1];
      double t = c1 > c0 ? (off - c0) / (c1 - c0) : 0.0;
      t = t < 0 ? 0 : (t > 1 ? 1 : t);
      double la = g.s_lat[k] + t * ((double)g.s_lat[k + 1] - g.s_lat[k]);
      double lo = g.s_lon[k] + t * ((double)g.s_lon[k + 1] - g.s_lon[k]);
      if (p->noise_sigma_m > 0) {
        double ny = rng.normal() * p->noise_sigma_m, nx = rng.normal() * p->noise_sigma_m;
        la += ny / kMpd;
        lo += nx / (kMpd * std::cos(la * kPi / 180.0));
      }
      lat[P] = (float)la;
      lon[P] = (float)lo;
      time[P] = p->t0 + s * p->interval_s;
      accuracy[P] = p->accuracy;
      if (true_edge) true_edge[P] = e;
      if (true_off) true_off[P] = (float)off;
      ++P;
      // advance (not past the last probe: the true path ends on its edge)
      if (s + 1 == p->points_per_vehicle) break;
      double dt = p->interval_s;
      int guard = 0;
      while (dt > 0 && guard++ < 10000) {
        double v = speed_of(e);
        double rem = g.e_len[e] - off;
        if (rem >= v * dt) {
          off += v * dt;
          dt = 0;
          break;
        }
        dt -= rem / v;
        int node = g.e_to[e];
        int o0 = g.out_off[node], o1 = g.out_off[node + 1];
        std::vector<int> opts;
        for (int o = o0; o < o1; ++o)
          if (o != g.e_opp[e]) opts.push_back(o);
        if (internal_run >= 2) {
          std::vector<int> ext;
          for (int o : opts)
            if (!(g.e_flags[o] & OTM_EDGE_INTERNAL)) ext.push_back(o);
          if (!ext.empty()) opts.swap(ext);
        }
        if (opts.empty()) opts.push_back(g.e_opp[e] >= 0 ? g.e_opp[e] : o0);
        int next = opts[0];
        if (opts.size() > 1) {
          if (rng.uni() < 0.7) {
            double h0 = heading(g, e, true), best = 1e9;
            for (int o : opts) {
              double d = std::fabs(std::remainder(heading(g, o, false) - h0, 2 * kPi));
              if (d < best) best = d, next = o;
            }
          } else {
            next = opts[rng.next() % opts.size()];
          }
        }
        internal_run = (g.e_flags[next] & OTM_EDGE_INTERNAL) ? internal_run + 1 : 0;
        e = next;
        off = 0;
        if (path) path->push_back(e);
        if (path && enter) enter->push_back(p->t0 + s * p->interval_s + (p->interval_s - dt));
      }
    }
  }
  trace_off[p->n_vehicles] = P;
  if (path) path_off[p->n_vehicles] = (int64_t)path->size();
  return OTM_OK;
}

}  // namespace otm

extern "C" int otm_synth_traces(const char* graph_path, const otm_synth_trace_params* p, int64_t* trace_off,
                                float* lat, float* lon, double* time, float* accuracy, int32_t* true_edge,
                                float* true_off) {
  otm::HostGraph g;
  std::string err;
  int rc = otm::load_graph(graph_path, &g, &err);
  if (rc) {
    otm::set_thread_error(err);
    return rc;
  }
  return otm::synth_traces(g, p, trace_off, lat, lon, time, accuracy, true_edge, true_off);
}

// The ground truth of otm_synth_traces: each vehicle's driven edge sequence
// (same generator, same seeds), for implementation-independent accuracy
// figures.  Fills path_off[n_vehicles + 1] and up to `cap` edges; returns the
// total edge count (call with cap 0 to size), or a negative error.
extern "C" int64_t otm_synth_true_paths_timed(const char* graph_path, const otm_synth_trace_params* p,
                                              int64_t* path_off, int32_t* path_edges, double* enter_time,
                                              int64_t cap) {
  otm::HostGraph g;
  std::string err;
  int rc = otm::load_graph(graph_path, &g, &err);
  if (rc) {
    otm::set_thread_error(err);
    return rc;
  }
  const size_t P = (size_t)p->n_vehicles * (size_t)p->points_per_vehicle;
  std::vector<int64_t> toff((size_t)p->n_vehicles + 1);
  std::vector<float> la(P), lo(P), acc(P);
  std::vector<double> tm(P);
  std::vector<int32_t> path;
  std::vector<double> ent;
  std::vector<int64_t> poff((size_t)p->n_vehicles + 1);
  rc = otm::synth_traces(g, p, toff.data(), la.data(), lo.data(), tm.data(), acc.data(), nullptr, nullptr, &path,
                         poff.data(), enter_time ? &ent : nullptr);
  if (rc) return rc;
  if (path_off) std::memcpy(path_off, poff.data(), poff.size() * 8);
  const size_t m = (size_t)std::min<int64_t>(std::max<int64_t>(cap, 0), (int64_t)path.size());
  if (path_edges && m) std::memcpy(path_edges, path.data(), m * 4);
  if (enter_time && m) std::memcpy(enter_time, ent.data(), m * 8);
  return (int64_t)path.size();
}

extern "C" int64_t otm_synth_true_paths(const char* graph_path, const otm_synth_trace_params* p, int64_t* path_off,
                                        int32_t* path_edges, int64_t cap) {
  return otm_synth_true_paths_timed(graph_path, p, path_off, path_edges, nullptr, cap);
}

// Kafka DefaultPartitioner: murmur2 (seed 0x9747b28c) over the key bytes.
extern "C" int32_t otm_murmur2(const char* key, size_t len) {
  const uint32_t m = 0x5bd1e995u;
  const int r = 24;
  uint32_t h = 0x9747b28cu ^ (uint32_t)len;
  const unsigned char* d = (const unsigned char*)key;
  size_t n4 = len / 4;
  for (size_t i = 0; i < n4; ++i) {
    uint32_t k = (uint32_t)d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) |
                 ((uint32_t)d[4 * i + 3] << 24);
    k *= m;
    k ^= k >> r;
    k *= m;
    h *= m;
    h ^= k;
  }
  size_t t = len & ~(size_t)3;
  switch (len % 4) {
    case 3: h ^= (uint32_t)d[t + 2] << 16; [[fallthrough]];
    case 2: h ^= (uint32_t)d[t + 1] << 8; [[fallthrough]];
    case 1: h ^= (uint32_t)d[t]; h *= m;
  }
  h ^= h >> 13;
  h *= m;
  h ^= h >> 15;
  return (int32_t)h;
}
