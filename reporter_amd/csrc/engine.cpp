// engine.cpp -- graph upload and per-batch orchestration of the kernels.
//
// Stands in for valhalla.Configure (py/reporter_service.py:279: load tiles
// once) and for one SegmentMatcher per worker (:52): here one engine per GPU
// holds the flattened graph in HBM and matches whole batches of traces.
#include "engine.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>

#include <cstring>

namespace otm {

#define HIPCHK(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      *err = std::string(#x) + ": " + hipGetErrorString(e_);                   \
      return OTM_EDEVICE;                                                      \
    }                                                                          \
  } while (0)

static int ensure(otm_engine::Buf& b, size_t bytes, std::string* err);
// host-pinned buffer of at least `bytes` (contents not kept on growth)
static int ensure_pinned(otm_engine::Buf& b, size_t bytes, std::string* err) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return OTM_OK;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  const size_t want = bytes + bytes / 4;
  HIPCHK(hipHostMalloc(&b.p, want, hipHostMallocDefault));
  b.cap = want;
  return OTM_OK;
}
#define ENS_F(buf, bytes) \
  if ((rc = ensure(E->buf, (bytes), err))) return rc;

static int ensure(otm_engine::Buf& b, size_t bytes, std::string* err) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return OTM_OK;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t want = bytes + bytes / 4;  // headroom against regrowth
  HIPCHK(hipMalloc(&b.p, want));
  b.cap = want;
  return OTM_OK;
}

// Grows an on-demand tier's table (the huge search and candidate tiers): the
// new allocation first, so that running out of HBM keeps the old table, and
// the failed hipMalloc's error taken off the runtime so the batch's later
// hipGetLastError checks do not report it.  OTM_TEST_GROW_OOM (tests only)
// asks for a size no device has, to drive that path for real.
static int ensure_grow(otm_engine::Buf& b, size_t bytes, std::string* err) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return OTM_OK;
  size_t want = bytes + bytes / 4;
  const char* oom = std::getenv("OTM_TEST_GROW_OOM");
  if (oom && *oom && *oom != '0') want = (size_t)1 << 62;
  void* p = nullptr;
  const hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *err = std::string("hipMalloc (tier table): ") + hipGetErrorString(e);
    return OTM_EDEVICE;
  }
  if (b.p) (void)hipFree(b.p);
  b.p = p;
  b.cap = want;
  return OTM_OK;
}

template <class T>
static T* P(otm_engine::Buf& b) {
  return (T*)b.p;
}

// A batch's host waits.  Large batches block on an event, so the waiting
// thread sleeps instead of spinning: with several batch contexts in flight
// (the async pipeline, the bench's in-flight contexts) spinning waiters hold
// CPUs the host threads need (the GPU box grants 16), and the cgroup then
// throttles the whole process.  Small batches (latency-bound single requests
// and batcher rounds) spin as hipStreamSynchronize does, and so do
// otm_match_device batches (their caller drives the GPU from its own threads:
// measured 1.27 vs 1.25G points/s on the bench's device leg, while the host
// leg went 0.57 -> 0.80G and the async JSON path 170 -> 221M with blocking
// waits).
static hipError_t wait_batch(otm_engine* E, hipStream_t s, int64_t points) {
  constexpr int64_t min_pts = 65536;
  if (points < min_pts || E->spin_waits) return hipStreamSynchronize(s);
  if (!E->sync_ev) {
    const hipError_t e = hipEventCreateWithFlags(&E->sync_ev, hipEventBlockingSync | hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  const hipError_t e = hipEventRecord(E->sync_ev, s);
  if (e != hipSuccess) return e;
  return hipEventSynchronize(E->sync_ev);
}

int build_index(otm_engine* E, std::string* err);

// exp(x), 0 <= x <= 4: Taylor series in double with a fixed term order, so the
// table is the same wherever it is computed (the CPU oracle's
// orc_turn_units does the same operations); no libm involved
static double exp_series(double x) {
  double term = 1.0, sum = 1.0;
  for (int n = 1; n <= 40; ++n) {
    term = term * x / (double)n;
    sum = sum + term;
  }
  return sum;
}
// turn cost of a turn deviating d degrees from straight on, in 1/64 m:
// round(factor * exp(-(180 - d) / 45) * 64) -- meili's turn table
// turn_penalty_factor * exp(-theta / 45) with theta the angle between the
// reversed incoming and the outgoing edge (theta = 180 - d)
uint32_t turn_units(float factor, int d) {
  if (!(factor > 0.0f)) return 0u;
  const double x = (double)(180 - d) / 45.0;
  return (uint32_t)std::floor((double)factor * 64.0 / exp_series(x) + 0.5);
}

// Grid multiplier when the config names none: the m that minimises the
// modelled cost of a probe's cell walk, ROW_COST x rows + entries scanned,
// with rows = box / (m cell) + 1 for a radius box of 2 x search_radius and
// entries = (entries per file cell) x m^2 x rows^2.  The row cost, in
// entries, grows as the graph thins -- 40 x sqrt(2.9 / density), an empirical
// fit to the candidate kernel's times on configs 2 and 4 (round 4,
// profiles/r04_ab/grid_inflight/): the city (2.9 entries per 56 m cell, 50 m
// radius) gets 2 (m = 1 / 2 / 3: 0.243 / 0.222 / 0.261 ms), the state graph
// (0.35 per cell, 200 m) 9 (m = 6 / 8 / 10 / 12 / 16: 1.77 / 1.59 / 1.57 /
// 1.59 / 1.70 ms, where round 3's constant 32 picked 5-6 at 1.84 ms).
static int auto_grid_mult(const otm_engine* E) {
  const auto& h = E->host.h;
  const double cells = std::max(1.0, (double)h.grid_rows * (double)h.grid_cols);
  const double dens = (double)h.n_cell_entries / cells;
  const double ROW_COST = std::min(160.0, std::max(32.0, 40.0 * std::sqrt(2.9 / std::max(dens, 1e-3))));
  const double cell_m = h.grid_cell_deg * 111195.0;
  const double box = 2.0 * std::max(1.0, (double)E->mc.search_radius);
  int best = 1;
  double best_cost = 1e300;
  for (int m = 1; m <= 16; ++m) {
    const double rows = box / (m * cell_m) + 1.0;
    const double cost = ROW_COST * rows + dens * (double)m * m * rows * rows;
    if (cost < best_cost) best_cost = cost, best = m;
  }
  return best;
}


int engine_init(otm_engine* E, const char* graph_path, int device, std::string* err) {
  int rc = load_graph(graph_path, &E->host, err);
  if (rc) return rc;
  if (E->host.h.n_edges >= (1 << 27)) {  // K2's lane-tier entries: edge << 4 below the node flag bit
    *err = "graph: 2^27 or more edges";
    return OTM_EINVAL;
  }
  if (E->grid_mult == 0) E->grid_mult = auto_grid_mult(E);
  E->device = device;
  HIPCHK(hipSetDevice(device));
  if (create_stream(0, &E->stream, false)) {
    *err = "stream creation failed";
    return OTM_EDEVICE;
  }
  const otmg_header& h = E->host.h;
  auto up = [&](int sec, const void** dst) -> int {
    void* d = nullptr;
    size_t n = h.sec[sec].bytes ? h.sec[sec].bytes : 16;
    HIPCHK(hipMalloc(&d, n));
    if (h.sec[sec].bytes) HIPCHK(hipMemcpy(d, E->host.section(sec), h.sec[sec].bytes, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    *dst = d;
    return OTM_OK;
  };
  DevGraph& g = E->g;
  const void* tmp;
#define UP(sec, field, T)                 \
  if ((rc = up(sec, &tmp))) return rc;    \
  g.field = (const T*)tmp;
  UP(OTMG_NODE_LAT, node_lat, float);
  UP(OTMG_NODE_LON, node_lon, float);
  UP(OTMG_NODE_OUT_OFF, out_off, int32_t);
  UP(OTMG_EDGE_FROM, e_from, int32_t);
  UP(OTMG_EDGE_TO, e_to, int32_t);
  UP(OTMG_EDGE_LEN, e_len, float);
  UP(OTMG_EDGE_SHAPE_OFF, e_shape_off, int32_t);
  UP(OTMG_EDGE_WAY, e_way, int64_t);
  UP(OTMG_EDGE_SEG, e_seg, int32_t);
  UP(OTMG_EDGE_SEG_POS, e_seg_pos, int32_t);
  UP(OTMG_EDGE_FLAGS, e_flags, uint8_t);
  UP(OTMG_SHAPE_LAT, s_lat, float);
  UP(OTMG_SHAPE_LON, s_lon, float);
  UP(OTMG_SHAPE_CUM, s_cum, float);
  UP(OTMG_SEG_ID, g_id, uint64_t);
  UP(OTMG_SEG_LEN, g_len, float);
  UP(OTMG_EDGE_HEAD_OUT, e_head_out, uint16_t);
  UP(OTMG_EDGE_HEAD_IN, e_head_in, uint16_t);
#undef UP
  {
    // turn units per deviation 0..180 degrees for the configured
    // turn_penalty_factor, one small device table
    uint32_t tu[TURN_TABLE];
    for (int d = 0; d < TURN_TABLE; ++d) tu[d] = turn_units(E->mc.turn_penalty_factor, d);
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof tu));
    HIPCHK(hipMemcpy(d, tu, sizeof tu, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    E->dp.turn_units = (const uint32_t*)d;
  }
  {
    // edge costs of the turn-aware searches: L(e) = round(len(e) x 64), in
    // 1/64 m (DESIGN.md §3 rule 4; the oracle computes the same from the file)
    const float* len = (const float*)E->host.section(OTMG_EDGE_LEN);
    std::vector<uint32_t> l64((size_t)h.n_edges + 1, 0u);
    for (int32_t e = 0; e < h.n_edges; ++e) l64[(size_t)e] = (uint32_t)std::floor((double)len[e] * 64.0 + 0.5);
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, l64.size() * 4));
    HIPCHK(hipMemcpy(d, l64.data(), l64.size() * 4, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    g.e_len64 = (const uint32_t*)d;
  }
  {
    // K7's edge record: what the segment pass reads per traversal -- length,
    // OSMLR segment, position in it, flags, way -- in one 16-byte word, so a
    // traversal's gather touches one line instead of five.
    // Ways are numbered through a table of the graph's distinct way ids (two
    // edges have the same way exactly when their numbers are equal).
    const float* len = (const float*)E->host.section(OTMG_EDGE_LEN);
    const int32_t* seg = (const int32_t*)E->host.section(OTMG_EDGE_SEG);
    const int32_t* pos = (const int32_t*)E->host.section(OTMG_EDGE_SEG_POS);
    const uint8_t* fl = (const uint8_t*)E->host.section(OTMG_EDGE_FLAGS);
    const int64_t* way = (const int64_t*)E->host.section(OTMG_EDGE_WAY);
    std::vector<int64_t> ways(way, way + h.n_edges);
    std::sort(ways.begin(), ways.end());
    ways.erase(std::unique(ways.begin(), ways.end()), ways.end());
    if (ways.size() >= (size_t)INT32_MAX) {
      *err = "graph: more than 2^31 distinct way ids";
      return OTM_EINVAL;
    }
    std::vector<uint32_t> rec((size_t)h.n_edges * 4 + 4, 0u);
    for (int32_t e = 0; e < h.n_edges; ++e) {
      if (seg[e] >= 0 && (pos[e] < 0 || pos[e] >= (1 << 24))) {
        *err = "graph: an edge's position in its OSMLR segment exceeds 2^24";
        return OTM_EINVAL;
      }
      uint32_t* r = &rec[(size_t)e * 4];
      std::memcpy(&r[0], &len[e], 4);
      r[1] = (uint32_t)seg[e];
      r[2] = ((uint32_t)(seg[e] >= 0 ? pos[e] : 0) & 0xFFFFFFu) | ((uint32_t)fl[e] << 24);
      r[3] = (uint32_t)(std::lower_bound(ways.begin(), ways.end(), way[e]) - ways.begin());
    }
    if (ways.empty()) ways.push_back(0);
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, rec.size() * 4));
    HIPCHK(hipMemcpy(d, rec.data(), rec.size() * 4, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    g.e_rec = (const uint4*)d;
    d = nullptr;
    HIPCHK(hipMalloc(&d, ways.size() * 8));
    HIPCHK(hipMemcpy(d, ways.data(), ways.size() * 8, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    g.way_tab = (const int64_t*)d;
    // {from, length bits} per edge: K4 stages a source candidate's index row
    // (from, for a node candidate) and start (length, for an edge candidate)
    // with one 8-byte load instead of two masked 4-byte ones
    const int32_t* from = (const int32_t*)E->host.section(OTMG_EDGE_FROM);
    std::vector<int32_t> fl2((size_t)h.n_edges * 2 + 2, 0);
    for (int32_t e = 0; e < h.n_edges; ++e) {
      fl2[(size_t)e * 2] = from[e];
      std::memcpy(&fl2[(size_t)e * 2 + 1], &len[e], 4);
    }
    d = nullptr;
    HIPCHK(hipMalloc(&d, fl2.size() * 4));
    HIPCHK(hipMemcpy(d, fl2.data(), fl2.size() * 4, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    g.e_fl = (const int2*)d;
  }
  {
    // The grid index of the candidate search.  The file's cells (meili's
    // 500 per 0.25 deg tile, ~55 m) may be merged m x m into coarser ones
    // (OTM_GRID_MULT, or grid_mult in the config): a probe's radius box then
    // spans fewer grid rows -- fewer dependent row loads -- at the price of
    // more entries scanned.  The candidates do not change: a shape segment is
    // listed in every cell its bbox touches, at either size, so every segment
    // within the radius is found and the per-edge best (sqdist, segment) is
    // the same minimum.  Only the cells / entries visited counts differ.
    const int m = E->grid_mult < 1 ? 1 : E->grid_mult;
    const int64_t* fo = (const int64_t*)E->host.section(OTMG_CELL_OFF);
    const uint32_t* fe = (const uint32_t*)E->host.section(OTMG_CELL_ENT);
    const int32_t R = (h.grid_rows + m - 1) / m, Cn = (h.grid_cols + m - 1) / m;
    std::vector<uint64_t> co_ent;  // (coarse cell << 32 | entry), coarse grids only
    const size_t nc = (size_t)R * (size_t)Cn + 1;
    std::vector<uint32_t> c32(nc, 0);
    std::vector<uint32_t> ent;
    if (m == 1) {
      if ((uint64_t)h.n_cell_entries >= (1ull << 32)) {
        *err = "graph: more than 2^32 cell entries (32-bit cell offsets)";
        return OTM_EINVAL;
      }
      for (size_t c = 0; c < nc; ++c) c32[c] = (uint32_t)fo[c];
      ent.assign(fe, fe + h.n_cell_entries);
    } else {
      co_ent.reserve((size_t)h.n_cell_entries);
      for (int32_t r = 0; r < h.grid_rows; ++r)
        for (int32_t c = 0; c < h.grid_cols; ++c) {
          const size_t f = (size_t)r * h.grid_cols + c;
          const uint64_t cc = (uint64_t)(r / m) * (uint64_t)Cn + (uint64_t)(c / m);
          for (int64_t q = fo[f]; q < fo[f + 1]; ++q) co_ent.push_back(cc << 32 | fe[q]);
        }
      std::sort(co_ent.begin(), co_ent.end());
      co_ent.erase(std::unique(co_ent.begin(), co_ent.end()), co_ent.end());
      if (co_ent.size() >= (1ull << 32)) {
        *err = "graph: more than 2^32 cell entries (32-bit cell offsets)";
        return OTM_EINVAL;
      }
      ent.resize(co_ent.size());
      for (size_t k = 0; k < co_ent.size(); ++k) {
        ent[k] = (uint32_t)co_ent[k];
        c32[(co_ent[k] >> 32) + 1]++;
      }
      for (size_t c = 0; c + 1 < nc; ++c) c32[c + 1] += c32[c];
      std::vector<uint64_t>().swap(co_ent);
    }
    E->grid_rows = R;
    E->grid_cols = Cn;
    E->grid_entries = (int64_t)ent.size();
    // cell offsets as 32-bit words in HBM: a sparse state-scale grid is
    // ~100M mostly-empty cells, and a probe's row range (2 offsets) then
    // usually sits in one cache line
    void* d = nullptr;
    HIPCHK(hipMalloc(&d, nc * 4));
    HIPCHK(hipMemcpy(d, c32.data(), nc * 4, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    g.cell_off = (const uint32_t*)d;
    d = nullptr;
    HIPCHK(hipMalloc(&d, ent.size() * 4 + 16));
    if (!ent.empty()) HIPCHK(hipMemcpy(d, ent.data(), ent.size() * 4, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    g.cell_ent = (const uint32_t*)d;
    // per cell entry: the shape segment's endpoints (lat_a, lon_a, lat_b,
    // lon_b), laid out in cell order so a probe's scan of one grid row is
    // one contiguous float4 stream (no edge -> shape indirection)
    const size_t ne = ent.size();
    const int32_t* soff = (const int32_t*)E->host.section(OTMG_EDGE_SHAPE_OFF);
    const float* slat = (const float*)E->host.section(OTMG_SHAPE_LAT);
    const float* slon = (const float*)E->host.section(OTMG_SHAPE_LON);
    std::vector<float> geo(ne * 4 + 4);
    for (size_t q = 0; q < ne; ++q) {
      const int32_t a = soff[ent[q] >> 4] + (int32_t)(ent[q] & 15u);
      geo[q * 4 + 0] = slat[a];
      geo[q * 4 + 1] = slon[a];
      geo[q * 4 + 2] = slat[a + 1];
      geo[q * 4 + 3] = slon[a + 1];
    }
    d = nullptr;
    HIPCHK(hipMalloc(&d, geo.size() * 4));
    HIPCHK(hipMemcpy(d, geo.data(), geo.size() * 4, hipMemcpyHostToDevice));
    E->graph_allocs.push_back(d);
    g.ent_geo = (const float4*)d;
    g.grid_rows = R;
    g.grid_cols = Cn;
    g.cell = h.grid_cell_deg * (double)m;
  }
  g.n_nodes = h.n_nodes;
  g.n_edges = h.n_edges;
  g.n_segments = h.n_segments;
  {
    // spatial-order tiles over the node bbox (a hair wider so max lands inside)
    const double h_deg = (h.bbox[2] - h.bbox[0]) * 1.0001 + 1e-9, w_deg = (h.bbox[3] - h.bbox[1]) * 1.0001 + 1e-9;
    g.bb_lat0 = (float)h.bbox[0];
    g.bb_lon0 = (float)h.bbox[1];
    g.bb_inv_h = (float)(ORDER_SIDE / h_deg);
    g.bb_inv_w = (float)(ORDER_SIDE / w_deg);
  }
  g.lat0 = h.grid_lat0;
  g.lon0 = h.grid_lon0;
  HIPCHK(hipMalloc((void**)&E->ctr, sizeof(DevCounters)));
  HIPCHK(hipMalloc((void**)&E->ctr_save, sizeof(DevCounters)));
  HIPCHK(hipMemset(E->ctr, 0, sizeof(DevCounters)));
  for (auto& e : E->kev) HIPCHK(hipEventCreate(&e));
  return build_index(E, err);
}

// The stream of batch context `slot` (0: the engine, k: its k-th clone), at
// normal priority (round 2: a prioritised context made the device leg slower,
// 0.78 -> 0.90-1.12 ms per step): from the runtime's pool of
// hardware queues (GPU_MAX_HW_QUEUES, shared round the process's streams), or,
// own_queue, on a hardware queue of its own -- a stream created with a CU mask
// (every CU) gets a new queue -- for the async pipeline's contexts, whose
// batches then run side by side instead of behind whatever other stream shares
// their queue (round 5: async 370-382M -> 538-553M points/s; the same for the
// one-call and device contexts was slower)
int create_stream(int slot, hipStream_t* s, bool own_queue) {
  (void)slot;
  if (own_queue) {
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && ncu > 0) {
      std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
      for (int c = 0; c < ncu; ++c) mask[(size_t)c / 32] |= 1u << (c % 32);
      if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) return 0;
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking) != hipSuccess;
}

int engine_clone(const otm_engine* P, otm_engine* C, std::string* err, bool own_queue) {
  C->parent = P;
  C->device = P->device;
  HIPCHK(hipSetDevice(C->device));
  const int slot = ++const_cast<otm_engine*>(P)->n_clones;
  if (create_stream(slot, &C->stream, own_queue)) {
    *err = "stream creation failed";
    return OTM_EDEVICE;
  }
  C->host.h = P->host.h;  // the header only: a clone reads no host graph sections
  C->g = P->g;
  C->idx = P->idx;
  for (int l = 0; l < NEAR_LEVELS; ++l) C->idxn[l] = P->idxn[l];
  for (int l = 0; l < NEAR_LEVELS; ++l) C->index_near_level_entries[l] = P->index_near_level_entries[l];
  C->index_rmax = P->index_rmax;
  C->index_entries = P->index_entries;
  C->index_slots = P->index_slots;
  C->index_near_slots = P->index_near_slots;
  C->index_incomplete_rows = P->index_incomplete_rows;
  C->index_build_ms = P->index_build_ms;
  C->small_points = P->small_points;
  C->trans_lanes = P->trans_lanes;
  C->mc = P->mc;
  C->rc = P->rc;
  C->dp = P->dp;
  C->drc = P->drc;
  HIPCHK(hipMalloc((void**)&C->ctr, sizeof(DevCounters)));
  HIPCHK(hipMalloc((void**)&C->ctr_save, sizeof(DevCounters)));
  HIPCHK(hipMemset(C->ctr, 0, sizeof(DevCounters)));
  for (auto& e : C->kev) HIPCHK(hipEventCreate(&e));
  (void)err;
  return OTM_OK;
}

// Index radius when the config names none: the road distance within which a
// row holds about INDEX_ROW_NODES nodes, from the graph's mean node density
// (a street grid holds ~2 rho R^2 nodes within road distance R), capped at
// the longest bound a transition can ask, max_route_distance_factor x
// breakage_distance.  The config-2 city (150 m blocks) gets 1.25 km, which
// covers every config-2 bound (5 x gc <= 952 m); the config-4 state graph
// (1.2 km blocks, 30 s sampling: bounds to ~5 km) gets the 10 km cap, with
// rows the same size as the city's.
static float auto_index_radius(const otm_engine* E) {
  constexpr double INDEX_ROW_NODES = 140.0;
  const auto& h = E->host.h;
  const double lat_mid = 0.5 * (h.bbox[0] + h.bbox[2]) * 3.14159265358979323846 / 180.0;
  const double h_m = (h.bbox[2] - h.bbox[0]) * 111195.0;
  const double w_m = (h.bbox[3] - h.bbox[1]) * 111195.0 * std::cos(lat_mid);
  const double area = std::max(h_m * w_m, 1.0);
  const double rho = std::max((double)h.n_nodes, 1.0) / area;
  double r = std::sqrt(INDEX_ROW_NODES / (2.0 * rho));
  r = std::min(r, (double)E->dp.factor * (double)E->dp.breakage);
  return (float)(std::ceil(r / 50.0) * 50.0);
}

// Bounded route index: part of flattening the graph into HBM, like the tile
// preprocessing behind valhalla.Configure (py/reporter_service.py:279).  One
// row per search source of the turn-aware route rule (DESIGN.md §3 rule 4):
// row e (< E) = the search from edge e's end node entered along e, row E + u =
// the search from node u with no heading (node candidates); a row holds every
// label within cost rmax x 64 (edge departure and node arrival labels) with
// its cost, route distance, turn units and predecessor edge, in a per-row
// open-addressing table.  Two passes of the same deterministic search: count,
// size + scan, insert.
namespace {
struct IndexBuilt {
  DevIndex X{};
  int64_t entries = 0, slots = 0;
  int32_t incomplete = 0;
};
// One index at radius *r: count, size + scan, insert.  The tables take the
// faster load (index_load_fast, 30 %) when they fit `budget`, else the denser
// (index_load_dense, 40 %: 40 B per entry).  With `shrink`, a radius whose
// dense tables still exceed `budget` is cut (rows shrink as R^2; the tables
// stay dense) and counted again, down to 100 m (then no index: *r = 0);
// without, such an index is left out (*r = 0).
int build_index_at(otm_engine* E, float* r, bool shrink, size_t budget, IndexBuilt& out, std::string* err) {
  out = IndexBuilt{};
  const int32_t N = E->g.n_edges + E->g.n_nodes;  // rows
  hipStream_t s = E->stream;
  int32_t* row_cnt = nullptr;
  int64_t* row_off = nullptr;
  IdxRow* rows = nullptr;
  HIPCHK(hipMalloc(&row_cnt, ((size_t)N + 1) * 4));
  HIPCHK(hipMalloc(&row_off, ((size_t)N + 1) * 8));
  HIPCHK(hipMalloc(&rows, ((size_t)N + 1) * sizeof(IdxRow)));
  size_t tmpb = scan_tmp_bytes(N) + 256;
  void* tmp = nullptr;
  HIPCHK(hipMalloc(&tmp, tmpb));
  int64_t total = 0;
  int pct = index_load_fast();
  auto size_rows = [&](int load) -> int {
    launch_row_sizes(row_cnt, row_off, N, load, s);
    scan_i64(row_off, N, tmp, tmpb, s);
    launch_row_pack(row_cnt, row_off, rows, N, s);
    HIPCHK(hipMemcpyAsync(&total, row_off + N, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return OTM_OK;
  };
  for (int attempt = 0;; ++attempt) {
    launch_index_build(E->g, E->dp.turn_units, index_cost_bound(*r), row_cnt, nullptr, nullptr, false, s);
    if (size_rows(pct)) return OTM_EDEVICE;
    if (pct != index_load_dense() && ((double)total + 1.0) * IDX_SLOT_BYTES > (double)budget) {
      // the same rows, denser tables -- and denser from here on: a radius
      // cut below costs the online tiers far more than the denser probes
      pct = index_load_dense();
      if (size_rows(pct)) return OTM_EDEVICE;
    }
    const double need = ((double)total + 1.0) * IDX_SLOT_BYTES;
    if (need <= (double)budget) break;
    const float rr = (float)(std::floor(*r * std::sqrt((double)budget / need) * 0.9 / 50.0) * 50.0);
    if (!shrink || attempt == 4 || rr < 100.0f) {
      (void)hipFree(tmp);
      (void)hipFree(rows);
      (void)hipFree(row_off);
      (void)hipFree(row_cnt);
      *r = 0.0f;  // no index
      return OTM_OK;
    }
    *r = rr;
  }
  (void)hipFree(tmp);
  E->graph_allocs.push_back(row_cnt);
  E->graph_allocs.push_back(row_off);
  E->graph_allocs.push_back(rows);
  void* slot = nullptr;
  HIPCHK(hipMalloc(&slot, ((size_t)total + 1) * IDX_SLOT_BYTES));
  E->graph_allocs.push_back(slot);
  HIPCHK(hipMemsetAsync(slot, 0xFF, ((size_t)total + 1) * IDX_SLOT_BYTES, s));
  launch_index_build(E->g, E->dp.turn_units, index_cost_bound(*r), row_cnt, rows, (uint4*)slot, true, s);
  HIPCHK(hipGetLastError());
  std::vector<int32_t> cnt((size_t)N);
  HIPCHK(hipMemcpyAsync(cnt.data(), row_cnt, (size_t)N * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (int32_t c : cnt) {
    out.incomplete += c < 0;
    out.entries += c > 0 ? c : 0;
  }
  out.slots = total;
  out.X.rmax = *r;
  out.X.cmax = index_cost_bound(*r);
  out.X.row = rows;
  out.X.slot = (const uint4*)slot;
  out.X.load_pct = pct;
  return OTM_OK;
}

// free HBM / 2, or OTM_INDEX_BUDGET_MB
size_t index_budget() {
  if (const char* bm = std::getenv("OTM_INDEX_BUDGET_MB")) return (size_t)std::strtoull(bm, nullptr, 0) << 20;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return 0;
  return fr / 2;
}
}  // namespace

int build_index(otm_engine* E, std::string* err) {
  E->idx = DevIndex{};
  for (auto& x : E->idxn) x = DevIndex{};
  E->idx.rmax = 0.0f;
  if (E->index_rmax < 0.0f) E->index_rmax = auto_index_radius(E);
  E->index_rmax = std::min(E->index_rmax, INDEX_RMAX_CAP);  // (slot costs below 2^24)
  if (!(E->index_rmax > 0.0f)) return OTM_OK;
  hipStream_t s = E->stream;
  hipEvent_t a, z;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&z));
  HIPCHK(hipEventRecord(a, s));
  // HBM budget for the slot tables (16 B per slot, the predecessor inside):
  // half of what is free after the graph.  A graph whose rows at
  // this radius exceed it gets a smaller radius; below 100 m the index is left
  // off and the online tiers answer everything (same results, slower).
  IndexBuilt full;
  int rc = build_index_at(E, &E->index_rmax, true, index_budget(), full, err);
  if (rc != OTM_OK) return rc;
  E->idx = full.X;
  E->index_entries = full.entries;
  E->index_slots = full.slots;
  E->index_incomplete_rows = full.incomplete;
  // the near indexes: the same rows at smaller radii, each for the columns
  // whose bound it is the smallest to cover (its tables a fraction of the
  // size, so their probes share lines and cache); one that does not fit what
  // is left is skipped
  std::vector<float> radii;
  if (E->index_near_set) {
    radii = E->index_near_m;
  } else if ((double)full.slots * IDX_SLOT_BYTES >= OTM_INDEX_NEAR_MIN_GB * 1e9) {
    for (float f : std::initializer_list<float> OTM_INDEX_NEAR_FRACS) radii.push_back(E->index_rmax * f);
  }
  for (float& r : radii) r = (float)(std::floor(r / 50.0) * 50.0);
  std::sort(radii.begin(), radii.end());
  radii.erase(std::unique(radii.begin(), radii.end()), radii.end());
  int nl = 0;
  for (float rn : radii) {
    if (nl == NEAR_LEVELS || !(E->idx.rmax > 0.0f) || rn < 100.0f || rn >= E->idx.rmax) continue;
    IndexBuilt near;
    rc = build_index_at(E, &rn, false, index_budget(), near, err);
    if (rc != OTM_OK) return rc;
    if (rn > 0.0f) {
      E->index_near_level_entries[nl] = near.entries;
      E->index_near_slots += near.slots;
      E->idxn[nl++] = near.X;
    }
  }
  HIPCHK(hipEventRecord(z, s));
  HIPCHK(hipEventSynchronize(z));
  HIPCHK(hipEventElapsedTime(&E->index_build_ms, a, z));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(z);
  return OTM_OK;
}

void engine_free(otm_engine* E) {
  if (E->device >= 0) (void)hipSetDevice(E->device);
  for (void* p : E->graph_allocs) (void)hipFree(p);
  E->graph_allocs.clear();
  otm_engine::Buf* bufs[] = {
      &E->in_off,        &E->in_lat,       &E->in_lon,         &E->in_time,        &E->in_acc,     &E->in_blob,
      &E->pt_trace,
      &E->is_col,        &E->prevc,        &E->nextc,        &E->gc,             &E->ncand,          &E->cand_eo,      &E->cand_em,
      &E->cand_xeo,      &E->cand_xem,
      &E->probe,         &E->col_prev,     &E->kq_prev,        &E->vmeta,  &E->colrec, &E->colrec_pos,        &E->trans_off,      &E->trans,          &E->bp,         &E->state,      &E->chosen,
      &E->chain_start,   &E->route_dist,   &E->ipos,   &E->path_off,       &E->path_len,       &E->path_pool,  &E->trace_err,
      &E->overflow_list0, &E->overflow_list2, &E->counters_i32, &E->scan_tmp, &E->snap,   &E->big_key,
      &E->big_lab,       &E->big_inq,      &E->big_fr,         &E->big_ins,        &E->big_prev,
      &E->huge_key,      &E->huge_lab,     &E->huge_inq,       &E->huge_fr,        &E->huge_ins,         &E->huge_prev,
      &E->cbig_key,      &E->cbig_val,     &E->cbig_skey,
      &E->overflow_list3, &E->o_traces,       &E->o_seg_cnt,  &E->o_way_cnt,
      &E->o_segments,    &E->o_seg_gidx,   &E->o_way_ids,      &E->o_reports,  &E->o_rep_cnt,  &E->seg_ub,
      &E->f_seg_off,     &E->f_way_off,    &E->f_rep_off,      &E->f_segs,     &E->f_ways,     &E->f_reps,
      &E->f_traces,
      &E->abort_flag,    &E->rs_blob,      &E->ord_tile,      &E->ord_cnt,      &E->ord_cursor,     &E->ord_grp,    &E->ord_item,
      &E->d_req,         &E->req_cnt,      &E->req_ok,     &E->req_lat,    &E->req_lon,    &E->req_time,   &E->req_acc,
      &E->resp_hdr,      &E->resp_seg,     &E->resp_rep,       &E->resp_hlen,      &E->resp_slen,  &E->resp_rlen,
      &E->resp_blen,     &E->resp_host,    &E->resp_blob};
  for (auto* b : bufs) {
    if (b->p) (void)hipFree(b->p);
    b->p = nullptr;
    b->cap = 0;
  }
  for (auto* b : {&E->h_traces, &E->h_segs, &E->h_reps_dense, &E->h_ways, &E->h_tot, &E->h_in, &E->h_status,
                  &E->h_req, &E->h_req_ok, &E->h_resp, &E->h_resp_meta}) {
    if (b->p) (void)hipHostFree(b->p);
    b->p = nullptr;
    b->cap = 0;
  }
  if (E->sync_ev) (void)hipEventDestroy(E->sync_ev);
  E->sync_ev = nullptr;
  for (hipEvent_t ev : E->req_ev) (void)hipEventDestroy(ev);
  E->req_ev.clear();
  if (E->req_copy) (void)hipStreamDestroy(E->req_copy);
  E->req_copy = nullptr;
  if (E->ctr) (void)hipFree(E->ctr);
  if (E->ctr_save) (void)hipFree(E->ctr_save);
  E->ctr = E->ctr_save = nullptr;
  for (auto& e : E->kev)
    if (e) (void)hipEventDestroy(e);
  if (E->stream) (void)hipStreamDestroy(E->stream);
  E->stream = nullptr;
}

// The growth cap of an on-demand tier (log2 of its table slots): the
// kernels.h default, or lower by env (a test hook)
static int max_log2(const char* env, int dflt) {
  const char* v = std::getenv(env);
  return v ? std::min(dflt, std::atoi(v)) : dflt;
}

// The candidate HBM tier's tables (kernels.h CAND_BIG_SLOTS): none until a
// probe outgrows the LDS tier; k_candidates<true> clears them per probe.
static int ensure_cand(otm_engine* E, std::string* err) {
  if (E->cand_log2 <= 0) return OTM_OK;
  const size_t n = (size_t)CAND_BIG_SLOTS << E->cand_log2;
  int rc;
  if ((rc = ensure_grow(E->cbig_key, n * 4, err))) return rc;
  if ((rc = ensure_grow(E->cbig_val, n * 8, err))) return rc;
  if ((rc = ensure_grow(E->cbig_skey, n / 2 * 8, err))) return rc;
  return OTM_OK;
}

// The huge search tier's tables (kernels.h HUGE_SLOTS): none until a search
// outgrows the global tier; then 2^huge_log2 slots each, grown 4x and the batch
// redone whenever a search does not fit (engine_match).
static int ensure_huge(otm_engine* E, std::string* err) {
  if (E->huge_log2 <= 0) return OTM_OK;
  const size_t n = (size_t)HUGE_SLOTS << E->huge_log2;
  int rc;
  if ((rc = ensure_grow(E->huge_key, n * 4, err))) return rc;
  if ((rc = ensure_grow(E->huge_lab, n * 8, err))) return rc;
  if ((rc = ensure_grow(E->huge_inq, n * 4, err))) return rc;
  if ((rc = ensure_grow(E->huge_fr, n * 8, err))) return rc;
  if ((rc = ensure_grow(E->huge_ins, (size_t)HUGE_SLOTS * huge_limit(E->huge_log2) * 4, err))) return rc;
  if ((rc = ensure_grow(E->huge_prev, (size_t)HUGE_SLOTS * 4, err))) return rc;
  if (E->huge_ready_log2 != E->huge_log2) {
    // (re)sized tables start clean, their "last inserted" lists marking the
    // whole table for the first search (-1)
    E->huge_ready_log2 = E->huge_log2;
    HIPCHK(hipMemsetAsync(E->huge_key.p, 0xFF, n * 4, E->stream));
    HIPCHK(hipMemsetAsync(E->huge_lab.p, 0xFF, n * 8, E->stream));
    HIPCHK(hipMemsetAsync(E->huge_inq.p, 0, n * 4, E->stream));
    HIPCHK(hipMemsetAsync(E->huge_prev.p, 0xFF, (size_t)HUGE_SLOTS * 4, E->stream));
  }
  return OTM_OK;
}

static int ensure_big(otm_engine* E, std::string* err) {
  const size_t n = (size_t)BIG_SLOTS * BIG_TABLE_CAP;
  int rc;
  const void* before = E->big_prev.p;
  if ((rc = ensure(E->big_key, n * 4, err))) return rc;
  if ((rc = ensure(E->big_lab, n * 8, err))) return rc;
  if ((rc = ensure(E->big_inq, n * 4, err))) return rc;
  if ((rc = ensure(E->big_fr, n * 8, err))) return rc;
  if ((rc = ensure(E->big_ins, (size_t)BIG_SLOTS * SEARCH_LIMIT * 4, err))) return rc;
  if ((rc = ensure(E->big_prev, (size_t)BIG_SLOTS * 4, err))) return rc;
  if (E->big_prev.p != before) {
    // fresh tables start clean (each search then clears only what the last
    // one inserted: kernels.hip ta_search)
    HIPCHK(hipMemsetAsync(E->big_key.p, 0xFF, n * 4, E->stream));
    HIPCHK(hipMemsetAsync(E->big_lab.p, 0xFF, n * 8, E->stream));
    HIPCHK(hipMemsetAsync(E->big_inq.p, 0, n * 4, E->stream));
    HIPCHK(hipMemsetAsync(E->big_prev.p, 0, (size_t)BIG_SLOTS * 4, E->stream));
  }
  return OTM_OK;
}

// One attempt at a batch, enqueued with no host synchronisation: buffers are
// sized from capacities (transition matrices, path pool) that the kernels
// check; an overflow sets w.abort, every later kernel returns at once, and
// engine_match grows the capacity and runs the batch again -- whole
// (from = RESUME_ALL), or from the on-demand tier that overflowed (Resume).
static int engine_match_once(otm_engine* E, const DevBatch& b, hipStream_t s, std::string* err,
                             int from = RESUME_ALL) {
  const int64_t NP = b.n_points;
  const int32_t NT = b.n_traces;
  const size_t Pn = (size_t)NP + 1;
  int rc;
#define ENS(buf, bytes) \
  if ((rc = ensure(E->buf, (bytes), err))) return rc;
  ENS(pt_trace, Pn * 4);
  ENS(is_col, Pn);
  ENS(prevc, Pn * 4);
  ENS(nextc, Pn * 4);
  ENS(gc, Pn * 4);
  ENS(ncand, Pn * 4);
  ENS(cand_eo, Pn * KIN * 8);  // inline candidate slots {edge, offset bits}
  ENS(cand_em, Pn * KIN * 4);  //   ... and their emissions
  ENS(cand_xeo, Pn * KX * 8);  // slots KIN.. (only the wider points touch them)
  ENS(cand_xem, Pn * KX * 4);
  ENS(probe, Pn * 16);
  ENS(col_prev, Pn * 4);
  ENS(kq_prev, Pn * 4);
  ENS(vmeta, Pn);
  ENS(colrec, Pn * 16);
  ENS(colrec_pos, Pn * 4);
  ENS(trans_off, Pn * 8);
  ENS(bp, Pn * KMAX);
  ENS(state, Pn * 4);
  ENS(chosen, Pn * 8);
  ENS(chain_start, Pn);
  ENS(route_dist, Pn * 4);
  ENS(ipos, Pn * 4);
  ENS(path_off, Pn * 4);
  ENS(path_len, Pn * 4);
  ENS(trace_err, ((size_t)NT + 1) * 4);
  ENS(overflow_list0, Pn * 4);
  ENS(overflow_list2, Pn * 4);
  ENS(overflow_list3, Pn * 4);
  ENS(counters_i32, 64 * 4);  // 64 counters (kernels.h DevWork::counters_i32)
  ENS(snap, 192 + sizeof(BatchStatus));
  ENS(abort_flag, 16);
  // Capacities of the transition matrices and the path pool: sized from the
  // batch (kept at the largest seen), so the abort -> regrow -> redo loop of
  // engine_match is the exception.  OTM_TRANS_CAP / OTM_POOL_CAP pin the
  // starting capacities instead (tests force the redo path with tiny ones).
  if (!E->caps_read) {
    E->caps_read = true;
    if (const char* v = std::getenv("OTM_TRANS_CAP")) E->trans_cap = std::max<int64_t>(1, std::atoll(v)), E->caps_pinned = true;
    if (const char* v = std::getenv("OTM_POOL_CAP")) E->pool_cap = (int32_t)std::max(1, std::atoi(v)), E->caps_pinned = true;
  }
  if (!E->caps_pinned) {
    E->trans_cap = std::max<int64_t>(E->trans_cap, (int64_t)Pn * 48 + 4096);
    E->pool_cap = std::max<int32_t>(E->pool_cap, (int32_t)std::min<size_t>(Pn * 8, (size_t)1 << 30));
  }
  ENS(o_traces, ((size_t)NT + 1) * sizeof(otm_trace_result));
  ENS(o_seg_cnt, ((size_t)NT + 1) * 4);
  ENS(o_way_cnt, ((size_t)NT + 1) * 4);
  ENS(scan_tmp, scan_tmp_bytes(NP > NT ? NP : NT) + 256);
  ENS(path_pool, (size_t)E->pool_cap * 4);

  // Small batches (the batcher's rounds) are latency bound: too few probes
  // to hide a lane's serial cell walk, and the spatial order's fixed cost
  // buys nothing.  They run in natural order with one wave per probe.
  DevParams dp = E->dp;
  if (NP < E->small_points) {
    dp.order_mask = 0;
    dp.cand_wave_all = 1;
  }

  DevWork w{};
  w.pt_trace = P<int32_t>(E->pt_trace);
  w.is_col = P<uint8_t>(E->is_col);
  w.prevc = P<int32_t>(E->prevc);
  w.nextc = P<int32_t>(E->nextc);
  w.gc = P<float>(E->gc);
  w.ncand = P<int32_t>(E->ncand);
  w.probe = P<float4>(E->probe);
  w.cand_eo = P<int2>(E->cand_eo);
  w.cand_em = P<float>(E->cand_em);
  w.cand_xeo = P<int2>(E->cand_xeo);
  w.cand_xem = P<float>(E->cand_xem);
  w.col_prev = P<int32_t>(E->col_prev);
  w.kq_prev = P<int32_t>(E->kq_prev);
  w.vmeta = P<uint8_t>(E->vmeta);
  {
    // ordered column records for K4 (spatial-order batches; the others read
    // the per-point arrays)
    w.colrec = P<int4>(E->colrec);
    w.colrec_pos = P<int32_t>(E->colrec_pos);
  }
  w.trans_off = P<int64_t>(E->trans_off);
  w.bp = P<uint8_t>(E->bp);
  w.state = P<int32_t>(E->state);
  w.chosen = P<int2>(E->chosen);
  w.chain_start = P<uint8_t>(E->chain_start);
  w.route_dist = P<float>(E->route_dist);
  w.ipos = P<float>(E->ipos);
  w.path_off = P<int32_t>(E->path_off);
  w.path_len = P<int32_t>(E->path_len);
  w.path_pool = P<int32_t>(E->path_pool);
  w.pool_cap = E->pool_cap;
  w.trace_err = P<int32_t>(E->trace_err);
  w.overflow_list0 = P<int32_t>(E->overflow_list0);
  w.overflow_list2 = P<int32_t>(E->overflow_list2);
  w.overflow_list3 = P<int32_t>(E->overflow_list3);
  w.idx = E->idx;
  for (int l = 0; l < NEAR_LEVELS; ++l) w.idxn[l] = E->idxn[l];
  w.counters_i32 = P<int32_t>(E->counters_i32);
  w.snap = P<int32_t>(E->snap);
  w.ctr = E->counting ? E->ctr : nullptr;
  if (E->counting && from == RESUME_ALL) HIPCHK(hipMemsetAsync(E->ctr, 0, sizeof(DevCounters), s));
  w.abort = P<int32_t>(E->abort_flag);
  // the counters' and abort flag's reset, the spill snapshots and the
  // transition capacity check ride in K1, K3, K4, K5 and K7 (OTM_FOLD_BOOKKEEPING)
  if (!fold_bookkeeping()) launch_batch_init(w.counters_i32, w.abort, s);  // [5] = candidate spill count
  Marks mk;
  mk.ev = E->timing ? E->kev : nullptr;
  ENS(ord_tile, Pn * 2);
  ENS(ord_cnt, ORDER_TILES * 4);
  ENS(ord_cursor, ORDER_TILES * 4);
  ENS(ord_grp, (ORDER_GROUPS + 1) * 4);
  ENS(ord_item, Pn * 4);
  w.ord.item = P<int32_t>(E->ord_item);
  w.ord.grp = P<int32_t>(E->ord_grp);
  w.ord.tile = P<uint16_t>(E->ord_tile);
  w.ord.tile_cnt = dp.order_mask ? P<int32_t>(E->ord_cnt) : nullptr;
  w.ord.cursor = P<int32_t>(E->ord_cursor);
  if (from == RESUME_ALL) {
    launch_columns(E->g, b, dp, w, s, mk);
    if (dp.order_mask) {
      launch_order(b, w, s, mk);
    } else if (E->timing) {
      mk.begin(KN_ORDER, s);
      mk.end(KN_ORDER, s);
    }
  }
  if ((rc = ensure_cand(E, err))) return rc;
  w.cand_final = E->cand_final;
  w.cbig_key = P<uint32_t>(E->cbig_key);
  w.cbig_val = P<unsigned long long>(E->cbig_val);
  w.cbig_skey = P<unsigned long long>(E->cbig_skey);
  w.cand_log2 = E->cand_log2;
  if (from <= RESUME_CAND_BIG) launch_candidates(E->g, b, dp, w, s, mk, from);
  // spill snapshot A: candidate probes the lane tier handed to the wave tier;
  // the counters start over for the transition tiers (links, scan and the
  // capacity check do not touch them)
  if (!fold_bookkeeping()) launch_snap(w.counters_i32, P<int32_t>(E->snap), true, s);
  if (from <= RESUME_CAND_BIG) {
    launch_links(b, dp, w, s, mk);
    mk.begin(KN_SCAN_TRANS, s);
    scan_i64(w.trans_off, NP, E->scan_tmp.p, E->scan_tmp.cap, s);
    mk.end(KN_SCAN_TRANS, s);
  }
  ENS(trans, ((size_t)E->trans_cap + 1) * 4);
  w.trans = P<float>(E->trans);
  w.trans_cap = E->trans_cap;
  if (!fold_bookkeeping()) launch_cap_check(b, w, s);
  if ((rc = ensure_big(E, err))) return rc;
  w.big_key = P<uint32_t>(E->big_key);
  w.big_lab = P<unsigned long long>(E->big_lab);
  w.big_inq = P<uint32_t>(E->big_inq);
  w.big_fr = P<uint32_t>(E->big_fr);
  w.big_ins = P<uint32_t>(E->big_ins);
  w.big_prev = P<int32_t>(E->big_prev);
  if ((rc = ensure_huge(E, err))) return rc;
  w.huge_key = P<uint32_t>(E->huge_key);
  w.huge_lab = P<unsigned long long>(E->huge_lab);
  w.huge_inq = P<uint32_t>(E->huge_inq);
  w.huge_fr = P<uint32_t>(E->huge_fr);
  w.huge_ins = P<uint32_t>(E->huge_ins);
  w.huge_prev = P<int32_t>(E->huge_prev);
  w.huge_log2 = E->huge_log2;
  w.huge_final = E->huge_final;
  if (from <= RESUME_TRANS_HUGE) launch_transitions(E->g, b, dp, w, s, mk, E->trans_lanes, from);
  // spill snapshot B: columns per transition tier (Viterbi does not touch
  // the counters; they start over for the route tiers)
  if (!fold_bookkeeping()) launch_snap(w.counters_i32, P<int32_t>(E->snap) + 16, true, s);
  if (from <= RESUME_TRANS_HUGE) launch_viterbi(b, w, s, mk);
  launch_route(E->g, b, dp, w, s, mk, from);
  // spill snapshot C: steps per route tier
  if (!fold_bookkeeping()) launch_snap(w.counters_i32, P<int32_t>(E->snap) + 32, false, s);

  // Segments, way ids and reports in ONE walk per trace, each trace writing
  // into a region sized by an upper bound (DevOut): every matched point adds
  // <= 2 + its path length, and the path lengths sum to at most the pool.
  const size_t cap = 2 * (size_t)NP + (size_t)E->pool_cap + 1;
  if (cap >= (size_t)INT32_MAX) {
    *err = "batch too large for one launch (segment regions exceed 2^31)";
    return OTM_EINVAL;
  }
  ENS(seg_ub, ((size_t)NT + 1) * 8);
  ENS(o_segments, cap * sizeof(otm_segment));
  ENS(o_seg_gidx, cap * 4);
  ENS(o_reports, cap * sizeof(otm_report_rec));
  ENS(o_way_ids, cap * 8);
  ENS(o_rep_cnt, ((size_t)NT + 1) * 4);
  DevOut o{};
  o.traces = E->o_traces.p;
  o.seg_cnt = P<int32_t>(E->o_seg_cnt);
  o.way_cnt = P<int32_t>(E->o_way_cnt);
  o.rep_cnt = P<int32_t>(E->o_rep_cnt);
  o.seg_base = P<int64_t>(E->seg_ub);
  o.segments = E->o_segments.p;
  o.seg_gidx = P<int32_t>(E->o_seg_gidx);
  o.reports = E->o_reports.p;
  o.way_ids = P<int64_t>(E->o_way_ids);
  {
    // the histogram binding lives on the parent; a clone reads it here
    otm_engine* H = E->parent ? const_cast<otm_engine*>(E->parent) : E;
    std::lock_guard<std::mutex> lk(H->hist_mu);
    o.hist = H->hist;
    o.speed_sum = H->speed_sum;
    o.nbins = H->nbins;
    o.bin_kph = H->bin_kph;
  }
  HIPCHK(hipMemsetAsync(E->seg_ub.p, 0, ((size_t)NT + 1) * 8, s));
  launch_seg_bound(E->g, b, dp, w, P<int64_t>(E->seg_ub), s, mk);
  mk.begin(KN_SEG_SCAN, s);
  scan_i64(P<int64_t>(E->seg_ub), NT, E->scan_tmp.p, E->scan_tmp.cap, s);
  mk.end(KN_SEG_SCAN, s);
  launch_segments(E->g, b, w, o, true, s, mk);
  launch_report(b, E->drc, w, o, s, mk);
  HIPCHK(hipGetLastError());
  E->last_T = NT;
  E->last_P = NP;
  E->last_S = -1;  // known after compaction (engine_fetch)
  E->last_W = -1;
#undef ENS
  return OTM_OK;
}

int engine_match(otm_engine* E, const DevBatch& b, hipStream_t s, std::string* err) {
  if (!s) s = E->stream;
  const int64_t NP = b.n_points;
  int rc;
  // A tier that ran out of HBM fails its overflowing traces for this batch
  // only: the next batch tries to grow it again (the growth cap, by contrast,
  // is final).  The guard lifts the batch's flags on every way out.
  struct OomGuard {
    otm_engine* E;
    bool huge = false, cand = false;
    ~OomGuard() {
      if (huge) E->huge_final = 0;
      if (cand) E->cand_final = 0;
    }
  } oom{E};
  int from = RESUME_ALL;
  E->last_resumes = 0;
  for (int attempt = 0;; ++attempt) {
    if ((rc = engine_match_once(E, b, s, err, from))) return rc;
    // the one synchronisation of a batch: did every capacity hold?
    // (gathered on the device, one copy into pinned memory)
    if ((rc = ensure_pinned(E->h_status, sizeof(BatchStatus), err))) return rc;
    BatchStatus* dst = (BatchStatus*)(P<char>(E->snap) + 192);
    launch_status(P<int32_t>(E->abort_flag), P<int64_t>(E->trans_off) + NP, P<int32_t>(E->counters_i32), dst, s);
    HIPCHK(hipMemcpyAsync(E->h_status.p, dst, sizeof(BatchStatus), hipMemcpyDeviceToHost, s));
    HIPCHK(wait_batch(E, s, NP));
    const BatchStatus st = *(const BatchStatus*)E->h_status.p;
    const int32_t ab = st.abort;
    const int64_t ttotal = st.ttotal;
    const int32_t cnt[3] = {st.cnt[0], st.cnt[1], st.cnt[2]};
    E->last_trans = ttotal;
    E->last_attempts = attempt + 1;
    if (!ab) break;
    if (attempt == 16) {
      *err = "batch capacities could not be sized";
      return OTM_EDEVICE;
    }
    if (ttotal > E->trans_cap) E->trans_cap = ttotal + ttotal / 4 + 4096;
    if (st.grow & 1) {
      // a search outgrew the huge tier's tables (or found none): 4x the slots,
      // or, past the cap or out of HBM, the overflowing traces fail alone
      const int32_t next = E->huge_log2 ? E->huge_log2 + 2 : 19;
      const int32_t prev = E->huge_log2;
      if (next > max_log2("OTM_HUGE_MAX_LOG2", HUGE_MAX_LOG2)) {
        E->huge_final = 1;
      } else {
        E->huge_log2 = next;
        if (ensure_huge(E, err) != OTM_OK) {
          E->huge_log2 = prev;
          E->huge_final = 1;
          oom.huge = true;
          E->huge_ready_log2 = 0;  // (a buffer regrown before the failure: cleared again)
          err->clear();
        }
      }
    }
    if (st.grow & 2) {
      // a probe had more distinct edges in its radius than the candidate
      // HBM tier's tables hold (or there were none): 4x the slots, or the
      // overflowing traces fail alone
      const int32_t next = E->cand_log2 ? E->cand_log2 + 2 : 13;
      const int32_t prev = E->cand_log2;
      if (next > max_log2("OTM_CAND_MAX_LOG2", CAND_MAX_LOG2)) {
        E->cand_final = 1;
      } else {
        E->cand_log2 = next;
        if (ensure_cand(E, err) != OTM_OK) {
          E->cand_log2 = prev;
          E->cand_final = 1;
          oom.cand = true;
          err->clear();
        }
      }
    }
    if (cnt[2]) E->pool_cap = (int32_t)std::min<size_t>((size_t)cnt[1] * 2 + 1024, (size_t)INT32_MAX / 2);
    // Where to resume: a matrix or path-pool overflow redoes
    // the whole batch (those buffers are reallocated); a tier whose tables
    // grew -- candidate HBM tier, or the huge search tier of the transition
    // or route stage -- runs again from itself: every earlier stage finished
    // and kept its results, every later one returned at once on the abort.
    // The spill counters go back to the snapshot the aborted attempt took at
    // that stage's boundary (A after the candidates, B after the transitions,
    // C after the routes), so the resumed kernels retake the same snapshots.
    const char* nr = std::getenv("OTM_NO_RESUME");  // A/B knob: every redo whole (rounds 1-5)
    const bool whole = !fold_bookkeeping() || ttotal > E->trans_cap || cnt[2] || !(st.grow & 3) ||
                       (nr && *nr && *nr != '0');
    from = whole ? RESUME_ALL
                 : (st.grow & 2) ? RESUME_CAND_BIG : (st.route_huge ? RESUME_ROUTE_HUGE : RESUME_TRANS_HUGE);
    if (from != RESUME_ALL) {
      const int snap = from == RESUME_CAND_BIG ? 0 : (from == RESUME_TRANS_HUGE ? 16 : 32);
      int32_t* ctr = P<int32_t>(E->counters_i32);
      HIPCHK(hipMemcpyAsync(ctr, P<int32_t>(E->snap) + snap, 16 * 4, hipMemcpyDeviceToDevice, s));
      HIPCHK(hipMemsetAsync(ctr + 23, 0, 4, s));  // the grow flags
      HIPCHK(hipMemsetAsync(ctr + 25, 0, 4, s));
      HIPCHK(hipMemsetAsync(E->abort_flag.p, 0, 4, s));
      E->last_resumes += 1;
    }
  }
  if (E->timing) {
    // kernel-only spans on the launch stream (the final attempt).  Stages are sums of their
    // kernels: columns | candidates (lane + wave tier) | links + scan |
    // transitions (index, lane, wave, global tiers) | viterbi | route (4 tiers)
    // | segments count + scans | segments write + report
    HIPCHK(hipEventSynchronize(E->kev[2 * KN_REPORT + 1]));
    for (int k = 0; k < KN_COUNT; ++k)
      HIPCHK(hipEventElapsedTime(&E->kernel_ms[k], E->kev[2 * k], E->kev[2 * k + 1]));
    const int first[8] = {KN_COLUMNS, KN_ORDER, KN_LINKS, KN_TRANS_INDEX, KN_VITERBI, KN_ROUTE_INDEX, KN_SEG_BOUND,
                          KN_SEG_WRITE};
    const int last[8] = {KN_COLUMNS, KN_CAND_WAVE, KN_SCAN_TRANS, KN_TRANS_GLOBAL, KN_VITERBI, KN_ROUTE_GLOBAL,
                         KN_SEG_SCAN, KN_REPORT};
    for (int k = 0; k < 8; ++k) {
      E->stage_ms[k] = 0.0f;
      for (int q = first[k]; q <= last[k]; ++q) E->stage_ms[k] += E->kernel_ms[q];
    }
  }
#undef ENS
  return OTM_OK;
}

// The large host<->device copies: hipMemcpyAsync on the batch's stream.
// Measured and not kept (profiles/r02_hostleg_ab/): a copy
// engine through hipMemcpyDeviceToDeviceNoCU, copies taking turns across the
// batch contexts, hipMemcpyWithStream, and the library's own copy kernel with
// 16-128 workgroups -- the leg runs at the sum of its PCIe bytes and kernels;
// round 5: the D2H copies on a stream of their own, and the library's copy
// kernel (16-64 workgroups) for the D2H copies -- both slower.
static hipError_t big_copy(void* dst, const void* src, size_t n, hipMemcpyKind k, hipStream_t s) {
  return hipMemcpyAsync(dst, src, n, k, s);
}

int engine_match_host(otm_engine* E, const otm_batch* in, std::string* err) {
  const int32_t NT = in->n_traces;
  if (NT < 0 || !in->trace_off) {
    *err = "invalid batch";
    return OTM_EINVAL;
  }
  const int64_t NP = in->trace_off[NT];
  if (in->trace_off[0] != 0 || NP < 0 || (in->n_points && in->n_points != NP)) {
    *err = "batch trace_off inconsistent with n_points";
    return OTM_EINVAL;
  }
  for (int32_t t = 0; t < NT; ++t)
    if (in->trace_off[t + 1] < in->trace_off[t]) {
      *err = "batch trace_off not monotonic";
      return OTM_EINVAL;
    }
  int rc;
  if ((rc = ensure(E->in_off, ((size_t)NT + 1) * 8, err))) return rc;
  if ((rc = ensure(E->in_lat, (size_t)NP * 4, err))) return rc;
  if ((rc = ensure(E->in_lon, (size_t)NP * 4, err))) return rc;
  if ((rc = ensure(E->in_time, (size_t)NP * 8, err))) return rc;
  if ((rc = ensure(E->in_acc, (size_t)NP * 4, err))) return rc;
  hipStream_t s = E->stream;
  const size_t b_off = ((size_t)NT + 1) * 8, b_pt = (size_t)NP * 4, b_tm = (size_t)NP * 8;
  DevBatch b;
  b.n_traces = NT;
  b.n_points = NP;
  if (NP <= (int64_t)1 << 18) {
    // small batches: one host copy into pinned staging, then ONE DMA into a
    // device blob laid out the same way (offsets, times, lat, lon, accuracy:
    // every section stays 8-byte aligned) -- the batcher's rounds, single requests
    const size_t total = b_off + b_tm + 3 * b_pt;
    if ((rc = ensure_pinned(E->h_in, total, err))) return rc;
    if ((rc = ensure(E->in_blob, total, err))) return rc;
    char* h = (char*)E->h_in.p;
    std::memcpy(h, in->trace_off, b_off);
    if (NP) {
      std::memcpy(h + b_off, in->time, b_tm);
      std::memcpy(h + b_off + b_tm, in->lat, b_pt);
      std::memcpy(h + b_off + b_tm + b_pt, in->lon, b_pt);
      std::memcpy(h + b_off + b_tm + 2 * b_pt, in->accuracy, b_pt);
    }
    HIPCHK(hipMemcpyAsync(E->in_blob.p, h, total, hipMemcpyHostToDevice, s));
    const char* d = (const char*)E->in_blob.p;
    b.trace_off = (const int64_t*)d;
    b.time = (const double*)(d + b_off);
    b.lat = (const float*)(d + b_off + b_tm);
    b.lon = (const float*)(d + b_off + b_tm + b_pt);
    b.acc = (const float*)(d + b_off + b_tm + 2 * b_pt);
    return engine_match(E, b, s, err);
  }
  const hipMemcpyKind h2d = hipMemcpyHostToDevice;
  HIPCHK(hipMemcpyAsync(E->in_off.p, in->trace_off, b_off, hipMemcpyHostToDevice, s));
  HIPCHK(big_copy(E->in_lat.p, in->lat, b_pt, h2d, s));
  HIPCHK(big_copy(E->in_lon.p, in->lon, b_pt, h2d, s));
  HIPCHK(big_copy(E->in_time.p, in->time, b_tm, h2d, s));
  HIPCHK(big_copy(E->in_acc.p, in->accuracy, b_pt, h2d, s));
  b.trace_off = (const int64_t*)E->in_off.p;
  b.lat = (const float*)E->in_lat.p;
  b.lon = (const float*)E->in_lon.p;
  b.time = (const double*)E->in_time.p;
  b.acc = (const float*)E->in_acc.p;
  return engine_match(E, b, s, err);
}

// otm_match_compact: the host's compact batch (14 B per point: lat, lon,
// an int32 time delta, an int16 accuracy; a per-trace int64 time base) to
// HBM, then widened on the device (k_expand_compact) into the arrays every
// stage reads.  Same results as engine_match_host on the widened batch;
// 10 B per point less over PCIe.
// The checks of a compact batch, for one engine and a multi-device engine
// alike (n_points 0: derived from trace_off); *np = the batch's point count.
int validate_compact(const otm_batch_compact* in, int64_t* np, std::string* err) {
  const int32_t NT = in->n_traces;
  if (NT < 0 || !in->trace_off || (NT > 0 && !in->time_base)) {
    *err = "invalid batch";
    return OTM_EINVAL;
  }
  const int64_t NP = in->trace_off[NT];
  if (in->trace_off[0] != 0 || NP < 0 || (in->n_points && in->n_points != NP)) {
    *err = "batch trace_off inconsistent with n_points";
    return OTM_EINVAL;
  }
  for (int32_t t = 0; t < NT; ++t)
    if (in->trace_off[t + 1] < in->trace_off[t]) {
      *err = "batch trace_off not monotonic";
      return OTM_EINVAL;
    }
  if (NP > 0 && (!in->lat || !in->lon || !in->time_delta || !in->accuracy)) {
    *err = "invalid batch";
    return OTM_EINVAL;
  }
  *np = NP;
  return OTM_OK;
}

int engine_match_compact(otm_engine* E, const otm_batch_compact* in, std::string* err) {
  const int32_t NT = in->n_traces;
  int64_t NP = 0;
  int rc;
  if ((rc = validate_compact(in, &NP, err))) return rc;
  const size_t b_off = ((size_t)NT + 1) * 8, b_base = (size_t)NT * 8, b_pt = (size_t)NP * 4,
               b_acc = ((size_t)NP * 2 + 7) & ~(size_t)7;
  // device: [offsets | time bases | lat | lon | time deltas | accuracies], each
  // section 256-B aligned (the runtime's copy kernels take an unaligned
  // destination on a slower path), then the widened time and accuracy arrays
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_base = al(b_off), o_lat = al(o_base + b_base), o_lon = al(o_lat + b_pt), o_dt = al(o_lon + b_pt),
               o_acc = al(o_dt + b_pt);
  const size_t total = o_acc + b_acc;
  if ((rc = ensure(E->in_blob, total, err))) return rc;
  if ((rc = ensure(E->in_time, (size_t)NP * 8 + 8, err))) return rc;
  if ((rc = ensure(E->in_acc, (size_t)NP * 4 + 8, err))) return rc;
  hipStream_t s = E->stream;
  char* d = (char*)E->in_blob.p;
  if (NP <= (int64_t)1 << 18) {
    // small batches: one host copy into pinned staging, then ONE DMA
    if ((rc = ensure_pinned(E->h_in, total, err))) return rc;
    char* h = (char*)E->h_in.p;
    std::memcpy(h, in->trace_off, b_off);
    if (NT) std::memcpy(h + o_base, in->time_base, b_base);
    if (NP) {
      std::memcpy(h + o_lat, in->lat, b_pt);
      std::memcpy(h + o_lon, in->lon, b_pt);
      std::memcpy(h + o_dt, in->time_delta, b_pt);
      std::memcpy(h + o_acc, in->accuracy, (size_t)NP * 2);
    }
    HIPCHK(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, s));
  } else {
    const hipMemcpyKind h2d = hipMemcpyHostToDevice;
    HIPCHK(hipMemcpyAsync(d, in->trace_off, b_off, h2d, s));
    if (NT) HIPCHK(hipMemcpyAsync(d + o_base, in->time_base, b_base, h2d, s));
    HIPCHK(big_copy(d + o_lat, in->lat, b_pt, h2d, s));
    HIPCHK(big_copy(d + o_lon, in->lon, b_pt, h2d, s));
    HIPCHK(big_copy(d + o_dt, in->time_delta, b_pt, h2d, s));
    HIPCHK(big_copy(d + o_acc, in->accuracy, (size_t)NP * 2, h2d, s));
  }
  launch_expand_compact((const int64_t*)d, (const int64_t*)(d + o_base), (const int32_t*)(d + o_dt),
                        (const int16_t*)(d + o_acc), (double*)E->in_time.p, (float*)E->in_acc.p, NT, s);
  DevBatch b;
  b.n_traces = NT;
  b.n_points = NP;
  b.trace_off = (const int64_t*)d;
  b.lat = (const float*)(d + o_lat);
  b.lon = (const float*)(d + o_lon);
  b.time = (const double*)E->in_time.p;
  b.acc = (const float*)E->in_acc.p;
  return engine_match(E, b, s, err);
}

// The staging blob of engine_match_requests: int64 offsets[n + 1] (padded to
// 16 bytes), then the body bytes (16-byte aligned: the readers load aligned
// 16-byte words), then REQ_PAD zero bytes (the last window's loads stay inside)
static constexpr size_t REQ_PAD = 64;
static size_t req_hdr_bytes(int32_t n) { return (((size_t)n + 1) * 8 + 15) & ~(size_t)15; }
static size_t req_blob_bytes(int32_t n, size_t bytes) { return req_hdr_bytes(n) + bytes + REQ_PAD; }

int engine_stage_requests(otm_engine* E, int32_t n, size_t bytes, bool bodies, int64_t** off, char** body,
                          std::string* err) {
  int rc;
  if (n < 0) {
    *err = "invalid request count";
    return OTM_EINVAL;
  }
  // the device side for the reads behind each pushed piece
  const size_t slots = req_sparse_slots(n, bytes);
  if ((rc = ensure(E->d_req, req_blob_bytes(n, bytes), err))) return rc;
  if ((rc = ensure(E->req_cnt, ((size_t)n + 1) * 8, err))) return rc;
  if ((rc = ensure(E->req_ok, (size_t)n + 1, err))) return rc;
  if ((rc = ensure(E->req_lat, slots * 4, err))) return rc;
  if ((rc = ensure(E->req_lon, slots * 4, err))) return rc;
  if ((rc = ensure(E->req_time, slots * 8, err))) return rc;
  if ((rc = ensure(E->req_acc, slots * 4, err))) return rc;
  E->req_read = 0;
  E->req_piece = 0;
  if (!bodies) {
    // every body goes to HBM from the caller's page-locked memory: the header alone
    if ((rc = ensure_pinned(E->h_req, req_hdr_bytes(n), err))) return rc;
    *off = (int64_t*)E->h_req.p;
    *body = nullptr;
    return OTM_OK;
  }
  if ((rc = ensure_pinned(E->h_req, req_blob_bytes(n, bytes), err))) return rc;
  char* h = (char*)E->h_req.p;
  std::memset(h + req_hdr_bytes(n) + bytes, 0, REQ_PAD);
  *off = (int64_t*)h;
  *body = h + req_hdr_bytes(n);
  return OTM_OK;
}

// the device copy of the staging blob, and one piece of it on its way: body
// bytes [from, to) (with the offsets header when from == 0, the padding when
// to == bytes), so the host can stage the next piece while this one moves.
// With src (page-locked host memory holding body bytes [from, to)) the bodies
// are copied from there instead of the staging buffer.
static DevBatch req_sparse(otm_engine* E) {
  DevBatch sp{};
  sp.lat = (const float*)E->req_lat.p;
  sp.lon = (const float*)E->req_lon.p;
  sp.time = (const double*)E->req_time.p;
  sp.acc = (const float*)E->req_acc.p;
  return sp;
}

// read requests [E->req_read, upto) of the device blob (requests.hip)
static void read_requests(otm_engine* E, int32_t n, int32_t upto) {
  if (upto <= E->req_read) return;
  const unsigned char* d = (const unsigned char*)E->d_req.p;
  launch_req_read(d + req_hdr_bytes(n), (const int64_t*)d, E->req_read, upto, n, P<int64_t>(E->req_cnt),
                  P<uint8_t>(E->req_ok), req_sparse(E), E->stream);
  E->req_read = upto;
}

// The request pieces' copy stream: the async pipeline's shared one, or E's own
static hipStream_t req_copy_stream(otm_engine* E) {
  if (E->req_shared) return E->req_shared;
  if (!E->req_copy && hipStreamCreateWithFlags(&E->req_copy, hipStreamNonBlocking) != hipSuccess) return nullptr;
  return E->req_copy;
}

// The pieces go to HBM on a copy stream (E's own, or with E->req_shared the
// async pipeline's one copy stream), each followed by an event that the batch
// stream waits on before it reads the piece's requests, so one piece's read
// overlaps the next piece's copy.
int engine_push_requests(otm_engine* E, int32_t n, size_t bytes, size_t from, size_t to, const char* src,
                         int32_t upto, std::string* err) {
  hipStream_t c = req_copy_stream(E);
  if (!c) {
    *err = "no request copy stream";
    return OTM_EDEVICE;
  }
  while (E->req_ev.size() < E->req_piece + 2) {  // [0]: the fence, [1 + p]: piece p
    hipEvent_t ev = nullptr;
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    E->req_ev.push_back(ev);
  }
  char* d = (char*)E->d_req.p;
  const char* h = (const char*)E->h_req.p;
  const size_t hdr = req_hdr_bytes(n);
  const hipMemcpyKind h2d = hipMemcpyHostToDevice;
  if (E->req_piece == 0) {
    // the copies must not overtake the batch stream's earlier work on d_req
    HIPCHK(hipEventRecord(E->req_ev[0], E->stream));
    HIPCHK(hipStreamWaitEvent(c, E->req_ev[0], 0));
  }
  if (!src) {
    const size_t a = from ? hdr + from : 0;
    const size_t b = hdr + (to >= bytes ? bytes + REQ_PAD : to);
    if (b > a) HIPCHK(big_copy(d + a, h + a, b - a, h2d, c));
  } else {
    if (from == 0) HIPCHK(hipMemcpyAsync(d, h, hdr, h2d, c));
    if (to > from) HIPCHK(big_copy(d + hdr + from, src, to - from, h2d, c));
    if (to >= bytes) HIPCHK(hipMemsetAsync(d + hdr + bytes, 0, REQ_PAD, c));
  }
  hipEvent_t ev = E->req_ev[1 + E->req_piece++];
  HIPCHK(hipEventRecord(ev, c));
  HIPCHK(hipStreamWaitEvent(E->stream, ev, 0));
  read_requests(E, n, upto < n ? upto : n);
  HIPCHK(hipGetLastError());
  return OTM_OK;
}

int engine_push_after(otm_engine* E, hipEvent_t ev) {
  hipStream_t c = req_copy_stream(E);
  return c && hipStreamWaitEvent(c, ev, 0) == hipSuccess ? OTM_OK : OTM_EDEVICE;
}

int engine_push_mark(otm_engine* E, hipEvent_t ev) {
  hipStream_t c = req_copy_stream(E);
  return c && hipEventRecord(ev, c) == hipSuccess ? OTM_OK : OTM_EDEVICE;
}

int engine_match_requests(otm_engine* E, int32_t n, size_t bytes, bool pushed, const uint8_t** ok,
                          int32_t* n_traces, std::string* err) {
  int rc;
  hipStream_t s = E->stream;
  const size_t total = req_blob_bytes(n, bytes);
  if ((rc = ensure_pinned(E->h_req_ok, (size_t)n + 8 + 8, err))) return rc;
  if ((rc = ensure(E->scan_tmp, scan_tmp_bytes(n) + 256, err))) return rc;
  // a valid point takes at least 39 bytes (`{"lat":0,"lon":0,"time":0,"accuracy":0}`)
  // plus its separator: the batch arrays sized by that bound before the count is known
  const size_t np_max = bytes / 39 + 1;
  if ((rc = ensure(E->in_off, ((size_t)n + 1) * 8, err))) return rc;
  if ((rc = ensure(E->in_lat, np_max * 4, err))) return rc;
  if ((rc = ensure(E->in_lon, np_max * 4, err))) return rc;
  if ((rc = ensure(E->in_time, np_max * 8, err))) return rc;
  if ((rc = ensure(E->in_acc, np_max * 4, err))) return rc;
  if (!pushed) HIPCHK(big_copy(E->d_req.p, E->h_req.p, total, hipMemcpyHostToDevice, s));
  const int64_t* off = (const int64_t*)E->d_req.p;
  int64_t* cnt = P<int64_t>(E->req_cnt);
  read_requests(E, n, n);  // (the requests no push read yet; n == 0: cnt[0] = 0)
  if (n == 0) HIPCHK(hipMemsetAsync(cnt, 0, 8, s));
  scan_i64(cnt, n, E->scan_tmp.p, E->scan_tmp.cap, s);
  DevBatch b{};
  b.trace_off = (const int64_t*)E->in_off.p;
  b.lat = (const float*)E->in_lat.p;
  b.lon = (const float*)E->in_lon.p;
  b.time = (const double*)E->in_time.p;
  b.acc = (const float*)E->in_acc.p;
  launch_req_compact(off, n, cnt, P<uint8_t>(E->req_ok), req_sparse(E), b, P<int64_t>(E->in_off), s);
  // the batch's size and the flags: one synchronisation before the match
  char* h = (char*)E->h_req_ok.p;
  HIPCHK(hipMemcpyAsync(h, cnt + n, 8, hipMemcpyDeviceToHost, s));
  if (n) HIPCHK(hipMemcpyAsync(h + 8, E->req_ok.p, (size_t)n, hipMemcpyDeviceToHost, s));
  HIPCHK(hipGetLastError());
  HIPCHK(wait_batch(E, s, (int64_t)(bytes / 40)));
  E->t_read_done = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  int64_t tot;
  std::memcpy(&tot, h, 8);
  b.n_traces = (int32_t)(tot >> 40);
  b.n_points = tot & (((int64_t)1 << 40) - 1);
  *ok = (const uint8_t*)(h + 8);
  *n_traces = b.n_traces;
  if ((size_t)b.n_points > np_max) {
    *err = "request reader: point count beyond its bound";
    return OTM_EDEVICE;
  }
  return engine_match(E, b, s, err);
}

// The last batch's results compacted on the device into the dense f_*
// arrays (traces with dense offsets); *NS / *NW / *NR their totals.
static int fetch_compact(otm_engine* E, int32_t* NS_, int32_t* NW_, int32_t* NR_, std::string* err) {
  hipStream_t s = E->stream;
  const int32_t NT = E->last_T;
  int rc;
  // dense offsets: exclusive scans of the per-trace counts, then one
  // compaction pass out of the per-trace regions
  ENS_F(f_seg_off, ((size_t)NT + 1) * 4);
  ENS_F(f_way_off, ((size_t)NT + 1) * 4);
  ENS_F(f_rep_off, ((size_t)NT + 1) * 4);
  int32_t* so = P<int32_t>(E->f_seg_off);
  int32_t* wo = P<int32_t>(E->f_way_off);
  int32_t* ro = P<int32_t>(E->f_rep_off);
  if ((rc = ensure_pinned(E->h_tot, 16, err))) return rc;
  int32_t* tot = (int32_t*)E->h_tot.p;
  tot[0] = tot[1] = tot[2] = 0;
  if (NT && NT <= FETCH_SCAN_MAX) {
    // small batches (the batcher's rounds): the three scans in one launch
    launch_fetch_scan(NT, P<int32_t>(E->o_seg_cnt), P<int32_t>(E->o_way_cnt), P<int32_t>(E->o_rep_cnt), so, wo, ro, s);
    HIPCHK(hipMemcpyAsync(tot, so + NT, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(tot + 1, wo + NT, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(tot + 2, ro + NT, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(wait_batch(E, s, E->last_P));
  } else if (NT) {
    HIPCHK(hipMemcpyAsync(so, E->o_seg_cnt.p, (size_t)NT * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(wo, E->o_way_cnt.p, (size_t)NT * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(ro, E->o_rep_cnt.p, (size_t)NT * 4, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemsetAsync(so + NT, 0, 4, s));
    HIPCHK(hipMemsetAsync(wo + NT, 0, 4, s));
    HIPCHK(hipMemsetAsync(ro + NT, 0, 4, s));
    scan_i32(so, NT, E->scan_tmp.p, E->scan_tmp.cap, s);
    scan_i32(wo, NT, E->scan_tmp.p, E->scan_tmp.cap, s);
    scan_i32(ro, NT, E->scan_tmp.p, E->scan_tmp.cap, s);
    HIPCHK(hipMemcpyAsync(tot, so + NT, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(tot + 1, wo + NT, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(tot + 2, ro + NT, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(wait_batch(E, s, E->last_P));
  }
  const int32_t NS = tot[0], NW = tot[1], NR = tot[2];
  ENS_F(f_segs, ((size_t)NS + 1) * sizeof(otm_segment));
  ENS_F(f_ways, ((size_t)NW + 1) * 8);
  ENS_F(f_reps, ((size_t)NR + 1) * sizeof(otm_report_rec));
  ENS_F(f_traces, ((size_t)NT + 1) * sizeof(otm_trace_result));
  if (NT) {
    DevOut o{};
    o.traces = E->o_traces.p;
    o.seg_cnt = P<int32_t>(E->o_seg_cnt);
    o.way_cnt = P<int32_t>(E->o_way_cnt);
    o.rep_cnt = P<int32_t>(E->o_rep_cnt);
    o.segments = E->o_segments.p;
    o.way_ids = P<int64_t>(E->o_way_ids);
    o.reports = E->o_reports.p;
    launch_compact(NT, o, so, wo, ro, E->f_segs.p, P<int64_t>(E->f_ways), E->f_reps.p, E->f_traces.p, s);
    HIPCHK(hipGetLastError());
  }
  E->last_S = NS;
  E->last_W = NW;
  *NS_ = NS;
  *NW_ = NW;
  *NR_ = NR;
  return OTM_OK;
}

int engine_fetch(otm_engine* E, otm_results* out, std::string* err) {
  hipStream_t s = E->stream;
  const int32_t NT = E->last_T;
  int32_t NS, NW, NR;
  int rc;
  if ((rc = fetch_compact(E, &NS, &NW, &NR, err))) return rc;
  if ((rc = ensure_pinned(E->h_traces, ((size_t)NT + 1) * sizeof(otm_trace_result), err))) return rc;
  if ((rc = ensure_pinned(E->h_segs, ((size_t)NS + 1) * sizeof(otm_segment), err))) return rc;
  if ((rc = ensure_pinned(E->h_reps_dense, ((size_t)NR + 1) * sizeof(otm_report_rec), err))) return rc;
  if ((rc = ensure_pinned(E->h_ways, ((size_t)NW + 1) * 8, err))) return rc;
  const hipMemcpyKind d2h = hipMemcpyDeviceToHost;
  hipStream_t c = s;
  if (NT) HIPCHK(big_copy(E->h_traces.p, E->f_traces.p, (size_t)NT * sizeof(otm_trace_result), d2h, c));
  if (NS) HIPCHK(big_copy(E->h_segs.p, E->f_segs.p, (size_t)NS * sizeof(otm_segment), d2h, c));
  if (NR) HIPCHK(big_copy(E->h_reps_dense.p, E->f_reps.p, (size_t)NR * sizeof(otm_report_rec), d2h, c));
  if (NW) HIPCHK(big_copy(E->h_ways.p, E->f_ways.p, (size_t)NW * 8, d2h, c));
  HIPCHK(wait_batch(E, c, E->last_P));
  out->n_traces = NT;
  out->n_segments = NS;
  out->n_reports = NR;
  out->n_way_ids = NW;
  out->traces = (const otm_trace_result*)E->h_traces.p;
  out->segments = (const otm_segment*)E->h_segs.p;
  out->reports = (const otm_report_rec*)E->h_reps_dense.p;
  out->way_ids = (const int64_t*)E->h_ways.p;
  return OTM_OK;
}

int engine_write_responses(otm_engine* E, const int64_t** off, const uint8_t** host,
                           const otm_trace_result** traces, int64_t* total, std::string* err) {
  hipStream_t s = E->stream;
  const int32_t NT = E->last_T;
  int32_t NS, NW, NR;
  int rc;
  if ((rc = fetch_compact(E, &NS, &NW, &NR, err))) return rc;
  const size_t hdr_b = (size_t)NT * RESP_HDR_SLOT + 64, seg_b = resp_seg_scratch(NS, NW),
               rep_b = (size_t)NR * RESP_REP_SLOT + 64;
  ENS_F(resp_hdr, hdr_b);
  ENS_F(resp_seg, seg_b);
  ENS_F(resp_rep, rep_b);
  ENS_F(resp_hlen, ((size_t)NT + 1) * 4);
  ENS_F(resp_slen, ((size_t)NS + 1) * 4);
  ENS_F(resp_rlen, ((size_t)NR + 1) * 4);
  ENS_F(resp_blen, ((size_t)NT + 1) * 8);
  ENS_F(resp_host, (size_t)NT + 1);
  // a body is at most its pieces plus the joins (commas, the fixed middle and end)
  const size_t blob_b = hdr_b + seg_b + rep_b + (size_t)NT * 97 + (size_t)NS + (size_t)NR;  // (+ the NULs)
  ENS_F(resp_blob, blob_b);
  if ((rc = ensure(E->scan_tmp, scan_tmp_bytes(NT) + 256, err))) return rc;
  RespIn in{NT, NS, NR, (const otm_trace_result*)E->f_traces.p, (const otm_segment*)E->f_segs.p,
            P<int64_t>(E->f_ways), (const otm_report_rec*)E->f_reps.p};
  RespWork w{P<char>(E->resp_hdr),   P<char>(E->resp_seg),     P<char>(E->resp_rep),    P<int32_t>(E->resp_hlen),
             P<int32_t>(E->resp_slen), P<int32_t>(E->resp_rlen), P<int64_t>(E->resp_blen), P<uint8_t>(E->resp_host)};
  if (NT) {
    launch_resp_items(in, w, s);
    launch_resp_len(in, w, s);
    scan_i64(w.blen, NT, E->scan_tmp.p, E->scan_tmp.cap, s);
    launch_resp_copy(in, w, w.blen, P<char>(E->resp_blob), s);
  }
  // the offsets, flags and trace records, then the bodies
  const size_t off_b = ((size_t)NT + 1) * 8;
  if ((rc = ensure_pinned(E->h_resp_meta, off_b + (size_t)NT + 8, err))) return rc;
  if ((rc = ensure_pinned(E->h_traces, ((size_t)NT + 1) * sizeof(otm_trace_result), err))) return rc;
  char* meta = (char*)E->h_resp_meta.p;
  std::memset(meta, 0, off_b);
  if (NT) {
    HIPCHK(hipMemcpyAsync(meta, w.blen, off_b, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(meta + off_b, w.host, (size_t)NT, hipMemcpyDeviceToHost, s));
    HIPCHK(big_copy(E->h_traces.p, E->f_traces.p, (size_t)NT * sizeof(otm_trace_result), hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipGetLastError());
  HIPCHK(wait_batch(E, s, E->last_P));
  *total = ((const int64_t*)meta)[NT];
  *off = (const int64_t*)meta;
  *host = (const uint8_t*)(meta + off_b);
  *traces = (const otm_trace_result*)E->h_traces.p;
  return OTM_OK;
}

// the body blob of the last engine_write_responses (total bytes) into dst --
// page-locked host memory (the caller's response arena) -- or, with dst null,
// into the engine's own pinned buffer; *blob: where it landed
int engine_copy_responses(otm_engine* E, char* dst, int64_t total, const char** blob, std::string* err) {
  int rc;
  if (!dst) {
    if ((rc = ensure_pinned(E->h_resp, (size_t)total + 16, err))) return rc;
    dst = (char*)E->h_resp.p;
  }
  if (total) {
    HIPCHK(big_copy(dst, E->resp_blob.p, (size_t)total, hipMemcpyDeviceToHost, E->stream));
    HIPCHK(wait_batch(E, E->stream, E->last_P));
  }
  *blob = dst;
  return OTM_OK;
}

// report() on the GPU over caller-supplied segments: the k_report kernel
// alone, with the per-trace segment regions laid out as the matcher's
// pipeline leaves them (DevOut: trace t's segments start at seg_base[t]).
int engine_report_segments(otm_engine* E, int32_t T, const int64_t* trace_off, const double* time,
                           const int32_t* seg_off, const otm_segment* segs, otm_trace_result* traces,
                           otm_report_rec* reports, std::string* err) {
  const int64_t NP = trace_off[T];
  const int32_t NS = seg_off[T];
  for (int32_t t = 0; t < T; ++t)
    if (trace_off[t + 1] <= trace_off[t]) {
      *err = "every trace needs at least one point (its end time)";
      return OTM_EINVAL;
    }
  int rc;
  // one device blob: trace_off, seg_base (per trace), time, segments,
  // seg_cnt, seg_gidx, trace_err, abort; outputs: traces, reports, rep_cnt
  const size_t b_off = ((size_t)T + 1) * 8, b_sb = ((size_t)T + 1) * 8, b_tm = (size_t)NP * 8;
  const size_t b_seg = ((size_t)NS + 1) * sizeof(otm_segment), b_cnt = ((size_t)T + 1) * 4;
  const size_t b_gidx = ((size_t)NS + 1) * 4, b_err = b_cnt, b_ab = 16;
  const size_t b_tr = ((size_t)T + 1) * sizeof(otm_trace_result), b_rep = ((size_t)NS + 1) * sizeof(otm_report_rec);
  size_t off[12];
  size_t tot = 0;
  const size_t sz[11] = {b_off, b_sb, b_tm, b_seg, b_cnt, b_gidx, b_err, b_ab, b_tr, b_rep, b_cnt};
  for (int k = 0; k < 11; ++k) {
    off[k] = tot;
    tot += (sz[k] + 255) & ~(size_t)255;
  }
  off[11] = tot;
  if ((rc = ensure(E->rs_blob, tot, err))) return rc;
  std::vector<char> h(off[8], 0);
  std::memcpy(h.data() + off[0], trace_off, b_off);
  int64_t* sb = (int64_t*)(h.data() + off[1]);
  int32_t* cnt = (int32_t*)(h.data() + off[4]);
  for (int32_t t = 0; t < T; ++t) {
    sb[t] = seg_off[t];
    cnt[t] = seg_off[t + 1] - seg_off[t];
  }
  if (NP) std::memcpy(h.data() + off[2], time, b_tm);
  if (NS) std::memcpy(h.data() + off[3], segs, (size_t)NS * sizeof(otm_segment));
  int32_t* gidx = (int32_t*)(h.data() + off[5]);
  for (int32_t k = 0; k < NS; ++k) gidx[k] = -1;  // no histogram for handed-in segments
  hipStream_t s = E->stream;
  char* d = (char*)E->rs_blob.p;
  HIPCHK(hipMemcpyAsync(d, h.data(), off[8], hipMemcpyHostToDevice, s));
  DevBatch b{};
  b.n_traces = T;
  b.n_points = NP;
  b.trace_off = (const int64_t*)(d + off[0]);
  b.time = (const double*)(d + off[2]);
  DevWork w{};
  w.trace_err = (int32_t*)(d + off[6]);
  w.abort = (int32_t*)(d + off[7]);
  w.ctr = nullptr;
  DevOut o{};
  o.traces = d + off[8];
  o.seg_cnt = (int32_t*)(d + off[4]);
  o.rep_cnt = (int32_t*)(d + off[10]);
  o.seg_base = (int64_t*)(d + off[1]);
  o.segments = d + off[3];
  o.seg_gidx = (int32_t*)(d + off[5]);
  o.reports = d + off[9];
  o.hist = nullptr;
  o.speed_sum = nullptr;
  launch_report(b, E->drc, w, o, s, Marks{});
  HIPCHK(hipGetLastError());
  if (T) HIPCHK(hipMemcpyAsync(traces, d + off[8], (size_t)T * sizeof(otm_trace_result), hipMemcpyDeviceToHost, s));
  if (NS) HIPCHK(hipMemcpyAsync(reports, d + off[9], (size_t)NS * sizeof(otm_report_rec), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  return OTM_OK;
}

int engine_debug_fetch(otm_engine* E, int what, void* dst, size_t bytes, size_t* needed, std::string* err) {
  const size_t Pn = (size_t)E->last_P;
  const void* src = nullptr;
  size_t n = 0;
  switch (what) {
    case 0: src = E->ncand.p; n = Pn * 4; break;
    case 1:
    case 2:
    case 3: {
      // candidate edges (1), offsets (2) or emissions (3) as [P*KMAX], slot
      // j of point p at p * KMAX + j (inline and overflow slots joined)
      n = Pn * KMAX * 4;
      if (needed) *needed = n;
      if (!dst) return OTM_OK;
      if (bytes < n) {
        *err = "debug buffer too small";
        return OTM_EINVAL;
      }
      if (!n) return OTM_OK;
      const bool rec = what != 3;
      std::vector<char> in(Pn * KIN * (rec ? 8 : 4)), ov(Pn * KX * (rec ? 8 : 4));
      HIPCHK(hipMemcpyAsync(in.data(), rec ? E->cand_eo.p : E->cand_em.p, in.size(), hipMemcpyDeviceToHost,
                            E->stream));
      HIPCHK(hipMemcpyAsync(ov.data(), rec ? E->cand_xeo.p : E->cand_xem.p, ov.size(), hipMemcpyDeviceToHost,
                            E->stream));
      HIPCHK(hipStreamSynchronize(E->stream));
      int32_t* d = (int32_t*)dst;
      for (size_t p = 0; p < Pn; ++p)
        for (int j = 0; j < KMAX; ++j) {
          const int32_t* src = j < KIN ? (const int32_t*)in.data() + (rec ? 2 : 1) * (p * KIN + j)
                                       : (const int32_t*)ov.data() + (rec ? 2 : 1) * (p * KX + (j - KIN));
          d[p * KMAX + j] = rec ? src[what - 1] : src[0];
        }
      return OTM_OK;
    }
    case 4: src = E->trans_off.p; n = (Pn + 1) * 8; break;
    case 5: src = E->trans.p; n = (size_t)E->last_trans * 4; break;
    case 6: src = E->state.p; n = Pn * 4; break;
    case 7: src = E->col_prev.p; n = Pn * 4; break;
    case 8: src = E->route_dist.p; n = Pn * 4; break;
    case 9: src = E->gc.p; n = Pn * 4; break;
    case 10: src = E->ipos.p; n = Pn * 4; break;
    // the last batch's inputs as the GPU request reader decoded them
    // (engine_match_requests; also a host batch of more than 2^18 points)
    case 11: src = E->in_off.p; n = ((size_t)E->last_T + 1) * 8; break;
    case 12: src = E->in_lat.p; n = Pn * 4; break;
    case 13: src = E->in_lon.p; n = Pn * 4; break;
    case 14: src = E->in_time.p; n = Pn * 8; break;
    case 15: src = E->in_acc.p; n = Pn * 4; break;
    default: *err = "unknown debug buffer"; return OTM_EINVAL;
  }
  if (needed) *needed = n;
  if (!dst) return OTM_OK;
  if (bytes < n) {
    *err = "debug buffer too small";
    return OTM_EINVAL;
  }
  if (n) HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, E->stream));
  HIPCHK(hipStreamSynchronize(E->stream));
  return OTM_OK;
}

int engine_spill_stats(otm_engine* E, otm_spill_stats* out) {
  int32_t v[48] = {};
  if (E->snap.p && hipMemcpy(v, E->snap.p, sizeof v, hipMemcpyDeviceToHost) != hipSuccess) return OTM_EDEVICE;
  // counters_i32 layout: [5] candidate spills; [4] index misses, [0] lane
  // spills, [3] LDS-wave spills (per stage)
  out->cand_wave = v[5];
  out->trans_online = v[16 + 4];
  out->trans_wave = v[16 + 4];
  out->trans_global = v[16 + 3];
  out->route_online = v[32 + 4];
  out->route_wave = v[32 + 4];
  out->route_global = v[32 + 3];
  int32_t c[32] = {};
  if (E->snap.p && hipMemcpy(c, E->counters_i32.p, sizeof c, hipMemcpyDeviceToHost) != hipSuccess) return OTM_EDEVICE;
  out->cand_big = c[24];
  out->trans_huge = c[21];
  out->route_huge = c[22];
  out->attempts = E->last_attempts;
  out->resumed = E->last_resumes;
  return OTM_OK;
}

int engine_counters(otm_engine* E, otm_work_counters* out) {
  DevCounters c;
  if (hipMemcpy(&c, E->ctr, sizeof c, hipMemcpyDeviceToHost) != hipSuccess) return OTM_EDEVICE;
  static_assert(sizeof(DevCounters) == sizeof(otm_work_counters), "counter layout");
  std::memcpy(out, &c, sizeof c);
  return OTM_OK;
}

}  // namespace otm
