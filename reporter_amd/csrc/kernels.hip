// kernels.hip -- the map-matching hot path as HIP kernels for gfx950 (CDNA4).
//
// Replaces valhalla.SegmentMatcher().Match (py/reporter_service.py:112) and
// report() (:110-215).  Every float expression below follows the evaluation
// order of the written spec (oracle/otm_oracle.c) and the file
// is compiled with -ffp-contract=off, so results are bit-identical to the CPU
// oracle: no FMA contraction, IEEE division and sqrt, and order-independent
// fixed points (label-correcting search == Dijkstra, see K4).
//
// Execution model: wave64.  The irregular stages run one wavefront per unit
// of work (probe, column pair, trace) in 64-thread workgroups, grid-striding,
// with their working sets (edge hash, search labels, frontiers) in LDS.  No
// stage is a dense contraction; MFMA is deliberately unused.  Graph arrays are
// read-only and small enough (tens of MB at city scale) to live in L2 / the
// 256 MB Infinity Cache after first touch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include <hipcub/hipcub.hpp>

#include "kernels.h"
#include "otmatch.h"

namespace otm {

namespace {

#define MPD_F 111319.4954833f  // (float)(20037581.187 / 180), Batch.java:33
constexpr uint32_t EMPTY = 0xFFFFFFFFu;
constexpr unsigned long long LAB_NONE = ~0ull;
constexpr int TB = 64;  // one wavefront per workgroup for the wave kernels
// A one-wavefront block's LDS operations execute in issue order, so its
// cross-lane LDS hand-offs need only the compiler kept from moving memory
// accesses across this point.  __syncthreads() would also wait for every
// global load and store in flight (s_waitcnt vmcnt(0)): the next chunks'
// prefetches, or the last item's result stores before the next item starts.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float cos_deg(float deg) {
  const float x = deg * 0.017453292519943295f;
  const float x2 = x * x;
  float c = -1.1470745597729725e-11f;
  c = c * x2 + 2.08767569878681e-09f;
  c = c * x2 - 2.755731922398589e-07f;
  c = c * x2 + 2.48015873015873e-05f;
  c = c * x2 - 0.001388888888888889f;
  c = c * x2 + 0.041666666666666664f;
  c = c * x2 - 0.5f;
  c = c * x2 + 1.0f;
  return c;
}

__device__ __forceinline__ float gc_dist(float la, float lo, float lb, float lob) {
  const float ls = MPD_F * cos_deg((la + lb) * 0.5f);
  const float dx = (lob - lo) * ls;
  const float dy = (lb - la) * MPD_F;
  return sqrtf(dx * dx + dy * dy);
}

// squared distance from the probe to shape segment a-b: the sqd half of
// project() below, same float evaluation order
__device__ __forceinline__ float seg_sqdist(float alat, float alon, float blat, float blon, float lat, float lon,
                                            float ls) {
  const float ax = (alon - lon) * ls;
  const float ay = (alat - lat) * MPD_F;
  const float bx = (blon - lon) * ls;
  const float by = (blat - lat) * MPD_F;
  const float vx = bx - ax;
  const float vy = by - ay;
  const float l2 = vx * vx + vy * vy;
  // branch-free: the quotient of a zero-length segment (inf / nan) is
  // selected away, so the lanes of the scan never split here
  const float dot = ax * vx + ay * vy;
  float t = -dot / l2;
  t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  t = l2 > 0.0f ? t : 0.0f;
  const float px = ax + t * vx;
  const float py = ay + t * vy;
  return px * px + py * py;
}

// (round 4 A/B, not kept: a division-free early out in the lane tier's scan
// for segments whose whole line lies beyond the radius measured slower --
// k_cand_lane 0.229 vs 0.221 ms on config 2, 1.89 vs 1.85 on config 4; the
// branch splits the wave where the division did not)

// A projection's inputs (the shape segment's two points and cumulative
// metres, the edge length and its last shape point), loaded apart from the
// arithmetic so a caller can issue several projections' loads at once.
struct ProjIn {
  float alon, alat, blon, blat, ca, cb, len;
  int32_t b, last;
};
__device__ __forceinline__ ProjIn proj_load(const DevGraph& g, int32_t e, int32_t k) {
  ProjIn in;
  const int32_t a = g.e_shape_off[e] + k, b = a + 1;
  in.last = g.e_shape_off[e + 1] - 1;
  in.alon = g.s_lon[a];
  in.alat = g.s_lat[a];
  in.blon = g.s_lon[b];
  in.blat = g.s_lat[b];
  in.ca = g.s_cum[a];
  in.cb = g.s_cum[b];
  in.len = g.e_len[e];
  in.b = b;
  return in;
}
__device__ __forceinline__ void proj_calc(const ProjIn& in, float lat, float lon, float ls, float& sqd,
                                          float& off_out, bool& at_end) {
  const float ax = (in.alon - lon) * ls;
  const float ay = (in.alat - lat) * MPD_F;
  const float bx = (in.blon - lon) * ls;
  const float by = (in.blat - lat) * MPD_F;
  const float vx = bx - ax;
  const float vy = by - ay;
  const float l2 = vx * vx + vy * vy;
  float t = 0.0f;
  if (l2 > 0.0f) {
    const float dot = ax * vx + ay * vy;
    t = -dot / l2;
    t = t < 0.0f ? 0.0f : (t > 1.0f ? 1.0f : t);
  }
  const float px = ax + t * vx;
  const float py = ay + t * vy;
  sqd = px * px + py * py;
  float off = in.ca + t * (in.cb - in.ca);
  off_out = off > in.len ? in.len : off;
  // clamped to the edge's last shape point: the projection is its end node
  at_end = t == 1.0f && in.b == in.last;
}
__device__ __forceinline__ void project(const DevGraph& g, int32_t e, int32_t k, float lat, float lon, float ls,
                                        float& sqd, float& off_out, bool& at_end) {
  proj_calc(proj_load(g, e, k), lat, lon, ls, sqd, off_out, at_end);
}
__device__ __forceinline__ void project(const DevGraph& g, int32_t e, int32_t k, float lat, float lon, float ls,
                                        float& sqd, float& off_out) {
  bool at_end;
  project(g, e, k, lat, lon, ls, sqd, off_out, at_end);
}
// node snap: the node an edge's best projection snaps to -- its
// start node at offset 0, its end node when clamped there and the node has an
// outgoing edge -- or -1.  The node candidate is carried as (the node's first
// outgoing edge, offset 0).
__device__ __forceinline__ int32_t snap_node(const DevGraph& g, int32_t e, float off, bool at_end) {
  if (off == 0.0f) return g.e_from[e];
  if (at_end) {
    const int32_t v = g.e_to[e];
    if (g.out_off[v + 1] > g.out_off[v]) return v;
  }
  return -1;
}

__device__ __forceinline__ float probe_radius(const DevParams& P, float acc) {
  const float a = acc > 0.0f ? acc : P.gps_accuracy;
  const float r = a > P.search_radius ? a : P.search_radius;
  return r < P.max_search_radius ? r : P.max_search_radius;
}

__device__ __forceinline__ uint32_t fbits(float f) { return __float_as_uint(f); }
__device__ __forceinline__ float bitsf(uint32_t u) { return __uint_as_float(u); }
__device__ __forceinline__ uint32_t hash32(uint32_t x) { return x * 2654435761u; }

__device__ __forceinline__ void cadd(unsigned long long* c, unsigned long long v) {
  if (c && v) atomicAdd(c, v);
}

// candidate slot j of point p (DevWork: KIN inline slots, the rest overflow)
__device__ __forceinline__ int2 crec(const DevWork& w, int64_t p, int j) {
  return j < KIN ? w.cand_eo[p * KIN + j] : w.cand_xeo[p * KX + (j - KIN)];
}
__device__ __forceinline__ float cemis(const DevWork& w, int64_t p, int j) {
  return j < KIN ? w.cand_em[p * KIN + j] : w.cand_xem[p * KX + (j - KIN)];
}
__device__ __forceinline__ void cput(const DevWork& w, int64_t p, int j, int32_t e, float off, float em) {
  if (j < KIN) {
    w.cand_eo[p * KIN + j] = make_int2(e, __float_as_int(off));
    w.cand_em[p * KIN + j] = em;
  } else {
    w.cand_xeo[p * KX + (j - KIN)] = make_int2(e, __float_as_int(off));
    w.cand_xem[p * KX + (j - KIN)] = em;
  }
}

// ============================================================== turn costs
// deviation from straight on (0..180 degrees) of the turn from an edge whose
// end heading is hin into an edge whose start heading is hout
__device__ __forceinline__ uint32_t turn_deg(uint32_t hin, uint32_t hout) {
  int d = (int)hout - (int)hin;
  d += d < 0 ? 360 : 0;
  return (uint32_t)(d <= 180 ? d : 360 - d);
}
// transition cost (turn_cost + |r - gc|) / beta of DESIGN.md §3; the turn
// cost is integer 1/64 m units summed over the route's turns (order-free),
// exact in a float below 2^24
__device__ __forceinline__ float trans_cost(uint32_t units, float r, float gcv, float beta) {
  units = units > TURN_UNITS_MAX ? TURN_UNITS_MAX : units;
  const float tc = (float)units * 0.015625f;
  const float diff = fabsf(r - gcv);
  return (tc + diff) / beta;
}

// ============================================================== node candidates
// DESIGN.md §3 node snap: a candidate at offset 0 is the node candidate of its
// edge's start node (K2 snaps every end-of-edge projection to the node, so
// an edge candidate never sits at offset 0).  Its routes start at the node
// with nothing left to drive, and it has no heading on its side of a route.
constexpr uint32_t NO_HEAD = 0xFFFFu;
__device__ __forceinline__ bool cand_node(float off) { return off == 0.0f; }
__device__ __forceinline__ int32_t src_node(const DevGraph& g, int32_t e, float off) {
  return cand_node(off) ? g.e_from[e] : g.e_to[e];
}
__device__ __forceinline__ float src_start(const DevGraph& g, int32_t e, float off) {
  return cand_node(off) ? 0.0f : g.e_len[e] - off;
}
__device__ __forceinline__ uint32_t src_head(const DevGraph& g, int32_t e, float off) {
  return cand_node(off) ? NO_HEAD : (uint32_t)g.e_head_in[e];
}
__device__ __forceinline__ uint32_t dst_head(const DevGraph& g, int32_t e, float off) {
  return cand_node(off) ? NO_HEAD : (uint32_t)g.e_head_out[e];
}
// DESIGN.md §3 rule 4, same edge: from (e, oi) to (e, oj) the route is along
// the edge when oj is not before oi; when oj is behind oi and both are edge
// candidates the step is a stay (GPS noise moved the later probe back; a
// vehicle does not reverse along a directed edge): route distance 0, no
// turns, no traversal, the position on the edge staying at the largest offset
// reached.  oracle/otm_oracle.c same_edge_step / same_edge_dist.
__device__ __forceinline__ bool same_edge_step(int32_t ei, float oi, int32_t ej, float oj) {
  return ei == ej && (oj >= oi || (!cand_node(oj) && !cand_node(oi)));
}
__device__ __forceinline__ float same_edge_dist(float oi, float oj) { return oj >= oi ? oj - oi : 0.0f; }
// turn units of one turn (none when either side is a node candidate)
__device__ __forceinline__ uint32_t turn_units(const uint32_t* TU, uint32_t hin, uint32_t hout) {
  return (hin == NO_HEAD || hout == NO_HEAD) ? 0u : TU[turn_deg(hin, hout)];
}

// wave-wide inclusive scan of an int (64 lanes)
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int n = __shfl_up(v, o, 64);
    if (lane >= o) v += n;
  }
  return v;
}

// The same bookkeeping folded into the stage kernels: each kernel boundary in
// a stream costs ~5-10 us, and these ran as five one-wave launches per batch.
#ifndef OTM_FOLD_BOOKKEEPING
#define OTM_FOLD_BOOKKEEPING 1
#endif
// one thread: spill snapshot k (16 counters), optionally resetting them
__device__ __forceinline__ void fold_snap(DevWork& w, int k, bool reset) {
  for (int t = 0; t < 16; ++t) {
    w.snap[16 * k + t] = w.counters_i32[t];
    if (reset) w.counters_i32[t] = 0;
  }
}
// every transition kernel's first test: the matrices' total against the
// buffer (the first kernel to run sets the abort flag for the rest)
__device__ __forceinline__ bool trans_over_cap(const DevBatch& b, const DevWork& w) {
  if (!OTM_FOLD_BOOKKEEPING) return false;
  if (w.trans_off[b.n_points] <= w.trans_cap) return false;
  *w.abort = 1;
  return true;
}

// ============================================================== spatial work order
__device__ __forceinline__ int hilbert_d(int x, int y) {
  int d = 0;
  for (int sft = ORDER_SIDE / 2; sft > 0; sft >>= 1) {
    const int rx = (x & sft) > 0;
    const int ry = (y & sft) > 0;
    d += sft * sft * ((3 * rx) ^ ry);
    if (ry == 0) {
      if (rx == 1) {
        x = ORDER_SIDE - 1 - x;
        y = ORDER_SIDE - 1 - y;
      }
      const int tmp = x;
      x = y;
      y = tmp;
    }
  }
  return d;
}

__device__ __forceinline__ int tile_of(const DevGraph& g, float lat, float lon) {
  int ty = (int)((lat - g.bb_lat0) * g.bb_inv_h);
  int tx = (int)((lon - g.bb_lon0) * g.bb_inv_w);
  ty = ty < 0 ? 0 : (ty >= ORDER_SIDE ? ORDER_SIDE - 1 : ty);
  tx = tx < 0 ? 0 : (tx >= ORDER_SIDE ? ORDER_SIDE - 1 : tx);
  return hilbert_d(tx, ty);
}

// Wave-aggregated atomicAdd(&ctr[key], 1): one atomic per distinct key in
// the wave; returns this lane's slot (consecutive points of a trace usually
// share a tile, so a wave makes one to three atomics).  All 64 lanes call it.
__device__ __forceinline__ int wave_agg_slot(int32_t* ctr, int key, bool active) {
  const int lane = threadIdx.x & 63;
  unsigned long long pending = __ballot(active);
  int pos = 0;
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const int k = __shfl(key, leader, 64);
    const unsigned long long grp = __ballot(((pending >> lane) & 1ull) && key == k);
    int base = 0;
    if (lane == leader) base = atomicAdd(&ctr[k], (int)__popcll(grp));
    base = __shfl(base, leader, 64);
    if ((grp >> lane) & 1ull) pos = base + (int)__popcll(grp & ((1ull << lane) - 1ull));
    pending &= ~grp;
  }
  return pos;
}

// one block: exclusive scan of the tile counts (Hilbert order), cursors, and
// the 8 group cuts at the tile boundaries nearest k/8 of the columns
__global__ __launch_bounds__(1024) void k_order_plan(const int32_t* tile_cnt, int32_t* cursor, int32_t* grp) {
  __shared__ int32_t part[1024];
  __shared__ int32_t cut[ORDER_GROUPS + 1];
  constexpr int PER = ORDER_TILES / 1024;
  const int tid = threadIdx.x;
  int32_t v[PER], sum = 0;
  for (int k = 0; k < PER; ++k) {
    v[k] = tile_cnt[tid * PER + k];
    sum += v[k];
  }
  part[tid] = sum;
  if (tid <= ORDER_GROUPS) cut[tid] = 0x7fffffff;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int32_t x = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += x;
    __syncthreads();
  }
  const int32_t total = part[1023];
  int32_t run = part[tid] - sum;
  // start of the tile before this thread's first one (-1 before tile 0)
  int32_t prev_start = tid == 0 ? -1 : run - tile_cnt[tid * PER - 1];
  for (int k = 0; k < PER; ++k) {
    cursor[tid * PER + k] = run;
    // group gi starts at the first tile whose start reaches gi/8 of the
    // columns: exactly one tile sees prev_start < want <= run
    for (int gi = 1; gi < ORDER_GROUPS; ++gi) {
      const int64_t want = ((int64_t)total * gi + ORDER_GROUPS - 1) / ORDER_GROUPS;
      if (run >= want && prev_start < want) cut[gi] = run;
    }
    prev_start = run;
    run += v[k];
  }
  __syncthreads();
  if (tid == 0) {
    grp[0] = 0;
    int32_t prev = 0;
    for (int gi = 1; gi < ORDER_GROUPS; ++gi) {
      const int32_t c = cut[gi] > total ? total : cut[gi];
      prev = c > prev ? c : prev;
      grp[gi] = prev;
    }
    grp[ORDER_GROUPS] = total;
  }
}

__global__ __launch_bounds__(256) void k_order_scatter(DevBatch b, DevWork w, const uint16_t* tile, int32_t* cursor,
                                                       int32_t* item) {
  for (int64_t p0 = (int64_t)blockIdx.x * 256; p0 < b.n_points; p0 += (int64_t)gridDim.x * 256) {
    const int64_t p = p0 + threadIdx.x;
    const bool col = p < b.n_points && w.is_col[p];
    const int t = col ? (int)tile[p] : 0;
    const int pos = wave_agg_slot(cursor, t, col);
    if (col) item[pos] = (int32_t)p;
    if (col && w.colrec_pos) w.colrec_pos[p] = pos;  // where K3 writes the column's K4 record
  }
}

// ============================================================== K1 columns
// One wavefront per trace: lanes stage the trace's coordinates in LDS and
// compute the distance of every point to its predecessor in parallel; lane 0
// then runs the interpolation filter (a point is a column iff it lies at least
// interpolation_distance from the last column) out of LDS, recomputing the
// distance only where the last column is not the immediate predecessor.
// points staged in LDS (longer traces take the serial form): 256 leaves room
// for 8 waves per SIMD (512: ~4.6), 0.050 -> 0.046 ms on config 2, 0.42 ->
// 0.37 ms on a config-3 shard
#ifndef OTM_COL_PTS
#define OTM_COL_PTS 256
#endif
constexpr int COL_PTS = OTM_COL_PTS;
__global__ __launch_bounds__(TB) void k_columns(DevGraph g, DevBatch b, DevParams P, DevWork w) {
  __shared__ float sLat[COL_PTS], sLon[COL_PTS], sGc[COL_PTS];
  __shared__ int32_t sPrev[COL_PTS];
  __shared__ uint8_t sCol[COL_PTS];
  const int lane = threadIdx.x;
  if (OTM_FOLD_BOOKKEEPING && blockIdx.x == 0) {
    // the batch's tier counters and abort flag start at zero (k_batch_init)
    if (lane < 32) w.counters_i32[lane] = 0;  // ([20]: the wide Viterbi list)
    if (lane == 0) *w.abort = 0;
  }
  for (int32_t t = blockIdx.x; t < b.n_traces; t += gridDim.x) {
    const int64_t a = b.trace_off[t], e = b.trace_off[t + 1];
    const int n = (int)(e - a);
    int ncols = 0;
    if (n > COL_PTS) {
      // long trace: the same filter straight from HBM
      if (lane == 0) {
        int64_t last = -1;
        for (int64_t p = a; p < e; ++p) {
          float gcv = 0.0f;
          if (last >= 0) gcv = gc_dist(b.lat[last], b.lon[last], b.lat[p], b.lon[p]);
          const bool col = last < 0 || gcv >= P.interp;
          w.is_col[p] = col ? 1 : 0;
          w.gc[p] = col ? gcv : 0.0f;
          w.prevc[p] = (int32_t)last;  // a non-column: the column before it (K7a)
          if (col) {
            last = p;
            ++ncols;
            if (w.ord.tile_cnt) {  // spatial order tile (serial here: long traces are rare)
              const int tl = tile_of(g, b.lat[p], b.lon[p]);
              w.ord.tile[p] = (uint16_t)tl;
              atomicAdd(&w.ord.tile_cnt[tl], 1);
            }
          }
        }
      }
      for (int64_t p = a + lane; p < e; p += TB) {
        w.probe[p] = make_float4(b.lat[p], b.lon[p], b.acc[p], 0.0f);
        w.pt_trace[p] = t;
        w.ncand[p] = 0;
        w.route_dist[p] = 0.0f;
        w.ipos[p] = -1.0f;
        w.nextc[p] = -1;
      }
    } else {
      for (int pl = lane; pl < n; pl += TB) {
        sLat[pl] = b.lat[a + pl];
        sLon[pl] = b.lon[a + pl];
      }
      __syncthreads();
      bool near = false;  // some step shorter than the interpolation distance
      for (int pl = lane; pl < n; pl += TB) {
        const float d = pl > 0 ? gc_dist(sLat[pl - 1], sLon[pl - 1], sLat[pl], sLon[pl]) : 0.0f;
        sGc[pl] = d;
        near = near || (pl > 0 && !(d >= P.interp));
      }
      __syncthreads();
      if (__ballot(near) == 0ull) {
        // every step is at least the interpolation distance: every point is a
        // column linked to the one before (what the serial filter below gives)
        for (int pl = lane; pl < n; pl += TB) {
          sCol[pl] = 1;
          sPrev[pl] = pl > 0 ? (int32_t)(a + pl - 1) : -1;
        }
        ncols = n;
      } else if (lane == 0) {
        int last = -1;
        for (int pl = 0; pl < n; ++pl) {
          float gcv = 0.0f;
          if (last >= 0) gcv = last == pl - 1 ? sGc[pl] : gc_dist(sLat[last], sLon[last], sLat[pl], sLon[pl]);
          const bool col = last < 0 || gcv >= P.interp;
          sCol[pl] = col ? 1 : 0;
          sGc[pl] = col ? gcv : 0.0f;
          sPrev[pl] = last >= 0 ? (int32_t)(a + last) : -1;  // a non-column: the column before it (K7a)
          if (col) {
            last = pl;
            ++ncols;
          }
        }
      }
      __syncthreads();
      for (int c0 = 0; c0 < n; c0 += TB) {
        const int pl = c0 + lane;
        const bool in = pl < n;
        const bool col = in && sCol[pl];
        if (in) {
          const int64_t p = a + pl;
          w.probe[p] = make_float4(sLat[pl], sLon[pl], b.acc[p], 0.0f);
          w.pt_trace[p] = t;
          w.is_col[p] = sCol[pl];
          w.gc[p] = sGc[pl];
          w.prevc[p] = sPrev[pl];
          // later stages write these for columns only (spatial work order)
          w.ncand[p] = 0;
          w.route_dist[p] = 0.0f;
          w.ipos[p] = -1.0f;
          w.nextc[p] = -1;
          // (path_len / path_off: K6 writes them for every column, and only
          // columns' are read)
        }
        if (w.ord.tile_cnt) {  // spatial order: this column's tile, counted per wave
          const int tl = col ? tile_of(g, sLat[pl], sLon[pl]) : 0;
          if (col) w.ord.tile[a + pl] = (uint16_t)tl;
          (void)wave_agg_slot(w.ord.tile_cnt, tl, col);
        }
      }
      __syncthreads();
    }
    if (lane == 0) {
      w.trace_err[t] = 0;
      if (w.ctr) {
        cadd(&w.ctr->points, (unsigned long long)n);
        cadd(&w.ctr->columns, (unsigned long long)ncols);
      }
    }
  }
}

// The items a block walks: the spatial order's group blockIdx % 8 (lanes
// or waves over it), or every point in natural order.  per_block = items
// per block per step (threads for lane kernels, 1 for wave kernels).
struct ItemRange {
  int64_t i0, i1, stride;
  bool ordered;
};
__device__ __forceinline__ ItemRange item_range(const DevWork& w, const DevBatch& b, bool ordered, int per_block) {
  ItemRange r;
  r.ordered = ordered;
  const int tid = per_block > 1 ? (int)threadIdx.x : 0;
  if (ordered) {
    const int grp = blockIdx.x % ORDER_GROUPS;
    r.i0 = w.ord.grp[grp] + (int64_t)(blockIdx.x / ORDER_GROUPS) * per_block + tid;
    r.i1 = w.ord.grp[grp + 1];
    r.stride = (int64_t)(gridDim.x / ORDER_GROUPS) * per_block;
  } else {
    r.i0 = (int64_t)blockIdx.x * per_block + tid;
    r.i1 = b.n_points;
    r.stride = (int64_t)gridDim.x * per_block;
  }
  return r;
}

// ============================================================== K2 candidates
constexpr int HCAP = 512;  // edge hash slots (>= 2 * MAX_HITS)
// a lane-tier entry that is a node candidate (edge << 4 keeps bits 4..30:
// graphs up to 2^27 edges, checked at engine load)
constexpr uint32_t NODE_ENT = 0x80000000u;
#ifndef OTM_CAND_LANE_CAP
#define OTM_CAND_LANE_CAP 8
#endif
// lane tier: distinct edges kept per probe.  8 measured best on config 2
// (0.39 ms with the wave tier vs 0.40 at 12, 0.45 at 16): a smaller LDS list
// buys occupancy; the ~1 % of probes with more edges in range spill.
constexpr int CAND_LANE_CAP = OTM_CAND_LANE_CAP;
// lane tier block size: 256 (round 4: k_cand_lane 1.518 vs 1.576 ms at 128 on
// config 4, 0.220 vs 0.222 on config 2; 64 no better, profiles/r04_ab/knobs/)
#ifndef OTM_CAND_TB
#define OTM_CAND_TB 256
#endif
// min waves per SIMD for the lane tier: 8 caps it at 64 VGPRs (0.276 ->
// 0.255 ms on config 2, 3.86 -> 3.76 ms on config 4; 6 measured no change)
#ifndef OTM_CAND_WAVES
#define OTM_CAND_WAVES 8
#endif
constexpr int CAND_TB = OTM_CAND_TB;
#ifndef OTM_CAND_INFL
#define OTM_CAND_INFL 2
#endif
constexpr int CAND_INFL = OTM_CAND_INFL;
// lane tier node snap: entries whose projection loads are issued together
// (more would spill under the 64-VGPR cap)
#ifndef OTM_SNAP_B
#define OTM_SNAP_B 2
#endif
constexpr int SNAP_B = OTM_SNAP_B;
// transition index tier: pairs per lane whose first slot loads are issued
// together.  Round 2 measured 2 best (0.337 -> 0.302 ms on config 2, 1.956 ->
// 1.888 ms on config 4; 3 and 4 slower: registers, spills); on round 4's
// kernel 1 is (0.213 / 0.251 / 0.298 ms for 1 / 2 / 3 on config 2, 2.164 /
// 2.351 / 2.478 ms on config 4, profiles/r04_ab/trans_batch/)
#ifndef OTM_TRANS_BATCH
#define OTM_TRANS_BATCH 1
#endif

// wave-reduce a per-lane count and add it to a device counter (all 64 lanes active)
__device__ __forceinline__ void wave_cadd(unsigned long long* c, unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v) atomicAdd(c, v);
}

// Lane tier of the candidate search: one probe per LANE.  The lane walks its
// probe's grid cells serially (the same cell range, entries and projection as
// the wave kernel below), keeps each edge's best (sqdist, shape segment) in a
// private LDS list of CAND_LANE_CAP slots (interleaved by thread), then
// selection-sorts the first max_candidates by (sqdist, edge).  Probes with
// more distinct edges in range spill to the wave kernel, which also applies
// the MAX_HITS spec limit.
template <bool CTR>
__global__ __launch_bounds__(CAND_TB, OTM_CAND_WAVES) void k_cand_lane(DevGraph g, DevBatch b, DevParams P, DevWork w) {
  __shared__ uint32_t sE[CAND_LANE_CAP * CAND_TB];  // edge << 4 | shape segment
  __shared__ float sQ[CAND_LANE_CAP * CAND_TB];     // best squared distance
  uint32_t* E = sE + threadIdx.x;
  float* Q = sQ + threadIdx.x;
  constexpr int S = CAND_TB;
  unsigned long long c_cells = 0, c_ent = 0, c_cand = 0;
  const ItemRange R = item_range(w, b, (P.order_mask & ORDER_CAND) != 0, CAND_TB);
  for (int64_t it = R.i0; it < R.i1; it += R.stride) {
    const int64_t p = R.ordered ? (int64_t)w.ord.item[it] : it;
    if (!R.ordered && !w.is_col[p]) continue;
    if (P.cand_wave_all) {
      const int slot = atomicAdd(&w.counters_i32[5], 1);
      w.overflow_list0[slot] = (int32_t)p;
      continue;
    }
    const float4 pr = w.probe[p];  // {lat, lon, accuracy} of the column (K1), one line
    const float lat = pr.x, lon = pr.y;
    const float r = probe_radius(P, pr.z);
    const float r2 = r * r;
    const float ls = MPD_F * cos_deg(lat);
    const float dlat = r / MPD_F;
    const float dlon = r / ls;
    const double la_lo = ((double)lat - (double)dlat - g.lat0) / g.cell;
    const double la_hi = ((double)lat + (double)dlat - g.lat0) / g.cell;
    const double lo_lo = ((double)lon - (double)dlon - g.lon0) / g.cell;
    const double lo_hi = ((double)lon + (double)dlon - g.lon0) / g.cell;
    const double R = g.grid_rows, Cn = g.grid_cols;
    int r0 = 0, r1 = -1, c0 = 0, c1 = -1;
    if (!(la_hi < 0.0 || lo_hi < 0.0 || la_lo >= R || lo_lo >= Cn)) {
      r0 = la_lo < 0.0 ? 0 : (int)floor(la_lo);
      r1 = la_hi >= R ? (int)R - 1 : (int)floor(la_hi);
      c0 = lo_lo < 0.0 ? 0 : (int)floor(lo_lo);
      c1 = lo_hi >= Cn ? (int)Cn - 1 : (int)floor(lo_hi);
    }
    int n = 0;
    bool spill = false;
    // cells c0..c1 of one grid row are adjacent in the row-major cell CSR:
    // each row's entries are one contiguous range
    const unsigned long long cells = (unsigned long long)(r1 - r0 + 1) * (unsigned long long)(c1 - c0 + 1);
    unsigned long long ents = 0;
    for (int rr = r0; rr <= r1 && !spill; ++rr) {
      {
        const size_t rbase = (size_t)rr * (size_t)g.grid_cols;
        const int64_t q0 = g.cell_off[rbase + c0], q1 = g.cell_off[rbase + c1 + 1];
        if (CTR) ents += (unsigned long long)(q1 - q0);
        // CAND_INFL entries' loads in flight per step, inserted in entry order: 2 keeps
        // the 64-VGPR cap without scratch (0.251 -> 0.246 ms config 2, 3.72 -> 3.66 ms config 4 against 4)
        for (int64_t q = q0; q < q1 && !spill; q += CAND_INFL) {
          float sq[CAND_INFL];
          uint32_t en[CAND_INFL];
#pragma unroll
          for (int u = 0; u < CAND_INFL; ++u) {
            sq[u] = INFINITY;
            en[u] = 0;
            if (q + u < q1) {
              const float4 G = g.ent_geo[q + u];
              sq[u] = seg_sqdist(G.x, G.y, G.z, G.w, lat, lon, ls);
            }
          }
          // the entry's id only for a hit (~1 in 7 entries): the scattered
          // load is issued by the lanes that need it, not by every lane
#pragma unroll
          for (int u = 0; u < CAND_INFL; ++u)
            if (sq[u] <= r2) en[u] = g.cell_ent[q + u];
#pragma unroll
          for (int u = 0; u < CAND_INFL; ++u) {
            const float sqd = sq[u];
            if (spill || !(sqd <= r2)) continue;
            const uint32_t ent = en[u];
            const uint32_t e = ent >> 4;
            // every slot's edge read at once and unconditionally -- slots past
            // n hold stale words, masked by the select -- so the compiler
            // emits eight LDS reads and selects, not eight guarded branches
            // (one LDS round trip per hit instead of up to 8)
            uint32_t ev[CAND_LANE_CAP];
#pragma unroll
            for (int m = 0; m < CAND_LANE_CAP; ++m) ev[m] = E[m * S];
            int f = -1;
#pragma unroll
            for (int m = 0; m < CAND_LANE_CAP; ++m) f = (m < n && (ev[m] >> 4) == e) ? m : f;
            if (f < 0) {
              if (n == CAND_LANE_CAP) {
                spill = true;
                continue;
              }
              E[n * S] = ent;
              Q[n * S] = sqd;
              ++n;
            } else {
              const float qf = Q[f * S];
              if (sqd < qf || (sqd == qf && (ent & 15u) < (E[f * S] & 15u))) {
                Q[f * S] = sqd;
                E[f * S] = ent;
              }
            }
          }
        }
      }
    }
    if (spill) {
      const int slot = atomicAdd(&w.counters_i32[5], 1);
      w.overflow_list0[slot] = (int32_t)p;
      continue;
    }
    // node snap: an entry whose projection snaps to a node becomes that
    // node's candidate (NODE_ENT | first outgoing edge << 4), one per node
    // at the smallest distance.  First every entry's snap, SNAP_B entries'
    // loads issued together (a pure function of the entry: round 6 -- the
    // entry-by-entry walk waited on 3-4 dependent loads per entry); then the
    // merge in entry order, out of LDS.
    for (int m0 = 0; m0 < n; m0 += SNAP_B) {
      uint32_t em[SNAP_B];
      ProjIn pin[SNAP_B];
#pragma unroll
      for (int u = 0; u < SNAP_B; ++u) {
        em[u] = m0 + u < n ? E[(m0 + u) * S] : 0u;
        if (m0 + u < n) pin[u] = proj_load(g, (int32_t)(em[u] >> 4), (int32_t)(em[u] & 15u));
      }
      int32_t vx[SNAP_B];
      bool node0[SNAP_B], at_end[SNAP_B];
#pragma unroll
      for (int u = 0; u < SNAP_B; ++u) {
        vx[u] = 0;
        node0[u] = at_end[u] = false;
        if (m0 + u < n) {
          float sqd, off;
          proj_calc(pin[u], lat, lon, ls, sqd, off, at_end[u]);
          node0[u] = off == 0.0f;
          const int32_t e = (int32_t)(em[u] >> 4);
          if (node0[u] || at_end[u]) vx[u] = node0[u] ? g.e_from[e] : g.e_to[e];
        }
      }
#pragma unroll
      for (int u = 0; u < SNAP_B; ++u) {
        // snap_node's rule: the start node at offset 0; the end node when
        // clamped there and it has an outgoing edge
        if (node0[u] || at_end[u]) {
          const int32_t o0 = g.out_off[vx[u]], o1 = g.out_off[vx[u] + 1];
          if (node0[u] || o1 > o0) E[(m0 + u) * S] = NODE_ENT | ((uint32_t)o0 << 4);
        }
      }
    }
    for (int m = 0; m < n; ++m) {
      const uint32_t key = E[m * S];
      if (!(key & NODE_ENT)) continue;
      int f = -1;
      for (int t = 0; t < m; ++t)
        if (E[t * S] == key) f = t;
      if (f >= 0) {
        const float qm = Q[m * S];
        if (qm < Q[f * S]) Q[f * S] = qm;
        --n;  // drop entry m: the last entry moves here and is examined next
        E[m * S] = E[n * S];
        Q[m * S] = Q[n * S];
        --m;
      }
    }
    const int K = n < P.max_candidates ? n : P.max_candidates;
    const float ds = (2.0f * P.sigma_z) * P.sigma_z;
    for (int j = 0; j < K; ++j) {
      // selection by (sqdist, edge, node before edge candidate)
      int m = j;
      float qm = Q[j * S];
      uint32_t em = E[j * S];
      for (int t = j + 1; t < n; ++t) {
        const float qt = Q[t * S];
        const uint32_t et = E[t * S];
        const uint32_t xt = (et & ~NODE_ENT) >> 4, xm = (em & ~NODE_ENT) >> 4;
        if (qt < qm || (qt == qm && (xt < xm || (xt == xm && et > em)))) {
          m = t;
          qm = qt;
          em = et;
        }
      }
      if (m != j) {
        Q[m * S] = Q[j * S];
        E[m * S] = E[j * S];
        Q[j * S] = qm;
        E[j * S] = em;
      }
    }
    // the K chosen, in order: the point's inline blocks whole (its 8-B
    // records in 16-B stores, its emissions in 16-B pieces; unused slots: edge
    // -1, emission +inf) -- whole lines to write back, not partially written
    // ones -- and any candidates past KIN one by one into its overflow slots
    int4* eo4 = (int4*)(w.cand_eo + p * KIN);
    float4* em4 = (float4*)(w.cand_em + p * KIN);
    float emv[4];
#pragma unroll
    for (int j = 0; j < (CAND_LANE_CAP > KIN ? CAND_LANE_CAP : KIN); j += 2) {
      if (j >= KIN && j >= K) break;
      int32_t e2[2];
      float o2[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int jj = j + u;
        e2[u] = -1;
        o2[u] = 0.0f;
        float emj = INFINITY;
        if (jj < K) {
          const uint32_t en = E[jj * S];
          const int32_t e = (int32_t)((en & ~NODE_ENT) >> 4);
          float sqd = Q[jj * S], off = 0.0f;
          if (!(en & NODE_ENT)) project(g, e, (int32_t)(en & 15u), lat, lon, ls, sqd, off);
          e2[u] = e;
          o2[u] = off;
          emj = sqd / ds;
        }
        emv[(j + u) & 3] = emj;
      }
      if (j < KIN) {
        eo4[j >> 1] = make_int4(e2[0], __float_as_int(o2[0]), e2[1], __float_as_int(o2[1]));
        if ((j & 3) == 2) em4[j >> 2] = make_float4(emv[0], emv[1], emv[2], emv[3]);
      } else {
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (j + u < K) {
            w.cand_xeo[p * KX + (j + u - KIN)] = make_int2(e2[u], __float_as_int(o2[u]));
            w.cand_xem[p * KX + (j + u - KIN)] = emv[(j + u) & 3];
          }
      }
    }

    w.ncand[p] = K;
    if (CTR) {
      c_cells += cells;
      c_ent += ents;
      c_cand += (unsigned long long)K;
    }
  }
  if (CTR) {
    wave_cadd(&w.ctr->cells_visited, c_cells);
    wave_cadd(&w.ctr->cell_entries_scanned, c_ent);
    wave_cadd(&w.ctr->candidates, c_cand);
  }
}

template <bool BIG>
struct Mem;
template <>
struct Mem<false> {  // LDS
  template <class T>
  __device__ static T ld(const T* p) {
    return *p;
  }
  template <class T>
  __device__ static void st(T* p, T v) {
    *p = v;
  }
};
template <>
struct Mem<true> {  // global scratch: keep every access at L2 (agent scope)
  template <class T>
  __device__ static T ld(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  template <class T>
  __device__ static void st(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
};

// Wave tier: one wavefront per spilled probe (list from the lane tier).
// BIG = false: LDS tables (MAX_HITS distinct edges); a probe with more goes
// to the list of the BIG form (overflow_list3, count [24]), whose tables
// (2^cand_log2 slots per block, in HBM) the host sizes: none until needed,
// grown 4x with the batch redone when a probe does not fit (no limit on the
// edges within a radius but memory; round 4 dropped the 256-edge spec limit).
template <bool BIG>
__global__ __launch_bounds__(TB) void k_candidates(DevGraph g, DevBatch b, DevParams P, DevWork w) {
  __shared__ uint32_t l_hkey[BIG ? 1 : HCAP];
  __shared__ unsigned long long l_hval[BIG ? 1 : HCAP];
  __shared__ unsigned long long l_skey[BIG ? 1 : MAX_HITS];
  __shared__ int64_t cstart[64];
  __shared__ int cexcl[64];
  __shared__ int s_count, s_over, s_n;
  const int lane = threadIdx.x;
  const int64_t nwork = BIG ? w.counters_i32[24] : w.counters_i32[5];
  const int32_t* list = BIG ? w.overflow_list3 : w.overflow_list0;
  if (BIG && nwork > 0 && w.cand_log2 == 0) {
    // no tables yet: the host makes them and redoes the batch -- or, when it
    // cannot (cand_final), these probes' traces answer 500 (OTM_TERR_CAND_OVERFLOW)
    for (int64_t it = (int64_t)blockIdx.x * TB + lane; it < nwork; it += (int64_t)gridDim.x * TB) {
      w.ncand[list[it]] = 0;
      if (w.cand_final) atomicCAS(&w.trace_err[w.pt_trace[list[it]]], 0, OTM_TERR_CAND_OVERFLOW);
    }
    if (!w.cand_final && blockIdx.x == 0 && lane == 0) {
      w.counters_i32[25] = 1;
      *w.abort = 1;
    }
    return;
  }
  const int hlog2 = BIG ? w.cand_log2 : 9;
  const int hcap = 1 << hlog2;
  const int max_hits = hcap / 2;
  uint32_t* hkey = BIG ? w.cbig_key + (size_t)blockIdx.x * hcap : l_hkey;
  unsigned long long* hval = BIG ? w.cbig_val + (size_t)blockIdx.x * hcap : l_hval;
  unsigned long long* skey = BIG ? w.cbig_skey + (size_t)blockIdx.x * max_hits : l_skey;
  for (int64_t it = blockIdx.x; it < nwork; it += gridDim.x) {
    const int64_t p = list[it];
    const float4 pr = w.probe[p];  // {lat, lon, accuracy} of the column (K1), one line
    const float lat = pr.x, lon = pr.y;
    const float r = probe_radius(P, pr.z);
    const float r2 = r * r;
    const float ls = MPD_F * cos_deg(lat);
    const float dlat = r / MPD_F;
    const float dlon = r / ls;
    const double la_lo = ((double)lat - (double)dlat - g.lat0) / g.cell;
    const double la_hi = ((double)lat + (double)dlat - g.lat0) / g.cell;
    const double lo_lo = ((double)lon - (double)dlon - g.lon0) / g.cell;
    const double lo_hi = ((double)lon + (double)dlon - g.lon0) / g.cell;
    const double R = g.grid_rows, Cn = g.grid_cols;
    int r0 = 0, r1 = -1, c0 = 0, c1 = -1;
    if (!(la_hi < 0.0 || lo_hi < 0.0 || la_lo >= R || lo_lo >= Cn)) {
      r0 = la_lo < 0.0 ? 0 : (int)floor(la_lo);
      r1 = la_hi >= R ? (int)R - 1 : (int)floor(la_hi);
      c0 = lo_lo < 0.0 ? 0 : (int)floor(lo_lo);
      c1 = lo_hi >= Cn ? (int)Cn - 1 : (int)floor(lo_hi);
    }
    const int ncols = c1 - c0 + 1;
    const int ncells = (r1 - r0 + 1) * ncols;
    for (int i = lane; i < hcap; i += TB) {
      Mem<BIG>::st(&hkey[i], (uint32_t)EMPTY);
      Mem<BIG>::st(&hval[i], (unsigned long long)LAB_NONE);
    }
    if (lane == 0) {
      s_count = 0;
      s_over = 0;
      s_n = 0;
    }
    __syncthreads();
    unsigned long long scanned = 0;
    for (int cb = 0; cb < ncells; cb += TB) {
      const int c = cb + lane;
      int cnt = 0;
      int64_t cs = 0;
      if (c < ncells) {
        const int rr = r0 + c / ncols, cc = c0 + c % ncols;
        const size_t cidx = (size_t)rr * (size_t)g.grid_cols + (size_t)cc;
        cs = g.cell_off[cidx];
        cnt = (int)(g.cell_off[cidx + 1] - cs);
      }
      const int incl = wave_incl_scan(cnt, lane);
      const int total = __shfl(incl, 63, 64);
      cexcl[lane] = incl - cnt;
      cstart[lane] = cs;
      __syncthreads();
      const int nc_here = min(TB, ncells - cb);
      for (int gi = lane; gi < total; gi += TB) {
        // cell holding entry gi: largest k with cexcl[k] <= gi
        int lo = 0, hi = nc_here - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (cexcl[mid] <= gi) lo = mid;
          else hi = mid - 1;
        }
        const uint32_t ent = g.cell_ent[cstart[lo] + (gi - cexcl[lo])];
        const int32_t e = (int32_t)(ent >> 4), k = (int32_t)(ent & 15u);
        float sqd, off;
        project(g, e, k, lat, lon, ls, sqd, off);
        if (!(sqd <= r2)) continue;
        uint32_t slot = hash32((uint32_t)e) >> (32 - hlog2);
        bool placed = false;
        for (int probe = 0; probe < hcap; ++probe) {
          const uint32_t old = atomicCAS(&hkey[slot], EMPTY, (uint32_t)e);
          if (old == EMPTY) {
            if (atomicAdd(&s_count, 1) >= max_hits) s_over = 1;
            placed = true;
            break;
          }
          if (old == (uint32_t)e) {
            placed = true;
            break;
          }
          slot = (slot + 1) & (uint32_t)(hcap - 1);
        }
        if (!placed) {
          s_over = 1;
          continue;
        }
        atomicMin(&hval[slot], ((unsigned long long)fbits(sqd) << 32) | (unsigned long long)k);
      }
      scanned += (unsigned long long)total;
      __syncthreads();
    }
    if (s_over) {
      if (lane == 0) {
        if (!BIG) {
          w.overflow_list3[atomicAdd(&w.counters_i32[24], 1)] = (int32_t)p;  // to the HBM tables
        } else if (w.cand_final) {
          // the tables are as large as they get: this probe's trace fails
          // alone (500, OTM_TERR_CAND_OVERFLOW), the batch goes on
          w.ncand[p] = 0;
          atomicCAS(&w.trace_err[w.pt_trace[p]], 0, OTM_TERR_CAND_OVERFLOW);
        } else {
          w.ncand[p] = 0;
          w.counters_i32[25] = 1;  // the tables are too small: grow, redo the batch
          *w.abort = 1;
        }
      }
      __syncthreads();
      continue;
    }
    // compact the distinct edges as sqdist bits << 32 | edge << 5 | shape
    // segment << 1; the edge table is then reused as the node table.  Each
    // edge is projected once, lane-parallel over the compacted list: an edge
    // candidate gets flag bit 1; one whose projection snaps to a node leaves
    // LAB_NONE (sorts last) and meets the other edges at that node in the node
    // table (key: the node's first outgoing edge; value: the smallest sqdist
    // bits << 32 | a slot of the group), which writes the node candidate
    // sqdist bits << 32 | first outgoing edge << 5 into that slot -- so a node
    // sorts before an edge candidate of the same edge at the same distance.
    for (int i = lane; i < hcap; i += TB) {
      const uint32_t hk = Mem<BIG>::ld(&hkey[i]);
      if (hk != EMPTY) {
        const unsigned long long hv = Mem<BIG>::ld(&hval[i]);
        const int idx = atomicAdd(&s_n, 1);
        Mem<BIG>::st(&skey[idx],
                     (hv & 0xFFFFFFFF00000000ull) | ((unsigned long long)hk << 5) | ((hv & 15ull) << 1));
      }
    }
    __syncthreads();
    for (int i = lane; i < hcap; i += TB) {
      Mem<BIG>::st(&hkey[i], (uint32_t)EMPTY);
      Mem<BIG>::st(&hval[i], (unsigned long long)LAB_NONE);
    }
    if (lane == 0) s_count = 0;  // from here: distinct candidates
    __syncthreads();
    const int n0 = s_n;
    for (int idx = lane; idx < n0; idx += TB) {
      const unsigned long long key = Mem<BIG>::ld(&skey[idx]);
      const int32_t e = (int32_t)(((uint32_t)key) >> 5);
      float sqd, off;
      bool at_end;
      project(g, e, (int32_t)((key >> 1) & 15ull), lat, lon, ls, sqd, off, at_end);
      const int32_t v = snap_node(g, e, off, at_end);
      if (v < 0) {
        Mem<BIG>::st(&skey[idx], key | 1ull);
        atomicAdd(&s_count, 1);
      } else {
        Mem<BIG>::st(&skey[idx], (unsigned long long)LAB_NONE);
        const uint32_t rep = (uint32_t)g.out_off[v];
        uint32_t slot = hash32(rep) >> (32 - hlog2);
        while (true) {
          const uint32_t old = atomicCAS(&hkey[slot], EMPTY, rep);
          if (old == EMPTY || old == rep) break;
          slot = (slot + 1) & (uint32_t)(hcap - 1);
        }
        atomicMin(&hval[slot], (key & 0xFFFFFFFF00000000ull) | (unsigned long long)idx);
      }
    }
    __syncthreads();
    for (int i = lane; i < hcap; i += TB) {
      const uint32_t hk = Mem<BIG>::ld(&hkey[i]);
      if (hk != EMPTY) {
        const unsigned long long hv = Mem<BIG>::ld(&hval[i]);
        Mem<BIG>::st(&skey[(int)(hv & 0xFFFFFFFFull)], (hv & 0xFFFFFFFF00000000ull) | ((unsigned long long)hk << 5));
        atomicAdd(&s_count, 1);
      }
    }
    __syncthreads();
    const int ns = n0;  // entries in skey (snapped edges past their node's slot: LAB_NONE)
    const int n = s_count;  // distinct candidates
    int N = 1;
    while (N < ns) N <<= 1;
    for (int i = ns + lane; i < N; i += TB) Mem<BIG>::st(&skey[i], (unsigned long long)LAB_NONE);
    __syncthreads();
    // bitonic sort ascending
    for (int kk = 2; kk <= N; kk <<= 1) {
      for (int j = kk >> 1; j > 0; j >>= 1) {
        for (int i = lane; i < N; i += TB) {
          const int ixj = i ^ j;
          if (ixj > i) {
            const unsigned long long x = Mem<BIG>::ld(&skey[i]), y = Mem<BIG>::ld(&skey[ixj]);
            const bool up = (i & kk) == 0;
            if ((x > y) == up) {
              Mem<BIG>::st(&skey[i], y);
              Mem<BIG>::st(&skey[ixj], x);
            }
          }
        }
        __syncthreads();
      }
    }
    const int K = n < P.max_candidates ? n : P.max_candidates;
    if (lane < K) {
      const unsigned long long key = Mem<BIG>::ld(&skey[lane]);
      const int32_t e = (int32_t)(((uint32_t)key) >> 5);
      float sqd = bitsf((uint32_t)(key >> 32)), off = 0.0f;
      if (key & 1ull) project(g, e, (int32_t)((key >> 1) & 15ull), lat, lon, ls, sqd, off);
      const float ds = (2.0f * P.sigma_z) * P.sigma_z;
      cput(w, p, lane, e, off, sqd / ds);
    } else if (lane < KIN) {
      cput(w, p, lane, -1, 0.0f, INFINITY);  // the rest of the inline block (whole lines written back)
    }
    if (lane == 0) {
      w.ncand[p] = K;
      if (w.ctr) {
        cadd(&w.ctr->cells_visited, (unsigned long long)ncells);
        cadd(&w.ctr->cell_entries_scanned, scanned);
        cadd(&w.ctr->candidates, (unsigned long long)K);
      }
    }
    __syncthreads();
  }
}

// ============================================================== K3 links
__global__ __launch_bounds__(256) void k_links(DevBatch b, DevParams P, DevWork w) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p > b.n_points) return;
  if (p == b.n_points) {
    w.trans_off[p] = 0;
    // spill snapshot A: candidate probes the lane tier handed to the wave
    // tier; the counters start over for the transition tiers
    if (OTM_FOLD_BOOKKEEPING) fold_snap(w, 0, true);
    return;
  }
  int32_t cp = -1, kq = 0;
  int64_t cnt = 0;
  if (w.is_col[p]) {
    const int32_t q = w.prevc[p];
    if (q >= 0 && p - q > 1) w.nextc[q] = (int32_t)p;  // interpolated points between: K7a finds p from them
    if (q >= 0 && w.ncand[p] > 0 && w.ncand[q] > 0 && w.gc[p] <= P.breakage) {
      cp = q;
      kq = w.ncand[q];
      cnt = (int64_t)kq * (int64_t)w.ncand[p];
    }
  }
  w.col_prev[p] = cp;
  w.kq_prev[p] = kq;
  w.trans_off[p] = cnt;
  // K4's record of the column in spatial-order position (k_trans_sub then
  // reads it with one coalesced load instead of an order lookup and five
  // scattered ones)
  if (w.colrec && (P.order_mask & ORDER_TRANS) && w.is_col[p])
    w.colrec[w.colrec_pos[p]] = make_int4((int32_t)p, cp, kq | (w.ncand[p] << 8), __float_as_int(w.gc[p]));
  // Viterbi's byte (k_viterbi_g): ncand <= KMAX = 32 fits six bits
  w.vmeta[p] = (uint8_t)((w.is_col[p] ? (w.ncand[p] | 0x40) : 0) | (cp >= 0 ? 0x80 : 0));
}

// Batch bookkeeping in single-wave kernels rather than memset / memcpy
// commands: each runtime copy or fill is its own blit dispatch (3.5-8 us
// each on the stream, ~60 us per batch before).
__global__ void k_batch_init(int32_t* counters, int32_t* abort) {
  const int t = threadIdx.x;
  if (t < 32) counters[t] = 0;
  if (t == 0) *abort = 0;
}
// spill snapshot: copy the 16 tier counters, optionally zeroing them for the
// next stage's tiers
__global__ void k_snap(int32_t* counters, int32_t* snap, int reset) {
  const int t = threadIdx.x;
  if (t < 16) {
    snap[t] = counters[t];
    if (reset) counters[t] = 0;
  }
}
// the batch's status for the host's one synchronisation: abort flag,
// transition total, path-pool counters
__global__ void k_status(const int32_t* abort, const int64_t* ttotal, const int32_t* counters, BatchStatus* out) {
  if (threadIdx.x == 0) {
    out->abort = *abort;
    out->grow = (counters[23] != 0 ? 1 : 0) | (counters[25] != 0 ? 2 : 0);
    out->ttotal = *ttotal;
    out->cnt[0] = counters[0];
    out->cnt[1] = counters[1];
    out->cnt[2] = counters[2];
    out->route_huge = counters[22];
  }
}

// the transition matrices' total (scan of K3's sizes) against the buffer
__global__ void k_cap_check(DevBatch b, DevWork w) {
  if (w.trans_off[b.n_points] > w.trans_cap) *w.abort = 1;
}



// ============================================================== turn-aware bounded search
// DESIGN.md §3 rule 4 (oracle ta_search): the route of a transition is the
// cheapest by distance plus turn penalty.  A search from node u entered with
// heading hin labels every edge g with its departure label -- the cheapest way
// to be at g's start, turned into it -- and every node v with its arrival
// label, each a 64-bit key cost << 32 | predecessor edge (costs in 1/64 m:
// L(e) = round(len x 64) per edge, turn units per turn), bounded by cost cmax.
// Label-correcting in one wavefront with 64-bit atomicMin: every label
// converges to the minimum over its in-steps, the unique fixed point (every
// step costs > 0), which the oracle's Dijkstra computes -- whatever the
// relaxation order.  A key enters the table once (the set of keys ever
// inserted is exactly those whose label is within cmax), so the count is
// order-free too.
struct Table {
  uint32_t* key;            // edge id, NODE_KEY | node, or EMPTY
  unsigned long long* lab;  // cost << 32 | predecessor edge
  uint32_t* inq;            // in next frontier
  uint32_t* fr0;            // frontier A (slot ids)
  uint32_t* fr1;            // frontier B
  int cap_log2;
  int limit;                // max labels before overflow
  // global tier only: the slots the last search inserted (its first `limit`)
  // and how many (*prev, -1: unknown), so the next search clears those instead
  // of the whole 128K-slot table (the tables start clean: engine.cpp ensure_big)
  uint32_t* ins = nullptr;
  int32_t* prev = nullptr;
};

struct SearchShared {
  int nfr, nnext, count, over;
};

template <bool BIG>
__device__ __forceinline__ int table_find(const Table& T, uint32_t v) {
  const uint32_t mask = (1u << T.cap_log2) - 1u;
  uint32_t slot = hash32(v) >> (32 - T.cap_log2);
  for (int i = 0; i <= (int)mask; ++i) {
    const uint32_t k = Mem<BIG>::ld(&T.key[slot]);
    if (k == v) return (int)slot;
    if (k == EMPTY) return -1;
    slot = (slot + 1) & mask;
  }
  return -1;
}

// lower key's label to nl (inserting the key); an edge key whose cost fell
// joins the next frontier
template <bool BIG>
__device__ __forceinline__ void ta_relax(const Table& T, SearchShared& S, uint32_t* nxt, uint32_t key,
                                         unsigned long long nl) {
  const uint32_t mask = (1u << T.cap_log2) - 1u;
  uint32_t slot = hash32(key) >> (32 - T.cap_log2);
  int found = -1;
  for (int i = 0; i <= (int)mask; ++i) {
    const uint32_t old = atomicCAS(&T.key[slot], EMPTY, key);
    if (old == EMPTY) {
      const int c = atomicAdd(&S.count, 1);
      if (c >= T.limit) S.over = 1;
      else if (BIG) Mem<true>::st(&T.ins[c], slot);
      found = (int)slot;
      break;
    }
    if (old == key) {
      found = (int)slot;
      break;
    }
    slot = (slot + 1) & mask;
  }
  if (found < 0) {
    S.over = 1;
    return;
  }
  const unsigned long long old = atomicMin(&T.lab[found], nl);
  // successors depend on the cost alone (their predecessor is this edge)
  if (!(key & NODE_KEY) && nl < old && (uint32_t)(old >> 32) != (uint32_t)(nl >> 32)) {
    if (atomicExch(&T.inq[found], 1u) == 0u) {
      const int idx = atomicAdd(&S.nnext, 1);
      Mem<BIG>::st(&nxt[idx], (uint32_t)found);
    }
  }
}

// returns >= 0 labels, or -1 on overflow (more than T.limit)
template <bool BIG>
__device__ int ta_search(const DevGraph& g, const uint32_t* TU, const Table& T, SearchShared& S, int32_t u,
                         uint32_t hin, uint32_t cmax, int lane) {
  const int cap = 1 << T.cap_log2;
  // a clean table: the LDS tier's whole, the global tier's the slots its last
  // search inserted (all of them after an overflow)
  const int pc = BIG ? Mem<true>::ld(T.prev) : -1;
  if (pc < 0) {
    for (int i = lane; i < cap; i += TB) {
      Mem<BIG>::st(&T.key[i], EMPTY);
      Mem<BIG>::st(&T.lab[i], LAB_NONE);
      Mem<BIG>::st(&T.inq[i], 0u);
    }
  } else {
    for (int i = lane; i < pc; i += TB) {
      const uint32_t sl = Mem<true>::ld(&T.ins[i]);
      Mem<BIG>::st(&T.key[sl], EMPTY);
      Mem<BIG>::st(&T.lab[sl], LAB_NONE);
      Mem<BIG>::st(&T.inq[sl], 0u);
    }
  }
  if (lane == 0) {
    S.nfr = 0;
    S.nnext = 0;
    S.count = 0;
    S.over = 0;
  }
  __syncthreads();
  uint32_t* cur = T.fr0;
  uint32_t* nxt = T.fr1;
  // the source node (arrival 0) and the route's possible first edges
  if (lane == 0) ta_relax<BIG>(T, S, nxt, NODE_KEY | (uint32_t)u, (unsigned long long)NONE_PRED);
  const int32_t e0 = g.out_off[u], e1 = g.out_off[u + 1];
  for (int32_t e = e0 + lane; e < e1; e += TB) {
    const uint32_t c = turn_units(TU, hin, g.e_head_out[e]);
    if (c <= cmax) ta_relax<BIG>(T, S, nxt, (uint32_t)e, ((unsigned long long)c << 32) | NONE_PRED);
  }
  __syncthreads();
  while (true) {
    if (lane == 0) {
      S.nfr = S.nnext;
      S.nnext = 0;
    }
    uint32_t* tmp = cur;
    cur = nxt;
    nxt = tmp;
    __syncthreads();
    const int nfr = S.nfr;
    if (nfr == 0 || S.over) break;
    for (int f = lane; f < nfr; f += TB) {
      const uint32_t sl = Mem<BIG>::ld(&cur[f]);
      if (BIG) atomicExch(&T.inq[sl], 0u);
      else T.inq[sl] = 0u;
      const int32_t e = (int32_t)Mem<BIG>::ld(&T.key[sl]);
      const unsigned long long ca =
          (unsigned long long)(uint32_t)(Mem<BIG>::ld(&T.lab[sl]) >> 32) + (unsigned long long)g.e_len64[e];
      if (ca > cmax) continue;
      const int32_t v = g.e_to[e];
      ta_relax<BIG>(T, S, nxt, NODE_KEY | (uint32_t)v, (ca << 32) | (uint32_t)e);
      const uint32_t hv = g.e_head_in[e];
      for (int32_t h = g.out_off[v]; h < g.out_off[v + 1]; ++h) {
        const unsigned long long c = ca + turn_units(TU, hv, g.e_head_out[h]);
        if (c <= cmax) ta_relax<BIG>(T, S, nxt, (uint32_t)h, (c << 32) | (uint32_t)e);
      }
    }
    __syncthreads();
  }
  const bool over = S.over != 0;
  const int count = S.count;
  if (BIG && lane == 0) Mem<true>::st(T.prev, over || count > T.limit ? -1 : count);
  __syncthreads();
  return over ? -1 : count;
}

// work counts of a converged search (oracle ta_search's counters): the
// departure labels, and the edges they relax (their end node's out-edges,
// when the arrival is within the bound)
template <bool BIG>
__device__ void ta_counts(const DevGraph& g, const Table& T, uint32_t cmax, int lane, unsigned long long& settled,
                          unsigned long long& relaxed) {
  unsigned long long st = 0, rl = 0;
  const int cap = 1 << T.cap_log2;
  for (int i = lane; i < cap; i += TB) {
    const uint32_t k = Mem<BIG>::ld(&T.key[i]);
    if (k == EMPTY || (k & NODE_KEY)) continue;
    ++st;
    const unsigned long long ca = (Mem<BIG>::ld(&T.lab[i]) >> 32) + (unsigned long long)g.e_len64[k];
    if (ca <= cmax) rl += (unsigned long long)(g.out_off[g.e_to[k] + 1] - g.out_off[g.e_to[k]]);
  }
  for (int o = 32; o > 0; o >>= 1) {
    st += __shfl_xor(st, o, 64);
    rl += __shfl_xor(rl, o, 64);
  }
  settled = st;
  relaxed = rl;
}

// The route a converged label ends: its predecessor chain (fully traversed
// edges), walked back from `pred0` into the lane's LDS buffer buf (stride TB,
// CHAIN_BUF entries; a longer chain is re-walked per edge), then summed in
// route order: the distance d and the turn units from heading hin through the
// chain, plus the turn into hout (NO_HEAD: none).  predof(e) = e's departure
// label's predecessor.
constexpr int CHAIN_BUF = 32;
template <class F>
__device__ void chain_sums(const DevGraph& g, const uint32_t* TU, F predof, uint32_t pred0, uint32_t hin,
                           uint32_t hout, int32_t* buf, float& d, uint32_t& units, int& n) {
  int cnt = 0;
  for (uint32_t p = pred0; p != NONE_PRED && cnt < (1 << 26); p = predof(p)) {
    if (cnt < CHAIN_BUF) buf[cnt * TB] = (int32_t)p;
    ++cnt;
  }
  float dd = 0.0f;
  unsigned long long un = 0;
  uint32_t h = hin;
  for (int m = cnt - 1; m >= 0; --m) {
    int32_t e;
    if (cnt <= CHAIN_BUF) {
      e = buf[m * TB];
    } else {
      uint32_t x = pred0;
      for (int k = 0; k < m; ++k) x = predof(x);
      e = (int32_t)x;
    }
    un += turn_units(TU, h, g.e_head_out[e]);
    dd = dd + g.e_len[e];
    h = g.e_head_in[e];
  }
  un += turn_units(TU, h, hout);
  d = dd;
  units = un > TURN_UNITS_MAX ? TURN_UNITS_MAX : (uint32_t)un;
  n = cnt;
}

// ============================================================== route index
__device__ __forceinline__ uint32_t idx_hash(uint32_t v) {
  v ^= v >> 16;
  v *= 0x85ebca6bu;
  v ^= v >> 13;
  v *= 0xc2b2ae35u;
  v ^= v >> 16;
  return v;
}

// A row's table: entries x 100 / pct slots rounded up to an even count (at
// least one slot empty, so every probe ends), the hash mapped onto its 2-slot
// buckets by a multiply-high.  A label's probe starts at its bucket's first
// slot and goes on linearly; a lookup loads the bucket's two slots (32 aligned
// bytes, one line) at once, which holds the label or ends the probe for most
// lookups.  A slot is 16 bytes with the predecessor inside (idx_slot_*).  The
// engine picks pct per index (engine.cpp build_index_at): IDX_LOAD_FAST (30 %,
// 53 B per entry) when the tables fit the HBM budget, IDX_LOAD_DENSE (40 %,
// 40 B per entry) when only that fits -- measured on configs 2 / 4 / 3,
// k_trans_sub at 40 % is 9 / 6 / 7 % slower than at 30 % (more lookups past
// their bucket), round 4's 20-B slots at 20 % (100 B per entry) 1 / 2 / 1 %
// faster.
constexpr int IDX_LOAD_FAST = 30, IDX_LOAD_DENSE = 40;
__host__ __device__ __forceinline__ int64_t idx_row_cap(int32_t c, int pct) {
  if (c <= 0) return 0;
  int64_t cap = ((int64_t)c * 100 + pct - 1) / pct;
  if (cap <= c) cap = (int64_t)c + 1;
  return (cap + 1) & ~(int64_t)1;
}
// first slot of a label's probe in row R (its bucket's first slot)
__device__ __forceinline__ uint32_t idx_slot0(uint32_t hh, const IdxRow& R) {
  return (uint32_t)(((uint64_t)hh * (uint64_t)(R.cap >> 1)) >> 32) << 1;
}
__device__ __forceinline__ uint32_t idx_next(uint32_t h, const IdxRow& R) {
  return h + 1u == R.cap ? 0u : h + 1u;
}
// A slot {key, cost | pred lo << 24, route distance bits, units | pred hi << 24}:
// cost and turn units below 2^24 (units <= cost <= the index's cmax, and the
// index radius is capped so that cmax < 2^24), the 16-bit predecessor slot in
// the row split over the two top bytes (IDX_NO_PRED: the route's first edge).
constexpr uint32_t IDX_LOW24 = 0xFFFFFFu;
constexpr uint32_t IDX_NO_PRED = 0xFFFFu;
static_assert((int64_t)INDEX_BUILD_LIMIT * 100 / IDX_LOAD_FAST + 2 < (int64_t)IDX_NO_PRED,
              "a row's slots must be numbered in 16 bits");
__host__ __device__ __forceinline__ uint32_t idx_slot_cost(const uint4& s) { return s.y & IDX_LOW24; }
__host__ __device__ __forceinline__ uint32_t idx_slot_units(const uint4& s) { return s.w & IDX_LOW24; }
__host__ __device__ __forceinline__ int32_t idx_slot_pred(const uint4& s) {
  const uint32_t p = (s.y >> 24) | ((s.w >> 24) << 8);
  return p == IDX_NO_PRED ? -1 : (int32_t)p;
}

// Row lookup: linear probing in the row's table from the key's bucket, a
// bucket (two slots) per load.  Returns the slot (its contents in *out) when
// the key is in the row, -1 when absent (its label beyond cmax), -2 when the
// row is incomplete.
__device__ __forceinline__ int64_t idx_find(const uint4* slot, const IdxRow& R, uint32_t v, uint4& out) {
  if (R.cnt < 0) return -2;
  if (R.cnt == 0) return -1;
  uint32_t h = idx_slot0(idx_hash(v), R);
  while (true) {
    const uint4 a = slot[R.off + h], b = slot[R.off + h + 1];
    if (a.x == v) {
      out = a;
      return R.off + h;
    }
    if (a.x == EMPTY) return -1;
    if (b.x == v) {
      out = b;
      return R.off + h + 1;
    }
    if (b.x == EMPTY) return -1;
    h = h + 2u == R.cap ? 0u : h + 2u;
  }
}
// the index row of a candidate as the source of a route: its edge's row
// (entered along the edge), or its node's (a node candidate, no heading)
__device__ __forceinline__ int64_t src_row(const DevGraph& g, int32_t e, float off) {
  return cand_node(off) ? (int64_t)g.n_edges + g.e_from[e] : (int64_t)e;
}
// the label a route to a candidate ends on: its edge's departure label, or its
// node's arrival label (a node candidate)
__device__ __forceinline__ uint32_t dst_key(const DevGraph& g, int32_t e, float off) {
  return cand_node(off) ? NODE_KEY | (uint32_t)g.e_from[e] : (uint32_t)e;
}

// Index build: one wavefront per row runs the row's search with bound cmax in
// an LDS table of INDEX_BUILD_CAP slots (the online tiers' fixed point), then
// inserts every label into the row's table with its cost, route distance and
// turn units (each lane walks its label's predecessor chain in the LDS table),
// and then, the row's slots all placed, its predecessor's slot in the row
// (the route's first edge: none), so a path is walked slot to slot.
template <bool WRITE>
__global__ __launch_bounds__(TB) void k_index_build(DevGraph g, const uint32_t* TU, uint32_t cmax, int32_t* row_cnt,
                                                    const IdxRow* rows, uint4* slot) {
  __shared__ uint32_t lkey[INDEX_BUILD_CAP];
  __shared__ unsigned long long llab[INDEX_BUILD_CAP];
  __shared__ uint32_t linq[INDEX_BUILD_CAP];
  __shared__ uint32_t lfr0[INDEX_BUILD_CAP];
  __shared__ uint32_t lfr1[INDEX_BUILD_CAP];
  __shared__ int32_t cbuf[CHAIN_BUF * TB];
  __shared__ SearchShared S;
  const int lane = threadIdx.x;
  const Table T{lkey, llab, linq, lfr0, lfr1, INDEX_BUILD_LOG2, INDEX_BUILD_LIMIT};
  const int64_t nrows = (int64_t)g.n_edges + g.n_nodes;
  for (int64_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const bool erow = r < g.n_edges;
    const int32_t u = erow ? g.e_to[r] : (int32_t)(r - g.n_edges);
    const uint32_t hin = erow ? (uint32_t)g.e_head_in[r] : NO_HEAD;
    const int n = ta_search<false>(g, TU, T, S, u, hin, cmax, lane);
    if (!WRITE) {
      if (lane == 0) row_cnt[r] = n;  // -1: incomplete row
      continue;
    }
    if (n < 0) continue;
    // insert the labels into the row's table (slot order depends on CAS
    // order; lookups do not)
    const IdxRow R = rows[r];
    auto predof = [&](uint32_t e) {
      const int sx = table_find<false>(T, e);
      return sx < 0 ? NONE_PRED : (uint32_t)(llab[sx] & 0xFFFFFFFFull);
    };
    for (int i = lane; i < INDEX_BUILD_CAP; i += TB) {
      const uint32_t k = lkey[i];
      if (k == EMPTY) continue;
      const unsigned long long lab = llab[i];
      const uint32_t pk = (uint32_t)(lab & 0xFFFFFFFFull);
      float d;
      uint32_t units;
      int len;
      chain_sums(g, TU, predof, pk, hin, (k & NODE_KEY) ? NO_HEAD : (uint32_t)g.e_head_out[k], cbuf + lane, d, units,
                 len);
      uint32_t h = idx_slot0(idx_hash(k), R);
      while (atomicCAS(&slot[R.off + h].x, EMPTY, k) != EMPTY) h = idx_next(h, R);
      // (cost <= cmax < 2^24 and units <= cost: the top bytes are the
      // predecessor's, written below)
      slot[R.off + h].y = (uint32_t)(lab >> 32) & IDX_LOW24;
      slot[R.off + h].z = fbits(d);
      slot[R.off + h].w = units & IDX_LOW24;
    }
    __syncthreads();
    for (int i = lane; i < INDEX_BUILD_CAP; i += TB) {
      const uint32_t k = lkey[i];
      if (k == EMPTY) continue;
      const uint32_t pk = (uint32_t)(llab[i] & 0xFFFFFFFFull);
      uint4 sk_v, tmp;
      const int64_t sk = idx_find(slot, R, k, sk_v);
      const int64_t sp = pk == NONE_PRED ? -1 : idx_find(slot, R, pk, tmp);
      const uint32_t ps = sp < 0 ? IDX_NO_PRED : (uint32_t)(sp - R.off);
      slot[sk].y = (sk_v.y & IDX_LOW24) | (ps & 0xFFu) << 24;
      slot[sk].w = (sk_v.w & IDX_LOW24) | (ps >> 8) << 24;
    }
    __syncthreads();
  }
}

// table capacity of a row (idx_row_cap at load pct)
__global__ void k_row_sizes(const int32_t* row_cnt, int64_t* sizes, int32_t n, int pct) {
  const int32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) sizes[u] = idx_row_cap(row_cnt[u], pct);
  if (u == n) sizes[n] = 0;
}

__global__ void k_row_pack(const int32_t* row_cnt, const int64_t* row_off, IdxRow* rows, int32_t n) {
  const int32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  const int64_t cap = row_off[u + 1] - row_off[u];
  rows[u] = IdxRow{row_off[u], row_cnt[u], (uint32_t)cap};
}

// K4 index tier: S lanes per column, TB / S columns in flight per wave,
// lanes over the column's Kq x Kp (source candidate, target candidate) pairs;
// each pair is one probe of its source's index row (row ei, or E + from(ei)
// for a node candidate) for its target's label (key ej, or NODE_KEY |
// from(ej) for a node candidate), whose 16-byte slot holds the label's cost,
// route distance and turn units.  A column is a chain of ~5 dependent round
// trips (point -> previous column -> candidates -> rows -> slots), so several
// columns per wave multiply the misses in flight at the same occupancy.
// Columns with more pairs than S loop within their group; columns the index
// cannot answer (cost bound > the index's, a source row incomplete, more than
// KC candidates) go to the search tiers (w.overflow_list0, count
// w.counters_i32[4]).
// At 8 lanes per column (8 columns per wave) a column with more than
// OTM_TRANS_KC8 candidates on either side goes to the wide list
// (w.overflow_list2, count w.counters_i32[6]), which a 16-lane pass (LIST)
// then answers from the index; KC8 keeps the LDS words within 8 waves per SIMD.
#ifndef OTM_TRANS_KC8
#define OTM_TRANS_KC8 8
#endif
// waves per SIMD the register budget is sized for
#ifndef OTM_TRANS_WAVES
#define OTM_TRANS_WAVES 8
#endif
template <int S, bool LIST>
__global__ __launch_bounds__(TB, OTM_TRANS_WAVES) void k_trans_sub(DevGraph g, DevBatch b, DevParams P, DevWork w) {
  if (*w.abort || trans_over_cap(b, w)) return;  // a capacity was exceeded: the host redoes the batch
  static_assert(S == 8 || S == 16, "8 lanes per column (two passes) or 16 (one pass / the wide pass)");
  constexpr int NS = TB / S;
  // a pair reads its target and source as one 16-byte LDS word each
  constexpr int KC = S >= 16 ? 16 : OTM_TRANS_KC8;
  constexpr bool WIDE = KC < 16;
  __shared__ int4 tg[NS][KC];  // target: edge, offset bits, label key, -
  __shared__ int4 sr[NS][KC];  // source: edge, offset bits, remaining-length bits, end heading
  __shared__ IdxRow rq[NS][KC];
  // slot of candidate k in its column group's row: XOR-swizzled so that the
  // groups a ds_read_b128 lane group spans (MI355X_MICROARCH.md §LDS: lanes
  // {0-3,12-15,20-27}, ...) read different banks when they read the same k
  // (a 128-B row at 8 lanes per column puts groups sg and sg + 2 on the same
  // 64 banks; at 16 lanes, every row spans all 64)
#ifndef OTM_TRANS_SWZ
#define OTM_TRANS_SWZ 1
#endif
  const int lane = threadIdx.x, sg = lane / S, sl = lane % S;
  const unsigned long long smask = ((1ull << S) - 1ull) << (sg * S);
  const int swz = !OTM_TRANS_SWZ ? 0 : (S == 8 ? ((sg >> 1) & 1) * 4 : (sg & 1) * 8);
  const DevIndex& X = w.idx;
  unsigned long long c_search = 0, c_settled = 0, c_relaxed = 0, c_trans = 0;
  const bool ordered = !LIST && (P.order_mask & ORDER_TRANS) != 0;
  int64_t base, end, stride;
  if (LIST) {
    base = (int64_t)blockIdx.x * NS;
    end = w.counters_i32[6];
    stride = (int64_t)gridDim.x * NS;
  } else if (ordered) {
    const int grp = blockIdx.x % ORDER_GROUPS;
    base = w.ord.grp[grp] + (int64_t)(blockIdx.x / ORDER_GROUPS) * NS;
    end = w.ord.grp[grp + 1];
    stride = (int64_t)(gridDim.x / ORDER_GROUPS) * NS;
  } else {
    base = (int64_t)blockIdx.x * NS;
    end = b.n_points;
    stride = (int64_t)gridDim.x * NS;
  }
  for (; base < end; base += stride) {
    const int64_t it = base + sg;
    bool act = it < end;
    int64_t p = 0;
    // the column's words in one round trip (K3 wrote the previous column's
    // candidate count beside the link): its ordered record, or the arrays
    int32_t q = -1;
    int Kp = 0, Kq = 0;
    float gcv = 0.0f;
    int64_t toff = 0;
    if (act && ordered && w.colrec) {
      const int4 A = w.colrec[it];
      p = A.x;
      toff = w.trans_off[p];  // (the scan's, after K3)
      q = A.y;
      Kq = A.z & 255;
      Kp = A.z >> 8;
      gcv = __int_as_float(A.w);
    } else if (act) {
      p = LIST ? (int64_t)w.overflow_list2[it] : (ordered ? (int64_t)w.ord.item[it] : it);
      q = w.col_prev[p];
      Kq = w.kq_prev[p];
      Kp = w.ncand[p];
      gcv = w.gc[p];
      toff = w.trans_off[p];
    }
    act = act && q >= 0;
    const float bound = P.factor * gcv;
    const uint32_t cq = index_cost_bound(bound);
    const bool idx_ok = X.rmax > 0.0f && cq <= X.cmax;
    // the near index when it covers the bound (same answers, smaller tables)
    const IdxRow* xrow = X.row;
    const uint4* xslot = X.slot;
#pragma unroll
    for (int l = NEAR_LEVELS - 1; l >= 0; --l) {
      if (w.idxn[l].rmax > 0.0f && cq <= w.idxn[l].cmax) {
        xrow = w.idxn[l].row;
        xslot = w.idxn[l].slot;
      }
    }
    const bool wide = WIDE && act && idx_ok && (Kp > KC || Kq > KC);
    if (wide && sl == 0) w.overflow_list2[atomicAdd(&w.counters_i32[6], 1)] = (int32_t)p;
    act = act && !wide;
    bool bad = act && (!idx_ok || Kp > KC || Kq > KC);
    // candidates of p (targets) and of q (sources), then rows
    for (int k = sl; k < KC; k += S) {
      if (act && k < Kp) {
        const int2 c = crec(w, p, k);
        const int32_t e = c.x;
        const float o = __int_as_float(c.y);
        const uint32_t key = dst_key(g, e, o);
        tg[sg][k ^ swz] = make_int4(e, __float_as_int(o), (int)key, (int)idx_hash(key));
      }
      if (act && k < Kq) {
        const int2 c = crec(w, q, k);
        const int32_t e = c.x;
        const float o = __int_as_float(c.y);
        // src_start and src_row from the edge's {from, length} pair (one
        // load); the heading only for the work counters (no load otherwise)
        const int2 fl = g.e_fl[e];
        const float start = cand_node(o) ? 0.0f : __int_as_float(fl.y) - o;
        sr[sg][k ^ swz] = make_int4(e, __float_as_int(o), __float_as_int(start), w.ctr ? (int)src_head(g, e, o) : 0);
        if (idx_ok) {
          const IdxRow R = xrow[cand_node(o) ? (int64_t)g.n_edges + fl.x : (int64_t)e];
          rq[sg][k ^ swz] = R;
          bad = bad || R.cnt < 0;
        }
      }
    }
    const bool spill = (__ballot(bad) & smask) != 0ull;
    if (spill && act && sl == 0) {
      const int slot = atomicAdd(&w.counters_i32[4], 1);
      w.overflow_list0[slot] = (int32_t)p;
    }
    act = act && !spill;
    wave_sync();
    if (act) {
      float* Tm = w.trans + toff;
      unsigned long long ntr = 0;
      // OTM_TRANS_BATCH pairs per lane per step: every pair's first bucket
      // (two slots, one aligned 32-B piece of a line) is loaded before any is
      // resolved, so their probes are in flight together
      constexpr int NB = OTM_TRANS_BATCH;
      const int npair = Kq * Kp;
      for (int idx0 = sl; idx0 < npair; idx0 += S * NB) {
        uint4 s0[NB], s1[NB];
        uint32_t h0[NB];
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int idx = idx0 + u * S;
          s0[u] = make_uint4(EMPTY, 0u, 0u, 0u);
          s1[u] = s0[u];
          h0[u] = 0u;
          if (idx < npair) {
            const int i = idx / Kp, j = idx - (idx / Kp) * Kp;
            const int4 T = tg[sg][j ^ swz], Sx = sr[sg][i ^ swz];
            const IdxRow R = rq[sg][i ^ swz];
            const bool same = same_edge_step(Sx.x, __int_as_float(Sx.y), T.x, __int_as_float(T.y));
            if (!same && R.cnt > 0) {
              h0[u] = idx_slot0((uint32_t)T.w, R);
              s0[u] = xslot[R.off + h0[u]];
              s1[u] = xslot[R.off + h0[u] + 1];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < NB; ++u) {
          const int idx = idx0 + u * S;
          if (idx >= npair) continue;
          const int i = idx / Kp, j = idx - (idx / Kp) * Kp;
          const int4 T = tg[sg][j ^ swz], Sx = sr[sg][i ^ swz];
          const uint32_t key = (uint32_t)T.z;
          const int32_t ej = T.x, ei = Sx.x;
          const float oj = __int_as_float(T.y), oi = __int_as_float(Sx.y), si = __int_as_float(Sx.z);
          float r = 0.0f;
          bool ok = true;
          uint32_t units = 0;
          if (same_edge_step(ei, oi, ej, oj)) {
            r = same_edge_dist(oi, oj);
          } else {
            const IdxRow R = rq[sg][i ^ swz];
            uint4 sv = s0[u];
            if (R.cnt > 0 && sv.x != key && sv.x != EMPTY) {
              sv = s1[u];
              uint32_t h = h0[u] + 1u;
              while (sv.x != key && sv.x != EMPTY) {  // the rest of the linear probe (rare)
                h = idx_next(h, R);
                sv = xslot[R.off + h];
              }
            }
            // a label of the row beyond this column's cost bound is not one
            // of its search's labels
            if (R.cnt > 0 && sv.x == key && idx_slot_cost(sv) <= cq) {
              const float sd = si + bitsf(sv.z);
              r = sd + oj;
              units = idx_slot_units(sv);
            } else {
              ok = false;
            }
          }
          float cost = INFINITY;
          if (ok && r <= bound) {
            cost = trans_cost(units, r, gcv, P.beta);
            ++ntr;
          }
          Tm[i * Kp + j] = cost;
        }
      }
      if (w.ctr) {
        // algorithmic counts of the equivalent searches (per-lane partials,
        // summed over the wave at the end): per distinct source (node,
        // heading), the row's departure labels within the bound and the
        // out-degrees of those whose edge end is within it too
        for (int i = 0; i < Kq; ++i) {
          const int4 Si = sr[sg][i ^ swz];
          const int32_t ui = src_node(g, Si.x, __int_as_float(Si.y));
          bool first = true;
          for (int k = 0; k < i; ++k) {
            const int4 Sk = sr[sg][k ^ swz];
            first = first && !(src_node(g, Sk.x, __int_as_float(Sk.y)) == ui && Sk.w == Si.w);
          }
          if (!first) continue;
          const IdxRow R = rq[sg][i ^ swz];
          for (int64_t k = sl; k < (int64_t)R.cap; k += S) {
            const uint4 slt = xslot[R.off + k];
            if (slt.x == EMPTY || (slt.x & NODE_KEY) || idx_slot_cost(slt) > cq) continue;
            ++c_settled;
            if ((unsigned long long)idx_slot_cost(slt) + g.e_len64[slt.x] <= cq) {
              const int32_t v = g.e_to[slt.x];
              c_relaxed += (unsigned long long)(g.out_off[v + 1] - g.out_off[v]);
            }
          }
          if (sl == 0) ++c_search;
        }
        c_trans += ntr;
      }
    }
    wave_sync();
  }
  if (w.ctr) {
    for (int sh = 32; sh > 0; sh >>= 1) {
      c_search += __shfl_xor(c_search, sh, 64);
      c_settled += __shfl_xor(c_settled, sh, 64);
      c_relaxed += __shfl_xor(c_relaxed, sh, 64);
      c_trans += __shfl_xor(c_trans, sh, 64);
    }
    if (lane == 0) {
      cadd(&w.ctr->searches, c_search);
      cadd(&w.ctr->nodes_settled, c_settled);
      cadd(&w.ctr->edges_relaxed, c_relaxed);
      cadd(&w.ctr->transitions, c_trans);
    }
  }
}

// K6 index tier: one lane per matched step; the route is the predecessor
// chain of its target's label in its source's row, one probe per edge.
// route / report waves-per-SIMD hints: 4 or 8 measured within noise (kept at 1)
#ifndef OTM_ROUTE_WAVES
#define OTM_ROUTE_WAVES 1
#endif
__global__ __launch_bounds__(256, OTM_ROUTE_WAVES) void k_route_index(DevGraph g, DevBatch b, DevParams P, DevWork w) {
  if (*w.abort) return;  // a capacity was exceeded: the host redoes the batch
  const DevIndex& X = w.idx;
  unsigned long long c_search = 0, c_settled = 0, c_relaxed = 0, c_edges = 0;
  const ItemRange R = item_range(w, b, (P.order_mask & ORDER_ROUTE) != 0, 256);
  // K4's column records (K3, spatial-order position) give p, its link and gc
  // in one coalesced load, so the link's chosen candidate loads with p's
  const bool rec = R.ordered && w.colrec && (P.order_mask & ORDER_TRANS);
  for (int64_t it = R.i0; it < R.i1; it += R.stride) {
    int64_t p;
    int32_t q = -1;
    float gcv = 0.0f;
    if (rec) {
      const int4 A = w.colrec[it];
      p = A.x;
      q = A.y;
      gcv = __int_as_float(A.w);
    } else {
      p = R.ordered ? (int64_t)w.ord.item[it] : it;
    }
    if (!R.ordered && !w.is_col[p]) continue;
    // (non-column points keep the zeros K1 wrote; a re-run after a path-pool
    // overflow rewrites every column)
    w.route_dist[p] = 0.0f;
    w.path_len[p] = 0;
    w.path_off[p] = 0;
    const int2 cq0 = w.chosen[q >= 0 ? q : p];  // (used only for a matched link)
    if (w.state[p] < 0 || w.chain_start[p]) continue;
    if (!rec) {
      q = w.col_prev[p];
      gcv = w.gc[p];
    }
    const int2 ci = rec ? cq0 : w.chosen[q], cj = w.chosen[p];
    const int32_t ei = ci.x, ej = cj.x;
    const float oi = __int_as_float(ci.y), oj = __int_as_float(cj.y);
    if (same_edge_step(ei, oi, ej, oj)) {
      w.route_dist[p] = same_edge_dist(oi, oj);
      continue;
    }
    const float bound = P.factor * gcv;
    const uint32_t cq = index_cost_bound(bound);
    IdxRow Rw{};
    int64_t sv = -1;
    uint4 lab{};
    // the near index when it covers the bound (the same labels and paths)
    int lvl = -1;
#pragma unroll
    for (int l = NEAR_LEVELS - 1; l >= 0; --l)
      if (w.idxn[l].rmax > 0.0f && cq <= w.idxn[l].cmax) lvl = l;
    const DevIndex& Xc = lvl >= 0 ? w.idxn[lvl] : X;
    // the source's row and start from its edge's {from, length} pair (one load)
    const int2 fli = g.e_fl[ei];
    if (X.rmax > 0.0f && cq <= X.cmax) {
      Rw = Xc.row[cand_node(oi) ? (int64_t)g.n_edges + fli.x : (int64_t)ei];
      sv = idx_find(Xc.slot, Rw, dst_key(g, ej, oj), lab);
    }
    if (sv < 0 || idx_slot_cost(lab) > cq) {
      const int slot = atomicAdd(&w.counters_i32[4], 1);
      w.overflow_list0[slot] = (int32_t)p;
      continue;
    }
    // the path: the label's predecessor slots in the row, back to the first
    // edge (a slot holds its label's edge and its predecessor's slot)
    int len = 0;
    for (int32_t ps = idx_slot_pred(lab); ps >= 0 && len <= Rw.cnt; ps = idx_slot_pred(Xc.slot[Rw.off + ps])) ++len;
    const int off = len ? atomicAdd(&w.counters_i32[1], len) : 0;
    if (off + len > w.pool_cap) {
      w.counters_i32[2] = 1;
      *w.abort = 1;
      w.path_len[p] = -1;
    } else {
      int k = len;
      for (int32_t ps = idx_slot_pred(lab); ps >= 0 && k > 0;) {
        const uint4 sl = Xc.slot[Rw.off + ps];
        w.path_pool[off + (--k)] = (int32_t)sl.x;
        ps = idx_slot_pred(sl);
      }
      w.path_off[p] = off;
      w.path_len[p] = len;
    }
    const float start = cand_node(oi) ? 0.0f : __int_as_float(fli.y) - oi;  // src_start
    const float sd = start + bitsf(lab.z);
    w.route_dist[p] = sd + oj;
    if (w.ctr) {
      unsigned long long st = 0, rl = 0;
      for (int64_t k = 0; k < (int64_t)Rw.cap; ++k) {
        const uint4 sl = Xc.slot[Rw.off + k];
        if (sl.x == EMPTY || (sl.x & NODE_KEY) || idx_slot_cost(sl) > cq) continue;
        ++st;
        if ((unsigned long long)idx_slot_cost(sl) + g.e_len64[sl.x] <= cq) {
          const int32_t v = g.e_to[sl.x];
          rl += (unsigned long long)(g.out_off[v + 1] - g.out_off[v]);
        }
      }
      ++c_search;
      c_settled += st;
      c_relaxed += rl;
      c_edges += (unsigned long long)len;
    }
  }
  if (w.ctr) {
    cadd(&w.ctr->route_searches, c_search);
    cadd(&w.ctr->route_nodes_settled, c_settled);
    cadd(&w.ctr->route_edges_relaxed, c_relaxed);
    cadd(&w.ctr->route_edges, c_edges);
  }
}

// ============================================================== K4 transitions (wave tiers)
// Columns the index tier could not answer (list in w.overflow_list0, count in
// w.counters_i32[4], read on the device: no host round trip): one turn-aware
// search per distinct source (node, heading), the wave's table in LDS.  The
// LDS tier spills to `w.overflow_list2` / counters_i32[3], which the
// global-memory tier (BIG) drains.
// the search table of a tier's block: LDS (0), global (1), huge (2)
template <int TIER>
__device__ __forceinline__ Table tier_table(const DevWork& w, uint32_t* lkey, unsigned long long* llab, uint32_t* linq,
                                            uint32_t* lfr0, uint32_t* lfr1) {
  if (TIER == 1) {
    const size_t base = (size_t)blockIdx.x * BIG_TABLE_CAP;
    return Table{w.big_key + base, w.big_lab + base, w.big_inq + base, w.big_fr + 2 * base,
                 w.big_fr + 2 * base + BIG_TABLE_CAP, BIG_TABLE_LOG2, SEARCH_LIMIT,
                 w.big_ins + (size_t)blockIdx.x * SEARCH_LIMIT, w.big_prev + blockIdx.x};
  }
  if (TIER == 2) {
    const size_t cap = (size_t)1 << w.huge_log2;
    const size_t base = (size_t)blockIdx.x * cap;
    const int lim = huge_limit(w.huge_log2);
    return Table{w.huge_key + base, w.huge_lab + base, w.huge_inq + base, w.huge_fr + 2 * base,
                 w.huge_fr + 2 * base + cap, w.huge_log2, lim, w.huge_ins + (size_t)blockIdx.x * lim,
                 w.huge_prev + blockIdx.x};
  }
  return Table{lkey, llab, linq, lfr0, lfr1, 8, LDS_TABLE_LIMIT};
}
// the huge tier has work but no tables yet: the host allocates them and
// redoes the batch -- or, when it cannot (huge_final), the listed columns'
// traces answer 500 (OTM_TERR_SEARCH_OVERFLOW) (returns true: the launch is done)
__device__ __forceinline__ bool huge_unready(DevWork& w, int64_t nwork, const int32_t* list) {
  if (nwork <= 0 || w.huge_log2 > 0) return false;
  if (w.huge_final) {
    for (int64_t it = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; it < nwork; it += (int64_t)gridDim.x * blockDim.x)
      atomicCAS(&w.trace_err[w.pt_trace[list[it]]], 0, OTM_TERR_SEARCH_OVERFLOW);
  } else if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.counters_i32[23] = 1;
    *w.abort = 1;
  }
  return true;
}
// a huge-tier search that outgrew its table: the host grows the tables and
// redoes the batch, or (huge_final) the column's trace answers 500
__device__ __forceinline__ void huge_overflow(DevWork& w, int64_t p) {
  if (w.huge_final) {
    atomicCAS(&w.trace_err[w.pt_trace[p]], 0, OTM_TERR_SEARCH_OVERFLOW);
  } else {
    w.counters_i32[23] = 1;  // the huge tables are too small: grow, redo
    *w.abort = 1;
  }
}

// TIER 0: LDS tables; 1: global tables (BIG_SLOTS x BIG_TABLE_CAP); 2: the
// huge tier (HUGE_SLOTS x 2^huge_log2).  Spills: 0 -> list2 ([3]) -> 1 ->
// list3 ([21]) -> 2 -> the host grows the huge tables and redoes the batch.
template <int TIER>
__global__ __launch_bounds__(TB) void k_transitions(DevGraph g, DevBatch b, DevParams P, DevWork w) {
  constexpr bool BIG = TIER > 0;
  if (*w.abort || trans_over_cap(b, w)) return;
  __shared__ uint32_t lkey[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ unsigned long long llab[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ uint32_t linq[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ uint32_t lfr0[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ uint32_t lfr1[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ int32_t cbuf[CHAIN_BUF * TB];
  __shared__ uint32_t TU[TURN_TABLE];
  __shared__ int32_t eq[KMAX], ep[KMAX];
  __shared__ float oq[KMAX], op[KMAX];
  __shared__ SearchShared S;
  const int lane = threadIdx.x;
  for (int k = lane; k < TURN_TABLE; k += TB) TU[k] = P.turn_units[k];
  Table T = tier_table<TIER>(w, lkey, llab, linq, lfr0, lfr1);
  auto predof = [&](uint32_t e) {
    const int sx = table_find<BIG>(T, e);
    return sx < 0 ? NONE_PRED : (uint32_t)(Mem<BIG>::ld(&T.lab[sx]) & 0xFFFFFFFFull);
  };
  const int32_t* list = TIER == 2 ? w.overflow_list3 : (BIG ? w.overflow_list2 : w.overflow_list0);
  const int64_t nwork = TIER == 2 ? (int64_t)w.counters_i32[21]
                                  : (BIG ? (int64_t)w.counters_i32[3] : (int64_t)w.counters_i32[4]);
  if (TIER == 2 && huge_unready(w, nwork, list)) return;
  __syncthreads();
  for (int64_t it = blockIdx.x; it < nwork; it += gridDim.x) {
    const int64_t p = (int64_t)list[it];
    const int32_t q = w.col_prev[p];
    if (q < 0) continue;
    const int Kq = w.ncand[q], Kp = w.ncand[p];
    const float gcv = w.gc[p];
    const float bound = P.factor * gcv;
    const uint32_t cq = index_cost_bound(bound);
    if (lane < Kq) {
      const int2 c = crec(w, q, lane);
      eq[lane] = c.x;
      oq[lane] = __int_as_float(c.y);
    }
    if (lane < Kp) {
      const int2 c = crec(w, p, lane);
      ep[lane] = c.x;
      op[lane] = __int_as_float(c.y);
    }
    __syncthreads();
    // distinct sources (node, heading), first occurrence order
    const int32_t u_l = lane < Kq ? src_node(g, eq[lane], oq[lane]) : -1;
    const uint32_t h_l = lane < Kq ? src_head(g, eq[lane], oq[lane]) : 0u;
    bool first = lane < Kq;
    for (int k = 0; k < Kq; ++k) {
      const int32_t uk = __shfl(u_l, k, 64);
      const uint32_t hk = __shfl(h_l, k, 64);
      if (k < lane && uk == u_l && hk == h_l) first = false;
    }
    unsigned long long srcmask = __ballot(first);
    float* Tm = w.trans + w.trans_off[p];
    bool failed = false;
    // work counts of this column, committed only if no search spilled (the
    // global tier redoes every source of a spilled column)
    unsigned long long c_search = 0, c_settled = 0, c_relaxed = 0, c_trans = 0;
    while (srcmask) {
      const int sl = __ffsll((long long)srcmask) - 1;
      srcmask &= srcmask - 1;
      const int32_t u = __shfl(u_l, sl, 64);
      const uint32_t hin = __shfl(h_l, sl, 64);
      const int labels = ta_search<BIG>(g, TU, T, S, u, hin, cq, lane);
      if (labels < 0) {
        failed = true;
        break;
      }
      unsigned long long ntr = 0;
      for (int idx = lane; idx < Kq * Kp; idx += TB) {
        const int i = idx / Kp, j = idx - (idx / Kp) * Kp;
        if (src_node(g, eq[i], oq[i]) != u || src_head(g, eq[i], oq[i]) != hin) continue;
        const int32_t ei = eq[i], ej = ep[j];
        const float start = src_start(g, ei, oq[i]);
        float r = 0.0f;
        uint32_t units = 0;
        bool ok = true;
        if (same_edge_step(ei, oq[i], ej, op[j])) {
          r = same_edge_dist(oq[i], op[j]);
        } else {
          const uint32_t key = dst_key(g, ej, op[j]);
          const int slot = table_find<BIG>(T, key);
          if (slot < 0) {
            ok = false;
          } else {
            float d;
            int n;
            chain_sums(g, TU, predof, (uint32_t)(Mem<BIG>::ld(&T.lab[slot]) & 0xFFFFFFFFull), hin,
                       (key & NODE_KEY) ? NO_HEAD : (uint32_t)g.e_head_out[ej], cbuf + lane, d, units, n);
            const float sd = start + d;
            r = sd + op[j];
          }
        }
        float cost = INFINITY;
        if (ok && r <= bound) {
          cost = trans_cost(units, r, gcv, P.beta);
          ++ntr;
        }
        Tm[i * Kp + j] = cost;
      }
      if (w.ctr) {
        unsigned long long st, rl;
        ta_counts<BIG>(g, T, cq, lane, st, rl);
        for (int o = 32; o > 0; o >>= 1) ntr += __shfl_xor(ntr, o, 64);
        c_search += 1;
        c_settled += st;
        c_relaxed += rl;
        c_trans += ntr;
      }
      __syncthreads();
    }
    if (w.ctr && !failed && lane == 0) {
      cadd(&w.ctr->searches, c_search);
      cadd(&w.ctr->nodes_settled, c_settled);
      cadd(&w.ctr->edges_relaxed, c_relaxed);
      cadd(&w.ctr->transitions, c_trans);
    }
    if (failed && lane == 0) {
      if (TIER == 0) {
        w.overflow_list2[atomicAdd(&w.counters_i32[3], 1)] = (int32_t)p;
      } else if (TIER == 1) {
        w.overflow_list3[atomicAdd(&w.counters_i32[21], 1)] = (int32_t)p;
      } else {
        huge_overflow(w, p);
      }
    }
    __syncthreads();
  }
}

// ============================================================== K5 viterbi
__device__ __forceinline__ void wave_argmin(float v, int idx, float& bv, int& bi) {
  // lexicographic (value, index) minimum over the wave; +inf never wins
  bv = v;
  bi = idx;
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ov < bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
}

// Global-memory form for one trace (traces too large for the LDS form).
__device__ void viterbi_trace_global(int64_t a, int64_t e, DevWork& w) {
  const int lane = threadIdx.x;
  {
    float prev = INFINITY;
    bool open = false;
    int64_t last = -1;
    auto backtrack = [&](int64_t endp) {
      const int Ke = w.ncand[endp];
      float bv;
      int bi;
      wave_argmin(lane < Ke ? prev : INFINITY, lane, bv, bi);
      __syncthreads();
      if (lane == 0) {
        int64_t pp = endp;
        int jj = bi;
        while (true) {
          w.state[pp] = jj;
          w.chosen[pp] = crec(w, pp, jj);
          if (w.chain_start[pp]) break;
          jj = w.bp[pp * KMAX + jj];
          pp = w.col_prev[pp];
        }
      }
    };
    for (int64_t p = a; p < e; ++p) {
      if (!w.is_col[p]) continue;
      const int Kp = w.ncand[p];
      if (Kp == 0) {
        if (open) backtrack(last);
        open = false;
        continue;
      }
      bool started = false;
      float cur = INFINITY;
      if (open && w.col_prev[p] == (int32_t)last) {
        const int Kq = w.ncand[last];
        const float* Tm = w.trans + w.trans_off[p];
        float best = INFINITY;
        int bi = -1;
        for (int i = 0; i < Kq; ++i) {
          const float pi = __shfl(prev, i, 64);
          if (lane < Kp) {
            const float v = pi + Tm[i * Kp + lane];
            if (v < best) {
              best = v;
              bi = i;
            }
          }
        }
        const bool alive = lane < Kp && bi >= 0;
        if (lane < Kp) {
          cur = alive ? best + cemis(w, p, lane) : INFINITY;
          w.bp[p * KMAX + lane] = alive ? (uint8_t)bi : (uint8_t)0xFF;
        }
        if (__ballot(alive) == 0ull) {
          backtrack(last);
        } else {
          started = true;
        }
      } else if (open) {
        backtrack(last);
      }
      if (!started) {
        cur = lane < Kp ? cemis(w, p, lane) : INFINITY;
        if (lane == 0) w.chain_start[p] = 1;
      }
      prev = cur;
      open = true;
      last = p;
    }
    __syncthreads();
    if (open) backtrack(last);
    __syncthreads();
  }
}
// LDS form: one wavefront per trace.  The trace's column metadata (and its
// backpointers, which never touch HBM) live in LDS for the whole trace; the
// transition block and emissions are streamed through LDS in windows of
// consecutive columns, each staged with coalesced loads.  The forward pass
// runs out of LDS with the previous column's scores broadcast by readlane;
// the backtrack walks LDS; state / chain_start go out coalesced.  Same
// recurrence, tie rules and chain breaks as viterbi_trace_global.
// LDS per trace (~5 KB at these sizes) and 64 VGPRs give 8 waves per SIMD
// (128 points of metadata: 0.218 -> 0.207 ms on config 2 against 256; 8
// waves instead of 7 with a 448-float window and 768 backpointers: 2.20 ->
// 1.96 ms on a config-3 shard, 0.201 -> 0.198 on config 2); a
// trace longer than VIT_PTS, whose candidates exceed VIT_BP, or with one
// column pair's block beyond VIT_TW, takes the global-memory form.
#ifndef OTM_VIT_TW
#define OTM_VIT_TW 448
#endif
#ifndef OTM_VIT_BP
#define OTM_VIT_BP 768
#endif
#ifndef OTM_VIT_PTS
#define OTM_VIT_PTS 128
#endif
constexpr int VIT_PTS = OTM_VIT_PTS; // points per trace (metadata held for the whole trace)
constexpr int VIT_BP = OTM_VIT_BP;   // candidates per trace (backpointers)
constexpr int VIT_TW = OTM_VIT_TW;   // transition floats per window (>= one column pair's block)
// emission floats per window (>= KMAX)
#ifndef OTM_VIT_EW
#define OTM_VIT_EW 256
#endif
constexpr int VIT_EW = OTM_VIT_EW;
static_assert(VIT_EW >= KMAX, "one column's emissions fit a window");

#ifndef OTM_VIT_WAVES
#define OTM_VIT_WAVES 8
#endif
// Measured and not kept (profiles/r02_ab_viterbi.txt): a one-read backtrack
// through trace-wide backpointer indices (0.159 vs 0.157 ms, and 16-bit
// backpointers cost occupancy), one global round trip per window (equal).
// list / list_n: the traces to decode (null: all); snap: this launch takes
// spill snapshot B (the first Viterbi launch of the batch)
__global__ __launch_bounds__(TB, OTM_VIT_WAVES) void k_viterbi(DevBatch b, DevWork w, const int32_t* list,
                                                               const int32_t* list_n, int snap) {
  // spill snapshot B: columns per transition tier (Viterbi does not touch the
  // counters; they start over for the route tiers)
  if (OTM_FOLD_BOOKKEEPING && snap && blockIdx.x == 0 && threadIdx.x == 0) fold_snap(w, 1, true);
  if (*w.abort) return;  // a capacity was exceeded: the host redoes the batch
  __shared__ float sT[VIT_TW];
  __shared__ float sEm[VIT_EW];
  __shared__ uint8_t sBp[VIT_BP];
  __shared__ int8_t sState[VIT_PTS];
  __shared__ uint8_t sCs[VIT_PTS];
  __shared__ int32_t sToff[VIT_PTS + 1];
  __shared__ int16_t sEoff[VIT_PTS + 1];
  __shared__ int16_t sCprev[VIT_PTS];
  __shared__ int8_t sKc[VIT_PTS];  // ncand of a column, -1 for a non-column point
  const int lane = threadIdx.x;
  const int32_t nwork = list ? *list_n : b.n_traces;
  for (int32_t it = blockIdx.x; it < nwork; it += gridDim.x) {
    const int32_t t = list ? list[it] : it;
    const int64_t a = b.trace_off[t], e = b.trace_off[t + 1];
    const int n = (int)(e - a);
    if (w.trace_err[t] != 0) {
      for (int64_t p = a + lane; p < e; p += TB) {
        w.state[p] = -1;
        w.chain_start[p] = 0;
      }
      continue;
    }
    const int64_t t0 = w.trans_off[a];
    int etot = 0;
    bool fits = n <= VIT_PTS;
    if (fits) {
      // column metadata + emission offsets (wave scan of ncand)
      bool big = false;  // a column pair's block beyond the window
      for (int c = 0; c < n; c += TB) {
        const int pl = c + lane;
        int kc = -1, cp = -1, to = 0;
        if (pl < n) {
          // independent loads (ncand / col_prev are defined for every point)
          const int64_t p = a + pl;
          const uint8_t ic = w.is_col[p];
          const int32_t nc = w.ncand[p];
          const int32_t q = w.col_prev[p];
          const int64_t tp = w.trans_off[p];
          const int64_t tn = w.trans_off[p + 1];
          if (ic) {
            kc = nc;
            cp = q >= 0 ? (int)(q - a) : -1;
          }
          to = (int)(tp - t0);
          big = big || tn - tp > VIT_TW;
        }
        const int k = kc > 0 ? kc : 0;
        const int incl = wave_incl_scan(k, lane);
        if (pl < n) {
          sKc[pl] = (int8_t)kc;
          sCprev[pl] = (int16_t)cp;
          sToff[pl] = to;
          sEoff[pl] = (int16_t)min(etot + incl - k, 32767);
          sState[pl] = -1;
          sCs[pl] = 0;
        }
        etot += __shfl(incl, 63, 64);
      }
      fits = etot <= VIT_BP && __ballot(big) == 0ull;
    }
    if (!fits) {
      __syncthreads();
      for (int64_t p = a + lane; p < e; p += TB) {
        w.state[p] = -1;
        w.chain_start[p] = 0;
      }
      __syncthreads();
      viterbi_trace_global(a, e, w);
      continue;
    }
    if (lane == 0) {
      sToff[n] = n > 0 ? (int)(w.trans_off[e] - t0) : 0;
      sEoff[n] = (int16_t)etot;
    }
    __syncthreads();
    float prev = INFINITY;
    bool open = false;
    int last = -1;
    int win_end = 0, wt0 = 0, we0 = 0;
    auto backtrack = [&](int endl, int Ke) {
      float bv;
      int bi;
      wave_argmin(lane < Ke ? prev : INFINITY, lane, bv, bi);
      __syncthreads();  // backpointers written by other lanes
      if (lane == 0) {
        int pl = endl;
        int jj = bi;
        while (true) {
          sState[pl] = (int8_t)jj;
          if (sCs[pl]) break;
          jj = sBp[sEoff[pl] + jj];
          pl = sCprev[pl];
        }
      }
    };
    // The forward pass walks the points in chunks of 64 whose metadata sits
    // in registers (lane k holds point c0 + k) and is read with readlane: the
    // per-column chain keeps one LDS round trip (emission + transition reads,
    // issued together) instead of five dependent ones.
    int lastK = 0;  // candidates of column `last`
    for (int c0 = 0; c0 < n; c0 += TB) {
      const int pk = c0 + lane;
      const int r_kc = pk < n ? (int)sKc[pk] : -1;
      const int r_eo = pk < n ? (int)sEoff[pk] : 0;
      const int r_cp = pk < n ? (int)sCprev[pk] : -1;
      const int r_to = pk < n ? sToff[pk] : 0;
      const int cend = n - c0 < TB ? n - c0 : TB;
      for (int k = 0; k < cend; ++k) {
        const int pl = c0 + k;
        const int Kp = __builtin_amdgcn_readlane(r_kc, k);
        if (Kp < 0) continue;
        if (Kp == 0) {
          if (open) backtrack(last, lastK);
          open = false;
          continue;
        }
        if (pl >= win_end) {
          // next window: the longest run of points from pl whose transitions
          // and emissions fit (one point always does)
          __syncthreads();
          wt0 = sToff[pl];
          we0 = sEoff[pl];
          // window end: Toff / Eoff are monotone, so the points that fit are
          // a prefix -- 64 candidates per LDS round trip, counted by ballot
          int we = pl + 1;
          while (we < n) {
            const int q = we + 1 + lane;
            const bool ok = q <= n && sToff[q] - wt0 <= VIT_TW && sEoff[q] - we0 <= VIT_EW;
            const int cnt = __popcll(__ballot(ok));
            we += cnt;
            if (cnt < TB) break;
          }
          win_end = we;
          const int nt = sToff[win_end] - wt0;
          for (int f0 = 0; f0 < nt; f0 += 8 * TB) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int f = f0 + u * TB + lane;
              v[u] = f < nt ? w.trans[t0 + wt0 + f] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              const int f = f0 + u * TB + lane;
              if (f < nt) sT[f] = v[u];
            }
          }
          // emissions point-parallel: lane q copies point q's candidates
          // (independent loads, no search for a candidate's point)
          for (int q0 = pl; q0 < win_end; q0 += TB) {
            const int q = q0 + lane;
            int kq = 0, eq = 0;
            if (q < win_end) {
              kq = sKc[q];
              eq = sEoff[q] - we0;
            }
            // the inline slots as two 16-byte loads of the point's 32-byte
            // block (consecutive lanes: consecutive blocks), the rest (points
            // with more than KIN candidates) from the overflow slots
            if (kq > 0) {
              const float4* e4 = (const float4*)(w.cand_em + (a + q) * KIN);
              const float4 x0 = e4[0];
              const float4 x1 = KIN > 4 && kq > 4 ? e4[KIN > 4 ? 1 : 0] : x0;
              const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
              for (int u = 0; u < KIN; ++u)
                if (u < kq) sEm[eq + u] = v[u];
            }
            for (int j0 = KIN; __ballot(j0 < kq) != 0ull; j0 += 4) {
              float v[4];
#pragma unroll
              for (int u = 0; u < 4; ++u)
                v[u] = j0 + u < kq ? w.cand_xem[(a + q) * KX + (j0 - KIN + u)] : 0.0f;
#pragma unroll
              for (int u = 0; u < 4; ++u)
                if (j0 + u < kq) sEm[eq + j0 + u] = v[u];
            }
          }
          __syncthreads();
        }
        const int eo = __builtin_amdgcn_readlane(r_eo, k);
        const float em = sEm[eo - we0 + (lane < Kp ? lane : 0)];
        bool started = false;
        float cur = INFINITY;
        if (open && __builtin_amdgcn_readlane(r_cp, k) == last) {
          const int Kq = lastK;
          const float* Tm = sT + (__builtin_amdgcn_readlane(r_to, k) - wt0) + (lane < Kp ? lane : 0);
          float best = INFINITY;
          int bi = -1;
          const int pbits = __float_as_int(prev);
          int i = 0;
          for (; i + 4 <= Kq; i += 4) {
            // four independent LDS reads in flight.  The four in i order with
            // strict < are: the chunk's minimum, if below best, at the first
            // u that reaches it -- a min tree and three selects instead of
            // four compare-and-select pairs (sums of costs >= +0: no NaN, no
            // -0, so min and == see exactly what < saw)
            float tv[4], pv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              tv[u] = Tm[(i + u) * Kp];
              pv[u] = __int_as_float(__builtin_amdgcn_readlane(pbits, i + u));
            }
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = pv[u] + tv[u];
            const float m = fminf(fminf(v[0], v[1]), fminf(v[2], v[3]));
            const int fu = v[0] == m ? 0 : (v[1] == m ? 1 : (v[2] == m ? 2 : 3));
            if (m < best) {
              best = m;
              bi = i + fu;
            }
          }
          for (; i < Kq; ++i) {
            const float v = __int_as_float(__builtin_amdgcn_readlane(pbits, i)) + Tm[i * Kp];
            if (v < best) {
              best = v;
              bi = i;
            }
          }
          const bool alive = lane < Kp && bi >= 0;
          if (lane < Kp) {
            cur = alive ? best + em : INFINITY;
            sBp[eo + lane] = alive ? (uint8_t)bi : (uint8_t)0xFF;
          }
          if (__ballot(alive) == 0ull) {
            backtrack(last, lastK);
          } else {
            started = true;
          }
        } else if (open) {
          backtrack(last, lastK);
        }
        if (!started) {
          cur = lane < Kp ? em : INFINITY;
          if (lane == 0) sCs[pl] = 1;
        }
        prev = cur;
        open = true;
        last = pl;
        lastK = Kp;
      }
    }
    if (open) backtrack(last, lastK);
    __syncthreads();
    for (int pl = lane; pl < n; pl += TB) {
      const int st = sState[pl];
      const int cs = sCs[pl];
      w.state[a + pl] = st;
      w.chain_start[a + pl] = (uint8_t)cs;
      // the chosen candidate, compact for the route and segment stages
      if (st >= 0) {
        w.chosen[a + pl] = crec(w, a + pl, st);
      }
    }
    __syncthreads();
  }
}

// K5, G lanes per trace (G = 8 or 16: 64 / G traces per wavefront; DESIGN.md
// §5 K5).  The wave-per-trace form above is VALU-issue bound (round 3 PMC:
// 534M VALU instructions over 10M points at config 4, 82 % of the SIMDs'
// cycles) with Kq <= 8 of its 64 lanes holding states; here one instruction
// stream steps 64 / G traces.  A group (lane j = state j) walks its trace's
// points in chunks of OTM_VG_CHUNK:
//  * a chunk's transition blocks (contiguous in the trace's stream, bounded
//    by K3's trans_off) and its points' emissions are loaded into registers
//    one chunk ahead -- in flight while the group steps through the current
//    chunk -- and staged through a per-group LDS window at the chunk's start
//    (a chunk whose blocks exceed the window reads them from HBM per step);
//    the per-point metadata is K3's one byte (vmeta), loaded two chunks ahead;
//  * a step reads its point's byte by shuffle and its block from LDS;
//  * a column's backpointers as one byte per state in LDS; a chain's end
//    records its argmin state;
//  * after the forward pass one lane per group walks the trace backward.
// (Round 4's first form loaded each step's block from HBM at the step: one
// exposed round trip per point, 0.645 ms on config 2 against 0.155 for the
// wave form.)  A trace with a column of more than G candidates, or more than
// VG_PTS points, goes to the next form's list (G = 8 -> G = 16 -> the wave
// form).  Same recurrence (min over i in order, strict <), tie rules and chain
// breaks as viterbi_trace_global: bit-identical to the oracle.
// The block is one wavefront (TB = 64): a chunk's staging needs only
// wave_sync(), not __syncthreads(), which would wait for the next chunks'
// prefetches.
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int x = __shfl_xor(v, o, 64);
    v = x > v ? x : v;
  }
  return v;
}
// waves per SIMD: 8 lanes per trace fits 4 in 128 VGPRs with a 12-float
// window per lane; 16 lanes per trace spills at 4, so 3
#ifndef OTM_VG8_WAVES
#define OTM_VG8_WAVES 4
#endif
#ifndef OTM_VG8_U
#define OTM_VG8_U 8
#endif
// points per chunk: 8 or 16 overflowed the 16-float-per-lane window on most of
// config 2's chunks (~20 transition floats per column), whose steps then read
// their blocks from HBM one round trip each (form 8: 0.699 ms, config 2)
#ifndef OTM_VG_CHUNK
#define OTM_VG_CHUNK 4
#endif
constexpr int VG_PTS = 128;  // points per trace
constexpr uint8_t VG_COL = 1, VG_CS = 2, VG_END = 4;  // point flags (VG_END: argmin state in bits 3..7)
template <int G>
__global__ __launch_bounds__(TB, G == 8 ? OTM_VG8_WAVES : 3) void k_viterbi_g(DevBatch b, DevWork w, const int32_t* list,
                                                                const int32_t* list_n, int32_t* rej, int32_t* rej_n,
                                                                int snap) {
  static_assert(G == 8 || G == 16, "8 or 16 lanes per trace");
  constexpr int NT = TB / G;
  constexpr int U = G == 8 ? OTM_VG8_U : 16;  // transition floats per lane per chunk
  constexpr int VT = U * G;                    // ... per chunk window
  constexpr int CH = OTM_VG_CHUNK;  // points per chunk (<= G)
  static_assert(CH <= G, "a chunk's metadata is one byte per lane");
  // spill snapshot B (see k_viterbi)
  if (OTM_FOLD_BOOKKEEPING && snap && blockIdx.x == 0 && threadIdx.x == 0) fold_snap(w, 1, true);
  if (*w.abort) return;
  // group rows padded by G words: group g's row starts g x G banks on, so the
  // wave's 64 lanes staging (or reading) the same offset j of their groups'
  // rows hit 64 different banks (round 4's one-word pad put group g + 1's
  // j on group g's j + 1: 39 % of the LDS cycles were bank conflicts, config 4)
  __shared__ float sT[NT][VT + G];
  __shared__ float sE[NT][CH * G + G];  // [point of the chunk][state]
  // backpointers, a nibble per state (15: dead), two states a byte: [point * G / 2 + state / 2]
  __shared__ uint8_t sBp[NT][VG_PTS * G / 2 + 4];
  __shared__ uint8_t sFl[NT][VG_PTS];  // flags; after the walk: VG_CS | (state + 1) << 3
  // each group's previous-column scores, so a step reads four of them with one
  // 16-byte broadcast read instead of four cross-lane shuffles
  __shared__ __attribute__((aligned(16))) float sP[NT][G];
  const int lane = threadIdx.x;
  const int g = lane / G, j = lane % G, gb = g * G;
  const unsigned long long gmask = (1ull << G) - 1ull;
  const int32_t ntr = list ? *list_n : b.n_traces;
  for (int32_t tb = blockIdx.x * NT; tb < ntr; tb += gridDim.x * NT) {
    const int32_t it = tb + g;
    bool act = it < ntr;
    const int32_t t = act ? (list ? list[it] : it) : 0;
    int64_t a = 0;
    int n = 0;
    int64_t t0 = 0;
    if (act) {
      a = b.trace_off[t];
      n = (int)(b.trace_off[t + 1] - a);
      t0 = w.trans_off[a];
      if (w.trace_err[t] != 0) {
        for (int pl = j; pl < n; pl += G) {
          w.state[a + pl] = -1;
          w.chain_start[a + pl] = 0;
        }
        act = false;
      }
    }
    // a trace this form cannot take: to the next form's list
    bool take = act && n <= VG_PTS;
    if (take) {
      bool wide = false;
      for (int pl = j; pl < n; pl += G) {
        const int vm = w.vmeta[a + pl];
        wide = wide || ((vm & 0x40) && (vm & 0x3F) > G);
      }
      take = ((__ballot(wide) >> gb) & gmask) == 0ull;
    }
    if (act && !take) {
      if (j == 0) rej[atomicAdd(rej_n, 1)] = t;
      act = false;
    }
    if (!act) n = 0;
    const int nch = (wave_max_i(n) + CH - 1) / CH;
    for (int pl = j; pl < n; pl += G) sFl[g][pl] = 0;
    // ---- the chunk pipeline: data two chunks ahead (two register sets, A for
    // even chunks, B for odd), metadata and T range four ahead
    // Every pipeline load is issued unconditionally (indices clamped into the
    // trace, results masked after): a fixed count per chunk lets the compiler
    // wait for exactly the older set, not for everything in flight.
    const int nl = n > 0 ? n - 1 : 0;  // (a trace's last point; 0 for an idle group)
    // (raw: a step reads lane k < CH's byte, and only for a point pl < n)
    auto ld_meta = [&](int c) {
      const int pl = c * CH + j;
      return (int)w.vmeta[a + (pl < nl ? pl : nl)];
    };
    // (the raw offsets: the subtraction waits for the loads, so it is done
    // where they are used, chunks later)
    auto ld_range = [&](int c, int64_t& lo, int64_t& hi) {
      const int p0 = c * CH < n ? c * CH : n, p1 = c * CH + CH < n ? c * CH + CH : n;
      lo = w.trans_off[a + p0];
      hi = w.trans_off[a + p1];
    };
    float pTa[U], pEa[CH], pTb[U], pEb[CH];
    auto ld_data = [&](int c, int m, int lo, int hi, float (&pT)[U], float (&pE)[CH]) {
      // raw values, no select on them here (a select would wait for the
      // load): the steps read only a window's valid floats and a point's
      // candidates (lo, hi: from the trace's first float; past hi, the
      // stream's capacity headroom)
      (void)m;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int f = lo + u * G + j;
        pT[u] = w.trans[t0 + (f < hi ? f : lo)];
      }
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int pl = c * CH + k < nl ? c * CH + k : nl;
        pE[k] = j < KIN ? w.cand_em[(a + pl) * KIN + j] : w.cand_xem[(a + pl) * KX + (j - KIN)];
      }
    };
    int m0 = ld_meta(0), m1 = ld_meta(1), m2 = ld_meta(2), m3 = ld_meta(3);
    int64_t lo0, hi0, lo1, hi1, lo2, hi2, lo3, hi3;
    ld_range(0, lo0, hi0);
    ld_range(1, lo1, hi1);
    ld_range(2, lo2, hi2);
    ld_range(3, lo3, hi3);
    ld_data(0, m0, (int)(lo0 - t0), (int)(hi0 - t0), pTa, pEa);
    ld_data(1, m1, (int)(lo1 - t0), (int)(hi1 - t0), pTb, pEb);
    // ---- forward pass (wave-uniform step count; groups predicated)
    float prev = INFINITY;
    sP[g][j] = INFINITY;
    bool open = false;
    int last = -1, lastK = 0;
    int acc = 0;  // the trace's transition floats before this column (K3's Kq x Kp counts, summed in order)
    auto end_chain = [&]() {
      // argmin (value, state) over the group's lanes < lastK, ties to the lower state
      float bv = j < lastK ? prev : INFINITY;
      int bi = j;
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) {
        const float ov = __shfl_xor(bv, o, G);
        const int oi = __shfl_xor(bi, o, G);
        if (ov < bv || (ov == bv && oi < bi)) {
          bv = ov;
          bi = oi;
        }
      }
      if (j == 0) sFl[g][last] = (uint8_t)(sFl[g][last] | VG_END | (bi << 3));
    };
    auto stage = [&](const float (&pT)[U], const float (&pE)[CH]) {
#pragma unroll
      for (int u = 0; u < U; ++u) sT[g][u * G + j] = pT[u];
#pragma unroll
      for (int k = 0; k < CH; ++k) sE[g][k * G + j] = pE[k];
    };
    auto chunk = [&](int c, int m_c, int lo_c, int hi_c) {
      // A step, for every group at once: its point's byte by shuffle, its
      // emission and block from LDS, Kq in fours (loads issued together), its
      // backpointers as one byte per state in LDS.  The loop bounds are
      // wave-uniform ballots, not unrolled to G (round 4's unrolled form spent
      // ~600 instructions per step).
      const bool big = hi_c - lo_c > VT;  // this group's chunk overflowed its window
      for (int k = 0; k < CH; ++k) {
        const int pl = c * CH + k;
        const int mk = __shfl(m_c, gb + k, TB);
        const bool on = pl < n && (mk & 0x40);
        const int Kp = mk & 0x3F;
        if (on && Kp == 0) {
          if (open) end_chain();
          open = false;
        }
        const bool col = on && Kp > 0;
        const bool link = col && open && (mk & 0x80);
        // a linked column's block follows the trace's earlier ones (its
        // previous column is the open chain's last)
        const int to = acc;
        if (link) acc += lastK * Kp;
        const int jj = j < Kp ? j : 0;
        const float em = sE[g][k * G + jj];
        int tb = to - lo_c;
        if (__ballot(big && link) != 0ull) {
          // the column's block (<= G x G floats) into the window first, so
          // the recurrence reads LDS only
          if (big) {
            tb = 0;
            if (link)
              for (int f = j; f < lastK * Kp; f += G) sT[g][f] = w.trans[t0 + to + f];
          }
        }
        bool started = false;
        float cur = INFINITY;
        if (__ballot(link) != 0ull) {
          float best = INFINITY;
          int bi = -1;
          const float* Tm = &sT[g][tb + jj];
          for (int i0 = 0; __ballot(link && i0 < lastK) != 0ull; i0 += 4) {
            float tv[4], pv[4];
            const float4 p4 = *(const float4*)&sP[g][i0 < G ? i0 : 0];
            pv[0] = p4.x;
            pv[1] = p4.y;
            pv[2] = p4.z;
            pv[3] = p4.w;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int i = i0 + u;
              tv[u] = link && i < lastK ? Tm[i * Kp] : INFINITY;
            }
            // (an i past lastK, or a lane of an unlinked group, reads +inf:
            // its sum is +inf and never below best.)  In i order with strict
            // <, the four are the chunk's minimum, if below best, at the first
            // u that reaches it (k_viterbi's form; costs >= +0: no NaN or -0)
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = pv[u] + tv[u];
            const float m = fminf(fminf(v[0], v[1]), fminf(v[2], v[3]));
            const int fu = v[0] == m ? 0 : (v[1] == m ? 1 : (v[2] == m ? 2 : 3));
            if (m < best) {
              best = m;
              bi = i0 + fu;
            }
          }
          const bool alive = link && j < Kp && bi >= 0;
          if (link) {
            cur = alive ? best + em : INFINITY;
            const int nib = alive ? bi : 15;
            // the neighbour lane's nibble by a DPP quad permute [1,0,3,2] (one VALU op, no
            // LDS-pipe shuffle); every lane of a linked group is here
            const int pair = __builtin_amdgcn_mov_dpp(nib, 0xB1, 0xF, 0xF, false);
            if (!(j & 1)) sBp[g][pl * (G / 2) + (j >> 1)] = (uint8_t)(nib | (pair << 4));
            if (((__ballot(alive) >> gb) & (unsigned long long)gmask) != 0ull) started = true;
            else end_chain();
          }
        }
        if (col && !link && open) end_chain();
        if (col) {
          if (!started) {
            cur = j < Kp ? em : INFINITY;
            if (j == 0) sFl[g][pl] = VG_COL | VG_CS;
          } else if (j == 0) {
            sFl[g][pl] = VG_COL;
          }
          prev = cur;
          sP[g][j] = cur;
          open = true;
          last = pl;
          lastK = Kp;
        }
      }
    };
    for (int c = 0; c < nch; c += 2) {
      // chunk c from set A; chunk c + 2's loads into A behind it
      stage(pTa, pEa);
      const int ma = m0, la = (int)(lo0 - t0), ha = (int)(hi0 - t0);
      const int mn0 = ld_meta(c + 4);
      int64_t ln0, hn0;
      ld_range(c + 4, ln0, hn0);
      wave_sync();
      ld_data(c + 2, m2, (int)(lo2 - t0), (int)(hi2 - t0), pTa, pEa);
      chunk(c, ma, la, ha);
      wave_sync();  // (the next chunk's staging overwrites the windows)
      if (c + 1 >= nch) break;
      // chunk c + 1 from set B; chunk c + 3's loads into B
      stage(pTb, pEb);
      const int mb = m1, lb = (int)(lo1 - t0), hb = (int)(hi1 - t0);
      const int mn1 = ld_meta(c + 5);
      int64_t ln1, hn1;
      ld_range(c + 5, ln1, hn1);
      wave_sync();
      ld_data(c + 3, m3, (int)(lo3 - t0), (int)(hi3 - t0), pTb, pEb);
      chunk(c + 1, mb, lb, hb);
      wave_sync();
      m0 = m2;
      lo0 = lo2;
      hi0 = hi2;
      m1 = m3;
      lo1 = lo3;
      hi1 = hi3;
      m2 = mn0;
      lo2 = ln0;
      hi2 = hn0;
      m3 = mn1;
      lo3 = ln1;
      hi3 = hn1;
    }
    if (act && open) end_chain();
    __syncthreads();
    // ---- backtrack: one lane per group walks the trace backward
    if (j == 0) {
      int sv = -1;
      for (int pl = n - 1; pl >= 0; --pl) {
        const uint32_t f = sFl[g][pl];
        if (!(f & VG_COL)) {
          sFl[g][pl] = 0;
          continue;
        }
        if (f & VG_END) sv = (int)(f >> 3);
        sFl[g][pl] = (uint8_t)((f & VG_CS) | ((sv + 1) << 3));
        if (sv >= 0) {
          if (f & VG_CS) {
            sv = -1;
          } else {
            sv = (sBp[g][pl * (G / 2) + (sv >> 1)] >> ((sv & 1) * 4)) & 15;
          }
        }
      }
    }
    __syncthreads();
    // ---- outputs, point-parallel within the group
    for (int pl = j; pl < n; pl += G) {
      const uint32_t f = sFl[g][pl];
      const int sv = (int)(f >> 3) - 1;
      const int64_t p = a + pl;
      w.state[p] = sv;
      w.chain_start[p] = (uint8_t)((f & VG_CS) ? 1 : 0);
      if (sv >= 0) w.chosen[p] = crec(w, p, sv);
    }
    __syncthreads();
  }
}

// ============================================================== K6 route
// Steps the index tier could not answer (w.overflow_list0 / counters_i32[4]):
// the winning search again, its target label's predecessor chain as the path.
// TIER as k_transitions (spill lists: list0 [4] -> list2 [3] -> list3 [22])
template <int TIER>
__global__ __launch_bounds__(TB) void k_route(DevGraph g, DevBatch b, DevParams P, DevWork w) {
  constexpr bool BIG = TIER > 0;
  if (*w.abort) return;
  __shared__ uint32_t lkey[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ unsigned long long llab[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ uint32_t linq[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ uint32_t lfr0[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ uint32_t lfr1[BIG ? 1 : LDS_TABLE_CAP];
  __shared__ int32_t cbuf[CHAIN_BUF * TB];
  __shared__ uint32_t TU[TURN_TABLE];
  __shared__ SearchShared S;
  const int lane = threadIdx.x;
  for (int k = lane; k < TURN_TABLE; k += TB) TU[k] = P.turn_units[k];
  Table T = tier_table<TIER>(w, lkey, llab, linq, lfr0, lfr1);
  auto predof = [&](uint32_t e) {
    const int sx = table_find<BIG>(T, e);
    return sx < 0 ? NONE_PRED : (uint32_t)(Mem<BIG>::ld(&T.lab[sx]) & 0xFFFFFFFFull);
  };
  const int32_t* list = TIER == 2 ? w.overflow_list3 : (BIG ? w.overflow_list2 : w.overflow_list0);
  const int64_t nwork = TIER == 2 ? (int64_t)w.counters_i32[22]
                                  : (BIG ? (int64_t)w.counters_i32[3] : (int64_t)w.counters_i32[4]);
  if (TIER == 2 && huge_unready(w, nwork, list)) return;
  __syncthreads();
  for (int64_t it = blockIdx.x; it < nwork; it += gridDim.x) {
    const int64_t p = (int64_t)list[it];
    const int32_t q = w.col_prev[p];
    const int2 ci = w.chosen[q], cj = w.chosen[p];
    const int32_t ei = ci.x, ej = cj.x;
    const float oi = __int_as_float(ci.y), oj = __int_as_float(cj.y);
    if (same_edge_step(ei, oi, ej, oj)) {
      if (lane == 0) w.route_dist[p] = same_edge_dist(oi, oj);
      continue;
    }
    const float bound = P.factor * w.gc[p];
    const uint32_t cq = index_cost_bound(bound);
    const int32_t u = src_node(g, ei, oi);
    const uint32_t hin = src_head(g, ei, oi);
    const int labels = ta_search<BIG>(g, TU, T, S, u, hin, cq, lane);
    if (labels < 0) {
      if (lane == 0) {
        if (TIER == 0) {
          w.overflow_list2[atomicAdd(&w.counters_i32[3], 1)] = (int32_t)p;
        } else if (TIER == 1) {
          w.overflow_list3[atomicAdd(&w.counters_i32[22], 1)] = (int32_t)p;
        } else {
          huge_overflow(w, p);
        }
      }
      __syncthreads();
      continue;
    }
    unsigned long long st = 0, rl = 0;
    if (w.ctr) ta_counts<BIG>(g, T, cq, lane, st, rl);
    if (lane == 0) {
      const uint32_t key = dst_key(g, ej, oj);
      const int vs = table_find<BIG>(T, key);
      if (vs < 0) {
        // (cannot happen: the step's transition was finite)
        atomicCAS(&w.trace_err[w.pt_trace[p]], 0, OTM_TERR_SEARCH_OVERFLOW);
      } else {
        const uint32_t pk = (uint32_t)(Mem<BIG>::ld(&T.lab[vs]) & 0xFFFFFFFFull);
        float d;
        uint32_t units;
        int n;
        chain_sums(g, TU, predof, pk, hin, NO_HEAD, cbuf, d, units, n);
        const int off = atomicAdd(&w.counters_i32[1], n);
        if (off + n > w.pool_cap) {
          w.counters_i32[2] = 1;
          *w.abort = 1;
          w.path_len[p] = -1;
        } else {
          int k = n;
          for (uint32_t pe = pk; pe != NONE_PRED && k > 0; pe = predof(pe)) w.path_pool[off + (--k)] = (int32_t)pe;
          w.path_off[p] = off;
          w.path_len[p] = n;
        }
        const float start = src_start(g, ei, oi);
        const float sd = start + d;
        w.route_dist[p] = sd + oj;
        if (w.ctr) {
          cadd(&w.ctr->route_searches, 1);
          cadd(&w.ctr->route_nodes_settled, st);
          cadd(&w.ctr->route_edges_relaxed, rl);
          cadd(&w.ctr->route_edges, (unsigned long long)n);
        }
      }
    }
    __syncthreads();
  }
}

// ============================================================== K7 segments
// Per-edge attributes the emitter needs, carried with each traversal so the
// serial grouping never goes back to HBM for a state edge.
struct EAttr {
  float len;
  int32_t seg, seg_pos;
  uint32_t flags;
  int64_t way;
  uint64_t gid;  // segment id / length of e_seg (when seg >= 0)
  float glen;
};

// the edge's K7 record (one 16-byte load): {len bits, seg, seg_pos | flags << 24, way number}
__device__ __forceinline__ uint4 edge_rec(const DevGraph& g, int32_t e) { return g.e_rec[e]; }
__device__ __forceinline__ float rec_len(const uint4& r) { return __uint_as_float(r.x); }
__device__ __forceinline__ int32_t rec_seg(const uint4& r) { return (int32_t)r.y; }
__device__ __forceinline__ int32_t rec_pos(const uint4& r) { return (int32_t)(r.z & 0xFFFFFFu); }
__device__ __forceinline__ uint32_t rec_flags(const uint4& r) { return r.z >> 24; }

__device__ __forceinline__ EAttr edge_attr(const DevGraph& g, int32_t e) {
  const uint4 r = edge_rec(g, e);
  EAttr a;
  a.len = rec_len(r);
  a.seg = rec_seg(r);
  a.seg_pos = a.seg >= 0 ? rec_pos(r) : 0;
  a.flags = rec_flags(r);
  a.way = g.way_tab[r.w];
  a.gid = a.seg >= 0 ? g.g_id[a.seg] : 0ull;
  a.glen = a.seg >= 0 ? g.g_len[a.seg] : 0.0f;
  return a;
}

struct Trav {
  int32_t edge;
  float off0, off1;
  double t0, t1;
  int32_t sh0, sh1;
  EAttr at;
};

template <bool WRITE>
struct SegEmitter {
  DevOut* o;
  int32_t seg_base, way_base;  // write positions (WRITE)
  int32_t nseg = 0, nway = 0;
  // open group
  bool has = false;
  Trav first, last;
  int32_t way_start = 0;
  int64_t last_way = 0;

  __device__ void add_way(const EAttr& at) {
    const int64_t way = at.way;
    if (nway > way_start && last_way == way) return;
    if (WRITE) o->way_ids[way_base + nway] = way;
    last_way = way;
    ++nway;
  }
  __device__ void flush() {
    if (!has) return;
    if (WRITE) {
      otm_segment s;
      const int32_t sg = first.at.seg;
      bool sv, ev;
      s.flags = 0u;
      if (sg >= 0) {
        sv = first.off0 == 0.0f && (first.at.flags & OTM_EDGE_SEG_BEGIN_D);
        ev = last.off1 == last.at.len && (last.at.flags & OTM_EDGE_SEG_END_D);
        s.segment_id = (int64_t)first.at.gid;
        s.length = (sv && ev) ? (int32_t)floor((double)first.at.glen + 0.5) : -1;
      } else {
        sv = first.off0 == 0.0f;
        ev = last.off1 == last.at.len;
        s.segment_id = -1;
        s.length = -1;
        if (first.at.flags & OTM_EDGE_INTERNAL_D) s.flags |= OTM_SEG_INTERNAL;
      }
      s.start_time = 0.0;
      s.end_time = 0.0;
      if (sv) {
        s.flags |= OTM_SEG_START_VALID;
        s.start_time = first.t0;
      }
      if (ev) {
        s.flags |= OTM_SEG_END_VALID;
        s.end_time = last.t1;
      }
      s.queue_length = 0;
      s.begin_shape_index = first.sh0;
      s.end_shape_index = last.sh1;
      s.way_off = way_base + way_start;
      s.way_cnt = nway - way_start;
      s.pad = 0u;
      ((otm_segment*)o->segments)[seg_base + nseg] = s;
      o->seg_gidx[seg_base + nseg] = sg;
    }
    ++nseg;
    has = false;
  }
  __device__ void push(const Trav& t) {
    bool join = false;
    if (has) {
      const int32_t s = t.at.seg, ps = last.at.seg;
      if (s >= 0) join = ps == s && t.at.seg_pos == last.at.seg_pos + 1;
      else join = ps < 0 && ((t.at.flags ^ last.at.flags) & OTM_EDGE_INTERNAL_D) == 0;
    }
    if (!join) {
      flush();
      has = true;
      first = t;
      way_start = nway;
    }
    last = t;
    add_way(t.at);
  }
  static constexpr uint32_t OTM_EDGE_INTERNAL_D = 0x01, OTM_EDGE_SEG_BEGIN_D = 0x02, OTM_EDGE_SEG_END_D = 0x04;
};

__device__ __forceinline__ double time_at(double ta, double tb, float x, float R) {
  if (R > 0.0f) return ta + (tb - ta) * ((double)x / (double)R);
  return ta;
}

// The boundary of step lp -> pl (trace-local points of the trace at a) at
// route distance x (DESIGN.md §3 rule 7, oracle step_bound): the step's
// anchors are lp (position 0), its placed interpolated points (K7a) and pl (R);
// the time is linear between the last anchor before pl at position <= x and
// the anchor after it, the shape index is the last anchor at position <= x.
// Without interpolated points: the two-state rule, bit for bit.
__device__ __forceinline__ void step_bound(const DevBatch& b, const DevWork& w, int64_t a, int lp, int pl, float R,
                                           double ta, double tb, float x, double& t, int& sh) {
  if (pl - lp < 2) {
    t = time_at(ta, tb, x, R);
    sh = x >= R ? pl : lp;
    return;
  }
  int iL = lp, k = lp + 1;
  float xL = 0.0f, xN = R, run = 0.0f;
  double tL = ta, tN = tb;
  for (; k < pl; ++k) {
    const float v = w.ipos[a + k];
    if (!(v >= run)) continue;  // unplaced, or behind an earlier anchor: no anchor
    if (!(v <= x)) break;
    iL = k;
    xL = v;
    tL = b.time[a + k];
    run = v;
  }
  for (; k < pl; ++k) {
    const float v = w.ipos[a + k];
    if (v >= run) {
      xN = v;
      tN = b.time[a + k];
      break;
    }
  }
  sh = R <= x ? pl : iL;
  const float den = xN - xL;
  t = den > 0.0f ? tL + (tN - tL) * ((double)(x - xL) / (double)den) : tL;
}

// Point data of one trace as the emitter reads it: straight from HBM ...
struct SegSrcGlobal {
  const DevGraph* g;
  const DevBatch* b;
  const DevWork* w;
  int64_t a;
  __device__ int state(int pl) const {
    const int64_t p = a + pl;
    return w->is_col[p] ? w->state[p] : -1;
  }
  __device__ bool cs(int pl) const { return w->chain_start[a + pl] != 0; }
  __device__ double time(int pl) const { return b->time[a + pl]; }
  __device__ float rd(int pl) const { return w->route_dist[a + pl]; }
  __device__ int32_t poff(int pl) const { return w->path_off[a + pl]; }
  __device__ int32_t plen(int pl) const { return w->path_len[a + pl]; }
  __device__ int32_t edge(int pl) const { return w->chosen[a + pl].x; }
  __device__ float off(int pl) const { return __int_as_float(w->chosen[a + pl].y); }
  __device__ EAttr attr(int pl) const { return edge_attr(*g, edge(pl)); }
};

// The traversal walk of one trace (one thread): states in order, chains,
// per step the close of the open traversal, the route's path edges and the
// re-open on the new edge; traversals grouped into OSMLR segments.
template <bool WRITE, class Src>
__device__ void segments_trace(const DevGraph& g, const DevWork& w, DevOut& o, int32_t t, int n, int32_t base,
                               const Src& S) {
  SegEmitter<WRITE> em;
  em.o = &o;
  em.seg_base = base;
  em.way_base = base;
  bool open = false;
  int nstate = 0;
  Trav cur{};
  int lastp = -1;
  float curmax = 0.0f;
  for (int p = 0; p <= n; ++p) {
    const int st = p < n ? S.state(p) : -1;
    if (p < n && st < 0) continue;
    const bool new_chain = p == n || S.cs(p);
    if (open && new_chain) {
      cur.off1 = curmax;  // the open traversal's largest state offset (rule 4's stays)
      cur.t1 = S.time(lastp);
      cur.sh1 = lastp;
      if (nstate >= 2) {
        // a chain ending on a node candidate ends at the node: the traversal
        // opened there never left it
        if (!cand_node(cur.off1)) em.push(cur);
        em.flush();
      }
      open = false;
    }
    if (p == n) break;
    const int32_t ej = S.edge(p);
    const float oj = S.off(p);
    if (new_chain) {
      cur.edge = ej;
      cur.at = S.attr(p);
      cur.off0 = oj;
      cur.t0 = S.time(p);
      cur.sh0 = p;
      curmax = oj;
      open = true;
      nstate = 1;
      lastp = p;
      continue;
    }
    const float Rd = S.rd(p);
    const double ta = S.time(lastp), tb = S.time(p);
    const int32_t ca = lastp, cb = p;
    const int32_t ei = cur.edge;
    const float oi = S.off(lastp);
    const bool same = same_edge_step(ei, oi, ej, oj);
    if (!same) {
      // close the traversal on the state's edge, unless the state is a node
      // candidate: its route starts at the node
      const float elen = cur.at.len;  // == e_len[ei]
      const float start = cand_node(oi) ? 0.0f : elen - oi;
      float x = start;
      cur.off1 = elen;
      int sh;
      step_bound(*S.b, w, S.a, ca, cb, Rd, ta, tb, x, cur.t1, sh);
      cur.sh1 = sh;
      if (!cand_node(oi)) em.push(cur);
      float dd = 0.0f;
      const int32_t po = S.poff(p), pl = S.plen(p);
      for (int k = 0; k < pl; ++k) {
        const int32_t pe = w.path_pool[po + k];
        Trav m;
        m.edge = pe;
        m.at = edge_attr(g, pe);
        m.off0 = 0.0f;
        m.off1 = m.at.len;
        const float xb = start + dd;
        dd = dd + m.at.len;
        const float xe = start + dd;
        step_bound(*S.b, w, S.a, ca, cb, Rd, ta, tb, xb, m.t0, sh);
        m.sh0 = sh;
        step_bound(*S.b, w, S.a, ca, cb, Rd, ta, tb, xe, m.t1, sh);
        m.sh1 = sh;
        em.push(m);
      }
      x = start + dd;
      cur.edge = ej;
      cur.at = S.attr(p);
      cur.off0 = 0.0f;
      step_bound(*S.b, w, S.a, ca, cb, Rd, ta, tb, x, cur.t0, sh);
      cur.sh0 = sh;
      curmax = oj;
    } else if (oj > curmax) {
      curmax = oj;
    }
    ++nstate;
    lastp = p;
  }
  o.seg_cnt[t] = em.nseg;
  o.way_cnt[t] = em.nway;
}

// One wavefront per trace, wave-parallel.  The serial walk
// above is a scan in disguise:
//  * the open traversal's edge at every step is the previous state's edge,
//    and it was opened by the latest "opener" state (a chain start, or a step
//    that left the edge) -- a max-scan over the states;
//  * each state emits a known number of traversals (close + route edges when
//    it leaves the edge, + the chain's final close) -- a sum-scan gives each
//    its slot; the lanes then write the traversals in parallel;
//  * a traversal joins its predecessor's group by a test of the two alone --
//    segment and way-id slots are counts of group starts / way changes.
// Float and double expressions are the walk's, in the walk's order (the route
// edges' f32 prefix sum stays sequential per state), so the records are
// bit-identical.  Traces beyond SEGP_PTS points or SEGP_TRAV traversals take
// the serial walk out of global memory (lane 0).
// Two LDS plans: a trace first tries the small one (128 states, 256
// traversals: 13.6 KB, 3 waves per SIMD); one that does not fit goes to a
// list for the large one (256 / 512: 26.6 KB); beyond that, the serial walk.
// Measured on config 2: 0.131 -> 0.111 ms against the large plan alone.
// Diagnostic phase timing of k_segments (a build with -DOTM_SEG_PROF only):
// per wave the clock between the phase boundaries, summed over the launch and
// printed by the launch's last wave for a launch over >= 50k traces.
#ifdef OTM_SEG_PROF
__device__ unsigned long long g_segp[10];
__device__ unsigned int g_segp_done, g_segp_prints;
#define SEGP_DECL unsigned long long segp_acc[9] = {}; long long segp_t = 0; unsigned long long segp_n = 0;
#define SEGP_START { segp_t = clock64(); ++segp_n; }
#define SEGP_MARK(i) { const long long _n = clock64(); segp_acc[i] += (unsigned long long)(_n - segp_t); segp_t = _n; }
#define SEGP_END                                                                                          \
  if (threadIdx.x == 0) {                                                                                 \
    for (int _i = 1; _i <= 8; ++_i) atomicAdd(&g_segp[_i], segp_acc[_i]);                                 \
    atomicAdd(&g_segp[9], segp_n);                                                                        \
    __threadfence();                                                                                      \
    if (atomicAdd(&g_segp_done, 1u) == gridDim.x - 1) {                                                   \
      unsigned long long v[10];                                                                           \
      for (int _i = 1; _i <= 9; ++_i) v[_i] = atomicAdd(&g_segp[_i], 0ull);                               \
      if (nwork >= 5000 && atomicAdd(&g_segp_prints, 1u) < 4)                                            \
        printf("SEGP traces %llu cycles/trace: states %llu scan %llu mark %llu fetch %llu opener %llu "  \
               "trav %llu group %llu record %llu\n", v[9], v[1] / v[9], v[2] / v[9], v[3] / v[9],      \
               v[4] / v[9], v[5] / v[9], v[6] / v[9], v[7] / v[9], v[8] / v[9]);                         \
      for (int _i = 0; _i <= 9; ++_i) atomicExch(&g_segp[_i], 0ull);                                     \
      atomicExch(&g_segp_done, 0u);                                                                       \
    }                                                                                                     \
  }
#else
#define SEGP_DECL
#define SEGP_START
#define SEGP_MARK(i)
#define SEGP_END
#endif

template <int PT, int TR>
struct SegParT {
  double o_t0[PT];  // per state: start time of the traversal it opens
  double t_t0[TR], t_t1[TR];
  float o_off0[PT];
  int32_t tbase[PT + 1];  // first traversal slot of each state
  int32_t t_edge[TR];
  float t_off0[TR], t_off1[TR];
  int16_t sidx[PT + 1];  // point of each state
  int16_t o_sh0[PT];
  int16_t lopen[PT];  // latest opener <= k
  int16_t chain[PT];
  int16_t t_sh0[TR], t_sh1[TR], t_chain[TR];
  int16_t g_first[TR], g_last[TR], g_w0[TR + 1];
  int32_t nt;
};
// small plan: 128 states / 160 traversals (~9.5 KB of LDS, 4 waves per SIMD);
// measured against 256 traversals (13.3 KB, 3 waves): 0.082 -> 0.075 ms on
// config 2, 1.04 -> 0.88 ms on a config-3 shard; 128-192 are within noise
#ifndef OTM_SEGP_TRAV_S
#define OTM_SEGP_TRAV_S 160
#endif
constexpr int SEGP_PTS_S = 128, SEGP_TRAV_S = OTM_SEGP_TRAV_S;
constexpr int SEGP_PTS = 256, SEGP_TRAV = 512;

__device__ __forceinline__ int wave_incl_max(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int n = __shfl_up(v, o, 64);
    if (lane >= o) v = n > v ? n : v;
  }
  return v;
}

// what a state contributes (recomputed in the two passes that need it).
// Every global load of a state is issued at once, unconditionally -- none
// depends on another (the neighbours' points come from LDS) -- so a pass
// costs one round trip for them, not three (round 6; the values and the
// arithmetic on them are the same as before).
struct StateStep {
  int32_t pts;     // point (low 16 bits) | previous state's point << 16
  uint32_t f;      // 1 chain start, 2 last state of its chain, 4 a step from lp, 8 stays on the open edge
  int32_t ei, ej;  // previous state's edge (== the open traversal's), own edge
  float oi, oj;
  int32_t plen, poff;
  double ta, tb;   // times of lp and pl
  float rd;        // the step's route distance
  __device__ int pl() const { return pts & 0xFFFF; }
  __device__ int lp() const { return pts >> 16; }
  __device__ bool cs() const { return f & 1u; }
  __device__ bool last() const { return f & 2u; }
  __device__ bool step() const { return f & 4u; }
  __device__ bool same() const { return f & 8u; }
};
template <class SP>
__device__ __forceinline__ StateStep state_step(const DevWork& w, const DevBatch& b, int64_t a, const SP& S, int k,
                                                int ns) {
  StateStep r;
  const int pl = S.sidx[k];
  const int nx = k + 1 < ns ? S.sidx[k + 1] : pl;
  const int pv = k > 0 ? S.sidx[k - 1] : pl;
  const int64_t p = a + pl;
  const bool csp = w.chain_start[p] != 0;
  const bool csn = w.chain_start[a + nx] != 0;
  const int2 cj = w.chosen[p];
  const int2 cv = w.chosen[a + pv];
  const int32_t pln = w.path_len[p], pof = w.path_off[p];
  const double tp = b.time[p], tv = b.time[a + pv];
  r.rd = w.route_dist[p];
  const bool last = k == ns - 1 || csn;
  const bool step = !csp && k > 0;
  const int lp = step ? pv : pl;
  r.pts = pl | (lp << 16);
  r.ej = cj.x;
  r.oj = __int_as_float(cj.y);
  const int2 ci = step ? cv : cj;
  r.ei = ci.x;
  r.oi = __int_as_float(ci.y);
  const bool same = step && same_edge_step(r.ei, r.oi, r.ej, r.oj);
  r.f = (csp ? 1u : 0u) | (last ? 2u : 0u) | (step ? 4u : 0u) | (same ? 8u : 0u);
  const bool leaves = step && !same;
  r.plen = leaves ? (pln > 0 ? pln : 0) : 0;
  r.poff = leaves ? pof : 0;
  r.tb = tp;
  r.ta = step ? tv : tp;
  return r;
}

// list / list_n: the traces to walk (null: all); spill / spill_n: where a
// trace beyond this plan goes (null: the serial walk)
template <int PT, int TR>
__global__ __launch_bounds__(TB, (PT <= 128 ? 4 : 2)) void k_segments(DevGraph g, DevBatch b, DevWork w, DevOut o, const int32_t* list,
                                                 const int32_t* list_n, int32_t* spill, int32_t* spill_n) {
  if (*w.abort) return;  // a capacity was exceeded: the host redoes the batch
  __shared__ SegParT<PT, TR> S;
  const int lane = threadIdx.x;
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int32_t nwork = list ? *list_n : b.n_traces;
  SEGP_DECL
  for (int32_t it = blockIdx.x; it < nwork; it += gridDim.x) {
    SEGP_START
    const int32_t t = list ? list[it] : it;
    const int64_t a = b.trace_off[t];
    const int n = (int)(b.trace_off[t + 1] - a);
    const int32_t base = (int32_t)o.seg_base[t];
    if (w.trace_err[t] != 0) {
      if (lane == 0) {
        o.seg_cnt[t] = 0;
        o.way_cnt[t] = 0;
      }
      continue;
    }
    if (n > PT) {
      if (lane == 0) {
        if (spill) spill[atomicAdd(spill_n, 1)] = t;
        else segments_trace<true>(g, w, o, t, n, base, SegSrcGlobal{&g, &b, &w, a});
      }
      continue;
    }
    // ---- states in point order (n <= PT here: every chunk's loads at once)
    constexpr int NCH = (PT + TB - 1) / TB;
    bool stv[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int pl = c * TB + lane;
      const bool in = pl < n;
      const uint8_t ic = in ? w.is_col[a + pl] : (uint8_t)0;
      const int32_t sv = in ? w.state[a + pl] : -1;
      stv[c] = ic && sv >= 0;
    }
    int ns = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const unsigned long long m = __ballot(stv[c]);
      if (stv[c]) S.sidx[ns + __popcll(m & lt)] = (int16_t)(c * TB + lane);
      ns += __popcll(m);
    }
    wave_sync();
    SEGP_MARK(1)
    // every state's loads at once, kept in registers for both passes below
    StateStep rs[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (c * TB + lane < ns) rs[c] = state_step(w, b, a, S, c * TB + lane, ns);
    // ---- per state: chain index, latest opener, slot counts (registers only);
    // the open edge's length of a state that leaves it is loaded here, so its
    // round trip overlaps the scans and the route-edge fetch below
    float elen[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) elen[c] = 0.0f;
    int c_chain = 0, c_open = -1, c_base = 0;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      if (c * TB >= ns) break;
      const int k = c * TB + lane;
      const bool valid = k < ns;
      int cs = 0, opener = -1, nem = 0;
      if (valid) {
        const StateStep& r = rs[c];
        cs = r.cs() ? 1 : 0;
        if (r.cs() || !r.same()) opener = k;
        if (!r.cs() && !r.same()) elen[c] = rec_len(edge_rec(g, r.ei));
        // the close of the open traversal (none from a node candidate), the
        // route's edges, the chain's final close (none at a node candidate)
        nem = (r.step() && !r.same() ? (cand_node(r.oi) ? 0 : 1) + r.plen : 0) +
              (r.last() && !r.cs() && !cand_node(r.oj) ? 1 : 0);
      }
      const int ch = c_chain + wave_incl_scan(cs, lane);
      int lo = wave_incl_max(opener, lane);
      lo = lo > c_open ? lo : c_open;
      const int inc = wave_incl_scan(nem, lane);
      if (valid) {
        S.chain[k] = (int16_t)(ch - 1);
        S.lopen[k] = (int16_t)lo;
        S.tbase[k] = c_base + inc - nem;
      }
      c_chain = __shfl(ch, 63, 64);
      c_open = __shfl(lo, 63, 64);
      c_base += __shfl(inc, 63, 64);
    }
    const int nt = c_base;
    wave_sync();
    SEGP_MARK(2)
    if (nt > TR) {
      if (lane == 0) {
        if (spill) spill[atomicAdd(spill_n, 1)] = t;
        else segments_trace<true>(g, w, o, t, n, base, SegSrcGlobal{&g, &b, &w, a});
      }
      wave_sync();
      continue;
    }
    // ---- the route edges: each state marks its route edges' slots with their
    // pool positions (every other slot -1), then the wave fetches every slot's
    // edge and length at once, a lane a slot -- one round trip for the
    // trace's path edges instead of two per edge along each state's path
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * TB + lane;
      if (k >= ns) continue;
      const StateStep& r = rs[c];
      int slot = S.tbase[k];
      if (r.step() && !r.same()) {
        if (!cand_node(r.oi)) S.t_edge[slot++] = -1;
        for (int i = 0; i < r.plen; ++i) S.t_edge[slot++] = -2 - (r.poff + i);
      }
      if (r.last() && !r.cs() && !cand_node(r.oj)) S.t_edge[slot] = -1;
    }
    wave_sync();
    SEGP_MARK(3)
    {
      constexpr int NTC = (TR + TB - 1) / TB;
      int32_t pe[NTC];
#pragma unroll
      for (int c = 0; c < NTC; ++c) {
        const int s = c * TB + lane;
        const int32_t v = s < nt ? S.t_edge[s] : -1;
        pe[c] = v <= -2 ? w.path_pool[-2 - v] : -1;
      }
#pragma unroll
      for (int c = 0; c < NTC; ++c) {
        const int s = c * TB + lane;
        if (pe[c] >= 0) {
          S.t_edge[s] = pe[c];
          S.t_off1[s] = rec_len(edge_rec(g, pe[c]));
        }
      }
    }
    wave_sync();
    SEGP_MARK(4)
    // ---- opener fields: a chain start's own, or the re-open on the new edge
    // at the end of the step's route (its length summed in route order)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * TB + lane;
      if (k >= ns) continue;
      const StateStep& r = rs[c];
      if (r.cs()) {
        S.o_t0[k] = r.tb;
        S.o_off0[k] = r.oj;
        S.o_sh0[k] = (int16_t)r.pl();
      } else if (!r.same()) {
        const float start = cand_node(r.oi) ? 0.0f : elen[c] - r.oi;  // src_start
        const int s0 = S.tbase[k] + (cand_node(r.oi) ? 0 : 1);
        float dd = 0.0f;
        for (int i = 0; i < r.plen; ++i) dd = dd + S.t_off1[s0 + i];
        const float x = start + dd;
        double t0;
        int sh;
        step_bound(b, w, a, r.lp(), r.pl(), r.rd, r.ta, r.tb, x, t0, sh);
        S.o_t0[k] = t0;
        S.o_off0[k] = 0.0f;
        S.o_sh0[k] = (int16_t)sh;
      }
    }
    wave_sync();
    SEGP_MARK(5)
    // ---- traversals, each state writing its own
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int k = c * TB + lane;
      if (k >= ns) continue;
      const StateStep& r = rs[c];
      int slot = S.tbase[k];
      const int16_t chk = S.chain[k];
      if (r.step() && !r.same()) {
        const float Rd = r.rd;
        const double ta = r.ta, tb = r.tb;
        const float el = elen[c];
        const float start = cand_node(r.oi) ? 0.0f : el - r.oi;  // src_start
        if (!cand_node(r.oi)) {
          const int jo = S.lopen[k - 1];
          S.t_edge[slot] = r.ei;
          S.t_off0[slot] = S.o_off0[jo];
          S.t_t0[slot] = S.o_t0[jo];
          S.t_sh0[slot] = S.o_sh0[jo];
          S.t_off1[slot] = el;
          double t1;
          int sh;
          step_bound(b, w, a, r.lp(), r.pl(), Rd, ta, tb, start, t1, sh);
          S.t_t1[slot] = t1;
          S.t_sh1[slot] = (int16_t)sh;
          S.t_chain[slot] = chk;
          ++slot;
        }
        float dd = 0.0f;
        for (int i = 0; i < r.plen; ++i) {
          const float len = S.t_off1[slot];  // (edge and length fetched above)
          const float xb = start + dd;
          dd = dd + len;
          const float xe = start + dd;
          S.t_off0[slot] = 0.0f;
          double tt;
          int sh;
          step_bound(b, w, a, r.lp(), r.pl(), Rd, ta, tb, xb, tt, sh);
          S.t_t0[slot] = tt;
          S.t_sh0[slot] = (int16_t)sh;
          step_bound(b, w, a, r.lp(), r.pl(), Rd, ta, tb, xe, tt, sh);
          S.t_t1[slot] = tt;
          S.t_sh1[slot] = (int16_t)sh;
          S.t_chain[slot] = chk;
          ++slot;
        }
      }
      if (r.last() && !r.cs() && !cand_node(r.oj)) {
        const int jo = S.lopen[k];
        // the traversal ends at the largest offset of its states (the opener
        // jo's and every stay after it: rule 4)
        float omax = r.oj;
        for (int kk = jo; kk < k; ++kk) {
          const float o2 = __int_as_float(w.chosen[a + S.sidx[kk]].y);
          omax = o2 > omax ? o2 : omax;
        }
        S.t_edge[slot] = r.ej;
        S.t_off0[slot] = S.o_off0[jo];
        S.t_t0[slot] = S.o_t0[jo];
        S.t_sh0[slot] = S.o_sh0[jo];
        S.t_off1[slot] = omax;
        S.t_t1[slot] = r.tb;
        S.t_sh1[slot] = (int16_t)r.pl();
        S.t_chain[slot] = chk;
      }
    }
    wave_sync();
    SEGP_MARK(6)
    // ---- groups (OSMLR segments) and way ids
    // (one 16-byte edge record per traversal; ways compared by number, the id
    // looked up only for the way ids written)
    int c_seg = 0, c_way = 0;
    int32_t p_seg = 0, p_pos = 0, p_ch = -1, p_way = -1;
    uint32_t p_fl = 0;
    for (int k0 = 0; k0 < nt; k0 += TB) {
      const int k = k0 + lane;
      const bool valid = k < nt;
      int32_t seg = -1, pos = 0, ch = -2, way = -1;
      uint32_t fl = 0;
      float elk = 0.0f;
      if (valid) {
        const uint4 er = edge_rec(g, S.t_edge[k]);
        elk = rec_len(er);
        seg = rec_seg(er);
        pos = rec_pos(er);
        fl = rec_flags(er);
        way = (int32_t)er.w;
        ch = S.t_chain[k];
      }
      int32_t qs = __shfl_up(seg, 1, 64), qp = __shfl_up(pos, 1, 64), qc = __shfl_up(ch, 1, 64);
      uint32_t qf = __shfl_up(fl, 1, 64);
      int32_t qw = __shfl_up(way, 1, 64);
      if (lane == 0) {
        qs = p_seg;
        qp = p_pos;
        qc = p_ch;
        qf = p_fl;
        qw = p_way;
      }
      bool join = false;
      if (valid && qc == ch) {
        if (seg >= 0) join = qs == seg && pos == qp + 1;
        else join = qs < 0 && ((fl ^ qf) & SegEmitter<true>::OTM_EDGE_INTERNAL_D) == 0;
      }
      const bool start = valid && !join;
      const bool wemit = valid && (start || way != qw);
      const unsigned long long ms = __ballot(start), mw = __ballot(wemit);
      const int gi = c_seg + __popcll(ms & lt) + (start ? 0 : -1);  // this traversal's group
      const int wi = c_way + __popcll(mw & lt);
      if (valid) {
        // what the record pass needs of this traversal's edge, kept in the two
        // slots it no longer reads (its edge and chain): the segment index, and
        // the flags with whether the traversal ends at the edge's end -- no
        // second and third gather of the edge record there
        S.t_edge[k] = seg;
        S.t_chain[k] = (int16_t)(fl | (S.t_off1[k] == elk ? 0x100u : 0u));
      }
      if (wemit) o.way_ids[base + wi] = g.way_tab[way];
      if (start) {
        S.g_first[gi] = (int16_t)k;
        S.g_w0[gi] = (int16_t)wi;
        if (gi > 0) S.g_last[gi - 1] = (int16_t)(k - 1);
      }
      c_seg += __popcll(ms);
      c_way += __popcll(mw);
      p_seg = __shfl(seg, 63, 64);
      p_pos = __shfl(pos, 63, 64);
      p_ch = __shfl(ch, 63, 64);
      p_fl = __shfl(fl, 63, 64);
      p_way = __shfl(way, 63, 64);
    }
    if (lane == 0 && c_seg > 0) {
      S.g_last[c_seg - 1] = (int16_t)(nt - 1);
      S.g_w0[c_seg] = (int16_t)c_way;
    }
    wave_sync();
    SEGP_MARK(7)
    // ---- one record per group (SegEmitter::flush)
    for (int s0 = 0; s0 < c_seg; s0 += TB) {
      const int si = s0 + lane;
      if (si >= c_seg) continue;
      const int kf = S.g_first[si], kl = S.g_last[si];
      EAttr fa;
      fa.seg = S.t_edge[kf];
      fa.flags = (uint32_t)S.t_chain[kf] & 0xFFu;
      fa.gid = fa.seg >= 0 ? g.g_id[fa.seg] : 0ull;
      fa.glen = fa.seg >= 0 ? g.g_len[fa.seg] : 0.0f;
      const uint32_t lfl = (uint32_t)S.t_chain[kl] & 0xFFu;
      const bool lfull = ((uint32_t)S.t_chain[kl] & 0x100u) != 0u;  // t_off1[kl] == the edge's length
      otm_segment sr;
      const int32_t sg = fa.seg;
      bool sv, ev;
      sr.flags = 0u;
      if (sg >= 0) {
        sv = S.t_off0[kf] == 0.0f && (fa.flags & SegEmitter<true>::OTM_EDGE_SEG_BEGIN_D);
        ev = lfull && (lfl & SegEmitter<true>::OTM_EDGE_SEG_END_D);
        sr.segment_id = (int64_t)fa.gid;
        sr.length = (sv && ev) ? (int32_t)floor((double)fa.glen + 0.5) : -1;
      } else {
        sv = S.t_off0[kf] == 0.0f;
        ev = lfull;
        sr.segment_id = -1;
        sr.length = -1;
        if (fa.flags & SegEmitter<true>::OTM_EDGE_INTERNAL_D) sr.flags |= OTM_SEG_INTERNAL;
      }
      sr.start_time = 0.0;
      sr.end_time = 0.0;
      if (sv) {
        sr.flags |= OTM_SEG_START_VALID;
        sr.start_time = S.t_t0[kf];
      }
      if (ev) {
        sr.flags |= OTM_SEG_END_VALID;
        sr.end_time = S.t_t1[kl];
      }
      sr.queue_length = 0;
      sr.begin_shape_index = S.t_sh0[kf];
      sr.end_shape_index = S.t_sh1[kl];
      sr.way_off = base + S.g_w0[si];
      sr.way_cnt = S.g_w0[si + 1] - S.g_w0[si];
      sr.pad = 0u;
      ((otm_segment*)o.segments)[base + si] = sr;
      o.seg_gidx[base + si] = sg;
    }
    if (lane == 0) {
      o.seg_cnt[t] = c_seg;
      o.way_cnt[t] = c_way;
    }
    wave_sync();
    SEGP_MARK(8)
  }
  SEGP_END
}

// ============================================================== K8 report
__device__ __forceinline__ bool in_lv(const int64_t* lv, int n, int64_t x) {
  for (int k = 0; k < n; ++k)
    if (lv[k] == x) return true;
  return false;
}

#ifndef OTM_REPORT_WAVES
#define OTM_REPORT_WAVES 1
#endif
// report() launch: 1 = a wave per trace over an LDS copy of its segments
// (k_report_wave), 0 = a thread per trace (k_report), 2 = the wave form up to
// REPW_MAX_TRACES traces (two rounds of 8 waves per SIMD), else the thread
// form.  Measured: config 2 (10k traces) 0.0445 -> 0.0392 ms with the wave
// form; config 4 (100k traces) 0.106 -> 0.290 ms, so it is not used there.
#ifndef OTM_REPORT_FORM
#define OTM_REPORT_FORM 2
#endif
constexpr int32_t REPW_MAX_TRACES = 2 * 8 * 4 * 256;
// report() (py/reporter_service.py:110-215) over one trace's segments, one
// thread per trace.  Segment times are Python values: a segment without
// START_VALID / END_VALID carries the int -1 (what the matcher emits), one
// with it the stored double, an int literal when START_INT / END_INT is set
// (segments handed in by otm_report_segments_device).  A report's t0 / t1
// inherit that int-ness for the JSON writer, and a zero duration raises
// Python's int or float ZeroDivisionError.  The histogram is added in a
// second pass, only for a trace that ends without an error: the reference
// posts nothing for a trace whose report() raised.
// The serial part of report() for trace t over its segments S (global memory,
// or the wave's LDS copy in k_report_wave): the trace result r and the reports
// written to REP, each carrying its reported segment's index in `pad` for the
// histogram pass (which clears it).  Returns the report count; an error trace
// (matcher error or ZeroDivisionError) gets code 500 and no reports.
__device__ int report_walk(int32_t t, const DevBatch& b, const DevReportCfg& rc, const DevWork& w,
                           const otm_segment* S, otm_trace_result& r, otm_report_rec* REP) {
  r.code = 200;
  r.rep_cnt = 0;
  r.shape_used = -1;
  r.successful_count = r.unreported_count = r.discontinuities = r.invalid_speeds = r.unassociated = 0;
  r.successful_length = r.unreported_length = -1;
  if (r.error_kind != 0) {
    r.code = 500;
    return 0;
  }
  const double end_time = b.time[b.trace_off[t + 1] - 1];
  auto ST = [&](const otm_segment& s) { return (s.flags & OTM_SEG_START_VALID) ? s.start_time : -1.0; };
  auto ET = [&](const otm_segment& s) { return (s.flags & OTM_SEG_END_VALID) ? s.end_time : -1.0; };
  auto ST_INT = [&](const otm_segment& s) {
    return !(s.flags & OTM_SEG_START_VALID) || (s.flags & OTM_SEG_START_INT) != 0u;
  };
  auto ET_INT = [&](const otm_segment& s) { return !(s.flags & OTM_SEG_END_VALID) || (s.flags & OTM_SEG_END_INT) != 0u; };
  int last_idx = r.seg_cnt - 1;
  while (last_idx >= 0 && end_time - ST(S[last_idx]) < rc.threshold_sec) --last_idx;
  r.shape_used = last_idx >= 0 ? S[last_idx].begin_shape_index : -1;
  bool have = false, first = true;
  int prior = -1;
  int64_t prior_level = -1;
  int nrep = 0;
  int zerodiv = 0;
  for (int idx = 0; idx <= last_idx; ++idx) {
    const otm_segment& s = S[idx];
    const bool internal = (s.flags & OTM_SEG_INTERNAL) != 0;
    if (idx != 0 && ST(s) == -1.0 && ET(S[idx - 1]) == -1.0) r.discontinuities++;
    const int64_t level = s.segment_id >= 0 ? (s.segment_id & 7) : -1;
    if (have && S[prior].segment_id >= 0 && S[prior].length > 0 && !internal) {
      const otm_segment& ps = S[prior];
      if (in_lv(rc.report_levels, rc.n_report, prior_level)) {
        const bool trans = in_lv(rc.transition_levels, rc.n_transition, level);
        const double t0 = ST(ps);
        const double t1 = trans ? ST(s) : ET(ps);
        const bool t0_int = ST_INT(ps);
        const bool t1_int = trans ? ST_INT(s) : ET_INT(ps);
        const double den = t1 - t0;
        if (den == 0.0) {
          // int / int raises "division by zero", anything else "float division by zero"
          zerodiv = t0_int && t1_int ? OTM_TERR_ZERODIV_INT : OTM_TERR_ZERODIV;
          break;
        }
        const double speed = ((double)ps.length / den) * 3.6;
        if (speed < 200.0) {
          otm_report_rec rep;
          rep.id = ps.segment_id;
          rep.next_id = (trans && s.segment_id >= 0) ? s.segment_id : -1;
          rep.t0 = t0;
          rep.t1 = t1;
          rep.flags = (t1_int ? OTM_REP_T1_INT : 0u) | (t0_int ? OTM_REP_T0_INT : 0u);
          rep.length = ps.length;
          rep.queue_length = ps.queue_length;
          rep.pad = (uint32_t)prior;  // the reported segment, for the histogram pass (cleared there)
          REP[nrep++] = rep;
          r.successful_count++;
          r.successful_length = ps.length;
        } else {
          r.invalid_speeds++;
        }
      } else {
        r.unreported_count++;
        r.unreported_length = ps.length;
      }
    }
    if (!(internal && !first)) {
      prior = idx;
      prior_level = level;
      have = true;
    }
    first = false;
    if (s.segment_id < 0 && !internal) r.unassociated++;
  }
  if (zerodiv) {
    r.code = 500;
    r.error_kind = zerodiv;
    r.shape_used = -1;
    r.successful_count = r.unreported_count = r.discontinuities = r.invalid_speeds = r.unassociated = 0;
    r.successful_length = r.unreported_length = -1;
    return 0;
  }
  return nrep;
}

// The histogram pass over one report: its speed bin and speed sum, for a
// trace that ended without an error (the reference posts nothing for a trace
// whose report() raised); a t1 that is the int -1 of a partial next segment
// gives no speed.  Clears the report's `pad`.
__device__ __forceinline__ void report_hist(const DevOut& o, int32_t seg_off, otm_report_rec& rep) {
  const int32_t ps = (int32_t)rep.pad;
  rep.pad = 0u;
  if (!o.hist) return;
  const double speed = ((double)rep.length / (rep.t1 - rep.t0)) * 3.6;
  const bool t1_minus1 = (rep.flags & OTM_REP_T1_INT) && rep.t1 == -1.0;
  const int32_t gi = o.seg_gidx[seg_off + ps];
  if (t1_minus1 || !(speed >= 0.0) || gi < 0) return;
  int bin = (int)(speed / (double)o.bin_kph);
  bin = bin < 0 ? 0 : (bin >= o.nbins ? o.nbins - 1 : bin);
  atomicAdd(&o.hist[(size_t)gi * o.nbins + bin], 1u);
  if (o.speed_sum) {
    // fixed point (1/1000 km/h) so the sums are exact and order-independent
    atomicAdd(&o.speed_sum[gi], (unsigned long long)(speed * 1000.0 + 0.5));
  }
}

// report() (py/reporter_service.py:110-215), one thread per trace (the
// OTM_REPORT_FORM 0 launch).
__global__ __launch_bounds__(256, OTM_REPORT_WAVES) void k_report(DevBatch b, DevReportCfg rc, DevWork w, DevOut o, int32_t n_seg_total) {
  if (*w.abort) return;  // a capacity was exceeded: the host redoes the batch
  const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= b.n_traces) return;
  otm_trace_result r;
  r.error_kind = w.trace_err[t];
  r.seg_off = (int32_t)o.seg_base[t];
  r.seg_cnt = o.seg_cnt[t];
  r.rep_off = r.seg_off;
  otm_report_rec* REP = (otm_report_rec*)o.reports + r.rep_off;
  const int nrep = report_walk(t, b, rc, w, (const otm_segment*)o.segments + r.seg_off, r, REP);
  for (int k = 0; k < nrep; ++k) report_hist(o, r.seg_off, REP[k]);
  r.rep_cnt = nrep;
  if (w.ctr && r.code == 200) {
    cadd(&w.ctr->segments_out, (unsigned long long)r.seg_cnt);
    cadd(&w.ctr->reports_out, (unsigned long long)nrep);
  }
  ((otm_trace_result*)o.traces)[t] = r;
  o.rep_cnt[t] = r.rep_cnt;
}

// report(), one wavefront per trace: the lanes copy the trace's segments into
// LDS with coalesced loads, lane 0 walks them there (the walk is serial: each
// step's global round trip becomes an LDS read), and the lanes run the
// histogram pass over the reports in parallel.  A trace with more segments
// than REPW_CAP is walked out of global memory.
constexpr int REPW_CAP = 64;
__global__ __launch_bounds__(TB) void k_report_wave(DevBatch b, DevReportCfg rc, DevWork w, DevOut o, int32_t n_seg_total) {
  if (*w.abort) return;  // a capacity was exceeded: the host redoes the batch
  __shared__ unsigned long long sSeg[REPW_CAP * sizeof(otm_segment) / 8];
  __shared__ int32_t sN;
  static_assert(sizeof(otm_segment) % 8 == 0, "segment words");
  constexpr int SW = (int)(sizeof(otm_segment) / 8);  // 8-byte words per segment
  const int lane = threadIdx.x;
  for (int32_t t = blockIdx.x; t < b.n_traces; t += gridDim.x) {
    otm_trace_result r;
    r.error_kind = w.trace_err[t];
    r.seg_off = (int32_t)o.seg_base[t];
    r.seg_cnt = o.seg_cnt[t];
    r.rep_off = r.seg_off;
    const otm_segment* G = (const otm_segment*)o.segments + r.seg_off;
    otm_report_rec* REP = (otm_report_rec*)o.reports + r.rep_off;
    const bool fits = r.seg_cnt <= REPW_CAP;
    if (fits && r.error_kind == 0) {
      const unsigned long long* gw = (const unsigned long long*)G;
      for (int k = lane; k < r.seg_cnt * SW; k += TB) sSeg[k] = gw[k];
    }
    __syncthreads();
    if (lane == 0) {
      const int nrep = report_walk(t, b, rc, w, fits ? (const otm_segment*)sSeg : G, r, REP);
      r.rep_cnt = nrep;
      sN = nrep;
      if (w.ctr && r.code == 200) {
        cadd(&w.ctr->segments_out, (unsigned long long)r.seg_cnt);
        cadd(&w.ctr->reports_out, (unsigned long long)nrep);
      }
      ((otm_trace_result*)o.traces)[t] = r;
      o.rep_cnt[t] = nrep;
      __threadfence_block();  // the reports, for the other lanes' histogram pass
    }
    __syncthreads();
    const int nrep = sN;
    for (int k = lane; k < nrep; k += TB) report_hist(o, r.seg_off, REP[k]);
    __syncthreads();
  }
}

// ============================================================== segment bound / compaction
// K7a, interpolated points (DESIGN.md §3 rule 7, oracle interp_pos): a point
// k between the two states q < k < p of a step that leaves its edge is placed
// on the step's route -- on each route piece (the rest of q's edge, the path's
// edges, p's edge up to p) its best projection onto the piece's edge,
// admissible inside the piece, costed sqdist / (2 sigma_z^2) + |pos - gc(q, k)|
// / beta; the cheapest wins (-1: none).  One thread per interpolated point
// (its step from prevc / nextc); the monotone filter (a point behind the
// step's running maximum is no anchor) is applied where the anchors are read
// (step_bound).
struct RoutePiece {
  int32_t edge;
  float o0, o1, xs;
};
__device__ float interp_pos(const DevGraph& g, const DevBatch& b, const DevParams& P, const DevWork& w, int64_t q,
                            int64_t p, int64_t k) {
  const int2 ci = w.chosen[q], cj = w.chosen[p];
  const int32_t ei = ci.x, ej = cj.x;
  const float oi = __int_as_float(ci.y), oj = __int_as_float(cj.y);
  const int32_t poff = w.path_off[p], plen = w.path_len[p];
  const bool has0 = !cand_node(oi);
  const int npc = (has0 ? 1 : 0) + plen + (cand_node(oj) ? 0 : 1);
  const float start = src_start(g, ei, oi);
  const float ds = (2.0f * P.sigma_z) * P.sigma_z;
  const float lat = b.lat[k], lon = b.lon[k];
  const float ls = MPD_F * cos_deg(lat);
  const float gcd = gc_dist(b.lat[q], b.lon[q], lat, lon);
  float best = INFINITY, bpos = -1.0f, dd = 0.0f;
  for (int m = 0; m < npc; ++m) {
    RoutePiece pc;
    const int pk = m - (has0 ? 1 : 0);
    if (has0 && m == 0) {
      pc = RoutePiece{ei, oi, g.e_len[ei], 0.0f};
    } else if (pk < plen) {
      const int32_t e = w.path_pool[poff + pk];
      const float len = g.e_len[e];
      pc = RoutePiece{e, 0.0f, len, start + dd};
      dd = dd + len;
    } else {
      pc = RoutePiece{ej, 0.0f, oj, start + dd};
    }
    const int32_t s0 = g.e_shape_off[pc.edge], nsh = g.e_shape_off[pc.edge + 1] - s0 - 1;
    float bsq = INFINITY, boff = 0.0f;
    for (int sg = 0; sg < nsh; ++sg) {
      float sqd, off;
      project(g, pc.edge, sg, lat, lon, ls, sqd, off);
      if (sqd < bsq) {
        bsq = sqd;
        boff = off;
      }
    }
    if (!(boff >= pc.o0 && boff <= pc.o1)) continue;
    const float pos = pc.xs + (boff - pc.o0);
    const float cost = bsq / ds + fabsf(pos - gcd) / P.beta;
    if (cost < best) {
      best = cost;
      bpos = pos;
    }
  }
  return bpos;
}

// Traversals a matched point can add: the close of the open traversal, its
// route's path edges, the re-open (+ the chain's final close): <= 2 + path.
// Summed per trace into tb[t] (scanned over traces into DevOut::seg_base): a
// wave's points are runs of whole traces, so a segmented suffix sum over the
// wave leaves each run's total on its first lane, which adds it with one
// atomic -- no per-point bound array, no point-length scan (round 6).  An
// interpolated point's thread places it instead (K7a).  Measured against a
// wave per trace (coalesced runs, no atomics): 0.027 vs 0.032 ms on config 2,
// 0.067 vs 0.064 on config 4; and against each trace's region taken from one
// cursor by k_segments (no bound pass at all): k_segments 0.047 -> 0.142 ms on
// config 2, the one address's atomics serialised (profiles/r06/k7/).
__global__ __launch_bounds__(256) void k_seg_bound(DevGraph g, DevBatch b, DevParams P, DevWork w, int64_t* tb) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // spill snapshot C: steps per route tier (kept for the status read)
  if (OTM_FOLD_BOOKKEEPING && k == b.n_points) fold_snap(w, 2, false);
  if (*w.abort) return;  // a capacity was exceeded: the host redoes the batch
  const int lane = threadIdx.x & 63;
  int64_t v = 0;
  int32_t t = -1;
  if (k < b.n_points) {
    t = w.pt_trace[k];
    if (w.is_col[k]) {
      if (w.state[k] >= 0) {
        const int32_t pl = w.path_len[k];
        v = 2 + (pl > 0 ? pl : 0);
      }
    } else {
      // the step q -> p around this point: linked, matched, leaving q's edge
      const int32_t q = w.prevc[k];
      const int32_t p = q >= 0 ? w.nextc[q] : -1;
      if (p >= 0 && w.col_prev[p] == q && !w.chain_start[p] && w.state[p] >= 0 && w.path_len[p] >= 0 &&
          w.trace_err[t] == 0) {
        const int2 ci = w.chosen[q], cj = w.chosen[p];
        if (!same_edge_step(ci.x, __int_as_float(ci.y), cj.x, __int_as_float(cj.y)))
          w.ipos[k] = interp_pos(g, b, P, w, q, p, k);
      }
    }
  }
  // segmented suffix sum over the wave's runs of equal t (lanes past the
  // batch's end have t = -1, a run of their own)
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int64_t vn = __shfl_down(v, d, 64);
    const int32_t tn = __shfl_down(t, d, 64);
    if (lane + d < 64 && tn == t) v += vn;
  }
  const int32_t tp = __shfl_up(t, 1, 64);
  if (t >= 0 && (lane == 0 || tp != t) && v != 0) atomicAdd((unsigned long long*)&tb[t], (unsigned long long)v);
}

// One wavefront per trace: copy its segments (way offsets rebased), way ids
// and reports from the trace's region to the dense arrays, and its result
// record with the dense offsets to `to` (the regions' records stay as they
// are, so fetching a batch twice gives the same arrays).
__global__ __launch_bounds__(TB) void k_compact(int32_t n_traces, DevOut o, const int32_t* seg_off, const int32_t* way_off,
                                                const int32_t* rep_off, otm_segment* so, int64_t* wo,
                                                otm_report_rec* ro, otm_trace_result* to) {
  const int lane = threadIdx.x;
  const otm_trace_result* TR = (const otm_trace_result*)o.traces;
  const otm_segment* SI = (const otm_segment*)o.segments;
  const otm_report_rec* RI = (const otm_report_rec*)o.reports;
  for (int32_t t = blockIdx.x; t < n_traces; t += gridDim.x) {
    const int32_t base = TR[t].seg_off;  // the region start k_report recorded
    const int32_t ns = o.seg_cnt[t], nw = o.way_cnt[t], nr = o.rep_cnt[t];
    const int32_t ds = seg_off[t], dw = way_off[t], dr = rep_off[t];
    for (int k = lane; k < ns; k += TB) {
      otm_segment x = SI[base + k];
      x.way_off = x.way_off - base + dw;
      so[ds + k] = x;
    }
    for (int k = lane; k < nw; k += TB) wo[dw + k] = o.way_ids[base + k];
    for (int k = lane; k < nr; k += TB) ro[dr + k] = RI[base + k];
    if (lane == 0) {
      otm_trace_result x = TR[t];
      x.seg_off = ds;
      x.rep_off = dr;
      to[t] = x;
    }
  }
}

// One block of 1024 threads: the three count arrays' exclusive scans, totals
// at o*[n].  (Round 4's form summed a contiguous chunk per thread: strided,
// uncoalesced loads, ~90 us per 10k traces with other batches in flight.)
__global__ __launch_bounds__(1024) void k_fetch_scan(int32_t n, const int32_t* c0, const int32_t* c1,
                                                     const int32_t* c2, int32_t* o0, int32_t* o1, int32_t* o2) {
  // tiles of 1024 consecutive counts (coalesced loads and stores), each tile
  // scanned in the block and added to the running carry
  __shared__ int32_t ws[3][16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int carry0 = 0, carry1 = 0, carry2 = 0;
  for (int base = 0; base < n; base += 1024) {
    const int i = base + t;
    const int s0 = i < n ? c0[i] : 0, s1 = i < n ? c1[i] : 0, s2 = i < n ? c2[i] : 0;
    // inclusive scans within the wave, then across the 16 waves
    int i0 = s0, i1 = s1, i2 = s2;
    for (int o = 1; o < 64; o <<= 1) {
      const int x0 = __shfl_up(i0, o, 64), x1 = __shfl_up(i1, o, 64), x2 = __shfl_up(i2, o, 64);
      if (lane >= o) {
        i0 += x0;
        i1 += x1;
        i2 += x2;
      }
    }
    if (lane == 63) {
      ws[0][wv] = i0;
      ws[1][wv] = i1;
      ws[2][wv] = i2;
    }
    __syncthreads();
    int b0 = 0, b1 = 0, b2 = 0, z0 = 0, z1 = 0, z2 = 0;
    for (int k = 0; k < 16; ++k) {
      const int w0 = ws[0][k], w1 = ws[1][k], w2 = ws[2][k];
      if (k < wv) {
        b0 += w0;
        b1 += w1;
        b2 += w2;
      }
      z0 += w0;
      z1 += w1;
      z2 += w2;
    }
    if (i < n) {
      o0[i] = carry0 + b0 + i0 - s0;
      o1[i] = carry1 + b1 + i1 - s1;
      o2[i] = carry2 + b2 + i2 - s2;
    }
    carry0 += z0;
    carry1 += z1;
    carry2 += z2;
    __syncthreads();  // (ws is rewritten by the next tile)
  }
  if (t == 0) {
    o0[n] = carry0;
    o1[n] = carry1;
    o2[n] = carry2;
  }
}

int grid_for(int64_t n, int per_block, int cap) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (int)(g > cap ? cap : g);
}

// ============================================================== launchers
constexpr int WAVE_GRID_CAP = 256 * 64;  // grid-stride cap for wave kernels
constexpr int TRANS_GRID_CAP = 65536;  // k_trans_sub waves (one per column, grid-striding beyond)

}  // namespace

void launch_fetch_scan(int32_t n, const int32_t* c0, const int32_t* c1, const int32_t* c2, int32_t* o0, int32_t* o1,
                       int32_t* o2, hipStream_t s) {
  hipLaunchKernelGGL(k_fetch_scan, dim3(1), dim3(1024), 0, s, n, c0, c1, c2, o0, o1, o2);
}


const char* const kKernelNames[KN_COUNT] = {
    "k_columns",       "spatial_order",  "k_cand_lane",    "k_candidates",     "k_links",         "scan_trans_off",  "k_trans_sub",
    "k_trans_wide",    "k_transitions",  "k_transitions_big", "k_viterbi",      "k_route_index",
    "k_route",         "k_route_big",    "k_seg_bound",      "scan_seg_bound",  "k_segments",       "k_report"};

namespace {
// The spill tiers run on lists the previous tier filled on the device; they
// read the list length themselves (fixed grids, no host round trip) and exit
// at once when the list is empty.
constexpr int SPILL_GRID = 4096;
#ifndef OTM_WIDE_GRID
#define OTM_WIDE_GRID 8192
#endif
// k_trans_sub's wide-column pass (grid-strides over its list): 8192 waves
// (eight per SIMD) rather than 2048: config 2 0.035 -> 0.030 ms (round 6)
constexpr int WIDE_GRID = OTM_WIDE_GRID;
}  // namespace

#define TIMED(k, launch) \
  do {                   \
    mk.begin(k, s);      \
    launch;              \
    mk.end(k, s);        \
  } while (0)

void launch_columns(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                    const Marks& mk) {
  if (w.ord.tile_cnt) (void)hipMemsetAsync(w.ord.tile_cnt, 0, ORDER_TILES * 4, s);
  TIMED(KN_COLUMNS, hipLaunchKernelGGL(k_columns, dim3(grid_for(b.n_traces, 1, WAVE_GRID_CAP)), dim3(TB), 0, s, g,
                                       b, p, w));
}
// grid for a kernel over the spatial order: a multiple of ORDER_GROUPS, with
// 25 % headroom per group over an even split
static int order_grid(int64_t n, int per_block, int cap) {
  const int64_t per_group = (n + ORDER_GROUPS - 1) / ORDER_GROUPS;
  int64_t gb = (per_group + per_group / 4 + per_block - 1) / per_block;
  if (gb < 1) gb = 1;
  int64_t gtot = gb * ORDER_GROUPS;
  if (gtot > cap) gtot = cap / ORDER_GROUPS * ORDER_GROUPS;
  return (int)gtot;
}

void launch_order(const DevBatch& b, DevWork& w, hipStream_t s, const Marks& mk) {
  // (the tile counts were made by K1)
  mk.begin(KN_ORDER, s);
  hipLaunchKernelGGL(k_order_plan, dim3(1), dim3(1024), 0, s, w.ord.tile_cnt, w.ord.cursor, w.ord.grp);
  hipLaunchKernelGGL(k_order_scatter, dim3(grid_for(b.n_points, 256, 8192)), dim3(256), 0, s, b, w, w.ord.tile,
                     w.ord.cursor, w.ord.item);
  mk.end(KN_ORDER, s);
}

void launch_candidates(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                       const Marks& mk, int from) {
  // (the work counters in their own instance: their registers cost the
  // uncounted one entries in flight)
  if (from < RESUME_CAND_BIG) {
    if (w.ctr)
      TIMED(KN_CAND_LANE, hipLaunchKernelGGL(k_cand_lane<true>, dim3(order_grid(b.n_points, CAND_TB, 1 << 30)),
                                             dim3(CAND_TB), 0, s, g, b, p, w));
    else
      TIMED(KN_CAND_LANE, hipLaunchKernelGGL(k_cand_lane<false>, dim3(order_grid(b.n_points, CAND_TB, 1 << 30)),
                                             dim3(CAND_TB), 0, s, g, b, p, w));
  }
  mk.begin(KN_CAND_WAVE, s);
  if (from < RESUME_CAND_BIG) hipLaunchKernelGGL(k_candidates<false>, dim3(4096), dim3(TB), 0, s, g, b, p, w);
  hipLaunchKernelGGL(k_candidates<true>, dim3(CAND_BIG_SLOTS), dim3(TB), 0, s, g, b, p, w);
  mk.end(KN_CAND_WAVE, s);
}
void launch_links(const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s, const Marks& mk) {
  TIMED(KN_LINKS, hipLaunchKernelGGL(k_links, dim3(grid_for(b.n_points + 1, 256, 1 << 30)), dim3(256), 0, s, b, p,
                                     w));
}
void launch_batch_init(int32_t* counters, int32_t* abort, hipStream_t s) {
  hipLaunchKernelGGL(k_batch_init, dim3(1), dim3(64), 0, s, counters, abort);
}
void launch_snap(int32_t* counters, int32_t* snap, bool reset, hipStream_t s) {
  hipLaunchKernelGGL(k_snap, dim3(1), dim3(64), 0, s, counters, snap, reset ? 1 : 0);
}
// The compact host batch (otm_match_compact) widened on the device: a wave per
// trace, its points' time = base + delta (whole seconds, exact in a double)
// and accuracy as float -- the arrays every stage reads.
__global__ __launch_bounds__(256) void k_expand_compact(const int64_t* trace_off, const int64_t* tbase,
                                                        const int32_t* dt, const int16_t* acc16, double* time,
                                                        float* acc, int32_t n_traces) {
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int64_t t = (int64_t)blockIdx.x * 4 + wv; t < n_traces; t += (int64_t)gridDim.x * 4) {
    const int64_t a = trace_off[t], e = trace_off[t + 1], base = tbase[t];
    for (int64_t i = a + lane; i < e; i += 64) {
      time[i] = (double)(base + (int64_t)dt[i]);
      acc[i] = (float)acc16[i];
    }
  }
}
void launch_expand_compact(const int64_t* trace_off, const int64_t* tbase, const int32_t* dt, const int16_t* acc16,
                           double* time, float* acc, int32_t n_traces, hipStream_t s) {
  if (n_traces <= 0) return;
  hipLaunchKernelGGL(k_expand_compact, dim3(grid_for(((int64_t)n_traces + 3) / 4, 1, 1 << 20)), dim3(256), 0, s,
                     trace_off, tbase, dt, acc16, time, acc, n_traces);
}
void launch_status(const int32_t* abort, const int64_t* ttotal, const int32_t* counters, BatchStatus* out,
                   hipStream_t s) {
  hipLaunchKernelGGL(k_status, dim3(1), dim3(64), 0, s, abort, ttotal, counters, out);
}
bool fold_bookkeeping() { return OTM_FOLD_BOOKKEEPING != 0; }
void launch_cap_check(const DevBatch& b, DevWork& w, hipStream_t s) {
  hipLaunchKernelGGL(k_cap_check, dim3(1), dim3(1), 0, s, b, w);
}
void launch_transitions(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                        const Marks& mk, int sub, int from) {
  if (from >= RESUME_TRANS_HUGE) {
    // the tiers below the huge one kept their matrices: the huge tier alone
    mk.begin(KN_TRANS_GLOBAL, s);
    hipLaunchKernelGGL(k_transitions<2>, dim3(HUGE_SLOTS), dim3(TB), 0, s, g, b, p, w);
    mk.end(KN_TRANS_GLOBAL, s);
    return;
  }
  // many more waves than fit at once (each column is a few dependent
  // round trips): measured 0.78 ms at 16K waves, 0.67 ms at 64K; a grid of
  // one resident round was slowest (0.92 ms, partial rounds at 7 waves/SIMD)
  // sub: lanes per column (engine trans_lanes)
  const int per = TB / sub;  // columns per wave step
  const int grid = order_grid((b.n_points + per - 1) / per, 1, TRANS_GRID_CAP);
  if (sub == 8) {
    // 8 lanes per column over the columns of <= OTM_TRANS_KC8 candidates a
    // side, then 16 lanes over the wide rest (a list filled on the device)
    TIMED(KN_TRANS_INDEX, hipLaunchKernelGGL((k_trans_sub<8, false>), dim3(grid), dim3(TB), 0, s, g, b, p, w));
    TIMED(KN_TRANS_WIDE, hipLaunchKernelGGL((k_trans_sub<16, true>), dim3(WIDE_GRID), dim3(TB), 0, s, g, b, p, w));
  } else {
    TIMED(KN_TRANS_INDEX, hipLaunchKernelGGL((k_trans_sub<16, false>), dim3(grid), dim3(TB), 0, s, g, b, p, w));
    mk.begin(KN_TRANS_WIDE, s);
    mk.end(KN_TRANS_WIDE, s);
  }
  TIMED(KN_TRANS_WAVE, hipLaunchKernelGGL(k_transitions<0>, dim3(SPILL_GRID), dim3(TB), 0, s, g, b, p, w));
  mk.begin(KN_TRANS_GLOBAL, s);
  hipLaunchKernelGGL(k_transitions<1>, dim3(BIG_SLOTS), dim3(TB), 0, s, g, b, p, w);
  hipLaunchKernelGGL(k_transitions<2>, dim3(HUGE_SLOTS), dim3(TB), 0, s, g, b, p, w);
  mk.end(KN_TRANS_GLOBAL, s);
}
void launch_viterbi(const DevBatch& b, DevWork& w, hipStream_t s, const Marks& mk) {
  // the form: OTM_VIT_FORM (8, 16 or 64) for the tests; by default the
  // grouped forms from 32,768 traces up, the wave form below:
  // a small batch's waves all fit the GPU at once, so its time is one wave's
  // (~100 steps of a latency-bound chain either way), while a large batch's
  // is wave rounds, which 8 traces per wave divide (round-4 A/B,
  // profiles/r04_ab/vit_form_*: config 2 0.157 ms wave form vs 0.50 grouped,
  // config 4 1.13 vs 0.73)
  // (read per batch: tests switch them)
  const char* fe = std::getenv("OTM_VIT_FORM");
  const int forced = fe ? std::atoi(fe) : 0;
  constexpr int gmin = 32768;
  const int form = forced ? forced : (b.n_traces >= gmin ? 8 : 64);
  if (form == 64) {
    TIMED(KN_VITERBI, hipLaunchKernelGGL(k_viterbi, dim3(grid_for(b.n_traces, 1, WAVE_GRID_CAP)), dim3(TB), 0, s, b,
                                         w, (const int32_t*)nullptr, (const int32_t*)nullptr, 1));
    return;
  }
  // 8 lanes per trace over every trace; what it cannot take (a column wider
  // than 8 candidates, more than VG_PTS points) to 16 lanes per trace; what
  // that cannot take to the wave-per-trace form.  Lists: overflow_list0 (count
  // counters_i32[20]) and overflow_list2 ([26]), both free between the
  // transition and route stages; the counts are zeroed by K1.
  int32_t* l8 = w.overflow_list0;
  int32_t* n8 = w.counters_i32 + 20;
  int32_t* l16 = w.overflow_list2;
  int32_t* n16 = w.counters_i32 + 26;
  mk.begin(KN_VITERBI, s);
  if (form == 16) {
    hipLaunchKernelGGL(k_viterbi_g<16>, dim3(grid_for(b.n_traces, TB / 16, WAVE_GRID_CAP)), dim3(TB), 0, s, b, w,
                       (const int32_t*)nullptr, (const int32_t*)nullptr, l16, n16, 1);
  } else {
    hipLaunchKernelGGL(k_viterbi_g<8>, dim3(grid_for(b.n_traces, TB / 8, WAVE_GRID_CAP)), dim3(TB), 0, s, b, w,
                       (const int32_t*)nullptr, (const int32_t*)nullptr, l8, n8, 1);
    // (sized for every trace: a block whose list entries ran out exits at once)
    hipLaunchKernelGGL(k_viterbi_g<16>, dim3(grid_for(b.n_traces, TB / 16, WAVE_GRID_CAP)), dim3(TB), 0, s, b, w,
                       (const int32_t*)l8, (const int32_t*)n8, l16, n16, 0);
  }
  hipLaunchKernelGGL(k_viterbi, dim3(grid_for(b.n_traces / 64 + 1, 1, 1024)), dim3(TB), 0, s, b, w,
                     (const int32_t*)l16, (const int32_t*)n16, 0);
  mk.end(KN_VITERBI, s);
}
void launch_route(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, hipStream_t s,
                  const Marks& mk, int from) {
  if (from >= RESUME_ROUTE_HUGE) {
    mk.begin(KN_ROUTE_GLOBAL, s);
    hipLaunchKernelGGL(k_route<2>, dim3(HUGE_SLOTS), dim3(TB), 0, s, g, b, p, w);
    mk.end(KN_ROUTE_GLOBAL, s);
    return;
  }
  TIMED(KN_ROUTE_INDEX, hipLaunchKernelGGL(k_route_index, dim3(order_grid(b.n_points, 256, 1 << 30)), dim3(256), 0,
                                           s, g, b, p, w));
  TIMED(KN_ROUTE_WAVE, hipLaunchKernelGGL(k_route<0>, dim3(SPILL_GRID), dim3(TB), 0, s, g, b, p, w));
  mk.begin(KN_ROUTE_GLOBAL, s);
  hipLaunchKernelGGL(k_route<1>, dim3(BIG_SLOTS), dim3(TB), 0, s, g, b, p, w);
  hipLaunchKernelGGL(k_route<2>, dim3(HUGE_SLOTS), dim3(TB), 0, s, g, b, p, w);
  mk.end(KN_ROUTE_GLOBAL, s);
}
void launch_segments(const DevGraph& g, const DevBatch& b, DevWork& w, DevOut& o, bool write, hipStream_t s,
                     const Marks& mk) {
  (void)write;
  const dim3 grid(grid_for(b.n_traces, 1, WAVE_GRID_CAP));
  // small LDS plan over every trace, the large one over its spills
  // (list in overflow_list0, count in counters_i32[8]: free after the route stage)
  int32_t* lst = w.overflow_list0;
  int32_t* cnt = w.counters_i32 + 8;
  mk.begin(KN_SEG_WRITE, s);
  hipLaunchKernelGGL((k_segments<SEGP_PTS_S, SEGP_TRAV_S>), grid, dim3(TB), 0, s, g, b, w, o, (const int32_t*)nullptr,
                     (const int32_t*)nullptr, lst, cnt);
  hipLaunchKernelGGL((k_segments<SEGP_PTS, SEGP_TRAV>), dim3(grid_for(b.n_traces, 1, 2048)), dim3(TB), 0, s, g, b, w,
                     o, (const int32_t*)lst, (const int32_t*)cnt, (int32_t*)nullptr, (int32_t*)nullptr);
  mk.end(KN_SEG_WRITE, s);
}
void launch_seg_bound(const DevGraph& g, const DevBatch& b, const DevParams& p, DevWork& w, int64_t* tb, hipStream_t s,
                      const Marks& mk) {
  TIMED(KN_SEG_BOUND, hipLaunchKernelGGL(k_seg_bound, dim3(grid_for(b.n_points + 1, 256, 1 << 30)), dim3(256), 0, s,
                                         g, b, p, w, tb));
}
void launch_compact(int32_t n_traces, const DevOut& o, const int32_t* seg_off, const int32_t* way_off,
                    const int32_t* rep_off, void* segs_out, int64_t* ways_out, void* reps_out, void* traces_out,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_compact, dim3(grid_for(n_traces, 1, WAVE_GRID_CAP)), dim3(TB), 0, s, n_traces, o, seg_off, way_off,
                     rep_off, (otm_segment*)segs_out, ways_out, (otm_report_rec*)reps_out,
                     (otm_trace_result*)traces_out);
}
void launch_report(const DevBatch& b, const DevReportCfg& rc, DevWork& w, DevOut& o, hipStream_t s,
                   const Marks& mk) {
  // thread per trace; the serial segment walk is latency-bound, so small
  // blocks spread the traces over more waves (0.053 -> 0.050 ms against 64 on
  // config 2)
  constexpr int tb = 16;
  if (OTM_REPORT_FORM == 1 || (OTM_REPORT_FORM == 2 && b.n_traces <= REPW_MAX_TRACES))
    TIMED(KN_REPORT, hipLaunchKernelGGL(k_report_wave, dim3(grid_for(b.n_traces, 1, WAVE_GRID_CAP)), dim3(TB), 0, s,
                                        b, rc, w, o, 0));
  else
    TIMED(KN_REPORT, hipLaunchKernelGGL(k_report, dim3(grid_for(b.n_traces, tb, 1 << 30)), dim3(tb), 0, s, b, rc, w,
                                        o, 0));
}
#undef TIMED

void launch_index_build(const DevGraph& g, const uint32_t* turn_units, uint32_t cmax, int32_t* row_cnt,
                        const IdxRow* rows, uint4* slot, bool write, hipStream_t s) {
  const int grid = grid_for((int64_t)g.n_edges + g.n_nodes, 1, 256 * 16);
  if (write)
    hipLaunchKernelGGL(k_index_build<true>, dim3(grid), dim3(TB), 0, s, g, turn_units, cmax, row_cnt, rows, slot);
  else
    hipLaunchKernelGGL(k_index_build<false>, dim3(grid), dim3(TB), 0, s, g, turn_units, cmax, row_cnt, rows, slot);
}
int index_load_fast() { return IDX_LOAD_FAST; }
int index_load_dense() { return IDX_LOAD_DENSE; }
void launch_row_sizes(const int32_t* row_cnt, int64_t* row_sizes, int32_t n, int pct, hipStream_t s) {
  hipLaunchKernelGGL(k_row_sizes, dim3(grid_for((int64_t)n + 1, 256, 1 << 30)), dim3(256), 0, s, row_cnt, row_sizes,
                     n, pct);
}
void launch_row_pack(const int32_t* row_cnt, const int64_t* row_off, IdxRow* rows, int32_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_row_pack, dim3(grid_for((int64_t)n, 256, 1 << 30)), dim3(256), 0, s, row_cnt, row_off, rows, n);
}

size_t scan_tmp_bytes(int64_t n) {
  size_t a = 0, c = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, a, (int64_t*)nullptr, (int64_t*)nullptr, (int)(n + 1));
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, c, (int32_t*)nullptr, (int32_t*)nullptr, (int)(n + 1));
  return a > c ? a : c;
}
void scan_i64(int64_t* d, int64_t n, void* tmp, size_t tmp_bytes, hipStream_t s) {
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, d, d, (int)(n + 1), s);
}
void scan_i32(int32_t* d, int64_t n, void* tmp, size_t tmp_bytes, hipStream_t s) {
  (void)hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, d, d, (int)(n + 1), s);
}

}  // namespace otm
