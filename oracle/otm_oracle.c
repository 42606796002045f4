/*
 * otm_oracle.c -- CPU oracle of the map-matching hot path.
 * TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker or the timed CPU baseline.
 *
 * This file IS the written spec of SegmentMatcher.Match
 * (py/reporter_service.py:112 -> Valhalla 2.2.7 meili, not present here;
 * DESIGN.md §3 restates the same rules in prose).  Every float operation is
 * spelled out in evaluation order and the library is built with
 * -ffp-contract=off so that the GPU kernels, which follow the same order,
 * agree bit for bit.  Parity against meili itself is UNPINNED.
 *
 *   S1 columns      interpolation_distance filter, chain links (gc, breakage)
 *   S2 candidates   grid cells in the radius box -> per-edge best projection
 *                   -> sort (sqdist, edge) -> first max_candidates
 *   S3 emission     sqdist / (2 sigma_z^2)
 *   S4 transitions  bounded Dijkstra per distinct source node, route distance
 *                   r, cost (turn_cost + |r - gc|) / beta when r <= factor * gc,
 *                   turn_cost summed over the turns of the shortest route
 *   S5 viterbi      min-sum, ties -> lowest index, dead column -> chain break
 *   S6 route        re-run the winning searches, predecessor edges
 *   S7 segments     traversals -> OSMLR groups, times linear in distance
 *   S8 report       py/reporter_service.py:110-215 on typed records
 */
#define _GNU_SOURCE
#include <fcntl.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "../include/otm_graph_format.h"
#include "orc_internal.h"
#include "otm_oracle.h"

#define MPD_F 111319.4954833f /* (float)(20037581.187 / 180), Batch.java:33 */
#define INF_F INFINITY

#define TERR_NONE 0
#define TERR_ZERODIV 1
#define TERR_CAND_OVERFLOW 2
#define TERR_SEARCH_OVERFLOW 3

static const char* terr_msg(int k) {
  switch (k) {
    case TERR_ZERODIV: return "float division by zero";
    case TERR_CAND_OVERFLOW: return "too many candidate edges within search radius";
    case TERR_SEARCH_OVERFLOW: return "route search exceeded node limit";
  }
  return "";
}

/* ================================================================== graph */
struct orc_graph {
  otmg_header h;
  void* map;
  size_t bytes;
  const float *nlat, *nlon;
  const int32_t* out_off;
  const int32_t *efrom, *eto;
  const float* elen;
  const int32_t* eshape;
  const int64_t* eway;
  const int32_t *eseg, *eseg_pos;
  const uint8_t* eflags;
  const float *slat, *slon, *scum;
  const uint64_t* gid;
  const float* glen;
  const int64_t* cell_off;
  const uint32_t* cell_ent;
  const uint16_t *ehead_out, *ehead_in;
  uint32_t* elen64; /* L(e) = round(len(e) x 64), computed once at load */
  uint64_t serial;  /* identifies this load to the per-thread workspace cache */
};
static atomic_uint_fast64_t graph_serial = 1;

orc_graph* orc_graph_load(const char* path) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) return NULL;
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(otmg_header)) {
    close(fd);
    return NULL;
  }
  void* m = mmap(NULL, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return NULL;
  orc_graph* g = (orc_graph*)calloc(1, sizeof(orc_graph));
  g->map = m;
  g->bytes = (size_t)st.st_size;
  memcpy(&g->h, m, sizeof(otmg_header));
  if (memcmp(g->h.magic, OTMG_MAGIC, 8) != 0 || g->h.version != OTMG_VERSION) {
    orc_graph_free(g);
    return NULL;
  }
#define SEC(s) ((const void*)((const char*)m + g->h.sec[s].offset))
  g->nlat = SEC(OTMG_NODE_LAT);
  g->nlon = SEC(OTMG_NODE_LON);
  g->out_off = SEC(OTMG_NODE_OUT_OFF);
  g->efrom = SEC(OTMG_EDGE_FROM);
  g->eto = SEC(OTMG_EDGE_TO);
  g->elen = SEC(OTMG_EDGE_LEN);
  g->eshape = SEC(OTMG_EDGE_SHAPE_OFF);
  g->eway = SEC(OTMG_EDGE_WAY);
  g->eseg = SEC(OTMG_EDGE_SEG);
  g->eseg_pos = SEC(OTMG_EDGE_SEG_POS);
  g->eflags = SEC(OTMG_EDGE_FLAGS);
  g->slat = SEC(OTMG_SHAPE_LAT);
  g->slon = SEC(OTMG_SHAPE_LON);
  g->scum = SEC(OTMG_SHAPE_CUM);
  g->gid = SEC(OTMG_SEG_ID);
  g->glen = SEC(OTMG_SEG_LEN);
  g->cell_off = SEC(OTMG_CELL_OFF);
  g->cell_ent = SEC(OTMG_CELL_ENT);
  g->ehead_out = SEC(OTMG_EDGE_HEAD_OUT);
  g->ehead_in = SEC(OTMG_EDGE_HEAD_IN);
#undef SEC
  g->elen64 = (uint32_t*)malloc(sizeof(uint32_t) * ((size_t)g->h.n_edges + 1));
  for (int32_t e = 0; e < g->h.n_edges; ++e) g->elen64[e] = (uint32_t)floor((double)g->elen[e] * 64.0 + 0.5);
  g->serial = atomic_fetch_add(&graph_serial, 1);
  return g;
}
void orc_graph_free(orc_graph* g) {
  if (!g) return;
  if (g->map) munmap(g->map, g->bytes);
  free(g->elen64);
  free(g);
}
int64_t orc_graph_count(const orc_graph* g, int what) {
  return what == 0 ? g->h.n_nodes : (what == 1 ? g->h.n_edges : g->h.n_segments);
}
void orc_params_default(orc_params* p) {
  p->sigma_z = 4.07f;
  p->beta = 3.0f;
  p->max_route_distance_factor = 5.0f;
  p->breakage_distance = 2000.0f;
  p->interpolation_distance = 10.0f;
  p->search_radius = 50.0f;
  p->max_search_radius = 100.0f;
  p->gps_accuracy = 5.0f;
  p->max_candidates = ORC_KMAX;
  p->turn_penalty_factor = 200.0f;
}
void orc_report_cfg_default(orc_report_cfg* c) {
  memset(c, 0, sizeof *c);
  c->n_report = 2;
  c->report_levels[0] = 0;
  c->report_levels[1] = 1;
  c->n_transition = 2;
  c->transition_levels[0] = 0;
  c->transition_levels[1] = 1;
  c->threshold_sec = 15.0;
}
void orc_free(void* p) { free(p); }

/* ================================================================== math */
/* cos of an angle in degrees: degree-14 Taylor polynomial in x^2, Horner
 * order, float.  |lat| <= 90 keeps |x| <= pi/2 (truncation < 1e-10). */
float orc_cos_deg(float deg) {
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
/* exp(x), 0 <= x <= 4: Taylor series in double, fixed term order (no libm:
 * the engine computes the same table with the same operations) */
static double orc_exp_series(double x) {
  double term = 1.0, sum = 1.0;
  for (int n = 1; n <= 40; ++n) {
    term = term * x / (double)n;
    sum = sum + term;
  }
  return sum;
}
uint32_t orc_turn_units(float factor, int d) {
  if (!(factor > 0.0f)) return 0u;
  const double x = (double)(180 - d) / 45.0;
  return (uint32_t)floor((double)factor * 64.0 / orc_exp_series(x) + 0.5);
}
/* deviation from straight on (0..180 degrees) of the turn from edge a's end
 * heading into edge b's start heading */
static int orc_turn_deg(unsigned hin, unsigned hout) {
  const int d = ((int)hout - (int)hin + 360) % 360;
  return d <= 180 ? d : 360 - d;
}
#define TURN_UNITS_MAX 0xFFFFFFu /* 2^24 - 1: a float holds the sum exactly */

/* equirectangular distance at the mean latitude (meters) */
static float orc_gc(float la, float lo, float lb, float lob) {
  const float ls = MPD_F * orc_cos_deg((la + lb) * 0.5f);
  const float dx = (lob - lo) * ls;
  const float dy = (lb - la) * MPD_F;
  return sqrtf(dx * dx + dy * dy);
}

/* ================================================================== S2 candidates */
typedef struct {
  int32_t edge;
  float sqd, off;
  int32_t k;
} hit;

/* (sqdist, edge, offset): a node candidate (offset 0) sorts before an
 * interior candidate of its representative edge at the same distance */
static int hit_cmp(const void* a, const void* b) {
  const hit* x = (const hit*)a;
  const hit* y = (const hit*)b;
  if (x->sqd < y->sqd) return -1;
  if (x->sqd > y->sqd) return 1;
  if (x->edge != y->edge) return (x->edge > y->edge) - (x->edge < y->edge);
  return (x->off > y->off) - (x->off < y->off);
}

/* projection of the probe (lat,lon) onto shape segment k of edge e */
static void project(const orc_graph* g, int32_t e, int32_t k, float lat, float lon, float ls, float* sqd_out,
                    float* off_out, int* at_end) {
  const int32_t a = g->eshape[e] + k, b = a + 1;
  const float ax = (g->slon[a] - lon) * ls;
  const float ay = (g->slat[a] - lat) * MPD_F;
  const float bx = (g->slon[b] - lon) * ls;
  const float by = (g->slat[b] - lat) * MPD_F;
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
  *sqd_out = px * px + py * py;
  float off = g->scum[a] + t * (g->scum[b] - g->scum[a]);
  const float len = g->elen[e];
  off = off > len ? len : off;
  *off_out = off;
  /* clamped to the edge's last shape point: the projection is its end node */
  *at_end = t == 1.0f && b == g->eshape[e + 1] - 1;
}

/* radius rule: max(search_radius, accuracy or gps_accuracy), capped */
static float probe_radius(const orc_params* P, float acc) {
  const float a = acc > 0.0f ? acc : P->gps_accuracy;
  float r = a > P->search_radius ? a : P->search_radius;
  return r < P->max_search_radius ? r : P->max_search_radius;
}

/* distinct edges one probe's scan projects (the §8(d) unique-edge term) */
#define SEEN_CAP 1024
typedef struct {
  int32_t key[SEEN_CAP];
  uint32_t stamp[SEEN_CAP];
  uint32_t gen;
} seen_set;
static void seen_add(const orc_graph* g, seen_set* S, int32_t e, orc_counters* C) {
  uint32_t h = ((uint32_t)e * 2654435761u) >> 22;
  for (int k = 0; k < SEEN_CAP; ++k, h = (h + 1) & (SEEN_CAP - 1)) {
    if (S->stamp[h] != S->gen) {
      S->stamp[h] = S->gen;
      S->key[h] = e;
      C->edges_projected++;
      C->edge_shape_points += g->eshape[e + 1] - g->eshape[e];
      return;
    }
    if (S->key[h] == e) return;
  }
}

/* returns the number of candidates; *hits / *hcap: the distinct edges in
 * range, grown as needed (no limit: round 4 dropped the 256-edge spec limit) */
static int candidates(const orc_graph* g, const orc_params* P, float lat, float lon, float acc, int32_t* c_edge,
                      float* c_off, float* c_emis, hit** hitsp, int* hcap, seen_set* seen, orc_counters* C) {
  hit* hits = *hitsp;
  const float r = probe_radius(P, acc);
  const float r2 = r * r;
  const float ls = MPD_F * orc_cos_deg(lat);
  const float dlat = r / MPD_F;
  const float dlon = r / ls;
  const double cell = g->h.grid_cell_deg;
  const double la_lo = ((double)lat - (double)dlat - g->h.grid_lat0) / cell;
  const double la_hi = ((double)lat + (double)dlat - g->h.grid_lat0) / cell;
  const double lo_lo = ((double)lon - (double)dlon - g->h.grid_lon0) / cell;
  const double lo_hi = ((double)lon + (double)dlon - g->h.grid_lon0) / cell;
  const double R = g->h.grid_rows, Cn = g->h.grid_cols;
  int nh = 0;
  if (seen && ++seen->gen == 0) {
    memset(seen->stamp, 0, sizeof seen->stamp);
    seen->gen = 1;
  }
  if (!(la_hi < 0.0 || lo_hi < 0.0 || la_lo >= R || lo_lo >= Cn)) {
    const int r0 = la_lo < 0.0 ? 0 : (int)floor(la_lo);
    const int r1 = la_hi >= R ? (int)R - 1 : (int)floor(la_hi);
    const int c0 = lo_lo < 0.0 ? 0 : (int)floor(lo_lo);
    const int c1 = lo_hi >= Cn ? (int)Cn - 1 : (int)floor(lo_hi);
    for (int rr = r0; rr <= r1; ++rr) {
      for (int cc = c0; cc <= c1; ++cc) {
        const size_t cidx = (size_t)rr * (size_t)g->h.grid_cols + (size_t)cc;
        C->cells_visited++;
        for (int64_t q = g->cell_off[cidx]; q < g->cell_off[cidx + 1]; ++q) {
          const uint32_t ent = g->cell_ent[q];
          const int32_t e = (int32_t)(ent >> 4), k = (int32_t)(ent & 15u);
          float sqd, off;
          int at_end;
          project(g, e, k, lat, lon, ls, &sqd, &off, &at_end);
          C->cell_entries_scanned++;
          if (seen) seen_add(g, seen, e, C);
          if (!(sqd <= r2)) continue;
          int f = -1;
          for (int h = 0; h < nh; ++h)
            if (hits[h].edge == e) {
              f = h;
              break;
            }
          if (f < 0) {
            if (nh == *hcap) {
              *hcap = *hcap ? *hcap * 2 : 256;
              hits = *hitsp = (hit*)realloc(hits, sizeof(hit) * (size_t)*hcap);
            }
            hits[nh].edge = e;
            hits[nh].sqd = sqd;
            hits[nh].off = off;
            hits[nh].k = k;
            ++nh;
          } else if (sqd < hits[f].sqd || (sqd == hits[f].sqd && k < hits[f].k)) {
            hits[f].sqd = sqd;
            hits[f].off = off;
            hits[f].k = k;
          }
        }
      }
    }
  }
  /* node snap: an edge's best projection
   * at its start node v (offset 0), or at its end node v when v has an
   * outgoing edge, becomes the node candidate of v -- one per node, shared by
   * all its edges, carried as (v's first outgoing edge, offset 0) at the
   * smallest distance of the projections that snapped to it */
  int nk = 0;
  for (int h = 0; h < nh; ++h) {
    const int32_t e = hits[h].edge;
    float sqd, off;
    int at_end;
    project(g, e, hits[h].k, lat, lon, ls, &sqd, &off, &at_end);
    hit x = hits[h];
    x.off = off;
    int32_t v = -1;
    if (off == 0.0f) v = g->efrom[e];
    else if (at_end && g->out_off[g->eto[e] + 1] > g->out_off[g->eto[e]]) v = g->eto[e];
    if (v >= 0) {
      x.edge = g->out_off[v];
      x.off = 0.0f;
      int f = -1;
      for (int m = 0; m < nk; ++m)
        if (hits[m].edge == x.edge && hits[m].off == 0.0f) f = m;
      if (f >= 0) {
        if (x.sqd < hits[f].sqd) hits[f].sqd = x.sqd;
        continue;
      }
    }
    hits[nk++] = x;
  }
  nh = nk;
  if (nh > 1) qsort(hits, (size_t)nh, sizeof(hit), hit_cmp);
  const int K = nh < P->max_candidates ? nh : P->max_candidates;
  const float ds = (2.0f * P->sigma_z) * P->sigma_z;
  for (int j = 0; j < K; ++j) {
    c_edge[j] = hits[j].edge;
    c_off[j] = hits[j].off;
    c_emis[j] = hits[j].sqd / ds;
  }
  C->candidates += K;
  return K;
}

/* ================================================================== S4/S6 turn-aware bounded search
 * a transition's route is the shortest by "distance cost
 * plus turn penalty" (DESIGN.md §3 rule 4).  The search labels every directed
 * edge g with the cheapest way to be at g's start, turned into it (its
 * departure label), and every node v with the cheapest way to arrive at v
 * (its arrival label).  Costs are integers in 1/64 m: an edge costs L(e) =
 * round(len(e) x 64), a turn its turn units; a label is the 64-bit key
 * cost << 32 | predecessor edge (0xFFFFFFFF: none), compared as one integer,
 * so ties go to the smaller predecessor and the labels are the search's
 * unique fixed point (every step costs > 0) -- the GPU's label-correcting
 * searches and index builder reach the same labels in any order.  A search
 * from source node u entered with heading hin (NO_HEAD for a node candidate):
 *   arrival(u) = (0, none); departure(g) = (turn(hin, g), none) for g out of u;
 *   a departure label (c, .) of g gives arrival(to(g)) <= (c + L(g), g) and
 *   departure(h) <= (c + L(g) + turn(g, h), g) for h out of to(g);
 * bounded: only labels with cost <= floor(B x 64), B = max_route_distance_factor
 * x gc.  A route's distance and turn units are summed along its edges in
 * route order (rule 4). */
#define NONE_PRED 0xFFFFFFFFu
typedef struct {
  uint64_t k;
  int32_t e;
} khn;

typedef struct ws {
  uint64_t *ek, *nk;      /* departure labels per edge, arrival labels per node */
  uint32_t *elab, *nlab;  /* stamps: labelled in this search */
  uint32_t stamp;
  int32_t* elist;         /* the labelled edges, in labelling order */
  int32_t ne, nn;         /* labelled edges / nodes */
  khn* heap;
  size_t hn, hcap;
  hit* hits; /* distinct edges of a probe (grown) */
  int hitcap;
  seen_set seen;
} ws;

static void hpush(ws* w, uint64_t k, int32_t e) {
  if (w->hn == w->hcap) {
    w->hcap = w->hcap ? w->hcap * 2 : 1024;
    w->heap = (khn*)realloc(w->heap, w->hcap * sizeof(khn));
  }
  size_t i = w->hn++;
  while (i > 0) {
    size_t q = (i - 1) / 2;
    if (w->heap[q].k <= k) break;
    w->heap[i] = w->heap[q];
    i = q;
  }
  w->heap[i].k = k;
  w->heap[i].e = e;
}
static khn hpop(ws* w) {
  khn top = w->heap[0], last = w->heap[--w->hn];
  size_t i = 0;
  while (1) {
    size_t c = 2 * i + 1;
    if (c >= w->hn) break;
    if (c + 1 < w->hn && w->heap[c + 1].k < w->heap[c].k) ++c;
    if (w->heap[c].k >= last.k) break;
    w->heap[i] = w->heap[c];
    i = c;
  }
  if (w->hn) w->heap[i] = last;
  return top;
}

/* ================================================================== per-batch state */
typedef struct tres {
  orc_segment* segs;
  int nseg, cseg;
  int64_t* ways;
  int nway, cway;
  orc_report_rec* reps;
  int nrep, crep;
  orc_trace_result tr;
} tres;

typedef struct batch {
  const orc_graph* g;
  const orc_params* P;
  const orc_report_cfg* rc;
  int32_t n_traces;
  const int64_t* toff_pts;
  const float *lat, *lon, *acc;
  const double* time;
  /* point-indexed stage arrays */
  uint8_t* is_col;
  uint8_t* chain_start;
  int32_t *ncand, *cand_edge, *state, *col_prev;
  float *cand_off, *cand_emis, *route_dist, *gc;
  float* ipos;   /* interpolated points: position along their step's route, -1 none (S7) */
  int32_t* terr; /* per trace error kind */
  int64_t* trans_off;
  float* trans;
  tres* res;
  atomic_int next;
  int phase;
  orc_counters* ctr; /* per thread */
  int count_unique;  /* count §8(d)'s unique projected edges (keep_stages) */
  const uint32_t* elen64;  /* L(e) = round(len(e) x 64): the search's edge costs */
  uint32_t turn_units[181]; /* orc_turn_units per deviation 0..180 */
} batch;

#define GROW(arr, n, cap, T)                                   \
  do {                                                         \
    if ((n) == (cap)) {                                        \
      (cap) = (cap) ? 2 * (cap) : 8;                           \
      (arr) = (T*)realloc((arr), sizeof(T) * (size_t)(cap));   \
    }                                                          \
  } while (0)

/* ------------------------------------------------------------ S1 + S2 */
static void phase_a(batch* B, ws* w, int32_t t, orc_counters* C) {
  const orc_graph* g = B->g;
  const orc_params* P = B->P;
  const int64_t a = B->toff_pts[t], b = B->toff_pts[t + 1];
  int64_t last = -1;
  for (int64_t p = a; p < b; ++p) {
    B->ncand[p] = 0;
    B->col_prev[p] = -1;
    B->gc[p] = 0.0f;
    B->is_col[p] = 0;
    C->points++;
    float gcv = 0.0f;
    if (last >= 0) {
      gcv = orc_gc(B->lat[last], B->lon[last], B->lat[p], B->lon[p]);
      if (!(gcv >= P->interpolation_distance)) continue;
    }
    B->is_col[p] = 1;
    C->columns++;
    B->gc[p] = gcv;
    int K = candidates(g, P, B->lat[p], B->lon[p], B->acc[p], B->cand_edge + p * ORC_KMAX,
                       B->cand_off + p * ORC_KMAX, B->cand_emis + p * ORC_KMAX, &w->hits, &w->hitcap,
                       B->count_unique ? &w->seen : NULL, C);
    if (K < 0) {
      if (!B->terr[t]) B->terr[t] = TERR_CAND_OVERFLOW;
      K = 0;
    }
    B->ncand[p] = K;
    if (last >= 0 && K > 0 && B->ncand[last] > 0 && gcv <= P->breakage_distance) B->col_prev[p] = (int32_t)last;
    last = p;
  }
}

/* ------------------------------------------------------------ S4 */
/* A candidate at offset 0 is a node candidate (S2's node snap): its routes
 * start at that node with nothing left to drive and no heading; an edge
 * candidate's start at its edge's end node after the rest of the edge,
 * entered with the edge's end heading. */
static int32_t src_node(const orc_graph* g, int32_t e, float off) { return off == 0.0f ? g->efrom[e] : g->eto[e]; }
static float src_start(const orc_graph* g, int32_t e, float off) { return off == 0.0f ? 0.0f : g->elen[e] - off; }
#define NO_HEAD 0xFFFFu /* a node candidate's side of a route: no turn */
static unsigned src_hin(const orc_graph* g, int32_t e, float off) { return off == 0.0f ? NO_HEAD : g->ehead_in[e]; }
static uint32_t turn_cost_units(const batch* B, unsigned hin, unsigned hout) {
  return (hin == NO_HEAD || hout == NO_HEAD) ? 0u : B->turn_units[orc_turn_deg(hin, hout)];
}
/* Rule 4's same-edge step from (e, oi) to (e, oj): the route along the edge
 * when oj is not before oi; when oj is behind oi and both are edge
 * candidates, a stay: GPS noise moved the later probe back along the edge
 * (vehicles do not reverse along a directed edge), so the step has route
 * distance 0, no turns and no traversal, and the position on the edge stays
 * at the largest offset reached.  (A backward step otherwise needs a loop
 * around the block, or a U-turn onto the opposite edge and back, which the
 * matched segments then show: VERDICT r3 #2) */
static int same_edge_step(int32_t ei, float oi, int32_t ej, float oj) {
  return ei == ej && (oj >= oi || (oj > 0.0f && oi > 0.0f));
}
static float same_edge_dist(float oi, float oj) { return oj >= oi ? oj - oi : 0.0f; }

/* the cost bound of a search bounded by B metres */
static uint32_t cost_bound(float B) { return (uint32_t)floor((double)B * 64.0); }

static int set_edge(ws* w, int32_t g, uint64_t k) {
  if (w->elab[g] != w->stamp) {
    w->elab[g] = w->stamp;
    w->elist[w->ne++] = g;
  } else if (k >= w->ek[g]) {
    return 0;
  }
  w->ek[g] = k;
  hpush(w, k, g);
  return 1;
}
static void set_node(ws* w, int32_t v, uint64_t k) {
  if (w->nlab[v] != w->stamp) {
    w->nlab[v] = w->stamp;
    w->nn++;
    w->nk[v] = k;
  } else if (k < w->nk[v]) {
    w->nk[v] = k;
  }
}

/* The labels of a search from node u entered with heading hin, bounded by
 * cost cmax.  Returns 0 (no label limit since round 4: the workspace holds
 * every edge and node of the graph). */
static int ta_search(const batch* B, ws* w, int32_t u, unsigned hin, uint32_t cmax, orc_counters* C, int route) {
  const orc_graph* g = B->g;
  if (++w->stamp == 0) {
    memset(w->elab, 0, sizeof(uint32_t) * (size_t)g->h.n_edges);
    memset(w->nlab, 0, sizeof(uint32_t) * (size_t)g->h.n_nodes);
    w->stamp = 1;
  }
  w->hn = 0;
  w->ne = w->nn = 0;
  set_node(w, u, NONE_PRED);
  for (int32_t e = g->out_off[u]; e < g->out_off[u + 1]; ++e) {
    const uint32_t c = turn_cost_units(B, hin, g->ehead_out[e]);
    if (c <= cmax) set_edge(w, e, ((uint64_t)c << 32) | NONE_PRED);
  }
  while (w->hn) {
    const khn h = hpop(w);
    const int32_t e = h.e;
    if (h.k != w->ek[e]) continue;
    const uint64_t ca = (h.k >> 32) + (uint64_t)B->elen64[e];
    if (ca > cmax) continue;
    const int32_t v = g->eto[e];
    set_node(w, v, (ca << 32) | (uint32_t)e);
    for (int32_t f = g->out_off[v]; f < g->out_off[v + 1]; ++f) {
      const uint64_t c = ca + turn_cost_units(B, g->ehead_in[e], g->ehead_out[f]);
      if (c <= cmax) set_edge(w, f, (c << 32) | (uint32_t)e);
    }
  }
  /* work counters: the departure labels, and the edges a label relaxes
     (its end node's out-edges, when the arrival is within the bound) */
  int64_t relaxed = 0;
  for (int k = 0; k < w->ne; ++k) {
    const int32_t e = w->elist[k];
    if ((w->ek[e] >> 32) + (uint64_t)B->elen64[e] <= cmax) relaxed += g->out_off[g->eto[e] + 1] - g->out_off[g->eto[e]];
  }
  if (route) {
    C->route_searches++;
    C->route_nodes_settled += w->ne;
    C->route_edges_relaxed += relaxed;
  } else {
    C->searches++;
    C->nodes_settled += w->ne;
    C->edges_relaxed += relaxed;
  }
  return 0;
}

/* The route of the last search to candidate (ej, oj): into edge ej (an edge
 * candidate: its departure label, the turn into ej included) or to node
 * from(ej) (a node candidate: its arrival label).  Returns 0 when unlabelled;
 * else the route's fully traversed edges in order (path, when non-NULL, up to
 * cap), their number, their summed length d (route order) and the route's
 * turn units (clamped to 2^24 - 1). */
static int ta_route(const batch* B, const ws* w, unsigned hin, int32_t ej, float oj, int32_t* path, int cap, int* plen,
                    float* d, uint32_t* units) {
  const orc_graph* g = B->g;
  uint64_t k;
  if (oj == 0.0f) {
    const int32_t v = g->efrom[ej];
    if (w->nlab[v] != w->stamp) return 0;
    k = w->nk[v];
  } else {
    if (w->elab[ej] != w->stamp) return 0;
    k = w->ek[ej];
  }
  int32_t tmp[64];
  int32_t* pp = path ? path : tmp;
  const int pc = path ? cap : 64;
  int n = 0;
  uint32_t pr = (uint32_t)k;
  while (pr != NONE_PRED) {
    if (n < pc) pp[n] = (int32_t)pr;
    ++n;
    pr = (uint32_t)w->ek[pr];
  }
  /* forward: route order; a chain longer than the buffer is walked again */
  float dd = 0.0f;
  uint64_t un = 0;
  unsigned h = hin;
  for (int m = n - 1; m >= 0; --m) {
    int32_t e;
    if (n <= pc) {
      e = pp[m];
    } else {
      int32_t x = (int32_t)(uint32_t)k;
      for (int s2 = 0; s2 < m; ++s2) x = (int32_t)(uint32_t)w->ek[x];
      e = x;
    }
    un += turn_cost_units(B, h, g->ehead_out[e]);
    dd = dd + g->elen[e];
    h = g->ehead_in[e];
  }
  if (oj != 0.0f) un += turn_cost_units(B, h, g->ehead_out[ej]);
  if (path && n <= pc)
    for (int a = 0, b = n - 1; a < b; ++a, --b) {
      const int32_t t = pp[a];
      pp[a] = pp[b];
      pp[b] = t;
    }
  *plen = n;
  *d = dd;
  *units = un > TURN_UNITS_MAX ? TURN_UNITS_MAX : (uint32_t)un;
  return 1;
}

static int transitions(batch* B, ws* w, int64_t p, orc_counters* C) {
  const orc_graph* g = B->g;
  const int64_t q = B->col_prev[p];
  const int Kq = B->ncand[q], Kp = B->ncand[p];
  const float gcv = B->gc[p];
  const float bound = B->P->max_route_distance_factor * gcv;
  const uint32_t cmax = cost_bound(bound);
  float* T = B->trans + B->trans_off[p];
  for (int k = 0; k < Kq * Kp; ++k) T[k] = INF_F;
  const int32_t* eq = B->cand_edge + q * ORC_KMAX;
  const float* oq = B->cand_off + q * ORC_KMAX;
  const int32_t* ep = B->cand_edge + p * ORC_KMAX;
  const float* op = B->cand_off + p * ORC_KMAX;
  /* one search per distinct source (node, heading) */
  for (int i0 = 0; i0 < Kq; ++i0) {
    const int32_t u = src_node(g, eq[i0], oq[i0]);
    const unsigned hin = src_hin(g, eq[i0], oq[i0]);
    int seen = 0;
    for (int k = 0; k < i0; ++k) seen |= src_node(g, eq[k], oq[k]) == u && src_hin(g, eq[k], oq[k]) == hin;
    if (seen) continue;
    if (ta_search(B, w, u, hin, cmax, C, 0) < 0) return -1;
    for (int i = i0; i < Kq; ++i) {
      if (src_node(g, eq[i], oq[i]) != u || src_hin(g, eq[i], oq[i]) != hin) continue;
      const float start = src_start(g, eq[i], oq[i]);
      for (int j = 0; j < Kp; ++j) {
        float r;
        uint32_t units = 0;
        if (same_edge_step(eq[i], oq[i], ep[j], op[j])) {
          r = same_edge_dist(oq[i], op[j]);
        } else {
          float d;
          int n;
          if (!ta_route(B, w, hin, ep[j], op[j], NULL, 0, &n, &d, &units)) continue;
          const float sd = start + d;
          r = sd + op[j];
        }
        if (r <= bound) {
          const float tc = (float)units * 0.015625f;
          const float diff = fabsf(r - gcv);
          T[i * Kp + j] = (tc + diff) / B->P->beta;
          C->transitions++;
        }
      }
    }
  }
  return 0;
}

/* ------------------------------------------------------------ S5 */
static void viterbi(batch* B, int32_t t, uint8_t* bp /* [npts*KMAX] */) {
  const int64_t a = B->toff_pts[t], b = B->toff_pts[t + 1];
  float prev[ORC_KMAX], cur[ORC_KMAX];
  int open = 0;
  int64_t last = -1;
#define BACKTRACK(endp)                                                                \
  do {                                                                                 \
    int64_t pp = (endp);                                                               \
    int bj = -1;                                                                       \
    float bv = INF_F;                                                                  \
    for (int j = 0; j < B->ncand[pp]; ++j)                                             \
      if (prev[j] < bv) {                                                              \
        bv = prev[j];                                                                  \
        bj = j;                                                                        \
      }                                                                                \
    int jj = bj;                                                                       \
    while (1) {                                                                        \
      B->state[pp] = jj;                                                               \
      if (B->chain_start[pp]) break;                                                   \
      jj = bp[(pp - a) * ORC_KMAX + jj];                                               \
      pp = B->col_prev[pp];                                                            \
    }                                                                                  \
  } while (0)
  for (int64_t p = a; p < b; ++p) {
    B->state[p] = -1;
    B->chain_start[p] = 0;
  }
  for (int64_t p = a; p < b; ++p) {
    if (!B->is_col[p]) continue;
    const int Kp = B->ncand[p];
    if (Kp == 0) {
      if (open) BACKTRACK(last);
      open = 0;
      continue;
    }
    const float* em = B->cand_emis + p * ORC_KMAX;
    int started = 0;
    if (open && B->col_prev[p] == last) {
      const int Kq = B->ncand[last];
      const float* T = B->trans + B->trans_off[p];
      int any = 0;
      for (int j = 0; j < Kp; ++j) {
        float best = INF_F;
        int bi = -1;
        for (int i = 0; i < Kq; ++i) {
          const float v = prev[i] + T[i * Kp + j];
          if (v < best) {
            best = v;
            bi = i;
          }
        }
        if (bi >= 0) {
          cur[j] = best + em[j];
          bp[(p - a) * ORC_KMAX + j] = (uint8_t)bi;
          any = 1;
        } else {
          cur[j] = INF_F;
          bp[(p - a) * ORC_KMAX + j] = 0xFF;
        }
      }
      if (!any) {
        BACKTRACK(last);
      } else {
        started = 1;
      }
    } else if (open) {
      BACKTRACK(last);
    }
    if (!started) {
      for (int j = 0; j < Kp; ++j) cur[j] = em[j];
      B->chain_start[p] = 1;
    }
    memcpy(prev, cur, sizeof(float) * (size_t)Kp);
    open = 1;
    last = p;
  }
  if (open) BACKTRACK(last);
#undef BACKTRACK
}

/* ------------------------------------------------------------ S6 + S7 */
typedef struct {
  int32_t edge;
  float off0, off1;
  double t0, t1;
  int32_t sh0, sh1;
} trav;

typedef struct {
  trav* v;
  int n, cap;
} travs;

static void tpush(travs* T, trav x) {
  GROW(T->v, T->n, T->cap, trav);
  T->v[T->n++] = x;
}

static void emit_group(batch* B, tres* R, const trav* f, const trav* l, const trav* all, int gi0, int gi1) {
  const orc_graph* g = B->g;
  GROW(R->segs, R->nseg, R->cseg, orc_segment);
  orc_segment* s = &R->segs[R->nseg++];
  memset(s, 0, sizeof *s);
  const int32_t sg = g->eseg[f->edge];
  int sv, ev;
  if (sg >= 0) {
    sv = f->off0 == 0.0f && (g->eflags[f->edge] & OTM_EDGE_SEG_BEGIN);
    ev = l->off1 == g->elen[l->edge] && (g->eflags[l->edge] & OTM_EDGE_SEG_END);
    s->segment_id = (int64_t)g->gid[sg];
    s->length = (sv && ev) ? (int32_t)floor((double)g->glen[sg] + 0.5) : -1;
  } else {
    sv = f->off0 == 0.0f;
    ev = l->off1 == g->elen[l->edge];
    s->segment_id = -1;
    s->length = -1;
    if (g->eflags[f->edge] & OTM_EDGE_INTERNAL) s->flags |= 4u;
  }
  if (sv) {
    s->flags |= 1u;
    s->start_time = f->t0;
  }
  if (ev) {
    s->flags |= 2u;
    s->end_time = l->t1;
  }
  s->queue_length = 0;
  s->begin_shape_index = f->sh0;
  s->end_shape_index = l->sh1;
  s->way_off = R->nway;
  for (int k = gi0; k <= gi1; ++k) {
    const int64_t way = g->eway[all[k].edge];
    if (R->nway > s->way_off && R->ways[R->nway - 1] == way) continue;
    GROW(R->ways, R->nway, R->cway, int64_t);
    R->ways[R->nway++] = way;
  }
  s->way_cnt = R->nway - s->way_off;
}

static void group_chain(batch* B, tres* R, const travs* T) {
  const orc_graph* g = B->g;
  int gs = -1; /* group start index */
  for (int k = 0; k < T->n; ++k) {
    const int32_t e = T->v[k].edge;
    int join = 0;
    if (gs >= 0) {
      const int32_t pe = T->v[k - 1].edge;
      const int32_t s = g->eseg[e], ps = g->eseg[pe];
      if (s >= 0) join = ps == s && g->eseg_pos[e] == g->eseg_pos[pe] + 1;
      else join = ps < 0 && ((g->eflags[e] ^ g->eflags[pe]) & OTM_EDGE_INTERNAL) == 0;
    }
    if (!join) {
      if (gs >= 0) emit_group(B, R, &T->v[gs], &T->v[k - 1], T->v, gs, k - 1);
      gs = k;
    }
  }
  if (gs >= 0) emit_group(B, R, &T->v[gs], &T->v[T->n - 1], T->v, gs, T->n - 1);
}

/* route of step p (from state at q = col_prev[p] to state at p) */
static int route_step(batch* B, ws* w, int64_t p, int32_t* path, int pcap, int* plen, int* same, float* R,
                      orc_counters* C) {
  const orc_graph* g = B->g;
  const int64_t q = B->col_prev[p];
  const int i = B->state[q], j = B->state[p];
  const int32_t ei = B->cand_edge[q * ORC_KMAX + i], ej = B->cand_edge[p * ORC_KMAX + j];
  const float oi = B->cand_off[q * ORC_KMAX + i], oj = B->cand_off[p * ORC_KMAX + j];
  *plen = 0;
  if (same_edge_step(ei, oi, ej, oj)) {
    *same = 1;
    *R = same_edge_dist(oi, oj);
    return 0;
  }
  *same = 0;
  const float bound = B->P->max_route_distance_factor * B->gc[p];
  const int32_t u = src_node(g, ei, oi);
  const unsigned hin = src_hin(g, ei, oi);
  if (ta_search(B, w, u, hin, cost_bound(bound), C, 1) < 0) return -1;
  float d;
  uint32_t units;
  if (!ta_route(B, w, hin, ej, oj, path, pcap, plen, &d, &units) || *plen > pcap) return -1;
  C->route_edges += *plen;
  const float start = src_start(g, ei, oi);
  const float sd = start + d;
  *R = sd + oj;
  return 0;
}

/* ------------------------------------------------------------ S7a interpolated points
 * a point within interpolation_distance of the previous
 * column gets no HMM state and is "projected onto the final route
 * afterwards"; README.md:162-163 defines begin/end_shape_index as the trace
 * index "before/at" a segment's start/end.  So the interpolated points of a
 * step q -> p (q < k < p; a step that stays on one edge has no boundary inside
 * it and needs none) are placed on the step's route:
 *   pieces, in route order: the rest of q's edge [off_q, len] (none for a node
 *   candidate), the path's edges [0, len], p's edge [0, off_p] (none for a node
 *   candidate); piece m starts at route distance xs_m;
 *   on each piece, the point's best projection onto that edge's polyline
 *   (lowest sqdist, ties the lowest shape segment) is admissible iff its
 *   offset lies inside the piece; its position is xs_m + (off - o0_m) and its
 *   cost sqdist / (2 sigma_z^2) + |position - gc(q, k)| / beta -- meili's
 *   emission plus a transition from q (no turns), the lowest cost winning
 *   (ties: the earliest piece);
 *   a point with no admissible piece stays unplaced (-1).
 * The step's anchors are its two states and the placed points that are not
 * behind an earlier anchor (position >= the running maximum, starting at q's
 * 0): their positions are nondecreasing in trace order.  A boundary at route distance x gets
 *   shape index = the last anchor (trace order) at position <= x;
 *   time = linear between the last anchor L before p with position <= x and
 *   the anchor N after it: t_L + (t_N - t_L) * ((x - x_L) / (x_N - x_L)),
 *   t_L when x_N == x_L.
 * A step without placed points is the two-state rule: t_q + (t_p - t_q) * x /
 * R, and q's index unless x reaches R. */
typedef struct {
  int32_t edge;
  float o0, o1, xs;
} piece;

static float interp_pos(const batch* B, const piece* pc, int npc, int64_t q, int64_t k) {
  const orc_graph* g = B->g;
  const float lat = B->lat[k], lon = B->lon[k];
  const float ls = MPD_F * orc_cos_deg(lat);
  const float gcd = orc_gc(B->lat[q], B->lon[q], lat, lon);
  const float ds = (2.0f * B->P->sigma_z) * B->P->sigma_z;
  float best = INF_F, bpos = -1.0f;
  for (int m = 0; m < npc; ++m) {
    const int32_t e = pc[m].edge;
    const int nsh = g->eshape[e + 1] - g->eshape[e] - 1;
    float bsq = INF_F, boff = 0.0f;
    for (int s = 0; s < nsh; ++s) {
      float sqd, off;
      int at_end;
      project(g, e, s, lat, lon, ls, &sqd, &off, &at_end);
      if (sqd < bsq) {
        bsq = sqd;
        boff = off;
      }
    }
    if (!(boff >= pc[m].o0 && boff <= pc[m].o1)) continue;
    const float pos = pc[m].xs + (boff - pc[m].o0);
    const float cost = bsq / ds + fabsf(pos - gcd) / B->P->beta;
    if (cost < best) {
      best = cost;
      bpos = pos;
    }
  }
  return bpos;
}

/* places the interpolated points of step q -> p (route: the rest of e_i from
   o_i, path[0..plen), e_j up to o_j) */
static void interp_step(batch* B, int64_t q, int64_t p, int32_t ei, float oi, int32_t ej, float oj,
                        const int32_t* path, int plen) {
  if (p - q < 2) return;
  const orc_graph* g = B->g;
  piece* pc = (piece*)malloc(sizeof(piece) * (size_t)(plen + 2));
  int n = 0;
  const float start = src_start(g, ei, oi);
  if (oi != 0.0f) pc[n++] = (piece){ei, oi, g->elen[ei], 0.0f};
  float dd = 0.0f;
  for (int k = 0; k < plen; ++k) {
    const float len = g->elen[path[k]];
    pc[n++] = (piece){path[k], 0.0f, len, start + dd};
    dd = dd + len;
  }
  if (oj != 0.0f) pc[n++] = (piece){ej, 0.0f, oj, start + dd};
  for (int64_t k = q + 1; k < p; ++k) B->ipos[k] = interp_pos(B, pc, n, q, k);
  free(pc);
}

/* time and shape index (relative to trace start a) of the boundary at route
   distance x of step q -> p */
static void step_bound(const batch* B, int64_t a, int64_t q, int64_t p, float R, float x, double* t, int32_t* sh) {
  int64_t iL = q, k = q + 1;
  float xL = 0.0f, xN = R, run = 0.0f;
  double tL = B->time[q], tN = B->time[p];
  for (; k < p; ++k) {
    const float v = B->ipos[k];
    if (!(v >= run)) continue; /* unplaced, or behind an earlier anchor: no anchor */
    if (!(v <= x)) break;
    iL = k;
    xL = v;
    tL = B->time[k];
    run = v;
  }
  for (; k < p; ++k)
    if (B->ipos[k] >= run) {
      xN = B->ipos[k];
      tN = B->time[k];
      break;
    }
  *sh = (int32_t)((R <= x ? p : iL) - a);
  const float den = xN - xL;
  *t = den > 0.0f ? tL + (tN - tL) * ((double)(x - xL) / (double)den) : tL;
}

static int segments_of_trace(batch* B, ws* w, int32_t t, tres* R, orc_counters* C) {
  const orc_graph* g = B->g;
  const int64_t a = B->toff_pts[t], b = B->toff_pts[t + 1];
  travs T = {0};
  int32_t* path = NULL;
  int pcap = 0;
  int open = 0;   /* a chain is open */
  int nstate = 0; /* states in the open chain */
  trav cur = {0};
  int64_t lastp = -1;
  int rc = 0;
  float curmax = 0.0f; /* the open traversal's largest state offset */
  for (int64_t p = a; p <= b; ++p) {
    const int is_state = p < b && B->is_col[p] && B->state[p] >= 0;
    if (p < b && !is_state) continue;
    const int new_chain = p == b || B->chain_start[p];
    if (open && new_chain) {
      /* close the open chain; a chain ending on a node candidate ends at the
         node: the traversal opened there never left it */
      cur.off1 = curmax; /* the largest offset of the open traversal's states (rule 4's stays) */
      cur.t1 = B->time[lastp];
      cur.sh1 = (int32_t)(lastp - a);
      if (cur.off1 != 0.0f) tpush(&T, cur);
      if (nstate >= 2) group_chain(B, R, &T);
      T.n = 0;
      open = 0;
    }
    if (p == b) break;
    const int j = B->state[p];
    const int32_t ej = B->cand_edge[p * ORC_KMAX + j];
    const float oj = B->cand_off[p * ORC_KMAX + j];
    if (new_chain) {
      cur.edge = ej;
      cur.off0 = oj;
      cur.t0 = B->time[p];
      cur.sh0 = (int32_t)(p - a);
      curmax = oj;
      open = 1;
      nstate = 1;
      lastp = p;
      continue;
    }
    /* step lastp -> p */
    if (pcap < g->h.n_edges + 1) {
      pcap = g->h.n_edges + 1; /* a route's edges are labelled edges of its search */
      path = (int32_t*)realloc(path, sizeof(int32_t) * (size_t)pcap);
    }
    int plen, same;
    float Rd;
    if (route_step(B, w, p, path, pcap, &plen, &same, &Rd, C) < 0) {
      rc = -1;
      break;
    }
    B->route_dist[p] = Rd;
    if (!same) {
      /* close the traversal on the state's edge, unless the state is a node
         candidate: its route starts at the node */
      const int32_t ei = cur.edge;
      const float oi = B->cand_off[lastp * ORC_KMAX + B->state[lastp]];
      interp_step(B, lastp, p, ei, oi, ej, oj, path, plen);
      const float start = src_start(g, ei, oi);
      float x = start;
      cur.off1 = g->elen[ei];
      step_bound(B, a, lastp, p, Rd, x, &cur.t1, &cur.sh1);
      if (oi != 0.0f) tpush(&T, cur);
      float dd = 0.0f;
      for (int k = 0; k < plen; ++k) {
        const int32_t pe = path[k];
        trav m;
        m.edge = pe;
        m.off0 = 0.0f;
        m.off1 = g->elen[pe];
        const float xb = start + dd;
        dd = dd + g->elen[pe];
        const float xe = start + dd;
        step_bound(B, a, lastp, p, Rd, xb, &m.t0, &m.sh0);
        step_bound(B, a, lastp, p, Rd, xe, &m.t1, &m.sh1);
        tpush(&T, m);
      }
      x = start + dd;
      cur.edge = ej;
      cur.off0 = 0.0f;
      step_bound(B, a, lastp, p, Rd, x, &cur.t0, &cur.sh0);
      curmax = oj;
    } else if (oj > curmax) {
      curmax = oj;
    }
    nstate++;
    lastp = p;
  }
  free(T.v);
  free(path);
  return rc;
}

/* ------------------------------------------------------------ S8 typed report */
static int in_lv(const int64_t* lv, int n, int64_t x) {
  for (int k = 0; k < n; ++k)
    if (lv[k] == x) return 1;
  return 0;
}
static int typed_report(batch* B, int32_t t, tres* R) {
  const orc_report_cfg* rc = B->rc;
  const double end_time = B->time[B->toff_pts[t + 1] - 1];
  orc_trace_result* o = &R->tr;
  int last_idx = R->nseg - 1;
#define ST(s) (((s).flags & 1u) ? (s).start_time : -1.0)
#define ET(s) (((s).flags & 2u) ? (s).end_time : -1.0)
  while (last_idx >= 0 && end_time - ST(R->segs[last_idx]) < rc->threshold_sec) --last_idx;
  o->shape_used = last_idx >= 0 ? R->segs[last_idx].begin_shape_index : -1;
  int have = 0, first = 1;
  const orc_segment* prior = NULL;
  int64_t prior_level = -1;
  o->successful_length = o->unreported_length = -1;
  for (int idx = 0; idx <= last_idx; ++idx) {
    const orc_segment* s = &R->segs[idx];
    const int internal = (s->flags & 4u) != 0;
    if (idx != 0 && ST(*s) == -1.0 && ET(R->segs[idx - 1]) == -1.0) o->discontinuities++;
    const int64_t level = s->segment_id >= 0 ? (s->segment_id & 7) : -1;
    if (have && prior->segment_id >= 0 && prior->length > 0 && !internal) {
      if (in_lv(rc->report_levels, rc->n_report, prior_level)) {
        const int trans = in_lv(rc->transition_levels, rc->n_transition, level);
        const double t0 = ST(*prior);
        const double t1 = trans ? ST(*s) : ET(*prior);
        const double den = t1 - t0;
        if (den == 0.0) return TERR_ZERODIV;
        const double speed = ((double)prior->length / den) * 3.6;
        if (speed < 200.0) {
          GROW(R->reps, R->nrep, R->crep, orc_report_rec);
          orc_report_rec* r = &R->reps[R->nrep++];
          memset(r, 0, sizeof *r);
          r->id = prior->segment_id;
          r->next_id = (trans && s->segment_id >= 0) ? s->segment_id : -1;
          r->t0 = t0;
          r->t1 = t1;
          if (trans && !(s->flags & 1u)) r->flags |= 1u;
          r->length = prior->length;
          r->queue_length = prior->queue_length;
          o->successful_count++;
          o->successful_length = prior->length;
        } else {
          o->invalid_speeds++;
        }
      } else {
        o->unreported_count++;
        o->unreported_length = prior->length;
      }
    }
    if (!(internal && !first)) {
      prior = s;
      prior_level = level;
      have = 1;
    }
    first = 0;
    if (s->segment_id < 0 && !internal) o->unassociated++;
  }
#undef ST
#undef ET
  return 0;
}

static void phase_b(batch* B, ws* w, int32_t t, orc_counters* C) {
  const int64_t a = B->toff_pts[t], b = B->toff_pts[t + 1];
  tres* R = &B->res[t];
  memset(R, 0, sizeof *R);
  R->tr.shape_used = -1;
  R->tr.successful_length = R->tr.unreported_length = -1;
  int err = B->terr[t];
  for (int64_t p = a; p < b; ++p) {
    B->route_dist[p] = 0.0f;
    B->ipos[p] = -1.0f;
  }
  if (!err) {
    for (int64_t p = a; p < b && !err; ++p)
      if (B->is_col[p] && B->col_prev[p] >= 0)
        if (transitions(B, w, p, C) < 0) err = TERR_SEARCH_OVERFLOW;
  }
  uint8_t* bp = (uint8_t*)malloc((size_t)(b - a) * ORC_KMAX + 1);
  if (!err) viterbi(B, t, bp);
  else
    for (int64_t p = a; p < b; ++p) B->state[p] = -1;
  free(bp);
  if (!err && segments_of_trace(B, w, t, R, C) < 0) err = TERR_SEARCH_OVERFLOW;
  if (!err) err = typed_report(B, t, R);
  if (err) {
    /* a report()-stage error (ZeroDivisionError) keeps the matched segments:
       Match succeeded, only the response is the error body */
    if (err != TERR_ZERODIV) R->nseg = R->nway = 0;
    R->nrep = 0;
    memset(&R->tr, 0, sizeof R->tr);
    R->tr.code = 500;
    R->tr.error_kind = err;
    R->tr.shape_used = -1;
    R->tr.successful_length = R->tr.unreported_length = -1;
  } else {
    R->tr.code = 200;
    C->segments_out += R->nseg;
    C->reports_out += R->nrep;
  }
}

/* ================================================================== threads */
typedef struct {
  batch* B;
  int tid;
} targ;

/* A search workspace per host thread, kept between calls (pthread key, freed
 * at thread exit): its label arrays span the graph, so allocating them per
 * call would cost O(graph) per /report request -- meili likewise keeps one
 * matcher with its label set per service thread (py/reporter_service.py:52).
 * The labels are stamp-validated, so reuse needs no clearing. */
typedef struct {
  uint64_t serial;
  ws w;
} ws_slot;
static pthread_key_t ws_key;
static pthread_once_t ws_once = PTHREAD_ONCE_INIT;
static void ws_release(ws* w) {
  free(w->ek);
  free(w->nk);
  free(w->elab);
  free(w->nlab);
  free(w->elist);
  free(w->heap);
  free(w->hits);
  memset(w, 0, sizeof *w);
}
static void ws_slot_free(void* p) {
  ws_slot* s = (ws_slot*)p;
  ws_release(&s->w);
  free(s);
}
static void ws_key_init(void) { pthread_key_create(&ws_key, ws_slot_free); }
static ws* ws_acquire(const orc_graph* g) {
  pthread_once(&ws_once, ws_key_init);
  ws_slot* s = (ws_slot*)pthread_getspecific(ws_key);
  if (!s) {
    s = (ws_slot*)calloc(1, sizeof(ws_slot));
    pthread_setspecific(ws_key, s);
  }
  if (s->serial != g->serial) {
    ws_release(&s->w);
    const size_t nn = (size_t)g->h.n_nodes, ne = (size_t)g->h.n_edges;
    s->w.ek = (uint64_t*)malloc(sizeof(uint64_t) * (ne + 1));
    s->w.nk = (uint64_t*)malloc(sizeof(uint64_t) * (nn + 1));
    s->w.elab = (uint32_t*)calloc(ne + 1, sizeof(uint32_t));
    s->w.nlab = (uint32_t*)calloc(nn + 1, sizeof(uint32_t));
    s->w.elist = (int32_t*)malloc(sizeof(int32_t) * (ne + 1));
    s->serial = g->serial;
  }
  return &s->w;
}

static void* worker(void* arg) {
  targ* A = (targ*)arg;
  batch* B = A->B;
  ws* w = ws_acquire(B->g);
  orc_counters* C = &B->ctr[A->tid];
  while (1) {
    int t = atomic_fetch_add(&B->next, 1);
    if (t >= B->n_traces) break;
    if (B->phase == 0) phase_a(B, w, t, C);
    else phase_b(B, w, t, C);
  }
  return NULL;
}

static void run_phase(batch* B, int phase, int nthreads) {
  B->phase = phase;
  atomic_store(&B->next, 0);
  if (nthreads <= 1) {
    targ a = {B, 0};
    worker(&a);
    return;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  targ* args = (targ*)malloc(sizeof(targ) * (size_t)nthreads);
  for (int i = 0; i < nthreads; ++i) {
    args[i].B = B;
    args[i].tid = i;
    pthread_create(&th[i], NULL, worker, &args[i]);
  }
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  free(th);
  free(args);
}

int orc_match_batch(const orc_graph* g, const orc_params* p, const orc_report_cfg* rc, int32_t n_traces,
                    const int64_t* trace_off, const float* lat, const float* lon, const double* time,
                    const float* accuracy, int nthreads, int keep_stages, orc_results* out) {
  memset(out, 0, sizeof *out);
  if (p->max_candidates < 1 || p->max_candidates > ORC_KMAX) return -1;
  if (nthreads < 1) nthreads = 1;
  const int64_t P = trace_off[n_traces];
  batch B;
  memset(&B, 0, sizeof B);
  B.g = g;
  B.P = p;
  B.rc = rc;
  B.n_traces = n_traces;
  B.toff_pts = trace_off;
  B.lat = lat;
  B.lon = lon;
  B.time = time;
  B.acc = accuracy;
  B.count_unique = keep_stages;
  B.elen64 = g->elen64;
  {
    /* the turn table per thread, rebuilt only when the factor changes (181
     * transcendental evaluations would otherwise dominate a short request) */
    static __thread uint32_t tu[181];
    static __thread uint32_t tu_bits;
    static __thread int tu_ok;
    uint32_t bits;
    memcpy(&bits, &p->turn_penalty_factor, 4);
    if (!tu_ok || bits != tu_bits) {
      for (int d = 0; d <= 180; ++d) tu[d] = orc_turn_units(p->turn_penalty_factor, d);
      tu_bits = bits;
      tu_ok = 1;
    }
    memcpy(B.turn_units, tu, sizeof tu);
  }
  const size_t PP = (size_t)P + 1;
  B.is_col = (uint8_t*)calloc(PP, 1);
  B.chain_start = (uint8_t*)calloc(PP, 1);
  B.ncand = (int32_t*)calloc(PP, 4);
  B.cand_edge = (int32_t*)calloc(PP * ORC_KMAX, 4);
  B.cand_off = (float*)calloc(PP * ORC_KMAX, 4);
  B.cand_emis = (float*)calloc(PP * ORC_KMAX, 4);
  B.state = (int32_t*)calloc(PP, 4);
  B.col_prev = (int32_t*)calloc(PP, 4);
  B.route_dist = (float*)calloc(PP, 4);
  B.gc = (float*)calloc(PP, 4);
  B.ipos = (float*)calloc(PP, 4);
  B.terr = (int32_t*)calloc((size_t)n_traces + 1, 4);
  B.trans_off = (int64_t*)calloc(PP, 8);
  B.res = (tres*)calloc((size_t)n_traces + 1, sizeof(tres));
  B.ctr = (orc_counters*)calloc((size_t)nthreads, sizeof(orc_counters));
  run_phase(&B, 0, nthreads);
  /* transition matrix offsets, point order */
  int64_t acc = 0;
  for (int64_t q = 0; q < P; ++q) {
    B.trans_off[q] = acc;
    if (B.is_col[q] && B.col_prev[q] >= 0) acc += (int64_t)B.ncand[B.col_prev[q]] * B.ncand[q];
  }
  B.trans_off[P] = acc;
  B.trans = (float*)malloc(sizeof(float) * (size_t)(acc + 1));
  run_phase(&B, 1, nthreads);
  /* gather */
  out->n_traces = n_traces;
  out->traces = (orc_trace_result*)calloc((size_t)n_traces + 1, sizeof(orc_trace_result));
  int64_t ns = 0, nw = 0, nr = 0;
  for (int32_t t = 0; t < n_traces; ++t) {
    ns += B.res[t].nseg;
    nw += B.res[t].nway;
    nr += B.res[t].nrep;
  }
  out->segments = (orc_segment*)calloc((size_t)ns + 1, sizeof(orc_segment));
  out->way_ids = (int64_t*)calloc((size_t)nw + 1, 8);
  out->reports = (orc_report_rec*)calloc((size_t)nr + 1, sizeof(orc_report_rec));
  ns = nw = nr = 0;
  for (int32_t t = 0; t < n_traces; ++t) {
    tres* R = &B.res[t];
    out->traces[t] = R->tr;
    out->traces[t].seg_off = (int32_t)ns;
    out->traces[t].seg_cnt = R->nseg;
    out->traces[t].rep_off = (int32_t)nr;
    out->traces[t].rep_cnt = R->nrep;
    for (int k = 0; k < R->nseg; ++k) {
      out->segments[ns + k] = R->segs[k];
      out->segments[ns + k].way_off += (int32_t)nw;
    }
    /* (count 0 leaves the source NULL: memcpy's arguments must not be) */
    if (R->nway) memcpy(out->way_ids + nw, R->ways, sizeof(int64_t) * (size_t)R->nway);
    if (R->nrep) memcpy(out->reports + nr, R->reps, sizeof(orc_report_rec) * (size_t)R->nrep);
    ns += R->nseg;
    nw += R->nway;
    nr += R->nrep;
    free(R->segs);
    free(R->ways);
    free(R->reps);
  }
  out->n_segments = (int32_t)ns;
  out->n_way_ids = (int32_t)nw;
  out->n_reports = (int32_t)nr;
  for (int i = 0; i < nthreads; ++i) {
    const int64_t* s = (const int64_t*)&B.ctr[i];
    int64_t* d = (int64_t*)&out->counters;
    for (size_t k = 0; k < sizeof(orc_counters) / 8; ++k) d[k] += s[k];
  }
  out->n_points = P;
  if (keep_stages) {
    out->ncand = B.ncand;
    out->cand_edge = B.cand_edge;
    out->cand_off = B.cand_off;
    out->cand_emis = B.cand_emis;
    out->trans_off = B.trans_off;
    out->trans = B.trans;
    out->state = B.state;
    out->col_prev = B.col_prev;
    out->route_dist = B.route_dist;
    out->gc = B.gc;
    out->ipos = B.ipos;
  } else {
    free(B.ncand);
    free(B.cand_edge);
    free(B.cand_off);
    free(B.cand_emis);
    free(B.trans_off);
    free(B.trans);
    free(B.state);
    free(B.col_prev);
    free(B.route_dist);
    free(B.gc);
    free(B.ipos);
  }
  free(B.is_col);
  free(B.chain_start);
  free(B.terr);
  free(B.res);
  free(B.ctr);
  return 0;
}

void orc_results_free(orc_results* r) {
  free(r->traces);
  free(r->segments);
  free(r->reports);
  free(r->way_ids);
  free(r->ncand);
  free(r->cand_edge);
  free(r->cand_off);
  free(r->cand_emis);
  free(r->trans_off);
  free(r->trans);
  free(r->state);
  free(r->col_prev);
  free(r->route_dist);
  free(r->gc);
  free(r->ipos);
  memset(r, 0, sizeof *r);
}

/* ================================================================== JSON Match */
static int num_of(const jv* v, double* d) {
  if (!v || (v->t != JV_INT && v->t != JV_FLOAT)) return 0;
  *d = v->t == JV_INT ? (double)v->i : v->d;
  return 1;
}

/* segments JSON of one trace (key order of README.md:136) */
static void write_segments(sbuf* out, const orc_results* r, int32_t t) {
  const orc_trace_result* tr = &r->traces[t];
  sb_puts(out, "{\"segments\":[");
  for (int k = 0; k < tr->seg_cnt; ++k) {
    const orc_segment* s = &r->segments[tr->seg_off + k];
    if (k) sb_puts(out, ",");
    sb_puts(out, "{");
    if (s->segment_id >= 0) sb_printf(out, "\"segment_id\":%lld,", (long long)s->segment_id);
    sb_puts(out, "\"way_ids\":[");
    for (int w = 0; w < s->way_cnt; ++w) sb_printf(out, w ? ",%lld" : "%lld", (long long)r->way_ids[s->way_off + w]);
    sb_puts(out, "],\"start_time\":");
    if (s->flags & 1u) py_float_repr(out, s->start_time);
    else sb_puts(out, "-1");
    sb_puts(out, ",\"end_time\":");
    if (s->flags & 2u) py_float_repr(out, s->end_time);
    else sb_puts(out, "-1");
    sb_printf(out, ",\"queue_length\":%d,\"length\":%d,\"internal\":%s,\"begin_shape_index\":%d,\"end_shape_index\":%d}",
              s->queue_length, s->length, (s->flags & 4u) ? "true" : "false", s->begin_shape_index,
              s->end_shape_index);
  }
  sb_puts(out, "]}");
}

int orc_match_dom(const orc_graph* g, const orc_params* p, const jv* req, sbuf* out, char** err) {
  const jv* tr = jv_get(req, "trace");
  if (!tr || tr->t != JV_ARR) {
    *err = strdup("trace must be an array of points");
    return 0;
  }
  const int64_t n = (int64_t)tr->n;
  float* lat = (float*)malloc(sizeof(float) * (size_t)(n + 1));
  float* lon = (float*)malloc(sizeof(float) * (size_t)(n + 1));
  float* acc = (float*)malloc(sizeof(float) * (size_t)(n + 1));
  double* tm = (double*)malloc(sizeof(double) * (size_t)(n + 1));
  for (int64_t k = 0; k < n; ++k) {
    const jv* pt = tr->items[k];
    double la, lo, ti, ac;
    if (!pt || pt->t != JV_OBJ || !num_of(jv_get(pt, "lat"), &la) || !num_of(jv_get(pt, "lon"), &lo) ||
        !num_of(jv_get(pt, "time"), &ti)) {
      char buf[128];
      snprintf(buf, sizeof buf, "trace point %lld must have numeric lat, lon and time", (long long)k);
      *err = strdup(buf);
      free(lat);
      free(lon);
      free(acc);
      free(tm);
      return 0;
    }
    lat[k] = (float)la;
    lon[k] = (float)lo;
    tm[k] = ti;
    acc[k] = num_of(jv_get(pt, "accuracy"), &ac) ? (float)ac : 0.0f;
  }
  int64_t off[2] = {0, n};
  orc_report_cfg rc;
  orc_report_cfg_default(&rc);
  orc_results r;
  orc_match_batch(g, p, &rc, 1, off, lat, lon, tm, acc, 1, 0, &r);
  free(lat);
  free(lon);
  free(acc);
  free(tm);
  int ok = 1;
  if (r.traces[0].code == 500 && r.traces[0].error_kind != TERR_ZERODIV) {
    *err = strdup(terr_msg(r.traces[0].error_kind));
    ok = 0;
  } else {
    write_segments(out, &r, 0);
  }
  orc_results_free(&r);
  return ok;
}

/* ================================================================== JSON batch (CPU baseline) */
typedef struct {
  const orc_graph* g;
  const orc_params* p;
  const orc_report_cfg* rc;
  int n;
  const char* const* bodies;
  const size_t* lens;
  int* codes;
  char** outs;
  size_t* out_lens;
  atomic_int next;
} jbatch;

static void* jworker(void* arg) {
  jbatch* J = (jbatch*)arg;
  while (1) {
    int i = atomic_fetch_add(&J->next, 1);
    if (i >= J->n) break;
    J->codes[i] = orc_handle_request(J->g, J->p, J->rc, "/report", J->bodies[i], J->lens[i], &J->outs[i],
                                     &J->out_lens[i]);
  }
  return NULL;
}

int orc_handle_batch(const orc_graph* g, const orc_params* p, const orc_report_cfg* rc, int n,
                     const char* const* bodies, const size_t* lens, int nthreads, int* codes, char** outs,
                     size_t* out_lens) {
  jbatch J = {g, p, rc, n, bodies, lens, codes, outs, out_lens, 0};
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, jworker, &J);
  for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
  free(th);
  return 0;
}

int orc_batcher_handler(void* ctx, int n, const char* const* reqs, const size_t* lens, char** resps,
                        size_t* resp_lens, int* codes) {
  const orc_handler_ctx* c = (const orc_handler_ctx*)ctx;
  return orc_handle_batch(c->g, c->p, c->rc, n, reqs, lens, c->nthreads, codes, resps, resp_lens);
}

/* ================================================================== polyline6 */
/* py/generate_test_trace.py:9-29 */
int64_t orc_decode_polyline6(const char* enc, size_t len, double* out, int64_t max_pairs) {
  int64_t prev[2] = {0, 0}, n = 0;
  size_t i = 0;
  while (i < len) {
    int64_t ll[2] = {0, 0};
    for (int j = 0; j < 2; ++j) {
      int shift = 0;
      int64_t byte = 0x20;
      while (byte >= 0x20) {
        if (i >= len) return -1;
        byte = (int64_t)(unsigned char)enc[i++] - 63;
        ll[j] |= (byte & 0x1f) << shift;
        shift += 5;
      }
      ll[j] = prev[j] + ((ll[j] & 1) ? ~(ll[j] >> 1) : (ll[j] >> 1));
      prev[j] = ll[j];
    }
    if (n < max_pairs) {
      char buf[64];
      const double inv = 1.0 / 1e6;
      snprintf(buf, sizeof buf, "%.6f", (double)ll[1] * inv);
      out[2 * n] = strtod(buf, NULL);
      snprintf(buf, sizeof buf, "%.6f", (double)ll[0] * inv);
      out[2 * n + 1] = strtod(buf, NULL);
    }
    ++n;
  }
  return n;
}
