// synth_graph.cpp -- seeded synthetic road network -> flat .otmg file.
//
// No Valhalla tiles exist in this environment, so the graph
// every config runs on is generated here, to the recipe of SURVEY.md §8(d):
// a perturbed Manhattan grid (block_m +- jitter_m), curved polylines of 2-6
// shape points, two-way streets, level 2 locals / level 1 every
// `arterial_every` line / level 0 every `highway_every` line, OSMLR segments
// = maximal same-line chains of associated edges <= seg_max_m, tile ids from
// py/get_tiles.py's hierarchy math (:30-72: 4 / 1 / 0.25 degree levels), and
// internal edges (4-node squares at crossings of `complex_every` lines) with
// no segment.  Output is the flat format of include/otm_graph_format.h, the
// stand-in for what valhalla.Configure loads (py/reporter_service.py:279).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "otm_graph_format.h"
#include "otm_internal.h"
#include "otmatch.h"

namespace otm {

namespace {

const double kMpd = 20037581.187 / 180.0;  // Batch.java:33
const double kPi = 3.14159265358979323846;

struct Pt {
  double x, y;  // metres, local frame
};

struct EdgeBuild {
  int from, to;
  std::vector<Pt> shape;
  int level;
  float speed;
  int64_t way;
  bool internal;
  bool assoc;
  int line_kind;  // 0 horizontal, 1 vertical, 2 internal
  int line;       // line index
  int pos;        // index along the line
  int dir;        // +1 increasing index, -1 decreasing
  int opp;        // index of reverse edge in build order
  // filled later
  std::vector<float> lat, lon, cum;
  int seg = -1, seg_pos = -1;
  unsigned flags = 0;
};

int line_level(int idx, int art, int hwy) {
  if (hwy > 0 && idx % hwy == 0) return 0;
  if (art > 0 && idx % art == 0) return 1;
  return 2;
}

float level_speed(int level) { return level == 0 ? 90.f : (level == 1 ? 50.f : 30.f); }

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

int synth_graph_write(const otm_synth_graph_params* p, const char* out_path, std::string* err) {
  if (p->block_m <= 2 * p->jitter_m + 30 || p->width_m < p->block_m || p->height_m < p->block_m) {
    *err = "synth_graph: invalid geometry parameters";
    return OTM_EINVAL;
  }
  Rng rng(p->seed);
  const int nc = (int)std::floor(p->width_m / p->block_m) + 1;
  const int nr = (int)std::floor(p->height_m / p->block_m) + 1;
  const double cos0 = std::cos(p->center_lat * kPi / 180.0);
  auto to_lat = [&](double y) { return p->center_lat + (y - p->height_m * 0.5) / kMpd; };
  auto to_lon = [&](double x) { return p->center_lon + (x - p->width_m * 0.5) / (kMpd * cos0); };

  // ---- nodes
  std::vector<Pt> node_pos;
  std::vector<int> gp_first(nr * nc);  // first node id of grid point
  std::vector<char> gp_complex(nr * nc, 0);
  for (int i = 0; i < nr; ++i) {
    for (int j = 0; j < nc; ++j) {
      double x = j * p->block_m + rng.uni(-p->jitter_m, p->jitter_m);
      double y = i * p->block_m + rng.uni(-p->jitter_m, p->jitter_m);
      bool cx = p->complex_every > 0 && i % p->complex_every == 0 && j % p->complex_every == 0;
      gp_first[i * nc + j] = (int)node_pos.size();
      gp_complex[i * nc + j] = cx;
      if (!cx) {
        node_pos.push_back({x, y});
      } else {  // SW, SE, NE, NW corners of a 20 m square
        node_pos.push_back({x - 10, y - 10});
        node_pos.push_back({x + 10, y - 10});
        node_pos.push_back({x + 10, y + 10});
        node_pos.push_back({x - 10, y + 10});
      }
    }
  }
  // side: 0 E, 1 N, 2 W, 3 S  ->  complex attach corner: E->NE(2) N->NW(3) W->SW(0) S->SE(1)
  auto attach = [&](int i, int j, int side) {
    int b = gp_first[i * nc + j];
    if (!gp_complex[i * nc + j]) return b;
    static const int corner[4] = {2, 3, 0, 1};
    return b + corner[side];
  };

  // ---- edges (build order)
  std::vector<EdgeBuild> E;
  auto add_street = [&](int a, int b, int kind, int line, int pos, int level, bool assoc, int64_t way) {
    Pt A = node_pos[a], B = node_pos[b];
    int k = (int)(rng.next() % 5);  // 0..4 interior points
    double amp = k ? rng.uni(-12.0, 12.0) : 0.0;
    double dx = B.x - A.x, dy = B.y - A.y, L = std::sqrt(dx * dx + dy * dy);
    double nx = -dy / L, ny = dx / L;
    std::vector<Pt> sh;
    sh.push_back(A);
    for (int m = 1; m <= k; ++m) {
      double f = (double)m / (k + 1);
      double o = amp * std::sin(kPi * f) + rng.uni(-2.0, 2.0);
      sh.push_back({A.x + f * dx + nx * o, A.y + f * dy + ny * o});
    }
    sh.push_back(B);
    EdgeBuild f{};
    f.from = a;
    f.to = b;
    f.shape = sh;
    f.level = level;
    f.speed = level_speed(level);
    f.way = way;
    f.internal = false;
    f.assoc = assoc;
    f.line_kind = kind;
    f.line = line;
    f.pos = pos;
    f.dir = +1;
    EdgeBuild r = f;
    r.from = b;
    r.to = a;
    std::reverse(r.shape.begin(), r.shape.end());
    r.dir = -1;
    f.opp = (int)E.size() + 1;
    r.opp = (int)E.size();
    E.push_back(f);
    E.push_back(r);
  };
  for (int i = 0; i < nr; ++i) {
    int lvl = line_level(i, p->arterial_every, p->highway_every);
    for (int j = 0; j + 1 < nc; ++j) {
      bool assoc = !(lvl == 2 && rng.uni() < p->unassoc_frac);
      int64_t way = (1ll << 40) | ((int64_t)i << 20) | (j / 3);
      add_street(attach(i, j, 0), attach(i, j + 1, 2), 0, i, j, lvl, assoc, way);
    }
  }
  for (int j = 0; j < nc; ++j) {
    int lvl = line_level(j, p->arterial_every, p->highway_every);
    for (int i = 0; i + 1 < nr; ++i) {
      bool assoc = !(lvl == 2 && rng.uni() < p->unassoc_frac);
      int64_t way = (2ll << 40) | ((int64_t)j << 20) | (i / 3);
      add_street(attach(i, j, 1), attach(i + 1, j, 3), 1, j, i, lvl, assoc, way);
    }
  }
  for (int g = 0; g < nr * nc; ++g) {
    if (!gp_complex[g]) continue;
    int b = gp_first[g];
    for (int s = 0; s < 4; ++s) {
      int a = b + s, c = b + (s + 1) % 4;
      EdgeBuild f{};
      f.from = a;
      f.to = c;
      f.shape = {node_pos[a], node_pos[c]};
      f.level = 1;
      f.speed = 25.f;
      f.way = (3ll << 40) | (int64_t)b;
      f.internal = true;
      f.assoc = false;
      f.line_kind = 2;
      f.line = g;
      f.pos = s;
      f.dir = +1;
      EdgeBuild r = f;
      r.from = c;
      r.to = a;
      std::reverse(r.shape.begin(), r.shape.end());
      r.dir = -1;
      f.opp = (int)E.size() + 1;
      r.opp = (int)E.size();
      E.push_back(f);
      E.push_back(r);
    }
  }

  // ---- geometry to float lat/lon + cumulative lengths
  for (auto& e : E) {
    size_t n = e.shape.size();
    e.lat.resize(n);
    e.lon.resize(n);
    e.cum.resize(n);
    double cum = 0.0;
    for (size_t k = 0; k < n; ++k) {
      e.lat[k] = (float)to_lat(e.shape[k].y);
      e.lon[k] = (float)to_lon(e.shape[k].x);
      if (k > 0) {
        double la0 = e.lat[k - 1], la1 = e.lat[k];
        double mid = 0.5 * (la0 + la1) * kPi / 180.0;
        double dx = ((double)e.lon[k] - (double)e.lon[k - 1]) * kMpd * std::cos(mid);
        double dy = (la1 - la0) * kMpd;
        cum += std::sqrt(dx * dx + dy * dy);
      }
      e.cum[k] = (float)cum;
    }
    if (e.cum[n - 1] < 1.0f) {
      *err = "synth_graph: degenerate edge";
      return OTM_EINVAL;
    }
  }

  // ---- OSMLR segments: walk each line in each direction
  struct SegB {
    int level;
    int first_edge_build;
    std::vector<int> edges;
    double len;
  };
  std::vector<SegB> segs;
  // index street edges per (kind, line, pos, dir)
  std::map<std::tuple<int, int, int, int>, int> street;
  for (int k = 0; k < (int)E.size(); ++k)
    if (E[k].line_kind < 2) street[std::make_tuple(E[k].line_kind, E[k].line, E[k].pos, E[k].dir)] = k;
  auto gp_of_join = [&](int kind, int line, int pos_between) {
    // grid point between street pos-1 and pos along a line
    return kind == 0 ? line * nc + pos_between : pos_between * nc + line;
  };
  for (int kind = 0; kind < 2; ++kind) {
    int nlines = kind == 0 ? nr : nc;
    int npos = kind == 0 ? nc - 1 : nr - 1;
    for (int line = 0; line < nlines; ++line) {
      for (int dir = +1; dir >= -1; dir -= 2) {
        SegB cur{};
        cur.len = 0;
        auto flush = [&]() {
          if (!cur.edges.empty()) segs.push_back(cur);
          cur = SegB{};
          cur.len = 0;
        };
        for (int s = 0; s < npos; ++s) {
          int pos = dir > 0 ? s : npos - 1 - s;
          int k = street[std::make_tuple(kind, line, pos, dir)];
          // break where the line crosses a complex intersection (internal edges between)
          if (s > 0) {
            int join = dir > 0 ? pos : pos + 1;
            if (gp_complex[gp_of_join(kind, line, join)]) flush();
          }
          if (!E[k].assoc) {
            flush();
            continue;
          }
          double L = E[k].cum.back();
          if (!cur.edges.empty() && cur.len + L > p->seg_max_m) flush();
          if (cur.edges.empty()) cur.level = E[k].level;
          cur.edges.push_back(k);
          cur.len += L;
        }
        flush();
      }
    }
  }
  std::map<std::pair<int, int64_t>, int64_t> tile_count;
  std::vector<uint64_t> seg_id(segs.size());
  std::vector<float> seg_len(segs.size());
  for (size_t g = 0; g < segs.size(); ++g) {
    auto& s = segs[g];
    const auto& e0 = E[s.edges[0]];
    int64_t t = otm::tile_id(s.level, e0.lat[0], e0.lon[0]);  // tiles.cpp (py/get_tiles.py:51-72)
    int64_t idx = tile_count[{s.level, t}]++;
    seg_id[g] = (uint64_t)s.level | ((uint64_t)t << 3) | ((uint64_t)idx << 25);
    float acc = 0.f;
    for (size_t m = 0; m < s.edges.size(); ++m) {
      auto& e = E[s.edges[m]];
      e.seg = (int)g;
      e.seg_pos = (int)m;
      if (m == 0) e.flags |= OTM_EDGE_SEG_BEGIN;
      if (m + 1 == s.edges.size()) e.flags |= OTM_EDGE_SEG_END;
      acc += e.cum.back();
    }
    seg_len[g] = acc;
  }
  for (auto& e : E)
    if (e.internal) e.flags |= OTM_EDGE_INTERNAL;

  // ---- CSR order: sort edges by (from, to, build index)
  const int NE = (int)E.size(), NN = (int)node_pos.size();
  std::vector<int> order(NE), rank(NE);
  for (int k = 0; k < NE; ++k) order[k] = k;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    if (E[a].from != E[b].from) return E[a].from < E[b].from;
    return E[a].to < E[b].to;
  });
  for (int k = 0; k < NE; ++k) rank[order[k]] = k;

  std::vector<float> nlat(NN), nlon(NN);
  for (int n = 0; n < NN; ++n) {
    nlat[n] = (float)to_lat(node_pos[n].y);
    nlon[n] = (float)to_lon(node_pos[n].x);
  }
  std::vector<int32_t> out_off(NN + 1, 0), efrom(NE), eto(NE), eshape_off(NE + 1), eseg(NE), eseg_pos(NE),
      eopp(NE);
  std::vector<float> elen(NE), espeed(NE);
  std::vector<int64_t> eway(NE);
  std::vector<uint8_t> eflags(NE), elevel(NE);
  std::vector<uint16_t> ehead_out(NE), ehead_in(NE);
  // bearing (whole degrees, clockwise from north) of shape segment a -> b
  auto bearing = [&](float la0, float lo0, float la1, float lo1) {
    const double mid = 0.5 * ((double)la0 + (double)la1) * kPi / 180.0;
    const double dx = ((double)lo1 - (double)lo0) * kMpd * std::cos(mid);
    const double dy = ((double)la1 - (double)la0) * kMpd;
    double b = std::atan2(dx, dy) * 180.0 / kPi;
    long r = std::lround(b < 0.0 ? b + 360.0 : b);
    return (uint16_t)(r % 360);
  };
  std::vector<float> slat, slon, scum;
  for (int k = 0; k < NE; ++k) {
    const auto& e = E[order[k]];
    efrom[k] = e.from;
    eto[k] = e.to;
    elen[k] = e.cum.back();
    eshape_off[k] = (int32_t)slat.size();
    for (size_t m = 0; m < e.lat.size(); ++m) {
      slat.push_back(e.lat[m]);
      slon.push_back(e.lon[m]);
      scum.push_back(e.cum[m]);
    }
    eway[k] = e.way;
    eseg[k] = e.seg;
    eseg_pos[k] = e.seg_pos;
    eflags[k] = (uint8_t)e.flags;
    elevel[k] = (uint8_t)e.level;
    espeed[k] = e.speed;
    eopp[k] = rank[e.opp];
    const size_t ns = e.lat.size();
    ehead_out[k] = bearing(e.lat[0], e.lon[0], e.lat[1], e.lon[1]);
    ehead_in[k] = bearing(e.lat[ns - 2], e.lon[ns - 2], e.lat[ns - 1], e.lon[ns - 1]);
    out_off[e.from + 1]++;
  }
  eshape_off[NE] = (int32_t)slat.size();
  for (int n = 0; n < NN; ++n) out_off[n + 1] += out_off[n];
  const int NG = (int)segs.size();
  std::vector<int32_t> gfirst(NG), gnedges(NG);
  for (int g = 0; g < NG; ++g) {
    gfirst[g] = rank[segs[g].edges[0]];
    gnedges[g] = (int32_t)segs[g].edges.size();
  }

  // ---- grid index
  double minlat = 1e9, minlon = 1e9, maxlat = -1e9, maxlon = -1e9;
  for (size_t s = 0; s < slat.size(); ++s) {
    minlat = std::min(minlat, (double)slat[s]);
    maxlat = std::max(maxlat, (double)slat[s]);
    minlon = std::min(minlon, (double)slon[s]);
    maxlon = std::max(maxlon, (double)slon[s]);
  }
  const double cell = p->cell_deg;
  const double lat0 = std::floor(minlat / cell) * cell - cell;
  const double lon0 = std::floor(minlon / cell) * cell - cell;
  const int rows = (int)std::ceil((maxlat - lat0) / cell) + 2;
  const int cols = (int)std::ceil((maxlon - lon0) / cell) + 2;
  std::vector<int64_t> cell_off((size_t)rows * cols + 1, 0);
  auto for_cells = [&](int k, int s, auto&& fn) {
    int a = eshape_off[k] + s;
    double la0 = std::min(slat[a], slat[a + 1]), la1 = std::max(slat[a], slat[a + 1]);
    double lo0 = std::min(slon[a], slon[a + 1]), lo1 = std::max(slon[a], slon[a + 1]);
    int r0 = (int)std::floor((la0 - lat0) / cell), r1 = (int)std::floor((la1 - lat0) / cell);
    int c0 = (int)std::floor((lo0 - lon0) / cell), c1 = (int)std::floor((lo1 - lon0) / cell);
    for (int r = r0; r <= r1; ++r)
      for (int c = c0; c <= c1; ++c) fn((size_t)r * cols + c);
  };
  for (int k = 0; k < NE; ++k) {
    int nseg = eshape_off[k + 1] - eshape_off[k] - 1;
    if (nseg > OTM_MAX_EDGE_SHAPE_SEGS) {
      *err = "synth_graph: too many shape points";
      return OTM_EINVAL;
    }
    for (int s = 0; s < nseg; ++s) for_cells(k, s, [&](size_t c) { cell_off[c + 1]++; });
  }
  for (size_t c = 0; c < (size_t)rows * cols; ++c) cell_off[c + 1] += cell_off[c];
  std::vector<uint32_t> cell_ent(cell_off.back());
  {
    std::vector<int64_t> fill(cell_off.begin(), cell_off.end() - 1);
    for (int k = 0; k < NE; ++k) {
      int nseg = eshape_off[k + 1] - eshape_off[k] - 1;
      for (int s = 0; s < nseg; ++s)
        for_cells(k, s, [&](size_t c) { cell_ent[fill[c]++] = ((uint32_t)k << 4) | (uint32_t)s; });
    }
  }

  // ---- write
  otmg_header h;
  std::memset(&h, 0, sizeof(h));
  std::memcpy(h.magic, OTMG_MAGIC, 8);
  h.version = OTMG_VERSION;
  h.header_bytes = sizeof(h);
  h.n_nodes = NN;
  h.n_edges = NE;
  h.n_shape = (int32_t)slat.size();
  h.n_segments = NG;
  h.grid_rows = rows;
  h.grid_cols = cols;
  h.n_cell_entries = (int64_t)cell_ent.size();
  h.grid_lat0 = lat0;
  h.grid_lon0 = lon0;
  h.grid_cell_deg = cell;
  double nb[4] = {1e9, 1e9, -1e9, -1e9};
  for (int n = 0; n < NN; ++n) {
    nb[0] = std::min(nb[0], (double)nlat[n]);
    nb[1] = std::min(nb[1], (double)nlon[n]);
    nb[2] = std::max(nb[2], (double)nlat[n]);
    nb[3] = std::max(nb[3], (double)nlon[n]);
  }
  std::memcpy(h.bbox, nb, sizeof(nb));
  h.seed = p->seed;
  struct Sec {
    const void* ptr;
    size_t bytes;
  } secs[OTMG_NUM_SECTIONS] = {
      {nlat.data(), (size_t)NN * 4},          {nlon.data(), (size_t)NN * 4},          {out_off.data(), ((size_t)NN + 1) * 4},
      {efrom.data(), (size_t)NE * 4},         {eto.data(), (size_t)NE * 4},           {elen.data(), (size_t)NE * 4},
      {eshape_off.data(), ((size_t)NE + 1) * 4}, {eway.data(), (size_t)NE * 8},       {eseg.data(), (size_t)NE * 4},
      {eseg_pos.data(), (size_t)NE * 4},      {eflags.data(), (size_t)NE},    {elevel.data(), (size_t)NE},
      {espeed.data(), (size_t)NE * 4},        {eopp.data(), (size_t)NE * 4},          {slat.data(), slat.size() * 4},
      {slon.data(), slon.size() * 4}, {scum.data(), scum.size() * 4}, {seg_id.data(), (size_t)NG * 8},
      {seg_len.data(), (size_t)NG * 4},       {gfirst.data(), (size_t)NG * 4},        {gnedges.data(), (size_t)NG * 4},
      {cell_off.data(), cell_off.size() * 8}, {cell_ent.data(), cell_ent.size() * 4},
      {ehead_out.data(), (size_t)NE * 2},     {ehead_in.data(), (size_t)NE * 2},
  };
  size_t off = align256(sizeof(h));
  for (int s = 0; s < OTMG_NUM_SECTIONS; ++s) {
    h.sec[s].offset = off;
    h.sec[s].bytes = secs[s].bytes;
    off = align256(off + secs[s].bytes);
  }
  FILE* f = std::fopen(out_path, "wb");
  if (!f) {
    *err = std::string("synth_graph: cannot open ") + out_path;
    return OTM_EIO;
  }
  std::vector<char> zeros(256, 0);
  bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1;
  size_t pos = sizeof(h);
  for (int s = 0; s < OTMG_NUM_SECTIONS && ok; ++s) {
    if (h.sec[s].offset > pos) ok = std::fwrite(zeros.data(), 1, h.sec[s].offset - pos, f) == h.sec[s].offset - pos;
    pos = h.sec[s].offset;
    if (ok && secs[s].bytes) ok = std::fwrite(secs[s].ptr, 1, secs[s].bytes, f) == secs[s].bytes;
    pos += secs[s].bytes;
  }
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) {
    *err = "synth_graph: write failed";
    return OTM_EIO;
  }
  return OTM_OK;
}

}  // namespace otm

extern "C" void otm_synth_graph_defaults(otm_synth_graph_params* p) {
  p->center_lat = 37.98;
  p->center_lon = 23.72;
  p->width_m = 20000;
  p->height_m = 20000;
  p->block_m = 150;
  p->jitter_m = 20;
  p->arterial_every = 8;
  p->highway_every = 32;
  p->unassoc_frac = 0.05;
  p->complex_every = 8;
  p->seg_max_m = 1000;
  p->cell_deg = 0.25 / 500.0;
  p->seed = 20171015ull;
}

extern "C" int otm_synth_graph(const otm_synth_graph_params* p, const char* out_path) {
  std::string err;
  int rc = otm::synth_graph_write(p, out_path, &err);
  if (rc) otm::set_thread_error(err);
  return rc;
}
