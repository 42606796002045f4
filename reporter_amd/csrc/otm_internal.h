// otm_internal.h -- shared host-side declarations of libotmatch.
#pragma once
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "otm_graph_format.h"
#include "otmatch.h"

namespace otm {

// ------------------------------------------------------------ errors
void set_thread_error(const std::string& msg);
const char* thread_error();

// ------------------------------------------------------------ rng (splitmix64)
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  double uni(double a, double b) { return a + (b - a) * uni(); }
  double normal() {  // Box-Muller
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

int synth_graph_write(const otm_synth_graph_params* p, const char* out_path, std::string* err);

// ------------------------------------------------------------ tile hierarchy (tiles.cpp, py/get_tiles.py:30-102)
int64_t tile_row(int level, double lat);
int64_t tile_col(int level, double lon);
int64_t tile_id(int level, double lat, double lon);  // -1 outside the world bbox
std::string tile_file(int64_t id, int level, const char* suffix);

// ------------------------------------------------------------ host graph view
// A read-only view over a mapped .otmg file (sections point into the map).
struct HostGraph {
  otmg_header h{};
  void* map = nullptr;
  size_t map_bytes = 0;
  const float *node_lat = nullptr, *node_lon = nullptr;
  const int32_t* out_off = nullptr;
  const int32_t *e_from = nullptr, *e_to = nullptr;
  const float* e_len = nullptr;
  const int32_t* e_shape_off = nullptr;
  const int64_t* e_way = nullptr;
  const int32_t *e_seg = nullptr, *e_seg_pos = nullptr;
  const uint8_t *e_flags = nullptr, *e_level = nullptr;
  const float* e_speed = nullptr;
  const int32_t* e_opp = nullptr;
  const float *s_lat = nullptr, *s_lon = nullptr, *s_cum = nullptr;
  const uint64_t* g_id = nullptr;
  const float* g_len = nullptr;
  const int32_t *g_first = nullptr, *g_nedges = nullptr;
  const int64_t* cell_off = nullptr;
  const uint32_t* cell_ent = nullptr;
  const uint16_t *e_head_out = nullptr, *e_head_in = nullptr;

  const void* section(int s) const { return (const char*)map + h.sec[s].offset; }
  ~HostGraph();
};
// Maps and validates the file.  Returns 0 or OTM_EIO with *err set.
int load_graph(const char* path, HostGraph* g, std::string* err);

// ------------------------------------------------------------ matcher config
struct MatchConfig {
  float sigma_z = 4.07f;
  float beta = 3.0f;
  float max_route_distance_factor = 5.0f;
  float breakage_distance = 2000.0f;
  float interpolation_distance = 10.0f;
  float search_radius = 50.0f;
  float max_search_radius = 100.0f;
  float gps_accuracy = 5.0f;
  int max_candidates = 32;
  // meili's turn penalty (auto costing: 200; the default costing's is 0):
  // the transition cost is (turn_cost + |route - gc|) / beta
  float turn_penalty_factor = 200.0f;
};

// reporter_service.py make_thread_locals (:51-62) state
struct ReportConfig {
  std::vector<int64_t> report_levels{0, 1};
  std::vector<int64_t> transition_levels{0, 1};
  // threshold_sec: int 15 by default, or bool True/False (== 1 / 0)
  double threshold_sec = 15.0;
  bool in_report(int64_t lvl) const {
    for (auto v : report_levels)
      if (v == lvl) return true;
    return false;
  }
  bool in_transition(int64_t lvl) const {
    for (auto v : transition_levels)
      if (v == lvl) return true;
    return false;
  }
};
// Reads REPORT_LEVELS / TRANSITION_LEVELS / THRESHOLD_SEC like
// make_thread_locals; returns false with the Python exception text in *err.
bool read_report_env(ReportConfig* rc, std::string* err);

}  // namespace otm
