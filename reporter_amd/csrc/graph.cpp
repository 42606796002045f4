// graph.cpp -- .otmg loading, thread errors, reporter env parsing.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cctype>
#include <cstdlib>
#include <cstring>

#include "otm_internal.h"

namespace otm {

static thread_local std::string g_thread_error;
void set_thread_error(const std::string& msg) { g_thread_error = msg; }
const char* thread_error() { return g_thread_error.c_str(); }

HostGraph::~HostGraph() {
  if (map) munmap(map, map_bytes);
}

int load_graph(const char* path, HostGraph* g, std::string* err) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) {
    *err = std::string("cannot open graph file ") + path;
    return OTM_EIO;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(otmg_header)) {
    close(fd);
    *err = std::string("graph file too small: ") + path;
    return OTM_EIO;
  }
  void* m = mmap(nullptr, st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    *err = "mmap failed";
    return OTM_EIO;
  }
  g->map = m;
  g->map_bytes = st.st_size;
  std::memcpy(&g->h, m, sizeof(otmg_header));
  const otmg_header& h = g->h;
  if (std::memcmp(h.magic, OTMG_MAGIC, 8) != 0 || h.version != OTMG_VERSION ||
      h.header_bytes != sizeof(otmg_header)) {
    *err = "bad graph file header";
    return OTM_EIO;
  }
  const uint64_t expect[OTMG_NUM_SECTIONS] = {
      4ull * h.n_nodes, 4ull * h.n_nodes, 4ull * (h.n_nodes + 1), 4ull * h.n_edges, 4ull * h.n_edges,
      4ull * h.n_edges, 4ull * (h.n_edges + 1), 8ull * h.n_edges, 4ull * h.n_edges, 4ull * h.n_edges,
      1ull * h.n_edges, 1ull * h.n_edges, 4ull * h.n_edges, 4ull * h.n_edges, 4ull * h.n_shape,
      4ull * h.n_shape, 4ull * h.n_shape, 8ull * h.n_segments, 4ull * h.n_segments, 4ull * h.n_segments,
      4ull * h.n_segments, 8ull * ((uint64_t)h.grid_rows * h.grid_cols + 1), 4ull * h.n_cell_entries,
      2ull * h.n_edges, 2ull * h.n_edges};
  for (int s = 0; s < OTMG_NUM_SECTIONS; ++s) {
    if (h.sec[s].bytes != expect[s] || h.sec[s].offset + h.sec[s].bytes > (uint64_t)st.st_size ||
        (h.sec[s].offset & 255)) {
      *err = "graph file section " + std::to_string(s) + " malformed";
      return OTM_EIO;
    }
  }
  g->node_lat = (const float*)g->section(OTMG_NODE_LAT);
  g->node_lon = (const float*)g->section(OTMG_NODE_LON);
  g->out_off = (const int32_t*)g->section(OTMG_NODE_OUT_OFF);
  g->e_from = (const int32_t*)g->section(OTMG_EDGE_FROM);
  g->e_to = (const int32_t*)g->section(OTMG_EDGE_TO);
  g->e_len = (const float*)g->section(OTMG_EDGE_LEN);
  g->e_shape_off = (const int32_t*)g->section(OTMG_EDGE_SHAPE_OFF);
  g->e_way = (const int64_t*)g->section(OTMG_EDGE_WAY);
  g->e_seg = (const int32_t*)g->section(OTMG_EDGE_SEG);
  g->e_seg_pos = (const int32_t*)g->section(OTMG_EDGE_SEG_POS);
  g->e_flags = (const uint8_t*)g->section(OTMG_EDGE_FLAGS);
  g->e_level = (const uint8_t*)g->section(OTMG_EDGE_LEVEL);
  g->e_speed = (const float*)g->section(OTMG_EDGE_SPEED);
  g->e_opp = (const int32_t*)g->section(OTMG_EDGE_OPP);
  g->s_lat = (const float*)g->section(OTMG_SHAPE_LAT);
  g->s_lon = (const float*)g->section(OTMG_SHAPE_LON);
  g->s_cum = (const float*)g->section(OTMG_SHAPE_CUM);
  g->g_id = (const uint64_t*)g->section(OTMG_SEG_ID);
  g->g_len = (const float*)g->section(OTMG_SEG_LEN);
  g->g_first = (const int32_t*)g->section(OTMG_SEG_FIRST_EDGE);
  g->g_nedges = (const int32_t*)g->section(OTMG_SEG_N_EDGES);
  g->cell_off = (const int64_t*)g->section(OTMG_CELL_OFF);
  g->cell_ent = (const uint32_t*)g->section(OTMG_CELL_ENT);
  g->e_head_out = (const uint16_t*)g->section(OTMG_EDGE_HEAD_OUT);
  g->e_head_in = (const uint16_t*)g->section(OTMG_EDGE_HEAD_IN);
  for (int32_t e = 0; e < h.n_edges; ++e)
    if (g->e_head_out[e] >= 360 || g->e_head_in[e] >= 360) {
      *err = "graph file: edge heading out of [0, 360)";
      return OTM_EIO;
    }
  // structural checks the kernels rely on (no bounds checks on device)
  if (g->out_off[0] != 0 || g->out_off[h.n_nodes] != h.n_edges || g->e_shape_off[0] != 0 ||
      g->e_shape_off[h.n_edges] != h.n_shape || g->cell_off[(size_t)h.grid_rows * h.grid_cols] != h.n_cell_entries) {
    *err = "graph file offsets inconsistent";
    return OTM_EIO;
  }
  for (int32_t e = 0; e < h.n_edges; ++e) {
    int32_t ns = g->e_shape_off[e + 1] - g->e_shape_off[e];
    if (g->e_from[e] < 0 || g->e_from[e] >= h.n_nodes || g->e_to[e] < 0 || g->e_to[e] >= h.n_nodes || ns < 2 ||
        ns - 1 > OTM_MAX_EDGE_SHAPE_SEGS || !(g->e_len[e] > 0.0f) || g->e_seg[e] >= h.n_segments) {
      *err = "graph file edge " + std::to_string(e) + " invalid";
      return OTM_EIO;
    }
    if (e > 0 && g->e_from[e] < g->e_from[e - 1]) {
      *err = "graph edges not in CSR order";
      return OTM_EIO;
    }
  }
  for (int64_t c = 0; c < h.n_cell_entries; ++c) {
    uint32_t ent = g->cell_ent[c];
    int32_t e = (int32_t)(ent >> 4), k = (int32_t)(ent & 15u);
    if (e >= h.n_edges || k + 1 >= g->e_shape_off[e + 1] - g->e_shape_off[e]) {
      *err = "graph cell entry invalid";
      return OTM_EIO;
    }
  }
  return OTM_OK;
}

// Python repr of a str (enough for env values: ASCII printable + escapes)
static std::string py_repr(const std::string& s) {
  bool has_sq = s.find('\'') != std::string::npos, has_dq = s.find('"') != std::string::npos;
  char q = (has_sq && !has_dq) ? '"' : '\'';
  std::string o(1, q);
  for (unsigned char c : s) {
    if (c == '\\') o += "\\\\";
    else if (c == (unsigned char)q) { o += '\\'; o += (char)c; }
    else if (c == '\n') o += "\\n";
    else if (c == '\r') o += "\\r";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == 0x7f) {
      char b[8];
      std::snprintf(b, sizeof b, "\\x%02x", c);
      o += b;
    } else o += (char)c;
  }
  o += q;
  return o;
}

// int(s) for base 10 as Python parses it: surrounding whitespace, sign,
// digits with single underscores between them.
static bool py_int(const std::string& s, int64_t* out) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) ++a;
  while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
  if (a == b) return false;
  bool neg = false;
  if (s[a] == '+' || s[a] == '-') {
    neg = s[a] == '-';
    ++a;
  }
  if (a == b || !std::isdigit((unsigned char)s[a]) || !std::isdigit((unsigned char)s[b - 1])) return false;
  int64_t v = 0;
  for (size_t i = a; i < b; ++i) {
    if (s[i] == '_') {
      if (s[i - 1] == '_') return false;
      continue;
    }
    if (!std::isdigit((unsigned char)s[i])) return false;
    v = v * 10 + (s[i] - '0');
  }
  *out = neg ? -v : v;
  return true;
}

static bool parse_levels(const char* env, const char* dflt, std::vector<int64_t>* out, std::string* err) {
  const char* v = std::getenv(env);
  std::string s = v ? v : dflt;
  out->clear();
  size_t start = 0;
  while (true) {
    size_t comma = s.find(',', start);
    std::string part = s.substr(start, comma == std::string::npos ? std::string::npos : comma - start);
    int64_t x;
    if (!py_int(part, &x)) {
      *err = "invalid literal for int() with base 10: " + py_repr(part);
      return false;
    }
    out->push_back(x);
    if (comma == std::string::npos) break;
    start = comma + 1;
  }
  return true;
}

bool read_report_env(ReportConfig* rc, std::string* err) {
  // reporter_service.py:55-56
  if (!parse_levels("REPORT_LEVELS", "0,1", &rc->report_levels, err)) return false;
  if (!parse_levels("TRANSITION_LEVELS", "0,1", &rc->transition_levels, err)) return false;
  // :59-62 -- bool(strtobool(str(THRESHOLD_SEC))) when set and non-empty
  rc->threshold_sec = 15.0;
  const char* t = std::getenv("THRESHOLD_SEC");
  if (t && *t) {
    std::string low;
    for (const char* c = t; *c; ++c) low += (char)std::tolower((unsigned char)*c);
    static const char* yes[] = {"y", "yes", "t", "true", "on", "1"};
    static const char* no[] = {"n", "no", "f", "false", "off", "0"};
    bool hit = false;
    for (auto y : yes)
      if (low == y) { rc->threshold_sec = 1.0; hit = true; }
    for (auto n : no)
      if (low == n) { rc->threshold_sec = 0.0; hit = true; }
    if (!hit) {
      *err = "invalid truth value " + py_repr(t);
      return false;
    }
  }
  return true;
}

}  // namespace otm
