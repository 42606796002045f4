// tiles.cpp -- Valhalla's tile hierarchy as the reference computes it
// (py/get_tiles.py:30-172, itself after baldr's tilehierarchy.cc /
// graphtile.cc): three levels over the world bbox -- 0 highway 4 deg,
// 1 arterial 1 deg, 2 local 0.25 deg -- tile id = row * ncolumns + col, and
// the tile file path "<level>/<id with thousands groups as dirs>.<suffix>".
//
// Used by the synthetic flattener for OSMLR ids (tile bits of the segment id)
// and by a real-tile flattener to name the .gph files of
// a bounding box.  Pinned against the reference script's own output by
// tests/golden/tile_cases.json (tests/golden/make_tile_golden.py).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "otm_internal.h"
#include "otmatch.h"

namespace otm {

namespace {

constexpr double kMinX = -180.0, kMinY = -90.0, kMaxX = 180.0, kMaxY = 90.0;

double tile_size(int level) { return level == 0 ? 4.0 : (level == 1 ? 1.0 : 0.25); }
int64_t ncolumns(int level) { return (int64_t)std::ceil((kMaxX - kMinX) / tile_size(level)); }
int64_t nrows(int level) { return (int64_t)std::ceil((kMaxY - kMinY) / tile_size(level)); }

// Tiles.Digits (:74-79): decimal digits of a non-negative id
int64_t digits(int64_t n) {
  int64_t d = n < 0 ? 1 : 0;
  while (n != 0) {
    n /= 10;
    ++d;
  }
  return d;
}

// '{:,}'.format(v).replace(',', '/')
std::string grouped(int64_t v) {
  std::string s = std::to_string(v), out;
  const int n = (int)s.size();
  for (int k = 0; k < n; ++k) {
    if (k && (n - k) % 3 == 0) out.push_back('/');
    out.push_back(s[(size_t)k]);
  }
  return out;
}

}  // namespace

// Tiles.Row (:51-60)
int64_t tile_row(int level, double y) {
  if (y < kMinY || y > kMaxY) return -1;
  if (y == kMaxY) return nrows(level) - 1;
  return (int64_t)((y - kMinY) / tile_size(level));
}

// Tiles.Col (:62-72)
int64_t tile_col(int level, double x) {
  if (x < kMinX || x > kMaxX) return -1;
  if (x == kMaxX) return ncolumns(level) - 1;
  const double col = (x - kMinX) / tile_size(level);
  return col >= 0.0 ? (int64_t)col : (int64_t)(col - 1.0);
}

int64_t tile_id(int level, double lat, double lon) {
  const int64_t r = tile_row(level, lat), c = tile_col(level, lon);
  if (r < 0 || c < 0) return -1;
  return r * ncolumns(level) + c;
}

// Tiles.GetFile (:82-102)
std::string tile_file(int64_t id, int level, const char* suffix) {
  int64_t max_length = digits(ncolumns(level) * nrows(level) - 1);
  const int64_t rem = max_length % 3;
  if (rem) max_length += 3 - rem;
  int64_t p = 1;
  for (int64_t k = 0; k < max_length; ++k) p *= 10;
  std::string f;
  if (level == 0) {
    f = grouped(p + id) + "." + suffix;
    f[0] = '0';  // "if it starts with a zero the pow trick doesn't work"
  } else {
    f = grouped((int64_t)level * p + id) + "." + suffix;
  }
  return f;
}

}  // namespace otm

extern "C" {

int64_t otm_tile_id(int level, double lat, double lon) {
  if (level < 0 || level > 2) return -1;
  return otm::tile_id(level, lat, lon);
}

int otm_tile_file(int64_t tile_id, int level, const char* suffix, char* out, size_t cap) {
  if (level < 0 || level > 2 || tile_id < 0 || !suffix) return OTM_EINVAL;
  const std::string f = otm::tile_file(tile_id, level, suffix);
  if (!out || cap < f.size() + 1) return (int)f.size() + 1;
  std::memcpy(out, f.c_str(), f.size() + 1);
  return OTM_OK;
}

// The main loop of get_tiles.py (:130-172): the tiles of a lon/lat bbox, the
// bbox split at the antimeridian, every level.  Levels in ascending order
// (the script walks its dict; py2 and py3 order it differently).
int otm_tile_files_bbox(double minx, double miny, double maxx, double maxy, const char* suffix, char** out,
                        size_t* out_len) {
  if (!suffix || !out) return OTM_EINVAL;
  struct BB {
    double minx, miny, maxx, maxy;
  } boxes[2];
  int nb = 0;
  if (minx >= maxx) minx -= 360.0;
  if (minx < -180.0 && maxx > -180.0) {
    boxes[nb++] = {-180.0, miny, maxx, maxy};
    boxes[nb++] = {minx + 360.0, miny, 180.0, maxy};
  } else if (minx < 180.0 && maxx > 180.0) {
    boxes[nb++] = {minx, miny, 180.0, maxy};
    boxes[nb++] = {-180.0, miny, maxx - 360.0, maxy};
  } else {
    boxes[nb++] = {minx, miny, maxx, maxy};
  }
  std::string s;
  for (int b = 0; b < nb; ++b) {
    for (int level = 0; level <= 2; ++level) {
      const int64_t mincol = otm::tile_col(level, boxes[b].minx);
      for (int64_t i = otm::tile_row(level, boxes[b].miny); i <= otm::tile_row(level, boxes[b].maxy); ++i) {
        int64_t id = i * otm::ncolumns(level) + mincol;
        for (int64_t j = mincol; j <= otm::tile_col(level, boxes[b].maxx); ++j) {
          s += otm::tile_file(id, level, suffix);
          s.push_back('\n');
          ++id;
        }
      }
    }
  }
  char* p = (char*)std::malloc(s.size() + 1);
  if (!p) return OTM_ENOMEM;
  std::memcpy(p, s.c_str(), s.size() + 1);
  *out = p;
  if (out_len) *out_len = s.size();
  return OTM_OK;
}

}  // extern "C"
