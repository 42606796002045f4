/*
 * otm_graph_format.h -- the flat, HBM-ready road-graph file (".otmg").
 *
 * This is the DATA contract between the graph flattener (product,
 * reporter_amd/csrc/synth_graph.cpp; the real-tile flattener of SURVEY.md
 * §8f row 2 will write the same format) and every reader: the engine
 * (reporter_amd/csrc/graph.cpp, which uploads each section verbatim to HBM)
 * and the CPU oracle (oracle/otm_oracle.c).  It replaces what baldr's
 * GraphReader/GraphTile serve to meili inside valhalla.SegmentMatcher
 * (called at py/reporter_service.py:112, configured at :279).
 *
 * Layout: a fixed header, then sections.  Every section starts at a 256-byte
 * aligned file offset so a memory map can hand each one to hipMemcpy as is.
 * All integers little-endian.  Arrays are structure-of-arrays so that a
 * wavefront's lanes read consecutive elements.
 *
 *   nodes      lat f32[N], lon f32[N], out_off i32[N+1] (CSR over edges)
 *   edges      (sorted by from-node, so edge ids are CSR order)
 *              from i32[E], to i32[E], len f32[E] (metres, == shape cum of
 *              the last shape point), shape_off i32[E+1], way i64[E],
 *              seg i32[E] (-1: no OSMLR association), seg_pos i32[E]
 *              (index of the edge inside its segment chain), flags u8[E],
 *              level u8[E], speed f32[E] (km/h), opp i32[E] (reverse edge
 *              or -1)
 *   shape      lat f32[S], lon f32[S], cum f32[S] (metres from edge start)
 *   segments   id u64[G] (OSMLR id: level in bits 0..2, tile 3..24,
 *              index 25..45), len f32[G], first_edge i32[G], n_edges i32[G]
 *   grid       cell_off i64[R*C+1], cell_ent u32[M]: entry = edge<<4 | k,
 *              meaning shape segment k (points k,k+1) of edge overlaps the
 *              cell's lat/lon box.  Cell (r,c) covers
 *              [lat0 + r*cell, lat0 + (r+1)*cell) x [lon0 + c*cell, ...).
 *   headings   (version 2) head_out u16[E], head_in u16[E]: the edge's
 *              bearing in whole degrees [0, 360), clockwise from north, at its
 *              start (first shape segment) and at its end (last shape
 *              segment), in the direction of travel -- what Valhalla keeps
 *              per node and edge for turn costs (the turn at a node is
 *              head_out(next) - head_in(prev)).
 */
#ifndef OTM_GRAPH_FORMAT_H
#define OTM_GRAPH_FORMAT_H

#include <stdint.h>

#define OTMG_MAGIC "OTMGRAPH"
#define OTMG_VERSION 2u

/* edge flags */
#define OTM_EDGE_INTERNAL 0x01u  /* intersection-internal / turn channel */
#define OTM_EDGE_SEG_BEGIN 0x02u /* first edge of its OSMLR segment      */
#define OTM_EDGE_SEG_END 0x04u   /* last edge of its OSMLR segment       */

/* max shape segments per edge: the grid entry packs k into 4 bits */
#define OTM_MAX_EDGE_SHAPE_SEGS 15

enum otmg_section {
  OTMG_NODE_LAT = 0,
  OTMG_NODE_LON,
  OTMG_NODE_OUT_OFF,
  OTMG_EDGE_FROM,
  OTMG_EDGE_TO,
  OTMG_EDGE_LEN,
  OTMG_EDGE_SHAPE_OFF,
  OTMG_EDGE_WAY,
  OTMG_EDGE_SEG,
  OTMG_EDGE_SEG_POS,
  OTMG_EDGE_FLAGS,
  OTMG_EDGE_LEVEL,
  OTMG_EDGE_SPEED,
  OTMG_EDGE_OPP,
  OTMG_SHAPE_LAT,
  OTMG_SHAPE_LON,
  OTMG_SHAPE_CUM,
  OTMG_SEG_ID,
  OTMG_SEG_LEN,
  OTMG_SEG_FIRST_EDGE,
  OTMG_SEG_N_EDGES,
  OTMG_CELL_OFF,
  OTMG_CELL_ENT,
  OTMG_EDGE_HEAD_OUT, /* version 2: turn costs */
  OTMG_EDGE_HEAD_IN,
  OTMG_NUM_SECTIONS
};

typedef struct otmg_section_desc {
  uint64_t offset; /* file offset, 256-byte aligned */
  uint64_t bytes;
} otmg_section_desc;

typedef struct otmg_header {
  char magic[8];
  uint32_t version;
  uint32_t header_bytes;
  int32_t n_nodes;
  int32_t n_edges;
  int32_t n_shape;
  int32_t n_segments;
  int32_t grid_rows;
  int32_t grid_cols;
  int64_t n_cell_entries;
  double grid_lat0;     /* south edge of row 0  */
  double grid_lon0;     /* west edge of column 0 */
  double grid_cell_deg; /* square cells, degrees */
  double bbox[4];       /* min_lat, min_lon, max_lat, max_lon of all nodes */
  uint64_t seed;        /* generator seed (0 for real tiles) */
  otmg_section_desc sec[OTMG_NUM_SECTIONS];
} otmg_header;

#endif /* OTM_GRAPH_FORMAT_H */
