// responses.hip -- the /report response bodies written on the GPU.
//
// report.cpp write_report_response's bytes (py/reporter_service.py:198-215,
// json.dumps of the handler's dict: Python 3 key order, float repr), from the
// batch's dense result arrays in HBM.  Three launches:
//   k_resp_items  a thread per piece: each trace's header (stats, shape_used,
//                 up to the segments' '['), each segment object, each
//                 datastore report object, formatted into a fixed-size slot
//                 with its length (-1: a float outside pyrepr.h's range);
//   k_resp_len    a thread per trace: the body's length from its pieces, or
//                 -1 (a 500 body or an unformattable float: the host writes it);
//   k_resp_copy   a wave per trace: the pieces and the fixed joins into the
//                 trace's place in one dense blob (offsets: a scan of the
//                 lengths), each body NUL-terminated, so that one copy into
//                 the caller's response arena leaves every body in place.
#include "kernels.h"
#include "otmatch.h"
#include "pyrepr.h"

namespace otm {
namespace {

constexpr int RESP_TB = 256;

// a piece's bytes, gathered 8 at a time and stored as whole 8-byte words
// (slots are 8-byte aligned; the last word may run past the piece into its
// slot's slack): a byte store per character cost a 64-line store instruction
struct Out {
  char* p;
  int n;
  uint64_t acc;
  __device__ __forceinline__ void put(char c) {
    acc |= (uint64_t)(uint8_t)c << (8 * (n & 7));
    if ((++n & 7) == 0) {
      *(uint64_t*)(p + n - 8) = acc;
      acc = 0;
    }
  }
  // m <= 8 bytes at once (w: byte j the j-th, zero above m)
  __device__ __forceinline__ void put8(uint64_t w, int m) {
    const int sh = 8 * (n & 7);
    acc |= w << sh;
    if ((n & 7) + m >= 8) {
      *(uint64_t*)(p + (n & ~7)) = acc;
      acc = sh ? w >> (64 - sh) : 0;
    }
    n += m;
  }
  // a literal, 8 characters a step, packed into constants at compile time (a
  // loop over the literal had read it from memory a byte at a time: one load
  // round trip per character)
  template <int N>
  __device__ __forceinline__ void lit(const char (&s)[N]) {
#pragma unroll
    for (int k0 = 0; k0 < N - 1; k0 += 8) {
      uint64_t w = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (k0 + j < N - 1) w |= (uint64_t)(uint8_t)s[k0 + j] << (8 * j);
      put8(w, N - 1 - k0 < 8 ? N - 1 - k0 : 8);
    }
  }
  __device__ __forceinline__ void i64(int64_t v) { pyrepr::put_i64(v, *this); }
  __device__ __forceinline__ bool f64(double d) { return pyrepr::py_repr(d, *this); }
  __device__ __forceinline__ int done() {
    if (n & 7) *(uint64_t*)(p + (n & ~7)) = acc;
    return n;
  }
};

__device__ const char kMid[] = "],\"mode\":\"auto\"},\"datastore\":{\"mode\":\"auto\"";
__device__ const char kReps[] = ",\"reports\":[";
constexpr int MID_LEN = sizeof(kMid) - 1;
constexpr int REPS_LEN = sizeof(kReps) - 1;

__device__ int64_t seg_slot(int32_t s, int32_t way_off) { return (int64_t)s * RESP_SEG_SLOT + 24ll * way_off; }

__global__ __launch_bounds__(RESP_TB) void k_resp_items(RespIn in, RespWork w) {
  const int64_t nitems = (int64_t)in.nt + in.ns + in.nr;
  for (int64_t it = (int64_t)blockIdx.x * RESP_TB + threadIdx.x; it < nitems; it += (int64_t)gridDim.x * RESP_TB) {
    if (it < in.nt) {
      const int32_t t = (int32_t)it;
      const otm_trace_result tr = in.traces[t];
      Out o{w.hdr + (int64_t)t * RESP_HDR_SLOT, 0, 0};
      bool ok = tr.code == 200;
      if (ok) {
        // write_report_response: the stats block, shape_used, up to the segments
        o.lit("{\"stats\":{\"successful_matches\":{\"count\":");
        o.i64(tr.successful_count);
        o.lit(",\"length\":");
        double v;
        if (tr.successful_length >= 0) ok = ok && pyrepr::py_round3((double)tr.successful_length * 0.001, &v) && o.f64(v);
        else o.lit("0");
        o.lit("},\"unreported_matches\":{\"count\":");
        o.i64(tr.unreported_count);
        o.lit(",\"length\":");
        if (tr.unreported_length >= 0) ok = ok && pyrepr::py_round3((double)tr.unreported_length * 0.001, &v) && o.f64(v);
        else o.lit("0");
        o.lit("},\"match_errors\":{\"discontinuities\":");
        o.i64(tr.discontinuities);
        o.lit(",\"invalid_speeds\":");
        o.i64(tr.invalid_speeds);
        o.lit("},\"unassociated_segments\":");
        o.i64(tr.unassociated);
        o.lit("}");
        if (tr.shape_used > 0) {
          o.lit(",\"shape_used\":");
          o.i64(tr.shape_used);
        }
        o.lit(",\"segment_matcher\":{\"segments\":[");
      }
      w.hlen[t] = o.done() >= 0 && ok ? o.n : -1;
    } else if (it < (int64_t)in.nt + in.ns) {
      const int32_t s = (int32_t)(it - in.nt);
      const otm_segment g = in.segs[s];
      Out o{w.seg + seg_slot(s, g.way_off), 0, 0};
      bool ok = true;
      o.lit("{");
      if (g.segment_id >= 0) {
        o.lit("\"segment_id\":");
        o.i64(g.segment_id);
        o.lit(",");
      }
      o.lit("\"way_ids\":[");
      for (int32_t k = 0; k < g.way_cnt; ++k) {
        if (k) o.lit(",");
        o.i64(in.ways[g.way_off + k]);
      }
      o.lit("],\"start_time\":");
      if (g.flags & OTM_SEG_START_VALID) ok = ok && o.f64(g.start_time);
      else o.lit("-1");
      o.lit(",\"end_time\":");
      if (g.flags & OTM_SEG_END_VALID) ok = ok && o.f64(g.end_time);
      else o.lit("-1");
      o.lit(",\"queue_length\":");
      o.i64(g.queue_length);
      o.lit(",\"length\":");
      o.i64(g.length);
      if (g.flags & OTM_SEG_INTERNAL) o.lit(",\"internal\":true");
      else o.lit(",\"internal\":false");
      o.lit(",\"begin_shape_index\":");
      o.i64(g.begin_shape_index);
      o.lit(",\"end_shape_index\":");
      o.i64(g.end_shape_index);
      o.lit("}");
      w.slen[s] = o.done() >= 0 && ok ? o.n : -1;
    } else {
      const int32_t r = (int32_t)(it - in.nt - in.ns);
      const otm_report_rec p = in.reps[r];
      Out o{w.rep + (int64_t)r * RESP_REP_SLOT, 0, 0};
      bool ok = true;
      o.lit("{\"id\":");
      o.i64(p.id);
      o.lit(",\"t0\":");
      if (p.flags & OTM_REP_T0_INT) o.i64((int64_t)p.t0);
      else ok = ok && o.f64(p.t0);
      o.lit(",\"t1\":");
      if (p.flags & OTM_REP_T1_INT) o.i64((int64_t)p.t1);
      else ok = ok && o.f64(p.t1);
      o.lit(",\"length\":");
      o.i64(p.length);
      o.lit(",\"queue_length\":");
      o.i64(p.queue_length);
      if (p.next_id >= 0) {
        o.lit(",\"next_id\":");
        o.i64(p.next_id);
      }
      o.lit("}");
      w.rlen[r] = o.done() >= 0 && ok ? o.n : -1;
    }
  }
}

// a trace's body length from its pieces (-1: the host writes it)
__global__ __launch_bounds__(RESP_TB) void k_resp_len(RespIn in, RespWork w) {
  const int32_t t = blockIdx.x * RESP_TB + threadIdx.x;
  if (t == in.nt) w.blen[t] = 0;
  if (t >= in.nt) return;
  const otm_trace_result tr = in.traces[t];
  int64_t n = w.hlen[t];
  bool ok = n >= 0;
  for (int32_t k = 0; ok && k < tr.seg_cnt; ++k) {
    const int32_t l = w.slen[tr.seg_off + k];
    ok = l >= 0;
    n += l + (k ? 1 : 0);
  }
  n += MID_LEN;
  if (tr.rep_cnt > 0) {
    n += REPS_LEN + 1;
    for (int32_t k = 0; ok && k < tr.rep_cnt; ++k) {
      const int32_t l = w.rlen[tr.rep_off + k];
      ok = ok && l >= 0;
      n += l + (k ? 1 : 0);
    }
  }
  n += 2;
  w.blen[t] = ok ? n + 1 : 0;  // + the NUL the caller's string needs
  w.host[t] = ok ? 0 : 1;
}

__device__ void copy_piece(char* dst, const char* src, int n, int lane) {
  for (int k = lane; k < n; k += 64) dst[k] = src[k];
}

// trace t's body into d, the wave's lanes copying each piece in turn (the
// form for a body larger than the LDS buffer below)
__device__ void body_serial(const RespIn& in, const RespWork& w, int32_t t, const otm_trace_result& tr, char* d,
                            int lane) {
  int64_t n = 0;
  const int hl = w.hlen[t];
  copy_piece(d, w.hdr + (int64_t)t * RESP_HDR_SLOT, hl, lane);
  n += hl;
  for (int32_t k = 0; k < tr.seg_cnt; ++k) {
    const int32_t s = tr.seg_off + k;
    if (k) {
      if (lane == 0) d[n] = ',';
      ++n;
    }
    const int l = w.slen[s];
    copy_piece(d + n, w.seg + seg_slot(s, in.segs[s].way_off), l, lane);
    n += l;
  }
  copy_piece(d + n, kMid, MID_LEN, lane);
  n += MID_LEN;
  if (tr.rep_cnt > 0) {
    copy_piece(d + n, kReps, REPS_LEN, lane);
    n += REPS_LEN;
    for (int32_t k = 0; k < tr.rep_cnt; ++k) {
      if (k) {
        if (lane == 0) d[n] = ',';
        ++n;
      }
      const int l = w.rlen[tr.rep_off + k];
      copy_piece(d + n, w.rep + (int64_t)(tr.rep_off + k) * RESP_REP_SLOT, l, lane);
      n += l;
    }
    if (lane == 0) d[n] = ']';
    ++n;
  }
  if (lane == 0) {
    d[n] = '}';
    d[n + 1] = '}';
    d[n + 2] = '\0';
  }
}

__device__ __forceinline__ int wave_scan_incl(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// one lane's piece (8-byte aligned slot, written as whole words) into LDS at L
__device__ __forceinline__ void piece_to_lds(char* L, const char* src, int l) {
  for (int q = 0; q < l; q += 8) {
    const uint64_t v = *(const uint64_t*)(src + q);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (q + j < l) L[q + j] = (char)(v >> (8 * j));
  }
}

// pieces [0, cnt) of one kind, a lane each (64 at a time), after a comma for
// every piece but the first; *at: the running LDS offset (uniform)
template <class Len, class Src>
__device__ __forceinline__ void pieces_to_lds(char* L, int* at, int32_t cnt, int lane, Len len, Src src) {
  for (int32_t k0 = 0; k0 < cnt; k0 += 64) {
    const int32_t k = k0 + lane;
    const bool has = k < cnt;
    const int l = has ? len(k) : 0;
    const int mine = has ? l + (k > 0 ? 1 : 0) : 0;
    const int incl = wave_scan_incl(mine, lane);
    if (has) {
      int p = *at + incl - mine;
      if (k > 0) L[p++] = ',';
      piece_to_lds(L + p, src(k), l);
    }
    *at += __shfl(incl, 63, 64);
  }
}

// a wave per trace: its pieces into the dense blob (boff: the scanned lengths).
// A body that fits BODY_LDS is assembled in LDS -- each lane copying whole
// pieces, their offsets from a wave scan of the lengths (no dependent length
// load per piece) -- and stored with 16-byte aligned words (bytes at its two
// ends, whose words it shares with its neighbours); a larger body is copied
// piece by piece (body_serial).
constexpr int BODY_LDS = 8192;
__global__ __launch_bounds__(64) void k_resp_copy(RespIn in, RespWork w, const int64_t* boff, char* blob) {
  __shared__ uint4 LW[BODY_LDS / 16];
  char* L = (char*)LW;
  const int lane = threadIdx.x;
  for (int32_t t = blockIdx.x; t < in.nt; t += gridDim.x) {
    if (w.host[t]) continue;
    const otm_trace_result tr = in.traces[t];
    const int64_t start = boff[t], end = boff[t + 1];  // (the body and its NUL)
    const int sh = (int)(start & 15);
    if (sh + (end - start) > BODY_LDS) {
      body_serial(in, w, t, tr, blob + start, lane);
      continue;
    }
    const int hl = w.hlen[t];
    const char* hdr = w.hdr + (int64_t)t * RESP_HDR_SLOT;
    for (int k = lane; k < hl; k += 64) L[sh + k] = hdr[k];
    int at = sh + hl;
    pieces_to_lds(
        L, &at, tr.seg_cnt, lane, [&](int32_t k) { return w.slen[tr.seg_off + k]; },
        [&](int32_t k) {
          const int32_t s = tr.seg_off + k;
          return (const char*)(w.seg + seg_slot(s, in.segs[s].way_off));
        });
    for (int k = lane; k < MID_LEN; k += 64) L[at + k] = kMid[k];
    at += MID_LEN;
    if (tr.rep_cnt > 0) {
      for (int k = lane; k < REPS_LEN; k += 64) L[at + k] = kReps[k];
      at += REPS_LEN;
      pieces_to_lds(
          L, &at, tr.rep_cnt, lane, [&](int32_t k) { return w.rlen[tr.rep_off + k]; },
          [&](int32_t k) { return (const char*)(w.rep + (int64_t)(tr.rep_off + k) * RESP_REP_SLOT); });
      if (lane == 0) L[at] = ']';
      ++at;
    }
    if (lane == 0) {
      L[at] = '}';
      L[at + 1] = '}';
      L[at + 2] = '\0';
    }
    __syncthreads();
    // LDS word i holds blob bytes [a0 + 16 i, a0 + 16 i + 16)
    const int64_t a0 = start - sh;
    const int nw = (int)((end - a0 + 15) >> 4);
    for (int i = lane; i < nw; i += 64) {
      const int64_t g = a0 + 16 * (int64_t)i;
      if (g >= start && g + 16 <= end) {
        *(uint4*)(blob + g) = LW[i];
      } else {
        for (int j = 0; j < 16; ++j)
          if (g + j >= start && g + j < end) blob[g + j] = L[16 * i + j];
      }
    }
    __syncthreads();  // (the next trace reuses the buffer)
  }
}

}  // namespace

size_t resp_seg_scratch(int32_t ns, int32_t nw) { return (size_t)ns * RESP_SEG_SLOT + 24ull * (size_t)nw + 64; }

void launch_resp_items(const RespIn& in, const RespWork& w, hipStream_t s) {
  const int64_t n = (int64_t)in.nt + in.ns + in.nr;
  int64_t g = (n + RESP_TB - 1) / RESP_TB;
  if (g < 1) g = 1;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_resp_items, dim3((unsigned)g), dim3(RESP_TB), 0, s, in, w);
}
void launch_resp_len(const RespIn& in, const RespWork& w, hipStream_t s) {
  hipLaunchKernelGGL(k_resp_len, dim3((unsigned)((in.nt + 1 + RESP_TB - 1) / RESP_TB)), dim3(RESP_TB), 0, s, in, w);
}
void launch_resp_copy(const RespIn& in, const RespWork& w, const int64_t* boff, char* blob, hipStream_t s) {
  const int g = in.nt < 65536 ? (in.nt > 0 ? in.nt : 1) : 65536;
  hipLaunchKernelGGL(k_resp_copy, dim3(g), dim3(64), 0, s, in, w, boff, blob);
}

}  // namespace otm
