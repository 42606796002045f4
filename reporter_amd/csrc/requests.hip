// requests.hip -- the /report request bytes read on the GPU.
//
// The Java batcher writes every request as
//   {"uuid":"K","trace":[{"lat":L,"lon":L,"time":T,"accuracy":A},...]}
// (Batch.java:52-61, Point.java:39-45).  otm_report_batch stages the bodies
// into one pinned blob, copies it to HBM once, and these kernels read it: one
// wavefront per request validates that exact form and decodes its points
// straight into the batch's SoA arrays, as host fast_request (report.cpp)
// would -- the same accepted grammar subset and the same number conversions,
// so a body the GPU accepts yields the host reader's points bit for bit.  A
// body outside the form (other key orders, whitespace, escapes, exponents,
// long literals, fewer than two points) is left to the host readers, whose
// results and error contract are unchanged.
//
// Per request: the header `{"uuid":"` + printable uuid + `","trace":[`, the
// trailer `]}`, and the points region in between.  The region is walked in
// 4 KB windows staged in LDS (+ a 256-byte margin: a point that starts in a
// window ends in its margin, or the body goes to the host); the '{' bytes are
// found in the loaded 16-byte words, listed in order in LDS, and lane j parses
// the window's point j from LDS, all lanes in lockstep (parsing inside a byte
// loop serialised the wave on every distinct offset: 2.4 -> 0.06 ms per pass;
// round 5 dropped the per-lane byte scan for the word masks).  Each point must be followed by
// ",{" or by the end of the region, and it starts with '{', so the checks
// cover every byte of the region; a '{' can occur nowhere else in a valid
// region, so the point count is the '{' count.
#include "kernels.h"

namespace otm {
namespace {

constexpr int RTB = 64;      // one wave per request
constexpr int CH = 4096;     // window step: 64 bytes per lane
constexpr int MARGIN = 256;  // a point starting in a step ends within this margin past it
constexpr int WBUF = CH + MARGIN + 16;  // + the 16-byte alignment of the window's loads
constexpr int WLOADS = (WBUF + 16 * RTB - 1) / (16 * RTB);  // 16-byte loads per lane per window

__constant__ double kP10[16] = {1e0, 1e1, 1e2,  1e3,  1e4,  1e5,  1e6,  1e7,
                                1e8, 1e9, 1e10, 1e11, 1e12, 1e13, 1e14, 1e15};

struct Cur {
  const unsigned char* L;  // window bytes (LDS)
  int i, lim;              // position, end of readable bytes
  __device__ int ch(int k) const { return k < lim ? (int)L[k] : -1; }
  // a key literal at i (its characters constants, the window reads
  // independent: a loop over the literal had read it from memory a byte at a
  // time, one round trip per character); on a mismatch the point fails, so i
  // moves only on a match
  template <int N>
  __device__ bool lit(const char (&w)[N]) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < N - 1; ++k) ok &= ch(i + k) == (int)(unsigned char)w[k];
    if (ok) i += N - 1;
    return ok;
  }
  __device__ bool digit(int k) const { return (unsigned)(ch(k) - '0') < 10u; }
  // a JSON number as report.cpp fast_request's num() reads it: int -> exact
  // double; float of <= 15 significant digits -> (double)m / 10^frac, the
  // correctly rounded value; anything else (exponent, longer literal) fails
  __device__ bool num(double* d) {
    const int a = i;
    const bool neg = ch(i) == '-';
    if (neg) ++i;
    if (!digit(i)) return false;
    unsigned long long m = 0;
    int nd = 0;
    if (ch(i) == '0') {
      ++i;
      nd = 1;
    } else {
      while (digit(i)) {
        m = m * 10ull + (unsigned long long)(ch(i) - '0');
        ++nd;
        ++i;
      }
    }
    if (ch(i) == '.') {
      if (!digit(i + 1)) return false;
      ++i;
      int frac = 0;
      while (digit(i)) {
        m = m * 10ull + (unsigned long long)(ch(i) - '0');
        ++nd;
        ++frac;
        ++i;
      }
      if (ch(i) == 'e' || ch(i) == 'E') return false;
      if (nd > 15) return false;  // host from_chars territory
      const double v = (double)m / kP10[frac];
      *d = neg ? -v : v;
      return true;
    }
    if (ch(i) == 'e' || ch(i) == 'E') return false;
    if (i - a > 18) return false;
    const long long v = neg ? -(long long)m : (long long)m;
    *d = (double)v;
    return true;
  }
};

// one point at window offset j; on success its values and the offset just
// past it (the region's end, or the next point's '{')
__device__ bool parse_point(const unsigned char* L, int j, int lim, int rend, double* la, double* lo, double* ti,
                            double* ac) {
  Cur c{L, j, lim};
  if (!c.lit("{\"lat\":") || !c.num(la)) return false;
  if (!c.lit(",\"lon\":") || !c.num(lo)) return false;
  if (!c.lit(",\"time\":") || !c.num(ti)) return false;
  if (!c.lit(",\"accuracy\":") || !c.num(ac)) return false;
  if (c.ch(c.i) != '}') return false;
  ++c.i;
  if (c.i == rend) return true;  // the region's last point
  return c.ch(c.i) == ',' && c.ch(c.i + 1) == '{';
}

// The header of request [a, e): the region [t0, t1) between `","trace":[`
// and the final `]}`, or false.  Lane-parallel search for the uuid's end.
__device__ bool req_header(const unsigned char* blob, int64_t a, int64_t e, int lane, int64_t* t0, int64_t* t1) {
  const char* H = "{\"uuid\":\"";
  if (e - a < 9 + 11 + 2) return false;
  bool ok = true;
  if (lane < 9) ok = blob[a + lane] == (unsigned char)H[lane];
  if (!__all(ok)) return false;
  // the uuid's closing quote: first '"' at >= a + 9; every byte before it
  // printable ASCII without a backslash
  int64_t q = -1;
  for (int64_t base = a + 9; base < e && q < 0; base += 64) {
    const int64_t k = base + lane;
    const int c = k < e ? (int)blob[k] : -1;
    const bool quote = c == '"';
    const bool bad = k < e && !quote && (c < 0x20 || c > 0x7e || c == '\\');
    const unsigned long long qm = __ballot(quote);
    const unsigned long long bm = __ballot(bad);
    const int first = qm ? __ffsll((long long)qm) - 1 : 64;
    // a bad byte before the quote (or before the end of this chunk with no quote)
    const unsigned long long before = first >= 64 ? ~0ull : ((1ull << first) - 1ull);
    if (bm & before) return false;
    if (qm) q = base + first;
  }
  if (q < 0) return false;
  const char* T = "\",\"trace\":[";
  if (q + 11 + 2 > e) return false;
  ok = true;
  if (lane < 11) ok = blob[q + lane] == (unsigned char)T[lane];
  if (!__all(ok)) return false;
  if (blob[e - 2] != ']' || blob[e - 1] != '}') return false;
  *t0 = q + 11;
  *t1 = e - 2;
  return *t1 > *t0;
}

// The '{' bytes of a 32-bit word: bit 8j+7 set for each byte j equal to '{'
// (exact, no borrow between bytes)
__device__ __forceinline__ uint32_t brace_bits(uint32_t x) {
  const uint32_t y = x ^ 0x7B7B7B7Bu;
  return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu);
}
// the flag bits (8j+7) of bytes j in [a, b) of a 64-bit word (a, b clamped to [0, 8])
__device__ __forceinline__ uint64_t byte_flags(int a, int b) {
  a = max(a, 0);
  b = min(b, 8);
  if (b <= a) return 0;
  const uint64_t below_b = b >= 8 ? ~0ull : ((1ull << (8 * b)) - 1ull);
  const uint64_t from_a = ~((1ull << (8 * a)) - 1ull);
  return below_b & from_a & 0x8080808080808080ull;
}

// Walk request r's points region: validate and count, and write each point
// that parses at out + base + its index (below cap).  Windows of
// CH bytes (+ MARGIN) are staged in LDS with 16-byte aligned loads, all of a
// lane's in flight at once.  The '{' bytes are found in the loaded words
// themselves (a 16-byte word holds at most one point start: a valid point is
// >= 39 bytes) and listed in LDS in order, so lane j parses the window's
// point j (no byte loop over LDS).
constexpr int PMAX = 128;  // point starts listed per window (a valid window holds <= CH / 39 + 1)
__device__ bool walk_points(const unsigned char* blob, int64_t t0, int64_t t1, int lane, unsigned char* L,
                            int16_t* PS, int64_t base, int64_t cap, const DevBatch* out, int* npts) {
  int count = 0;
  bool good = true;
  for (int64_t w0 = t0; w0 < t1; w0 += CH) {
    const int64_t al = w0 & ~(int64_t)15;  // the blob is 16-byte aligned and padded past its end
    const int sh = (int)(w0 - al);
    const int lim = (int)min<int64_t>((int64_t)(CH + MARGIN), t1 - w0);
    const uint4* src = (const uint4*)(blob + al);
    const int nld = (sh + lim + 15) >> 4;  // 16-byte words covering [w0, w0 + lim)
    uint4 v[WLOADS];
#pragma unroll
    for (int u = 0; u < WLOADS; ++u) {
      const int k = u * RTB + lane;
      v[u] = k < nld ? src[k] : make_uint4(0u, 0u, 0u, 0u);
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < WLOADS; ++u) {
      const int k = u * RTB + lane;
      if (k < nld) ((uint4*)L)[k] = v[u];
    }
    // the point starts of this step (window offsets [0, min(CH, lim))), in
    // order: word k = u * RTB + lane covers offsets [16k - sh, 16k - sh + 16)
    const int send = min(CH, lim);
    int listed = 0;
#pragma unroll
    for (int u = 0; u < WLOADS; ++u) {
      const int k = u * RTB + lane;
      int at = -1;
      if (k < nld) {
        const uint32_t b0 = brace_bits(v[u].x), b1 = brace_bits(v[u].y), b2 = brace_bits(v[u].z),
                       b3 = brace_bits(v[u].w);
        const uint64_t lo = (uint64_t)b0 | ((uint64_t)b1 << 32), hi = (uint64_t)b2 | ((uint64_t)b3 << 32);
        // bytes of the word inside [0, send): o = 16k - sh + j
        const int o0 = 16 * k - sh;
        const int j0 = o0 < 0 ? -o0 : 0, j1 = min(16, send - o0);
        const uint64_t flo = lo & byte_flags(j0, j1), fhi = hi & byte_flags(j0 - 8, j1 - 8);
        const int nb = __popcll(flo) + __popcll(fhi);
        if (nb > 1) good = false;  // two point starts within 16 bytes: no valid body has them
        if (nb >= 1) at = o0 + (flo ? (__ffsll((long long)flo) - 1) >> 3 : 8 + ((__ffsll((long long)fhi) - 1) >> 3));
      }
      const unsigned long long m = __ballot(at >= 0);
      const int pos = listed + __popcll(m & ((1ull << lane) - 1ull));
      if (at >= 0 && pos < PMAX) PS[pos] = (int16_t)at;
      listed += __popcll(m);
    }
    if (listed > PMAX) good = false;  // more starts than a valid window holds
    __syncthreads();
    const unsigned char* W = L + sh;  // W[0] = byte w0
    if (w0 == t0 && lane == 0 && W[0] != '{') good = false;  // the region starts with a point
    // lane j parses the step's point j (then j + 64)
    const int np = min(listed, PMAX);
    for (int j = lane; j - lane < np; j += RTB) {
      if (j >= np) continue;
      const int k = PS[j];
      double la, lo, ti, ac;
      const bool ok = parse_point(W, k, lim, (int)(t1 - w0), &la, &lo, &ti, &ac);
      good = good && ok;
      const int idx = count + j;
      if (ok && idx < cap) {  // (cap: an invalid body's stray '{'s write nothing past its range)
        const int64_t p = base + idx;
        // extract_points' conversions (report.cpp)
        ((float*)out->lat)[p] = (float)la;
        ((float*)out->lon)[p] = (float)lo;
        ((double*)out->time)[p] = ti;
        ((float*)out->acc)[p] = (float)ac;
      }
    }
    count += listed;
    if (!__all(good)) return false;
  }
  *npts = count;
  return good;
}

// Request r's points land in a sparse slot range first: a valid point takes
// >= 39 bytes, so request r (len_r bytes) holds at most len_r / 39 points and
// the ranges [r + off[r] / 39, + len_r / 39) never overlap (floor(a/39) +
// floor(b/39) <= floor((a+b)/39)).  So one pass can validate, count and
// write, piece by piece as the blob arrives, and a compaction after the scan
// of the counts moves the accepted points into the dense batch.
__device__ __forceinline__ int64_t sparse_base(int32_t r, int64_t a) { return (int64_t)r + a / 39; }

// per request of [r0, r1): accepted << 40 | points in cnt (0: the host
// readers take it), ok[r], its points at their sparse slots
__global__ __launch_bounds__(RTB) void k_req_read(const unsigned char* blob, const int64_t* off, int32_t r0,
                                                  int32_t r1, int32_t n, int64_t* cnt, uint8_t* ok, DevBatch sp) {
  __shared__ __attribute__((aligned(16))) unsigned char L[WBUF];
  __shared__ int16_t PS[PMAX];
  const int lane = threadIdx.x;
  for (int32_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
    const int64_t a = off[r], e = off[r + 1];
    int64_t t0 = 0, t1 = 0;
    int np = 0;
    bool acc = req_header(blob, a, e, lane, &t0, &t1);
    acc = acc && walk_points(blob, t0, t1, lane, L, PS, sparse_base(r, a), (e - a) / 39, &sp, &np) && np >= 2;
    if (lane == 0) {
      cnt[r] = acc ? ((int64_t)1 << 40) | (int64_t)np : 0;
      ok[r] = acc ? 1 : 0;
    }
  }
  if (r1 == n && blockIdx.x == 0 && lane == 0) cnt[n] = 0;
}

// (cnt scanned into pre) the accepted requests' points from their sparse
// slots into the dense batch, and the trace offsets: a wave per request
__global__ __launch_bounds__(RTB) void k_req_compact(const int64_t* off, int32_t n, const int64_t* pre,
                                                     const uint8_t* ok, DevBatch sp, DevBatch out,
                                                     int64_t* trace_off) {
  const int lane = threadIdx.x;
  constexpr int64_t MASK = ((int64_t)1 << 40) - 1;
  if (blockIdx.x == 0 && lane == 0) trace_off[pre[n] >> 40] = pre[n] & MASK;
  for (int32_t r = blockIdx.x; r < n; r += gridDim.x) {
    if (!ok[r]) continue;
    const int64_t d = pre[r] & MASK, m = (pre[r + 1] & MASK) - d;
    const int64_t s = sparse_base(r, off[r]);
    if (lane == 0) trace_off[pre[r] >> 40] = d;
    for (int64_t i = lane; i < m; i += RTB) {
      ((float*)out.lat)[d + i] = sp.lat[s + i];
      ((float*)out.lon)[d + i] = sp.lon[s + i];
      ((double*)out.time)[d + i] = sp.time[s + i];
      ((float*)out.acc)[d + i] = sp.acc[s + i];
    }
  }
}

}  // namespace

size_t req_sparse_slots(int32_t n, size_t bytes) { return (size_t)n + bytes / 39 + 1; }

void launch_req_read(const unsigned char* blob, const int64_t* off, int32_t r0, int32_t r1, int32_t n, int64_t* cnt,
                     uint8_t* ok, const DevBatch& sparse, hipStream_t s) {
  const int32_t m = r1 - r0;
  const int grid = m < 65536 ? (m > 0 ? m : 1) : 65536;
  hipLaunchKernelGGL(k_req_read, dim3(grid), dim3(RTB), 0, s, blob, off, r0, r1, n, cnt, ok, sparse);
}

void launch_req_compact(const int64_t* off, int32_t n, const int64_t* pre, const uint8_t* ok, const DevBatch& sparse,
                        const DevBatch& out, int64_t* trace_off, hipStream_t s) {
  const int grid = n < 65536 ? (n > 0 ? n : 1) : 65536;
  hipLaunchKernelGGL(k_req_compact, dim3(grid), dim3(RTB), 0, s, off, n, pre, ok, sparse, out, trace_off);
}

}  // namespace otm
