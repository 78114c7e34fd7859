// ge_rows.hpp -- CSR row kernels with an in-order edge sum.
//
// The reference adds a row's edge terms to its force one after the other in
// stored order (include/forceatlas.hpp:169-203, :415-467), so a row's sum is a
// serial chain; but each TERM depends only on the two endpoints.  So the terms
// are evaluated in parallel and only the adds are serial:
//   heavy (deg > kTileCap)     one block per row: three waves evaluate the next
//                              chunk while the first adds the current one;
//   tiles (many rows)          consecutive rows packed into tiles of <= kTileRows
//                              rows and <= kTileCap entries: one thread per
//                              entry evaluates its term into LDS (coalesced
//                              index reads, every gather of the tile in flight
//                              at once), then one lane per (row, dimension)
//                              adds the row's terms in order;
//   medium / light (few rows, a small level: latency, not throughput)
//                              one wave per row / one thread per row.
// In the serial adds, lane k carries dimension k: one dependent add per term.
// A term computed alone is 0 + t, equal to t up to the sign of zero; the
// accumulator starts at +0 and a round-to-nearest sum is -0 only when both
// operands are, so it is never -0 and adding the stored term later gives the
// reference's bits.
//
// classed_rows_kernel: blocks [0, nheavy) take heavy rows (scheduled first:
// longest chains), then 4 medium rows per block, then 256 light rows per block.
// tile_rows_kernel takes the tiles, on the caller's stream, while the heavy
// rows run beside it on a side stream (launch_rows).  `rows` lists heavy rows, then the tiled rows (in
// the caller's order, so a tile's CSR rows are usually contiguous), then
// medium, then light rows; the tile boundaries follow them in the same array.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace ge {

constexpr int kRowT = 256;
constexpr int kMedDeg = 32;
constexpr int kHeavyDeg = 2048;
#ifndef GE_TILE_ROWS
#define GE_TILE_ROWS 64
#endif
#ifndef GE_TILE_CAP
#define GE_TILE_CAP 512
#endif
#ifndef GE_ROWS_MINBLOCKS
#define GE_ROWS_MINBLOCKS 1
#endif
constexpr int kTileRows = GE_TILE_ROWS;  // <= 128 (two-wave scan)
constexpr int kTileCap = GE_TILE_CAP;    // entries per tile (multiple of kRowT); longer rows are heavy
constexpr int kTileMinRows = 65536;  // fewer rows: medium / light classes
// kSegStore: heavy rows of at least this many entries are "early" (launch_rows): their
// segments and chains run first, on the side stream, so that the longest chains do not
// start after the last segment.  C4 level 0: 299 rows of 8 192-135 339 entries (12 261
// segments); the other heavy rows have <= 6 224.
constexpr int kChainEarly = 16 * kTileCap;

struct RowClasses {
  const int* rows = nullptr;
  const int* tile_ptr = nullptr;  // ntiles + 1 offsets into rows
  const int* seg = nullptr;       // nseg x {heavy row slot, first, last entry offset in the row}
  long long* hacc = nullptr;      // nheavy x D x {S, A}: binade sums of the segments (zeroed)
  int* hflag = nullptr;           // nheavy: a segment could not use the binade sum
  double* hterm = nullptr;        // kSegStore: the heavy rows' terms, row h at hoff[h], dim-major
  const long long* hoff = nullptr;
  int seg_mode = 0;               // kSegBinade / kSegStore when nseg > 0
  int nheavy = 0, ntiles = 0, nmed = 0, nlight = 0, nseg = 0;
  // kSegStore: heavy rows [0, nearly) (the longest: heavy rows are in descending
  // degree order) and their segments [0, nseg_early) run first, on the side stream
  int nearly = 0, nseg_early = 0;
  int tile_off = 0;  // where tile_ptr starts in the host array
  int seg_off = 0;   // where seg starts in the host array
  int grid() const { return nheavy + (nmed + 3) / 4 + (nlight + kRowT - 1) / kRowT; }
  void bind(const int* dev) {
    rows = dev;
    tile_ptr = dev + tile_off;
    seg = dev + seg_off;
  }
};

// Host: order `ids` (row ids with their degrees) into classes; `out` gets the
// row list followed by the tile boundaries (upload all of it, then bind()).
// GE_ROWS_MED / GE_ROWS_HEAVY / GE_ROWS_TILES override the choices (tuning).
// Heavy rows in tile mode are split into segments of <= kTileCap entries,
// evaluated as tiles, and then summed by one of:
//   kSegBinade  integer sums in the binade of the row's force (its sum starts far
//               above its edge terms: single-level forceAtlas), serial fallback;
//   kSegStore   the terms stored in HBM, then one wave per row adds them in order
//               (the multilevel member rows, whose sums leave the binade).
// kSegNone keeps heavy rows whole (one block per row, on a side stream).
constexpr int kSegNone = 0, kSegBinade = 1, kSegStore = 2;
inline void classify_rows(const std::vector<int>& ids, const std::vector<int>& deg,
                          std::vector<int>& out, RowClasses& rc, int seg_mode,
                          std::vector<int>* heavy_deg = nullptr) {
  bool tiles = ids.size() >= (size_t)kTileMinRows;
  if (const char* e = std::getenv("GE_ROWS_TILES")) tiles = std::atoi(e) != 0;
  // few rows (a small level): latency, not throughput -- rows of more than 4
  // entries take a wave (n = 536: attraction 26 -> 13 us per iteration)
  int med = ids.size() <= 65536 ? 4 : kMedDeg, heavy = tiles ? kTileCap : kHeavyDeg;
  if (const char* e = std::getenv("GE_ROWS_MED")) med = std::atoi(e);
  if (const char* e = std::getenv("GE_ROWS_HEAVY")) heavy = std::min(std::atoi(e), tiles ? kTileCap : 1 << 30);
  out.clear();
  if (heavy_deg) heavy_deg->clear();
  // heavy rows longest first: their chains bound the pass (a row's sum does not depend
  // on where it sits in the list)
  std::vector<int> hq;
  for (size_t q = 0; q < ids.size(); ++q)
    if (deg[q] > heavy) hq.push_back((int)q);
  std::stable_sort(hq.begin(), hq.end(), [&](int x, int y) { return deg[x] > deg[y]; });
  for (int q : hq) {
    out.push_back(ids[q]);
    if (heavy_deg) heavy_deg->push_back(deg[q]);
  }
  rc.nheavy = (int)out.size();
  std::vector<int> tp;
  if (tiles) {
    int rows = 0, ents = 0;
    for (size_t q = 0; q < ids.size(); ++q) {
      if (deg[q] > heavy) continue;
      if (rows == 0 || rows == kTileRows || ents + deg[q] > kTileCap) {
        tp.push_back((int)out.size());
        rows = ents = 0;
      }
      out.push_back(ids[q]);
      ++rows;
      ents += deg[q];
    }
    rc.ntiles = (int)tp.size();
    tp.push_back((int)out.size());
    rc.nmed = rc.nlight = 0;
  } else {
    rc.ntiles = 0;
    for (size_t q = 0; q < ids.size(); ++q)
      if (deg[q] > med && deg[q] <= heavy) out.push_back(ids[q]);
    rc.nmed = (int)out.size() - rc.nheavy;
    for (size_t q = 0; q < ids.size(); ++q)
      if (deg[q] <= med && deg[q] <= heavy) out.push_back(ids[q]);
    rc.nlight = (int)out.size() - rc.nheavy - rc.nmed;
  }
  rc.tile_off = (int)out.size();
  out.insert(out.end(), tp.begin(), tp.end());
  // heavy rows as segments of <= kTileCap entries (tile mode; GE_ROWS_SEGMENTS=0: whole rows
  // on a side stream instead)
  bool segs = tiles && seg_mode != kSegNone;
  if (const char* e = std::getenv("GE_ROWS_SEGMENTS")) segs = segs && std::atoi(e) != 0;
  rc.seg_mode = segs ? seg_mode : kSegNone;
  rc.seg_off = (int)out.size();
  rc.nseg = 0;
  rc.nearly = rc.nseg_early = 0;
  if (segs) {
    int h = 0;
    for (int q : hq) {
      for (int a = 0; a < deg[q]; a += kTileCap) {
        out.push_back(h);
        out.push_back(a);
        out.push_back(std::min(deg[q], a + kTileCap));
        ++rc.nseg;
      }
      ++h;
      if (seg_mode == kSegStore && deg[q] >= kChainEarly) {
        rc.nearly = h;
        rc.nseg_early = rc.nseg;
      }
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Lane k (< D) of the summing wave carries dimension k's running sum; the
// other lanes shadow lane D-1.  One dependent add per term instead of D, so the
// serial chain -- the floor for a hub row -- is D times shorter.  Terms sit in
// LDS dimension-major (buf[k * stride + term]), so a lane's 8 next terms are
// 4 contiguous 16-byte reads.
template <int D>
__device__ __forceinline__ double lane_dim_value(const double (&acc)[D], int kd) {
  // bitwise blend: a select chain over acc[] is turned into a dynamically
  // indexed (scratch) load by the compiler
  long long a = __double_as_longlong(acc[0]);
#pragma unroll
  for (int k = 1; k < D; ++k) {
    const long long m = -(long long)(kd == k);
    a = (a & ~m) | (__double_as_longlong(acc[k]) & m);
  }
  return __longlong_as_double(a);
}

// a += p[0] + p[1] + ... + p[cnt-1], in order (p 16-byte aligned).  Software
// pipelined: the reads of the next 16 terms are issued before the adds of the
// current 16, so the LDS latency is hidden behind the dependent add chain
// (without it every 16 terms paid a full LDS round trip).
template <int B = 16>  // terms per block
__device__ __forceinline__ double lane_chain(double a, const double* p, int cnt) {
  constexpr int R = B / 2;  // 16-byte reads per block
  const double2* q = reinterpret_cast<const double2*>(p);
  const int np = cnt / (2 * B);  // pairs of blocks: ping-pong without branches
  if (np > 0) {
    double2 x[R], y[R];
#pragma unroll
    for (int r = 0; r < R; ++r) x[r] = q[r];
    for (int b = 0; b < np; ++b) {
#pragma unroll
      for (int r = 0; r < R; ++r) y[r] = q[(2 * b + 1) * R + r];
      __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the adds
#pragma unroll
      for (int r = 0; r < R; ++r) {
        a = a + x[r].x;
        a = a + x[r].y;
      }
      const int b2 = min(2 * b + 2, 2 * np - 1);  // past the end: re-read (unused)
#pragma unroll
      for (int r = 0; r < R; ++r) x[r] = q[b2 * R + r];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        a = a + y[r].x;
        a = a + y[r].y;
      }
    }
  }
  for (int l = np * 2 * B; l < cnt; ++l) a = a + p[l];
  return a;
}

// acc += term(e0) + term(e0+1) + ... in order, by one wave (lane 0..63); buf
// holds D * 64 * U doubles.  Every lane ends with the full acc.
template <int D, int U, class Term>
__device__ __forceinline__ void ordered_edge_sum(int e0, int e1, int lane, double* buf, Term&& term,
                                                 double (&acc)[D]) {
  constexpr int kStride = 64 * U;
  const int kd = lane < D ? lane : D - 1;
  double a = lane_dim_value<D>(acc, kd);
  for (int b = e0; b < e1; b += kStride) {
    wave_lds_sync();  // the previous chunk has been read
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = b + lane + 64 * u;
      if (e < e1) {
        double t[D];
#pragma unroll
        for (int k = 0; k < D; ++k) t[k] = 0.0;
        term(e, t);
#pragma unroll
        for (int k = 0; k < D; ++k) buf[k * kStride + lane + 64 * u] = t[k];
      }
    }
    wave_lds_sync();
    a = lane_chain(a, buf + kd * kStride, min(kStride, e1 - b));
  }
#pragma unroll
  for (int k = 0; k < D; ++k) acc[k] = __shfl(a, k);
}

// Heavy rows (one 256-thread block per row): waves 1-3 evaluate the next chunk
// of kSplitChunk terms while wave 0 adds the current one in order, so the
// serial add chain overlaps the gathers.  buf holds two chunks, each
// dimension-major.  Only wave 0's acc is the row's sum.
#ifndef GE_SPLIT_U
#define GE_SPLIT_U 4
#endif
constexpr int kSplitU = GE_SPLIT_U;
constexpr int kSplitChunk = 192 * kSplitU;  // 3 computing waves x 64 lanes x U

template <int D, class Term>
__device__ __forceinline__ void ordered_edge_sum_split(int e0, int e1, int tid, double* buf,
                                                       Term&& term, double (&acc)[D]) {
  const bool summer = tid < 64;
  const int w = tid - 64;  // computing lane 0..191
  // branch-free over the U terms of a lane (indices clamped into the row, the
  // surplus terms dropped by the summer's count), so the compiler can issue
  // all U gathers before the arithmetic
  auto compute = [&](int b, double* dst) {
    double t[kSplitU][D];
#pragma unroll
    for (int u = 0; u < kSplitU; ++u) {
      const int e = min(b + w + 192 * u, e1 - 1);
#pragma unroll
      for (int k = 0; k < D; ++k) t[u][k] = 0.0;
      term(e, t[u]);
    }
#pragma unroll
    for (int u = 0; u < kSplitU; ++u)
#pragma unroll
      for (int k = 0; k < D; ++k) dst[k * kSplitChunk + w + 192 * u] = t[u][k];
  };
  const int kd = tid < D ? tid : D - 1;
  double a = lane_dim_value<D>(acc, kd);
  if (!summer && e0 < e1) compute(e0, buf);
  __syncthreads();
  int c = 0;
  for (int b = e0; b < e1; b += kSplitChunk, ++c) {
    double* cur = buf + (c & 1) * kSplitChunk * D;
    if (summer)
      a = lane_chain(a, cur + kd * kSplitChunk, min(kSplitChunk, e1 - b));
    else if (b + kSplitChunk < e1)
      compute(b + kSplitChunk, buf + ((c + 1) & 1) * kSplitChunk * D);
    __syncthreads();
  }
  if (summer)
#pragma unroll
    for (int k = 0; k < D; ++k) acc[k] = __shfl(a, k);
}

// a += p[0] + ... + p[cnt-1] in order, p 8-byte aligned (8 reads ahead)
__device__ __forceinline__ double lane_chain_any(double a, const double* p, int cnt) {
  int l = 0;
  for (; l + 8 <= cnt; l += 8) {
    double v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = p[l + t];
#pragma unroll
    for (int t = 0; t < 8; ++t) a = a + v[t];
  }
  for (; l < cnt; ++l) a = a + p[l];
  return a;
}

// ---------------------------------------------------------------------------
// Exact ordered sums without the serial chain (heavy rows).
//
// A row's sum starts at s0 = its repulsion force (a normal double, usually far
// larger than the edge terms) and adds the terms in stored order, rounding each
// step to nearest.  Let u = ulp(s0) = 2^(e-52) and P0 = s0/u, an integer with
// 2^52 <= |P0| < 2^53.  If the running value stays in s0's binade, every
// representable number there is a multiple of u, so each step rounds the exact
// Q*u + t to (Q + rint(t/u))*u -- unless t/u is a half-integer (a tie, decided
// by Q's parity).  Hence, with r_i = rint(t_i/u), no ties and every prefix
// P0 + r_1 + ... + r_k strictly inside (2^52, 2^53) in magnitude, the serial
// result is (P0 + sum r_i)*u bit for bit: integer sums, so any order and any
// split of the row gives it.  |prefix - P0| <= A = sum |r_i|, so
// 2^52 < |P0| - A and |P0| + A < 2^53 covers every prefix.  Segments of a heavy
// row accumulate S = sum r_i and A in int64 (|r_i| < 2^36 or the row is
// flagged); rows that fail any test (s0 zero/subnormal/non-finite, a tie, a
// large term, a binade crossing) are summed serially in stored order instead.
constexpr double kBinadeMagic = 0x1.8p52;  // f + M rounds f (|f| < 2^51) to an integer
constexpr double kBinadeBig = 0x1p36;

__device__ __forceinline__ bool binade_base(double s0, int& uexp, long long& P0) {
  const long long b = __double_as_longlong(s0);
  const int ex = (int)((b >> 52) & 0x7ff);
  if (ex == 0 || ex == 0x7ff) return false;  // zero, subnormal, inf, nan
  uexp = ex - 1023 - 52;
  P0 = (b & ((1ll << 52) - 1)) | (1ll << 52);  // |s0| / u
  if (b < 0) P0 = -P0;
  return true;
}

// rint(t / 2^uexp) as an integer; flag on a tie or |t / 2^uexp| >= 2^36 (or nan)
__device__ __forceinline__ long long binade_term(double t, int uexp, int& flag) {
  const double f = ldexp(t, -uexp);  // exact unless |f| < 2^-1022 (then rint(f) = 0)
  if (!(fabs(f) < kBinadeBig)) {
    flag = 1;
    return 0;
  }
  const double y = f + kBinadeMagic;  // round to nearest even integer
  const double r = y - kBinadeMagic;
  if (fabs(f - r) == 0.5) flag = 1;  // exact difference; a tie depends on the parity of Q
  return __double_as_longlong(y) - __double_as_longlong(kBinadeMagic);
}

// (P0 + S) * u when every prefix stays in the binade, else false
__device__ __forceinline__ bool binade_result(long long P0, int uexp, long long S, long long A,
                                              double& out) {
  const long long m = P0 < 0 ? -P0 : P0;
  if (!(m - A > (1ll << 52) && m + A < (1ll << 53))) return false;
  out = ldexp((double)(P0 + S), uexp);  // |P0 + S| < 2^53: exact
  return true;
}

// LDS bytes of the classed kernel (heavy / medium rows) and of a tile.
template <int D, class P>
struct RowsLds {
  static constexpr size_t heavy = sizeof(double) * 2 * kSplitChunk * D;
  static constexpr size_t medium = sizeof(double) * 4 * 64 * D;
  static constexpr size_t bytes = heavy > medium ? heavy : medium;
  static constexpr size_t tile = sizeof(double) * kTileCap * D +
                                 sizeof(typename P::State) * kTileRows + sizeof(int) * (kTileRows + 2);
};

// One tile: rows L.rows[r0 .. r1), entries of all of them <= kTileCap.
template <int D, class P>
__device__ __forceinline__ void tile_rows(const RowClasses& L, const P& p, int t, char* lds) {
  using State = typename P::State;
  double* tb = reinterpret_cast<double*>(lds);  // [D][kTileCap]
  State* sst = reinterpret_cast<State*>(lds + sizeof(double) * kTileCap * D);
  int* soff = reinterpret_cast<int*>(lds + sizeof(double) * kTileCap * D + sizeof(State) * kTileRows);
  const int tid = threadIdx.x;
  const int r0 = L.tile_ptr[t], nr = L.tile_ptr[t + 1] - r0;
  // phase 0: row states; exclusive scan of the row lengths (rows < 128: waves 0-1)
  int len = 0;
  if (tid < nr) {
    State st;
    p.load(L.rows[r0 + tid], st);
    sst[tid] = st;
    len = st.e1 - st.e0;
  }
  const int lane = tid & 63;
  int inc = len;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o);
    if (lane >= o) inc += v;
  }
  if (tid == 63) soff[kTileRows + 1] = inc;  // wave 0's total (scratch)
  __syncthreads();
  if (tid < 64) soff[tid + 1] = inc;
  else if (tid < 128) soff[tid + 1] = inc + soff[kTileRows + 1];
  if (tid == 0) soff[0] = 0;
  __syncthreads();
  const int total = soff[nr];
  // phase 1: one thread per entry; a fixed trip count with the entry index
  // clamped into the tile, so all of a thread's gathers can be in flight at once
  if (total > 0) {
    constexpr int U = kTileCap / kRowT;
    int es[U], ss[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = min(tid + kRowT * u, total - 1);
      int lo = 0, hi = nr;  // last s with soff[s] <= q
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (soff[mid] <= q) lo = mid;
        else hi = mid;
      }
      ss[u] = lo;
      es[u] = q - soff[lo];
    }
    double tt[U][D];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const State& st = sst[ss[u]];
#pragma unroll
      for (int k = 0; k < D; ++k) tt[u][k] = 0.0;
      p.term(st, st.e0 + es[u], tt[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (tid + kRowT * u < total)
#pragma unroll
        for (int k = 0; k < D; ++k) tb[k * kTileCap + tid + kRowT * u] = tt[u][k];
  }
  __syncthreads();
  // phase 2: one lane per (row, dimension), the row's terms in order
  for (int x = tid; x < nr * D; x += kRowT) {
    const int s = x / D, k = x - s * D;
    const int b = soff[s];
    sst[s].acc[k] = lane_chain_any(sst[s].acc[k], tb + k * kTileCap + b, soff[s + 1] - b);
  }
  __syncthreads();
  if (tid < nr) {
    State st = sst[tid];
    p.finish(st, true);
  }
}

// One segment of a heavy row (entries [a, b) of it, b - a <= kTileCap): the
// binade sums of its terms, added to the row's accumulators.
template <int D, class P>
__device__ __forceinline__ void segment_rows(const RowClasses& L, const P& p, int q, char* lds) {
  using State = typename P::State;
  long long* red = reinterpret_cast<long long*>(lds);  // [4 waves][2D]
  int* rflag = reinterpret_cast<int*>(lds + sizeof(long long) * 4 * 2 * D);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int h = L.seg[3 * q], a = L.seg[3 * q + 1], b = L.seg[3 * q + 2];
  State st;
  p.load(L.rows[h], st);
  int uexp[D];
  long long P0[D], S[D], A[D];
  int flag = 0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    if (!binade_base(st.acc[k], uexp[k], P0[k])) flag = 1;
    S[k] = A[k] = 0;
  }
  if (!flag) {
    constexpr int U = kTileCap / kRowT;
    double tt[U][D];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = st.e0 + min(a + tid + kRowT * u, b - 1);
#pragma unroll
      for (int k = 0; k < D; ++k) tt[u][k] = 0.0;
      p.term(st, e, tt[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (a + tid + kRowT * u < b)
#pragma unroll
        for (int k = 0; k < D; ++k) {
          const long long r = binade_term(tt[u][k], uexp[k], flag);
          S[k] += r;
          A[k] += r < 0 ? -r : r;
        }
  }
#pragma unroll
  for (int k = 0; k < D; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      S[k] += __shfl_xor(S[k], o);
      A[k] += __shfl_xor(A[k], o);
    }
  const bool any = __any(flag);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < D; ++k) {
      red[wv * 2 * D + 2 * k] = S[k];
      red[wv * 2 * D + 2 * k + 1] = A[k];
    }
    rflag[wv] = any ? 1 : 0;
  }
  __syncthreads();
  if (tid < 2 * D) {
    const long long v = red[tid] + red[2 * D + tid] + red[4 * D + tid] + red[6 * D + tid];
    atomicAdd(reinterpret_cast<unsigned long long*>(L.hacc + (size_t)h * 2 * D + tid),
              (unsigned long long)v);
  }
  if (tid == 0 && (rflag[0] | rflag[1] | rflag[2] | rflag[3])) atomicOr(L.hflag + h, 1);
}

// After every segment: one wave per heavy row turns its binade sums into the
// row's force (or, when they do not apply, adds its terms serially in stored
// order), then gravity and the update; the accumulators are zeroed for the
// next pass.
template <int D, class P>
__global__ void __launch_bounds__(kRowT) heavy_finish_kernel(RowClasses L, P p) {
  __shared__ __attribute__((aligned(16))) double buf[4 * 64 * D];
  const int tid = threadIdx.x, lane = tid & 63;
  const int h = blockIdx.x * 4 + (tid >> 6);
  if (h >= L.nheavy) return;  // wave-uniform
  typename P::State st;
  p.load(L.rows[h], st);
  long long* acc = L.hacc + (size_t)h * 2 * D;
  bool ok = L.hflag[h] == 0;
  double sum[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    int uexp;
    long long P0;
    ok = ok && binade_base(st.acc[k], uexp, P0) && binade_result(P0, uexp, acc[2 * k], acc[2 * k + 1], sum[k]);
  }
  if (ok) {
#pragma unroll
    for (int k = 0; k < D; ++k) st.acc[k] = sum[k];
  } else {
    ordered_edge_sum<D, 1>(st.e0, st.e1, lane, buf + (tid >> 6) * 64 * D,
                           [&](int e, double (&t)[D]) { p.term(st, e, t); }, st.acc);
  }
  p.finish(st, lane == 0);
  wave_lds_sync();  // every lane has read the accumulators
  if (lane < 2 * D) acc[lane] = 0;
  if (lane == 0) L.hflag[h] = 0;
}

// kSegStore, phase A: the terms of one segment of a heavy row, stored
// dimension-major in the row's region of L.hterm.
template <int D, class P>
__device__ __forceinline__ void segment_store(const RowClasses& L, const P& p, int q) {
  using State = typename P::State;
  const int tid = threadIdx.x;
  const int h = L.seg[3 * q], a = L.seg[3 * q + 1], b = L.seg[3 * q + 2];
  State st;
  p.load(L.rows[h], st);
  const int deg = st.e1 - st.e0;
  double* out = L.hterm + L.hoff[h];
  constexpr int U = kTileCap / kRowT;
  double tt[U][D];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = st.e0 + min(a + tid + kRowT * u, b - 1);
#pragma unroll
    for (int k = 0; k < D; ++k) tt[u][k] = 0.0;
    p.term(st, e, tt[u]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int l = a + tid + kRowT * u;
    if (l < b)
#pragma unroll
      for (int k = 0; k < D; ++k) out[(size_t)k * deg + l] = tt[u][k];
  }
}

// kSegStore, phase B: one wave per heavy row adds the stored terms in order
// (lane k: dimension k) while the whole wave loads the next chunk of them from
// HBM into registers; then the chunk goes to LDS (one buffer: it is written after
// the adds of the one before), and at the end gravity and the update.
constexpr int kStoreChunk = 512;  // terms per dimension per chunk
// CH: terms per dimension per chunk, B: lane_chain's block.  The early rows (long
// chains) take 512 / 16; the others 256 / 8, which halves the registers and so
// doubles the waves in flight: their launch is many short chains, bound by the
// latency of each one's loads rather than by its adds.  (Round 5 kept two LDS
// buffers of 512: 24 KB per one-wave block at D = 3 held a CU to 6 chain waves.)
template <int D, class P, int CH = kStoreChunk, int B = 16>
__global__ void __launch_bounds__(64) heavy_chain_kernel(RowClasses L, P p, int h0 = 0) {
  __shared__ __attribute__((aligned(16))) double buf[D * CH];
  const int lane = threadIdx.x;
  const int h = blockIdx.x + h0;
  typename P::State st;
  p.load(L.rows[h], st);
  const int deg = st.e1 - st.e0;
  const double* in = L.hterm + L.hoff[h];
  const int kd = lane < D ? lane : D - 1;
  double a = lane_dim_value<D>(st.acc, kd);
  constexpr int PER = D * CH / 64;  // values per lane per chunk
  double v[PER];
  auto fetch = [&](int c0) {  // chunk [c0, c0 + CH) of every dimension
#pragma unroll
    for (int r = 0; r < PER; ++r) {
      const int x = lane + 64 * r;  // dimension x / CH, item x % CH
      const int k = x / CH, l = c0 + x % CH;
      v[r] = l < deg ? in[(size_t)k * deg + l] : 0.0;
    }
  };
  auto put = [&](double* dst) {
#pragma unroll
    for (int r = 0; r < PER; ++r) dst[lane + 64 * r] = v[r];
  };
  if (deg > 0) {
    fetch(0);
    put(buf);
  }
  for (int c0 = 0; c0 < deg; c0 += CH) {
    wave_lds_sync();  // the chunk at c0 is in buf
    const bool more = c0 + CH < deg;
    if (more) fetch(c0 + CH);  // in flight during the adds below
    a = lane_chain<B>(a, buf + kd * CH, min(CH, deg - c0));
    wave_lds_sync();  // every lane has read the chunk
    if (more) put(buf);
  }
#pragma unroll
  for (int k = 0; k < D; ++k) st.acc[k] = __shfl(a, k);
  p.finish(st, lane == 0);
}

// Tiles get their own kernel: without the heavy path's registers and LDS it
// keeps several blocks per CU in flight (the pass is gather-latency bound).
// Block b: tile tile0 + b (b < nt), else heavy-row segment seg0 + (b - nt): every
// tile then every segment, or (kSegStore) the tiles alone / a range of segments alone.

template <int D, class P>
__global__ void __launch_bounds__(kRowT) tile_rows_kernel(RowClasses L, P p, int tile0, int nt,
                                                          int seg0) {
  __shared__ __attribute__((aligned(16))) char lds[RowsLds<D, P>::tile];
  const int b = (int)blockIdx.x;
  if (b < nt)
    tile_rows<D>(L, p, tile0 + b, lds);
  else if (L.seg_mode == kSegStore)
    segment_store<D>(L, p, seg0 + b - nt);
  else
    segment_rows<D>(L, p, seg0 + b - nt, lds);
}

// P: a row policy with
//   struct State (holds acc[D] and the edge range e0, e1; trivially copyable)
//   load(row, State&), term(const State&, e, t[D]), finish(State&, bool writer).
template <int D, class P>
__global__ void __launch_bounds__(kRowT, GE_ROWS_MINBLOCKS) classed_rows_kernel(RowClasses L, P p) {
  __shared__ __attribute__((aligned(16))) char lds[RowsLds<D, P>::bytes];
  double* buf = reinterpret_cast<double*>(lds);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  typename P::State st;
  if (b < L.nheavy) {
    p.load(L.rows[b], st);
    ordered_edge_sum_split<D>(st.e0, st.e1, tid, buf,
                              [&](int e, double (&t)[D]) { p.term(st, e, t); }, st.acc);
    p.finish(st, tid == 0);
    return;
  }
  const int r_med = L.tile_off - L.nmed - L.nlight;  // first medium row
  const int mblocks = (L.nmed + 3) / 4;
  const int bm = b - L.nheavy;
  if (bm < mblocks) {
    const int q = bm * 4 + (tid >> 6);
    if (q >= L.nmed) return;  // wave-uniform; no block barrier on this path
    const int lane = tid & 63;
    p.load(L.rows[r_med + q], st);
    ordered_edge_sum<D, 1>(
        st.e0, st.e1, lane, buf + (tid >> 6) * 64 * D,
        [&](int e, double (&t)[D]) { p.term(st, e, t); }, st.acc);
    p.finish(st, lane == 0);
    return;
  }
  const int q = (bm - mblocks) * kRowT + tid;
  if (q >= L.nlight) return;
  p.load(L.rows[r_med + L.nmed + q], st);
  for (int e = st.e0; e < st.e1; ++e) {
    double t[D];
#pragma unroll
    for (int k = 0; k < D; ++k) t[k] = 0.0;
    p.term(st, e, t);
#pragma unroll
    for (int k = 0; k < D; ++k) st.acc[k] = st.acc[k] + t[k];
  }
  p.finish(st, true);
}

// Per-plan row resources: the side stream + events for running whole heavy rows
// beside the tiles, and the heavy rows' binade accumulators (segment mode).
struct RowStreams {
  DevBuf<long long> hacc, hoff;
  DevBuf<int> hflag;
  DevBuf<double> hterm;
  int nheavy = 0;
  // allocate (and zero) the heavy rows' segment buffers; deg: their entry
  // counts in rows order (kSegStore)
  void attach(RowClasses& rc, int D, hipStream_t s, const std::vector<int>& heavy_deg = {}) {
    if (rc.nseg == 0) return;
    if (rc.seg_mode == kSegStore) {
      std::vector<long long> off(rc.nheavy + 1, 0);
      for (int h = 0; h < rc.nheavy; ++h) off[h + 1] = off[h] + (long long)heavy_deg.at(h) * D;
      hoff.alloc(rc.nheavy + 1);
      hoff.upload(off.data(), off.size(), s);
      GE_HIP(hipStreamSynchronize(s));  // off is a local
      hterm.alloc(std::max<long long>(off[rc.nheavy], 1));
      rc.hoff = hoff.p;
      rc.hterm = hterm.p;
      return;
    }
    hacc.alloc((size_t)rc.nheavy * 2 * D);
    hflag.alloc(rc.nheavy);
    GE_HIP(hipMemsetAsync(hacc.p, 0, sizeof(long long) * hacc.n, s));
    GE_HIP(hipMemsetAsync(hflag.p, 0, sizeof(int) * hflag.n, s));
    rc.hacc = hacc.p;
    rc.hflag = hflag.p;
    nheavy = rc.nheavy;
  }
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, mid = nullptr;
  RowStreams() = default;
  RowStreams(const RowStreams&) = delete;
  RowStreams& operator=(const RowStreams&) = delete;
  ~RowStreams() {
    if (side) {
      (void)hipStreamSynchronize(side);
      (void)hipStreamDestroy(side);
    }
    if (fork) (void)hipEventDestroy(fork);
    if (join) (void)hipEventDestroy(join);
    if (mid) (void)hipEventDestroy(mid);
  }
  void ensure() {
    if (side) return;
    GE_HIP(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    GE_HIP(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    GE_HIP(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    GE_HIP(hipEventCreateWithFlags(&mid, hipEventDisableTiming));
  }
};

// All rows of `rc` on stream s (the heavy ones on rs.side when there are tiles;
// s waits for them before returning to the caller's next work).  Round 4 also
// queued the heavy rows' segment terms beside the multilevel repulsion launch
// (they need only the coordinates): bit-exact, the pass fell from 3.54 to 2.2-2.4 ms
// but the repulsion launch beside it rose from 136.3 to 141-142 ms
// (profiles/r04/ab_rows_early.log); removed in round 5.
template <int D, class P>
inline void launch_rows(const RowClasses& rc, const P& p, hipStream_t s, RowStreams& rs) {
  const int tgrid = rc.ntiles + rc.nseg;
  if (rc.nseg > 0 && rc.seg_mode == kSegStore && rc.ntiles > 0 &&
      !std::getenv("GE_ROWS_SERIAL")) {
    // a heavy row's chain (its terms stored by its segment blocks, then one dependent
    // add per term) is independent of the tiles.  The early rows (the longest chains)
    // store their segments and run their chains on the side stream; the caller's
    // stream stores the other heavy rows' segments and then runs the tiles, while the
    // side stream, once those segments are stored, runs their (short) chains.  C4
    // (profiles/r06/rows_timeline_c4.txt): early segments 0-0.2 ms, early chains to
    // 1.2 ms; other segments to 1.2 ms, tiles to 2.6 ms beside the other chains
    // (1.22-1.58 ms).  Round 5 stored all segments and then ran all chains on the side
    // stream beside the tiles (2.07 + 1.43 ms: the 135 339-entry row's chain started
    // last); DESIGN.md 5d has the variants measured.
    const int nlate = rc.nseg - rc.nseg_early;
    rs.ensure();
    GE_HIP(hipEventRecord(rs.fork, s));
    GE_HIP(hipStreamWaitEvent(rs.side, rs.fork, 0));
    if (rc.nearly > 0) {
      hipLaunchKernelGGL((tile_rows_kernel<D, P>), dim3(rc.nseg_early), dim3(kRowT), 0, rs.side,
                         rc, p, 0, 0, 0);
      hipLaunchKernelGGL((heavy_chain_kernel<D, P>), dim3(rc.nearly), dim3(64), 0, rs.side, rc, p,
                         0);
    }
    if (nlate > 0) {
      hipLaunchKernelGGL((tile_rows_kernel<D, P>), dim3(nlate), dim3(kRowT), 0, s, rc, p, 0, 0,
                         rc.nseg_early);
      GE_HIP(hipEventRecord(rs.mid, s));
      GE_HIP(hipStreamWaitEvent(rs.side, rs.mid, 0));
      hipLaunchKernelGGL((heavy_chain_kernel<D, P, 256, 8>), dim3(rc.nheavy - rc.nearly), dim3(64),
                         0, rs.side, rc, p, rc.nearly);
    }
    hipLaunchKernelGGL((tile_rows_kernel<D, P>), dim3(rc.ntiles), dim3(kRowT), 0, s, rc, p, 0,
                       rc.ntiles, 0);
    GE_HIP(hipEventRecord(rs.join, rs.side));
    GE_HIP(hipStreamWaitEvent(s, rs.join, 0));
    return;
  }
  if (rc.nseg > 0) {  // heavy rows as segments, then their sums and finish
    hipLaunchKernelGGL((tile_rows_kernel<D, P>), dim3(tgrid), dim3(kRowT), 0, s, rc, p, 0,
                       rc.ntiles, 0);
    if (rc.seg_mode == kSegStore)
      hipLaunchKernelGGL((heavy_chain_kernel<D, P>), dim3(rc.nheavy), dim3(64), 0, s, rc, p);
    else
      hipLaunchKernelGGL((heavy_finish_kernel<D, P>), dim3((rc.nheavy + 3) / 4), dim3(kRowT), 0,
                         s, rc, p);
    return;
  }
  if (rc.ntiles > 0 && rc.nheavy > 0 && std::getenv("GE_ROWS_SERIAL")) {  // tuning: no overlap
    hipLaunchKernelGGL((classed_rows_kernel<D, P>), dim3(rc.nheavy), dim3(kRowT), 0, s, rc, p);
    hipLaunchKernelGGL((tile_rows_kernel<D, P>), dim3(tgrid), dim3(kRowT), 0, s, rc, p, 0,
                       rc.ntiles, 0);
  } else if (rc.ntiles > 0 && rc.nheavy > 0) {
    rs.ensure();
    GE_HIP(hipEventRecord(rs.fork, s));
    GE_HIP(hipStreamWaitEvent(rs.side, rs.fork, 0));
    hipLaunchKernelGGL((classed_rows_kernel<D, P>), dim3(rc.nheavy), dim3(kRowT), 0, rs.side, rc, p);
    hipLaunchKernelGGL((tile_rows_kernel<D, P>), dim3(tgrid), dim3(kRowT), 0, s, rc, p, 0,
                       rc.ntiles, 0);
    GE_HIP(hipEventRecord(rs.join, rs.side));
    GE_HIP(hipStreamWaitEvent(s, rs.join, 0));
  } else if (rc.ntiles > 0) {
    hipLaunchKernelGGL((tile_rows_kernel<D, P>), dim3(tgrid), dim3(kRowT), 0, s, rc, p, 0,
                       rc.ntiles, 0);
  } else if (rc.grid() > 0) {
    hipLaunchKernelGGL((classed_rows_kernel<D, P>), dim3(rc.grid()), dim3(kRowT), 0, s, rc, p);
  }
}

}  // namespace ge
