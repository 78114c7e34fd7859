// ge_partition_dev.hip -- the coarsening hierarchy (partition::partition,
// src/partitioner.cpp:1550-1893) on gfx950, bit-exact with the reference.
//
// What one round of the reference does, and what it amounts to:
//
//  * scan (:1703-1726): every alive vertex i with !notouch[i] (or max_eta = -inf)
//    takes the neighbour j with the largest eta = 2*(a_ij/T - alpha_i*alpha_j)
//    over untouched j; the ascending-j walk with strict `>` selects the
//    smallest j among the maxima.  That is a segmented argmax under the total
//    order (eta desc, j asc), so any split of a neighbourhood across lanes
//    reduces to the same (max_eta, max_ind).
//  * greedy resolve (:1728-1753): in `used` order, i merges with j = max_ind[i]
//    when neither is touched yet, !(max_eta[i] < max_eta[j]) and (under
//    positiveMerging) max_eta[i] > 0.  max_eta / max_ind do not change during
//    the resolve, only the touched flags do, so the resolve is the greedy
//    matching of the candidate edges (i, max_ind[i]) taken in the order of the
//    proposer's `used` slot.  That matching is what the parallel "locally
//    dominant" rounds compute exactly: an edge whose rank is the smallest among
//    the live edges at both its endpoints is taken, edges touching a taken
//    vertex die, repeat (the globally smallest live edge is always taken, so the
//    loop ends).
//  * contraction (:1756-1779): the round's merges form a matching, so the new
//    adjacency is the quotient graph with summed weights and
//    alpha[i'] = alpha[i'] + alpha[j'].  For integer weights every sum is exact
//    in any order, so lists are rebuilt with hash tables and atomics.  Non-integer
//    weights keep the host path (ge_partition.cpp), where the += order is the
//    reference's.
//  * swap-pop of `used`, union-find, snapshots (:1797-1834): O(merges) per round,
//    sequential and order-dependent -> on the host, mirrored into the device
//    rank array (rank[v] = pointer[v]) by uploading only the changed slots.
//
// Data on the device: per-vertex neighbour lists (keys int32, weights fp64) in
// a pool with per-vertex offset / length / capacity.  Lists keep no order
// (the scan is order-free) and no duplicate keys (so the list length is the
// reference's map size, which orients each merge, :1737-1743).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <numeric>
#include <memory>
#include <vector>

#include "ge_internal.hpp"
#include "ge_prim.hpp"

namespace ge {
namespace {

constexpr int kNone = 0x7F7F7F7F;  // lock sentinel (memset byte 0x7F), above every rank
constexpr int kSmallLen = 16;      // scan: one thread per vertex up to this many entries
constexpr int kMidLen = 512;       // scan: one wave per vertex up to this many entries
constexpr int kBigLen = 16384;     // scan: one 256-thread block up to this, then 1024 threads
constexpr int kWaveNeed = 64;      // rebuild: one wave (128-slot LDS table) up to this
constexpr int kBlockNeed = 2048;   // rebuild: one block (4096-slot LDS table) up to this
constexpr int kBlockSlots = 4096;
// Hub lists (longer than kPatchMin) are patched in place after a round instead of
// rebuilt (patch_list): at most kPatchGone absorbed neighbours and a partner list
// of at most kPatchGone entries, in LDS sets of kPatchSet slots.
constexpr int kPatchMin = kBlockNeed;
constexpr int kPatchGone = 1024;
constexpr int kPatchSet = 4096;
constexpr int kPairCap = 1 << 22;
constexpr int kPatchU = 16;
constexpr int kSpecMerges = 4096;  // merge records copied with the round's counts

enum {
  C_SMALL,
  C_MID,
  C_BIG,
  C_PROP,
  C_CAND,
  C_MERGE,
  C_DIRTY,
  C_W,
  C_B,
  C_G,
  C_OVF,
  C_BAD,  // eligibility flags
  C_ALIVE2,
  C_CAND2,
  C_HUGE,
  C_PAIR,   // (hub, absorbed neighbour) pairs of this round's contraction
  C_PATCH,  // hub lists patched in place this round (profiling)
  C_PTOP,   // bucket space handed out to the hubs' absorbed-neighbour lists
  C_PF_SHORT, C_PF_SIZE, C_PF_FIT,  // lists rebuilt instead: short, sets too small, no room
  // the per-pass and per-contraction counters are zeroed by the kernels that
  // follow their last reader (no memset per round); their final values are kept
  // here for the profile
  C_SH_SMALL, C_SH_MID, C_SH_BIG, C_SH_PROP, C_SH_CAND, C_SH_HUGE,
  C_SH_DIRTY, C_SH_W, C_SH_B, C_SH_G,
  C_R_CHG, C_R_BOUND, C_R_PASS,  // rescans of lists > kSmallLen by reason (profile)
  NCNT
};

struct MergeRec {
  int keep, gone, rank, pass;
  double eta;
  int len_keep, len_gone;
};

struct Dev {
  int N;
  int positive;
  int incremental;  // all weights > 0: alphas only grow, see classify_scan_kernel
  double T;
  int* akey;
  double* aw;
  long long* aoff;
  int* alen;
  int* acap;
  double* alpha;
  int* alive;
  int* touched;
  int* rank;
  double* best;
  int* arg;
  int* rep;
  int* partner;
  int* dirty;
  int* lk;
  int* alist;   // alive vertices (may hold dead entries until the next compaction)
  int* alist2;
  int* late;    // last scan was a pass >= 1 scan (touched neighbours excluded)
  int* chg;     // round of the last change of the vertex's list or alpha
  int* kst;     // round in which the vertex last kept a merge (its alpha grew)
  int* small;
  int* mid;
  int* big;
  int* huge;
  int* prop;
  int* cand;
  int* cand2;
  int* cnt;
  MergeRec* mrec;
  int* dlist;
  int* lw;
  int* lb;
  int* lg;
  long long* gofs;
  int* gmask;
  int* gkey;
  double* gw;
  unsigned long long* gtop;
  unsigned long long* pool_top;
  long long pool_cap;
  int2* pairs;  // (hub, absorbed neighbour), kPairCap
  int* pcnt;    // per hub: pairs counted (mark_dirty), then the bucket fill cursor
  int2* pinfo;  // per hub: (bucket offset, pair count)
  int* pbuf;    // the buckets: each hub's absorbed neighbours, kPairCap
  // what the last pass-0 scan of a vertex found besides its argmax: the argmax,
  // its entry's weight and the best eta of every other entry (see classify_scan)
  int* t2arg;
  double* t2w;
  double* t2b2;
  // ... and its runner-up (key, weight) with the best eta of the remaining entries
  int* t2arg2;
  double* t2w2;
  double* t2b3;
  int patch;    // 0: every dirty list is rebuilt (GE_PARTITION_NO_PATCH)
  int prof;     // GE_PROFILE_PARTITION: count rescans by reason
};

__device__ inline int lane_id() { return threadIdx.x & 63; }

// Append `value` to list[] when pred (one atomic per wave).  Every lane of the
// wave that is still running must call it.
__device__ inline void wave_append(int* list, int* counter, bool pred, int value) {
  const unsigned long long m = __ballot(pred);
  if (!m) return;
  const int lane = lane_id();
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, __popcll(m));
  base = __shfl(base, leader);
  if (pred) list[base + __popcll(m & ((1ull << lane) - 1ull))] = value;
}

// Append `value` to lists[q] where pred[q], q < L, with one global atomic per
// list per block (a wave-level atomic per list contends at the L2 when every wave
// of a large grid appends).  Every thread of the block must call it; s: LDS int[2L].
template <int L>
__device__ inline void block_append(int* const (&lists)[L], int* const (&ctrs)[L],
                                    const bool (&pred)[L], int value, int* s) {
  const int lane = lane_id();
  if (threadIdx.x < L) s[threadIdx.x] = 0;
  __syncthreads();
  unsigned long long m[L];
  int woff[L];
#pragma unroll
  for (int q = 0; q < L; ++q) {
    m[q] = __ballot(pred[q]);
    int o = 0;
    if (lane == 0 && m[q]) o = atomicAdd(&s[q], __popcll(m[q]));
    woff[q] = __shfl(o, 0);
  }
  __syncthreads();
  if (threadIdx.x < L && s[threadIdx.x]) s[L + threadIdx.x] = atomicAdd(ctrs[threadIdx.x], s[threadIdx.x]);
  __syncthreads();
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int q = 0; q < L; ++q)
    if (pred[q]) lists[q][s[L + q] + woff[q] + __popcll(m[q] & below)] = value;
  __syncthreads();
}

// (eta desc, index asc): the reference's ascending walk with strict `>`
__device__ inline bool better(double e, int k, double be, int bk) {
  return e > be || (e == be && k < bk);
}

// Wait for this wave's outstanding memory operations (vmcnt/lgkmcnt = 0).  Before a
// __syncthreads() it orders this block's global atomics before the other waves'
// reads after the barrier -- the workgroup-scope fence of __syncthreads() does not
// wait for vector memory, and __threadfence() would write back the whole L2.
__device__ inline void drain() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

__device__ inline int agent_load(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline double eta_of(const Dev& d, double w, double au, int k) {
  return 2.0 * (w / d.T - au * d.alpha[k]);  // :1715 (no contraction: -ffp-contract=off)
}

// Running (argmax, runner-up, best eta of the other entries) of a scan, under
// the scan's total order (eta desc, index asc); merge() combines two partial
// scans of disjoint entry sets.
struct Top {
  double be = -INFINITY, bw = 0.0, e2 = -INFINITY, w2 = 0.0, e3 = -INFINITY;
  int bk = INT_MAX, k2 = INT_MAX;
  __device__ void add(double e, int k, double w) {
    if (better(e, k, be, bk)) {
      e3 = fmax(e3, e2);
      e2 = be;
      k2 = bk;
      w2 = bw;
      be = e;
      bk = k;
      bw = w;
    } else if (better(e, k, e2, k2)) {
      e3 = fmax(e3, e2);
      e2 = e;
      k2 = k;
      w2 = w;
    } else {
      e3 = fmax(e3, e);
    }
  }
  __device__ void merge(const Top& o) {
    e3 = fmax(e3, o.e3);
    add(o.be, o.bk, o.bw);
    add(o.e2, o.k2, o.w2);
  }
  __device__ Top shfl_xor(int m) const {
    Top o;
    o.be = __shfl_xor(be, m);
    o.bw = __shfl_xor(bw, m);
    o.e2 = __shfl_xor(e2, m);
    o.w2 = __shfl_xor(w2, m);
    o.e3 = __shfl_xor(e3, m);
    o.bk = __shfl_xor(bk, m);
    o.k2 = __shfl_xor(k2, m);
    return o;
  }
};

__device__ inline void scan_store(const Dev& d, int u, int pass, const Top& t, bool& prop) {
  d.best[u] = t.be;
  d.arg[u] = t.bk == INT_MAX ? -1 : t.bk;
  prop = t.bk != INT_MAX && (!d.positive || t.be > 0.0);
  if (pass == 0) {
    d.t2arg[u] = t.bk == INT_MAX ? -1 : t.bk;
    d.t2w[u] = t.bw;
    d.t2b2[u] = fmax(t.e2, t.e3);
    d.t2arg2[u] = t.k2 == INT_MAX ? -1 : t.k2;
    d.t2w2[u] = t.w2;
    d.t2b3[u] = t.e3;
  }
}

// ---- scan (:1703-1726) -----------------------------------------------------
// Which alive vertices the reference's scan would give a different answer than
// the one each vertex already holds; those are rescanned, the others keep their
// (max_eta, max_ind) -- the same values a rescan returns:
//  * pass 0: a vertex whose list or alpha changed in the last contraction
//    (chg), whose max_ind kept a merge (its alpha grew, so the eta towards it
//    fell), or whose last scan excluded touched neighbours (late).  With
//    positive weights every alpha is positive and only grows, so the eta towards
//    any other neighbour can only fall (RN rounding is monotone): the argmax and
//    its eta stay.
//  * pass >= 1 (:1706, untouched j only at :1712): an untouched vertex whose
//    max_ind is untouched keeps it -- the max over a subset that holds the old
//    argmax -- so only those whose max_ind was touched rescan (and touched ones
//    with max_eta = -inf, the reference's own rule).
// Vertices that keep their result and have a usable candidate go straight to the
// proposer list; the rescans are split by list length.
__global__ void classify_scan_kernel(Dev d, int pass, int L, int round, int full, int last) {
  __shared__ int s_app[6];
  if (pass == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
    // the previous contraction's counters (every reader has run) and the merge count
    for (int q = 0; q < 4; ++q) {
      d.cnt[C_SH_DIRTY + q] = d.cnt[C_DIRTY + q];  // DIRTY W B G
      d.cnt[C_DIRTY + q] = 0;
    }
    *d.gtop = 0;
    d.cnt[C_MERGE] = 0;
  }
  const int stride = gridDim.x * blockDim.x;
  const int rounds = (L + stride - 1) / stride;
  for (int r = 0; r < rounds; ++r) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x + r * stride;
    int u = 0;
    bool resc = false, keepprop = false;
    int len = 0, why = 0;
    if (x < L) {
      u = d.alist[x];
      if (d.alive[u]) {
        const bool tu = d.touched[u];
        const int a = d.arg[u];
        if (pass == 0) {
          resc = full || !d.incremental || d.chg[u] == round - 1;
          why = resc ? 1 : 0;
          if (!resc && (d.late[u] || (a >= 0 && d.kst[a] == round - 1))) {
            why = 2;
            // The last pass-0 scan's argmax a0 may have lost eta (its alpha grew)
            // or been excluded since (late).  u's list and alpha are unchanged
            // since that scan (chg), and every other alpha only grew, so every
            // other entry's eta is still <= the be2 that scan recorded: if a0's
            // eta now, computed as a scan computes it, exceeds be2, a0 is the
            // argmax and that eta the max -- what a rescan returns.
            const int a0 = d.t2arg[u];
            bool skip = false;
            if (a0 >= 0) {
              const double e = eta_of(d, d.t2w[u], d.alpha[u], a0);
              if (e > d.t2b2[u]) {
                d.best[u] = e;
                d.arg[u] = a0;
                d.late[u] = 0;
                skip = true;
              }
            }
            resc = !skip;
          }
        } else if (!tu) {
          resc = !d.incremental || (a >= 0 && d.touched[a]);
          why = 3;
          const int k2 = d.t2arg2[u];
          if (resc && d.incremental && a >= 0 && a == d.t2arg[u] && k2 >= 0 && !d.touched[k2]) {
            // The argmax a of the last pass-0 scan is touched.  Every entry but a
            // and its runner-up k2 has eta <= the b3 that scan recorded (the bound
            // argument above), so if k2 is untouched and its eta now exceeds b3,
            // k2 is the best untouched entry -- what the rescan returns.
            const double e = eta_of(d, d.t2w2[u], d.alpha[u], k2);
            if (e > d.t2b3[u]) {
              d.best[u] = e;
              d.arg[u] = k2;
              d.late[u] = 1;
              resc = false;
            }
          }
          if (resc && d.incremental && last && d.positive && a >= 0 && a == d.t2arg[u] &&
              d.t2b2[u] <= 0.0) {
            // The last pass under positiveMerging: every entry but a has eta <=
            // be2 <= 0 (the pass-0 bound above), so u's best over its untouched
            // entries is <= 0.  u cannot propose, and a proposer i pointing at u
            // (best[i] > 0) passes !(best[i] < best[u]) for any best[u] <= 0: the
            // bound stands in for the rescan.  Nothing reads it after this pass
            // (late: the next pass 0 goes through the bound or rescans).
            d.best[u] = d.t2b2[u];
            d.arg[u] = -1;
            d.late[u] = 1;
            resc = false;
          }
        } else {
          resc = d.best[u] == -INFINITY;
        }
        if (resc) len = d.alen[u];
        else keepprop = !tu && d.arg[u] >= 0 && (!d.positive || d.best[u] > 0.0);
      }
    }
    int* const lists[3] = {d.small, d.mid, d.prop};
    int* const ctrs[3] = {&d.cnt[C_SMALL], &d.cnt[C_MID], &d.cnt[C_PROP]};
    const bool pr[3] = {resc && len <= kSmallLen, resc && len > kSmallLen, keepprop};
    block_append<3>(lists, ctrs, pr, u, s_app);
    if (d.prof) {
#pragma unroll
      for (int q = 1; q <= 3; ++q) {
        const unsigned long long m = __ballot(resc && len > kSmallLen && why == q);
        if (lane_id() == 0 && m) atomicAdd(&d.cnt[C_R_CHG + q - 1], __popcll(m));
      }
    }
  }
}

// one thread per vertex of the small list
__global__ void scan_small_kernel(Dev d, int pass) {
  __shared__ int s_app[2];
  const int count = d.cnt[C_SMALL];
  const int stride = gridDim.x * blockDim.x;
  const int rounds = (count + stride - 1) / stride;
  for (int r = 0; r < rounds; ++r) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x + r * stride;
    bool prop = false;
    int u = 0;
    if (x < count) {
      u = d.small[x];
      const int len = d.alen[u];
      Top b;
      const double au = d.alpha[u];
      const long long o = d.aoff[u];
      for (int t = 0; t < len; ++t) {
        const int k = d.akey[o + t];
        if (pass > 0 && d.touched[k]) continue;
        const double w = d.aw[o + t];
        b.add(eta_of(d, w, au, k), k, w);
      }
      scan_store(d, u, pass, b, prop);
      d.late[u] = pass > 0;
      prop = prop && !d.touched[u];
    }
    int* const lists[1] = {d.prop};
    int* const ctrs[1] = {&d.cnt[C_PROP]};
    const bool pr[1] = {prop};
    block_append<1>(lists, ctrs, pr, u, s_app);
  }
}

// Scan entries [b, e) of u's list with `stride` cooperating threads, 4 in flight.
__device__ inline void scan_range(const Dev& d, int pass, int u, int b, int e, int stride,
                                  Top& bt) {
  const double au = d.alpha[u];
  const long long o = d.aoff[u];
  int t = b;
  for (; t + 3 * stride < e; t += 4 * stride) {
    int k[4];
    double w[4], a[4];
    int tc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      k[q] = d.akey[o + t + q * stride];
      w[q] = d.aw[o + t + q * stride];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = d.alpha[k[q]];
      tc[q] = pass > 0 ? d.touched[k[q]] : 0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (tc[q]) continue;
      bt.add(2.0 * (w[q] / d.T - au * a[q]), k[q], w[q]);  // eta_of
    }
  }
  for (; t < e; t += stride) {
    const int k = d.akey[o + t];
    if (pass > 0 && d.touched[k]) continue;
    const double w = d.aw[o + t];
    bt.add(eta_of(d, w, au, k), k, w);
  }
}

__device__ inline void wave_argmax(Top& b) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) b.merge(b.shfl_xor(o));
}

// one wave per vertex of the mid list; longer lists go on to the big list
__global__ void __launch_bounds__(256) scan_mid_kernel(Dev d, int pass) {
  __shared__ int s_app[6];
  const int lane = lane_id();
  const int wib = threadIdx.x >> 6;  // wave in block (4 waves)
  const int count = d.cnt[C_MID];
  for (int base = blockIdx.x * 4; base < count; base += gridDim.x * 4) {
    const int x = base + wib;
    int u = 0, len = 0;
    bool prop = false;
    if (x < count) {
      u = d.mid[x];
      len = d.alen[u];
      if (len <= kMidLen) {
        Top b;
        scan_range(d, pass, u, lane, len, 64, b);
        wave_argmax(b);
        if (lane == 0) {
          scan_store(d, u, pass, b, prop);
          d.late[u] = pass > 0;
          prop = prop && !d.touched[u];
        }
      }
    }
    // appends aggregated per block (same-address atomics from every wave serialise)
    int* const lists[3] = {d.prop, d.big, d.huge};
    int* const ctrs[3] = {&d.cnt[C_PROP], &d.cnt[C_BIG], &d.cnt[C_HUGE]};
    const bool pr[3] = {prop, lane == 0 && x < count && len > kMidLen && len <= kBigLen,
                        lane == 0 && x < count && len > kBigLen};
    block_append<3>(lists, ctrs, pr, u, s_app);
  }
}

// one block per vertex of the big (T = 256) or huge (T = 1024) list
template <int T>
__global__ void __launch_bounds__(T) scan_big_kernel(Dev d, int pass) {
  __shared__ __attribute__((aligned(16))) char st_raw[16 * sizeof(Top)];  // (Top has initialisers)
  Top* st = reinterpret_cast<Top*>(st_raw);
  const int count = d.cnt[T == 1024 ? C_HUGE : C_BIG];
  const int* list = T == 1024 ? d.huge : d.big;
  const int tid = threadIdx.x;
  for (int x = blockIdx.x; x < count; x += gridDim.x) {
    const int u = list[x];
    const int len = d.alen[u];
    Top b;
    scan_range(d, pass, u, tid, len, blockDim.x, b);
    wave_argmax(b);
    if (lane_id() == 0) st[tid >> 6] = b;
    __syncthreads();
    if (tid < 64) {
      Top c;
      if (tid < (int)(blockDim.x >> 6)) c = st[tid];
      wave_argmax(c);
      if (tid == 0) {
        bool prop;
        scan_store(d, u, pass, c, prop);
        d.late[u] = pass > 0;
        if (prop && !d.touched[u]) d.prop[atomicAdd(&d.cnt[C_PROP], 1)] = u;
      }
    }
    __syncthreads();
  }
}

// Lists longer than kBigLen (hubs: up to 652 K entries at C4): kHugeChunks
// blocks per list, each scanning one contiguous chunk into a partial (argmax,
// weight, runner-up) -- the order-free reduction of the same (eta desc, index
// asc) total order -- and one wave per list combining the partials.
constexpr int kHugeChunks = 64;

__global__ void __launch_bounds__(1024) scan_huge_part_kernel(Dev d, int pass, Top* part,
                                                               int cap) {
  __shared__ __attribute__((aligned(16))) char st_raw[16 * sizeof(Top)];  // (Top has initialisers)
  Top* st = reinterpret_cast<Top*>(st_raw);
  const int count = min(d.cnt[C_HUGE], cap);  // (cap: nnz / kBigLen + 2 > any count)
  const int tid = threadIdx.x;
  for (int li = blockIdx.y; li < count; li += gridDim.y) {
    const int u = d.huge[li];
    const long long len = d.alen[u];
    const int b = (int)(len * blockIdx.x / kHugeChunks);
    const int e = (int)(len * (blockIdx.x + 1) / kHugeChunks);
    Top t;
    scan_range(d, pass, u, b + tid, e, blockDim.x, t);
    wave_argmax(t);
    if (lane_id() == 0) st[tid >> 6] = t;
    __syncthreads();
    if (tid < 64) {
      Top c;
      if (tid < (int)(blockDim.x >> 6)) c = st[tid];
      wave_argmax(c);
      if (tid == 0) part[(size_t)li * kHugeChunks + blockIdx.x] = c;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) scan_huge_final_kernel(Dev d, int pass, const Top* part,
                                                              int cap) {
  const int count = min(d.cnt[C_HUGE], cap);
  const int lane = lane_id();
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  static_assert(kHugeChunks == 64, "one partial per lane");
  for (int li = wave; li < count; li += nw) {
    Top c = part[(size_t)li * kHugeChunks + lane];
    wave_argmax(c);
    if (lane == 0) {
      const int u = d.huge[li];
      bool prop;
      scan_store(d, u, pass, c, prop);
      d.late[u] = pass > 0;
      if (prop && !d.touched[u]) d.prop[atomicAdd(&d.cnt[C_PROP], 1)] = u;
    }
  }
}

// ---- resolve (:1728-1753) ---------------------------------------------------
// candidate edges: untouched i, untouched j = max_ind[i], !(max_eta[i] < max_eta[j])
__global__ void filter_kernel(Dev d) {
  __shared__ int s_app[2];
  const int count = d.cnt[C_PROP];
  const int stride = gridDim.x * blockDim.x;
  const int first = blockIdx.x * blockDim.x + threadIdx.x;
  // uniform trip count per wave (wave_append needs every lane)
  const int rounds = (count + stride - 1) / stride;
  for (int r = 0; r < rounds; ++r) {
    const int x = first + r * stride;
    bool c = false;
    int i = 0;
    if (x < count) {
      i = d.prop[x];
      const int j = d.arg[i];
      c = !d.touched[i] && !d.touched[j] && !(d.best[i] < d.best[j]);
    }
    int* const lists[1] = {d.cand};
    int* const ctrs[1] = {&d.cnt[C_CAND]};
    const bool pr[1] = {c};
    block_append<1>(lists, ctrs, pr, i, s_app);
  }
}

__device__ inline void record_merge(const Dev& d, int i, int j, int r, int pass) {
  // :1737-1743: the larger map keeps (ties: the proposer i)
  const int li = d.alen[i], lj = d.alen[j];
  MergeRec m;
  if (li < lj) {
    m.keep = j;
    m.gone = i;
    m.len_keep = lj;
    m.len_gone = li;
  } else {
    m.keep = i;
    m.gone = j;
    m.len_keep = li;
    m.len_gone = lj;
  }
  m.rank = r;
  m.pass = pass;
  m.eta = d.best[i];
  d.mrec[atomicAdd(&d.cnt[C_MERGE], 1)] = m;
  d.touched[i] = 1;
  d.touched[j] = 1;
}

// The first locally-dominant round over the whole grid (most candidates of a
// late round are leaves pointing at the same hub: one round removes them).
// lk[v] = the smallest rank of the candidates touching v.  Most candidates of a
// late round propose to one of a few hubs (C4 round 2490: 371 679 candidates, 98
// merges), so the hub endpoints' minima are first taken in a per-block LDS table
// (keyed by vertex, open addressing over kMinSlots) and each table entry then
// makes one global atomicMin: the same minima with far fewer contended atomics.
// The proposer's own lock (distinct per candidate) goes straight to global.
constexpr int kMinSlots = 512;
__global__ void __launch_bounds__(256) resolve_min_kernel(Dev d) {
  __shared__ int s_key[kMinSlots];
  __shared__ int s_min[kMinSlots];
  for (int q = threadIdx.x; q < kMinSlots; q += blockDim.x) {
    s_key[q] = -1;
    s_min[q] = kNone;
  }
  __syncthreads();
  const int n = d.cnt[C_CAND];
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const int i = d.cand[c];
    const int j = d.arg[i];
    const int r = d.rank[i];
    atomicMin(&d.lk[i], r);
    bool done = false;
    int h = (int)(((unsigned)j * 2654435761u) >> 23) & (kMinSlots - 1);
    for (int probe = 0; probe < 8 && !done; ++probe, h = (h + 1) & (kMinSlots - 1)) {
      const int k = atomicCAS(&s_key[h], -1, j);
      if (k == -1 || k == j) {
        atomicMin(&s_min[h], r);
        done = true;
      }
    }
    if (!done) atomicMin(&d.lk[j], r);  // table crowded: directly
  }
  __syncthreads();
  for (int q = threadIdx.x; q < kMinSlots; q += blockDim.x)
    if (s_key[q] >= 0) atomicMin(&d.lk[s_key[q]], s_min[q]);
}

__global__ void resolve_select_kernel(Dev d, int pass) {
  const int n = d.cnt[C_CAND];
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n; c += gridDim.x * blockDim.x) {
    const int i = d.cand[c];
    const int j = d.arg[i];
    const int r = d.rank[i];
    if (d.lk[i] == r && d.lk[j] == r) record_merge(d, i, j, r, pass);
  }
}

__global__ void resolve_filter_kernel(Dev d) {
  __shared__ int s_app[2];
  const int n = d.cnt[C_CAND];
  const int stride = gridDim.x * blockDim.x;
  const int rounds = (n + stride - 1) / stride;
  for (int r = 0; r < rounds; ++r) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x + r * stride;
    int i = 0;
    bool live = false;
    if (c < n) {
      i = d.cand[c];
      const int j = d.arg[i];
      d.lk[i] = kNone;
      d.lk[j] = kNone;
      live = !d.touched[i] && !d.touched[j];
    }
    int* const lists[1] = {d.cand2};
    int* const ctrs[1] = {&d.cnt[C_CAND2]};
    const bool pr[1] = {live};
    block_append<1>(lists, ctrs, pr, i, s_app);
  }
}

constexpr int kLocalCand = 1024;   // LDS phase: candidates
constexpr int kLocalSlots = 4096;  // LDS phase: endpoint table (load <= 1/2)

// Greedy matching in rank order via locally-dominant rounds; one block.  While
// more than kLocalCand candidates are live the rounds run on global memory
// (vertex-indexed lock array); the rest runs in LDS (endpoints hashed to slots).
__device__ void resolve_block(Dev d, int pass, int cidx);

// The round's counters, pool top and first `spec` merge records written straight
// into pinned host memory by the round's last kernel (no blit copies, each of
// which waited ~15 us behind the last kernel).  System-scope vector stores; the
// stream synchronisation that follows completes the kernel and its release before
// the host reads them.
struct RoundExport {
  const unsigned long long* tops = nullptr;
  int* hcnt = nullptr;  // nullptr: not the round's last pass
  unsigned long long* htop = nullptr;
  int* hrec = nullptr;
  int* hseq = nullptr;  // the round number, written last (the host spins on it)
  int seq = 0;
  int spec = 0;
};

__device__ void export_round(const Dev& d, const RoundExport& ex) {
  const int t = threadIdx.x;
  for (int c = t; c < NCNT; c += blockDim.x)
    __hip_atomic_store(&ex.hcnt[c], d.cnt[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (t == 0) __hip_atomic_store(ex.htop, ex.tops[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int nw = min(d.cnt[C_MERGE], ex.spec) * (int)(sizeof(MergeRec) / sizeof(int));
  const int* src = reinterpret_cast<const int*>(d.mrec);
  for (int w = t; w < nw; w += blockDim.x)
    __hip_atomic_store(&ex.hrec[w], src[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // every thread's stores are complete at the system level before the round number
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t == 0) __hip_atomic_store(ex.hseq, ex.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The matching's last kernel of a pass; then the pass's list counters are zeroed
// for the next pass (every reader of them has run).  The round's last pass also
// exports the round (ex.hcnt set).
__global__ void __launch_bounds__(1024) resolve_kernel(Dev d, int pass, int cidx, RoundExport ex) {
  resolve_block(d, pass, cidx);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int from[6] = {C_SMALL, C_MID, C_BIG, C_PROP, C_CAND, C_HUGE};
    for (int q = 0; q < 6; ++q) {
      d.cnt[C_SH_SMALL + q] = d.cnt[from[q]];
      d.cnt[from[q]] = 0;
    }
    d.cnt[C_CAND2] = 0;
  }
  if (ex.hcnt) {
    __syncthreads();  // the merge records and the moved counters are complete
    export_round(d, ex);
  }
}

__device__ void resolve_block(Dev d, int pass, int cidx) {
  __shared__ int s_live;
  __shared__ int hk[kLocalSlots];
  __shared__ int hl[kLocalSlots];
  __shared__ unsigned char ht[kLocalSlots];
  __shared__ int ci[kLocalCand], cj[kLocalCand], cr[kLocalCand];
  __shared__ short si[kLocalCand], sj[kLocalCand];
  __shared__ short cl[2][kLocalCand];
  int* cur = d.cand;
  int* nxt = d.cand2;
  int n = d.cnt[cidx];
  const int tid = threadIdx.x, nt = blockDim.x;
  int iters = 0;
  while (n > kLocalCand) {
    if (++iters > (1 << 22)) {  // cannot happen: the smallest live rank is taken every round
      if (tid == 0) atomicMax(&d.cnt[C_OVF], 2);
      return;
    }
    for (int c = tid; c < n; c += nt) {
      const int i = cur[c];
      const int r = d.rank[i];
      atomicMin(&d.lk[i], r);
      atomicMin(&d.lk[d.arg[i]], r);
    }
    if (tid == 0) s_live = 0;
    drain();  // the L2 atomics are complete before any lane reads lk
    __syncthreads();
    for (int c = tid; c < n; c += nt) {
      const int i = cur[c];
      const int j = d.arg[i];
      const int r = d.rank[i];
      if (agent_load(&d.lk[i]) == r && agent_load(&d.lk[j]) == r) record_merge(d, i, j, r, pass);
    }
    drain();
    __syncthreads();
    for (int c = tid; c < n; c += nt) {
      const int i = cur[c];
      const int j = d.arg[i];
      atomicExch(&d.lk[i], kNone);
      atomicExch(&d.lk[j], kNone);
      if (!d.touched[i] && !d.touched[j]) nxt[atomicAdd(&s_live, 1)] = i;
    }
    drain();
    __syncthreads();
    n = s_live;
    int* t = cur;
    cur = nxt;
    nxt = t;
    __syncthreads();
  }
  if (n == 0) return;
  // ---- LDS phase
  for (int s = tid; s < kLocalSlots; s += nt) {
    hk[s] = -1;
    hl[s] = kNone;
    ht[s] = 0;
  }
  __syncthreads();
  for (int c = tid; c < n; c += nt) {
    const int i = cur[c];
    const int j = d.arg[i];
    ci[c] = i;
    cj[c] = j;
    cr[c] = d.rank[i];
    for (int e = 0; e < 2; ++e) {
      const int v = e == 0 ? i : j;
      unsigned h = ((unsigned)v * 2654435761u) & (kLocalSlots - 1);
      while (true) {
        const int prev = atomicCAS(&hk[h], -1, v);
        if (prev == -1 || prev == v) break;
        h = (h + 1) & (kLocalSlots - 1);
      }
      (e == 0 ? si : sj)[c] = (short)h;
    }
    cl[0][c] = (short)c;
  }
  __syncthreads();
  int b = 0;
  while (n > 0) {
    for (int x = tid; x < n; x += nt) {
      const int c = cl[b][x];
      atomicMin(&hl[si[c]], cr[c]);
      atomicMin(&hl[sj[c]], cr[c]);
    }
    if (tid == 0) s_live = 0;
    __syncthreads();
    for (int x = tid; x < n; x += nt) {
      const int c = cl[b][x];
      if (hl[si[c]] == cr[c] && hl[sj[c]] == cr[c]) {
        record_merge(d, ci[c], cj[c], cr[c], pass);
        ht[si[c]] = 1;
        ht[sj[c]] = 1;
      }
    }
    __syncthreads();
    for (int x = tid; x < n; x += nt) {
      const int c = cl[b][x];
      hl[si[c]] = kNone;
      hl[sj[c]] = kNone;
      if (!ht[si[c]] && !ht[sj[c]]) cl[b ^ 1][atomicAdd(&s_live, 1)] = (short)c;
    }
    __syncthreads();
    n = s_live;
    b ^= 1;
    __syncthreads();
  }
}

// ---- contraction (:1756-1779) -----------------------------------------------
__global__ void merge_apply_kernel(Dev d, int round) {
  const int count = d.cnt[C_MERGE];
  const int stride = gridDim.x * blockDim.x;
  const int rounds = (count + stride - 1) / stride;
  for (int r = 0; r < rounds; ++r) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x + r * stride;
    bool ok = x < count;
    int keep = 0;
    if (ok) {
      const MergeRec m = d.mrec[x];
      keep = m.keep;
      d.rep[m.gone] = keep;
      d.alive[m.gone] = 0;
      d.alpha[keep] = d.alpha[keep] + d.alpha[m.gone];  // :1770
      d.partner[keep] = m.gone;
      d.kst[keep] = round;
      d.dirty[keep] = 1;
      d.touched[keep] = 0;  // :1830
      d.touched[m.gone] = 0;
    }
    wave_append(d.dlist, &d.cnt[C_DIRTY], ok, keep);
  }
}

// every alive neighbour of an absorbed vertex gets a renamed entry: dirty
__global__ void mark_dirty_kernel(Dev d) {
  const int lane = lane_id();
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  const int count = d.cnt[C_MERGE];
  for (int x = wave; x < count; x += nw) {
    const int keep = d.mrec[x].keep, gone = d.mrec[x].gone;
    const int len = d.alen[gone];
    const long long o = d.aoff[gone];
    for (int b = 0; b < len; b += 64) {
      const int t = b + lane;
      bool mk = false, pr = false;
      int k = 0;
      if (t < len) {
        k = d.akey[o + t];
        const bool live = k != keep && d.rep[k] == k;
        mk = live && atomicCAS(&d.dirty[k], 0, 1) == 0;
        pr = d.patch && live && d.alen[k] > kPatchMin;  // a hub: patched, not rebuilt
      }
      wave_append(d.dlist, &d.cnt[C_DIRTY], mk, k);
      const unsigned long long pm = __ballot(pr);
      if (pm) {  // the pair (k, gone), capped (over the cap: no hub is patched this round)
        const int leader = __ffsll((long long)pm) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(&d.cnt[C_PAIR], __popcll(pm));
        base = __shfl(base, leader);
        const int at = base + __popcll(pm & ((1ull << lane) - 1ull));
        if (pr && at < kPairCap) d.pairs[at] = make_int2(k, gone);
        if (pr) atomicAdd(&d.pcnt[k], 1);
      }
    }
  }
}

__device__ inline unsigned pow2_at_least(unsigned x) {
  unsigned p = 1;
  while (p < x) p <<= 1;
  return p;
}

__global__ void classify_kernel(Dev d) {
  const int count = d.cnt[C_DIRTY];
  const int stride = gridDim.x * blockDim.x;
  const int rounds = (count + stride - 1) / stride;
  for (int r = 0; r < rounds; ++r) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x + r * stride;
    int u = 0, need = 0;
    if (x < count) {
      u = d.dlist[x];
      const int g = d.partner[u];
      need = d.alen[u] + (g >= 0 ? d.alen[g] : 0);
    }
    const bool w = x < count && need <= kWaveNeed;
    const bool b = x < count && need > kWaveNeed && need <= kBlockNeed;
    wave_append(d.lw, &d.cnt[C_W], w, u);
    wave_append(d.lb, &d.cnt[C_B], b, u);
    if (x < count && need > kBlockNeed) {
      const unsigned slots = pow2_at_least(2u * (unsigned)need);
      const int at = atomicAdd(&d.cnt[C_G], 1);
      d.lg[at] = u;
      d.gofs[at] = (long long)atomicAdd(d.gtop, (unsigned long long)slots);
      d.gmask[at] = (int)slots - 1;
      const int pc = d.pcnt[u];  // this hub's bucket of absorbed neighbours
      d.pinfo[u] = make_int2(pc > 0 ? atomicAdd(&d.cnt[C_PTOP], pc) : 0, pc);
      d.pcnt[u] = 0;
    }
  }
}

template <class T>
__device__ inline T tab_load(T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ inline unsigned slot_hash(int k) { return (unsigned)k * 2654435761u; }

// Rebuild u's list as sum_{members} (rep(k), w), dropping rep(k) == u, into a
// hash table (LDS or global) of mask+1 slots shared by `nt` threads; then write
// it back in place (fits) or to fresh pool space.
template <class Key, class W>
__device__ void rebuild_list(const Dev& d, int u, Key* tk, W* tw, int mask, int tid, int nt,
                             int* s_cnt, long long* s_dst) {
  for (int s = tid; s <= mask; s += nt) {
    tk[s] = -1;
    tw[s] = 0.0;
  }
  if (tid == 0) *s_cnt = 0;
  drain();
  __syncthreads();
  const int g = d.partner[u];
  for (int m = 0; m < 2; ++m) {
    const int v = m == 0 ? u : g;
    if (v < 0) break;
    const int len = d.alen[v];
    const long long o = d.aoff[v];
    for (int t = tid; t < len; t += nt) {
      const int r = d.rep[d.akey[o + t]];
      if (r == u) continue;  // the merged pair's own edge: into alpha (:1767-1770)
      const double w = d.aw[o + t];
      unsigned h = slot_hash(r) & (unsigned)mask;
      while (true) {
        const int prev = atomicCAS(&tk[h], -1, r);
        if (prev == -1 || prev == r) {
          atomicAdd(&tw[h], w);  // integer weights: exact in any order
          break;
        }
        h = (h + 1) & (unsigned)mask;
      }
    }
  }
  drain();  // (global tables) the atomics are complete before the table is read
  __syncthreads();
  for (int s0 = 0; s0 <= mask; s0 += nt) {  // used slots, one LDS atomic per wave
    const int s = s0 + tid;
    const unsigned long long m = __ballot(s <= mask && tab_load(&tk[s]) >= 0);
    if (lane_id() == 0 && m) atomicAdd(s_cnt, __popcll(m));
  }
  __syncthreads();
  const int count = *s_cnt;
  if (tid == 0) {
    long long dst = d.aoff[u];
    if (count > d.acap[u]) {
      const int cap = count + count / 2 + 4;
      dst = (long long)atomicAdd(d.pool_top, (unsigned long long)cap);
      if (dst + cap > d.pool_cap) {
        // atomicMax: a resolve that did not converge earlier in the round (2, a bug)
        // must not be masked by this capacity code (1, rerun on the host)
        atomicMax(&d.cnt[C_OVF], 1);
        dst = -1;
      } else {
        d.aoff[u] = dst;
        d.acap[u] = cap;
      }
    }
    *s_dst = dst;
    *s_cnt = 0;
    if (dst >= 0) d.alen[u] = count;
  }
  __syncthreads();
  const long long dst = *s_dst;
  if (dst >= 0) {
    for (int s0 = 0; s0 <= mask; s0 += nt) {
      const int s = s0 + tid;
      const int k = s <= mask ? tab_load(&tk[s]) : -1;
      const unsigned long long m = __ballot(k >= 0);
      int base = 0;
      if (lane_id() == 0 && m) base = atomicAdd(s_cnt, __popcll(m));
      base = __shfl(base, 0);
      if (k >= 0) {
        const int at = base + __popcll(m & ((1ull << lane_id()) - 1ull));
        d.akey[dst + at] = k;
        d.aw[dst + at] = tab_load(&tw[s]);
      }
    }
  }
  __syncthreads();
}

// the pairs into their hubs' buckets (when every pair was stored)
__global__ void pair_scatter_kernel(Dev d) {
  const int np = d.cnt[C_PAIR];
  if (np > kPairCap) return;
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < np; x += gridDim.x * blockDim.x) {
    const int2 pr = d.pairs[x];
    const int at = d.pinfo[pr.x].x + atomicAdd(&d.pcnt[pr.x], 1);
    if (at >= 0 && at < kPairCap) d.pbuf[at] = pr.y;  // (always: every pair's hub is in lg)
  }
}

// ---- hub lists patched in place ----------------------------------------------
// A hub's list changes in a round only where a neighbour was absorbed: that
// entry goes and its weight moves to the keeper's entry (which may be new), and
// when the hub itself kept a merge its partner's entries (renamed) are added and
// the partner's own entry goes.  mark_dirty_kernel recorded (hub, absorbed) pairs;
// the hub's list is read twice (coalesced, no gathers): once to find the absorbed
// entries, once to find the entries of the keys that receive weight.  The result
// is the rebuild's list up to entry order (lists keep no order; integer weights
// sum exactly in any order).  Returns false, having written nothing, when a set
// would overflow or the list outgrows its capacity: the caller rebuilds.
struct PatchLds {
  int gk[kPatchSet];    // absorbed neighbours in the list (set)
  int ik[kPatchSet];    // keys that receive weight (set)
  int ipos[kPatchSet];  // their position in the list, -1: a new entry
  double iw[kPatchSet];
  int del[kPatchGone + 1];  // positions of the absorbed entries
  int ngone, ndel, nnew, fill, ok;
};

__device__ inline int set_insert(int* keys, int key) {
  unsigned h = slot_hash(key) & (kPatchSet - 1);
  while (true) {
    const int prev = atomicCAS(&keys[h], -1, key);
    if (prev == -1 || prev == key) return (int)h;
    h = (h + 1) & (kPatchSet - 1);
  }
}

__device__ inline int set_find(const int* keys, int key) {
  unsigned h = slot_hash(key) & (kPatchSet - 1);
  while (true) {
    const int k = keys[h];
    if (k == key) return (int)h;
    if (k == -1) return -1;
    h = (h + 1) & (kPatchSet - 1);
  }
}

__device__ bool patch_list(const Dev& d, int u, PatchLds& s, int tid, int nt) {
  const int npairs = d.cnt[C_PAIR];
  const int g = d.partner[u];
  const int len = d.alen[u];
  const long long o = d.aoff[u];
  if (!d.patch) return false;
  if (len <= kPatchMin || npairs > kPairCap || (g >= 0 && d.alen[g] > kPatchGone)) {
    if (tid == 0) atomicAdd(&d.cnt[len <= kPatchMin ? C_PF_SHORT : C_PF_SIZE], 1);
    return false;  // uniform over the block
  }
  for (int x = tid; x < kPatchSet; x += nt) {
    s.gk[x] = -1;
    s.ik[x] = -1;
    s.ipos[x] = -1;
    s.iw[x] = 0.0;
  }
  if (tid == 0) {
    s.ngone = g >= 0 ? 1 : 0;
    s.ndel = s.nnew = s.fill = 0;
  }
  __syncthreads();
  const int2 pi = d.pinfo[u];
  if (pi.y + s.ngone > kPatchGone) {  // uniform
    if (tid == 0) atomicAdd(&d.cnt[C_PF_SIZE], 1);
    return false;
  }
  if (tid == 0 && g >= 0) set_insert(s.gk, g);  // the partner's own entry goes
  for (int x = tid; x < pi.y; x += nt) set_insert(s.gk, d.pbuf[pi.x + x]);
  __syncthreads();
  if (tid == 0) s.ngone += pi.y;
  // the keys that receive weight: the absorbed neighbours' keepers, and the
  // partner's entries renamed (its edge to u goes into alpha, :1767-1770)
  for (int x = tid; x < pi.y; x += nt) {
    const int r = d.rep[d.pbuf[pi.x + x]];
    if (r != u) set_insert(s.ik, r);
  }
  if (g >= 0) {
    const int glen = d.alen[g];
    const long long go = d.aoff[g];
    for (int t = tid; t < glen; t += nt) {
      const int r = d.rep[d.akey[go + t]];
      if (r != u) atomicAdd(&s.iw[set_insert(s.ik, r)], d.aw[go + t]);
    }
  }
  __syncthreads();
  // one pass over the list (kPatchU coalesced loads in flight per thread): the
  // absorbed entries go (their weight to their keeper's key), and the entries of
  // the keys that receive weight are located
  for (int t0 = 0; t0 < len; t0 += nt * kPatchU) {
    int k[kPatchU];
#pragma unroll
    for (int q = 0; q < kPatchU; ++q) {
      const int t = t0 + q * nt + tid;
      k[q] = t < len ? d.akey[o + t] : -1;
    }
#pragma unroll
    for (int q = 0; q < kPatchU; ++q) {
      if (k[q] < 0) continue;
      const int t = t0 + q * nt + tid;
      if (set_find(s.gk, k[q]) >= 0) {
        s.del[atomicAdd(&s.ndel, 1)] = t;
        const int r = d.rep[k[q]];
        const int sl = r != u ? set_find(s.ik, r) : -1;  // (inserted above)
        if (sl >= 0) atomicAdd(&s.iw[sl], d.aw[o + t]);
      } else {
        const int sl = set_find(s.ik, k[q]);
        if (sl >= 0) s.ipos[sl] = t;
      }
    }
  }
  __syncthreads();
  for (int x = tid; x < kPatchSet; x += nt)
    if (s.ik[x] >= 0 && s.ipos[x] < 0) atomicAdd(&s.nnew, 1);
  __syncthreads();
  const int ndel = s.ndel, nnew = s.nnew;
  const int newlen = len - ndel + nnew;
  // every absorbed neighbour was found (the lists are symmetric), and the list fits
  if (ndel != s.ngone || newlen > d.acap[u]) {
    if (tid == 0) atomicAdd(&d.cnt[C_PF_FIT], 1);
    return false;
  }
  for (int x = tid; x < kPatchSet; x += nt) {
    const int k = s.ik[x];
    if (k < 0) continue;
    if (s.ipos[x] >= 0) {
      d.aw[o + s.ipos[x]] = d.aw[o + s.ipos[x]] + s.iw[x];  // integers: exact
    } else {
      const int f = atomicAdd(&s.fill, 1);
      const int at = f < ndel ? s.del[f] : len + (f - ndel);
      d.akey[o + at] = k;
      d.aw[o + at] = s.iw[x];
    }
  }
  drain();
  __syncthreads();
  // close the remaining holes H = del[nnew, ndel) in parallel: the list ends at
  // L = len - |H|; the holes below L take the live entries of [L, len) (the
  // tail holds exactly as many live entries as there are holes below L)
  const int nh = ndel > nnew ? ndel - nnew : 0;
  if (nh > 0) {
    const int* h = s.del + nnew;
    const int L = len - nh;
    int* tail = s.gk;                    // [nh] flags: tail slot is a hole
    int* below = s.gk + kPatchGone + 1;  // holes below L
    int* live = s.ipos;                  // live tail positions (ipos is no longer needed)
    for (int x = tid; x < nh; x += nt) tail[x] = 0;
    if (tid == 0) s.fill = 0;  // reused: count of holes below L
    __syncthreads();
    for (int x = tid; x < nh; x += nt) {
      if (h[x] >= L) tail[h[x] - L] = 1;
      else below[atomicAdd(&s.fill, 1)] = h[x];
    }
    if (tid == 0) s.nnew = 0;  // reused: count of live tail slots
    __syncthreads();
    for (int y = tid; y < nh; y += nt)
      if (!tail[y]) live[atomicAdd(&s.nnew, 1)] = L + y;
    __syncthreads();
    for (int x = tid; x < s.fill; x += nt) {
      d.akey[o + below[x]] = d.akey[o + live[x]];
      d.aw[o + below[x]] = d.aw[o + live[x]];
    }
  }
  if (tid == 0) {
    d.alen[u] = newlen;
    atomicAdd(&d.cnt[C_PATCH], 1);
  }
  __syncthreads();
  return true;
}

__global__ void __launch_bounds__(64) rebuild_wave_kernel(Dev d) {
  __shared__ int tk[2 * kWaveNeed];
  __shared__ double tw[2 * kWaveNeed];
  __shared__ int s_cnt;
  __shared__ long long s_dst;
  const int count = d.cnt[C_W];
  for (int x = blockIdx.x; x < count; x += gridDim.x)
    rebuild_list(d, d.lw[x], tk, tw, 2 * kWaveNeed - 1, threadIdx.x, 64, &s_cnt, &s_dst);
}

__global__ void __launch_bounds__(256) rebuild_block_kernel(Dev d) {
  __shared__ int tk[kBlockSlots];
  __shared__ double tw[kBlockSlots];
  __shared__ int s_cnt;
  __shared__ long long s_dst;
  const int count = d.cnt[C_B];
  for (int x = blockIdx.x; x < count; x += gridDim.x) {
    const int u = d.lb[x];
    const int g = d.partner[u];
    const int need = d.alen[u] + (g >= 0 ? d.alen[g] : 0);
    const int slots = (int)pow2_at_least(2u * (unsigned)need);  // <= kBlockSlots
    rebuild_list(d, u, tk, tw, slots - 1, threadIdx.x, 256, &s_cnt, &s_dst);
  }
}

__global__ void __launch_bounds__(1024) rebuild_global_kernel(Dev d) {
  __shared__ int s_cnt;
  __shared__ long long s_dst;
  __shared__ PatchLds s_patch;
  const int count = d.cnt[C_G];
  for (int x = blockIdx.x; x < count; x += gridDim.x) {
    const bool patched = patch_list(d, d.lg[x], s_patch, threadIdx.x, (int)blockDim.x);
    if (threadIdx.x == 0) d.pcnt[d.lg[x]] = 0;  // the bucket cursor, for the next round
    if (patched) continue;
    __syncthreads();
    rebuild_list(d, d.lg[x], d.gkey + d.gofs[x], d.gw + d.gofs[x], d.gmask[x], threadIdx.x,
                 (int)blockDim.x, &s_cnt, &s_dst);
  }
}

__global__ void dirty_reset_kernel(Dev d, int round) {
  const int count = d.cnt[C_DIRTY];
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // for the next contraction
    d.cnt[C_PAIR] = 0;
    d.cnt[C_PTOP] = 0;
  }
  for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < count; x += gridDim.x * blockDim.x) {
    const int u = d.dlist[x];
    d.dirty[u] = 0;
    d.partner[u] = -1;
    d.chg[u] = round;
  }
}

__global__ void alive_compact_kernel(Dev d, int L) {
  __shared__ int s_app[2];
  const int stride = gridDim.x * blockDim.x;
  const int rounds = (L + stride - 1) / stride;
  for (int r = 0; r < rounds; ++r) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x + r * stride;
    int u = 0;
    if (x < L) u = d.alist[x];
    int* const lists[1] = {d.alist2};
    int* const ctrs[1] = {&d.cnt[C_ALIVE2]};
    const bool pr[1] = {x < L && d.alive[u]};
    block_append<1>(lists, ctrs, pr, u, s_app);
  }
}

__global__ void rank_update_kernel(Dev d, int count, const int2* __restrict__ ch) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x < count) d.rank[ch[x].x] = ch[x].y;
}


// ---- set-up ------------------------------------------------------------------
// Eligibility (rows strictly ascending -> no duplicate keys; integer weights;
// A symmetric with equal weights) and the lists: row i minus its diagonal
// entry (:1569-1571).  One wave per row.
__global__ void init_lists_kernel(int n, const int* __restrict__ ip, const int* __restrict__ ix,
                                  const double* __restrict__ dx, Dev d, double* __restrict__ rowsum,
                                  double* __restrict__ abs_total, double* __restrict__ self_total) {
  const int lane = lane_id();
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nw = (gridDim.x * blockDim.x) >> 6;
  for (int i = wave; i < n; i += nw) {
    const int b = ip[i], e = ip[i + 1];
    int self = -1;
    bool bad = false;
    double s = 0.0, sa = 0.0, sd = 0.0;
    for (int t = b + lane; t < e; t += 64) {
      const int j = ix[t];
      const double w = dx[t];
      if (j < 0 || j >= n || (t + 1 < e && !(j < ix[t + 1]))) bad = true;
      if (!(w == trunc(w)) || !(fabs(w) <= 1099511627776.0)) bad = true;  // |w| <= 2^40
      if (j == i) {
        self = t;
        sd += w;
      } else if (!bad) {
        // mirror entry (j, i) with the same weight: binary search in row j
        int lo = ip[j], hi = ip[j + 1] - 1;
        bool found = false;
        while (lo <= hi) {
          const int mid = lo + ((hi - lo) >> 1);  // entry offsets reach 2^31 / 2 (C5)
          const int c = ix[mid];
          if (c == i) {
            found = dx[mid] == w;
            break;
          }
          if (c < i) lo = mid + 1;
          else hi = mid - 1;
        }
        if (!found) bad = true;
      }
      s += w;
      sa += fabs(w);
    }
    if (__ballot(bad)) {
      if (lane == 0) atomicOr(&d.cnt[C_BAD], 1);
    }
    const unsigned long long sm = __ballot(self >= 0);
    const int sp = sm ? __shfl(self, __ffsll((long long)sm) - 1) : -1;
    for (int t = b + lane; t < e; t += 64) {
      if (t == sp) continue;
      const int o = (sp >= 0 && t > sp) ? t - 1 : t;
      d.akey[o] = ix[t];
      d.aw[o] = dx[t];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s += __shfl_xor(s, o);  // integers: exact in any order
      sa += __shfl_xor(sa, o);
      sd += __shfl_xor(sd, o);
    }
    if (lane == 0) {
      d.aoff[i] = b;
      d.alen[i] = (e - b) - (sp >= 0 ? 1 : 0);
      d.acap[i] = e - b;
      rowsum[i] = s;
      atomicAdd(abs_total, sa);
      if (sd != 0.0) atomicAdd(self_total, sd);
    }
  }
}

__global__ void init_state_kernel(Dev d, const double* __restrict__ rowsum) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= d.N) return;
  d.alpha[i] = rowsum[i] / d.T;  // :1595
  d.alive[i] = 1;
  d.touched[i] = 0;
  d.rank[i] = i;
  d.best[i] = -INFINITY;
  d.arg[i] = -1;
  d.rep[i] = i;
  d.partner[i] = -1;
  d.dirty[i] = 0;
  d.alist[i] = i;
  d.late[i] = 0;
  d.chg[i] = -1;
  d.kst[i] = -1;
}

// compaction of the pool: new capacity per alive list, then copy
__global__ void compact_size_kernel(Dev d, long long* __restrict__ cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < d.N) cap[i] = d.alive[i] ? (long long)d.alen[i] + d.alen[i] / 4 + 4 : 0;
}

__global__ void compact_copy_kernel(Dev d, const long long* __restrict__ noff,
                                    int* __restrict__ nkey, double* __restrict__ nw) {
  const int lane = lane_id();
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwv = (gridDim.x * blockDim.x) >> 6;
  for (int i = wave; i < d.N; i += nwv) {
    if (!d.alive[i]) continue;
    const long long o = d.aoff[i], q = noff[i];
    const int len = d.alen[i];
    for (int t = lane; t < len; t += 64) {
      nkey[q + t] = d.akey[o + t];
      nw[q + t] = d.aw[o + t];
    }
    if (lane == 0) {
      d.aoff[i] = q;
      d.acap[i] = (int)(noff[i + 1] - q);
    }
  }
}

inline unsigned blocks_for(long long n, int t) { return (unsigned)std::max<long long>(1, (n + t - 1) / t); }

}  // namespace

// Device path of partition::partition.  Returns nullptr (nothing computed) when
// the input needs the host path: non-integer or too large weights, an
// asymmetric matrix, or rows that are not strictly ascending.
ge_hier* partition_device(ge_ctx* ctx, int n, const int* I, const int* J, const double* Dv,
                          double cf, bool printing, bool positive, double stall, int matching) {
  DeviceGuard guard(ctx);
  hipStream_t st = ctx->stream;
  const bool prof = std::getenv("GE_PROFILE_PARTITION") != nullptr;
  // GE_PROGRESS: a line on stderr every ~10 s (long device runs, e.g. C5, stay visibly alive)
  const bool progress = std::getenv("GE_PROGRESS") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto secs = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  const auto t_start = now();
  auto note = [&](const char* what) {
    if (progress) std::fprintf(stderr, "partition_device: %s (%.1f s)\n", what, secs(t_start, now()));
  };
  const long long nnz = I[n];
  // ---- buffers
  DevBuf<int> d_ip(n + 1), d_ix(std::max<long long>(nnz, 1));
  DevBuf<double> d_dx(std::max<long long>(nnz, 1));
  d_ip.upload(I, n + 1, st);
  d_ix.upload(J, nnz, st);
  d_dx.upload(Dv, nnz, st);
  note("input uploaded");
  const long long pool_cap = 3 * nnz + 4 * (long long)n + 1024;
  DevBuf<int> key_a(pool_cap), key_b(pool_cap);
  DevBuf<double> w_a(pool_cap), w_b(pool_cap);
  DevBuf<long long> aoff(n + 1), capbuf(n + 1);
  DevBuf<int> huge(n), alen(n), acap(n), alive(n), touched(n), rank(n), arg(n), rep(n), partner(n),
      dirty(n), lk(n), alist(n), alist2(n), late(n), chg(n), kst(n), small(n), mid(n), big(n), prop(n), cand(n), cand2(n), dlist(n), lw(n), lb(n), lg(n),
      gmask(n), cnt(NCNT);
  DevBuf<long long> gofs(n);
  DevBuf<double> alpha(n), best(n), rowsum(n), sums(2);
  DevBuf<MergeRec> mrec(n / 2 + 1);
  const long long gcap = 4 * (nnz + 64) + 2 * (long long)kBlockSlots;
  DevBuf<int> gkey(gcap);
  DevBuf<double> gw(gcap);
  DevBuf<unsigned long long> tops(2);  // [0] pool top, [1] global-table top
  DevBuf<int2> pairs(kPairCap), pinfo(n);
  DevBuf<int> pcnt(n), pbuf(kPairCap), t2arg(n), t2arg2(n);
  DevBuf<double> t2w(n), t2b2(n), t2w2(n), t2b3(n);
  const int hcap = (int)(nnz / kBigLen + 2);  // lists longer than kBigLen: entries <= nnz
  DevBuf<Top> hpart((size_t)hcap * kHugeChunks);
  GE_HIP(hipMemsetAsync(pcnt.p, 0, sizeof(int) * n, st));

  Dev d{};
  d.N = n;
  d.positive = positive ? 1 : 0;
  // incremental scans need every alpha > 0 and growing: all weights positive
  d.incremental = std::getenv("GE_PARTITION_FULL_SCANS") == nullptr;
  d.akey = key_a.p;
  d.aw = w_a.p;
  d.aoff = aoff.p;
  d.alen = alen.p;
  d.acap = acap.p;
  d.alpha = alpha.p;
  d.alive = alive.p;
  d.touched = touched.p;
  d.rank = rank.p;
  d.best = best.p;
  d.arg = arg.p;
  d.rep = rep.p;
  d.partner = partner.p;
  d.dirty = dirty.p;
  d.lk = lk.p;
  d.alist = alist.p;
  d.alist2 = alist2.p;
  d.late = late.p;
  d.chg = chg.p;
  d.kst = kst.p;
  d.small = small.p;
  d.mid = mid.p;
  d.big = big.p;
  d.huge = huge.p;
  d.prop = prop.p;
  d.cand = cand.p;
  d.cand2 = cand2.p;
  d.cnt = cnt.p;
  d.mrec = mrec.p;
  d.dlist = dlist.p;
  d.lw = lw.p;
  d.lb = lb.p;
  d.lg = lg.p;
  d.gofs = gofs.p;
  d.gmask = gmask.p;
  d.gkey = gkey.p;
  d.gw = gw.p;
  d.gtop = tops.p + 1;
  d.pool_top = tops.p;
  d.pool_cap = pool_cap;
  d.pairs = pairs.p;
  d.pcnt = pcnt.p;
  d.pinfo = pinfo.p;
  d.pbuf = pbuf.p;
  d.t2arg = t2arg.p;
  d.t2w = t2w.p;
  d.t2b2 = t2b2.p;
  d.t2arg2 = t2arg2.p;
  d.t2w2 = t2w2.p;
  d.t2b3 = t2b3.p;
  d.patch = std::getenv("GE_PARTITION_NO_PATCH") == nullptr;
  d.prof = prof ? 1 : 0;

  note("buffers allocated");
  GE_HIP(hipMemsetAsync(cnt.p, 0, sizeof(int) * NCNT, st));
  GE_HIP(hipMemsetAsync(sums.p, 0, sizeof(double) * 2, st));
  GE_HIP(hipMemsetAsync(lk.p, 0x7F, sizeof(int) * n, st));
  hipLaunchKernelGGL(init_lists_kernel, dim3(2048), dim3(256), 0, st, n, d_ip.p, d_ix.p, d_dx.p, d,
                     rowsum.p, sums.p, sums.p + 1);
  GE_HIP(hipGetLastError());
  int bad = 0;
  double h_sums[2];
  GE_HIP(hipMemcpyAsync(&bad, cnt.p + C_BAD, sizeof(int), hipMemcpyDeviceToHost, st));
  GE_HIP(hipMemcpyAsync(h_sums, sums.p, sizeof(h_sums), hipMemcpyDeviceToHost, st));
  GE_HIP(hipStreamSynchronize(st));
  note("lists built");
  if (bad || !(h_sums[0] < 4503599627370496.0)) {  // sum |w| < 2^52
    if (progress)
      std::fprintf(stderr, "partition_device: input needs the host path (%s)\n",
                   bad ? "non-integer weights, asymmetric or unsorted rows"
                       : "weights sum to 2^52 or more");
    return nullptr;
  }
  {
    bool pos = true;
    for (long long e = 0; e < nnz && pos; ++e) pos = Dv[e] > 0.0;
    if (!pos) d.incremental = 0;
  }
  d_ix.release();
  d_dx.release();
  d_ip.release();
  // T = sum of all entries (:1580-1591): exact (integers), any order
  std::vector<double> h_rowsum(n);
  rowsum.download(h_rowsum.data(), n, st);
  GE_HIP(hipStreamSynchronize(st));
  double T = 0.0;
  for (int i = 0; i < n; ++i) T += h_rowsum[i];
  const double d_sum = h_sums[1];
  d.T = T;
  hipLaunchKernelGGL(init_state_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, st, d, rowsum.p);
  unsigned long long top0 = (unsigned long long)nnz;
  GE_HIP(hipMemcpyAsync(tops.p, &top0, sizeof(top0), hipMemcpyHostToDevice, st));
  double Q = 0.0;
  if (printing) {  // Q = d_sum/T - sum alpha^2, serial (:1601-1605)
    std::vector<double> h_alpha(n);
    alpha.download(h_alpha.data(), n, st);
    GE_HIP(hipStreamSynchronize(st));
    Q = d_sum / T;
    for (int i = 0; i < n; ++i) Q += -h_alpha[i] * h_alpha[i];
  }

  // ---- host mirrors of the order-dependent state (:1610-1620)
  std::unique_ptr<ge_hier> hier(new ge_hier());  // released on success only
  ge_hier* h = hier.get();
  std::vector<int> used(n), pointer(n), id(n), basis(n);
  std::iota(used.begin(), used.end(), 0);
  pointer = id = basis = used;
  int N = n, M = n, M_prev = M;
  auto find = [&](int i) {  // :1622-1633
    int root = i;
    while (id[root] != root) root = id[root];
    while (id[i] != root) {
      const int a = id[i];
      id[i] = root;
      i = a;
    }
    return root;
  };
  auto snap = [&]() {  // :1799-1808 + interpolationMatrix (:29-65)
    std::vector<int> cntr(M + 1, 0), rowof(basis.size());
    for (size_t y = 0; y < basis.size(); ++y) {
      rowof[y] = pointer[find(basis[y])];
      cntr[rowof[y] + 1]++;
    }
    for (int r = 0; r < M; ++r) cntr[r + 1] += cntr[r];
    std::vector<int> ix(basis.size());
    std::vector<int> fill(cntr.begin(), cntr.end() - 1);
    for (size_t y = 0; y < basis.size(); ++y) ix[fill[rowof[y]]++] = (int)y;
    h->rows.push_back(M);
    h->cols.push_back(N);
    h->indptr.push_back(std::move(cntr));
    h->indices.push_back(std::move(ix));
  };

  note("host state ready");
  MergeRec* h_mrec = nullptr;
  int2* h_changes = nullptr;
  GE_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_mrec), sizeof(MergeRec) * (n / 2 + 1)));
  GE_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_changes), sizeof(int2) * (n / 2 + 1)));
  struct PinnedFree {
    void* a;
    void* b;
    ~PinnedFree() {
      (void)hipHostFree(a);
      (void)hipHostFree(b);
    }
  } pinned_free{h_mrec, h_changes};
  struct {
    int merges;
    unsigned long long top;
  } rb{};
  int* h_cnt = nullptr;
  GE_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_cnt), sizeof(int) * NCNT));
  struct PinnedCnt {
    int* p;
    ~PinnedCnt() { (void)hipHostFree(p); }
  } pinned_cnt{h_cnt};
  unsigned long long* h_top = nullptr;
  GE_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_top), sizeof(unsigned long long)));
  struct PinnedTop {
    unsigned long long* p;
    ~PinnedTop() { (void)hipHostFree(p); }
  } pinned_top{h_top};
  int* h_seq = nullptr;  // the last exported round (RoundExport::hseq)
  GE_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_seq), sizeof(int)));
  *h_seq = 0;
  struct PinnedSeq {
    int* p;
    ~PinnedSeq() { (void)hipHostFree(p); }
  } pinned_seq{h_seq};

  int alist_len = n;
  const int mid_blocks = 1024;  // 512 / 2 048 measured no better
  const int spec = std::min(kSpecMerges, n / 2 + 1);
  double t_dev = 0, t_host = 0, t_compact = 0;
  long long total_merges = 0;
  int rounds = 0, compactions = 0;
  std::vector<MergeRec> order;
  std::vector<int> stamp(n, 0), moved(n / 2 + 1);
  auto t_last_note = now();
  long long stat[NCNT] = {0};
  int rstat[NCNT] = {0};  // this round's list sizes (GE_PROFILE_ROUNDS)
  const bool prof_rounds = prof && std::getenv("GE_PROFILE_ROUNDS");
  // A pass is its scans (classify_scan .. filter: they read lists, alphas and the
  // touched flags, never the rank array) and its resolve (the greedy matching in
  // `used` order: reads the rank array).  Round r + 1's first scans are queued right
  // behind round r's contraction, before the host's swap-pop of round r, and round
  // r's rank update behind them: the device runs the scans while the host does the
  // order-dependent bookkeeping (round 6: it waited for it before, 0.53 s at C4 in
  // gaps before rank_update_kernel and classify_scan_kernel,
  // profiles/r06/partition_c4_gaps_start.txt).
  auto launch_scans = [&](int pass, int round) {
    hipLaunchKernelGGL(classify_scan_kernel, dim3(blocks_for(alist_len, 256)), dim3(256), 0, st, d,
                       pass, alist_len, round, round == 1 ? 1 : 0, pass == matching - 1 ? 1 : 0);
    hipLaunchKernelGGL(scan_small_kernel, dim3(1024), dim3(256), 0, st, d, pass);
    hipLaunchKernelGGL(scan_mid_kernel, dim3(mid_blocks), dim3(256), 0, st, d, pass);
    hipLaunchKernelGGL(scan_big_kernel<256>, dim3(1024), dim3(256), 0, st, d, pass);
    hipLaunchKernelGGL(scan_huge_part_kernel, dim3(kHugeChunks, 64), dim3(1024), 0, st, d, pass,
                       hpart.p, hcap);
    hipLaunchKernelGGL(scan_huge_final_kernel, dim3(64), dim3(256), 0, st, d, pass, hpart.p, hcap);
    hipLaunchKernelGGL(filter_kernel, dim3(1024), dim3(256), 0, st, d);
  };
  bool scans_queued = false;  // pass 0's scans of the coming round are already queued
  do {
    std::fill(rstat, rstat + NCNT, 0);
    ++rounds;
    const auto t0 = now();
    for (int pass = 0; pass < matching; ++pass) {
      if (!(pass == 0 && scans_queued)) launch_scans(pass, rounds);
      hipLaunchKernelGGL(resolve_min_kernel, dim3(512), dim3(256), 0, st, d);
      hipLaunchKernelGGL(resolve_select_kernel, dim3(512), dim3(256), 0, st, d, pass);
      hipLaunchKernelGGL(resolve_filter_kernel, dim3(512), dim3(256), 0, st, d);
      {
        Dev d2 = d;  // the survivors are in cand2
        std::swap(d2.cand, d2.cand2);
        RoundExport ex;  // the round's last pass exports its counts and records
        if (pass == matching - 1) {
          ex.tops = tops.p;
          ex.hcnt = h_cnt;
          ex.htop = h_top;
          ex.hrec = reinterpret_cast<int*>(h_mrec);
          ex.hseq = h_seq;
          ex.seq = rounds;
          ex.spec = spec;
        }
        hipLaunchKernelGGL(resolve_kernel, dim3(1), dim3(1024), 0, st, d2, pass, (int)C_CAND2, ex);
      }
      if (prof) {  // per-pass list sizes (extra synchronisation: profiling only)
        GE_HIP(hipMemcpyAsync(h_cnt, cnt.p, sizeof(int) * NCNT, hipMemcpyDeviceToHost, st));
        GE_HIP(hipStreamSynchronize(st));
        // (resolve_kernel moved the pass's counts to the C_SH_* slots)
        const int from[6] = {C_SMALL, C_MID, C_BIG, C_PROP, C_CAND, C_HUGE};
        for (int q = 0; q < 6; ++q) {
          stat[from[q]] += h_cnt[C_SH_SMALL + q];
          rstat[from[q]] += h_cnt[C_SH_SMALL + q];
        }
      }
    }
    GE_HIP(hipGetLastError());
    // The round's last resolve_kernel writes its counts and the first `spec` merge
    // records into pinned memory and then the round number into *h_seq (system-scope
    // release): the host spins on it instead of a stream synchronisation, whose
    // wake-up cost ~25 us per round (0.26 s at C4 in the gap before merge_apply_kernel).
    // A stream that finished or failed without writing it ends the spin (the error
    // is then reported by the synchronisation).
    for (long long spins = 1;; ++spins) {
      if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) == rounds) break;
      if ((spins & 1023) == 0 && hipStreamQuery(st) != hipErrorNotReady) {
        GE_HIP(hipStreamSynchronize(st));
        if (__atomic_load_n(h_seq, __ATOMIC_ACQUIRE) != rounds)
          throw Error(GE_ERR_STATE, "partition_device: a round ended without its export");
        break;
      }
    }
    if (rounds <= 2) note("round: matching passes done");
    rb.merges = h_cnt[C_MERGE];
    if (prof) {
      for (int q = 0; q < 4; ++q) {  // previous round's contraction (DIRTY W B G)
        stat[C_DIRTY + q] += h_cnt[C_SH_DIRTY + q];
        rstat[C_DIRTY + q] = h_cnt[C_SH_DIRTY + q];
      }
      for (int c : {(int)C_PATCH, (int)C_PF_SHORT, (int)C_PF_SIZE, (int)C_PF_FIT}) {
        rstat[c] = h_cnt[c] - (int)stat[c];  // these counters accumulate
        stat[c] = h_cnt[c];
      }
    }
    rb.top = *h_top;
    if (h_cnt[C_OVF] == 2)  // a bug, not a capacity limit: never retried on the host
      throw Error(GE_ERR_STATE, "partition_device: resolve did not converge");
    if (h_cnt[C_OVF])
      throw Error(GE_ERR_CAPACITY, "partition_device: list pool overflow");
    const int nm = rb.merges;
    if (nm > 0) {
      if (nm > spec) {
        GE_HIP(hipMemcpyAsync(h_mrec + spec, mrec.p + spec, sizeof(MergeRec) * (nm - spec),
                              hipMemcpyDeviceToHost, st));
        GE_HIP(hipStreamSynchronize(st));
      }
      // fresh pool space this round needs at most 1.5 x (both lists) + 4 per keeper
      long long worst = 0;
      for (int x = 0; x < nm; ++x)
        worst += (long long)h_mrec[x].len_keep + h_mrec[x].len_gone +
                 ((long long)h_mrec[x].len_keep + h_mrec[x].len_gone) / 2 + 4;
      if ((long long)rb.top + worst > pool_cap) {
        const auto tc = now();
        ++compactions;
        hipLaunchKernelGGL(compact_size_kernel, dim3(blocks_for(n, 256)), dim3(256), 0, st, d,
                           capbuf.p);
        GE_HIP(hipMemsetAsync(capbuf.p + n, 0, sizeof(long long), st));
        DevBuf<long long> noff(n + 1);
        prim_exclusive_sum(st, capbuf.p, noff.p, (size_t)n + 1);
        int* nkey = (d.akey == key_a.p) ? key_b.p : key_a.p;
        double* nwt = (d.aw == w_a.p) ? w_b.p : w_a.p;
        hipLaunchKernelGGL(compact_copy_kernel, dim3(2048), dim3(256), 0, st, d, noff.p, nkey, nwt);
        GE_HIP(hipGetLastError());
        GE_HIP(hipMemcpyAsync(tops.p, noff.p + n, sizeof(long long), hipMemcpyDeviceToDevice, st));
        GE_HIP(hipMemcpyAsync(h_top, tops.p, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        GE_HIP(hipStreamSynchronize(st));
        d.akey = nkey;
        d.aw = nwt;
        if ((long long)*h_top + worst > pool_cap)
          throw Error(GE_ERR_CAPACITY, "partition_device: list pool exhausted after compaction");
        t_compact += secs(tc, now());
      }
      // contraction on the device (asynchronous) while the host does the
      // order-dependent bookkeeping
      hipLaunchKernelGGL(merge_apply_kernel, dim3(blocks_for(nm, 256)), dim3(256), 0, st, d, rounds);
      hipLaunchKernelGGL(mark_dirty_kernel, dim3(blocks_for(nm, 4)), dim3(256), 0, st, d);
      hipLaunchKernelGGL(classify_kernel, dim3(1024), dim3(256), 0, st, d);
      hipLaunchKernelGGL(pair_scatter_kernel, dim3(1024), dim3(256), 0, st, d);
      hipLaunchKernelGGL(rebuild_wave_kernel, dim3(8192), dim3(64), 0, st, d);
      hipLaunchKernelGGL(rebuild_block_kernel, dim3(1024), dim3(256), 0, st, d);
      hipLaunchKernelGGL(rebuild_global_kernel, dim3(256), dim3(1024), 0, st, d);
      hipLaunchKernelGGL(dirty_reset_kernel, dim3(1024), dim3(256), 0, st, d, rounds);
      GE_HIP(hipGetLastError());
      if (rounds <= 2 && progress) {  // profiling the first rounds: wait for the contraction
        GE_HIP(hipStreamSynchronize(st));
        note("round: contraction done");
      }
    }
    M_prev = M;
    M -= nm;  // the swap-pop below removes nm entries of `used`
    const bool more = 1.0 * M / M_prev < stall;  // :1838
    if (more) {
      if (alist_len > M + M / 4 + 1024) {  // drop the dead entries of the alive list
        GE_HIP(hipMemsetAsync(cnt.p + C_ALIVE2, 0, sizeof(int), st));
        hipLaunchKernelGGL(alive_compact_kernel, dim3(blocks_for(alist_len, 256)), dim3(256), 0, st,
                           d, alist_len);
        GE_HIP(hipGetLastError());
        std::swap(d.alist, d.alist2);
        alist_len = M;
      }
      launch_scans(0, rounds + 1);  // the next round's first scans (no rank reads)
      GE_HIP(hipGetLastError());
      scans_queued = true;
    }
    const auto t1 = now();
    t_dev += secs(t0, t1);
    // ---- host: merges in the reference's order (pass, then `used` slot)
    order.assign(h_mrec, h_mrec + nm);
    std::sort(order.begin(), order.end(), [](const MergeRec& a, const MergeRec& b) {
      return a.pass != b.pass ? a.pass < b.pass : a.rank < b.rank;
    });
    double dQ = 0.0;
    for (const auto& m : order) dQ += m.eta;  // :1749
    Q += dQ;                                  // :1784
    if (1.0 * M_prev / N <= cf) {  // :1797-1815 (before this round's swap-pop)
      const int M_now = M;
      M = M_prev;  // snap() reads the pre-round count
      snap();
      M = M_now;
      basis = used;
      N = M_prev;
    }
    int nch = 0;
    for (const auto& m : order) {  // :1819-1834
      const int idx = pointer[m.gone];
      const int last = used.back();
      std::swap(used[idx], used.back());
      used.pop_back();
      pointer[last] = idx;
      id[m.gone] = m.keep;
      if (stamp[last] != rounds) {  // a vertex may move several times: upload its final slot
        stamp[last] = rounds;
        moved[nch++] = last;
      }
    }
    for (int x = 0; x < nch; ++x) h_changes[x] = make_int2(moved[x], pointer[moved[x]]);
    total_merges += nm;
    if (nch > 0 && more) {
      // the kernel reads the pinned changes directly (no H2D blit); the host next
      // writes h_changes after the next round's export, past this kernel
      hipLaunchKernelGGL(rank_update_kernel, dim3(blocks_for(nch, 256)), dim3(256), 0, st, d, nch,
                         (const int2*)h_changes);
      GE_HIP(hipGetLastError());
    }
    t_host += secs(t1, now());
    if (progress && (rounds <= 3 || secs(t_last_note, now()) > 10.0)) {
      t_last_note = now();
      std::fprintf(stderr, "partition_device: round %d, %d aggregates, %lld merges, %.0f s\n",
                   rounds, M, total_merges, secs(t_start, t_last_note));
    }
    if (prof_rounds)  // rescans by class (both passes), proposers, candidates; the
                      // previous round's contraction: dirty lists by table class
      std::fprintf(stderr,
                   "round %d alive %d merges %d pool %llu small %d mid %d big %d huge %d prop %d "
                   "cand %d dirty %d w %d b %d g %d patched %d rebuilt short %d size %d fit %d\n",
                   rounds, M, nm, rb.top, rstat[C_SMALL], rstat[C_MID], rstat[C_BIG],
                   rstat[C_HUGE], rstat[C_PROP], rstat[C_CAND], rstat[C_DIRTY], rstat[C_W],
                   rstat[C_B], rstat[C_G], rstat[C_PATCH], rstat[C_PF_SHORT], rstat[C_PF_SIZE],
                   rstat[C_PF_FIT]);
    if (!more) break;
  } while (true);
  GE_HIP(hipStreamSynchronize(st));
  snap();  // :1840-1852
  if (prof)
    std::fprintf(stderr,
                 "partition_device: n=%d nnz=%lld %d rounds %lld merges %.3fs (device rounds "
                 "%.3fs, host %.3fs, %d compactions %.3fs)\n",
                 n, nnz, rounds, total_merges, secs(t_start, now()), t_dev, t_host, compactions,
                 t_compact);
  if (prof)
    std::fprintf(stderr,
                 "partition_device lists (sums over passes): rescans small %lld mid %lld big %lld "
                 "huge %lld, proposers %lld, candidates %lld; dirty %lld (wave %lld block %lld "
                 "global %lld, of which patched %lld; rebuilt: short %lld, sets %lld, room %lld)\n",
                 stat[C_SMALL], stat[C_MID], stat[C_BIG], stat[C_HUGE], stat[C_PROP], stat[C_CAND],
                 stat[C_DIRTY],
                 stat[C_W], stat[C_B], stat[C_G], stat[C_PATCH], stat[C_PF_SHORT], stat[C_PF_SIZE],
                 stat[C_PF_FIT]);
  if (prof)
    std::fprintf(stderr,
                 "partition_device rescans of lists > %d entries by reason: changed %d, bound "
                 "failed %d, argmax touched %d\n",
                 kSmallLen, h_cnt[C_R_CHG], h_cnt[C_R_BOUND], h_cnt[C_R_PASS]);
  if (printing) {  // :1880-1889
    std::cout << "modularity: " << Q << std::endl;
    std::cout << "level 0: " << n << " aggregates" << std::endl;
    for (size_t l = 0; l < h->rows.size(); ++l)
      std::cout << "level " << l + 1 << ": " << h->rows[l] << " aggregates" << std::endl;
  }
  return hier.release();
}

}  // namespace ge
