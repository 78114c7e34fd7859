// ge_dist.hip -- multi-GPU inside libge: a communicator per context (RCCL over
// xGMI, or a caller transport) and the sharded forms of the path's calls.
//
// The reference runs on one node with OpenMP and has no multi-GPU code; the
// sharding follows SURVEY.md 8(e):
//   * forceAtlas (include/forceatlas.hpp:146-270): every new position depends on
//     all positions of the previous iteration and on nothing else global (the
//     swing / traction sums are dead, :228, :242), so ranks own contiguous row
//     blocks and one in-place all-gather of the fp64 coordinates follows each
//     iteration.  Levels small enough for the fused single-launch kernels (the
//     coarsest level's 1e5 iterations) run as replicas: an all-gather per
//     microsecond-scale iteration would cost more than it saves.
//   * forceAtlasMultilevel (:314-574): aggregates exchange nothing during the
//     iterations (:454, :462 read only the frozen coarse coordinates), so they are
//     dealt to ranks by cost (longest processing time first) and one all-gather
//     of the members' coordinates completes the call.
//   * P^T A P: ranks take contiguous blocks of coarse rows of equal expanded work
//     (ge_ptap.hip with a row range); one all-gather of the coarse rows.
// Every rank computes its rows with the single-GPU kernels on the same inputs, so
// the results are bit-identical to the single-GPU calls.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <queue>
#include <vector>

#include "ge_internal.hpp"

namespace ge {
namespace {

#define GE_NCCL(call)                                                                    \
  do {                                                                                   \
    ncclResult_t _r = (call);                                                            \
    if (_r != ncclSuccess)                                                               \
      throw ::ge::Error(GE_ERR_HIP, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)

// A C-ABI call made from inside the library: a failure becomes an exception.
void abi(int rc) {
  if (rc != GE_OK) throw Error(rc, ge_last_error());
}

ncclComm_t nccl_of(const ge_comm* c) { return (ncclComm_t)c->nccl; }

}  // namespace

// All-gather of equal blocks of `bytes` bytes between device buffers (d_send may
// be d_recv + rank * bytes: in place), enqueued on stream s; the transport path
// synchronises s.
void allgather_stream(ge_comm* c, hipStream_t s, const void* d_send, void* d_recv, size_t bytes) {
  char* recv = (char*)d_recv;
  if (c->nranks == 1) {
    if (d_send != d_recv && bytes)
      GE_HIP(hipMemcpyAsync(recv, d_send, bytes, hipMemcpyDeviceToDevice, s));
    return;
  }
  if (c->nccl) {
    GE_NCCL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, nccl_of(c), s));
    return;
  }
  std::vector<unsigned char> hs(std::max<size_t>(bytes, 1)), hr(std::max<size_t>(bytes * c->nranks, 1));
  if (bytes) GE_HIP(hipMemcpyAsync(hs.data(), d_send, bytes, hipMemcpyDeviceToHost, s));
  GE_HIP(hipStreamSynchronize(s));
  if (c->tp.allgather(c->tp.user, hs.data(), hr.data(), bytes) != 0)
    throw Error(GE_ERR_STATE, "transport all-gather failed");
  if (bytes) GE_HIP(hipMemcpyAsync(recv, hr.data(), bytes * c->nranks, hipMemcpyHostToDevice, s));
  GE_HIP(hipStreamSynchronize(s));
}

namespace {

// The same on the context's stream.
void allgather_dev(ge_comm* c, const void* d_send, void* d_recv, size_t bytes) {
  allgather_stream(c, c->ctx->stream, d_send, d_recv, bytes);
}

// All-gather of small host arrays (counts, sizes).
template <class T>
std::vector<T> allgather_host(ge_comm* c, const T* v, size_t count) {
  std::vector<T> out(count * c->nranks);
  if (c->nranks == 1) {
    std::copy(v, v + count, out.begin());
    return out;
  }
  const size_t bytes = sizeof(T) * count;
  if (c->nccl) {
    DevBuf<unsigned char> d(bytes * c->nranks);
    GE_HIP(hipMemcpyAsync(d.p + bytes * c->rank, v, bytes, hipMemcpyHostToDevice, c->ctx->stream));
    allgather_dev(c, d.p + bytes * c->rank, d.p, bytes);
    GE_HIP(hipMemcpyAsync(out.data(), d.p, bytes * c->nranks, hipMemcpyDeviceToHost,
                          c->ctx->stream));
    GE_HIP(hipStreamSynchronize(c->ctx->stream));
    return out;
  }
  if (c->tp.allgather(c->tp.user, v, out.data(), bytes) != 0)
    throw Error(GE_ERR_STATE, "transport all-gather failed");
  return out;
}

// All-gather of one variable-size host byte block per rank.
std::vector<std::vector<unsigned char>> allgatherv_host(ge_comm* c,
                                                        const std::vector<unsigned char>& mine) {
  const long long sz = (long long)mine.size();
  const std::vector<long long> sizes = allgather_host(c, &sz, 1);
  const size_t width = (size_t)std::max(1ll, *std::max_element(sizes.begin(), sizes.end()));
  std::vector<std::vector<unsigned char>> out(c->nranks);
  DevBuf<unsigned char> d(width * c->nranks);
  hipStream_t s = c->ctx->stream;
  if (sz) GE_HIP(hipMemcpyAsync(d.p + width * c->rank, mine.data(), sz, hipMemcpyHostToDevice, s));
  allgather_dev(c, d.p + width * c->rank, d.p, width);
  std::vector<unsigned char> all(width * c->nranks);
  GE_HIP(hipMemcpyAsync(all.data(), d.p, all.size(), hipMemcpyDeviceToHost, s));
  GE_HIP(hipStreamSynchronize(s));
  for (int r = 0; r < c->nranks; ++r)
    out[r].assign(all.begin() + width * r, all.begin() + width * r + sizes[r]);
  return out;
}

__global__ void pack_rows_kernel(int count, int dim, const int* __restrict__ rows,
                                 const double* __restrict__ x, double* __restrict__ out) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < (long long)count * dim) out[t] = x[(size_t)rows[t / dim] * dim + t % dim];
}

// rows of every rank but `self`: block r of recv holds counts[r] rows of width
__global__ void unpack_rows_kernel(int nranks, int self, int width, int dim,
                                   const int* __restrict__ counts, const int* __restrict__ first,
                                   const int* __restrict__ rows, const double* __restrict__ recv,
                                   double* __restrict__ x) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)width * dim;
  if (t >= per * nranks) return;
  const int r = (int)(t / per);
  const int q = (int)((t % per) / dim);
  const int k = (int)(t % dim);
  if (r == self || q >= counts[r]) return;
  x[(size_t)rows[first[r] + q] * dim + k] = recv[t];
}

inline unsigned grid_for(long long L) { return (unsigned)((L + 255) / 256); }

// Levels up to this many rows run as replicas in the sharded forceAtlas.
int replica_max() {
  if (const char* e = std::getenv("GE_DIST_REPLICA_MAX")) return std::atoi(e);
  return 65536;
}

void check_comm(const ge_comm* c) {
  GE_REQUIRE(c && c->ctx, "null communicator");
}

}  // namespace

// Cost of an aggregate per iteration: ordered pairs + its members' CSR entries.
std::vector<double> aggregate_costs(int m, const int* pip, const int* pix, const int* ip) {
  std::vector<double> cost(m);
  for (int a = 0; a < m; ++a) {
    const double s = pip[a + 1] - pip[a];
    double c = s * (s - 1);
    if (ip && s > 0) {
      double e = 0.0;
      for (int q = pip[a]; q < pip[a + 1]; ++q) e += ip[pix[q] + 1] - ip[pix[q]];
      c = c + e;
    }
    cost[a] = c;
  }
  return cost;
}

// Longest-processing-time list scheduling of aggregates; split
// aggregates (split[a] != 0) get owner -1 and load every rank with an equal share.
std::vector<int> assign_aggregates(int m, const int* pip, const int* pix, const int* ip,
                                   int nranks, const std::vector<char>* split) {
  const std::vector<double> cost = aggregate_costs(m, pip, pix, ip);
  std::vector<int> order;
  for (int a = 0; a < m; ++a)
    if (!split || !(*split)[a]) order.push_back(a);
  std::stable_sort(order.begin(), order.end(),
                   [&](int x, int y) { return cost[x] > cost[y]; });  // ties: lower id first
  using Load = std::pair<double, int>;  // (load, rank): least load, then lowest rank
  std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
  for (int r = 0; r < nranks; ++r) heap.emplace(0.0, r);
  std::vector<int> owner(m, -1);
  for (int a : order) {
    const Load top = heap.top();
    heap.pop();
    owner[a] = top.second;
    heap.emplace(top.first + cost[a], top.second);
  }
  return owner;
}

void allgather_members(ge_comm* c, double* d_x, int dim, int m, const int* pip, const int* pix,
                       const int* owner) {
  if (c->nranks == 1) return;
  const int N = c->nranks;
  std::vector<int> counts(N, 0), first(N + 1, 0);
  for (int a = 0; a < m; ++a) counts[owner[a]] += pip[a + 1] - pip[a];
  for (int r = 0; r < N; ++r) first[r + 1] = first[r] + counts[r];
  std::vector<int> rows(first[N]), fill(first.begin(), first.end() - 1);
  for (int a = 0; a < m; ++a)  // aggregates ascending, members in P_T order
    for (int q = pip[a]; q < pip[a + 1]; ++q) rows[fill[owner[a]]++] = pix[q];
  const int width = std::max(1, *std::max_element(counts.begin(), counts.end()));
  hipStream_t s = c->ctx->stream;
  DevBuf<int> d_rows(std::max(1, first[N])), d_counts(N), d_first(N + 1);
  d_rows.upload(rows.data(), rows.size(), s);
  d_counts.upload(counts.data(), N, s);
  d_first.upload(first.data(), N + 1, s);
  DevBuf<double> recv((size_t)width * dim * N);
  double* mine = recv.p + (size_t)width * dim * c->rank;
  const long long own = (long long)counts[c->rank] * dim;
  if (own)
    hipLaunchKernelGGL(pack_rows_kernel, dim3(grid_for(own)), dim3(256), 0, s, counts[c->rank],
                       dim, d_rows.p + first[c->rank], d_x, mine);
  allgather_dev(c, mine, recv.p, sizeof(double) * width * dim);
  const long long all = (long long)width * dim * N;
  hipLaunchKernelGGL(unpack_rows_kernel, dim3(grid_for(all)), dim3(256), 0, s, N, c->rank, width,
                     dim, d_counts.p, d_first.p, d_rows.p, recv.p, d_x);
  GE_HIP(hipGetLastError());
  GE_HIP(hipStreamSynchronize(s));
}

// Rows of d_x listed per rank (d_rows: rank r's h_counts[r] positions from
// h_first[r]) exchanged so every rank holds every rank's rows: pack this rank's into
// its block of d_buf (nranks x width x dim), all-gather on stream s, unpack the
// others.  Stream-ordered (RCCL); the transport path synchronises s.
void exchange_rows(ge_comm* c, hipStream_t s, int dim, const int* d_rows, const int* d_counts,
                   const int* d_first, const int* h_counts, const int* h_first, int width,
                   double* d_buf, double* d_x) {
  const int N = c->nranks;
  double* mine = d_buf + (size_t)width * dim * c->rank;
  const long long own = (long long)h_counts[c->rank] * dim;
  if (own)
    hipLaunchKernelGGL(pack_rows_kernel, dim3(grid_for(own)), dim3(256), 0, s, h_counts[c->rank],
                       dim, d_rows + h_first[c->rank], d_x, mine);
  allgather_stream(c, s, mine, d_buf, sizeof(double) * (size_t)width * dim);
  const long long all = (long long)width * dim * N;
  hipLaunchKernelGGL(unpack_rows_kernel, dim3(grid_for(all)), dim3(256), 0, s, N, c->rank, width,
                     dim, d_counts, d_first, d_rows, d_buf, d_x);
  GE_HIP(hipGetLastError());
}

// Aggregates split by row tiles across ranks: an aggregate whose
// ordered pairs s(s-1) exceed half of a rank's average load cannot be balanced as a
// whole.  min_members > 0 splits every aggregate of at least that many members
// (tests); 0 splits none; < 0 the automatic rule (GE_DIST_SPLIT_MIN overrides it).
std::vector<char> split_aggregates(int m, const int* pip, const int* pix, const int* ip,
                                   int nranks, int min_members) {
  std::vector<char> out(m, 0);
  if (nranks <= 1) return out;
  if (min_members < 0)
    if (const char* e = std::getenv("GE_DIST_SPLIT_MIN")) min_members = std::atoi(e);
  if (min_members > 0) {
    for (int a = 0; a < m; ++a) out[a] = pip[a + 1] - pip[a] >= std::max(min_members, 2);
    return out;
  }
  if (min_members == 0) return out;
  const std::vector<double> cost = aggregate_costs(m, pip, pix, ip);
  double W = 0.0;
  for (double c : cost) W += c;
  for (int a = 0; a < m; ++a) out[a] = pip[a + 1] - pip[a] >= 128 && cost[a] > 0.5 * W / nranks;
  return out;
}

void fa_host_dist(ge_comm* c, int n, const int* ip, const int* ix, const double* dx, int dim,
                  double* X, bool init_random, int iterations, const ge_fa_params& p) {
  if (init_random) uniform_stream(p.seed, (size_t)n * dim, X);  // :118-125
  if (c->nranks == 1 || n <= replica_max() || iterations <= 0) {
    fa_host(c->ctx, n, ip, ix, dx, dim, X, false, iterations, p);  // replicas
    return;
  }
  const int N = c->nranks;
  const int chunk = (n + N - 1) / N;
  const int rb = std::min(n, c->rank * chunk), re = std::min(n, (c->rank + 1) * chunk);
  hipStream_t s = c->ctx->stream;
  DevCsr A(n, ip, ix, dx, s);
  const size_t padded = (size_t)N * chunk * dim;
  DevBuf<double> xa(padded), xb(padded);
  GE_HIP(hipMemsetAsync(xa.p, 0, sizeof(double) * padded, s));
  GE_HIP(hipMemsetAsync(xb.p, 0, sizeof(double) * padded, s));
  xa.upload(X, (size_t)n * dim, s);
  ge_fa_plan* plan = nullptr;
  abi(ge_fa_plan_create(c->ctx, n, A.nnz, A.ip.p, A.ix.p, A.dx.p, dim, &p, rb, re, &plan));
  double *cur = xa.p, *nxt = xb.p;
  try {
    for (int it = 0; it < iterations; ++it) {
      if (re > rb) abi(ge_fa_plan_step(plan, cur, nxt));
      allgather_dev(c, nxt + (size_t)c->rank * chunk * dim, nxt,
                    sizeof(double) * (size_t)chunk * dim);
      std::swap(cur, nxt);
    }
  } catch (...) {
    ge_fa_plan_destroy(plan);
    throw;
  }
  abi(ge_fa_plan_destroy(plan));
  GE_HIP(hipMemcpyAsync(X, cur, sizeof(double) * n * dim, hipMemcpyDeviceToHost, s));
  GE_HIP(hipStreamSynchronize(s));
  if (p.normalize) normalize_host(X, n, dim);
}

void faml_host_dist(ge_comm* c, int n, const int* ip, const int* ix, const double* dx, int m,
                    const int* pip, const int* pix, const int* vA, const double* cA,
                    const double* rA, double* X, int dim, int iterations,
                    const ge_fa_params& p) {
  if (c->nranks == 1) {
    faml_host(c->ctx, n, ip, ix, dx, m, pip, pix, vA, cA, rA, X, dim, iterations, p);
    return;
  }
  // aggregates too large for a rank's share are split by row tiles over all ranks
  // (their members exchanged after every iteration inside the plan); the rest are
  // dealt whole by cost
  const std::vector<char> split = split_aggregates(m, pip, pix, ip, c->nranks, -1);
  std::vector<int> owner = assign_aggregates(m, pip, pix, ip, c->nranks, &split);
  std::vector<int> mine, shared;
  for (int a = 0; a < m; ++a) {
    if (split[a]) shared.push_back(a);
    else if (owner[a] == c->rank) mine.push_back(a);
  }
  hipStream_t s = c->ctx->stream;
  std::vector<double> init((size_t)pip[m] * dim);
  uniform_stream(p.seed, init.size(), init.data());  // P_T storage order (:356-360)
  DevCsr A(n, ip, ix, dx, s);
  DevBuf<int> dpip(m + 1), dpix(std::max(pip[m], 1)), dvA(std::max(n, 1));
  DevBuf<double> dcA(std::max<size_t>((size_t)m * dim, 1)), drA(std::max(m, 1)),
      dinit(std::max<size_t>(init.size(), 1)), dX(std::max<size_t>((size_t)n * dim, 1));
  dpip.upload(pip, m + 1, s);
  dpix.upload(pix, pip[m], s);
  dvA.upload(vA, n, s);
  dcA.upload(cA, (size_t)m * dim, s);
  drA.upload(rA, m, s);
  dinit.upload(init.data(), init.size(), s);
  GE_HIP(hipMemsetAsync(dX.p, 0, sizeof(double) * dX.n, s));
  if (!mine.empty() || !shared.empty()) {
    ge_faml_plan* plan = nullptr;
    abi(ge_faml_plan_create_shard(c->ctx, c, n, A.ip.p, A.ix.p, A.dx.p, m, pip, dpip.p, dpix.p,
                                  dvA.p, dim, &p, iterations, mine.data(), (int)mine.size(),
                                  shared.data(), (int)shared.size(), &plan));
    const int rc = ge_faml_plan_run(plan, dcA.p, drA.p, dinit.p, dX.p);
    ge_faml_plan_destroy(plan);
    abi(rc);
  }
  for (int a : shared) owner[a] = 0;  // every rank holds the split aggregates' members
  allgather_members(c, dX.p, dim, m, pip, pix, owner.data());
  dX.download(X, (size_t)n * dim, s);
  GE_HIP(hipStreamSynchronize(s));
}

// Coarse-row blocks of equal expanded work (members' CSR entries + 1 per row).
std::vector<int> ptap_row_blocks(int m, const int* pip, const int* pix, const int* ip,
                                 int nranks) {
  std::vector<double> pre(m + 1, 0.0);
  for (int a = 0; a < m; ++a) {
    double w = 1.0;
    for (int q = pip[a]; q < pip[a + 1]; ++q) w += ip[pix[q] + 1] - ip[pix[q]];
    pre[a + 1] = pre[a] + w;
  }
  std::vector<int> b(nranks + 1, m);
  b[0] = 0;
  for (int r = 1; r < nranks; ++r) {
    const double target = pre[m] * r / nranks;
    b[r] = std::max(b[r - 1], (int)(std::lower_bound(pre.begin(), pre.end(), target) - pre.begin()));
    b[r] = std::min(b[r], m);
  }
  return b;
}

}  // namespace ge

// ===========================================================================
// C ABI

using ge::guarded;

extern "C" {

int ge_comm_unique_id(unsigned char* id) {
  return guarded([&] {
    GE_REQUIRE(id, "null argument");
    ncclUniqueId u;
    GE_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, GE_COMM_ID_BYTES);
  });
}

int ge_comm_create(ge_ctx* ctx, int nranks, int rank, const unsigned char* id, ge_comm** out) {
  return guarded([&] {
    GE_REQUIRE(ctx && id && out, "null argument");
    GE_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / size");
    ge::DeviceGuard g(ctx);
    ncclUniqueId u;
    std::memcpy(u.internal, id, GE_COMM_ID_BYTES);
    ncclComm_t nc = nullptr;
    GE_NCCL(ncclCommInitRank(&nc, nranks, u, rank));
    auto* c = new ge_comm();
    c->ctx = ctx;
    c->nranks = nranks;
    c->rank = rank;
    c->nccl = nc;
    *out = c;
  });
}

int ge_comm_create_transport(ge_ctx* ctx, int nranks, int rank, const ge_transport* t,
                             ge_comm** out) {
  return guarded([&] {
    GE_REQUIRE(ctx && t && t->allgather && out, "null argument");
    GE_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / size");
    auto* c = new ge_comm();
    c->ctx = ctx;
    c->nranks = nranks;
    c->rank = rank;
    c->tp = *t;
    *out = c;
  });
}

int ge_comm_info(const ge_comm* c, int* nranks, int* rank, int* is_rccl) {
  return guarded([&] {
    GE_REQUIRE(c && nranks && rank && is_rccl, "null argument");
    *nranks = c->nranks;
    *rank = c->rank;
    *is_rccl = c->nccl ? 1 : 0;
  });
}

int ge_comm_destroy(ge_comm* c) {
  return guarded([&] {
    if (!c) return;
    if (c->nccl) {
      ge::DeviceGuard g(c->ctx);
      (void)hipStreamSynchronize(c->ctx->stream);
      ncclCommDestroy(ge::nccl_of(c));
    }
    delete c;
  });
}

int ge_row_shard(int n, int nranks, int rank, int* rb, int* re, int* rows_per_rank) {
  return guarded([&] {
    GE_REQUIRE(rb && re && rows_per_rank, "null argument");
    GE_REQUIRE(n >= 0 && nranks >= 1 && rank >= 0 && rank < nranks, "bad arguments");
    const int chunk = (n + nranks - 1) / nranks;
    *rows_per_rank = chunk;
    *rb = std::min(n, rank * chunk);
    *re = std::min(n, (rank + 1) * chunk);
  });
}

int ge_allgather_coords(ge_comm* c, double* d_x, long long rows_per_rank, int dim) {
  return guarded([&] {
    ge::check_comm(c);
    GE_REQUIRE(d_x && rows_per_rank >= 0 && dim >= 1, "bad arguments");
    ge::DeviceGuard g(c->ctx);
    const size_t block = (size_t)rows_per_rank * dim;
    ge::allgather_dev(c, d_x + block * c->rank, d_x, sizeof(double) * block);
  });
}

int ge_assign_aggregates(int m, const int* pip, const int* pix, const int* ip, int nranks,
                         int* owner) {
  return guarded([&] {
    GE_REQUIRE(m >= 0 && pip && (pix || !ip) && owner && nranks >= 1, "bad arguments");
    const std::vector<int> o = ge::assign_aggregates(m, pip, pix, ip, nranks, nullptr);
    std::copy(o.begin(), o.end(), owner);
  });
}

int ge_assign_aggregates_split(int m, const int* pip, const int* pix, const int* ip, int nranks,
                               int min_members, int* owner) {
  return guarded([&] {
    GE_REQUIRE(m >= 0 && pip && (pix || !ip) && owner && nranks >= 1, "bad arguments");
    const std::vector<char> split = ge::split_aggregates(m, pip, pix, ip, nranks, min_members);
    const std::vector<int> o = ge::assign_aggregates(m, pip, pix, ip, nranks, &split);
    std::copy(o.begin(), o.end(), owner);
  });
}

int ge_allgather_members(ge_comm* c, double* d_x, int dim, int m, const int* pip,
                         const int* pix, const int* owner) {
  return guarded([&] {
    ge::check_comm(c);
    GE_REQUIRE(d_x && pip && pix && owner && dim >= 1 && m >= 0, "bad arguments");
    for (int a = 0; a < m; ++a)
      GE_REQUIRE(owner[a] >= 0 && owner[a] < c->nranks, "owner out of range");
    ge::DeviceGuard g(c->ctx);
    ge::allgather_members(c, d_x, dim, m, pip, pix, owner);
  });
}

int ge_force_atlas_dist(ge_comm* c, int n, const int* ip, const int* ix, const double* dx, int dim,
                        double* coords, int init_random, int iterations, const ge_fa_params* p) {
  return guarded([&] {
    ge::check_comm(c);
    GE_REQUIRE(p && (coords || n == 0), "null argument");
    GE_REQUIRE(dim >= 1 && dim <= 4, "dimension must be 1..4");
    GE_REQUIRE(iterations >= 0, "negative iteration count");
    GE_REQUIRE(n == 0 || (ip && ix && dx && ip[0] == 0), "bad CSR");
    if (n > 0) ge::check_csr(n, ip, ix, dx);  // indices in range, as the one-GPU calls
    ge::DeviceGuard g(c->ctx);
    ge::fa_host_dist(c, n, ip, ix, dx, dim, coords, init_random != 0, iterations, *p);
  });
}

int ge_force_atlas_ml_dist(ge_comm* c, int n, const int* ip, const int* ix, const double* dx,
                           int m, const int* pip, const int* pix, const int* vA,
                           const double* cA, const double* rA, double* coords, int dim,
                           int iterations, const ge_fa_params* p) {
  return guarded([&] {
    ge::check_comm(c);
    GE_REQUIRE(p && pip && pix && vA && cA && rA && (coords || n == 0), "null argument");
    GE_REQUIRE(dim >= 1 && dim <= 4, "dimension must be 1..4");
    GE_REQUIRE(n == 0 || (ip && ix && dx && ip[0] == 0), "bad CSR");
    if (n > 0) ge::check_csr(n, ip, ix, dx);  // indices in range, as the one-GPU calls
    GE_REQUIRE(m >= 0 && pip[0] == 0 && pip[m] == n, "P_T must have one entry per fine vertex");
    if (n == 0) return;
    ge::DeviceGuard g(c->ctx);
    ge::faml_host_dist(c, n, ip, ix, dx, m, pip, pix, vA, cA, rA, coords, dim, iterations, *p);
  });
}

int ge_ptap_dist(ge_comm* c, int n, const int* ip, const int* ix, const double* dx, int m,
                 const int* pip, const int* pix, ge_csr** out) {
  return guarded([&] {
    ge::check_comm(c);
    GE_REQUIRE(out && pip && pix, "null argument");
    GE_REQUIRE(n == 0 || (ip && ix && dx && ip[0] == 0), "bad CSR");
    if (n > 0) ge::check_csr(n, ip, ix, dx);  // indices in range, as the one-GPU calls
    GE_REQUIRE(m >= 0 && pip[0] == 0 && pip[m] == n, "P_T must have one entry per fine vertex");
    ge::DeviceGuard g(c->ctx);
    hipStream_t s = c->ctx->stream;
    const std::vector<int> blk = ge::ptap_row_blocks(m, pip, pix, ip, c->nranks);
    const int a0 = blk[c->rank], a1 = blk[c->rank + 1];
    ge_csr part;
    {
      ge::DevCsr A(n, ip, ix, dx, s);
      ge::DevBuf<int> dpip(m + 1), dpix(std::max(n, 1));
      dpip.upload(pip, m + 1, s);
      dpix.upload(pix, n, s);
      ge::ptap_device(c->ctx, n, A.ip.p, A.ix.p, A.dx.p, A.nnz, m, pip, dpip.p, dpix.p, a0, a1,
                      &part);
    }
    // one block per rank: its rows' lengths, column indices, values
    const size_t nr = (size_t)(a1 - a0), nz = part.indices.size();
    std::vector<unsigned char> mine(sizeof(int) * (nr + nz) + sizeof(double) * nz);
    std::vector<int> lens(nr);
    for (size_t r = 0; r < nr; ++r) lens[r] = part.indptr[r + 1] - part.indptr[r];
    unsigned char* w = mine.data();
    std::memcpy(w, lens.data(), sizeof(int) * nr);
    std::memcpy(w + sizeof(int) * nr, part.indices.data(), sizeof(int) * nz);
    std::memcpy(w + sizeof(int) * (nr + nz), part.data.data(), sizeof(double) * nz);
    const auto blocks = ge::allgatherv_host(c, mine);
    auto* C = new ge_csr();
    C->rows = C->cols = m;
    C->indptr.assign(m + 1, 0);
    for (int r = 0; r < c->nranks; ++r) {
      const size_t rr = (size_t)(blk[r + 1] - blk[r]);
      const unsigned char* b = blocks[r].data();
      const size_t rz = (blocks[r].size() - sizeof(int) * rr) / (sizeof(int) + sizeof(double));
      std::vector<int> rl(rr);
      if (rr) std::memcpy(rl.data(), b, sizeof(int) * rr);
      for (size_t q = 0; q < rr; ++q)
        C->indptr[blk[r] + q + 1] = C->indptr[blk[r] + q] + rl[q];
      const size_t base = C->indices.size();
      C->indices.resize(base + rz);
      C->data.resize(base + rz);
      if (rz) {
        std::memcpy(C->indices.data() + base, b + sizeof(int) * rr, sizeof(int) * rz);
        std::memcpy(C->data.data() + base, b + sizeof(int) * (rr + rz), sizeof(double) * rz);
      }
    }
    *out = C;
  });
}

}  // extern "C"
