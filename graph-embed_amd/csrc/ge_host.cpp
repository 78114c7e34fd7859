// ge_host.cpp -- host side of libge.so: the C ABI entry points, the coarsening
// hierarchy, the radius step, embed orchestration and synthetic graph inputs.
//
// Device work lives in ge_fa.hip / ge_faml.hip / ge_ptap.hip; this file moves
// data, sequences levels and runs the host-resident algorithms:
//   * partition hierarchy: ge_partition.cpp (incremental, bit-exact).
//   * radius ("kinetic ball") step (src/embed.cpp:615-777) with an ordered set
//     instead of a full re-sort after every event; the popped sequence (always
//     the largest (time, i, j) tuple) and every time update are the
//     reference's.

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <mutex>
#include <numeric>
#include <set>
#include <tuple>
#include <unordered_map>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "ge_internal.hpp"

namespace ge {

static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }

// Host CSR arguments: indptr starts at 0 and never decreases, every column index
// is a row id (the kernels gather by it).  O(n + nnz), OpenMP.
void check_csr(int n, const int* ip, const int* ix, const double* dx) {
  GE_REQUIRE(n >= 0, "negative row count");
  GE_REQUIRE(n == 0 || (ip && ix && dx), "null CSR array");
  if (n == 0) return;
  GE_REQUIRE(ip[0] == 0 && ip[n] >= 0, "bad indptr");
  long long bad_rows = 0, bad_cols = 0;
#pragma omp parallel for reduction(+ : bad_rows) schedule(static)
  for (int i = 0; i < n; ++i) bad_rows += ip[i + 1] < ip[i];
  GE_REQUIRE(bad_rows == 0, "indptr decreases");
  const long long nnz = ip[n];
#pragma omp parallel for reduction(+ : bad_cols) schedule(static)
  for (long long e = 0; e < nnz; ++e) bad_cols += (unsigned)ix[e] >= (unsigned)n;
  GE_REQUIRE(bad_cols == 0, "column index out of range");
}

namespace {

constexpr double kEps = 0.00001;

inline double dist_to(const double* from, const double* to, int dim) {
  double acc = 0.0;
  for (int k = 0; k < dim; ++k) {
    double t = to[k] - from[k];
    acc += t * t;
  }
  return std::sqrt(acc);
}

inline double norm_of(const double* v, int dim) {
  double acc = 0.0;
  for (int k = 0; k < dim; ++k) acc += v[k] * v[k];
  return std::sqrt(acc);
}

// ---------------------------------------------------------------------------
// radius step (src/embed.cpp:615-777)

using Event = std::tuple<double, int, int>;

// Event loop of :636-678 / :713-755.  `limit` = coords_A.size() in both.
void run_events(std::vector<Event> ev, double* r, int limit) {
  std::set<std::pair<Event, int>> live;  // (event, id) -- id breaks exact-duplicate ties
  std::unordered_map<int, std::vector<int>> touching;
  std::vector<double> when(ev.size());
  for (int id = 0; id < (int)ev.size(); ++id) {
    live.emplace(ev[id], id);
    when[id] = std::get<0>(ev[id]);
    touching[std::get<1>(ev[id])].push_back(id);
    touching[std::get<2>(ev[id])].push_back(id);
  }
  std::vector<char> gone(ev.size(), 0);
  int assigned = 0;
  auto shift = [&](int v, double t) {
    auto it = touching.find(v);
    if (it == touching.end()) return;
    for (int id : it->second) {
      if (gone[id]) continue;
      live.erase({Event(when[id], std::get<1>(ev[id]), std::get<2>(ev[id])), id});
      when[id] = -(2 * (-when[id]) - (-t));
      live.emplace(Event(when[id], std::get<1>(ev[id]), std::get<2>(ev[id])), id);
    }
  };
  while (assigned < limit && !live.empty()) {
    auto top = std::prev(live.end());
    const int id = top->second;
    const double t = std::get<0>(top->first);
    const int i = std::get<1>(top->first), j = std::get<2>(top->first);
    live.erase(top);
    gone[id] = 1;
    const double d = -t;
    if (r[i] <= 0.0 && r[j] > 0.0) {
      r[i] = d;
      shift(i, t);
      assigned += 1;
    } else if (r[i] > 0.0 && r[j] <= 0.0) {
      r[j] = d;
      shift(j, t);
      assigned += 1;
    } else if (r[i] <= 0 && r[j] <= 0) {
      r[i] = d;
      r[j] = d;
      // every live entry touching i or j moves once (:668-673)
      std::vector<int> ids;
      for (int v : {i, j}) {
        auto it = touching.find(v);
        if (it != touching.end()) ids.insert(ids.end(), it->second.begin(), it->second.end());
      }
      std::sort(ids.begin(), ids.end());
      ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
      for (int e : ids) {
        if (gone[e]) continue;
        live.erase({Event(when[e], std::get<1>(ev[e]), std::get<2>(ev[e])), e});
        when[e] = -(2 * (-when[e]) - (-t));
        live.emplace(Event(when[e], std::get<1>(ev[e]), std::get<2>(ev[e])), e);
      }
      assigned += 2;
    }
  }
}

void radius_step(int m, double* cA, double* rA, int dim, bool base, int mc, const int* PIc,
                 const int* PJc, const double* cAc, const double* rAc, const int* AcI,
                 const int* AcJ) {
  std::fill(rA, rA + m, 0.0);
  if (base) {  // :616-679, all pairs of the coarsest level
    std::vector<Event> ev;
    ev.reserve((size_t)m * (m - 1) / 2);
    for (int i = 0; i < m; ++i)
      for (int j = i + 1; j < m; ++j)
        ev.emplace_back(-dist_to(cA + (size_t)i * dim, cA + (size_t)j * dim, dim) / 2, i, j);
    run_events(std::move(ev), rA, m);
    return;
  }
  std::vector<int> grp(m);
  for (int b = 0; b < mc; ++b)
    for (int c = PIc[b]; c < PIc[b + 1]; ++c) grp[PJc[c]] = b;
#pragma omp parallel for schedule(dynamic, 1)
  for (int b = 0; b < mc; ++b) {  // :686-756, groups touch disjoint r_A entries
    const int s = PIc[b + 1] - PIc[b];
    if (s == 1) {
      rA[PJc[PIc[b]]] = rAc[b];
      continue;
    }
    std::vector<Event> ev;
    for (int x = 0; x < s; ++x) {
      const int a = PJc[PIc[b] + x];
      for (int kk = AcI[a]; kk < AcI[a + 1]; ++kk) {
        const int j = AcJ[kk];
        if (a < j && grp[j] == grp[a])
          ev.emplace_back(-dist_to(cA + (size_t)a * dim, cA + (size_t)j * dim, dim) / 2, a, j);
      }
    }
    run_events(std::move(ev), rA, m);
  }
  for (int b = 0; b < mc; ++b) {  // :757-777
    const double* cb = cAc + (size_t)b * dim;
    double reach = 0.0;
    for (int c = PIc[b]; c < PIc[b + 1]; ++c) {
      const int a = PJc[c];
      const double d = dist_to(cb, cA + (size_t)a * dim, dim) + rA[a];
      if (d > reach) reach = d;
    }
    if (reach < 0.000001) reach = 0.000001;
    for (int c = PIc[b]; c < PIc[b + 1]; ++c) {
      const int a = PJc[c];
      for (int k = 0; k < dim; ++k) {
        double& x = cA[(size_t)a * dim + k];
        x = cb[k] + (rAc[b] / reach) * (x - cb[k]);
      }
      rA[a] = (rAc[b] / reach) * rA[a];
    }
  }
}

}  // namespace

void radius_step_host(int m, double* cA, double* rA, int dim, bool base, int mc, const int* PIc,
                      const int* PJc, const double* cAc, const double* rAc, const int* AcI,
                      const int* AcJ) {
  radius_step(m, cA, rA, dim, base, mc, PIc, PJc, cAc, rAc, AcI, AcJ);
}

// ---------------------------------------------------------------------------
// multilevel FA on the device from host arrays

void faml_host(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, int m,
               const int* pip, const int* pix, const int* vA, const double* cA,
               const double* rA, double* X, int dim, int iterations, const ge_fa_params& p) {
  hipStream_t s = ctx->stream;
  std::vector<double> init((size_t)pip[m] * dim);
  uniform_stream(p.seed, init.size(), init.data());
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
  faml_run_device(ctx, n, A.ip.p, A.ix.p, A.dx.p, m, pip, dpip.p, dpix.p, dvA.p, dcA.p, drA.p,
                  dinit.p, dX.p, dim, iterations, p);
  dX.download(X, (size_t)n * dim, s);
  GE_HIP(hipStreamSynchronize(s));
}

// normalize (include/forceatlas.hpp:272-303), serial as the reference
void normalize_host(double* X, int n, int dim) {
  std::vector<double> avg(dim, 0.0);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < dim; ++k) avg[k] = avg[k] + X[(size_t)i * dim + k];
  for (int k = 0; k < dim; ++k) avg[k] = avg[k] / n;
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < dim; ++k) X[(size_t)i * dim + k] -= avg[k];
  double longest = 0.0;
  for (int i = 0; i < n; ++i) {
    double len = norm_of(X + (size_t)i * dim, dim);
    if (longest < len) longest = len;
  }
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < dim; ++k) X[(size_t)i * dim + k] = X[(size_t)i * dim + k] / longest;
}

void fa_host(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, int dim,
             double* X, bool init_random, int iterations, const ge_fa_params& p) {
  if (init_random) uniform_stream(p.seed, (size_t)n * dim, X);  // :118-125
  if (n == 0) return;
  hipStream_t s = ctx->stream;
  DevCsr A(n, ip, ix, dx, s);
  DevBuf<double> dX((size_t)n * dim);
  dX.upload(X, (size_t)n * dim, s);
  fa_run_device(ctx, n, A.nnz, A.ip.p, A.ix.p, A.dx.p, dim, dX.p, iterations, p);
  dX.download(X, (size_t)n * dim, s);
  GE_HIP(hipStreamSynchronize(s));
  if (p.normalize) normalize_host(X, n, dim);
}

// ---------------------------------------------------------------------------
// embed orchestration (src/embed.cpp:561-796): the coarsest level's forceAtlas
// (:586), then per finer level the radius step (:615-777) and
// forceAtlasMultilevel (:793).  With a communicator of more than one rank the
// level calls run sharded (ge_dist.hip); the host radius step is replicated.

void embed_impl(ge_ctx* ctx, ge_comm* comm, int levels, const int* a_n, const int* a_off,
                const int* a_nz_off, const int* a_ip, const int* a_ix, const double* a_dx,
                const int* p_rows, const int* p_off, const int* p_nz_off, const int* p_ip,
                const int* p_ix, int dim, int base_iterations, int ml_iterations,
                int print_progress, const ge_fa_params& p, double* coords_out) {
  const bool dist = comm && comm->nranks > 1;
  auto fa_level = [&](int n, const int* ip, const int* ix, const double* dx, int d, double* X,
                      bool init, int it, const ge_fa_params& pr) {
    if (dist) fa_host_dist(comm, n, ip, ix, dx, d, X, init, it, pr);
    else fa_host(ctx, n, ip, ix, dx, d, X, init, it, pr);
  };
  auto faml_level = [&](int n, const int* ip, const int* ix, const double* dx, int m,
                        const int* pip, const int* pix, const int* vA, const double* cA,
                        const double* rA, double* X, int d, int it, const ge_fa_params& pr) {
    if (dist) faml_host_dist(comm, n, ip, ix, dx, m, pip, pix, vA, cA, rA, X, d, it, pr);
    else faml_host(ctx, n, ip, ix, dx, m, pip, pix, vA, cA, rA, X, d, it, pr);
  };
  GE_REQUIRE(coords_out && a_n && a_off && a_nz_off, "null argument");
  GE_REQUIRE(levels >= 0 && dim >= 1 && dim <= 4, "bad levels or dimension");
  for (int l = 0; l < levels; ++l)  // src/embed.cpp:564-570
    GE_REQUIRE(p_rows[l] == a_n[l + 1], "As[l+1].Rows() must equal P_Ts[l].Rows()");
  auto Aip = [&](int l) { return a_ip + a_off[l]; };
  auto Aix = [&](int l) { return a_ix + a_nz_off[l]; };
  auto Adx = [&](int l) { return a_dx + a_nz_off[l]; };
  auto Pip = [&](int l) { return p_ip + p_off[l]; };
  auto Pix = [&](int l) { return p_ix + p_nz_off[l]; };
  for (int l = 0; l < levels; ++l)
    GE_REQUIRE(Pip(l)[p_rows[l]] == a_n[l], "As[l].Rows() must equal P_Ts[l].Cols()");

  const int L = levels;
  const bool prof = std::getenv("GE_PROFILE_EMBED") != nullptr;
  const char* rh = std::getenv("GE_RADIUS_HOST");
  const bool radius_host = rh && *rh && *rh != '0';
  auto clk = [] { return std::chrono::steady_clock::now(); };
  auto secs = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
  if (print_progress) std::cout << "embedding layer " << L + 1 << ": getting base coords" << std::endl;
  std::vector<double> coarse((size_t)a_n[L] * dim);
  auto t0 = clk();
  fa_level(a_n[L], Aip(L), Aix(L), Adx(L), dim, coarse.data(), true, base_iterations, p);
  if (prof)
    std::fprintf(stderr, "embed: coarsest forceAtlas n=%d %d iterations %.3fs\n", a_n[L],
                 base_iterations, secs(t0, clk()));
  std::vector<double> r_coarse, cAc;
  for (int l = L - 1; l >= 0; --l) {
    if (print_progress) std::cout << "embeding layer " << l + 1 << std::endl;  // sic (:613)
    const int m = a_n[l + 1];
    const bool base = (l + 1 == L);
    std::vector<double> rA(m);
    auto t1 = clk();
    // on the device (ge_radius.hip) unless GE_RADIUS_HOST is set or a zero
    // distance needs the serial replay
    const int mc = base ? 0 : p_rows[l + 1];
    const int* PIc = base ? nullptr : Pip(l + 1);
    const int* PJc = base ? nullptr : Pix(l + 1);
    const double* cAcp = base ? nullptr : cAc.data();
    const double* rAcp = base ? nullptr : r_coarse.data();
    if (!radius_host && radius_step_device(ctx, m, coarse.data(), rA.data(), dim, base, mc, PIc,
                                           PJc, cAcp, rAcp, Aip(l + 1), Aix(l + 1))) {
    } else {
      radius_step(m, coarse.data(), rA.data(), dim, base, mc, PIc, PJc, cAcp, rAcp, Aip(l + 1),
                  Aix(l + 1));
    }
    auto t2 = clk();
    std::vector<int> vA(a_n[l]);
    for (int a = 0; a < m; ++a)
      for (int c = Pip(l)[a]; c < Pip(l)[a + 1]; ++c) vA[Pix(l)[c]] = a;
    std::vector<double> fine((size_t)a_n[l] * dim, 0.0);
    faml_level(a_n[l], Aip(l), Aix(l), Adx(l), m, Pip(l), Pix(l), vA.data(), coarse.data(),
               rA.data(), fine.data(), dim, ml_iterations, p);
    if (prof)
      std::fprintf(stderr, "embed: level %d n=%d: radius step %.3fs, forceAtlasMultilevel %.3fs\n",
                   l, a_n[l], secs(t1, t2), secs(t2, clk()));
    cAc = std::move(coarse);
    r_coarse = std::move(rA);
    coarse = std::move(fine);
  }
  std::memcpy(coords_out, coarse.data(), sizeof(double) * coarse.size());
}

namespace {

// ---------------------------------------------------------------------------
// synthetic R-MAT + LCC (definition: tests/graphs.py)

inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void csr_from_pairs(int n, std::vector<std::pair<int, int>>& pairs, ge_csr* out) {
  out->rows = out->cols = n;
  out->indptr.assign(n + 1, 0);
  for (const auto& pr : pairs) out->indptr[pr.first + 1]++;
  for (int i = 0; i < n; ++i) out->indptr[i + 1] += out->indptr[i];
  std::vector<int> cols(pairs.size());
  std::vector<int> fill(out->indptr.begin(), out->indptr.end() - 1);
  for (const auto& pr : pairs) cols[fill[pr.first]++] = pr.second;
  std::vector<int> newp(n + 1, 0);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int i = 0; i < n; ++i) {
    auto b = cols.begin() + out->indptr[i], e = cols.begin() + out->indptr[i + 1];
    std::sort(b, e);
    newp[i + 1] = (int)(std::unique(b, e) - b);
  }
  for (int i = 0; i < n; ++i) newp[i + 1] += newp[i];
  out->indices.resize(newp[n]);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int i = 0; i < n; ++i)
    std::copy(cols.begin() + out->indptr[i], cols.begin() + out->indptr[i] + (newp[i + 1] - newp[i]),
              out->indices.begin() + newp[i]);
  out->indptr = std::move(newp);
  out->data.assign(out->indices.size(), 1.0);
}

}  // namespace
}  // namespace ge

// ===========================================================================
// C ABI

using ge::guarded;

extern "C" {

const char* ge_last_error(void) { return ge::g_last_error.c_str(); }
const char* ge_version(void) { return "graph-embed_amd 0.1 (gfx950)"; }

void ge_fa_params_default(ge_fa_params* p) {
  p->ks = 0.1;
  p->ksmax = 1.0;
  p->repel = 1.0;
  p->attract = 1.0;
  p->gravity = 1.0;
  p->delta = 1.0;
  p->tolerate = 1.0;
  p->use_weights = 1;
  p->linlog = 0;
  p->nohubs = 0;
  p->normalize = 0;
  p->seed = 12345u;
  p->mode = GE_MODE_STRICT;
}

int ge_device_count(int* count) {
  return guarded([&] {
    GE_REQUIRE(count, "null argument");
    int c = 0;
    GE_HIP(hipGetDeviceCount(&c));
    *count = c;
  });
}

int ge_ctx_create(int device, ge_ctx** out) {
  return guarded([&] {
    GE_REQUIRE(out, "null argument");
    int c = 0;
    GE_HIP(hipGetDeviceCount(&c));
    GE_REQUIRE(device >= 0 && device < c, "no such device");
    auto* ctx = new ge_ctx();
    ctx->device = device;
    ge::DeviceGuard g(ctx);
    hipError_t e = hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete ctx;
      GE_HIP(e);
    }
    ctx->stream = ctx->own;
    *out = ctx;
  });
}

int ge_ctx_destroy(ge_ctx* ctx) {
  return guarded([&] {
    if (!ctx) return;
    if (ctx->own) {
      ge::DeviceGuard g(ctx);
      (void)hipStreamSynchronize(ctx->own);
      (void)hipStreamDestroy(ctx->own);
    }
    delete ctx;
  });
}

int ge_ctx_set_stream(ge_ctx* ctx, void* s) {
  return guarded([&] {
    GE_REQUIRE(ctx, "null context");
    ctx->stream = s ? (hipStream_t)s : ctx->own;
  });
}

int ge_ctx_sync(ge_ctx* ctx) {
  return guarded([&] {
    GE_REQUIRE(ctx, "null context");
    ge::DeviceGuard g(ctx);
    GE_HIP(hipStreamSynchronize(ctx->stream));
  });
}

int ge_force_atlas(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, int dim,
                   double* coords, int init_random, int iterations, const ge_fa_params* p) {
  return guarded([&] {
    GE_REQUIRE(ctx && p && (coords || n == 0), "null argument");
    GE_REQUIRE(dim >= 1 && dim <= 4, "dimension must be 1..4");
    GE_REQUIRE(iterations >= 0, "negative iteration count");
    ge::check_csr(n, ip, ix, dx);
    ge::DeviceGuard g(ctx);
    ge::fa_host(ctx, n, ip, ix, dx, dim, coords, init_random != 0, iterations, *p);
  });
}

int ge_force_atlas_ml(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, int m,
                      const int* pip, const int* pix, const int* vA, const double* cA,
                      const double* rA, double* coords, int dim, int iterations,
                      const ge_fa_params* p) {
  return guarded([&] {
    GE_REQUIRE(ctx && p && pip && pix && vA && cA && rA && (coords || n == 0),
               "null argument");
    GE_REQUIRE(dim >= 1 && dim <= 4, "dimension must be 1..4");
    ge::check_csr(n, ip, ix, dx);
    GE_REQUIRE(m >= 0 && pip[0] == 0 && pip[m] == n, "P_T must have one entry per fine vertex");
    if (n == 0) return;
    ge::DeviceGuard g(ctx);
    ge::faml_host(ctx, n, ip, ix, dx, m, pip, pix, vA, cA, rA, coords, dim, iterations, *p);
  });
}

int ge_partition(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, double cf,
                 int printing, int positive, double stall, int matching, int merge_leaves,
                 ge_hier** out) {
  return guarded([&] {
    GE_REQUIRE(out, "null argument");
    GE_REQUIRE(n > 0, "empty graph");
    GE_REQUIRE(!merge_leaves, "mergeLeaves is not supported (off by default; buggy in the "
                              "reference, src/partitioner.cpp:1680)");
    ge::check_csr(n, ip, ix, dx);
    *out = nullptr;
    // with a context: the device path (integer weights, symmetric, ascending rows);
    // otherwise, or when the input needs it, the host path
    const char* force_host = std::getenv("GE_PARTITION_HOST");
    if (ctx && !(force_host && *force_host && *force_host != '0')) {
      try {
        *out = ge::partition_device(ctx, n, ip, ix, dx, cf, printing != 0, positive != 0, stall,
                                    matching);
      } catch (const ge::Error& e) {
        // only a device capacity limit (the list pool) falls back: the host path
        // computes the same hierarchy.  Anything else -- a resolve that did not
        // converge included -- is a device-path failure and is reported, not
        // masked as a slow host run.  GE_PARTITION_DEVICE_REQUIRE=1 (tests) makes
        // the capacity limit an error too.
        const char* req = std::getenv("GE_PARTITION_DEVICE_REQUIRE");
        if (e.code != GE_ERR_CAPACITY || (req && *req == '1')) throw;
        std::fprintf(stderr, "ge_partition: %s; using the host path\n", e.what());
        *out = nullptr;
      }
    }
    if (!*out)
      *out = ge::partition_incremental(n, ip, ix, dx, cf, printing != 0, positive != 0, stall,
                                       matching);
  });
}

int ge_hier_levels(const ge_hier* h, int* levels) {
  return guarded([&] {
    GE_REQUIRE(h && levels, "null argument");
    *levels = (int)h->rows.size();
  });
}

int ge_hier_shape(const ge_hier* h, int l, int* rows, int* cols) {
  return guarded([&] {
    GE_REQUIRE(h && rows && cols, "null argument");
    GE_REQUIRE(l >= 0 && l < (int)h->rows.size(), "level out of range");
    *rows = h->rows[l];
    *cols = h->cols[l];
  });
}

int ge_hier_copy(const ge_hier* h, int l, int* ip, int* ix) {
  return guarded([&] {
    GE_REQUIRE(h && ip && ix, "null argument");
    GE_REQUIRE(l >= 0 && l < (int)h->rows.size(), "level out of range");
    std::memcpy(ip, h->indptr[l].data(), sizeof(int) * h->indptr[l].size());
    std::memcpy(ix, h->indices[l].data(), sizeof(int) * h->indices[l].size());
  });
}

int ge_hier_free(ge_hier* h) {
  delete h;
  return GE_OK;
}

int ge_interpolation_matrix(int num_cols, int num_rows, const int* offsets, const int* sets,
                            ge_csr** out) {
  return guarded([&] {
    GE_REQUIRE(out && offsets && (sets || num_cols == 0), "null argument");
    GE_REQUIRE(offsets[0] == 0 && offsets[num_rows] == num_cols,
               "set sizes must sum to numCols (src/partitioner.cpp:63)");
    auto* c = new ge_csr();
    c->rows = num_rows;
    c->cols = num_cols;
    c->indptr.assign(offsets, offsets + num_rows + 1);
    c->indices.assign(sets, sets + num_cols);
    c->data.assign(num_cols, 1.0);
    *out = c;
  });
}

int ge_ptap(ge_ctx* ctx, int n, const int* ip, const int* ix, const double* dx, int m,
            const int* pip, const int* pix, ge_csr** out) {
  return guarded([&] {
    GE_REQUIRE(ctx && out && pip && pix, "null argument");
    ge::check_csr(n, ip, ix, dx);
    GE_REQUIRE(m >= 0 && pip[0] == 0 && pip[m] == n, "P_T must have one entry per fine vertex");
    ge::DeviceGuard g(ctx);
    hipStream_t s = ctx->stream;
    auto* c = new ge_csr();
    try {
      ge::DevCsr A(n, ip, ix, dx, s);
      ge::DevBuf<int> dpip(m + 1), dpix(std::max(n, 1));
      dpip.upload(pip, m + 1, s);
      dpix.upload(pix, n, s);
      ge::ptap_device(ctx, n, A.ip.p, A.ix.p, A.dx.p, A.nnz, m, pip, dpip.p, dpix.p, 0, m, c);
    } catch (...) {
      delete c;
      throw;
    }
    *out = c;
  });
}

int ge_csr_shape(const ge_csr* c, int* rows, int* cols, long long* nnz) {
  return guarded([&] {
    GE_REQUIRE(c && rows && cols && nnz, "null argument");
    *rows = c->rows;
    *cols = c->cols;
    *nnz = (long long)c->indices.size();
  });
}

int ge_csr_copy(const ge_csr* c, int* ip, int* ix, double* dx) {
  return guarded([&] {
    GE_REQUIRE(c && ip && (ix || c->indices.empty()) && (dx || c->data.empty()),
               "null argument");
    std::memcpy(ip, c->indptr.data(), sizeof(int) * c->indptr.size());
    if (!c->indices.empty()) std::memcpy(ix, c->indices.data(), sizeof(int) * c->indices.size());
    if (!c->data.empty()) std::memcpy(dx, c->data.data(), sizeof(double) * c->data.size());
  });
}

int ge_csr_free(ge_csr* c) {
  delete c;
  return GE_OK;
}

int ge_modularity(int n, const int* ip, const int* ix, const double* dx, int m, const int* vA,
                  double* q) {
  return guarded([&] {
    GE_REQUIRE(q && vA, "null argument");
    ge::check_csr(n, ip, ix, dx);
    std::vector<double> in(m, 0.0), outw(m, 0.0);
    double T = 0.0;
    for (int i = 0; i < n; ++i)
      for (int e = ip[i]; e < ip[i + 1]; ++e) {
        const int w = (int)dx[e];  // sic: int truncation (src/partitioner.cpp:90)
        if (vA[i] == vA[ix[e]]) in[vA[i]] += w;
        else outw[vA[i]] += w;
        T += w;
      }
    double s = 0.0;
    for (int a = 0; a < m; ++a) {
      const double al = (in[a] + outw[a]) / T;
      s += in[a] / T - al * al;
    }
    *q = s;
  });
}

int ge_embed(ge_ctx* ctx, int levels, const int* a_n, const int* a_off, const int* a_nz_off,
             const int* a_ip, const int* a_ix, const double* a_dx, const int* p_rows,
             const int* p_off, const int* p_nz_off, const int* p_ip, const int* p_ix, int dim,
             int base_iterations, int ml_iterations, int print_progress, const ge_fa_params* pp,
             double* coords_out) {
  return guarded([&] {
    GE_REQUIRE(ctx && pp, "null argument");
    ge::DeviceGuard g(ctx);
    ge::embed_impl(ctx, nullptr, levels, a_n, a_off, a_nz_off, a_ip, a_ix, a_dx, p_rows, p_off,
                   p_nz_off, p_ip, p_ix, dim, base_iterations, ml_iterations, print_progress, *pp,
                   coords_out);
  });
}

int ge_embed_dist(ge_comm* comm, int levels, const int* a_n, const int* a_off,
                  const int* a_nz_off, const int* a_ip, const int* a_ix, const double* a_dx,
                  const int* p_rows, const int* p_off, const int* p_nz_off, const int* p_ip,
                  const int* p_ix, int dim, int base_iterations, int ml_iterations,
                  int print_progress, const ge_fa_params* pp, double* coords_out) {
  return guarded([&] {
    GE_REQUIRE(comm && comm->ctx && pp, "null argument");
    ge::DeviceGuard g(comm->ctx);
    ge::embed_impl(comm->ctx, comm, levels, a_n, a_off, a_nz_off, a_ip, a_ix, a_dx, p_rows, p_off,
                   p_nz_off, p_ip, p_ix, dim, base_iterations, ml_iterations,
                   print_progress && comm->rank == 0, *pp, coords_out);
  });
}

int ge_radius_step(int m, double* cA, double* rA, int dim, int base, int mc, const int* PIc,
                   const int* PJc, const double* cAc, const double* rAc, const int* AcI,
                   const int* AcJ) {
  return guarded([&] {
    GE_REQUIRE(m >= 0 && cA && rA && dim >= 1, "bad radius-step arguments");
    GE_REQUIRE(base || (PIc && PJc && cAc && rAc && AcI && AcJ), "null argument");
    ge::radius_step(m, cA, rA, dim, base != 0, mc, PIc, PJc, cAc, rAc, AcI, AcJ);
  });
}

int ge_uniform_stream(unsigned seed, long long count, double* out) {
  return guarded([&] {
    GE_REQUIRE(count >= 0 && (out || count == 0), "bad arguments");
    ge::uniform_stream(seed, (size_t)count, out);
  });
}

int ge_rmat_csr(int n, long long draws, unsigned long long seed, ge_csr** out) {
  return guarded([&] {
    GE_REQUIRE(out && n > 1 && draws >= 0, "bad R-MAT arguments");
    int scale = 1;
    while ((1ll << scale) < n) ++scale;
    const uint64_t base = ge::splitmix64(seed);
    const double a = 0.57, b = 0.19, c = 0.19;
    std::vector<int> src(draws), dst(draws);
    std::vector<char> ok(draws);
#pragma omp parallel for schedule(static)
    for (long long e = 0; e < draws; ++e) {
      long long s = 0, d = 0;
      for (int l = 0; l < scale; ++l) {
        const uint64_t h = ge::splitmix64(base + (uint64_t)e * 64ull + (uint64_t)l);
        const double u = (double)(h >> 11) * 0x1.0p-53;
        const int q = u < a ? 0 : (u < a + b ? 1 : (u < a + b + c ? 2 : 3));
        s = (s << 1) | (q >> 1);
        d = (d << 1) | (q & 1);
      }
      ok[e] = (s < n && d < n && s != d);
      src[e] = (int)s;
      dst[e] = (int)d;
    }
    std::vector<std::pair<int, int>> pairs;
    pairs.reserve((size_t)draws * 2);
    for (long long e = 0; e < draws; ++e)
      if (ok[e]) {
        pairs.emplace_back(src[e], dst[e]);
        pairs.emplace_back(dst[e], src[e]);
      }
    auto* g = new ge_csr();
    ge::csr_from_pairs(n, pairs, g);
    *out = g;
  });
}

int ge_largest_component(int n, const int* ip, const int* ix, const double* dx, ge_csr** out) {
  return guarded([&] {
    GE_REQUIRE(out, "null argument");
    ge::check_csr(n, ip, ix, dx);
    std::vector<int> comp(n, -1), stack;
    int nc = 0;
    std::vector<int> sizes;
    for (int s = 0; s < n; ++s) {
      if (comp[s] != -1) continue;
      comp[s] = nc;
      int cnt = 0;
      stack.push_back(s);
      while (!stack.empty()) {
        const int v = stack.back();
        stack.pop_back();
        ++cnt;
        for (int e = ip[v]; e < ip[v + 1]; ++e)
          if (comp[ix[e]] == -1) {
            comp[ix[e]] = nc;
            stack.push_back(ix[e]);
          }
      }
      sizes.push_back(cnt);
      ++nc;
    }
    int best = 0;
    for (int c = 1; c < nc; ++c)
      if (sizes[c] > sizes[best]) best = c;  // first largest wins (embedder.cpp:80-84)
    std::vector<int> newid(n, -1);
    int k = 0;
    for (int v = 0; v < n; ++v)
      if (nc > 0 && comp[v] == best) newid[v] = k++;
    auto* g = new ge_csr();
    g->rows = g->cols = k;
    g->indptr.assign(k + 1, 0);
    for (int v = 0; v < n; ++v) {
      if (newid[v] < 0) continue;
      for (int e = ip[v]; e < ip[v + 1]; ++e)
        if (newid[ix[e]] >= 0) {
          g->indices.push_back(newid[ix[e]]);
          g->data.push_back(dx[e]);
        }
      g->indptr[newid[v] + 1] = (int)g->indices.size();
    }
    *out = g;
  });
}

}  // extern "C"
