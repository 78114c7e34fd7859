// ge_oracle.cpp -- CPU restatement of graph-embed's hot path.
//
// TEST INFRASTRUCTURE ONLY (see ge_oracle.h): the checker for the HIP path and
// the timed CPU baseline.  PARITY UNPINNED against the reference build (the
// reference needs the absent linalgcpp and ships no fixtures); cross-checked
// against tests/pyref.py.
//
// Build: see oracle/Makefile.  Compiled with -O2 -ffp-contract=off so every
// multiply and add rounds separately, as in the reference's x86-64 -O2 build.
//
// The arithmetic below keeps the reference's expression trees exactly
// (operand order, parenthesisation, serial accumulation order).  The code
// structure is our own: flat arrays, one helper per reference loop nest.

#include "ge_oracle.h"

#include <algorithm>
#include <cassert>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <random>
#include <tuple>
#include <unordered_map>
#include <utility>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

constexpr int kMaxDim = 16;
constexpr double kEps = 0.00001;  // include/forceatlas.hpp:110, :337

void set_threads(int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
}

// distance(v1, v2) of include/forceatlas.hpp:70-78: sum of (v2-v1)^2 over k in
// ascending k starting from 0.0, then sqrt.
inline double dist_to(const double* from, const double* to, int dim) {
  double acc = 0.0;
  for (int k = 0; k < dim; ++k) {
    double t = to[k] - from[k];
    acc += t * t;
  }
  return std::sqrt(acc);
}

// magnitude(v) of include/forceatlas.hpp:80-87.
inline double norm_of(const double* v, int dim) {
  double acc = 0.0;
  for (int k = 0; k < dim; ++k) {
    double t = v[k];
    acc += t * t;
  }
  return std::sqrt(acc);
}

inline double clamp_eps(double x) { return (x < kEps) ? kEps : x; }

// Attraction magnitude, include/forceatlas.hpp:176-196 (and :424-444).
inline double attraction_magnitude(double dis, double a_ij, double deg_ip1,
                                   const orc_fa_params& p) {
  double f = dis;
  if (p.linlog) f = std::log(1 + f);
  if (p.delta == 1.0) {
    f = f * a_ij;
  } else if (p.delta != 0.0) {
    double sgn = (a_ij < 0) ? -1.0 : 1.0;
    double mag = (a_ij < 0) ? -a_ij : a_ij;
    f = sgn * std::pow(mag, p.delta) * f;
  }
  if (p.nohubs) f = f / deg_ip1;
  return p.attract * f;
}

// One row of the single-level force pass, include/forceatlas.hpp:148-211.
// frep != nullptr: the repulsion sums are supplied (the value acc holds after
// :151-167) and only the attraction, gravity part is evaluated.
void fa_force_row(int i, int n, const int* I, const int* J, const double* D, int dim,
                  const double* X, const double* deg, const orc_fa_params& p,
                  double* F_row, const double* frep = nullptr) {
  double acc[kMaxDim];
  for (int k = 0; k < dim; ++k) acc[k] = frep ? frep[k] : 0.0;
  const double* xi = X + (size_t)i * dim;
  const double dip1 = deg[i] + 1;
  // repulsion: every j != i in ascending j  (:151-167)
  for (int j = 0; j < (frep ? 0 : n); ++j) {
    if (j == i) continue;
    const double* xj = X + (size_t)j * dim;
    const double djp1 = deg[j] + 1;
    const double dis = clamp_eps(dist_to(xi, xj, dim));
    const double val = dip1 * djp1 * p.repel / (dis * dis);
    for (int k = 0; k < dim; ++k) {
      double dir = -(xj[k] - xi[k]) / dis;
      acc[k] += dir * val;
    }
  }
  // attraction: CSR row in stored order  (:169-203)
  for (int e = I[i]; e < I[i + 1]; ++e) {
    const double* xj = X + (size_t)J[e] * dim;
    const double dis = clamp_eps(dist_to(xi, xj, dim));
    const double a_ij = p.use_weights ? D[e] : 1.0;
    const double Fa = attraction_magnitude(dis, a_ij, dip1, p);
    for (int k = 0; k < dim; ++k) {
      double dir = (xj[k] - xi[k]) / dis;
      acc[k] += dir * Fa;
    }
  }
  // gravity  (:205-211), mag deliberately not clamped
  const double mag = norm_of(xi, dim);
  for (int k = 0; k < dim; ++k) {
    double unit = -xi[k] / mag;
    double g = unit * p.gravity * dip1;
    F_row[k] = acc[k] + g;
  }
}

// Swing + speed + position update for one vertex, include/forceatlas.hpp:214-261
// (single level: swing not clamped) and :477-530 (multilevel: clamped).
inline void fa_update_vertex(double* x, const double* F, const double* Fprev, int dim,
                             const orc_fa_params& p, bool clamp_swing) {
  double sw = dist_to(F, Fprev, dim);
  if (clamp_swing && sw < kEps) sw = kEps;
  // globalSwing / globalTraction are overwritten with 1.0 (:228, :242)
  const double gS = p.tolerate * 1.0 / 1.0;
  const double totalF = norm_of(F, dim);
  double speed = p.ks * gS / (1 + gS * std::sqrt(sw));
  const double cap = p.ksmax / totalF;
  if (speed > cap) speed = cap;
  for (int k = 0; k < dim; ++k) x[k] = F[k] * speed + x[k];
}

void degrees(int n, const int* I, const double* D, bool use_weights, double* deg) {
  for (int i = 0; i < n; ++i) {
    if (use_weights) {
      double s = 0.0;
      for (int e = I[i]; e < I[i + 1]; ++e) s += D[e];
      deg[i] = s;
    } else {
      deg[i] = 1.0 * (I[i + 1] - I[i]);
    }
  }
}

}  // namespace

extern "C" {

void orc_fa_params_default(orc_fa_params* p) {
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
}

void orc_uniform_stream(unsigned seed, long long count, double* out) {
  std::mt19937 gen(seed);
  std::uniform_real_distribution<double> u(-1.0, 1.0);
  for (long long c = 0; c < count; ++c) out[c] = u(gen);
}

void orc_degrees(int n, const int* indptr, const double* data, int use_weights,
                 double* deg) {
  degrees(n, indptr, data, use_weights != 0, deg);
}

int orc_fa_forces_rows(int n, const int* I, const int* J, const double* D, int dim,
                       const double* X, const double* deg, int rb, int re,
                       const orc_fa_params* p, double* F, int nthreads) {
  if (dim < 1 || dim > kMaxDim) return 1;
  set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
  for (int i = rb; i < re; ++i)
    fa_force_row(i, n, I, J, D, dim, X, deg, *p, F + (size_t)(i - rb) * dim);
  return 0;
}

int orc_fa_step_rows(int n, const int* I, const int* J, const double* D, int dim,
                     const double* X, const double* deg, int rb, int re, const orc_fa_params* p,
                     double* Fprev, double* Xn, int nthreads) {
  if (dim < 1 || dim > kMaxDim) return 1;
  set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
  for (int i = rb; i < re; ++i) {
    double F[kMaxDim];
    fa_force_row(i, n, I, J, D, dim, X, deg, *p, F);
    double x[kMaxDim];
    for (int k = 0; k < dim; ++k) x[k] = X[(size_t)i * dim + k];
    double* fp = Fprev + (size_t)(i - rb) * dim;
    fa_update_vertex(x, F, fp, dim, *p, false);
    for (int k = 0; k < dim; ++k) {
      Xn[(size_t)i * dim + k] = x[k];
      fp[k] = F[k];
    }
  }
  return 0;
}

// orc_fa_step_rows with the repulsion sums supplied (Frep: (re - rb) x dim, the
// value each row's force holds after :151-167) -- the check for
// ge_fa_plan_attract at sizes whose all-pairs repulsion is out of reach.
int orc_fa_step_rows_frep(int n, const int* I, const int* J, const double* D, int dim,
                          const double* X, const double* deg, int rb, int re,
                          const orc_fa_params* p, const double* Frep, double* Fprev, double* Xn,
                          int nthreads) {
  if (dim < 1 || dim > kMaxDim) return 1;
  set_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
  for (int i = rb; i < re; ++i) {
    double F[kMaxDim];
    fa_force_row(i, n, I, J, D, dim, X, deg, *p, F, Frep + (size_t)(i - rb) * dim);
    double x[kMaxDim];
    for (int k = 0; k < dim; ++k) x[k] = X[(size_t)i * dim + k];
    double* fp = Fprev + (size_t)(i - rb) * dim;
    fa_update_vertex(x, F, fp, dim, *p, false);
    for (int k = 0; k < dim; ++k) {
      Xn[(size_t)i * dim + k] = x[k];
      fp[k] = F[k];
    }
  }
  return 0;
}

int orc_force_atlas(int n, const int* I, const int* J, const double* D, int dim,
                    double* X, int init_random, unsigned seed, int iterations,
                    const orc_fa_params* pp, int nthreads) {
  if (dim < 1 || dim > kMaxDim) return 1;
  const orc_fa_params p = *pp;
  set_threads(nthreads);
  if (init_random) orc_uniform_stream(seed, (long long)n * dim, X);  // :118-125

  std::vector<double> deg(n);
  degrees(n, I, D, p.use_weights != 0, deg.data());
  std::vector<double> F((size_t)n * dim, 0.0), Fprev((size_t)n * dim, 0.0);

  // rows are independent within an iteration; small levels (the coarsest, 1e5
  // iterations) stay on one thread: a fork/join per iteration would dominate
  const bool par = n >= 256;
  for (int it = 0; it < iterations; ++it) {
#pragma omp parallel for schedule(dynamic, 16) if (par)
    for (int i = 0; i < n; ++i)
      fa_force_row(i, n, I, J, D, dim, X, deg.data(), p, &F[(size_t)i * dim]);
#pragma omp parallel for schedule(static) if (par)
    for (int i = 0; i < n; ++i)
      fa_update_vertex(X + (size_t)i * dim, &F[(size_t)i * dim], &Fprev[(size_t)i * dim],
                       dim, p, false);
    std::swap(F, Fprev);  // forces_prev = forces (:263); F is rewritten next pass
  }

  if (p.normalize) {  // :272-303
    double avg[kMaxDim];
    for (int k = 0; k < dim; ++k) avg[k] = 0.0;
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
  return 0;
}

// forceAtlasMultilevel for the aggregates aggs[0..n_aggs) (all m when aggs is
// null).  Single-thread draw order of :340-360: aggregates ascending, members in
// P_T row order, k ascending -> draw c*dim+k for P_T storage position c, whichever
// aggregates are evaluated.
int orc_force_atlas_ml_aggs(int n, const int* I, const int* J, const double* D, int m,
                            const int* PI, const int* PJ, const int* vA, const double* cA,
                            const double* rA, double* X, int dim, int iterations,
                            unsigned seed, const orc_fa_params* pp, const int* aggs,
                            int n_aggs, int nthreads) {
  if (dim < 1 || dim > kMaxDim) return 1;
  const orc_fa_params p = *pp;
  set_threads(nthreads);
  (void)n;
  const long long total = (long long)PI[m] * dim;
  std::vector<double> draws(total);
  orc_uniform_stream(seed, total, draws.data());
  const int na = aggs ? n_aggs : m;
  // Aggregates are independent (the reference's `omp parallel for` over them,
  // :340); inside one, the force rows of an iteration are independent too (each
  // row's sum is its own serial loop), so an aggregate of kInnerRows members or
  // more runs alone with its rows on the threads -- same arithmetic, and the C4/C5
  // hub aggregates (4e4-1e5 members) no longer hold one thread for minutes.
  constexpr int kInnerRows = 8192;
  auto run_agg = [&](int a, bool inner) {
    const int base = PI[a];
    const int s = PI[a + 1] - PI[a];
    const int* v = PJ + base;
    for (int i = 0; i < s; ++i)
      for (int k = 0; k < dim; ++k)
        X[(size_t)v[i] * dim + k] = draws[(size_t)(base + i) * dim + k];

    std::vector<double> deg(s);  // :362-383, internal neighbours only
#pragma omp parallel for schedule(dynamic, 64) if (inner)
    for (int i = 0; i < s; ++i) {
      double acc = 0.0;
      for (int e = I[v[i]]; e < I[v[i] + 1]; ++e)
        if (vA[J[e]] == a) acc += p.use_weights ? D[e] : 1.0;
      deg[i] = acc;
    }

    std::vector<double> F((size_t)s * dim, 0.0), Fprev((size_t)s * dim, 0.0);
    const double* ca = cA + (size_t)a * dim;
    for (int it = 0; it < iterations; ++it) {
#pragma omp parallel for schedule(dynamic, 64) if (inner)
      for (int i = 0; i < s; ++i) {
        double acc[kMaxDim];
        for (int k = 0; k < dim; ++k) acc[k] = 0.0;
        const double* xi = X + (size_t)v[i] * dim;
        const double dip1 = deg[i] + 1;
        for (int j = 0; j < s; ++j) {  // :394-410
          if (j == i) continue;
          const double* xj = X + (size_t)v[j] * dim;
          const double djp1 = deg[j] + 1;
          const double dis = clamp_eps(dist_to(xi, xj, dim));
          const double val = dip1 * djp1 * p.repel / (dis * dis);
          for (int k = 0; k < dim; ++k) {
            double dir = -(xj[k] - xi[k]) / dis;
            acc[k] += dir * val;
          }
        }
        double mag = norm_of(xi, dim);  // :411-414
        if (mag < kEps) mag = kEps;
        for (int e = I[v[i]]; e < I[v[i] + 1]; ++e) {  // :415-467
          const int j = J[e];
          if (vA[j] == a && j != i) {  // sic: local i against global j (:417)
            const double* xj = X + (size_t)j * dim;
            const double dis = clamp_eps(dist_to(xi, xj, dim));
            const double a_ij = p.use_weights ? D[e] : 1.0;
            const double Fa = attraction_magnitude(dis, a_ij, dip1, p);
            for (int k = 0; k < dim; ++k) {
              double dir = (xj[k] - xi[k]) / dis;
              acc[k] += dir * Fa;
            }
          } else {
            const double* cb = cA + (size_t)vA[j] * dim;
            const double dis = clamp_eps(dist_to(ca, cb, dim));
            const double pull = 100.0 * 1.0;  // pull * fao_ij (:453-459)
            for (int k = 0; k < dim; ++k) {
              double dir = (cb[k] - ca[k]) / dis;
              acc[k] += dir * pull / mag;
            }
          }
        }
        for (int k = 0; k < dim; ++k) {  // :469-474
          double unit = -xi[k] / mag;
          double g = unit * p.gravity * dip1;
          F[(size_t)i * dim + k] = acc[k] + g;
        }
      }
      for (int i = 0; i < s; ++i)  // :477-530
        fa_update_vertex(X + (size_t)v[i] * dim, &F[(size_t)i * dim], &Fprev[(size_t)i * dim],
                         dim, p, true);
      std::swap(F, Fprev);
    }

    // centre, scale into the ball coords_A[a] + r_A[a] * x / max  (:539-570)
    double avg[kMaxDim];
    for (int k = 0; k < dim; ++k) avg[k] = 0.0;
    for (int i = 0; i < s; ++i)
      for (int k = 0; k < dim; ++k) avg[k] = avg[k] + X[(size_t)v[i] * dim + k];
    for (int k = 0; k < dim; ++k) avg[k] = avg[k] / s;
    for (int i = 0; i < s; ++i)
      for (int k = 0; k < dim; ++k) X[(size_t)v[i] * dim + k] -= avg[k];
    double biggest = 0.0;
    for (int i = 0; i < s; ++i) {
      double len = norm_of(X + (size_t)v[i] * dim, dim);
      if (len > biggest) biggest = len;
    }
    if (biggest < kEps) biggest = kEps;
    for (int i = 0; i < s; ++i)
      for (int k = 0; k < dim; ++k) {
        double& x = X[(size_t)v[i] * dim + k];
        x = ca[k] + rA[a] * (x / biggest);
      }
  };
  for (int x = 0; x < na; ++x) {
    const int a = aggs ? aggs[x] : x;
    if (PI[a + 1] - PI[a] >= kInnerRows) run_agg(a, true);
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int x = 0; x < na; ++x) {
    const int a = aggs ? aggs[x] : x;
    if (PI[a + 1] - PI[a] < kInnerRows) run_agg(a, false);
  }
  return 0;
}

int orc_force_atlas_ml(int n, const int* I, const int* J, const double* D, int m,
                       const int* PI, const int* PJ, const int* vA, const double* cA,
                       const double* rA, double* X, int dim, int iterations,
                       unsigned seed, const orc_fa_params* pp, int nthreads) {
  return orc_force_atlas_ml_aggs(n, I, J, D, m, PI, PJ, vA, cA, rA, X, dim, iterations, seed,
                                 pp, nullptr, 0, nthreads);
}

// ---------------------------------------------------------------------------
// partition hierarchy (src/partitioner.cpp:1550-1893), default mergeLeaves=false

struct orc_hier {
  std::vector<int> rows, cols;
  std::vector<std::vector<int>> indptr, indices;
};

orc_hier* orc_partition(int n, const int* I, const int* J, const double* D, double cf,
                        int positive_merging, double stall, int matching_iterations) {
  const double inf = std::numeric_limits<double>::infinity();
  auto* h = new orc_hier();
  int N = n, M = n;

  std::vector<std::map<int, double>> adj(n);  // :1561-1577
  std::vector<double> alpha(n);
  for (int i = 0; i < n; ++i) {
    double s = 0.0;
    for (int e = I[i]; e < I[i + 1]; ++e) {
      if (J[e] != i) adj[i].insert(std::make_pair(J[e], D[e]));
      s += D[e];
    }
    alpha[i] = s;
  }
  double T = 0.0;  // :1580-1591 (d_sum only feeds Q, which does not steer)
  for (int i = 0; i < n; ++i)
    for (int e = I[i]; e < I[i + 1]; ++e) T += D[e];
  for (int i = 0; i < n; ++i) alpha[i] /= T;

  std::vector<int> basis(n), used(n), pos(n), parent(n);
  for (int i = 0; i < n; ++i) basis[i] = used[i] = pos[i] = parent[i] = i;
  auto root_of = [&](int x) {  // union-find with path compression (:1622-1633)
    int r = x;
    while (parent[r] != r) r = parent[r];
    while (parent[x] != r) {
      int nx = parent[x];
      parent[x] = r;
      x = nx;
    }
    return r;
  };
  std::vector<double> best_eta(n, -inf), best_ind(n, 0.0);
  std::vector<char> touched(n, 0);

  auto snapshot = [&]() {  // :1797-1815 / :1840-1852 + interpolationMatrix :29-65
    std::vector<std::vector<int>> groups(M);
    for (int y = 0; y < (int)basis.size(); ++y) groups[pos[root_of(basis[y])]].push_back(y);
    std::vector<int> ip(M + 1), ix;
    ix.reserve(N);
    ip[0] = 0;
    for (int r = 0; r < M; ++r) {
      for (int y : groups[r]) ix.push_back(y);
      ip[r + 1] = (int)ix.size();
    }
    h->rows.push_back(M);
    h->cols.push_back(N);
    h->indptr.push_back(std::move(ip));
    h->indices.push_back(std::move(ix));
  };

  const bool progress = std::getenv("ORC_PROGRESS") != nullptr;  // long runs (C4 digest)
  long rounds = 0;
  int M_prev = M;
  do {
    std::vector<std::pair<int, int>> merges;
    for (int pass = 0; pass < matching_iterations; ++pass) {
      // scan (:1703-1726, `omp parallel for` there too): argmax over untouched
      // neighbours, ascending j, strict >; each x writes only its own slots
#pragma omp parallel for schedule(dynamic, 512)
      for (int x = 0; x < (int)used.size(); ++x) {
        const int i = used[x];
        if (touched[i] && best_eta[i] != -inf) continue;
        double top = -inf;
        int arg = -1;
        for (const auto& kv : adj[i]) {
          if (touched[kv.first]) continue;
          double eta = 2 * (kv.second / T - alpha[i] * alpha[kv.first]);
          if (eta > top) {
            top = eta;
            arg = kv.first;
          }
        }
        best_eta[i] = top;
        best_ind[i] = arg;
      }
      // greedy resolve in `used` order (:1728-1753)
      for (int x = 0; x < (int)used.size(); ++x) {
        const int i = used[x];
        if (touched[i]) continue;
        const int j = (int)best_ind[i];
        if (j == -1 || touched[j] || best_eta[i] < best_eta[j]) continue;
        if (positive_merging && !(best_eta[i] > 0)) continue;
        if (adj[i].size() < adj[j].size())
          merges.push_back(std::make_pair(j, i));
        else
          merges.push_back(std::make_pair(i, j));
        touched[i] = touched[j] = 1;
      }
    }
    // contraction (:1756-1779)
    for (const auto& mg : merges) {
      const int keep = mg.first, gone = mg.second;
      for (const auto& kv : adj[gone]) {
        const int k = kv.first;
        adj[k].erase(adj[k].find(gone));
        best_eta[k] = -inf;
        if (k == keep) {
          alpha[keep] = alpha[keep] + alpha[gone];
        } else {
          adj[keep][k] += kv.second;
          adj[k][keep] += kv.second;
        }
      }
    }
    M_prev = M;
    if (1.0 * M / N <= cf) {
      snapshot();
      basis = used;
      N = M;
    }
    // swap-pop + union (:1819-1834)
    for (const auto& mg : merges) {
      const int keep = mg.first, gone = mg.second;
      const int slot = pos[gone];
      const int last = used.back();
      std::swap(used[slot], used[used.size() - 1]);
      used.pop_back();
      pos[last] = slot;
      parent[gone] = keep;
      touched[keep] = 0;
      M -= 1;
    }
    if (progress && (++rounds % 50) == 0)
      std::fprintf(stderr, "orc_partition: round %ld M %d levels %zu\n", rounds, M,
                   h->rows.size());
  } while (1.0 * M / M_prev < stall);
  snapshot();
  return h;
}

// The same loop (src/partitioner.cpp:1550-1893) with the per-vertex std::map
// replaced by an unordered entry list, for the C4 digest: the std::map version
// spends hours chasing tree nodes in the scans (~7 s per round at C4, 9 969 rounds).
// Every operation of the loop above is performed in the same order on the same
// cells; only the container differs, and nothing the loop computes depends on the
// container's iteration order:
//   * scan (:1703-1726): the reference walks a[i] in ascending j and keeps the
//     first strict maximum, i.e. the smallest j among the entries with the largest
//     eta; an unordered walk keeps (eta > top) or (eta == top and j < arg), which is
//     the same entry (eta is finite: weights / T and alpha products), and top is that
//     entry's eta either way;
//   * contraction (:1756-1779): one merge touches, for each neighbour k of j', the
//     cells a[k][j'] (erased), a[i'][k] and a[k][i'] (one += each) and best_eta[k];
//     distinct k touch distinct cells, so the walk order of a[j'] changes no value
//     (across merges the order is the merge order, as above);
//   * representative choice (:1737-1743): list sizes only.
// a[i][k] += w on a missing key inserts 0.0 and adds, as std::map::operator[] does.
// tests/test_oracle.py checks it against orc_partition on R-MAT / ER graphs with
// every option, and tests/golden/make_partition_digest.py reproduces the committed
// C3 digest (std::map version) before it runs C4.
namespace {
struct FlatAdj {
  std::vector<int> key;
  std::vector<double> w;
  std::unordered_map<int, int>* idx = nullptr;  // key -> slot, for long lists
  static constexpr size_t kIndexAt = 48;
  ~FlatAdj() { delete idx; }
  int find(int k) const {
    if (idx) {
      auto it = idx->find(k);
      return it == idx->end() ? -1 : it->second;
    }
    for (size_t s = 0; s < key.size(); ++s)
      if (key[s] == k) return (int)s;
    return -1;
  }
  void erase(int k) {  // the key is present (:1763 dereferences find)
    const int s = find(k);
    assert(s >= 0);
    const int last = (int)key.size() - 1;
    if (s != last) {
      key[s] = key[last];
      w[s] = w[last];
      if (idx) (*idx)[key[s]] = s;
    }
    key.pop_back();
    w.pop_back();
    if (idx) idx->erase(k);
  }
  void insert(int k, double v) {  // a new key with its value (std::map::insert)
    key.push_back(k);
    w.push_back(0.0);
    w.back() = v;
    if (idx) {
      (*idx)[k] = (int)key.size() - 1;
    } else if (key.size() > kIndexAt) {
      idx = new std::unordered_map<int, int>();
      idx->reserve(2 * key.size());
      for (size_t q = 0; q < key.size(); ++q) (*idx)[key[q]] = (int)q;
    }
  }
  void add(int k, double v) {  // a[i][k] += v
    int s = find(k);
    if (s < 0) {
      s = (int)key.size();
      key.push_back(k);
      w.push_back(0.0);
      if (idx) {
        (*idx)[k] = s;
      } else if (key.size() > kIndexAt) {
        idx = new std::unordered_map<int, int>();
        idx->reserve(2 * key.size());
        for (size_t q = 0; q < key.size(); ++q) (*idx)[key[q]] = (int)q;
      }
    }
    w[s] = w[s] + v;
  }
};
}  // namespace

orc_hier* orc_partition_flat(int n, const int* I, const int* J, const double* D, double cf,
                             int positive_merging, double stall, int matching_iterations) {
  const double inf = std::numeric_limits<double>::infinity();
  auto* h = new orc_hier();
  int N = n, M = n;

  std::vector<FlatAdj> adj(n);  // :1561-1577 (duplicate entries of a row: the map keeps the first)
  std::vector<double> alpha(n);
  for (int i = 0; i < n; ++i) {
    double s = 0.0;
    for (int e = I[i]; e < I[i + 1]; ++e) {
      if (J[e] != i && adj[i].find(J[e]) < 0) adj[i].insert(J[e], D[e]);
      s += D[e];
    }
    alpha[i] = s;
  }
  double T = 0.0;  // :1580-1591
  for (int i = 0; i < n; ++i)
    for (int e = I[i]; e < I[i + 1]; ++e) T += D[e];
  for (int i = 0; i < n; ++i) alpha[i] /= T;

  std::vector<int> basis(n), used(n), pos(n), parent(n);
  for (int i = 0; i < n; ++i) basis[i] = used[i] = pos[i] = parent[i] = i;
  auto root_of = [&](int x) {  // :1622-1633
    int r = x;
    while (parent[r] != r) r = parent[r];
    while (parent[x] != r) {
      int nx = parent[x];
      parent[x] = r;
      x = nx;
    }
    return r;
  };
  std::vector<double> best_eta(n, -inf), best_ind(n, 0.0);
  std::vector<char> touched(n, 0);

  auto snapshot = [&]() {  // :1797-1815 / :1840-1852 + interpolationMatrix :29-65
    std::vector<std::vector<int>> groups(M);
    for (int y = 0; y < (int)basis.size(); ++y) groups[pos[root_of(basis[y])]].push_back(y);
    std::vector<int> ip(M + 1), ix;
    ix.reserve(N);
    ip[0] = 0;
    for (int r = 0; r < M; ++r) {
      for (int y : groups[r]) ix.push_back(y);
      ip[r + 1] = (int)ix.size();
    }
    h->rows.push_back(M);
    h->cols.push_back(N);
    h->indptr.push_back(std::move(ip));
    h->indices.push_back(std::move(ix));
  };

  const bool progress = std::getenv("ORC_PROGRESS") != nullptr;
  long rounds = 0;
  int M_prev = M;
  do {
    std::vector<std::pair<int, int>> merges;
    for (int pass = 0; pass < matching_iterations; ++pass) {
#pragma omp parallel for schedule(dynamic, 512)
      for (int x = 0; x < (int)used.size(); ++x) {  // :1703-1726
        const int i = used[x];
        if (touched[i] && best_eta[i] != -inf) continue;
        double top = -inf;
        int arg = -1;
        const FlatAdj& a = adj[i];
        const double ai = alpha[i];
        for (size_t s = 0; s < a.key.size(); ++s) {
          const int k = a.key[s];
          if (touched[k]) continue;
          double eta = 2 * (a.w[s] / T - ai * alpha[k]);
          if (eta > top || (eta == top && k < arg)) {
            top = eta;
            arg = k;
          }
        }
        best_eta[i] = top;
        best_ind[i] = arg;
      }
      for (int x = 0; x < (int)used.size(); ++x) {  // :1728-1753
        const int i = used[x];
        if (touched[i]) continue;
        const int j = (int)best_ind[i];
        if (j == -1 || touched[j] || best_eta[i] < best_eta[j]) continue;
        if (positive_merging && !(best_eta[i] > 0)) continue;
        if (adj[i].key.size() < adj[j].key.size())
          merges.push_back(std::make_pair(j, i));
        else
          merges.push_back(std::make_pair(i, j));
        touched[i] = touched[j] = 1;
      }
    }
    for (const auto& mg : merges) {  // :1756-1779
      const int keep = mg.first, gone = mg.second;
      const FlatAdj& g = adj[gone];
      for (size_t s = 0; s < g.key.size(); ++s) {
        const int k = g.key[s];
        const double wk = g.w[s];
        adj[k].erase(gone);
        best_eta[k] = -inf;
        if (k == keep) {
          alpha[keep] = alpha[keep] + alpha[gone];
        } else {
          adj[keep].add(k, wk);
          adj[k].add(keep, wk);
        }
      }
    }
    M_prev = M;
    if (1.0 * M / N <= cf) {
      snapshot();
      basis = used;
      N = M;
    }
    for (const auto& mg : merges) {  // :1819-1834
      const int keep = mg.first, gone = mg.second;
      const int slot = pos[gone];
      const int last = used.back();
      std::swap(used[slot], used[used.size() - 1]);
      used.pop_back();
      pos[last] = slot;
      parent[gone] = keep;
      touched[keep] = 0;
      M -= 1;
      std::vector<int>().swap(adj[gone].key);  // j' is never read again
      std::vector<double>().swap(adj[gone].w);
      delete adj[gone].idx;
      adj[gone].idx = nullptr;
    }
    if (progress && (++rounds % 50) == 0)
      std::fprintf(stderr, "orc_partition_flat: round %ld M %d levels %zu\n", rounds, M,
                   h->rows.size());
  } while (1.0 * M / M_prev < stall);
  snapshot();
  return h;
}

int orc_hier_levels(const orc_hier* h) { return (int)h->rows.size(); }
void orc_hier_shape(const orc_hier* h, int l, int* rows, int* cols) {
  *rows = h->rows[l];
  *cols = h->cols[l];
}
void orc_hier_copy(const orc_hier* h, int l, int* ip, int* ix) {
  std::memcpy(ip, h->indptr[l].data(), sizeof(int) * h->indptr[l].size());
  std::memcpy(ix, h->indices[l].data(), sizeof(int) * h->indices[l].size());
}
void orc_hier_free(orc_hier* h) { delete h; }

double orc_modularity(int n, const int* I, const int* J, const double* D, int m,
                      const int* agg) {
  std::vector<double> inside(m, 0.0), outside(m, 0.0);
  double T = 0.0;
  for (int i = 0; i < n; ++i)
    for (int e = I[i]; e < I[i + 1]; ++e) {
      int w = (int)D[e];  // sic: truncation to int (:90)
      if (agg[i] == agg[J[e]])
        inside[agg[i]] += w;
      else
        outside[agg[i]] += w;
      T += w;
    }
  double q = 0.0;
  for (int a = 0; a < m; ++a) {
    double al = (inside[a] + outside[a]) / T;
    q += inside[a] / T - al * al;
  }
  return q;
}

// ---------------------------------------------------------------------------
// P^T A P.  Pinned order: B = P_T A with row a = sum over members i (P_T row
// order) of A row i, columns ascending; then C = B P with C[a][agg(c)] summed
// over B's columns c ascending.  Output rows sorted ascending.

struct orc_csr {
  int rows;
  std::vector<int> indptr, indices;
  std::vector<double> data;
};

orc_csr* orc_ptap(int n, const int* I, const int* J, const double* D, int m,
                  const int* PI, const int* PJ) {
  std::vector<int> agg(n, -1);
  for (int a = 0; a < m; ++a)
    for (int c = PI[a]; c < PI[a + 1]; ++c) agg[PJ[c]] = a;
  auto* out = new orc_csr();
  out->rows = m;
  out->indptr.assign(m + 1, 0);
  std::map<int, double> rowB, rowC;
  for (int a = 0; a < m; ++a) {
    rowB.clear();
    rowC.clear();
    for (int c = PI[a]; c < PI[a + 1]; ++c) {
      const int i = PJ[c];
      for (int e = I[i]; e < I[i + 1]; ++e) rowB[J[e]] += D[e];
    }
    for (const auto& kv : rowB) rowC[agg[kv.first]] += kv.second * 1.0;
    for (const auto& kv : rowC) {
      out->indices.push_back(kv.first);
      out->data.push_back(kv.second);
    }
    out->indptr[a + 1] = (int)out->indices.size();
  }
  return out;
}

void orc_csr_shape(const orc_csr* c, int* rows, int* nnz) {
  *rows = c->rows;
  *nnz = (int)c->indices.size();
}
void orc_csr_copy(const orc_csr* c, int* ip, int* ix, double* dx) {
  std::memcpy(ip, c->indptr.data(), sizeof(int) * c->indptr.size());
  std::memcpy(ix, c->indices.data(), sizeof(int) * c->indices.size());
  std::memcpy(dx, c->data.data(), sizeof(double) * c->data.size());
}
void orc_csr_free(orc_csr* c) { delete c; }

// ---------------------------------------------------------------------------
// radius step (src/embed.cpp:615-777)

namespace {

using Event = std::tuple<double, int, int>;

// The kinetic event loop shared by both branches (:636-678 and :713-755).
// `limit` is the reference's `m` (coords_A.size(), also in the per-group loop).
void run_events(std::vector<Event>& ev, double* r, int limit) {
  std::sort(ev.begin(), ev.end());
  int assigned = 0;
  while (assigned < limit && !ev.empty()) {
    const Event top = ev.back();
    ev.pop_back();
    const double t = std::get<0>(top);
    const int i = std::get<1>(top), j = std::get<2>(top);
    const double d = -t;
    auto shift = [&](int a, int b) {
      for (auto& e : ev) {
        const int p = std::get<1>(e), q = std::get<2>(e);
        if (p == a || q == a || p == b || q == b) {
          double cur = std::get<0>(e);
          std::get<0>(e) = -(2 * (-cur) - (-t));
        }
      }
      std::sort(ev.begin(), ev.end());
    };
    if (r[i] <= 0.0 && r[j] > 0.0) {
      r[i] = d;
      shift(i, i);
      assigned += 1;
    } else if (r[i] > 0.0 && r[j] <= 0.0) {
      r[j] = d;
      shift(j, j);
      assigned += 1;
    } else if (r[i] <= 0 && r[j] <= 0) {
      r[i] = d;
      r[j] = d;
      shift(i, j);
      assigned += 2;
    }
  }
}

}  // namespace

int orc_radius_step(int m, double* cA, double* rA, int dim, int coarse_is_base, int mc,
                    const int* PIc, const int* PJc, const double* cAc, const double* rAc,
                    const int* AcI, const int* AcJ) {
  for (int a = 0; a < m; ++a) rA[a] = 0.0;
  if (coarse_is_base) {  // :616-679
    std::vector<Event> ev;
    for (int i = 0; i < m; ++i)
      for (int j = i + 1; j < m; ++j)
        ev.emplace_back(-dist_to(cA + (size_t)i * dim, cA + (size_t)j * dim, dim) / 2, i, j);
    run_events(ev, rA, m);
    return 0;
  }
  std::vector<int> vAc(m);  // P_Ts[l+1].Transpose().GetIndices()
  for (int b = 0; b < mc; ++b)
    for (int c = PIc[b]; c < PIc[b + 1]; ++c) vAc[PJc[c]] = b;
  for (int b = 0; b < mc; ++b) {  // :686-756 (groups are independent)
    const int s = PIc[b + 1] - PIc[b];
    std::vector<Event> ev;
    for (int x = 0; x < s; ++x) {
      const int a = PJc[PIc[b] + x];
      for (int kk = AcI[a]; kk < AcI[a + 1]; ++kk) {
        const int j = AcJ[kk];
        if (a < j && vAc[j] == vAc[a])
          ev.emplace_back(-dist_to(cA + (size_t)a * dim, cA + (size_t)j * dim, dim) / 2, a, j);
      }
    }
    if (s == 1) {
      rA[PJc[PIc[b]]] = rAc[b];
      continue;
    }
    run_events(ev, rA, m);
  }
  for (int b = 0; b < mc; ++b) {  // :757-777
    double reach = 0.0;
    const double* cb = cAc + (size_t)b * dim;
    for (int c = PIc[b]; c < PIc[b + 1]; ++c) {
      const int a = PJc[c];
      double d = dist_to(cb, cA + (size_t)a * dim, dim) + rA[a];
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
  return 0;
}

// ---------------------------------------------------------------------------
// embed (src/embed.cpp:561-796): recursion unrolled from the coarsest level up.

// ---------------------------------------------------------------------------
// embedViaMinimization (src/embed.cpp:341-559), restated serially with the
// reference's vector-of-vectors layout and loop order.

int orc_embed_via_minimization(int n, const int* I, const int* J, int d, double* coords,
                               int init_random, unsigned seed, int ITER) {
  const double inf = std::numeric_limits<double>::infinity();
  const double epsilon = 10e-12;
  std::vector<std::vector<double>> X(n, std::vector<double>(d));
  if (init_random) {
    std::mt19937 gen(seed);
    std::uniform_real_distribution<double> random(-1.0, 1.0);
    for (int i = 0; i < n; i++)
      for (int k = 0; k < d; k++) X[i][k] = random(gen);
  } else {
    for (int i = 0; i < n; i++)
      for (int k = 0; k < d; k++) X[i][k] = coords[(size_t)i * d + k];
  }
  std::vector<std::vector<double>> dirs;
  for (int k = 0; k < d; k++) {  // :363-379 (the d = 2, 3 literals list the same order)
    std::vector<double> e(d, 0.0);
    e[k] = 1;
    dirs.push_back(e);
    e[k] = -1;
    dirs.push_back(e);
  }
  for (int iter = 0; iter < ITER; iter++) {
    for (int i = 0; i < n; i++) {
      std::vector<double>& x_i = X[i];
      int count = 0;
      for (int kk = I[i]; kk < I[i + 1]; kk++)
        if (J[kk] != i) count++;
      if (count == 0) continue;
      double min_J_loc = inf;
      double min_t = 0.0f;
      double min_s = -1;
      const double w = 1000000.0;
      for (int s = 0; s < (int)dirs.size(); s++) {
        const std::vector<double>& x_s = dirs[s];
        double t = 0.5;
        double jump = 0.25;
        do {
          double dJ_loc_dt = 0.0;
          for (int r = 0; r < n; r++) {
            if (i == r) continue;
            const std::vector<double>& x_r = X[r];
            double term1 = 0.0;
            double term2 = 0.0;
            for (int k = 0; k < d; k++) {
              double u_k = x_s[k] - x_i[k];
              double v_k = x_i[k] - x_r[k];
              double z_k = (u_k * t + v_k);
              term1 = term1 + z_k * z_k;
              term2 = term2 + z_k * u_k;
            }
            if (term1 < epsilon) term1 = epsilon;
            dJ_loc_dt += -((1.0 / sqrt(term1 * term1 * term1)) * term2);
          }
          for (int kk = I[i]; kk < I[i + 1]; kk++) {
            int r = J[kk];
            if (i == r) continue;
            const std::vector<double>& x_r = X[r];
            double term = 0.0;
            for (int k = 0; k < d; k++) {
              double a = (1 - t) * x_i[k] + t * x_s[k] - x_r[k];
              term += w * 2.0 * a * (x_s[k] - x_i[k]);
            }
            dJ_loc_dt += term;
          }
          if (dJ_loc_dt < 0.0) t = t + jump;
          else t = t - jump;
          jump = jump / 2.0;
        } while (jump > 1.e-4);
        double J_loc = 0.0;
        for (int r = 0; r < n; r++) {
          if (i == r) continue;
          const std::vector<double>& x_r = X[r];
          double term1 = 0.0;
          for (int k = 0; k < d; k++) {
            double u_k = x_s[k] - x_i[k];
            double v_k = x_i[k] - x_r[k];
            double z_k = (u_k * t + v_k);
            term1 = term1 + z_k * z_k;
          }
          if (term1 < epsilon) term1 = epsilon;
          J_loc = J_loc + 1.0 / sqrt(term1);
        }
        for (int kk = I[i]; kk < I[i + 1]; kk++) {
          int r = J[kk];
          if (i == r) continue;
          const std::vector<double>& x_r = X[r];
          double term = 0.0;
          for (int k = 0; k < d; k++) {
            double a = (1 - t) * x_i[k] + t * x_s[k] - x_r[k];
            term += a * a;
          }
          J_loc += w * term;
        }
        if (J_loc < min_J_loc) {
          min_J_loc = J_loc;
          min_t = t;
          min_s = s;
        }
      }
      if (min_s >= 0)
        for (int k = 0; k < d; k++)
          X[i][k] = X[i][k] * (1 - min_t) + dirs[(int)min_s][k] * min_t;
    }
  }
  if (n > 1) {
    std::vector<double> avg(d);
    for (int i = 1; i < n; i++)
      for (int k = 0; k < d; k++) avg[k] = avg[k] + X[i][k];
    for (int k = 0; k < d; k++) avg[k] = avg[k] / (n - 1);
    for (int i = 0; i < n; i++)
      for (int k = 0; k < d; k++) X[i][k] -= avg[k];
    double max_length = 0.0;
    for (int i = 1; i < n; i++) {
      double sum = 0.0;
      for (int k = 0; k < d; k++) sum += X[i][k] * X[i][k];
      double length = sqrt(sum);
      if (max_length < length) max_length = length;
    }
    for (int i = 0; i < n; i++)
      for (int k = 0; k < d; k++) X[i][k] = X[i][k] / max_length;
  }
  for (int i = 0; i < n; i++)
    for (int k = 0; k < d; k++) coords[(size_t)i * d + k] = X[i][k];
  return 0;
}

namespace {

// anyToMultilevel(minimizer) applied to one level (src/embed.cpp:23-83): per
// aggregate a, the members' internal edges as an r x r matrix of counts (the
// CooMatrix of 1.0 entries summed by ToSparse), the minimizer on it, then the
// result normalised by its largest norm and placed in a's ball.
void any_to_multilevel_minimization(int n, const int* I, const int* J, int m, const int* PI,
                                    const int* PJ, const int* v_A, const double* cA,
                                    const double* rA, double* coords, int d, unsigned seed,
                                    int min_iterations) {
  (void)n;
  for (int a = 0; a < m; a++) {
    std::vector<int> v(PJ + PI[a], PJ + PI[a + 1]);
    const int r = (int)v.size();
    std::vector<std::map<int, double>> rows(r);
    for (int i = 0; i < r; i++)
      for (int k2 = I[v[i]]; k2 < I[v[i] + 1]; k2++) {
        const int j = J[k2];
        if (v_A[j] == a) {
          int jp = -1;
          for (int j2 = 0; j2 < r; j2++)
            if (j == v[j2]) jp = j2;
          rows[i][jp] += 1.0;
        }
      }
    std::vector<int> ci(r + 1, 0), cj;
    for (int i = 0; i < r; i++) {
      for (const auto& e : rows[i]) cj.push_back(e.first);
      ci[i + 1] = (int)cj.size();
    }
    // embedViaMinimization(A, d) starts from r x d zeros (:341-345), so it never
    // draws: the empty-coords branch (:353) is not taken
    std::vector<double> nc((size_t)r * d, 0.0);
    orc_embed_via_minimization(r, ci.data(), cj.data(), d, nc.data(), 0, seed, min_iterations);
    double mx = 0.0;
    for (int i = 0; i < r; i++) {
      double sum = 0.0;
      for (int k = 0; k < d; k++) sum += nc[(size_t)i * d + k] * nc[(size_t)i * d + k];
      const double mag = sqrt(sum);
      if (mag > mx) mx = mag;
    }
    for (int i = 0; i < r; i++)
      for (int k = 0; k < d; k++)
        coords[(size_t)v[i] * d + k] = cA[(size_t)a * d + k] + rA[a] * (nc[(size_t)i * d + k] / mx);
  }
}

}  // namespace

static int embed_levels(int levels, const int* a_n, const int* a_off, const int* a_nz_off,
                        const int* a_ip, const int* a_ix, const double* a_dx, const int* p_rows,
                        const int* p_off, const int* p_nz_off, const int* p_ip, const int* p_ix,
                        int dim, unsigned seed, int base_iterations, int ml_iterations,
                        int min_iterations, double* coords_out, int nthreads) {
  for (int l = 0; l < levels; ++l)  // shape asserts (:564-570)
    if (p_rows[l] != a_n[l + 1]) return 2;
  orc_fa_params p;
  orc_fa_params_default(&p);
  auto A_ip = [&](int l) { return a_ip + a_off[l]; };
  auto A_ix = [&](int l) { return a_ix + a_nz_off[l]; };
  auto A_dx = [&](int l) { return a_dx + a_nz_off[l]; };
  auto P_ip = [&](int l) { return p_ip + p_off[l]; };
  auto P_ix = [&](int l) { return p_ix + p_nz_off[l]; };

  // base: forceAtlas(As[L], d) with random init (:582-587)
  const int L = levels;
  std::vector<double> coarse((size_t)a_n[L] * dim);
  int rc = orc_force_atlas(a_n[L], A_ip(L), A_ix(L), A_dx(L), dim, coarse.data(), 1, seed,
                           base_iterations, &p, nthreads);
  if (rc) return rc;
  std::vector<double> r_coarse;  // r_Ac of the level below (empty at the base)
  std::vector<double> cAc;       // coords_Ac
  for (int l = L - 1; l >= 0; --l) {
    const int m = a_n[l + 1];
    std::vector<double> rA(m);
    const bool base = (l + 1 == L);
    rc = orc_radius_step(m, coarse.data(), rA.data(), dim, base ? 1 : 0,
                         base ? 0 : p_rows[l + 1], base ? nullptr : P_ip(l + 1),
                         base ? nullptr : P_ix(l + 1), base ? nullptr : cAc.data(),
                         base ? nullptr : r_coarse.data(), A_ip(l + 1), A_ix(l + 1));
    if (rc) return rc;
    std::vector<int> vA(a_n[l]);
    for (int a = 0; a < m; ++a)
      for (int c = P_ip(l)[a]; c < P_ip(l)[a + 1]; ++c) vA[P_ix(l)[c]] = a;
    std::vector<double> fine((size_t)a_n[l] * dim, 0.0);
    if (l == 0 && min_iterations >= 0) {  // embedVia: the finest level's embedder
      any_to_multilevel_minimization(a_n[l], A_ip(l), A_ix(l), m, P_ip(l), P_ix(l), vA.data(),
                                     coarse.data(), rA.data(), fine.data(), dim, seed,
                                     min_iterations);
      cAc = std::move(coarse);
      r_coarse = std::move(rA);
      coarse = std::move(fine);
      continue;
    }
    rc = orc_force_atlas_ml(a_n[l], A_ip(l), A_ix(l), A_dx(l), m, P_ip(l), P_ix(l), vA.data(),
                            coarse.data(), rA.data(), fine.data(), dim, ml_iterations, seed,
                            &p, nthreads);
    if (rc) return rc;
    cAc = std::move(coarse);
    r_coarse = std::move(rA);
    coarse = std::move(fine);
  }
  std::memcpy(coords_out, coarse.data(), sizeof(double) * coarse.size());
  return 0;
}

int orc_embed(int levels, const int* a_n, const int* a_off, const int* a_nz_off,
              const int* a_ip, const int* a_ix, const double* a_dx, const int* p_rows,
              const int* p_off, const int* p_nz_off, const int* p_ip, const int* p_ix,
              int dim, unsigned seed, int base_iterations, int ml_iterations,
              double* coords_out, int nthreads) {
  return embed_levels(levels, a_n, a_off, a_nz_off, a_ip, a_ix, a_dx, p_rows, p_off, p_nz_off,
                      p_ip, p_ix, dim, seed, base_iterations, ml_iterations, -1, coords_out,
                      nthreads);
}

int orc_embed_via_minimization_ml(int levels, const int* a_n, const int* a_off,
                                  const int* a_nz_off, const int* a_ip, const int* a_ix,
                                  const double* a_dx, const int* p_rows, const int* p_off,
                                  const int* p_nz_off, const int* p_ip, const int* p_ix,
                                  int dim, unsigned seed, int base_iterations, int ml_iterations,
                                  int min_iterations, double* coords_out, int nthreads) {
  if (levels < 1 || min_iterations < 0) return 2;
  return embed_levels(levels, a_n, a_off, a_nz_off, a_ip, a_ix, a_dx, p_rows, p_off, p_nz_off,
                      p_ip, p_ix, dim, seed, base_iterations, ml_iterations, min_iterations,
                      coords_out, nthreads);
}

}  // extern "C"
