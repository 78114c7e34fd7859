// ge_partition.cpp -- the coarsening hierarchy (partition::partition,
// src/partitioner.cpp:1550-1893), bit-exact, with work proportional to what
// changes per round instead of to the graph.
//
// The reference runs rounds of greedy modularity pair matching until a round
// merges nothing.  Rounds grow with the largest aggregate (a hub absorbs one
// neighbour per round: 1255 rounds for a 148K-vertex R-MAT LCC), and every
// round rescans every alive vertex's adjacency (std::map) twice.  Here:
//
//  * Adjacency: one open-addressing hash table per vertex (O(1) find/insert/
//    erase).  The scan takes the largest eta with ties to the smallest
//    neighbour id -- exactly what the reference's ascending map walk with
//    strict `>` selects (:1710-1720) -- so iteration order does not matter.
//    The contraction adds each weight once per merge, in merge order, like
//    `a[i'][k] += w; a[k][i'] += w` (:1772-1773).
//  * Scan skipping: a vertex is rescanned only if an input of its scan changed
//    since its last scan (its neighbours or their weights, alpha of it or of a
//    neighbour, a neighbour's busy flag).  A clean vertex would recompute the
//    same (max_eta, max_ind), so best/arg stay identical to the reference's
//    arrays at every step.  The reference's own skip rule
//    (`notouch[i] && max_eta[i] != -inf`, :1706) is applied on top.
//  * Resolve: only vertices with a usable candidate (max_ind != -1, and
//    max_eta > 0 under positiveMerging) can merge (:1730-1735).  They are kept
//    in a bitmap over `used` slots and visited in slot order -- the reference's
//    `used` order -- so the greedy decisions are the same.

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <limits>
#include <new>
#include <numeric>
#include <vector>

#include "ge_internal.hpp"

namespace ge {
namespace {

// int -> double map: entries kept dense (iteration touches live entries only).
// Up to kSmall entries live inline in the object (most vertices of a
// power-law graph: one cache line, no pointer chase); larger maps keep
// keys/vals arrays on the heap located through an open-addressing index table
// (linear probing, tombstones).  Erase moves the last entry into the hole.
class NbrMap {
 public:
  static constexpr int kSmall = 3;
  static constexpr int kEmpty = -1, kTomb = -2;
  NbrMap() = default;
  NbrMap(const NbrMap&) = delete;
  NbrMap& operator=(const NbrMap&) = delete;
  ~NbrMap() { clear(); }
  int size() const { return size_; }
  const int* keys() const { return big() ? u_.b.keys : u_.s.k; }
  const double* vals() const { return big() ? u_.b.vals : u_.s.v; }

  void reserve(int want) {
    if (want > kSmall) make_big(want);
  }
  // first insertion wins (std::map::insert semantics)
  void insert_new(int k, double v) {
    if (index_of(k) >= 0) return;
    append(k, v);
  }
  // m[k] += v (operator[] then +=: 0.0 + v for a new key)
  void add(int k, double v) {
    const int x = index_of(k);
    if (x >= 0) {
      mvals()[x] += v;
      return;
    }
    append(k, 0.0 + v);
  }
  const double* find(int k) const {
    const int x = index_of(k);
    return x < 0 ? nullptr : vals() + x;
  }
  void erase(int k) {
    if (!big()) {
      for (int x = 0; x < size_; ++x)
        if (u_.s.k[x] == k) {
          --size_;
          u_.s.k[x] = u_.s.k[size_];
          u_.s.v[x] = u_.s.v[size_];
          return;
        }
      return;
    }
    const int at = locate(k);
    if (at < 0) return;
    int* t = u_.b.table;
    const int idx = t[at];
    t[at] = kTomb;
    const int last = size_ - 1;
    if (idx != last) {
      t[locate(u_.b.keys[last])] = idx;
      u_.b.keys[idx] = u_.b.keys[last];
      u_.b.vals[idx] = u_.b.vals[last];
    }
    --size_;
  }
  // visit entries [b, e) of the dense order (for splitting one map across threads)
  template <class F>
  void for_range(int b, int e, F&& f) const {
    const int* kk = keys();
    const double* vv = vals();
    for (int x = b; x < e; ++x) f(kk[x], vv[x]);
  }
  template <class F>
  void for_each(F&& f) const {
    for_range(0, size_, f);
  }
  void clear() {
    if (big()) {
      std::free(u_.b.keys);
      std::free(u_.b.vals);
      std::free(u_.b.table);
    }
    size_ = kcap_ = tcap_ = used_ = 0;
  }

 private:
  struct Small {
    int k[kSmall];
    double v[kSmall];
  };
  struct Big {
    int* keys;
    double* vals;
    int* table;
  };
  bool big() const { return kcap_ > 0; }
  double* mvals() { return big() ? u_.b.vals : u_.s.v; }
  static int hash(int k) { return (int)(((uint32_t)k * 2654435761u) >> 1); }
  int index_of(int k) const {
    if (!big()) {
      for (int x = 0; x < size_; ++x)
        if (u_.s.k[x] == k) return x;
      return -1;
    }
    const int at = locate(k);
    return at < 0 ? -1 : u_.b.table[at];
  }
  // table slot holding k, or -1
  int locate(int k) const {
    const int mask = tcap_ - 1;
    const int* t = u_.b.table;
    for (int h = hash(k) & mask;; h = (h + 1) & mask) {
      const int x = t[h];
      if (x == kEmpty) return -1;
      if (x >= 0 && u_.b.keys[x] == k) return h;
    }
  }
  void append(int k, double v) {
    if (!big()) {
      if (size_ < kSmall) {
        u_.s.k[size_] = k;
        u_.s.v[size_] = v;
        ++size_;
        return;
      }
      make_big(2 * kSmall);
    }
    if (size_ == kcap_) {
      kcap_ *= 2;
      u_.b.keys = static_cast<int*>(std::realloc(u_.b.keys, sizeof(int) * kcap_));
      u_.b.vals = static_cast<double*>(std::realloc(u_.b.vals, sizeof(double) * kcap_));
      if (!u_.b.keys || !u_.b.vals) throw std::bad_alloc();
    }
    if (2 * (used_ + 1) > tcap_) {
      int cap = 4;
      while (cap < 4 * (size_ + 1)) cap <<= 1;  // load <= 1/4 after rehash
      rehash(cap);
    }
    // first free slot on k's chain (k is absent)
    const int mask = tcap_ - 1;
    int* t = u_.b.table;
    int at = hash(k) & mask;
    while (t[at] >= 0) at = (at + 1) & mask;
    if (t[at] == kEmpty) ++used_;
    t[at] = size_;
    u_.b.keys[size_] = k;
    u_.b.vals[size_] = v;
    ++size_;
  }
  void make_big(int want) {
    if (big()) {
      if (want <= kcap_) return;
      u_.b.keys = static_cast<int*>(std::realloc(u_.b.keys, sizeof(int) * want));
      u_.b.vals = static_cast<double*>(std::realloc(u_.b.vals, sizeof(double) * want));
      if (!u_.b.keys || !u_.b.vals) throw std::bad_alloc();
      kcap_ = want;
      int cap = 4;
      while (cap < 2 * want) cap <<= 1;
      if (cap > tcap_) rehash(cap);
      return;
    }
    Small old = u_.s;
    const int n = size_;
    kcap_ = std::max(want, 2 * kSmall);
    u_.b.keys = static_cast<int*>(std::malloc(sizeof(int) * kcap_));
    u_.b.vals = static_cast<double*>(std::malloc(sizeof(double) * kcap_));
    u_.b.table = nullptr;
    if (!u_.b.keys || !u_.b.vals) throw std::bad_alloc();
    for (int x = 0; x < n; ++x) {
      u_.b.keys[x] = old.k[x];
      u_.b.vals[x] = old.v[x];
    }
    int cap = 4;
    while (cap < 2 * kcap_) cap <<= 1;
    tcap_ = 0;
    rehash(cap);
  }
  void rehash(int cap) {
    int* t = static_cast<int*>(std::malloc(sizeof(int) * cap));
    if (!t) throw std::bad_alloc();
    std::fill(t, t + cap, kEmpty);
    const int mask = cap - 1;
    for (int x = 0; x < size_; ++x) {
      int at = hash(u_.b.keys[x]) & mask;
      while (t[at] != kEmpty) at = (at + 1) & mask;
      t[at] = x;
    }
    std::free(u_.b.table);
    u_.b.table = t;
    tcap_ = cap;
    used_ = size_;
  }
  union {
    Small s;
    Big b;
  } u_;
  int size_ = 0, kcap_ = 0, tcap_ = 0, used_ = 0;
};

struct Bitmap {
  std::vector<uint64_t> w;
  void resize(size_t bits) { w.assign((bits + 63) / 64, 0); }
  void set(int i) { w[i >> 6] |= 1ull << (i & 63); }
  void clr(int i) { w[i >> 6] &= ~(1ull << (i & 63)); }
  bool get(int i) const { return (w[i >> 6] >> (i & 63)) & 1ull; }
};

}  // namespace

ge_hier* partition_incremental(int n, const int* I, const int* J, const double* Dv, double cf,
                               bool printing, bool positive, double stall, int matching) {
  const double inf = std::numeric_limits<double>::infinity();
  const bool prof = std::getenv("GE_PROFILE_PARTITION") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto secs = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double>(b - a).count();
  };
  const auto t_start = now();
  auto* h = new ge_hier();
  int N = n, M = n;

  std::vector<NbrMap> adj(n);
  std::vector<double> alpha(n);
#pragma omp parallel for schedule(dynamic, 256)
  for (int i = 0; i < n; ++i) {  // :1561-1577
    adj[i].reserve(I[i + 1] - I[i]);
    double s = 0.0;
    for (int e = I[i]; e < I[i + 1]; ++e) {
      if (J[e] != i) adj[i].insert_new(J[e], Dv[e]);
      s += Dv[e];
    }
    alpha[i] = s;
  }
  double T = 0.0, self_sum = 0.0;  // :1580-1591
  for (int i = 0; i < n; ++i)
    for (int e = I[i]; e < I[i + 1]; ++e) {
      if (J[e] == i) self_sum += Dv[e];
      T += Dv[e];
    }
  for (int i = 0; i < n; ++i) alpha[i] /= T;
  double Q = self_sum / T;
  for (int i = 0; i < n; ++i) Q += -alpha[i] * alpha[i];

  std::vector<int> basis(n), alive(n), slot(n), up(n);
  std::iota(basis.begin(), basis.end(), 0);
  alive = slot = up = basis;
  std::vector<char> dead(n, 0), busy(n, 0), dirty(n, 1);
  std::vector<double> best(n, -inf);
  std::vector<int> arg(n, 0);
  // runner-up of each clean vertex's last scan (value, index) under the same
  // order (eta descending, index ascending).  Etas only fall while a vertex stays
  // clean, so it is an upper bound on the current runner-up.  second_idx = -1:
  // the scan found no runner-up; kUnknown: not known (after a demotion).
  constexpr int kUnknown = -2;
  std::vector<double> second(n, -inf);
  std::vector<int> second_idx(n, -1);
  std::vector<int> work(n);  // dirty vertices
  std::iota(work.begin(), work.end(), 0);
  Bitmap cand;  // over `alive` slots: max_ind != -1 (and max_eta > 0 if positive)
  cand.resize(n);

  long long msrc[6] = {0, 0, 0, 0, 0, 0};
  int mcur = 0;
  auto mark = [&](int v) {
    if (!dirty[v]) {
      dirty[v] = 1;
      work.push_back(v);
      ++msrc[mcur];
    }
  };
  auto mark_nbrs = [&](int v) { adj[v].for_each([&](int k, double) { mark(k); }); };
  auto set_cand = [&](int v) {
    const bool c = arg[v] != -1 && (!positive || best[v] > 0);
    if (c) cand.set(slot[v]);
    else cand.clr(slot[v]);
  };
  // watch[v]: clean vertices whose max_ind is v (entries may be stale; checked
  // on use).  Invariant: every clean k with arg[k] = v >= 0 is in watch[v].
  std::vector<std::vector<int>> watch(n);
  auto consume = [&](int v) {
    for (int k : watch[v])
      if (arg[k] == v) mark(k);
    std::vector<int>().swap(watch[v]);
  };
  // v became busy: a clean watcher k whose only candidate was v (no runner-up)
  // now has none -- exactly what its rescan would find -- and gets v back at
  // the end of the round if v survives; the others rescan.
  std::vector<std::pair<int, int>> lost, pending, demoted;
  // pass >= 2 scans skip busy neighbours; up to kSkip of them are remembered so
  // the vertex can take them back at the end of the round without a rescan
  // (skipn = number skipped; > kSkip: rescan)
  constexpr int kSkip = 8;
  std::vector<int> skipv((size_t)n * kSkip, -1), skipn(n, 0);
  std::vector<char> late_scan(n, 0);
  long long ustat = 0;
  auto consume_busy = [&](int v) {
    for (int k : watch[v]) {
      if (arg[k] != v || dirty[k]) continue;
      if (second_idx[k] == -1) {
        best[k] = -inf;
        arg[k] = -1;
        set_cand(k);
        lost.emplace_back(k, v);
      } else if (second_idx[k] >= 0) {
        pending.emplace_back(k, v);  // demoted to its runner-up after this resolve
      } else {
        ++ustat;
        mark(k);
      }
    }
    std::vector<int>().swap(watch[v]);
  };
  auto eta_of = [&](int k, int j, double& eta) {
    const double* w = adj[k].find(j);
    if (!w) return false;
    eta = 2 * (*w / T - alpha[k] * alpha[j]);
    return true;
  };
  // After a resolve: a clean k whose max v became busy.  The reference rescans
  // k in the next pass and finds the best non-busy neighbour.  If k's recorded
  // runner-up s is not busy and its eta is unchanged, s is that neighbour: every
  // other candidate was <= it at k's last scan and etas only fell since.  The
  // runner-up behind s is then unknown.  (k, v) is remembered so that v, free
  // again at the end of the round, can be compared back in without a rescan.
  long long pstat[5] = {0, 0, 0, 0, 0};
  auto apply_pending = [&]() {
    for (const auto& kv : pending) {
      const int k = kv.first, v = kv.second;
      if (dirty[k] || dead[k] || arg[k] != v) continue;
      if (late_scan[k]) {  // its skip record would not cover v: rescan
        mark(k);
        continue;
      }
      const int sidx = second_idx[k];
      double eta;
      if (prof) {
        if (sidx < 0) ++pstat[0];
        else if (busy[sidx]) ++pstat[1];
        else if (dead[sidx]) ++pstat[2];
        else if (!eta_of(k, sidx, eta) || eta != second[k]) ++pstat[3];
        else ++pstat[4];
      }
      if (sidx >= 0 && !busy[sidx] && !dead[sidx] && eta_of(k, sidx, eta) && eta == second[k]) {
        best[k] = eta;
        arg[k] = sidx;
        second_idx[k] = kUnknown;
        set_cand(k);
        watch[sidx].push_back(k);
        demoted.emplace_back(k, v);
      } else {
        mark(k);
      }
    }
    pending.clear();
  };
  // keep's alpha grew: a clean watcher k keeps keep as its max if the new eta
  // still beats the (upper bound of the) runner-up; then only max_eta changes.
  std::vector<int> stay;
  auto reeval = [&](int v) {
    stay.clear();
    for (int k : watch[v]) {
      if (arg[k] != v || dirty[k]) continue;
      if (second_idx[k] == kUnknown) {
        mark(k);
        continue;
      }
      const double* w = adj[k].find(v);
      bool kept = false;
      if (w) {
        const double eta = 2 * (*w / T - alpha[k] * alpha[v]);
        if (second_idx[k] < 0 || eta > second[k] || (eta == second[k] && v < second_idx[k])) {
          best[k] = eta;
          set_cand(k);
          stay.push_back(k);
          kept = true;
        }
      }
      if (!kept) mark(k);
    }
    watch[v].swap(stay);
  };
  // With positive weights every alpha is positive, so a merge only lowers the
  // eta of keep's neighbours towards keep: only vertices whose max_ind is keep
  // (watchers) can change, plus anything scanned while keep was busy.
  bool positive_weights = true;
  for (long long e = 0; e < (long long)I[n]; ++e) positive_weights = positive_weights && Dv[e] > 0;
  auto root = [&](int x) {
    int r = x;
    while (up[r] != r) r = up[r];
    while (up[x] != r) {
      const int nx = up[x];
      up[x] = r;
      x = nx;
    }
    return r;
  };
  auto snap = [&]() {  // :1797-1815 / :1840-1852 and interpolationMatrix :29-65
    std::vector<int> cnt(M + 1, 0), rowof(basis.size());
    for (size_t y = 0; y < basis.size(); ++y) {
      rowof[y] = slot[root(basis[y])];
      cnt[rowof[y] + 1]++;
    }
    for (int r = 0; r < M; ++r) cnt[r + 1] += cnt[r];
    std::vector<int> ix(basis.size());
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (size_t y = 0; y < basis.size(); ++y) ix[fill[rowof[y]]++] = (int)y;
    h->rows.push_back(M);
    h->cols.push_back(N);
    h->indptr.push_back(std::move(cnt));
    h->indices.push_back(std::move(ix));
  };

  double t_scan = 0, t_resolve = 0, t_merge = 0, t_pop = 0, t_cls = 0, t_par = 0;
  double t_snap = 0, t_swap = 0, t_lost = 0;
  long long rescans = 0, slots_scanned = 0, slots_big = 0, live_scanned = 0;
  long long hist_n[21] = {0}, hist_e[21] = {0}, hist_p2 = 0;
  int rounds = 0;
  std::vector<int> todo, keep_dirty, late, late_fix, big, small_todo;
  int M_prev = M;
  do {
    ++rounds;
    std::vector<std::pair<int, int>> merges;
    double dQ = 0.0;
    for (int pass = 0; pass < matching; ++pass) {
      const auto t0 = now();
      // ---- scan (:1703-1726) over the dirty vertices the reference would scan
      todo.clear();
      keep_dirty.clear();
      for (int v : work) {
        if (dead[v]) {
          dirty[v] = 0;
        } else if (busy[v] && best[v] != -inf) {
          keep_dirty.push_back(v);  // not scanned this pass; stays dirty
        } else {
          todo.push_back(v);
          dirty[v] = 0;
        }
      }
      work.swap(keep_dirty);
      const auto tA = now();
      t_cls += secs(t0, tA);
      const int nt = (int)todo.size();
      rescans += nt;
      // top-2 under (eta descending, index ascending): a total order, so any
      // split of a neighbourhood reduces to the same result
      struct Top2 {
        double e1 = -std::numeric_limits<double>::infinity(), e2 = e1;
        int i1 = -1, i2 = -1;
        void offer(double e, int j) {
          if (i1 < 0 || e > e1 || (e == e1 && j < i1)) {
            e2 = e1;
            i2 = i1;
            e1 = e;
            i1 = j;
          } else if (i2 < 0 || e > e2 || (e == e2 && j < i2)) {
            e2 = e;
            i2 = j;
          }
        }
      };
      auto scan_range = [&](int i, int b, int e, Top2& t, int* sk) {
        const double ai = alpha[i];
        adj[i].for_range(b, e, [&](int j, double w) {
          if (busy[j]) {
            if (sk[kSkip] < kSkip) sk[sk[kSkip]] = j;
            ++sk[kSkip];
            return;
          }
          t.offer(2 * (w / T - ai * alpha[j]), j);
        });
      };
      auto store = [&](int i, const Top2& t) {
        best[i] = t.e1;
        arg[i] = t.i1;
        second[i] = t.e2;
        second_idx[i] = t.i2;
      };
      big.clear();
      small_todo.clear();
      for (int x = 0; x < nt; ++x) {
        const int cap = adj[todo[x]].size();
        (cap > 4096 ? big : small_todo).push_back(todo[x]);
        if (prof) {
          int bkt = 0;
          while ((2 << bkt) <= cap && bkt < 20) ++bkt;
          hist_n[bkt] += 1;
          hist_e[bkt] += cap;
          if (late_scan[todo[x]] == 0 && pass > 0) ++hist_p2;
          slots_scanned += cap;
          if (cap > 8192) slots_big += cap;
          live_scanned += adj[todo[x]].size();
        }
      }
      const int nsm = (int)small_todo.size();
#pragma omp parallel for schedule(dynamic, 64)
      for (int x = 0; x < nsm; ++x) {
        Top2 t;
        int sk[kSkip + 1];
        sk[kSkip] = 0;
        const int i = small_todo[x];
        scan_range(i, 0, adj[i].size(), t, sk);
        store(i, t);
        for (int q = 0; q < std::min(sk[kSkip], kSkip); ++q) skipv[(size_t)i * kSkip + q] = sk[q];
        skipn[i] = sk[kSkip];
      }
      for (int i : big) {  // one large neighbourhood split across threads
        const int cap = adj[i].size();
        skipn[i] = 0;
        Top2 acc;
#pragma omp parallel
        {
          Top2 t;
          int sk[kSkip + 1];
          sk[kSkip] = 0;
#pragma omp for schedule(static) nowait
          for (int b = 0; b < cap; b += 1024) scan_range(i, b, std::min(cap, b + 1024), t, sk);
          if (sk[kSkip] > 0) {
#pragma omp atomic
            skipn[i] += kSkip + 1;  // a split scan does not keep the ids: rescan
          }
#pragma omp critical
          {
            if (t.i1 >= 0) acc.offer(t.e1, t.i1);
            if (t.i2 >= 0) acc.offer(t.e2, t.i2);
          }
        }
        store(i, acc);
      }
      const auto tB = now();
      t_par += secs(tA, tB);
      for (int x = 0; x < nt; ++x) {
        const int i = todo[x];
        set_cand(i);
        if (arg[i] >= 0) watch[arg[i]].push_back(i);
        if (pass > 0) {  // scanned while this round's pairs were busy
          late.push_back(i);
          late_scan[i] = 1;
        }
      }
      const auto t1 = now();
      t_scan += secs(t0, t1);
      // ---- greedy resolve in `used` order (:1728-1753)
      const int words = (int)((alive.size() + 63) / 64);
      for (int wi = 0; wi < words; ++wi) {
        uint64_t bits = cand.w[wi];
        while (bits) {
          const int x = wi * 64 + __builtin_ctzll(bits);
          bits &= bits - 1;
          if (x >= (int)alive.size()) break;
          const int i = alive[x];
          if (busy[i]) continue;
          const int j = arg[i];
          if (j == -1 || busy[j] || best[i] < best[j]) continue;
          if (positive && !(best[i] > 0)) continue;
          if (adj[i].size() < adj[j].size())
            merges.emplace_back(j, i);
          else
            merges.emplace_back(i, j);
          busy[i] = busy[j] = 1;
          mcur = 1;
          if (positive_weights) {  // only vertices whose max_ind is i or j lose their max
            consume_busy(i);
            consume_busy(j);
          } else {
            mark_nbrs(i);
            mark_nbrs(j);
          }
          dQ += best[i];
        }
      }
      apply_pending();
      t_resolve += secs(t1, now());
    }
    // ---- contraction (:1756-1779)
    const auto t2 = now();
    for (const auto& mg : merges) {
      const int keep = mg.first, gone = mg.second;
      mcur = 2;
      adj[gone].for_each([&](int k, double w) {
        adj[k].erase(gone);
        best[k] = -inf;
        cand.clr(slot[k]);
        mark(k);
        if (k == keep) {
          alpha[keep] = alpha[keep] + alpha[gone];
        } else {
          adj[keep].add(k, w);
          adj[k].add(keep, w);
        }
      });
      adj[gone].clear();
      mark(keep);
      mcur = 3;
      if (positive_weights) {
        reeval(keep);  // eta towards keep fell for everyone; only its watchers can change
        consume(gone);
      } else {
        mark_nbrs(keep);
      }
    }
    // vertices scanned in passes >= 2 excluded this round's busy pairs; the
    // surviving ones become available again now
    mcur = 4;
    for (int v : late) {
      late_scan[v] = 0;
      if (skipn[v] > kSkip) mark(v);
      else if (!dirty[v] && !dead[v]) late_fix.push_back(v);
    }
    late.clear();
    Q += dQ;
    M_prev = M;
    const auto t3 = now();
    t_merge += secs(t2, t3);
    if (1.0 * M / N <= cf) {
      snap();
      basis = alive;
      N = M;
    }
    const auto t4 = now();
    t_snap += secs(t3, t4);
    // ---- swap-pop + union (:1819-1834); the candidate bit moves with its vertex
    for (const auto& mg : merges) {
      const int keep = mg.first, gone = mg.second;
      const int s = slot[gone];
      const int L = (int)alive.size() - 1;
      const int last = alive[L];
      const bool bit_last = cand.get(L);
      std::swap(alive[s], alive[L]);
      alive.pop_back();
      slot[last] = s;
      if (bit_last) cand.set(s);
      else cand.clr(s);
      cand.clr(L);
      dead[gone] = 1;
      up[gone] = keep;
      busy[keep] = 0;
      M -= 1;
    }
    const auto t5 = now();
    t_swap += secs(t4, t5);
    // single-candidate vertices that lost their partner to busy get it back
    // (it was scanned in pass 1, when nothing was busy, so v is its only
    // neighbour; any change to its adjacency would have marked it dirty)
    for (const auto& kv : lost) {
      const int k = kv.first, v = kv.second;
      if (dirty[k] || dead[k] || arg[k] != -1) continue;
      const double* w = dead[v] ? nullptr : adj[k].find(v);
      if (!w) {
        mark(k);
        continue;
      }
      best[k] = 2 * (*w / T - alpha[k] * alpha[v]);
      arg[k] = v;
      set_cand(k);
      watch[v].push_back(k);
    }
    lost.clear();
    const auto t6 = now();
    t_lost += secs(t5, t6);
    // demoted vertices: their old max v is free again (or dead, and then k's
    // adjacency changed and k is dirty).  v comes back if it beats the current
    // max under the scan order; the other candidates are <= the current max.
    for (const auto& kv : demoted) {
      const int k = kv.first, v = kv.second;
      if (dirty[k] || dead[k] || dead[v] || arg[k] < 0 || busy[k]) continue;
      double eta;
      if (!eta_of(k, v, eta)) {
        mark(k);
        continue;
      }
      const int a = arg[k];
      if (eta > best[k] || (eta == best[k] && v < a)) {
        second[k] = best[k];
        second_idx[k] = a;
        best[k] = eta;
        arg[k] = v;
        watch[v].push_back(k);
      } else {
        second_idx[k] = kUnknown;
      }
      set_cand(k);
    }
    demoted.clear();
    // late scans: the skipped (busy) neighbours come back.  The scan's top-2
    // is exact over the others, whose etas did not change (none of them merged
    // this round, and a merge touching the vertex's adjacency made it dirty).
    for (int k : late_fix) {
      if (dirty[k] || dead[k]) continue;
      bool redo = false;
      for (int q = 0; q < skipn[k] && !redo; ++q) {
        const int u = skipv[(size_t)k * kSkip + q];
        double eta;
        if (dead[u] || !eta_of(k, u, eta)) {
          redo = true;
          break;
        }
        if (arg[k] < 0 || eta > best[k] || (eta == best[k] && u < arg[k])) {
          second[k] = best[k];
          second_idx[k] = arg[k];
          best[k] = eta;
          arg[k] = u;
        } else if (second_idx[k] < 0 || eta > second[k] || (eta == second[k] && u < second_idx[k])) {
          second[k] = eta;
          second_idx[k] = u;
        }
      }
      if (redo) {
        mark(k);
        continue;
      }
      set_cand(k);
      if (arg[k] >= 0) watch[arg[k]].push_back(k);
    }
    late_fix.clear();
    t_pop += secs(t3, now());
    if (prof && std::getenv("GE_PROFILE_ROUNDS"))
      std::fprintf(stderr, "round %d alive %d merges %zu rescans_total %lld\n", rounds, M,
                   merges.size(), rescans);
  } while (1.0 * M / M_prev < stall);
  snap();
  if (prof)
    std::fprintf(stderr,
                 "partition: n=%d %d rounds %.3fs: scan %.3fs (%lld rescans) resolve %.3fs "
                 "merge %.3fs snap+pop %.3fs\n",
                 n, rounds, secs(t_start, now()), t_scan, rescans, t_resolve, t_merge, t_pop);
  if (prof)
    std::fprintf(stderr, "scan split: classify %.3fs parallel %.3fs; slots %lld (big maps %lld), live entries %lld\n",
                 t_cls, t_par, slots_scanned, slots_big, live_scanned);
  if (prof) {
    std::fprintf(stderr, "rescans by size 2^b: ");
    for (int b = 0; b < 21; ++b)
      if (hist_n[b]) std::fprintf(stderr, "[%d] %lld/%lld  ", b, hist_n[b], hist_e[b]);
    std::fprintf(stderr, " pass2 %lld\n", hist_p2);
  }
  if (prof)
    std::fprintf(stderr, "snap+pop split: snap %.3fs swap-pop %.3fs lost %.3fs demoted %.3fs\n",
                 t_snap, t_swap, t_lost, t_pop - t_snap - t_swap - t_lost);
  if (prof)
    std::fprintf(stderr, "demotions: no-runner-up %lld runner-up busy %lld dead %lld changed %lld ok %lld; unknown->mark %lld\n",
                 pstat[0], pstat[1], pstat[2], pstat[3], pstat[4], ustat);
  if (prof)
    std::fprintf(stderr, "marks: init %lld resolve %lld gone-nbrs %lld keep %lld late %lld\n",
                 msrc[0], msrc[1], msrc[2], msrc[3], msrc[4]);
  if (printing) {  // :1880-1889
    std::cout << "modularity: " << Q << std::endl;
    std::cout << "level 0: " << n << " aggregates" << std::endl;
    for (size_t l = 0; l < h->rows.size(); ++l)
      std::cout << "level " << l + 1 << ": " << h->rows[l] << " aggregates" << std::endl;
  }
  return h;
}

}  // namespace ge
