// Drop-in for include/embed.hpp (LLNL/graph-embed).
//   embed(As, ps, d)                                     src/embed.cpp:561-574
//   embedMultilevel(As, ps, d, index, r_A, coords_A)     src/embed.cpp:576-796
// embed() is one libge call (ge_embed); embedMultilevel() composes the same
// steps from the C ABI (forceAtlas on the coarsest level, radius step,
// forceAtlasMultilevel per level) so its r_A / coords_A out-parameters are
// available.  Both print the reference's "embedding layer" lines.
// The alternative embedders (embedViaMinimization, anyToMultilevel, embedVia,
// embedViaMultilevel, src/embed.cpp:23-559) are implemented at the end.
#ifndef EMBED_HPP
#define EMBED_HPP

#include <algorithm>
#include <functional>
#include <iostream>
#include <vector>

#include "forceatlas.hpp"
#include "partitioner.hpp"

namespace partition {

using MultilevelEmbedder =
    std::function<void(const SparseMatrix&, const SparseMatrix&, const std::vector<int>&,
                       const std::vector<std::vector<double>>&, const std::vector<double>&,
                       std::vector<std::vector<double>>&, const int)>;

inline std::vector<std::vector<double>> embed(const std::vector<SparseMatrix>& As,
                                              const std::vector<SparseMatrix>& ps, const int d) {
  const int levels = (int)ps.size();
  if ((int)As.size() != levels + 1)
    throw std::invalid_argument("embed: As.size() must equal P_Ts.size() + 1 (src/embed.cpp:564)");
  std::vector<int> a_n, a_off, a_nz, a_ip, a_ix, p_rows, p_off, p_nz, p_ip, p_ix;
  std::vector<double> a_dx;
  for (const auto& A : As) {
    a_n.push_back(A.Rows());
    a_off.push_back((int)a_ip.size());
    a_nz.push_back((int)a_ix.size());
    a_ip.insert(a_ip.end(), A.GetIndptr().begin(), A.GetIndptr().end());
    a_ix.insert(a_ix.end(), A.GetIndices().begin(), A.GetIndices().end());
    a_dx.insert(a_dx.end(), A.GetData().begin(), A.GetData().end());
  }
  for (const auto& P : ps) {
    p_rows.push_back(P.Rows());
    p_off.push_back((int)p_ip.size());
    p_nz.push_back((int)p_ix.size());
    p_ip.insert(p_ip.end(), P.GetIndptr().begin(), P.GetIndptr().end());
    p_ix.insert(p_ix.end(), P.GetIndices().begin(), P.GetIndices().end());
  }
  p_rows.push_back(0);
  p_off.push_back((int)p_ip.size());
  p_nz.push_back((int)p_ix.size());
  p_ip.push_back(0);
  p_ix.push_back(0);
  ge_fa_params p;
  ge_fa_params_default(&p);
  p.seed = detail::seed_ref();
  std::vector<double> X((size_t)As[0].Rows() * d);
  detail::check(ge_embed(detail::context(), levels, a_n.data(), a_off.data(), a_nz.data(),
                         a_ip.data(), a_ix.data(), a_dx.data(), p_rows.data(), p_off.data(),
                         p_nz.data(), p_ip.data(), p_ix.data(), d, 100000, 100, 1, &p, X.data()));
  std::vector<std::vector<double>> coords;
  detail::unflatten(X, As[0].Rows(), d, coords);
  return coords;
}

namespace detail {

// The radius step between level index+1 and level index (src/embed.cpp:615-777)
// on the device (ge_radius_step_device): coords_A (level index+1) is rescaled in
// place, r_A receives its radii.
inline void radius_step(const std::vector<SparseMatrix>& As, const std::vector<SparseMatrix>& ps,
                        int index, int d, const std::vector<double>& r_Ac,
                        const std::vector<std::vector<double>>& coords_Ac,
                        std::vector<std::vector<double>>& coords_A, std::vector<double>& r_A) {
  const SparseMatrix& A_c = As[index + 1];
  const int m = (int)coords_A.size();
  std::vector<double> cA = flatten(coords_A, m, d);
  r_A.assign(m, 0.0);
  const bool base = r_Ac.empty();
  std::vector<double> cAc;
  if (!base) cAc = flatten(coords_Ac, (int)coords_Ac.size(), d);
  const SparseMatrix* P_Tc = base ? nullptr : &ps[index + 1];
  check(ge_radius_step_device(context(), m, cA.data(), r_A.data(), d, base ? 1 : 0,
                              base ? 0 : P_Tc->Rows(), base ? nullptr : P_Tc->GetIndptr().data(),
                              base ? nullptr : P_Tc->GetIndices().data(),
                              base ? nullptr : cAc.data(), base ? nullptr : r_Ac.data(),
                              A_c.GetIndptr().data(), A_c.GetIndices().data(), nullptr));
  unflatten(cA, m, d, coords_A);
}

}  // namespace detail

inline std::vector<std::vector<double>> embedMultilevel(const std::vector<SparseMatrix>& As,
                                                        const std::vector<SparseMatrix>& ps,
                                                        const int d, const int index,
                                                        std::vector<double>& r_A,
                                                        std::vector<std::vector<double>>& coords_A) {
  if (index == (int)ps.size()) {  // :582-587
    std::cout << "embedding layer " << index + 1 << ": getting base coords" << std::endl;
    r_A.clear();
    coords_A.clear();
    return forceAtlas(As[index], d);
  }
  std::vector<double> r_Ac;
  std::vector<std::vector<double>> coords_Ac;
  coords_A = embedMultilevel(As, ps, d, index + 1, r_Ac, coords_Ac);  // :593
  std::cout << "embeding layer " << index + 1 << std::endl;           // sic (:613)
  detail::radius_step(As, ps, index, d, r_Ac, coords_Ac, coords_A, r_A);
  const SparseMatrix& P_T = ps[index];
  const std::vector<int> vertex_A = detail::vertex_of(P_T);
  std::vector<std::vector<double>> coords(As[index].Rows(), std::vector<double>(d));
  forceAtlasMultilevel(As[index], P_T, vertex_A, coords_A, r_A, coords, d, 100);  // :793
  return coords;
}

// ---------------------------------------------------------------------------
// Alternative embedders (src/embed.cpp:23-559).  embedViaMinimization runs in
// libge (ge_embed_via_minimization, host: its line searches are serial sums);
// anyToMultilevel and embedVia compose it (or any user embedder) with the
// device hierarchy steps above, as the reference composes them.

inline void embedViaMinimization(const SparseMatrix& A, const int d,
                                 std::vector<std::vector<double>>& coords, const int ITER = 10) {
  const int n = A.Rows();
  const bool init = coords.empty();  // :353-361
  std::vector<double> X = init ? std::vector<double>((size_t)n * d) : detail::flatten(coords, n, d);
  detail::check(ge_embed_via_minimization(n, A.GetIndptr().data(), A.GetIndices().data(), d,
                                          X.data(), init ? 1 : 0, detail::seed_ref(), ITER));
  detail::unflatten(X, n, d, coords);
}

inline std::vector<std::vector<double>> embedViaMinimization(const SparseMatrix& A, const int d) {
  std::vector<std::vector<double>> coords(A.Rows(), std::vector<double>(d, 0.0));  // :341-345
  embedViaMinimization(A, d, coords, 1000);
  return coords;
}

// :23-83.  Per aggregate a: the members' internal edges as an r x r matrix of
// counts (the reference adds 1.0 per stored entry and sums duplicates in
// ToSparse), the single-level embedder on it, the result normalised by its
// largest norm and placed in a's ball.
inline MultilevelEmbedder anyToMultilevel(
    std::function<std::vector<std::vector<double>>(const SparseMatrix&, const int)> embedder) {
  return [embedder](const SparseMatrix& A, const SparseMatrix& P_T, const std::vector<int>& v_A,
                    const std::vector<std::vector<double>>& coords_A,
                    const std::vector<double>& r_A, std::vector<std::vector<double>>& coords,
                    const int d) {
    const std::vector<int>& I = A.GetIndptr();
    const std::vector<int>& J = A.GetIndices();
    const std::vector<int>& PI = P_T.GetIndptr();
    const std::vector<int>& PJ = P_T.GetIndices();
    for (int a = 0; a < P_T.Rows(); ++a) {
      const std::vector<int> v(PJ.begin() + PI[a], PJ.begin() + PI[a + 1]);
      const int r = (int)v.size();
      std::vector<std::vector<int>> cols(r);
      for (int i = 0; i < r; ++i)
        for (int k2 = I[v[i]]; k2 < I[v[i] + 1]; ++k2) {
          const int j = J[k2];
          if (v_A[j] != a) continue;
          int jp = -1;  // last match, as the reference's scan
          for (int j2 = 0; j2 < r; ++j2)
            if (v[j2] == j) jp = j2;
          cols[i].push_back(jp);
        }
      std::vector<int> ci(r + 1, 0), cj;
      std::vector<double> cd;
      for (int i = 0; i < r; ++i) {
        std::sort(cols[i].begin(), cols[i].end());
        for (size_t q = 0; q < cols[i].size(); ++q) {
          if (q > 0 && cols[i][q] == cols[i][q - 1]) {
            cd.back() += 1.0;
          } else {
            cj.push_back(cols[i][q]);
            cd.push_back(1.0);
          }
        }
        ci[i + 1] = (int)cj.size();
      }
      const std::vector<std::vector<double>> nc = embedder(SparseMatrix(ci, cj, cd, r, r), d);
      double mx = 0.0;
      for (int i = 0; i < r; ++i) {
        const double mg = magnitude(nc[i]);
        if (mg > mx) mx = mg;
      }
      for (int i = 0; i < r; ++i)
        for (int k = 0; k < d; ++k) coords[v[i]][k] = coords_A[a][k] + r_A[a] * (nc[i][k] / mx);
    }
  };
}

// :108-338.  The coarser levels are embedMultilevel (the reference recurses into
// it, not into itself); the finest level runs the radius step, then `embedder`.
inline std::vector<std::vector<double>> embedViaMultilevel(
    const std::vector<SparseMatrix>& As, const std::vector<SparseMatrix>& ps, const int d,
    const int index, std::vector<double>& r_A, std::vector<std::vector<double>>& coords_A,
    MultilevelEmbedder embedder) {
  if (index == (int)ps.size()) {  // :121-139: a 1-row P_T over the whole graph (sic)
    std::cout << "embedding layer " << index + 1 << ": getting base coords" << std::endl;
    r_A.clear();
    coords_A.clear();
    const int n = As[index].Rows();
    std::vector<int> I(n + 1), J(n, 0);
    for (int i = 0; i <= n; ++i) I[i] = i;
    const SparseMatrix P_T(I, J, std::vector<double>(n, 1.0), 1, n);
    // the reference leaves the rows empty (writes through them are undefined);
    // here they hold d zeros
    std::vector<std::vector<double>> coords(n, std::vector<double>(d, 0.0));
    const std::vector<std::vector<double>> origin = {std::vector<double>(d, 0.0)};
    embedder(As[index], P_T, std::vector<int>(n, 0), origin, std::vector<double>{1.0}, coords, d);
    return coords;
  }
  std::vector<double> r_Ac;
  std::vector<std::vector<double>> coords_Ac;
  coords_A = embedMultilevel(As, ps, d, index + 1, r_Ac, coords_Ac);  // :143
  std::cout << "embeding layer " << index + 1 << std::endl;
  detail::radius_step(As, ps, index, d, r_Ac, coords_Ac, coords_A, r_A);
  const SparseMatrix& P_T = ps[index];
  std::vector<std::vector<double>> coords(As[index].Rows(), std::vector<double>(d));
  embedder(As[index], P_T, detail::vertex_of(P_T), coords_A, r_A, coords, d);  // :336
  return coords;
}

inline std::vector<std::vector<double>> embedVia(const std::vector<SparseMatrix>& As,
                                                 const std::vector<SparseMatrix>& ps, const int d,
                                                 MultilevelEmbedder embedder) {
  if (As.size() != ps.size() + 1)  // :95-103
    throw std::invalid_argument("embedVia: As.size() must equal P_Ts.size() + 1");
  for (size_t i = 0; i < ps.size(); ++i)
    if (As[i].Rows() != ps[i].Cols() || As[i + 1].Rows() != ps[i].Rows())
      throw std::invalid_argument("embedVia: level shapes do not chain");
  std::vector<double> none;
  std::vector<std::vector<double>> none2;
  return embedViaMultilevel(As, ps, d, 0, none, none2, embedder);
}

}  // namespace partition

#endif  // EMBED_HPP
