/*
 * ge_oracle.h -- CPU restatement of LLNL/graph-embed's hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle.so, and only as the checker /
 * the timed CPU baseline -- never as the product path.
 *
 * PARITY UNPINNED against the reference itself: the reference cannot be built
 * here (its only dependency, linalgcpp, is not vendored and not installed, and
 * the rules forbid a stand-in header), and it ships no tests, fixtures or golden
 * vectors.  This file is an independent restatement of the
 * reference algorithm, written from the reference source read as text, with each
 * function citing the reference lines it follows.  It is cross-checked bit-for-bit
 * against a second, independent pure-Python restatement (tests/pyref.py) on small
 * cases.
 *
 * Conventions (all pinned here; the reference leaves them to random_device /
 * the absent linalgcpp):
 *   - Every RNG is std::mt19937(seed) feeding
 *     std::uniform_real_distribution<double>(-1, 1) (libstdc++), consumed in the
 *     reference's single-thread draw order.
 *   - CSR inputs: int32 indptr/indices, double data, rows in caller order.
 *   - P^T A P output rows have ascending column indices.
 *
 * Arrays are flat and row-major: coordinates are n*dim doubles (vertex-major).
 */
#ifndef GE_ORACLE_H
#define GE_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_fa_params {
  double ks, ksmax, repel, attract, gravity, delta, tolerate;
  int use_weights, linlog, nohubs, normalize;
} orc_fa_params;

/* Defaults of include/forceatlas.hpp:89-103. */
void orc_fa_params_default(orc_fa_params* p);

/* First `count` values of uniform_real_distribution<double>(-1,1) over
 * mt19937(seed). */
void orc_uniform_stream(unsigned seed, long long count, double* out);

/* forceAtlas (include/forceatlas.hpp:89-305).  If init_random != 0, coords are
 * (re)initialised from mt19937(seed) exactly as :118-125; otherwise the given
 * coords are used.  nthreads <= 0 -> OpenMP default. */
int orc_force_atlas(int n, const int* indptr, const int* indices, const double* data,
                    int dim, double* coords, int init_random, unsigned seed,
                    int iterations, const orc_fa_params* p, int nthreads);

/* One forceAtlas iteration restricted to rows [row_begin,row_end): writes the
 * force rows (forces[i][k] at include/forceatlas.hpp:210) for those rows only.
 * deg must be precomputed (orc_degrees).  Used for the bounded CPU baseline. */
int orc_fa_forces_rows(int n, const int* indptr, const int* indices, const double* data,
                       int dim, const double* coords, const double* deg,
                       int row_begin, int row_end, const orc_fa_params* p,
                       double* forces_out, int nthreads);

/* One forceAtlas iteration for rows [row_begin,row_end) only (the loop body
 * of include/forceatlas.hpp:146-269 restricted to a row shard): reads all of
 * coords, updates fprev_rows ((row_end-row_begin)*dim, in/out) and writes rows
 * [row_begin,row_end) of coords_next. */
int orc_fa_step_rows(int n, const int* indptr, const int* indices, const double* data, int dim,
                     const double* coords, const double* deg, int row_begin, int row_end,
                     const orc_fa_params* p, double* fprev_rows, double* coords_next,
                     int nthreads);

/* deg[i] of include/forceatlas.hpp:127-140. */
void orc_degrees(int n, const int* indptr, const double* data, int use_weights, double* deg);

/* forceAtlasMultilevel (include/forceatlas.hpp:314-574), single-thread draw
 * order.  m = rows of P_T. */
int orc_force_atlas_ml(int n, const int* indptr, const int* indices, const double* data,
                       int m, const int* pt_indptr, const int* pt_indices,
                       const int* vertex_A, const double* coords_A, const double* r_A,
                       double* coords, int dim, int iterations, unsigned seed,
                       const orc_fa_params* p, int nthreads);

/* ---- partition hierarchy (src/partitioner.cpp:1550-1893) ---- */
typedef struct orc_hier orc_hier;
orc_hier* orc_partition(int n, const int* indptr, const int* indices, const double* data,
                        double coarsening_factor, int positive_merging,
                        double stall_stop_threshold, int matching_iterations);
/* the same loop over unordered entry lists (ge_oracle.cpp: identical results, faster) */
orc_hier* orc_partition_flat(int n, const int* indptr, const int* indices, const double* data,
                        double coarsening_factor, int positive_merging,
                        double stall_stop_threshold, int matching_iterations);
int orc_hier_levels(const orc_hier* h);
/* rows/cols of P_T[l]; indptr has rows+1 entries, indices has cols entries */
void orc_hier_shape(const orc_hier* h, int l, int* rows, int* cols);
void orc_hier_copy(const orc_hier* h, int l, int* indptr, int* indices);
void orc_hier_free(orc_hier* h);

/* modularity (src/partitioner.cpp:69-114) */
double orc_modularity(int n, const int* indptr, const int* indices, const double* data,
                      int m, const int* vertex_A);

/* ---- P^T A P (examples/embed.cpp:96-98) ---- */
typedef struct orc_csr orc_csr;
orc_csr* orc_ptap(int n, const int* indptr, const int* indices, const double* data,
                  int m, const int* pt_indptr, const int* pt_indices);
void orc_csr_shape(const orc_csr* c, int* rows, int* nnz);
void orc_csr_copy(const orc_csr* c, int* indptr, int* indices, double* data);
void orc_csr_free(orc_csr* c);

/* ---- embed (src/embed.cpp:561-796) ----
 * levels = number of P_T matrices (As has levels+1 entries).  a_* arrays are
 * concatenations of As[0..levels] CSR blocks; p_* of P_Ts[0..levels-1].
 * a_off[l] = start of level l in a_indptr (each level has n_l+1 entries),
 * a_nz_off[l] = start of level l in a_indices/a_data; similarly p_off, p_nz_off.
 * base_iterations is the coarsest forceAtlas iteration count (reference: 100000);
 * ml_iterations the per-level multilevel count (reference: 100). */
int orc_embed(int levels, const int* a_n, const int* a_off, const int* a_nz_off,
              const int* a_indptr, const int* a_indices, const double* a_data,
              const int* p_rows, const int* p_off, const int* p_nz_off,
              const int* p_indptr, const int* p_indices,
              int dim, unsigned seed, int base_iterations, int ml_iterations,
              double* coords_out, int nthreads);

/* Radius ("kinetic ball") step of src/embed.cpp:615-777 for one level.
 * coarse_is_base != 0 selects the base-case branch (:616-679); then r_Ac,
 * coords_Ac, P_Ts[l+1] are unused.  coords_A (m*dim) is updated in place in the
 * non-base branch (:757-777).  r_A (m) is written. */
int orc_radius_step(int m, double* coords_A, double* r_A, int dim, int coarse_is_base,
                    int mc, const int* ptc_indptr, const int* ptc_indices,
                    const double* coords_Ac, const double* r_Ac,
                    const int* ac_indptr, const int* ac_indices);

/* embedViaMinimization (src/embed.cpp:341-559): coords n*dim in/out; init_random
 * != 0 draws U(-1,1) from mt19937(seed) first (the empty-coords branch, :353-361). */
int orc_embed_via_minimization(int n, const int* indptr, const int* indices, int dim,
                               double* coords, int init_random, unsigned seed, int iterations);

/* embedVia(As, P_Ts, d, anyToMultilevel(minimizer)) (src/embed.cpp:23-106,
 * :108-338) with minimizer(A, d) = embedViaMinimization(A, d) (:341-345: r x d
 * zeros, min_iterations sweeps; the reference uses 1000): the levels >= 1 are
 * embedMultilevel (forceAtlas, radius steps, forceAtlasMultilevel), level 0 is
 * the radius step then the per-aggregate minimizer.  levels >= 1. */
int orc_embed_via_minimization_ml(int levels, const int* a_n, const int* a_off,
                                  const int* a_nz_off, const int* a_indptr, const int* a_indices,
                                  const double* a_data, const int* p_rows, const int* p_off,
                                  const int* p_nz_off, const int* p_indptr, const int* p_indices,
                                  int dim, unsigned seed, int base_iterations, int ml_iterations,
                                  int min_iterations, double* coords_out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
