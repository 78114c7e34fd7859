/*
 * ge.h -- C ABI of libge.so, the MI355X-native (gfx950) implementation of
 * graph-embed's hot path: multilevel modularity coarsening + ForceAtlas.
 *
 * Plain C: pointers and sizes only, no C++ or torch types.  Every function
 * returns 0 on success or a non-zero GE_ERR_* / HIP error code; the text of the
 * last error on the calling thread is ge_last_error().  (The reference reports
 * errors only through assert; the drop-in headers in graph-embed_amd/include turn a non-zero
 * status into std::runtime_error.)
 *
 * Memory: functions named *_plan_* and ge_fa_plan_step take DEVICE pointers
 * (data resident in HBM); every other entry point takes HOST pointers and moves
 * the data itself.  All device work is enqueued on the context's stream.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to LLNL/graph-embed).
 */
#ifndef GE_H
#define GE_H

#ifdef __cplusplus
extern "C" {
#endif

#define GE_OK 0
#define GE_ERR_ARG 1001     /* invalid argument / shape mismatch */
#define GE_ERR_HIP 1002     /* a HIP runtime call failed */
#define GE_ERR_STATE 1003   /* object used in the wrong state */
#define GE_ERR_NOMEM 1004   /* host allocation failed */
#define GE_ERR_CAPACITY 1005 /* a device-side capacity limit (e.g. the partition's list pool) */

#define GE_MODE_STRICT 0 /* bit-exact with the reference's serial op order */
#define GE_MODE_FAST 1   /* re-associated / FMA / rsqrt; 1e-5 relative bar */

typedef struct ge_ctx ge_ctx;
typedef struct ge_hier ge_hier;
typedef struct ge_csr ge_csr;
typedef struct ge_fa_plan ge_fa_plan;

/* ForceAtlas parameters.  Defaults (ge_fa_params_default) are those of
 * forceAtlas / forceAtlasMultilevel, include/forceatlas.hpp:89-103, :320-331. */
typedef struct ge_fa_params {
  double ks, ksmax, repel, attract, gravity, delta, tolerate;
  int use_weights, linlog, nohubs, normalize;
  unsigned seed; /* mt19937 seed replacing std::random_device (:104-105, :332-333) */
  int mode;      /* GE_MODE_STRICT (default) or GE_MODE_FAST */
} ge_fa_params;

void ge_fa_params_default(ge_fa_params* p);
const char* ge_last_error(void);
const char* ge_version(void);

/* ---- context: one device + one stream; reentrant, no global mutable state ---- */
int ge_device_count(int* count);
int ge_ctx_create(int device, ge_ctx** out);
int ge_ctx_destroy(ge_ctx* ctx);
/* Enqueue on an external hipStream_t (e.g. torch's current stream); NULL
 * restores the context's own stream. */
int ge_ctx_set_stream(ge_ctx* ctx, void* hip_stream);
int ge_ctx_sync(ge_ctx* ctx);

/* ---- single-level ForceAtlas ----
 * Replaces partition::forceAtlas(A, dim, coords, iterations, ks, ksmax, repel,
 * attract, gravity, useWeights, linlog, nohubs, delta, tolerate, normalize)
 * (include/forceatlas.hpp:89-305) and, with init_random = 1 and
 * iterations = 100000, partition::forceAtlas(A, dim) (:307-312).
 * coords: n*dim row-major, in/out.  init_random != 0 draws U(-1,1) from
 * mt19937(p->seed) in the reference order (:118-125). */
int ge_force_atlas(ge_ctx* ctx, int n, const int* indptr, const int* indices,
                   const double* data, int dim, double* coords, int init_random,
                   int iterations, const ge_fa_params* p);

/* Device-resident ForceAtlas iteration over rows [row_begin, row_end) -- the
 * loop body of include/forceatlas.hpp:146-270 -- for row-sharded multi-GPU use.
 * The plan keeps d_indptr/d_indices/d_data by pointer (caller owns them). */
int ge_fa_plan_create(ge_ctx* ctx, int n, int nnz, const int* d_indptr,
                      const int* d_indices, const double* d_data, int dim,
                      const ge_fa_params* p, int row_begin, int row_end,
                      ge_fa_plan** out);
/* d_x_cur: all n*dim coordinates of this iteration; writes rows
 * [row_begin,row_end) of d_x_next (must not alias d_x_cur). */
int ge_fa_plan_step(ge_fa_plan* plan, const double* d_x_cur, double* d_x_next);
/* The second half of the iteration alone -- attraction in CSR order, gravity,
 * swing and update (include/forceatlas.hpp:169-269) -- with the repulsion sums
 * supplied by the caller (d_frep: (row_end - row_begin)*dim, the value each
 * row's force holds after :151-167).  For measuring the attraction pass at
 * sizes whose all-pairs repulsion is out of reach (configs[4]).  Always runs
 * the CSR row kernels (tiles / heavy segments), also for small levels. */
int ge_fa_plan_attract(ge_fa_plan* plan, const double* d_x_cur, const double* d_frep,
                       double* d_x_next);
/* Kernel timing with HIP events on the plan's stream (0 = off). */
int ge_fa_plan_set_profiling(ge_fa_plan* plan, int enable);
/* Average device ms per launch of the repulsion and attraction/update kernels
 * since profiling was enabled; *launches = steps timed. Synchronises. */
int ge_fa_plan_kernel_ms(ge_fa_plan* plan, double* repulsion_ms, double* attraction_ms,
                         int* launches);
int ge_fa_plan_destroy(ge_fa_plan* plan);

/* ---- multilevel ForceAtlas ----
 * Replaces partition::forceAtlasMultilevel(A, P, v_A, coords_A, r_A, coords,
 * dim, iterations, ks, ksmax, useWeights, linlog, nohubs, repel, attract,
 * gravity, delta, tolerate) (include/forceatlas.hpp:314-574), in the reference's
 * single-thread random draw order.  m = P_T rows; coords: n*dim out. */
int ge_force_atlas_ml(ge_ctx* ctx, int n, const int* indptr, const int* indices,
                      const double* data, int m, const int* pt_indptr,
                      const int* pt_indices, const int* vertex_A, const double* coords_A,
                      const double* r_A, double* coords, int dim, int iterations,
                      const ge_fa_params* p);

/* Device-resident multilevel level (the bench and multi-GPU path).  Aggregates
 * [agg_begin, agg_end) of P_T are processed; h_pt_indptr is a HOST copy of
 * P_T's indptr (used to bucket aggregates by size), every other array is on the
 * device.  Run: d_init = the n*dim draws in P_T storage order (ge_uniform_stream),
 * d_coords receives the members' coordinates (fine-vertex order). */
typedef struct ge_faml_plan ge_faml_plan;
int ge_faml_plan_create(ge_ctx* ctx, int n, const int* d_indptr, const int* d_indices,
                        const double* d_data, int m, const int* h_pt_indptr,
                        const int* d_pt_indptr, const int* d_pt_indices, const int* d_vertex_A,
                        int dim, const ge_fa_params* p, int iterations, int agg_begin,
                        int agg_end, ge_faml_plan** out);
/* The same for an arbitrary set of aggregates (h_aggs: n_aggs strictly increasing
 * ids) -- one rank's share when aggregates are dealt to GPUs by cost
 * (ge_amd.dist.assign_aggregates). */
int ge_faml_plan_create_subset(ge_ctx* ctx, int n, const int* d_indptr, const int* d_indices,
                               const double* d_data, int m, const int* h_pt_indptr,
                               const int* d_pt_indptr, const int* d_pt_indices,
                               const int* d_vertex_A, int dim, const ge_fa_params* p,
                               int iterations, const int* h_aggs, int n_aggs,
                               ge_faml_plan** out);
/* One rank's plan when aggregates are also split across GPUs (SURVEY.md 8(e);
 * include/forceatlas.hpp:394-410 is a per-row ordered sum, so rows of one aggregate
 * can live on different ranks): h_aggs are this rank's whole aggregates, h_split the
 * aggregates split by 64-row tiles over all ranks of comm (the same list on every
 * rank; rank r takes tiles [T r / N, T (r + 1) / N)).  The split aggregates' rows are
 * all-gathered over comm after every iteration inside ge_faml_plan_run, and every
 * rank ends with all their members' coordinates.  Every rank must run its plan. */
typedef struct ge_comm ge_comm;
int ge_faml_plan_create_shard(ge_ctx* ctx, ge_comm* comm, int n, const int* d_indptr,
                              const int* d_indices, const double* d_data, int m,
                              const int* h_pt_indptr, const int* d_pt_indptr,
                              const int* d_pt_indices, const int* d_vertex_A, int dim,
                              const ge_fa_params* p, int iterations, const int* h_aggs,
                              int n_aggs, const int* h_split, int n_split, ge_faml_plan** out);
int ge_faml_plan_run(ge_faml_plan* plan, const double* d_coords_A, const double* d_r_A,
                     const double* d_init, double* d_coords);
int ge_faml_plan_set_profiling(ge_faml_plan* plan, int enable);
/* Average device ms of the resident (LDS) kernels and of the streamed path per run. */
int ge_faml_plan_kernel_ms(ge_faml_plan* plan, double* resident_ms, double* streamed_ms,
                           int* runs);
/* Average device ms of one streamed-path repulsion launch (faml_big_repulse, one
 * per iteration) over the profiled runs, and the ordered pairs one launch
 * evaluates (sum of s(s-1) over the streamed aggregates); 0 launches if none. */
int ge_faml_plan_repulse_ms(ge_faml_plan* plan, double* ms_per_launch, int* launches,
                            double* pairs_per_launch);
/* Average device ms of one pass over the streamed members' rows (FamlRows: CSR
 * attraction / external pull, :415-467, gravity and update, :469-530; one per
 * iteration), the passes profiled, and the rows and CSR entries one pass reads. */
int ge_faml_plan_rows_ms(ge_faml_plan* plan, double* ms_per_pass, int* passes,
                         long long* rows, long long* entries);
/* The plan's schedule of the streamed aggregates' repulsion: how many run as
 * plain symmetric sweeps, in bands (pre row blocks / in-band sweeps / post row
 * blocks: a shorter dependency chain), as whole row blocks, and the units of
 * one launch.  Diagnostics; the results do not depend on it. */
int ge_faml_plan_schedule(ge_faml_plan* plan, int* sweeps, int* banded, int* row_blocks,
                          int* units);
int ge_faml_plan_destroy(ge_faml_plan* plan);

/* ---- coarsening hierarchy ----
 * Replaces std::vector<SparseMatrix> partition::partition(A, coarseningFactor,
 * printing, positiveMerging, stallStopThreshold, matchingIterations,
 * mergeLeaves) (include/partitioner.hpp:52-53, src/partitioner.cpp:1550-1893).
 * A must be symmetric.  Level l of the result is P_T[l] (rows x cols, one 1.0
 * per column).  ctx != NULL builds the hierarchy on the context's device
 * (graph-embed_amd/csrc/ge_partition_dev.hip) when A has integer weights and
 * strictly ascending rows; ctx == NULL, other inputs, or GE_PARTITION_HOST=1 take
 * the host path.  Both give the reference's P_T arrays. */
int ge_partition(ge_ctx* ctx, int n, const int* indptr, const int* indices,
                 const double* data, double coarsening_factor, int printing,
                 int positive_merging, double stall_stop_threshold,
                 int matching_iterations, int merge_leaves, ge_hier** out);
int ge_hier_levels(const ge_hier* h, int* levels);
int ge_hier_shape(const ge_hier* h, int level, int* rows, int* cols);
/* indptr: rows+1 ints, indices: cols ints */
int ge_hier_copy(const ge_hier* h, int level, int* indptr, int* indices);
int ge_hier_free(ge_hier* h);

/* Replaces partition::interpolationMatrix(numCols, partition)
 * (src/partitioner.cpp:29-65) in flattened form: sets[offsets[r]..offsets[r+1])
 * are row r's columns. */
int ge_interpolation_matrix(int num_cols, int num_rows, const int* offsets,
                            const int* sets, ge_csr** out);

/* ---- P^T A P on the device ----
 * Replaces P_T.Mult(A).Mult(P_T.Transpose()) (examples/embed.cpp:96-98,
 * examples/embedder.cpp:213-216; linalgcpp).  Output rows sorted ascending. */
int ge_ptap(ge_ctx* ctx, int n, const int* indptr, const int* indices, const double* data,
            int m, const int* pt_indptr, const int* pt_indices, ge_csr** out);
int ge_csr_shape(const ge_csr* c, int* rows, int* cols, long long* nnz);
int ge_csr_copy(const ge_csr* c, int* indptr, int* indices, double* data);
int ge_csr_free(ge_csr* c);

/* ---- modularity (src/partitioner.cpp:69-114) ---- */
int ge_modularity(int n, const int* indptr, const int* indices, const double* data,
                  int m, const int* vertex_A, double* q);
/* The same with the CSR and vertex_A on the device (O(nnz) pass as 64-bit integer
 * sums -- exact, the weights being truncated to int -- then the O(M) final sum on
 * the host in the reference's order).  Same result bits as ge_modularity. */
int ge_modularity_device(ge_ctx* ctx, int n, const int* d_indptr, const int* d_indices,
                         const double* d_data, int m, const int* d_vertex_A, double* q);

/* ---- multilevel embed ----
 * Replaces partition::embed(As, P_Ts, d) (include/embed.hpp:70-72,
 * src/embed.cpp:561-796).  levels = P_Ts.size(); As has levels+1 entries.
 * a_* are the concatenated CSR arrays of As[0..levels], p_* of
 * P_Ts[0..levels-1]; a_n[l] = rows of As[l]; *_off / *_nz_off = start of each
 * level in the indptr / indices arrays.  base_iterations / ml_iterations:
 * reference values 100000 and 100.  print_progress mirrors the reference's
 * "embedding layer" stdout lines (:583, :613). */
int ge_embed(ge_ctx* ctx, int levels, const int* a_n, const int* a_off,
             const int* a_nz_off, const int* a_indptr, const int* a_indices,
             const double* a_data, const int* p_rows, const int* p_off,
             const int* p_nz_off, const int* p_indptr, const int* p_indices, int dim,
             int base_iterations, int ml_iterations, int print_progress,
             const ge_fa_params* p, double* coords_out);

/* Radius ("kinetic ball") step between levels, src/embed.cpp:615-777 (host).
 * m coarse vertices with coords_A (m*dim, updated in place by the rescale of
 * :757-777 unless coarse_is_base) -> r_A (m).  coarse_is_base selects the
 * all-pairs base case (:616-679); otherwise P_T[l+1] (mc rows), coords_Ac /
 * r_Ac of level l+2 and A_c = As[l+1] (ac_indptr/ac_indices) are used. */
int ge_radius_step(int m, double* coords_A, double* r_A, int dim, int coarse_is_base, int mc,
                   const int* ptc_indptr, const int* ptc_indices, const double* coords_Ac,
                   const double* r_Ac, const int* ac_indptr, const int* ac_indices);

/* The same step on the device (graph-embed_amd/csrc/ge_radius.hip): the events
 * pop in parallel rounds with the serial loop's result bits.  When an event
 * distance is 0 (coincident coarse coordinates) the host loop runs instead;
 * *used_device (may be NULL) tells which ran.  embed uses this form. */
int ge_radius_step_device(ge_ctx* ctx, int m, double* coords_A, double* r_A, int dim,
                          int coarse_is_base, int mc, const int* ptc_indptr,
                          const int* ptc_indices, const double* coords_Ac, const double* r_Ac,
                          const int* ac_indptr, const int* ac_indices, int* used_device);

/* ---- multi-GPU: one process per GPU, a communicator per context ----
 * The reference has no multi-GPU path (it is OpenMP on one node); these entry
 * points shard the same computations across ranks and return
 * the same bits on every rank as the single-GPU calls:
 *   - forceAtlas: contiguous row shards + one all-gather of the fp64
 *     coordinates per iteration (include/forceatlas.hpp:146-270 reads all
 *     coordinates of the previous iteration, nothing else is global: :228, :242);
 *     levels small enough for the fused single-launch kernels run as replicas.
 *   - forceAtlasMultilevel: aggregates dealt to ranks by cost (longest
 *     processing time first), no exchange during the iterations (:454, :462 read
 *     only the frozen coarse coordinates), one all-gather of the members'
 *     coordinates at the end.
 *   - P^T A P: coarse rows dealt to ranks in contiguous blocks of equal expanded
 *     work, one all-gather of the coarse rows.
 * A communicator is RCCL (ncclCommInitRank over xGMI: ge_comm_unique_id on
 * rank 0, shipped to the others out of band) or a caller transport (host
 * all-gather callback, e.g. MPI or gloo; data are staged through host memory).
 * Every rank passes the same inputs; collective calls must be made by all ranks
 * in the same order. */
#define GE_COMM_ID_BYTES 128
typedef struct ge_transport {
  void* user;
  /* All-gather of equal blocks: recv (nranks * bytes, rank-major) receives every
   * rank's `bytes` bytes of send.  Host pointers.  Returns 0 on success. */
  int (*allgather)(void* user, const void* send, void* recv, unsigned long long bytes);
} ge_transport;

int ge_comm_unique_id(unsigned char* id /* GE_COMM_ID_BYTES */);
/* RCCL communicator on the context's device; collectives run on its stream. */
int ge_comm_create(ge_ctx* ctx, int nranks, int rank, const unsigned char* id, ge_comm** out);
int ge_comm_create_transport(ge_ctx* ctx, int nranks, int rank, const ge_transport* t,
                             ge_comm** out);
int ge_comm_info(const ge_comm* comm, int* nranks, int* rank, int* is_rccl);
int ge_comm_destroy(ge_comm* comm);

/* Row shard of rank `rank`: rows [*row_begin, *row_end) of n, blocks of
 * *rows_per_rank = ceil(n / nranks) rows (coordinate buffers hold
 * nranks * rows_per_rank rows so every rank's block has the same size). */
int ge_row_shard(int n, int nranks, int rank, int* row_begin, int* row_end, int* rows_per_rank);
/* In-place all-gather of rank blocks of a device coordinate array
 * d_x[nranks * rows_per_rank * dim]: rank r contributes rows
 * [r * rows_per_rank, (r + 1) * rows_per_rank). */
int ge_allgather_coords(ge_comm* comm, double* d_x, long long rows_per_rank, int dim);
/* Deal aggregates to ranks by cost s(s-1) + (CSR entries of the members, when
 * indptr != NULL): descending cost (ties: lower id) to the least-loaded rank
 * (ties: lower rank).  owner[m] receives each aggregate's rank.  Host only. */
int ge_assign_aggregates(int m, const int* pt_indptr, const int* pt_indices, const int* indptr,
                         int nranks, int* owner);
/* After every rank wrote the coordinates of the members of its own aggregates
 * into d_x (n * dim, fine-vertex order; e.g. ge_faml_plan_run of a subset plan),
 * every rank holds all of them.  h_owner: ge_assign_aggregates' result;
 * h_pt_indptr / h_pt_indices: P_T on the host. */
/* ge_assign_aggregates with the giant aggregates split (owner -1): those with at
 * least min_members members (min_members > 0), none (0), or (< 0) those whose
 * ordered pairs exceed half a rank's average load (GE_DIST_SPLIT_MIN overrides). */
int ge_assign_aggregates_split(int m, const int* pt_indptr, const int* pt_indices,
                               const int* indptr, int nranks, int min_members, int* owner);
int ge_allgather_members(ge_comm* comm, double* d_x, int dim, int m, const int* h_pt_indptr,
                         const int* h_pt_indices, const int* h_owner);

/* Sharded forms of ge_force_atlas, ge_force_atlas_ml, ge_ptap and ge_embed (same
 * arguments, the context is the communicator's).  Results are identical on
 * every rank and bit-identical to the single-GPU calls. */
int ge_force_atlas_dist(ge_comm* comm, int n, const int* indptr, const int* indices,
                        const double* data, int dim, double* coords, int init_random,
                        int iterations, const ge_fa_params* p);
int ge_force_atlas_ml_dist(ge_comm* comm, int n, const int* indptr, const int* indices,
                           const double* data, int m, const int* pt_indptr,
                           const int* pt_indices, const int* vertex_A, const double* coords_A,
                           const double* r_A, double* coords, int dim, int iterations,
                           const ge_fa_params* p);
int ge_ptap_dist(ge_comm* comm, int n, const int* indptr, const int* indices, const double* data,
                 int m, const int* pt_indptr, const int* pt_indices, ge_csr** out);
int ge_embed_dist(ge_comm* comm, int levels, const int* a_n, const int* a_off,
                  const int* a_nz_off, const int* a_indptr, const int* a_indices,
                  const double* a_data, const int* p_rows, const int* p_off,
                  const int* p_nz_off, const int* p_indptr, const int* p_indices, int dim,
                  int base_iterations, int ml_iterations, int print_progress,
                  const ge_fa_params* p, double* coords_out);

/* ---- alternative embedder ----
 * Replaces partition::embedViaMinimization(A, d, coords, ITER) (include/embed.hpp:22-23,
 * src/embed.cpp:341-559): `iterations` Gauss-Seidel sweeps of a per-vertex line
 * search towards the 2d unit directions, then centring and scaling.  coords:
 * n*dim in/out; init_random != 0 first draws U(-1,1) from mt19937(seed) (the
 * reference's empty-coords branch, :353-361).  Edge weights are not read (the
 * reference ignores them).  Host code (off the embed path; the line searches are
 * chains of serial n-term sums); the 2d directions run on OpenMP threads.
 * anyToMultilevel / embedVia / embedViaMultilevel (src/embed.cpp:23-338) are
 * header-only in graph-embed_amd/include/embed.hpp on top of this ABI. */
int ge_embed_via_minimization(int n, const int* indptr, const int* indices, int dim,
                              double* coords, int init_random, unsigned seed, int iterations);

/* The reference's initial-coordinate stream: the first `count` values of
 * uniform_real_distribution<double>(-1,1) over mt19937(seed) (libstdc++). */
int ge_uniform_stream(unsigned seed, long long count, double* out);

/* Diagnostics: checks on the device that the strict kernels' shared-reciprocal
 * division (graph-embed_amd/csrc/ge_math.hpp) returns the same bits as IEEE
 * division for `samples` random and adversarial operand triples. */
int ge_selftest_math(ge_ctx* ctx, long long samples, unsigned long long seed,
                     long long* mismatches);

/* ---- synthetic inputs (bench / tests) ----
 * Graph500 R-MAT (0.57, 0.19, 0.19, 0.05) with a counter-based SplitMix64
 * generator (definition: tests/graphs.py), symmetrised, deduplicated, unit
 * weights; and the largest connected component as examples/embedder.cpp:35-93. */
int ge_rmat_csr(int n, long long draws, unsigned long long seed, ge_csr** out);
int ge_largest_component(int n, const int* indptr, const int* indices, const double* data,
                         ge_csr** out);
/* The same two on the device (graph-embed_amd/csrc/ge_graph.hip), same results:
 * R-MAT by counter-based generation + radix sort + compaction, lcc != 0 returns
 * its largest connected component (hooking + pointer jumping, vertices renumbered
 * in ascending original id, examples/embedder.cpp:35-93). */
int ge_rmat_csr_device(ge_ctx* ctx, int n, long long draws, unsigned long long seed, int lcc,
                       ge_csr** out);
int ge_largest_component_device(ge_ctx* ctx, int n, const int* indptr, const int* indices,
                                const double* data, ge_csr** out);

#ifdef __cplusplus
}
#endif
#endif /* GE_H */
