/*
 * gsparse.h -- C ABI of libgsparse.so, the MI355X (gfx950) edge-scoring engine.
 *
 * This is the drop-in boundary below the reference's Python API
 * (/root/reference/src/sparsification): the host mirror
 * gnn-sparsification-research_amd/gsparse/ binds these entry points with
 * ctypes and keeps the reference's names, argument meaning and error
 * behaviour.  The reference has no FFI of its own (it is NumPy/SciPy), so
 * each entry point below cites the reference function whose arithmetic it
 * replaces.  Conventions:
 *   - every function returns 0 (GS_OK) or a negative GS_E* code and never
 *     throws; gs_last_error() gives the message (thread-local);
 *   - "loc" arguments say where a pointer lives: GS_HOST or GS_DEVICE;
 *   - scores are float64, one per canonical-CSR entry, in CSR order
 *     (the reference's adj.nonzero() order, metrics.py:47,115,236,348);
 *   - calls are synchronous with respect to host pointers; device-pointer
 *     outputs are complete when the call returns unless gs_set_async(1).
 */
#ifndef GSPARSE_H
#define GSPARSE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_API_VERSION 3

enum {
    GS_OK = 0,
    GS_EINVAL = -1,       /* bad argument (Python shim raises ValueError)      */
    GS_EHIP = -2,         /* HIP runtime error                                 */
    GS_ENOMEM = -3,       /* device allocation failed                          */
    GS_ESTATE = -4,       /* call out of order (e.g. no graph set)             */
    GS_EUNSUPPORTED = -5, /* input outside the implemented contract            */
    GS_EINDEX = -6        /* an array shorter than the index range it must cover
                             (Python shim raises IndexError, as NumPy does)     */
};

enum { GS_HOST = 0, GS_DEVICE = 1 };

typedef struct gs_ctx gs_ctx;

/* ---- library / context ------------------------------------------------- */
int gs_api_version(void);
const char *gs_last_error(void);
int gs_device_count(int *count);
/* One context per (process, device); not re-entrant per context. */
int gs_create(int device, gs_ctx **out);
void gs_destroy(gs_ctx *ctx);
/* Use an external hipStream_t (e.g. torch.cuda.current_stream()); NULL =
 * the context's own stream. */
int gs_set_stream(gs_ctx *ctx, void *hip_stream);
/* Stream ordering without a host sync (hip_stream NULL = the null stream):
 * gs_stream_wait -- work the context enqueues from now on runs after
 *   everything already enqueued on hip_stream (call it before handing the
 *   library device buffers that another stream produced or last used, e.g.
 *   torch.cuda.current_stream());
 * gs_stream_signal -- work enqueued on hip_stream from now on runs after
 *   everything the context has enqueued (device outputs in async mode). */
int gs_stream_wait(gs_ctx *ctx, void *hip_stream);
int gs_stream_signal(gs_ctx *ctx, void *hip_stream);
int gs_synchronize(gs_ctx *ctx);
/* 1: device-pointer outputs may still be in flight on return. */
int gs_set_async(gs_ctx *ctx, int async_);

/* Kernel timing on the context's stream (hipEvents around every launch). */
int gs_profile_enable(gs_ctx *ctx, int on);
int gs_profile_reset(gs_ctx *ctx);
/* i-th profiled kernel name; -1 past the end. ms = summed launch time. */
int gs_profile_get(gs_ctx *ctx, int i, char *name, int name_len, int64_t *launches,
                   double *ms, double *bytes);

/* ---- graph --------------------------------------------------------------
 * Replaces GraphSparsifier.__init__'s COO->CSR build (core.py:70-74):
 * sp.csr_matrix((ones(E), (ei[0], ei[1])), (n, n)) -- duplicates summed
 * (data = multiplicity), columns sorted.  Built on the device. */
int gs_graph_from_edge_index(gs_ctx *ctx, int64_t n, int64_t E, const int64_t *src,
                             const int64_t *dst, int loc);
/* Canonical CSR given directly (sorted columns, no duplicates), e.g. the
 * adj argument of the metrics.py module functions. data may be NULL (=1). */
int gs_graph_from_csr(gs_ctx *ctx, int64_t n, int64_t nnz, const int64_t *indptr,
                      const int32_t *indices, const double *data, int loc);
int gs_graph_shape(gs_ctx *ctx, int64_t *n, int64_t *nnz, int *symmetric);
/* Canonical edge list for the dataset loader (gsparse/loader.py, standing in
 * for the reference's absent src/data; PyG's to_undirected + coalesce):
 * undirected != 0 adds every reversed pair; remove_self_loops != 0 drops
 * u == v; the result is sorted by (row, col) with duplicates removed.
 * *out_E: capacity on entry (2E suffices), edge count on return. */
int gs_coalesce_edges(gs_ctx *ctx, int64_t n, int64_t E, const int64_t *src, const int64_t *dst,
                      int undirected, int remove_self_loops, int64_t *out_src, int64_t *out_dst,
                      int64_t *out_E, int loc);
int gs_graph_copy_csr(gs_ctx *ctx, int64_t *indptr, int32_t *indices, double *data, int loc);

/* ---- scorers: out[e - e0] for CSR entries e in [e0, e1) ------------------ */
/* calculate_jaccard_scores, metrics.py:17-64 (bit-exact). */
int gs_jaccard(gs_ctx *ctx, int64_t e0, int64_t e1, double *out, int loc);
/* Part `part` of `nparts` of the whole-graph Jaccard (multi-GPU sharding,
 * SURVEY 8(e)): out[nnz] holds this part's pairs (both CSR entries of each
 * undirected pair on a symmetric graph; an edge range on a directed one) and
 * 0.0 elsewhere, so the element-wise sum of the nparts outputs equals
 * gs_jaccard(0, nnz) bit for bit. */
int gs_jaccard_part(gs_ctx *ctx, int part, int nparts, double *out, int loc);
/* Sharded Jaccard with an all-gather of per-pair counts (multi-GPU, SURVEY
 * 8(e); symmetric graphs, else GS_EUNSUPPORTED).  The owner of an undirected
 * pair {u, v} is the endpoint of larger degree (ties: smaller id); its CSR
 * entry (u, v) is the pair's owner entry.  Part p of nparts owns the owner
 * entries of rows [row_cut[p], row_cut[p+1]) -- contiguous row ranges cut at
 * equal shares of the intersection work, the same on every rank -- which are
 * owner entries [owner_off[p], owner_off[p+1]) in CSR order.
 *   gs_jaccard_shares: row_cut[nparts+1], owner_off[nparts+1] (host; either
 *     may be NULL).
 *   gs_jaccard_part_counts: counts[i] = |N(u) ∩ N(v)| of part p's i-th owner
 *     entry (uint32, owner_off[p+1] - owner_off[p] values).
 *   gs_jaccard_from_counts: every part's counts (part p's at counts + p*stride,
 *     e.g. an all-gather of the shares padded to stride) -> out[nnz], the
 *     score of both CSR entries of every pair (the reference's single fp64
 *     division of metrics.py:54-59): bit-identical to gs_jaccard(0, nnz).
 *     A part longer than stride is GS_EINDEX. */
int gs_jaccard_shares(gs_ctx *ctx, int nparts, int64_t *row_cut, int64_t *owner_off);
int gs_jaccard_part_counts(gs_ctx *ctx, int part, int nparts, uint32_t *counts, int loc);
int gs_jaccard_from_counts(gs_ctx *ctx, int nparts, const uint32_t *counts, int64_t stride,
                           int c_loc, double *out, int loc);
/* Distributed global top-k of Jaccard-T (GraphSparsifier.sparsify, core.py:229-240, over N
 * ranks; SURVEY 8(e) "top-k alone: histogram all-reduce") without gathering scores.  Each
 * rank selects over its own owner pairs (gs_jaccard_part_counts; a pair's two CSR entries
 * share one score, multiplicity 2, a self-loop 1):
 *   gs_jsel_begin   scores (scores may be NULL: this part's pairs, owner order) and keys of
 *                   the own pairs; hist (device, GS_JSEL_BINS uint64) = the weighted
 *                   histogram of the keys' top 12 bits.  0 < num_keep < nnz.
 *   gs_jsel_step    hist holds the SUM over ranks of the last histogram: picks the digit
 *                   of the cut's rank and writes the next digit's histogram into hist;
 *                   GS_JSEL_PASSES calls (12 + 4 x 13 bits), *passes_left counts down.
 *   gs_jsel_result  the cut score, the entries strictly beyond it and the tie block (the
 *                   same on every rank, = gs_topk_mask's), and this rank's tied positions.
 *   gs_jsel_tie_positions  this rank's tied CSR positions (npos >= my_tied).
 *   gs_jsel_keep    2-bit keep codes of the own pairs (bit 0 the owner entry, bit 1 the
 *                   reverse entry), pair i in bits 2 (i % 4) of byte i / 4: ceil(pairs / 4)
 *                   bytes.  need = num_keep - n_beyond; when 0 < need < n_tied the cut is
 *                   ambiguous and tie_pos must hold every rank's tied positions (ntie =
 *                   n_tied, any order): the block is resolved as np.argsort(kind='stable')
 *                   resolves it (top: the highest positions; keep_lowest: the lowest).
 *   gs_jsel_mask    every rank's codes (part p's at keep_all + p * stride bytes, an
 *                   all-gather padded to stride) -> the CSR keep mask mask[nnz], bit-identical
 *                   to gs_topk_mask on the gathered scores.
 * Symmetric graphs with nnz < 2^31 (else GS_EUNSUPPORTED). */
enum { GS_JSEL_BINS = 8192, GS_JSEL_PASSES = 5 };
int gs_jsel_begin(gs_ctx *ctx, int part, int nparts, const uint32_t *counts, int c_loc,
                  int64_t num_keep, int keep_lowest, uint64_t *hist, double *scores, int s_loc);
int gs_jsel_step(gs_ctx *ctx, uint64_t *hist, int *passes_left);
int gs_jsel_result(gs_ctx *ctx, double *cut, int64_t *n_beyond, int64_t *n_tied, int64_t *my_tied);
int gs_jsel_tie_positions(gs_ctx *ctx, int64_t *pos, int64_t npos, int loc);
int gs_jsel_keep(gs_ctx *ctx, const int64_t *tie_pos, int64_t ntie, int t_loc, int64_t need,
                 uint8_t *keep, int k_loc);
int gs_jsel_mask(gs_ctx *ctx, int nparts, const uint8_t *keep_all, int64_t stride, int k_loc,
                 uint8_t *mask, int m_loc);
/* calculate_adamic_adar_scores, metrics.py:67-121 (bit-exact).  c[w] =
 * 1/sqrt(max(log(deg_w+1),1e-10)) as NumPy computes it (metrics.py:104-108),
 * n values. */
int gs_adamic_adar(gs_ctx *ctx, const double *c, int c_loc, int64_t e0, int64_t e1,
                   double *out, int loc);
/* compute_scores('degree'), core.py:167-172 (bit-exact). */
int gs_degree(gs_ctx *ctx, int64_t e0, int64_t e1, double *out, int loc);
/* calculate_feature_cosine_scores, metrics.py:301-358 (bit-exact, x's dtype). */
int gs_feature_cosine_f32(gs_ctx *ctx, const float *x, int64_t f, int x_loc, int64_t e0,
                          int64_t e1, double *out, int loc);
int gs_feature_cosine_f64(gs_ctx *ctx, const double *x, int64_t f, int x_loc, int64_t e0,
                          int64_t e1, double *out, int loc);

/* ---- ApproxER: calculate_approx_effective_resistance_scores,
 *      metrics.py:178-298 -------------------------------------------------
 * gs_er_prepare: edges u<v in CSR order (m of them, :236-242), L_reg =
 *   diag(rowsum A) - A + reg*I (:251-256); allocates Y/Z (n x k, row-major).
 * gs_er_project_rows: streams rows [e0, e1) of the raw standard-normal
 *   matrix (row-major, k per row, NumPy Generator order) and folds
 *   Y = B @ (raw / sqrt_k) (:272-275) in ascending edge id.  Rows must be
 *   streamed in order, each exactly once.
 * gs_er_project_pcg64: the same, drawing the normals on the device from
 *   NumPy's PCG64 state (state_hi/lo, inc_hi/lo) with NumPy's ziggurat.
 * gs_er_solve: CG on columns [col0, col1) (:284-289), SciPy 1.15 cg
 *   recurrence with OpenBLAS-SkylakeX ddot order for blas_threads threads
 *   (more than 64 run as 64: OpenBLAS's MAX_THREADS in NumPy's build).
 * gs_er_scores: out[e-e0] = sum over columns [col0,col1) of (Z_u - Z_v)^2 in
 *   NumPy pairwise order (:292-293).  [col0,col1) must be a node of the
 *   pairwise tree of k (the whole range, or a gs_er_split() block); when
 *   finalize != 0 the clamp of :296-297 is applied.
 * gs_er_iterations: CG iterations each column ran (k values).
 * gs_er_copy_z: the solved Z columns [col0, col1) (metrics.py:285-289's
 *   Z[:, i] = cg(...)), n rows x (col1 - col0) row-major -- a parity read-out. */
int gs_er_prepare(gs_ctx *ctx, int64_t k, double reg, int64_t *m_out);
int gs_er_project_rows(gs_ctx *ctx, int64_t e0, int64_t e1, const double *raw, int loc,
                       double sqrt_k);
int gs_er_project_pcg64(gs_ctx *ctx, uint64_t state_hi, uint64_t state_lo, uint64_t inc_hi,
                        uint64_t inc_lo, double sqrt_k);
/* Column-slice forms (a rank's JL columns): the normal stream /
 * the host rows are the same whole NumPy stream, but only Y[:, col0:col1] is
 * formed; gs_er_solve then accepts column ranges inside [col0, col1). */
int gs_er_project_pcg64_cols(gs_ctx *ctx, uint64_t state_hi, uint64_t state_lo, uint64_t inc_hi,
                             uint64_t inc_lo, double sqrt_k, int64_t col0, int64_t col1);
int gs_er_project_rows_cols(gs_ctx *ctx, int64_t e0, int64_t e1, const double *raw, int loc,
                            double sqrt_k, int64_t col0, int64_t col1);
int gs_er_solve(gs_ctx *ctx, int64_t col0, int64_t col1, int32_t maxiter, double rtol,
                int32_t blas_threads);
int gs_er_scores(gs_ctx *ctx, int64_t col0, int64_t col1, int64_t e0, int64_t e1,
                 int finalize, double *out, int loc);
int gs_er_iterations(gs_ctx *ctx, int32_t *iters, int loc);
int gs_er_copy_z(gs_ctx *ctx, int64_t col0, int64_t col1, double *out, int loc);
/* Column blocks of the pairwise tree of k at depth log2(parts): bounds has
 * parts+1 entries.  parts must be a power of two. */
int gs_er_split(int64_t k, int32_t parts, int64_t *bounds);

/* ---- selection: GraphSparsifier.sparsify core.py:229-242 -----------------
 * mask[E] (uint8): the num_keep highest (keep_lowest: lowest) of the nnz
 * scores, ties broken as np.argsort(kind='stable') does (top: highest
 * indices; lowest: lowest indices); num_keep == 0 keeps all nnz for top
 * (the reference's idx[-0:] quirk) and none for keep_lowest.  Also returns
 * the cut key, #strictly-beyond-cut and #tied-at-cut (n_tied > needed means
 * the reference's unstable argsort may resolve the tie block differently). */
int gs_topk_mask(gs_ctx *ctx, const double *scores, int s_loc, int64_t nnz, int64_t E,
                 int64_t num_keep, int keep_lowest, uint8_t *mask, int m_loc,
                 double *cut, int64_t *n_beyond, int64_t *n_tied);

/* ---- metric backbone: compute_metric_backbone, metric_backbone.py:28-141
 * keep[idx] for every edge_index column idx=(src,dst): shortest-path
 * distance d from src in the undirected graph of the src<dst columns
 * (min weight over duplicates), keep iff d == inf or w[idx] <= d + eps.
 * nw = number of entries of w: nw < E is GS_EINDEX (the reference reads
 * edge_weights[idx] for every column, metric_backbone.py:73-74, and raises
 * IndexError).  n_relax (optional) returns the number of edge relaxations
 * performed. */
/* sparsify_degree_aware phase 1 (core.py:415-428, min_edges_per_node = 1):
 * for every node u, pick[u] = the edge_index column i (src[i] == u) holding
 * the unique maximum of scores[i], -1 if u has no column, -2 when the
 * reference's np.argsort order decides (ties at the maximum or a NaN).
 * scores are indexed by column as the reference indexes them (needs E <=
 * nscores, else GS_EINVAL, the reference's IndexError). */
int gs_segment_argmax(gs_ctx *ctx, const double *scores, int s_loc, int64_t nscores,
                      const int64_t *src, int src_loc, int64_t E, int64_t n, int64_t *pick,
                      int pick_loc);

int gs_metric_backbone(gs_ctx *ctx, int64_t n, int64_t E, const int64_t *src,
                       const int64_t *dst, const double *w, int64_t nw, int loc, double eps,
                       uint8_t *keep, int keep_loc, int64_t *n_relax);
/* Part `part` of `nparts` of gs_metric_backbone (multi-GPU): keep
 * bytes of the columns (u, v) with max(u, v) % nparts == part -- both directions
 * of a pair in one part, ids as the library labels them (graphs without id
 * locality are relabeled by descending degree, so max(u, v) is the pair's
 * lower-degree endpoint) -- 0 elsewhere; the element-wise sum over parts equals
 * the whole keep mask. */
int gs_metric_backbone_part(gs_ctx *ctx, int64_t n, int64_t E, const int64_t *src,
                            const int64_t *dst, const double *w, int64_t nw, int loc, double eps,
                            int part, int nparts, uint8_t *keep, int keep_loc, int64_t *n_relax);

/* The metric backbone in stages, for N ranks (metric_backbone.py:86-111
 * decided by sources split over the ranks).  Every rank calls the stages in order
 * with its own part / nparts and exchanges between them:
 *   gs_bb_begin        relabel, G, and the landmark searches l = part (mod nparts);
 *                      n_landmarks = K.  Exchange: the K x n landmark labels
 *                      (gs_bb_landmarks_io, element-wise MIN over ranks; +inf where
 *                      another rank searched) and the K completeness flags (MAX).
 *   gs_bb_certify      2-hop witness and certificates of this part's column range.
 *                      Exchange: the E column states (gs_bb_state_io, element-wise
 *                      MAX: 0 open, 1 keep, 2 prune; every rule is exact, so ranks
 *                      that decide a column decide it alike).
 *   gs_bb_plan         the sources with open columns (the same on every rank) and
 *                      nbatch, the search batches in their processing order.
 *   gs_bb_search       batches [b0, b1) (0 <= b0 <= b1 <= nbatch), this part's every
 *                      nparts-th one; exchange the states (MAX) after each range.
 *   gs_bb_finish       keep bytes of every column (state 1).
 * dir 0 copies the library's buffer out to D / complete / state, 1 copies it in;
 * loc: GS_HOST or GS_DEVICE.  With one part and one range this is gs_metric_backbone. */
int gs_bb_begin(gs_ctx *ctx, int64_t n, int64_t E, const int64_t *src, const int64_t *dst,
                const double *w, int64_t nw, int loc, double eps, int part, int nparts,
                int32_t *n_landmarks);
int gs_bb_landmarks_io(gs_ctx *ctx, double *D, int32_t *complete, int loc, int dir);
int gs_bb_certify(gs_ctx *ctx, int part, int nparts);
int gs_bb_state_io(gs_ctx *ctx, uint8_t *state, int loc, int dir);
int gs_bb_plan(gs_ctx *ctx, int64_t *nbatch);
int gs_bb_search(gs_ctx *ctx, int64_t b0, int64_t b1, int part, int nparts);
int gs_bb_finish(gs_ctx *ctx, uint8_t *keep, int keep_loc, int64_t *n_relax);

/* Decision classes of the metric backbone (a diagnostic: which exact rule decided each
 * column of metric_backbone.py:97-111's comparison).  gs_bb_classes(ctx, 1) makes the
 * following backbone runs on ctx record a class byte per column; gs_bb_class_counts
 * returns, for the last run, counts[k] = columns decided by class k on this rank
 * (ncounts >= GS_BB_WHY_CLASSES; counts[GS_BB_WHY_OPEN] = columns this rank left to
 * others) and, when why != NULL, the E class bytes (nwhy >= E, else GS_EINDEX;
 * why_loc: GS_HOST / GS_DEVICE); n_columns (may be NULL) = E of that run. */
enum {
    GS_BB_WHY_OPEN = 0,
    GS_BB_WHY_SELF,         /* self-loop: d(u, u) = 0 */
    GS_BB_WHY_ISOLATED,     /* an endpoint without edges in G: keep */
    GS_BB_WHY_DEG1,         /* an endpoint of degree 1 whose neighbour is the other: d = w_G */
    GS_BB_WHY_DIRECT,       /* w > fl(w_G(u, v) + eps): prune */
    GS_BB_WHY_LOCAL2,       /* local lower bound from both endpoints' least other edges: keep */
    GS_BB_WHY_LM_COMP,      /* a complete landmark search reaches one endpoint only: keep */
    GS_BB_WHY_LM_PRUNE,     /* landmark upper bound: prune */
    GS_BB_WHY_LM_KEEP,      /* landmark lower bound: keep */
    GS_BB_WHY_WITNESS,      /* 2-hop witness path: prune */
    GS_BB_WHY_LOCAL34,      /* 2- / 3- / 4-edge local lower bound: keep */
    GS_BB_WHY_SEARCH_PRUNE, /* the source row's bounded search: prune */
    GS_BB_WHY_SEARCH_KEEP,  /* the source row's bounded search: keep */
    GS_BB_WHY_REV_EXACT,    /* the reverse row's search, exact rule */
    GS_BB_WHY_REV_PRUNE,    /* the reverse row's search, upper bound: prune */
    GS_BB_WHY_REV_KEEP,     /* the reverse row's search, unreached within its bound: keep */
    GS_BB_WHY_MITM,         /* meet-in-the-middle certificate (GSPARSE_BB_MITM=1) */
    GS_BB_WHY_CLASSES
};
int gs_bb_classes(gs_ctx *ctx, int on);
int gs_bb_class_counts(gs_ctx *ctx, int64_t *counts, int ncounts, uint8_t *why, int64_t nwhy,
                       int why_loc, int64_t *n_columns);

/* Exact shortest-path distances for nq node pairs (qs[q], qt[q]) (host arrays;
 * out host) in the graph metric_backbone.py:70-79 builds from the columns
 * (src, dst, w): undirected, the columns with src < dst, weight the minimum
 * over duplicates; w == NULL: unit weights (hop counts); nw = entries of w
 * (nw < E: GS_EINDEX).  +inf when
 * unreachable; 0 when qs == qt.  Bit-identical to NetworkX Dijkstra's
 * left-fold path sums.  Replaces the nx.shortest_path_length calls of
 * verify_geodesic_preservation (metric_backbone.py:144-225) and
 * compute_geodesic_preservation (metrics.py:361-442). */
int gs_pair_distances(gs_ctx *ctx, int64_t n, int64_t E, const int64_t *src, const int64_t *dst,
                      const double *w, int64_t nw, int loc, int64_t nq, const int64_t *qs,
                      const int64_t *qt, double *out);

/* Exact effective resistance of the resident (symmetric) graph, one score per
 * CSR entry.  Replaces calculate_effective_resistance_scores (metrics.py:124-175:
 * dense pinv of L + 1e-10 I).  Computed as G_uu + G_vv - 2 G_uv with G the
 * inverse of the grounded Laplacian M (one ground node per connected
 * component, its row/column read as zero), G from a blocked fp64-MFMA Cholesky
 * M = L L^T and L^-1 (GSPARSE_XER_METHOD=ns: Newton-Schulz); max(., 1e-10) as
 * the reference clamps.  Dense: n <= 32768 (GS_EUNSUPPORTED above, and for a
 * directed adjacency).  *iterations (may be NULL) receives the number of 64-row
 * blocks (Cholesky) or Newton-Schulz steps. */
int gs_exact_er(gs_ctx *ctx, double *out, int out_loc, int32_t *iterations);

/* ---- compute_topology_metrics (metrics.py:445-520) on the resident graph ----
 * The resident graph must be symmetric; the clustering and the counts expect
 * it self-loop-free (NetworkX drops v from its own neighbour set).
 *
 * |N(u) ∩ N(v)| per CSR entry (exact integers as float64). */
int gs_common_neighbors(gs_ctx *ctx, double *out, int out_loc);
/* nx.average_clustering in NetworkX's operation order (bit-identical):
 * c_v = 0 if t == 0 else t / (d (d - 1)), t = sum of the counts of v's entries,
 * summed left to right from 0 in node order, / n.  per_node (may be NULL,
 * location per_loc) receives c_v. */
int gs_clustering(gs_ctx *ctx, double *avg, double *per_node, int per_loc);
/* Connected components (nx.connected_components): labels[u] = smallest node id
 * of u's component (may be NULL), *count, *largest (size of the largest). */
int gs_components(gs_ctx *ctx, int32_t *labels, int labels_loc, int64_t *count,
                  int64_t *largest);
/* Algebraic connectivity (nx.algebraic_connectivity, weighted, unnormalised)
 * of a connected resident graph, n <= 32768: 1 / lambda_max(P G P), G the
 * grounded inverse of L (fp64-MFMA Cholesky), P = I - 11^T/n, by Lanczos with
 * full reorthogonalisation until the Ritz value changes by <= tol (relative)
 * or max_iter (<= 500) steps.  GS_EINVAL if the graph is not connected. */
int gs_fiedler(gs_ctx *ctx, double tol, int32_t max_iter, double *value, int32_t *iterations);

#ifdef __cplusplus
}
#endif
#endif /* GSPARSE_H */
