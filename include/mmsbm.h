/*
 * mmsbm.h — C ABI of the MI355X MMSBM EM engine (libmmsbm.so).
 *
 * Drop-in boundary for the triplet-link E/M loop of
 * AleixMT/TrigenicInteractionPredictor, src/TrigenicInteractionPredictor.py.
 * The reference boundary is a Python method API, not an FFI; each entry point
 * below names the reference method it replaces.  The Python host mirror
 * (trigenicinteractionpredictor_amd/model.py, class Model) binds these through
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - every call returns MMSBM_OK (0) or a negative MMSBM_ERR_* code;
 *    mmsbm_last_error() returns the message of the last failure (thread-local);
 *  - all array pointers are DEVICE pointers (memory owned by the caller, e.g.
 *    PyTorch tensors) unless the parameter name ends in _host;
 *  - kernels are enqueued on the caller's hipStream_t (passed as void*); only
 *    setup calls (set_links / set_genes) synchronise;
 *  - a context is not thread-safe: one host thread per context, one process
 *    per GPU.
 *
 * Device layouts
 *  - obs    int32[n_obs_pad][4] = (id1, id2, id3, n): one row per OBSERVED
 *           (link, rating) pair, ids in the reference's string-sorted key order
 *           (:349-358), n = links[key][r] (:360-368).  Rows are grouped by
 *           rating r; every group starts on a multiple of MMSBM_TILE and is
 *           padded with (0,0,0,0) rows (weight 0, contributes exactly 0).
 *  - theta  f64[B][P][K]          membership vectors of B batched samples (:117-121)
 *  - pr     f64[B][R][K][K][K]    rating-major copy of the reference's
 *           pr[K][K][K][R] (:124-139)
 *  - gene CSR: gene_ptr int32[P+1], gene_inc int32[nnz] with entries
 *           obs_row*3 + slot, listing every (observation, slot) of gene g in
 *           ascending order; deg int32[P] = the reference's `counter`
 *           (:986-994: one per link slot, independent of the counts).
 */
#ifndef MMSBM_H
#define MMSBM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMSBM_OK 0
#define MMSBM_ERR_INVALID -1      /* bad argument / call order */
#define MMSBM_ERR_HIP -2          /* a HIP runtime call failed */
#define MMSBM_ERR_ZERO_DEGREE -3  /* a gene has no train link: the reference raises
                                     ZeroDivisionError at :1018 */
#define MMSBM_ERR_UNSUPPORTED -4  /* shape outside the compiled kernel set */

#define MMSBM_TILE 256            /* observations per workgroup tile */
#define MMSBM_MAX_K 32
#define MMSBM_SET_TRAIN 0         /* `links` (:57) */
#define MMSBM_SET_TEST 1          /* `test_links` (:61) */

typedef struct mmsbm_ctx mmsbm_ctx;

int mmsbm_version(void);
int mmsbm_tile(void);
const char *mmsbm_last_error(void);

/* Context = one GPU + one problem shape.  Replaces the per-process `Model()`
 * state of :39-88 for the hot path. */
int mmsbm_create(int device, mmsbm_ctx **out);
int mmsbm_destroy(mmsbm_ctx *ctx);

/* K groups, R ratings (2 in the reference, :79), B batched samples
 * (independent restarts, :1253), P genes (:413), eps (:88). */
int mmsbm_set_shape(mmsbm_ctx *ctx, int32_t K, int32_t R, int32_t B, int32_t P, double eps);

/* Device edge list of one link set (MMSBM_SET_TRAIN = `links`,
 * MMSBM_SET_TEST = `test_links`), built by the host from get_traintest's
 * dicts (:321-423).  seg_host[R+1]: start row of each rating group
 * (seg_host[R] = n_obs_pad); every entry a multiple of MMSBM_TILE. */
int mmsbm_set_links(mmsbm_ctx *ctx, int32_t which, const int32_t *obs, int64_t n_obs_pad,
                    const int64_t *seg_host);

/* Gene incidence CSR of the TRAIN set for the theta M-step (:1016-1018).  Call after
 * mmsbm_set_links(MMSBM_SET_TRAIN) (re-setting the train links requires calling it again).
 * The engine inverts it once on the device: every observation's three responsibility rows
 * are then written straight to their gene's contiguous CSR run.
 * Validates deg > 0 for every gene (copies deg to the host once); a zero
 * returns MMSBM_ERR_ZERO_DEGREE and makes mmsbm_iterate fail the same way. */
int mmsbm_set_genes(mmsbm_ctx *ctx, const int32_t *gene_ptr, const int32_t *gene_inc,
                    int64_t nnz, const int32_t *deg);

/* Scratch the engine needs (responsibility rows, per-tile partial sums). */
int mmsbm_workspace_bytes(const mmsbm_ctx *ctx, int64_t *bytes);
int mmsbm_set_workspace(mmsbm_ctx *ctx, void *ws, int64_t bytes);

/* n_iters EM iterations on all B samples, in place.
 * Replaces Model.make_iteration (:984-1043) called n_iters times. */
int mmsbm_iterate(mmsbm_ctx *ctx, double *theta, double *pr, int32_t n_iters, void *stream);

/* Log-likelihood of link set `which` for every sample into out[B] (device).
 * Replaces Model.compute_likelihood(selected_set) (:952-974). */
int mmsbm_loglik(mmsbm_ctx *ctx, int32_t which, const double *theta, const double *pr,
                 double *out, void *stream);

/* P(r = 1) for n rows of ids int32[n][3] into out[B][n] (device).
 * Replaces Model.do_prediction (:530-547), used by calculate_test_set_results
 * (:557-569). */
int mmsbm_predict(mmsbm_ctx *ctx, const int32_t *ids, int64_t n, const double *theta,
                  const double *pr, double *out, void *stream);

/* Link-sharded iteration (single sample over N ranks): each rank's context
 * holds 1/N of the train links (mmsbm_set_links) and the GLOBAL degree (mmsbm_set_genes' deg).
 * Step 1, the accumulation half of make_iteration (:986-1012) over this rank's links:
 *   nth[B][P][K]   = per gene, the sum of its local c-scaled (Y | Z | W) rows (theta not applied)
 *   S[B][R][K^3]   = the S lattice sums,  npr = p S.
 * The caller sums nth and S over ranks (one all-reduce of one buffer), then step 2 applies the
 * M-step (:1016-1028): theta <- theta nth / deg, p_r <- p_r S_r / (eps + sum_r p_r S_r).
 * Called on one rank with all links, the pair equals mmsbm_iterate(n = 1). */
int mmsbm_accumulate(mmsbm_ctx *ctx, const double *theta, const double *pr, double *nth, double *S,
                     void *stream);
int mmsbm_mstep(mmsbm_ctx *ctx, double *theta, double *pr, const double *nth, const double *S,
                void *stream);

/* Which E-step path mmsbm_iterate runs: 1 = fused FP64-MFMA KR-image kernel (E-step and S
 * accumulation in one kernel, then M2; K <= 10), 2 = the lean fused kernel (K = 11, 12, or
 * MMSBM_ESTEP=5), 3 = the large-K FP64-MFMA pair (E-step kernel, S-accumulation kernel, M2;
 * 13 <= K <= 32), 0 = the VALU E-step + M1 + M2 (MMSBM_ESTEP=1/2). */
int mmsbm_fused(const mmsbm_ctx *ctx, int32_t *fused);

/* Kernel timing for measurement (bench.py): with stride n > 0, mmsbm_iterate records a HIP
 * event pair on the launch stream around every kernel of every n-th iteration (kernel ids:
 * 0 E-step, 1 M1 = S accumulation + theta gather, 2 M2 = p update); 0 disables.
 * mmsbm_timing resets the counters; mmsbm_timing_result waits for the last event and returns
 * the summed device time (ms) and the number of timed launches of that kernel. */
int mmsbm_timing(mmsbm_ctx *ctx, int32_t stride);

/* Measurement: n back-to-back launches of the E-step kernel mmsbm_iterate would run (the fused
 * kernel, or the VALU E-step) on the current theta / pr, between one HIP event pair on
 * `stream`; *avg_ms = elapsed / n.  The E-step only reads theta / pr, so the parameters are
 * unchanged.  Synchronises the stream. */
int mmsbm_time_estep(mmsbm_ctx *ctx, double *theta, double *pr, int32_t n, void *stream,
                     double *avg_ms);
int mmsbm_timing_result(mmsbm_ctx *ctx, int32_t kernel, double *total_ms, int64_t *count);

#ifdef __cplusplus
}
#endif
#endif /* MMSBM_H */
