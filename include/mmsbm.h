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
 *  - pointers whose name ends in _host are HOST arrays; every other array
 *    pointer is a DEVICE pointer (memory owned by the caller, e.g. PyTorch
 *    tensors);
 *  - kernels are enqueued on the caller's hipStream_t (passed as void*); the
 *    setup calls (set_links, set_degree, set_workspace) synchronise;
 *  - every call runs on the context's device and restores the caller's current
 *    device on return;
 *  - a context is not thread-safe: one host thread per context.
 *
 * Device layouts
 *  - theta  f64[B][P][K]          membership vectors of B batched samples (:117-121)
 *  - pr     f64[B][R][K][K][K]    rating-major copy of the reference's
 *           pr[K][K][K][R] (:124-139)
 *  The engine's own work plan (observation streams ordered by each slot's gene,
 *  DESIGN.md) is built inside mmsbm_set_links from the host link table.
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

#define MMSBM_CHUNK 4             /* observations per MFMA k-step (one pivot gene each) */
#define MMSBM_MAX_K 32
#define MMSBM_SET_TRAIN 0         /* `links` (:57) */
#define MMSBM_SET_TEST 1          /* `test_links` (:61) */

typedef struct mmsbm_ctx mmsbm_ctx;

int mmsbm_version(void);
int mmsbm_chunk(void);
/* 16 hex digits naming the build (sha256 of the sources, headers, arch and flags): profile
 * records are stamped with it so a measurement can be matched to the library it came from. */
const char *mmsbm_build_id(void);
const char *mmsbm_last_error(void);

/* Context = one GPU + one problem shape.  Replaces the per-process `Model()`
 * state of :39-88 for the hot path. */
int mmsbm_create(int device, mmsbm_ctx **out);
int mmsbm_destroy(mmsbm_ctx *ctx);

/* K groups, R ratings (2 in the reference, :79), B batched samples
 * (independent restarts, :1253), P genes (:413), eps (:88).  Changing K, R or P
 * drops the link sets, the degree and the workspace (call mmsbm_set_links and
 * mmsbm_set_workspace again); changing B drops the workspace. */
int mmsbm_set_shape(mmsbm_ctx *ctx, int32_t K, int32_t R, int32_t B, int32_t P, double eps);

/* One link set (MMSBM_SET_TRAIN = `links`, MMSBM_SET_TEST = `test_links`) as the
 * reference holds it after get_traintest (:321-423), in dict insertion order:
 * ids_host[E][3] = the key's gene ids in its string-sorted order ('10_2_9' ->
 * 10, 2, 9; :349-358), counts_host[E][R] = links[key] (:360-368).  Builds the
 * device work plan.  For the train set it also computes the degree (the
 * reference's `counter`, :986-994: one per link slot) unless mmsbm_set_degree
 * fixed it.  Invalidates the workspace (query mmsbm_workspace_bytes again). */
int mmsbm_set_links(mmsbm_ctx *ctx, int32_t which, const int32_t *ids_host,
                    const int32_t *counts_host, int64_t E);

/* Kernel family of the small-K plans (K <= 12; one family above): the three-stream fused
 * E-step (SK_U) or the stream-0 E-step with Y entries (SK_Y).  Both follow the reference's sums
 * (:996-1028) and agree with it to ~1e-12; their sums are ordered differently, so a sample's bits
 * depend on the family, and within one family on nothing else (not B, not the sample's slot, not
 * the rank).  AUTO picks from B at every mmsbm_set_shape (B = 1: SK_U, the one-sample latency
 * winner; B >= 2: SK_Y, the throughput winner); a driver whose engines hold different B for one
 * run (a ragged last batch, ranks with unequal shares, a pool that shrinks) fixes the family from
 * its configured batch instead, so every sample of the run gets the same bits.  A change of the
 * effective family drops the link plans (call mmsbm_set_links again).  The environment variable
 * MMSBM_SK_Y=0/1 overrides it (measurement).  Replaces nothing in the reference (a scheduling
 * choice of this engine). */
#define MMSBM_FAMILY_AUTO 0
#define MMSBM_FAMILY_SKU 1
#define MMSBM_FAMILY_SKY 2
int mmsbm_set_family(mmsbm_ctx *ctx, int32_t family);

/* Active samples: mmsbm_iterate, mmsbm_loglik, mmsbm_accumulate, mmsbm_mstep and mmsbm_predict
 * process samples [0, n) of the B and leave the others untouched (n = 0 or n >= B: all B; the
 * default).  A restart driver that retires converged samples compacts the live ones to the front
 * and shrinks n instead of iterating finished slots (the reference ends a sample at convergence,
 * :1270-1276).  mmsbm_set_shape resets it to B. */
int mmsbm_set_active(mmsbm_ctx *ctx, int32_t n);

/* deg_host[P]: the degree the M-step divides by (:1016-1018) — for a
 * link-sharded rank the counter over ALL train links, not its own block.  A
 * zero makes mmsbm_iterate / mmsbm_mstep fail with MMSBM_ERR_ZERO_DEGREE.
 * The degree is pinned for the NEXT mmsbm_set_links(MMSBM_SET_TRAIN) only: a
 * train link set given without a preceding mmsbm_set_degree is counted afresh. */
int mmsbm_set_degree(mmsbm_ctx *ctx, const int32_t *deg_host);

/* Scratch the engine needs (c per observation, partial rows, S partials). */
int mmsbm_workspace_bytes(const mmsbm_ctx *ctx, int64_t *bytes);
int mmsbm_set_workspace(mmsbm_ctx *ctx, void *ws, int64_t bytes);

/* n_iters EM iterations on all B samples, in place.
 * Replaces Model.make_iteration (:984-1043) called n_iters times. */
int mmsbm_iterate(mmsbm_ctx *ctx, double *theta, double *pr, int32_t n_iters, void *stream);

/* Log-likelihood of link set `which` for every sample into out[B] (device).
 * Replaces Model.compute_likelihood(selected_set) (:952-974). */
int mmsbm_loglik(mmsbm_ctx *ctx, int32_t which, const double *theta, const double *pr,
                 double *out, void *stream);

/* P(r = 1) for n rows of ids int32[n][3] into out[B][n] (device); an id outside
 * [0, P) gives NaN.  Replaces Model.do_prediction (:530-547), used by
 * calculate_test_set_results (:557-569). */
int mmsbm_predict(mmsbm_ctx *ctx, const int32_t *ids, int64_t n, const double *theta,
                  const double *pr, double *out, void *stream);

/* Link-sharded iteration (single sample over N ranks): each rank's context
 * holds 1/N of the train links (mmsbm_set_links) and the GLOBAL degree (mmsbm_set_degree).
 * Step 1, the accumulation half of make_iteration (:986-1012) over this rank's links:
 *   nth[B][P][K]   = per gene, the sum of its c-scaled responsibility marginals (theta not applied)
 *   S[B][R][K^3]   = the S lattice sums,  npr = p S.
 * The caller sums nth and S over ranks (one all-reduce of one buffer), then step 2 applies the
 * M-step (:1016-1028): theta <- theta nth / deg, p_r <- p_r S_r / (eps + sum_r p_r S_r).
 * Called on one rank with all links, the pair equals mmsbm_iterate(n = 1). */
int mmsbm_accumulate(mmsbm_ctx *ctx, const double *theta, const double *pr, double *nth, double *S,
                     void *stream);
int mmsbm_mstep(mmsbm_ctx *ctx, double *theta, double *pr, const double *nth, const double *S,
                void *stream);

/* Joint digenic + trigenic model (include/mmsbm_pairs.h): nth_add[B][P][K] (device; NULL = none)
 * is added to every gene's triplet sums before the division by the counter in mmsbm_iterate
 * (the pair loop's ntheta, :1608-1642 of src/TrigenicInteractionPredictor_23.py), and to nth in
 * mmsbm_accumulate.  The pointer is read at every launch; it stays set until replaced. */
int mmsbm_set_theta_addend(mmsbm_ctx *ctx, const double *nth_add);

/* Measurement: info[16] = observations, plan rows (3 streams on the small-K plans, stream 0 on the
 * large-K ones), stream-0 rows, stream-0 workgroups, stream-1/2 workgroups, S partials, partial
 * rows, most genes per stream-0 workgroup (per unit for the small-K plan), V tables computed per
 * iteration, stream-0 partial rows, 1 if the plan is the small-K one (K <= 12, sk.h; 2: with the
 * fused E-step launch, pass A then runs all three streams and pass B is empty; 0: the large-K
 * kernels), units (waves of work), [12] the compute-unit count the fused plan sized its units
 * from (0: the plan does not depend on it), [13] that plan's unit target, [14] Y entries of the
 * large-K plan (2 per observation), [15] the large-K gm_kernel's workgroups per S part for the
 * current active batch (1 or 2; it follows the batch, the bits do not: its X rows are formed in
 * two fixed halves either way; 0 on the small-K plans).  The fused plan's unit length, and so the
 * order of its sums, follows [12]: results are bitwise reproducible on one device model /
 * partition mode. */
int mmsbm_plan_info(const mmsbm_ctx *ctx, int32_t which, int64_t *info);

/* Kernel timing for measurement (bench.py): with stride n > 0, mmsbm_iterate records a HIP
 * event pair on the launch stream around every kernel of every n-th iteration (kernel ids:
 * 0 = pass A (large-K: stream 0 + Y entries; fused small-K: the whole E-step), 1 = the large-K
 * gene kernel (x0, S partials, Y sums) / the small-K pass B, 2 = fin (theta / p update));
 * 0 disables.  mmsbm_timing resets the counters; mmsbm_timing_result waits for the last event
 * and returns the summed device time (ms) and the number of timed launches of that kernel. */
int mmsbm_timing(mmsbm_ctx *ctx, int32_t stride);
int mmsbm_timing_result(mmsbm_ctx *ctx, int32_t kernel, double *total_ms, int64_t *count);

/* Measurement: n back-to-back launches of kernel `kernel` (ids as above) on the current theta /
 * pr, between one HIP event pair on `stream`; *avg_ms = elapsed / n.  The passes only read
 * theta / pr and fin runs in its sums-out mode into workspace scratch, so the parameters are
 * unchanged.  Synchronises the stream. */
int mmsbm_time_kernel(mmsbm_ctx *ctx, int32_t kernel, double *theta, double *pr, int32_t n,
                      void *stream, double *avg_ms);

#ifdef __cplusplus
}
#endif
#endif /* MMSBM_H */
