/* ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into the product path.
 *
 * Plain-C restatement of the reference MMSBM EM path
 * (AleixMT/TrigenicInteractionPredictor, src/TrigenicInteractionPredictor.py).
 * Same loop order and the same binary64 operation order as the reference
 * (compiled with -ffp-contract=off, no fast-math), so it is bit-identical to
 * the reference under CPython and to oracle/mmsbm_oracle.py; this is checked
 * against the golden fixtures in tests/test_oracle_golden.py and
 * tests/test_oracle_c.py.  It exists because the pure-Python oracle needs
 * ~2 us x K^3 per link; the C one checks fold0-sized inputs in seconds.
 *
 * Layouts (host memory):
 *   ids    int32[E][3]  gene ids of each link in `links` dict order, slots in
 *                       the reference's string-sorted key order (:349-358)
 *   counts int32[E][R]  rating counts n_r (:360-368)
 *   theta  f64[P][K]    (:117-121)
 *   pr     f64[K][K][K][R] (:124-139)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* compute_likelihood, :952-974 */
double oracle_loglik(int64_t E, const int32_t *ids, const int32_t *counts,
                     int K, int R, double eps, const double *theta, const double *pr)
{
    double total = 0.0;
    double d[16];
    for (int64_t e = 0; e < E; ++e) {
        const double *t1 = theta + (int64_t)ids[3 * e + 0] * K;
        const double *t2 = theta + (int64_t)ids[3 * e + 1] * K;
        const double *t3 = theta + (int64_t)ids[3 * e + 2] * K;
        for (int r = 0; r < R; ++r) d[r] = eps;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b)
                for (int c = 0; c < K; ++c) {
                    const double *cell = pr + (((int64_t)a * K + b) * K + c) * R;
                    for (int r = 0; r < R; ++r) d[r] += t1[a] * t2[b] * t3[c] * cell[r];
                }
        for (int r = 0; r < R; ++r) total += (double)counts[e * R + r] * log(d[r]);
    }
    return total;
}

/* Per-link loop of :986-1012, adding into nth[P][K], npr[K^3][R], deg[P]. */
static void tri_accumulate(int64_t E, const int32_t *ids, const int32_t *counts, int K, int R,
                           double eps, const double *theta, const double *pr, double *nth,
                           double *npr, int64_t *deg)
{
    double d[16];
    for (int64_t e = 0; e < E; ++e) {
        const int g1 = ids[3 * e + 0], g2 = ids[3 * e + 1], g3 = ids[3 * e + 2];
        const double *t1 = theta + (int64_t)g1 * K;
        const double *t2 = theta + (int64_t)g2 * K;
        const double *t3 = theta + (int64_t)g3 * K;
        const int32_t *n = counts + e * R;
        deg[g1] += 1; deg[g2] += 1; deg[g3] += 1;
        for (int r = 0; r < R; ++r) d[r] = eps;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b)
                for (int c = 0; c < K; ++c) {
                    const double *cell = pr + (((int64_t)a * K + b) * K + c) * R;
                    for (int r = 0; r < R; ++r) d[r] += t1[a] * t2[b] * t3[c] * cell[r];
                }
        double *n1 = nth + (int64_t)g1 * K, *n2 = nth + (int64_t)g2 * K, *n3 = nth + (int64_t)g3 * K;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b)
                for (int c = 0; c < K; ++c) {
                    const int64_t cidx = (((int64_t)a * K + b) * K + c) * R;
                    for (int r = 0; r < R; ++r) {
                        const double w = (t1[a] * t2[b] * t3[c] * pr[cidx + r]) / d[r];
                        const double nr = (double)n[r];
                        n1[a] += w * nr;
                        n2[b] += w * nr;
                        n3[c] += w * nr;
                        npr[cidx + r] += w * nr;
                    }
                }
    }
}

/* The accumulation half of make_iteration (:986-1012) over a subset of the links, adding into
 * nth[P][K] and npr[K^3][R] (zeroed by the caller): the sums a gene's theta' needs (:1016-1018)
 * are complete when every link holding the gene is in the subset (tests: config-5 genes checked
 * at full size, with the degree counted over all links). */
void oracle_accumulate(int64_t E, const int32_t *ids, const int32_t *counts, int P, int K, int R,
                       double eps, const double *theta, const double *pr, double *nth, double *npr)
{
    int64_t *deg = calloc((size_t)P, sizeof(int64_t));
    tri_accumulate(E, ids, counts, K, R, eps, theta, pr, nth, npr, deg);
    free(deg);
}

/* cells[n][R] <- cells / (eps + sum_r cells), :1021-1028 */
static void normalise_cells(int64_t n, int R, double eps, double *cells)
{
    for (int64_t cell = 0; cell < n; ++cell) {
        double s = eps;
        for (int r = 0; r < R; ++r) s += cells[cell * R + r];
        for (int r = 0; r < R; ++r) cells[cell * R + r] /= s;
    }
}

/* make_iteration, :984-1043.  Returns 0, or -1 when a gene has zero degree
 * (the reference raises ZeroDivisionError at :1018; nothing is modified). */
int oracle_make_iteration(int64_t E, const int32_t *ids, const int32_t *counts,
                          int P, int K, int R, double eps, double *theta, double *pr)
{
    const int64_t K3 = (int64_t)K * K * K;
    double *nth = calloc((size_t)P * K, sizeof(double));
    double *npr = calloc((size_t)K3 * R, sizeof(double));
    int64_t *deg = calloc((size_t)P, sizeof(int64_t));
    tri_accumulate(E, ids, counts, K, R, eps, theta, pr, nth, npr, deg);
    for (int g = 0; g < P; ++g)
        if (deg[g] == 0) { free(nth); free(npr); free(deg); return -1; }
    for (int g = 0; g < P; ++g)
        for (int a = 0; a < K; ++a) nth[(int64_t)g * K + a] /= (double)deg[g];
    normalise_cells(K3, R, eps, npr);
    memcpy(theta, nth, sizeof(double) * (size_t)P * K);
    memcpy(pr, npr, sizeof(double) * (size_t)K3 * R);
    free(nth); free(npr); free(deg);
    return 0;
}

/* ---- joint digenic + trigenic model, src/TrigenicInteractionPredictor_23.py ----
 * pair links: ids2 int32[E2][2] (`dlinks` keys, string-sorted ids), counts2 int32[E2][R],
 * qr f64[K][K][R] (:163-174). */

/* compute_likelihood's pair loop, :1549-1559, continuing the running sum `start` of the
 * triplet loop (:1535-1547) */
double oracle_pair_loglik(int64_t E, const int32_t *ids, const int32_t *counts,
                          int K, int R, double eps, const double *theta, const double *qr,
                          double start)
{
    double total = start;
    double d[16];
    for (int64_t e = 0; e < E; ++e) {
        const double *t1 = theta + (int64_t)ids[2 * e + 0] * K;
        const double *t2 = theta + (int64_t)ids[2 * e + 1] * K;
        for (int r = 0; r < R; ++r) d[r] = eps;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b) {
                const double *cell = qr + ((int64_t)a * K + b) * R;
                for (int r = 0; r < R; ++r) d[r] += t1[a] * t2[b] * cell[r];
            }
        for (int r = 0; r < R; ++r) total += (double)counts[e * R + r] * log(d[r]);
    }
    return total;
}

/* make_iteration of the joint model, :1572-1687: the triplet loop, the pair loop (:1608-1635)
 * into the same ntheta / counter, then theta, pr and qr normalised.  -1 on a zero degree. */
int oracle_joint_make_iteration(int64_t E3, const int32_t *ids3, const int32_t *counts3,
                                int64_t E2, const int32_t *ids2, const int32_t *counts2,
                                int P, int K, int R, double eps, double *theta, double *pr,
                                double *qr)
{
    const int64_t K2 = (int64_t)K * K, K3 = K2 * K;
    double *nth = calloc((size_t)P * K, sizeof(double));
    double *npr = calloc((size_t)K3 * R, sizeof(double));
    double *nqr = calloc((size_t)K2 * R, sizeof(double));
    int64_t *deg = calloc((size_t)P, sizeof(int64_t));
    double d[16];
    tri_accumulate(E3, ids3, counts3, K, R, eps, theta, pr, nth, npr, deg);
    for (int64_t e = 0; e < E2; ++e) {
        const int g1 = ids2[2 * e + 0], g2 = ids2[2 * e + 1];
        const double *t1 = theta + (int64_t)g1 * K;
        const double *t2 = theta + (int64_t)g2 * K;
        const int32_t *n = counts2 + e * R;
        deg[g1] += 1; deg[g2] += 1;
        for (int r = 0; r < R; ++r) d[r] = eps;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b) {
                const double *cell = qr + ((int64_t)a * K + b) * R;
                for (int r = 0; r < R; ++r) d[r] += t1[a] * t2[b] * cell[r];
            }
        double *n1 = nth + (int64_t)g1 * K, *n2 = nth + (int64_t)g2 * K;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b) {
                const int64_t cidx = ((int64_t)a * K + b) * R;
                for (int r = 0; r < R; ++r) {
                    const double w = (t1[a] * t2[b] * qr[cidx + r]) / d[r];
                    const double nr = (double)n[r];
                    n1[a] += w * nr;
                    n2[b] += w * nr;
                    nqr[cidx + r] += w * nr;
                }
            }
    }
    for (int g = 0; g < P; ++g)
        if (deg[g] == 0) { free(nth); free(npr); free(nqr); free(deg); return -1; }
    for (int g = 0; g < P; ++g)
        for (int a = 0; a < K; ++a) nth[(int64_t)g * K + a] /= (double)deg[g];
    normalise_cells(K3, R, eps, npr);
    normalise_cells(K2, R, eps, nqr);
    memcpy(theta, nth, sizeof(double) * (size_t)P * K);
    memcpy(pr, npr, sizeof(double) * (size_t)K3 * R);
    memcpy(qr, nqr, sizeof(double) * (size_t)K2 * R);
    free(nth); free(npr); free(nqr); free(deg);
    return 0;
}

/* do_prediction of a pair, :957-962 (rating 1, no epsilon) for each of E pairs. */
void oracle_pair_predict(int64_t E, const int32_t *ids, int K, int R,
                         const double *theta, const double *qr, double *out)
{
    for (int64_t e = 0; e < E; ++e) {
        const double *t1 = theta + (int64_t)ids[2 * e + 0] * K;
        const double *t2 = theta + (int64_t)ids[2 * e + 1] * K;
        double p = 0.0;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b)
                p += t1[a] * t2[b] * qr[((int64_t)a * K + b) * R + 1];
        out[e] = p;
    }
}

/* do_prediction, :530-547 (rating 1, no epsilon) for each of E links. */
void oracle_predict(int64_t E, const int32_t *ids, int K, int R,
                    const double *theta, const double *pr, double *out)
{
    for (int64_t e = 0; e < E; ++e) {
        const double *t1 = theta + (int64_t)ids[3 * e + 0] * K;
        const double *t2 = theta + (int64_t)ids[3 * e + 1] * K;
        const double *t3 = theta + (int64_t)ids[3 * e + 2] * K;
        double p = 0.0;
        for (int a = 0; a < K; ++a)
            for (int b = 0; b < K; ++b)
                for (int c = 0; c < K; ++c)
                    p += t1[a] * t2[b] * t3[c] * pr[(((int64_t)a * K + b) * K + c) * R + 1];
        out[e] = p;
    }
}
