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

/* make_iteration, :984-1043.  Returns 0, or -1 when a gene has zero degree
 * (the reference raises ZeroDivisionError at :1018; nothing is modified). */
int oracle_make_iteration(int64_t E, const int32_t *ids, const int32_t *counts,
                          int P, int K, int R, double eps, double *theta, double *pr)
{
    const int64_t K3 = (int64_t)K * K * K;
    double *nth = calloc((size_t)P * K, sizeof(double));
    double *npr = calloc((size_t)K3 * R, sizeof(double));
    int64_t *deg = calloc((size_t)P, sizeof(int64_t));
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
    for (int g = 0; g < P; ++g)
        if (deg[g] == 0) { free(nth); free(npr); free(deg); return -1; }
    for (int g = 0; g < P; ++g)
        for (int a = 0; a < K; ++a) nth[(int64_t)g * K + a] /= (double)deg[g];
    for (int64_t cell = 0; cell < K3; ++cell) {
        double s = eps;
        for (int r = 0; r < R; ++r) s += npr[cell * R + r];
        for (int r = 0; r < R; ++r) npr[cell * R + r] /= s;
    }
    memcpy(theta, nth, sizeof(double) * (size_t)P * K);
    memcpy(pr, npr, sizeof(double) * (size_t)K3 * R);
    free(nth); free(npr); free(deg);
    return 0;
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
