/* mmsbm_io.h — native fold-file ingestion (host C++, libmmsbm_io.so).
 *
 * Replaces the per-line Python loop of Model.get_traintest
 * (AleixMT/TrigenicInteractionPredictor, src/TrigenicInteractionPredictor.py:321-423) for
 * large link sets: one pass over each file, the same gene id
 * assignment (first appearance, train file first, then test), the same per-gene interaction
 * counts (`uniqueg`), the same link keys (ids sorted as decimal STRINGS, :349-358) in the same
 * first-appearance order, and the same per-rating counts.
 *
 * The native reader takes the canonical fold format only: printable ASCII + TAB, '\n' line
 * ends, three '_'-separated genes, a rating field that Python's int() reads as 0 or 1.  Any
 * other input (other line ends or bytes, another number of genes, a missing or unparsable
 * rating, ratings other than 0/1, an unreadable file) returns MMSBM_IO_FALLBACK, and the caller
 * runs the reference-semantics Python reader, which reproduces the reference's exceptions and
 * messages for those inputs.
 */
#ifndef MMSBM_IO_H
#define MMSBM_IO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMSBM_IO_OK 0
#define MMSBM_IO_FALLBACK 1   /* input outside the native fast path: use the Python reader */
#define MMSBM_IO_INVALID (-1) /* bad arguments */

typedef struct mmsbm_fold mmsbm_fold;

/* Parse train then test (:321-423).  On MMSBM_IO_OK *out owns the result. */
int mmsbm_fold_parse(const char *train_path, const char *test_path, mmsbm_fold **out);

/* Sizes for the export buffers: genes P, unique train / test links, bytes of the gene-name
 * block (names in id order, each followed by a '\0'), train lines (for `uniqueg` checks). */
int mmsbm_fold_sizes(const mmsbm_fold *f, int64_t *P, int64_t *E_train, int64_t *E_test,
                     int64_t *names_bytes);

/* Copy out: names[names_bytes]; uniqueg int32[P] (:339-341); train_ids int32[E_train][3] and
 * test_ids int32[E_test][3] in key order (the reference's 'i_j_k' key split into ints);
 * train_counts / test_counts int32[E][2] (:361-366, :404-408), rows in first-appearance order. */
int mmsbm_fold_export(const mmsbm_fold *f, char *names, int32_t *uniqueg, int32_t *train_ids,
                      int32_t *train_counts, int32_t *test_ids, int32_t *test_counts);

void mmsbm_fold_free(mmsbm_fold *f);

#ifdef __cplusplus
}
#endif

#endif /* MMSBM_IO_H */
