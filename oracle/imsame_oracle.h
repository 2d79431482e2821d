/*
 * imsame_oracle.h -- TEST INFRASTRUCTURE: CPU restatement of IMSAME's
 * seed-and-extend path, used ONLY as the parity checker by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Nothing in the
 * product (imsame_amd/, include/) links or calls it.
 *
 * Parity of this restatement is pinned against the reference itself, compiled
 * from /root/reference/src into oracle/_ref/ (see oracle/Makefile) and frozen
 * as golden vectors under tests/golden/ (tests/golden/make_golden.py).
 */
#ifndef IMSAME_ORACLE_H
#define IMSAME_ORACLE_H
#include <stdint.h>
#include <stddef.h>
#include "../include/imsame_dev.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Result of one gapped alignment (NW + backtracking + text identities). */
typedef struct {
    int64_t  score;
    uint64_t bx, by;
    uint64_t length, identities, igaps, egaps;
    uint64_t head_x, head_y;
} or_nw_out;

/* Result of one ungapped extension (alignmentFromQuickHits). */
typedef struct {
    uint64_t x_start, y_start, t_len, raw;
    long double e_value;
    double e_value_d;     /* convenience copy for Python */
    int pass;             /* e_value < min_e */
} or_ug_out;

int or_nw(const char *X, uint64_t xlen, const char *Y, uint64_t ylen, int64_t igap, int64_t egap,
          or_nw_out *out, char *text, uint64_t text_cap, uint64_t *text_len);

int or_ungapped(const uint8_t *db, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
                const uint8_t *q, uint64_t q_len, const uint64_t *q_start, uint64_t n_q,
                uint64_t pos_db, uint64_t pos_q, uint64_t read, uint64_t dbseq,
                double min_e /* <0: reference default 1/powl(10,20) */, or_ug_out *out);

/* Whole read-vs-database pass, per-read results (same struct the device
 * returns).  db_brk: optional bitmap (1 bit per filtered DB base, LSB-first)
 * of k-mer resets, as produced by the FASTA loader; NULL = record starts only.
 * Returns 0, or IMSAME_E_READ_TOO_LONG with *err_read set. */
int or_align(const uint8_t *db, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
             const uint8_t *db_brk,
             const uint8_t *q, uint64_t q_len, const uint64_t *q_start, uint64_t n_q,
             const imsame_params *prm, uint64_t n_threads, imsame_read_result *res,
             uint64_t *err_read);

/* or_align over the reads of DISJOINT windows [from[w], to[w]) only, with the whole
 * query's chunk heads (res has n_q entries; the windows' are written). */
int or_align_windows(const uint8_t *db, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
                     const uint8_t *db_brk, const uint8_t *q, uint64_t q_len, const uint64_t *q_start, uint64_t n_q,
                     const imsame_params *prm, uint64_t n_threads, uint64_t nwin, const uint64_t *from,
                     const uint64_t *to, imsame_read_result *res, uint64_t *err_read);

/* Reverse complement of a FASTA byte image (reverseComplement.c semantics). */
int or_revcomp(const uint8_t *in, uint64_t in_len, uint8_t *out, uint64_t out_cap, uint64_t *out_len);
/* test-speed option: skip re-running NW for (read, record) pairs already
 * rejected for the read (identical results) */
void or_set_memo_rejected(int on);

void or_params_default(imsame_params *p);

/* Full CLI (IMSAME argv semantics). */
int or_main(int argc, char **argv);

#ifdef __cplusplus
}
#endif
#endif
