/* imsame_host.h -- host-side helpers of the CLI: FASTA loading with the
 * reference's rules and .align text rendering from device paths. */
#ifndef IMSAME_HOST_H
#define IMSAME_HOST_H
#include <stdint.h>
#include <stddef.h>
#include "../../../include/imsame_dev.h"

typedef struct {
    uint8_t  *seq;     /* ACGT-filtered concatenation           */
    uint64_t *start;   /* n + 1 entries (start[n] = len)        */
    uint64_t  n, len;
    uint8_t  *brk;     /* database: k-mer reset bitmap, else NULL */
} host_seqs;

typedef struct { char *buf; size_t len, cap; } host_text;

/* IMSAME.c:194-289 (want_brk = 1, database) / :320-371 (query) */
int  host_parse_fasta(const uint8_t *b, uint64_t nb, int want_brk, host_seqs *s);
int  host_load_fasta(const char *path, int want_brk, host_seqs *s);
void host_free_seqs(host_seqs *s);

/* Same result as host_parse_fasta, parsed by up to nthreads threads over
 * pieces of at least min_piece bytes (0 = 4 MiB) cut before line-initial
 * '>' (SURVEY 8(f) row 2).  host_load_fasta uses it with host_threads(). */
#define HOST_MAX_THREADS 64
int  host_parse_fasta_mt(const uint8_t *b, uint64_t nb, int want_brk, int nthreads, uint64_t min_piece,
                         host_seqs *s);
int  host_threads(void);        /* IMSAME_HOST_THREADS, else online CPUs capped at 16 */
int  host_read_file(const char *path, uint8_t **buf, uint64_t *len);

/* backtrackingNW's strings (alignmentFunctions.c:493-560) rebuilt from a
 * device path, then build_alignment's 60-column text (:230-271).
 * Returns the identities counted by the text loop. */
uint64_t host_render(const uint8_t *X, uint64_t xlen, const uint8_t *Y, uint64_t ylen,
                     const imsame_read_result *r, const uint32_t *path, host_text *t);
/* host_render APPENDING to t, with caller-owned scratch reused across
 * records (no allocation per record once it has grown) */
uint64_t host_render_scratch(const uint8_t *X, uint64_t xlen, const uint8_t *Y, uint64_t ylen,
                             const imsame_read_result *r, const uint32_t *path, host_text *t, host_text *scratch);
/* exact byte count of the text host_render produces for r */
uint64_t host_render_size(uint64_t xlen, uint64_t ylen, const imsame_read_result *r);

#endif
