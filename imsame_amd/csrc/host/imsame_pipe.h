/* imsame_pipe.h -- one IMSAME run over G device contexts, shared by the
 * imsame CLI and the all-vs-all driver.
 *
 * The reference fans reads out to -n_threads pthreads that each write their
 * accepted records to one FILE* as they go (IMSAME.c:414-467,
 * alignmentFunctions.c:165-168).  Here reads are cut into G contiguous
 * shards, one per device context (chunk heads stay those of -n_threads over
 * the whole query); each device aligns its shard in one
 * call (or batches of batch_reads) that hands over its lanes' reads as they
 * become final, and the host renders those parts in read order with a pool
 * of threads while the devices continue.  Records land in
 * ascending read order (= the reference's -n_threads 1 file). */
#ifndef IMSAME_PIPE_H
#define IMSAME_PIPE_H
#include <stdint.h>
#include "imsame_host.h"

#define PIPE_MAX_DEV 64

typedef struct {
    int device;
    imsame_ctx *ctx;
    const host_seqs *db_now, *q_now;  /* what the context holds (avoid re-uploads) */
    uint64_t q_lo, q_hi;
} pipe_dev;

typedef struct {
    uint64_t T;                  /* -n_threads semantics                     */
    imsame_params prm;           /* want_paths is set from out_fd            */
    int out_fd;                  /* -1: no .align output                     */
    int render_threads;          /* host threads rendering (0: host_threads) */
    uint64_t batch_reads;        /* reads per device call (0: the whole shard) */
} pipe_opts;

typedef struct {
    int rc;                      /* 0, IMSAME_E_READ_TOO_LONG, or an error   */
    uint64_t stop;               /* reads [0, stop) were decided and written  */
    uint64_t accepted;           /* accepted reads among them                */
    uint64_t bytes_out, batches; /* batches: parts rendered                  */
    imsame_stats st;             /* summed over devices (ms_total: max)      */
    double t_align;              /* first align call -> last part delivered  */
    double t_render;             /* render threads' busy wall, summed per part */
    double t_write;              /* pwrite wall, summed per part             */
    double t_tail;               /* last part delivered -> output complete   */
    double t_pwrite_sum, t_pwrite_max;   /* seconds in pwrite: summed over threads, one thread's most */
    double t_wait_max;           /* IMSAME_ONE_WRITER: longest a render thread waited for the writer */
    uint64_t bytes_ok;           /* a file: bytes [0, bytes_ok) are complete (parts fully written) */
    int write_errno;             /* the first output write error (0: none)   */
} pipe_result;

/* parse "-devices" values: "N" (devices 0..N-1) or "d0,d1,..." */
int pipe_parse_devices(const char *spec, int *devs, int max);
/* open / close contexts */
int pipe_open(pipe_dev *d, const int *devs, int G);
void pipe_close(pipe_dev *d, int G);
/* index the database on every context (in parallel); no-op where held */
int pipe_index(pipe_dev *d, int G, const host_seqs *db);
/* upload shard g = [g*n/G, (g+1)*n/G) of the query to context g */
int pipe_set_query(pipe_dev *d, int G, const host_seqs *q);
/* align every read (shards as uploaded) and write the .align records */
int pipe_align_render(pipe_dev *d, int G, const host_seqs *db, const host_seqs *q, const pipe_opts *o,
                      pipe_result *r);
/* render reads [from, to) of res (paths: one arena for them) to fd at
 * *off (seekable: parallel pwrite) -- used for a single prepared batch */
int pipe_render_range(const host_seqs *db, const host_seqs *q, const imsame_read_result *res,
                      const uint32_t *paths, uint64_t from, uint64_t to, int fd, int threads, uint64_t *off,
                      pipe_result *r);
double pipe_now(void);

#endif
