/*
 * imsame_dev.h -- C-ABI drop-in boundary of the MI355X seed-and-extend path.
 *
 * Plain C types only (no HIP / torch types).  The reference has no plugin
 * API: its seam for this path is the pthread worker
 *     void *computeAlignmentsByThread(void *HashTableArgs)
 *         /root/reference/src/alignmentFunctions.h:51 (decl), .c:43-208 (body)
 * fed by the index built inline in main()
 *         /root/reference/src/IMSAME.c:194-289 (DB load + 12-mer insert)
 * and the stand-alone tool
 *         /root/reference/src/reverseComplement.c:21-118.
 * Each entry point below names the reference code it replaces.
 *
 * Ownership: the caller owns every host buffer (borrowed for the call);
 * the context owns device copies, the index and scratch.  One host thread
 * per context; contexts on different devices may run concurrently.
 * Errors are returned as negative IMSAME_E_* codes -- the library never
 * calls exit() (the reference's terror() does, commonFunctions.c:10-13);
 * the CLI maps codes back onto the reference's fatal messages.
 */
#ifndef IMSAME_DEV_H
#define IMSAME_DEV_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IMSAME_OK                 0
#define IMSAME_E_HIP             -1   /* HIP runtime error / no device              */
#define IMSAME_E_OOM             -2   /* device or host allocation failed           */
#define IMSAME_E_READ_TOO_LONG   -3   /* xlen or ylen > max_read_size on an e-value
                                         passing hit: the reference's terror(
                                         "Read size reached for gapped alignment.")
                                         alignmentFunctions.c:155                   */
#define IMSAME_E_ARG             -4   /* bad argument                                */
#define IMSAME_E_RANGE           -5   /* gap parameters could overflow int32 scores  */
#define IMSAME_E_PATHS           -6   /* path arena too small (retry with more)      */
#define IMSAME_E_STATE           -7   /* index / query not loaded                    */

/* Reference constants restated (structs.h:13-19). */
#define IMSAME_FIXED_K        12
#define IMSAME_POINT           4
#define IMSAME_MAX_READ_SIZE 3000
#define IMSAME_ALIGN_LEN      60

/* Alignment parameters, same meaning and defaults as IMSAME.c:44-49 /
 * init_args (IMSAME.c:520-578).  igap/egap are the NEGATIVE values the
 * reference uses internally (CLI "-igap 5" => igap = -5). */
typedef struct imsame_params {
    long double min_e;          /* e-value threshold: pass iff e <  min_e   */
    long double min_coverage;   /* accept iff len/ylen    >= min_coverage  */
    long double min_identity;   /* accept iff ident/len   >= min_identity  */
    int64_t     igap;
    int64_t     egap;
    uint64_t    max_read_size;  /* IMSAME_MAX_READ_SIZE unless raised (C5)  */
    uint32_t    want_paths;     /* 1: return alignment paths of accepted reads */
    uint32_t    flags;          /* IMSAME_FLAG_* (0 = defaults)                 */
} imsame_params;

/* flags: force the int32 NW kernel even where the packed int16 one fits,
 * or the packed kernel for every launch it fits however few candidates it
 * has (by default launches of < 3000 candidates take the int32 kernel: lower
 * latency).  Results are identical; the tests use both to cover both kernels. */
#define IMSAME_FLAG_NW32 1u
#define IMSAME_FLAG_NW16 2u
/* the packed kernel in ONE pass (traceback of every row) instead of its
 * default two passes (score-only sweep + a traceback band under the best
 * cell, nw16_kernel.hip).  Results are identical. */
#define IMSAME_FLAG_NW16_ONEPASS 4u

/* Fill the reference defaults: min_e = 1/powl(10,20), cov = id = 0.5,
 * igap = -5, egap = -2, max_read_size = 3000, want_paths = 0. */
void imsame_params_default(imsame_params *p);

/* Per-read outcome, 64 bytes.  For an accepted read the fields describe the
 * FIRST accepted (read, db record) pair in the reference's visiting order
 * (alignmentFunctions.c:91-195); for other reads only ylen is set. */
typedef struct imsame_read_result {
    uint64_t db_seq;        /* accepted database record (global 0-based index) */
    int64_t  score;         /* best cell score  (NW bc.score)                   */
    uint32_t bx, by;        /* best cell        (bc.xpos, bc.ypos)              */
    uint32_t length;        /* BasicAlignment.length                            */
    uint32_t identities;    /* BasicAlignment.identities                        */
    uint32_t igaps, egaps;  /* BasicAlignment.igaps / egaps                     */
    uint32_t head_x, head_y;/* backtrackingNW ret_head_x / ret_head_y           */
    uint32_t ylen;          /* read length                                      */
    uint32_t status;        /* 0 = not found, 1 = accepted                      */
    uint32_t path_off;      /* first entry of this read's path in the arena     */
    uint32_t path_len;      /* number of path entries (0 if none)               */
} imsame_read_result;

/* A path is the backtrack of the accepted alignment, walked from the best
 * cell towards the origin (backtrackingNW order), as u32 runs:
 *   bits 31..30 = move (IMSAME_MOVE_*), bits 29..0 = run length / jump size. */
#define IMSAME_MOVE_DIAG 0u   /* n diagonal steps: X[px],Y[py] pairs           */
#define IMSAME_MOVE_UP   1u   /* one jump of n rows: X[px..px-n+1] vs '-'      */
#define IMSAME_MOVE_LEFT 2u   /* one jump of n cols: '-' vs Y[py..py-n+1]      */

#define IMSAME_LAUNCH_STATS 64
typedef struct imsame_stats {
    uint64_t n_reads;       /* reads processed                       */
    uint64_t n_accepted;    /* reads accepted                        */
    uint64_t n_nw;          /* gapped alignments computed            */
    uint64_t nw_cells;      /* sum xlen*ylen over computed NW         */
    uint64_t n_hits;        /* ungapped extensions evaluated          */
    uint64_t rounds;        /* seed->NW rounds                        */
    uint64_t err_read;      /* IMSAME_E_READ_TOO_LONG: offending read */
    uint64_t err_dbseq;     /* ... and database record                */
    double   ms_seed;       /* device time in seed/ungapped kernels   */
    double   ms_nw;         /* device time in NW kernels              */
    double   ms_total;      /* wall time of imsame_dev_align          */
    double   nw_launch_ms;  /* average NW kernel launch duration      */
    uint64_t nw_launches;
    uint64_t nw_bytes;      /* 2 B per NW cell (traceback floor) */
    /* per NW launch, in launch order (first IMSAME_LAUNCH_STATS launches):
     * candidates (read, record) pairs aligned and device milliseconds */
    uint64_t launch_cand[IMSAME_LAUNCH_STATS];
    double   launch_ms[IMSAME_LAUNCH_STATS];
    uint64_t n_rewalk;      /* accepted reads whose path overflowed the device
                               arena and was re-walked (want_paths)      */
    double   ms_setup;      /* host: tables, buffers, until the first kernel */
    double   ms_d2h;        /* results (64 B per read) device -> host        */
    double   ms_nw_busy;    /* wall time the device ran NW launches (union of
                               the launch intervals of all lanes)        */
    uint64_t lanes;         /* concurrent lanes the call ran (1-8)     */
    uint64_t nw_redo;       /* two-pass NW: second-sweep retries of waves whose
                               traceback band missed a path (4 bands, then
                               from row 1)                                  */
    uint64_t launch_pk;     /* bit k: NW launch k ran the packed int16 kernel
                               (nw16_kernel), else the int32 nw_kernel     */
    uint64_t nw_win;        /* two-pass NW: candidates whose path was walked in
                               the first sweep's predicted traceback window  */
    double   ms_nw_first;   /* first NW launch start / last NW launch end, ms
                               after the call's first device operation     */
    double   ms_nw_last;
    uint64_t launch_k5;     /* bit k: packed NW launch k ran 5 columns per lane
                               (latency-bound launches), else 10           */
    uint64_t launch_np;     /* bit k: NW launch k was non-persistent (one wave
                               per task, arena slots per XCD)             */
    uint64_t launch_k19;    /* bit k: packed NW launch k ran the 19-column
                               form (8 lanes per pair, reads of one length
                               150: every lane of the wave busy)          */
    uint64_t launch_nwp;    /* bit k: NW launch k ran the packed long-read
                               kernel (two long reads per wave, int16
                               halves in per-lane frames)                 */
    uint64_t nw_fallback;   /* packed long-read waves whose values left the
                               int16 range proof: their pairs ran the int32
                               long-read path instead (same results)      */
    uint64_t seed_windows;  /* seed scan work (seed roofline): k-mer windows
                               probed (two CSR offsets each), CSR entries
                               read, 16-byte chunk pairs (database + query)
                               loaded by ungapped extensions              */
    uint64_t seed_entries;
    uint64_t seed_ext_chunks;
    uint64_t nw_spec_waste; /* NW work the reference never does: candidates a
                               read emitted past the one it accepted (speculation,
                               round_policy.h).  n_nw - nw_spec_waste are the
                               distinct (read, record) pairs of the reference's
                               NW calls (alignmentFunctions.c:126-186), which
                               also repeats a rejected record at each of its
                               e-value-passing hits                        */
    uint64_t launch_k3;     /* bit k: packed NW launch k ran the 3-column
                               latency form (one pair per wave, 50 lanes at
                               150 bp: the fewest instructions per row step) */
} imsame_stats;

typedef struct imsame_ctx imsame_ctx;

/* Number of visible HIP devices (0 without a GPU).  The reference has no
 * device notion; the all-vs-all driver uses it to pick its shard count. */
int  imsame_dev_count(void);

/* Open device `device` (HIP ordinal).  Fails with IMSAME_E_HIP if no GPU.
 * Several contexts may be opened on one device (each owns its own streams
 * and buffers).  A context runs a large imsame_dev_align call as up to 8
 * concurrent lanes, one per hardware queue: the library reads
 * GPU_MAX_HW_QUEUES (HIP's default 4 when unset) once and never changes it.
 * A host program that wants 8 lanes sets GPU_MAX_HW_QUEUES=8 (<= 32) in its
 * environment before its first HIP call (the imsame CLI and bench.py do);
 * results never depend on it. */
int  imsame_dev_open(int device, imsame_ctx **out);
void imsame_dev_close(imsame_ctx *ctx);
const char *imsame_strerror(int code);

/* Replaces the 12-mer insert loop IMSAME.c:232-281 (Container + llpos pools,
 * alignmentFunctions.h:4-6, structs.h:26-30): builds the direct-address
 * 4^12 bucket index in HBM (CSR; hits visited in the reference's LIFO order).
 *   db_seq   : ACGT-filtered concatenation (IMSAME.c:216-221), db_len bases
 *   db_start : n_db record starts (IMSAME.c:200)
 *   db_brk   : optional bitmap, bit p (LSB-first) = k-mer reset before base p
 *              (non-ACGT, non-'\n' byte: IMSAME.c:229-231); record starts are
 *              resets implicitly.  NULL = none besides record starts.
 * Sizes: db_len is u64 (databases past 4 Gbases index with 8-byte entries
 * {pos - record start, record}); n_db and each record's length must be
 * below 2^32 - 16 (IMSAME_E_ARG).  HBM: db_len x 5 B during the build,
 * plus 8 B per k-mer and 128 MB of bucket offsets.
 * Bases: db_seq (and every query below) holds only the bytes 'A', 'C', 'G',
 * 'T' -- what IMSAME's loaders keep (toupper, then drop the rest).  The seed
 * stage compares 2-bit codes, which alias every other byte to one of them, so
 * the build checks every byte and returns IMSAME_E_ARG on any other one;
 * imsame_dev_align* do the same for the bytes of the reads they align (the
 * check runs inside the query's 2-bit packing kernel). */
int imsame_dev_index(imsame_ctx *ctx, const uint8_t *db_seq, uint64_t db_len,
                     const uint64_t *db_start, uint64_t n_db, const uint8_t *db_brk);

/* Upload the query (IMSAME.c:320-371 output): ACGT-filtered concatenation
 * and n_q read starts. */
int imsame_dev_set_query(imsame_ctx *ctx, const uint8_t *q_seq, uint64_t q_len,
                         const uint64_t *q_start, uint64_t n_q);

/* imsame_dev_set_query for a SHARD: the host arrays are the whole query (as
 * the loader produced it), but only reads [read_from, read_to) -- their
 * bases, one preceding base (a read borrows the previous read's last base,
 * SURVEY Appendix A Q4) and their starts -- are copied to HBM.  Chunk heads
 * keep the whole query's meaning (IMSAME.c:414: i*floor(n_q/T)), so
 * imsame_dev_align over any sub-range of the shard gives the per-read
 * results of a run over the whole query.  This is the per-GPU upload of a
 * multi-GPU run: each device receives 1/N of the query. */
int imsame_dev_set_query_range(imsame_ctx *ctx, const uint8_t *q_seq, uint64_t q_len,
                               const uint64_t *q_start, uint64_t n_q,
                               uint64_t read_from, uint64_t read_to);

/* imsame_dev_set_query_range without waiting for the copies: they are queued
 * in parts on the context's stream, and each internal lane of the next
 * imsame_dev_align* starts as soon as the parts holding its reads are in HBM,
 * so the upload overlaps the first lanes' seed scans.  q_seq must stay valid
 * and unchanged until that call (or imsame_dev_sync) returns; it should be
 * page-locked (imsame_host_alloc) for the copies to run asynchronously. */
int imsame_dev_set_query_range_async(imsame_ctx *ctx, const uint8_t *q_seq, uint64_t q_len,
                                     const uint64_t *q_start, uint64_t n_q,
                                     uint64_t read_from, uint64_t read_to);

/* Wait for the context's queued work (an asynchronous query upload). */
int imsame_dev_sync(imsame_ctx *ctx);

/* Replaces T x computeAlignmentsByThread (alignmentFunctions.c:43-208) over
 * reads [read_from, read_to) of the loaded query (inside the uploaded range).  n_threads_semantic is the
 * reference's -n_threads: it fixes the chunk heads {i*floor(n/T)}
 * (IMSAME.c:414,430-452) whose first k-mer does not borrow the previous
 * read's last base, so results equal the reference's
 * for that -n_threads.  res[k] describes read read_from+k.  paths/paths_cap:
 * u32 arena for want_paths (may be NULL when want_paths == 0).  The device
 * keeps its own arena, sized to what the alignments need (paths that
 * overflow it are re-walked for exactly the reads concerned, never the whole
 * call).  On ANY return, *paths_used > paths_cap means the paths were NOT
 * copied and wait on the device: the call returns IMSAME_E_PATHS with res[]
 * complete -- or IMSAME_E_READ_TOO_LONG, which takes precedence, with res[]
 * complete below the offending read -- so callers compare *paths_used with
 * paths_cap whatever the code, grow the host arena and call
 * imsame_dev_fetch_paths.
 * A call over short reads is cut into up to 8 parts ("lanes") that run
 * concurrently on their own streams (internal contexts sharing the index
 * and the query): one lane per 40,000 reads, at most one per hardware queue
 * (GPU_MAX_HW_QUEUES, see imsame_dev_open).  Results do not depend on it
 * (IMSAME_LANES=n forces n lanes, 1 turns it off). */
int imsame_dev_align(imsame_ctx *ctx, uint64_t read_from, uint64_t read_to,
                     uint64_t n_threads_semantic, const imsame_params *prm,
                     imsame_read_result *res, uint32_t *paths, uint64_t paths_cap,
                     uint64_t *paths_used, imsame_stats *stats);

/* imsame_dev_align that hands the results over as they become final -- the
 * reference's workers write each accepted record as soon as it is found
 * (alignmentFunctions.c:165-168), so its output starts long before the last
 * thread joins (IMSAME.c:460-462).  The call runs its lanes as
 * imsame_dev_align does and, as soon as lane k's reads [a, b) are final,
 * calls part(user, a, b, status, err_read, paths, n_paths) from that lane's
 * host thread: res[a - read_from .. b - read_from) are complete, and when
 * prm->want_paths their path_off index `paths` (n_paths entries, valid
 * during the callback only).  status: IMSAME_OK, IMSAME_E_READ_TOO_LONG (rows
 * below err_read are complete) or another IMSAME_E_* code.  The parts cover
 * [read_from, read_to) exactly, arrive in any order and may run
 * concurrently; the call returns when every part's callback has returned,
 * with the first failure it saw (IMSAME_E_PATHS never: the paths go through
 * the callbacks; imsame_dev_fetch_paths does not apply). */
typedef void (*imsame_part_fn)(void *user, uint64_t read_from, uint64_t read_to, int status, uint64_t err_read,
                               const uint32_t *paths, uint64_t n_paths);
int imsame_dev_align_parts(imsame_ctx *ctx, uint64_t read_from, uint64_t read_to, uint64_t n_threads_semantic,
                           const imsame_params *prm, imsame_read_result *res, imsame_part_fn part, void *user,
                           imsame_stats *stats);

/* imsame_dev_align on the loaded index when it holds ONE SLICE (whole
 * records) of a larger database: ev_db_len is the whole database's length
 * for the e-value (0 = the loaded index's), win_cap[k] (host, may be NULL)
 * limits read read_from+k to windows p < win_cap[k] (p = query position of
 * the k-mer's last base, the reference's curr_pos), win_start[k] (host, may
 * be NULL) makes its scan begin at window max(first, win_start[k]), and win[k] (host, out)
 * receives the window of each accepted read's hit (~0 if none).  res[k].db_seq
 * is slice-local.  For a database cut into slices s = 0, 1, ... from its
 * highest records down, the reference's first accepted pair is, per read,
 * the accepted result with the smallest (win, s): slices on one GPU
 * (imsame_dev_align_sliced) or shards across GPUs (a min all-reduce). */
int imsame_dev_align_windows(imsame_ctx *ctx, uint64_t read_from, uint64_t read_to,
                             uint64_t n_threads_semantic, const imsame_params *prm, uint64_t ev_db_len,
                             const uint64_t *win_start, const uint64_t *win_cap,
                             imsame_read_result *res, uint64_t *win,
                             uint32_t *paths, uint64_t paths_cap, uint64_t *paths_used,
                             imsame_stats *stats);

/* imsame_dev_align against a database whose index is built and searched in
 * slices of at most slice_bases bases (whole records; a record longer than
 * that is a slice of its own), one slice's index in HBM at a time: the
 * memory-capped multi-pass form of IMSAME.c:232-281 + the worker.  Results
 * (db_seq global) equal imsame_dev_align over the whole database (the
 * e-value uses the whole db_len).  Slices run from the highest records down
 * (a bucket's LIFO order, IMSAME.c:255-276); a read accepted at window w
 * scans only windows < w of later slices.  Two phases: every slice over each
 * read's first windows (where most reads accept, and where the smallest key
 * is final), then the rest for reads still open.  Restriction: every record and
 * read must fit max_read_size (the reference's size abort is not sliced):
 * IMSAME_E_ARG otherwise.  Needs a loaded query; leaves the last slice's
 * index loaded.  n_slices (may be NULL) receives the slice count. */
int imsame_dev_align_sliced(imsame_ctx *ctx, const uint8_t *db_seq, uint64_t db_len,
                            const uint64_t *db_start, uint64_t n_db, const uint8_t *db_brk,
                            uint64_t slice_bases, uint64_t read_from, uint64_t read_to,
                            uint64_t n_threads_semantic, const imsame_params *prm,
                            imsame_read_result *res, uint32_t *paths, uint64_t paths_cap,
                            uint64_t *paths_used, uint64_t *n_slices, imsame_stats *stats);

/* Copy the paths of the last imsame_dev_align / _align_windows /
 * _align_sliced call (after IMSAME_E_PATHS) into paths[0 .. *paths_used):
 * IMSAME_E_PATHS again if paths_cap is still too small. */
int imsame_dev_fetch_paths(imsame_ctx *ctx, uint32_t *paths, uint64_t paths_cap, uint64_t *paths_used);

/* Page-locked host memory for query/database buffers (faster H2D than
 * pageable memory); NULL without a GPU.  Free with imsame_host_free. */
void *imsame_host_alloc(uint64_t bytes);
void  imsame_host_free(void *p);

/* Unit-level entry replacing build_alignment (alignmentFunctions.c:210-274:
 * NW + backtrackingNW + identities) plus the acceptance test (:163) for
 * explicit pairs: X_k = xs[x_start[k] .. x_start[k+1]) (database record,
 * rows), Y_k likewise (read, columns); x_start/y_start have npairs+1 entries.
 * res[k].status = 1 accepted / 2 rejected.  kernel_ms: device time. */
int imsame_dev_nw_pairs(imsame_ctx *ctx, const uint8_t *xs, const uint64_t *x_start,
                        const uint8_t *ys, const uint64_t *y_start, uint64_t npairs,
                        const imsame_params *prm, imsame_read_result *res, uint32_t *paths,
                        uint64_t paths_cap, uint64_t *paths_used, double *kernel_ms);

/* Replaces reverseComplement.c:21-118: FASTA image -> records in reverse
 * order, header line kept, letters reversed and complemented (A<->T, C<->G,
 * U->A, case kept), one sequence line per record.  If out_cap is too small
 * the call returns IMSAME_E_ARG with *out_len = the size required
 * (in_len + records + 1 suffices unless headers contain '>'). */
int imsame_dev_revcomp(imsame_ctx *ctx, const uint8_t *in, uint64_t in_len,
                       uint8_t *out, uint64_t out_cap, uint64_t *out_len);

#ifdef __cplusplus
}
#endif
#endif
