/*
 * imsame_cli.c -- the IMSAME command line over the MI355X C-ABI.
 *
 * Same flags, defaults, stdout lines and .align output as the reference's
 * main()/init_args() (/root/reference/src/IMSAME.c:34-578); the alignment
 * itself runs on the GPU through include/imsame_dev.h.  Records are written
 * in ascending read order -- the reference's -n_threads 1 file order; with
 * -n_threads T the record set equals the reference's (its own file
 * interleaves thread output at fprintf granularity).
 *
 * Extra flags (not in the reference): -device D, -devices N|d0,d1,... (the
 * reads are sharded over several device contexts, the multi-GPU form of the
 * reference's -n_threads fan-out, IMSAME.c:414-467), -max_read_size N (raise
 * the 3000-base NW cap of structs.h:19; the reference has it compile-time
 * only), -slice_bases N, -render_threads N, -batch_reads N.  The .align records are rendered by a thread pool as the device hands over
 * finished parts of the reads, while it aligns the rest (imsame_pipe.c).  Timing lines report wall-clock seconds (the reference
 * prints clock(), i.e. CPU time summed over threads); a JSON phase line goes
 * to stderr.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <time.h>
#include <inttypes.h>
#include "../../../include/imsame_dev.h"
#include <fcntl.h>
#include <pthread.h>
#include <unistd.h>
#include "imsame_host.h"
#include "imsame_pipe.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}
/* diagnostics: seconds since the wall-clock instant IMSAME_T_LAUNCH (set by
 * bench.py just before it starts the process), -1 without it */
static double since_launch(void) {
    const char *e = getenv("IMSAME_T_LAUNCH");
    if (!e) return -1;
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9 - atof(e);
}

/* terror(), commonFunctions.c:10-13 */
static void terror(const char *s) {
    printf("ERR**** %s ****\n", s);
    exit(-1);
}

/* The output could not be written: the parts are written in parallel into
 * ranges allocated ahead (fallocate), so a failed run would leave zero-filled
 * holes after the last complete part -- cut the file back to the bytes known
 * complete (a prefix of whole records), then fail as the reference does. */
static void out_failed(int fd, uint64_t bytes_ok) {
    if (ftruncate(fd, (off_t)bytes_ok) != 0 && errno != EINVAL && errno != ESPIPE)
        fprintf(stderr, "[imsame] could not cut the output back: %s\n", strerror(errno));
    terror("Could not write the output file");
}

/* device contexts, opened on a thread of their own (overlapping the parse) */
static pipe_dev dv_all[PIPE_MAX_DEV];
typedef struct { pipe_dev *d; const int *devs; int G, rc; double secs; } open_job;
static void *open_run(void *a) {
    open_job *j = a;
    const double t = now_s();
    j->rc = pipe_open(j->d, j->devs, j->G);
    j->secs = now_s() - t;
    return NULL;
}

static void usage(void) {
    printf("USAGE:\n");
    printf("           IMSAME -query [query] -db [database]\n");
    printf("OPTIONAL:\n");
    printf("           -n_threads  [Integer:   0<n_threads] (default 4)\n");
    printf("           -evalue     [Double:    0<=pval<1] (default: 1 * 10^-20)\n");
    printf("           -coverage   [Double:    0<coverage<=1 (default: 0.5)\n");
    printf("           -identity   [Double:    0<identity<=1 (default: 0.5)\n");
    printf("           -igap       [Integer:   (default: 5)\n");
    printf("           -egap       [Integer:   (default: 2)\n");
    printf("           -out        [File path]\n");
    printf("           --verbose   Turns verbose on\n");
    printf("           --help      Shows help for program usage\n");
    printf("           -device     [Integer: HIP device] (default 0)\n");
    printf("           -devices    [N | d0,d1,...: shard the reads over these HIP devices]\n");
    printf("           -max_read_size [Integer] (default 3000)\n");
    printf("           -slice_bases [Integer: index the database in slices of at most this many bases]\n");
    printf("           -render_threads [Integer: host threads writing the .align records]\n");
    printf("           -batch_reads [Integer: reads per device call]\n");
    exit(1);
}

int main(int argc, char **argv) {
    const double t_main = since_launch();
    /* one hardware queue per alignment lane (include/imsame_dev.h: the library
     * runs at most one lane per queue and never sets this itself); a value in
     * the environment is kept.  Before the first HIP call. */
    setenv("GPU_MAX_HW_QUEUES", "8", 0);
    const char *qpath = NULL, *dpath = NULL, *opath = NULL, *devspec = NULL;
    imsame_params prm;
    imsame_params_default(&prm);
    uint64_t T = 4;                                   /* IMSAME.c:49 */
    int device = 0, render_threads = 0;
    uint64_t slice_bases = 0, batch_reads = 0;       /* 0: one index (the reference's) */
    /* init_args, IMSAME.c:520-578 (same strcmp scan over every argv slot) */
    for (int a = 0; a < argc; a++) {
        if (!strcmp(argv[a], "--help")) usage();
        if (a + 1 >= argc) continue;
        if (!strcmp(argv[a], "-query")) qpath = argv[a + 1];
        if (!strcmp(argv[a], "-db")) dpath = argv[a + 1];
        if (!strcmp(argv[a], "-out")) opath = argv[a + 1];
        if (!strcmp(argv[a], "-evalue")) {
            prm.min_e = (long double)atof(argv[a + 1]);
            if (prm.min_e < 0) terror("Min-e-value must be larger than zero");
        }
        if (!strcmp(argv[a], "-coverage")) {
            prm.min_coverage = (long double)atof(argv[a + 1]);
            if (prm.min_coverage <= 0) terror("Min-coverage must be larger than zero");
        }
        if (!strcmp(argv[a], "-identity")) {
            prm.min_identity = (long double)atof(argv[a + 1]);
            if (prm.min_identity <= 0) terror("Min-identity must be larger than zero");
        }
        if (!strcmp(argv[a], "-igap")) prm.igap = -atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-egap")) prm.egap = -atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-n_threads")) T = (uint64_t)atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-device")) device = atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-devices")) devspec = argv[a + 1];
        if (!strcmp(argv[a], "-max_read_size")) prm.max_read_size = strtoull(argv[a + 1], NULL, 10);
        if (!strcmp(argv[a], "-slice_bases")) slice_bases = strtoull(argv[a + 1], NULL, 10);
        if (!strcmp(argv[a], "-render_threads")) render_threads = atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-batch_reads")) batch_reads = strtoull(argv[a + 1], NULL, 10);
    }
    if (!qpath || !dpath) terror("A query and database is required");
    /* the reference fopen()s "wt" and never checks it (IMSAME.c:541-551) */
    int out_fd = opath ? open(opath, O_WRONLY | O_CREAT | O_TRUNC, 0666) : -1;
    int devs[PIPE_MAX_DEV], G = 1;
    devs[0] = device;
    if (devspec) G = pipe_parse_devices(devspec, devs, PIPE_MAX_DEV);
    if (G < 1) terror("Could not open the GPU device");
    if (slice_bases && G > 1) terror("-slice_bases runs on one device");

    const double t_wall = now_s();
    /* The device runtime starts (a few hundred ms) on its own thread while
     * the FASTA files are parsed; the [INFO] lines keep the reference's order
     * and each reports its own phase. */
    open_job oj = {.d = dv_all, .devs = devs, .G = G};
    pthread_t oth;
    const int othr = pthread_create(&oth, NULL, open_run, &oj) == 0;
    if (!othr) open_run(&oj);
    double t0 = now_s();
    host_seqs db, q;
    const int db_bad = host_load_fasta(dpath, 1, &db);
    const double t_parse_db = now_s() - t0;
    t0 = now_s();
    const int q_bad = db_bad ? 1 : host_load_fasta(qpath, 0, &q);
    const double t_parse_q = now_s() - t0;
    if (othr) pthread_join(oth, NULL);
    pipe_dev *dv = dv_all;
    printf("[INFO] Init. quick table\n");
    if (oj.rc) terror("Could not open the GPU device");
    printf("[INFO] Initialization took %e seconds \n", oj.secs);

    printf("[INFO] Loading database\n");
    if (db_bad) terror("Could not open database file");
    t0 = now_s();
    if (db.n == 0) slice_bases = 0;                  /* nothing to slice */
    int rc = slice_bases ? IMSAME_OK : pipe_index(dv, G, &db);
    if (rc) terror(imsame_strerror(rc));
    const double t_index = now_s() - t0;
    printf("[INFO] Database loaded and of length %" PRIu64 ". Hash table building took %e seconds\n", db.len,
           t_parse_db + t_index);

    t0 = now_s();
    printf("[INFO] Loading query.\n");
    if (q_bad) terror("Could not open query file");
    rc = pipe_set_query(dv, G, &q);
    if (rc) terror(imsame_strerror(rc));
    const double t_upload = now_s() - t0;
    printf("[INFO] Query loaded and of length %" PRIu64 ". Took %e seconds\n", q.len, t_parse_q + t_upload);

    t0 = now_s();
    printf("[INFO] Computing alignments.\n");
    /* per-thread banner of computeAlignmentsByThread (alignmentFunctions.c:88) */
    {
        uint64_t TT = T ? T : 1, rpt = (uint64_t)floorl((long double)q.n / (long double)TT);
        for (uint64_t t = 0; t < TT; t++)
            printf("Going from %" PRIu64 " to %" PRIu64 "\n", t * rpt, t == TT - 1 ? q.n : (t + 1) * rpt);
        fflush(stdout);
    }
    pipe_result pr;
    memset(&pr, 0, sizeof pr);
    if (slice_bases) {
        /* one device, database indexed slice by slice: one batch */
        imsame_read_result *res = calloc(q.n + 1, sizeof *res);
        uint64_t cap = out_fd >= 0 ? 2 * q.n + 1024 : 0, used = 0;
        uint32_t *paths = cap ? malloc(cap * sizeof(uint32_t)) : NULL;
        if (!res || (cap && !paths)) terror("Could not allocate memory for results");
        prm.want_paths = out_fd >= 0;
        const double ta = now_s();
        rc = imsame_dev_align_sliced(dv[0].ctx, db.seq, db.len, db.start, db.n, db.brk, slice_bases, 0, q.n, T, &prm,
                                     res, paths, cap, &used, NULL, &pr.st);
        if (rc == IMSAME_E_PATHS) {
            uint32_t *p2 = realloc(paths, (used + 1) * sizeof(uint32_t));
            if (!p2) terror("Could not allocate memory for results");
            paths = p2;
            rc = imsame_dev_fetch_paths(dv[0].ctx, paths, used, &used);
        }
        pr.t_align = now_s() - ta;
        if (rc == IMSAME_E_ARG) terror("-slice_bases needs every record and read within -max_read_size");
        if (rc) terror(imsame_strerror(rc));
        const double tr = now_s();
        uint64_t off = 0;
        if (out_fd >= 0 && pipe_render_range(&db, &q, res, paths, 0, q.n, out_fd, render_threads, &off, &pr))
            out_failed(out_fd, pr.bytes_ok);
        pr.t_tail = now_s() - tr;
        pr.stop = q.n;
        for (uint64_t r = 0; r < q.n; r++) pr.accepted += res[r].status == 1;
        free(res);
        free(paths);
    } else {
        pipe_opts po = {.T = T, .prm = prm, .out_fd = out_fd, .render_threads = render_threads,
                        .batch_reads = batch_reads};
        rc = pipe_align_render(dv, G, &db, &q, &po, &pr);
        if (pr.write_errno && out_fd >= 0) out_failed(out_fd, pr.bytes_ok);
        if (rc && rc != IMSAME_E_READ_TOO_LONG) terror(imsame_strerror(rc));
    }
    if (out_fd >= 0 && close(out_fd) != 0) terror("Could not write the output file");
    if (rc == IMSAME_E_READ_TOO_LONG) terror("Read size reached for gapped alignment.");
    const uint64_t acc = pr.accepted;
    printf("[INFO] Alignments computed in %e seconds.\n", now_s() - t0);
    printf("[INFO] %" PRIu64 " reads (%" PRIu64 ") from the query were found in the database (%" PRIu64
           ") at a minimum e-value of %Le and minimum coverage of %d%%.\n",
           acc, q.n, db.n, prm.min_e, (int)(100 * prm.min_coverage));
    printf("[INFO] The Jaccard-index is: %Le\n", (long double)acc / ((db.n + q.n) - acc));
    printf("[INFO] Deallocating heap memory.\n");
    if (fflush(stdout) != 0 || ferror(stdout)) {       /* a late error on stdout is an error */
        fprintf(stderr, "[imsame] error writing stdout\n");
        _exit(1);
    }
    fprintf(stderr, "[imsame] rounds=%" PRIu64 " nw=%" PRIu64 " cells=%" PRIu64 " seed_ms=%.3f nw_ms=%.3f total_ms=%.3f\n",
            pr.st.rounds, pr.st.n_nw, pr.st.nw_cells, pr.st.ms_seed, pr.st.ms_nw, pr.st.ms_total);
    fprintf(stderr, "[imsame] phases {\"devices\": %d, \"parts\": %" PRIu64 ", \"open_s\": %.4f, \"parse_db_s\": %.4f, \"index_s\": %.4f, "
            "\"parse_query_s\": %.4f, \"upload_s\": %.4f, \"align_s\": %.4f, \"render_busy_s\": %.4f, "
            "\"write_busy_s\": %.4f, \"render_tail_s\": %.4f, \"pwrite_sum_s\": %.4f, \"pwrite_max_s\": %.4f, \"writer_wait_max_s\": %.4f, "
            "\"bytes_out\": %" PRIu64 ", \"accepted\": %" PRIu64 ", \"wall_s\": %.4f}\n",
            G, pr.batches, oj.secs, t_parse_db, t_index, t_parse_q, t_upload, pr.t_align, pr.t_render, pr.t_write, pr.t_tail,
            pr.t_pwrite_sum, pr.t_pwrite_max, pr.t_wait_max, pr.bytes_out, acc, now_s() - t_wall);
    /* The device contexts and the heap are left to process exit (the output
     * is closed and stdout flushed; the kernel driver releases the GPU
     * memory): hipFree of the arenas and the runtime's exit handlers cost
     * 0.04-0.14 s of a 0.7-0.9 s C2 run (profiles/r4l/, r4m/).
     * IMSAME_CLEAN_EXIT=1 tears everything down (leak checks). */
    const char *ce = getenv("IMSAME_CLEAN_EXIT"), *fe = getenv("IMSAME_FAST_EXIT");
    if (!(ce && atoi(ce)) && !(fe && !atoi(fe))) {
        fprintf(stderr, "[imsame] teardown {\"close_s\": 0, \"fast_exit\": 1, \"main_at_s\": %.4f, \"exit_at_s\": %.4f}\n",
                t_main, since_launch());
        fflush(stderr);
        _exit(0);
    }
    const double t_close = now_s();
    host_free_seqs(&db);
    host_free_seqs(&q);
    pipe_close(dv, G);
    fprintf(stderr, "[imsame] teardown {\"close_s\": %.4f, \"main_at_s\": %.4f, \"exit_at_s\": %.4f}\n",
            now_s() - t_close, t_main, since_launch());
    return 0;
}
