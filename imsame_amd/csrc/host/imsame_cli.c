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
 * Extra flags (not in the reference): -device D, -max_read_size N (raise the
 * 3000-base NW cap of structs.h:19; the reference has it compile-time only).
 * Timing lines report wall-clock seconds (the reference prints clock(),
 * i.e. CPU time summed over threads).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <time.h>
#include <inttypes.h>
#include "../../../include/imsame_dev.h"
#include "imsame_host.h"

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* terror(), commonFunctions.c:10-13 */
static void terror(const char *s) {
    printf("ERR**** %s ****\n", s);
    exit(-1);
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
    printf("           -max_read_size [Integer] (default 3000)\n");
    printf("           -slice_bases [Integer: index the database in slices of at most this many bases]\n");
    exit(1);
}

int main(int argc, char **argv) {
    const char *qpath = NULL, *dpath = NULL, *opath = NULL;
    imsame_params prm;
    imsame_params_default(&prm);
    uint64_t T = 4;                                   /* IMSAME.c:49 */
    int device = 0;
    uint64_t slice_bases = 0;                        /* 0: one index (the reference's) */
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
        if (!strcmp(argv[a], "-max_read_size")) prm.max_read_size = strtoull(argv[a + 1], NULL, 10);
        if (!strcmp(argv[a], "-slice_bases")) slice_bases = strtoull(argv[a + 1], NULL, 10);
    }
    if (!qpath || !dpath) terror("A query and database is required");
    FILE *out = NULL;
    if (opath) out = fopen(opath, "wt");

    double t0 = now_s();
    printf("[INFO] Init. quick table\n");
    imsame_ctx *ctx = NULL;
    int rc = imsame_dev_open(device, &ctx);
    if (rc) terror("Could not open the GPU device");
    printf("[INFO] Initialization took %e seconds \n", now_s() - t0);

    printf("[INFO] Loading database\n");
    t0 = now_s();
    host_seqs db, q;
    if (host_load_fasta(dpath, 1, &db)) terror("Could not open database file");
    if (db.n == 0) slice_bases = 0;                  /* nothing to slice */
    rc = slice_bases ? IMSAME_OK : imsame_dev_index(ctx, db.seq, db.len, db.start, db.n, db.brk);
    if (rc) terror(imsame_strerror(rc));
    printf("[INFO] Database loaded and of length %" PRIu64 ". Hash table building took %e seconds\n", db.len,
           now_s() - t0);

    t0 = now_s();
    printf("[INFO] Loading query.\n");
    if (host_load_fasta(qpath, 0, &q)) terror("Could not open query file");
    rc = imsame_dev_set_query(ctx, q.seq, q.len, q.start, q.n);
    if (rc) terror(imsame_strerror(rc));
    printf("[INFO] Query loaded and of length %" PRIu64 ". Took %e seconds\n", q.len, now_s() - t0);

    t0 = now_s();
    printf("[INFO] Computing alignments.\n");
    /* per-thread banner of computeAlignmentsByThread (alignmentFunctions.c:88) */
    {
        uint64_t TT = T ? T : 1, rpt = (uint64_t)floorl((long double)q.n / (long double)TT);
        for (uint64_t t = 0; t < TT; t++)
            printf("Going from %" PRIu64 " to %" PRIu64 "\n", t * rpt, t == TT - 1 ? q.n : (t + 1) * rpt);
        fflush(stdout);
    }
    imsame_read_result *res = calloc(q.n + 1, sizeof *res);
    uint64_t cap = out ? (q.n + 1) * 8 + 1024 : 0, used = 0;
    uint32_t *paths = out ? malloc(cap * sizeof(uint32_t)) : NULL;
    prm.want_paths = out ? 1 : 0;
    imsame_stats st;
    for (;;) {
        rc = slice_bases ? imsame_dev_align_sliced(ctx, db.seq, db.len, db.start, db.n, db.brk, slice_bases, 0, q.n,
                                                   T, &prm, res, paths, cap, &used, NULL, &st)
                         : imsame_dev_align(ctx, 0, q.n, T, &prm, res, paths, cap, &used, &st);
        if (rc != IMSAME_E_PATHS) break;
        cap = used + used / 4 + 1024 > 2 * cap ? used + used / 4 + 1024 : 2 * cap;   /* too small: grow, redo */
        paths = realloc(paths, cap * sizeof(uint32_t));
    }
    if (rc == IMSAME_E_ARG && slice_bases)
        terror("-slice_bases needs every record and read within -max_read_size");
    if (rc && rc != IMSAME_E_READ_TOO_LONG) terror(imsame_strerror(rc));
    const uint64_t stop = (rc == IMSAME_E_READ_TOO_LONG) ? st.err_read : q.n;
    uint64_t acc = 0;
    host_text txt = {0};
    for (uint64_t r = 0; r < stop; r++) {
        const imsame_read_result *x = &res[r];
        if (x->status != 1) continue;
        acc++;
        if (!out) continue;
        const uint64_t yl = x->ylen;
        /* alignmentFunctions.c:167 */
        const uint64_t pid = 100 * (uint64_t)x->identities / x->length, pcv = 100 * (uint64_t)x->length / yl;
        fprintf(out, "(%" PRIu64 ", %" PRIu64 ") : %d%% %d%% %" PRIu64 "\n $$$$$$$ \n", r, x->db_seq,
                (int)pid < 100 ? (int)pid : 100, (int)pcv < 100 ? (int)pcv : 100, yl);
        const uint64_t s = x->db_seq;
        host_render(db.seq + db.start[s], db.start[s + 1] - db.start[s], q.seq + q.start[r], yl, x,
                    paths + x->path_off, &txt);
        fwrite(txt.buf, 1, txt.len, out);
    }
    if (out) fclose(out);
    if (rc == IMSAME_E_READ_TOO_LONG) terror("Read size reached for gapped alignment.");
    printf("[INFO] Alignments computed in %e seconds.\n", now_s() - t0);
    printf("[INFO] %" PRIu64 " reads (%" PRIu64 ") from the query were found in the database (%" PRIu64
           ") at a minimum e-value of %Le and minimum coverage of %d%%.\n",
           acc, q.n, db.n, prm.min_e, (int)(100 * prm.min_coverage));
    printf("[INFO] The Jaccard-index is: %Le\n", (long double)acc / ((db.n + q.n) - acc));
    printf("[INFO] Deallocating heap memory.\n");
    fprintf(stderr, "[imsame] rounds=%" PRIu64 " nw=%" PRIu64 " cells=%" PRIu64 " seed_ms=%.3f nw_ms=%.3f total_ms=%.3f\n",
            st.rounds, st.n_nw, st.nw_cells, st.ms_seed, st.ms_nw, st.ms_total);
    free(txt.buf);
    free(res);
    free(paths);
    host_free_seqs(&db);
    host_free_seqs(&q);
    imsame_dev_close(ctx);
    return 0;
}
