/*
 * imsame_avav.c -- bin/all_vs_all_metagenomes_IMSAME.sh as ONE multi-GPU job
 * (BASELINE.json configs[3]).
 *
 *   imsame_all_vs_all metagenomes_directory coverage similarity threads file_extension outpath
 *                     [-devices N | -devices d0,d1,...] [-dry_run]
 *
 * The reference script (/root/reference/bin/all_vs_all_metagenomes_IMSAME.sh)
 *   - lists  $DIR/<*>.$EXT  (ls order) and names each file by what precedes the
 *     first match of awk's field-separator REGEX ".$EXT" in its basename
 *     (:21-26);
 *   - for every pair i < j (:28-33), unless $OUT/X-Y.align exists (:38), runs
 *         IMSAME -query X -db Y -n_threads THR -coverage COV -identity SIM -out $OUT/X-Y.align
 *     and, unless $OUT/X-Y.r.align exists (:47), runs revComp Y > Y.r.EXT and
 *         IMSAME -query X -db Y.r.EXT ... -out $OUT/X-Y.r.align   (:49-51).
 * Here the same runs happen in the same order with the same outputs, but:
 *   - every metagenome is read and parsed once (multi-threaded parse) and kept
 *     in host memory; the reverse complement of Y is computed on the GPU by
 *     imsame_dev_revcomp (reverseComplement.c:21-118, no 1M-record limit) and
 *     parsed with the DATABASE rules, once per Y -- nothing is written into
 *     the metagenome directory (the script writes and deletes Y.r.EXT);
 *   - each run's reads are split into contiguous shards, one per device
 *     context, each device holding a replica of the run's index; chunk heads
 *     come from -n_threads THR, independent of the shard count,
 *     so every record is the one the stock tool computes; the shards' records
 *     are rendered in parallel and written in ascending read order (= the
 *     stock file for THR = 1, the same record set for THR > 1).
 * stdout carries, per run, the [INFO] lines IMSAME prints.  An IMSAME run that
 * would die with "Read size reached" prints that line, keeps the records of
 * the reads before the failing one, and the job continues with the next run
 * as the script does.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <time.h>
#include <glob.h>
#include <pthread.h>
#include <inttypes.h>
#include <sys/stat.h>
#include "../../../include/imsame_dev.h"
#include <fcntl.h>
#include <unistd.h>
#include "imsame_host.h"
#include "imsame_pipe.h"

#define MAX_DEV PIPE_MAX_DEV

/* wall seconds per phase over the job (stderr summary) */
static double ph_read, ph_parse, ph_revcomp, ph_index, ph_align, ph_render, ph_write, ph_tail;

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void die(const char *s) {
    printf("ERR**** %s ****\n", s);
    exit(-1);
}

/* ---- metagenome cache ----------------------------------------------------- */
typedef struct {
    char *name, *path;
    uint8_t *raw;
    uint64_t raw_len;
    host_seqs fwd;      /* database rules (brk bitmap); also serves as query */
    host_seqs rc;       /* parse of revComp(raw), database rules            */
    int have_raw, have_fwd, have_rc;
} mgen;

/* awk -F ".$EXT" '{print $1}': text before the first match of the regex
 * <any char> EXT (EXT taken literally; a match at offset 0 gives ""). */
static char *script_name(const char *base, const char *ext) {
    const size_t n = strlen(base), e = strlen(ext);
    size_t k = n;
    for (size_t i = 0; i + 1 + e <= n; ++i)
        if (memcmp(base + i + 1, ext, e) == 0) { k = i; break; }
    return strndup(base, k);
}

static int is_file(const char *p) {
    struct stat sb;
    return stat(p, &sb) == 0 && S_ISREG(sb.st_mode);
}

/* One IMSAME run (IMSAME.c:34-478 semantics, as imsame_cli.c) over the G
 * contexts: shards, batches and parallel rendering by imsame_pipe.c. */
static void imsame_run(pipe_dev *dv, int G, const host_seqs *q, const host_seqs *db, uint64_t T,
                       const imsame_params *prm, const char *opath) {
    const int out_fd = open(opath, O_WRONLY | O_CREAT | O_TRUNC, 0666);
    double t0 = now_s();
    printf("[INFO] Init. quick table\n");
    printf("[INFO] Initialization took %e seconds \n", now_s() - t0);
    printf("[INFO] Loading database\n");
    double tp = now_s();
    int rc = pipe_index(dv, G, db);
    if (rc) die(imsame_strerror(rc));
    ph_index += now_s() - tp;
    printf("[INFO] Database loaded and of length %" PRIu64 ". Hash table building took %e seconds\n", db->len,
           now_s() - t0);
    printf("[INFO] Loading query.\n");
    t0 = now_s();
    rc = pipe_set_query(dv, G, q);
    if (rc) die(imsame_strerror(rc));
    printf("[INFO] Query loaded and of length %" PRIu64 ". Took %e seconds\n", q->len, now_s() - t0);
    t0 = now_s();
    printf("[INFO] Computing alignments.\n");
    {
        const uint64_t n = q->n, TT = T ? T : 1, rpt = (uint64_t)floorl((long double)n / (long double)TT);
        for (uint64_t t = 0; t < TT; t++)
            printf("Going from %" PRIu64 " to %" PRIu64 "\n", t * rpt, t == TT - 1 ? n : (t + 1) * rpt);
    }
    fflush(stdout);
    pipe_opts po = {.T = T, .prm = *prm, .out_fd = out_fd, .render_threads = 0, .batch_reads = 0};
    pipe_result pr;
    rc = pipe_align_render(dv, G, db, q, &po, &pr);
    if (out_fd >= 0) close(out_fd);
    ph_align += pr.t_align; ph_render += pr.t_render; ph_write += pr.t_write; ph_tail += pr.t_tail;
    if (rc == IMSAME_E_READ_TOO_LONG) {
        printf("ERR**** Read size reached for gapped alignment. ****\n");
        fflush(stdout);
        return;
    }
    if (rc) die(imsame_strerror(rc));
    const uint64_t acc = pr.accepted, n = q->n;
    printf("[INFO] Alignments computed in %e seconds.\n", now_s() - t0);
    printf("[INFO] %" PRIu64 " reads (%" PRIu64 ") from the query were found in the database (%" PRIu64
           ") at a minimum e-value of %Le and minimum coverage of %d%%.\n",
           acc, n, db->n, prm->min_e, (int)(100 * prm->min_coverage));
    printf("[INFO] The Jaccard-index is: %Le\n", (long double)acc / ((db->n + n) - acc));
    printf("[INFO] Deallocating heap memory.\n");
    fflush(stdout);
    fprintf(stderr, "[imsame_all_vs_all] %s: reads=%" PRIu64 " accepted=%" PRIu64 " nw=%" PRIu64 " cells=%" PRIu64
            " shards=%d batches=%" PRIu64 " align_ms(max)=%.3f\n", opath, n, acc, pr.st.n_nw, pr.st.nw_cells, G,
            pr.batches, pr.st.ms_total);
}

static void load_raw(mgen *m) {
    if (m->have_raw) return;
    const double t = now_s();
    if (host_read_file(m->path, &m->raw, &m->raw_len)) die("Could not open query file");
    m->have_raw = 1;
    ph_read += now_s() - t;
}

static void load_fwd(mgen *m) {
    if (m->have_fwd) return;
    load_raw(m);
    const double t = now_s();
    if (host_parse_fasta_mt(m->raw, m->raw_len, 1, host_threads(), 0, &m->fwd)) die("Could not parse FASTA");
    m->have_fwd = 1;
    ph_parse += now_s() - t;
}

static void load_rc(mgen *m, imsame_ctx *ctx) {
    if (m->have_rc) return;
    load_raw(m);
    double t = now_s();
    uint64_t cap = m->raw_len + m->raw_len / 64 + 4096, got = 0;
    uint8_t *img = malloc(cap);
    int rc = imsame_dev_revcomp(ctx, m->raw, m->raw_len, img, cap, &got);
    if (rc == IMSAME_E_ARG && got > cap) {
        cap = got;
        img = realloc(img, cap);
        rc = imsame_dev_revcomp(ctx, m->raw, m->raw_len, img, cap, &got);
    }
    if (rc) die(imsame_strerror(rc));
    ph_revcomp += now_s() - t;
    t = now_s();
    if (host_parse_fasta_mt(img, got, 1, host_threads(), 0, &m->rc)) die("Could not parse FASTA");
    ph_parse += now_s() - t;
    free(img);
    m->have_rc = 1;
}

int main(int argc, char **argv) {
    setenv("GPU_MAX_HW_QUEUES", "8", 0);     /* one hardware queue per lane (see imsame_cli.c) */
    /* positional arguments exactly as the script; options after them */
    int npos = 0, dry = 0;
    const char *pos[6] = {0}, *devspec = NULL;
    for (int a = 1; a < argc; a++) {
        if (!strcmp(argv[a], "-devices") && a + 1 < argc) devspec = argv[++a];
        else if (!strcmp(argv[a], "-dry_run")) dry = 1;
        else if (npos < 6) pos[npos++] = argv[a];
        else npos = 7;
    }
    if (npos != 6) {
        printf("***ERROR*** Use: %s metagenomes_directory coverage similarity threads file_extension outpath\n",
               argv[0]);
        return 255;
    }
    const char *dir = pos[0], *ext = pos[4], *outdir = pos[5];
    imsame_params prm;
    imsame_params_default(&prm);
    /* IMSAME's init_args: atof coverage/identity, atoi threads (IMSAME.c:520-578) */
    prm.min_coverage = (long double)atof(pos[1]);
    prm.min_identity = (long double)atof(pos[2]);
    if (prm.min_coverage <= 0) die("Min-coverage must be larger than zero");
    if (prm.min_identity <= 0) die("Min-identity must be larger than zero");
    const uint64_t T = (uint64_t)atoi(pos[3]);

    /* ls -d $DIR/<*>.$EXT (C-locale order) */
    char pat[4096];
    snprintf(pat, sizeof pat, "%s/*.%s", dir, ext);
    glob_t gl;
    int grc = glob(pat, 0, NULL, &gl);
    const size_t nm = grc == 0 ? gl.gl_pathc : 0;
    mgen *m = calloc(nm + 1, sizeof *m);
    for (size_t k = 0; k < nm; ++k) {
        const char *p = gl.gl_pathv[k], *b = strrchr(p, '/');
        m[k].name = script_name(b ? b + 1 : p, ext);
        if (asprintf(&m[k].path, "%s/%s.%s", dir, m[k].name, ext) < 0) die("out of memory");
    }

    int devs[MAX_DEV], G = 0;
    if (!dry) {
        if (devspec) G = pipe_parse_devices(devspec, devs, MAX_DEV);
        else
            for (int g = 0, avail = imsame_dev_count(); g < avail && g < MAX_DEV; ++g) devs[G++] = g;
        if (G == 0) die("Could not open the GPU device");
    }
    pipe_dev dv[MAX_DEV];
    if (G && pipe_open(dv, devs, G)) die("Could not open the GPU device");

    char op[8192];
    const double t_job = now_s();
    uint64_t runs = 0, skipped = 0;
    for (size_t i = 0; i < nm; ++i)
        for (size_t j = i; j < nm; ++j) {
            if (i == j) continue;
            for (int rev = 0; rev < 2; ++rev) {
                snprintf(op, sizeof op, "%s/%s-%s%s.align", outdir, m[i].name, m[j].name, rev ? ".r" : "");
                if (is_file(op)) { skipped++; if (dry) printf("SKIP %s\n", op); continue; }
                runs++;
                if (dry) {
                    printf("RUN -query %s -db %s%s -n_threads %" PRIu64 " -out %s\n", m[i].path, m[j].path,
                           rev ? " (reverse complement)" : "", T, op);
                    continue;
                }
                load_fwd(&m[i]);
                if (rev) load_rc(&m[j], dv[0].ctx);
                else load_fwd(&m[j]);
                imsame_run(dv, G, &m[i].fwd, rev ? &m[j].rc : &m[j].fwd, T, &prm, op);
            }
        }
    fprintf(stderr, "[imsame_all_vs_all] phase read=%.3f parse=%.3f revcomp=%.3f index=%.3f align=%.3f render=%.3f "
            "write=%.3f render_tail=%.3f\n", ph_read, ph_parse, ph_revcomp, ph_index, ph_align, ph_render, ph_write,
            ph_tail);
    fprintf(stderr, "[imsame_all_vs_all] %zu metagenomes, %" PRIu64 " runs, %" PRIu64 " skipped, %d device contexts, %.3f s\n",
            nm, runs, skipped, G, now_s() - t_job);
    pipe_close(dv, G);
    for (size_t k = 0; k < nm; ++k) {
        free(m[k].name); free(m[k].path); free(m[k].raw);
        host_free_seqs(&m[k].fwd); host_free_seqs(&m[k].rc);
    }
    free(m);
    if (grc == 0) globfree(&gl);
    return 0;
}
