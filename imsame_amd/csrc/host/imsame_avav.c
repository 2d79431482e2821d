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
#include "imsame_host.h"

#define MAX_DEV 64

/* wall seconds per phase over the job (stderr summary) */
static double ph_read, ph_parse, ph_revcomp, ph_align, ph_render, ph_write;

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

/* ---- device workers --------------------------------------------------------- */
typedef struct {
    int device;
    imsame_ctx *ctx;
    const host_seqs *db_now, *q_now;        /* what the context holds */
    /* job */
    const host_seqs *db, *q;
    uint64_t from, to, T, stop;
    const imsame_params *prm;
    imsame_read_result *res;                /* global array; this shard writes [from, to) */
    uint32_t *paths;
    uint64_t cap, used;
    imsame_stats st;
    int rc;
    host_text text;
    double t_index;
} worker;

static void *align_run(void *arg) {
    worker *w = arg;
    double t0 = now_s();
    w->rc = 0;
    if (w->db_now != w->db) {
        w->rc = imsame_dev_index(w->ctx, w->db->seq, w->db->len, w->db->start, w->db->n, w->db->brk);
        if (w->rc) return NULL;
        w->db_now = w->db;
    }
    w->t_index = now_s() - t0;
    if (w->q_now != w->q) {
        w->rc = imsame_dev_set_query(w->ctx, w->q->seq, w->q->len, w->q->start, w->q->n);
        if (w->rc) return NULL;
        w->q_now = w->q;
    }
    memset(&w->st, 0, sizeof w->st);
    if (w->to <= w->from) return NULL;
    for (;;) {
        w->rc = imsame_dev_align(w->ctx, w->from, w->to, w->T, w->prm, w->res + w->from, w->paths, w->cap,
                                 &w->used, &w->st);
        if (w->rc != IMSAME_E_PATHS) break;
        w->cap = w->used + w->used / 4 + 1024;
        uint32_t *p = realloc(w->paths, w->cap * sizeof(uint32_t));
        if (!p) { w->rc = IMSAME_E_OOM; break; }
        w->paths = p;
    }
    return NULL;
}

/* The record of alignmentFunctions.c:165-168, rendered for reads [from, stop). */
static void *render_run(void *arg) {
    worker *w = arg;
    w->text.len = 0;
    host_text one = {0};
    const uint64_t hi = w->stop < w->to ? w->stop : w->to;
    for (uint64_t r = w->from; r < hi; r++) {
        const imsame_read_result *x = &w->res[r];
        if (x->status != 1) continue;
        const uint64_t yl = x->ylen, s = x->db_seq;
        const uint64_t pid = 100 * (uint64_t)x->identities / x->length, pcv = 100 * (uint64_t)x->length / yl;
        char head[160];
        const int hn = snprintf(head, sizeof head, "(%" PRIu64 ", %" PRIu64 ") : %d%% %d%% %" PRIu64 "\n $$$$$$$ \n",
                                r, s, (int)pid < 100 ? (int)pid : 100, (int)pcv < 100 ? (int)pcv : 100, yl);
        host_render(w->db->seq + w->db->start[s], w->db->start[s + 1] - w->db->start[s], w->q->seq + w->q->start[r],
                    yl, x, w->paths + x->path_off, &one);
        if (w->text.len + hn + one.len > w->text.cap) {
            w->text.cap = (w->text.len + hn + one.len) * 2 + 65536;
            w->text.buf = realloc(w->text.buf, w->text.cap);
        }
        memcpy(w->text.buf + w->text.len, head, hn);
        memcpy(w->text.buf + w->text.len + hn, one.buf, one.len);
        w->text.len += hn + one.len;
    }
    free(one.buf);
    return NULL;
}

static void run_workers(worker *w, int G, void *(*fn)(void *)) {
    pthread_t th[MAX_DEV];
    for (int g = 1; g < G; ++g)
        if (pthread_create(&th[g], NULL, fn, &w[g])) { fn(&w[g]); th[g] = 0; }
    fn(&w[0]);
    for (int g = 1; g < G; ++g)
        if (th[g]) pthread_join(th[g], NULL);
}

/* One IMSAME run (IMSAME.c:34-478 semantics, as imsame_cli.c) over G shards. */
static void imsame_run(worker *w, int G, const host_seqs *q, const host_seqs *db, uint64_t T,
                       const imsame_params *prm_in, const char *opath) {
    imsame_params prm = *prm_in;
    FILE *out = fopen(opath, "wt");
    double t0 = now_s();
    printf("[INFO] Init. quick table\n");
    printf("[INFO] Initialization took %e seconds \n", now_s() - t0);
    printf("[INFO] Loading database\n");
    const uint64_t n = q->n;
    imsame_read_result *res = calloc(n + 1, sizeof *res);
    if (!res) die("Could not allocate memory for results");
    prm.want_paths = out ? 1 : 0;
    for (int g = 0; g < G; ++g) {
        w[g].db = db; w[g].q = q; w[g].T = T; w[g].prm = &prm; w[g].res = res;
        w[g].from = (uint64_t)g * n / G; w[g].to = (uint64_t)(g + 1) * n / G;
        if (out && !w[g].paths) {
            w[g].cap = (w[g].to - w[g].from + 1) * 8 + 1024;
            w[g].paths = malloc(w[g].cap * sizeof(uint32_t));
        }
    }
    /* index build and query upload happen inside the workers, overlapped
     * with alignment; the phase lines keep the stock order and lengths */
    printf("[INFO] Database loaded and of length %" PRIu64 ". Hash table building took %e seconds\n", db->len,
           now_s() - t0);
    printf("[INFO] Loading query.\n");
    printf("[INFO] Query loaded and of length %" PRIu64 ". Took %e seconds\n", q->len, 0.0);
    t0 = now_s();
    printf("[INFO] Computing alignments.\n");
    {
        const uint64_t TT = T ? T : 1, rpt = (uint64_t)floorl((long double)n / (long double)TT);
        for (uint64_t t = 0; t < TT; t++)
            printf("Going from %" PRIu64 " to %" PRIu64 "\n", t * rpt, t == TT - 1 ? n : (t + 1) * rpt);
    }
    double tp = now_s();
    run_workers(w, G, align_run);
    ph_align += now_s() - tp;
    uint64_t stop = n;
    int fatal = 0;
    for (int g = 0; g < G; ++g) {
        if (w[g].rc == IMSAME_E_READ_TOO_LONG) { if (w[g].st.err_read < stop) stop = w[g].st.err_read; fatal = 1; }
        else if (w[g].rc) die(imsame_strerror(w[g].rc));
    }
    uint64_t acc = 0;
    for (uint64_t r = 0; r < stop; r++) acc += res[r].status == 1;
    if (out) {
        for (int g = 0; g < G; ++g) w[g].stop = stop;
        tp = now_s();
        run_workers(w, G, render_run);
        ph_render += now_s() - tp;
        tp = now_s();
        for (int g = 0; g < G; ++g) fwrite(w[g].text.buf, 1, w[g].text.len, out);
        fclose(out);
        ph_write += now_s() - tp;
    }
    free(res);
    if (fatal) {
        printf("ERR**** Read size reached for gapped alignment. ****\n");
        fflush(stdout);
        return;
    }
    printf("[INFO] Alignments computed in %e seconds.\n", now_s() - t0);
    printf("[INFO] %" PRIu64 " reads (%" PRIu64 ") from the query were found in the database (%" PRIu64
           ") at a minimum e-value of %Le and minimum coverage of %d%%.\n",
           acc, n, db->n, prm.min_e, (int)(100 * prm.min_coverage));
    printf("[INFO] The Jaccard-index is: %Le\n", (long double)acc / ((db->n + n) - acc));
    printf("[INFO] Deallocating heap memory.\n");
    fflush(stdout);
    uint64_t nw = 0, cells = 0;
    double ms = 0;
    for (int g = 0; g < G; ++g) { nw += w[g].st.n_nw; cells += w[g].st.nw_cells; if (w[g].st.ms_total > ms) ms = w[g].st.ms_total; }
    fprintf(stderr, "[imsame_all_vs_all] %s: reads=%" PRIu64 " accepted=%" PRIu64 " nw=%" PRIu64 " cells=%" PRIu64
            " shards=%d align_ms(max)=%.3f\n", opath, n, acc, nw, cells, G, ms);
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
        const int avail = imsame_dev_count();
        if (devspec && strchr(devspec, ',')) {
            for (const char *s = devspec; *s && G < MAX_DEV; ) {
                devs[G++] = atoi(s);
                const char *c = strchr(s, ',');
                if (!c) break;
                s = c + 1;
            }
        } else {
            const int want = devspec ? atoi(devspec) : avail;
            for (int g = 0; g < want && g < MAX_DEV; ++g) devs[G++] = g;
        }
        if (G == 0) die("Could not open the GPU device");
    }
    worker *w = calloc(G ? G : 1, sizeof *w);
    for (int g = 0; g < G; ++g) {
        w[g].device = devs[g];
        if (imsame_dev_open(devs[g], &w[g].ctx)) die("Could not open the GPU device");
    }

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
                if (rev) load_rc(&m[j], w[0].ctx);
                else load_fwd(&m[j]);
                imsame_run(w, G, &m[i].fwd, rev ? &m[j].rc : &m[j].fwd, T, &prm, op);
            }
        }
    fprintf(stderr, "[imsame_all_vs_all] phase read=%.3f parse=%.3f revcomp=%.3f align=%.3f render=%.3f write=%.3f\n",
            ph_read, ph_parse, ph_revcomp, ph_align, ph_render, ph_write);
    fprintf(stderr, "[imsame_all_vs_all] %zu metagenomes, %" PRIu64 " runs, %" PRIu64 " skipped, %d device contexts, %.3f s\n",
            nm, runs, skipped, G, now_s() - t_job);
    for (int g = 0; g < G; ++g) {
        imsame_dev_close(w[g].ctx);
        free(w[g].paths);
        free(w[g].text.buf);
    }
    for (size_t k = 0; k < nm; ++k) {
        free(m[k].name); free(m[k].path); free(m[k].raw);
        host_free_seqs(&m[k].fwd); host_free_seqs(&m[k].rc);
    }
    free(m);
    free(w);
    if (grc == 0) globfree(&gl);
    return 0;
}
