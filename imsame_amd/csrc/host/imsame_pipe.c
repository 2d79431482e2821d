/* imsame_pipe.c -- see imsame_pipe.h.
 *
 * Threads: one per device context (index build, query upload, the batches of
 * its shard), plus a pool of render threads per finished batch.  The main
 * thread walks the batches in read order; when batch b is done it renders b
 * (records into per-thread buffers, then each buffer written at its file
 * offset) while the devices align b+1, b+2, ...  The record of a read is the
 * reference's (alignmentFunctions.c:165-168):
 *     "(%lu, %lu) : %d%% %d%% %lu\n $$$$$$$ \n" + build_alignment's text. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <errno.h>
#include <fcntl.h>
#include <inttypes.h>
#include <pthread.h>
#include <time.h>
#include <unistd.h>
#include "imsame_pipe.h"

double pipe_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int pipe_parse_devices(const char *spec, int *devs, int max) {
    int G = 0;
    if (!spec || !*spec) return 0;
    if (strchr(spec, ',')) {
        for (const char *s = spec; *s && G < max;) {
            devs[G++] = atoi(s);
            const char *c = strchr(s, ',');
            if (!c) break;
            s = c + 1;
        }
        return G;
    }
    const int n = atoi(spec);
    for (int g = 0; g < n && g < max; ++g) devs[G++] = g;
    return G;
}

int pipe_open(pipe_dev *d, const int *devs, int G) {
    memset(d, 0, sizeof *d * (size_t)G);
    for (int g = 0; g < G; ++g) {
        d[g].device = devs[g];
        const int rc = imsame_dev_open(devs[g], &d[g].ctx);
        if (rc) { pipe_close(d, g); return rc; }
    }
    return 0;
}

void pipe_close(pipe_dev *d, int G) {
    for (int g = 0; g < G; ++g) {
        imsame_dev_close(d[g].ctx);
        d[g].ctx = NULL;
    }
}

/* ---- per-device phases, in parallel over the contexts -------------------- */
typedef struct { pipe_dev *d; const host_seqs *s; uint64_t from, to; int rc; } dev_job;

static void for_devices(dev_job *j, int G, void *(*fn)(void *)) {
    pthread_t th[PIPE_MAX_DEV];
    int started[PIPE_MAX_DEV] = {0};
    for (int g = 1; g < G; ++g) started[g] = pthread_create(&th[g], NULL, fn, &j[g]) == 0;
    fn(&j[0]);
    for (int g = 1; g < G; ++g) {
        if (started[g]) pthread_join(th[g], NULL);
        else fn(&j[g]);
    }
}

static void *index_run(void *a) {
    dev_job *j = a;
    j->rc = 0;
    if (j->d->db_now == j->s) return NULL;
    j->d->db_now = NULL;
    j->rc = imsame_dev_index(j->d->ctx, j->s->seq, j->s->len, j->s->start, j->s->n, j->s->brk);
    if (!j->rc) j->d->db_now = j->s;
    return NULL;
}

static void *query_run(void *a) {
    dev_job *j = a;
    j->rc = 0;
    pipe_dev *d = j->d;
    if (d->q_now == j->s && d->q_lo == j->from && d->q_hi == j->to) return NULL;
    d->q_now = NULL;
    j->rc = imsame_dev_set_query_range(d->ctx, j->s->seq, j->s->len, j->s->start, j->s->n, j->from, j->to);
    if (!j->rc) { d->q_now = j->s; d->q_lo = j->from; d->q_hi = j->to; }
    return NULL;
}

static int first_rc(const dev_job *j, int G) {
    for (int g = 0; g < G; ++g)
        if (j[g].rc) return j[g].rc;
    return 0;
}

int pipe_index(pipe_dev *d, int G, const host_seqs *db) {
    dev_job j[PIPE_MAX_DEV];
    for (int g = 0; g < G; ++g) j[g] = (dev_job){.d = &d[g], .s = db};
    for_devices(j, G, index_run);
    return first_rc(j, G);
}

static void shard(uint64_t n, int g, int G, uint64_t *from, uint64_t *to) {
    *from = n * (uint64_t)g / (uint64_t)G;           /* imsame_amd.dist.shard_range */
    *to = n * (uint64_t)(g + 1) / (uint64_t)G;
}

int pipe_set_query(pipe_dev *d, int G, const host_seqs *q) {
    dev_job j[PIPE_MAX_DEV];
    for (int g = 0; g < G; ++g) {
        j[g] = (dev_job){.d = &d[g], .s = q};
        shard(q->n, g, G, &j[g].from, &j[g].to);
    }
    for_devices(j, G, query_run);
    return first_rc(j, G);
}

/* ---- rendering ------------------------------------------------------------ */
typedef struct {
    const host_seqs *db, *q;
    const imsame_read_result *res;     /* global: res[r] is read r */
    const uint32_t *paths;             /* the arena of reads [from, to) */
    uint64_t from, to;
    host_text text, scratch;           /* reused across batches */
    uint64_t off;
    int fd, err;
} rtask;

static void *render_task(void *a) {
    rtask *t = a;
    t->text.len = 0;
    for (uint64_t r = t->from; r < t->to; r++) {
        const imsame_read_result *x = &t->res[r];
        if (x->status != 1) continue;
        const uint64_t yl = x->ylen, s = x->db_seq;
        const uint64_t pid = 100 * (uint64_t)x->identities / x->length, pcv = 100 * (uint64_t)x->length / yl;
        if (t->text.len + 160 > t->text.cap) {
            t->text.cap = (t->text.len + 160) * 2 + 65536;
            char *b = realloc(t->text.buf, t->text.cap);
            if (!b) { t->err = ENOMEM; return NULL; }
            t->text.buf = b;
        }
        /* alignmentFunctions.c:167-168 */
        t->text.len += (size_t)snprintf(t->text.buf + t->text.len, 160,
                                        "(%" PRIu64 ", %" PRIu64 ") : %d%% %d%% %" PRIu64 "\n $$$$$$$ \n", r, s,
                                        (int)pid < 100 ? (int)pid : 100, (int)pcv < 100 ? (int)pcv : 100, yl);
        host_render_scratch(t->db->seq + t->db->start[s], t->db->start[s + 1] - t->db->start[s],
                            t->q->seq + t->q->start[r], yl, x, t->paths + x->path_off, &t->text, &t->scratch);
    }
    return NULL;
}

static int write_all(int fd, const char *b, uint64_t n, uint64_t off, int seekable) {
    while (n) {
        const ssize_t w = seekable ? pwrite(fd, b, n, (off_t)off) : write(fd, b, n);
        if (w < 0) {
            if (errno == EINTR) continue;
            return errno;
        }
        b += w; n -= (uint64_t)w; off += (uint64_t)w;
    }
    return 0;
}

static void *write_task(void *a) {
    rtask *t = a;
    t->err = write_all(t->fd, t->text.buf, t->text.len, t->off, 1);
    return NULL;
}

static void run_pool(rtask *t, int n, void *(*fn)(void *)) {
    pthread_t th[HOST_MAX_THREADS];
    int started[HOST_MAX_THREADS] = {0};
    for (int k = 1; k < n; ++k) started[k] = pthread_create(&th[k], NULL, fn, &t[k]) == 0;
    fn(&t[0]);
    for (int k = 1; k < n; ++k) {
        if (started[k]) pthread_join(th[k], NULL);
        else fn(&t[k]);
    }
}

/* render reads [from, to) into the task buffers t[0..*nt) and give each its
 * file offset from *off (advanced past the batch); *nt = tasks used */
static int render_part(rtask *t, int *nt, const host_seqs *db, const host_seqs *q, const imsame_read_result *res,
                       const uint32_t *paths, uint64_t from, uint64_t to, int fd, uint64_t *off, pipe_result *r) {
    if (to <= from) { *nt = 0; return 0; }
    const uint64_t n = to - from;
    if ((uint64_t)*nt > n) *nt = (int)n;
    for (int k = 0; k < *nt; ++k) {
        t[k].db = db; t[k].q = q; t[k].res = res; t[k].paths = paths; t[k].fd = fd; t[k].err = 0;
        t[k].from = from + n * (uint64_t)k / (uint64_t)*nt;
        t[k].to = from + n * (uint64_t)(k + 1) / (uint64_t)*nt;
    }
    const double t0 = pipe_now();
    run_pool(t, *nt, render_task);
    r->t_render += pipe_now() - t0;
    for (int k = 0; k < *nt; ++k) {
        if (t[k].err) return t[k].err;
        t[k].off = *off;
        *off += t[k].text.len;
    }
    r->bytes_out = *off;
    return 0;
}

/* write what render_part left in t[0..nt): parallel pwrite at the offsets, or
 * ordered write() for pipes; returns an errno and the wall time in *secs */
static int write_part(rtask *t, int nt, int fd, int seekable, double *secs) {
    const double t0 = pipe_now();
    int err = 0;
    if (seekable) {
        run_pool(t, nt, write_task);
        for (int k = 0; k < nt && !err; ++k) err = t[k].err;
    } else {
        for (int k = 0; k < nt && !err; ++k) err = write_all(fd, t[k].text.buf, t[k].text.len, 0, 0);
    }
    *secs = pipe_now() - t0;
    return err;
}

static int render_batch(rtask *t, int nt, const host_seqs *db, const host_seqs *q, const imsame_read_result *res,
                        const uint32_t *paths, uint64_t from, uint64_t to, int fd, int seekable, uint64_t *off,
                        pipe_result *r) {
    int err = render_part(t, &nt, db, q, res, paths, from, to, fd, off, r);
    if (err || !nt) return err;
    double w = 0;
    err = write_part(t, nt, fd, seekable, &w);
    r->t_write += w;
    return err;
}

/* Output of batch k is written by a writer thread while the main thread
 * renders batch k+1 into the other buffer set (the kernel copies one file's
 * writes into the page cache one at a time, so writing -- not rendering --
 * sets the output rate; overlapping the two hides the rendering). */
typedef struct { rtask *t; int nt, fd, seekable, err, running; double secs; pthread_t th; } writer;

static void *writer_run(void *a) {
    writer *w = a;
    w->err = write_part(w->t, w->nt, w->fd, w->seekable, &w->secs);
    return NULL;
}

static int writer_join(writer *w, pipe_result *r) {
    if (!w->running) return 0;
    pthread_join(w->th, NULL);
    w->running = 0;
    r->t_write += w->secs;
    return w->err;
}

static int writer_start(writer *w, rtask *t, int nt, int fd, int seekable) {
    *w = (writer){.t = t, .nt = nt, .fd = fd, .seekable = seekable};
    if (!nt) return 0;
    if (pthread_create(&w->th, NULL, writer_run, w) != 0) return writer_run(w), w->err;
    w->running = 1;
    return 0;
}

static int render_threads(int want) {
    int n = want > 0 ? want : host_threads();
    return n > HOST_MAX_THREADS ? HOST_MAX_THREADS : n < 1 ? 1 : n;
}

int pipe_render_range(const host_seqs *db, const host_seqs *q, const imsame_read_result *res, const uint32_t *paths,
                      uint64_t from, uint64_t to, int fd, int threads, uint64_t *off, pipe_result *r) {
    const int nt = render_threads(threads);
    rtask *t = calloc((size_t)nt, sizeof *t);
    if (!t) return ENOMEM;
    const int seekable = lseek(fd, 0, SEEK_CUR) >= 0;
    const int err = render_batch(t, nt, db, q, res, paths, from, to, fd, seekable, off, r);
    for (int k = 0; k < nt; ++k) { free(t[k].text.buf); free(t[k].scratch.buf); }
    free(t);
    return err;
}

/* ---- alignment: device workers over batches ------------------------------- */
typedef struct {
    uint64_t from, to;
    uint32_t *paths;
    uint64_t npaths;
    imsame_stats st;
    int rc, done;
    double t_done;
} batch;

typedef struct {
    pipe_dev *d;
    batch *b;
    int nb;
    const pipe_opts *o;
    const imsame_params *prm;
    imsame_read_result *res;
    pthread_mutex_t *mu;
    pthread_cond_t *cv;
    uint64_t *stop_read;               /* min erroring read so far (shared)  */
} worker;

static void *align_worker(void *a) {
    worker *w = a;
    for (int k = 0; k < w->nb; ++k) {
        batch *b = &w->b[k];
        pthread_mutex_lock(w->mu);
        const int skip = b->from >= *w->stop_read;     /* past a fatal read: never written */
        pthread_mutex_unlock(w->mu);
        uint64_t used = 0;
        int rc = 0;
        if (!skip) {
            const uint64_t cap = w->prm->want_paths ? 2 * (b->to - b->from) + 1024 : 0;
            b->paths = cap ? malloc(cap * sizeof(uint32_t)) : NULL;
            if (cap && !b->paths) rc = IMSAME_E_OOM;
            if (!rc)
                rc = imsame_dev_align(w->d->ctx, b->from, b->to, w->o->T, w->prm, w->res + b->from, b->paths, cap,
                                      &used, &b->st);
            /* paths not copied (IMSAME_E_PATHS, or a size abort whose paths did
             * not fit either, include/imsame_dev.h): fetch them */
            if ((rc == IMSAME_E_PATHS || rc == IMSAME_E_READ_TOO_LONG) && cap && used > cap) {
                uint32_t *p = realloc(b->paths, (used + 1) * sizeof(uint32_t));
                const int rf = p ? imsame_dev_fetch_paths(w->d->ctx, p, used, &used) : IMSAME_E_OOM;
                if (p) b->paths = p;
                if (rc == IMSAME_E_PATHS || rf) rc = rf;
            }
        }
        b->npaths = used;
        pthread_mutex_lock(w->mu);
        b->rc = skip ? IMSAME_E_STATE : rc;
        if (rc == IMSAME_E_READ_TOO_LONG && b->st.err_read < *w->stop_read) *w->stop_read = b->st.err_read;
        b->done = 1;
        b->t_done = pipe_now();
        pthread_cond_broadcast(w->cv);
        pthread_mutex_unlock(w->mu);
    }
    return NULL;
}

static void add_stats(imsame_stats *t, const imsame_stats *s) {
    t->n_reads += s->n_reads; t->n_accepted += s->n_accepted; t->n_nw += s->n_nw; t->nw_cells += s->nw_cells;
    t->n_hits += s->n_hits; t->rounds = s->rounds > t->rounds ? s->rounds : t->rounds;
    t->ms_seed += s->ms_seed; t->ms_nw += s->ms_nw; t->nw_launches += s->nw_launches; t->nw_bytes += s->nw_bytes;
    t->n_rewalk += s->n_rewalk;
}

int pipe_align_render(pipe_dev *d, int G, const host_seqs *db, const host_seqs *q, const pipe_opts *o,
                      pipe_result *r) {
    memset(r, 0, sizeof *r);
    r->st.err_read = ~0ull;
    const uint64_t n = q->n;
    imsame_params prm = o->prm;
    prm.want_paths = o->out_fd >= 0;
    imsame_read_result *res = calloc(n + 1, sizeof *res);
    if (!res) return IMSAME_E_OOM;
    /* batches: each device's shard in pieces (several when rendering, so
     * the host renders batch b while the device aligns b+1) */
    int nb[PIPE_MAX_DEV], total = 0;
    uint64_t from[PIPE_MAX_DEV], to[PIPE_MAX_DEV], bsz[PIPE_MAX_DEV];
    for (int g = 0; g < G; ++g) {
        shard(n, g, G, &from[g], &to[g]);
        const uint64_t m = to[g] - from[g];
        uint64_t b = o->batch_reads;
        if (!b) b = prm.want_paths ? (m + 3) / 4 : m;          /* 4 batches when rendering */
        if (prm.want_paths && !o->batch_reads && b < 131072) b = 131072;
        if (b == 0) b = 1;
        bsz[g] = b;
        nb[g] = m ? (int)((m + b - 1) / b) : 0;
        total += nb[g];
    }
    batch *B = calloc((size_t)total + 1, sizeof *B);
    const int nt = render_threads(o->render_threads);
    rtask *rt = prm.want_paths ? calloc(2 * (size_t)nt, sizeof *rt) : NULL;       /* two buffer sets */
    if (!B || (prm.want_paths && !rt)) {
        free(B); free(rt); free(res);
        return r->rc = IMSAME_E_OOM;
    }
    worker W[PIPE_MAX_DEV];
    pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
    pthread_cond_t cv = PTHREAD_COND_INITIALIZER;
    uint64_t stop_read = n;
    int k = 0;
    for (int g = 0; g < G; ++g) {
        W[g] = (worker){.d = &d[g], .b = B + k, .nb = nb[g], .o = o, .prm = &prm, .res = res, .mu = &mu, .cv = &cv,
                        .stop_read = &stop_read};
        for (int j = 0; j < nb[g]; ++j, ++k) {
            B[k].from = from[g] + (uint64_t)j * bsz[g];
            B[k].to = B[k].from + bsz[g] < to[g] ? B[k].from + bsz[g] : to[g];
        }
    }
    r->batches = (uint64_t)total;
    const double t0 = pipe_now();
    pthread_t th[PIPE_MAX_DEV];
    int started[PIPE_MAX_DEV] = {0};
    for (int g = 0; g < G; ++g) started[g] = pthread_create(&th[g], NULL, align_worker, &W[g]) == 0;
    for (int g = 0; g < G; ++g)
        if (!started[g]) align_worker(&W[g]);
    /* walk the batches in read order: render each as it completes */
    const int seekable = prm.want_paths && lseek(o->out_fd, 0, SEEK_CUR) >= 0;
    uint64_t off = seekable ? (uint64_t)lseek(o->out_fd, 0, SEEK_CUR) : 0;
    int rc = 0, werr = 0, nrend = 0;
    writer wr = {0};
    double t_last = t0;
    for (k = 0; k < total; ++k) {
        pthread_mutex_lock(&mu);
        while (!B[k].done) pthread_cond_wait(&cv, &mu);
        const uint64_t sr = stop_read;
        pthread_mutex_unlock(&mu);
        if (B[k].t_done > t_last) t_last = B[k].t_done;
        if (B[k].from >= sr) continue;                        /* past the fatal read */
        if (B[k].rc && B[k].rc != IMSAME_E_READ_TOO_LONG) { if (!rc) rc = B[k].rc; continue; }
        if (B[k].rc == IMSAME_E_READ_TOO_LONG && !rc) rc = IMSAME_E_READ_TOO_LONG;
        const uint64_t hi = B[k].to < sr ? B[k].to : sr;
        if (rt && !werr && (rc == 0 || rc == IMSAME_E_READ_TOO_LONG)) {
            /* set nrend & 1 was last written two batches ago: that writer is joined */
            rtask *set = rt + (size_t)(nrend & 1) * nt;
            int used = nt;
            werr = render_part(set, &used, db, q, res, B[k].paths, B[k].from, hi, o->out_fd, &off, r);
            const int e = writer_join(&wr, r);              /* batch k-1's output is out */
            if (!werr) werr = e;
            if (!werr) werr = writer_start(&wr, set, used, o->out_fd, seekable);
            nrend++;
        }
        /* its paths are no longer needed once rendered (the text is in the set) */
        free(B[k].paths);
        B[k].paths = NULL;
    }
    {
        const int e = writer_join(&wr, r);
        if (!werr) werr = e;
    }
    for (int g = 0; g < G; ++g)
        if (started[g]) pthread_join(th[g], NULL);
    if (stop_read < n && !rc) rc = IMSAME_E_READ_TOO_LONG;       /* its batch may start at the read */
    for (k = 0; k < total; ++k) {
        if (B[k].t_done > t_last) t_last = B[k].t_done;
        add_stats(&r->st, &B[k].st);
        free(B[k].paths);
    }
    double dev_ms[PIPE_MAX_DEV] = {0};
    for (int g = 0; g < G; ++g)
        for (int j = 0; j < nb[g]; ++j) dev_ms[g] += W[g].b[j].st.ms_total;
    for (int g = 0; g < G; ++g)
        if (dev_ms[g] > r->st.ms_total) r->st.ms_total = dev_ms[g];
    r->t_align = t_last - t0;
    r->t_tail = pipe_now() - t_last;
    r->stop = stop_read;
    r->st.err_read = stop_read < n ? stop_read : ~0ull;
    for (uint64_t x = 0; x < stop_read; ++x) r->accepted += res[x].status == 1;
    if (rt) {
        for (int j = 0; j < 2 * nt; ++j) { free(rt[j].text.buf); free(rt[j].scratch.buf); }
        free(rt);
    }
    free(B);
    free(res);
    if (werr) { fprintf(stderr, "[imsame] write error: %s\n", strerror(werr)); if (!rc) rc = IMSAME_E_ARG; }
    r->rc = rc;
    return rc;
}
