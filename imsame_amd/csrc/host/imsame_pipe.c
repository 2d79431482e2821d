/* imsame_pipe.c -- see imsame_pipe.h.
 *
 * Threads: one per device context (index build, query upload, the
 * alignment calls of its shard), the library's lane threads (each hands its
 * reads over as soon as they are final, imsame_dev_align_parts), plus a pool
 * of render threads.  The main thread takes the parts in read order; while
 * the devices finish later parts it renders part p (records into per-thread
 * buffers) and a writer thread writes part p-1's buffers at their file
 * offsets.  The record of a read is the reference's
 * (alignmentFunctions.c:165-168):
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
    uint64_t bytes;                    /* record bytes of [from, to) (size_task) */
    int fd, err;
    double t_pw;                       /* seconds in pwrite (render_write_task) */
    host_text spare;                   /* the piece the part's writer holds */
    int inflight;                      /* spare is queued or being written */
    struct wqueue *wq;
} rtask;

/* A part's single writer (IMSAME_ONE_WRITER=1): the render threads hand it
 * full pieces (one in flight per thread, double-buffered), it pwrites them at
 * their offsets.  The write-rate micro reached ~21 GB/s from one writer with
 * a cache-hot source (profiles/r4g/wrate_r4g.txt); with freshly rendered
 * pieces it reached ~9.7 GB/s, below 16 writers' ~12.7 (profiles/r4n/). */
typedef struct wqueue {
    pthread_mutex_t mu;
    pthread_cond_t cv_item, cv_free;
    struct { const char *buf; size_t len; uint64_t off; rtask *owner; } q[HOST_MAX_THREADS];
    int head, count, producers, fd, err;
    double t_busy;
} wqueue;

static int digits(uint64_t v) {
    int d = 1;
    while (v >= 10) { v /= 10; d++; }
    return d;
}

/* bytes of read r's record: the header line of alignmentFunctions.c:167-168
 * ("(%lu, %lu) : %d%% %d%% %lu\n $$$$$$$ \n": 22 fixed bytes + the digits)
 * and build_alignment's text (host_render_size) -- a function of the result
 * row alone, so every record's file offset is known before any is rendered */
static uint64_t record_size(const host_seqs *db, const imsame_read_result *x, uint64_t r) {
    const uint64_t yl = x->ylen, s = x->db_seq;
    const uint64_t pid = 100 * (uint64_t)x->identities / x->length, pcv = 100 * (uint64_t)x->length / yl;
    const uint64_t head = 22 + digits(r) + digits(s) + digits(pid < 100 ? pid : 100) + digits(pcv < 100 ? pcv : 100) +
                          digits(yl);
    return head + host_render_size(db->start[s + 1] - db->start[s], yl, x);
}

static void *size_task(void *a) {
    rtask *t = a;
    uint64_t n = 0;
    for (uint64_t r = t->from; r < t->to; r++)
        if (t->res[r].status == 1) n += record_size(t->db, &t->res[r], r);
    t->bytes = n;
    return NULL;
}

/* read r's record appended to t->text */
static void render_one(rtask *t, uint64_t r) {
    const imsame_read_result *x = &t->res[r];
    const uint64_t yl = x->ylen, s = x->db_seq;
    const uint64_t pid = 100 * (uint64_t)x->identities / x->length, pcv = 100 * (uint64_t)x->length / yl;
    if (t->text.len + 160 > t->text.cap) {
        t->text.cap = (t->text.len + 160) * 2 + 65536;
        char *b = realloc(t->text.buf, t->text.cap);
        if (!b) { t->err = ENOMEM; return; }
        t->text.buf = b;
    }
    /* alignmentFunctions.c:167-168 */
    t->text.len += (size_t)snprintf(t->text.buf + t->text.len, 160,
                                    "(%" PRIu64 ", %" PRIu64 ") : %d%% %d%% %" PRIu64 "\n $$$$$$$ \n", r, s,
                                    (int)pid < 100 ? (int)pid : 100, (int)pcv < 100 ? (int)pcv : 100, yl);
    host_render_scratch(t->db->seq + t->db->start[s], t->db->start[s + 1] - t->db->start[s],
                        t->q->seq + t->q->start[r], yl, x, t->paths + x->path_off, &t->text, &t->scratch);
}

static void *render_task(void *a) {
    rtask *t = a;
    t->text.len = 0;
    for (uint64_t r = t->from; r < t->to && !t->err; r++)
        if (t->res[r].status == 1) render_one(t, r);
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

static int write_all(int fd, const char *b, uint64_t n, uint64_t off, int seekable);

/* render [from, to) and hand it to the part's writer at t->off as it goes,
 * in pieces of RW_PIECE bytes: rendering goes on while the previous piece is
 * written, and the pieces of all threads land at their offsets (the
 * reference's threads share one FILE*, alignmentFunctions.c:165-168) */
#ifndef RW_PIECE
#define RW_PIECE (4u << 20)
#endif
static void render_one(rtask *t, uint64_t r);
/* queue t->text as the piece at file offset off; t->text becomes the spare */
static void hand_piece(rtask *t, uint64_t off) {
    wqueue *w = t->wq;
    const double w0 = pipe_now();
    if (!w) {                                  /* no writer thread: write it here */
        t->err = write_all(t->fd, t->text.buf, t->text.len, off, 1);
        t->t_pw += pipe_now() - w0;
        t->text.len = 0;
        return;
    }
    pthread_mutex_lock(&w->mu);
    while (t->inflight) pthread_cond_wait(&w->cv_free, &w->mu);
    t->inflight = 1;
    const int k = (w->head + w->count) % HOST_MAX_THREADS;
    w->q[k].buf = t->text.buf; w->q[k].len = t->text.len; w->q[k].off = off; w->q[k].owner = t;
    w->count++;
    pthread_cond_signal(&w->cv_item);
    pthread_mutex_unlock(&w->mu);
    t->t_pw += pipe_now() - w0;                /* time waiting for the writer */
    const host_text x = t->text;
    t->text = t->spare;
    t->spare = x;
    t->text.len = 0;
}
static void *writer_task(void *a) {
    wqueue *w = a;
    pthread_mutex_lock(&w->mu);
    for (;;) {
        while (w->count == 0 && w->producers > 0) pthread_cond_wait(&w->cv_item, &w->mu);
        if (w->count == 0) break;
        const int k = w->head;
        w->head = (w->head + 1) % HOST_MAX_THREADS;
        w->count--;
        const char *b = w->q[k].buf;
        const size_t n = w->q[k].len;
        const uint64_t off = w->q[k].off;
        rtask *o = w->q[k].owner;
        const int failed = w->err;
        pthread_mutex_unlock(&w->mu);
        const double t0 = pipe_now();
        const int e = failed ? 0 : write_all(w->fd, b, n, off, 1);
        const double dt = pipe_now() - t0;
        pthread_mutex_lock(&w->mu);
        w->t_busy += dt;
        if (e && !w->err) w->err = e;
        o->inflight = 0;
        pthread_cond_broadcast(&w->cv_free);
    }
    pthread_mutex_unlock(&w->mu);
    return NULL;
}
static void *render_write_task(void *a) {
    rtask *t = a;
    t->text.len = 0;
    uint64_t done = 0;
    for (uint64_t r = t->from; r < t->to && !t->err; r++) {
        if (t->res[r].status != 1) continue;
        render_one(t, r);
        if (t->text.len >= RW_PIECE) {
            const uint64_t n = t->text.len;
            hand_piece(t, t->off + done);
            done += n;
        }
    }
    if (!t->err && t->text.len) {
        const uint64_t n = t->text.len;
        hand_piece(t, t->off + done);
        done += n;
    }
    t->text.len = 0;
    wqueue *w = t->wq;                         /* this thread is done: its last piece out before the buffers go */
    if (w) {
        pthread_mutex_lock(&w->mu);
        w->producers--;
        pthread_cond_signal(&w->cv_item);
        while (t->inflight) pthread_cond_wait(&w->cv_free, &w->mu);
        if (w->err && !t->err) t->err = w->err;
        pthread_mutex_unlock(&w->mu);
    }
    if (!t->err && done != t->bytes) {                 /* record_size must be exact */
        fprintf(stderr, "[imsame] internal error: rendered %llu bytes, sized %llu\n", (unsigned long long)done,
                (unsigned long long)t->bytes);
        t->err = EIO;
    }
    return NULL;
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

/* write what render_part left in t[0..nt): parallel pwrite at the offsets,
 * or ordered write() for pipes; returns an errno and the wall time in *secs.
 * (Writing through a shared mapping of the file instead -- parallel page
 * faults, no file lock -- measured 3.6x slower on the GPU box's overlay
 * filesystem: 1.42 s vs 0.40 s for the 3 GB of C2, profiles/r3c_e2e_*.) */
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

/* seekable output: every slice of [from, to) sized (record_size, in
 * parallel), given its file offset from *off, then rendered and pwritten by
 * its thread at once -- no stage waits for a whole part's text */
static int render_write_part(rtask *t, int nt, const host_seqs *db, const host_seqs *q,
                             const imsame_read_result *res, const uint32_t *paths, uint64_t from, uint64_t to, int fd,
                             uint64_t *off, pipe_result *r) {
    if (to <= from) return 0;
    const uint64_t n = to - from;
    if ((uint64_t)nt > n) nt = (int)n;
    for (int k = 0; k < nt; ++k) {
        t[k].db = db; t[k].q = q; t[k].res = res; t[k].paths = paths; t[k].fd = fd; t[k].err = 0;
        t[k].from = from + n * (uint64_t)k / (uint64_t)nt;
        t[k].to = from + n * (uint64_t)(k + 1) / (uint64_t)nt;
    }
    const double t0 = pipe_now();
    run_pool(t, nt, size_task);
    for (int k = 0; k < nt; ++k) {
        t[k].off = *off;
        *off += t[k].bytes;
    }
    r->bytes_out = *off;
    /* the part's blocks allocated before its writes, so the threads' pwrites
     * only copy (C2 on the box's overlay fs: render tail 0.24 -> 0.19 s and
     * 0.33 -> 0.29 s in two A/B pairs, profiles/r4n, r4o).  fallocate(2), not
     * posix_fallocate: where the filesystem lacks it this is a no-op instead
     * of glibc's byte-per-block emulation.  IMSAME_FALLOCATE=0 turns it off. */
    const char *fa = getenv("IMSAME_FALLOCATE");
    if ((!fa || atoi(fa)) && nt) {
        const uint64_t a = t[0].off;
        if (*off > a) (void)fallocate(fd, 0, (off_t)a, (off_t)(*off - a));
    }
    const double t1 = pipe_now();
    wqueue w = {.mu = PTHREAD_MUTEX_INITIALIZER, .cv_item = PTHREAD_COND_INITIALIZER,
                .cv_free = PTHREAD_COND_INITIALIZER, .producers = nt, .fd = fd};
    for (int k = 0; k < nt; ++k) { t[k].t_pw = 0; t[k].inflight = 0; t[k].wq = &w; }
    /* every render thread pwrites its own pieces (the default: ~12.7 GB/s of
     * the box's page cache for the 3 GB of C2), or IMSAME_ONE_WRITER=1 hands
     * them to one writer thread (measured ~9.7 GB/s: the copies into the page
     * cache then run on one core, profiles/r4n/) */
    const char *ow = getenv("IMSAME_ONE_WRITER");
    pthread_t wth;
    const int wstarted = ow && atoi(ow) && pthread_create(&wth, NULL, writer_task, &w) == 0;
    if (!wstarted)                             /* no writer thread: every render thread writes its own pieces */
        for (int k = 0; k < nt; ++k) t[k].wq = NULL;
    run_pool(t, nt, render_write_task);
    if (wstarted) pthread_join(wth, NULL);
    r->t_render += t1 - t0;                /* sizing */
    r->t_write += pipe_now() - t1;         /* render + write, overlapped */
    if (wstarted) {                        /* diagnostics: the writer's pwrite seconds, and the */
        r->t_pwrite_sum += w.t_busy;       /* longest a render thread waited for it */
        if (w.t_busy > r->t_pwrite_max) r->t_pwrite_max = w.t_busy;
        for (int k = 0; k < nt; ++k)
            if (t[k].t_pw > r->t_wait_max) r->t_wait_max = t[k].t_pw;
    } else {                               /* every render thread's own pwrite seconds */
        for (int k = 0; k < nt; ++k) {
            r->t_pwrite_sum += t[k].t_pw;
            if (t[k].t_pw > r->t_pwrite_max) r->t_pwrite_max = t[k].t_pw;
        }
    }
    for (int k = 0; k < nt; ++k)
        if (t[k].err) return t[k].err;
    return 0;
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
    const uint64_t start = *off;
    const int err = seekable ? render_write_part(t, nt, db, q, res, paths, from, to, fd, off, r)
                             : render_batch(t, nt, db, q, res, paths, from, to, fd, seekable, off, r);
    if (r) {                                       /* bytes known complete, for a caller that must cut */
        r->bytes_ok = err ? start : *off;          /* a failed file back to them */
        if (err && !r->write_errno) r->write_errno = err;
    }
    for (int k = 0; k < nt; ++k) { free(t[k].text.buf); free(t[k].spare.buf); free(t[k].scratch.buf); }
    free(t);
    return err;
}

/* ---- alignment: device workers, results handed over in parts ---------------
 * Each device aligns its shard in one imsame_dev_align_parts call (or
 * batches of -batch_reads); the library hands over each lane's reads as soon
 * as they are final (imsame_dev.h), in any order.  The main thread renders
 * the parts in read order -- the part starting at the next unwritten read --
 * while the devices finish the others. */
typedef struct part {
    uint64_t from, to, err;
    int status;
    uint32_t *paths;                   /* copy of the part's paths (path_off index it) */
    struct part *next;
} part;

typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    part *ready;                       /* delivered, not rendered yet          */
    uint64_t stop_read;                /* min erroring read so far             */
    int fatal;                         /* a hard error (not the size abort)    */
    int workers_left;
    double t_last;                     /* last part delivered                  */
} exchange;

typedef struct {
    pipe_dev *d;
    uint64_t from, to, bsz;
    const pipe_opts *o;
    const imsame_params *prm;
    imsame_read_result *res;
    exchange *x;
    imsame_stats st;                   /* summed over the worker's calls       */
    double ms_calls;
    int batches;
} worker;

static void on_part(void *user, uint64_t a, uint64_t b, int status, uint64_t err, const uint32_t *paths,
                    uint64_t np) {
    worker *w = user;
    exchange *x = w->x;
    part *pt = calloc(1, sizeof *pt);
    uint32_t *pp = np ? malloc(np * sizeof(uint32_t)) : NULL;
    if (pt && (pp || !np)) {
        if (np) memcpy(pp, paths, np * sizeof(uint32_t));
        *pt = (part){.from = a, .to = b, .err = err, .status = status, .paths = pp};
    } else {
        free(pt); free(pp);
        pt = NULL;
    }
    pthread_mutex_lock(&x->mu);
    if (!pt) x->fatal = x->fatal ? x->fatal : IMSAME_E_OOM;
    else {
        pt->next = x->ready;
        x->ready = pt;
        if (status == IMSAME_E_READ_TOO_LONG && err < x->stop_read) x->stop_read = err;
        else if (status && status != IMSAME_E_READ_TOO_LONG && !x->fatal) x->fatal = status;
    }
    x->t_last = pipe_now();
    pthread_cond_broadcast(&x->cv);
    pthread_mutex_unlock(&x->mu);
}

static void add_stats(imsame_stats *t, const imsame_stats *s) {
    t->n_reads += s->n_reads; t->n_accepted += s->n_accepted; t->n_nw += s->n_nw; t->nw_cells += s->nw_cells;
    t->n_hits += s->n_hits; t->rounds = s->rounds > t->rounds ? s->rounds : t->rounds;
    t->ms_seed += s->ms_seed; t->ms_nw += s->ms_nw; t->nw_launches += s->nw_launches; t->nw_bytes += s->nw_bytes;
    t->n_rewalk += s->n_rewalk;
    t->lanes = s->lanes > t->lanes ? s->lanes : t->lanes;
}

static void *align_worker(void *a) {
    worker *w = a;
    exchange *x = w->x;
    for (uint64_t f = w->from; f < w->to; f += w->bsz) {
        const uint64_t t = f + w->bsz < w->to ? f + w->bsz : w->to;
        pthread_mutex_lock(&x->mu);
        const int skip = f >= x->stop_read || x->fatal;    /* past a fatal read: never written */
        pthread_mutex_unlock(&x->mu);
        if (skip) break;
        imsame_stats st;
        memset(&st, 0, sizeof st);
        const int rc = imsame_dev_align_parts(w->d->ctx, f, t, w->o->T, w->prm, w->res + f, on_part, w, &st);
        add_stats(&w->st, &st);
        w->ms_calls += st.ms_total;
        w->batches++;
        if (rc && rc != IMSAME_E_READ_TOO_LONG) {          /* parts may be missing: stop the run */
            pthread_mutex_lock(&x->mu);
            if (!x->fatal) x->fatal = rc;
            pthread_cond_broadcast(&x->cv);
            pthread_mutex_unlock(&x->mu);
            break;
        }
    }
    pthread_mutex_lock(&x->mu);
    x->workers_left--;
    pthread_cond_broadcast(&x->cv);
    pthread_mutex_unlock(&x->mu);
    return NULL;
}

/* the delivered part starting at read `at` (unlinked), or NULL */
static part *take_part(exchange *x, uint64_t at) {
    for (part **pp = &x->ready; *pp; pp = &(*pp)->next)
        if ((*pp)->from == at) {
            part *p = *pp;
            *pp = p->next;
            return p;
        }
    return NULL;
}

int pipe_align_render(pipe_dev *d, int G, const host_seqs *db, const host_seqs *q, const pipe_opts *o,
                      pipe_result *r) {
    memset(r, 0, sizeof *r);
    r->st.err_read = ~0ull;
    const uint64_t n = q->n;
    imsame_params prm = o->prm;
    prm.want_paths = o->out_fd >= 0;
    imsame_read_result *res = calloc(n + 1, sizeof *res);
    const int nt = render_threads(o->render_threads);
    rtask *rt = prm.want_paths ? calloc(2 * (size_t)nt, sizeof *rt) : NULL;       /* two buffer sets */
    if (!res || (prm.want_paths && !rt)) {
        free(res); free(rt);
        return r->rc = IMSAME_E_OOM;
    }
    exchange x = {.mu = PTHREAD_MUTEX_INITIALIZER, .cv = PTHREAD_COND_INITIALIZER, .stop_read = n, .workers_left = G};
    worker W[PIPE_MAX_DEV];
    for (int g = 0; g < G; ++g) {
        uint64_t f, t;
        shard(n, g, G, &f, &t);
        W[g] = (worker){.d = &d[g], .from = f, .to = t, .bsz = o->batch_reads ? o->batch_reads : (t - f ? t - f : 1),
                        .o = o, .prm = &prm, .res = res, .x = &x};
    }
    const double t0 = pipe_now();
    x.t_last = t0;
    pthread_t th[PIPE_MAX_DEV];
    int started[PIPE_MAX_DEV] = {0};
    for (int g = 0; g < G; ++g) started[g] = pthread_create(&th[g], NULL, align_worker, &W[g]) == 0;
    for (int g = 0; g < G; ++g)
        if (!started[g]) align_worker(&W[g]);
    /* render the parts in read order as they arrive */
    const int seekable = prm.want_paths && lseek(o->out_fd, 0, SEEK_CUR) >= 0;
    uint64_t off = seekable ? (uint64_t)lseek(o->out_fd, 0, SEEK_CUR) : 0;
    int rc = 0, werr = 0, nrend = 0;
    writer wr = {0};
    uint64_t nxt = 0;
    for (;;) {
        pthread_mutex_lock(&x.mu);
        part *pt = NULL;
        while (nxt < x.stop_read && !x.fatal && !(pt = take_part(&x, nxt)) && x.workers_left > 0)
            pthread_cond_wait(&x.cv, &x.mu);
        if (!pt && nxt < x.stop_read && !x.fatal) pt = take_part(&x, nxt);   /* workers done meanwhile */
        const uint64_t sr = x.stop_read;
        if (x.fatal && !rc) rc = x.fatal;
        pthread_mutex_unlock(&x.mu);
        if (!pt) break;                                     /* done, past the fatal read, or failed */
        nxt = pt->to;
        const uint64_t hi = pt->to < sr ? pt->to : sr;
        if (rt && !werr && !rc && hi > pt->from && seekable) {
            /* a file: offsets from the rows, every thread renders and writes */
            werr = render_write_part(rt, nt, db, q, res, pt->paths, pt->from, hi, o->out_fd, &off, r);
            if (!werr) r->bytes_ok = off;                   /* this part is complete in the file */
        } else if (rt && !werr && !rc && hi > pt->from) {
            /* a pipe: ordered writes.  Set nrend & 1 was last written two
             * parts ago: that writer is joined */
            rtask *set = rt + (size_t)(nrend & 1) * nt;
            int used = nt;
            werr = render_part(set, &used, db, q, res, pt->paths, pt->from, hi, o->out_fd, &off, r);
            const int e = writer_join(&wr, r);              /* the previous part's output is out */
            if (!werr) werr = e;
            if (!werr) werr = writer_start(&wr, set, used, o->out_fd, seekable);
            nrend++;
        }
        free(pt->paths);                                    /* rendered: the text is in the set */
        free(pt);
        r->batches++;
    }
    {
        const int e = writer_join(&wr, r);
        if (!werr) werr = e;
    }
    for (int g = 0; g < G; ++g)
        if (started[g]) pthread_join(th[g], NULL);
    for (part *p = x.ready; p;) {                           /* parts past the stop */
        part *nx = p->next;
        free(p->paths);
        free(p);
        p = nx;
    }
    if (x.fatal && !rc) rc = x.fatal;
    if (!rc && x.stop_read < n) rc = IMSAME_E_READ_TOO_LONG;
    for (int g = 0; g < G; ++g) {
        add_stats(&r->st, &W[g].st);
        if (W[g].ms_calls > r->st.ms_total) r->st.ms_total = W[g].ms_calls;
    }
    r->st.err_read = x.stop_read < n ? x.stop_read : ~0ull;
    r->t_align = x.t_last - t0;
    r->t_tail = pipe_now() - x.t_last;
    r->stop = x.stop_read;
    for (uint64_t k = 0; k < x.stop_read; ++k) r->accepted += res[k].status == 1;
    if (rt) {
        for (int j = 0; j < 2 * nt; ++j) { free(rt[j].text.buf); free(rt[j].spare.buf); free(rt[j].scratch.buf); }
        free(rt);
    }
    free(res);
    if (werr) {
        fprintf(stderr, "[imsame] write error: %s\n", strerror(werr));
        r->write_errno = werr;
        if (!rc) rc = IMSAME_E_ARG;
    }
    r->rc = rc;
    return rc;
}
