/* pipe_race.c -- TEST INFRASTRUCTURE: drives the host side of the imsame CLI
 * (imsame_host.c, imsame_pipe.c) with every thread it starts, for the
 * sanitizer builds of scripts/sanitize.sh (ThreadSanitizer; Address +
 * UndefinedBehavior), against fake_dev.c instead of the GPU:
 *   1. host_parse_fasta_mt (6 threads, 4 KiB pieces) == host_parse_fasta on an
 *      adversarial FASTA (CRLF, N, lowercase, empty records, '>' inside lines);
 *   2. pipe_align_render with 3 contexts x 3 lanes, 37-read batches and 4
 *      render threads writes the same bytes as 1 context, whole shard, 1
 *      render thread -- and as a serial host_render of every record;
 *   3. pipe_render_range with 5 threads appends the same bytes again.
 * The reference's threads share one FILE* (alignmentFunctions.c:165-168);
 * this is the exchange that replaces it.  Exit status 0 = all equal. */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/resource.h>
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include "../../imsame_amd/csrc/host/imsame_pipe.h"

void fake_result(const imsame_ctx *c, uint64_t r, imsame_read_result *o, uint32_t *path);

static uint64_t rng = 88172645463325252ull;
static uint64_t nxt(void) { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

static char *make_fasta(int nrec, int minlen, int maxlen, int adversarial, size_t *len) {
    size_t cap = (size_t)nrec * (maxlen + maxlen / 10 + 64) + 64, n = 0;
    char *b = malloc(cap);
    for (int k = 0; k < nrec; ++k) {
        n += (size_t)sprintf(b + n, ">rec_%d%s\n", k, adversarial && k % 11 == 0 ? " some > text" : "");
        int L = minlen + (int)(nxt() % (uint64_t)(maxlen - minlen + 1));
        if (adversarial && k % 13 == 5) L = 0;                   /* empty record */
        for (int i = 0; i < L; ++i) {
            char ch = "ACGT"[nxt() & 3];
            if (adversarial && nxt() % 97 == 0) ch = 'N';
            if (adversarial && nxt() % 89 == 0) ch = (char)(ch + 32);
            b[n++] = ch;
            if ((i + 1) % 60 == 0 && i + 1 < L) {
                if (adversarial && k % 3 == 1) b[n++] = '\r';
                b[n++] = '\n';
            }
        }
        if (adversarial && k % 3 == 1) b[n++] = '\r';
        b[n++] = '\n';
    }
    *len = n;
    return b;
}

static int same_seqs(const host_seqs *a, const host_seqs *b) {
    if (a->n != b->n || a->len != b->len) return 0;
    if (memcmp(a->seq, b->seq, a->len) || memcmp(a->start, b->start, (a->n + 1) * 8)) return 0;
    if ((a->brk == NULL) != (b->brk == NULL)) return 0;
    return !a->brk || !memcmp(a->brk, b->brk, (a->len + 7) / 8);
}

static char *slurp(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    char *b = malloc(*len + 1);
    if (fread(b, 1, *len, f) != *len) { fclose(f); free(b); return NULL; }
    fclose(f);
    return b;
}

static int run_pipe_r(const host_seqs *db, const host_seqs *q, int G, int rt, uint64_t batch, const char *path,
                      uint64_t *acc, pipe_result *out);
static int run_pipe(const host_seqs *db, const host_seqs *q, int G, int rt, uint64_t batch, const char *path,
                    uint64_t *acc) {
    pipe_result r;
    return run_pipe_r(db, q, G, rt, batch, path, acc, &r);
}
static int run_pipe_r(const host_seqs *db, const host_seqs *q, int G, int rt, uint64_t batch, const char *path,
                      uint64_t *acc, pipe_result *out) {
    pipe_dev d[8];
    int devs[8] = {0};
    if (pipe_open(d, devs, G) || pipe_index(d, G, db) || pipe_set_query(d, G, q)) return 1;
    pipe_opts o;
    memset(&o, 0, sizeof o);
    o.T = 4;
    imsame_params_default(&o.prm);
    o.render_threads = rt;
    o.batch_reads = batch;
    o.out_fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
    pipe_result r;
    const int rc = pipe_align_render(d, G, db, q, &o, &r);
    close(o.out_fd);
    pipe_close(d, G);
    *acc = r.accepted;
    *out = r;
    return rc;
}

void imsame_params_default(imsame_params *p) {
    memset(p, 0, sizeof *p);
    p->min_e = 1e-20L; p->min_coverage = 0.5; p->min_identity = 0.5;
    p->igap = -5; p->egap = -2; p->max_read_size = IMSAME_MAX_READ_SIZE;
}

int main(int argc, char **argv) {
    const char *dir = argc > 1 ? argv[1] : "/tmp";
    int fails = 0;
    /* 1. parallel parse == serial parse */
    size_t nd, nq;
    char *fd_ = make_fasta(400, 300, 1200, 1, &nd);
    char *fq = make_fasta(6000, 20, 150, 1, &nq);
    host_seqs db, db2, q, q2;
    if (host_parse_fasta((uint8_t *)fd_, nd, 1, &db) || host_parse_fasta_mt((uint8_t *)fd_, nd, 1, 6, 4096, &db2) ||
        host_parse_fasta((uint8_t *)fq, nq, 0, &q) || host_parse_fasta_mt((uint8_t *)fq, nq, 0, 6, 4096, &q2)) {
        fprintf(stderr, "parse failed\n");
        return 2;
    }
    if (!same_seqs(&db, &db2) || !same_seqs(&q, &q2)) { fprintf(stderr, "FAIL parse_mt != parse\n"); fails++; }
    /* 2. the pipeline: threaded cut vs one context, whole shard, one render thread */
    char p1[512], p2[512], p3[512];
    snprintf(p1, sizeof p1, "%s/pipe_race_1.align", dir);
    snprintf(p2, sizeof p2, "%s/pipe_race_2.align", dir);
    snprintf(p3, sizeof p3, "%s/pipe_race_3.align", dir);
    uint64_t a1 = 0, a2 = 0;
    if (run_pipe(&db, &q, 1, 1, 0, p1, &a1) || run_pipe(&db, &q, 3, 4, 37, p2, &a2)) {
        fprintf(stderr, "pipeline failed\n");
        return 2;
    }
    size_t l1, l2, l3;
    char *b1 = slurp(p1, &l1), *b2 = slurp(p2, &l2);
    if (!b1 || !b2 || l1 != l2 || memcmp(b1, b2, l1) || a1 != a2) { fprintf(stderr, "FAIL threaded pipeline output\n"); fails++; }
    /* the serial rendering of every record */
    imsame_ctx *c = NULL;
    imsame_dev_open(0, &c);
    imsame_dev_index(c, db.seq, db.len, db.start, db.n, db.brk);
    imsame_dev_set_query_range(c, q.seq, q.len, q.start, q.n, 0, q.n);
    imsame_read_result *res = calloc(q.n + 1, sizeof *res);
    uint32_t *paths = calloc(q.n + 1, sizeof *paths);
    host_text t = {0}, one = {0};
    uint64_t np = 0;
    for (uint64_t r = 0; r < q.n; ++r) {
        fake_result(c, r, &res[r], paths + np);
        if (res[r].status != 1) continue;
        res[r].path_off = (uint32_t)np;
        np += res[r].path_len;
        const imsame_read_result *x = &res[r];
        char head[160];
        const uint64_t yl = x->ylen, s = x->db_seq;
        const int pid = (int)(100 * (uint64_t)x->identities / x->length), pcv = (int)(100 * (uint64_t)x->length / yl);
        const int hn = snprintf(head, sizeof head, "(%" PRIu64 ", %" PRIu64 ") : %d%% %d%% %" PRIu64 "\n $$$$$$$ \n",
                                r, s, pid < 100 ? pid : 100, pcv < 100 ? pcv : 100, yl);
        host_render(db.seq + db.start[s], db.start[s + 1] - db.start[s], q.seq + q.start[r], yl, x,
                    paths + x->path_off, &one);
        t.buf = realloc(t.buf, t.len + (size_t)hn + one.len + 1);
        memcpy(t.buf + t.len, head, (size_t)hn); t.len += (size_t)hn;
        memcpy(t.buf + t.len, one.buf, one.len); t.len += one.len;
    }
    if (t.len != l1 || memcmp(t.buf, b1, l1)) { fprintf(stderr, "FAIL pipeline != serial render\n"); fails++; }
    /* 3. pipe_render_range with 5 threads */
    int fd3 = open(p3, O_CREAT | O_TRUNC | O_WRONLY, 0644);
    uint64_t off = 0;
    pipe_result pr;
    memset(&pr, 0, sizeof pr);
    if (pipe_render_range(&db, &q, res, paths, 0, q.n, fd3, 5, &off, &pr)) { fprintf(stderr, "render_range failed\n"); fails++; }
    close(fd3);
    char *b3 = slurp(p3, &l3);
    if (!b3 || l3 != t.len || memcmp(b3, t.buf, l3)) { fprintf(stderr, "FAIL render_range\n"); fails++; }
    /* 4. a write that fails part-way (file size limit): the pipeline reports
     * the error and how many leading bytes are complete -- whole parts, a
     * prefix of the serial text -- for the CLI to cut the file back to */
    {
        char p4[512];
        snprintf(p4, sizeof p4, "%s/pipe_race_4.align", dir);
        signal(SIGXFSZ, SIG_IGN);
        struct rlimit old, lim;
        getrlimit(RLIMIT_FSIZE, &old);
        lim = old;
        lim.rlim_cur = (rlim_t)(l1 * 2 / 3);
        setrlimit(RLIMIT_FSIZE, &lim);
        uint64_t a4 = 0;
        pipe_result r4;
        const int rc4 = run_pipe_r(&db, &q, 3, 4, 997, p4, &a4, &r4);
        setrlimit(RLIMIT_FSIZE, &old);
        size_t l4;
        char *b4 = slurp(p4, &l4);
        if (rc4 == 0 || r4.write_errno != EFBIG || r4.bytes_ok == 0 || r4.bytes_ok > (uint64_t)lim.rlim_cur ||
            !b4 || l4 < r4.bytes_ok || memcmp(b4, b1, r4.bytes_ok)) {
            fprintf(stderr, "FAIL write error: rc %d errno %d bytes_ok %" PRIu64 " file %zu\n", rc4, r4.write_errno,
                    r4.bytes_ok, b4 ? l4 : 0);
            fails++;
        }
        free(b4);
        unlink(p4);
    }
    printf("pipe_race: %" PRIu64 " reads, %" PRIu64 " accepted, %zu bytes, %s\n", q.n, a1, l1, fails ? "FAIL" : "ok");
    imsame_dev_close(c);
    free(res); free(paths); free(t.buf); free(one.buf); free(b1); free(b2); free(b3); free(fd_); free(fq);
    host_free_seqs(&db); host_free_seqs(&db2); host_free_seqs(&q); host_free_seqs(&q2);
    unlink(p1); unlink(p2); unlink(p3);
    return fails ? 1 : 0;
}
