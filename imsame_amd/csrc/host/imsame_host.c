/* imsame_host.c -- FASTA loading and .align rendering for the CLI. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <emmintrin.h>
#include <pthread.h>
#include <unistd.h>
#include "imsame_host.h"

static inline int is_acgt(uint8_t c) { return c == 'A' || c == 'C' || c == 'G' || c == 'T'; }

/* One pass over the byte image.  IMSAME.c:197-289: the outer loop looks for
 * '>' (text before it is skipped; a '>' as the very last byte opens nothing),
 * the header runs to '\n', the body loop reads bytes (toupper) until a '>'.
 * Database: non-ACGT bytes other than '\n' reset the k-mer (:229-231); a new
 * record resets it too (:283).  Reset = bit set on the next stored base. */
int host_parse_fasta(const uint8_t *b, uint64_t nb, int want_brk, host_seqs *s) {
    uint64_t cap_n = 1024;
    memset(s, 0, sizeof *s);
    s->seq = malloc(nb + 1);
    s->start = malloc(cap_n * sizeof(uint64_t));
    if (want_brk) s->brk = calloc(nb / 8 + 2, 1);
    if (!s->seq || !s->start || (want_brk && !s->brk)) return -1;
    uint64_t i = 0, len = 0, n = 0;
    int reset = 0;
    while (i < nb) {
        const uint8_t *gt = memchr(b + i, '>', nb - i);
        if (!gt) break;
        i = (uint64_t)(gt - b);
        if (i + 1 == nb) break;
        if (n + 2 > cap_n) {
            cap_n *= 2;
            s->start = realloc(s->start, cap_n * sizeof(uint64_t));
            if (!s->start) return -1;
        }
        s->start[n++] = len;
        reset = 1;
        const uint8_t *nl = memchr(b + i, '\n', nb - i);
        i = nl ? (uint64_t)(nl - b) + 1 : nb;
        for (; i < nb; ++i) {
            uint8_t c = b[i];
            if (c == '>') break;
            if (c >= 'a' && c <= 'z') c -= 32;
            if (is_acgt(c)) {
                if (reset && want_brk) s->brk[len >> 3] |= (uint8_t)(1u << (len & 7));
                reset = 0;
                s->seq[len++] = c;
            } else if (c != '\n') {
                reset = 1;
            }
        }
    }
    s->start[n] = len;
    s->n = n;
    s->len = len;
    return 0;
}

/* ---- multi-threaded parse ------------------------------
 * A '>' that begins a line always opens a record: a header ends at its first
 * '\n', so the byte after any '\n' is never inside a header, and text before
 * the first '>' is skipped anyway.  Cutting the image just before such '>'
 * gives pieces that parse independently (each opens with a record, which
 * resets the k-mer), so piece k produces exactly the bases, starts and reset
 * positions the serial loop produces over that stretch.  Pieces parse into
 * private buffers; the concatenation is a prefix sum + parallel copy. */
typedef struct {
    const uint8_t *b;
    uint64_t lo, hi, nb;          /* [lo, hi) of the image of nb bytes       */
    uint8_t  *seq;                /* private bases                           */
    uint64_t *start, n, cap_n, len;
    uint64_t *rst, nr, cap_r;     /* positions (piece-local) with a reset bit */
    uint64_t base_off, rec_off;   /* filled after the prefix sum             */
    host_seqs *dst;
    int want_brk, err;
} parse_piece;

static int push_u64(uint64_t **a, uint64_t *n, uint64_t *cap, uint64_t v) {
    if (*n == *cap) {
        *cap = *cap ? 2 * *cap : 256;
        uint64_t *p = realloc(*a, *cap * sizeof(uint64_t));
        if (!p) return -1;
        *a = p;
    }
    (*a)[(*n)++] = v;
    return 0;
}

static void *parse_piece_run(void *arg) {
    parse_piece *p = arg;
    const uint8_t *b = p->b;
    p->seq = malloc(p->hi - p->lo + 1);
    if (!p->seq) { p->err = 1; return NULL; }
    uint64_t i = p->lo, len = 0;
    int reset = 0;
    while (i < p->hi) {
        const uint8_t *gt = memchr(b + i, '>', p->hi - i);
        if (!gt) break;
        i = (uint64_t)(gt - b);
        if (i + 1 == p->nb) break;          /* '>' as the image's last byte */
        if (push_u64(&p->start, &p->n, &p->cap_n, len)) { p->err = 1; return NULL; }
        reset = 1;
        const uint8_t *nl = memchr(b + i, '\n', p->hi - i);
        i = nl ? (uint64_t)(nl - b) + 1 : p->hi;
        for (; i < p->hi; ++i) {
            uint8_t c = b[i];
            if (c == '>') break;
            if (c >= 'a' && c <= 'z') c -= 32;
            if (is_acgt(c)) {
                if (reset && p->want_brk && push_u64(&p->rst, &p->nr, &p->cap_r, len)) { p->err = 1; return NULL; }
                reset = 0;
                p->seq[len++] = c;
            } else if (c != '\n') {
                reset = 1;
            }
        }
    }
    p->len = len;
    return NULL;
}

static void *copy_piece_run(void *arg) {
    parse_piece *p = arg;
    memcpy(p->dst->seq + p->base_off, p->seq, p->len);
    for (uint64_t k = 0; k < p->n; ++k) p->dst->start[p->rec_off + k] = p->start[k] + p->base_off;
    return NULL;
}

static void run_pieces(parse_piece *pc, int np, void *(*fn)(void *)) {
    pthread_t th[HOST_MAX_THREADS];
    int started[HOST_MAX_THREADS] = {0};
    for (int k = 1; k < np; ++k) started[k] = pthread_create(&th[k], NULL, fn, &pc[k]) == 0;
    fn(&pc[0]);
    for (int k = 1; k < np; ++k) {
        if (started[k]) pthread_join(th[k], NULL);
        else fn(&pc[k]);
    }
}

int host_parse_fasta_mt(const uint8_t *b, uint64_t nb, int want_brk, int nthreads, uint64_t min_piece,
                        host_seqs *s) {
    if (nthreads > HOST_MAX_THREADS) nthreads = HOST_MAX_THREADS;
    if (min_piece == 0) min_piece = 1u << 22;
    uint64_t np_want = nb / min_piece;
    if (nthreads <= 1 || np_want < 2) return host_parse_fasta(b, nb, want_brk, s);
    if (np_want > (uint64_t)nthreads) np_want = (uint64_t)nthreads;
    parse_piece pc[HOST_MAX_THREADS];
    memset(pc, 0, sizeof pc);
    /* cut points: first "\n>" at or after k*nb/np (cut before the '>') */
    uint64_t cut[HOST_MAX_THREADS + 1];
    int np = 0;
    cut[0] = 0;
    for (uint64_t k = 1; k < np_want; ++k) {
        uint64_t x = k * nb / np_want;
        if (x <= cut[np]) x = cut[np] + 1;
        uint64_t c = nb;
        while (x < nb) {
            const uint8_t *gt = memchr(b + x, '>', nb - x);
            if (!gt) break;
            const uint64_t g = (uint64_t)(gt - b);
            if (g > 0 && b[g - 1] == '\n') { c = g; break; }
            x = g + 1;
        }
        if (c >= nb) break;
        cut[++np] = c;
    }
    cut[++np] = nb;
    for (int k = 0; k < np; ++k)
        pc[k] = (parse_piece){.b = b, .lo = cut[k], .hi = cut[k + 1], .nb = nb, .want_brk = want_brk};
    run_pieces(pc, np, parse_piece_run);
    int err = 0;
    uint64_t len = 0, n = 0;
    for (int k = 0; k < np; ++k) {
        err |= pc[k].err;
        pc[k].base_off = len;
        pc[k].rec_off = n;
        len += pc[k].len;
        n += pc[k].n;
    }
    memset(s, 0, sizeof *s);
    if (!err) {
        s->seq = malloc(len + 1);
        s->start = malloc((n + 1) * sizeof(uint64_t));
        if (want_brk) s->brk = calloc(len / 8 + 2, 1);
        err = !s->seq || !s->start || (want_brk && !s->brk);
    }
    if (!err) {
        for (int k = 0; k < np; ++k) pc[k].dst = s;
        run_pieces(pc, np, copy_piece_run);
        if (want_brk)
            for (int k = 0; k < np; ++k)
                for (uint64_t r = 0; r < pc[k].nr; ++r) {
                    const uint64_t q = pc[k].rst[r] + pc[k].base_off;
                    s->brk[q >> 3] |= (uint8_t)(1u << (q & 7));
                }
        s->start[n] = len;
        s->n = n;
        s->len = len;
    }
    for (int k = 0; k < np; ++k) { free(pc[k].seq); free(pc[k].start); free(pc[k].rst); }
    if (err) { host_free_seqs(s); return -1; }
    return 0;
}

int host_read_file(const char *path, uint8_t **buf, uint64_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseeko(f, 0, SEEK_END);
    const uint64_t sz = (uint64_t)ftello(f);
    fseeko(f, 0, SEEK_SET);
    *buf = malloc(sz + 1);
    if (!*buf) { fclose(f); return -1; }
    *len = fread(*buf, 1, sz, f);
    fclose(f);
    return 0;
}

int host_load_fasta(const char *path, int want_brk, host_seqs *s) {
    uint8_t *buf;
    uint64_t n;
    if (host_read_file(path, &buf, &n)) return -1;
    const int rc = host_parse_fasta_mt(buf, n, want_brk, host_threads(), 0, s);
    free(buf);
    return rc;
}

int host_threads(void) {
    const char *e = getenv("IMSAME_HOST_THREADS");
    long t = e ? strtol(e, NULL, 10) : sysconf(_SC_NPROCESSORS_ONLN);
    if (t > 16 && !e) t = 16;               /* GPU boxes show the whole machine's CPUs */
    if (t < 1) t = 1;
    if (t > HOST_MAX_THREADS) t = HOST_MAX_THREADS;
    return (int)t;
}

void host_free_seqs(host_seqs *s) {
    free(s->seq); free(s->start); free(s->brk);
    memset(s, 0, sizeof *s);
}

static void text_reserve(host_text *t, size_t n) {
    if (t->len + n <= t->cap) return;
    t->cap = (t->len + n) * 2 + 4096;
    char *b = realloc(t->buf, t->cap);
    if (!b) { fprintf(stderr, "[imsame] out of host memory (render)\n"); exit(-1); }
    t->buf = b;
}

/* bytes of build_alignment's text (alignmentFunctions.c:233-271) for a path
 * whose strings start at head_x+1 / head_y+1 of 2*max(xlen, ylen) */
uint64_t host_render_size(uint64_t xlen, uint64_t ylen, const imsame_read_result *r) {
    const uint64_t M = 2 * (xlen > ylen ? xlen : ylen);
    uint64_t i = (uint64_t)r->head_x + 1, j = (uint64_t)r->head_y + 1, n = 1;
    while (i <= M && j <= M) {
        const uint64_t nx = M - i + 1 < IMSAME_ALIGN_LEN ? M - i + 1 : IMSAME_ALIGN_LEN;
        const uint64_t ny = M - j + 1 < IMSAME_ALIGN_LEN ? M - j + 1 : IMSAME_ALIGN_LEN;
        n += 2 * nx + ny + 3;
        i += nx; j += ny;
    }
    return n;
}

/* backtrackingNW's strings (:493-560) from the path, right to left into
 * rx/ry (scratch of >= 2M+2 bytes each, reused across records), then the
 * 60-column blocks appended to t. */
uint64_t host_render_scratch(const uint8_t *X, uint64_t xlen, const uint8_t *Y, uint64_t ylen,
                             const imsame_read_result *r, const uint32_t *path, host_text *t, host_text *scratch) {
    const uint64_t M = 2 * (xlen > ylen ? xlen : ylen);
    if (scratch->cap < 2 * (M + 2) + IMSAME_ALIGN_LEN + 8) {
        free(scratch->buf);
        scratch->cap = 2 * (M + 2) + 4096;
        scratch->buf = malloc(scratch->cap);
        if (!scratch->buf) { fprintf(stderr, "[imsame] out of host memory (render)\n"); exit(-1); }
    }
    char *rx = scratch->buf, *ry = scratch->buf + M + 2;
    /* the last block's match line pairs X with up to 60 bytes past ry[M]:
     * zero there, as in the reference's memset buffers (never a '*') */
    memset(ry + M + 1, 0, IMSAME_ALIGN_LEN + 4);
    /* right to left; every run is a contiguous copy or fill ending at hx / hy */
    uint64_t hx = M, hy = M;
#define FILL(buf, h, c, n) do { const uint64_t n_ = (n); memset((buf) + (h) + 1 - n_, (c), n_); (h) -= n_; } while (0)
#define COPY(buf, h, src, p, n) do { const uint64_t n_ = (n); memcpy((buf) + (h) + 1 - n_, (src) + (p) + 1 - n_, n_); (h) -= n_; } while (0)
    FILL(rx, hx, '-', xlen - 1 - r->bx);
    FILL(ry, hy, '-', ylen - 1 - r->by);
    uint64_t px = r->bx, py = r->by;
    for (uint32_t e = 0; e < r->path_len; ++e) {
        const uint32_t mv = path[e] >> 30, n = path[e] & 0x3FFFFFFFu;
        if (mv == IMSAME_MOVE_DIAG) {
            COPY(rx, hx, X, px, n); COPY(ry, hy, Y, py, n);
            px -= n; py -= n;
        } else if (mv == IMSAME_MOVE_UP) {
            FILL(ry, hy, '-', n); COPY(rx, hx, X, px, n);
            px -= n; py -= 1;
        } else {
            FILL(rx, hx, '-', n); COPY(ry, hy, Y, py, n);
            py -= n; px -= 1;
        }
    }
    FILL(rx, hx, '-', px);
    FILL(ry, hy, '-', py);
    if (px >= py) FILL(ry, hy, ' ', px);
    else          FILL(rx, hx, ' ', py);
#undef FILL
#undef COPY
    /* build_alignment's loop (:233-271): the strings are [hx+1, M] and [hy+1, M]
     * (the reference prints bytes of rec_X/rec_Y up to index M) */
    text_reserve(t, host_render_size(xlen, ylen, r));
    char *o = t->buf + t->len;
    uint64_t i = hx + 1, j = hy + 1, ident = 0;
    const __m128i dash = _mm_set1_epi8('-'), star = _mm_set1_epi8('*'), space = _mm_set1_epi8(' ');
    while (i <= M && j <= M) {
        const uint64_t nx = M - i + 1 < IMSAME_ALIGN_LEN ? M - i + 1 : IMSAME_ALIGN_LEN;
        const uint64_t ny = M - j + 1 < IMSAME_ALIGN_LEN ? M - j + 1 : IMSAME_ALIGN_LEN;
        memcpy(o, rx + i, nx); o += nx; *o++ = '\n';
        memcpy(o, ry + j, ny); o += ny; *o++ = '\n';
        /* the match line, 16 columns at a time: '*' where both are the same
         * base (neither a gap) */
        uint64_t b = 0;
        for (; b + 16 <= nx; b += 16) {
            const __m128i a = _mm_loadu_si128((const __m128i *)(rx + i + b));
            const __m128i c = _mm_loadu_si128((const __m128i *)(ry + j + b));
            const __m128i m = _mm_andnot_si128(_mm_cmpeq_epi8(a, dash), _mm_cmpeq_epi8(a, c));
            _mm_storeu_si128((__m128i *)(o + b), _mm_or_si128(_mm_and_si128(m, star), _mm_andnot_si128(m, space)));
            ident += (uint64_t)__builtin_popcount((unsigned)_mm_movemask_epi8(m));
        }
        for (; b < nx; b++) {
            const char a = rx[i + b], c = ry[j + b];
            const int st = a != '-' && c != '-' && a == c;
            ident += st;
            o[b] = st ? '*' : ' ';
        }
        o += nx;
        *o++ = '\n';
        i += nx; j += ny;
    }
    *o++ = '\n';
    t->len = (size_t)(o - t->buf);
    return ident;
}

uint64_t host_render(const uint8_t *X, uint64_t xlen, const uint8_t *Y, uint64_t ylen, const imsame_read_result *r,
                     const uint32_t *path, host_text *t) {
    host_text scratch = {0};
    t->len = 0;
    const uint64_t ident = host_render_scratch(X, xlen, Y, ylen, r, path, t, &scratch);
    free(scratch.buf);
    return ident;
}
