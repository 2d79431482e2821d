/*
 * imsame_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Clean-room CPU restatement of IMSAME's read-vs-database seed-and-extend
 * path (Bitlab-UMA/IMSAME).  It is the parity CHECKER: tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (imsame_amd/, include/) never does.
 *
 * Every function cites the reference code it restates.  Deliberately plain:
 * full int64 NW table, literal per-thread scan state machine, x87
 * long-double e-value/coverage/identity tests, no memoisation -- so that it
 * shares no shortcut with the HIP path it checks.
 *
 * Pinned against the reference compiled from /root/reference/src
 * (oracle/Makefile 'ref' target) through tests/golden/ fixtures.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <pthread.h>
#include <unistd.h>
#include <time.h>
#include <inttypes.h>
#include "imsame_oracle.h"

#define K   IMSAME_FIXED_K
#define PT  IMSAME_POINT
#define NB  (1u << 24)                      /* 4^12 buckets */

/* ------------------------------------------------------------------ */
/* sequences                                                           */
/* ------------------------------------------------------------------ */
typedef struct {
    uint8_t  *seq;      /* ACGT-filtered concatenation           */
    uint64_t *start;    /* n+1 entries, start[n] = len            */
    uint64_t  n, len;
    uint8_t  *brk;      /* DB only: k-mer reset bitmap (bit/base) */
    int       own;      /* 1: buffers malloc'd here               */
} or_seqs;

static int base_code(uint8_t c) {
    switch (c) { case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3; }
    return -1;
}

/* FASTA -> filtered concatenation.  IMSAME.c:194-289 (database) and
 * IMSAME.c:320-371 (query).
 *  - text before the first '>' is skipped; a '>' that is the file's very last
 *    byte starts nothing (the outer loop condition fails first, :197);
 *  - a header runs to '\n' (:212) -- a header cut by EOF ends the file;
 *  - body bytes are toupper()'d, only A/C/G/T are kept (:216-221);
 *  - database only: any other byte except '\n' resets the running k-mer
 *    (:229-231), as does a new record (:283).  Stored as bit p of brk =
 *    "reset before base p". */
static void or_parse_fasta(const uint8_t *b, uint64_t nb, or_seqs *s, int want_brk) {
    uint64_t ncap = 64, i = 0;
    s->seq = malloc(nb + 1);
    s->start = malloc(ncap * sizeof(uint64_t));
    s->n = 0; s->len = 0; s->own = 1;
    s->brk = want_brk ? calloc(nb / 8 + 2, 1) : NULL;
    int pending = 0;
    while (i < nb) {
        if (b[i] != '>' || i + 1 == nb) { i++; continue; }
        if (s->n + 2 > ncap) { ncap *= 2; s->start = realloc(s->start, ncap * sizeof(uint64_t)); }
        s->start[s->n++] = s->len;
        pending = 1;
        while (i < nb && b[i] != '\n') i++;
        if (i < nb) i++;                                  /* consume the header's '\n' */
        while (i < nb) {
            uint8_t c = b[i++];
            if (c >= 'a' && c <= 'z') c = (uint8_t)(c - 'a' + 'A');
            if (c == '>') { i--; break; }                 /* outer loop sees the '>' */
            if (base_code(c) >= 0) {
                if (pending && s->brk) s->brk[s->len >> 3] |= (uint8_t)(1u << (s->len & 7));
                pending = 0;
                s->seq[s->len++] = c;
            } else if (c != '\n') {
                pending = 1;
            }
        }
    }
    s->start[s->n] = s->len;
}

static void or_free_seqs(or_seqs *s) {
    if (s->own) { free(s->seq); free(s->start); free(s->brk); }
}

/* ------------------------------------------------------------------ */
/* 12-mer index                                                        */
/* ------------------------------------------------------------------ */
/* Reference: 4^12 table of LIFO linked lists (IMSAME.c:232-281), so a
 * bucket is visited in DESCENDING insertion position.  Here: CSR filled in
 * descending position order. */
typedef struct {
    uint64_t *off;       /* NB+1 */
    uint64_t *pos;       /* reference pos (u64: databases past 4 Gbases) */
    uint32_t *sid;
} or_index;

static int brk_at(const or_seqs *d, uint64_t b) { return d->brk ? (d->brk[b >> 3] >> (b & 7)) & 1 : 0; }

static uint32_t kmer_code(const uint8_t *s) {
    uint32_t c = 0;
    for (int k = 0; k < K; k++) c = (c << 2) | (uint32_t)base_code(s[k]);
    return c;
}

/* The index build splits the database by record ranges: thread t computes
 * the rolling codes of its records and counts its k-mers per bucket; bucket
 * c then gets, per thread, a fill cursor that leaves room for every later
 * range's entries first (descending position = higher ranges first), and
 * each thread scatters its own positions in descending order.  Every pass
 * is O(len / T). */
typedef struct { const or_seqs *d; uint32_t *code; uint64_t *cnt; or_index *ix; uint64_t lo, hi, total; int pass; } ix_part;

static void *ix_part_run(void *arg) {
    ix_part *t = arg;
    const or_seqs *d = t->d;
    if (t->pass == 0) {
        const uint32_t mask = (uint32_t)((1ull << (2 * K)) - 1);
        for (uint64_t rec = t->lo; rec < t->hi; rec++) {
            uint32_t c = 0, run = 0;
            for (uint64_t p = d->start[rec]; p < d->start[rec + 1]; p++) {
                run = (p == d->start[rec] || brk_at(d, p)) ? 1 : run + 1;
                c = ((c << 2) | (uint32_t)base_code(d->seq[p])) & mask;
                t->code[p] = (run >= K) ? c : ~0u;
                if (run >= K) { t->cnt[c]++; t->total++; }
            }
        }
    } else {
        uint64_t *fill = t->cnt;                 /* this range's cursor per bucket */
        for (uint64_t rec = t->hi; rec-- > t->lo;)
            for (uint64_t p = d->start[rec + 1]; p-- > d->start[rec];) {
                const uint32_t c = t->code[p];
                if (c == ~0u) continue;
                t->ix->pos[fill[c]] = p + 1;             /* pos = last base + 1 (IMSAME.c:247) */
                t->ix->sid[fill[c]] = (uint32_t)rec;     /* s_id = current record (:249)     */
                fill[c]++;
            }
    }
    return NULL;
}

#define IX_THREADS 16

static void or_build_index(const or_seqs *d, or_index *ix) {
    /* a k-mer ending at p is valid when the K bases p-K+1..p lie in one
     * record and no break flag sits on p-K+2..p -- i.e. the run of bases
     * since the last record start/break is at least K long. */
    uint32_t *code = malloc((d->len + 1) * sizeof(uint32_t));
    ix->off = calloc(NB + 1, sizeof(uint64_t));
    const char *th_env = getenv("OR_INDEX_THREADS");     /* tests: force a thread count */
    const long ncpu = th_env ? atol(th_env) : sysconf(_SC_NPROCESSORS_ONLN);
    int T = d->len > (1u << 22) ? (int)(ncpu < 1 ? 1 : ncpu > IX_THREADS ? IX_THREADS : ncpu) : 1;
    if (d->n > 0 && (uint64_t)T > d->n) T = (int)d->n;
    pthread_t th[IX_THREADS];
    ix_part part[IX_THREADS];
    uint64_t total = 0;
    for (int pass = 0; pass < 2; pass++) {
        if (pass == 1) {
            for (uint64_t c = 0; c < NB; c++) {
                uint64_t n = 0;
                for (int t = 0; t < T; t++) n += part[t].cnt[c];
                ix->off[c + 1] = ix->off[c] + n;
                uint64_t run = ix->off[c];
                for (int t = T; t-- > 0;) { const uint64_t k = part[t].cnt[c]; part[t].cnt[c] = run; run += k; }
            }
            for (int t = 0; t < T; t++) total += part[t].total;
            ix->pos = malloc((total + 1) * sizeof(uint64_t));
            ix->sid = malloc((total + 1) * sizeof(uint32_t));
        }
        for (int t = 0; t < T; t++) {
            if (pass == 0) part[t] = (ix_part){ d, code, calloc(NB, sizeof(uint64_t)), ix, d->n * t / T, d->n * (t + 1) / T, 0, 0 };
            part[t].pass = pass;
            pthread_create(&th[t], NULL, ix_part_run, &part[t]);
        }
        for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    }
    for (int t = 0; t < T; t++) free(part[t].cnt);
    free(code);
}

static void or_free_index(or_index *ix) { free(ix->off); free(ix->pos); free(ix->sid); }

/* ------------------------------------------------------------------ */
/* ungapped extension + e-value: alignmentFromQuickHits,               */
/* alignmentFunctions.c:276-387                                        */
/* ------------------------------------------------------------------ */
static uint64_t rec_hi(const or_seqs *s, uint64_t r) {
    /* last record's bound is total_len itself (:280-293) */
    return (r == s->n - 1) ? s->len : s->start[r + 1] - 1;
}

static void ungapped(const or_seqs *db, const or_seqs *q, uint64_t pd0, uint64_t pq0,
                     uint64_t r, uint64_t s, or_ug_out *o) {
    int64_t xs = (int64_t)db->start[s], xe = (int64_t)rec_hi(db, s);
    int64_t ys = (int64_t)q->start[r],  ye = (int64_t)rec_hi(q, r);
    int64_t end_x = (int64_t)pd0 - 1, beg_x = end_x - K + 1, beg_y = (int64_t)pq0 - K;
    int64_t sc = K * PT, best_r = sc, best_l = sc;
    uint64_t idents = K;
    /* forward from the base after the seed (:318-333) */
    for (int64_t x = (int64_t)pd0, y = (int64_t)pq0;
         sc > 0 && x < (int64_t)db->len && y < (int64_t)q->len && x <= xe && y <= ye; x++, y++) {
        if (db->seq[x] == q->seq[y]) { sc += PT; idents++; } else sc -= PT;
        if (best_r <= sc) { best_r = sc; end_x = x; }
    }
    /* backward from the base before the seed; the running score restarts at
     * the forward maximum while the left maximum keeps its initial 48 (:336-357) */
    sc = best_r;
    for (int64_t x = (int64_t)pd0 - K - 1, y = (int64_t)pq0 - K - 1;
         sc > 0 && x >= 0 && y >= 0 && x >= xs && y >= ys; x--, y--) {
        if (db->seq[x] == q->seq[y]) { sc += PT; idents++; } else sc -= PT;
        if (best_l <= sc) { best_l = sc; beg_x = x; beg_y = y; }
    }
    uint64_t t_len = (uint64_t)(end_x - beg_x);              /* not +1 (:359) */
    uint64_t raw = idents * PT - (t_len - idents) * PT;      /* u64 wrap arithmetic (:373) */
    long double rl = (r == q->n - 1) ? (long double)q->len - q->start[r]
                                     : (long double)q->start[r + 1] - q->start[r];
    o->x_start = (uint64_t)beg_x; o->y_start = (uint64_t)beg_y; o->t_len = t_len; o->raw = raw;
    /* same association order as :384 */
    o->e_value = (long double)0.333 * rl * db->len * expl(-0.275 * (long double)raw);
    o->e_value_d = (double)o->e_value;
}

/* ------------------------------------------------------------------ */
/* gapped alignment                                                    */
/* ------------------------------------------------------------------ */
typedef struct { int64_t s; uint32_t fx, fy; } ncell;
typedef struct {
    ncell   *T;   uint64_t Tcap;
    int64_t *cmS; uint64_t *cmX; uint64_t cmcap;
    char    *rx, *ry; uint64_t rcap;
    uint64_t hx, hy, M;         /* last backtrack heads */
} nw_work;

static void work_reserve(nw_work *w, uint64_t xl, uint64_t yl) {
    if (xl * yl > w->Tcap) { free(w->T); w->Tcap = xl * yl; w->T = malloc(w->Tcap * sizeof(ncell)); }
    if (yl > w->cmcap) {
        free(w->cmS); free(w->cmX); w->cmcap = yl;
        w->cmS = malloc(yl * sizeof(int64_t)); w->cmX = malloc(yl * sizeof(uint64_t));
    }
    uint64_t m = 2 * (xl > yl ? xl : yl) + 2;
    if (m > w->rcap) { free(w->rx); free(w->ry); w->rcap = m; w->rx = malloc(m); w->ry = malloc(m); }
}

static void work_free(nw_work *w) { free(w->T); free(w->cmS); free(w->cmX); free(w->rx); free(w->ry); }

/* NW, alignmentFunctions.c:389-489.  X = database record (rows), Y = read
 * (columns).  Row/column "jump" gap model with the reference's lags:
 *  - the row state is tested against T[i][j-2] but takes T[i-1][j-2] (:434-438)
 *  - column j-1's state holds the max over rows <= i-3, earliest on ties (:476-480)
 *  - ties: diagonal >=, then up > left (:457-472)
 *  - best cell over the last row / last column, ">=" in row-major order (:481-484). */
static void nw_fill(const uint8_t *X, uint64_t xl, const uint8_t *Y, uint64_t yl,
                    int64_t ig, int64_t eg, nw_work *w, int64_t *bs, uint64_t *bx, uint64_t *by) {
    ncell *T = w->T;
#define C(i, j) T[(uint64_t)(i) * yl + (j)]
    for (uint64_t j = 0; j < yl; j++) {
        C(0, j).s = (X[0] == Y[j]) ? PT : -PT;
        w->cmS[j] = C(0, j).s; w->cmX[j] = 0;
    }
    int64_t best = INT64_MIN; uint64_t bi = 0, bj = 0;
    for (uint64_t i = 1; i < xl; i++) {
        C(i, 0).s = (X[i] == Y[0]) ? PT : -PT;
        int64_t rs = C(i, 0).s; uint64_t rx = i, ry = 0;
        for (uint64_t j = 1; j < yl; j++) {
            if (j > 1 && rs <= C(i, j - 2).s) { rs = C(i - 1, j - 2).s; rx = i - 1; ry = j - 2; }
            int64_t m = (X[i] == Y[j]) ? PT : -PT;
            int64_t dg = C(i - 1, j - 1).s + m;
            int64_t lf = (j > 1) ? rs + ig + (int64_t)(j - ry - 1) * eg + m : INT64_MIN;
            int64_t up = (i > 1) ? w->cmS[j - 1] + ig + (int64_t)(i - w->cmX[j - 1] - 1) * eg + m : INT64_MIN;
            ncell *c = &C(i, j);
            if (dg >= lf && dg >= up)   { c->s = dg; c->fx = (uint32_t)(i - 1); c->fy = (uint32_t)(j - 1); }
            else if (up > lf)           { c->s = up; c->fx = (uint32_t)w->cmX[j - 1]; c->fy = (uint32_t)(j - 1); }
            else                        { c->s = lf; c->fx = (uint32_t)rx; c->fy = (uint32_t)ry; }
            if (i > 1 && j > 1 && C(i - 2, j - 1).s > w->cmS[j - 1]) {
                w->cmS[j - 1] = C(i - 2, j - 1).s; w->cmX[j - 1] = i - 2;
            }
            if ((i == xl - 1 || j == yl - 1) && c->s >= best) { best = c->s; bi = i; bj = j; }
        }
    }
    *bs = best; *bx = bi; *by = bj;
#undef C
}

/* backtrackingNW, alignmentFunctions.c:493-560: writes the two gapped
 * strings right-to-left from index M = 2*max(xlen,ylen).  A jump emits the
 * run of the longer side against '-' and drops the other side's character;
 * the origin cell itself is never emitted; leading '-' and ' ' padding. */
static void nw_back(const uint8_t *X, uint64_t xl, const uint8_t *Y, uint64_t yl, nw_work *w,
                    uint64_t bx, uint64_t by, or_nw_out *o) {
    ncell *T = w->T;
    uint64_t M = 2 * (xl > yl ? xl : yl);
    uint64_t hx = M, hy = M, k;
    char *rx = w->rx, *ry = w->ry;
    for (k = xl - 1; k > bx; k--) rx[hx--] = '-';
    for (k = yl - 1; k > by; k--) ry[hy--] = '-';
    uint64_t px = bx, py = by, cx = bx, cy = by;
    o->length = o->igaps = o->egaps = 0;
    while (cx > 0 && cy > 0) {
        ncell *c = &T[px * yl + py];
        cx = c->fx; cy = c->fy;
        if (cx + 1 == px && cy + 1 == py) {
            rx[hx--] = (char)X[px]; ry[hy--] = (char)Y[py]; o->length++;
        } else if (px - cx > py - cy) {
            for (k = px; k > cx; k--) { ry[hy--] = '-'; rx[hx--] = (char)X[k]; o->length++; o->egaps++; }
            o->igaps++; o->egaps--;
        } else {
            for (k = py; k > cy; k--) { rx[hx--] = '-'; ry[hy--] = (char)Y[k]; o->length++; o->egaps++; }
            o->igaps++; o->egaps--;
        }
        px = cx; py = cy;
    }
    for (k = 0; k < cx; k++) rx[hx--] = '-';
    for (k = 0; k < cy; k++) ry[hy--] = '-';
    if (cx >= cy) for (k = 0; k < cx; k++) ry[hy--] = ' ';
    else          for (k = 0; k < cy; k++) rx[hx--] = ' ';
    w->hx = hx; w->hy = hy; w->M = M;
    o->head_x = hx; o->head_y = hy;
}

/* build_alignment text loop, alignmentFunctions.c:230-271: 60-column X and Y
 * lines plus a '*' match line over X's span; identities are counted there.
 * text == NULL: count only.  Returns text length. */
static uint64_t nw_text(nw_work *w, char *text, uint64_t cap, uint64_t *idents) {
    uint64_t i = w->hx + 1, j = w->hy + 1, M = w->M, n = 0, id = 0;
    const char *rx = w->rx, *ry = w->ry;
#define PUT(ch) do { if (text && n < cap) text[n] = (ch); n++; } while (0)
    while (i <= M && j <= M) {
        uint64_t bi = i, bj = j, o;
        for (o = 0; o < IMSAME_ALIGN_LEN && i <= M; o++, i++) PUT(rx[i]);
        PUT('\n');
        for (o = 0; o < IMSAME_ALIGN_LEN && j <= M; o++, j++) PUT(ry[j]);
        PUT('\n');
        for (; bi < i; bi++, bj++) {
            /* short-circuit: Y is only read where X is not '-' */
            int star = rx[bi] != '-' && bj <= M && ry[bj] != '-' && rx[bi] == ry[bj];
            if (star) id++;
            PUT(star ? '*' : ' ');
        }
        PUT('\n');
    }
    PUT('\n');
#undef PUT
    *idents = id;
    return n;
}

static void nw_full(const uint8_t *X, uint64_t xl, const uint8_t *Y, uint64_t yl, int64_t ig, int64_t eg,
                    nw_work *w, or_nw_out *o) {
    work_reserve(w, xl, yl);
    nw_fill(X, xl, Y, yl, ig, eg, w, &o->score, &o->bx, &o->by);
    nw_back(X, xl, Y, yl, w, o->bx, o->by, o);
    nw_text(w, NULL, 0, &o->identities);
}

int or_nw(const char *X, uint64_t xl, const char *Y, uint64_t yl, int64_t ig, int64_t eg,
          or_nw_out *o, char *text, uint64_t cap, uint64_t *tlen) {
    if (xl < 2 || yl < 2) return IMSAME_E_ARG;          /* reference reads an unset best cell */
    nw_work w; memset(&w, 0, sizeof w);
    nw_full((const uint8_t *)X, xl, (const uint8_t *)Y, yl, ig, eg, &w, o);
    uint64_t id;
    uint64_t n = nw_text(&w, text, cap, &id);
    if (tlen) *tlen = n;
    work_free(&w);
    return 0;
}

int or_ungapped(const uint8_t *db, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
                const uint8_t *q, uint64_t q_len, const uint64_t *q_start, uint64_t n_q,
                uint64_t pos_db, uint64_t pos_q, uint64_t read, uint64_t dbseq,
                double min_e, or_ug_out *o) {
    or_seqs d = { (uint8_t *)db, (uint64_t *)db_start, n_db, db_len, NULL, 0 };
    or_seqs s = { (uint8_t *)q, (uint64_t *)q_start, n_q, q_len, NULL, 0 };
    ungapped(&d, &s, pos_db, pos_q, read, dbseq, o);
    long double me = (min_e < 0) ? 1 / powl(10, 20) : (long double)min_e;
    o->pass = o->e_value < me;
    return 0;
}

/* ------------------------------------------------------------------ */
/* per-thread scan: computeAlignmentsByThread, alignmentFunctions.c:43-208 */
/* ------------------------------------------------------------------ */
typedef struct {
    const or_seqs *db, *q;
    const or_index *ix;
    const imsame_params *prm;
    uint64_t from, to;
    imsame_read_result *res;       /* indexed by global read */
    char **texts;                  /* optional: text of accepted reads */
    int status; uint64_t err_read, err_dbseq;
    uint64_t n_nw;
    int mid;                       /* window view: start inside the chunk at read `from`,
                                      having borrowed start[from]-1 from the read before */
} or_chunk;

/* Test-speed option, off by default: skip the NW of a (read, record) pair
 * already rejected for this read.  Results are identical (NW is pure,
 * SURVEY Appendix A Q18); the reference recomputes, which makes long-read
 * (C5) cases with hundreds of e-value passes per read take minutes. */
static int g_memo_rejected;
void or_set_memo_rejected(int on) { g_memo_rejected = on; }

static void *scan_chunk(void *arg) {
    or_chunk *ch = arg;
    uint64_t memo_read = ~0ull, nmemo = 0, capmemo = 0, *memo = NULL;
    const or_seqs *db = ch->db, *q = ch->q;
    const imsame_params *prm = ch->prm;
    nw_work w; memset(&w, 0, sizeof w);
    uint64_t r = ch->from;
    /* An empty read at a chunk head makes the reference scan the rest of the
     * query as that read and reach NW with ylen = 0 (undefined behaviour).
     * Restated contract: skip it and let the next read open the chunk. */
    if (!ch->mid)
        while (r < ch->to && r + 1 < q->n && q->start[r] == q->start[r + 1]) r++;
    /* mid-chunk (a window): every read before `from` left p at start[from]-1,
     * accepted (:190) or scanned to its end (:93-105) */
    uint64_t p = ch->mid ? q->start[r] - 1 : (r < q->n) ? q->start[r] : q->len;
    unsigned run = 0;                  /* consecutive bases buffered (crrSeqL) */
    while (r < ch->to && p < q->len) {
        uint64_t lim = (r + 1 < q->n) ? q->start[r + 1] - 1 : q->len;
        if (p == lim) { run = 0; r++; continue; }  /* next read keeps p: borrows a base */
        run++;
        int done = 0;
        if (run >= K) {
            uint32_t code = kmer_code(q->seq + p + 1 - K);
            for (uint64_t h = ch->ix->off[code]; h < ch->ix->off[code + 1] && !done; h++) {
                uint64_t s = ch->ix->sid[h];
                or_ug_out u;
                ungapped(db, q, ch->ix->pos[h], p + 1, r, s, &u);
                if (!(u.e_value < prm->min_e)) continue;
                uint64_t xl = db->start[s + 1] - db->start[s];
                uint64_t yl = q->start[r + 1] - q->start[r];
                if (xl > prm->max_read_size || yl > prm->max_read_size) {
                    ch->status = IMSAME_E_READ_TOO_LONG; ch->err_read = r; ch->err_dbseq = s;
                    work_free(&w);
                    free(memo);
                    return NULL;
                }
                if (g_memo_rejected) {
                    if (memo_read != r) { memo_read = r; nmemo = 0; }
                    uint64_t k = 0;
                    while (k < nmemo && memo[k] != s) k++;
                    if (k < nmemo) continue;
                }
                or_nw_out o;
                nw_full(db->seq + db->start[s], xl, q->seq + q->start[r], yl, prm->igap, prm->egap, &w, &o);
                ch->n_nw++;
                if ((long double)o.length / yl >= prm->min_coverage &&
                    (long double)o.identities / o.length >= prm->min_identity) {
                    imsame_read_result *rr = &ch->res[r];
                    rr->db_seq = s; rr->score = o.score; rr->bx = (uint32_t)o.bx; rr->by = (uint32_t)o.by;
                    rr->length = (uint32_t)o.length; rr->identities = (uint32_t)o.identities;
                    rr->igaps = (uint32_t)o.igaps; rr->egaps = (uint32_t)o.egaps;
                    rr->head_x = (uint32_t)o.head_x; rr->head_y = (uint32_t)o.head_y;
                    rr->status = 1;
                    if (ch->texts) {
                        uint64_t id, n = nw_text(&w, NULL, 0, &id);
                        char *t = malloc(n + 1);
                        nw_text(&w, t, n, &id);
                        t[n] = 0;
                        ch->texts[r] = t;
                    }
                    done = 1;
                } else if (g_memo_rejected) {
                    if (nmemo == capmemo) {
                        capmemo = capmemo ? 2 * capmemo : 16;
                        memo = realloc(memo, capmemo * sizeof *memo);
                    }
                    memo[nmemo++] = s;
                }
            }
            if (!done) run--;
        }
        if (done) {
            if (r + 1 >= q->n) break;  /* reference jumps via start_pos[n] (unset): read over */
            p = q->start[r + 1] - 1;   /* == reference's start[r+1]-2 then ++ (:190,:198) */
            continue;
        }
        p++;
    }
    work_free(&w);
    free(memo);
    return NULL;
}

/* wall time of the last alignment phase (threads only, no loading/index) */
static double g_align_seconds;
double or_last_align_seconds(void) { return g_align_seconds; }
/* NW calls of the last or_align (distinct pairs when the rejected-pair memo is on) */
static uint64_t g_last_nw;
uint64_t or_last_nw(void) { return g_last_nw; }

/* Partition, IMSAME.c:414,430-452: rpt = floor(n/T); chunk i = [i*rpt,(i+1)*rpt),
 * the last chunk runs to n. */
static int run_chunks(const or_seqs *db, const or_seqs *q, const or_index *ix, const imsame_params *prm,
                      uint64_t T, imsame_read_result *res, char **texts, uint64_t *err_read,
                      uint64_t *err_dbseq, uint64_t *n_nw, int print_going) {
    if (T == 0) T = 1;
    uint64_t rpt = (uint64_t)floorl((long double)q->n / (long double)T);
    or_chunk *ch = calloc(T, sizeof(or_chunk));
    pthread_t *th = calloc(T, sizeof(pthread_t));
    for (uint64_t r = 0; r < q->n; r++) {
        memset(&res[r], 0, sizeof res[r]);
        res[r].ylen = (uint32_t)(q->start[r + 1] - q->start[r]);
    }
    for (uint64_t t = 0; t < T; t++) {
        ch[t].db = db; ch[t].q = q; ch[t].ix = ix; ch[t].prm = prm;
        ch[t].from = t * rpt; ch[t].to = (t == T - 1) ? q->n : (t + 1) * rpt;
        ch[t].res = res; ch[t].texts = texts;
        if (print_going) printf("Going from %" PRIu64 " to %" PRIu64 "\n", ch[t].from, ch[t].to);
    }
    if (print_going) fflush(stdout);
    struct timespec a0, a1;
    clock_gettime(CLOCK_MONOTONIC, &a0);
    for (uint64_t t = 0; t < T; t++) pthread_create(&th[t], NULL, scan_chunk, &ch[t]);
    for (uint64_t t = 0; t < T; t++) pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &a1);
    g_align_seconds = (a1.tv_sec - a0.tv_sec) + (a1.tv_nsec - a0.tv_nsec) * 1e-9;
    int st = 0;
    uint64_t nn = 0;
    for (uint64_t t = 0; t < T; t++) {
        nn += ch[t].n_nw;
        if (ch[t].status && (!st || ch[t].err_read < *err_read)) {
            st = ch[t].status; *err_read = ch[t].err_read; *err_dbseq = ch[t].err_dbseq;
        }
    }
    if (n_nw) *n_nw = nn;
    free(ch); free(th);
    return st;
}

int or_align(const uint8_t *dbs, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
             const uint8_t *db_brk,
             const uint8_t *qs, uint64_t q_len, const uint64_t *q_start, uint64_t n_q,
             const imsame_params *prm, uint64_t T, imsame_read_result *res, uint64_t *err_read) {
    or_seqs db = { (uint8_t *)dbs, malloc((n_db + 1) * sizeof(uint64_t)), n_db, db_len, NULL, 0 };
    or_seqs q  = { (uint8_t *)qs,  malloc((n_q + 1) * sizeof(uint64_t)),  n_q,  q_len,  NULL, 0 };
    memcpy(db.start, db_start, n_db * sizeof(uint64_t)); db.start[n_db] = db_len;
    memcpy(q.start, q_start, n_q * sizeof(uint64_t));    q.start[n_q] = q_len;
    /* record starts are resets: add them to a private copy of the bitmap */
    db.brk = calloc(db_len / 8 + 2, 1);
    if (db_brk) memcpy(db.brk, db_brk, (db_len + 7) / 8);
    for (uint64_t s = 0; s < n_db; s++)
        if (db.start[s] < db_len) db.brk[db.start[s] >> 3] |= (uint8_t)(1u << (db.start[s] & 7));
    or_index ix;
    struct timespec t0, t1, t2;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    or_build_index(&db, &ix);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    uint64_t er = 0, es = 0;
    int st = run_chunks(&db, &q, &ix, prm, T, res, NULL, &er, &es, &g_last_nw, 0);
    clock_gettime(CLOCK_MONOTONIC, &t2);
    if (getenv("OR_TIMING"))
        fprintf(stderr, "[oracle] index %.2f s, align %.2f s\n", (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec),
                (t2.tv_sec - t1.tv_sec) + 1e-9 * (t2.tv_nsec - t1.tv_nsec));
    if (err_read) *err_read = er;
    or_free_index(&ix);
    free(db.start); free(q.start); free(db.brk);
    return st;
}

/* or_align restricted to the reads of windows [from[w], to[w]) of the WHOLE
 * query: the same chunk heads (IMSAME.c:414,430-452), each chunk's part
 * inside a window scanned with the state the reference's thread has on
 * reaching it (a read inside a chunk borrows the previous read's last base,
 * Q4).  Lets tests compare windows deep inside a large query without
 * running all of it; the index is built once.  res: n_q entries (only the
 * windows' are written). */
int or_align_windows(const uint8_t *dbs, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
                     const uint8_t *db_brk, const uint8_t *qs, uint64_t q_len, const uint64_t *q_start, uint64_t n_q,
                     const imsame_params *prm, uint64_t T, uint64_t nwin, const uint64_t *wfrom, const uint64_t *wto,
                     imsame_read_result *res, uint64_t *err_read) {
    or_seqs db = { (uint8_t *)dbs, malloc((n_db + 1) * sizeof(uint64_t)), n_db, db_len, NULL, 0 };
    or_seqs q  = { (uint8_t *)qs,  malloc((n_q + 1) * sizeof(uint64_t)),  n_q,  q_len,  NULL, 0 };
    memcpy(db.start, db_start, n_db * sizeof(uint64_t)); db.start[n_db] = db_len;
    memcpy(q.start, q_start, n_q * sizeof(uint64_t));    q.start[n_q] = q_len;
    db.brk = calloc(db_len / 8 + 2, 1);
    if (db_brk) memcpy(db.brk, db_brk, (db_len + 7) / 8);
    for (uint64_t s = 0; s < n_db; s++)
        if (db.start[s] < db_len) db.brk[db.start[s] >> 3] |= (uint8_t)(1u << (db.start[s] & 7));
    or_index ix;
    or_build_index(&db, &ix);
    if (T == 0) T = 1;
    const uint64_t rpt = (uint64_t)floorl((long double)n_q / (long double)T);
    const uint64_t nc = T * nwin;
    or_chunk *ch = calloc(nc, sizeof(or_chunk));
    pthread_t *th = calloc(nc, sizeof(pthread_t));
    int *started = calloc(nc, sizeof(int));
    for (uint64_t w = 0; w < nwin; w++)
        for (uint64_t r = wfrom[w]; r < wto[w]; r++) {
            memset(&res[r], 0, sizeof res[r]);
            res[r].ylen = (uint32_t)(q.start[r + 1] - q.start[r]);
        }
    for (uint64_t w = 0; w < nwin; w++)
        for (uint64_t t = 0; t < T; t++) {
            const uint64_t f = t * rpt, e = (t == T - 1) ? n_q : (t + 1) * rpt;
            const uint64_t lo = f > wfrom[w] ? f : wfrom[w], hi = e < wto[w] ? e : wto[w];
            if (lo >= hi) continue;
            or_chunk *c = &ch[w * T + t];
            c->db = &db; c->q = &q; c->ix = &ix; c->prm = prm; c->res = res;
            c->from = lo; c->to = hi;
            /* the chunk's head role passes over empty reads: mid-chunk only
             * if a read of [f, lo) has bases */
            c->mid = lo > f && q.start[f] != q.start[lo];
            started[w * T + t] = pthread_create(&th[w * T + t], NULL, scan_chunk, c) == 0 ? 1 : 2;
            if (started[w * T + t] == 2) scan_chunk(c);
        }
    int st = 0;
    uint64_t er = 0, nn = 0;
    for (uint64_t k = 0; k < nc; k++) {
        if (started[k] == 1) pthread_join(th[k], NULL);
        if (started[k] && ch[k].status && (!st || ch[k].err_read < er)) { st = ch[k].status; er = ch[k].err_read; }
        nn += ch[k].n_nw;
    }
    g_last_nw = nn;
    if (err_read) *err_read = er;
    free(ch); free(th); free(started);
    or_free_index(&ix);
    free(db.start); free(q.start); free(db.brk);
    return st;
}

/* ------------------------------------------------------------------ */
/* reverse complement: reverseComplement.c:21-118                      */
/* ------------------------------------------------------------------ */
static uint8_t rc_base(uint8_t c) {
    switch (c) {
    case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; case 'U': return 'A';
    case 'a': return 't'; case 'c': return 'g'; case 'g': return 'c'; case 't': return 'a'; case 'u': return 'a';
    }
    return c;
}

int or_revcomp(const uint8_t *in, uint64_t n, uint8_t *out, uint64_t cap, uint64_t *out_len) {
    /* every '>' byte opens a record (:48-54), emitted last-to-first (:56) */
    uint64_t nr = 0, i, o = 0;
    for (i = 0; i < n; i++) nr += in[i] == '>';
    uint64_t *off = malloc((nr + 1) * sizeof(uint64_t));
    nr = 0;
    for (i = 0; i < n; i++) if (in[i] == '>') off[nr++] = i;
    for (uint64_t r = nr; r-- > 0;) {
        /* header: fgets up to and including '\n' (:59-62) */
        for (i = off[r]; i < n; i++) { if (o < cap) out[o] = in[i]; o++; if (in[i] == '\n') { i++; break; } }
        /* body: bytes up to the next '>' (:64-70); letters only, reversed */
        uint64_t b0 = i;
        while (i < n && in[i] != '>') i++;
        for (uint64_t k = i; k-- > b0;) {
            uint8_t c = in[k];
            if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z')) { if (o < cap) out[o] = rc_base(c); o++; }
        }
        if (o < cap) out[o] = '\n';
        o++;
    }
    free(off);
    *out_len = o;
    return o <= cap ? 0 : IMSAME_E_ARG;
}

/* ------------------------------------------------------------------ */
/* CLI: main + init_args, IMSAME.c:34-578                              */
/* ------------------------------------------------------------------ */
static int read_file(const char *path, uint8_t **buf, uint64_t *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseeko(f, 0, SEEK_END);
    uint64_t sz = (uint64_t)ftello(f);
    fseeko(f, 0, SEEK_SET);
    *buf = malloc(sz + 1);
    *n = fread(*buf, 1, sz, f);
    fclose(f);
    return 0;
}

static void die(const char *s) { printf("ERR**** %s ****\n", s); exit(-1); }

static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* IMSAME.c:44-49 defaults */
void or_params_default(imsame_params *p) {
    memset(p, 0, sizeof *p);
    p->min_e = 1 / powl(10, 20); p->min_coverage = 0.5; p->min_identity = 0.5;
    p->igap = -5; p->egap = -2; p->max_read_size = IMSAME_MAX_READ_SIZE;
}

int or_main(int argc, char **argv) {
    const char *qpath = NULL, *dpath = NULL, *opath = NULL;
    imsame_params prm;
    or_params_default(&prm);
    uint64_t T = 4;
    for (int a = 0; a < argc; a++) {
        if (!strcmp(argv[a], "--help")) {
            printf("USAGE:\n           IMSAME -query [query] -db [database]\n");
            exit(1);
        }
        if (a + 1 >= argc) continue;
        if (!strcmp(argv[a], "-query")) qpath = argv[a + 1];
        if (!strcmp(argv[a], "-db")) dpath = argv[a + 1];
        if (!strcmp(argv[a], "-out")) opath = argv[a + 1];
        if (!strcmp(argv[a], "-evalue")) { prm.min_e = (long double)atof(argv[a + 1]); if (prm.min_e < 0) die("Min-e-value must be larger than zero"); }
        if (!strcmp(argv[a], "-coverage")) { prm.min_coverage = (long double)atof(argv[a + 1]); if (prm.min_coverage <= 0) die("Min-coverage must be larger than zero"); }
        if (!strcmp(argv[a], "-identity")) { prm.min_identity = (long double)atof(argv[a + 1]); if (prm.min_identity <= 0) die("Min-identity must be larger than zero"); }
        if (!strcmp(argv[a], "-igap")) prm.igap = -atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-egap")) prm.egap = -atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-n_threads")) T = (uint64_t)atoi(argv[a + 1]);
        if (!strcmp(argv[a], "-max_read_size")) prm.max_read_size = strtoull(argv[a + 1], NULL, 10);
    }
    if (!qpath || !dpath) die("A query and database is required");
    double t0 = now_s();
    printf("[INFO] Init. quick table\n");
    printf("[INFO] Initialization took %e seconds \n", now_s() - t0);
    printf("[INFO] Loading database\n");
    uint8_t *buf; uint64_t nb;
    or_seqs db, q;
    t0 = now_s();
    if (read_file(dpath, &buf, &nb)) die("Could not open database file");
    or_parse_fasta(buf, nb, &db, 1);
    free(buf);
    or_index ix;
    or_build_index(&db, &ix);
    printf("[INFO] Database loaded and of length %" PRIu64 ". Hash table building took %e seconds\n", db.len, now_s() - t0);
    t0 = now_s();
    printf("[INFO] Loading query.\n");
    if (read_file(qpath, &buf, &nb)) die("Could not open query file");
    or_parse_fasta(buf, nb, &q, 0);
    free(buf);
    printf("[INFO] Query loaded and of length %" PRIu64 ". Took %e seconds\n", q.len, now_s() - t0);
    t0 = now_s();
    printf("[INFO] Computing alignments.\n");
    imsame_read_result *res = calloc(q.n + 1, sizeof *res);
    char **texts = calloc(q.n + 1, sizeof(char *));
    uint64_t er = 0, es = 0, nn = 0;
    int st = run_chunks(&db, &q, &ix, &prm, T, res, opath ? texts : NULL, &er, &es, &nn, 1);
    double ta = now_s() - t0;
    FILE *out = opath ? fopen(opath, "wt") : NULL;
    uint64_t acc = 0;
    for (uint64_t r = 0; r < q.n; r++) {
        if (st && r >= er) break;
        if (res[r].status != 1) continue;
        acc++;
        if (out) {
            uint64_t yl = res[r].ylen;
            uint64_t pid = 100 * (uint64_t)res[r].identities / res[r].length;
            uint64_t pcv = 100 * (uint64_t)res[r].length / yl;
            fprintf(out, "(%" PRIu64 ", %" PRIu64 ") : %d%% %d%% %" PRIu64 "\n $$$$$$$ \n", r, res[r].db_seq,
                    (int)pid < 100 ? (int)pid : 100, (int)pcv < 100 ? (int)pcv : 100, yl);
            fputs(texts[r], out);
        }
    }
    if (out) fclose(out);
    if (st == IMSAME_E_READ_TOO_LONG) die("Read size reached for gapped alignment.");
    printf("[INFO] Alignments computed in %e seconds.\n", ta);
    printf("[INFO] %" PRIu64 " reads (%" PRIu64 ") from the query were found in the database (%" PRIu64
           ") at a minimum e-value of %Le and minimum coverage of %d%%.\n",
           acc, q.n, db.n, prm.min_e, (int)(100 * prm.min_coverage));
    printf("[INFO] The Jaccard-index is: %Le\n", (long double)acc / ((db.n + q.n) - acc));
    printf("[INFO] Deallocating heap memory.\n");
    fprintf(stderr, "[ORACLE] nw=%" PRIu64 " align_s=%.6f\n", nn, ta);
    for (uint64_t r = 0; r < q.n; r++) free(texts[r]);
    free(texts); free(res);
    or_free_index(&ix); or_free_seqs(&db); or_free_seqs(&q);
    return 0;
}

#ifdef ORACLE_MAIN
int main(int argc, char **argv) { return or_main(argc, argv); }
#endif

/* test helper: run the loader on a byte image; caller buffers: seq n+1,
 * starts n+2 entries, brk n/8+2 bytes */
int or_parse(const uint8_t *buf, uint64_t n, int want_brk, uint8_t *seq, uint64_t *len, uint64_t *starts,
             uint64_t *nrec, uint8_t *brk) {
    or_seqs s;
    or_parse_fasta(buf, n, &s, want_brk);
    memcpy(seq, s.seq, s.len);
    memcpy(starts, s.start, (s.n + 1) * sizeof(uint64_t));
    if (want_brk && brk) memcpy(brk, s.brk, n / 8 + 2);
    *len = s.len; *nrec = s.n;
    or_free_seqs(&s);
    return 0;
}

/* test helper: glibc "%La" rendering of a long double held in memory */
int or_fmt_ld(const long double *x, char *buf, int cap) { return snprintf(buf, (size_t)cap, "%La", *x); }

/* test helpers: the reference's e-value and identity tests on given integers */
int or_epass(uint64_t raw, uint64_t ylen, uint64_t Ldb, const imsame_params *p) {
    long double e = (long double)0.333 * (long double)ylen * Ldb * expl(-0.275 * (long double)raw);
    return e < p->min_e;
}
int or_ident_ok(uint64_t ident, uint64_t len, const imsame_params *p) {
    return (long double)ident / len >= p->min_identity;
}
