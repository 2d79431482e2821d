/* imsame_host.c -- FASTA loading and .align rendering for the CLI. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
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

int host_load_fasta(const char *path, int want_brk, host_seqs *s) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseeko(f, 0, SEEK_END);
    const uint64_t sz = (uint64_t)ftello(f);
    fseeko(f, 0, SEEK_SET);
    uint8_t *buf = malloc(sz + 1);
    if (!buf) { fclose(f); return -1; }
    const uint64_t got = fread(buf, 1, sz, f);
    fclose(f);
    const int rc = host_parse_fasta(buf, got, want_brk, s);
    free(buf);
    return rc;
}

void host_free_seqs(host_seqs *s) {
    free(s->seq); free(s->start); free(s->brk);
    memset(s, 0, sizeof *s);
}

static void text_reserve(host_text *t, size_t n) {
    if (t->len + n <= t->cap) return;
    t->cap = (t->len + n) * 2 + 4096;
    t->buf = realloc(t->buf, t->cap);
}

uint64_t host_render(const uint8_t *X, uint64_t xlen, const uint8_t *Y, uint64_t ylen, const imsame_read_result *r,
                     const uint32_t *path, host_text *t) {
    const uint64_t M = 2 * (xlen > ylen ? xlen : ylen);
    char *rx = malloc(2 * M + 4), *ry = malloc(2 * M + 4);
    memset(rx, 0, 2 * M + 4);
    memset(ry, 0, 2 * M + 4);
    uint64_t hx = M, hy = M, k;
    for (k = xlen - 1; k > r->bx; k--) rx[hx--] = '-';
    for (k = ylen - 1; k > r->by; k--) ry[hy--] = '-';
    uint64_t px = r->bx, py = r->by;
    for (uint32_t e = 0; e < r->path_len; ++e) {
        const uint32_t mv = path[e] >> 30, n = path[e] & 0x3FFFFFFFu;
        if (mv == IMSAME_MOVE_DIAG) {
            for (uint32_t d = 0; d < n; ++d) { rx[hx--] = (char)X[px--]; ry[hy--] = (char)Y[py--]; }
        } else if (mv == IMSAME_MOVE_UP) {
            for (uint32_t d = 0; d < n; ++d) { ry[hy--] = '-'; rx[hx--] = (char)X[px - d]; }
            px -= n; py -= 1;
        } else {
            for (uint32_t d = 0; d < n; ++d) { rx[hx--] = '-'; ry[hy--] = (char)Y[py - d]; }
            py -= n; px -= 1;
        }
    }
    for (k = 0; k < px; k++) rx[hx--] = '-';
    for (k = 0; k < py; k++) ry[hy--] = '-';
    if (px >= py) for (k = 0; k < px; k++) ry[hy--] = ' ';
    else          for (k = 0; k < py; k++) rx[hx--] = ' ';
    /* build_alignment's loop (:233-271) */
    t->len = 0;
    uint64_t i = hx + 1, j = hy + 1, ident = 0;
    while (i <= M && j <= M) {
        text_reserve(t, 3 * IMSAME_ALIGN_LEN + 8);
        uint64_t bi = i, bj = j, o;
        for (o = 0; o < IMSAME_ALIGN_LEN && i <= M; o++, i++) t->buf[t->len++] = rx[i];
        t->buf[t->len++] = '\n';
        for (o = 0; o < IMSAME_ALIGN_LEN && j <= M; o++, j++) t->buf[t->len++] = ry[j];
        t->buf[t->len++] = '\n';
        for (; bi < i; bi++, bj++) {
            const int star = rx[bi] != '-' && ry[bj] != '-' && rx[bi] == ry[bj];
            ident += star;
            t->buf[t->len++] = star ? '*' : ' ';
        }
        t->buf[t->len++] = '\n';
    }
    text_reserve(t, 2);
    t->buf[t->len++] = '\n';
    free(rx);
    free(ry);
    return ident;
}
