/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
 *
 * A small harness that links the *unmodified* reference sources
 * (/root/reference/src/alignmentFunctions.c, commonFunctions.c) and calls
 * their external symbols on arbitrary inputs, so that golden vectors can be
 * generated for the unit-level parity tests:
 *
 *   NW                      /root/reference/src/alignmentFunctions.c:389-489
 *   backtrackingNW          /root/reference/src/alignmentFunctions.c:493-560
 *   build_alignment         /root/reference/src/alignmentFunctions.c:210-274
 *   alignmentFromQuickHits  /root/reference/src/alignmentFunctions.c:276-387
 *
 * Built by oracle/Makefile into oracle/_ref/ref_driver (git-ignored).
 *
 * Protocol (stdin, one command per line, whitespace separated):
 *   nw <igap> <egap> <X> <Y>
 *       -> "score bx by length identities igaps egaps head_x head_y textlen\n"
 *          followed by the alignment text exactly as build_alignment renders it
 *          (textlen bytes) and a terminating "\n".
 *   db <n> <seq0> ... <seq{n-1}>     (load database records, ACGT only)
 *   q  <n> <seq0> ... <seq{n-1}>     (load query reads)
 *   ug <pos_db> <pos_q> <read> <dbseq>
 *       -> "x_start y_start t_len e_hex e_dec\n"  (long double printed %La / %.21Le)
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <inttypes.h>
#include "structs.h"
#include "alignmentFunctions.h"
#include "commonFunctions.h"

static struct cell **g_table;
static struct positioned_cell *g_mc;
static char *g_rx, *g_ry, *g_text;
static unsigned char *g_mx, *g_my;

static SeqInfo g_db, g_q;

static char *read_token(void) {
    static char *buf = NULL;
    static size_t cap = 0;
    int c;
    size_t n = 0;
    do { c = getchar(); } while (c == ' ' || c == '\n' || c == '\t' || c == '\r');
    if (c == EOF) return NULL;
    while (c != EOF && c != ' ' && c != '\n' && c != '\t' && c != '\r') {
        if (n + 2 > cap) { cap = cap ? cap * 2 : 4096; buf = realloc(buf, cap); }
        buf[n++] = (char)c;
        c = getchar();
    }
    buf[n] = 0;
    return buf;
}

static void load_seqs(SeqInfo *si) {
    uint64_t n = strtoull(read_token(), NULL, 10), i, total = 0;
    free(si->sequences); free(si->start_pos);
    si->start_pos = malloc((n + 1) * sizeof(uint64_t));
    si->sequences = NULL;
    size_t cap = 0;
    for (i = 0; i < n; i++) {
        char *t = read_token();
        size_t l = (t[0] == '.') ? 0 : strlen(t);      /* "." denotes an empty record */
        if (total + l + 1 > cap) { cap = (total + l + 1) * 2; si->sequences = realloc(si->sequences, cap); }
        si->start_pos[i] = total;
        memcpy(si->sequences + total, t, l);
        total += l;
    }
    if (!si->sequences) si->sequences = malloc(1);
    si->n_seqs = n;
    si->total_len = total;
}

int main(void) {
    uint64_t i;
    g_table = malloc(MAX_READ_SIZE * sizeof(struct cell *));
    for (i = 0; i < MAX_READ_SIZE; i++) g_table[i] = malloc(MAX_READ_SIZE * sizeof(struct cell));
    g_mc = malloc(MAX_READ_SIZE * sizeof(struct positioned_cell));
    g_mx = malloc(MAX_READ_SIZE + 8);
    g_my = malloc(MAX_READ_SIZE + 8);
    /* +8: the reference writes rec[2*MAX_READ_SIZE] when a length is exactly MAX_READ_SIZE */
    g_rx = malloc(2 * MAX_READ_SIZE + 8);
    g_ry = malloc(2 * MAX_READ_SIZE + 8);
    g_text = malloc((size_t)MAX_READ_SIZE * MAX_READ_SIZE);
    memset(&g_db, 0, sizeof g_db);
    memset(&g_q, 0, sizeof g_q);

    char *cmd;
    while ((cmd = read_token()) != NULL) {
        if (strcmp(cmd, "nw") == 0) {
            int igap = atoi(read_token());
            int egap = atoi(read_token());
            char *tx = strdup(read_token());
            char *ty = strdup(read_token());
            uint64_t xlen = strlen(tx), ylen = strlen(ty);
            SeqInfo dx = { (unsigned char *)tx, NULL, xlen, 1 };
            SeqInfo dy = { (unsigned char *)ty, NULL, ylen, 1 };
            uint64_t s0 = 0;
            dx.start_pos = &s0; dy.start_pos = &s0;
            HashTableArgs hta;
            memset(&hta, 0, sizeof hta);
            hta.database = &dx; hta.query = &dy; hta.igap = igap; hta.egap = egap;
            memcpy(g_mx, tx, xlen); memcpy(g_my, ty, ylen);
            struct positioned_cell bc = NW(g_mx, 0, xlen, g_my, 0, ylen, igap, egap, g_table, g_mc, 0);
            BasicAlignment ba;
            ba.identities = ba.length = ba.igaps = ba.egaps = 0;
            /* build_alignment recomputes NW itself (NW is pure: SURVEY Appendix A Q18). */
            build_alignment(g_rx, g_ry, 0, 0, &hta, g_mx, g_my, g_table, g_mc, g_text, &ba, xlen, ylen);
            uint64_t hx, hy;
            BasicAlignment ba2;
            ba2.identities = ba2.length = ba2.igaps = ba2.egaps = 0;
            NW(g_mx, 0, xlen, g_my, 0, ylen, igap, egap, g_table, g_mc, 0);
            backtrackingNW(g_mx, 0, xlen, g_my, 0, ylen, g_table, g_rx, g_ry, &bc, &hx, &hy, &ba2);
            size_t tl = strlen(g_text);
            printf("%" PRId64 " %" PRIu64 " %" PRIu64 " %" PRIu64 " %" PRIu64 " %" PRIu64 " %" PRIu64
                   " %" PRIu64 " %" PRIu64 " %zu\n",
                   bc.score, bc.xpos, bc.ypos, ba.length, ba.identities, ba.igaps, ba.egaps, hx, hy, tl);
            fwrite(g_text, 1, tl, stdout);
            printf("\n");
            fflush(stdout);
            free(tx); free(ty);
        } else if (strcmp(cmd, "db") == 0) {
            load_seqs(&g_db);
        } else if (strcmp(cmd, "q") == 0) {
            load_seqs(&g_q);
        } else if (strcmp(cmd, "ug") == 0) {
            uint64_t pd = strtoull(read_token(), NULL, 10);
            uint64_t pq = strtoull(read_token(), NULL, 10);
            uint64_t r = strtoull(read_token(), NULL, 10);
            uint64_t s = strtoull(read_token(), NULL, 10);
            Quickfrag qf;
            memset(&qf, 0, sizeof qf);
            alignmentFromQuickHits(&g_db, &g_q, pd, pq, r, s, &qf);
            printf("%" PRIu64 " %" PRIu64 " %" PRIu64 " %La %.21Le\n", qf.x_start, qf.y_start, qf.t_len,
                   qf.e_value, qf.e_value);
            fflush(stdout);
        } else {
            fprintf(stderr, "unknown command %s\n", cmd);
            return 2;
        }
    }
    return 0;
}
