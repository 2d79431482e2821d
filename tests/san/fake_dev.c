/* fake_dev.c -- TEST INFRASTRUCTURE for the host sanitizer runs
 * (scripts/sanitize.sh): a CPU stand-in for the five device entry points the
 * host pipeline calls (include/imsame_dev.h), so imsame_pipe.c's threads --
 * per-device workers, the library's lane threads delivering parts through the
 * callback, the render pool and the writer -- run under ThreadSanitizer /
 * AddressSanitizer without a GPU.  Results are synthetic but valid (a
 * diagonal path inside the record) and depend only on the read index, so a
 * run's output is independent of how the work was cut.  Never linked into the
 * product. */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "../../include/imsame_dev.h"

struct imsame_ctx {
    const uint64_t *db_start;
    uint64_t n_db, db_len;
    const uint64_t *q_start;
    uint64_t n_q, q_len;
};

int imsame_dev_open(int device, imsame_ctx **out) {
    (void)device;
    *out = calloc(1, sizeof **out);
    return *out ? IMSAME_OK : IMSAME_E_OOM;
}

void imsame_dev_close(imsame_ctx *c) { free(c); }

int imsame_dev_index(imsame_ctx *c, const uint8_t *db_seq, uint64_t db_len, const uint64_t *db_start, uint64_t n_db,
                     const uint8_t *db_brk) {
    (void)db_seq; (void)db_brk;
    c->db_start = db_start; c->n_db = n_db; c->db_len = db_len;
    return IMSAME_OK;
}

int imsame_dev_set_query_range(imsame_ctx *c, const uint8_t *q_seq, uint64_t q_len, const uint64_t *q_start,
                               uint64_t n_q, uint64_t read_from, uint64_t read_to) {
    (void)q_seq; (void)read_from; (void)read_to;
    c->q_start = q_start; c->n_q = n_q; c->q_len = q_len;
    return IMSAME_OK;
}

/* the synthetic outcome of read r (1 diagonal run of ylen-1 steps) */
void fake_result(const imsame_ctx *c, uint64_t r, imsame_read_result *o, uint32_t *path) {
    memset(o, 0, sizeof *o);
    const uint64_t yl = c->q_start[r + 1] - c->q_start[r];
    o->ylen = (uint32_t)yl;
    if (yl < 2 || r % 7 == 3) return;                        /* not found */
    const uint64_t s = (r * 2654435761u) % c->n_db;
    const uint64_t xl = c->db_start[s + 1] - c->db_start[s];
    if (xl <= yl + 1) return;
    const uint64_t off = 1 + (r * 37) % (xl - yl - 1);
    o->status = 1; o->db_seq = s;
    o->bx = (uint32_t)(off + yl - 1); o->by = (uint32_t)(yl - 1);
    o->length = (uint32_t)(yl - 1); o->identities = (uint32_t)(yl - 1 - r % 5);
    /* backtrackingNW's string heads as the device reports them (nw_finish:
     * M - ((xlen-1-bx) + length + tail), tail = the walk's end px + py = off) */
    const uint64_t M = 2 * (xl > yl ? xl : yl);
    o->head_x = (uint32_t)(M - (xl - 1)); o->head_y = (uint32_t)(M - (yl - 1 + off));
    o->path_len = 1;
    *path = (IMSAME_MOVE_DIAG << 30) | (uint32_t)(yl - 1);
}

typedef struct {
    imsame_ctx *c;
    const uint64_t *cut;              /* piece i = reads [cut[i], cut[i+1]) */
    int k, nl, np;                    /* this lane runs pieces k, k + nl, ... */
    imsame_read_result *res;          /* res[r - base] */
    uint64_t base;
    imsame_part_fn fn;
    void *user;
    int want_paths;
} lane;

static void *lane_run(void *p) {
    lane *l = p;
    for (int i = l->k; i < l->np; i += l->nl) {
        const uint64_t a = l->cut[i], b = l->cut[i + 1];
        uint32_t *paths = malloc((b - a + 1) * sizeof *paths);
        uint64_t np = 0;
        for (uint64_t r = a; r < b; ++r) {
            imsame_read_result *o = &l->res[r - l->base];
            fake_result(l->c, r, o, paths + np);
            if (o->status == 1 && l->want_paths) { o->path_off = (uint32_t)np; np += o->path_len; }
        }
        /* a lane hands over each piece from its own thread, as the library's do */
        l->fn(l->user, a, b, IMSAME_OK, ~0ull, np ? paths : NULL, np);
        free(paths);
    }
    return NULL;
}

/* as imsame_dev.hip:align_impl with a callback: NL lanes on their own
 * threads, each lane's share cut into IMSAME_LANE_PARTS pieces (3 by
 * default), piece i on lane i mod NL, handed over as each one ends */
int imsame_dev_align_parts(imsame_ctx *c, uint64_t read_from, uint64_t read_to, uint64_t n_threads_semantic,
                           const imsame_params *prm, imsame_read_result *res, imsame_part_fn part, void *user,
                           imsame_stats *stats) {
    (void)n_threads_semantic;
    enum { NL = 3 };
    const char *pe = getenv("IMSAME_LANE_PARTS");
    int ns = pe ? atoi(pe) : 3;
    ns = ns < 1 ? 1 : ns > 16 ? 16 : ns;
    const int np = NL * ns;
    uint64_t cut[3 * 16 + 1];
    lane L[NL];
    pthread_t th[NL];
    const uint64_t n = read_to - read_from;
    for (int i = 0; i <= np; ++i) cut[i] = read_from + n * (uint64_t)i / (uint64_t)np;
    for (int k = 0; k < NL; ++k)
        L[k] = (lane){c, cut, k, NL, np, res, read_from, part, user, prm->want_paths};
    for (int k = 1; k < NL; ++k) pthread_create(&th[k], NULL, lane_run, &L[k]);
    lane_run(&L[0]);
    for (int k = 1; k < NL; ++k) pthread_join(th[k], NULL);
    if (stats) { memset(stats, 0, sizeof *stats); stats->n_reads = n; stats->lanes = NL; stats->err_read = ~0ull; }
    return IMSAME_OK;
}
