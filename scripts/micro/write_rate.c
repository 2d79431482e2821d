/* write_rate.c -- how fast can one process put N GB of .align text into ONE
 * file on this filesystem?  (the CLI's output is ~3 GB at C2.)
 *   gcc -O2 -pthread -o write_rate write_rate.c && ./write_rate DIR [GB]
 * Modes: buffered pwrite from 1 / 4 / 16 threads at disjoint offsets (the
 * CLI's form), and O_DIRECT pwrite from 16 threads with 2 MiB aligned pieces
 * where the filesystem allows it.  Prints GB/s per mode. */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <sys/mman.h>
#include <unistd.h>
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }

typedef struct { int fd; char *buf; uint64_t off, len, piece; int err; } job;

static void *run(void *a) {
    job *j = a;
    for (uint64_t o = 0; o < j->len; o += j->piece) {
        uint64_t n = j->len - o < j->piece ? j->len - o : j->piece;
        const char *b = j->buf + (o % (64ull << 20));
        while (n) {
            ssize_t w = pwrite(j->fd, b, n, (off_t)(j->off + o));
            if (w < 0) { if (errno == EINTR) continue; j->err = errno; return NULL; }
            n -= (uint64_t)w; b += w; o += (uint64_t)w;
            if (n) o -= (uint64_t)w;
        }
    }
    return NULL;
}

static double trial(const char *path, int threads, int direct, uint64_t total, uint64_t piece, char *buf) {
    int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY | (direct ? O_DIRECT : 0), 0644);
    if (fd < 0) return -1;
    pthread_t th[64];
    job J[64];
    const double t0 = now();
    for (int k = 0; k < threads; ++k) {
        uint64_t a = total / threads * k, b = k + 1 == threads ? total : total / threads * (k + 1);
        a &= ~((uint64_t)(2 << 20) - 1); if (k + 1 < threads) b &= ~((uint64_t)(2 << 20) - 1);
        J[k] = (job){fd, buf, a, b - a, piece, 0};
        pthread_create(&th[k], NULL, run, &J[k]);
    }
    int err = 0;
    for (int k = 0; k < threads; ++k) { pthread_join(th[k], NULL); if (J[k].err) err = J[k].err; }
    const double t = now() - t0;
    close(fd);
    unlink(path);
    return err ? -err : total / t / 1e9;
}

/* a shared writable mapping of the file, pre-faulted by 16 threads
 * (MADV_POPULATE_WRITE) and then filled by 16 threads with memcpy: the two
 * phases timed apart (the first can run before the text exists) */
typedef struct { char *m; uint64_t a, b; const char *buf; int err; int pop; } mjob;
static void *mrun(void *p) {
    mjob *j = p;
    if (j->pop) { if (madvise(j->m + j->a, j->b - j->a, MADV_POPULATE_WRITE)) j->err = errno; return NULL; }
    for (uint64_t o = j->a; o < j->b; o += 8 << 20) {
        uint64_t n = j->b - o < (8u << 20) ? j->b - o : 8u << 20;
        memcpy(j->m + o, j->buf + (o % (64ull << 20)), n);
    }
    return NULL;
}
static void mmap_trial(const char *path, uint64_t total, const char *buf) {
    int fd = open(path, O_CREAT | O_TRUNC | O_RDWR, 0644);
    if (fd < 0 || ftruncate(fd, (off_t)total)) { printf("mmap: open/ftruncate failed\n"); return; }
    char *m = mmap(NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) { printf("mmap failed\n"); close(fd); return; }
    pthread_t th[16];
    mjob J[16];
    double ph[2];
    for (int pop = 1; pop >= 0; --pop) {
        const double t0 = now();
        for (int k = 0; k < 16; ++k) {
            uint64_t a = (total / 16 * k) & ~4095ull, b = k == 15 ? total : (total / 16 * (k + 1)) & ~4095ull;
            J[k] = (mjob){m, a, b, buf, 0, pop};
            pthread_create(&th[k], NULL, mrun, &J[k]);
        }
        int err = 0;
        for (int k = 0; k < 16; ++k) { pthread_join(th[k], NULL); if (J[k].err) err = J[k].err; }
        ph[pop] = err ? -err : now() - t0;
    }
    const double t1 = now();
    munmap(m, total);
    close(fd);
    const double tu = now() - t1;
    printf("mmap 16 threads: populate %.3f s, memcpy %.3f s (%.2f GB/s), munmap+close %.3f s\n", ph[1], ph[0],
           total / ph[0] / 1e9, tu);
    unlink(path);
}

int main(int argc, char **argv) {
    const char *dir = argc > 1 ? argv[1] : "/tmp";
    const double gb = argc > 2 ? atof(argv[2]) : 3.0;
    const uint64_t total = (uint64_t)(gb * 1e9);
    char path[512];
    snprintf(path, sizeof path, "%s/write_rate.tmp", dir);
    char *buf = aligned_alloc(1 << 21, (64ull << 20) + (16 << 20));
    for (uint64_t k = 0; k < (64ull << 20) + (16 << 20); ++k) buf[k] = "ACGT*- \n"[k & 7];
    const int T[] = {1, 4, 16};
    for (int i = 0; i < 3; ++i)
        printf("buffered pwrite %2d threads: %6.2f GB/s\n", T[i], trial(path, T[i], 0, total, 8 << 20, buf));
    printf("O_DIRECT pwrite 16 threads: %6.2f GB/s (negative: errno)\n", trial(path, 16, 1, total, 2 << 20, buf));
    printf("buffered pwrite 16 threads, 64 KiB pieces: %6.2f GB/s\n", trial(path, 16, 0, total, 64 << 10, buf));
    mmap_trial(path, total, buf);
    free(buf);
    return 0;
}
