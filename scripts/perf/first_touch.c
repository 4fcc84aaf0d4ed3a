// First-touch (zero-fill page fault) cost of fresh host memory, as the
// public API's result arrays pay it: one thread vs several, with and without
// MADV_HUGEPAGE, and a warm rewrite for the memory bandwidth itself.
#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
typedef struct { char* p; size_t n; } Arg;
static void* touch(void* a_) { Arg* a = a_; for (size_t i = 0; i < a->n; i += 4096) a->p[i] = 1; return 0; }
static double now(void) { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + t.tv_nsec * 1e-9; }
static double run(size_t n, int T, int huge) {
    char* p = mmap(0, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (huge) madvise(p, n, MADV_HUGEPAGE);
    double t0 = now();
    pthread_t th[64]; Arg a[64];
    for (int i = 0; i < T; ++i) { a[i].p = p + i * (n / T); a[i].n = n / T; pthread_create(&th[i], 0, touch, &a[i]); }
    for (int i = 0; i < T; ++i) pthread_join(th[i], 0);
    double ms = (now() - t0) * 1e3;
    t0 = now(); memset(p, 2, n); double warm = (now() - t0) * 1e3;
    munmap(p, n);
    printf("520 MB: threads %2d hugepage %d: first touch %.1f ms (warm memset %.1f ms)\n", T, huge, ms, warm);
    return ms;
}
int main(void) {
    size_t n = 520ull << 20;
    FILE* f = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r");
    char buf[128] = {0};
    if (f) { fgets(buf, sizeof buf, f); fclose(f); }
    printf("THP: %s", buf);
    for (int h = 0; h <= 1; ++h) for (int T = 1; T <= 16; T *= 2) run(n, T, h);
    return 0;
}
