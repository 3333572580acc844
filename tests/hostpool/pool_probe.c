/* CPU probe of the rank host-thread pool (host/host_cpus.c): argv[1] engines
 * each submit a job of argv[2] items (a few hundred microseconds of work
 * each) with width argv[3], 100 times, all at once; prints
 * "budget B threads T peak P items I" where T is the number of distinct
 * threads that ran items, P the most items running at once and I the items
 * run (every item exactly once). Built and run by tests/test_host_budget.py. */
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "host/gpu_engine.h"

static atomic_int g_inside, g_peak, g_items, g_nthreads;
static pthread_barrier_t g_bar;
static int g_n, g_width;
static __thread int t_seen;

static void item(void* ctx, int i) {
  atomic_int* hits = (atomic_int*)ctx;
  atomic_fetch_add(&hits[i], 1);
  if (!t_seen) { t_seen = 1; atomic_fetch_add(&g_nthreads, 1); }
  const int v = atomic_fetch_add(&g_inside, 1) + 1;
  int p = atomic_load(&g_peak);
  while (v > p && !atomic_compare_exchange_weak(&g_peak, &p, v)) {}
  usleep(200);
  atomic_fetch_sub(&g_inside, 1);
  atomic_fetch_add(&g_items, 1);
}

static void* engine(void* arg) {
  (void)arg;
  atomic_int* hits = calloc((size_t)g_n, sizeof(atomic_int));
  for (int it = 0; it < 100; ++it) {
    pthread_barrier_wait(&g_bar);
    memset(hits, 0, (size_t)g_n * sizeof(atomic_int));
    vp8g_job j;
    vp8g_job_submit(0, &j, item, hits, g_n, g_width);
    vp8g_job_join(&j);
    for (int i = 0; i < g_n; ++i)
      if (atomic_load(&hits[i]) != 1) { printf("item %d ran %d times\n", i, hits[i]); exit(1); }
  }
  free(hits);
  return NULL;
}

int main(int argc, char** argv) {
  const int engines = argc > 1 ? atoi(argv[1]) : 6;
  g_n = argc > 2 ? atoi(argv[2]) : 64;
  g_width = argc > 3 ? atoi(argv[3]) : 15;
  pthread_t th[64];
  pthread_barrier_init(&g_bar, NULL, (unsigned)engines);
  for (int e = 0; e < engines; ++e) pthread_create(&th[e], NULL, engine, NULL);
  for (int e = 0; e < engines; ++e) pthread_join(th[e], NULL);
  printf("budget %d threads %d peak %d items %d\n", vp8g_rank_threads(0),
         atomic_load(&g_nthreads), atomic_load(&g_peak), atomic_load(&g_items));
  return 0;
}
