/* CPU probe of the rank host-thread pool (host/host_cpus.c): argv[1] engines
 * run a host phase at the same time, each asking for argv[2] helpers; prints
 * "budget B peak P helpers H" where P is the most threads (callers + granted
 * helpers) and H the most granted helpers inside host phases at once. Built and run by tests/test_host_budget.py. */
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

int vp8g_rank_threads(int device);
int vp8g_helpers_take(int device, int want);
void vp8g_helpers_give(int grant);

static atomic_int g_inside, g_peak, g_help, g_hpeak;
static pthread_barrier_t g_bar;
static int g_want;

static void bump(atomic_int* cur, atomic_int* peak, int k) {
  const int v = atomic_fetch_add(cur, k) + k;
  int p = atomic_load(peak);
  while (v > p && !atomic_compare_exchange_weak(peak, &p, v)) {}
}

static void* engine(void* arg) {
  (void)arg;
  for (int it = 0; it < 200; ++it) {
    pthread_barrier_wait(&g_bar);
    const int grant = vp8g_helpers_take(0, g_want);
    bump(&g_inside, &g_peak, grant + 1);
    bump(&g_help, &g_hpeak, grant);
    usleep(50);
    atomic_fetch_sub(&g_help, grant);
    atomic_fetch_sub(&g_inside, grant + 1);
    vp8g_helpers_give(grant);
  }
  return NULL;
}

int main(int argc, char** argv) {
  const int engines = argc > 1 ? atoi(argv[1]) : 6;
  g_want = argc > 2 ? atoi(argv[2]) : 15;
  pthread_t th[64];
  pthread_barrier_init(&g_bar, NULL, (unsigned)engines);
  for (int e = 0; e < engines; ++e) pthread_create(&th[e], NULL, engine, NULL);
  for (int e = 0; e < engines; ++e) pthread_join(th[e], NULL);
  printf("budget %d peak %d helpers %d\n", vp8g_rank_threads(0), atomic_load(&g_peak),
         atomic_load(&g_hpeak));
  return 0;
}
