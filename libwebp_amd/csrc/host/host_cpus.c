/* Host-thread placement ("each GPU runs its own batch
 * pipeline and host-tail pool; pin host threads to the GPU's NUMA node").
 *
 * The CPUs an engine's host threads may use: the NUMA node of its GPU (from
 * the device's PCI address in sysfs), intersected with this process's
 * affinity mask, split evenly between the ranks that share the node. Ranks
 * are one process per GPU with local rank r on device r (torchrun's
 * LOCAL_WORLD_SIZE ranks over the visible devices); a single process (no
 * LOCAL_WORLD_SIZE) keeps the whole node. When the node is unknown (no sysfs
 * entry, a node with none of our CPUs) nothing is pinned.
 * WEBP_AMD_NO_PIN=1 turns placement off. */
#define _GNU_SOURCE
#include <ctype.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "gpu_engine.h"
#include "webp/encode_gpu.h"

#define MAX_DEV 64

typedef struct {
  int done, ncpu;
  cpu_set_t set;
} DevCpus;

static DevCpus g_dev[MAX_DEV];
static pthread_mutex_t g_lock = PTHREAD_MUTEX_INITIALIZER;

static int device_numa_node(int device) {
  char bus[64], path[160];
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), device) != hipSuccess) return -1;
  for (char* p = bus; *p; ++p) *p = (char)tolower((unsigned char)*p);
  snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node;
}

/* "0-23,48-71" -> set; returns the number of CPUs read */
static int read_cpulist(int node, cpu_set_t* set) {
  char path[96], buf[4096];
  snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  CPU_ZERO(set);
  int count = 0;
  for (char* p = buf; *p;) {
    if (!isdigit((unsigned char)*p)) { ++p; continue; }
    char* end;
    const long a = strtol(p, &end, 10);
    long b = a;
    if (*end == '-') b = strtol(end + 1, &end, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) {
      if (!CPU_ISSET((int)c, set)) ++count;
      CPU_SET((int)c, set);
    }
    p = end;
  }
  return count;
}

static void compute(int device, DevCpus* d) {
  d->ncpu = 0;
  const char* off = getenv("WEBP_AMD_NO_PIN");
  if (off && off[0] == '1') return;
  const int node = device_numa_node(device);
  if (node < 0) return;
  cpu_set_t nodeset, mine;
  if (read_cpulist(node, &nodeset) <= 0) return;
  if (sched_getaffinity(0, sizeof(mine), &mine) != 0) return;
  int cpus[CPU_SETSIZE], n = 0;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &nodeset) && CPU_ISSET(c, &mine)) cpus[n++] = c;
  if (n == 0) return;
  /* ranks on this node: local rank k drives device k mod the device count
   * (one rank per GPU, or every rank on one GPU in a one-GPU test); this
   * process's slot comes from LOCAL_RANK when the launcher sets it, else
   * from the device index */
  int ndev = 0, ranks = 1, idx = 0;
  const char* lw = getenv("LOCAL_WORLD_SIZE");
  const char* lr = getenv("LOCAL_RANK");
  const int local_world = lw ? atoi(lw) : 1;
  const int local_rank = lr ? atoi(lr) : device;
  if (local_world > 1 && hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
    ranks = 0;
    for (int k = 0; k < local_world; ++k) {
      if (device_numa_node(k % ndev) != node) continue;
      if (k < local_rank) ++idx;
      ++ranks;
    }
    if (ranks < 1) ranks = 1;
    if (idx >= ranks) idx = ranks - 1;
  }
  int share = n / ranks;
  if (share < 1) share = 1;
  const int lo = (idx * share) % n;
  CPU_ZERO(&d->set);
  for (int k = 0; k < share; ++k) CPU_SET(cpus[(lo + k) % n], &d->set);
  d->ncpu = share;
}

/* The CPU set of `device`'s host threads (NULL: no placement); *ncpu its size. */
const cpu_set_t* vp8g_device_cpus(int device, int* ncpu) {
  *ncpu = 0;
  if (device < 0 || device >= MAX_DEV) return NULL;
  pthread_mutex_lock(&g_lock);
  DevCpus* d = &g_dev[device];
  if (!d->done) {
    compute(device, d);
    d->done = 1;
  }
  pthread_mutex_unlock(&g_lock);
  *ncpu = d->ncpu;
  return d->ncpu > 0 ? &d->set : NULL;
}

/* pthread_create with the device's CPU set (plain create without one) */
int vp8g_thread_create(pthread_t* th, void* (*fn)(void*), void* arg, int device) {
  int ncpu = 0;
  const cpu_set_t* set = vp8g_device_cpus(device, &ncpu);
  if (!set) return pthread_create(th, NULL, fn, arg);
  pthread_attr_t attr;
  if (pthread_attr_init(&attr) != 0) return pthread_create(th, NULL, fn, arg);
  int rc = pthread_attr_setaffinity_np(&attr, sizeof(cpu_set_t), set);
  rc = rc == 0 ? pthread_create(th, &attr, fn, arg) : pthread_create(th, NULL, fn, arg);
  pthread_attr_destroy(&attr);
  return rc;
}

int WebPGpuHostCpus(int device, int* cpus, int max_cpus) {
  int ncpu = 0, k = 0;
  const cpu_set_t* set = vp8g_device_cpus(device, &ncpu);
  if (!set) return 0;
  for (int c = 0; c < CPU_SETSIZE && k < ncpu; ++c)
    if (CPU_ISSET(c, set)) {
      if (cpus && k < max_cpus) cpus[k] = c;
      ++k;
    }
  return k;
}

int vp8g_device_ncpu(int device) {
  int ncpu = 0;
  (void)vp8g_device_cpus(device, &ncpu);
  return ncpu;
}

/* ---- host-thread budget of a rank ---------------------------------------
 * A rank's host threads share its CPU quota: the cgroup CPU quota (v2
 * cpu.max, v1 cfs_quota_us; WEBP_AMD_CPU_QUOTA overrides it, tests use that)
 * divided by the ranks of the node (LOCAL_WORLD_SIZE), capped by the pinned
 * NUMA share above and by the online CPUs. Every engine of the process runs
 * the per-frame items of its host phases on one persistent pool of budget - 1
 * threads (below) plus its own calling thread, so six engines per rank and
 * eight ranks per node stay at about one busy host thread per quota CPU. */

/* CPUs granted by the cgroup CPU quota, 0 when there is none */
static double cgroup_quota(void) {
  const char* o = getenv("WEBP_AMD_CPU_QUOTA");
  if (o && atof(o) > 0) return atof(o);
  FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r");
  if (f) {
    char q[32] = {0};
    long per = 0;
    const int got = fscanf(f, "%31s %ld", q, &per);
    fclose(f);
    if (got == 2 && strcmp(q, "max") != 0 && per > 0) return atof(q) / (double)per;
  }
  long q = 0, per = 0;
  f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r");
  if (f) {
    if (fscanf(f, "%ld", &q) != 1) q = 0;
    fclose(f);
  }
  f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r");
  if (f) {
    if (fscanf(f, "%ld", &per) != 1) per = 0;
    fclose(f);
  }
  return (q > 0 && per > 0) ? (double)q / (double)per : 0.0;
}

int vp8g_rank_threads(int device) {
  long n = sysconf(_SC_NPROCESSORS_ONLN);
  const int pinned = vp8g_device_ncpu(device);
  if (pinned > 0 && pinned < n) n = pinned;
  const double quota = cgroup_quota();
  if (quota > 0) {
    const char* lw = getenv("LOCAL_WORLD_SIZE");
    const int ranks = (lw && atoi(lw) > 0) ? atoi(lw) : 1;
    long q = (long)(quota / ranks + 0.5);
    if (q < 1) q = 1;
    if (q < n) n = q;
  }
  return n < 1 ? 1 : (int)n;
}

/* One persistent pool of host threads per process (a rank is one process
 * per GPU, so per rank): budget - 1 threads pinned like vp8g_thread_create
 * for the first device that submits work, fed from a queue of jobs. A job
 * is n independent items (one frame each); any idle pool thread takes items
 * of the oldest job that still has some, up to the job's width at once, and
 * the submitting thread takes items too when it joins. The pool is
 * work-conserving (one engine alone gets every thread, several share them)
 * and never holds more threads than the budget, however many engines -- or
 * devices: a process that drives several GPUs shares the one pool between
 * them instead of starting a full-budget pool per device, which would
 * oversubscribe the quota by the device count. */
typedef struct {
  pthread_mutex_t lock;
  pthread_cond_t work, done;
  vp8g_job* head;
  int started, nthreads, busy;
} DevPool;

static DevPool g_pool;
static pthread_mutex_t g_pools_lock = PTHREAD_MUTEX_INITIALIZER;

static int pool_size(int device) {
  const char* e = getenv("WEBP_AMD_THREADS");   /* explicit override of the budget */
  if (e && atoi(e) > 0) return atoi(e);
  return vp8g_rank_threads(device);
}

static void* pool_thread(void* arg) {
  DevPool* P = (DevPool*)arg;
  pthread_mutex_lock(&P->lock);
  for (;;) {
    vp8g_job* j = P->head;
    while (j && (atomic_load(&j->next) >= j->n || j->active >= j->width)) j = j->link;
    if (!j) {
      pthread_cond_wait(&P->work, &P->lock);
      continue;
    }
    ++j->active;
    ++P->busy;
    pthread_mutex_unlock(&P->lock);
    for (;;) {
      const int i = atomic_fetch_add(&j->next, 1);
      if (i >= j->n) break;
      j->fn(j->ctx, i);
      atomic_fetch_add(&j->done, 1);
    }
    pthread_mutex_lock(&P->lock);
    --P->busy;
    if (--j->active == 0) pthread_cond_broadcast(&P->done);
  }
  return NULL;
}

static DevPool* pool_get(int device) {
  if (device < 0 || device >= MAX_DEV) device = 0;
  DevPool* P = &g_pool;
  pthread_mutex_lock(&g_pools_lock);
  if (!P->started) {
    pthread_mutex_init(&P->lock, NULL);
    pthread_cond_init(&P->work, NULL);
    pthread_cond_init(&P->done, NULL);
    P->head = NULL;
    P->started = 1;
    const int want = pool_size(device) - 1;
    for (int k = 0; k < want; ++k) {
      pthread_t th;
      if (vp8g_thread_create(&th, pool_thread, P, device) != 0) break;
      pthread_detach(th);
      ++P->nthreads;
    }
  }
  pthread_mutex_unlock(&g_pools_lock);
  return P;
}

void vp8g_job_submit(int device, vp8g_job* j, void (*fn)(void*, int), void* ctx, int n, int width) {
  j->fn = fn;
  j->ctx = ctx;
  j->n = n > 0 ? n : 0;
  j->width = width;
  atomic_init(&j->next, 0);
  atomic_init(&j->done, 0);
  j->active = 0;
  j->link = NULL;
  j->pool = NULL;
  if (j->n <= 1 || width <= 0) return;   /* the caller does it alone in vp8g_job_join */
  DevPool* P = pool_get(device);
  if (P->nthreads == 0) return;
  j->pool = P;
  pthread_mutex_lock(&P->lock);
  vp8g_job** q = &P->head;
  while (*q) q = &(*q)->link;
  *q = j;
  pthread_cond_broadcast(&P->work);
  pthread_mutex_unlock(&P->lock);
}

void vp8g_job_join(vp8g_job* j) {
  for (;;) {   /* the caller takes items too */
    const int i = atomic_fetch_add(&j->next, 1);
    if (i >= j->n) break;
    j->fn(j->ctx, i);
    atomic_fetch_add(&j->done, 1);
  }
  DevPool* P = (DevPool*)j->pool;
  if (!P) return;
  pthread_mutex_lock(&P->lock);
  vp8g_job** q = &P->head;   /* off the queue: no thread starts on it any more */
  while (*q && *q != j) q = &(*q)->link;
  if (*q) *q = j->link;
  while (j->active > 0 || atomic_load(&j->done) < j->n) pthread_cond_wait(&P->done, &P->lock);
  pthread_mutex_unlock(&P->lock);
  j->pool = NULL;
}

int WebPGpuHostThreadBudget(int device, int* busy) {
  const int n = pool_size(device);
  if (busy) {
    *busy = 0;
    if (g_pool.started) {
      pthread_mutex_lock(&g_pool.lock);
      *busy = g_pool.busy;
      pthread_mutex_unlock(&g_pool.lock);
    }
  }
  return n;
}
