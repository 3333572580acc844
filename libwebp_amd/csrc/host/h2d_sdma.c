/* Host <-> device copies of pinned buffers on a copy (SDMA) engine.
 *
 * With hipMemcpyAsync the host-input bench line sat ≈ 32 ms per 256 × 1080p
 * batch below the HBM-resident one -- about the upload's PCIe time
 * (2.1 GB at 57 GB/s), i.e. the upload did not overlap the other encoder
 * instances' kernels, as a copy kernel would not: while another instance's
 * K3 holds every CU (its VGPRs fill the register file) a blit kernel waits
 * for it and then holds CU slots for the whole transfer.
 * hsa_amd_memory_async_copy puts the transfer on an SDMA engine, which needs
 * no CU. The batch's big downloads (the packed .webp partitions, the MB
 * info) go the same way: as blit kernels they waited behind the other
 * instances' K3 (up to 100 ms in kernel_stats_r4z.csv). The calling engine thread waits for the copy's signal
 * (its own stream is idle at that point: every batch call drains it before
 * returning). */
#include "h2d_sdma.h"

#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define MAX_DEV 64

typedef struct {
  int ok;              /* 1 usable, -1 unusable, 0 not looked up yet */
  hsa_agent_t gpu, cpu;
  pthread_mutex_t up;  /* one upload at a time per device (see below) */
  pthread_mutex_t down;
} dev_agents;

static dev_agents g_dev[MAX_DEV];
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_hsa = 0;   /* 1 initialised, -1 failed */

typedef struct {
  uint32_t bdfid, domain;
  int found_gpu, found_cpu;
  hsa_agent_t gpu, cpu;
} find_ctx;

static hsa_status_t find_agent(hsa_agent_t a, void* data) {
  find_ctx* c = (find_ctx*)data;
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !c->found_cpu) {
    c->cpu = a;
    c->found_cpu = 1;
  } else if (t == HSA_DEVICE_TYPE_GPU && !c->found_gpu) {
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
        bdf == c->bdfid && dom == c->domain) {
      c->gpu = a;
      c->found_gpu = 1;
    }
  }
  return HSA_STATUS_SUCCESS;
}

static int lookup(int device) {
  if (device < 0 || device >= MAX_DEV) return 0;
  pthread_mutex_lock(&g_mu);
  if (!g_hsa) g_hsa = hsa_init() == HSA_STATUS_SUCCESS ? 1 : -1;   /* refcounted with HIP's */
  if (g_hsa > 0 && !g_dev[device].ok) {
    int bus = 0, dev = 0, dom = 0;
    find_ctx c = {0, 0, 0, 0, {0}, {0}};
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) == hipSuccess &&
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) == hipSuccess &&
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) == hipSuccess) {
      c.bdfid = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
      c.domain = (uint32_t)dom;
      hsa_iterate_agents(find_agent, &c);
    }
    g_dev[device].ok = (c.found_gpu && c.found_cpu) ? 1 : -1;
    pthread_mutex_init(&g_dev[device].up, NULL);
    pthread_mutex_init(&g_dev[device].down, NULL);
    g_dev[device].gpu = c.gpu;
    g_dev[device].cpu = c.cpu;
  }
  const int ok = g_hsa > 0 && g_dev[device].ok > 0;
  pthread_mutex_unlock(&g_mu);
  return ok;
}

static int sdma_mode(void) {   /* LIBWEBP_AMD_H2D=hip keeps the runtime's copies (A/B) */
  static int mode = -1;
  if (mode < 0) {
    const char* v = getenv("LIBWEBP_AMD_H2D");
    mode = (v && v[0] == 'h') ? 0 : 1;
  }
  return mode;
}

static int sdma_copy(pthread_mutex_t* mu, void* dst, hsa_agent_t dst_agent, const void* src,
                     hsa_agent_t src_agent, size_t bytes) {
  pthread_mutex_lock(mu);
  hsa_signal_t sig;
  if (hsa_signal_create(1, 0, NULL, &sig) != HSA_STATUS_SUCCESS) {
    pthread_mutex_unlock(mu);
    return 0;
  }
  const hsa_status_t st = hsa_amd_memory_async_copy(dst, dst_agent, src, src_agent, bytes, 0, NULL, sig);
  int ok = 0;
  if (st == HSA_STATUS_SUCCESS) {
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                     HSA_WAIT_STATE_BLOCKED) >= 1) {
    }
    ok = 1;
  }
  hsa_signal_destroy(sig);
  pthread_mutex_unlock(mu);
  return ok;
}

int h2d_sdma_upload(int device, void* dst, const void* src, size_t bytes) {
  if (!sdma_mode() || !lookup(device)) return 0;
  /* Uploads to one device go one after another: they share the PCIe link
     anyway, and in turn the first engine's frames are on the device after one
     transfer time instead of all engines' after three (its kernels start
     while the next engine uploads). */
  dev_agents* d = &g_dev[device];
  return sdma_copy(&d->up, dst, d->gpu, src, d->cpu, bytes);
}

int h2d_sdma_upload_start(int device, void* dst, const void* src, size_t bytes, uint64_t* handle) {
  if (!sdma_mode() || !lookup(device)) return 0;
  /* no per-device lock: it runs while this engine's batch encodes, beside
     the other engines' (blocking) uploads, which share the link with it */
  dev_agents* d = &g_dev[device];
  hsa_signal_t sig;
  if (hsa_signal_create(1, 0, NULL, &sig) != HSA_STATUS_SUCCESS) return 0;
  if (hsa_amd_memory_async_copy(dst, d->gpu, src, d->cpu, bytes, 0, NULL, sig) != HSA_STATUS_SUCCESS) {
    hsa_signal_destroy(sig);
    return 0;
  }
  *handle = sig.handle;
  return 1;
}

void h2d_sdma_finish(uint64_t handle) {
  hsa_signal_t sig;
  sig.handle = handle;
  while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                   HSA_WAIT_STATE_BLOCKED) >= 1) {
  }
  hsa_signal_destroy(sig);
}

int d2h_sdma_download(int device, void* dst, const void* src, size_t bytes) {
  if (!bytes) return 1;
  if (!sdma_mode() || !lookup(device)) return 0;
  dev_agents* d = &g_dev[device];
  return sdma_copy(&d->down, dst, d->cpu, src, d->gpu, bytes);
}

/* GPU memory-fault report (diagnostics, WEBP_AMD_FAULT_REPORT=1): the
 * runtime's memory-fault event carries the faulting virtual address and the
 * reason; HIP itself only returns "an illegal memory access". Printed to
 * stderr next to the engines' buffer ranges (gpu_batch.c), it names the
 * buffer (or none) an access went out of. */
static hsa_status_t fault_event(const hsa_amd_event_t* ev, void* data) {
  (void)data;
  if (ev->event_type == HSA_AMD_GPU_MEMORY_FAULT_EVENT)
    fprintf(stderr, "WEBP_AMD_FAULT address 0x%llx reason 0x%x\n",
            (unsigned long long)ev->memory_fault.virtual_address,
            (unsigned)ev->memory_fault.fault_reason_mask);
  return HSA_STATUS_SUCCESS;
}
static pthread_once_t g_fault_once = PTHREAD_ONCE_INIT;
static void fault_init(void) {
  if (hsa_amd_register_system_event_handler(fault_event, NULL) != HSA_STATUS_SUCCESS)
    fprintf(stderr, "WEBP_AMD_FAULT report: handler not registered\n");
}
void vp8g_fault_report_init(void) { pthread_once(&g_fault_once, fault_init); }
