/* Batched GPU engine: device buffers, the K1 -> K2 -> host setup -> K3
 * pipeline, and the host thread pool that runs the boolean-coder tail.
 * Host C over the HIP runtime C API; kernels live in hip/vp8_kernels.hip. */
#include "h2d_sdma.h"
#include <math.h>
#include <stdio.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "gpu_engine.h"
#include "vp8_host.h"
#include "webp/encode_gpu.h"

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

/* gamma tables for the RGB->YUV import (picture_csp_enc.c:103-117) */
static uint16_t g_g2l[256];
static int32_t g_l2g[33];
static pthread_once_t g_gamma_once = PTHREAD_ONCE_INIT;
static void gamma_init(void) {
  const double scale = (double)(1 << 7) / 4095;
  const double norm = 1. / 255.;
  for (int v = 0; v < 256; ++v) g_g2l[v] = (uint16_t)(pow(norm * v, 0.80) * 4095 + .5);
  for (int v = 0; v <= 32; ++v) g_l2g[v] = (int)(255. * pow(scale * v, 1. / 0.80) + .5);
}

int WebPGpuSynthRGBA(void* rgba, size_t fstride, int w, int h, int first, int n, int seed,
                     void* stream) {
  if (!rgba || w <= 0 || h <= 0 || n <= 0 || fstride < (size_t)w * h * 4) return 0;
  if (!vp8g_launch_synth((uint8_t*)rgba, fstride, w, h, first, n, seed, stream)) return 0;
  return hipStreamSynchronize((hipStream_t)stream) == hipSuccess;
}

int WebPGpuDeviceCount(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

/* host threads of an engine: WEBP_AMD_THREADS, else at most 16 and no more
 * than the rank's host-thread budget (cgroup quota over the node's ranks, the
 * rank's share of its GPU's NUMA node; host_cpus.c). The helpers of each
 * host phase are drawn from the process-wide pool of that budget, so several
 * engines per rank do not multiply it. */
/* WEBP_AMD_WATCH=1 (diagnostics): frame 0's progress word is polled during
 * every K3 launch of the batch API too, and each change is printed with the
 * time since the launch -- how far a stalled launch got, without touching
 * the kernel's code */
static double watch_t0;
static int watch_rows(void* ctx, int rows, int total) {
  (void)ctx;
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  const double t = ts.tv_sec + 1e-9 * ts.tv_nsec;
  if (rows <= 0) watch_t0 = t;
  fprintf(stderr, "[watch] frame 0: %d / %d rows folded at %.3f s\n", rows, total, t - watch_t0);
  return 1;
}

static int default_threads(int device) {
  const char* e = getenv("WEBP_AMD_THREADS");
  if (e && atoi(e) > 0) return atoi(e);
  const int n = vp8g_rank_threads(device);
  return n > 16 ? 16 : n;
}

static __thread char g_last_error[256];

void vp8g_set_error(const char* where, const char* what) {
  snprintf(g_last_error, sizeof(g_last_error), "%s: %s", where, what);
}

const char* WebPGpuLastError(void) { return g_last_error; }

#define CHK(x)                                                         \
  do {                                                                 \
    const hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) {                                            \
      char loc_[64];                                                   \
      snprintf(loc_, sizeof(loc_), "gpu_batch.c:%d", __LINE__);        \
      vp8g_set_error(loc_, hipGetErrorString(e_));                     \
      goto fail;                                                       \
    }                                                                  \
  } while (0)

WebPGpuBatch* WebPGpuBatchNew(int device, int width, int height, int max_frames,
                              const WebPConfig* config, int host_threads) {
  if (!config || width <= 0 || height <= 0 || width > WEBP_MAX_DIMENSION ||
      height > WEBP_MAX_DIMENSION || max_frames <= 0)
    return NULL;
  if (!WebPValidateConfig(config)) return NULL;
  WebPGpuBatch* b = (WebPGpuBatch*)calloc(1, sizeof(*b));
  if (!b) return NULL;
  if (config->lossless) {   /* VP8L engine (host/vp8l_batch.c) */
    b->device = device;
    b->w = width; b->h = height;
    b->max_frames = max_frames;
    b->cfg = *config;
    b->threads = host_threads > 0 ? host_threads : default_threads(device);
    CHK(hipSetDevice(device));
    CHK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
    for (int i = 0; i < 6; ++i) CHK(hipEventCreate(&b->ev[i]));
    b->l = vp8l_engine_new(width, height, max_frames, config->method, 0);
    if (!b->l) goto fail;
    vp8l_engine_set_near_lossless(b->l, config->near_lossless);
    vp8l_engine_set_exact(b->l, config->exact);
    return b;
  }
  vp8h_frame probe;
  if (!vp8h_frame_init(&probe, config, width, height)) { free(b); return NULL; }
  pthread_once(&g_gamma_once, gamma_init);
  b->device = device;
  b->w = width; b->h = height;
  b->max_frames = max_frames;
  b->cfg = *config;
  b->mbw = (width + 15) >> 4; b->mbh = (height + 15) >> 4;
  b->nmb = b->mbw * b->mbh;
  b->uvw = (width + 1) >> 1; b->uvh = (height + 1) >> 1;
  b->yfb = (size_t)width * height + 2 * (size_t)b->uvw * b->uvh;
  b->yfb = (b->yfb + 255) & ~(size_t)255;
  b->tok_cap = 0;   /* d_tokens: sized per run (tokens_for_run) */
  b->sharp = vp8h_use_sharp(config, width, height);
  b->dither = b->sharp ? 0.f : vp8h_import_dithering(config);
  b->threads = host_threads > 0 ? host_threads : default_threads(device);
  b->host_emit = 0;
  {   /* where partition 0 is coded: WEBP_AMD_P0=host / gpu, else by the rank's
         host-thread budget (use_gpu_p0) */
    const char* e = getenv("WEBP_AMD_P0");
    b->gpu_p0 = e && !strcmp(e, "gpu") ? 1 : e && !strcmp(e, "host") ? 0 : -1;
  }
  {   /* test knob: start with token rows of 64 tokens, so the first call
         re-runs K3 with wider rows (k3_settle's regrow) */
    const char* tt = getenv("WEBP_AMD_TEST_TINY_TOKENS");
    b->tiny_tokens = tt && tt[0] == '1';
  }
#ifdef WEBP_AMD_DIAG
  {   /* diagnostic build only: WEBP_AMD_HOST_EMIT=1 boolean-codes partition 1
         on the host threads (A/B of K4; libwebp_amd_diag.so) */
    const char* he = getenv("WEBP_AMD_HOST_EMIT");
    b->host_emit = he && he[0] == '1';
  }
#endif

  const size_t N = (size_t)max_frames, nmb = (size_t)b->nmb;
  CHK(hipSetDevice(device));
  CHK(hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking));
  for (int i = 0; i < 6; ++i) CHK(hipEventCreate(&b->ev[i]));
  CHK(hipMalloc((void**)&b->d_g2l, 256 * sizeof(uint16_t) + 33 * sizeof(int32_t)));
  b->d_l2g = (int32_t*)(b->d_g2l + 256);
  CHK(hipMemcpy(b->d_g2l, g_g2l, 256 * sizeof(uint16_t), hipMemcpyHostToDevice));
  CHK(hipMemcpy(b->d_l2g, g_l2g, 33 * sizeof(int32_t), hipMemcpyHostToDevice));
  CHK(hipMalloc((void**)&b->d_yuv, N * b->yfb));
  CHK(hipMalloc((void**)&b->d_aflags, N * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&b->d_aplane, N * (size_t)width * height));
  CHK(hipMalloc((void**)&b->d_alpha, N * nmb));
  CHK(hipMalloc((void**)&b->d_uva, N * nmb * sizeof(uint16_t)));
  CHK(hipMalloc((void**)&b->d_amode, N * nmb));
  CHK(hipMalloc((void**)&b->d_segmap, N * nmb));
  CHK(hipMalloc((void**)&b->d_params, N * sizeof(vp8g_frame_params)));
  CHK(hipMalloc((void**)&b->d_mbinfo, N * nmb * VP8G_MBINFO_BYTES));
  CHK(hipMalloc((void**)&b->d_mboff, N * nmb * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&b->d_rerun, N * VP8G_RERUN_STATE_BYTES));
  if (N <= VP8G_XSPLIT_MAX_FRAMES)   /* few frames: K3 splits each over several CUs */
    CHK(hipMalloc((void**)&b->d_xsync, N * vp8g_xsync_bytes(width, height)));
  CHK(hipMalloc((void**)&b->d_wsnap, N * vp8g_wsnap_bytes(width, height)));
  CHK(hipMalloc((void**)&b->d_results, N * sizeof(vp8g_frame_result)));
  /* K4 streams: one per token partition; the WebPEncode pool changes the
   * config of an engine between calls, so room for the most partitions */
  const size_t NS = N * (VP8G_MAX_PARTS + 1);   /* + partition 0 (gpu_p0) */
  CHK(hipMalloc((void**)&b->d_psize, NS * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&b->d_emeta, NS * sizeof(vp8g_emit_meta)));
  CHK(hipMalloc((void**)&b->d_pinfo, N * 16 * sizeof(uint32_t)));
  CHK(hipHostMalloc((void**)&b->h_pinfo, N * 16 * sizeof(uint32_t), 0));
  CHK(hipHostMalloc((void**)&b->h_aflags, N * sizeof(uint32_t), 0));
  CHK(hipHostMalloc((void**)&b->h_alpha, N * nmb, 0));
  CHK(hipHostMalloc((void**)&b->h_uva, N * nmb * sizeof(uint16_t), 0));
  CHK(hipHostMalloc((void**)&b->h_segmap, N * nmb, 0));
  CHK(hipHostMalloc((void**)&b->h_params, N * sizeof(vp8g_frame_params), 0));
  CHK(hipHostMalloc((void**)&b->h_mbinfo, N * nmb * VP8G_MBINFO_BYTES, 0));
  CHK(hipHostMalloc((void**)&b->h_results, N * sizeof(vp8g_frame_result), 0));
  CHK(hipHostMalloc((void**)&b->h_psize, NS * sizeof(uint32_t), 0));
  CHK(hipHostMalloc((void**)&b->h_poff, (NS + 1) * sizeof(uint64_t), 0));
  CHK(hipMalloc((void**)&b->d_poff, (NS + 1) * sizeof(uint64_t)));
  CHK(hipHostMalloc((void**)&b->h_emeta, NS * sizeof(vp8g_emit_meta), 0));
  b->frames = (vp8h_frame*)calloc(N, sizeof(vp8h_frame));
  b->tok_off = (size_t*)calloc(N + 1, sizeof(size_t));
  b->p0 = (vp8h_bw*)calloc(N, sizeof(vp8h_bw));
  b->out = (uint8_t**)calloc(N, sizeof(uint8_t*));
  b->out_cap = (size_t*)calloc(N, sizeof(size_t));
  b->out_size = (size_t*)calloc(N, sizeof(size_t));
  b->err = (int*)calloc(N, sizeof(int));
  b->hdr = (int*)calloc(2 * N, sizeof(int));
  b->araw = (uint8_t**)calloc(N, sizeof(uint8_t*));
  b->fin_cost = (int*)calloc(N, sizeof(int));
  b->pass_act = (uint8_t*)calloc(N, 1);
  b->asse = (uint64_t*)calloc(N, sizeof(uint64_t));
  if (!b->frames || !b->tok_off || !b->p0 || !b->out || !b->out_cap || !b->out_size || !b->err || !b->hdr ||
      !b->araw || !b->fin_cost || !b->pass_act || !b->asse)
    goto fail;
  if (getenv("WEBP_AMD_WATCH")) b->progress = watch_rows;
  return b;
fail:
  WebPGpuBatchDelete(b);
  return NULL;
}

void WebPGpuBatchDelete(WebPGpuBatch* b) {
  if (!b) return;
  hipSetDevice(b->device);
  if (b->stream) hipStreamSynchronize(b->stream);
  if (b->pf_busy) h2d_sdma_finish(b->pf_sig);
  hipFree(b->d_rgba2);
  hipFree(b->d_g2l); hipFree(b->d_rgba); hipFree(b->d_yuv); hipFree(b->d_aflags); hipFree(b->d_alpha);
  hipFree(b->d_uva); hipFree(b->d_amode); hipFree(b->d_segmap); hipFree(b->d_params); hipFree(b->d_tokens);
  hipFree(b->d_rowtok); hipHostFree(b->h_rowtok); hipFree(b->d_rerun_snap); hipFree(b->d_edesc);
  hipFree(b->d_mbinfo); hipFree(b->d_mboff); hipFree(b->d_rerun); hipFree(b->d_xsync); hipFree(b->d_wsnap); hipFree(b->d_results); hipFree(b->d_psize); hipFree(b->d_emeta);
  hipFree(b->d_poff); hipFree(b->d_part); hipFree(b->d_pinfo);
  hipFree(b->d_emap); hipFree(b->d_eshift); hipFree(b->d_esegs); hipFree(b->d_nbuf);
  hipFree(b->d_eimg);
  hipFree(b->d_stabs); hipFree(b->d_sharp); hipFree(b->d_sstate);
  hipFree(b->d_rnd_y); hipFree(b->d_rnd_uv);
  hipFree(b->d_active); hipFree(b->d_tbits);
  hipFree(b->d_ahist); hipFree(b->d_amaps); hipHostFree(b->h_ahist); hipHostFree(b->h_amaps);
  hipFree(b->d_lmstats); hipFree(b->d_lmi); hipHostFree(b->h_lmstats); hipHostFree(b->h_lmi);
  free(b->asse);
  hipFree(b->d_recon); hipFree(b->d_mbval); hipFree(b->d_afp); hipFree(b->d_aflevel);
  hipHostFree(b->h_afp); hipHostFree(b->h_aflevel);
  hipHostFree(b->h_state); hipHostFree(b->h_active); hipHostFree(b->h_tbits);
  hipHostFree(b->h_prog);
  hipHostFree(b->h_aflags); hipHostFree(b->h_alpha); hipHostFree(b->h_uva);
  hipHostFree(b->h_segmap); hipHostFree(b->h_params); hipHostFree(b->h_mbinfo);
  hipHostFree(b->h_results); hipHostFree(b->h_tokens); hipHostFree(b->h_psize);
  hipHostFree(b->h_part); hipHostFree(b->h_emeta); hipHostFree(b->h_poff); hipHostFree(b->h_pinfo);
  hipHostFree(b->h_p0hdr); hipHostFree(b->h_p0par); hipFree(b->d_p0hdr); hipFree(b->d_p0par);
  vp8l_engine_free(b->l);
  vp8l_engine_free(b->la);
  hipFree(b->d_aplane);
  if (b->araw)
    for (int i = 0; i < b->max_frames; ++i) free(b->araw[i]);
  free(b->araw);
  free(b->fin_cost); free(b->pass_act);
  for (int i = 0; i < 6; ++i)
    if (b->ev[i]) hipEventDestroy(b->ev[i]);
  if (b->stream) hipStreamDestroy(b->stream);
  if (b->out)
    for (int i = 0; i < b->max_frames; ++i) free(b->out[i]);
  free(b->out); free(b->out_cap); free(b->out_size); free(b->err); free(b->hdr);
  if (b->p0)
    for (int i = 0; i < b->max_frames; ++i) vp8h_bw_free(&b->p0[i]);
  free(b->frames); free(b->tok_off); free(b->p0);
  free(b);
}

/* ---- the per-frame host phases, on the rank's thread pool (host_cpus.c) ---- */

typedef struct {
  WebPGpuBatch* b;
  int phase;   /* 0: partition 0; 1: partition 1 + RIFF write; 2: frame setup;
                  3: partition 0's header tokens (gpu_p0) */
  vp8g_job job;
} TailJob;

/* Partition 0 of frame f: needs only K3's results and modes. */
static void frame_head(WebPGpuBatch* b, int f) {
  vp8h_frame* fr = &b->frames[f];
  const vp8g_frame_result* res = &b->h_results[f];
  b->out_size[f] = 0;   /* b->out[f] (capacity b->out_cap[f]) is reused */
  vp8h_bw_free(&b->p0[f]);
  if (b->err[f] != VP8_ENC_OK) return;
  if (res->error) {
    if (getenv("WEBP_AMD_SYNC_K3"))   /* fault localisation: K3's raw error (wait site << 4) */
      fprintf(stderr, "frame %d: K3 error 0x%x\n", f, (unsigned)res->error);
    /* wait site 6: the progress hook asked to stop (WebPEncode) */
    b->err[f] = (res->error >> 4) == 6 ? VP8_ENC_ERROR_USER_ABORT : VP8_ENC_ERROR_OUT_OF_MEMORY;
    return;
  }
  b->err[f] = vp8h_build_p0(fr, res, b->h_mbinfo + (size_t)f * b->nmb * VP8G_MBINFO_BYTES,
                            &b->p0[f], b->hdr + 2 * f);
}

/* Partition 0 on the device (gpu_p0): the frame header as tokens for
 * k_p0_modes, which appends the MB modes; K4 codes the stream. */
static void frame_head_dev(WebPGpuBatch* b, int f) {
  vp8h_frame* fr = &b->frames[f];
  const vp8g_frame_result* res = &b->h_results[f];
  b->out_size[f] = 0;
  vp8h_bw_free(&b->p0[f]);
  int nh = -1;
  if (b->err[f] == VP8_ENC_OK && res->error)
    b->err[f] = (res->error >> 4) == 6 ? VP8_ENC_ERROR_USER_ABORT : VP8_ENC_ERROR_OUT_OF_MEMORY;
  if (b->err[f] == VP8_ENC_OK) {
    nh = vp8h_p0_header(fr, res, b->h_p0hdr + (size_t)f * VP8G_P0_HDR_CAP, VP8G_P0_HDR_CAP,
                        b->hdr + 2 * f);
    if (nh < 0) b->err[f] = VP8_ENC_ERROR_OUT_OF_MEMORY;
  }
  vp8h_p0_par(fr, res, nh, &b->h_p0par[f]);
}

/* Join partition 0 with partition 1 (K4's bytes, or coded here under
 * WEBP_AMD_HOST_EMIT=1) into the RIFF/WEBP file. */
static void frame_finish(WebPGpuBatch* b, int f) {
  const vp8g_frame_result* res = &b->h_results[f];
  if (b->err[f] != VP8_ENC_OK) { vp8h_bw_free(&b->p0[f]); return; }
  vp8h_bw part1[VP8G_MAX_PARTS];
  const int np = b->nparts;
  if (b->host_emit) {   /* boolean-code the tokens here (token_enc.c:200-223) */
    vp8h_bw_init(&part1[0], (size_t)res->ntokens / 8 + 4096);
    vp8h_emit_tokens(&part1[0], b->h_tokens + b->tok_off[f], res->ntokens, res->probas);
    vp8h_bw_finish(&part1[0]);
  } else {              /* the token partitions, already coded by K4 */
    for (int p = 0; p < np; ++p) {
      const size_t s = (size_t)f * np + p;
      memset(&part1[p], 0, sizeof(part1[p]));
      part1[p].buf = b->h_part + b->h_poff[s];
      part1[p].pos = b->h_psize[s];
    }
  }
  if (b->p0_dev) {   /* partition 0 coded by K4: borrowed from the packed bytes */
    const size_t s = (size_t)b->last_ns + f;
    memset(&b->p0[f], 0, sizeof(b->p0[f]));
    b->p0[f].buf = b->h_part + b->h_poff[s];
    b->p0[f].pos = b->h_psize[s];
    b->hdr[2 * f + 1] = (int)b->h_psize[s] - b->hdr[2 * f];
    if (b->h_psize[s] >= (1u << 19)) {   /* syntax_enc.c / vp8h_build_p0's check */
      b->err[f] = VP8_ENC_ERROR_PARTITION0_OVERFLOW;
      memset(&b->p0[f], 0, sizeof(b->p0[f]));
      return;
    }
  }
  int err = VP8_ENC_OK;
  vp8h_alpha alpha, *ap = NULL;
  if (b->h_aflags[f]) {   /* ALPH chunk (alpha_enc.c:110-182) */
    if (b->araw[f]) {
      alpha.header = 0;   /* ALPHA_NO_COMPRESSION */
      alpha.data = b->araw[f];
      alpha.size = (size_t)b->w * b->h;
    } else {
      alpha.header = 1;   /* ALPHA_LOSSLESS_COMPRESSION, no filter */
      alpha.data = vp8l_engine_output(b->la, f);
      alpha.size = vp8l_engine_out_size(b->la, f);
    }
    if (b->cfg.alpha_quality < 100) alpha.header |= 1 << 4;   /* ALPHA_PREPROCESSED_LEVELS */
    ap = &alpha;
  }
  b->out_size[f] = vp8h_write_riff(&b->frames[f], &b->p0[f], part1, b->host_emit ? 1 : np, ap,
                                   &b->out[f], &b->out_cap[f], &err);
  b->err[f] = err;
  if (b->host_emit) vp8h_bw_free(&part1[0]);
}

/* Frame header state and the segment map from K2's per-MB alphas
 * (vp8h_analyze_segments: analysis_enc.c's k-means). */
static void frame_setup(WebPGpuBatch* b, int f) {
  if (b->err[f] != VP8_ENC_OK) return;
  const size_t nmb = (size_t)b->nmb;
  vp8h_frame_init(&b->frames[f], &b->cfg, b->w, b->h);
  vp8h_analyze_segments(&b->frames[f], b->h_alpha + f * nmb, b->h_uva + f * nmb,
                        b->h_segmap + f * nmb);
}

static void tail_item(void* arg, int f) {
  TailJob* j = (TailJob*)arg;
  if (j->phase == 0) frame_head(j->b, f);
  else if (j->phase == 1) frame_finish(j->b, f);
  else if (j->phase == 3) frame_head_dev(j->b, f);
  else frame_setup(j->b, f);
}

/* queue the phase's frames on the pool (at most b->threads - 1 pool threads
 * on it at once); the caller joins in later */
static void tail_spawn(TailJob* j, WebPGpuBatch* b, int n, int phase, int extra) {
  j->b = b;
  j->phase = phase;
  vp8g_job_submit(b->device, &j->job, tail_item, j, n, extra);
}

static void tail_join(TailJob* j) { vp8g_job_join(&j->job); }

static void run_tails(WebPGpuBatch* b, int n, int phase) {
  TailJob job;
  tail_spawn(&job, b, n, phase, b->threads - 1);
  tail_join(&job);
}

/* ---- pipeline ---- */

/* frame 0's progress words into the parameters of the next K3 launch
 * (WebPEncode with a progress hook), every other frame none */
static int stamp_progress(WebPGpuBatch* b, int n) {
  if (b->progress && !b->h_prog) {
    void* dp = NULL;
    if (hipHostMalloc((void**)&b->h_prog, 2 * sizeof(uint32_t), hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer(&dp, b->h_prog, 0) != hipSuccess) {
      vp8g_set_error("stamp_progress", "host-mapped progress words");
      return 0;
    }
    b->d_prog = (uint64_t)(uintptr_t)dp;
  }
  if (b->progress) {
    __atomic_store_n(&b->h_prog[0], 0u, __ATOMIC_RELAXED);
    __atomic_store_n(&b->h_prog[1], 0u, __ATOMIC_RELAXED);
  }
  for (int f = 0; f < n; ++f) b->h_params[f].progress_addr = (f == 0 && b->progress) ? b->d_prog : 0;
  return 1;
}

/* wait for the stream; with a progress hook, poll the rows K3 has folded
 * and pass them on (WebPReportProgress per MB row, iterator_enc.c:89-99); a
 * hook returning 0 raises the abort word K3 checks after each row it folds,
 * and the hook is not called again */
static hipError_t engine_wait(WebPGpuBatch* b, hipStream_t st) {
  if (!b->progress || !b->h_prog) return hipStreamSynchronize(st);
  int last = -1;
  for (;;) {
    const hipError_t e = hipStreamQuery(st);
    if (e != hipErrorNotReady) {
      if (b->progress == watch_rows) fprintf(stderr, "[watch] K3 launch done (status %d)\n", (int)e);
      return e;
    }
    const int rows = (int)__atomic_load_n(&b->h_prog[0], __ATOMIC_RELAXED);
    if (rows != last && !__atomic_load_n(&b->h_prog[1], __ATOMIC_RELAXED)) {
      last = rows;
      if (!b->progress(b->progress_ctx, rows, b->mbh))
        __atomic_store_n(&b->h_prog[1], 1u, __ATOMIC_RELAXED);
    }
    usleep(200);
  }
}

/* ALPH chunks of the frames with alpha (h_aflags): the alpha planes in
 * d_aplane through the VP8L engine in ALPH mode (alpha_enc.c:50-98), or raw
 * (alpha_compression 0, or when the stream would not be smaller). */
static int encode_alpha(WebPGpuBatch* b, int n) {
  int any = 0;
  for (int f = 0; f < n; ++f) {
    free(b->araw[f]);
    b->araw[f] = NULL;
    any |= b->h_aflags[f] != 0;
  }
  if (!any) return 1;
  const size_t plane = (size_t)b->w * b->h;
  double t[10] = {0};
  const int reduce_levels = b->cfg.alpha_quality < 100;
  if (reduce_levels) {   /* QuantizeLevels on the device planes (alpha_enc.c:342-349) */
    if (!b->d_ahist) {
      const size_t N = (size_t)b->max_frames;
      CHK(hipMalloc((void**)&b->d_ahist, N * 256 * sizeof(uint32_t)));
      CHK(hipMalloc((void**)&b->d_amaps, N * 256));
      CHK(hipHostMalloc((void**)&b->h_ahist, N * 256 * sizeof(uint32_t), 0));
      CHK(hipHostMalloc((void**)&b->h_amaps, N * 256, 0));
    }
    if (!vp8g_launch_alpha_hist(b->d_aplane, plane, b->d_aflags, n, b->d_ahist, b->stream))
      return 0;
    CHK(hipMemcpyAsync(b->h_ahist, b->d_ahist, n * 256 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       b->stream));
    CHK(hipStreamSynchronize(b->stream));
    const int levels = vp8h_alpha_levels(b->cfg.alpha_quality);
    for (int f = 0; f < n; ++f)
      if (b->h_aflags[f])
        vp8h_quantize_levels_map(b->h_ahist + (size_t)f * 256, plane, levels,
                                 b->h_amaps + (size_t)f * 256, &b->asse[f]);
    CHK(hipMemcpyAsync(b->d_amaps, b->h_amaps, n * 256, hipMemcpyHostToDevice, b->stream));
    if (!vp8g_launch_alpha_remap(b->d_aplane, plane, b->d_aflags, n, b->d_amaps, b->stream))
      return 0;
    CHK(hipStreamSynchronize(b->stream));
  }
  if (b->cfg.alpha_compression) {
    /* the ALPH effort follows config->method on every call (alpha_enc.c:76,
     * 379); the WebPEncode pool hands an engine configs of other methods */
    if (b->la && b->la->method != b->cfg.method) {
      vp8l_engine_free(b->la);
      b->la = NULL;
    }
    if (!b->la) b->la = vp8l_engine_new(b->w, b->h, b->max_frames, b->cfg.method, 1);
    if (!b->la) return 0;
    if (!vp8l_engine_encode(b->la, b->stream, b->threads, b->d_aplane, plane, b->w, n, t))
      return 0;
  }
  for (int f = 0; f < n; ++f) {
    if (!b->h_aflags[f]) continue;
    if (b->cfg.alpha_compression && !vp8l_engine_error(b->la, f) &&
        vp8l_engine_out_size(b->la, f) <= plane)
      continue;
    b->araw[f] = (uint8_t*)malloc(plane);
    if (!b->araw[f] ||
        hipMemcpy(b->araw[f], b->d_aplane + (size_t)f * plane, plane, hipMemcpyDeviceToHost) !=
            hipSuccess)
      return 0;
  }
  b->timings[9] = t[0] + t[1] + t[2] + t[3] + t[4];
  return 1;
fail:
  return 0;
}

/* ---- token buffers ----------------------------------------------------
 * The token loop (methods 3-6 without low_memory) runs K3 with token rows:
 * every MB's tokens are written once, where K4 reads them -- frame f's MB
 * row y at d_tokens + f * tok_cap + y * rowcap, the MBs of the row one after
 * another in raster order (vp8g_rows) -- and a row that runs out of room
 * makes k3_settle widen the rows and run the launch again. The other paths
 * (methods 0-2, low_memory, VP8EncLoop's searches) keep per-MB slots of the
 * worst case VP8G_MAX_TOKENS_PER_MB and a compact stream per frame. Both
 * take d_tokens with a frame stride of tok_cap tokens; behind the frames'
 * slabs lies each frame's partition-0 stream (gpu_p0). */
static int rows_mode(const WebPGpuBatch* b) {
  return b->cfg.method >= 3 && !b->cfg.low_memory && !b->host_emit;
}

/* d_tokens with a frame stride of tok_cap tokens; the first keep frames'
 * token rows (rowcap apart, the old layout) move to the new layout */
static int alloc_tokens(WebPGpuBatch* b, size_t tok_cap, size_t rowcap, int keep) {
  uint16_t* old = b->d_tokens;
  const size_t old_rowcap = b->rowcap, old_cap = b->tok_cap;
  uint16_t* nt = NULL;
  const size_t p0cap = vp8g_p0_cap(b->nmb);
  CHK(hipMalloc((void**)&nt, (size_t)b->max_frames * (tok_cap + p0cap) * sizeof(uint16_t)));
  if (old && keep > 0 && old_rowcap) {   /* row y of frame f: f * cap + y * rowcap */
    for (int f = 0; f < keep; ++f)
      CHK(hipMemcpy2DAsync(nt + (size_t)f * tok_cap, rowcap * sizeof(uint16_t),
                           old + (size_t)f * old_cap, old_rowcap * sizeof(uint16_t),
                           old_rowcap * sizeof(uint16_t), (size_t)b->mbh, hipMemcpyDeviceToDevice,
                           b->stream));
    CHK(hipStreamSynchronize(b->stream));
  }
  hipFree(old);
  b->d_tokens = nt;
  b->tok_cap = tok_cap;
  b->p0_cap = p0cap;
  /* the rows: as asked, else the widest the stride holds (a slot-sized
     buffer); a multiple of 64 tokens, so every row and every K4 segment
     starts on a 128-byte line (K4 stages segments in 128-byte strips: a
     strip across two lines doubled k_emit_seg's reads, r6i) */
  b->rowcap = rowcap ? rowcap : (tok_cap / (size_t)b->mbh) & ~(size_t)63;
  return 1;
fail:
  hipFree(nt);
  return 0;
}

/* d_tokens with a stride of at least cap tokens per frame (grows only) */
static int ensure_tok_cap(WebPGpuBatch* b, size_t cap) {
  cap = (cap + 255) & ~(size_t)255;
  if (b->d_tokens && b->tok_cap >= cap) return 1;
  return alloc_tokens(b, cap, 0, 0);
}

/* token rows of at least rowcap tokens (grows only, at most the worst case
 * of a row); keep: frames whose rows must survive a regrow */
static int ensure_rows(WebPGpuBatch* b, size_t rowcap, int keep) {
  const size_t most = (size_t)VP8G_MAX_TOKENS_PER_MB * b->mbw;
  rowcap = (rowcap + 63) & ~(size_t)63;
  if (rowcap > most) rowcap = (most + 63) & ~(size_t)63;
  if (!b->d_rowtok) {
    CHK(hipMalloc((void**)&b->d_rowtok, (size_t)b->max_frames * b->mbh * sizeof(uint32_t)));
    CHK(hipHostMalloc((void**)&b->h_rowtok, (size_t)b->max_frames * b->mbh * sizeof(uint32_t), 0));
    CHK(hipMalloc((void**)&b->d_rerun_snap, (size_t)b->max_frames * VP8G_RERUN_STATE_BYTES));
  }
  if (b->d_tokens && b->rowcap >= rowcap) return 1;
  /* the K4 reads of a row's last 8-token piece stay inside the slab: + 8;
     frames 512-byte aligned */
  return alloc_tokens(b, ((size_t)b->mbh * rowcap + 8 + 255) & ~(size_t)255, rowcap, keep);
fail:
  return 0;
}

/* the token buffers of this run's path (before K3's first launch) */
static int tokens_for_run(WebPGpuBatch* b) {
  const size_t nmb = (size_t)b->nmb;
  if (!rows_mode(b)) return ensure_tok_cap(b, nmb * VP8G_MAX_TOKENS_PER_MB);
  if (b->tiny_tokens)   /* test knob: k3_settle's regrow runs on the first call */
    return ensure_rows(b, 64, 0);
  /* ~2.3x the tokens per MB of a -q 75 frame of natural content in a row
   * (batches); single pictures (K3X) start at 4096 per MB (a 4096-wide q90
   * m6 row holds ~2900 per MB) */
  return ensure_rows(b, (size_t)b->mbw * (b->max_frames <= VP8G_XSPLIT_MAX_FRAMES ? 4096 : 2048), 0);
}

/* K3 over the frames of h_params (already on the device). The caller copies
 * the results back and calls k3_settle. */
static int launch_k3(WebPGpuBatch* b, int n, uint8_t* recon) {
  hipStream_t st = b->stream;
  vp8g_rows R, *rp = NULL;
  if (rows_mode(b)) {
    int reread = 0;   /* a pass that starts from d_rerun: keep a copy for a re-run */
    for (int f = 0; f < n; ++f)
      reread |= b->h_params[f].pass_mode == 1 || b->h_params[f].pass_mode == 3;
    if (reread)
      CHK(hipMemcpyAsync(b->d_rerun_snap, b->d_rerun, (size_t)n * VP8G_RERUN_STATE_BYTES,
                         hipMemcpyDeviceToDevice, st));
    R.rowcap = (uint32_t)b->rowcap;
    R.rowtok = b->d_rowtok;
    rp = &R;
  }
  if (!vp8g_launch_encode(b->d_yuv, b->yfb, b->w, b->h, n, b->d_segmap, b->d_params, b->d_tokens,
                          b->tok_cap, b->d_mbinfo, b->d_mboff, b->cfg.method >= 5, b->d_results,
                          b->d_rerun, recon, b->d_xsync, b->d_wsnap, rp, st))
    return 0;
  return 1;
fail:
  return 0;
}

/* after launch_k3 and the results' copy to h_results (stream drained): a
 * launch in which some frame's token row ran out of room runs again (from
 * the saved d_rerun) with rows wide enough for the longest row it reported
 * (K3 counts a row's tokens on after the room is gone). The frames this
 * launch skipped (pass_mode 2) keep their rows. Returns 2 when K3 ran again
 * (d_rerun changed), 1 else. */
static int k3_settle(WebPGpuBatch* b, int n, uint8_t* recon) {
  if (!rows_mode(b)) return 1;
  hipStream_t st = b->stream;
  int rerun = 0;
  for (int tries = 0;; ++tries) {
    int over = 0;
    for (int f = 0; f < n; ++f)
      if (b->h_params[f].pass_mode != 2 && (b->h_results[f].error & VP8G_ERR_ARENA)) over = 1;
    if (!over) return rerun ? 2 : 1;
    const size_t nr = (size_t)n * b->mbh;
    CHK(hipMemcpy(b->h_rowtok, b->d_rowtok, nr * sizeof(uint32_t), hipMemcpyDeviceToHost));
    size_t longest = 0;
    for (int f = 0; f < n; ++f)
      if (b->h_params[f].pass_mode != 2)
        for (int y = 0; y < b->mbh; ++y)
          if (b->h_rowtok[(size_t)f * b->mbh + y] > longest) longest = b->h_rowtok[(size_t)f * b->mbh + y];
    size_t want = longest + longest / 8 + 64;
    if (want < 2 * b->rowcap) want = 2 * b->rowcap;
    if (tries > 4 || b->rowcap >= (size_t)VP8G_MAX_TOKENS_PER_MB * b->mbw || !ensure_rows(b, want, n)) {
      vp8g_set_error("k_encode", "token rows cannot grow");
      return 0;
    }
    int reread = 0;
    for (int f = 0; f < n; ++f)
      reread |= b->h_params[f].pass_mode == 1 || b->h_params[f].pass_mode == 3;
    if (reread)
      CHK(hipMemcpyAsync(b->d_rerun, b->d_rerun_snap, (size_t)n * VP8G_RERUN_STATE_BYTES,
                         hipMemcpyDeviceToDevice, st));
    if (!launch_k3(b, n, recon)) return 0;
    rerun = 1;
    CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                       hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
  }
fail:
  return 0;
}

/* VP8AdjustFilterStrength reads dqm->max_edge_, which StoreMaxDelta raises in
 * every RD_OPT_BASIC decision since the last SetupMatrices: the last StatLoop
 * pass and the final pass share one set of segment parameters, so the final
 * maxima include the last StatLoop pass's (lm_max_edge). */
static void merge_stat_max_edge(WebPGpuBatch* b, int n) {
  for (int f = 0; f < n; ++f) {
    vp8g_frame_result* R = &b->h_results[f];
    if (b->err[f] != VP8_ENC_OK || R->error) continue;
    for (int sg = 0; sg < 4; ++sg)
      if (b->frames[f].lm_max_edge[sg] > R->max_edge[sg]) R->max_edge[sg] = b->frames[f].lm_max_edge[sg];
  }
}

/* low_memory with methods 3-6: VP8EncLoop (frame_enc.c:614-775). StatLoop
 * passes run K3 at RD_OPT_BASIC with the default probabilities and no cost
 * refreshes; k_lowmem replays the statistics of the probe MBs (method 3: half
 * the frame) from the compact token stream and counts their skips. The host
 * then finalises the probabilities and the skip flag, and the final K3 pass
 * runs the method's RD level with those costs frozen; k_lowmem drops the
 * tokens of skipped MBs when the skip flag pays. */
static int lowmem_passes(WebPGpuBatch* b, int n) {
  const size_t nmb = (size_t)b->nmb, N = (size_t)b->max_frames;
  hipStream_t st = b->stream;
  uint8_t* act = b->pass_act;
  if (!b->d_lmstats) {
    CHK(hipMalloc((void**)&b->d_lmstats, N * VP8G_NUM_SLOTS * sizeof(uint32_t)));
    CHK(hipMalloc((void**)&b->d_lmi, 2 * N * sizeof(int32_t)));
    CHK(hipHostMalloc((void**)&b->h_lmstats, N * VP8G_NUM_SLOTS * sizeof(uint32_t), 0));
    CHK(hipHostMalloc((void**)&b->h_lmi, 2 * N * sizeof(int32_t), 0));
  }
  if (!b->h_active) {
    CHK(hipHostMalloc((void**)&b->h_active, N, 0));
    CHK(hipMalloc((void**)&b->d_active, N));
  }
  if (!b->h_state)
    CHK(hipHostMalloc((void**)&b->h_state, N * VP8G_RERUN_STATE_BYTES, 0));
  int32_t* h_nb = b->h_lmi;          /* probe MBs per frame */
  int32_t* h_nskip = b->h_lmi + N;   /* their skips (last pass) */
  const int nb = b->cfg.method == 3 ? ((nmb > 200) ? (int)(nmb >> 1) : 100) : (int)nmb;
  CHK(hipMemsetAsync(b->d_lmstats, 0, n * VP8G_NUM_SLOTS * sizeof(uint32_t), st));
  for (int f = 0; f < n; ++f) {
    h_nb[f] = nb;
    memset(b->frames[f].lm_max_edge, 0, sizeof(b->frames[f].lm_max_edge));
    act[f] = b->err[f] == VP8_ENC_OK && vp8h_pass_start(&b->frames[f]);
  }
  CHK(hipMemcpyAsync(b->d_lmi, b->h_lmi, 2 * n * sizeof(int32_t), hipMemcpyHostToDevice, st));
  int first = 1;
  for (;;) {   /* StatLoop (frame_enc.c:614-674), no search */
    int nact = 0;
    for (int f = 0; f < n; ++f) {
      vp8g_frame_params* P = &b->h_params[f];
      b->h_active[f] = act[f];
      if (!act[f]) { P->pass_mode = 2; continue; }
      vp8h_frame* fr = &b->frames[f];
      vp8h_set_loop_params(fr, fr->ps_q, b->h_segmap + f * nmb, P);
      P->rd_opt = 1;                /* RD_OPT_BASIC */
      P->max_count = 0x7fffffff;    /* no refreshes: the default probabilities' costs */
      P->pass_mode = 0;
      P->recon_addr = 0;
      ++nact;
    }
    if (!nact) break;
    if (!stamp_progress(b, n)) return 0;
    CHK(hipMemcpyAsync(b->d_segmap, b->h_segmap, n * nmb, hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_params, b->h_params, n * sizeof(vp8g_frame_params),
                       hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_active, b->h_active, n, hipMemcpyHostToDevice, st));
    if (first) CHK(hipEventRecord(b->ev[2], st));
    first = 0;
    if (!vp8g_launch_encode(b->d_yuv, b->yfb, b->w, b->h, n, b->d_segmap, b->d_params,
                            b->d_tokens, b->tok_cap, b->d_mbinfo, b->d_mboff, b->cfg.method >= 5,
                            b->d_results, b->d_rerun, NULL, b->d_xsync, b->d_wsnap, NULL, st))
      return 0;
    if (!vp8g_launch_lowmem(b->d_tokens, b->tok_cap, b->d_mboff, b->d_results, b->d_mbinfo,
                            (int)nmb, n, b->d_lmi, b->d_active, 0, b->d_lmstats, b->d_lmi + N, st))
      return 0;
    CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                       hipMemcpyDeviceToHost, st));
    const int probe = nb < (int)nmb;   /* method 3: OneStatPass covers the first nb MBs */
    if (probe)
      CHK(hipMemcpyAsync(b->h_mbinfo, b->d_mbinfo, n * nmb * VP8G_MBINFO_BYTES,
                         hipMemcpyDeviceToHost, st));
    CHK(engine_wait(b, st));   /* per-row progress and the hook's abort */
    for (int f = 0; f < n; ++f) {
      if (!act[f]) continue;
      vp8h_frame* fr = &b->frames[f];
      const vp8g_frame_result* R = &b->h_results[f];
      if (R->error) { act[f] = 0; continue; }
      /* K3's maxima span the whole frame: merged only when the pass covers
       * every MB (a method-3 probe's own maxima are not available) */
      if (!probe)
        for (int sg = 0; sg < 4; ++sg) fr->lm_max_edge[sg] = R->max_edge[sg];
      /* size_p0 of the probe (frame_enc.c:596, 651-655): K3 sums every MB's
       * info.H; the probe's sum comes from the MBs' modes */
      const uint64_t hdr = probe ? vp8h_mode_header_bits(
                                       b->h_mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES,
                                       fr->mbw, nb)
                                 : R->size_p0;
      act[f] = vp8h_pass_finish(fr, hdr + (uint64_t)fr->seg_hdr_size) && vp8h_pass_start(fr);
    }
  }
  /* FinalizeSkipProba + FinalizeTokenProbas + VP8CalculateLevelCosts */
  CHK(hipMemcpyAsync(b->h_lmstats, b->d_lmstats, n * VP8G_NUM_SLOTS * sizeof(uint32_t),
                     hipMemcpyDeviceToHost, st));
  CHK(hipMemcpyAsync(b->h_lmi + N, b->d_lmi + N, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  int nfinal = 0;
  for (int f = 0; f < n; ++f) {
    vp8g_frame_params* P = &b->h_params[f];
    b->h_active[f] = 0;
    if (b->err[f] != VP8_ENC_OK || b->h_results[f].error) { P->pass_mode = 2; continue; }
    uint8_t* S = b->h_state + (size_t)f * VP8G_RERUN_STATE_BYTES;
    int dirty = 0;
    vp8h_finalize_probas(b->h_lmstats + (size_t)f * VP8G_NUM_SLOTS, S + VP8G_STATE_COEFFS, &dirty);
    if (dirty) memcpy(S, S + VP8G_STATE_COEFFS, VP8G_NUM_SLOTS);
    else vp8h_default_probas(S);
    const int skip_proba = (int)((uint64_t)(nmb - h_nskip[f]) * 255 / nmb);
    b->frames[f].lm_skip_proba = skip_proba;
    b->h_active[f] = skip_proba < 250;   /* use_skip_proba */
    P->rd_opt = b->frames[f].rd_opt;   /* the final pass: the method's RD level */
    P->max_count = 0x7fffffff;
    P->pass_mode = 1;                  /* costs + probabilities from the state */
    P->max_i4_header_bits = b->frames[f].max_i4_header_bits;
    P->recon_addr = b->cfg.autofilter ? (uint64_t)(uintptr_t)(b->d_recon + (size_t)f * nmb * 512) : 0;
    ++nfinal;
  }
  if (first) CHK(hipEventRecord(b->ev[2], st));
  if (!nfinal) {
    CHK(hipEventRecord(b->ev[3], st));
    return 1;
  }
  CHK(hipMemcpyAsync(b->d_rerun, b->h_state, n * VP8G_RERUN_STATE_BYTES, hipMemcpyHostToDevice, st));
  if (!stamp_progress(b, n)) return 0;
  CHK(hipMemcpyAsync(b->d_params, b->h_params, n * sizeof(vp8g_frame_params),
                     hipMemcpyHostToDevice, st));
  if (!vp8g_launch_encode(b->d_yuv, b->yfb, b->w, b->h, n, b->d_segmap, b->d_params, b->d_tokens,
                          b->tok_cap, b->d_mbinfo, b->d_mboff, b->cfg.method >= 5, b->d_results,
                          b->d_rerun, b->cfg.autofilter ? b->d_recon : NULL, b->d_xsync, b->d_wsnap, NULL, st))
    return 0;
  CHK(hipEventRecord(b->ev[3], st));
  CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                     hipMemcpyDeviceToHost, st));
  CHK(engine_wait(b, st));   /* per-row progress and the hook's abort */
  /* the emitted probabilities are StatLoop's, not the final pass's */
  for (int f = 0; f < n; ++f) {
    if (b->h_params[f].pass_mode != 1 || b->h_results[f].error) continue;
    vp8g_frame_result* R = &b->h_results[f];
    memcpy(R->probas, b->h_state + (size_t)f * VP8G_RERUN_STATE_BYTES + VP8G_STATE_COEFFS,
           VP8G_NUM_SLOTS);
    R->use_skip = (int16_t)b->h_active[f];
    R->skip_proba = (int16_t)b->frames[f].lm_skip_proba;
  }
  CHK(hipMemcpyAsync(b->d_results, b->h_results, n * sizeof(vp8g_frame_result),
                     hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(b->d_active, b->h_active, n, hipMemcpyHostToDevice, st));
  if (!vp8g_launch_lowmem(b->d_tokens, b->tok_cap, b->d_mboff, b->d_results, b->d_mbinfo,
                          (int)nmb, n, b->d_lmi, b->d_active, 1, b->d_lmstats, b->d_lmi + N, st))
    return 0;
  CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                     hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  merge_stat_max_edge(b, n);
  return 1;
fail:
  return 0;
}

/* VP8EncLoop with a size / PSNR search (methods 0-2, or low_memory;
 * frame_enc.c:574-672, 739-774): StatLoop's passes decide at RD_OPT_BASIC
 * over every MB (no fast probe while searching) -> K3 with the level costs of
 * the current probabilities and no refreshes (intra-4 only from method 2,
 * quant_enc.c:1375-1377), k_lowmem adds every MB's token statistics (kept
 * across passes, ResetTokenStats runs once) and counts the skips. A size
 * search finalises the skip flag and the probabilities after each pass
 * (OneStatPass, :602-607; the next pass's costs follow them when they
 * changed) and values the pass at (sum R + H + both finalize costs + header
 * estimate) in bytes; a PSNR search values it by its distortion and
 * finalises once at the end. The final pass keeps the last pass's segment
 * parameters: K3 at the method's RD level (low_memory) then k_lowmem's skip
 * drop, or K3N (methods 0-2) with the StatLoop statistics and skip count. */
static int statloop_search(WebPGpuBatch* b, int n) {
  const size_t nmb = (size_t)b->nmb, N = (size_t)b->max_frames;
  hipStream_t st = b->stream;
  uint8_t* act = b->pass_act;
  const int m012 = b->cfg.method < 3;
  if (!b->d_lmstats) {
    CHK(hipMalloc((void**)&b->d_lmstats, N * VP8G_NUM_SLOTS * sizeof(uint32_t)));
    CHK(hipMalloc((void**)&b->d_lmi, 2 * N * sizeof(int32_t)));
    CHK(hipHostMalloc((void**)&b->h_lmstats, N * VP8G_NUM_SLOTS * sizeof(uint32_t), 0));
    CHK(hipHostMalloc((void**)&b->h_lmi, 2 * N * sizeof(int32_t), 0));
  }
  if (!b->h_active) {
    CHK(hipHostMalloc((void**)&b->h_active, N, 0));
    CHK(hipMalloc((void**)&b->d_active, N));
  }
  if (!b->h_state)
    CHK(hipHostMalloc((void**)&b->h_state, N * VP8G_RERUN_STATE_BYTES, 0));
  int32_t* h_nb = b->h_lmi;          /* statistics MBs per frame: all of them */
  int32_t* h_nskip = b->h_lmi + N;   /* their skips */
  CHK(hipMemsetAsync(b->d_lmstats, 0, n * VP8G_NUM_SLOTS * sizeof(uint32_t), st));
  for (int f = 0; f < n; ++f) {
    h_nb[f] = (int32_t)nmb;
    uint8_t* S = b->h_state + (size_t)f * VP8G_RERUN_STATE_BYTES;
    vp8h_default_probas(S);                        /* the probabilities of the level costs */
    vp8h_default_probas(S + VP8G_STATE_COEFFS);    /* the current probabilities */
    b->frames[f].npass = 0;
    b->frames[f].lm_nskip = 0;
    b->frames[f].lm_skip_proba = 255;
    memset(b->frames[f].lm_max_edge, 0, sizeof(b->frames[f].lm_max_edge));
    act[f] = b->err[f] == VP8_ENC_OK && vp8h_pass_start(&b->frames[f]);
  }
  CHK(hipMemcpyAsync(b->d_lmi, b->h_lmi, 2 * n * sizeof(int32_t), hipMemcpyHostToDevice, st));
  int first = 1;
  for (;;) {
    int nact = 0;
    for (int f = 0; f < n; ++f) {
      vp8g_frame_params* P = &b->h_params[f];
      b->h_active[f] = act[f];
      if (!act[f]) { P->pass_mode = 2; continue; }
      vp8h_frame* fr = &b->frames[f];
      vp8h_set_loop_params(fr, fr->ps_q, b->h_segmap + f * nmb, P);
      P->rd_opt = 1;                /* RD_OPT_BASIC */
      P->max_count = 0x7fffffff;    /* no refreshes inside a pass */
      P->pass_mode = fr->npass == 0 ? 0 : 1;   /* later passes: the costs of S */
      P->max_i4_header_bits = fr->method >= 2 ? fr->max_i4_header_bits : 0;
      P->recon_addr = 0;
      ++fr->npass;
      ++nact;
    }
    if (!nact) break;
    if (!stamp_progress(b, n)) return 0;
    CHK(hipMemcpyAsync(b->d_segmap, b->h_segmap, n * nmb, hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_params, b->h_params, n * sizeof(vp8g_frame_params),
                       hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_active, b->h_active, n, hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_rerun, b->h_state, n * VP8G_RERUN_STATE_BYTES, hipMemcpyHostToDevice,
                       st));
    if (first) CHK(hipEventRecord(b->ev[2], st));
    first = 0;
    /* RD_OPT_BASIC: the instantiation without trellis paths (it sums R + H) */
    if (!vp8g_launch_encode(b->d_yuv, b->yfb, b->w, b->h, n, b->d_segmap, b->d_params,
                            b->d_tokens, b->tok_cap, b->d_mbinfo, b->d_mboff, 0,
                            b->d_results, b->d_rerun, NULL, b->d_xsync, b->d_wsnap, NULL, st))
      return 0;
    if (!vp8g_launch_lowmem(b->d_tokens, b->tok_cap, b->d_mboff, b->d_results, b->d_mbinfo,
                            (int)nmb, n, b->d_lmi, b->d_active, 0, b->d_lmstats, b->d_lmi + N, st))
      return 0;
    CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                       hipMemcpyDeviceToHost, st));
    CHK(hipMemcpyAsync(b->h_lmstats, b->d_lmstats, n * VP8G_NUM_SLOTS * sizeof(uint32_t),
                       hipMemcpyDeviceToHost, st));
    CHK(hipMemcpyAsync(h_nskip, b->d_lmi + N, n * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    CHK(engine_wait(b, st));   /* per-row progress and the hook's abort */
    for (int f = 0; f < n; ++f) {
      if (!act[f]) continue;
      vp8h_frame* fr = &b->frames[f];
      const vp8g_frame_result* R = &b->h_results[f];
      if (R->error) { act[f] = 0; continue; }
      fr->lm_nskip = h_nskip[f];
      for (int sg = 0; sg < 4; ++sg) fr->lm_max_edge[sg] = R->max_edge[sg];
      const uint64_t size_p0 = R->size_p0 + (uint64_t)fr->seg_hdr_size;
      if (fr->do_size_search) {   /* OneStatPass, :602-607 */
        uint8_t* S = b->h_state + (size_t)f * VP8G_RERUN_STATE_BYTES;
        int use_skip = 0, dirty = 0;
        uint64_t size = R->size_rh;
        size += (uint64_t)vp8h_finalize_skip(h_nskip[f], (int)nmb, &fr->lm_skip_proba, &use_skip);
        size += (uint64_t)vp8h_finalize_probas(b->h_lmstats + (size_t)f * VP8G_NUM_SLOTS,
                                               S + VP8G_STATE_COEFFS, &dirty);
        if (dirty) memcpy(S, S + VP8G_STATE_COEFFS, VP8G_NUM_SLOTS);   /* VP8CalculateLevelCosts */
        fr->ps_value = (double)(((size + size_p0 + 1024) >> 11) + (12 + 8 + 10));
      } else {
        fr->ps_value = vp8h_psnr(R->distortion, (uint64_t)nmb * 384);
      }
      act[f] = vp8h_statloop_finish(fr, size_p0) && vp8h_pass_start(fr);
    }
  }
  /* the final pass */
  int nfinal = 0;
  for (int f = 0; f < n; ++f) {
    vp8g_frame_params* P = &b->h_params[f];
    vp8h_frame* fr = &b->frames[f];
    b->h_active[f] = 0;
    if (b->err[f] != VP8_ENC_OK || b->h_results[f].error) { P->pass_mode = 2; continue; }
    uint8_t* S = b->h_state + (size_t)f * VP8G_RERUN_STATE_BYTES;
    const uint32_t* stats = b->h_lmstats + (size_t)f * VP8G_NUM_SLOTS;
    if (!fr->do_size_search) {   /* StatLoop's own finalisation, :665-669 */
      int use_skip = 0, dirty = 0;
      vp8h_finalize_skip(fr->lm_nskip, (int)nmb, &fr->lm_skip_proba, &use_skip);
      vp8h_finalize_probas(stats, S + VP8G_STATE_COEFFS, &dirty);
      if (dirty) memcpy(S, S + VP8G_STATE_COEFFS, VP8G_NUM_SLOTS);
    }
    /* the segment parameters stay those of the last pass (P as set then) */
    P->max_i4_header_bits = fr->max_i4_header_bits;
    P->recon_addr = b->cfg.autofilter ? (uint64_t)(uintptr_t)(b->d_recon + (size_t)f * nmb * 512) : 0;
    if (m012) {   /* K3N with StatLoop's statistics and skip count */
      P->rd_opt = 0;
      P->max_count = 0x7fffffff;
      P->pass_mode = 3;
      P->nb_stat = 0;
      P->none_finalize = 1;
      P->skip_count = fr->lm_nskip;
      memcpy(S + VP8G_STATE_STATS, stats, VP8G_NUM_SLOTS * sizeof(uint32_t));
    } else {      /* K3 at the method's RD level with the costs frozen */
      b->h_active[f] = fr->lm_skip_proba < 250;   /* use_skip_proba */
      P->rd_opt = fr->rd_opt;
      P->max_count = 0x7fffffff;
      P->pass_mode = 1;
    }
    ++nfinal;
  }
  if (!nfinal) {
    CHK(hipEventRecord(b->ev[3], st));
    return 1;
  }
  if (m012 && b->cfg.method < 2) {
    /* RefineUsingDistortion's presets for methods 0-1 are the MB type and UV
     * mode the last StatLoop pass chose (PickBestIntra16/4/UV set them in
     * the MB info, quant_enc.c:1058,1161,1215): K3N's mode byte, bit 1 =
     * intra-4, bits 0 and 2 = the UV mode */
    CHK(hipMemcpyAsync(b->h_mbinfo, b->d_mbinfo, n * nmb * VP8G_MBINFO_BYTES,
                       hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
    uint8_t* am = (uint8_t*)malloc(n * nmb);
    if (!am) return 0;
    for (size_t k = 0; k < n * nmb; ++k) {
      const uint8_t* in = b->h_mbinfo + k * VP8G_MBINFO_BYTES;
      am[k] = (uint8_t)((in[1] & 1) | ((in[0] == 0) << 1) | ((in[1] >> 1) << 2));
    }
    const hipError_t e1 = hipMemcpy(b->d_amode, am, n * nmb, hipMemcpyHostToDevice);
    free(am);
    CHK(e1);
  }
  CHK(hipMemcpyAsync(b->d_rerun, b->h_state, n * VP8G_RERUN_STATE_BYTES, hipMemcpyHostToDevice, st));
  if (!stamp_progress(b, n)) return 0;
  CHK(hipMemcpyAsync(b->d_params, b->h_params, n * sizeof(vp8g_frame_params),
                     hipMemcpyHostToDevice, st));
  if (m012) {
    if (!vp8g_launch_encode_none(b->d_yuv, b->yfb, b->w, b->h, n, b->d_segmap, b->d_amode,
                                 b->d_params, b->d_tokens, b->tok_cap, b->d_mbinfo, b->d_mboff,
                                 b->d_results, b->d_rerun, st))
      return 0;
    CHK(hipEventRecord(b->ev[3], st));
    CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                       hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
    merge_stat_max_edge(b, n);
    return 1;
  }
  if (!vp8g_launch_encode(b->d_yuv, b->yfb, b->w, b->h, n, b->d_segmap, b->d_params, b->d_tokens,
                          b->tok_cap, b->d_mbinfo, b->d_mboff, b->cfg.method >= 5, b->d_results,
                          b->d_rerun, b->cfg.autofilter ? b->d_recon : NULL, b->d_xsync, b->d_wsnap, NULL, st))
    return 0;
  CHK(hipEventRecord(b->ev[3], st));
  CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                     hipMemcpyDeviceToHost, st));
  CHK(engine_wait(b, st));   /* per-row progress and the hook's abort */
  for (int f = 0; f < n; ++f) {   /* the emitted probabilities are StatLoop's */
    if (b->h_params[f].pass_mode != 1 || b->h_results[f].error) continue;
    vp8g_frame_result* R = &b->h_results[f];
    memcpy(R->probas, b->h_state + (size_t)f * VP8G_RERUN_STATE_BYTES + VP8G_STATE_COEFFS,
           VP8G_NUM_SLOTS);
    R->use_skip = (int16_t)b->h_active[f];
    R->skip_proba = (int16_t)b->frames[f].lm_skip_proba;
  }
  CHK(hipMemcpyAsync(b->d_results, b->h_results, n * sizeof(vp8g_frame_result),
                     hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(b->d_active, b->h_active, n, hipMemcpyHostToDevice, st));
  if (!vp8g_launch_lowmem(b->d_tokens, b->tok_cap, b->d_mboff, b->d_results, b->d_mbinfo,
                          (int)nmb, n, b->d_lmi, b->d_active, 1, b->d_lmstats, b->d_lmi + N, st))
    return 0;
  CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                     hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  merge_stat_max_edge(b, n);
  return 1;
fail:
  return 0;
}

/* VP8EncTokenLoop's pass loop (frame_enc.c:808-880) for every frame of the
 * batch in lock step. Each round sets the loop parameters of each unfinished
 * frame for its pass (SetLoopParams with the frame's current q) and runs K3
 * over the batch (finished frames skip it, pass_mode 2). A size search
 * (target_size) then finalises the probabilities from each frame's token
 * statistics on the host and estimates the token bits on the device
 * (k_token_cost); each frame decides on its own whether another pass follows
 * (search step, or the partition-0 overflow retry of :869-876). */
static int run_passes(WebPGpuBatch* b, int n) {
  const size_t nmb = (size_t)b->nmb;
  hipStream_t st = b->stream;
  int* fin_cost = b->fin_cost;
  uint8_t* act = b->pass_act;
  const int af = b->cfg.autofilter != 0;
  if (af && !b->d_recon) {
    const size_t N = (size_t)b->max_frames;
    CHK(hipMalloc((void**)&b->d_recon, N * nmb * 512));
    CHK(hipMalloc((void**)&b->d_mbval, N * nmb * 64 * sizeof(double)));
    CHK(hipMalloc((void**)&b->d_afp, N * sizeof(vp8g_af_frame)));
    CHK(hipMalloc((void**)&b->d_aflevel, N * 4));
    CHK(hipHostMalloc((void**)&b->h_afp, N * sizeof(vp8g_af_frame), 0));
    CHK(hipHostMalloc((void**)&b->h_aflevel, N * 4, 0));
    if (!b->h_active) {
      CHK(hipHostMalloc((void**)&b->h_active, N, 0));
      CHK(hipMalloc((void**)&b->d_active, N));
    }
  }
  int round = 0;
  /* low_memory only changes methods 3-6 (they switch to VP8EncLoop,
   * webp_enc.c:115-122); methods 0-2 already run VP8EncLoop and encode exactly
   * as without the flag */
  const int lowmem = b->cfg.low_memory && b->cfg.method >= 3;
  /* a size / PSNR search under VP8EncLoop (methods 0-2 or low_memory) */
  const int search = (b->cfg.method < 3 || b->cfg.low_memory) &&
                     (b->cfg.target_size > 0 || b->cfg.target_PSNR > 0);
  if (search) {
    if (!statloop_search(b, n)) return 0;
    round = 1;
  } else if (lowmem) {
    if (!lowmem_passes(b, n)) return 0;
    round = 1;
  }
  for (int f = 0; f < n; ++f)
    act[f] = !lowmem && !search && b->err[f] == VP8_ENC_OK && vp8h_pass_start(&b->frames[f]);
  for (;;) {
    int nact = 0, nsize = 0;
    for (int f = 0; f < n; ++f) {
      vp8g_frame_params* P = &b->h_params[f];
      if (!act[f]) { P->pass_mode = 2; continue; }
      vp8h_frame* fr = &b->frames[f];
      vp8h_set_loop_params(fr, fr->ps_q, b->h_segmap + f * nmb, P);
      /* StatLoop (RD_OPT_NONE) never resets its statistics between passes */
      P->pass_mode = fr->npass == 0 ? 0 : (fr->is_last_pass && fr->rd_opt > 0) ? 1 : 3;
      P->recon_addr = af ? (uint64_t)(uintptr_t)(b->d_recon + (size_t)f * nmb * 512) : 0;
      ++fr->npass;
      ++nact;
      nsize += fr->do_size_search && !fr->is_last_pass;
    }
    if (!nact) break;
    if (!stamp_progress(b, n)) return 0;
    CHK(hipMemcpyAsync(b->d_segmap, b->h_segmap, n * nmb, hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_params, b->h_params, n * sizeof(vp8g_frame_params),
                       hipMemcpyHostToDevice, st));
    if (round == 0) CHK(hipEventRecord(b->ev[2], st));
    if (b->cfg.method < 3) {   /* methods 0-2: VP8EncLoop's RD_OPT_NONE encoder */
      if (!vp8g_launch_encode_none(b->d_yuv, b->yfb, b->w, b->h, n, b->d_segmap, b->d_amode,
                                   b->d_params, b->d_tokens, b->tok_cap, b->d_mbinfo, b->d_mboff,
                                   b->d_results, b->d_rerun, st))
        return 0;
    } else if (!launch_k3(b, n, af ? b->d_recon : NULL)) {   /* the token loop */
      return 0;
    }
    CHK(hipEventRecord(b->ev[3], st));
    CHK(hipMemcpyAsync(b->h_results, b->d_results, n * sizeof(vp8g_frame_result),
                       hipMemcpyDeviceToHost, st));
    if (nsize) {
      /* each buffer on its own first use: low_memory passes allocate h_state too */
      if (!b->h_state)
        CHK(hipHostMalloc((void**)&b->h_state, (size_t)b->max_frames * VP8G_RERUN_STATE_BYTES, 0));
      if (!b->h_tbits)
        CHK(hipHostMalloc((void**)&b->h_tbits, b->max_frames * sizeof(unsigned long long), 0));
      if (!b->d_tbits)
        CHK(hipMalloc((void**)&b->d_tbits, b->max_frames * sizeof(unsigned long long)));
      if (!b->h_active) {
        CHK(hipHostMalloc((void**)&b->h_active, b->max_frames, 0));
        CHK(hipMalloc((void**)&b->d_active, b->max_frames));
      }
      CHK(hipMemcpyAsync(b->h_state, b->d_rerun, (size_t)n * VP8G_RERUN_STATE_BYTES,
                         hipMemcpyDeviceToHost, st));
    }
    CHK(engine_wait(b, st));
    if (b->cfg.method >= 3) {
      const int rc = k3_settle(b, n, af ? b->d_recon : NULL);
      if (!rc) return 0;
      if (rc == 2 && nsize)   /* K3 ran again: the state the size search reads */
        CHK(hipMemcpy(b->h_state, b->d_rerun, (size_t)n * VP8G_RERUN_STATE_BYTES,
                      hipMemcpyDeviceToHost));
    }
    if (nsize) {   /* FinalizeTokenProbas, then VP8EstimateTokenSize on the device */
      for (int f = 0; f < n; ++f) {
        vp8h_frame* fr = &b->frames[f];
        b->h_active[f] = act[f] && fr->do_size_search && !fr->is_last_pass &&
                         !b->h_results[f].error;
        if (!b->h_active[f]) continue;
        uint8_t* S = b->h_state + (size_t)f * VP8G_RERUN_STATE_BYTES;
        int dirty = 0;
        fin_cost[f] = vp8h_finalize_probas((const uint32_t*)(S + VP8G_STATE_STATS),
                                           S + VP8G_STATE_COEFFS, &dirty);
        /* VP8CalculateLevelCosts at the next pass start recomputes the level
         * costs only when the update left a non-default probability */
        if (dirty) memcpy(S, S + VP8G_STATE_COEFFS, VP8G_NUM_SLOTS);
      }
      CHK(hipMemcpyAsync(b->d_rerun, b->h_state, (size_t)n * VP8G_RERUN_STATE_BYTES,
                         hipMemcpyHostToDevice, st));
      CHK(hipMemcpyAsync(b->d_active, b->h_active, n, hipMemcpyHostToDevice, st));
      vp8g_rows R = {(uint32_t)b->rowcap, b->d_rowtok};
      if (!vp8g_launch_token_cost(b->d_tokens, b->tok_cap, rows_mode(b) ? &R : NULL, b->mbh, n,
                                  b->d_results, b->d_rerun, b->d_active, b->d_tbits, st))
        return 0;
      CHK(hipMemcpyAsync(b->h_tbits, b->d_tbits, n * sizeof(unsigned long long),
                         hipMemcpyDeviceToHost, st));
      CHK(hipStreamSynchronize(st));
    }
    for (int f = 0; f < n; ++f) {
      if (!act[f]) continue;
      vp8h_frame* fr = &b->frames[f];
      const vp8g_frame_result* R = &b->h_results[f];
      if (R->error) { act[f] = 0; continue; }
      const uint64_t size_p0 = R->size_p0 + (uint64_t)fr->seg_hdr_size;
      if (fr->do_size_search)
        fr->ps_value = fr->is_last_pass ? 0.
                     : vp8h_pass_size_value((uint64_t)fin_cost[f], b->h_tbits[f], size_p0);
      else
        fr->ps_value = vp8h_psnr(R->distortion, (uint64_t)nmb * 384);
      act[f] = vp8h_pass_finish(fr, size_p0) && vp8h_pass_start(fr);
    }
    ++round;
  }
  if (round == 0) {   /* no frame to encode: keep the K3 timing events valid */
    CHK(hipEventRecord(b->ev[2], st));
    CHK(hipEventRecord(b->ev[3], st));
  }
  if (af && round > 0) {   /* VP8StoreFilterStats + VP8AdjustFilterStrength on the device */
    for (int f = 0; f < n; ++f) {
      const vp8h_frame* fr = &b->frames[f];
      vp8g_af_frame* A = &b->h_afp[f];
      b->h_active[f] = b->err[f] == VP8_ENC_OK && !b->h_results[f].error;
      A->simple = (uint8_t)fr->f_simple;
      A->sharpness = (uint8_t)fr->filter_sharpness;
      for (int s = 0; s < 4; ++s) {
        A->level0[s] = (uint8_t)fr->seg_fstrength[s];
        A->quant[s] = (uint8_t)fr->seg_quant[s];
      }
    }
    CHK(hipMemcpyAsync(b->d_afp, b->h_afp, n * sizeof(vp8g_af_frame), hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_active, b->h_active, n, hipMemcpyHostToDevice, st));
    if (!vp8g_launch_autofilter(b->d_yuv, b->yfb, b->w, b->h, n, b->d_mbinfo, b->d_recon,
                                b->d_afp, b->d_active, b->d_mbval, b->d_aflevel, st))
      return 0;
    CHK(hipMemcpyAsync(b->h_aflevel, b->d_aflevel, n * 4, hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
    for (int f = 0; f < n; ++f)
      if (b->h_active[f])
        for (int s = 0; s < 4; ++s) b->frames[f].seg_fstrength[s] = b->h_aflevel[4 * f + s];
  }
  CHK(hipStreamSynchronize(st));
  if (!d2h_sdma_download(b->device, b->h_mbinfo, b->d_mbinfo, n * nmb * VP8G_MBINFO_BYTES)) {
    CHK(hipMemcpyAsync(b->h_mbinfo, b->d_mbinfo, n * nmb * VP8G_MBINFO_BYTES,
                       hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
  }
  return 1;
fail:
  return 0;
}

/* Partition 0 on the device when asked (WEBP_AMD_P0=gpu), or, by default,
 * when the rank's host-thread budget is small: coding it is ~1 ms of one CPU
 * per 1080p frame (the intra-4 modes), which a budget of a few threads shared
 * by several engines cannot keep up with, while on the
 * device it adds a K4 stream of ~1/13 of the frame's tokens. */
#define P0_DEVICE_BELOW 8   /* host threads per rank */
/* Partition 0 on the device when the host has few threads (the 8-rank
 * budget) or the call has few frames: a single picture's host tail (1.2 ms
 * for 1080p) is latency with nothing beside it to hide behind, the device
 * path adds 0.3 ms of K4 (one 1080p frame 32.4 -> 31.6 ms,
 * profiles/r6/k3x/p0/); a batch's host tails overlap the other instances'
 * kernels (256 x 1080p at 16 threads: 4782 host vs 4663 MP/s device) */
static int use_gpu_p0(const WebPGpuBatch* b, int n) {
  if (b->gpu_p0 >= 0) return b->gpu_p0;
  return b->threads < P0_DEVICE_BELOW || n <= VP8G_XSPLIT_MAX_FRAMES;
}

int vp8g_engine_run_yuv(WebPGpuBatch* b, int n) {
  const size_t nmb = (size_t)b->nmb;
  double t0 = now_us(), t1, t2, t3, t4;
  hipStream_t st = b->stream;
  TailJob head;
  int head_running = 0;
  b->timings[9] = 0;
  if (!tokens_for_run(b)) return 0;
  if (getenv("WEBP_AMD_FAULT_REPORT")) {   /* diagnostics: buffer ranges for a fault address */
    vp8g_fault_report_init();
    fprintf(stderr,
            "WEBP_AMD_BUFFERS tokens %p +%zu yuv %p +%zu mbinfo %p +%zu mboff %p +%zu "
            "wsnap %p +%zu results %p +%zu params %p segmap %p rowtok %p\n",
            (void*)b->d_tokens, (size_t)b->max_frames * (b->tok_cap + b->p0_cap) * 2, (void*)b->d_yuv,
            (size_t)b->max_frames * b->yfb, (void*)b->d_mbinfo, (size_t)b->max_frames * nmb * 20,
            (void*)b->d_mboff, (size_t)b->max_frames * nmb * 4, (void*)b->d_wsnap,
            (size_t)b->max_frames * vp8g_wsnap_bytes(b->w, b->h), (void*)b->d_results,
            (size_t)b->max_frames * sizeof(vp8g_frame_result), (void*)b->d_params,
            (void*)b->d_segmap, (void*)b->d_rowtok);
  }
  if (!encode_alpha(b, n)) return 0;
  if (!b->ev0_recorded) CHK(hipEventRecord(b->ev[0], st));
  b->ev0_recorded = 0;
  if (!vp8g_launch_analysis(b->d_yuv, b->yfb, b->w, b->h, n, b->d_alpha, b->d_uva,
                            b->cfg.method <= 1 ? (int)b->cfg.quality : -1, b->d_amode, st))
    return 0;
  CHK(hipEventRecord(b->ev[1], st));
  CHK(hipMemcpyAsync(b->h_alpha, b->d_alpha, n * nmb, hipMemcpyDeviceToHost, st));
  CHK(hipMemcpyAsync(b->h_uva, b->d_uva, n * nmb * sizeof(uint16_t), hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  t1 = now_us();
  run_tails(b, n, 2);   /* per-frame setup + segment k-means on the host threads */
  t2 = now_us();
  if (!run_passes(b, n)) return 0;
  /* token partitions: VP8EncLoop only (vp8h_frame_init) */
  const int np = (b->cfg.method < 3 || b->cfg.low_memory) ? 1 << b->cfg.partitions : 1;
  const int ns = n * np;   /* K4 streams */
  b->nparts = np;
  if (np > 1 && b->host_emit) {
    vp8g_set_error("WebPGpuBatch", "WEBP_AMD_HOST_EMIT codes a single token partition");
    return 0;
  }
  if (!b->host_emit && np > 1) {   /* token partitions: rows regrouped per partition */
    if (!vp8g_launch_partition(b->d_tokens, b->tok_cap, n, b->d_mboff, b->d_results, b->d_mbinfo,
                               b->mbw, b->mbh, b->cfg.method < 3 ? 0 : 1, np, b->d_pinfo, st))
      return 0;
    CHK(hipMemcpyAsync(b->h_pinfo, b->d_pinfo, (size_t)n * 16 * sizeof(uint32_t),
                       hipMemcpyDeviceToHost, st));
    CHK(hipStreamSynchronize(st));
  }
  /* partition 0: coded on the host threads while K4 runs, or (gpu_p0) its
     header tokens built here and the rest done by k_p0_modes + K4 */
  const int p0dev = !b->host_emit && use_gpu_p0(b, n);
  b->p0_dev = p0dev;
  b->last_ns = ns;
  if (p0dev) {
    if (!b->h_p0hdr) {
      const size_t N = (size_t)b->max_frames;
      CHK(hipHostMalloc((void**)&b->h_p0hdr, N * VP8G_P0_HDR_CAP * sizeof(uint16_t), 0));
      CHK(hipHostMalloc((void**)&b->h_p0par, N * sizeof(vp8g_p0_par), 0));
      CHK(hipMalloc((void**)&b->d_p0hdr, N * VP8G_P0_HDR_CAP * sizeof(uint16_t)));
      CHK(hipMalloc((void**)&b->d_p0par, N * sizeof(vp8g_p0_par)));
    }
    run_tails(b, n, 3);
    uint32_t nh_max = 0;
    for (int f = 0; f < n; ++f)
      if (b->h_p0par[f].nhdr != 0xffffffffu && b->h_p0par[f].nhdr > nh_max) nh_max = b->h_p0par[f].nhdr;
    CHK(hipMemcpy2DAsync(b->d_p0hdr, VP8G_P0_HDR_CAP * sizeof(uint16_t), b->h_p0hdr,
                         VP8G_P0_HDR_CAP * sizeof(uint16_t), nh_max * sizeof(uint16_t) + 2, n,
                         hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(b->d_p0par, b->h_p0par, n * sizeof(vp8g_p0_par), hipMemcpyHostToDevice, st));
  }
  const int nst = ns + (p0dev ? n : 0);   /* K4 streams: partitions, then partition 0 */
  if (!b->host_emit) {   /* K4 on the device, sized from the token counts */
    const int rows = rows_mode(b) && np == 1;
    uint32_t max_ntok = 0, max_seg = 0;
    size_t segs = 0, words = 0;
    for (int s = ns; s < nst; ++s) {   /* partition 0: k_p0_modes sets ntok / nseg */
      const int f = s - ns;
      vp8g_emit_meta* m = &b->h_emeta[s];
      const uint32_t bound = (uint32_t)(b->p0_cap - VP8G_EMIT_SEG);
      m->ntok = bound;
      m->frame = (uint32_t)f;
      m->nrows = 0;
      m->rowcap = 0;
      m->pad = 0;
      m->tok_off = (uint64_t)b->max_frames * b->tok_cap + (uint64_t)f * b->p0_cap;
      m->nseg = (bound + VP8G_EMIT_SEG - 1) / VP8G_EMIT_SEG;
    }
    for (int s = 0; s < nst; ++s) {
      if (s >= ns) {   /* partition 0 (bounds; its meta fields above) */
        vp8g_emit_meta* m = &b->h_emeta[s];
        m->seg_base = (uint32_t)segs;
        m->nb_base = (uint32_t)words;
        m->S = m->L = 0;
        segs += m->nseg;
        words += (7 * (size_t)m->ntok + 17 + 8 + 63) / 32 + 4;
        if (m->ntok > max_ntok) max_ntok = m->ntok;
        if (m->nseg > max_seg) max_seg = m->nseg;
        continue;
      }
      const int f = s / np, p = s % np;
      vp8g_emit_meta* m = &b->h_emeta[s];
      const uint32_t* pi = np > 1 ? b->h_pinfo + 16 * (size_t)f : NULL;
      if (pi && pi[0] == 0xffffffffu && !b->h_results[f].error && b->err[f] == VP8_ENC_OK)
        b->err[f] = VP8_ENC_ERROR_OUT_OF_MEMORY;   /* the partitions did not fit the slab */
      const int ok = !b->h_results[f].error && !(pi && pi[0] == 0xffffffffu);
      m->ntok = !ok ? 0 : pi ? pi[8 + p] : b->h_results[f].ntokens;
      m->frame = (uint32_t)f;
      /* the token loop's streams lie in K3's token rows (k_emit_desc cuts them
         row by row: the count below is a bound, set exactly on the device) */
      m->nrows = rows && ok ? (uint32_t)b->mbh : 0;
      m->rowcap = rows ? (uint32_t)b->rowcap : 0;
      m->pad = 0;
      m->tok_off = (uint64_t)f * b->tok_cap + (ok && pi ? pi[p] : 0);
      m->nseg = (m->ntok + VP8G_EMIT_SEG - 1) / VP8G_EMIT_SEG + (ok ? m->nrows : 0);
      m->seg_base = (uint32_t)segs;
      m->nb_base = (uint32_t)words;
      m->S = m->L = 0;
      segs += m->nseg;
      words += (7 * (size_t)m->ntok + 17 + 8 + 63) / 32 + 4;
      if (m->ntok > max_ntok) max_ntok = m->ntok;
      if (m->nseg > max_seg) max_seg = m->nseg;
    }
    if (segs > b->emit_seg_cap) {
      hipFree(b->d_emap); hipFree(b->d_eshift); hipFree(b->d_esegs); hipFree(b->d_eimg);
      hipFree(b->d_edesc);
      b->d_emap = NULL; b->d_eshift = NULL; b->d_esegs = NULL; b->d_eimg = NULL; b->d_edesc = NULL;
      b->emit_seg_cap = 0;
      const size_t cap = segs + segs / 4 + 64;
      CHK(hipMalloc((void**)&b->d_emap, cap * 128));
      CHK(hipMalloc((void**)&b->d_edesc, cap * sizeof(vp8g_emit_desc)));
      CHK(hipMalloc((void**)&b->d_eshift, cap * 128 * sizeof(uint16_t)));
      CHK(hipMalloc((void**)&b->d_esegs, cap * sizeof(vp8g_emit_seg)));
      CHK(hipMalloc((void**)&b->d_eimg, cap * 17));
      b->emit_seg_cap = cap;
    }
    if (words > b->emit_word_cap) {
      hipFree(b->d_nbuf);
      b->d_nbuf = NULL; b->emit_word_cap = 0;
      const size_t cap = words + words / 4 + 256;
      CHK(hipMalloc((void**)&b->d_nbuf, cap * sizeof(uint32_t)));
      b->emit_word_cap = cap;
    }
    CHK(hipEventRecord(b->ev[5], st));
    CHK(hipMemsetAsync(b->d_nbuf, 0, words * sizeof(uint32_t), st));
    CHK(hipMemcpyAsync(b->d_emeta, b->h_emeta, nst * sizeof(vp8g_emit_meta),
                       hipMemcpyHostToDevice, st));
    if (p0dev && !vp8g_launch_p0_modes(b->d_mbinfo, b->mbw, b->mbh, n, b->d_p0par, b->d_p0hdr,
                                       b->d_tokens, b->d_emeta, ns, st))
      return 0;
    if (!vp8g_launch_emit(b->d_tokens, b->tok_cap, nst, b->d_results, b->d_emeta, b->d_rowtok,
                          max_ntok, max_seg, b->d_emap, b->d_eshift, b->d_eimg, b->d_edesc,
                          b->d_esegs, b->d_nbuf, b->d_psize, st))
      return 0;
    CHK(hipEventRecord(b->ev[4], st));
    CHK(hipMemcpyAsync(b->h_psize, b->d_psize, nst * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    if (!p0dev) {   /* partition 0 on the host threads while K4 runs on the device */
      tail_spawn(&head, b, n, 0, b->threads - 1);
      head_running = 1;
    }
    CHK(hipStreamSynchronize(st));
  }
  t3 = now_us();
  if (b->host_emit) {
    b->tok_off[0] = 0;
    for (int f = 0; f < n; ++f) b->tok_off[f + 1] = b->tok_off[f] + b->h_results[f].ntokens;
    const size_t total = b->tok_off[n];
    if (total > b->h_tok_cap) {
      hipHostFree(b->h_tokens);
      b->h_tokens = NULL;
      b->h_tok_cap = 0;
      const size_t cap = total + total / 4 + 1024;
      CHK(hipHostMalloc((void**)&b->h_tokens, cap * sizeof(uint16_t), 0));
      b->h_tok_cap = cap;
    }
    for (int f = 0; f < n; ++f)
      if (b->h_results[f].ntokens)
        CHK(hipMemcpyAsync(b->h_tokens + b->tok_off[f], b->d_tokens + (size_t)f * b->tok_cap,
                           b->h_results[f].ntokens * sizeof(uint16_t), hipMemcpyDeviceToHost, st));
  } else {
    /* one packed D2H of every frame's token partitions (k_pack) */
    uint32_t max_size = 0;
    b->h_poff[0] = 0;
    for (int s = 0; s < nst; ++s) {
      b->h_poff[s + 1] = b->h_poff[s] + ((b->h_psize[s] + 15u) & ~15u);
      if (b->h_psize[s] > max_size) max_size = b->h_psize[s];
    }
    const size_t total = b->h_poff[nst];
    if (total > b->h_part_cap) {
      hipHostFree(b->h_part);
      b->h_part = NULL;
      b->h_part_cap = 0;
      const size_t cap = total + total / 4 + 4096;
      CHK(hipHostMalloc((void**)&b->h_part, cap, 0));
      b->h_part_cap = cap;
    }
    if (total > b->d_part_cap) {
      hipFree(b->d_part);
      b->d_part = NULL;
      b->d_part_cap = 0;
      const size_t cap = total + total / 4 + 4096;
      CHK(hipMalloc((void**)&b->d_part, cap));
      b->d_part_cap = cap;
    }
    if (total) {
      CHK(hipMemcpyAsync(b->d_poff, b->h_poff, (nst + 1) * sizeof(uint64_t), hipMemcpyHostToDevice,
                         st));
      if (!vp8g_launch_pack(b->d_tokens, b->d_emeta, nst, b->d_poff, b->d_psize, max_size, b->d_part,
                            st))
        goto fail;
      CHK(hipStreamSynchronize(st));   /* then the bytes come back on a copy engine */
      if (!d2h_sdma_download(b->device, b->h_part, b->d_part, total))
        CHK(hipMemcpyAsync(b->h_part, b->d_part, total, hipMemcpyDeviceToHost, st));
    }
  }
  CHK(hipStreamSynchronize(st));
  t4 = now_us();
  if (head_running) {
    tail_join(&head);
    head_running = 0;
  } else if (!p0dev) {
    run_tails(b, n, 0);
  }
  const double t4b = now_us();
  run_tails(b, n, 1);
  const double t5 = now_us();
  if (getenv("LIBWEBP_AMD_TAIL_TIMING"))
    fprintf(stderr, "tail: head join %.0f us, finish %.0f us, threads %d\n", t4b - t4, t5 - t4b,
            b->threads);
  float k3_ms = 0.f, k12_ms = 0.f, k4_ms = 0.f;
  CHK(hipEventElapsedTime(&k3_ms, b->ev[2], b->ev[3]));
  CHK(hipEventElapsedTime(&k12_ms, b->ev[0], b->ev[1]));
  if (!b->host_emit) CHK(hipEventElapsedTime(&k4_ms, b->ev[5], b->ev[4]));
  b->timings[6] = 1e3 * k3_ms;
  b->timings[7] = 1e3 * k12_ms;
  b->timings[8] = 1e3 * k4_ms;
  b->timings[1] = t2 - t1;
  b->timings[2] = t3 - t2;
  b->timings[3] = t4 - t3;
  b->timings[4] = t5 - t4;
  b->timings[0] += t1 - t0;
  b->last_n = n;
  return 1;
fail:
  if (head_running) tail_join(&head);
  return 0;
}

/* RGBA -> YUV420 of n frames on the engine stream: K1, or the sharp-YUV
 * kernels (hip/vp8_sharp.hip) when requested. */
static int launch_import(WebPGpuBatch* b, const uint8_t* rgba, size_t fstride, int rstride, int n,
                         int sharp) {
  if (!sharp) {
    if (b->dither > 0.f && b->dither != b->dither_built) {
      /* dithered import (preprocessing & 2): the VP8Random rounding terms
       * depend only on the size and amplitude, so every frame shares them */
      const size_t ny = (size_t)b->w * b->h, nuv = 2 * (size_t)b->uvw * b->uvh;
      uint16_t* ry = (uint16_t*)malloc(ny * sizeof(uint16_t));
      uint32_t* ruv = (uint32_t*)malloc(nuv * sizeof(uint32_t));
      int ok = ry && ruv;
      if (ok) vp8h_dither_rounders(b->w, b->h, b->dither, ry, ruv);
      if (ok && !b->d_rnd_y)
        ok = hipMalloc((void**)&b->d_rnd_y, ny * sizeof(uint16_t)) == hipSuccess &&
             hipMalloc((void**)&b->d_rnd_uv, nuv * sizeof(uint32_t)) == hipSuccess;
      ok = ok && hipMemcpy(b->d_rnd_y, ry, ny * sizeof(uint16_t), hipMemcpyHostToDevice) ==
                     hipSuccess &&
           hipMemcpy(b->d_rnd_uv, ruv, nuv * sizeof(uint32_t), hipMemcpyHostToDevice) == hipSuccess;
      free(ry);
      free(ruv);
      if (!ok) {
        vp8g_set_error("launch_import", "dither rounders");
        return 0;
      }
      b->dither_built = b->dither;
    }
    const int dith = b->dither > 0.f;
    return vp8g_launch_import(rgba, fstride, rstride, b->w, b->h, n, b->d_yuv, b->yfb,
                              b->d_aflags, b->d_aplane, b->d_g2l, b->d_l2g,
                              dith ? b->d_rnd_y : NULL, dith ? b->d_rnd_uv : NULL, b->stream);
  }
  if (!vp8g_launch_extract_alpha(rgba, fstride, rstride, b->w, b->h, n, NULL, b->d_aplane,
                                 b->stream))
    return 0;
  if (!b->d_sharp) {   /* first sharp call: scratch for max_frames frames */
    const uint32_t *g2l, *l2g;
    vp8h_sharp_tables(&g2l, &l2g);
    CHK(hipMalloc((void**)&b->d_stabs, (1026 + 514) * sizeof(uint32_t)));
    CHK(hipMemcpy(b->d_stabs, g2l, 1026 * sizeof(uint32_t), hipMemcpyHostToDevice));
    CHK(hipMemcpy(b->d_stabs + 1026, l2g, 514 * sizeof(uint32_t), hipMemcpyHostToDevice));
    CHK(hipMalloc((void**)&b->d_sstate, b->max_frames * sizeof(vp8g_sharp_state)));
    CHK(hipMalloc((void**)&b->d_sharp, b->max_frames * vp8g_sharp_frame_bytes(b->w, b->h)));
  }
  return vp8g_launch_sharp(rgba, fstride, rstride, b->w, b->h, n, b->d_yuv, b->yfb, b->d_aflags,
                           b->d_sharp, b->d_sstate, b->d_stabs, b->d_stabs + 1026, b->stream);
fail:
  return 0;
}

static int run_rgba(WebPGpuBatch* b, const void* rgba_dev, size_t fstride, int rstride, int n,
                    void* stream) {
  const double t0 = now_us();
  if (n <= 0 || n > b->max_frames) return 0;
  if (rstride < 4 * b->w) return 0;
  if (n > 1 && fstride < (size_t)rstride * b->h) return 0;
  CHK(hipSetDevice(b->device));
  if (stream) {   /* order after the caller's producer work */
    hipEvent_t ev;
    CHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    CHK(hipEventRecord(ev, (hipStream_t)stream));
    CHK(hipStreamWaitEvent(b->stream, ev, 0));
    hipEventDestroy(ev);
  }
  if (b->l) {   /* lossless (VP8L) */
    const int ok = vp8l_engine_run(b, (const uint8_t*)rgba_dev, fstride, rstride, n);
    b->timings[5] = now_us() - t0;
    return ok;
  }
  for (int f = 0; f < n; ++f) b->err[f] = VP8_ENC_OK;
  CHK(hipMemsetAsync(b->d_aflags, 0, n * sizeof(uint32_t), b->stream));
  CHK(hipEventRecord(b->ev[0], b->stream));
  b->ev0_recorded = 1;
  if (!launch_import(b, (const uint8_t*)rgba_dev, fstride, rstride, n, b->sharp)) return 0;
  CHK(hipMemcpyAsync(b->h_aflags, b->d_aflags, n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                     b->stream));
  CHK(hipStreamSynchronize(b->stream));
  {
    int any = 0;
    for (int f = 0; f < n; ++f) {
      any |= b->h_aflags[f] != 0;
    }
    /* the alpha planes of the frames K1 found not opaque (K1 writes none) */
    if (any && !b->sharp &&
        !vp8g_launch_extract_alpha((const uint8_t*)rgba_dev, fstride, rstride, b->w, b->h, n,
                                   b->d_aflags, b->d_aplane, b->stream))
      return 0;
    /* webp_enc.c:369-371: smooth/flatten the fully transparent areas */
    if (any && !b->cfg.exact &&
        !vp8g_launch_cleanup_alpha(b->d_yuv, b->yfb, b->d_aplane, b->d_aflags, b->w, b->h, n,
                                   b->stream))
      return 0;
  }
  b->timings[0] = now_us() - t0;
  const int ok = vp8g_engine_run_yuv(b, n);
  b->timings[5] = now_us() - t0;
  return ok;
fail:
  return 0;
}

int WebPGpuBatchEncodeRGBA(WebPGpuBatch* b, const void* rgba_dev, size_t fstride, int rstride,
                           int n, void* stream) {
  if (!b || !rgba_dev) return 0;
  return run_rgba(b, rgba_dev, fstride, rstride, n, stream);
}

/* host memory the DMA engines can read directly (page-locked by HIP) */
static int byte_is_pinned(const void* p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();   /* an unregistered pointer reports an error: clear it */
    return 0;
  }
  return at.type == hipMemoryTypeHost;
}

/* the whole range [p, p + n) page-locked (a caller may have hipHostRegister-ed
 * only part of a buffer, or several pieces of it; the SDMA engine must not
 * read pageable pages): walk the registrations that cover it, from each one's
 * start address and size, until the range is covered -- a gap, or a byte HIP
 * does not know, means pageable. Should the runtime not report a range
 * (older runtimes), every 64 MB and the last byte are sampled instead. */
static int host_is_pinned(const void* p, size_t n) {
  const uint8_t* c = (const uint8_t*)p;
  const uint8_t* end = c + (n ? n : 1);
  while (c < end) {
    if (!byte_is_pinned(c)) return 0;
    void* base = NULL;
    size_t size = 0;
    if (hipPointerGetAttribute(&base, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                               (hipDeviceptr_t)(uintptr_t)c) != hipSuccess ||
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                               (hipDeviceptr_t)(uintptr_t)c) != hipSuccess ||
        !base || size == 0 || (const uint8_t*)base > c ||
        (const uint8_t*)base + size <= c) {
      (void)hipGetLastError();
      for (size_t o = (size_t)(c - (const uint8_t*)p); o < n; o += (size_t)64 << 20)
        if (!byte_is_pinned((const uint8_t*)p + o)) return 0;
      return byte_is_pinned(end - 1);
    }
    c = (const uint8_t*)base + size;   /* the next registration, if any, starts here */
  }
  return 1;
}

/* Encode n frames from host memory; with `next` (pinned, same geometry),
 * also start uploading the next batch into the spare buffer while this one
 * encodes: a later call for `next` then finds its frames on the device. */
static int encode_host(WebPGpuBatch* b, const uint8_t* rgba, const uint8_t* next, size_t fstride,
                       int rstride, int n) {
  if (!b || !rgba || n <= 0 || n > b->max_frames || rstride < 4 * b->w) return 0;
  if (n > 1 && fstride < (size_t)rstride * b->h) return 0;
  CHK(hipSetDevice(b->device));
  const size_t need = (size_t)(n - 1) * fstride + (size_t)rstride * b->h;
  int have = 0;   /* this batch's frames already uploaded by the previous call */
  if (b->pf_busy) {
    h2d_sdma_finish(b->pf_sig);
    b->pf_busy = 0;
    if (b->pf_src == rgba && b->pf_need == need && b->pf_fstride == fstride &&
        b->pf_rstride == rstride && b->pf_n == n) {
      uint8_t* t = b->d_rgba;
      const size_t tc = b->d_rgba_cap;
      b->d_rgba = b->d_rgba2;
      b->d_rgba_cap = b->d_rgba2_cap;
      b->d_rgba2 = t;
      b->d_rgba2_cap = tc;
      have = 1;
    }
  }
  if (!have) {
    if (need > b->d_rgba_cap) {
      hipFree(b->d_rgba);
      b->d_rgba = NULL;
      b->d_rgba_cap = 0;
      CHK(hipMalloc((void**)&b->d_rgba, need));
      b->d_rgba_cap = need;
    }
    if (host_is_pinned(rgba, need)) {
      /* page-locked (hipHostMalloc / hipHostRegister): one copy on an SDMA
         engine (host/h2d_sdma.c) -- it runs beside the other engines' kernels,
         where the runtime's copy kernel would wait for CUs a running K3 holds */
      CHK(hipStreamSynchronize(b->stream));   /* (idle between batch calls) */
      if (!h2d_sdma_upload(b->device, b->d_rgba, rgba, need))   /* an SDMA engine, no CU */
        CHK(hipMemcpyAsync(b->d_rgba, rgba, need, hipMemcpyHostToDevice, b->stream));
    } else {
      /* pageable: an async copy of it on our non-blocking stream is not safe
         on this platform (the runtime may read it from the GPU directly), so
         drain the stream and copy synchronously */
      CHK(hipStreamSynchronize(b->stream));
      CHK(hipMemcpy(b->d_rgba, rgba, need, hipMemcpyHostToDevice));
    }
  }
  if (next && host_is_pinned(next, need)) {
    /* the spare buffer was last read by the previous call's kernels, which
       that call drained before returning */
    if (need > b->d_rgba2_cap) {
      hipFree(b->d_rgba2);
      b->d_rgba2 = NULL;
      b->d_rgba2_cap = 0;
      CHK(hipMalloc((void**)&b->d_rgba2, need));
      b->d_rgba2_cap = need;
    }
    if (h2d_sdma_upload_start(b->device, b->d_rgba2, next, need, &b->pf_sig)) {
      b->pf_busy = 1;
      b->pf_src = next;
      b->pf_need = need;
      b->pf_fstride = fstride;
      b->pf_rstride = rstride;
      b->pf_n = n;
    }
  }
  return run_rgba(b, b->d_rgba, fstride, rstride, n, NULL);
fail:
  return 0;
}

int WebPGpuBatchEncodeRGBAHost(WebPGpuBatch* b, const uint8_t* rgba, size_t fstride, int rstride,
                               int n) {
  return encode_host(b, rgba, NULL, fstride, rstride, n);
}

int WebPGpuBatchEncodeRGBAHostPrefetch(WebPGpuBatch* b, const uint8_t* rgba,
                                       const uint8_t* rgba_next, size_t fstride, int rstride,
                                       int n) {
  return encode_host(b, rgba, rgba_next, fstride, rstride, n);
}

size_t WebPGpuBatchOutputSize(const WebPGpuBatch* b, int f) {
  if (!b || f < 0 || f >= b->last_n) return 0;
  return b->l ? vp8l_engine_out_size(b->l, f) : b->out_size[f];
}
const uint8_t* WebPGpuBatchOutput(const WebPGpuBatch* b, int f) {
  if (!b || f < 0 || f >= b->last_n) return NULL;
  if (b->l) return vp8l_engine_output(b->l, f);
  return b->out[f];
}
int WebPGpuBatchStageCycles(const WebPGpuBatch* b, int f, uint64_t cycles[8]) {
  if (!b || b->l || f < 0 || f >= b->last_n || !cycles) return 0;
  for (int i = 0; i < 8; ++i) cycles[i] = b->h_results[f].stamps[i];
  return 1;
}
size_t WebPGpuBatchTokenCount(const WebPGpuBatch* b, int f) {
  return (b && !b->l && f >= 0 && f < b->last_n) ? b->h_results[f].ntokens : 0;
}
int WebPGpuBatchError(const WebPGpuBatch* b, int f) {
  if (!b || f < 0 || f >= b->last_n) return VP8_ENC_ERROR_NULL_PARAMETER;
  return b->l ? vp8l_engine_error(b->l, f) : b->err[f];
}
void WebPGpuBatchTimings(const WebPGpuBatch* b, double t[10]) {
  for (int i = 0; i < 10; ++i) t[i] = b ? b->timings[i] : 0.;
}

int WebPGpuBatchGetYUV(const WebPGpuBatch* b, int f, uint8_t* dst) {
  if (!b || f < 0 || f >= b->max_frames || !dst) return 0;
  const size_t bytes = (size_t)b->w * b->h + 2 * (size_t)b->uvw * b->uvh;
  hipSetDevice(b->device);
  return hipMemcpy(dst, b->d_yuv + (size_t)f * b->yfb, bytes, hipMemcpyDeviceToHost) == hipSuccess;
}

int WebPGpuBatchGetTokens(const WebPGpuBatch* b, int f, uint16_t* dst, size_t max_tokens) {
  if (!b || f < 0 || f >= b->last_n || !dst || !b->host_emit) return 0;
  const size_t n = b->h_results[f].ntokens < max_tokens ? b->h_results[f].ntokens : max_tokens;
  hipSetDevice(b->device);
  return hipMemcpy(dst, b->d_tokens + (size_t)f * b->tok_cap, n * sizeof(uint16_t),
                   hipMemcpyDeviceToHost) == hipSuccess;
}

int WebPGpuBatchGetMBInfo(const WebPGpuBatch* b, int f, uint8_t* dst) {
  if (!b || f < 0 || f >= b->last_n || !dst) return 0;
  memcpy(dst, b->h_mbinfo + (size_t)f * b->nmb * VP8G_MBINFO_BYTES,
         (size_t)b->nmb * VP8G_MBINFO_BYTES);
  return 1;
}

int vp8g_engine_upload_yuv(WebPGpuBatch* b, int f, const uint8_t* y, int ys, const uint8_t* u,
                           const uint8_t* v, int uvs, const uint8_t* a, int as) {
  uint8_t* dst = b->d_yuv + (size_t)f * b->yfb;
  if (hipSetDevice(b->device) != hipSuccess) return 0;
  if (hipMemcpy2D(dst, b->w, y, ys, b->w, b->h, hipMemcpyHostToDevice) != hipSuccess) return 0;
  dst += (size_t)b->w * b->h;
  if (hipMemcpy2D(dst, b->uvw, u, uvs, b->uvw, b->uvh, hipMemcpyHostToDevice) != hipSuccess)
    return 0;
  dst += (size_t)b->uvw * b->uvh;
  if (hipMemcpy2D(dst, b->uvw, v, uvs, b->uvw, b->uvh, hipMemcpyHostToDevice) != hipSuccess)
    return 0;
  b->h_aflags[f] = a != NULL;   /* the caller passes a plane only when it is not opaque */
  if (a && hipMemcpy2D(b->d_aplane + (size_t)f * b->w * b->h, b->w, a, as, b->w, b->h,
                       hipMemcpyHostToDevice) != hipSuccess)
    return 0;
  b->err[f] = VP8_ENC_OK;
  return 1;
}

int vp8g_engine_import(WebPGpuBatch* b, const uint8_t* rgba, int stride, uint8_t* y,
                       uint8_t* u, uint8_t* v, uint8_t* a, int* has_alpha, int sharp,
                       float dither) {
  /* synchronous single-frame RGBA -> YUV through K1 (used by the
   * WebPPictureImport* API); output written to the caller's host planes */
  if (hipSetDevice(b->device) != hipSuccess) return 0;
  b->dither = dither;
  const size_t need = (size_t)stride * b->h;
  if (need > b->d_rgba_cap) {
    hipFree(b->d_rgba);
    b->d_rgba = NULL;
    b->d_rgba_cap = 0;
    if (hipMalloc((void**)&b->d_rgba, need) != hipSuccess) return 0;
    b->d_rgba_cap = need;
  }
  if (hipMemcpy(b->d_rgba, rgba, need, hipMemcpyHostToDevice) != hipSuccess) return 0;
  if (hipMemsetAsync(b->d_aflags, 0, sizeof(uint32_t), b->stream) != hipSuccess) return 0;
  if (!launch_import(b, b->d_rgba, need, stride, 1, sharp && b->w >= 4 && b->h >= 4)) return 0;
  if (hipStreamSynchronize(b->stream) != hipSuccess) return 0;
  uint32_t flag = 0;
  if (hipMemcpy(&flag, b->d_aflags, 4, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  *has_alpha = flag != 0;
  /* K1 writes no alpha plane (the sharp-YUV import extracts its own): the
   * plane of a frame with alpha comes from the RGBA here */
  const int sharp_used = sharp && b->w >= 4 && b->h >= 4;
  if (a && flag && !sharp_used &&
      (!vp8g_launch_extract_alpha(b->d_rgba, need, stride, b->w, b->h, 1, NULL, b->d_aplane,
                                  b->stream) ||
       hipStreamSynchronize(b->stream) != hipSuccess))
    return 0;
  const uint8_t* src = b->d_yuv;
  if (hipMemcpy(y, src, (size_t)b->w * b->h, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  src += (size_t)b->w * b->h;
  if (hipMemcpy(u, src, (size_t)b->uvw * b->uvh, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  src += (size_t)b->uvw * b->uvh;
  if (hipMemcpy(v, src, (size_t)b->uvw * b->uvh, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  if (a && hipMemcpy(a, b->d_aplane, (size_t)b->w * b->h, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return 1;
}
