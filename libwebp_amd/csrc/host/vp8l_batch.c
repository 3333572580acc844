/* Lossless (VP8L) batch engine: device buffers, the L0 analysis and the
 * per-frame entropy-mode decision, the L1 -> L5 kernels, the per-frame header
 * on host threads, the L6/L7 bit writer and the RIFF assembly. One call
 * encodes n same-sized RGBA frames resident in HBM; every .webp lands in one
 * pinned host buffer per engine (the root engine's for the spatial / direct
 * frames, a palette engine's per bundling for the colour-indexed ones). */
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "h2d_sdma.h"
#include "gpu_engine.h"
#include "vp8l_batch.h"
#include "vp8l_host.h"

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

#define CHK(x)                                                         \
  do {                                                                 \
    const hipError_t e_ = (x);                                         \
    if (e_ != hipSuccess) {                                            \
      char loc_[64];                                                   \
      snprintf(loc_, sizeof(loc_), "vp8l_batch.c:%d", __LINE__);       \
      vp8g_set_error(loc_, hipGetErrorString(e_));                     \
      goto fail;                                                       \
    }                                                                  \
  } while (0)

static int sub_sample(int size, int bits) { return (size + (1 << bits) - 1) >> bits; }

void vp8l_engine_free(vp8l_engine* l) {
  if (!l) return;
  for (int i = 0; i < 6; ++i) vp8l_engine_free(l->sub[i]);
  hipFree(l->d_rep); hipHostFree(l->h_rep);
  free(l->route_eng); free(l->route_slot);
  hipFree(l->d_minb); hipFree(l->d_cseg); hipFree(l->d_prov); hipFree(l->d_chist); hipFree(l->d_cbits);
  hipFree(l->d_ehist); hipFree(l->d_scan); hipFree(l->d_fidx); hipFree(l->d_fmode);
  hipFree(l->d_psort); hipFree(l->d_psidx); hipFree(l->d_npal);
  hipHostFree(l->h_ehist); hipHostFree(l->h_scan); hipHostFree(l->h_fidx); hipHostFree(l->h_fmode);
  hipHostFree(l->h_cbits); hipHostFree(l->h_psort); hipHostFree(l->h_psidx); hipHostFree(l->h_npal);
  free(l->h_pal);
  hipFree(l->d_nl[0]); hipFree(l->d_nl[1]); hipFree(l->d_nlapply); hipHostFree(l->h_nlapply);
  hipFree(l->d_tabs); hipFree(l->d_argb); hipFree(l->d_modes); hipFree(l->d_mult);
  hipFree(l->d_aflag); hipFree(l->d_pflag); hipFree(l->d_pexact); hipHostFree(l->h_pexact);
  hipFree(l->d_ops); hipFree(l->d_feat); hipFree(l->d_tl); hipFree(l->d_tn);
  hipFree(l->d_hc); hipFree(l->d_assign); hipFree(l->d_ctab); hipFree(l->d_gtile);
  hipFree(l->d_start); hipFree(l->d_bsum); hipFree(l->d_boff); hipFree(l->d_end); hipFree(l->d_out);
  hipFree(l->d_packed); hipFree(l->d_poff); hipFree(l->d_hpack); hipFree(l->d_hoff);
  hipFree(l->d_hwords);
  hipHostFree(l->h_modes); hipHostFree(l->h_mult); hipHostFree(l->h_aflag); hipHostFree(l->h_hc);
  hipHostFree(l->h_assign); hipHostFree(l->h_ctab); hipHostFree(l->h_gtile);
  hipHostFree(l->h_start); hipHostFree(l->h_end); hipHostFree(l->h_hdr); hipHostFree(l->h_out);
  hipHostFree(l->h_poff); hipHostFree(l->h_hpack); hipHostFree(l->h_hoff); hipHostFree(l->h_hwords);
  free(l->hdr_bytes); free(l->out_off); free(l->out_size); free(l->err);
  hipFree(l->lz.runs); hipFree(l->lz.htab); hipFree(l->lz.chain); hipFree(l->lz.hoff);
  hipFree(l->lz.hlen); hipFree(l->lz.loff); hipFree(l->lz.llen); hipFree(l->lz.costs);
  hipFree(l->lz.costs_row); hipFree(l->lz.est);
  hipFree(l->d_dcodes);
  hipFree(l->d_dpcand); hipFree(l->d_dpcost);
  for (int i = 0; i < 5; ++i)
    if (l->ev[i]) hipEventDestroy(l->ev[i]);
  free(l);
}

static vp8l_engine* engine_alloc(const vp8l_params* p, int max_frames, int method, int root) {
  vp8l_engine* l = (vp8l_engine*)calloc(1, sizeof(*l));
  if (!l) return NULL;
  l->p = *p;
  const int w = p->w, h = p->h;
  l->method = method;
  if (hipGetDevice(&l->device) != hipSuccess) l->device = 0;
  l->max_frames = max_frames;
  l->npix = (size_t)w * h;
  l->ntt = sub_sample(w, l->p.tb) * sub_sample(h, l->p.tb);
  l->nht = sub_sample(w, l->p.hb) * sub_sample(h, l->p.hb);
  l->nblk = (int)((l->npix + VP8L_BLOCK - 1) / VP8L_BLOCK);
  l->hdr_cap = ((size_t)16 * l->ntt + (size_t)8 * l->nht + ((size_t)256 << 10) + 255) & ~(size_t)255;
  l->out_cap = (l->npix * 5 + l->hdr_cap + 255) & ~(size_t)255;
  const size_t N = (size_t)max_frames, np = l->npix;
  for (int i = 0; i < 5; ++i) CHK(hipEventCreate(&l->ev[i]));
  CHK(hipMalloc((void**)&l->d_tabs, VP8L_TAB_WORDS * sizeof(int32_t)));
  CHK(hipMemcpy(l->d_tabs + VP8L_TAB_FSLOG, vp8l_float_tables(), 512 * sizeof(float),
                hipMemcpyHostToDevice));
  CHK(hipMemcpy(l->d_tabs, vp8l_nlogn_table(), 4097 * sizeof(int32_t), hipMemcpyHostToDevice));
  CHK(hipMemcpy(l->d_tabs + 4097, vp8l_flog2_table(), 1024 * sizeof(int32_t),
                hipMemcpyHostToDevice));
  CHK(hipMalloc((void**)&l->d_argb, N * np * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_ops, N * np * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_minb, N * np));
  if (l->p.cache_bits) {
    CHK(hipMalloc((void**)&l->d_prov, N * np * sizeof(uint16_t)));
    CHK(hipMalloc((void**)&l->d_chist, N * VP8L_CHIST * sizeof(uint32_t)));
    CHK(hipMalloc((void**)&l->d_cseg, N * VP8L_CACHE_SEGS * VP8L_CACHE_TAB * 2 * sizeof(uint32_t)));
  }
  CHK(hipMalloc((void**)&l->d_cbits, N));
  CHK(hipMalloc((void**)&l->d_fidx, N * sizeof(int)));
  CHK(hipMalloc((void**)&l->d_fmode, N));
  CHK(hipMalloc((void**)&l->d_nlapply, N));
  CHK(hipHostMalloc((void**)&l->h_nlapply, N, 0));
  CHK(hipHostMalloc((void**)&l->h_fidx, N * sizeof(int), 0));
  CHK(hipHostMalloc((void**)&l->h_fmode, N, 0));
  CHK(hipHostMalloc((void**)&l->h_cbits, N, 0));
  if (root) {
    CHK(hipMalloc((void**)&l->d_ehist, N * VP8L_EHIST * sizeof(uint32_t)));
    CHK(hipMalloc((void**)&l->d_scan, N * VP8L_PAL_STRIDE * sizeof(uint32_t)));
    CHK(hipHostMalloc((void**)&l->h_ehist, N * VP8L_EHIST * sizeof(uint32_t), 0));
    CHK(hipHostMalloc((void**)&l->h_scan, N * VP8L_PAL_STRIDE * sizeof(uint32_t), 0));
    CHK(hipMalloc((void**)&l->d_rep, N * 2 * sizeof(uint32_t)));
    CHK(hipHostMalloc((void**)&l->h_rep, N * 2 * sizeof(uint32_t), 0));
    l->route_eng = (vp8l_engine**)calloc(N, sizeof(*l->route_eng));
    l->route_slot = (int*)calloc(N, sizeof(int));
    if (!l->route_eng || !l->route_slot) goto fail;
  }
  if (l->p.palette || l->p.lz) {   /* the cost-model parse (vp8l_launch_analyze with lz) */
    CHK(hipMalloc((void**)&l->lz.runs, N * np * sizeof(uint16_t)));
    CHK(hipMalloc((void**)&l->lz.htab, N * VP8L_LZ_HASH_SIZE * sizeof(int32_t)));
    CHK(hipMalloc((void**)&l->lz.chain, N * np * sizeof(int32_t)));
    CHK(hipMalloc((void**)&l->lz.hoff, N * np * sizeof(uint32_t)));
    CHK(hipMalloc((void**)&l->lz.hlen, N * np * sizeof(uint16_t)));
    CHK(hipMalloc((void**)&l->lz.loff, N * np * sizeof(uint32_t)));
    CHK(hipMalloc((void**)&l->lz.llen, N * np * sizeof(uint16_t)));
    CHK(hipMalloc((void**)&l->lz.costs, N * VP8L_LZ_NCOST * sizeof(int32_t)));
    CHK(hipMalloc((void**)&l->lz.costs_row, N * VP8L_LZ_NCOST * sizeof(int32_t)));
    CHK(hipMalloc((void**)&l->lz.est, 2 * N * sizeof(unsigned long long)));
    {
      const int nd = vp8l_plane_dcodes(w, NULL);
      uint8_t* tab = (uint8_t*)malloc((size_t)nd);
      if (!tab) goto fail;
      vp8l_plane_dcodes(w, tab);
      const hipError_t e1 = hipMalloc((void**)&l->d_dcodes, (size_t)nd);
      const hipError_t e2 = e1 == hipSuccess ? hipMemcpy(l->d_dcodes, tab, (size_t)nd,
                                                         hipMemcpyHostToDevice) : e1;
      free(tab);
      CHK(e2);
      l->lz.dcodes = l->d_dcodes;
      l->lz.nd = nd;
    }
  }
  if (l->p.palette) {
    CHK(hipMalloc((void**)&l->d_psort, N * VP8L_MAX_PALETTE * sizeof(uint32_t)));
    CHK(hipMalloc((void**)&l->d_psidx, N * VP8L_MAX_PALETTE));
    CHK(hipMalloc((void**)&l->d_npal, N * sizeof(int)));
    CHK(hipHostMalloc((void**)&l->h_psort, N * VP8L_MAX_PALETTE * sizeof(uint32_t), 0));
    CHK(hipHostMalloc((void**)&l->h_psidx, N * VP8L_MAX_PALETTE, 0));
    CHK(hipHostMalloc((void**)&l->h_npal, N * sizeof(int), 0));
    l->h_pal = (uint32_t*)calloc(N * VP8L_MAX_PALETTE, sizeof(uint32_t));
    if (!l->h_pal) goto fail;
  }
  if (!l->p.palette && !l->p.alpha) {   /* the shortest-path parse (frames without a predictor) */
    int32_t cand[VP8L_DP_NC * 4];
    memset(cand, 0, sizeof(cand));
    l->dp_ncand = vp8l_dp_candidates(w, cand);
    CHK(hipMalloc((void**)&l->d_dpcand, sizeof(cand)));
    CHK(hipMemcpy(l->d_dpcand, cand, sizeof(cand), hipMemcpyHostToDevice));
    CHK(hipMalloc((void**)&l->d_dpcost, N * VP8L_DP_NCOST * sizeof(int32_t)));
  }
  CHK(hipMalloc((void**)&l->d_modes, N * l->ntt));
  CHK(hipMalloc((void**)&l->d_mult, N * l->ntt * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_aflag, N * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_pflag, N * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_pexact, N));
  CHK(hipHostMalloc((void**)&l->h_pexact, N, 0));
  CHK(hipMalloc((void**)&l->d_feat, N * l->nht * sizeof(int64_t)));
  CHK(hipMalloc((void**)&l->d_tl, N * l->nht * VP8L_TILE_CAP(l->p.hb) * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_tn, N * l->nht * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_hc, N * VP8L_KMAX * VP8L_NS * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_assign, N * l->nht));
  CHK(hipMalloc((void**)&l->d_ctab, N * VP8L_KMAX * VP8L_NS * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_gtile, N * l->nht));
  CHK(hipMalloc((void**)&l->d_start, N * sizeof(uint64_t)));
  CHK(hipMalloc((void**)&l->d_end, N * sizeof(uint64_t)));
  CHK(hipMalloc((void**)&l->d_bsum, N * l->nblk * sizeof(uint32_t)));
  CHK(hipMalloc((void**)&l->d_boff, N * l->nblk * sizeof(uint64_t)));
  CHK(hipMalloc((void**)&l->d_out, N * l->out_cap));
  CHK(hipHostMalloc((void**)&l->h_modes, N * l->ntt, 0));
  CHK(hipHostMalloc((void**)&l->h_mult, N * l->ntt * sizeof(uint32_t), 0));
  CHK(hipHostMalloc((void**)&l->h_aflag, N * sizeof(uint32_t), 0));
  CHK(hipHostMalloc((void**)&l->h_hc, N * VP8L_KMAX * VP8L_NS * sizeof(uint32_t), 0));
  CHK(hipHostMalloc((void**)&l->h_assign, N * l->nht, 0));
  CHK(hipHostMalloc((void**)&l->h_ctab, N * VP8L_KMAX * VP8L_NS * sizeof(uint32_t), 0));
  CHK(hipHostMalloc((void**)&l->h_gtile, N * l->nht, 0));
  CHK(hipHostMalloc((void**)&l->h_start, N * sizeof(uint64_t), 0));
  CHK(hipHostMalloc((void**)&l->h_end, N * sizeof(uint64_t), 0));
  CHK(hipHostMalloc((void**)&l->h_hdr, N * l->hdr_cap, 0));
  CHK(hipMalloc((void**)&l->d_poff, (N + 1) * sizeof(uint64_t)));
  CHK(hipMalloc((void**)&l->d_hoff, (N + 1) * sizeof(uint64_t)));
  CHK(hipMalloc((void**)&l->d_hwords, N * sizeof(uint32_t)));
  CHK(hipHostMalloc((void**)&l->h_poff, (N + 1) * sizeof(uint64_t), 0));
  CHK(hipHostMalloc((void**)&l->h_hoff, (N + 1) * sizeof(uint64_t), 0));
  CHK(hipHostMalloc((void**)&l->h_hwords, N * sizeof(uint32_t), 0));
  l->hdr_bytes = (size_t*)calloc(N, sizeof(size_t));
  l->out_off = (size_t*)calloc(N + 1, sizeof(size_t));
  l->out_size = (size_t*)calloc(N, sizeof(size_t));
  l->err = (int*)calloc(N, sizeof(int));
  if (!l->hdr_bytes || !l->out_off || !l->out_size || !l->err) goto fail;
  return l;
fail:
  vp8l_engine_free(l);
  return NULL;
}

vp8l_engine* vp8l_engine_new(int w, int h, int max_frames, int method, int alpha) {
  vp8l_params p;
  vp8l_setup_params(&p, w, h, max_frames, method, alpha);
  return engine_alloc(&p, max_frames, method, 1);
}

void vp8l_engine_set_near_lossless(vp8l_engine* l, int quality) {
  const int bits = quality >= 100 ? 0 : 5 - quality / 20;   /* VP8LNearLosslessBits */
  /* VP8ApplyNearLossless leaves pictures under 64x64 or 3 rows as they are;
   * the predictor's quantisation (spatial modes) has no such exception */
  l->nl_bits = ((l->p.w < 64 && l->p.h < 64) || l->p.h < 3 || l->p.alpha) ? 0 : bits;
  l->p.nlq_bits = l->p.alpha ? 0 : bits;
}

void vp8l_engine_set_exact(vp8l_engine* l, int exact) {
  if (!l->p.alpha) l->p.exact = exact != 0;
}

static void route(const vp8l_engine* l, int f, const vp8l_engine** e, int* s) {
  if (l->route_eng && l->route_eng[f]) { *e = l->route_eng[f]; *s = l->route_slot[f]; }
  else { *e = l; *s = f; }
}

/* ---- per-frame headers on host threads ---- */

typedef struct {
  vp8l_engine* l;
  int n;
  atomic_int next;
} HdrJob;

static void frame_header(vp8l_engine* l, int f) {
  vp8l_bw bw;
  const vp8l_params* p = &l->p;
  vp8l_bw_init(&bw, 1 << 16);
  const int emode = p->palette ? VP8L_MODE_PALETTE : l->h_fmode[f];
  const int ok = vp8l_build_header(p, l->h_aflag[f] != 0, emode, l->h_cbits[f],
                                   p->palette ? l->h_pal + (size_t)f * VP8L_MAX_PALETTE : NULL,
                                   p->palette ? l->h_npal[f] : 0,
                                   l->h_modes + (size_t)f * l->ntt,
                                   l->h_mult + (size_t)f * l->ntt,
                                   l->h_hc + (size_t)f * VP8L_KMAX * VP8L_NS,
                                   l->h_assign + (size_t)f * l->nht, &bw,
                                   l->h_ctab + (size_t)f * VP8L_KMAX * VP8L_NS,
                                   l->h_gtile + (size_t)f * l->nht);
  l->h_start[f] = bw.nbits;
  const size_t nb = vp8l_bw_finish(&bw);
  if (!ok || bw.oom) {
    l->err[f] = VP8_ENC_ERROR_OUT_OF_MEMORY;
  } else if (nb > l->hdr_cap) {
    l->err[f] = VP8_ENC_ERROR_BITSTREAM_OUT_OF_MEMORY;
  } else {
    uint8_t* d = l->h_hdr + (size_t)f * l->hdr_cap;
    memcpy(d, bw.buf, nb);
    memset(d + nb, 0, ((nb + 3) & ~(size_t)3) - nb);
    l->hdr_bytes[f] = nb;
  }
  if (l->err[f]) { l->h_start[f] = 0; l->hdr_bytes[f] = 0; }
  vp8l_bw_free(&bw);
}

static void hdr_item(void* arg, int f) { frame_header(((HdrJob*)arg)->l, f); }

/* the frames' headers on the rank's thread pool (host_cpus.c), at most
 * threads - 1 pool threads at once, the caller taking frames too */
static void run_headers(vp8l_engine* l, int n, int threads) {
  HdrJob job;
  job.l = l; job.n = n;
  vp8g_job pj;
  vp8g_job_submit(l->device, &pj, hdr_item, &job, n, threads - 1);
  vp8g_job_join(&pj);
}

/* ---- pipeline ---- */

int vp8l_engine_run(struct WebPGpuBatch* b, const uint8_t* rgba, size_t fstride, int rstride, int n) {
  const int ok = vp8l_engine_encode(b->l, b->stream, b->threads, rgba, fstride, rstride, n,
                                    b->timings);
  if (ok) b->last_n = n;
  return ok;
}

/* One engine's stages over its n slots. identity: slot f = frame f (the
 * ALPH engine); else h_fidx / h_fmode (and the palettes) were filled. */
static int pipeline(vp8l_engine* l, hipStream_t st, int threads, const uint8_t* rgba,
                    size_t fstride, int rstride, int n, int identity, const uint32_t* ehist,
                    double timings[10]) {
  const size_t N = (size_t)n;
  double t0 = now_us(), t1, t2, t3, t4, t5;
  vp8l_params p = l->p;
  p.n = n;
  const int* fidx_in = identity ? NULL : l->d_fidx;
  for (int f = 0; f < n; ++f) l->err[f] = VP8_ENC_OK;
  CHK(hipMemsetAsync(l->d_aflag, 0, N * sizeof(uint32_t), st));
  int any_exact = 0;
  if (!identity) {
    CHK(hipMemcpyAsync(l->d_fidx, l->h_fidx, N * sizeof(int), hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(l->d_fmode, l->h_fmode, N, hipMemcpyHostToDevice, st));
    for (int f = 0; f < n; ++f) any_exact |= l->h_pexact[f];
    CHK(hipMemcpyAsync(l->d_pexact, l->h_pexact, N, hipMemcpyHostToDevice, st));
  }
  if (p.palette) {
    CHK(hipMemcpyAsync(l->d_psort, l->h_psort, N * VP8L_MAX_PALETTE * sizeof(uint32_t),
                       hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(l->d_psidx, l->h_psidx, N * VP8L_MAX_PALETTE, hipMemcpyHostToDevice, st));
    CHK(hipMemcpyAsync(l->d_npal, l->h_npal, N * sizeof(int), hipMemcpyHostToDevice, st));
  }
  int nl_any = 0;   /* VP8ApplyNearLossless: direct / subtract-green frames only
                       (vp8l_enc.c:1537-1538; the spatial ones quantise in L1a) */
  if (l->nl_bits && !p.palette && !identity)
    for (int f = 0; f < n; ++f) {
      l->h_nlapply[f] = !(l->h_fmode[f] & VP8L_MODE_SPATIAL);
      nl_any |= l->h_nlapply[f];
    }
  if (nl_any) {   /* near-lossless passes into slot-indexed buffers */
    const size_t fb = l->npix * 4;
    for (int i = 0; i < 2; ++i)
      if (!l->d_nl[i]) CHK(hipMalloc((void**)&l->d_nl[i], (size_t)l->max_frames * fb));
    CHK(hipMemcpyAsync(l->d_nlapply, l->h_nlapply, N, hipMemcpyHostToDevice, st));
    const uint8_t* nl = NULL;
    if (!vp8l_launch_near_lossless(rgba, fstride, rstride, l->d_fidx, l->d_nlapply, p.w, p.h, n,
                                   l->nl_bits, l->d_nl[0], l->d_nl[1], &nl, st))
      goto fail;
    rgba = nl; fstride = fb; rstride = p.w * 4;
    fidx_in = NULL;
  }
  CHK(hipEventRecord(l->ev[0], st));
  if (p.palette) {
    if (!vp8l_launch_palette_apply(rgba, fstride, rstride, &p, fidx_in,
                                   l->d_psort, l->d_psidx, l->d_npal, l->d_argb, l->d_aflag, st))
      goto fail;
  } else {
    int sg_mask = 0;
    for (int f = 0; f < n; ++f) sg_mask |= identity ? 1 : 1 << ((l->h_fmode[f] >> 1) & 1);
    /* the transform search scores against the input frame's L0 histograms */
    if (!vp8l_launch_transform(rgba, fstride, rstride, &p, fidx_in, identity ? NULL : l->d_fidx,
                               identity ? NULL : l->d_fmode, ehist, l->d_tabs, sg_mask,
                               l->d_argb, l->d_modes, identity ? NULL : l->d_pexact, any_exact,
                               l->d_pflag, l->d_mult, l->d_aflag, st))
      goto fail;
  }
  CHK(hipEventRecord(l->ev[1], st));
  vp8l_dp dp = {NULL, NULL, 0, NULL};
  if (VP8L_DP_ENABLED && !identity && l->d_dpcand && !p.low_effort) {   /* model: dp_parse's frames */
    dp.fmode = l->d_fmode;
    dp.cand = l->d_dpcand;
    dp.ncand = l->dp_ncand;
    dp.costs = l->d_dpcost;
  }
  if (!vp8l_launch_analyze(l->d_argb, &p, l->d_tabs, l->d_minb, l->d_cseg, l->d_prov, l->d_chist,
                           l->d_cbits, l->d_ops, l->d_feat, l->d_tl, l->d_tn, l->d_hc,
                           l->d_assign, (p.palette || p.lz) ? &l->lz : NULL, &dp, st))
    goto fail;
  CHK(hipEventRecord(l->ev[2], st));
  {   /* debugging aid: LIBWEBP_AMD_VP8L_DUMP=<prefix> writes slot 0's
       * coded image, cache sizes, parse ops and cache bits */
    const char* dump = getenv("LIBWEBP_AMD_VP8L_DUMP");
    if (dump) {
      fprintf(stderr, "vp8l dump: n %d palette %d tb %d hb %d exact %d nlq_bits %d low_effort %d "
              "nl_bits %d\n", n, p.palette, p.tb, p.hb, p.exact, p.nlq_bits, p.low_effort,
              l->nl_bits);
      const size_t np = l->npix;
      uint8_t* buf = (uint8_t*)malloc(np * 4 + 1);
      char path[512];
      const struct { const void* d; size_t bytes; const char* tag; } parts[] = {
          {l->d_argb, np * 4, "argb"}, {l->d_ops, np * 4, "ops"}, {l->d_cbits, 1, "cbits"},
          {l->d_modes, (size_t)l->ntt, "modes"}, {l->d_mult, (size_t)l->ntt * 4, "mult"},
          {l->d_pflag, 4, "pflag"}};
      for (int i = 0; buf && i < 6; ++i) {
        if (p.palette && i >= 3) break;
        CHK(hipStreamSynchronize(st));
        CHK(hipMemcpy(buf, parts[i].d, parts[i].bytes, hipMemcpyDeviceToHost));
        snprintf(path, sizeof(path), "%s.%s", dump, parts[i].tag);
        FILE* fp = fopen(path, "wb");
        if (fp) { fwrite(buf, 1, parts[i].bytes, fp); fclose(fp); }
      }
      free(buf);
    }
  }
  if (!p.palette) {
    CHK(hipMemcpyAsync(l->h_modes, l->d_modes, N * l->ntt, hipMemcpyDeviceToHost, st));
    CHK(hipMemcpyAsync(l->h_mult, l->d_mult, N * l->ntt * sizeof(uint32_t),
                       hipMemcpyDeviceToHost, st));
  }
  CHK(hipMemcpyAsync(l->h_aflag, l->d_aflag, N * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  CHK(hipMemcpyAsync(l->h_cbits, l->d_cbits, N, hipMemcpyDeviceToHost, st));
  CHK(hipMemcpyAsync(l->h_hc, l->d_hc, N * VP8L_KMAX * VP8L_NS * sizeof(uint32_t),
                     hipMemcpyDeviceToHost, st));
  CHK(hipMemcpyAsync(l->h_assign, l->d_assign, N * l->nht, hipMemcpyDeviceToHost, st));
  /* the output slabs must start zeroed (the bit writer ORs its edge words) */
  CHK(hipMemsetAsync(l->d_out, 0, N * l->out_cap, st));
  CHK(hipStreamSynchronize(st));
  t1 = now_us();
  run_headers(l, n, threads);
  t2 = now_us();
  /* headers back to back (4-byte aligned), one upload, scattered on device */
  l->h_hoff[0] = 0;
  for (int f = 0; f < n; ++f) {
    l->h_hwords[f] = (uint32_t)((l->hdr_bytes[f] + 3) >> 2);
    l->h_hoff[f + 1] = l->h_hoff[f] + 4 * (uint64_t)l->h_hwords[f];
  }
  if (l->h_hoff[n] > l->h_hpack_cap) {
    hipHostFree(l->h_hpack); hipFree(l->d_hpack);
    l->h_hpack = NULL; l->d_hpack = NULL;
    l->h_hpack_cap = l->d_hpack_cap = 0;
    const size_t cap = l->h_hoff[n] + l->h_hoff[n] / 4 + 4096;
    CHK(hipHostMalloc((void**)&l->h_hpack, cap, 0));
    l->h_hpack_cap = cap;
    CHK(hipMalloc((void**)&l->d_hpack, cap));
    l->d_hpack_cap = cap;
  }
  for (int f = 0; f < n; ++f)
    memcpy(l->h_hpack + l->h_hoff[f], l->h_hdr + (size_t)f * l->hdr_cap, 4 * (size_t)l->h_hwords[f]);
  if (l->h_hoff[n])
    CHK(hipMemcpyAsync(l->d_hpack, l->h_hpack, l->h_hoff[n], hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(l->d_hoff, l->h_hoff, N * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(l->d_hwords, l->h_hwords, N * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  if (!vp8l_launch_put_headers(l->d_hpack, l->d_hoff, l->d_hwords, n, l->d_out, l->out_cap, st))
    goto fail;
  CHK(hipMemcpyAsync(l->d_ctab, l->h_ctab, N * VP8L_KMAX * VP8L_NS * sizeof(uint32_t),
                     hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(l->d_gtile, l->h_gtile, N * l->nht, hipMemcpyHostToDevice, st));
  CHK(hipMemcpyAsync(l->d_start, l->h_start, N * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  CHK(hipEventRecord(l->ev[3], st));
  if (!vp8l_launch_write(l->d_argb, l->d_ops, &p, l->d_cbits, l->d_ctab, l->d_gtile, l->d_start,
                         l->d_bsum, l->d_boff, l->d_end, l->d_out, l->out_cap, st))
    goto fail;
  CHK(hipEventRecord(l->ev[4], st));
  CHK(hipMemcpyAsync(l->h_end, l->d_end, N * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  CHK(hipStreamSynchronize(st));
  t3 = now_us();
  /* packed pinned output: per frame 20-byte RIFF/VP8L header, payload, pad */
  l->out_off[0] = 0;
  for (int f = 0; f < n; ++f) {
    size_t sz = 0;
    if (!l->err[f]) {
      const size_t bytes = (size_t)((l->h_end[f] + 7) >> 3);
      if (bytes > l->out_cap) l->err[f] = VP8_ENC_ERROR_BITSTREAM_OUT_OF_MEMORY;
      else sz = 20 + bytes + (bytes & 1);   /* ALPH mode: the 20-byte slot stays unused */
    }
    l->out_size[f] = sz;
    l->out_off[f + 1] = l->out_off[f] + ((sz + 15) & ~(size_t)15);
  }
  if (l->out_off[n] + 16 > l->h_out_cap) {
    hipHostFree(l->h_out); hipFree(l->d_packed);
    l->h_out = NULL; l->d_packed = NULL;
    l->h_out_cap = l->d_packed_cap = 0;
    const size_t cap = l->out_off[n] + l->out_off[n] / 4 + 4096;
    CHK(hipHostMalloc((void**)&l->h_out, cap, 0));
    l->h_out_cap = cap;
    CHK(hipMalloc((void**)&l->d_packed, cap));
    l->d_packed_cap = cap;
  }
  /* one gather kernel + one device-to-host copy of every frame */
  for (int f = 0; f <= n; ++f) l->h_poff[f] = l->out_off[f];
  CHK(hipMemcpyAsync(l->d_poff, l->h_poff, (N + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  if (!vp8l_launch_pack(l->d_out, l->out_cap, l->d_poff, l->d_end, n, l->d_packed, st)) goto fail;
  {
    const size_t down = l->out_off[n] + 16 <= l->d_packed_cap ? l->out_off[n] + 16 : l->out_off[n];
    CHK(hipStreamSynchronize(st));   /* the bytes come back on a copy engine (h2d_sdma.c) */
    if (!d2h_sdma_download(l->device, l->h_out, l->d_packed, down)) {
      CHK(hipMemcpyAsync(l->h_out, l->d_packed, down, hipMemcpyDeviceToHost, st));
      CHK(hipStreamSynchronize(st));
    }
  }
  t4 = now_us();
  for (int f = 0; f < n; ++f) {
    if (!l->out_size[f]) continue;
    uint8_t* o = l->h_out + l->out_off[f];
    const size_t bytes = (size_t)((l->h_end[f] + 7) >> 3);
    if (l->p.alpha) {   /* bare VP8L stream for an ALPH chunk */
      l->out_size[f] = bytes;
      continue;
    }
    vp8l_riff_header(o, bytes);
    if (bytes & 1) o[20 + bytes] = 0;
  }
  t5 = now_us();
  {
    float k_ms = 0.f, a_ms = 0.f, w_ms = 0.f;
    CHK(hipEventElapsedTime(&k_ms, l->ev[0], l->ev[1]));
    CHK(hipEventElapsedTime(&a_ms, l->ev[1], l->ev[2]));
    CHK(hipEventElapsedTime(&w_ms, l->ev[3], l->ev[4]));
    timings[0] += t1 - t0;   /* transform + analysis kernels + side copies (wall) */
    timings[1] += t2 - t1;   /* host headers */
    timings[2] += t3 - t2;   /* header upload + bit writer (wall) */
    timings[3] += t4 - t3;   /* output copies */
    timings[4] += t5 - t4;   /* RIFF */
    timings[6] += 1e3 * a_ms;   /* cache + parse + tiles + clustering */
    timings[7] += 1e3 * k_ms;   /* transform */
    timings[8] += 1e3 * w_ms;   /* bit writer */
  }
  return 1;
fail:
  return 0;
}

static int xbits_of(int npal) { return npal <= 2 ? 3 : npal <= 4 ? 2 : npal <= 16 ? 1 : 0; }

static int u32_less(const void* a, const void* b) {
  const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return x < y ? -1 : x > y;
}

/* The root engine's call: L0 analysis of every frame, the entropy mode of
 * each (AnalyzeEntropy restated, host/vp8l_host.c), then one pipeline per
 * engine with its slots. */
int vp8l_engine_encode(vp8l_engine* l, void* stream, int threads, const uint8_t* rgba,
                       size_t fstride, int rstride, int n, double timings[10]) {
  hipStream_t st = (hipStream_t)stream;
  const size_t N = (size_t)n;
  for (int i = 0; i < 10; ++i) timings[i] = 0.;
  const double t0 = now_us();
  CHK(hipMemsetAsync(l->d_ehist, 0, N * VP8L_EHIST * sizeof(uint32_t), st));
  if (!vp8l_launch_scan(rgba, fstride, rstride, l->p.w, l->p.h, n, l->p.alpha, l->d_ehist,
                        l->d_scan, st))
    goto fail;
  CHK(hipMemcpyAsync(l->h_ehist, l->d_ehist, N * VP8L_EHIST * sizeof(uint32_t),
                     hipMemcpyDeviceToHost, st));
  CHK(hipMemcpyAsync(l->h_scan, l->d_scan, N * VP8L_PAL_STRIDE * sizeof(uint32_t),
                     hipMemcpyDeviceToHost, st));
  /* repeat-heavy frames (oracle/vp8l_model.py: repeat_heavy) take the hash
     chain; not for ALPH planes nor method 0 */
  const int rep_on = !l->p.alpha && !l->p.low_effort && l->p.w >= 8;
  if (rep_on) {
    if (!vp8l_launch_repeat(rgba, fstride, rstride, l->p.w, l->p.h, n,
                            vp8l_repeat_ystep(l->p.w, l->p.h), l->d_rep, st))
      goto fail;
    CHK(hipMemcpyAsync(l->h_rep, l->d_rep, N * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  }
  CHK(hipStreamSynchronize(st));
  {
    /* [0..3] palette engines by xbits, [4] root, [5] sub[4]: non-palette
       frames whose colours fit a palette take the palette histogram bits */
    int cnt[7] = {0, 0, 0, 0, 0, 0, 0};   /* [6] sub[5] */
    const int ntt_pal = sub_sample(l->p.w, vp8l_transform_bits(l->method,
                                   vp8l_histo_bits_palette(l->method, l->p.w, l->p.h)));
    const int ntiles_pal = ntt_pal * sub_sample(l->p.h, vp8l_transform_bits(l->method,
                                   vp8l_histo_bits_palette(l->method, l->p.w, l->p.h)));
    uint8_t* mode = (uint8_t*)malloc(N);
    if (!mode) goto fail;
    for (int f = 0; f < n; ++f) {
      const uint32_t* sc = l->h_scan + (size_t)f * VP8L_PAL_STRIDE;
      const int npal = sc[0] <= VP8L_MAX_PALETTE ? (int)sc[0] : 0;
      const int ntiles = npal ? ntiles_pal : l->ntt;
      /* method 0 skips AnalyzeEntropy: palette or spatial + subtract green (vp8l_enc.c:302-308) */
      mode[f] = l->p.low_effort ? (uint8_t)(npal ? VP8L_MODE_PALETTE : VP8L_MODE_SPATIAL_SUBGREEN)
                                : (uint8_t)vp8l_entropy_choice(l->h_ehist + (size_t)f * VP8L_EHIST,
                                                               npal, ntiles);
      if (mode[f] == VP8L_MODE_PALETTE) cnt[xbits_of(npal)]++;
      else if (!npal && rep_on && vp8l_repeat_heavy(l->h_rep + 2 * (size_t)f)) cnt[6]++;
      else cnt[npal ? 5 : 4]++;
    }
    if (cnt[5] && !(l->sub[4] && l->sub[4]->max_frames >= cnt[5])) {
      vp8l_engine_free(l->sub[4]);
      vp8l_params pp;
      vp8l_setup_params_palette_hb(&pp, l->p.w, l->p.h, cnt[5], l->method, l->p.alpha);
      l->sub[4] = engine_alloc(&pp, cnt[5], l->method, 0);
      if (!l->sub[4]) { free(mode); goto fail; }
    }
    if (cnt[6] && !(l->sub[5] && l->sub[5]->max_frames >= cnt[6])) {
      vp8l_engine_free(l->sub[5]);
      vp8l_params pp = l->p;
      pp.lz = 1;
      l->sub[5] = engine_alloc(&pp, cnt[6], l->method, 0);
      if (!l->sub[5]) { free(mode); goto fail; }
    }
    if (l->sub[5]) {
      l->sub[5]->nl_bits = l->nl_bits;
      l->sub[5]->p.nlq_bits = l->p.nlq_bits;
      l->sub[5]->p.exact = l->p.exact;
      l->sub[5]->p.low_effort = l->p.low_effort;
    }
    if (l->sub[4]) {   /* the root's per-call settings */
      l->sub[4]->nl_bits = l->nl_bits;
      l->sub[4]->p.nlq_bits = l->p.nlq_bits;
      l->sub[4]->p.exact = l->p.exact;
      l->sub[4]->p.low_effort = l->p.low_effort;
    }
    for (int xb = 0; xb < 4; ++xb) {
      if (!cnt[xb] || (l->sub[xb] && l->sub[xb]->max_frames >= cnt[xb])) continue;
      vp8l_engine_free(l->sub[xb]);
      vp8l_params pp;
      vp8l_setup_palette_params(&pp, l->p.w, l->p.h, cnt[xb], l->method, xb, l->p.alpha);
      l->sub[xb] = engine_alloc(&pp, cnt[xb], l->method, 0);
      if (!l->sub[xb]) { free(mode); goto fail; }
    }
    int used[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int f = 0; f < n; ++f) {
      const uint32_t* sc = l->h_scan + (size_t)f * VP8L_PAL_STRIDE;
      if (mode[f] != VP8L_MODE_PALETTE) {
        const int lzf = sc[0] > VP8L_MAX_PALETTE && rep_on &&
                        vp8l_repeat_heavy(l->h_rep + 2 * (size_t)f);
        vp8l_engine* e = lzf ? l->sub[5] : sc[0] <= VP8L_MAX_PALETTE ? l->sub[4] : l;
        const int s = used[lzf ? 6 : e == l ? 4 : 5]++;
        e->h_fidx[s] = f;
        e->h_fmode[s] = mode[f];
        /* the reference's own predictor choice where GetResidual updates the
           picture (model: needs_exact_predictor): near-lossless, or -- without
           exact -- any transparent pixel (predictor_enc.c:273-288), counted by
           L0 over every pixel */
        e->h_pexact[s] = !l->p.exact && (l->p.nlq_bits > 0 ||
                                         l->h_ehist[(size_t)f * VP8L_EHIST + VP8L_EH_TRANSP] > 0);
        l->route_eng[f] = e;
        l->route_slot[f] = s;
        continue;
      }
      const int npal = (int)sc[0], xb = xbits_of(npal);
      vp8l_engine* e = l->sub[xb];
      const int s = used[xb]++;
      uint32_t* pal = e->h_pal + (size_t)s * VP8L_MAX_PALETTE;
      memcpy(pal, sc + 1, (size_t)npal * sizeof(uint32_t));
      vp8l_palette_order(pal, npal);
      uint32_t* srt = e->h_psort + (size_t)s * VP8L_MAX_PALETTE;
      memcpy(srt, pal, (size_t)npal * sizeof(uint32_t));
      qsort(srt, (size_t)npal, sizeof(uint32_t), u32_less);
      for (int i = 0; i < npal; ++i) {   /* stored index of each sorted colour */
        int lo = 0, hi = npal;
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (srt[mid] <= pal[i]) lo = mid; else hi = mid;
        }
        e->h_psidx[(size_t)s * VP8L_MAX_PALETTE + lo] = (uint8_t)i;
      }
      e->h_npal[s] = npal;
      e->h_fidx[s] = f;
      e->h_fmode[s] = VP8L_MODE_PALETTE;
      l->route_eng[f] = e;
      l->route_slot[f] = s;
    }
    free(mode);
    timings[9] = now_us() - t0;   /* L0 analysis + decision */
    if (used[4] && !pipeline(l, st, threads, rgba, fstride, rstride, used[4], 0, l->d_ehist,
                             timings))
      goto fail;
    if (used[5] && !pipeline(l->sub[4], st, threads, rgba, fstride, rstride, used[5], 0,
                             l->d_ehist, timings))
      goto fail;
    if (used[6] && !pipeline(l->sub[5], st, threads, rgba, fstride, rstride, used[6], 0,
                             l->d_ehist, timings))
      goto fail;
    for (int xb = 0; xb < 4; ++xb)
      if (used[xb] &&
          !pipeline(l->sub[xb], st, threads, rgba, fstride, rstride, used[xb], 0, l->d_ehist,
                    timings))
        goto fail;
  }
  return 1;
fail:
  return 0;
}

const uint8_t* vp8l_engine_output(const vp8l_engine* l, int f) {
  const vp8l_engine* e; int s;
  route(l, f, &e, &s);
  if (!e->out_size[s]) return NULL;
  return e->h_out + e->out_off[s] + (e->p.alpha ? 20 : 0);
}

size_t vp8l_engine_out_size(const vp8l_engine* l, int f) {
  const vp8l_engine* e; int s;
  route(l, f, &e, &s);
  return e->out_size[s];
}

int vp8l_engine_error(const vp8l_engine* l, int f) {
  const vp8l_engine* e; int s;
  route(l, f, &e, &s);
  return e->err[s];
}

void vp8l_engine_frame_info(const vp8l_engine* l, int f, vp8l_frame_info* info) {
  const vp8l_engine* e; int s;
  route(l, f, &e, &s);
  memset(info, 0, sizeof(*info));
  const int mode = e->p.palette ? VP8L_MODE_PALETTE : e->h_fmode[s];
  /* transforms used (vp8l_enc.c:1628-1632): 1 predictor, 2 cross colour,
   * 4 subtract green, 8 palette */
  info->features = mode == VP8L_MODE_PALETTE ? 8 :
                   ((mode & VP8L_MODE_SPATIAL) ? 3 : 0) | ((mode & VP8L_MODE_SUBGREEN) ? 4 : 0);
  info->histogram_bits = e->p.hb;
  info->transform_bits = e->p.palette ? l->p.tb : e->p.tb;
  info->cache_bits = e->h_cbits[s];
  info->palette_size = e->p.palette ? e->h_npal[s] : 0;
  info->hdr_bytes = (int)((e->h_start[s] + 7) >> 3);
  info->data_bytes = (int)((e->h_end[s] - e->h_start[s] + 7) >> 3);
}
