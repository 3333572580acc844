/* The libwebp encoder C ABI (include/webp/encode.h) on top of the GPU
 * engine. Behaviour follows the reference API functions cited per item. */
#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "gpu_engine.h"
#include "vp8_host.h"
#include "webp/encode.h"
#include "webp/encode_gpu.h"
#include "picture_internal.h"

#define set_error vp8h_pic_error

/* ---- single-picture GPU engines: a process-wide pool ----
 * The reference is re-entrant for distinct pictures (all state lives in the
 * per-call VP8Encoder, webp_enc.c:330-410). Here each call takes an idle
 * engine of its picture's size and kind from the pool (creating one when none
 * is idle), runs on that engine's own HIP stream without any process-wide
 * lock, and hands it back: concurrent callers encode in parallel on the GPU,
 * and engines of other sizes stay cached instead of being torn down. */
#define POOL_SLOTS 32

typedef struct {
  WebPGpuBatch* e;   /* NULL while being created */
  int used;          /* slot taken (engine present or being created) */
  int busy;          /* a call is using it */
  int w, h, lossless, method;
  uint64_t stamp;    /* last release, for LRU eviction */
} PoolSlot;

static pthread_mutex_t g_pool_lock = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_pool_cv = PTHREAD_COND_INITIALIZER;
static PoolSlot g_pool[POOL_SLOTS];
static uint64_t g_pool_clock = 0;

/* lossless engines are specific to the method (VP8L search effort); lossy
 * engines take the call's config at every run */
static int pool_match(const PoolSlot* s, int w, int h, int lossless, int method) {
  return s->used && s->w == w && s->h == h && s->lossless == lossless &&
         (!lossless || s->method == method);
}

static WebPGpuBatch* pool_get(const WebPConfig* cfg, int w, int h, int lossless) {
  if (WebPGpuDeviceCount() <= 0) return NULL;
  pthread_mutex_lock(&g_pool_lock);
  for (;;) {
    int idle = -1, empty = -1, lru = -1;
    for (int i = 0; i < POOL_SLOTS; ++i) {
      PoolSlot* s = &g_pool[i];
      if (!s->used) {
        if (empty < 0) empty = i;
      } else if (!s->busy && s->e != NULL) {
        if (pool_match(s, w, h, lossless, cfg->method)) { idle = i; break; }
        if (lru < 0 || s->stamp < g_pool[lru].stamp) lru = i;
      }
    }
    if (idle >= 0) {
      PoolSlot* s = &g_pool[idle];
      s->busy = 1;
      pthread_mutex_unlock(&g_pool_lock);
      if (!lossless) s->e->cfg = *cfg;
      return s->e;
    }
    int slot = empty;
    WebPGpuBatch* evict = NULL;
    if (slot < 0 && lru >= 0) {   /* full: replace the least recently used idle engine */
      slot = lru;
      evict = g_pool[lru].e;
    }
    if (slot >= 0) {
      PoolSlot* s = &g_pool[slot];
      s->used = 1; s->busy = 1; s->e = NULL;
      s->w = w; s->h = h; s->lossless = lossless; s->method = cfg->method;
      pthread_mutex_unlock(&g_pool_lock);
      if (evict) WebPGpuBatchDelete(evict);
      WebPGpuBatch* e = WebPGpuBatchNew(0, w, h, 1, cfg, 1);
      pthread_mutex_lock(&g_pool_lock);
      if (e == NULL) {
        s->used = 0; s->busy = 0;
        pthread_cond_broadcast(&g_pool_cv);
        pthread_mutex_unlock(&g_pool_lock);
        return NULL;
      }
      s->e = e;
      pthread_mutex_unlock(&g_pool_lock);
      return e;
    }
    pthread_cond_wait(&g_pool_cv, &g_pool_lock);   /* every slot busy */
  }
}

static void pool_put(WebPGpuBatch* e) {
  if (e == NULL) return;
  pthread_mutex_lock(&g_pool_lock);
  for (int i = 0; i < POOL_SLOTS; ++i)
    if (g_pool[i].e == e) {
      g_pool[i].busy = 0;
      g_pool[i].stamp = ++g_pool_clock;
      break;
    }
  pthread_cond_broadcast(&g_pool_cv);
  pthread_mutex_unlock(&g_pool_lock);
}

/* ---- import (picture_csp_enc.c:474-619, 732-844) ---- */

static int import_packed_d(WebPPicture* pic, const uint8_t* src, int stride, int step,
                           int swap_rb, int with_alpha, int sharp, float dither);
static int import_packed(WebPPicture* pic, const uint8_t* src, int stride, int step, int swap_rb,
                         int with_alpha, int sharp) {
  return import_packed_d(pic, src, stride, step, swap_rb, with_alpha, sharp, 0.f);
}

/* dither > 0: the dithered conversion of WebPPictureARGBToYUVADithered
 * (picture_csp_enc.c:520-619), amplitude in [0, 1] */
static int import_packed_d(WebPPicture* pic, const uint8_t* src, int stride, int step,
                           int swap_rb, int with_alpha, int sharp, float dither) {
  const int w = pic->width, h = pic->height;
  if (abs(stride) < (with_alpha ? 4 : step) * w) return 0;
  const int ri = swap_rb ? 2 : 0, bi = swap_rb ? 0 : 2;
  if (pic->use_argb) {   /* ARGB container (lossless path, WebPPictureARGBToYUVA) */
    if (!WebPPictureAlloc(pic)) return 0;
    for (int y = 0; y < h; ++y) {
      const uint8_t* s = src + (size_t)y * stride;
      for (int x = 0; x < w; ++x, s += step) {
        const uint32_t a = with_alpha ? s[3] : 0xff;
        pic->argb[y * pic->argb_stride + x] =
            (a << 24) | ((uint32_t)s[ri] << 16) | ((uint32_t)s[1] << 8) | s[bi];
      }
    }
    return 1;
  }
  /* repack to RGBA (alpha forced opaque when the source has none), convert
   * on the GPU (K1) */
  uint8_t* rgba = (uint8_t*)malloc((size_t)w * h * 4);
  if (!rgba) return set_error(pic, VP8_ENC_ERROR_OUT_OF_MEMORY);
  for (int y = 0; y < h; ++y) {
    const uint8_t* s = src + (size_t)y * stride;
    uint8_t* d = rgba + (size_t)y * w * 4;
    for (int x = 0; x < w; ++x, s += step, d += 4) {
      d[0] = s[ri]; d[1] = s[1]; d[2] = s[bi]; d[3] = with_alpha ? s[3] : 0xff;
    }
  }
  /* CheckNonOpaque (picture_csp_enc.c:52-66): YUV420A only with alpha */
  int translucent = 0;
  if (with_alpha)
    for (size_t i = 0; i < (size_t)w * h && !translucent; ++i) translucent = rgba[4 * i + 3] != 0xff;
  pic->colorspace = translucent ? WEBP_YUV420A : WEBP_YUV420;
  int ok = vp8h_pic_alloc_yuva(pic);
  if (ok) {
    WebPConfig cfg;
    WebPConfigInitInternal(&cfg, WEBP_PRESET_DEFAULT, 75.f, WEBP_ENCODER_ABI_VERSION);
    WebPGpuBatch* e = pool_get(&cfg, w, h, 0);
    int has_alpha = 0;
    ok = e != NULL && vp8g_engine_import(e, rgba, 4 * w, pic->y, pic->u, pic->v,
                                         translucent ? pic->a : NULL, &has_alpha, sharp,
                                         sharp ? 0.f : dither);
    pool_put(e);
    if (!ok) set_error(pic, VP8_ENC_ERROR_OUT_OF_MEMORY);
  }
  free(rgba);
  return ok;
}

int WebPPictureImportRGB(WebPPicture* p, const uint8_t* s, int st) {
  return (p && s) ? import_packed(p, s, st, 3, 0, 0, 0) : 0;
}
int WebPPictureImportRGBA(WebPPicture* p, const uint8_t* s, int st) {
  return (p && s) ? import_packed(p, s, st, 4, 0, 1, 0) : 0;
}
int WebPPictureImportRGBX(WebPPicture* p, const uint8_t* s, int st) {
  return (p && s) ? import_packed(p, s, st, 4, 0, 0, 0) : 0;
}
int WebPPictureImportBGR(WebPPicture* p, const uint8_t* s, int st) {
  return (p && s) ? import_packed(p, s, st, 3, 1, 0, 0) : 0;
}
int WebPPictureImportBGRA(WebPPicture* p, const uint8_t* s, int st) {
  return (p && s) ? import_packed(p, s, st, 4, 1, 1, 0) : 0;
}
int WebPPictureImportBGRX(WebPPicture* p, const uint8_t* s, int st) {
  return (p && s) ? import_packed(p, s, st, 4, 1, 0, 0) : 0;
}

/* picture_csp_enc.c:622-664: ARGB container -> YUV420 through K1, or the
 * sharp-YUV kernels when `sharp` */
static int argb_to_yuva(WebPPicture* p, WebPEncCSP csp, int sharp, float dither) {
  if (p == NULL) return 0;
  if (p->argb == NULL) return set_error(p, VP8_ENC_ERROR_NULL_PARAMETER);
  if ((csp & WEBP_CSP_UV_MASK) != WEBP_YUV420)
    return set_error(p, VP8_ENC_ERROR_INVALID_CONFIGURATION);
  const int w = p->width, h = p->height;
  uint8_t* bgra = (uint8_t*)malloc((size_t)w * h * 4);
  if (!bgra) return set_error(p, VP8_ENC_ERROR_OUT_OF_MEMORY);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const uint32_t v = p->argb[y * p->argb_stride + x];
      uint8_t* d = bgra + ((size_t)y * w + x) * 4;
      d[0] = v & 0xff; d[1] = (v >> 8) & 0xff; d[2] = (v >> 16) & 0xff; d[3] = v >> 24;
    }
  void* keep_argb = p->memory_argb_;
  uint32_t* keep_ptr = p->argb;
  const int keep_stride = p->argb_stride;
  p->use_argb = 0;
  p->memory_argb_ = NULL;   /* keep ARGB alive across the YUV allocation */
  const int ok = import_packed_d(p, bgra, 4 * w, 4, 1, 1, sharp, dither);
  p->memory_argb_ = keep_argb;
  p->argb = keep_ptr;
  p->argb_stride = keep_stride;
  free(bgra);
  return ok;
}

int WebPPictureARGBToYUVA(WebPPicture* p, WebPEncCSP csp) {
  return argb_to_yuva(p, csp, 0, 0.f);
}

int WebPPictureSharpARGBToYUVA(WebPPicture* p) { return argb_to_yuva(p, WEBP_YUV420, 1, 0.f); }
int WebPPictureSmartARGBToYUVA(WebPPicture* p) { return WebPPictureSharpARGBToYUVA(p); }

/* picture_csp_enc.c:649-652: the VP8Random rounding terms (same for every
 * picture of a size and amplitude, host/vp8_host.c) feed K1 */
int WebPPictureARGBToYUVADithered(WebPPicture* p, WebPEncCSP csp, float dithering) {
  if (p == NULL) return 0;
  return argb_to_yuva(p, csp, 0, dithering > 0.f ? dithering : 0.f);
}

/* ---- WebPEncode (webp_enc.c:330-410) ---- */

/* StoreSideInfo's per-MB map (frame_enc.c:503-518) from the final pass's
 * MB records: 1 intra type, 2 segment, 3 segment quantiser, 4 intra-16 mode
 * (0xff for intra-4), 5 chroma mode, 7 analysis alpha (its class centre).
 * Type 6 (coded bits per MB) is only set by the reference's VP8EncLoop path
 * (frame_enc.c:354-355; uninitialised in its token loop) and is stored as 0
 * here, like every other type. */
static void store_extra_info(WebPPicture* pic, const vp8h_frame* fr, const uint8_t* mbinfo,
                             const uint8_t* mb_alpha) {
  const int nmb = fr->mbw * fr->mbh;
  for (int i = 0; i < nmb; ++i) {
    const uint8_t* m = mbinfo + (size_t)i * VP8G_MBINFO_BYTES;   /* is_i16, uv, seg, skip, modes */
    uint8_t v;
    switch (pic->extra_info_type) {
      case 1: v = m[0]; break;
      case 2: v = m[2]; break;
      case 3: v = (uint8_t)fr->seg_quant[m[2]]; break;
      case 4: v = m[0] ? m[4] : 0xff; break;
      case 5: v = m[1]; break;
      case 7: v = fr->alpha_center[mb_alpha[i]]; break;
      default: v = 0; break;
    }
    pic->extra_info[i] = v;
  }
}

static int report(const WebPPicture* pic, int percent) {
  if (pic->progress_hook && !pic->progress_hook(percent, pic))
    return set_error(pic, VP8_ENC_ERROR_USER_ABORT);
  return 1;
}

/* the token loop's progress, one call per MB row folded (VP8IteratorProgress,
 * iterator_enc.c:89-99, between WebPEncode's 20 and 90), deduplicated like
 * WebPReportProgress (webp_enc.c:317-327) and kept monotone over the passes
 * of a size / PSNR search (each K3 pass folds the rows from the top again) */
typedef struct {
  const WebPPicture* pic;
  int last;
} ProgressCtx;
static int progress_rows(void* ctx, int rows, int total) {
  ProgressCtx* c = (ProgressCtx*)ctx;
  const int pct = 20 + (69 * rows) / (total > 0 ? total : 1);   /* 90 follows */
  if (pct <= c->last) return 1;
  c->last = pct;
  return report(c->pic, pct);
}

static double psnr(uint64_t err, uint64_t size) {
  return (err > 0 && size > 0) ? 10. * log10(255. * 255. * size / err) : 99.;
}

/* webp_enc.c:396-407: ARGB samples (converted from YUVA when needed),
 * fully transparent pixels zeroed unless `exact`, then the VP8L engine
 * (host/vp8l_batch.c) on one frame. */
static int encode_lossless(const WebPConfig* config, WebPPicture* pic) {
  if (pic->argb == NULL && !WebPPictureYUVAToARGB(pic)) return 0;
  const int w = pic->width, h = pic->height;
  uint8_t* rgba = (uint8_t*)malloc((size_t)w * h * 4);
  if (!rgba) return set_error(pic, VP8_ENC_ERROR_OUT_OF_MEMORY);
  for (int y = 0; y < h; ++y) {
    const uint32_t* s = pic->argb + (size_t)y * pic->argb_stride;
    uint8_t* d = rgba + (size_t)y * w * 4;
    for (int x = 0; x < w; ++x, d += 4) {
      uint32_t v = s[x];
      if (!config->exact && (v >> 24) == 0) v = 0;   /* WebPReplaceTransparentPixels */
      d[0] = (uint8_t)(v >> 16); d[1] = (uint8_t)(v >> 8); d[2] = (uint8_t)v;
      d[3] = (uint8_t)(v >> 24);
    }
  }
  if (!report(pic, 5)) { free(rgba); return 0; }
  WebPGpuBatch* e = pool_get(config, w, h, 1);
  if (e) {   /* per call */
    vp8l_engine_set_near_lossless(e->l, config->near_lossless);
    vp8l_engine_set_exact(e->l, config->exact);
  }
  int ok = e != NULL && WebPGpuBatchEncodeRGBAHost(e, rgba, (size_t)w * h * 4, 4 * w, 1);
  free(rgba);
  const int err = ok ? WebPGpuBatchError(e, 0) : VP8_ENC_ERROR_OUT_OF_MEMORY;
  const size_t size = ok && !err ? WebPGpuBatchOutputSize(e, 0) : 0;
  uint8_t* out = size ? (uint8_t*)malloc(size) : NULL;
  if (out) memcpy(out, WebPGpuBatchOutput(e, 0), size);
  vp8l_frame_info li;
  memset(&li, 0, sizeof(li));
  if (ok && !err) vp8l_engine_frame_info(e->l, 0, &li);
  pool_put(e);
  if (!ok || err != VP8_ENC_OK || out == NULL) {
    free(out);
    return set_error(pic, err != VP8_ENC_OK ? (WebPEncodingError)err : VP8_ENC_ERROR_OUT_OF_MEMORY);
  }
  ok = report(pic, 90) && pic->writer(out, size, pic);
  free(out);
  if (!ok) return pic->error_code != VP8_ENC_OK ? 0 : set_error(pic, VP8_ENC_ERROR_BAD_WRITE);
  if (pic->stats != NULL) {   /* vp8l_enc.c:1628-1639,1841-1881 */
    WebPAuxStats* s = pic->stats;
    memset(s, 0, sizeof(*s));
    for (int i = 0; i < 5; ++i) s->PSNR[i] = 99.f;
    s->coded_size = (int)size;
    s->lossless_size = (int)size;
    s->lossless_features = li.features;
    s->histogram_bits = li.histogram_bits;
    s->transform_bits = li.transform_bits;
    s->cache_bits = li.cache_bits;
    s->palette_size = li.palette_size;
    s->lossless_hdr_size = li.hdr_bytes;
    s->lossless_data_size = li.data_bytes;
  }
  if (pic->extra_info != NULL)   /* vp8l_enc.c:1884-1888 */
    memset(pic->extra_info, 0, (size_t)((w + 15) >> 4) * ((h + 15) >> 4));
  return report(pic, 100);
}

int WebPEncode(const WebPConfig* config, WebPPicture* pic) {
  if (pic == NULL) return 0;
  pic->error_code = VP8_ENC_OK;
  if (config == NULL) return set_error(pic, VP8_ENC_ERROR_NULL_PARAMETER);
  if (!WebPValidateConfig(config)) return set_error(pic, VP8_ENC_ERROR_INVALID_CONFIGURATION);
  if (!vp8h_pic_validate(pic)) return 0;
  if (pic->width > WEBP_MAX_DIMENSION || pic->height > WEBP_MAX_DIMENSION)
    return set_error(pic, VP8_ENC_ERROR_BAD_DIMENSION);
  if (pic->stats != NULL) memset(pic->stats, 0, sizeof(*pic->stats));
  if (config->lossless) return encode_lossless(config, pic);
  vp8h_frame probe;
  if (!vp8h_frame_init(&probe, config, pic->width, pic->height))
    return set_error(pic, VP8_ENC_ERROR_INVALID_CONFIGURATION);
  if (pic->use_argb || pic->y == NULL || pic->u == NULL || pic->v == NULL) {
    /* webp_enc.c:351-367 */
    const int sharp = config->use_sharp_yuv || (config->preprocessing & 4);
    if (!(sharp ? WebPPictureSharpARGBToYUVA(pic)
                : WebPPictureARGBToYUVADithered(pic, WEBP_YUV420, vp8h_import_dithering(config))))
      return 0;
  }
  if (!config->exact) WebPCleanupTransparentArea(pic);   /* webp_enc.c:369-371 */
  const int has_alpha = pic->a != NULL && WebPPictureHasTransparency(pic);

  WebPGpuBatch* e = pool_get(config, pic->width, pic->height, 0);
  int ok = e != NULL;
  if (!ok) return set_error(pic, VP8_ENC_ERROR_OUT_OF_MEMORY);
  ProgressCtx pc = {pic, 20};
  e->progress = pic->progress_hook ? progress_rows : NULL;
  e->progress_ctx = &pc;
  ok = vp8g_engine_upload_yuv(e, 0, pic->y, pic->y_stride, pic->u, pic->v, pic->uv_stride,
                              has_alpha ? pic->a : NULL, pic->a_stride) &&
       report(pic, 20) && vp8g_engine_run_yuv(e, 1);
  e->progress = NULL;
  e->progress_ctx = NULL;
  int err = ok ? e->err[0] : VP8_ENC_ERROR_OUT_OF_MEMORY;
  uint8_t* out = ok ? e->out[0] : NULL;
  const size_t size = ok ? e->out_size[0] : 0;
  if (ok) {   /* take ownership */
    e->out[0] = NULL;
    e->out_cap[0] = 0;
  }
  vp8h_frame fr;
  vp8g_frame_result res;
  memset(&fr, 0, sizeof(fr));
  memset(&res, 0, sizeof(res));
  int hdr[2] = {0, 0};
  uint64_t asse = 0;
  if (ok) {
    asse = has_alpha ? e->asse[0] : 0;
    fr = e->frames[0];
    res = e->h_results[0];
    hdr[0] = e->hdr[0];
    hdr[1] = e->hdr[1];
    if (pic->extra_info != NULL && err == VP8_ENC_OK)
      store_extra_info(pic, &fr, e->h_mbinfo, e->h_alpha);
  }
  pool_put(e);
  if (pic->error_code != VP8_ENC_OK) { free(out); return 0; }
  if (!ok || err != VP8_ENC_OK || out == NULL) {
    free(out);
    return set_error(pic, err != VP8_ENC_OK ? (WebPEncodingError)err : VP8_ENC_ERROR_OUT_OF_MEMORY);
  }
  ok = report(pic, 90) && pic->writer(out, size, pic);
  free(out);
  if (!ok) return pic->error_code != VP8_ENC_OK ? 0 : set_error(pic, VP8_ENC_ERROR_BAD_WRITE);
  if (pic->stats != NULL) {   /* StoreStats, webp_enc.c:271-304 */
    WebPAuxStats* s = pic->stats;
    const uint64_t count = (uint64_t)fr.mbw * fr.mbh * 256;
    s->coded_size = (int)size;
    s->PSNR[0] = (float)psnr(res.sse[0], count);
    s->PSNR[1] = (float)psnr(res.sse[1], count / 4);
    s->PSNR[2] = (float)psnr(res.sse[2], count / 4);
    s->PSNR[3] = (float)psnr(res.sse[0] + res.sse[1] + res.sse[2], count * 3 / 2);
    s->PSNR[4] = (float)psnr(asse, count);   /* enc->sse_[3], alpha_enc.c:362 */
    for (int i = 0; i < 3; ++i) s->block_count[i] = res.block_count[i];
    s->header_bytes[0] = hdr[0];
    s->header_bytes[1] = hdr[1];
    for (int i = 0; i < 4; ++i) {
      s->segment_size[i] = fr.segment_size[i];
      s->segment_quant[i] = fr.seg_quant[i];
      s->segment_level[i] = fr.seg_fstrength[i];
    }
  }
  return report(pic, 100);
}

/* ---- one-shot API (picture_enc.c:238-302) ---- */

typedef int (*Importer)(WebPPicture*, const uint8_t*, int);

static size_t encode_oneshot(const uint8_t* px, int w, int h, int stride, Importer imp, float q,
                             int lossless, uint8_t** output) {
  WebPPicture pic;
  WebPConfig cfg;
  WebPMemoryWriter wrt;
  if (output == NULL) return 0;
  if (!WebPConfigInitInternal(&cfg, WEBP_PRESET_DEFAULT, q, WEBP_ENCODER_ABI_VERSION) ||
      !WebPPictureInitInternal(&pic, WEBP_ENCODER_ABI_VERSION))
    return 0;
  cfg.lossless = !!lossless;
  pic.use_argb = !!lossless;
  pic.width = w;
  pic.height = h;
  pic.writer = WebPMemoryWrite;
  pic.custom_ptr = &wrt;
  WebPMemoryWriterInit(&wrt);
  const int ok = imp(&pic, px, stride) && WebPEncode(&cfg, &pic);
  WebPPictureFree(&pic);
  if (!ok) {
    WebPMemoryWriterClear(&wrt);
    *output = NULL;
    return 0;
  }
  *output = wrt.mem;
  return wrt.size;
}

size_t WebPEncodeRGB(const uint8_t* p, int w, int h, int s, float q, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportRGB, q, 0, o);
}
size_t WebPEncodeBGR(const uint8_t* p, int w, int h, int s, float q, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportBGR, q, 0, o);
}
size_t WebPEncodeRGBA(const uint8_t* p, int w, int h, int s, float q, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportRGBA, q, 0, o);
}
size_t WebPEncodeBGRA(const uint8_t* p, int w, int h, int s, float q, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportBGRA, q, 0, o);
}

/* picture_enc.c:285-297: lossless one-shot API at quality 70 */
#define LOSSLESS_DEFAULT_QUALITY 70.f
size_t WebPEncodeLosslessRGB(const uint8_t* p, int w, int h, int s, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportRGB, LOSSLESS_DEFAULT_QUALITY, 1, o);
}
size_t WebPEncodeLosslessBGR(const uint8_t* p, int w, int h, int s, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportBGR, LOSSLESS_DEFAULT_QUALITY, 1, o);
}
size_t WebPEncodeLosslessRGBA(const uint8_t* p, int w, int h, int s, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportRGBA, LOSSLESS_DEFAULT_QUALITY, 1, o);
}
size_t WebPEncodeLosslessBGRA(const uint8_t* p, int w, int h, int s, uint8_t** o) {
  return encode_oneshot(p, w, h, s, WebPPictureImportBGRA, LOSSLESS_DEFAULT_QUALITY, 1, o);
}
