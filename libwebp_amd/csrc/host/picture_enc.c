/* The HIP-free part of the libwebp encoder C ABI (include/webp/encode.h):
 * version and memory helpers, WebPConfig, WebPPicture buffers and the memory
 * writer. Behaviour follows the reference API functions cited per item.
 * (webp_api.c holds the entry points that drive the GPU engines.) */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "picture_internal.h"
#include "webp/encode.h"

#define set_error vp8h_pic_error

/* ---- misc (webp_enc.c:32-34, utils.c) ---- */

int WebPGetEncoderVersion(void) { return (1 << 16) | (3 << 8) | 2; }
void* WebPMalloc(size_t size) { return malloc(size); }
void WebPFree(void* ptr) { free(ptr); }

int vp8h_pic_error(const WebPPicture* pic, WebPEncodingError e) {   /* webp_enc.c:306-315 */
  if (pic->error_code == VP8_ENC_OK) ((WebPPicture*)pic)->error_code = e;
  return 0;
}

/* ---- WebPConfig (config_enc.c:24-157) ---- */

int WebPConfigInitInternal(WebPConfig* c, WebPPreset preset, float quality, int version) {
  if (WEBP_ABI_IS_INCOMPATIBLE(version, WEBP_ENCODER_ABI_VERSION)) return 0;
  if (c == NULL) return 0;
  memset(c, 0, sizeof(*c));
  c->quality = quality;
  c->method = 4;
  c->sns_strength = 50;
  c->filter_strength = 60;
  c->filter_type = 1;
  c->segments = 4;
  c->pass = 1;
  c->qmax = 100;
  c->alpha_compression = 1;
  c->alpha_filtering = 1;
  c->alpha_quality = 100;
  c->near_lossless = 100;
  c->image_hint = WEBP_HINT_DEFAULT;
  switch (preset) {
    case WEBP_PRESET_PICTURE:
      c->sns_strength = 80; c->filter_sharpness = 4; c->filter_strength = 35;
      c->preprocessing &= ~2;
      break;
    case WEBP_PRESET_PHOTO:
      c->sns_strength = 80; c->filter_sharpness = 3; c->filter_strength = 30;
      c->preprocessing |= 2;
      break;
    case WEBP_PRESET_DRAWING:
      c->sns_strength = 25; c->filter_sharpness = 6; c->filter_strength = 10;
      break;
    case WEBP_PRESET_ICON:
      c->sns_strength = 0; c->filter_strength = 0; c->preprocessing &= ~2;
      break;
    case WEBP_PRESET_TEXT:
      c->sns_strength = 0; c->filter_strength = 0; c->preprocessing &= ~2; c->segments = 2;
      break;
    default:
      break;
  }
  return WebPValidateConfig(c);
}

#define IN_RANGE(v, lo, hi) ((v) >= (lo) && (v) <= (hi))
int WebPValidateConfig(const WebPConfig* c) {
  if (c == NULL) return 0;
  return IN_RANGE(c->quality, 0, 100) && c->target_size >= 0 && c->target_PSNR >= 0 &&
         IN_RANGE(c->method, 0, 6) && IN_RANGE(c->segments, 1, 4) &&
         IN_RANGE(c->sns_strength, 0, 100) && IN_RANGE(c->filter_strength, 0, 100) &&
         IN_RANGE(c->filter_sharpness, 0, 7) && IN_RANGE(c->filter_type, 0, 1) &&
         IN_RANGE(c->autofilter, 0, 1) && IN_RANGE(c->pass, 1, 10) && c->qmin >= 0 &&
         c->qmax <= 100 && c->qmin <= c->qmax && IN_RANGE(c->show_compressed, 0, 1) &&
         IN_RANGE(c->preprocessing, 0, 7) && IN_RANGE(c->partitions, 0, 3) &&
         IN_RANGE(c->partition_limit, 0, 100) && c->alpha_compression >= 0 &&
         c->alpha_filtering >= 0 && IN_RANGE(c->alpha_quality, 0, 100) &&
         IN_RANGE(c->lossless, 0, 1) && IN_RANGE(c->near_lossless, 0, 100) &&
         c->image_hint < WEBP_HINT_LAST && IN_RANGE(c->emulate_jpeg_size, 0, 1) &&
         IN_RANGE(c->thread_level, 0, 1) && IN_RANGE(c->low_memory, 0, 1) &&
         IN_RANGE(c->exact, 0, 1) && IN_RANGE(c->use_delta_palette, 0, 1) &&
         IN_RANGE(c->use_sharp_yuv, 0, 1);
}

int WebPConfigLosslessPreset(WebPConfig* c, int level) {
  static const uint8_t kMethod[10] = {0, 1, 2, 3, 3, 4, 4, 4, 5, 6};
  static const uint8_t kQuality[10] = {0, 20, 25, 30, 50, 50, 75, 90, 90, 100};
  if (c == NULL || level < 0 || level > 9) return 0;
  c->lossless = 1;
  c->method = kMethod[level];
  c->quality = kQuality[level];
  return 1;
}

/* ---- WebPPicture (picture_enc.c:25-183) ---- */

static int DummyWriter(const uint8_t* d, size_t n, const WebPPicture* p) {
  (void)d; (void)n; (void)p;
  return 1;
}

int WebPPictureInitInternal(WebPPicture* pic, int version) {
  if (WEBP_ABI_IS_INCOMPATIBLE(version, WEBP_ENCODER_ABI_VERSION)) return 0;
  if (pic != NULL) {
    memset(pic, 0, sizeof(*pic));
    pic->writer = DummyWriter;
    pic->error_code = VP8_ENC_OK;
  }
  return 1;
}

int vp8h_pic_validate(const WebPPicture* pic) {
  if (pic == NULL) return 0;
  if (pic->width <= 0 || pic->height <= 0 || pic->width / 4 > INT_MAX / 4 ||
      pic->height / 4 > INT_MAX / 4)
    return set_error(pic, VP8_ENC_ERROR_BAD_DIMENSION);
  if (pic->colorspace != WEBP_YUV420 && pic->colorspace != WEBP_YUV420A)
    return set_error(pic, VP8_ENC_ERROR_INVALID_CONFIGURATION);
  return 1;
}

void vp8h_pic_reset_argb(WebPPicture* p) { p->memory_argb_ = NULL; p->argb = NULL; p->argb_stride = 0; }
void vp8h_pic_reset_yuva(WebPPicture* p) {
  p->memory_ = NULL;
  p->y = p->u = p->v = p->a = NULL;
  p->y_stride = p->uv_stride = p->a_stride = 0;
}

int vp8h_pic_alloc_argb(WebPPicture* p) {
  if (!vp8h_pic_validate(p)) return 0;
  free(p->memory_argb_);
  vp8h_pic_reset_argb(p);
  void* m = malloc((size_t)p->width * p->height * 4 + 64);
  if (!m) return set_error(p, VP8_ENC_ERROR_OUT_OF_MEMORY);
  p->memory_argb_ = m;
  p->argb = (uint32_t*)(((uintptr_t)m + 31) & ~(uintptr_t)31);
  p->argb_stride = p->width;
  return 1;
}

int vp8h_pic_alloc_yuva(WebPPicture* p) {
  if (!vp8h_pic_validate(p)) return 0;
  const int has_alpha = (int)p->colorspace & WEBP_CSP_ALPHA_BIT;
  const int w = p->width, h = p->height;
  const int uvw = (int)(((int64_t)w + 1) >> 1), uvh = (int)(((int64_t)h + 1) >> 1);
  const uint64_t ys = (uint64_t)w * h, uvs = (uint64_t)uvw * uvh;
  const uint64_t as = has_alpha ? (uint64_t)w * h : 0;
  free(p->memory_);
  vp8h_pic_reset_yuva(p);
  uint8_t* m = (uint8_t*)malloc(ys + as + 2 * uvs);
  if (!m) return set_error(p, VP8_ENC_ERROR_OUT_OF_MEMORY);
  p->memory_ = m;
  p->y_stride = w;
  p->uv_stride = uvw;
  p->a_stride = has_alpha ? w : 0;
  p->y = m;
  p->u = m + ys;
  p->v = p->u + uvs;
  if (as) p->a = p->v + uvs;
  return 1;
}

int WebPPictureAlloc(WebPPicture* p) {
  if (p != NULL) {
    WebPPictureFree(p);
    return p->use_argb ? vp8h_pic_alloc_argb(p) : vp8h_pic_alloc_yuva(p);
  }
  return 1;
}

void WebPPictureFree(WebPPicture* p) {
  if (p != NULL) {
    free(p->memory_);
    free(p->memory_argb_);
    vp8h_pic_reset_argb(p);
    vp8h_pic_reset_yuva(p);
  }
}

int WebPPictureCopy(const WebPPicture* src, WebPPicture* dst) {   /* picture_rescale_enc.c */
  if (src == NULL || dst == NULL) return 0;
  if (src == dst) return 1;
  *dst = *src;
  vp8h_pic_reset_argb(dst);
  vp8h_pic_reset_yuva(dst);
  if (!WebPPictureAlloc(dst)) return 0;
  if (!src->use_argb) {
    const int uvw = (src->width + 1) >> 1, uvh = (src->height + 1) >> 1;
    for (int y = 0; y < src->height; ++y)
      memcpy(dst->y + y * dst->y_stride, src->y + y * src->y_stride, src->width);
    for (int y = 0; y < uvh; ++y) {
      memcpy(dst->u + y * dst->uv_stride, src->u + y * src->uv_stride, uvw);
      memcpy(dst->v + y * dst->uv_stride, src->v + y * src->uv_stride, uvw);
    }
    if (dst->a)
      for (int y = 0; y < src->height; ++y)
        memcpy(dst->a + y * dst->a_stride, src->a + y * src->a_stride, src->width);
  } else {
    for (int y = 0; y < src->height; ++y)
      memcpy(dst->argb + y * dst->argb_stride, src->argb + y * src->argb_stride,
             4 * (size_t)src->width);
  }
  return 1;
}

int WebPPictureHasTransparency(const WebPPicture* p) {   /* picture_csp_enc.c:69-81 */
  if (p == NULL) return 0;
  if (p->use_argb) {
    if (p->argb == NULL) return 0;
    for (int y = 0; y < p->height; ++y)
      for (int x = 0; x < p->width; ++x)
        if ((p->argb[y * p->argb_stride + x] >> 24) != 0xff) return 1;
    return 0;
  }
  if (p->a == NULL) return 0;
  for (int y = 0; y < p->height; ++y)
    for (int x = 0; x < p->width; ++x)
      if (p->a[y * p->a_stride + x] != 0xff) return 1;
  return 0;
}

/* ---- WebPMemoryWriter (picture_enc.c:188-233) ---- */

void WebPMemoryWriterInit(WebPMemoryWriter* w) {
  w->mem = NULL;
  w->size = 0;
  w->max_size = 0;
}

void WebPMemoryWriterClear(WebPMemoryWriter* w) {
  if (w != NULL) {
    free(w->mem);
    WebPMemoryWriterInit(w);
  }
}

int WebPMemoryWrite(const uint8_t* data, size_t n, const WebPPicture* pic) {
  WebPMemoryWriter* const w = (WebPMemoryWriter*)pic->custom_ptr;
  if (w == NULL) return 1;
  const uint64_t next = (uint64_t)w->size + n;
  if (next > w->max_size) {
    uint64_t cap = 2ULL * w->max_size;
    if (cap < next) cap = next;
    if (cap < 8192ULL) cap = 8192ULL;
    uint8_t* m = (uint8_t*)malloc((size_t)cap);
    if (m == NULL) return 0;
    if (w->size > 0) memcpy(m, w->mem, w->size);
    free(w->mem);
    w->mem = m;
    w->max_size = (size_t)cap;
  }
  if (n > 0) {
    memcpy(w->mem + w->size, data, n);
    w->size += n;
  }
  return 1;
}

