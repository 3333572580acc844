/* WebPPicture utilities of the libwebp encoder ABI that sit beside the
 * encode path: views and crops, the rescaler, YUV->ARGB
 * with the "fancy" chroma upsampler, PSNR/SSIM/LSIM distortion, transparent
 * area cleanup and alpha blending. Host C over the caller's host buffers —
 * these are per-picture API conveniences for cwebp (-crop, -resize,
 * -print_psnr/-print_ssim, -blend_alpha), not the batched GPU encode path.
 * Integer behaviour is bit-exact with the reference; each block cites the
 * reference file:line it restates (paths relative to the reference root). */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "picture_internal.h"
#include "webp/encode.h"

#define HALVE(x) (((x) + 1) >> 1)

static void copy_plane(const uint8_t* src, int ss, uint8_t* dst, int ds, int w, int h) {
  for (int y = 0; y < h; ++y) memcpy(dst + (size_t)y * ds, src + (size_t)y * ss, (size_t)w);
}

/* PictureGrabSpecs, src/enc/picture_rescale_enc.c:30-35 */
static void grab_specs(const WebPPicture* src, WebPPicture* dst) {
  *dst = *src;
  vp8h_pic_reset_argb(dst);
  vp8h_pic_reset_yuva(dst);
}

/* AdjustAndCheckRectangle + SnapTopLeftPosition, :39-58 */
static int check_rect(const WebPPicture* pic, int* left, int* top, int w, int h) {
  if (!pic->use_argb) {
    *left &= ~1;
    *top &= ~1;
  }
  if (*left < 0 || *top < 0 || w <= 0 || h <= 0) return 0;
  return *left + w <= pic->width && *top + h <= pic->height;
}

/* ---- views and crops: picture_rescale_enc.c:87-165 ---- */

int WebPPictureIsView(const WebPPicture* pic) {
  if (pic == NULL) return 0;
  return pic->use_argb ? pic->memory_argb_ == NULL : pic->memory_ == NULL;
}

int WebPPictureView(const WebPPicture* src, int left, int top, int width, int height,
                    WebPPicture* dst) {
  if (src == NULL || dst == NULL) return 0;
  if (!check_rect(src, &left, &top, width, height)) return 0;
  if (src != dst) grab_specs(src, dst);   /* aliasing: keep memory_ of src */
  dst->width = width;
  dst->height = height;
  if (!src->use_argb) {
    dst->y = src->y + top * src->y_stride + left;
    dst->u = src->u + (top >> 1) * src->uv_stride + (left >> 1);
    dst->v = src->v + (top >> 1) * src->uv_stride + (left >> 1);
    dst->y_stride = src->y_stride;
    dst->uv_stride = src->uv_stride;
    if (src->a != NULL) {
      dst->a = src->a + top * src->a_stride + left;
      dst->a_stride = src->a_stride;
    }
  } else {
    dst->argb = src->argb + top * src->argb_stride + left;
    dst->argb_stride = src->argb_stride;
  }
  return 1;
}

int WebPPictureCrop(WebPPicture* pic, int left, int top, int width, int height) {
  WebPPicture tmp;
  if (pic == NULL) return 0;
  if (!check_rect(pic, &left, &top, width, height)) return 0;
  grab_specs(pic, &tmp);
  tmp.width = width;
  tmp.height = height;
  if (!WebPPictureAlloc(&tmp)) return vp8h_pic_error(pic, tmp.error_code);
  if (!pic->use_argb) {
    const int yo = top * pic->y_stride + left;
    const int uvo = (top / 2) * pic->uv_stride + left / 2;
    copy_plane(pic->y + yo, pic->y_stride, tmp.y, tmp.y_stride, width, height);
    copy_plane(pic->u + uvo, pic->uv_stride, tmp.u, tmp.uv_stride, HALVE(width), HALVE(height));
    copy_plane(pic->v + uvo, pic->uv_stride, tmp.v, tmp.uv_stride, HALVE(width), HALVE(height));
    if (tmp.a != NULL)
      copy_plane(pic->a + top * pic->a_stride + left, pic->a_stride, tmp.a, tmp.a_stride, width,
                 height);
  } else {
    copy_plane((const uint8_t*)(pic->argb + top * pic->argb_stride + left), 4 * pic->argb_stride,
               (uint8_t*)tmp.argb, 4 * tmp.argb_stride, 4 * width, height);
  }
  WebPPictureFree(pic);
  *pic = tmp;
  return 1;
}

/* ---- rescaler: src/utils/rescaler_utils.c:24-160, src/dsp/rescaler.c ---- */

#define RFIX 32
#define RONE (1ull << RFIX)
#define RFRAC(x, y) ((uint32_t)(((uint64_t)(x) << RFIX) / (y)))
#define MULT_FIX(x, y) ((uint32_t)(((uint64_t)(x) * (y) + (RONE >> 1)) >> RFIX))
#define MULT_FIX_FLOOR(x, y) ((uint32_t)(((uint64_t)(x) * (y)) >> RFIX))

typedef struct {
  int x_expand, y_expand, nc;
  uint32_t fx_scale, fy_scale, fxy_scale;
  int y_accum, y_add, y_sub, x_add, x_sub;
  int src_w, src_h, dst_w, dst_h, src_y, dst_y;
  uint8_t* dst;
  int dst_stride;
  uint32_t *irow, *frow;
} Rescaler;

static void rs_init(Rescaler* r, int sw, int sh, uint8_t* dst, int dw, int dh, int ds, int nc,
                    uint32_t* work) {   /* WebPRescalerInit, rescaler_utils.c:24-79 */
  memset(r, 0, sizeof(*r));
  r->x_expand = sw < dw;
  r->y_expand = sh < dh;
  r->src_w = sw; r->src_h = sh; r->dst_w = dw; r->dst_h = dh;
  r->dst = dst; r->dst_stride = ds; r->nc = nc;
  r->x_add = r->x_expand ? dw - 1 : sw;
  r->x_sub = r->x_expand ? sw - 1 : dw;
  if (!r->x_expand) r->fx_scale = RFRAC(1, r->x_sub);
  r->y_add = r->y_expand ? sh - 1 : sh;
  r->y_sub = r->y_expand ? dh - 1 : dh;
  r->y_accum = r->y_expand ? r->y_sub : r->y_add;
  if (!r->y_expand) {
    const uint64_t ratio = (uint64_t)dh * RONE / ((uint64_t)r->x_add * r->y_add);
    r->fxy_scale = ratio != (uint32_t)ratio ? 0 : (uint32_t)ratio;
    r->fy_scale = RFRAC(1, r->y_sub);
  } else {
    r->fy_scale = RFRAC(1, r->x_add);
  }
  r->irow = work;
  r->frow = work + (size_t)nc * dw;
  memset(work, 0, 2 * sizeof(uint32_t) * nc * dw);
}

static void rs_import_row(Rescaler* r, const uint8_t* src) {   /* rescaler.c:27-97 */
  const int xs = r->nc, xmax = r->dst_w * r->nc;
  for (int c = 0; c < xs; ++c) {
    int x_in = c, x_out = c;
    if (r->x_expand) {   /* bilinear */
      int accum = r->x_add;
      uint32_t left = src[x_in];
      uint32_t right = r->src_w > 1 ? src[x_in + xs] : left;
      x_in += xs;
      for (;;) {
        r->frow[x_out] = right * r->x_add + (left - right) * accum;
        x_out += xs;
        if (x_out >= xmax) break;
        accum -= r->x_sub;
        if (accum < 0) {
          left = right;
          x_in += xs;
          right = src[x_in];
          accum += r->x_add;
        }
      }
    } else {             /* box average with fractional edges */
      uint32_t sum = 0;
      int accum = 0;
      while (x_out < xmax) {
        uint32_t base = 0;
        accum += r->x_add;
        while (accum > 0) {
          accum -= r->x_sub;
          base = src[x_in];
          sum += base;
          x_in += xs;
        }
        const uint32_t frac = base * (uint32_t)(-accum);
        r->frow[x_out] = sum * r->x_sub - frac;
        sum = (uint32_t)(int)MULT_FIX(frac, r->fx_scale);
        x_out += xs;
      }
    }
  }
}

static void rs_export_row(Rescaler* r) {   /* rescaler.c:102-170, :176-209 */
  const int xmax = r->dst_w * r->nc;
  uint8_t* const dst = r->dst;
  if (r->y_expand) {
    if (r->y_accum == 0) {
      for (int x = 0; x < xmax; ++x) {
        const int v = (int)MULT_FIX(r->frow[x], r->fy_scale);
        dst[x] = v > 255 ? 255 : (uint8_t)v;
      }
    } else {
      const uint32_t B = RFRAC(-r->y_accum, r->y_sub);
      const uint32_t A = (uint32_t)(RONE - B);
      for (int x = 0; x < xmax; ++x) {
        const uint64_t I = (uint64_t)A * r->frow[x] + (uint64_t)B * r->irow[x];
        const uint32_t J = (uint32_t)((I + (RONE >> 1)) >> RFIX);
        const int v = (int)MULT_FIX(J, r->fy_scale);
        dst[x] = v > 255 ? 255 : (uint8_t)v;
      }
    }
  } else if (r->fxy_scale) {
    const uint32_t yscale = r->fy_scale * (uint32_t)(-r->y_accum);
    for (int x = 0; x < xmax; ++x) {
      if (yscale) {
        const uint32_t frac = MULT_FIX_FLOOR(r->frow[x], yscale);
        const int v = (int)MULT_FIX(r->irow[x] - frac, r->fxy_scale);
        dst[x] = v > 255 ? 255 : (uint8_t)v;
        r->irow[x] = frac;
      } else {
        const int v = (int)MULT_FIX(r->irow[x], r->fxy_scale);
        dst[x] = v > 255 ? 255 : (uint8_t)v;
        r->irow[x] = 0;
      }
    }
  } else {   /* 1-pixel-wide source, same height (:189-196) */
    for (int x = 0; x < xmax; ++x) {
      dst[x] = (uint8_t)r->irow[x];
      r->irow[x] = 0;
    }
  }
  r->y_accum += r->y_add;
  r->dst += r->dst_stride;
  ++r->dst_y;
}

static void rescale_plane(const uint8_t* src, int sw, int sh, int ss, uint8_t* dst, int dw,
                          int dh, int ds, uint32_t* work, int nc) {   /* picture_rescale_enc.c:170-189 */
  Rescaler r;
  rs_init(&r, sw, sh, dst, dw, dh, ds, nc, work);
  int y = 0;
  while (y < sh) {
    /* WebPRescalerImport (rescaler_utils.c:121-145) */
    while (y < sh && !(r.dst_y < r.dst_h && r.y_accum <= 0)) {
      if (r.y_expand) {
        uint32_t* t = r.irow;
        r.irow = r.frow;
        r.frow = t;
      }
      rs_import_row(&r, src + (size_t)y * ss);
      if (!r.y_expand)
        for (int x = 0; x < nc * dw; ++x) r.irow[x] += r.frow[x];
      ++r.src_y;
      ++y;
      r.y_accum -= r.y_sub;
    }
    while (r.dst_y < r.dst_h && r.y_accum <= 0) rs_export_row(&r);   /* WebPRescalerExport */
  }
}

/* alpha premultiplication, src/dsp/alpha_processing.c:25-33,134-176 (the
 * non-table variant; 24-bit fixed point, uint32 arithmetic) */
static inline uint32_t amul(uint32_t x, uint32_t m) { return (x * m + (1u << 23)) >> 24; }
static inline uint32_t ascale(uint32_t a, int inverse) {
  return inverse ? (255u << 24) / a : a * ((1u << 24) / 255u);
}
static void mult_argb_rows(uint32_t* p, int stride, int w, int h, int inverse) {
  for (int y = 0; y < h; ++y, p += stride)
    for (int x = 0; x < w; ++x) {
      const uint32_t v = p[x];
      if (v >= 0xff000000u) continue;
      if (v <= 0x00ffffffu) {
        p[x] = 0;
        continue;
      }
      const uint32_t s = ascale(v >> 24, inverse);
      p[x] = (v & 0xff000000u) | amul(v & 0xff, s) | (amul((v >> 8) & 0xff, s) << 8) |
             (amul((v >> 16) & 0xff, s) << 16);
    }
}
static void mult_rows(uint8_t* p, int ps, const uint8_t* a, int as, int w, int h, int inverse) {
  for (int y = 0; y < h; ++y, p += ps, a += as)
    for (int x = 0; x < w; ++x) {
      if (a[x] == 255) continue;
      p[x] = a[x] == 0 ? 0 : (uint8_t)amul(p[x], ascale(a[x], inverse));
    }
}

int WebPPictureRescale(WebPPicture* pic, int width, int height) {   /* picture_rescale_enc.c:207-270 */
  WebPPicture tmp;
  if (pic == NULL) return 0;
  const int pw = pic->width, ph = pic->height;
  {   /* WebPRescalerGetScaledDimensions, rescaler_utils.c:81-107 */
    if (width == 0 && ph > 0) width = (int)(((uint64_t)pw * height + ph - 1) / ph);
    if (height == 0 && pw > 0) height = (int)(((uint64_t)ph * width + pw - 1) / pw);
    if (width <= 0 || height <= 0 || width > 0x3fffffff || height > 0x3fffffff)
      return vp8h_pic_error(pic, VP8_ENC_ERROR_BAD_DIMENSION);
  }
  grab_specs(pic, &tmp);
  tmp.width = width;
  tmp.height = height;
  if (!WebPPictureAlloc(&tmp)) return vp8h_pic_error(pic, tmp.error_code);
  const int nc = pic->use_argb ? 4 : 1;
  uint32_t* work = (uint32_t*)malloc(2 * sizeof(uint32_t) * (size_t)width * nc);
  if (work == NULL) {
    WebPPictureFree(&tmp);
    return vp8h_pic_error(pic, VP8_ENC_ERROR_OUT_OF_MEMORY);
  }
  if (!pic->use_argb) {
    if (pic->a != NULL)
      rescale_plane(pic->a, pw, ph, pic->a_stride, tmp.a, width, height, tmp.a_stride, work, 1);
    if (pic->a != NULL) mult_rows(pic->y, pic->y_stride, pic->a, pic->a_stride, pw, ph, 0);
    rescale_plane(pic->y, pw, ph, pic->y_stride, tmp.y, width, height, tmp.y_stride, work, 1);
    rescale_plane(pic->u, HALVE(pw), HALVE(ph), pic->uv_stride, tmp.u, HALVE(width),
                  HALVE(height), tmp.uv_stride, work, 1);
    rescale_plane(pic->v, HALVE(pw), HALVE(ph), pic->uv_stride, tmp.v, HALVE(width),
                  HALVE(height), tmp.uv_stride, work, 1);
    if (tmp.a != NULL) mult_rows(tmp.y, tmp.y_stride, tmp.a, tmp.a_stride, width, height, 1);
  } else {
    mult_argb_rows(pic->argb, pic->argb_stride, pw, ph, 0);
    rescale_plane((const uint8_t*)pic->argb, pw, ph, 4 * pic->argb_stride, (uint8_t*)tmp.argb,
                  width, height, 4 * tmp.argb_stride, work, 4);
    mult_argb_rows(tmp.argb, tmp.argb_stride, width, height, 1);
  }
  WebPPictureFree(pic);
  free(work);
  *pic = tmp;
  return 1;
}

/* ---- YUV(A) -> ARGB: picture_csp_enc.c:669-727 with the fancy upsampler
 * (src/dsp/upsampling.c:35-95) and VP8YuvToBgra (src/dsp/yuv.h:59-138) ---- */

static inline int mult_hi(int v, int c) { return (v * c) >> 8; }
static inline int clip8_6(int v) { return (v & ~16383) == 0 ? (v >> 6) : (v < 0) ? 0 : 255; }
static inline uint32_t yuv_to_argb(int y, int u, int v) {
  const int r = clip8_6(mult_hi(y, 19077) + mult_hi(v, 26149) - 14234);
  const int g = clip8_6(mult_hi(y, 19077) - mult_hi(u, 6419) - mult_hi(v, 13320) + 8708);
  const int b = clip8_6(mult_hi(y, 19077) + mult_hi(u, 33050) - 17685);
  return 0xff000000u | ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
}
#define LOAD_UV(u, v) ((uint32_t)(u) | ((uint32_t)(v) << 16))

static void upsample_pair(const uint8_t* ty, const uint8_t* by, const uint8_t* tu,
                          const uint8_t* tv, const uint8_t* cu, const uint8_t* cv, uint32_t* td,
                          uint32_t* bd, int len) {
  const int last = (len - 1) >> 1;
  uint32_t tl = LOAD_UV(tu[0], tv[0]), l = LOAD_UV(cu[0], cv[0]);
  {
    const uint32_t uv0 = (3 * tl + l + 0x00020002u) >> 2;
    td[0] = yuv_to_argb(ty[0], uv0 & 0xff, uv0 >> 16);
  }
  if (by) {
    const uint32_t uv0 = (3 * l + tl + 0x00020002u) >> 2;
    bd[0] = yuv_to_argb(by[0], uv0 & 0xff, uv0 >> 16);
  }
  for (int x = 1; x <= last; ++x) {
    const uint32_t t = LOAD_UV(tu[x], tv[x]), uv = LOAD_UV(cu[x], cv[x]);
    const uint32_t avg = tl + t + l + uv + 0x00080008u;
    const uint32_t d12 = (avg + 2 * (t + l)) >> 3, d03 = (avg + 2 * (tl + uv)) >> 3;
    {
      const uint32_t uv0 = (d12 + tl) >> 1, uv1 = (d03 + t) >> 1;
      td[2 * x - 1] = yuv_to_argb(ty[2 * x - 1], uv0 & 0xff, uv0 >> 16);
      td[2 * x] = yuv_to_argb(ty[2 * x], uv1 & 0xff, uv1 >> 16);
    }
    if (by) {
      const uint32_t uv0 = (d03 + l) >> 1, uv1 = (d12 + uv) >> 1;
      bd[2 * x - 1] = yuv_to_argb(by[2 * x - 1], uv0 & 0xff, uv0 >> 16);
      bd[2 * x] = yuv_to_argb(by[2 * x], uv1 & 0xff, uv1 >> 16);
    }
    tl = t;
    l = uv;
  }
  if (!(len & 1)) {
    {
      const uint32_t uv0 = (3 * tl + l + 0x00020002u) >> 2;
      td[len - 1] = yuv_to_argb(ty[len - 1], uv0 & 0xff, uv0 >> 16);
    }
    if (by) {
      const uint32_t uv0 = (3 * l + tl + 0x00020002u) >> 2;
      bd[len - 1] = yuv_to_argb(by[len - 1], uv0 & 0xff, uv0 >> 16);
    }
  }
}

int WebPPictureYUVAToARGB(WebPPicture* pic) {
  if (pic == NULL) return 0;
  if (pic->y == NULL || pic->u == NULL || pic->v == NULL)
    return vp8h_pic_error(pic, VP8_ENC_ERROR_NULL_PARAMETER);
  if ((pic->colorspace & WEBP_CSP_ALPHA_BIT) && pic->a == NULL)
    return vp8h_pic_error(pic, VP8_ENC_ERROR_NULL_PARAMETER);
  if ((pic->colorspace & WEBP_CSP_UV_MASK) != WEBP_YUV420)
    return vp8h_pic_error(pic, VP8_ENC_ERROR_INVALID_CONFIGURATION);
  if (!vp8h_pic_alloc_argb(pic)) return 0;
  pic->use_argb = 1;
  const int w = pic->width, h = pic->height;
  uint32_t* dst = pic->argb;
  const uint8_t *cu = pic->u, *cv = pic->v, *cy = pic->y;
  upsample_pair(cy, NULL, cu, cv, cu, cv, dst, NULL, w);   /* first row */
  cy += pic->y_stride;
  dst += pic->argb_stride;
  for (int y = 1; y + 1 < h; y += 2) {
    const uint8_t *tu = cu, *tv = cv;
    cu += pic->uv_stride;
    cv += pic->uv_stride;
    upsample_pair(cy, cy + pic->y_stride, tu, tv, cu, cv, dst, dst + pic->argb_stride, w);
    cy += 2 * pic->y_stride;
    dst += 2 * pic->argb_stride;
  }
  if (h > 1 && !(h & 1)) upsample_pair(cy, NULL, cu, cv, cu, cv, dst, NULL, w);
  if (pic->colorspace & WEBP_CSP_ALPHA_BIT)
    for (int y = 0; y < h; ++y) {
      uint32_t* d = pic->argb + y * pic->argb_stride;
      const uint8_t* a = pic->a + y * pic->a_stride;
      for (int x = 0; x < w; ++x) d[x] = (d[x] & 0x00ffffffu) | ((uint32_t)a[x] << 24);
    }
  return 1;
}

/* ---- distortion: src/enc/picture_psnr_enc.c:24-224, src/dsp/ssim.c ---- */

static const uint32_t kSsimW[7] = {1, 2, 3, 4, 3, 2, 1};

static double ssim_from_stats(uint32_t w, uint32_t xm, uint32_t ym, uint32_t xxm, uint32_t xym,
                              uint32_t yym, uint32_t N) {   /* ssim.c:30-53 */
  const uint32_t w2 = N * N, C1 = 20 * w2, C2 = 60 * w2, C3 = 8 * 8 * w2;
  const uint64_t xmxm = (uint64_t)xm * xm, ymym = (uint64_t)ym * ym;
  (void)w;
  if (xmxm + ymym >= C3) {
    const int64_t xmym = (int64_t)xm * ym;
    const int64_t sxy = (int64_t)xym * N - xmym;
    const uint64_t sxx = (uint64_t)xxm * N - xmxm, syy = (uint64_t)yym * N - ymym;
    const uint64_t num_S = (2 * (uint64_t)(sxy < 0 ? 0 : sxy) + C2) >> 8;
    const uint64_t den_S = (sxx + syy + C2) >> 8;
    const uint64_t fnum = (2 * xmym + C1) * num_S, fden = (xmxm + ymym + C1) * den_S;
    return (double)fnum / fden;
  }
  return 1.;
}

/* one SSIM sample centred on (xo, yo), window clipped to the plane
 * (ssim.c:63-110; the unclipped interior variant is the same arithmetic
 * with w = 256) */
static double ssim_at(const uint8_t* s1, int st1, const uint8_t* s2, int st2, int xo, int yo,
                      int W, int H) {
  uint32_t w = 0, xm = 0, ym = 0, xxm = 0, xym = 0, yym = 0;
  const int ymin = yo - 3 < 0 ? 0 : yo - 3, ymax = yo + 3 > H - 1 ? H - 1 : yo + 3;
  const int xmin = xo - 3 < 0 ? 0 : xo - 3, xmax = xo + 3 > W - 1 ? W - 1 : xo + 3;
  for (int y = ymin; y <= ymax; ++y)
    for (int x = xmin; x <= xmax; ++x) {
      const uint32_t k = kSsimW[3 + x - xo] * kSsimW[3 + y - yo];
      const uint32_t a = s1[y * st1 + x], b = s2[y * st2 + x];
      w += k;
      xm += k * a;
      ym += k * b;
      xxm += k * a * a;
      xym += k * a * b;
      yym += k * b * b;
    }
  return ssim_from_stats(w, xm, ym, xxm, xym, yym, w);
}

static double acc_ssim(const uint8_t* s, int ss, const uint8_t* r, int rs, int w, int h) {
  double sum = 0.;   /* raster order, as picture_psnr_enc.c:76-110 visits */
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) sum += ssim_at(s, ss, r, rs, x, y, w, h);
  return sum;
}

static double acc_sse(const uint8_t* s, int ss, const uint8_t* r, int rs, int w, int h) {
  double total = 0.;   /* :62-73, per-row uint32 sums (ssim.c:117-129) */
  for (int y = 0; y < h; ++y) {
    uint32_t row = 0;
    for (int x = 0; x < w; ++x) {
      const int d = s[y * ss + x] - r[y * rs + x];
      row += (uint32_t)(d * d);
    }
    total += row;
  }
  return total;
}

static double acc_lsim(const uint8_t* s, int ss, const uint8_t* r, int rs, int w, int h) {
  double total = 0.;   /* :34-59, radius 2 */
  for (int y = 0; y < h; ++y) {
    const int y0 = y - 2 < 0 ? 0 : y - 2, y1 = y + 3 >= h ? h : y + 3;
    for (int x = 0; x < w; ++x) {
      const int x0 = x - 2 < 0 ? 0 : x - 2, x1 = x + 3 >= w ? w : x + 3;
      double best = 255. * 255.;
      const double value = (double)r[y * rs + x];
      for (int j = y0; j < y1; ++j)
        for (int i = x0; i < x1; ++i) {
          const double d = s[j * ss + i] - value;
          if (d * d < best) best = d * d;
        }
      total += best;
    }
  }
  return total;
}

static double get_psnr(double v, double size) {   /* :117-120 */
  return (v > 0. && size > 0.) ? -4.3429448 * log(v / (size * 255 * 255.)) : 99.;
}
static double get_log_ssim(double v, double size) {   /* :122-125 */
  v = (size > 0.) ? v / size : 1.;
  return (v < 1.) ? -10.0 * log10(1. - v) : 99.;
}

int WebPPlaneDistortion(const uint8_t* src, size_t src_stride, const uint8_t* ref,
                        size_t ref_stride, int width, int height, size_t x_step, int type,
                        float* distortion, float* result) {   /* :127-163 */
  uint8_t* tmp = NULL;
  if (src == NULL || ref == NULL || src_stride < x_step * width || ref_stride < x_step * width ||
      result == NULL || distortion == NULL)
    return 0;
  if (x_step != 1) {   /* extract packed planes */
    tmp = (uint8_t*)malloc(2 * (size_t)width * height);
    if (tmp == NULL) return 0;
    for (int y = 0; y < height; ++y)
      for (int x = 0; x < width; ++x) {
        tmp[x + (size_t)y * width] = src[x * x_step + y * src_stride];
        tmp[(size_t)width * height + x + (size_t)y * width] = ref[x * x_step + y * ref_stride];
      }
    src = tmp;
    ref = tmp + (size_t)width * height;
  }
  /* the metric always walks rows of `width` bytes (:155), whatever the
   * strides given for x_step == 1 */
  const double d = type == 0 ? acc_sse(src, width, ref, width, width, height)
                 : type == 1 ? acc_ssim(src, width, ref, width, width, height)
                             : acc_lsim(src, width, ref, width, width, height);
  *distortion = (float)d;
  free(tmp);
  *result = type == 1 ? (float)get_log_ssim(*distortion, (double)width * height)
                      : (float)get_psnr(*distortion, (double)width * height);
  return 1;
}

int WebPPictureDistortion(const WebPPicture* src, const WebPPicture* ref, int type,
                          float results[5]) {   /* :172-224 */
  WebPPicture p0, p1;
  double total_size = 0., total_d = 0.;
  int ok = 0;
  if (src == NULL || ref == NULL || src->width != ref->width || src->height != ref->height ||
      results == NULL)
    return 0;
  if (!WebPPictureInitInternal(&p0, WEBP_ENCODER_ABI_VERSION) ||
      !WebPPictureInitInternal(&p1, WEBP_ENCODER_ABI_VERSION))
    return 0;
  const int w = src->width, h = src->height;
  if (!WebPPictureView(src, 0, 0, w, h, &p0)) goto Error;
  if (!WebPPictureView(ref, 0, 0, w, h, &p1)) goto Error;
  if (p0.use_argb == 0 && !WebPPictureYUVAToARGB(&p0)) goto Error;
  if (p1.use_argb == 0 && !WebPPictureYUVAToARGB(&p1)) goto Error;
  for (int c = 0; c < 4; ++c) {   /* results in B, G, R, A order (little endian) */
    float d;
    if (!WebPPlaneDistortion((const uint8_t*)p0.argb + c, 4 * (size_t)p0.argb_stride,
                             (const uint8_t*)p1.argb + c, 4 * (size_t)p1.argb_stride, w, h, 4,
                             type, &d, results + c))
      goto Error;
    total_d += d;
    total_size += w * h;
  }
  results[4] = type == 1 ? (float)get_log_ssim(total_d, total_size)
                         : (float)get_psnr(total_d, total_size);
  ok = 1;
Error:
  WebPPictureFree(&p0);
  WebPPictureFree(&p1);
  return ok;
}

/* ---- transparency helpers: src/enc/picture_tools_enc.c:19-270 ---- */

static int smoothen_block(const uint8_t* a, int as, uint8_t* y, int ys, int w, int h) {
  int sum = 0, count = 0;   /* :54-80 */
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i)
      if (a[j * as + i] != 0) {
        ++count;
        sum += y[j * ys + i];
      }
  if (count > 0 && count < w * h) {
    const uint8_t avg = (uint8_t)(sum / count);
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i)
        if (a[j * as + i] == 0) y[j * ys + i] = avg;
  }
  return count == 0;
}

static void flatten(uint8_t* p, int v, int stride, int size) {
  for (int j = 0; j < size; ++j) memset(p + j * stride, v, size);
}

void WebPCleanupTransparentArea(WebPPicture* pic) {   /* :95-168, 8x8 blocks */
  if (pic == NULL) return;
  const int bw = pic->width / 8, bh = pic->height / 8;
  if (pic->use_argb) {
    uint32_t value = 0;
    for (int by = 0; by < bh; ++by) {
      int need_reset = 1;
      for (int bx = 0; bx < bw; ++bx) {
        uint32_t* p = pic->argb + (by * pic->argb_stride + bx) * 8;
        int transparent = 1;
        for (int j = 0; j < 8 && transparent; ++j)
          for (int i = 0; i < 8; ++i)
            if (p[j * pic->argb_stride + i] & 0xff000000u) { transparent = 0; break; }
        if (transparent) {
          if (need_reset) {
            value = p[0];
            need_reset = 0;
          }
          for (int j = 0; j < 8; ++j)
            for (int i = 0; i < 8; ++i) p[j * pic->argb_stride + i] = value;
        } else {
          need_reset = 1;
        }
      }
    }
    return;
  }
  const int width = pic->width, height = pic->height;
  uint8_t *yp = pic->y, *up = pic->u, *vp = pic->v;
  const uint8_t* ap = pic->a;
  int values[3] = {0, 0, 0};
  if (ap == NULL || yp == NULL || up == NULL || vp == NULL) return;
  int y, x;
  for (y = 0; y + 8 <= height; y += 8) {
    int need_reset = 1;
    for (x = 0; x + 8 <= width; x += 8) {
      if (smoothen_block(ap + x, pic->a_stride, yp + x, pic->y_stride, 8, 8)) {
        if (need_reset) {
          values[0] = yp[x];
          values[1] = up[x >> 1];
          values[2] = vp[x >> 1];
          need_reset = 0;
        }
        flatten(yp + x, values[0], pic->y_stride, 8);
        flatten(up + (x >> 1), values[1], pic->uv_stride, 4);
        flatten(vp + (x >> 1), values[2], pic->uv_stride, 4);
      } else {
        need_reset = 1;
      }
    }
    if (x < width) smoothen_block(ap + x, pic->a_stride, yp + x, pic->y_stride, width - x, 8);
    ap += 8 * pic->a_stride;
    yp += 8 * pic->y_stride;
    up += 4 * pic->uv_stride;
    vp += 4 * pic->uv_stride;
  }
  if (y < height) {
    const int sub = height - y;
    for (x = 0; x + 8 <= width; x += 8)
      smoothen_block(ap + x, pic->a_stride, yp + x, pic->y_stride, 8, sub);
    if (x < width) smoothen_block(ap + x, pic->a_stride, yp + x, pic->y_stride, width - x, sub);
  }
}

#define BLEND(V0, V1, A) ((((V0) * (255 - (A)) + (V1) * (A)) * 0x101 + 256) >> 16)
#define BLEND_10BIT(V0, V1, A) ((((V0) * (1020 - (A)) + (V1) * (A)) * 0x101 + 1024) >> 18)

void WebPBlendAlpha(WebPPicture* pic, uint32_t background_rgb) {   /* :180-270 */
  const int red = (background_rgb >> 16) & 0xff, green = (background_rgb >> 8) & 0xff,
            blue = background_rgb & 0xff;
  if (pic == NULL) return;
  if (!pic->use_argb) {
    const int uv_width = pic->width >> 1;
    /* VP8RGBToY/U/V (yuv.h:186-204) of the background; U/V on 4x sums */
    const int Y0 = (16839 * red + 33059 * green + 6420 * blue + (1 << 15) + (16 << 16)) >> 16;
    int U0 = -9719 * 4 * red - 19081 * 4 * green + 28800 * 4 * blue;
    int V0 = 28800 * 4 * red - 24116 * 4 * green - 4684 * 4 * blue;
    U0 = (U0 + 4 * (1 << 15) + (128 << 18)) >> 18;
    V0 = (V0 + 4 * (1 << 15) + (128 << 18)) >> 18;
    U0 = (U0 & ~0xff) == 0 ? U0 : U0 < 0 ? 0 : 255;
    V0 = (V0 & ~0xff) == 0 ? V0 : V0 < 0 ? 0 : 255;
    const int has_alpha = pic->colorspace & WEBP_CSP_ALPHA_BIT;
    uint8_t *yp = pic->y, *up = pic->u, *vp = pic->v, *ap = pic->a;
    if (!has_alpha || ap == NULL) return;
    for (int y = 0; y < pic->height; ++y) {
      for (int x = 0; x < pic->width; ++x) {
        const uint8_t a = ap[x];
        if (a < 0xff) yp[x] = BLEND(Y0, yp[x], a);
      }
      if ((y & 1) == 0) {
        const uint8_t* a2 = (y + 1 == pic->height) ? ap : ap + pic->a_stride;
        int x;
        for (x = 0; x < uv_width; ++x) {
          const uint32_t a = ap[2 * x] + ap[2 * x + 1] + a2[2 * x] + a2[2 * x + 1];
          up[x] = BLEND_10BIT(U0, up[x], a);
          vp[x] = BLEND_10BIT(V0, vp[x], a);
        }
        if (pic->width & 1) {
          const uint32_t a = 2 * (ap[2 * x] + a2[2 * x]);
          up[x] = BLEND_10BIT(U0, up[x], a);
          vp[x] = BLEND_10BIT(V0, vp[x], a);
        }
      } else {
        up += pic->uv_stride;
        vp += pic->uv_stride;
      }
      memset(ap, 0xff, pic->width);
      ap += pic->a_stride;
      yp += pic->y_stride;
    }
  } else {
    uint32_t* argb = pic->argb;
    const uint32_t bg = 0xff000000u | (red << 16) | (green << 8) | blue;
    for (int y = 0; y < pic->height; ++y, argb += pic->argb_stride)
      for (int x = 0; x < pic->width; ++x) {
        const int a = (argb[x] >> 24) & 0xff;
        if (a == 0xff) continue;
        if (a > 0) {
          const int r = BLEND(red, (argb[x] >> 16) & 0xff, a);
          const int g = BLEND(green, (argb[x] >> 8) & 0xff, a);
          const int b = BLEND(blue, argb[x] & 0xff, a);
          argb[x] = 0xff000000u | (r << 16) | (g << 8) | b;
        } else {
          argb[x] = bg;
        }
      }
  }
}
