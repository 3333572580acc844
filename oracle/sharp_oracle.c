/* Test infrastructure ONLY (see vp8_oracle.h): scalar CPU restatement of
 * libwebp v1.3.2's "sharp" (iterative) RGB -> YUV420 conversion as the lossy
 * encoder calls it (src/enc/picture_csp_enc.c:176-186: SharpYuvConvert with
 * 8-bit RGB in, 8-bit YUV out, the WebP matrix, sRGB transfer). Structure and
 * names are our own; each block cites the reference file:line it restates
 * (paths relative to the reference root). */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "vp8_oracle.h"

/* sRGB gamma tables, sharpyuv/sharpyuv_gamma.c:22-78 (built with double pow
 * exactly like the reference; 1024+2 gamma->linear, 512+2 linear->gamma) */
static uint32_t s_g2l[1024 + 2], s_l2g[512 + 2];
static volatile int s_ready = 0;

void vp8o_sharp_tables(uint32_t g2l[1026], uint32_t l2g[514]) {
  if (!s_ready) {
    const double a = 0.09929682680944, thresh = 0.018053968510807;
    const double gamma = 1. / 0.45, scale = 1 << 16;
    for (int v = 0; v <= 1024; ++v) {
      const double g = v / 1024.;
      const double x = (g <= thresh * 4.5) ? g / 4.5 : pow((g + a) / (1. + a), gamma);
      s_g2l[v] = (uint32_t)(x * scale + .5);
    }
    s_g2l[1025] = s_g2l[1024];
    for (int v = 0; v <= 512; ++v) {
      const double g = v / 512.;
      const double x = (g <= thresh) ? 4.5 * g : (1. + a) * pow(g, 1. / gamma) - a;
      s_l2g[v] = (uint32_t)(scale * x + .5);
    }
    s_l2g[513] = s_l2g[512];
    s_ready = 1;
  }
  if (g2l) memcpy(g2l, s_g2l, sizeof(s_g2l));
  if (l2g) memcpy(l2g, s_l2g, sizeof(s_l2g));
}

/* 10-bit working precision (8-bit input + 2, sharpyuv.c:44-49):
 * gamma->linear is a plain table read (sharpyuv_gamma.c:101-107, shift 0),
 * linear->gamma interpolates the 512-entry table (:84-99, :109-114). */
static inline uint32_t to_lin(int v) { return s_g2l[v]; }
static inline int to_gamma(uint32_t v) {
  const uint32_t pos = v >> 7, x = v - (pos << 7);
  const uint32_t v0 = s_l2g[pos] >> 6, v1 = s_l2g[pos + 1] >> 6;
  return (int)(v0 + (((v1 - v0) * x + 64) >> 7));
}
static inline int gray(int64_t r, int64_t g, int64_t b) {   /* sharpyuv.c:67-70 */
  return (int)((13933 * r + 46871 * g + 4732 * b + (1 << 15)) >> 16);
}
static inline int clip10(int v) { return v < 0 ? 0 : v > 1023 ? 1023 : v; }
static inline int clip8s(int v) {   /* clip_8b on an int16 (sharpyuv.c:56-58) */
  const int16_t s = (int16_t)v;
  return (!(s & ~0xff)) ? s : (s < 0) ? 0 : 255;
}

/* W (gray of the linearised pixel, re-gammaed): UpdateW, sharpyuv.c:85-101 */
static inline int wval(int r, int g, int b) {
  return to_gamma((uint32_t)gray(to_lin(r), to_lin(g), to_lin(b)));
}
/* one chroma sample from a 2x2 block of 10-bit RGB: UpdateChroma + ScaleDown,
 * sharpyuv.c:72-83, :103-128 */
static void chroma(const int p[4][3], int16_t out[3]) {
  int c[3];
  for (int k = 0; k < 3; ++k)
    c[k] = to_gamma((to_lin(p[0][k]) + to_lin(p[1][k]) + to_lin(p[2][k]) + to_lin(p[3][k]) + 2) >> 2);
  const int W = gray(c[0], c[1], c[2]);
  for (int k = 0; k < 3; ++k) out[k] = (int16_t)(c[k] - W);
}

/* RGB (R,G,B,x byte order, stride bytes) -> Y/U/V planes (strides w and
 * (w+1)/2). Returns 1. Pictures smaller than 4 in either dimension are not
 * sharp-converted by the reference (picture_csp_enc.c:165,493-496); the caller
 * handles that case. */
int vp8o_sharp_import_rgba(const uint8_t* rgba, int width, int height, int stride,
                           uint8_t* Y, uint8_t* U, uint8_t* V) {
  const int w = (width + 1) & ~1, h = (height + 1) & ~1;
  const int uvw = w >> 1, uvh = h >> 1;
  vp8o_sharp_tables(NULL, NULL);
  uint16_t* by = (uint16_t*)malloc(sizeof(uint16_t) * w * h);
  uint16_t* ty = (uint16_t*)malloc(sizeof(uint16_t) * w * h);
  int16_t* buv = (int16_t*)malloc(sizeof(int16_t) * 3 * uvw * uvh);
  int16_t* tuv = (int16_t*)malloc(sizeof(int16_t) * 3 * uvw * uvh);
  uint16_t* src = (uint16_t*)malloc(sizeof(uint16_t) * 6 * w);   /* 2 rows x RGB planes */
  if (!by || !ty || !buv || !tuv || !src) {
    free(by); free(ty); free(buv); free(tuv); free(src);
    return 0;
  }
  /* import: sharpyuv.c:152-180 (x4, replicate last column), :318-346 */
  for (int j = 0; j < uvh; ++j) {
    for (int r = 0; r < 2; ++r) {
      const int yy = (2 * j + r < height) ? 2 * j + r : height - 1;   /* odd last row: copy */
      const uint8_t* p = rgba + (size_t)yy * stride;
      uint16_t* d = src + r * 3 * w;
      for (int x = 0; x < w; ++x) {
        const int xx = x < width ? x : width - 1;
        for (int k = 0; k < 3; ++k) d[k * w + x] = (uint16_t)(p[4 * xx + k] << 2);
      }
      for (int x = 0; x < w; ++x) {
        const int R = d[x], G = d[w + x], B = d[2 * w + x];
        by[(2 * j + r) * w + x] = (uint16_t)gray(R, G, B);   /* StoreGray :130-136 */
        ty[(2 * j + r) * w + x] = (uint16_t)wval(R, G, B);
      }
    }
    for (int i = 0; i < uvw; ++i) {
      int p[4][3];
      for (int k = 0; k < 3; ++k) {
        p[0][k] = src[k * w + 2 * i];
        p[1][k] = src[k * w + 2 * i + 1];
        p[2][k] = src[3 * w + k * w + 2 * i];
        p[3][k] = src[3 * w + k * w + 2 * i + 1];
      }
      int16_t c[3];
      chroma(p, c);
      for (int k = 0; k < 3; ++k) tuv[(j * 3 + k) * uvw + i] = buv[(j * 3 + k) * uvw + i] = c[k];
    }
  }
  /* iterations: sharpyuv.c:348-418. best_uv is updated in place, so row
   * pair j interpolates with the *updated* row j-1 and the old rows j, j+1. */
  uint64_t prev_sum = ~0ULL;
  const uint64_t thresh = (uint64_t)(3.0 * w * h);
  int16_t* rgb_uv = (int16_t*)src;   /* reuse: 3 x uvw */
  uint16_t out[2][3][2];
  for (int iter = 0; iter < 4; ++iter) {
    uint64_t sum = 0;
    for (int j = 0; j < uvh; ++j) {
      const int16_t* prev = buv + 3 * uvw * (j > 0 ? j - 1 : 0);
      const int16_t* cur = buv + 3 * uvw * j;
      const int16_t* next = buv + 3 * uvw * (j < uvh - 1 ? j + 1 : j);
      /* per 2x2 block: InterpolateTwoRows (:182-219) + SharpYuvFilterRow_C
       * (sharpyuv_dsp.c:53-65) + Filter2 (:138-141) at both ends */
      for (int i = 0; i < uvw; ++i) {
        int px[4][3];
        for (int r = 0; r < 2; ++r) {
          const int16_t* B = r ? next : prev;
          for (int k = 0; k < 3; ++k) {
            const int16_t* A = cur + k * uvw;
            const int16_t* Bk = B + k * uvw;
            for (int s = 0; s < 2; ++s) {
              const int x = 2 * i + s;
              const int wy = by[(2 * j + r) * w + x];
              int v;
              if (x == 0 || x == w - 1) {
                v = ((A[i] * 3 + Bk[i] + 2) >> 2) + wy;
              } else if (s == 1) {   /* x = 1 + 2i: v0 of filter index i */
                v = wy + ((A[i] * 9 + A[i + 1] * 3 + Bk[i] * 3 + Bk[i + 1] + 8) >> 4);
              } else {               /* x = 2 + 2(i-1): v1 of filter index i-1 */
                v = wy + ((A[i] * 9 + A[i - 1] * 3 + Bk[i] * 3 + Bk[i - 1] + 8) >> 4);
              }
              px[2 * r + s][k] = clip10(v);
            }
          }
        }
        for (int r = 0; r < 2; ++r)
          for (int s = 0; s < 2; ++s) {
            /* SharpYuvUpdateY_C, sharpyuv_dsp.c:28-41 */
            const int idx = (2 * j + r) * w + 2 * i + s;
            const int d = ty[idx] - wval(px[2 * r + s][0], px[2 * r + s][1], px[2 * r + s][2]);
            by[idx] = (uint16_t)clip10(by[idx] + d);
            sum += (uint64_t)abs(d);
          }
        int16_t c[3];
        chroma(px, c);
        for (int k = 0; k < 3; ++k) rgb_uv[k * uvw + i] = c[k];
      }
      (void)out;
      /* SharpYuvUpdateRGB_C, sharpyuv_dsp.c:43-51 (in place, after the row
       * pair is interpolated) */
      for (int k = 0; k < 3; ++k)
        for (int i = 0; i < uvw; ++i) {
          const int t = (j * 3 + k) * uvw + i;
          buv[t] = (int16_t)(buv[t] + tuv[t] - rgb_uv[k * uvw + i]);
        }
    }
    if (iter > 0 && (sum < thresh || sum > prev_sum)) break;   /* :408-413 */
    prev_sum = sum;
  }
  /* ConvertWRGBToYUV, sharpyuv.c:221-268, with the WebP matrix
   * (sharpyuv_csp.c:62-66) rescaled for the 2 extra bits (:511-514) */
  for (int j = 0; j < height; ++j)
    for (int i = 0; i < width; ++i) {
      const int Wy = by[j * w + i];
      const int16_t* uv = buv + 3 * uvw * (j >> 1);
      const int r = uv[i >> 1] + Wy, g = uv[uvw + (i >> 1)] + Wy, b = uv[2 * uvw + (i >> 1)] + Wy;
      Y[(size_t)j * width + i] =
          (uint8_t)clip8s((16839 * r + 33059 * g + 6420 * b + (16 << 18) + (1 << 17)) >> 18);
    }
  for (int j = 0; j < uvh; ++j)
    for (int i = 0; i < uvw; ++i) {
      const int16_t* uv = buv + 3 * uvw * j;
      const int r = uv[i], g = uv[uvw + i], b = uv[2 * uvw + i];
      U[(size_t)j * uvw + i] =
          (uint8_t)clip8s((-9719 * r - 19081 * g + 28800 * b + (128 << 18) + (1 << 17)) >> 18);
      V[(size_t)j * uvw + i] =
          (uint8_t)clip8s((28800 * r - 24116 * g - 4684 * b + (128 << 18) + (1 << 17)) >> 18);
    }
  free(by); free(ty); free(buv); free(tuv); free(src);
  return 1;
}
