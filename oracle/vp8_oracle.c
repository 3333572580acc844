/* Test infrastructure ONLY (see vp8_oracle.h): scalar CPU restatement of the
 * libwebp v1.3.2 lossy encode path. Structure and names are our own; every
 * block cites the reference file:line whose behaviour it restates
 * (paths relative to the reference root, /root/reference). */
#include "vp8_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define VP8T_DECL static const
#include "vp8_tables.h"

#define BPS 32                    /* scratch stride, src/dsp/dsp.h:28 */
#define Y_BLK(n) (((n) >> 2) * 4 * BPS + ((n) & 3) * 4)
#define QFIX 17                   /* src/enc/vp8i_enc.h:112 */
#define MAX_LEVEL 2047            /* src/enc/vp8i_enc.h:39 */
#define MAX_VLEVEL 67             /* src/enc/vp8i_enc.h:38 */
#define MAX_COST ((int64_t)0x7fffffffffffffLL)   /* vp8i_enc.h:110 */
#define P0_LIMIT (((1ULL << 19) - 2048ULL) << 11) /* frame_enc.c:32 */

typedef int64_t score_t;

static int g_passes;   /* passes of the last encode (> 1: partition-0 retry) */
static uint64_t g_size_p0;   /* header estimate of the last pass (1/256 bit) */

static const uint8_t kZz[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
static const uint8_t kBand[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};

static inline int clip8(int v) { return (v & ~0xff) == 0 ? v : (v < 0 ? 0 : 255); }
static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
static inline int iabs(int v) { return v < 0 ? -v : v; }
static inline int bit_cost(int bit, int p) {      /* cost_enc.h:59-61 */
  return bit ? kVP8EntropyCost[255 - p] : kVP8EntropyCost[p];
}

/* ------------------------------------------------------------------------ */
/* RGBA -> YUV420, opaque path: src/enc/picture_csp_enc.c:103-138,375-457,
 * 474-619 and src/dsp/yuv.h:186-204 */

static uint16_t g_g2l[256];
static int g_l2g[33];
static volatile int g_gamma_ready = 0;

static void gamma_tables(void) {
  if (g_gamma_ready) return;
  const double scale = (double)(1 << 7) / 4095;
  const double norm = 1. / 255.;
  for (int v = 0; v < 256; ++v) g_g2l[v] = (uint16_t)(pow(norm * v, 0.80) * 4095 + .5);
  for (int v = 0; v <= 32; ++v) g_l2g[v] = (int)(255. * pow(scale * v, 1. / 0.80) + .5);
  g_gamma_ready = 1;
}

static inline int lin_to_gamma(uint32_t sum, int shift) {
  const int v = (int)(sum << shift);
  const int pos = v >> 9, frac = v & 511;
  const int y = g_l2g[pos + 1] * frac + g_l2g[pos] * (512 - frac);
  return (y + 64) >> 7;
}

static inline int rgb_to_y(int r, int g, int b) {
  return (16839 * r + 33059 * g + 6420 * b + (1 << 15) + (16 << 16)) >> 16;
}
static inline int clip_uv(int v) {
  v = (v + (1 << 17) + (128 << 18)) >> 18;
  return (v & ~0xff) == 0 ? v : (v < 0 ? 0 : 255);
}

int vp8o_import_rgba(const uint8_t* rgba, int w, int h, int stride,
                     uint8_t* Y, uint8_t* U, uint8_t* V) {
  const int uvw = (w + 1) >> 1;
  gamma_tables();
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i)
      if (rgba[j * stride + 4 * i + 3] != 0xff) return 0;
  for (int j = 0; j < h; ++j) {
    const uint8_t* p = rgba + j * stride;
    for (int i = 0; i < w; ++i) Y[j * w + i] = rgb_to_y(p[4 * i], p[4 * i + 1], p[4 * i + 2]);
  }
  for (int j = 0; j < (h + 1) >> 1; ++j) {
    const uint8_t* r0 = rgba + 2 * j * stride;
    /* the odd last row pairs with itself (rgb_stride = 0, :604-605) */
    const uint8_t* r1 = (2 * j + 1 < h) ? r0 + stride : r0;
    for (int i = 0; i < uvw; ++i) {
      int c[3];
      for (int k = 0; k < 3; ++k) {
        if (2 * i + 1 < w) {       /* SUM4 */
          const uint32_t s = g_g2l[r0[8 * i + k]] + g_g2l[r0[8 * i + 4 + k]] +
                             g_g2l[r1[8 * i + k]] + g_g2l[r1[8 * i + 4 + k]];
          c[k] = lin_to_gamma(s, 0);
        } else {                   /* SUM2: odd last column */
          const uint32_t s = g_g2l[r0[8 * i + k]] + g_g2l[r1[8 * i + k]];
          c[k] = lin_to_gamma(s, 1);
        }
      }
      U[j * uvw + i] = clip_uv(-9719 * c[0] - 19081 * c[1] + 28800 * c[2]);
      V[j * uvw + i] = clip_uv(28800 * c[0] - 24116 * c[1] - 4684 * c[2]);
    }
  }
  return 1;
}

/* Dithered import (WebPPictureARGBToYUVADithered, picture_csp_enc.c:520-619;
 * VP8Random, src/utils/random_utils.{h,c}; webp_enc.c:357-365 for the
 * amplitude of preprocessing & 2): the same conversion with the rounding
 * terms drawn from Knuth's difference generator, in the reference's order
 * (two luma rows, then the U,V pairs of their chroma row). Opaque input. */
typedef struct { int i1, i2, amp; uint32_t tab[55]; } Rng;
static const uint32_t kRngTable[55] = {
    0x0de15230, 0x03b31886, 0x775faccb, 0x1c88626a, 0x68385c55, 0x14b3b828, 0x4a85fef8,
    0x49ddb84b, 0x64fcf397, 0x5c550289, 0x4a290000, 0x0d7ec1da, 0x5940b7ab, 0x5492577d,
    0x4e19ca72, 0x38d38c69, 0x0c01ee65, 0x32a1755f, 0x5437f652, 0x5abb2c32, 0x0faa57b1,
    0x73f533e7, 0x685feeda, 0x7563cce2, 0x6e990e83, 0x4730a7ed, 0x4fc0d9c6, 0x496b153c,
    0x4f1403fa, 0x541afb0c, 0x73990b32, 0x26d7cb1c, 0x6fcc3706, 0x2cbb77d8, 0x75762f2a,
    0x6425ccdd, 0x24b35461, 0x0a7d8715, 0x220414a8, 0x141ebf67, 0x56b41583, 0x73e502e3,
    0x44cab16f, 0x28264d42, 0x73baaefb, 0x0a50ebed, 0x1d6ab6fb, 0x0d3ad40b, 0x35db3b68,
    0x2b081e83, 0x77ce6b95, 0x5181e5f0, 0x78853bbc, 0x009f9494, 0x27e5ed3c};
static int rng_bits(Rng* rg, int nb) {
  uint32_t d = rg->tab[rg->i1] - rg->tab[rg->i2];
  if ((int32_t)d < 0) d += 1u << 31;
  rg->tab[rg->i1] = d;
  rg->i1 = rg->i1 == 54 ? 0 : rg->i1 + 1;
  rg->i2 = rg->i2 == 54 ? 0 : rg->i2 + 1;
  int v = (int32_t)(d << 1) >> (32 - nb);
  v = (v * rg->amp) >> 8;
  return v + (1 << (nb - 1));
}

int vp8o_import_rgba_dithered(const uint8_t* rgba, int w, int h, int stride, float dithering,
                              uint8_t* Y, uint8_t* U, uint8_t* V) {
  const int uvw = (w + 1) >> 1;
  Rng rg;
  gamma_tables();
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i)
      if (rgba[j * stride + 4 * i + 3] != 0xff) return 0;
  memcpy(rg.tab, kRngTable, sizeof(rg.tab));
  rg.i1 = 0; rg.i2 = 31;
  rg.amp = dithering < 0.0 ? 0 : dithering > 1.0 ? 256 : (int)(uint32_t)(256 * dithering);
  for (int j = 0; j < (h + 1) >> 1; ++j) {
    for (int r = 2 * j; r < 2 * j + 2 && r < h; ++r) {
      const uint8_t* p = rgba + r * stride;
      for (int i = 0; i < w; ++i)
        Y[r * w + i] = (16839 * p[4 * i] + 33059 * p[4 * i + 1] + 6420 * p[4 * i + 2] +
                        rng_bits(&rg, 16) + (16 << 16)) >> 16;
    }
    const uint8_t* r0 = rgba + 2 * j * stride;
    const uint8_t* r1 = (2 * j + 1 < h) ? r0 + stride : r0;
    for (int i = 0; i < uvw; ++i) {
      int c[3];
      for (int k = 0; k < 3; ++k) {
        if (2 * i + 1 < w) {
          const uint32_t s = g_g2l[r0[8 * i + k]] + g_g2l[r0[8 * i + 4 + k]] +
                             g_g2l[r1[8 * i + k]] + g_g2l[r1[8 * i + 4 + k]];
          c[k] = lin_to_gamma(s, 0);
        } else {
          c[k] = lin_to_gamma(g_g2l[r0[8 * i + k]] + g_g2l[r1[8 * i + k]], 1);
        }
      }
      for (int ch = 0; ch < 2; ++ch) {   /* ConvertRowsToUV: U then V */
        const int uv = ch ? 28800 * c[0] - 24116 * c[1] - 4684 * c[2]
                          : -9719 * c[0] - 19081 * c[1] + 28800 * c[2];
        int v = (uv + rng_bits(&rg, 18) + (128 << 18)) >> 18;
        v = (v & ~0xff) == 0 ? v : (v < 0 ? 0 : 255);
        (ch ? V : U)[j * uvw + i] = (uint8_t)v;
      }
    }
  }
  return 1;
}

/* ------------------------------------------------------------------------ */
/* Boolean coder: src/utils/bit_writer_utils.c:26-179 */

typedef struct {
  int32_t range, value;
  int run, nb_bits;
  uint8_t* buf;
  size_t pos, cap;
  int error;
} BW;

static void bw_init(BW* b) {
  memset(b, 0, sizeof(*b));
  b->range = 254;
  b->nb_bits = -8;
}

static int bw_reserve(BW* b, size_t extra) {
  if (b->pos + extra <= b->cap) return 1;
  size_t n = b->cap * 2;
  if (n < b->pos + extra) n = b->pos + extra;
  if (n < 1024) n = 1024;
  uint8_t* nb = (uint8_t*)realloc(b->buf, n);
  if (!nb) { b->error = 1; return 0; }
  b->buf = nb;
  b->cap = n;
  return 1;
}

static void bw_flush(BW* b) {
  const int s = 8 + b->nb_bits;
  const int32_t bits = b->value >> s;
  b->value -= bits << s;
  b->nb_bits -= 8;
  if ((bits & 0xff) != 0xff) {
    size_t pos = b->pos;
    if (!bw_reserve(b, b->run + 1)) return;
    if ((bits & 0x100) && pos > 0) b->buf[pos - 1]++;
    for (; b->run > 0; --b->run) b->buf[pos++] = (bits & 0x100) ? 0x00 : 0xff;
    b->buf[pos++] = bits & 0xff;
    b->pos = pos;
  } else {
    b->run++;
  }
}

/* renormalisation: shift so that range >= 127 (kNorm / kNewRange, :83-106) */
static inline void bw_renorm(BW* b) {
  if (b->range < 127) {
    const int shift = __builtin_clz((unsigned)(b->range + 1)) - 24;  /* 7-log2(r+1) */
    b->range = ((b->range + 1) << shift) - 1;
    b->value <<= shift;
    b->nb_bits += shift;
    if (b->nb_bits > 0) bw_flush(b);
  }
}

static int bw_put(BW* b, int bit, int prob) {
  const int split = (b->range * prob) >> 8;
  if (bit) { b->value += split + 1; b->range -= split + 1; }
  else { b->range = split; }
  bw_renorm(b);
  return bit;
}

static int bw_put_uniform(BW* b, int bit) {
  const int split = b->range >> 1;
  if (bit) { b->value += split + 1; b->range -= split + 1; }
  else { b->range = split; }
  bw_renorm(b);
  return bit;
}

static void bw_put_bits(BW* b, uint32_t v, int n) {
  for (uint32_t m = 1u << (n - 1); m; m >>= 1) bw_put_uniform(b, (v & m) != 0);
}

static void bw_put_signed(BW* b, int v, int n) {
  if (!bw_put_uniform(b, v != 0)) return;
  if (v < 0) bw_put_bits(b, ((-v) << 1) | 1, n + 1);
  else bw_put_bits(b, v << 1, n + 1);
}

static void bw_finish(BW* b) {
  bw_put_bits(b, 0, 9 - b->nb_bits);
  b->nb_bits = 0;
  bw_flush(b);
}

/* ------------------------------------------------------------------------ */
/* 4x4 transforms: src/dsp/enc.c:112-222, src/dsp/dec.c:137-162 */

static void fdct4(const uint8_t* src, int ss, const uint8_t* ref, int rs, int16_t out[16]) {
  int t[16];
  for (int i = 0; i < 4; ++i) {
    const int d0 = src[i * ss + 0] - ref[i * rs + 0];
    const int d1 = src[i * ss + 1] - ref[i * rs + 1];
    const int d2 = src[i * ss + 2] - ref[i * rs + 2];
    const int d3 = src[i * ss + 3] - ref[i * rs + 3];
    const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
    t[4 * i + 0] = (a0 + a1) * 8;
    t[4 * i + 1] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
    t[4 * i + 2] = (a0 - a1) * 8;
    t[4 * i + 3] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
  }
  for (int i = 0; i < 4; ++i) {
    const int a0 = t[i] + t[12 + i], a1 = t[4 + i] + t[8 + i];
    const int a2 = t[4 + i] - t[8 + i], a3 = t[i] - t[12 + i];
    out[i] = (int16_t)((a0 + a1 + 7) >> 4);
    out[4 + i] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
    out[8 + i] = (int16_t)((a0 - a1 + 7) >> 4);
    out[12 + i] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
  }
}

#define IMUL(a, b) (((a) * (b)) >> 16)
static void idct4(const uint8_t* ref, int rs, const int16_t in[16], uint8_t* dst, int ds) {
  const int c1 = 20091 + (1 << 16), c2 = 35468;
  int t[16];
  for (int i = 0; i < 4; ++i) {          /* columns */
    const int a = in[i] + in[8 + i], b = in[i] - in[8 + i];
    const int c = IMUL(in[4 + i], c2) - IMUL(in[12 + i], c1);
    const int d = IMUL(in[4 + i], c1) + IMUL(in[12 + i], c2);
    t[4 * i + 0] = a + d; t[4 * i + 1] = b + c;
    t[4 * i + 2] = b - c; t[4 * i + 3] = a - d;
  }
  for (int i = 0; i < 4; ++i) {          /* rows */
    const int dc = t[i] + 4;
    const int a = dc + t[8 + i], b = dc - t[8 + i];
    const int c = IMUL(t[4 + i], c2) - IMUL(t[12 + i], c1);
    const int d = IMUL(t[4 + i], c1) + IMUL(t[12 + i], c2);
    const int v[4] = {a + d, b + c, b - c, a - d};
    for (int k = 0; k < 4; ++k) dst[i * ds + k] = clip8(ref[i * rs + k] + (v[k] >> 3));
  }
}

/* forward WHT over the 16 luma DCs (dc[k] = DC of block k, raster order) */
static void fwht(const int16_t dc[16], int16_t out[16]) {
  int t[16];
  for (int i = 0; i < 4; ++i) {
    const int a0 = dc[4 * i + 0] + dc[4 * i + 2], a1 = dc[4 * i + 1] + dc[4 * i + 3];
    const int a2 = dc[4 * i + 1] - dc[4 * i + 3], a3 = dc[4 * i + 0] - dc[4 * i + 2];
    t[4 * i + 0] = a0 + a1; t[4 * i + 1] = a3 + a2;
    t[4 * i + 2] = a3 - a2; t[4 * i + 3] = a0 - a1;
  }
  for (int i = 0; i < 4; ++i) {
    const int a0 = t[i] + t[8 + i], a1 = t[4 + i] + t[12 + i];
    const int a2 = t[4 + i] - t[12 + i], a3 = t[i] - t[8 + i];
    out[i] = (int16_t)((a0 + a1) >> 1);
    out[4 + i] = (int16_t)((a3 + a2) >> 1);
    out[8 + i] = (int16_t)((a3 - a2) >> 1);
    out[12 + i] = (int16_t)((a0 - a1) >> 1);
  }
}

/* inverse WHT: returns the 16 per-block DCs in raster block order */
static void iwht(const int16_t in[16], int16_t dc[16]) {
  int t[16];
  for (int i = 0; i < 4; ++i) {
    const int a0 = in[i] + in[12 + i], a1 = in[4 + i] + in[8 + i];
    const int a2 = in[4 + i] - in[8 + i], a3 = in[i] - in[12 + i];
    t[i] = a0 + a1; t[8 + i] = a0 - a1;
    t[4 + i] = a3 + a2; t[12 + i] = a3 - a2;
  }
  for (int i = 0; i < 4; ++i) {
    const int d = t[4 * i] + 3;
    const int a0 = d + t[4 * i + 3], a1 = t[4 * i + 1] + t[4 * i + 2];
    const int a2 = t[4 * i + 1] - t[4 * i + 2], a3 = d - t[4 * i + 3];
    dc[4 * i + 0] = (int16_t)((a0 + a1) >> 3);
    dc[4 * i + 1] = (int16_t)((a3 + a2) >> 3);
    dc[4 * i + 2] = (int16_t)((a0 - a1) >> 3);
    dc[4 * i + 3] = (int16_t)((a3 - a2) >> 3);
  }
}

static int sse(const uint8_t* a, int as, const uint8_t* b, int bs, int w, int h) {
  int s = 0;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) { const int d = a[y * as + x] - b[y * bs + x]; s += d * d; }
  return s;
}

/* Hadamard "texture" measure, src/dsp/enc.c:590-641 */
static int hadamard_w(const uint8_t* in, int st, const uint16_t* w) {
  int t[16], sum = 0;
  for (int i = 0; i < 4; ++i) {
    const uint8_t* p = in + i * st;
    const int a0 = p[0] + p[2], a1 = p[1] + p[3], a2 = p[1] - p[3], a3 = p[0] - p[2];
    t[4 * i + 0] = a0 + a1; t[4 * i + 1] = a3 + a2;
    t[4 * i + 2] = a3 - a2; t[4 * i + 3] = a0 - a1;
  }
  for (int i = 0; i < 4; ++i) {
    const int a0 = t[i] + t[8 + i], a1 = t[4 + i] + t[12 + i];
    const int a2 = t[4 + i] - t[12 + i], a3 = t[i] - t[8 + i];
    sum += w[i] * iabs(a0 + a1) + w[4 + i] * iabs(a3 + a2) +
           w[8 + i] * iabs(a3 - a2) + w[12 + i] * iabs(a0 - a1);
  }
  return sum;
}
static int tdisto4(const uint8_t* a, int as, const uint8_t* b, int bs) {
  return iabs(hadamard_w(b, bs, kVP8WeightY) - hadamard_w(a, as, kVP8WeightY)) >> 5;
}
static int tdisto16(const uint8_t* a, int as, const uint8_t* b, int bs) {
  int d = 0;
  for (int y = 0; y < 16; y += 4)
    for (int x = 0; x < 16; x += 4) d += tdisto4(a + y * as + x, as, b + y * bs + x, bs);
  return d;
}

/* ------------------------------------------------------------------------ */
/* Intra predictors: src/dsp/enc.c:231-531 (NULL edge = missing neighbour) */

static void fill(uint8_t* d, int ds, int v, int n) {
  for (int y = 0; y < n; ++y) memset(d + y * ds, v, n);
}
static void pred_v(uint8_t* d, int ds, const uint8_t* top, int n) {
  if (!top) { fill(d, ds, 127, n); return; }
  for (int y = 0; y < n; ++y) memcpy(d + y * ds, top, n);
}
static void pred_h(uint8_t* d, int ds, const uint8_t* left, int n) {
  if (!left) { fill(d, ds, 129, n); return; }
  for (int y = 0; y < n; ++y) memset(d + y * ds, left[y], n);
}
static void pred_tm(uint8_t* d, int ds, const uint8_t* left, const uint8_t* top, int n) {
  if (left && top) {
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x) d[y * ds + x] = clip8(top[x] + left[y] - left[-1]);
  } else if (left) {
    pred_h(d, ds, left, n);
  } else if (top) {
    pred_v(d, ds, top, n);
  } else {
    fill(d, ds, 129, n);
  }
}
static void pred_dc(uint8_t* d, int ds, const uint8_t* left, const uint8_t* top, int n, int shift) {
  int dc = 0;
  if (top) {
    for (int j = 0; j < n; ++j) dc += top[j];
    if (left) { for (int j = 0; j < n; ++j) dc += left[j]; }
    else dc += dc;
    dc = (dc + n) >> shift;
  } else if (left) {
    for (int j = 0; j < n; ++j) dc += left[j];
    dc += dc;
    dc = (dc + n) >> shift;
  } else {
    dc = 0x80;
  }
  fill(d, ds, dc, n);
}

/* 16x16 luma: 4 modes in DC, TM, VE, HE order; d[m] is 16x16 stride 16 */
static void preds16(uint8_t d[4][256], const uint8_t* left, const uint8_t* top) {
  pred_dc(d[0], 16, left, top, 16, 5);
  pred_tm(d[1], 16, left, top, 16);
  pred_v(d[2], 16, top, 16);
  pred_h(d[3], 16, left, 16);
}
/* chroma: d[m] is 16 wide (U | V) x 8 rows, stride 16 */
static void preds_uv(uint8_t d[4][128], const uint8_t* uleft, const uint8_t* vleft,
                     const uint8_t* top) {
  for (int c = 0; c < 2; ++c) {
    const uint8_t* l = uleft ? (c ? vleft : uleft) : NULL;
    const uint8_t* t = top ? top + 8 * c : NULL;
    pred_dc(d[0] + 8 * c, 16, l, t, 8, 4);
    pred_tm(d[1] + 8 * c, 16, l, t, 8);
    pred_v(d[2] + 8 * c, 16, t, 8);
    pred_h(d[3] + 8 * c, 16, l, 8);
  }
}

#define AVG3(a, b, c) (((a) + 2 * (b) + (c) + 2) >> 2)
#define AVG2(a, b) (((a) + (b) + 1) >> 1)
/* e[0..12] = L K J I X A B C D E F G H (left bottom->top, corner, top, top-right);
 * out[m][16] = 4x4 prediction of mode m (B_DC..B_HU order) */
static void preds4(uint8_t out[10][16], const uint8_t e[13]) {
  const int L = e[0], K = e[1], J = e[2], I = e[3], X = e[4];
  const int A = e[5], B = e[6], C = e[7], D = e[8], E = e[9], F = e[10], G = e[11], H = e[12];
  uint8_t* p;
#define P(x, y) p[(y) * 4 + (x)]
  { int dc = 4; for (int i = 0; i < 4; ++i) dc += e[5 + i] + e[i];
    memset(out[0], dc >> 3, 16); }
  p = out[1];
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) P(x, y) = clip8(e[5 + x] + e[3 - y] - X);
  p = out[2];
  for (int y = 0; y < 4; ++y) {
    P(0, y) = AVG3(X, A, B); P(1, y) = AVG3(A, B, C);
    P(2, y) = AVG3(B, C, D); P(3, y) = AVG3(C, D, E);
  }
  p = out[3];
  { const int r[4] = {AVG3(X, I, J), AVG3(I, J, K), AVG3(J, K, L), AVG3(K, L, L)};
    for (int y = 0; y < 4; ++y) memset(p + 4 * y, r[y], 4); }
  p = out[4];   /* RD */
  P(0, 3) = AVG3(J, K, L);
  P(0, 2) = P(1, 3) = AVG3(I, J, K);
  P(0, 1) = P(1, 2) = P(2, 3) = AVG3(X, I, J);
  P(0, 0) = P(1, 1) = P(2, 2) = P(3, 3) = AVG3(A, X, I);
  P(1, 0) = P(2, 1) = P(3, 2) = AVG3(B, A, X);
  P(2, 0) = P(3, 1) = AVG3(C, B, A);
  P(3, 0) = AVG3(D, C, B);
  p = out[5];   /* VR */
  P(0, 0) = P(1, 2) = AVG2(X, A);
  P(1, 0) = P(2, 2) = AVG2(A, B);
  P(2, 0) = P(3, 2) = AVG2(B, C);
  P(3, 0) = AVG2(C, D);
  P(0, 3) = AVG3(K, J, I);
  P(0, 2) = AVG3(J, I, X);
  P(0, 1) = P(1, 3) = AVG3(I, X, A);
  P(1, 1) = P(2, 3) = AVG3(X, A, B);
  P(2, 1) = P(3, 3) = AVG3(A, B, C);
  P(3, 1) = AVG3(B, C, D);
  p = out[6];   /* LD */
  P(0, 0) = AVG3(A, B, C);
  P(1, 0) = P(0, 1) = AVG3(B, C, D);
  P(2, 0) = P(1, 1) = P(0, 2) = AVG3(C, D, E);
  P(3, 0) = P(2, 1) = P(1, 2) = P(0, 3) = AVG3(D, E, F);
  P(3, 1) = P(2, 2) = P(1, 3) = AVG3(E, F, G);
  P(3, 2) = P(2, 3) = AVG3(F, G, H);
  P(3, 3) = AVG3(G, H, H);
  p = out[7];   /* VL */
  P(0, 0) = AVG2(A, B);
  P(1, 0) = P(0, 2) = AVG2(B, C);
  P(2, 0) = P(1, 2) = AVG2(C, D);
  P(3, 0) = P(2, 2) = AVG2(D, E);
  P(0, 1) = AVG3(A, B, C);
  P(1, 1) = P(0, 3) = AVG3(B, C, D);
  P(2, 1) = P(1, 3) = AVG3(C, D, E);
  P(3, 1) = P(2, 3) = AVG3(D, E, F);
  P(3, 2) = AVG3(E, F, G);
  P(3, 3) = AVG3(F, G, H);
  p = out[8];   /* HD */
  P(0, 0) = P(2, 1) = AVG2(I, X);
  P(0, 1) = P(2, 2) = AVG2(J, I);
  P(0, 2) = P(2, 3) = AVG2(K, J);
  P(0, 3) = AVG2(L, K);
  P(3, 0) = AVG3(A, B, C);
  P(2, 0) = AVG3(X, A, B);
  P(1, 0) = P(3, 1) = AVG3(I, X, A);
  P(1, 1) = P(3, 2) = AVG3(J, I, X);
  P(1, 2) = P(3, 3) = AVG3(K, J, I);
  P(1, 3) = AVG3(L, K, J);
  p = out[9];   /* HU */
  P(0, 0) = AVG2(I, J);
  P(2, 0) = P(0, 1) = AVG2(J, K);
  P(2, 1) = P(0, 2) = AVG2(K, L);
  P(1, 0) = AVG3(I, J, K);
  P(3, 0) = P(1, 1) = AVG3(J, K, L);
  P(3, 1) = P(1, 2) = AVG3(K, L, L);
  P(3, 2) = P(2, 2) = P(0, 3) = P(1, 3) = P(2, 3) = P(3, 3) = L;
#undef P
}
#undef AVG3
#undef AVG2

/* ------------------------------------------------------------------------ */
/* Encoder state (the subset of src/enc/vp8i_enc.h:140-413 that the lossy
 * token path reads) */

typedef struct {
  uint16_t q[16], iq[16];
  uint32_t bias[16], zthresh[16];
  uint16_t sharpen[16];
} Mtx;

typedef struct {
  Mtx y1, y2, uv;
  int alpha, beta, quant, fstrength, max_edge, min_disto, i4_penalty;
  int lambda_i16, lambda_i4, lambda_uv, lambda_mode, tlambda;
  int lambda_trellis_i16, lambda_trellis_i4, lambda_trellis_uv;
} Seg;

typedef struct {
  const uint8_t *Y, *U, *V;
  int ys, uvs, w, h, mbw, mbh;
  vp8o_config cfg;
  int method, rd_opt;           /* rd_opt: 1 basic, 2 trellis-final, 3 trellis-all */
  int max_i4_header_bits;
  /* per-MB info */
  uint8_t *mb_type, *mb_uv, *mb_skip, *mb_seg, *mb_alpha;
  uint8_t* preds_mem; uint8_t* preds; int preds_w;
  uint32_t* nz_mem; uint32_t* nz;   /* nz[-1] == 0 */
  uint8_t *y_top, *uv_top;
  int8_t (*top_derr)[2][2];
  /* segment / quant */
  Seg dqm[4];
  int num_segments, update_map, seg_hdr_size;
  uint8_t seg_probas[3];
  int base_quant, alpha, uv_alpha, dq_uv_dc, dq_uv_ac;
  /* filter header */
  int f_simple, f_level, f_sharpness;
  /* probabilities */
  uint8_t coeffs[4][8][3][11];
  uint32_t stats[4][8][3][11];
  uint16_t lcost[4][8][3][MAX_VLEVEL + 1];
  int dirty;
  /* token buffer */
  uint16_t* tok; size_t ntok, tcap;
  int tok_err;
  int no_tokens, no_stats;       /* RecordResiduals (stats only) / CodeResiduals (tokens only) */
  /* VP8EncLoop (m0-2): skip probability (frame_enc.c:99-127) */
  int nb_skip, use_skip, skip_proba;
  score_t mb_header_limit;
  /* token partitions (webp_enc.c:115-122, 209; iterator_enc.c:48): row y's
   * tokens go to partition y & (num_parts - 1); row_tok[y] = the row's first
   * token in the final pass */
  int num_parts;
  size_t* row_tok;
} Enc;

typedef struct {
  int x, y;
  uint8_t yin[BPS * 16], yout[BPS * 16], yout2[BPS * 16];
  uint8_t* out;  uint8_t* out2;      /* swap-able views on yout/yout2 */
  uint8_t p16[4][256], puv[4][128];
  uint8_t yl_mem[17], ul_mem[9], vl_mem[9];
  uint8_t *yl, *ul, *vl;             /* index -1 valid (top-left) */
  const uint8_t *ytop, *uvtop;
  int top_nz[9], left_nz[9];
  int8_t lderr[2][2];
  int do_trellis;
  uint8_t* preds;                    /* this MB's entry in the 4x4 mode plane */
  uint32_t* nz;                      /* this MB's column in the nz context row */
} It;

typedef struct {
  score_t D, SD, H, R, score;
  int16_t y_dc[16], y_ac[16][16], uv[8][16];
  int mode_i16, mode_uv;
  uint8_t modes_i4[16];
  uint32_t nz;
  int8_t derr[2][3];
} Score;

/* ------------------------------------------------------------------------ */
/* Iterator: src/enc/iterator_enc.c:22-174,234-326 */

static void it_init_left(It* it, const Enc* e) {
  it->yl[-1] = it->ul[-1] = it->vl[-1] = (it->y > 0) ? 129 : 127;
  memset(it->yl, 129, 16);
  memset(it->ul, 129, 8);
  memset(it->vl, 129, 8);
  it->left_nz[8] = 0;
  if (e->top_derr) memset(it->lderr, 0, sizeof(it->lderr));
}

static void it_set_row(It* it, Enc* e, int y) {
  it->x = 0; it->y = y;
  it->preds = e->preds + y * 4 * e->preds_w;
  it->nz = e->nz;
  it->ytop = e->y_top;
  it->uvtop = e->uv_top;
  it_init_left(it, e);
}

static void it_reset(It* it, Enc* e) {
  memset(it, 0, sizeof(*it));
  it->yl = it->yl_mem + 1; it->ul = it->ul_mem + 1; it->vl = it->vl_mem + 1;
  it->out = it->yout; it->out2 = it->yout2;
  memset(e->y_top, 127, 2 * e->mbw * 16);
  memset(e->nz, 0, e->mbw * sizeof(*e->nz));
  if (e->top_derr) memset(e->top_derr, 0, e->mbw * sizeof(*e->top_derr));
  it_set_row(it, e, 0);
}

static int it_next(It* it, Enc* e) {
  if (++it->x == e->mbw) {
    if (it->y + 1 == e->mbh) return 0;
    it_set_row(it, e, it->y + 1);
  } else {
    it->preds += 4; it->nz += 1; it->ytop += 16; it->uvtop += 16;
  }
  return 1;
}

/* copy a w x h block into an n x n cache, replicating the right/bottom edge */
static void import_block(const uint8_t* src, int ss, uint8_t* dst, int w, int h, int n) {
  for (int i = 0; i < h; ++i) {
    memcpy(dst + i * BPS, src + i * ss, w);
    if (w < n) memset(dst + i * BPS + w, dst[i * BPS + w - 1], n - w);
  }
  for (int i = h; i < n; ++i) memcpy(dst + i * BPS, dst + (i - 1) * BPS, n);
}

static void it_import(It* it, const Enc* e) {
  const int x = it->x, y = it->y;
  const int w = e->w - 16 * x < 16 ? e->w - 16 * x : 16;
  const int h = e->h - 16 * y < 16 ? e->h - 16 * y : 16;
  import_block(e->Y + 16 * (y * e->ys + x), e->ys, it->yin, w, h, 16);
  import_block(e->U + 8 * (y * e->uvs + x), e->uvs, it->yin + 16, (w + 1) >> 1, (h + 1) >> 1, 8);
  import_block(e->V + 8 * (y * e->uvs + x), e->uvs, it->yin + 24, (w + 1) >> 1, (h + 1) >> 1, 8);
}

static void line_copy(const uint8_t* src, int step, uint8_t* dst, int len, int total) {
  int i = 0;
  for (; i < len; ++i) dst[i] = src[i * step];
  for (; i < total; ++i) dst[i] = dst[len - 1];
}

/* analysis-only boundary from *source* samples (iterator_enc.c:147-173) */
static void it_import_src_boundary(It* it, const Enc* e, uint8_t tmp32[32]) {
  const int x = it->x, y = it->y;
  const uint8_t* ys = e->Y + 16 * (y * e->ys + x);
  const uint8_t* us = e->U + 8 * (y * e->uvs + x);
  const uint8_t* vs = e->V + 8 * (y * e->uvs + x);
  const int w = e->w - 16 * x < 16 ? e->w - 16 * x : 16;
  const int h = e->h - 16 * y < 16 ? e->h - 16 * y : 16;
  const int uw = (w + 1) >> 1, uh = (h + 1) >> 1;
  if (x == 0) {
    it_init_left(it, e);
  } else {
    if (y == 0) {
      it->yl[-1] = it->ul[-1] = it->vl[-1] = 127;
    } else {
      it->yl[-1] = ys[-1 - e->ys];
      it->ul[-1] = us[-1 - e->uvs];
      it->vl[-1] = vs[-1 - e->uvs];
    }
    line_copy(ys - 1, e->ys, it->yl, h, 16);
    line_copy(us - 1, e->uvs, it->ul, uh, 8);
    line_copy(vs - 1, e->uvs, it->vl, uh, 8);
  }
  it->ytop = tmp32;
  it->uvtop = tmp32 + 16;
  if (y == 0) {
    memset(tmp32, 127, 32);
  } else {
    line_copy(ys - e->ys, 1, tmp32, w, 16);
    line_copy(us - e->uvs, 1, tmp32 + 16, uw, 8);
    line_copy(vs - e->uvs, 1, tmp32 + 24, uw, 8);
  }
}

/* nz context word <-> per-block flags (iterator_enc.c:220-283) */
static void nz_to_flags(It* it) {
  const uint32_t t = it->nz[0], l = it->nz[-1];
  static const int tb[9] = {12, 13, 14, 15, 18, 19, 22, 23, 24};
  static const int lb[8] = {3, 7, 11, 15, 17, 19, 21, 23};
  for (int i = 0; i < 9; ++i) it->top_nz[i] = (t >> tb[i]) & 1;
  for (int i = 0; i < 8; ++i) it->left_nz[i] = (l >> lb[i]) & 1;
}
static void flags_to_nz(It* it) {
  uint32_t nz = 0;
  nz |= (it->top_nz[0] << 12) | (it->top_nz[1] << 13) | (it->top_nz[2] << 14) |
        (it->top_nz[3] << 15) | (it->top_nz[4] << 18) | (it->top_nz[5] << 19) |
        (it->top_nz[6] << 22) | (it->top_nz[7] << 23) | (it->top_nz[8] << 24);
  nz |= (it->left_nz[0] << 3) | (it->left_nz[1] << 7) | (it->left_nz[2] << 11) |
        (it->left_nz[4] << 17) | (it->left_nz[6] << 21);
  it->nz[0] = nz;
}

static void it_save_boundary(It* it, Enc* e) {
  const uint8_t* o = it->out;
  if (it->x < e->mbw - 1) {
    for (int i = 0; i < 16; ++i) it->yl[i] = o[15 + i * BPS];
    for (int i = 0; i < 8; ++i) { it->ul[i] = o[16 + 7 + i * BPS]; it->vl[i] = o[24 + 7 + i * BPS]; }
    it->yl[-1] = it->ytop[15];
    it->ul[-1] = it->uvtop[7];
    it->vl[-1] = it->uvtop[15];
  }
  if (it->y < e->mbh - 1) {
    memcpy((uint8_t*)it->ytop, o + 15 * BPS, 16);
    memcpy((uint8_t*)it->uvtop, o + 16 + 7 * BPS, 16);
  }
}

static void set_i16_mode(It* it, Enc* e, int mode) {   /* iterator_enc.c:331-339 */
  for (int y = 0; y < 4; ++y) memset(it->preds + y * e->preds_w, mode, 4);
  e->mb_type[it->y * e->mbw + it->x] = 1;
}
static void set_i4_modes(It* it, Enc* e, const uint8_t* modes) {
  for (int y = 0; y < 4; ++y) memcpy(it->preds + y * e->preds_w, modes + 4 * y, 4);
  e->mb_type[it->y * e->mbw + it->x] = 0;
}

/* ------------------------------------------------------------------------ */
/* Analysis: src/enc/analysis_enc.c:28-333,422-482; histogram from
 * src/dsp/enc.c:46-81 */

static int histo_alpha(const uint8_t* src, const uint8_t* pred, int ps,
                       const int* offs_src, const int* offs_pred, int nblk) {
  int dist[32] = {0};
  for (int b = 0; b < nblk; ++b) {
    int16_t c[16];
    fdct4(src + offs_src[b], BPS, pred + offs_pred[b], ps, c);
    for (int k = 0; k < 16; ++k) {
      int v = iabs(c[k]) >> 3;
      dist[v > 31 ? 31 : v]++;
    }
  }
  int maxv = 0, last = 1;
  for (int k = 0; k < 32; ++k)
    if (dist[k] > 0) { if (dist[k] > maxv) maxv = dist[k]; last = k; }
  return maxv > 1 ? 510 * last / maxv : 0;
}

/* FastMBAnalyze (analysis_enc.c:255-276), methods 0 and 1: intra-16 DC when
 * the 16 4x4 block sums vary little, else intra-4 DC; susceptibility 0 */
static int fast_mb_analyze(It* it, Enc* e) {
  const int q = (int)e->cfg.quality;
  const uint32_t thr = 8 + (17 - 8) * q / 100;
  uint32_t m = 0, m2 = 0;
  for (int k = 0; k < 16; ++k) {   /* VP8Mean16x4 (dsp/enc.c:594-608): block sums */
    uint32_t dc = 0;
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) dc += it->yin[Y_BLK(k) + y * BPS + x];
    m += dc;
    m2 += dc * dc;
  }
  if (thr * m2 < m * m) {
    set_i16_mode(it, e, 0);
  } else {
    static const uint8_t kDC4[16] = {0};
    set_i4_modes(it, e, kDC4);
  }
  return 0;
}

static void mb_analyze(It* it, Enc* e, int* alphas, int* sum_a, int* sum_uva) {
  int so[16], po[16], suv[8], puv[8];
  for (int b = 0; b < 16; ++b) { so[b] = (b >> 2) * 4 * BPS + (b & 3) * 4; po[b] = (b >> 2) * 64 + (b & 3) * 4; }
  for (int b = 0; b < 8; ++b) {
    const int c = b >> 2, k = b & 3;
    suv[b] = 16 + 8 * c + (k >> 1) * 4 * BPS + (k & 1) * 4;
    puv[b] = 8 * c + (k >> 1) * 64 + (k & 1) * 4;
  }
  const uint8_t* left = it->x ? it->yl : NULL;
  const uint8_t* top = it->y ? it->ytop : NULL;
  const int mi = it->y * e->mbw + it->x;
  int best_a = -1, best_mode = 0;
  set_i16_mode(it, e, 0);   /* MBAnalyze defaults (analysis_enc.c:312-314) */
  if (e->method <= 1) {
    best_a = fast_mb_analyze(it, e);
  } else {
    preds16(it->p16, left, top);
    for (int m = 0; m < 2; ++m) {   /* DC and TM only (MAX_INTRA16_MODE) */
      const int a = histo_alpha(it->yin, it->p16[m], 16, so, po, 16);
      if (a > best_a) { best_a = a; best_mode = m; }
    }
    set_i16_mode(it, e, best_mode);
  }
  preds_uv(it->puv, it->x ? it->ul : NULL, it->x ? it->vl : NULL, it->y ? it->uvtop : NULL);
  int best_uv = -1, smallest = 0, uv_mode = 0;
  for (int m = 0; m < 2; ++m) {
    const int a = histo_alpha(it->yin, it->puv[m], 16, suv, puv, 8);
    if (a > best_uv) best_uv = a;
    if (m == 0 || a < smallest) { smallest = a; uv_mode = m; }
  }
  e->mb_uv[mi] = uv_mode;   /* VP8SetIntraUVMode: kept by method 0 (no UV refinement) */
  int a = (3 * best_a + best_uv + 2) >> 2;
  a = clampi(255 - a, 0, 255);
  alphas[a]++;
  e->mb_alpha[it->y * e->mbw + it->x] = a;
  *sum_a += a;
  *sum_uva += best_uv;
}

static void smooth_segments(Enc* e) {   /* analysis_enc.c:28-67 */
  const int w = e->mbw, h = e->mbh;
  uint8_t* tmp = (uint8_t*)malloc(w * h);
  if (!tmp) return;
  for (int y = 1; y < h - 1; ++y)
    for (int x = 1; x < w - 1; ++x) {
      int cnt[4] = {0};
      const uint8_t* s = e->mb_seg + x + w * y;
      int maj = s[0];
      cnt[s[-w - 1]]++; cnt[s[-w]]++; cnt[s[-w + 1]]++; cnt[s[-1]]++;
      cnt[s[1]]++; cnt[s[w - 1]]++; cnt[s[w]]++; cnt[s[w + 1]]++;
      for (int n = 0; n < 4; ++n) if (cnt[n] >= 5) { maj = n; break; }
      tmp[x + y * w] = maj;
    }
  for (int y = 1; y < h - 1; ++y)
    for (int x = 1; x < w - 1; ++x) e->mb_seg[x + w * y] = tmp[x + y * w];
  free(tmp);
}

static void assign_segments(Enc* e, const int* alphas) {   /* :132-216 */
  const int nb = e->num_segments < 4 ? e->num_segments : 4;
  int centers[4], map[256], accum[4], dist[4];
  int n, k, a, wavg = 0, min_a, max_a;
  for (n = 0; n <= 255 && alphas[n] == 0; ++n) {}
  min_a = n;
  for (n = 255; n > min_a && alphas[n] == 0; --n) {}
  max_a = n;
  const int range = max_a - min_a;
  for (k = 0, n = 1; k < nb; ++k, n += 2) centers[k] = min_a + (n * range) / (2 * nb);
  for (k = 0; k < 6; ++k) {
    int tw = 0, displaced = 0;
    for (n = 0; n < nb; ++n) accum[n] = dist[n] = 0;
    n = 0;
    for (a = min_a; a <= max_a; ++a) {
      if (alphas[a]) {
        while (n + 1 < nb && iabs(a - centers[n + 1]) < iabs(a - centers[n])) n++;
        map[a] = n;
        dist[n] += a * alphas[a];
        accum[n] += alphas[a];
      }
    }
    wavg = 0;
    for (n = 0; n < nb; ++n) {
      if (accum[n]) {
        const int c = (dist[n] + accum[n] / 2) / accum[n];
        displaced += iabs(centers[n] - c);
        centers[n] = c;
        wavg += c * accum[n];
        tw += accum[n];
      }
    }
    wavg = (wavg + tw / 2) / tw;
    if (displaced < 5) break;
  }
  for (n = 0; n < e->mbw * e->mbh; ++n) {
    const int al = e->mb_alpha[n];
    e->mb_seg[n] = map[al];
    e->mb_alpha[n] = centers[map[al]];
  }
  if (nb > 1 && (e->cfg.preprocessing & 1)) smooth_segments(e);
  /* SetSegmentAlphas, :76-97 */
  int mn = centers[0], mx = centers[0];
  if (nb > 1)
    for (n = 0; n < nb; ++n) { if (mn > centers[n]) mn = centers[n]; if (mx < centers[n]) mx = centers[n]; }
  if (mx == mn) mx = mn + 1;
  for (n = 0; n < nb; ++n) {
    e->dqm[n].alpha = clampi(255 * (centers[n] - wavg) / (mx - mn), -127, 127);
    e->dqm[n].beta = clampi(255 * (centers[n] - mn) / (mx - mn), 0, 255);
  }
}

static void analyze(Enc* e) {
  const int do_seg = e->cfg.emulate_jpeg_size || e->num_segments > 1 || e->method <= 1;
  if (do_seg) {
    int alphas[256] = {0}, sa = 0, suva = 0;
    It it;
    uint8_t tmp32[32];
    it_reset(&it, e);
    do {
      it_import(&it, e);
      it_import_src_boundary(&it, e, tmp32);
      mb_analyze(&it, e, alphas, &sa, &suva);
    } while (it_next(&it, e));
    const int total = e->mbw * e->mbh;
    e->alpha = sa / total;
    e->uv_alpha = suva / total;
    assign_segments(e, alphas);
  } else {
    memset(e->mb_seg, 0, e->mbw * e->mbh);
    memset(e->mb_alpha, 0, e->mbw * e->mbh);
    e->dqm[0].alpha = e->dqm[0].beta = 0;
    e->alpha = e->uv_alpha = 0;
  }
}

void vp8o_analyze(const uint8_t* Y, const uint8_t* U, const uint8_t* V,
                  int w, int h, int ys, int uvs,
                  uint8_t* mb_alpha, int* uv_alpha_sum, int* histo256) {
  Enc e;
  memset(&e, 0, sizeof(e));
  e.Y = Y; e.U = U; e.V = V; e.ys = ys; e.uvs = uvs; e.w = w; e.h = h;
  e.mbw = (w + 15) >> 4; e.mbh = (h + 15) >> 4;
  e.mb_alpha = mb_alpha;
  e.mb_type = (uint8_t*)calloc(e.mbw * e.mbh, 1);
  e.y_top = (uint8_t*)calloc(2 * e.mbw * 16, 1);
  e.uv_top = e.y_top + 16 * e.mbw;
  e.nz_mem = (uint32_t*)calloc(e.mbw + 1, 4); e.nz = e.nz_mem + 1;
  e.preds_w = 4 * e.mbw + 1;
  e.preds_mem = (uint8_t*)calloc(e.preds_w * (4 * e.mbh + 1), 1);
  e.preds = e.preds_mem + 1 + e.preds_w;
  int sa = 0, suva = 0;
  memset(histo256, 0, 256 * sizeof(int));
  It it;
  uint8_t tmp32[32];
  it_reset(&it, &e);
  do {
    it_import(&it, &e);
    it_import_src_boundary(&it, &e, tmp32);
    mb_analyze(&it, &e, histo256, &sa, &suva);
  } while (it_next(&it, &e));
  *uv_alpha_sum = suva;
  free(e.mb_type); free(e.y_top); free(e.nz_mem); free(e.preds_mem);
}

/* ------------------------------------------------------------------------ */
/* Segment parameters: src/enc/quant_enc.c:205-455, filter_enc.c:59-63 */

static int expand_matrix(Mtx* m, int type) {
  for (int i = 0; i < 2; ++i) {
    m->iq[i] = (1 << QFIX) / m->q[i];
    m->bias[i] = kVP8BiasMtx[type][i > 0] << (QFIX - 8);
    m->zthresh[i] = ((1 << QFIX) - 1 - m->bias[i]) / m->iq[i];
  }
  for (int i = 2; i < 16; ++i) {
    m->q[i] = m->q[1]; m->iq[i] = m->iq[1];
    m->bias[i] = m->bias[1]; m->zthresh[i] = m->zthresh[1];
  }
  int sum = 0;
  for (int i = 0; i < 16; ++i) {
    m->sharpen[i] = type == 0 ? (kVP8FreqSharpen[i] * m->q[i]) >> 11 : 0;
    sum += m->q[i];
  }
  return (sum + 8) >> 4;
}

static void setup_matrices(Enc* e) {
  const int tls = e->method >= 4 ? e->cfg.sns_strength : 0;
  for (int i = 0; i < e->num_segments; ++i) {
    Seg* m = &e->dqm[i];
    const int q = m->quant;
    m->y1.q[0] = kVP8DcQ[clampi(q, 0, 127)];
    m->y1.q[1] = kVP8AcQ[clampi(q, 0, 127)];
    m->y2.q[0] = kVP8DcQ[clampi(q, 0, 127)] * 2;
    m->y2.q[1] = kVP8AcQ2[clampi(q, 0, 127)];
    m->uv.q[0] = kVP8DcQ[clampi(q + e->dq_uv_dc, 0, 117)];
    m->uv.q[1] = kVP8AcQ[clampi(q + e->dq_uv_ac, 0, 127)];
    const int q_i4 = expand_matrix(&m->y1, 0);
    const int q_i16 = expand_matrix(&m->y2, 1);
    const int q_uv = expand_matrix(&m->uv, 2);
#define ATLEAST1(v) ((v) < 1 ? 1 : (v))
    m->lambda_i4 = ATLEAST1((3 * q_i4 * q_i4) >> 7);
    m->lambda_i16 = ATLEAST1(3 * q_i16 * q_i16);
    m->lambda_uv = ATLEAST1((3 * q_uv * q_uv) >> 6);
    m->lambda_mode = ATLEAST1((1 * q_i4 * q_i4) >> 7);
    m->lambda_trellis_i4 = ATLEAST1((7 * q_i4 * q_i4) >> 3);
    m->lambda_trellis_i16 = ATLEAST1((q_i16 * q_i16) >> 2);
    m->lambda_trellis_uv = ATLEAST1((q_uv * q_uv) << 1);
    m->tlambda = ATLEAST1((tls * q_i4) >> 5);
#undef ATLEAST1
    m->min_disto = 20 * m->y1.q[0];
    m->i4_penalty = 1000 * q_i4 * q_i4;
    m->max_edge = 0;
  }
}

static double quality_to_compression(double c) {
  const double lin = (c < 0.75) ? c * (2. / 3.) : 2. * c - 1.;
  return pow(lin, 1 / 3.);
}
static double quality_to_jpeg_compression(double c, double alpha) {
  const double amin = 0.30, amax = 0.85, emin = 0.4, emax = 0.9;
  const double slope = (emin - emax) / (amax - amin);
  const double expn = (alpha > amax) ? emin : (alpha < amin) ? emax : emax + slope * (alpha - amin);
  return pow(c, expn);
}

static void set_segment_params(Enc* e, float quality) {
  const int ns = e->num_segments;
  const double amp = 0.9 * e->cfg.sns_strength / 100. / 128.;
  const double Q = quality / 100.;
  const double cbase = e->cfg.emulate_jpeg_size ? quality_to_jpeg_compression(Q, e->alpha / 255.)
                                                : quality_to_compression(Q);
  for (int i = 0; i < ns; ++i) {
    const double expn = 1. - amp * e->dqm[i].alpha;
    const double c = pow(cbase, expn);
    e->dqm[i].quant = clampi((int)(127. * (1. - c)), 0, 127);
  }
  e->base_quant = e->dqm[0].quant;
  for (int i = ns; i < 4; ++i) e->dqm[i].quant = e->base_quant;
  int dq_uv_ac = (e->uv_alpha - 64) * (6 - (-4)) / (100 - 30);
  dq_uv_ac = dq_uv_ac * e->cfg.sns_strength / 100;
  dq_uv_ac = clampi(dq_uv_ac, -4, 6);
  int dq_uv_dc = -4 * e->cfg.sns_strength / 100;
  dq_uv_dc = clampi(dq_uv_dc, -15, 15);
  e->dq_uv_dc = dq_uv_dc;
  e->dq_uv_ac = dq_uv_ac;
  /* SetupFilterStrength (:296-314): note it reads the *current* header
   * sharpness before overwriting it with the config value. */
  const int level0 = 5 * e->cfg.filter_strength;
  for (int i = 0; i < 4; ++i) {
    Seg* m = &e->dqm[i];
    const int qstep = kVP8AcQ[clampi(m->quant, 0, 127)] >> 2;
    const int pos = qstep < 64 ? qstep : 63;
    const int base = kVP8LevelsFromDelta[e->f_sharpness][pos];
    const int f = base * level0 / (256 + m->beta);
    m->fstrength = (f < 2) ? 0 : (f > 63) ? 63 : f;
  }
  e->f_level = e->dqm[0].fstrength;
  e->f_simple = (e->cfg.filter_type == 0);
  e->f_sharpness = e->cfg.filter_sharpness;
  /* SimplifySegments (:362-400) */
  if (ns > 1) {
    int map[4] = {0, 1, 2, 3}, nfinal = 1;
    for (int s1 = 1; s1 < ns; ++s1) {
      int s2, found = 0;
      for (s2 = 0; s2 < nfinal; ++s2)
        if (e->dqm[s1].quant == e->dqm[s2].quant && e->dqm[s1].fstrength == e->dqm[s2].fstrength) {
          found = 1;
          break;
        }
      map[s1] = s2;
      if (!found) {
        if (nfinal != s1) e->dqm[nfinal] = e->dqm[s1];
        ++nfinal;
      }
    }
    if (nfinal < ns) {
      for (int i = 0; i < e->mbw * e->mbh; ++i) e->mb_seg[i] = map[e->mb_seg[i]];
      e->num_segments = nfinal;
      for (int i = nfinal; i < ns; ++i) e->dqm[i] = e->dqm[nfinal - 1];
    }
  }
  setup_matrices(e);
}

static int get_proba(int a, int b) {   /* frame_enc.c:185-189 */
  const int t = a + b;
  return t == 0 ? 255 : (255 * a + t / 2) / t;
}

static void set_segment_probas(Enc* e) {   /* frame_enc.c:198-231 */
  int p[4] = {0};
  for (int n = 0; n < e->mbw * e->mbh; ++n) p[e->mb_seg[n]]++;
  if (e->num_segments > 1) {
    uint8_t* pr = e->seg_probas;
    pr[0] = get_proba(p[0] + p[1], p[2] + p[3]);
    pr[1] = get_proba(p[0], p[1]);
    pr[2] = get_proba(p[2], p[3]);
    e->update_map = (pr[0] != 255) || (pr[1] != 255) || (pr[2] != 255);
    if (!e->update_map) memset(e->mb_seg, 0, e->mbw * e->mbh);
    e->seg_hdr_size = p[0] * (bit_cost(0, pr[0]) + bit_cost(0, pr[1])) +
                      p[1] * (bit_cost(0, pr[0]) + bit_cost(1, pr[1])) +
                      p[2] * (bit_cost(1, pr[0]) + bit_cost(0, pr[2])) +
                      p[3] * (bit_cost(1, pr[0]) + bit_cost(1, pr[2]));
  } else {
    e->update_map = 0;
    e->seg_hdr_size = 0;
  }
}

/* ------------------------------------------------------------------------ */
/* Probabilities and costs: src/enc/cost_enc.c:42-90, frame_enc.c:131-180 */

static void level_costs(Enc* e) {
  if (!e->dirty) return;
  for (int t = 0; t < 4; ++t)
    for (int b = 0; b < 8; ++b)
      for (int c = 0; c < 3; ++c) {
        const uint8_t* p = e->coeffs[t][b][c];
        uint16_t* tab = e->lcost[t][b][c];
        const int c0 = c > 0 ? bit_cost(1, p[0]) : 0;
        const int base = bit_cost(1, p[1]) + c0;
        tab[0] = bit_cost(0, p[1]) + c0;
        for (int v = 1; v <= MAX_VLEVEL; ++v) {
          int pat = kVP8LevelCodes[v - 1][0], bits = kVP8LevelCodes[v - 1][1], cost = 0;
          for (int i = 2; pat; ++i, pat >>= 1, bits >>= 1)
            if (pat & 1) cost += bit_cost(bits & 1, p[i]);
          tab[v] = base + cost;
        }
      }
  e->dirty = 0;
}

/* FinalizeTokenProbas (frame_enc.c:146-180): a pure function of the
 * statistics (old_p is the default table, not the previous value); returns
 * the header cost of the proba updates in 1/256 bits */
static int finalize_token_probas(Enc* e) {
  int changed = 0, size = 0;
  for (int t = 0; t < 4; ++t)
    for (int b = 0; b < 8; ++b)
      for (int c = 0; c < 3; ++c)
        for (int p = 0; p < 11; ++p) {
          const uint32_t st = e->stats[t][b][c][p];
          const int nb = st & 0xffff, total = (st >> 16) & 0xffff;
          const int upd = kVP8CoeffUpdateProba[t][b][c][p];
          const int old_p = kVP8CoeffProba0[t][b][c][p];
          const int new_p = nb ? (255 - nb * 255 / total) : 255;
          const int old_cost = nb * bit_cost(1, old_p) + (total - nb) * bit_cost(0, old_p) + bit_cost(0, upd);
          const int new_cost = nb * bit_cost(1, new_p) + (total - nb) * bit_cost(0, new_p) +
                               bit_cost(1, upd) + 8 * 256;
          const int use_new = old_cost > new_cost;
          size += bit_cost(use_new, upd);
          if (use_new) {
            e->coeffs[t][b][c][p] = new_p;
            changed |= (new_p != old_p);
            size += 8 * 256;
          } else {
            e->coeffs[t][b][c][p] = old_p;
          }
        }
  e->dirty = changed;
  return size;
}

static inline int level_cost(const uint16_t* tab, int level) {
  return kVP8LevelFixedCost[level] + tab[level > MAX_VLEVEL ? MAX_VLEVEL : level];
}

/* GetResidualCost_C, src/dsp/cost.c:322-355. levels in zigzag order. */
static int residual_cost(const Enc* e, int ctx0, int type, int first, const int16_t* lv) {
  int last = -1;
  for (int n = 15; n >= 0; --n) if (lv[n]) { last = n; break; }
  const int p0 = e->coeffs[type][first][ctx0][0];
  if (last < 0) return bit_cost(0, p0);
  int cost = ctx0 == 0 ? bit_cost(1, p0) : 0;
  const uint16_t* t = e->lcost[type][kBand[first]][ctx0];
  int n = first;
  for (; n < last; ++n) {
    const int v = iabs(lv[n]);
    cost += level_cost(t, v);
    t = e->lcost[type][kBand[n + 1]][v >= 2 ? 2 : v];
  }
  const int v = iabs(lv[n]);
  cost += level_cost(t, v);
  if (n < 15) cost += bit_cost(0, e->coeffs[type][kBand[n + 1]][v == 1 ? 1 : 2][0]);
  return cost;
}

/* ------------------------------------------------------------------------ */
/* Quantisation: src/dsp/enc.c:653-686, src/enc/quant_enc.c:593-763,860-920 */

static int quantize(int16_t in[16], int16_t out[16], const Mtx* m) {
  int last = -1;
  for (int n = 0; n < 16; ++n) {
    const int j = kZz[n];
    const int neg = in[j] < 0;
    const uint32_t coeff = (uint32_t)(neg ? -in[j] : in[j]) + m->sharpen[j];
    if (coeff > m->zthresh[j]) {
      int level = (int)((coeff * m->iq[j] + m->bias[j]) >> QFIX);
      if (level > MAX_LEVEL) level = MAX_LEVEL;
      if (neg) level = -level;
      in[j] = (int16_t)(level * (int)m->q[j]);
      out[n] = (int16_t)level;
      if (level) last = n;
    } else {
      out[n] = 0;
      in[j] = 0;
    }
  }
  return last >= 0;
}

typedef struct { int8_t prev, sign; int16_t level; } TNode;

static int trellis(const Enc* e, int16_t in[16], int16_t out[16], int ctx0, int type,
                   const Mtx* m, int lambda) {
  const int first = type == 0 ? 1 : 0;
  TNode nodes[16][2];
  score_t ss_score[2][2];
  const uint16_t* ss_cost[2][2];
  int cur = 0, prv = 1;
  int best_path[3] = {-1, -1, -1};
  score_t best_score;
  int n, last;
  const int thresh = m->q[1] * m->q[1] / 4;
  const int last_proba = e->coeffs[type][kBand[first]][ctx0][0];
  last = first - 1;
  for (n = 15; n >= first; --n) {
    const int j = kZz[n];
    if (in[j] * in[j] > thresh) { last = n; break; }
  }
  if (last < 15) ++last;
  best_score = (score_t)bit_cost(0, last_proba) * lambda;
  for (int k = 0; k < 2; ++k) {
    ss_score[cur][k] = (score_t)(ctx0 == 0 ? bit_cost(1, last_proba) : 0) * lambda;
    ss_cost[cur][k] = e->lcost[type][kBand[first]][ctx0];
  }
  for (n = first; n <= last; ++n) {
    const int j = kZz[n];
    const uint32_t Q = m->q[j], iQ = m->iq[j];
    const int neg = in[j] < 0;
    const uint32_t coeff0 = (uint32_t)(neg ? -in[j] : in[j]) + m->sharpen[j];
    int level0 = (int)((coeff0 * iQ) >> QFIX);
    int thr_level = (int)((coeff0 * iQ + (0x80 << (QFIX - 8))) >> QFIX);
    if (thr_level > MAX_LEVEL) thr_level = MAX_LEVEL;
    if (level0 > MAX_LEVEL) level0 = MAX_LEVEL;
    cur ^= 1; prv ^= 1;
    for (int k = 0; k < 2; ++k) {
      TNode* nd = &nodes[n][k];
      const int level = level0 + k;
      const int ctx = level > 2 ? 2 : level;
      const int band = kBand[n + 1];
      ss_cost[cur][k] = e->lcost[type][band][ctx];
      if (level < 0 || level > thr_level) { ss_score[cur][k] = MAX_COST; continue; }
      const int new_err = (int)coeff0 - level * (int)Q;
      const int delta = kVP8WeightTrellis[j] * (new_err * new_err - (int)(coeff0 * coeff0));
      const score_t base = (score_t)256 * delta;
      score_t best_cur = ss_score[prv][0] + (score_t)level_cost(ss_cost[prv][0], level) * lambda;
      int best_prev = 0;
      const score_t s1 = ss_score[prv][1] + (score_t)level_cost(ss_cost[prv][1], level) * lambda;
      if (s1 < best_cur) { best_cur = s1; best_prev = 1; }
      best_cur += base;
      nd->sign = neg; nd->level = level; nd->prev = best_prev;
      ss_score[cur][k] = best_cur;
      if (level != 0 && best_cur < best_score) {
        const score_t lc = (n < 15) ? bit_cost(0, e->coeffs[type][band][ctx][0]) : 0;
        const score_t sc = best_cur + lc * lambda;
        if (sc < best_score) {
          best_score = sc;
          best_path[0] = n; best_path[1] = k; best_path[2] = best_prev;
        }
      }
    }
  }
  if (type == 0) {
    memset(in + 1, 0, 15 * sizeof(*in));
    memset(out + 1, 0, 15 * sizeof(*out));
  } else {
    memset(in, 0, 16 * sizeof(*in));
    memset(out, 0, 16 * sizeof(*out));
  }
  if (best_path[0] == -1) return 0;
  int nz = 0, node = best_path[1];
  n = best_path[0];
  nodes[n][node].prev = best_path[2];
  for (; n >= first; --n) {
    const TNode* nd = &nodes[n][node];
    const int j = kZz[n];
    out[n] = nd->sign ? -nd->level : nd->level;
    nz |= nd->level;
    in[j] = out[n] * m->q[j];
    node = nd->prev;
  }
  return nz != 0;
}

/* ------------------------------------------------------------------------ */
/* Reconstruction + RD mode search: src/enc/quant_enc.c:772-1398 */

static const int kUVBlk[8] = {16, 20, 16 + 4 * BPS, 20 + 4 * BPS, 24, 28, 24 + 4 * BPS, 28 + 4 * BPS};
#define P16_BLK(n) (((n) >> 2) * 64 + ((n) & 3) * 4)
static const int kUVPred[8] = {0, 4, 64, 68, 8, 12, 72, 76};

static int recon_i16(It* it, Enc* e, Score* rd, uint8_t* yout, int mode) {
  const uint8_t* ref = it->p16[mode];
  const Seg* dq = &e->dqm[e->mb_seg[it->y * e->mbw + it->x]];
  int16_t tmp[16][16], dcs[16], dc_tmp[16];
  int nz = 0;
  for (int n = 0; n < 16; ++n) fdct4(it->yin + Y_BLK(n), BPS, ref + P16_BLK(n), 16, tmp[n]);
  for (int n = 0; n < 16; ++n) dcs[n] = tmp[n][0];
  fwht(dcs, dc_tmp);
  nz |= quantize(dc_tmp, rd->y_dc, &dq->y2) << 24;
  if (it->do_trellis) {
    nz_to_flags(it);
    for (int y = 0, n = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x, ++n) {
        const int ctx = it->top_nz[x] + it->left_nz[y];
        const int b = trellis(e, tmp[n], rd->y_ac[n], ctx, 0, &dq->y1, dq->lambda_trellis_i16);
        it->top_nz[x] = it->left_nz[y] = b;
        rd->y_ac[n][0] = 0;
        nz |= b << n;
      }
  } else {
    for (int n = 0; n < 16; ++n) {
      tmp[n][0] = 0;
      nz |= quantize(tmp[n], rd->y_ac[n], &dq->y1) << n;
    }
  }
  iwht(dc_tmp, dcs);
  for (int n = 0; n < 16; ++n) {
    tmp[n][0] = dcs[n];
    idct4(ref + P16_BLK(n), 16, tmp[n], yout + Y_BLK(n), BPS);
  }
  return nz;
}

static int recon_i4(It* it, Enc* e, int16_t levels[16], const uint8_t* src,
                    const uint8_t* pred, uint8_t* dst, int dst_stride, int i4) {
  const Seg* dq = &e->dqm[e->mb_seg[it->y * e->mbw + it->x]];
  int16_t tmp[16];
  int nz;
  fdct4(src, BPS, pred, 4, tmp);
  if (it->do_trellis) {
    const int ctx = it->top_nz[i4 & 3] + it->left_nz[i4 >> 2];
    nz = trellis(e, tmp, levels, ctx, 3, &dq->y1, dq->lambda_trellis_i4);
  } else {
    nz = quantize(tmp, levels, &dq->y1);
  }
  idct4(pred, 4, tmp, dst, dst_stride);
  return nz;
}

static int8_t quant_single(int16_t* v, const Mtx* m) {   /* :860-873 */
  int V = *v;
  const int neg = V < 0;
  if (neg) V = -V;
  if (V > (int)m->zthresh[0]) {
    const int qV = (int)(((uint32_t)V * m->iq[0] + m->bias[0]) >> QFIX) * m->q[0];
    const int err = V - qV;
    *v = (int16_t)(neg ? -qV : qV);
    return (int8_t)((neg ? -err : err) >> 1);
  }
  *v = 0;
  return (int8_t)((neg ? -V : V) >> 1);
}

static void correct_dc(It* it, Enc* e, const Mtx* m, int16_t tmp[8][16], Score* rd) {
  for (int ch = 0; ch <= 1; ++ch) {
    const int8_t* top = e->top_derr[it->x][ch];
    const int8_t* left = it->lderr[ch];
    int16_t (*c)[16] = &tmp[ch * 4];
    int e0, e1, e2, e3;
    c[0][0] += (7 * top[0] + 8 * left[0]) >> 3;
    e0 = quant_single(&c[0][0], m);
    c[1][0] += (7 * top[1] + 8 * e0) >> 3;
    e1 = quant_single(&c[1][0], m);
    c[2][0] += (7 * e0 + 8 * left[1]) >> 3;
    e2 = quant_single(&c[2][0], m);
    c[3][0] += (7 * e1 + 8 * e2) >> 3;
    e3 = quant_single(&c[3][0], m);
    rd->derr[ch][0] = (int8_t)e1;
    rd->derr[ch][1] = (int8_t)e2;
    rd->derr[ch][2] = (int8_t)e3;
  }
}

static void store_derr(It* it, Enc* e, const Score* rd) {
  for (int ch = 0; ch <= 1; ++ch) {
    int8_t* top = e->top_derr[it->x][ch];
    int8_t* left = it->lderr[ch];
    left[0] = rd->derr[ch][0];
    left[1] = 3 * rd->derr[ch][2] >> 2;
    top[0] = rd->derr[ch][1];
    top[1] = rd->derr[ch][2] - left[1];
  }
}

/* yout: 32-stride UV area (U at col 16, V at col 24) */
static int recon_uv(It* it, Enc* e, Score* rd, uint8_t* yout, int mode) {
  const uint8_t* ref = it->puv[mode];
  const Seg* dq = &e->dqm[e->mb_seg[it->y * e->mbw + it->x]];
  int16_t tmp[8][16];
  int nz = 0;
  for (int n = 0; n < 8; ++n) fdct4(it->yin + kUVBlk[n], BPS, ref + kUVPred[n], 16, tmp[n]);
  if (e->top_derr) correct_dc(it, e, &dq->uv, tmp, rd);
  for (int n = 0; n < 8; ++n) nz |= quantize(tmp[n], rd->uv[n], &dq->uv) << n;
  for (int n = 0; n < 8; ++n) idct4(ref + kUVPred[n], 16, tmp[n], yout + kUVBlk[n], BPS);
  return nz << 16;
}

static int is_flat(const int16_t* lv, int nblk, int thresh) {   /* dsp/quant.h:61-73 */
  int score = 0;
  for (int b = 0; b < nblk; ++b, lv += 16)
    for (int i = 1; i < 16; ++i) {
      score += (lv[i] != 0);
      if (score > thresh) return 0;
    }
  return 1;
}

static int is_flat_source16(const uint8_t* src) {
  for (int y = 0; y < 16; ++y)
    for (int x = 0; x < 16; ++x)
      if (src[y * BPS + x] != src[0]) return 0;
  return 1;
}

static inline void set_score(int lambda, Score* s) {
  s->score = (s->R + s->H) * lambda + 256 * (s->D + s->SD);
}

static int cost_luma16(It* it, Enc* e, const Score* rd) {   /* cost_enc.c:232-256 */
  int R = 0;
  nz_to_flags(it);
  R += residual_cost(e, it->top_nz[8] + it->left_nz[8], 1, 0, rd->y_dc);
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) {
      const int16_t* lv = rd->y_ac[x + 4 * y];
      R += residual_cost(e, it->top_nz[x] + it->left_nz[y], 0, 1, lv);
      int nzb = 0;
      for (int k = 0; k < 16; ++k) nzb |= lv[k];
      it->top_nz[x] = it->left_nz[y] = nzb != 0;
    }
  return R;
}

static int cost_uv(It* it, Enc* e, const Score* rd) {   /* cost_enc.c:258-278 */
  int R = 0;
  nz_to_flags(it);
  for (int ch = 0; ch <= 2; ch += 2)
    for (int y = 0; y < 2; ++y)
      for (int x = 0; x < 2; ++x) {
        const int16_t* lv = rd->uv[2 * ch + x + 2 * y];
        R += residual_cost(e, it->top_nz[4 + ch + x] + it->left_nz[4 + ch + y], 2, 0, lv);
        int nzb = 0;
        for (int k = 0; k < 16; ++k) nzb |= lv[k];
        it->top_nz[4 + ch + x] = it->left_nz[4 + ch + y] = nzb != 0;
      }
  return R;
}

static void pick_i16(It* it, Enc* e, Score* rd) {   /* :1002-1058 */
  Seg* dq = &e->dqm[e->mb_seg[it->y * e->mbw + it->x]];
  Score cand[2];
  Score* best = &cand[0];
  Score* cur = &cand[1];
  int flat = is_flat_source16(it->yin);
  for (int mode = 0; mode < 4; ++mode) {
    uint8_t* dst = it->out2;
    cur->mode_i16 = mode;
    cur->nz = recon_i16(it, e, cur, dst, mode);
    cur->D = sse(it->yin, BPS, dst, BPS, 16, 16);
    cur->SD = dq->tlambda ? (dq->tlambda * tdisto16(it->yin, BPS, dst, BPS) + 128) >> 8 : 0;
    cur->H = kVP8ModeCostI16[mode];
    cur->R = cost_luma16(it, e, cur);
    if (flat) {
      flat = is_flat(cur->y_ac[0], 16, 0);
      if (flat) { cur->D *= 2; cur->SD *= 2; }
    }
    set_score(dq->lambda_i16, cur);
    if (mode == 0 || cur->score < best->score) {
      Score* t = cur; cur = best; best = t;
      uint8_t* o = it->out; it->out = it->out2; it->out2 = o;
    }
  }
  *rd = *best;
  set_score(dq->lambda_mode, rd);
  set_i16_mode(it, e, rd->mode_i16);
  if ((rd->nz & 0x100ffff) == 0x1000000 && rd->D > dq->min_disto) {
    int mv = iabs(rd->y_dc[1]);
    if (iabs(rd->y_dc[2]) > mv) mv = iabs(rd->y_dc[2]);
    if (iabs(rd->y_dc[4]) > mv) mv = iabs(rd->y_dc[4]);
    if (mv > dq->max_edge) dq->max_edge = mv;
  }
}

/* Build the 13 edge samples for 4x4 block i4 from a canvas holding the MB's
 * top row (+ top-right), left column and the blocks reconstructed so far.
 * Equivalent to the snake boundary of iterator_enc.c:367-457. */
typedef struct { uint8_t c[17][21]; } Canvas;   /* c[0][0]=corner, row0=top, col0=left */

static void canvas_init(Canvas* cv, It* it, Enc* e) {
  cv->c[0][0] = it->yl[-1];
  for (int i = 0; i < 16; ++i) cv->c[0][1 + i] = it->ytop[i];
  for (int i = 0; i < 4; ++i)
    cv->c[0][17 + i] = (it->x < e->mbw - 1) ? it->ytop[16 + i] : it->ytop[15];
  for (int i = 0; i < 16; ++i) cv->c[1 + i][0] = it->yl[i];
}
static void canvas_edges(const Canvas* cv, int i4, uint8_t ed[13]) {
  const int bx = i4 & 3, by = i4 >> 2, r = 4 * by, c = 4 * bx;
  for (int k = 0; k < 4; ++k) ed[3 - k] = cv->c[r + 1 + k][c];    /* I J K L -> e[3..0] */
  ed[4] = cv->c[r][c];
  for (int k = 0; k < 4; ++k) ed[5 + k] = cv->c[r][c + 1 + k];
  for (int k = 0; k < 4; ++k)
    ed[9 + k] = (by > 0 && bx == 3) ? cv->c[0][17 + k] : cv->c[r][c + 5 + k];
}
static void canvas_put(Canvas* cv, int i4, const uint8_t* blk, int st) {
  const int r = 4 * (i4 >> 2), c = 4 * (i4 & 3);
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) cv->c[r + 1 + y][c + 1 + x] = blk[y * st + x];
}

static int pick_i4(It* it, Enc* e, Score* rd) {   /* :1072-1165 */
  const Seg* dq = &e->dqm[e->mb_seg[it->y * e->mbw + it->x]];
  const int pw = e->preds_w;
  uint8_t* best_blocks = it->out2;     /* Y area of the scratch output */
  int total_hdr = 0;
  Score acc;
  Canvas cv;
  if (e->max_i4_header_bits == 0) return 0;
  memset(&acc, 0, sizeof(acc));
  acc.H = 211;
  set_score(dq->lambda_mode, &acc);
  canvas_init(&cv, it, e);
  nz_to_flags(it);
  for (int i4 = 0; i4 < 16; ++i4) {
    const int bx = i4 & 3, by = i4 >> 2;
    const int left = bx == 0 ? it->preds[by * pw - 1] : rd->modes_i4[i4 - 1];
    const int top = by == 0 ? it->preds[-pw + bx] : rd->modes_i4[i4 - 4];
    const uint16_t* mcost = kVP8ModeCostI4[top][left];
    const uint8_t* src = it->yin + Y_BLK(i4);
    uint8_t ed[13], pred[10][16], rec[2][16];
    int cur_slot = 0, best_slot = -1;
    int16_t lv[16];
    Score bi;      /* best for this sub-block */
    int best_mode = -1;
    memset(&bi, 0, sizeof(bi));
    bi.score = MAX_COST;
    canvas_edges(&cv, i4, ed);
    preds4(pred, ed);
    for (int mode = 0; mode < 10; ++mode) {
      Score t;
      uint8_t* dst = rec[cur_slot];
      t.nz = recon_i4(it, e, lv, src, pred[mode], dst, 4, i4) << i4;
      t.D = sse(src, BPS, dst, 4, 4, 4);
      t.SD = dq->tlambda ? (dq->tlambda * tdisto4(src, BPS, dst, 4) + 128) >> 8 : 0;
      t.H = mcost[mode];
      t.R = (mode > 0 && is_flat(lv, 1, 3)) ? 140 : 0;
      set_score(dq->lambda_i4, &t);
      if (best_mode >= 0 && t.score >= bi.score) continue;
      t.R += residual_cost(e, it->top_nz[bx] + it->left_nz[by], 3, 0, lv);
      set_score(dq->lambda_i4, &t);
      if (best_mode < 0 || t.score < bi.score) {
        bi.D = t.D; bi.SD = t.SD; bi.R = t.R; bi.H = t.H; bi.nz = t.nz; bi.score = t.score;
        best_mode = mode;
        best_slot = cur_slot;
        cur_slot ^= 1;
        memcpy(acc.y_ac[i4], lv, sizeof(lv));
      }
    }
    set_score(dq->lambda_mode, &bi);
    acc.D += bi.D; acc.SD += bi.SD; acc.R += bi.R; acc.H += bi.H;
    acc.nz |= bi.nz; acc.score += bi.score;
    if (acc.score >= rd->score) return 0;
    total_hdr += (int)bi.H;
    if (total_hdr > e->max_i4_header_bits) return 0;
    for (int y = 0; y < 4; ++y) memcpy(best_blocks + Y_BLK(i4) + y * BPS, rec[best_slot] + 4 * y, 4);
    canvas_put(&cv, i4, rec[best_slot], 4);
    rd->modes_i4[i4] = best_mode;
    it->top_nz[bx] = it->left_nz[by] = bi.nz ? 1 : 0;
  }
  rd->D = acc.D; rd->SD = acc.SD; rd->R = acc.R; rd->H = acc.H;
  rd->nz = acc.nz; rd->score = acc.score;
  set_i4_modes(it, e, rd->modes_i4);
  { uint8_t* o = it->out; it->out = it->out2; it->out2 = o; }
  memcpy(rd->y_ac, acc.y_ac, sizeof(rd->y_ac));
  return 1;
}

static void pick_uv(It* it, Enc* e, Score* rd) {   /* :1169-1217 */
  const Seg* dq = &e->dqm[e->mb_seg[it->y * e->mbw + it->x]];
  uint8_t buf[2][BPS * 8];
  int cur_slot = 0, best_slot = -1;
  Score best;
  memset(&best, 0, sizeof(best));
  best.score = MAX_COST;
  rd->mode_uv = -1;
  for (int mode = 0; mode < 4; ++mode) {
    Score t;
    uint8_t* dst = buf[cur_slot] - 16;    /* so that dst + kUVBlk[n] is in buf */
    t.nz = recon_uv(it, e, &t, dst, mode);
    t.D = sse(it->yin + 16, BPS, dst + 16, BPS, 16, 8);
    t.SD = 0;
    t.H = kVP8ModeCostUV[mode];
    t.R = cost_uv(it, e, &t);
    if (mode > 0 && is_flat(t.uv[0], 8, 2)) t.R += 140 * 8;
    set_score(dq->lambda_uv, &t);
    if (mode == 0 || t.score < best.score) {
      best.D = t.D; best.SD = t.SD; best.R = t.R; best.H = t.H; best.nz = t.nz; best.score = t.score;
      rd->mode_uv = mode;
      memcpy(rd->uv, t.uv, sizeof(rd->uv));
      if (e->top_derr) memcpy(rd->derr, t.derr, sizeof(rd->derr));
      best_slot = cur_slot;
      cur_slot ^= 1;
    }
  }
  e->mb_uv[it->y * e->mbw + it->x] = rd->mode_uv;
  rd->D += best.D; rd->SD += best.SD; rd->R += best.R; rd->H += best.H;
  rd->nz |= best.nz; rd->score += best.score;
  for (int y = 0; y < 8; ++y) memcpy(it->out + 16 + y * BPS, buf[best_slot] + y * BPS, 16);
  if (e->top_derr) store_derr(it, e, rd);
}

/* m5 final pass: re-quantise the chosen modes with trellis (:1222-1245) */
static void simple_quantize(It* it, Enc* e, Score* rd) {
  const int mbi = it->y * e->mbw + it->x;
  int nz = 0;
  if (e->mb_type[mbi] == 1) {
    nz = recon_i16(it, e, rd, it->out, it->preds[0]);
  } else {
    Canvas cv;
    canvas_init(&cv, it, e);
    nz_to_flags(it);
    for (int i4 = 0; i4 < 16; ++i4) {
      const int mode = it->preds[(i4 & 3) + (i4 >> 2) * e->preds_w];
      uint8_t ed[13], pred[10][16];
      canvas_edges(&cv, i4, ed);
      preds4(pred, ed);
      nz |= recon_i4(it, e, rd->y_ac[i4], it->yin + Y_BLK(i4), pred[mode],
                     it->out + Y_BLK(i4), BPS, i4) << i4;
      canvas_put(&cv, i4, it->out + Y_BLK(i4), BPS);
    }
  }
  nz |= recon_uv(it, e, rd, it->out, e->mb_uv[mbi]);
  rd->nz = nz;
}

/* RefineUsingDistortion (quant_enc.c:1248-1350): RD_OPT_NONE (methods 0-2)
 * picks modes by prediction SSE plus fixed mode costs, no rate */
static void refine_using_distortion(It* it, Enc* e, int try_both, int refine_uv, Score* rd) {
  const int mi = it->y * e->mbw + it->x, pw = e->preds_w;
  const Seg* dq = &e->dqm[e->mb_seg[mi]];
  score_t best_score = MAX_COST;
  int nz = 0;
  int is_i16 = try_both || e->mb_type[mi] == 1;
  score_t score_i4 = dq->i4_penalty, i4_bit_sum = 0;
  const score_t bit_limit = try_both ? e->mb_header_limit : MAX_COST;
  if (is_i16) {
    int best_mode = -1;
    for (int mode = 0; mode < 4; ++mode) {
      const score_t score = (score_t)sse(it->yin, BPS, it->p16[mode], 16, 16, 16) * 256 +
                            kVP8ModeCostI16[mode] * 106;
      if (mode > 0 && kVP8ModeCostI16[mode] > bit_limit) continue;
      if (score < best_score) { best_mode = mode; best_score = score; }
    }
    if ((it->x == 0 || it->y == 0) && is_flat_source16(it->yin)) {   /* bug #432 */
      best_mode = (it->x == 0) ? 0 : 2;
      try_both = 0;
    }
    set_i16_mode(it, e, best_mode);
  }
  if (try_both || !is_i16) {
    Canvas cv;
    is_i16 = 0;
    canvas_init(&cv, it, e);
    for (int i4 = 0; i4 < 16; ++i4) {
      const int bx = i4 & 3, by = i4 >> 2;
      const int left = bx == 0 ? it->preds[by * pw - 1] : rd->modes_i4[i4 - 1];
      const int top = by == 0 ? it->preds[-pw + bx] : rd->modes_i4[i4 - 4];
      const uint16_t* mcost = kVP8ModeCostI4[top][left];
      const uint8_t* src = it->yin + Y_BLK(i4);
      uint8_t ed[13], pred[10][16], rec[16];
      int best = -1;
      score_t best_i4 = MAX_COST;
      canvas_edges(&cv, i4, ed);
      preds4(pred, ed);
      for (int mode = 0; mode < 10; ++mode) {
        const score_t score = (score_t)sse(src, BPS, pred[mode], 4, 4, 4) * 256 + mcost[mode] * 11;
        if (score < best_i4) { best = mode; best_i4 = score; }
      }
      i4_bit_sum += mcost[best];
      rd->modes_i4[i4] = best;
      score_i4 += best_i4;
      if (score_i4 >= best_score || i4_bit_sum > bit_limit) { is_i16 = 1; break; }
      nz |= recon_i4(it, e, rd->y_ac[i4], src, pred[best], rec, 4, i4) << i4;
      for (int y = 0; y < 4; ++y) memcpy(it->out2 + Y_BLK(i4) + y * BPS, rec + 4 * y, 4);
      canvas_put(&cv, i4, rec, 4);
    }
  }
  if (!is_i16) {
    set_i4_modes(it, e, rd->modes_i4);
    { uint8_t* o = it->out; it->out = it->out2; it->out2 = o; }
    best_score = score_i4;
  } else {
    nz = recon_i16(it, e, rd, it->out, it->preds[0]);
  }
  if (refine_uv) {
    int best_mode = -1;
    score_t best_uv = MAX_COST;
    for (int mode = 0; mode < 4; ++mode) {
      const score_t score = (score_t)sse(it->yin + 16, BPS, it->puv[mode], 16, 16, 8) * 256 +
                            kVP8ModeCostUV[mode] * 120;
      if (score < best_uv) { best_mode = mode; best_uv = score; }
    }
    e->mb_uv[mi] = best_mode;
  }
  nz |= recon_uv(it, e, rd, it->out, e->mb_uv[mi]);
  rd->nz = nz;
  rd->score = best_score;
}

static int decimate(It* it, Enc* e, Score* rd) {   /* :1364-1398 */
  memset(rd, 0, sizeof(*rd));
  rd->score = MAX_COST;
  preds16(it->p16, it->x ? it->yl : NULL, it->y ? it->ytop : NULL);
  preds_uv(it->puv, it->x ? it->ul : NULL, it->x ? it->vl : NULL, it->y ? it->uvtop : NULL);
  if (e->rd_opt == 0) {   /* RD_OPT_NONE */
    it->do_trellis = 0;
    refine_using_distortion(it, e, e->method >= 2, e->method >= 1, rd);
  } else {
    it->do_trellis = e->rd_opt >= 3;
    pick_i16(it, e, rd);
    if (e->method >= 2) pick_i4(it, e, rd);
    pick_uv(it, e, rd);
    if (e->rd_opt == 2) {
      it->do_trellis = 1;
      simple_quantize(it, e, rd);
    }
  }
  const int skip = rd->nz == 0;
  e->mb_skip[it->y * e->mbw + it->x] = skip;
  return skip;
}

/* ------------------------------------------------------------------------ */
/* Token recording: src/enc/token_enc.c:87-193, frame_enc.c:411-453,
 * cost_enc.h:45-56 */

static inline void tok_push(Enc* e, uint32_t t) {
  if (e->no_tokens) return;
  if (e->ntok == e->tcap) {
    size_t n = e->tcap ? 2 * e->tcap : 65536;
    uint16_t* p = (uint16_t*)realloc(e->tok, n * sizeof(*p));
    if (!p) { e->tok_err = 1; return; }
    e->tok = p; e->tcap = n;
  }
  e->tok[e->ntok++] = (uint16_t)t;
}
static inline void record(uint32_t* s, int bit) {
  uint32_t p = *s;
  if (p >= 0xfffe0000u) p = ((p + 1u) >> 1) & 0x7fff7fffu;
  *s = p + 0x00010000u + bit;
}
/* dynamic-probability token: slot id for the proba, separate stats slot */
static inline int tok_dyn(Enc* e, int bit, int proba_id, uint32_t* stat) {
  tok_push(e, ((uint32_t)bit << 15) | proba_id);
  if (!e->no_stats) record(stat, bit);
  return bit;
}
static inline void tok_fix(Enc* e, int bit, int proba) {
  tok_push(e, ((uint32_t)bit << 15) | (1u << 14) | proba);
}

static int record_block(Enc* e, int ctx, int type, int first, const int16_t* lv) {
  int last = -1;
  for (int n = 15; n >= 0; --n) if (lv[n]) { last = n; break; }
  int n = first;
  int base = 11 * (ctx + 3 * (kBand[n] + 8 * type));
  uint32_t* s = e->stats[type][kBand[n]][ctx];
  if (!tok_dyn(e, last >= 0, base + 0, s + 0)) return 0;
  while (n < 16) {
    const int c = lv[n++];
    const int neg = c < 0;
    const uint32_t v = neg ? -c : c;
    if (!tok_dyn(e, v != 0, base + 1, s + 1)) {
      base = 11 * (0 + 3 * (kBand[n] + 8 * type));
      s = e->stats[type][kBand[n]][0];
      continue;
    }
    if (!tok_dyn(e, v > 1, base + 2, s + 2)) {
      base = 11 * (1 + 3 * (kBand[n] + 8 * type));
      s = e->stats[type][kBand[n]][1];
    } else {
      if (!tok_dyn(e, v > 4, base + 3, s + 3)) {
        if (tok_dyn(e, v != 2, base + 4, s + 4)) tok_dyn(e, v == 4, base + 5, s + 5);
      } else if (!tok_dyn(e, v > 10, base + 6, s + 6)) {
        if (!tok_dyn(e, v > 6, base + 7, s + 7)) {
          tok_fix(e, v == 6, 159);
        } else {
          tok_fix(e, v >= 9, 165);
          tok_fix(e, !(v & 1), 145);
        }
      } else {
        const uint8_t* tab;
        int mask;
        uint32_t res = v - 3;
        if (res < (8 << 1)) {
          tok_dyn(e, 0, base + 8, s + 8); tok_dyn(e, 0, base + 9, s + 9);
          res -= 8 << 0; mask = 1 << 2; tab = kVP8Cat3;
        } else if (res < (8 << 2)) {
          tok_dyn(e, 0, base + 8, s + 8); tok_dyn(e, 1, base + 9, s + 9);
          res -= 8 << 1; mask = 1 << 3; tab = kVP8Cat4;
        } else if (res < (8 << 3)) {
          /* proba slot 10, but the token recorder's statistic lands in slot 9
           * (token_enc.c:168); RecordResiduals' VP8RecordCoeffs uses slot 10
           * (cost_enc.c:315-318) */
          tok_dyn(e, 1, base + 8, s + 8); tok_dyn(e, 0, base + 10, s + (e->no_tokens ? 10 : 9));
          res -= 8 << 2; mask = 1 << 4; tab = kVP8Cat5;
        } else {
          tok_dyn(e, 1, base + 8, s + 8); tok_dyn(e, 1, base + 10, s + (e->no_tokens ? 10 : 9));
          res -= 8 << 3; mask = 1 << 10; tab = kVP8Cat6;
        }
        for (; mask; mask >>= 1) tok_fix(e, (res & mask) != 0, *tab++);
      }
      base = 11 * (2 + 3 * (kBand[n] + 8 * type));
      s = e->stats[type][kBand[n]][2];
    }
    tok_fix(e, neg, 128);
    if (n == 16 || !tok_dyn(e, n <= last, base + 0, s + 0)) return 1;
  }
  return 1;
}

static void record_tokens(It* it, Enc* e, const Score* rd) {
  nz_to_flags(it);
  int type = 3, first = 0;
  if (e->mb_type[it->y * e->mbw + it->x] == 1) {
    const int ctx = it->top_nz[8] + it->left_nz[8];
    it->top_nz[8] = it->left_nz[8] = record_block(e, ctx, 1, 0, rd->y_dc);
    type = 0; first = 1;
  }
  for (int y = 0; y < 4; ++y)
    for (int x = 0; x < 4; ++x) {
      const int ctx = it->top_nz[x] + it->left_nz[y];
      it->top_nz[x] = it->left_nz[y] = record_block(e, ctx, type, first, rd->y_ac[x + 4 * y]);
    }
  for (int ch = 0; ch <= 2; ch += 2)
    for (int y = 0; y < 2; ++y)
      for (int x = 0; x < 2; ++x) {
        const int ctx = it->top_nz[4 + ch + x] + it->left_nz[4 + ch + y];
        it->top_nz[4 + ch + x] = it->left_nz[4 + ch + y] =
            record_block(e, ctx, 2, 0, rd->uv[2 * ch + x + 2 * y]);
      }
  flags_to_nz(it);
}

/* ------------------------------------------------------------------------ */
/* Frame loop and bitstream: frame_enc.c:563-572,783-894,
 * tree_enc.c:270-347,485-504, syntax_enc.c:149-389, filter_enc.c:194-233 */

static void code_intra_modes(Enc* e, BW* bw) {
  const int pw = e->preds_w;
  for (int y = 0; y < e->mbh; ++y)
    for (int x = 0; x < e->mbw; ++x) {
      const int i = y * e->mbw + x;
      const uint8_t* preds = e->preds + 4 * y * pw + 4 * x;
      if (e->update_map) {
        const int s = e->mb_seg[i];
        const uint8_t* p = e->seg_probas;
        if (bw_put(bw, s >= 2, p[0])) p += 1;
        bw_put(bw, s & 1, p[1]);
      }
      if (e->use_skip) bw_put(bw, e->mb_skip[i], e->skip_proba);   /* tree_enc.c:323-325 */
      if (bw_put(bw, e->mb_type[i] != 0, 145)) {
        const int m = preds[0];
        if (bw_put(bw, m == 1 || m == 3, 156)) bw_put(bw, m == 1, 128);
        else bw_put(bw, m == 2, 163);
      } else {
        const uint8_t* top = preds - pw;
        for (int yy = 0; yy < 4; ++yy) {
          int left = preds[-1];
          for (int xx = 0; xx < 4; ++xx) {
            const uint8_t* pr = kVP8BModeProba[top[xx]][left];
            const int m = preds[xx];
            if (bw_put(bw, m != 0, pr[0]) && bw_put(bw, m != 1, pr[1]) &&
                bw_put(bw, m != 2, pr[2])) {
              if (!bw_put(bw, m >= 6, pr[3])) {
                if (bw_put(bw, m != 3, pr[4])) bw_put(bw, m != 4, pr[5]);
              } else if (bw_put(bw, m != 6, pr[6])) {
                if (bw_put(bw, m != 7, pr[7])) bw_put(bw, m != 8, pr[8]);
              }
            }
            left = m;
          }
          top = preds;
          preds += pw;
        }
      }
      const int uvm = e->mb_uv[i];
      if (bw_put(bw, uvm != 0, 142) && bw_put(bw, uvm != 2, 114)) bw_put(bw, uvm != 3, 183);
    }
}

static void put_le32(uint8_t* p, uint32_t v) { p[0] = v; p[1] = v >> 8; p[2] = v >> 16; p[3] = v >> 24; }

static size_t write_stream(Enc* e, BW* parts, int nparts, uint8_t** out) {
  BW bw;
  bw_init(&bw);
  bw_put_uniform(&bw, 0);   /* colorspace */
  bw_put_uniform(&bw, 0);   /* clamp type */
  if (bw_put_uniform(&bw, e->num_segments > 1)) {
    bw_put_uniform(&bw, e->update_map);
    bw_put_uniform(&bw, 1);   /* update data */
    bw_put_uniform(&bw, 1);   /* absolute values */
    for (int s = 0; s < 4; ++s) bw_put_signed(&bw, e->dqm[s].quant, 7);
    for (int s = 0; s < 4; ++s) bw_put_signed(&bw, e->dqm[s].fstrength, 6);
    if (e->update_map)
      for (int s = 0; s < 3; ++s)
        if (bw_put_uniform(&bw, e->seg_probas[s] != 255u)) bw_put_bits(&bw, e->seg_probas[s], 8);
  }
  bw_put_uniform(&bw, e->f_simple);
  bw_put_bits(&bw, e->f_level, 6);
  bw_put_bits(&bw, e->f_sharpness, 3);
  bw_put_uniform(&bw, 0);       /* no lf delta */
  bw_put_bits(&bw, nparts == 8 ? 3 : nparts == 4 ? 2 : nparts == 2 ? 1 : 0, 2);
  bw_put_bits(&bw, e->base_quant, 7);
  bw_put_signed(&bw, 0, 4);
  bw_put_signed(&bw, 0, 4);
  bw_put_signed(&bw, 0, 4);
  bw_put_signed(&bw, e->dq_uv_dc, 4);
  bw_put_signed(&bw, e->dq_uv_ac, 4);
  bw_put_uniform(&bw, 0);       /* no proba refresh */
  for (int t = 0; t < 4; ++t)
    for (int b = 0; b < 8; ++b)
      for (int c = 0; c < 3; ++c)
        for (int p = 0; p < 11; ++p) {
          const int v = e->coeffs[t][b][c][p];
          if (bw_put(&bw, v != kVP8CoeffProba0[t][b][c][p], kVP8CoeffUpdateProba[t][b][c][p]))
            bw_put_bits(&bw, v, 8);
        }
  if (bw_put_uniform(&bw, e->use_skip)) bw_put_bits(&bw, e->skip_proba, 8);   /* tree_enc.c:500-502 */
  code_intra_modes(e, &bw);
  bw_finish(&bw);
  if (bw.error || bw.pos >= (1u << 19)) { free(bw.buf); return 0; }
  size_t size1 = 0;   /* the token partitions, EmitPartitionsSize (syntax_enc.c:248-265) */
  for (int p = 0; p < nparts; ++p) {
    if (parts[p].error || (p < nparts - 1 && parts[p].pos >= (1u << 24))) {
      free(bw.buf);
      return 0;
    }
    size1 += parts[p].pos;
  }
  const size_t size0 = bw.pos;
  size_t vp8_size = 10 + size0 + 3 * (size_t)(nparts - 1) + size1;
  const size_t pad = vp8_size & 1;
  vp8_size += pad;
  const size_t riff_size = 4 + 8 + vp8_size;
  const size_t total = 8 + riff_size;
  uint8_t* o = (uint8_t*)malloc(total);
  if (!o) { free(bw.buf); return 0; }
  memcpy(o, "RIFF", 4); put_le32(o + 4, (uint32_t)riff_size); memcpy(o + 8, "WEBP", 4);
  memcpy(o + 12, "VP8 ", 4); put_le32(o + 16, (uint32_t)vp8_size);
  const int use_filter = e->cfg.filter_strength > 0 || e->cfg.autofilter > 0;
  const int profile = use_filter ? (e->cfg.filter_type == 1 ? 0 : 1) : 2;
  const uint32_t bits = 0 | (profile << 1) | (1 << 4) | ((uint32_t)size0 << 5);
  uint8_t* f = o + 20;
  f[0] = bits; f[1] = bits >> 8; f[2] = bits >> 16;
  f[3] = 0x9d; f[4] = 0x01; f[5] = 0x2a;
  f[6] = e->w & 0xff; f[7] = e->w >> 8; f[8] = e->h & 0xff; f[9] = e->h >> 8;
  memcpy(o + 30, bw.buf, size0);
  uint8_t* d = o + 30 + size0;
  for (int p = 0; p < nparts - 1; ++p) {
    d[0] = (uint8_t)parts[p].pos; d[1] = (uint8_t)(parts[p].pos >> 8);
    d[2] = (uint8_t)(parts[p].pos >> 16);
    d += 3;
  }
  for (int p = 0; p < nparts; ++p) {
    if (parts[p].pos) memcpy(d, parts[p].buf, parts[p].pos);
    d += parts[p].pos;
  }
  if (pad) *d = 0;
  free(bw.buf);
  *out = o;
  return total;
}


/* ------------------------------------------------------------------------ */
/* Multi-pass convergence: frame_enc.c:26-80, 554-556, token_enc.c:226-247 */

#define DQ_LIMIT 0.4
#define HEADER_SIZE_ESTIMATE (12 + 8 + 10)

typedef struct {
  int is_first;
  float dq;
  float q, last_q;
  float qmin, qmax;
  double value, last_value;
  double target;
  int do_size_search;
} PassStats;

static float clampf(float v, float lo, float hi) { return (v < lo) ? lo : (v > hi) ? hi : v; }

static void init_pass_stats(PassStats* s, const vp8o_config* cfg) {
  const uint64_t target_size = (uint64_t)cfg->target_size;
  const int do_size_search = (target_size != 0);
  const float target_PSNR = cfg->target_PSNR;
  s->is_first = 1;
  s->dq = 10.f;
  s->qmin = 1.f * cfg->qmin;
  s->qmax = 1.f * cfg->qmax;
  s->q = s->last_q = clampf(cfg->quality, s->qmin, s->qmax);
  s->target = do_size_search ? (double)target_size : (target_PSNR > 0.) ? target_PSNR : 40.;
  s->value = s->last_value = 0.;
  s->do_size_search = do_size_search;
}

static float compute_next_q(PassStats* s) {
  float dq;
  if (s->is_first) {
    dq = (s->value > s->target) ? -s->dq : s->dq;
    s->is_first = 0;
  } else if (s->value != s->last_value) {
    const double slope = (s->target - s->value) / (s->last_value - s->value);
    dq = (float)(slope * (s->last_q - s->q));
  } else {
    dq = 0.;
  }
  s->dq = clampf(dq, -30.f, 30.f);
  s->last_q = s->q;
  s->last_value = s->value;
  s->q = clampf(s->q + s->dq, s->qmin, s->qmax);
  return s->q;
}

static double psnr_of(uint64_t mse, uint64_t size) {
  return (mse > 0 && size > 0) ? 10. * log10(255. * 255. * size / mse) : 99;
}

static uint64_t estimate_token_size(const Enc* e) {
  uint64_t size = 0;
  for (size_t k = 0; k < e->ntok; ++k) {
    const uint16_t t = e->tok[k];
    const int bit = (t >> 15) & 1;
    size += bit_cost(bit, (t & (1u << 14)) ? (t & 0xffu) : ((const uint8_t*)e->coeffs)[t & 0x3fffu]);
  }
  return size;
}


/* ------------------------------------------------------------------------ */
/* Autofilter (config->autofilter): per-MB SSIM of the reconstruction filtered
 * at the candidate levels, filter_enc.c:70-233, with the in-loop filters of
 * src/dsp/dec.c:484-692 and the SSIM of src/dsp/ssim.c:22-108 */

static inline int sclip1(int v) { return v < -128 ? -128 : v > 127 ? 127 : v; }   /* VP8ksclip1 */
static inline int sclip2(int v) { return v < -16 ? -16 : v > 15 ? 15 : v; }       /* VP8ksclip2 */
static inline int uclip1(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }         /* VP8kclip1 */

static void lf_filter2(uint8_t* p, int step) {   /* DoFilter2_C */
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
  p[-step] = uclip1(p0 + a2);
  p[0] = uclip1(q0 - a1);
}
static void lf_filter4(uint8_t* p, int step) {   /* DoFilter4_C */
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  const int a = 3 * (q0 - p0);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
  p[-2 * step] = uclip1(p1 + a3);
  p[-step] = uclip1(p0 + a2);
  p[0] = uclip1(q0 - a1);
  p[step] = uclip1(q1 - a3);
}
static int lf_hev(const uint8_t* p, int step, int t) {
  return iabs(p[-2 * step] - p[-step]) > t || iabs(p[step] - p[0]) > t;
}
static int lf_needs(const uint8_t* p, int step, int t) {   /* NeedsFilter_C */
  return 4 * iabs(p[-step] - p[0]) + iabs(p[-2 * step] - p[step]) <= t;
}
static int lf_needs2(const uint8_t* p, int step, int t, int it) {   /* NeedsFilter2_C */
  const int p3 = p[-4 * step], p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
  const int q0 = p[0], q1 = p[step], q2 = p[2 * step], q3 = p[3 * step];
  if (4 * iabs(p0 - q0) + iabs(p1 - q1) > t) return 0;
  return iabs(p3 - p2) <= it && iabs(p2 - p1) <= it && iabs(p1 - p0) <= it &&
         iabs(q3 - q2) <= it && iabs(q2 - q1) <= it && iabs(q1 - q0) <= it;
}
/* FilterLoop24_C: the inner-edge complex filter along one edge */
static void lf_loop24(uint8_t* p, int hs, int vs, int size, int thresh, int ithresh, int hev) {
  const int t2 = 2 * thresh + 1;
  for (; size-- > 0; p += vs)
    if (lf_needs2(p, hs, t2, ithresh)) {
      if (lf_hev(p, hs, hev)) lf_filter2(p, hs); else lf_filter4(p, hs);
    }
}
static void lf_simple(uint8_t* p, int hs, int vs, int thresh) {   /* Simple[HV]Filter16_C */
  const int t2 = 2 * thresh + 1;
  for (int i = 0; i < 16; ++i, p += vs)
    if (lf_needs(p, hs, t2)) lf_filter2(p, hs);
}

static int lf_ilevel(int sharpness, int level) {   /* GetILevel, filter_enc.c:70-83 */
  if (sharpness > 0) {
    level >>= (sharpness > 4) ? 2 : 1;
    if (level > 9 - sharpness) level = 9 - sharpness;
  }
  return level < 1 ? 1 : level;
}

static void lf_do_filter(const Enc* e, const uint8_t* rec, uint8_t* out, int level) {   /* :85-107 */
  const int ilevel = lf_ilevel(e->cfg.filter_sharpness, level);
  const int limit = 2 * level + ilevel;
  memcpy(out, rec, BPS * 16);
  if (e->f_simple) {
    for (int k = 1; k <= 3; ++k) lf_simple(out + 4 * k, 1, BPS, limit);        /* H, 16i */
    for (int k = 1; k <= 3; ++k) lf_simple(out + 4 * k * BPS, BPS, 1, limit);  /* V, 16i */
  } else {
    const int hev = (level >= 40) ? 2 : (level >= 15) ? 1 : 0;
    for (int k = 1; k <= 3; ++k) lf_loop24(out + 4 * k, 1, BPS, 16, limit, ilevel, hev);
    lf_loop24(out + 16 + 4, 1, BPS, 8, limit, ilevel, hev);          /* HFilter8i: u, v */
    lf_loop24(out + 24 + 4, 1, BPS, 8, limit, ilevel, hev);
    for (int k = 1; k <= 3; ++k) lf_loop24(out + 4 * k * BPS, BPS, 1, 16, limit, ilevel, hev);
    lf_loop24(out + 16 + 4 * BPS, BPS, 1, 8, limit, ilevel, hev);    /* VFilter8i */
    lf_loop24(out + 24 + 4 * BPS, BPS, 1, 8, limit, ilevel, hev);
  }
}

static double ssim_clipped(const uint8_t* s1, const uint8_t* s2, int xo, int yo, int W, int H) {
  static const uint32_t kW[7] = {1, 2, 3, 4, 3, 2, 1};
  uint32_t w = 0, xm = 0, ym = 0, xxm = 0, xym = 0, yym = 0;
  const int ymin = yo - 3 < 0 ? 0 : yo - 3, ymax = yo + 3 > H - 1 ? H - 1 : yo + 3;
  const int xmin = xo - 3 < 0 ? 0 : xo - 3, xmax = xo + 3 > W - 1 ? W - 1 : xo + 3;
  for (int y = ymin; y <= ymax; ++y)
    for (int x = xmin; x <= xmax; ++x) {
      const uint32_t wt = kW[3 + x - xo] * kW[3 + y - yo];
      const uint32_t a = s1[y * BPS + x], b = s2[y * BPS + x];
      w += wt; xm += wt * a; ym += wt * b;
      xxm += wt * a * a; xym += wt * a * b; yym += wt * b * b;
    }
  /* SSIMCalculation with N = w (ssim.c:28-52) */
  const uint32_t N = w, w2 = N * N;
  const uint32_t C1 = 20 * w2, C2 = 60 * w2, C3 = 8 * 8 * w2;
  const uint64_t xmxm = (uint64_t)xm * xm, ymym = (uint64_t)ym * ym;
  if (xmxm + ymym >= C3) {
    const int64_t xmym = (int64_t)xm * ym;
    const int64_t sxy = (int64_t)xym * N - xmym;
    const uint64_t sxx = (uint64_t)xxm * N - xmxm, syy = (uint64_t)yym * N - ymym;
    const uint64_t num_S = (2 * (uint64_t)(sxy < 0 ? 0 : sxy) + C2) >> 8;
    const uint64_t den_S = (sxx + syy + C2) >> 8;
    const uint64_t fnum = (2 * xmym + C1) * num_S;
    const uint64_t fden = (xmxm + ymym + C1) * den_S;
    return (double)fnum / fden;
  }
  return 1.;
}

static double mb_ssim(const uint8_t* a, const uint8_t* b) {   /* GetMBSSIM, :112-132 */
  double sum = 0.;
  for (int y = 3; y < 16 - 3; ++y)
    for (int x = 3; x < 16 - 3; ++x) sum += ssim_clipped(a, b, x, y, 16, 16);
  for (int x = 1; x < 7; ++x)
    for (int y = 1; y < 7; ++y) {
      sum += ssim_clipped(a + 16, b + 16, x, y, 8, 8);
      sum += ssim_clipped(a + 24, b + 24, x, y, 8, 8);
    }
  return sum;
}

static void store_filter_stats(const It* it, const Enc* e, double lf[4][64]) {   /* :156-192 */
  const int mi = it->y * e->mbw + it->x;
  const int s = e->mb_seg[mi];
  const int level0 = e->dqm[s].fstrength;
  const int dmin = -e->dqm[s].quant, dmax = e->dqm[s].quant;
  const int step = (dmax - dmin >= 4) ? 4 : 1;
  if (e->mb_type[mi] == 1 && e->mb_skip[mi]) return;
  lf[s][0] += mb_ssim(it->yin, it->out);
  uint8_t tmp[BPS * 16];
  for (int d = dmin; d <= dmax; d += step) {
    const int level = level0 + d;
    if (level <= 0 || level >= 64) continue;
    lf_do_filter(e, it->out, tmp, level);
    lf[s][level] += mb_ssim(it->yin, tmp);
  }
}

void vp8o_default_config(vp8o_config* c) {   /* config_enc.c:24-98 */
  memset(c, 0, sizeof(*c));
  c->quality = 75.f; c->method = 4; c->segments = 4; c->sns_strength = 50;
  c->filter_strength = 60; c->filter_sharpness = 0; c->filter_type = 1;
  c->pass = 1; c->qmin = 0; c->qmax = 100;
}

/* VP8EncLoop (frame_enc.c:740-775) for methods 0-2: StatLoop (:614-674,
 * without search) collects the token statistics over the first MBs
 * (method 0: a quarter of them) and the skip count, then the final pass codes
 * every MB with the final probabilities, skipping the residuals of all-zero
 * MBs when the skip probability pays (FinalizeSkipProba, :111-127). With
 * RD_OPT_NONE the decisions do not depend on the statistics, so both passes
 * decide the same. */
static void enc_loop(Enc* e, const vp8o_config* cfg, vp8o_mb_trace* trace, double (*lf)[64]) {
  const int nmb = e->mbw * e->mbh;
  int nb = nmb;
  It it;
  int stats_ok = 1;
  /* StatLoop decides with RD_OPT_BASIC from method 3 on (low_memory), else
   * RD_OPT_NONE; the final pass with the method's own level */
  const int final_rd = e->rd_opt, stat_rd = e->method >= 3 ? 1 : 0;
  if (e->method == 0) nb = (nmb > 200) ? nmb >> 2 : 50;   /* fast probe */
  if (e->method == 3) nb = (nmb > 200) ? nmb >> 1 : 100;
  memset(e->stats, 0, sizeof(e->stats));
  g_passes = 0;
  e->rd_opt = stat_rd;
  for (int pass = 0, npass = cfg->pass < 1 ? 1 : cfg->pass; pass < npass; ++pass) {
    int left = nb;   /* OneStatPass */
    uint64_t size_p0 = 0;
    it_reset(&it, e);
    const float q = cfg->quality < (float)cfg->qmin ? (float)cfg->qmin
                  : cfg->quality > (float)cfg->qmax ? (float)cfg->qmax : cfg->quality;
    set_segment_params(e, q < 0.f ? 0.f : q > 100.f ? 100.f : q);
    set_segment_probas(e);
    level_costs(e);
    e->nb_skip = 0;
    e->no_tokens = 1;
    do {
      Score rd;
      it_import(&it, e);
      if (decimate(&it, e, &rd)) ++e->nb_skip;
      record_tokens(&it, e, &rd);   /* RecordResiduals: statistics only */
      size_p0 += rd.H;
      it_save_boundary(&it, e);
    } while (it_next(&it, e) && --left > 0);
    ++g_passes;
    size_p0 += e->seg_hdr_size;
    if (e->max_i4_header_bits > 0 && size_p0 > P0_LIMIT) {   /* frame_enc.c:651-655 */
      e->max_i4_header_bits >>= 1;
      ++npass;
      continue;
    }
    /* OneStatPass returns the header estimate: the mode costs (0 with
     * RD_OPT_NONE) plus the segment header, and StatLoop gives up when it is
     * 0 (frame_enc.c:645-646), before FinalizeSkipProba/FinalizeTokenProbas:
     * default probabilities and no skip flags then */
    if (size_p0 == 0) { stats_ok = 0; break; }
    if (e->max_i4_header_bits == 0) break;   /* is_last_pass */
  }
  e->no_tokens = 0;
  if (stats_ok) {   /* FinalizeSkipProba + FinalizeTokenProbas */
    e->skip_proba = nmb ? (int)((uint64_t)(nmb - e->nb_skip) * 255 / nmb) : 255;
    e->use_skip = e->skip_proba < 250;
    finalize_token_probas(e);
    level_costs(e);
  } else {
    e->use_skip = 0;
  }
  /* final pass: the method's RD level with the level costs frozen */
  e->rd_opt = final_rd;
  if (lf) memset(lf, 0, 4 * 64 * sizeof(double));
  e->no_stats = 1;
  e->ntok = 0;
  it_reset(&it, e);
  do {
    Score rd;
    if (it.x == 0 && e->row_tok) e->row_tok[it.y] = e->ntok;
    it_import(&it, e);
    const int skip = decimate(&it, e, &rd);
    e->no_tokens = skip && e->use_skip;   /* ResetAfterSkip == the nz of coding zeros */
    record_tokens(&it, e, &rd);
    e->no_tokens = 0;
    if (trace) {
      vp8o_mb_trace* t = &trace[it.y * e->mbw + it.x];
      const int mi = it.y * e->mbw + it.x;
      t->segment = e->mb_seg[mi]; t->type = e->mb_type[mi];
      t->uv_mode = e->mb_uv[mi]; t->skip = e->mb_skip[mi];
      t->alpha = e->mb_alpha[mi];
      for (int k = 0; k < 16; ++k) t->modes[k] = it.preds[(k >> 2) * e->preds_w + (k & 3)];
      memcpy(t->y_dc, rd.y_dc, sizeof(t->y_dc));
      memcpy(t->y_ac, rd.y_ac, sizeof(t->y_ac));
      memcpy(t->uv, rd.uv, sizeof(t->uv));
    }
    if (lf) store_filter_stats(&it, e, lf);
    it_save_boundary(&it, e);
  } while (it_next(&it, e));
  e->no_stats = 0;
}

size_t vp8o_encode_yuv(const uint8_t* Y, const uint8_t* U, const uint8_t* V,
                       int w, int h, int ys, int uvs, const vp8o_config* cfg,
                       uint8_t** out, vp8o_mb_trace* trace) {
  Enc* e = (Enc*)calloc(1, sizeof(Enc));
  size_t result = 0;
  if (!e || cfg->method < 0 || cfg->method > 6) { free(e); return 0; }
  /* methods 0-2 with a size / PSNR search take StatLoop's RD_OPT_BASIC
   * passes (frame_enc.c:614-674): not restated */
  if ((cfg->method < 3 || cfg->low_memory) && (cfg->target_size > 0 || cfg->target_PSNR > 0)) {
    free(e);
    return 0;
  }
  e->Y = Y; e->U = U; e->V = V; e->ys = ys; e->uvs = uvs; e->w = w; e->h = h;
  e->mbw = (w + 15) >> 4; e->mbh = (h + 15) >> 4;
  e->cfg = *cfg;
  const int nmb = e->mbw * e->mbh;
  e->mb_type = (uint8_t*)calloc(nmb, 1); e->mb_uv = (uint8_t*)calloc(nmb, 1);
  e->mb_skip = (uint8_t*)calloc(nmb, 1); e->mb_seg = (uint8_t*)calloc(nmb, 1);
  e->mb_alpha = (uint8_t*)calloc(nmb, 1);
  e->preds_w = 4 * e->mbw + 1;
  e->preds_mem = (uint8_t*)calloc(e->preds_w * (4 * e->mbh + 1), 1);  /* border = B_DC_PRED */
  e->preds = e->preds_mem + 1 + e->preds_w;
  e->nz_mem = (uint32_t*)calloc(e->mbw + 1, sizeof(uint32_t));
  e->nz = e->nz_mem + 1;
  e->y_top = (uint8_t*)calloc(2 * 16 * e->mbw, 1);
  e->uv_top = e->y_top + 16 * e->mbw;
  if (cfg->quality <= 98 || cfg->pass > 1)   /* webp_enc.c:162-164 */
    e->top_derr = calloc(e->mbw, sizeof(*e->top_derr));
  /* MapConfigToTools, webp_enc.c:95-123 */
  e->method = cfg->method;
  e->rd_opt = cfg->method >= 6 ? 3 : cfg->method >= 5 ? 2 : cfg->method >= 3 ? 1 : 0;
  e->mb_header_limit = (score_t)256 * 510 * 8 * 1024 / (e->mbw * e->mbh);   /* webp_enc.c:109 */
  {
    const int lim = 100 - cfg->partition_limit;
    e->max_i4_header_bits = 256 * 16 * 16 * (lim * lim) / (100 * 100);
  }
  memcpy(e->coeffs, kVP8CoeffProba0, sizeof(e->coeffs));
  e->dirty = 1;
  memset(e->seg_probas, 255, 3);
  e->num_segments = cfg->segments;
  e->update_map = e->num_segments > 1;
  e->f_simple = 1; e->f_level = 0; e->f_sharpness = 0;

  analyze(e);

  BW part1[8];
  e->num_parts = (e->rd_opt == 0 || cfg->low_memory) ? 1 << cfg->partitions : 1;
  for (int p = 0; p < e->num_parts; ++p) bw_init(&part1[p]);
  if (e->num_parts > 1) e->row_tok = (size_t*)calloc((size_t)e->mbh + 1, sizeof(size_t));
  It it;
  double (*lf)[64] = cfg->autofilter ? (double (*)[64])calloc(4 * 64, sizeof(double)) : NULL;
  if (e->rd_opt == 0 || cfg->low_memory) {   /* VP8EncLoop: webp_enc.c:115-122 */
    enc_loop(e, cfg, trace, lf);
  } else {
    /* VP8EncTokenLoop (frame_enc.c:783-894): `pass` entropy passes, the
     * size / PSNR search of InitPassStats / ComputeNextQ (:47-80) and the
     * partition-0 overflow retry (:869-876) */
    g_passes = 0;
    const int max_count = (nmb >> 3) < 96 ? 96 : (nmb >> 3);
    PassStats ps;
    init_pass_stats(&ps, cfg);
    const int do_search = cfg->target_size > 0 || cfg->target_PSNR > 0;
    const uint64_t pixel_count = (uint64_t)nmb * 384;
    int num_pass_left = cfg->pass < 1 ? 1 : cfg->pass;
    while (num_pass_left-- > 0) {
      const int is_last_pass = (fabs(ps.dq) <= DQ_LIMIT) || (num_pass_left == 0) ||
                               (e->max_i4_header_bits == 0);
      uint64_t size_p0 = 0, distortion = 0;
      int cnt = max_count;
      it_reset(&it, e);
      /* SetLoopParams (:563-572) */
      const float q = ps.q < 0.f ? 0.f : ps.q > 100.f ? 100.f : ps.q;
      set_segment_params(e, q);
      set_segment_probas(e);
      level_costs(e);
      if (is_last_pass) memset(e->stats, 0, sizeof(e->stats));
      if (is_last_pass && lf) memset(lf, 0, 4 * 64 * sizeof(double));   /* VP8InitFilter */
      e->ntok = 0;
      do {
        Score rd;
        it_import(&it, e);
        if (--cnt < 0) {
          finalize_token_probas(e);
          level_costs(e);
          cnt = max_count;
        }
        decimate(&it, e, &rd);
        record_tokens(&it, e, &rd);
        size_p0 += rd.H;
        distortion += rd.D;
        if (is_last_pass && lf) store_filter_stats(&it, e, lf);
        if (trace && is_last_pass) {
          vp8o_mb_trace* t = &trace[it.y * e->mbw + it.x];
          const int mi = it.y * e->mbw + it.x;
          t->segment = e->mb_seg[mi]; t->type = e->mb_type[mi];
          t->uv_mode = e->mb_uv[mi]; t->skip = e->mb_skip[mi];
          t->alpha = e->mb_alpha[mi];
          for (int k = 0; k < 16; ++k) t->modes[k] = it.preds[(k >> 2) * e->preds_w + (k & 3)];
          memcpy(t->y_dc, rd.y_dc, sizeof(t->y_dc));
          memcpy(t->y_ac, rd.y_ac, sizeof(t->y_ac));
          memcpy(t->uv, rd.uv, sizeof(t->uv));
        }
        it_save_boundary(&it, e);
      } while (it_next(&it, e));
      size_p0 += e->seg_hdr_size;
      ++g_passes;
      g_size_p0 = size_p0;
      if (e->tok_err) break;
      if (ps.do_size_search) {
        uint64_t size = (uint64_t)finalize_token_probas(e);
        size += estimate_token_size(e);
        size = (size + size_p0 + 1024) >> 11;
        size += HEADER_SIZE_ESTIMATE;
        ps.value = (double)size;
      } else {
        ps.value = psnr_of(distortion, pixel_count);
      }
      if (e->max_i4_header_bits > 0 && size_p0 > P0_LIMIT) {
        ++num_pass_left;
        e->max_i4_header_bits >>= 1;
        continue;
      }
      if (is_last_pass) break;
      if (do_search) compute_next_q(&ps);
    }
  }
  if (e->tok_err) goto done;
  if (e->rd_opt > 0 && !cfg->low_memory)   /* enc_loop has settled its probabilities */
    finalize_token_probas(e);
  if (e->row_tok) e->row_tok[e->mbh] = e->ntok;
  for (int y = 0; y < (e->row_tok ? e->mbh : 1); ++y) {   /* VP8EmitTokens per partition */
    BW* pb = &part1[y & (e->num_parts - 1)];
    const size_t k0 = e->row_tok ? e->row_tok[y] : 0, k1 = e->row_tok ? e->row_tok[y + 1] : e->ntok;
    for (size_t k = k0; k < k1; ++k) {
      const uint16_t t = e->tok[k];
      const int bit = t >> 15;
      bw_put(pb, bit, (t & (1u << 14)) ? (t & 0xff) : ((const uint8_t*)e->coeffs)[t & 0x3fff]);
    }
  }
  for (int p = 0; p < e->num_parts; ++p) bw_finish(&part1[p]);
  if (lf) {   /* VP8AdjustFilterStrength with -af (filter_enc.c:197-212) */
    for (int sg = 0; sg < 4; ++sg) {
      int best_level = 0;
      double best_v = 1.00001 * lf[sg][0];
      for (int i = 1; i < 64; ++i)
        if (lf[sg][i] > best_v) { best_v = lf[sg][i]; best_level = i; }
      e->dqm[sg].fstrength = best_level;
    }
  } else if (cfg->filter_strength > 0) {   /* VP8AdjustFilterStrength without -af */
    int max_level = 0;
    for (int s = 0; s < 4; ++s) {
      Seg* d = &e->dqm[s];
      const int delta = (d->max_edge * d->y2.q[1]) >> 3;
      const int lvl = kVP8LevelsFromDelta[e->f_sharpness][delta < 64 ? delta : 63];
      if (lvl > d->fstrength) d->fstrength = lvl;
      if (max_level < d->fstrength) max_level = d->fstrength;
    }
    e->f_level = max_level;
  }
  result = write_stream(e, part1, e->num_parts, out);
done:
  free(lf);
  for (int p = 0; p < e->num_parts; ++p) free(part1[p].buf);
  free(e->row_tok);
  free(e->tok); free(e->mb_type); free(e->mb_uv); free(e->mb_skip); free(e->mb_seg);
  free(e->mb_alpha); free(e->preds_mem); free(e->nz_mem); free(e->y_top); free(e->top_derr);
  free(e);
  return result;
}

size_t vp8o_encode_rgba(const uint8_t* rgba, int w, int h, int stride,
                        const vp8o_config* cfg, uint8_t** out) {
  const int uw = (w + 1) >> 1, uh = (h + 1) >> 1;
  uint8_t* buf = (uint8_t*)malloc((size_t)w * h + 2 * (size_t)uw * uh);
  if (!buf) return 0;
  uint8_t *Y = buf, *U = buf + (size_t)w * h, *V = U + (size_t)uw * uh;
  size_t r = 0;
  /* sharp conversion only from 4x4 up (picture_csp_enc.c:165,493-496) */
  const int sharp = cfg->use_sharp_yuv && w >= 4 && h >= 4;
  int opaque = 1;
  for (int j = 0; j < h && opaque; ++j)
    for (int i = 0; i < w; ++i)
      if (rgba[(size_t)j * stride + 4 * i + 3] != 0xff) { opaque = 0; break; }
  float dither = 0.f;   /* preprocessing & 2, webp_enc.c:357-365 */
  if (cfg->preprocessing & 2) {
    const float x = cfg->quality / 100.f;
    const float x2 = x * x;
    dither = 1.0f + (0.5f - 1.0f) * x2 * x2;
  }
  if (opaque && (sharp ? vp8o_sharp_import_rgba(rgba, w, h, stride, Y, U, V)
                 : dither > 0.f ? vp8o_import_rgba_dithered(rgba, w, h, stride, dither, Y, U, V)
                                : vp8o_import_rgba(rgba, w, h, stride, Y, U, V)))
    r = vp8o_encode_yuv(Y, U, V, w, h, w, uw, cfg, out, NULL);
  free(buf);
  return r;
}

void vp8o_free(void* p) { free(p); }
int vp8o_last_pass_count(void) { return g_passes; }
double vp8o_last_p0_fraction(void) { return (double)g_size_p0 / (double)P0_LIMIT; }
