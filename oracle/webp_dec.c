/* Test infrastructure only (see oracle/Makefile): an own WebP decoder, so
 * that decode-side checks (lossy decode, lossless
 * pixel exactness, the ALPH plane) run on the GPU box without any reference
 * code. It restates the normative decode of libwebp 1.3.2 -- not its
 * structure: whole frames, no incremental decoding, no SIMD, no row cache.
 *
 *   container  src/dec/webp_dec.c (RIFF, VP8 / VP8L / VP8X + ALPH chunks)
 *   VP8        src/dec/vp8_dec.c:160-640 (headers, residuals), tree_dec.c
 *              (modes, probabilities), quant_dec.c:62-111 (dequantisation),
 *              frame_dec.c:60-314 (reconstruction, filter strengths),
 *              src/dsp/dec.c (transforms, intra predictors, loop filters)
 *   VP8L       src/dec/vp8l_dec.c (Huffman codes, LZ77, colour cache,
 *              transforms), src/dsp/lossless.c (inverse transforms)
 *   ALPH       src/dec/alpha_dec.c, src/dsp/filters.c:192-234 (unfilters)
 *   RGBA       src/dec/io_dec.c:57-111 + src/dsp/upsampling.c:37-97 (fancy
 *              upsampler) + src/dsp/yuv.h (VP8YuvToRgb)
 *
 * Entry points (C ABI, bound by oracle/oracle.py):
 *   odec_info(data, size, &w, &h, &has_alpha, &lossless)
 *   odec_decode_rgba(data, size, out[w*h*4])          -- WebPDecodeRGBA
 *   odec_decode_yuv(data, size, y[w*h], u[uw*uh], v)  -- VP8 only
 * Each returns 1 on success, 0 on a malformed or unsupported bitstream. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "vp8_tables.h"

/* ======================================================================
 * VP8 boolean decoder (RFC 6386 section 7; equivalent to
 * src/utils/bit_reader_utils.c + bit_reader_inl_utils.h: zeros past the end) */
typedef struct {
  const uint8_t *p, *end;
  uint32_t value, range;
  int bit_count;
} BoolDec;

static uint32_t bd_byte(BoolDec* d) { return d->p < d->end ? *d->p++ : 0; }

static void bd_init(BoolDec* d, const uint8_t* p, size_t n) {
  d->p = p;
  d->end = p + n;
  d->range = 255;
  d->bit_count = 0;
  d->value = bd_byte(d) << 8;
  d->value |= bd_byte(d);
}

static int bd_bit(BoolDec* d, int prob) {
  const uint32_t split = 1 + (((d->range - 1) * (uint32_t)prob) >> 8);
  const uint32_t big = split << 8;
  int bit;
  if (d->value >= big) {
    bit = 1;
    d->range -= split;
    d->value -= big;
  } else {
    bit = 0;
    d->range = split;
  }
  while (d->range < 128) {
    d->value <<= 1;
    d->range <<= 1;
    if (++d->bit_count == 8) {
      d->bit_count = 0;
      d->value |= bd_byte(d);
    }
  }
  return bit;
}

static int bd_value(BoolDec* d, int nbits) {   /* VP8GetValue: MSB first */
  int v = 0;
  while (nbits-- > 0) v = (v << 1) | bd_bit(d, 0x80);
  return v;
}

static int bd_signed_value(BoolDec* d, int nbits) {   /* VP8GetSignedValue */
  const int v = bd_value(d, nbits);
  return bd_bit(d, 0x80) ? -v : v;
}

/* ======================================================================
 * VP8 frame */
#define BPS 32
enum { B_DC = 0, B_TM, B_VE, B_HE, B_RD, B_VR, B_LD, B_VL, B_HD, B_HU };
enum { DC_PRED = 0, TM_PRED, V_PRED, H_PRED };

static const uint8_t kZigzag[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
static const uint8_t kBands[17] = {0, 1, 2, 3, 6, 4, 5, 6, 6, 6, 6, 6, 6, 6, 6, 7, 0};

typedef struct {
  int w, h, mbw, mbh;
  int use_segment, update_map, absolute_delta;
  int quantizer[4], filter_strength[4];
  uint8_t seg_proba[3];
  int simple, level, sharpness, use_lf_delta;
  int ref_lf_delta[4], mode_lf_delta[4];
  int nparts;
  BoolDec br, parts[8];
  int q[4][3][2];   /* segment, {y1, y2, uv}, {dc, ac} */
  uint8_t proba[4][8][3][11];
  int use_skip, skip_p;
} VP8Frame;

static inline int clip_q(int v, int m) { return v < 0 ? 0 : v > m ? m : v; }

/* vp8_dec.c:261-378 + quant_dec.c:62-111 + tree_dec.c:500-537 */
static int vp8_headers(VP8Frame* F, const uint8_t* buf, size_t size) {
  memset(F, 0, sizeof(*F));
  if (size < 10) return 0;
  const uint32_t bits = buf[0] | (buf[1] << 8) | (buf[2] << 16);
  const int key = !(bits & 1), show = (bits >> 4) & 1;
  const uint32_t p0len = bits >> 5;
  if (!key || !show || ((bits >> 1) & 7) > 3) return 0;
  if (buf[3] != 0x9d || buf[4] != 0x01 || buf[5] != 0x2a) return 0;
  F->w = ((buf[7] << 8) | buf[6]) & 0x3fff;
  F->h = ((buf[9] << 8) | buf[8]) & 0x3fff;
  if (F->w == 0 || F->h == 0) return 0;
  F->mbw = (F->w + 15) >> 4;
  F->mbh = (F->h + 15) >> 4;
  buf += 10;
  size -= 10;
  if (p0len > size) return 0;
  BoolDec* br = &F->br;
  bd_init(br, buf, p0len);
  buf += p0len;
  size -= p0len;
  bd_bit(br, 0x80);   /* colorspace */
  bd_bit(br, 0x80);   /* clamp type */
  memset(F->seg_proba, 255, 3);
  F->use_segment = bd_bit(br, 0x80);
  if (F->use_segment) {   /* ParseSegmentHeader, vp8_dec.c:161-190 */
    F->update_map = bd_bit(br, 0x80);
    if (bd_bit(br, 0x80)) {
      F->absolute_delta = bd_bit(br, 0x80);
      for (int s = 0; s < 4; ++s) F->quantizer[s] = bd_bit(br, 0x80) ? bd_signed_value(br, 7) : 0;
      for (int s = 0; s < 4; ++s)
        F->filter_strength[s] = bd_bit(br, 0x80) ? bd_signed_value(br, 6) : 0;
    }
    if (F->update_map)
      for (int s = 0; s < 3; ++s) F->seg_proba[s] = bd_bit(br, 0x80) ? bd_value(br, 8) : 255;
  }
  /* ParseFilterHeader, vp8_dec.c:238-259 */
  F->simple = bd_bit(br, 0x80);
  F->level = bd_value(br, 6);
  F->sharpness = bd_value(br, 3);
  F->use_lf_delta = bd_bit(br, 0x80);
  if (F->use_lf_delta && bd_bit(br, 0x80)) {
    for (int i = 0; i < 4; ++i)
      if (bd_bit(br, 0x80)) F->ref_lf_delta[i] = bd_signed_value(br, 6);
    for (int i = 0; i < 4; ++i)
      if (bd_bit(br, 0x80)) F->mode_lf_delta[i] = bd_signed_value(br, 6);
  }
  /* ParsePartitions, vp8_dec.c:201-235 */
  F->nparts = 1 << bd_value(br, 2);
  const size_t last = (size_t)F->nparts - 1;
  if (size < 3 * last) return 0;
  const uint8_t* sz = buf;
  const uint8_t* start = buf + 3 * last;
  size_t left = size - 3 * last;
  for (size_t p = 0; p < last; ++p) {
    size_t ps = sz[0] | (sz[1] << 8) | (sz[2] << 16);
    if (ps > left) ps = left;
    bd_init(&F->parts[p], start, ps);
    start += ps;
    left -= ps;
    sz += 3;
  }
  bd_init(&F->parts[last], start, left);
  /* VP8ParseQuant, quant_dec.c:62-111 */
  const int base_q0 = bd_value(br, 7);
  int dq[5];
  for (int i = 0; i < 5; ++i) dq[i] = bd_bit(br, 0x80) ? bd_signed_value(br, 4) : 0;
  for (int s = 0; s < 4; ++s) {
    int q = base_q0;
    if (F->use_segment) {
      q = F->quantizer[s] + (F->absolute_delta ? 0 : base_q0);
    } else if (s > 0) {
      memcpy(F->q[s], F->q[0], sizeof(F->q[0]));
      continue;
    }
    F->q[s][0][0] = kVP8DcQ[clip_q(q + dq[0], 127)];
    F->q[s][0][1] = kVP8AcQ[clip_q(q, 127)];
    F->q[s][1][0] = kVP8DcQ[clip_q(q + dq[1], 127)] * 2;
    F->q[s][1][1] = (kVP8AcQ[clip_q(q + dq[2], 127)] * 101581) >> 16;   /* x * 155 / 100 */
    if (F->q[s][1][1] < 8) F->q[s][1][1] = 8;
    F->q[s][2][0] = kVP8DcQ[clip_q(q + dq[3], 117)];
    F->q[s][2][1] = kVP8AcQ[clip_q(q + dq[4], 127)];
  }
  bd_bit(br, 0x80);   /* update_proba (ignored for key frames) */
  /* VP8ParseProba, tree_dec.c:500-537 */
  for (int t = 0; t < 4; ++t)
    for (int b = 0; b < 8; ++b)
      for (int c = 0; c < 3; ++c)
        for (int p = 0; p < 11; ++p)
          F->proba[t][b][c][p] = bd_bit(br, kVP8CoeffUpdateProba[t][b][c][p])
                                     ? (uint8_t)bd_value(br, 8)
                                     : kVP8CoeffProba0[t][b][c][p];
  F->use_skip = bd_bit(br, 0x80);
  if (F->use_skip) F->skip_p = bd_value(br, 8);
  return 1;
}

/* one macroblock's parse results (VP8MBData) */
typedef struct {
  int segment, skip, is_i4, uvmode;
  uint8_t imodes[16];
  int16_t coeffs[384];   /* 16 Y, 4 U, 4 V blocks of 16, natural order, dequantised */
  int nonzero;           /* any coefficient */
} MB;

/* ParseIntraMode, tree_dec.c:290-358 */
static void parse_modes(VP8Frame* F, BoolDec* br, MB* mb, uint8_t* top, uint8_t* left) {
  if (F->update_map) {
    mb->segment = !bd_bit(br, F->seg_proba[0]) ? bd_bit(br, F->seg_proba[1])
                                               : bd_bit(br, F->seg_proba[2]) + 2;
  } else {
    mb->segment = 0;
  }
  mb->skip = F->use_skip ? bd_bit(br, F->skip_p) : 0;
  mb->is_i4 = !bd_bit(br, 145);
  if (!mb->is_i4) {
    const int ymode = bd_bit(br, 156) ? (bd_bit(br, 128) ? TM_PRED : H_PRED)
                                      : (bd_bit(br, 163) ? V_PRED : DC_PRED);
    mb->imodes[0] = (uint8_t)ymode;
    memset(top, ymode, 4);
    memset(left, ymode, 4);
  } else {
    for (int y = 0; y < 4; ++y) {
      int ymode = left[y];
      for (int x = 0; x < 4; ++x) {
        const uint8_t* pr = kVP8BModeProba[top[x]][ymode];
        /* the intra-4 mode tree (RFC 6386 11.2; tree_dec.c:327-344) */
        if (!bd_bit(br, pr[0])) ymode = B_DC;
        else if (!bd_bit(br, pr[1])) ymode = B_TM;
        else if (!bd_bit(br, pr[2])) ymode = B_VE;
        else if (!bd_bit(br, pr[3]))
          ymode = !bd_bit(br, pr[4]) ? B_HE : (!bd_bit(br, pr[5]) ? B_RD : B_VR);
        else
          ymode = !bd_bit(br, pr[6]) ? B_LD
                  : (!bd_bit(br, pr[7]) ? B_VL : (!bd_bit(br, pr[8]) ? B_HD : B_HU));
        top[x] = (uint8_t)ymode;
      }
      memcpy(mb->imodes + 4 * y, top, 4);
      left[y] = (uint8_t)ymode;
    }
  }
  mb->uvmode = !bd_bit(br, 142) ? DC_PRED
               : !bd_bit(br, 114) ? V_PRED
               : bd_bit(br, 183) ? TM_PRED : H_PRED;
}

/* GetLargeValue, vp8_dec.c:403-438 */
static int large_value(BoolDec* br, const uint8_t* p) {
  int v;
  if (!bd_bit(br, p[3])) {
    if (!bd_bit(br, p[4])) v = 2;
    else v = 3 + bd_bit(br, p[5]);
  } else if (!bd_bit(br, p[6])) {
    if (!bd_bit(br, p[7])) {
      v = 5 + bd_bit(br, 159);
    } else {
      v = 7 + 2 * bd_bit(br, 165);
      v += bd_bit(br, 145);
    }
  } else {
    const int bit1 = bd_bit(br, p[8]);
    const int bit0 = bd_bit(br, p[9 + bit1]);
    const int cat = 2 * bit1 + bit0;
    static const uint8_t* const kCats[4] = {kVP8Cat3, kVP8Cat4, kVP8Cat5, kVP8Cat6};
    static const int kCatLen[4] = {3, 4, 5, 11};
    v = 0;
    for (int i = 0; i < kCatLen[cat]; ++i) v += v + bd_bit(br, kCats[cat][i]);
    v += 3 + (8 << cat);
  }
  return v;
}

/* GetCoeffs, vp8_dec.c:441-470: returns the last non-zero position + 1 */
static int get_coeffs(BoolDec* br, const uint8_t (*band)[3][11], int ctx, const int dq[2], int n,
                      int16_t* out) {
  const uint8_t* p = band[kBands[n]][ctx];
  for (; n < 16; ++n) {
    if (!bd_bit(br, p[0])) return n;
    while (!bd_bit(br, p[1])) {
      ++n;
      if (n == 16) return 16;
      p = band[kBands[n]][0];
    }
    int v;
    if (!bd_bit(br, p[2])) {
      v = 1;
      p = band[kBands[n + 1]][1];
    } else {
      v = large_value(br, p);
      p = band[kBands[n + 1]][2];
    }
    const int s = bd_bit(br, 0x80) ? -v : v;
    out[kZigzag[n]] = (int16_t)(s * dq[n > 0]);
  }
  return 16;
}

/* ParseResiduals, vp8_dec.c:510-608. tnz/lnz: this column's / the row's
 * left nz bits (4 Y, 2 U, 2 V), tdc/ldc the Y2 flags. Returns 1 when some
 * coefficient is non-zero. */
static int parse_residuals(VP8Frame* F, BoolDec* br, MB* mb, uint8_t* tnz_p, uint8_t* lnz_p,
                           uint8_t* tdc, uint8_t* ldc) {
  const int (*q)[2] = F->q[mb->segment];
  int16_t* dst = mb->coeffs;
  memset(dst, 0, sizeof(mb->coeffs));
  int first, any = 0;
  const uint8_t (*ac)[3][11];
  if (!mb->is_i4) {
    int16_t dc[16] = {0};
    const int nz = get_coeffs(br, F->proba[1], *tdc + *ldc, q[1], 0, dc);
    *tdc = *ldc = nz > 0;
    /* TransformWHT_C (src/dsp/dec.c:137-162) into the blocks' DC */
    int tmp[16];
    for (int i = 0; i < 4; ++i) {
      const int a0 = dc[0 + i] + dc[12 + i], a1 = dc[4 + i] + dc[8 + i];
      const int a2 = dc[4 + i] - dc[8 + i], a3 = dc[0 + i] - dc[12 + i];
      tmp[0 + i] = a0 + a1;
      tmp[8 + i] = a0 - a1;
      tmp[4 + i] = a3 + a2;
      tmp[12 + i] = a3 - a2;
    }
    for (int i = 0; i < 4; ++i) {
      const int d = tmp[0 + 4 * i] + 3;
      const int a0 = d + tmp[3 + 4 * i], a1 = tmp[1 + 4 * i] + tmp[2 + 4 * i];
      const int a2 = tmp[1 + 4 * i] - tmp[2 + 4 * i], a3 = d - tmp[3 + 4 * i];
      dst[64 * i + 0] = (int16_t)((a0 + a1) >> 3);
      dst[64 * i + 16] = (int16_t)((a3 + a2) >> 3);
      dst[64 * i + 32] = (int16_t)((a0 - a1) >> 3);
      dst[64 * i + 48] = (int16_t)((a3 - a2) >> 3);
    }
    first = 1;
    ac = F->proba[0];
  } else {
    first = 0;
    ac = F->proba[3];
  }
  uint8_t tnz = *tnz_p, lnz = *lnz_p;
  uint8_t ntnz = 0, nlnz = 0;
  for (int y = 0; y < 4; ++y) {
    int l = (lnz >> y) & 1;
    for (int x = 0; x < 4; ++x) {
      const int t = (tnz >> x) & 1;
      int16_t* blk = dst + 16 * (4 * y + x);
      const int nz = get_coeffs(br, ac, l + t, q[0], first, blk);
      l = nz > first;
      tnz = (uint8_t)((tnz & ~(1u << x)) | (l << x));
      if (nz > 1 || blk[0] != 0) any = 1;   /* NzCodeBits != 0, vp8_dec.c:503-507 */
    }
    nlnz |= (uint8_t)(l << y);
  }
  ntnz = tnz & 0x0f;
  for (int ch = 0; ch < 2; ++ch) {
    int16_t* base = dst + 256 + 64 * ch;
    uint8_t t2 = (uint8_t)((tnz >> (4 + 2 * ch)) & 3), l2 = (uint8_t)((lnz >> (4 + 2 * ch)) & 3);
    for (int y = 0; y < 2; ++y) {
      int l = (l2 >> y) & 1;
      for (int x = 0; x < 2; ++x) {
        const int t = (t2 >> x) & 1;
        int16_t* blk = base + 16 * (2 * y + x);
        const int nz = get_coeffs(br, F->proba[2], l + t, q[2], 0, blk);
        l = nz > 0;
        t2 = (uint8_t)((t2 & ~(1u << x)) | (l << x));
        if (nz > 1 || blk[0] != 0) any = 1;
      }
      l2 = (uint8_t)((l2 & ~(1u << y)) | (l << y));
    }
    ntnz |= (uint8_t)(t2 << (4 + 2 * ch));
    nlnz |= (uint8_t)(l2 << (4 + 2 * ch));
  }
  *tnz_p = ntnz;
  *lnz_p = nlnz;
  return any;
}

/* ---- reconstruction (frame_dec.c:72-190; src/dsp/dec.c) ---- */
static inline uint8_t clip8(int v) { return (v & ~0xff) == 0 ? (uint8_t)v : v < 0 ? 0 : 255; }

#define MUL1(a) ((((a) * 20091) >> 16) + (a))
#define MUL2(a) (((a) * 35468) >> 16)
static void itransform_add(const int16_t* in, uint8_t* dst) {   /* TransformOne_C */
  int C[16], *tmp = C;
  for (int i = 0; i < 4; ++i, ++in, tmp += 4) {
    const int a = in[0] + in[8], b = in[0] - in[8];
    const int c = MUL2(in[4]) - MUL1(in[12]), d = MUL1(in[4]) + MUL2(in[12]);
    tmp[0] = a + d;
    tmp[1] = b + c;
    tmp[2] = b - c;
    tmp[3] = a - d;
  }
  tmp = C;
  for (int i = 0; i < 4; ++i, ++tmp, dst += BPS) {
    const int dc = tmp[0] + 4;
    const int a = dc + tmp[8], b = dc - tmp[8];
    const int c = MUL2(tmp[4]) - MUL1(tmp[12]), d = MUL1(tmp[4]) + MUL2(tmp[12]);
    dst[0] = clip8(dst[0] + ((a + d) >> 3));
    dst[1] = clip8(dst[1] + ((b + c) >> 3));
    dst[2] = clip8(dst[2] + ((b - c) >> 3));
    dst[3] = clip8(dst[3] + ((a - d) >> 3));
  }
}
#undef MUL1
#undef MUL2

static void add_block(const int16_t* in, uint8_t* dst) {
  for (int i = 0; i < 16; ++i)
    if (in[i]) { itransform_add(in, dst); return; }
}

#define AVG3(a, b, c) ((uint8_t)(((a) + 2 * (b) + (c) + 2) >> 2))
#define AVG2(a, b) (((a) + (b) + 1) >> 1)
#define DST(x, y) dst[(x) + (y) * BPS]

static void pred_tm(uint8_t* dst, int size) {   /* TrueMotion */
  const uint8_t* top = dst - BPS;
  const int tl = top[-1];
  for (int y = 0; y < size; ++y, dst += BPS)
    for (int x = 0; x < size; ++x) dst[x] = clip8(top[x] + dst[-1] - tl);
}
static void pred_fill(uint8_t* dst, int size, int v) {
  for (int y = 0; y < size; ++y) memset(dst + y * BPS, v, size);
}
/* 16x16 / 8x8 (dec.c:201-262, 415-477); mode as CheckMode returns it:
 * DC_PRED variants by edge availability */
static void pred_block(uint8_t* dst, int size, int mode, int has_left, int has_top) {
  const int sh = size == 16 ? 4 : 3;
  if (mode == TM_PRED) {
    pred_tm(dst, size);
  } else if (mode == V_PRED) {
    for (int y = 0; y < size; ++y) memcpy(dst + y * BPS, dst - BPS, size);
  } else if (mode == H_PRED) {
    for (int y = 0; y < size; ++y) memset(dst + y * BPS, dst[y * BPS - 1], size);
  } else {   /* DC */
    int dc = 0;
    if (has_left && has_top) {
      for (int j = 0; j < size; ++j) dc += dst[-1 + j * BPS] + dst[j - BPS];
      dc = (dc + size) >> (sh + 1);
    } else if (has_left) {
      for (int j = 0; j < size; ++j) dc += dst[-1 + j * BPS];
      dc = (dc + (size >> 1)) >> sh;
    } else if (has_top) {
      for (int j = 0; j < size; ++j) dc += dst[j - BPS];
      dc = (dc + (size >> 1)) >> sh;
    } else {
      dc = 0x80;
    }
    pred_fill(dst, size, dc);
  }
}

/* 4x4 predictors, dec.c:283-412 */
static void pred4(uint8_t* dst, int mode) {
  const int I = dst[-1], J = dst[-1 + BPS], K = dst[-1 + 2 * BPS], L = dst[-1 + 3 * BPS];
  const int X = dst[-1 - BPS], A = dst[-BPS], B = dst[1 - BPS], C = dst[2 - BPS];
  const int D = dst[3 - BPS], E = dst[4 - BPS], F = dst[5 - BPS], G = dst[6 - BPS];
  const int H = dst[7 - BPS];
  switch (mode) {
    case B_DC: {
      int dc = 4;
      for (int i = 0; i < 4; ++i) dc += dst[i - BPS] + dst[-1 + i * BPS];
      pred_fill(dst, 4, dc >> 3);
      break;
    }
    case B_TM: pred_tm(dst, 4); break;
    case B_VE: {
      const uint8_t v[4] = {AVG3(X, A, B), AVG3(A, B, C), AVG3(B, C, D), AVG3(C, D, E)};
      for (int i = 0; i < 4; ++i) memcpy(dst + i * BPS, v, 4);
      break;
    }
    case B_HE: {
      const uint8_t r[4] = {AVG3(X, I, J), AVG3(I, J, K), AVG3(J, K, L), AVG3(K, L, L)};
      for (int i = 0; i < 4; ++i) memset(dst + i * BPS, r[i], 4);
      break;
    }
    case B_RD:
      DST(0, 3) = AVG3(J, K, L);
      DST(1, 3) = DST(0, 2) = AVG3(I, J, K);
      DST(2, 3) = DST(1, 2) = DST(0, 1) = AVG3(X, I, J);
      DST(3, 3) = DST(2, 2) = DST(1, 1) = DST(0, 0) = AVG3(A, X, I);
      DST(3, 2) = DST(2, 1) = DST(1, 0) = AVG3(B, A, X);
      DST(3, 1) = DST(2, 0) = AVG3(C, B, A);
      DST(3, 0) = AVG3(D, C, B);
      break;
    case B_LD:
      DST(0, 0) = AVG3(A, B, C);
      DST(1, 0) = DST(0, 1) = AVG3(B, C, D);
      DST(2, 0) = DST(1, 1) = DST(0, 2) = AVG3(C, D, E);
      DST(3, 0) = DST(2, 1) = DST(1, 2) = DST(0, 3) = AVG3(D, E, F);
      DST(3, 1) = DST(2, 2) = DST(1, 3) = AVG3(E, F, G);
      DST(3, 2) = DST(2, 3) = AVG3(F, G, H);
      DST(3, 3) = AVG3(G, H, H);
      break;
    case B_VR:
      DST(0, 0) = DST(1, 2) = AVG2(X, A);
      DST(1, 0) = DST(2, 2) = AVG2(A, B);
      DST(2, 0) = DST(3, 2) = AVG2(B, C);
      DST(3, 0) = AVG2(C, D);
      DST(0, 3) = AVG3(K, J, I);
      DST(0, 2) = AVG3(J, I, X);
      DST(0, 1) = DST(1, 3) = AVG3(I, X, A);
      DST(1, 1) = DST(2, 3) = AVG3(X, A, B);
      DST(2, 1) = DST(3, 3) = AVG3(A, B, C);
      DST(3, 1) = AVG3(B, C, D);
      break;
    case B_VL:
      DST(0, 0) = AVG2(A, B);
      DST(1, 0) = DST(0, 2) = AVG2(B, C);
      DST(2, 0) = DST(1, 2) = AVG2(C, D);
      DST(3, 0) = DST(2, 2) = AVG2(D, E);
      DST(0, 1) = AVG3(A, B, C);
      DST(1, 1) = DST(0, 3) = AVG3(B, C, D);
      DST(2, 1) = DST(1, 3) = AVG3(C, D, E);
      DST(3, 1) = DST(2, 3) = AVG3(D, E, F);
      DST(3, 2) = AVG3(E, F, G);
      DST(3, 3) = AVG3(F, G, H);
      break;
    case B_HU:
      DST(0, 0) = AVG2(I, J);
      DST(2, 0) = DST(0, 1) = AVG2(J, K);
      DST(2, 1) = DST(0, 2) = AVG2(K, L);
      DST(1, 0) = AVG3(I, J, K);
      DST(3, 0) = DST(1, 1) = AVG3(J, K, L);
      DST(3, 1) = DST(1, 2) = AVG3(K, L, L);
      DST(3, 2) = DST(2, 2) = DST(0, 3) = DST(1, 3) = DST(2, 3) = DST(3, 3) = L;
      break;
    default:   /* B_HD */
      DST(0, 0) = DST(2, 1) = AVG2(I, X);
      DST(0, 1) = DST(2, 2) = AVG2(J, I);
      DST(0, 2) = DST(2, 3) = AVG2(K, J);
      DST(0, 3) = AVG2(L, K);
      DST(3, 0) = AVG3(A, B, C);
      DST(2, 0) = AVG3(X, A, B);
      DST(1, 0) = DST(3, 1) = AVG3(I, X, A);
      DST(1, 1) = DST(3, 2) = AVG3(J, I, X);
      DST(1, 2) = DST(3, 3) = AVG3(K, J, I);
      DST(1, 3) = AVG3(L, K, J);
      break;
  }
}
#undef DST

/* decoded frame: planes of the full MB grid, unfiltered then filtered */
typedef struct {
  int yw, uvw;   /* strides: 16 * mbw, 8 * mbw */
  uint8_t *y, *u, *v;
  uint8_t* finfo;   /* per MB: filter limit (0 = none) */
  uint8_t* fil;     /* per MB: ilevel */
  uint8_t* fin;     /* per MB: inner edges */
  uint8_t* fhev;    /* per MB: hev threshold */
} Planes;

/* ReconstructRow for one MB, frame_dec.c:72-190: edges into a BPS work area,
 * predict + add residuals, copy back */
static void reconstruct_mb(const VP8Frame* F, Planes* P, const MB* mb, int mx, int my) {
  uint8_t ws[(1 + 16 + 1 + 8) * BPS];
  uint8_t* y = ws + BPS + 8;
  uint8_t* u = ws + (1 + 16 + 1) * BPS + 8;
  uint8_t* v = u + 16;
  const int ys = P->yw, us = P->uvw;
  uint8_t* Y = P->y + (size_t)my * 16 * ys + mx * 16;
  uint8_t* U = P->u + (size_t)my * 8 * us + mx * 8;
  uint8_t* V = P->v + (size_t)my * 8 * us + mx * 8;
  /* left column (129 at the frame edge) */
  for (int j = 0; j < 16; ++j) y[j * BPS - 1] = mx > 0 ? Y[j * ys - 1] : 129;
  for (int j = 0; j < 8; ++j) {
    u[j * BPS - 1] = mx > 0 ? U[j * us - 1] : 129;
    v[j * BPS - 1] = mx > 0 ? V[j * us - 1] : 129;
  }
  /* top row + top-left: 127 on the first row; 129 top-left at the left edge */
  if (my == 0) {
    memset(y - BPS - 1, 127, 16 + 4 + 1);
    memset(u - BPS - 1, 127, 9);
    memset(v - BPS - 1, 127, 9);
  } else {
    memcpy(y - BPS, Y - ys, 16);
    memcpy(u - BPS, U - us, 8);
    memcpy(v - BPS, V - us, 8);
    y[-BPS - 1] = mx > 0 ? Y[-ys - 1] : 129;
    u[-BPS - 1] = mx > 0 ? U[-us - 1] : 129;
    v[-BPS - 1] = mx > 0 ? V[-us - 1] : 129;
  }
  if (mb->is_i4) {
    uint8_t* tr = y - BPS + 16;
    if (my > 0) {
      if (mx >= F->mbw - 1) memset(tr, Y[-ys + 15], 4);
      else memcpy(tr, Y - ys + 16, 4);
    }
    for (int r = 1; r < 4; ++r) memcpy(tr + 4 * r * BPS, tr, 4);   /* replicated below */
    for (int n = 0; n < 16; ++n) {
      uint8_t* d = y + (n >> 2) * 4 * BPS + (n & 3) * 4;
      pred4(d, mb->imodes[n]);
      add_block(mb->coeffs + 16 * n, d);
    }
  } else {
    pred_block(y, 16, mb->imodes[0], mx > 0, my > 0);
    for (int n = 0; n < 16; ++n)
      add_block(mb->coeffs + 16 * n, y + (n >> 2) * 4 * BPS + (n & 3) * 4);
  }
  pred_block(u, 8, mb->uvmode, mx > 0, my > 0);
  pred_block(v, 8, mb->uvmode, mx > 0, my > 0);
  for (int n = 0; n < 4; ++n) {
    add_block(mb->coeffs + 256 + 16 * n, u + (n >> 1) * 4 * BPS + (n & 1) * 4);
    add_block(mb->coeffs + 320 + 16 * n, v + (n >> 1) * 4 * BPS + (n & 1) * 4);
  }
  for (int j = 0; j < 16; ++j) memcpy(Y + j * ys, y + j * BPS, 16);
  for (int j = 0; j < 8; ++j) {
    memcpy(U + j * us, u + j * BPS, 8);
    memcpy(V + j * us, v + j * BPS, 8);
  }
}

/* ---- loop filter, src/dsp/dec.c:480-700 ---- */
static inline int sclip1(int v) { return v < -128 ? -128 : v > 127 ? 127 : v; }   /* VP8ksclip1 */
static inline int sclip2(int v) { return v < -16 ? -16 : v > 15 ? 15 : v; }       /* VP8ksclip2 */
static inline int iabs(int v) { return v < 0 ? -v : v; }

static void do_filter2(uint8_t* p, int step) {
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
  p[-step] = clip8(p0 + a2);
  p[0] = clip8(q0 - a1);
}
static void do_filter4(uint8_t* p, int step) {
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  const int a = 3 * (q0 - p0);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
  p[-2 * step] = clip8(p1 + a3);
  p[-step] = clip8(p0 + a2);
  p[0] = clip8(q0 - a1);
  p[step] = clip8(q1 - a3);
}
static void do_filter6(uint8_t* p, int step) {
  const int p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
  const int q0 = p[0], q1 = p[step], q2 = p[2 * step];
  const int a = sclip1(3 * (q0 - p0) + sclip1(p1 - q1));
  const int a1 = (27 * a + 63) >> 7, a2 = (18 * a + 63) >> 7, a3 = (9 * a + 63) >> 7;
  p[-3 * step] = clip8(p2 + a3);
  p[-2 * step] = clip8(p1 + a2);
  p[-step] = clip8(p0 + a1);
  p[0] = clip8(q0 - a1);
  p[step] = clip8(q1 - a2);
  p[2 * step] = clip8(q2 - a3);
}
static int hev(const uint8_t* p, int step, int t) {
  return iabs(p[-2 * step] - p[-step]) > t || iabs(p[step] - p[0]) > t;
}
static int needs(const uint8_t* p, int step, int t) {
  return 4 * iabs(p[-step] - p[0]) + iabs(p[-2 * step] - p[step]) <= t;
}
static int needs2(const uint8_t* p, int step, int t, int it) {
  const int p3 = p[-4 * step], p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
  const int q0 = p[0], q1 = p[step], q2 = p[2 * step], q3 = p[3 * step];
  if (4 * iabs(p0 - q0) + iabs(p1 - q1) > t) return 0;
  return iabs(p3 - p2) <= it && iabs(p2 - p1) <= it && iabs(p1 - p0) <= it &&
         iabs(q3 - q2) <= it && iabs(q2 - q1) <= it && iabs(q1 - q0) <= it;
}
/* FilterLoop26_C / FilterLoop24_C */
static void loop(uint8_t* p, int hs, int vs, int size, int thresh, int ithresh, int hevt,
                 int six) {
  const int t2 = 2 * thresh + 1;
  for (int i = 0; i < size; ++i, p += vs) {
    if (!needs2(p, hs, t2, ithresh)) continue;
    if (hev(p, hs, hevt)) do_filter2(p, hs);
    else if (six) do_filter6(p, hs);
    else do_filter4(p, hs);
  }
}
static void simple_edge(uint8_t* p, int hs, int vs, int thresh) {   /* Simple[HV]Filter16_C */
  const int t2 = 2 * thresh + 1;
  for (int i = 0; i < 16; ++i, p += vs)
    if (needs(p, hs, t2)) do_filter2(p, hs);
}

/* DoFilter, frame_dec.c:214-259, in raster order over the whole frame */
static void filter_frame(const VP8Frame* F, Planes* P) {
  const int ys = P->yw, us = P->uvw;
  for (int my = 0; my < F->mbh; ++my)
    for (int mx = 0; mx < F->mbw; ++mx) {
      const int i = my * F->mbw + mx;
      const int limit = P->finfo[i];
      if (limit == 0) continue;
      const int il = P->fil[i], inner = P->fin[i], ht = P->fhev[i];
      uint8_t* y = P->y + (size_t)my * 16 * ys + mx * 16;
      if (F->simple) {
        if (mx > 0) simple_edge(y, 1, ys, limit + 4);
        if (inner)
          for (int k = 1; k < 4; ++k) simple_edge(y + 4 * k, 1, ys, limit);
        if (my > 0) simple_edge(y, ys, 1, limit + 4);
        if (inner)
          for (int k = 1; k < 4; ++k) simple_edge(y + 4 * k * ys, ys, 1, limit);
      } else {
        uint8_t* u = P->u + (size_t)my * 8 * us + mx * 8;
        uint8_t* v = P->v + (size_t)my * 8 * us + mx * 8;
        if (mx > 0) {
          loop(y, 1, ys, 16, limit + 4, il, ht, 1);
          loop(u, 1, us, 8, limit + 4, il, ht, 1);
          loop(v, 1, us, 8, limit + 4, il, ht, 1);
        }
        if (inner) {
          for (int k = 1; k < 4; ++k) loop(y + 4 * k, 1, ys, 16, limit, il, ht, 0);
          loop(u + 4, 1, us, 8, limit, il, ht, 0);
          loop(v + 4, 1, us, 8, limit, il, ht, 0);
        }
        if (my > 0) {
          loop(y, ys, 1, 16, limit + 4, il, ht, 1);
          loop(u, us, 1, 8, limit + 4, il, ht, 1);
          loop(v, us, 1, 8, limit + 4, il, ht, 1);
        }
        if (inner) {
          for (int k = 1; k < 4; ++k) loop(y + 4 * k * ys, ys, 1, 16, limit, il, ht, 0);
          loop(u + 4 * us, us, 1, 8, limit, il, ht, 0);
          loop(v + 4 * us, us, 1, 8, limit, il, ht, 0);
        }
      }
    }
}

/* PrecomputeFilterStrengths, frame_dec.c:266-314 */
static void filter_strength(const VP8Frame* F, int seg, int i4, int* limit, int* ilevel,
                            int* hevt) {
  int level = F->level;
  if (F->use_segment) level = F->filter_strength[seg] + (F->absolute_delta ? 0 : F->level);
  if (F->use_lf_delta) {
    level += F->ref_lf_delta[0];
    if (i4) level += F->mode_lf_delta[0];
  }
  level = level < 0 ? 0 : level > 63 ? 63 : level;
  *limit = 0;
  if (level > 0) {
    int il = level;
    if (F->sharpness > 0) {
      il >>= F->sharpness > 4 ? 2 : 1;
      if (il > 9 - F->sharpness) il = 9 - F->sharpness;
    }
    if (il < 1) il = 1;
    *ilevel = il;
    *limit = 2 * level + il;
    *hevt = level >= 40 ? 2 : level >= 15 ? 1 : 0;
  }
}

/* VP8 key frame -> Y/U/V planes of the MB grid (caller frees P->y/u/v) */
static int vp8_decode(const uint8_t* data, size_t size, VP8Frame* F, Planes* P) {
  if (!vp8_headers(F, data, size)) return 0;
  const int mbw = F->mbw, mbh = F->mbh, nmb = mbw * mbh;
  P->yw = 16 * mbw;
  P->uvw = 8 * mbw;
  P->y = (uint8_t*)calloc((size_t)P->yw * 16 * mbh, 1);
  P->u = (uint8_t*)calloc((size_t)P->uvw * 8 * mbh, 1);
  P->v = (uint8_t*)calloc((size_t)P->uvw * 8 * mbh, 1);
  P->finfo = (uint8_t*)calloc((size_t)nmb * 4, 1);
  uint8_t* intra_t = (uint8_t*)calloc((size_t)4 * mbw, 1);
  uint8_t* tnz = (uint8_t*)calloc((size_t)mbw, 1);
  uint8_t* tdc = (uint8_t*)calloc((size_t)mbw, 1);
  MB* mb = (MB*)malloc(sizeof(MB));
  int ok = P->y && P->u && P->v && P->finfo && intra_t && tnz && tdc && mb;
  if (ok) {
    P->fil = P->finfo + nmb;
    P->fin = P->fil + nmb;
    P->fhev = P->fin + nmb;
    const int filter_type = F->level == 0 ? 0 : F->simple ? 1 : 2;
    for (int my = 0; my < mbh; ++my) {
      uint8_t intra_l[4] = {B_DC, B_DC, B_DC, B_DC};
      uint8_t lnz = 0, ldc = 0;
      BoolDec* tb = &F->parts[my & (F->nparts - 1)];
      for (int mx = 0; mx < mbw; ++mx) {
        parse_modes(F, &F->br, mb, intra_t + 4 * mx, intra_l);
        int skip = mb->skip;
        if (!skip) {
          skip = !parse_residuals(F, tb, mb, &tnz[mx], &lnz, &tdc[mx], &ldc);
        } else {   /* VP8DecodeMB, vp8_dec.c:612-625 */
          memset(mb->coeffs, 0, sizeof(mb->coeffs));
          tnz[mx] = lnz = 0;
          if (!mb->is_i4) tdc[mx] = ldc = 0;
        }
        reconstruct_mb(F, P, mb, mx, my);
        if (filter_type > 0) {
          int limit, il = 0, ht = 0;
          filter_strength(F, mb->segment, mb->is_i4, &limit, &il, &ht);
          const int i = my * mbw + mx;
          P->finfo[i] = (uint8_t)limit;
          P->fil[i] = (uint8_t)il;
          P->fin[i] = (uint8_t)(mb->is_i4 | !skip);
          P->fhev[i] = (uint8_t)ht;
        }
      }
    }
    if (filter_type > 0) filter_frame(F, P);
  }
  free(intra_t);
  free(tnz);
  free(tdc);
  free(mb);
  free(P->finfo);
  P->finfo = NULL;
  if (!ok) {
    free(P->y); free(P->u); free(P->v);
    P->y = P->u = P->v = NULL;
  }
  return ok;
}

/* ======================================================================
 * VP8L (src/dec/vp8l_dec.c; LSB-first bit reader) */
typedef struct {
  const uint8_t* p;
  size_t n, pos;   /* bit position */
  int eos;
} LBits;

static uint32_t lb_read(LBits* b, int nbits) {   /* VP8LReadBits */
  uint32_t v = 0;
  for (int i = 0; i < nbits; ++i, ++b->pos) {
    const size_t byte = b->pos >> 3;
    if (byte >= b->n) { b->eos = 1; continue; }
    v |= (uint32_t)((b->p[byte] >> (b->pos & 7)) & 1) << i;
  }
  return v;
}

/* canonical Huffman code as (length, code) per symbol, decoded bit by bit
 * through a first-code / offset table per length (the code the table of
 * huffman_utils.c:BuildHuffmanTable describes) */
typedef struct {
  int nsym, single;   /* single: one used symbol, read with 0 bits */
  int count[16], first[16], offset[16];
  int* sorted;        /* symbols by (length, value) */
} Huff;

static int huff_build(Huff* h, const int* lens, int n) {
  memset(h, 0, sizeof(*h));
  h->sorted = (int*)malloc(sizeof(int) * (n > 0 ? n : 1));
  if (!h->sorted) return 0;
  int used = 0, last = 0;
  for (int i = 0; i < n; ++i)
    if (lens[i] > 0) { h->count[lens[i]]++; ++used; last = i; }
  h->nsym = used;
  if (used == 0) return 0;
  if (used == 1) { h->single = 1; h->sorted[0] = last; return 1; }
  /* completeness (huffman_utils.c:170-185: incomplete or over-subscribed codes fail) */
  int left = 1;
  for (int l = 1; l < 16; ++l) {
    left <<= 1;
    left -= h->count[l];
    if (left < 0) return 0;
  }
  if (left != 0) return 0;
  int code = 0, k = 0;
  for (int l = 1; l < 16; ++l) {
    h->first[l] = code;
    h->offset[l] = k;
    code = (code + h->count[l]) << 1;
    k += h->count[l];
  }
  int fill[16];
  memcpy(fill, h->offset, sizeof(fill));
  for (int i = 0; i < n; ++i)
    if (lens[i] > 0) h->sorted[fill[lens[i]]++] = i;
  return 1;
}

static int huff_read(const Huff* h, LBits* b) {
  if (h->single) return h->sorted[0];
  int code = 0;
  for (int l = 1; l < 16; ++l) {
    code = (code << 1) | (int)lb_read(b, 1);   /* codes are stored MSB-first, bit by bit */
    const int d = code - h->first[l];
    if (d < h->count[l]) return h->sorted[h->offset[l] + d];
  }
  b->eos = 1;
  return 0;
}

static const int kAlphabet[5] = {256 + 24, 256, 256, 256, 40};
static const uint8_t kCodeLengthOrder[19] = {17, 18, 0, 1, 2, 3, 4, 5, 16, 6,
                                             7, 8, 9, 10, 11, 12, 13, 14, 15};
static const uint8_t kCodeToPlane[120] = {
    0x18, 0x07, 0x17, 0x19, 0x28, 0x06, 0x27, 0x29, 0x16, 0x1a, 0x26, 0x2a, 0x38, 0x05, 0x37,
    0x39, 0x15, 0x1b, 0x36, 0x3a, 0x25, 0x2b, 0x48, 0x04, 0x47, 0x49, 0x14, 0x1c, 0x35, 0x3b,
    0x46, 0x4a, 0x24, 0x2c, 0x58, 0x45, 0x4b, 0x34, 0x3c, 0x03, 0x57, 0x59, 0x13, 0x1d, 0x56,
    0x5a, 0x23, 0x2d, 0x44, 0x4c, 0x55, 0x5b, 0x33, 0x3d, 0x68, 0x02, 0x67, 0x69, 0x12, 0x1e,
    0x66, 0x6a, 0x22, 0x2e, 0x54, 0x5c, 0x43, 0x4d, 0x65, 0x6b, 0x32, 0x3e, 0x78, 0x01, 0x77,
    0x79, 0x53, 0x5d, 0x11, 0x1f, 0x64, 0x6c, 0x42, 0x4e, 0x76, 0x7a, 0x21, 0x2f, 0x75, 0x7b,
    0x31, 0x3f, 0x63, 0x6d, 0x52, 0x5e, 0x00, 0x74, 0x7c, 0x41, 0x4f, 0x10, 0x20, 0x62, 0x6e,
    0x30, 0x73, 0x7d, 0x51, 0x5f, 0x40, 0x72, 0x7e, 0x61, 0x6f, 0x50, 0x71, 0x7f, 0x60, 0x70};

/* ReadHuffmanCode / ReadHuffmanCodeLengths, vp8l_dec.c:257-358 */
static int read_huff(LBits* b, int alphabet, Huff* h) {
  int* lens = (int*)calloc((size_t)alphabet, sizeof(int));
  if (!lens) return 0;
  int ok = 0;
  if (lb_read(b, 1)) {   /* simple code: 1 or 2 symbols */
    const int nsym = (int)lb_read(b, 1) + 1;
    const int first8 = (int)lb_read(b, 1);
    int s = (int)lb_read(b, first8 ? 8 : 1);
    if (s < alphabet) lens[s] = 1;
    if (nsym == 2) {
      s = (int)lb_read(b, 8);
      if (s < alphabet) lens[s] = 1;
    }
    ok = 1;
  } else {
    int cl[19] = {0};
    const int ncodes = (int)lb_read(b, 4) + 4;
    for (int i = 0; i < ncodes; ++i) cl[kCodeLengthOrder[i]] = (int)lb_read(b, 3);
    Huff lh;
    if (huff_build(&lh, cl, 19)) {
      int max_symbol = alphabet;
      ok = 1;
      if (lb_read(b, 1)) {
        const int nbits = 2 + 2 * (int)lb_read(b, 3);
        max_symbol = 2 + (int)lb_read(b, nbits);
        if (max_symbol > alphabet) ok = 0;
      }
      int sym = 0, prev = 8;
      while (ok && sym < alphabet) {
        if (max_symbol-- == 0) break;
        const int c = huff_read(&lh, b);
        if (c < 16) {
          lens[sym++] = c;
          if (c) prev = c;
        } else {
          static const int kExtra[3] = {2, 3, 7}, kOff[3] = {3, 3, 11};
          const int rep = (int)lb_read(b, kExtra[c - 16]) + kOff[c - 16];
          if (sym + rep > alphabet) { ok = 0; break; }
          const int v = c == 16 ? prev : 0;
          for (int k = 0; k < rep; ++k) lens[sym++] = v;
        }
      }
    }
    free(lh.sorted);
  }
  ok = ok && !b->eos && huff_build(h, lens, alphabet);
  free(lens);
  return ok;
}

typedef struct { Huff h[5]; } HGroup;

static inline int subsample(int size, int bits) { return (size + (1 << bits) - 1) >> bits; }

static uint32_t* decode_image_stream(LBits* b, int xs, int ys, int level0, int* out_xs);

static int copy_distance(int sym, LBits* b) {   /* GetCopyDistance, vp8l_dec.c:159-168 */
  if (sym < 4) return sym + 1;
  const int eb = (sym - 2) >> 1;
  const int off = (2 + (sym & 1)) << eb;
  return off + (int)lb_read(b, eb) + 1;
}

/* DecodeImageData, vp8l_dec.c:1138-1275 (colour cache filled in pixel order) */
/* analysis only (odec_vp8l_stats): the main image's coding, filled by the
 * level-0 decode of the calling thread */
static _Thread_local long long* t_lstats;      /* requested */
static _Thread_local long long* t_lstats_px;   /* armed for the main image's pixels */
enum { LS_HDR_BITS, LS_NGROUPS, LS_HBITS, LS_CACHE_BITS, LS_NLIT, LS_NCOPY, LS_NCACHE,
       LS_BLIT, LS_BCOPY, LS_BCACHE, LS_COPY_PX, LS_N };

static int decode_pixels(LBits* b, uint32_t* data, int xs, int ys, int cache_bits,
                         const HGroup* groups, const uint32_t* himg, int hbits) {
  long long* st = t_lstats_px;
  t_lstats_px = NULL;
  const int hxs = hbits ? subsample(xs, hbits) : 0;
  uint32_t* cache = cache_bits ? (uint32_t*)calloc((size_t)1 << cache_bits, 4) : NULL;
  if (cache_bits && !cache) return 0;
  const size_t total = (size_t)xs * ys;
  size_t pos = 0, cached = 0;
  int ok = 1;
#define CACHE_UPTO(end)                                                         \
  while (cache && cached < (end)) {                                             \
    const uint32_t px_ = data[cached++];                                        \
    cache[(0x1e35a7bdu * px_) >> (32 - cache_bits)] = px_;                      \
  }
  while (pos < total && ok) {
    const int x = (int)(pos % xs), y = (int)(pos / xs);
    const HGroup* g = groups + (hbits ? himg[(y >> hbits) * hxs + (x >> hbits)] : 0);
    const size_t p0 = b->pos, pos0 = pos;
    const int code = huff_read(&g->h[0], b);
    if (code < 256) {
      const int r = huff_read(&g->h[1], b), bl = huff_read(&g->h[2], b);
      const int a = huff_read(&g->h[3], b);
      data[pos++] = ((uint32_t)a << 24) | ((uint32_t)r << 16) | ((uint32_t)code << 8) | (uint32_t)bl;
    } else if (code < 256 + 24) {
      const int len = copy_distance(code - 256, b);
      const int dsym = huff_read(&g->h[4], b);
      const int dcode = copy_distance(dsym, b);
      int dist;
      if (dcode > 120) {
        dist = dcode - 120;
      } else {   /* PlaneCodeToDistance, vp8l_dec.c:176-186 */
        const int dc = kCodeToPlane[dcode - 1];
        dist = (dc >> 4) * xs + (8 - (dc & 0xf));
        if (dist < 1) dist = 1;
      }
      if ((size_t)dist > pos || total - pos < (size_t)len) { ok = 0; break; }
      for (int k = 0; k < len; ++k, ++pos) data[pos] = data[pos - dist];
    } else {
      const int key = code - (256 + 24);
      if (!cache || key >= (1 << cache_bits)) { ok = 0; break; }
      CACHE_UPTO(pos);
      data[pos++] = cache[key];
    }
    CACHE_UPTO(pos);
    if (b->eos) ok = 0;
    if (st) {
      const int k = code < 256 ? 0 : code < 256 + 24 ? 1 : 2;
      st[LS_NLIT + k] += 1;
      st[LS_BLIT + k] += (long long)(b->pos - p0);
      if (k == 1) st[LS_COPY_PX] += (long long)(pos - pos0);
    }
  }
#undef CACHE_UPTO
  free(cache);
  return ok;
}

typedef struct {
  int type, bits, xs, ys;
  uint32_t* data;
} LTransform;

static inline uint32_t avg2(uint32_t a, uint32_t b) {
  return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b);
}
static inline uint32_t clip255(uint32_t a) { return a < 256 ? a : ~a >> 24; }
static inline int sub3(int a, int b, int c) { return iabs(b - c) - iabs(a - c); }
static uint32_t select_px(uint32_t a, uint32_t b, uint32_t c) {   /* Select, lossless.c:98-105 */
  int d = 0;
  for (int s = 0; s < 32; s += 8) d += sub3((a >> s) & 0xff, (b >> s) & 0xff, (c >> s) & 0xff);
  return d <= 0 ? a : b;
}
static uint32_t add_sub_full(uint32_t c0, uint32_t c1, uint32_t c2) {
  uint32_t out = 0;
  for (int s = 0; s < 32; s += 8)
    out |= clip255((uint32_t)((int)((c0 >> s) & 0xff) + (int)((c1 >> s) & 0xff) -
                              (int)((c2 >> s) & 0xff)))
           << s;
  return out;
}
static uint32_t add_sub_half(uint32_t c0, uint32_t c1, uint32_t c2) {
  const uint32_t ave = avg2(c0, c1);
  uint32_t out = 0;
  for (int s = 0; s < 32; s += 8) {
    const int a = (int)((ave >> s) & 0xff), b = (int)((c2 >> s) & 0xff);
    out |= clip255((uint32_t)(a + (a - b) / 2)) << s;
  }
  return out;
}
static uint32_t predict_px(int mode, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
  switch (mode) {   /* VP8LPredictor0..13_C, lossless.c:110-182 */
    case 1: return L;
    case 2: return T;
    case 3: return TR;
    case 4: return TL;
    case 5: return avg2(avg2(L, TR), T);
    case 6: return avg2(L, TL);
    case 7: return avg2(L, T);
    case 8: return avg2(TL, T);
    case 9: return avg2(T, TR);
    case 10: return avg2(avg2(L, TL), avg2(T, TR));
    case 11: return select_px(T, L, TL);
    case 12: return add_sub_full(L, T, TL);
    case 13: return add_sub_half(L, T, TL);
    default: return 0xff000000u;   /* 0, and the unused 14/15 */
  }
}
static inline uint32_t add_px(uint32_t a, uint32_t b) {   /* VP8LAddPixels */
  return (((a & 0xff00ff00u) + (b & 0xff00ff00u)) & 0xff00ff00u) |
         (((a & 0x00ff00ffu) + (b & 0x00ff00ffu)) & 0x00ff00ffu);
}

/* VP8LInverseTransform (lossless.c) over the whole image; in has width
 * t->xs (colour indexing: packed width) */
static uint32_t* inverse_transform(const LTransform* t, uint32_t* in, int in_xs) {
  const int w = t->xs, h = t->ys;
  if (t->type == 0) {   /* predictor, lossless.c:215-257 */
    uint32_t* out = in;
    const int tw = subsample(w, t->bits);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        uint32_t pred;
        uint32_t* o = out + (size_t)y * w + x;
        if (y == 0) pred = x == 0 ? 0xff000000u : o[-1];
        else if (x == 0) pred = o[-w];
        else {
          const int mode = (t->data[(y >> t->bits) * tw + (x >> t->bits)] >> 8) & 0xf;
          /* top-right of the last column = the first pixel of this row */
          pred = predict_px(mode, o[-1], o[-w], o[-w - 1], o[-w + 1]);
        }
        *o = add_px(*o, pred);
      }
    return out;
  }
  if (t->type == 1) {   /* cross colour, VP8LTransformColorInverse_C */
    const int tw = subsample(w, t->bits);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const uint32_t m = t->data[(y >> t->bits) * tw + (x >> t->bits)];
        const int8_t g2r = (int8_t)(m & 0xff), g2b = (int8_t)((m >> 8) & 0xff);
        const int8_t r2b = (int8_t)((m >> 16) & 0xff);
        uint32_t* p = in + (size_t)y * w + x;
        const uint32_t argb = *p;
        const int8_t g = (int8_t)(argb >> 8);
        int r = (argb >> 16) & 0xff, bl = argb & 0xff;
        r = (r + ((g2r * g) >> 5)) & 0xff;
        bl += (g2b * g) >> 5;
        bl += (r2b * (int8_t)r) >> 5;
        bl &= 0xff;
        *p = (argb & 0xff00ff00u) | ((uint32_t)r << 16) | (uint32_t)bl;
      }
    return in;
  }
  if (t->type == 2) {   /* add green */
    for (size_t i = 0; i < (size_t)w * h; ++i) {
      const uint32_t argb = in[i], g = (argb >> 8) & 0xff;
      in[i] = (argb & 0xff00ff00u) | ((((argb >> 16) + g) & 0xff) << 16) | ((argb + g) & 0xff);
    }
    return in;
  }
  /* colour indexing, VP8LColorIndexInverseTransform: t->data is the
   * expanded colour map (1 << (8 >> bits) entries) */
  uint32_t* out = (uint32_t*)malloc((size_t)w * h * 4);
  if (!out) { free(in); return NULL; }
  const int bpp = 8 >> t->bits, ppb = 1 << t->bits, cmask = ppb - 1, bmask = (1 << bpp) - 1;
  for (int y = 0; y < h; ++y) {
    const uint32_t* src = in + (size_t)y * in_xs;
    uint32_t packed = 0;
    for (int x = 0; x < w; ++x) {
      if ((x & cmask) == 0) packed = (*src++ >> 8) & 0xff;
      out[(size_t)y * w + x] = t->data[packed & bmask];
      packed >>= bpp;
    }
  }
  free(in);
  return out;
}

/* DecodeImageStream, vp8l_dec.c:1455-1530 (+ ReadTransform :1330-1384,
 * ReadHuffmanCodes :367-452) */
static uint32_t* decode_image_stream(LBits* b, int xs, int ys, int level0, int* out_xs) {
  LTransform tr[4];
  int ntr = 0, seen = 0, txs = xs;
  uint32_t* data = NULL;
  HGroup* groups = NULL;
  uint32_t* himg = NULL;
  int ngroups = 1, hbits = 0, ok = 1;
  memset(tr, 0, sizeof(tr));
  if (level0) {
    while (ok && lb_read(b, 1)) {
      LTransform* t = &tr[ntr];
      t->type = (int)lb_read(b, 2);
      if (seen & (1 << t->type)) { ok = 0; break; }
      seen |= 1 << t->type;
      t->xs = txs;
      t->ys = ys;
      ++ntr;
      if (t->type == 0 || t->type == 1) {
        t->bits = (int)lb_read(b, 3) + 2;
        t->data = decode_image_stream(b, subsample(txs, t->bits), subsample(ys, t->bits), 0, NULL);
        ok = t->data != NULL;
      } else if (t->type == 3) {
        const int ncol = (int)lb_read(b, 8) + 1;
        t->bits = ncol > 16 ? 0 : ncol > 4 ? 1 : ncol > 2 ? 2 : 3;
        txs = subsample(t->xs, t->bits);
        uint32_t* pal = decode_image_stream(b, ncol, 1, 0, NULL);
        ok = pal != NULL;
        if (ok) {   /* ExpandColorMap, vp8l_dec.c:1305-1328 */
          const int fin = 1 << (8 >> t->bits);
          t->data = (uint32_t*)calloc((size_t)fin, 4);
          ok = t->data != NULL;
          if (ok) {
            t->data[0] = pal[0];
            for (int i = 1; i < ncol && i < fin; ++i) t->data[i] = add_px(pal[i], t->data[i - 1]);
          }
          free(pal);
        }
      }
    }
  }
  int cache_bits = 0;
  if (ok && lb_read(b, 1)) {
    cache_bits = (int)lb_read(b, 4);
    ok = cache_bits >= 1 && cache_bits <= 11;
  }
  if (ok && level0 && lb_read(b, 1)) {   /* meta Huffman codes */
    hbits = (int)lb_read(b, 3) + 2;
    const int hx = subsample(txs, hbits), hy = subsample(ys, hbits);
    himg = decode_image_stream(b, hx, hy, 0, NULL);
    ok = himg != NULL;
    if (ok) {
      for (int i = 0; i < hx * hy; ++i) {
        himg[i] = (himg[i] >> 8) & 0xffff;
        if ((int)himg[i] >= ngroups) ngroups = (int)himg[i] + 1;
      }
    }
  }
  if (ok) {
    groups = (HGroup*)calloc((size_t)ngroups, sizeof(HGroup));
    ok = groups != NULL;
    for (int g = 0; ok && g < ngroups; ++g)
      for (int j = 0; ok && j < 5; ++j)
        ok = read_huff(b, kAlphabet[j] + (j == 0 && cache_bits ? 1 << cache_bits : 0),
                       &groups[g].h[j]);
  }
  if (ok) {
    data = (uint32_t*)malloc((size_t)txs * ys * 4 + 4);
    if (level0 && t_lstats) {
      t_lstats[LS_HDR_BITS] = (long long)b->pos;
      t_lstats[LS_NGROUPS] = ngroups;
      t_lstats[LS_HBITS] = hbits;
      t_lstats[LS_CACHE_BITS] = cache_bits;
      t_lstats_px = t_lstats;
    }
    ok = data && decode_pixels(b, data, txs, ys, cache_bits, groups, himg, hbits);
  }
  if (groups)
    for (int g = 0; g < ngroups; ++g)
      for (int j = 0; j < 5; ++j) free(groups[g].h[j].sorted);
  free(groups);
  free(himg);
  if (ok) {
    int cur_xs = txs;
    for (int i = ntr - 1; i >= 0 && data; --i) {
      data = inverse_transform(&tr[i], data, cur_xs);
      cur_xs = tr[i].xs;
    }
    ok = data != NULL;
    if (out_xs) *out_xs = cur_xs;
  }
  for (int i = 0; i < ntr; ++i) free(tr[i].data);
  if (!ok) {
    free(data);
    return NULL;
  }
  return data;
}

/* VP8L chunk payload -> ARGB (w x h) */
static uint32_t* vp8l_decode(const uint8_t* p, size_t n, int* w, int* h) {
  LBits b = {p, n, 0, 0};
  if (n < 5 || lb_read(&b, 8) != 0x2f) return NULL;
  *w = (int)lb_read(&b, 14) + 1;
  *h = (int)lb_read(&b, 14) + 1;
  lb_read(&b, 1);   /* alpha hint */
  if (lb_read(&b, 3) != 0) return NULL;
  return decode_image_stream(&b, *w, *h, 1, NULL);
}

/* ALPH chunk -> alpha plane (alpha_dec.c:41-120, filters.c:192-234) */
static int alpha_decode(const uint8_t* p, size_t n, int w, int h, uint8_t* a) {
  if (n < 1) return 0;
  const int method = p[0] & 3, filter = (p[0] >> 2) & 3;
  if ((p[0] >> 6) & 3) return 0;
  if (method == 0) {
    if (n - 1 < (size_t)w * h) return 0;
    memcpy(a, p + 1, (size_t)w * h);
  } else if (method == 1) {
    LBits b = {p + 1, n - 1, 0, 0};
    uint32_t* argb = decode_image_stream(&b, w, h, 1, NULL);
    if (!argb) return 0;
    for (size_t i = 0; i < (size_t)w * h; ++i) a[i] = (uint8_t)(argb[i] >> 8);
    free(argb);
  } else {
    return 0;
  }
  for (int y = 0; y < h; ++y) {   /* WebPUnfilters[filter](prev, row, row) */
    uint8_t* row = a + (size_t)y * w;
    const uint8_t* prev = y ? row - w : NULL;
    if (filter == 0) continue;
    if (prev == NULL || filter == 1) {
      uint8_t pred = prev ? prev[0] : 0;
      for (int x = 0; x < w; ++x) { row[x] = (uint8_t)(pred + row[x]); pred = row[x]; }
    } else if (filter == 2) {
      for (int x = 0; x < w; ++x) row[x] = (uint8_t)(prev[x] + row[x]);
    } else {
      int top, tl = prev[0], left = prev[0];
      for (int x = 0; x < w; ++x) {
        top = prev[x];
        int g = left + top - tl;
        g = g < 0 ? 0 : g > 255 ? 255 : g;
        left = (uint8_t)(row[x] + g);
        tl = top;
        row[x] = (uint8_t)left;
      }
    }
  }
  return 1;
}

/* ======================================================================
 * YUV -> RGBA, fancy upsampling (upsampling.c:37-97, io_dec.c:57-111, yuv.h) */
static inline int clip8_6(int v) { return (v & ~16383) == 0 ? v >> 6 : v < 0 ? 0 : 255; }
static inline int mult_hi(int v, int c) { return (v * c) >> 8; }
static void yuv_px(int y, int u, int v, uint8_t* d) {
  d[0] = (uint8_t)clip8_6(mult_hi(y, 19077) + mult_hi(v, 26149) - 14234);
  d[1] = (uint8_t)clip8_6(mult_hi(y, 19077) - mult_hi(u, 6419) - mult_hi(v, 13320) + 8708);
  d[2] = (uint8_t)clip8_6(mult_hi(y, 19077) + mult_hi(u, 33050) - 17685);
}
static void upsample_pair(const uint8_t* ty, const uint8_t* by, const uint8_t* tu,
                          const uint8_t* tv, const uint8_t* cu, const uint8_t* cv,
                          uint8_t* td, uint8_t* bd, int len) {
#define LOAD_UV(u, v) ((uint32_t)(u) | ((uint32_t)(v) << 16))
  const int last = (len - 1) >> 1;
  uint32_t tl = LOAD_UV(tu[0], tv[0]), l = LOAD_UV(cu[0], cv[0]);
  {
    const uint32_t uv0 = (3 * tl + l + 0x00020002u) >> 2;
    yuv_px(ty[0], uv0 & 0xff, uv0 >> 16, td);
  }
  if (by) {
    const uint32_t uv0 = (3 * l + tl + 0x00020002u) >> 2;
    yuv_px(by[0], uv0 & 0xff, uv0 >> 16, bd);
  }
  for (int x = 1; x <= last; ++x) {
    const uint32_t t = LOAD_UV(tu[x], tv[x]), uv = LOAD_UV(cu[x], cv[x]);
    const uint32_t avg = tl + t + l + uv + 0x00080008u;
    const uint32_t d12 = (avg + 2 * (t + l)) >> 3, d03 = (avg + 2 * (tl + uv)) >> 3;
    {
      const uint32_t uv0 = (d12 + tl) >> 1, uv1 = (d03 + t) >> 1;
      yuv_px(ty[2 * x - 1], uv0 & 0xff, uv0 >> 16, td + (2 * x - 1) * 4);
      yuv_px(ty[2 * x], uv1 & 0xff, uv1 >> 16, td + 2 * x * 4);
    }
    if (by) {
      const uint32_t uv0 = (d03 + l) >> 1, uv1 = (d12 + uv) >> 1;
      yuv_px(by[2 * x - 1], uv0 & 0xff, uv0 >> 16, bd + (2 * x - 1) * 4);
      yuv_px(by[2 * x], uv1 & 0xff, uv1 >> 16, bd + 2 * x * 4);
    }
    tl = t;
    l = uv;
  }
  if (!(len & 1)) {
    {
      const uint32_t uv0 = (3 * tl + l + 0x00020002u) >> 2;
      yuv_px(ty[len - 1], uv0 & 0xff, uv0 >> 16, td + (len - 1) * 4);
    }
    if (by) {
      const uint32_t uv0 = (3 * l + tl + 0x00020002u) >> 2;
      yuv_px(by[len - 1], uv0 & 0xff, uv0 >> 16, bd + (len - 1) * 4);
    }
  }
#undef LOAD_UV
}

static void planes_to_rgba(const Planes* P, int w, int h, uint8_t* out) {
  const uint8_t *y = P->y, *u = P->u, *v = P->v;
  const int ys = P->yw, us = P->uvw, os = 4 * w;
  upsample_pair(y, NULL, u, v, u, v, out, NULL, w);
  int r = 1;
  for (; r + 1 < h; r += 2) {
    const int ur = (r - 1) >> 1;
    upsample_pair(y + (size_t)r * ys, y + (size_t)(r + 1) * ys, u + (size_t)ur * us,
                  v + (size_t)ur * us, u + (size_t)(ur + 1) * us, v + (size_t)(ur + 1) * us,
                  out + (size_t)r * os, out + (size_t)(r + 1) * os, w);
  }
  if (h > 1 && !(h & 1)) {
    const int ur = (h - 2) >> 1;
    upsample_pair(y + (size_t)(h - 1) * ys, NULL, u + (size_t)ur * us, v + (size_t)ur * us,
                  u + (size_t)ur * us, v + (size_t)ur * us, out + (size_t)(h - 1) * os, NULL, w);
  }
  for (size_t i = 0; i < (size_t)w * h; ++i) out[4 * i + 3] = 0xff;
}

/* ======================================================================
 * container (webp_dec.c ParseHeadersInternal: RIFF, VP8X, ALPH, VP8/VP8L) */
typedef struct {
  const uint8_t *vp8, *vp8l, *alph;
  size_t vp8_n, vp8l_n, alph_n;
  int w, h;
} Chunks;

static uint32_t le32(const uint8_t* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24); }

static int parse_container(const uint8_t* d, size_t n, Chunks* c) {
  memset(c, 0, sizeof(*c));
  if (n < 12 || memcmp(d, "RIFF", 4) || memcmp(d + 8, "WEBP", 4)) return 0;
  size_t riff = le32(d + 4) + 8;
  if (riff > n) riff = n;
  size_t pos = 12;
  while (pos + 8 <= riff) {
    const uint8_t* tag = d + pos;
    const size_t len = le32(d + pos + 4);
    const uint8_t* pay = d + pos + 8;
    if (pos + 8 + len > riff) return 0;
    if (!memcmp(tag, "VP8 ", 4)) { c->vp8 = pay; c->vp8_n = len; }
    else if (!memcmp(tag, "VP8L", 4)) { c->vp8l = pay; c->vp8l_n = len; }
    else if (!memcmp(tag, "ALPH", 4)) { c->alph = pay; c->alph_n = len; }
    pos += 8 + len + (len & 1);
  }
  if (c->vp8) {
    if (c->vp8_n < 10) return 0;
    c->w = ((c->vp8[7] << 8) | c->vp8[6]) & 0x3fff;
    c->h = ((c->vp8[9] << 8) | c->vp8[8]) & 0x3fff;
    return 1;
  }
  if (c->vp8l) {
    if (c->vp8l_n < 5 || c->vp8l[0] != 0x2f) return 0;
    const uint32_t b = le32(c->vp8l + 1);
    c->w = (int)(b & 0x3fff) + 1;
    c->h = (int)((b >> 14) & 0x3fff) + 1;
    return 1;
  }
  return 0;
}

/* analysis only: how a VP8L file's main image is coded -- out[LS_N]: header
 * bits (transforms, cache, meta image, codes), code groups, meta bits, cache
 * bits, literal / copy / cache-hit counts and their bits, pixels copied */
int odec_vp8l_stats(const uint8_t* data, size_t size, long long* out) {
  for (int i = 0; i < LS_N; ++i) out[i] = 0;
  if (size < 20 || memcmp(data + 12, "VP8L", 4)) return 0;
  int w = 0, h = 0;
  t_lstats = out;
  uint32_t* argb = vp8l_decode(data + 20, size - 20, &w, &h);
  t_lstats = NULL;
  free(argb);
  return argb != NULL;
}

int odec_info(const uint8_t* data, size_t size, int* w, int* h, int* has_alpha, int* lossless) {
  Chunks c;
  if (!parse_container(data, size, &c)) return 0;
  *w = c.w;
  *h = c.h;
  *lossless = c.vp8 == NULL;
  *has_alpha = c.vp8 ? c.alph != NULL : (c.vp8l_n > 4 && ((c.vp8l[4] >> 4) & 1));
  return 1;
}

int odec_decode_yuv(const uint8_t* data, size_t size, uint8_t* y, uint8_t* u, uint8_t* v) {
  Chunks c;
  if (!parse_container(data, size, &c) || !c.vp8) return 0;
  VP8Frame* F = (VP8Frame*)malloc(sizeof(VP8Frame));
  Planes P;
  memset(&P, 0, sizeof(P));
  const int ok = F && vp8_decode(c.vp8, c.vp8_n, F, &P) && F->w == c.w && F->h == c.h;
  if (ok) {
    const int uw = (c.w + 1) >> 1, uh = (c.h + 1) >> 1;
    for (int j = 0; j < c.h; ++j) memcpy(y + (size_t)j * c.w, P.y + (size_t)j * P.yw, c.w);
    for (int j = 0; j < uh; ++j) {
      memcpy(u + (size_t)j * uw, P.u + (size_t)j * P.uvw, uw);
      memcpy(v + (size_t)j * uw, P.v + (size_t)j * P.uvw, uw);
    }
  }
  free(P.y); free(P.u); free(P.v);
  free(F);
  return ok;
}

int odec_decode_rgba(const uint8_t* data, size_t size, uint8_t* out) {
  Chunks c;
  if (!parse_container(data, size, &c)) return 0;
  const size_t npx = (size_t)c.w * c.h;
  if (c.vp8) {
    VP8Frame* F = (VP8Frame*)malloc(sizeof(VP8Frame));
    Planes P;
    memset(&P, 0, sizeof(P));
    int ok = F && vp8_decode(c.vp8, c.vp8_n, F, &P) && F->w == c.w && F->h == c.h;
    if (ok) planes_to_rgba(&P, c.w, c.h, out);
    free(P.y); free(P.u); free(P.v);
    free(F);
    if (ok && c.alph) {
      uint8_t* a = (uint8_t*)malloc(npx);
      ok = a && alpha_decode(c.alph, c.alph_n, c.w, c.h, a);
      if (ok)
        for (size_t i = 0; i < npx; ++i) out[4 * i + 3] = a[i];
      free(a);
    }
    return ok;
  }
  int w, h;
  uint32_t* argb = vp8l_decode(c.vp8l, c.vp8l_n, &w, &h);
  if (!argb) return 0;
  const int ok = w == c.w && h == c.h;
  if (ok)
    for (size_t i = 0; i < npx; ++i) {
      const uint32_t p = argb[i];
      out[4 * i] = (uint8_t)(p >> 16);
      out[4 * i + 1] = (uint8_t)(p >> 8);
      out[4 * i + 2] = (uint8_t)p;
      out[4 * i + 3] = (uint8_t)(p >> 24);
    }
  free(argb);
  return ok;
}
