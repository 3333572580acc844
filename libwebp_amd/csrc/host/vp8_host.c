/* Host C: per-frame segment setup and the boolean-coder / bitstream tail of
 * the VP8 lossy encoder. Reference behaviour cited per function. */
#include "vp8_host.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define VP8T_DECL static const
#include "../vp8_tables.h"

#define QFIX 17

static inline int clampi(int v, int lo, int hi) { return v < lo ? lo : v > hi ? hi : v; }
static inline int iabs(int v) { return v < 0 ? -v : v; }
static inline float clampf(float v, float lo, float hi) {   /* frame_enc.c:34-36 */
  return (v < lo) ? lo : (v > hi) ? hi : v;
}
static inline int bit_cost(int bit, int p) {   /* cost_enc.h:59-61 */
  return bit ? kVP8EntropyCost[255 - p] : kVP8EntropyCost[p];
}

static uint32_t g_sg2l[1026], g_sl2g[514];
static pthread_once_t g_sharp_once = PTHREAD_ONCE_INIT;
static void sharp_tables_init(void) {
  const double a = 0.09929682680944, lin_thresh = 0.018053968510807;
  const double scale = 65536.;
  for (int i = 0; i <= 1024; ++i) {   /* gamma -> linear */
    const double g = (1. / 1024) * i;
    const double x = g <= lin_thresh * 4.5 ? g / 4.5 : pow((1. / (1. + a)) * (g + a), 1. / 0.45);
    g_sg2l[i] = (uint32_t)(x * scale + .5);
  }
  g_sg2l[1025] = g_sg2l[1024];
  for (int i = 0; i <= 512; ++i) {    /* linear -> gamma */
    const double l = (1. / 512) * i;
    const double x = l <= lin_thresh ? 4.5 * l : (1. + a) * pow(l, 1. / (1. / 0.45)) - a;
    g_sl2g[i] = (uint32_t)(scale * x + .5);
  }
  g_sl2g[513] = g_sl2g[512];
}
void vp8h_sharp_tables(const uint32_t** g2l, const uint32_t** l2g) {
  pthread_once(&g_sharp_once, sharp_tables_init);
  *g2l = g_sg2l;
  *l2g = g_sl2g;
}
int vp8h_use_sharp(const WebPConfig* cfg, int w, int h) {
  return (cfg->use_sharp_yuv || (cfg->preprocessing & 4)) && w >= 4 && h >= 4;
}

int vp8h_frame_init(vp8h_frame* fr, const WebPConfig* cfg, int w, int h) {
  memset(fr, 0, sizeof(*fr));
  if (cfg->method < 0 || cfg->method > 6) return 0;
  /* token partitions: VP8EncLoop writes MB row y into partition
   * y & (2^partitions - 1); the token loop (methods 3-6 without low_memory)
   * keeps one (webp_enc.c:115-122, 209) */
  fr->num_parts = (cfg->method < 3 || cfg->low_memory) ? 1 << cfg->partitions : 1;
  fr->w = w; fr->h = h;
  fr->mbw = (w + 15) >> 4; fr->mbh = (h + 15) >> 4;
  fr->method = cfg->method;
  fr->rd_opt = cfg->method >= 6 ? 3 : cfg->method >= 5 ? 2 : cfg->method >= 3 ? 1 : 0;
  {
    const int lim = 100 - cfg->partition_limit;
    fr->max_i4_header_bits = 256 * 16 * 16 * (lim * lim) / (100 * 100);
  }
  {
    const int use_filter = cfg->filter_strength > 0 || cfg->autofilter > 0;
    fr->profile = use_filter ? ((cfg->filter_type == 1) ? 0 : 1) : 2;
  }
  fr->quality = cfg->quality;
  fr->sns_strength = cfg->sns_strength;
  fr->filter_strength = cfg->filter_strength;
  fr->filter_sharpness = cfg->filter_sharpness;
  fr->filter_type = cfg->filter_type;
  fr->preprocessing = cfg->preprocessing;
  fr->emulate_jpeg_size = cfg->emulate_jpeg_size;
  fr->cfg_segments = cfg->segments;
  fr->num_segments = cfg->segments;
  fr->update_map = fr->num_segments > 1;
  memset(fr->seg_probas, 255, 3);
  fr->f_simple = 1;     /* ResetFilterHeader, webp_enc.c:47-53 */
  fr->f_level = 0;
  fr->f_sharpness = 0;
  /* InitPassStats (frame_enc.c:47-62), enc->do_search_ (webp_enc.c:114) */
  fr->pass_left = fr->cfg_pass = cfg->pass;
  fr->autofilter = cfg->autofilter;
  fr->do_search = cfg->target_size > 0 || cfg->target_PSNR > 0;
  fr->do_size_search = cfg->target_size != 0;
  fr->ps_is_first = 1;
  fr->ps_dq = 10.f;
  fr->ps_qmin = 1.f * cfg->qmin;
  fr->ps_qmax = 1.f * cfg->qmax;
  fr->ps_q = fr->ps_last_q = clampf(cfg->quality, fr->ps_qmin, fr->ps_qmax);
  fr->ps_target = fr->do_size_search ? (double)(uint64_t)cfg->target_size
                : (cfg->target_PSNR > 0.) ? cfg->target_PSNR : 40.;
  fr->ps_value = fr->ps_last_value = 0.;
  return 1;
}

/* ------------------------------------------------------------------------ */
/* multi-pass convergence: frame_enc.c:26-80, 146-180, 554-556, 808-880 */

#define DQ_LIMIT 0.4
#define HEADER_SIZE_ESTIMATE (12 + 8 + 10)   /* RIFF + chunk + VP8 frame headers */

int vp8h_pass_start(vp8h_frame* fr) {
  if (fr->pass_left-- <= 0) return 0;
  /* StatLoop (RD_OPT_NONE, no search): no q changes, dq stays 10 */
  fr->is_last_pass = (fabs(fr->ps_dq) <= DQ_LIMIT) || (fr->pass_left == 0) ||
                     (fr->max_i4_header_bits == 0);
  return 1;
}

static void compute_next_q(vp8h_frame* s) {   /* ComputeNextQ, :60-80 */
  float dq;
  if (s->ps_is_first) {
    dq = (s->ps_value > s->ps_target) ? -s->ps_dq : s->ps_dq;
    s->ps_is_first = 0;
  } else if (s->ps_value != s->ps_last_value) {
    const double slope = (s->ps_target - s->ps_value) / (s->ps_last_value - s->ps_value);
    dq = (float)(slope * (s->ps_last_q - s->ps_q));
  } else {
    dq = 0.;
  }
  s->ps_dq = clampf(dq, -30.f, 30.f);
  s->ps_last_q = s->ps_q;
  s->ps_last_value = s->ps_value;
  s->ps_q = clampf(s->ps_q + s->ps_dq, s->ps_qmin, s->ps_qmax);
}

/* StatLoop's pass control (frame_enc.c:640-664): like the token loop's, but a
 * search step that lands within DQ_LIMIT ends the loop at once (the new q is
 * never run: the final pass keeps the last pass's segment parameters) */
int vp8h_statloop_finish(vp8h_frame* fr, uint64_t size_p0) {
  if (size_p0 == 0) return 0;   /* :646 */
  if (fr->max_i4_header_bits > 0 && size_p0 > VP8H_P0_LIMIT) {
    ++fr->pass_left;
    fr->max_i4_header_bits >>= 1;
    return 1;
  }
  if (fr->is_last_pass) return 0;
  if (fr->do_search) {
    compute_next_q(fr);
    if (fabs(fr->ps_dq) <= DQ_LIMIT) return 0;
  }
  return fr->pass_left > 0;
}

/* FinalizeSkipProba (frame_enc.c:111-127): the skip probability from the
 * pass's skip count, whether it pays, and its header cost (1/256 bit) */
int vp8h_finalize_skip(int nb_skip, int nmb, int* skip_proba, int* use_skip) {
  const int p = nmb ? (int)((uint64_t)(nmb - nb_skip) * 255 / nmb) : 255;   /* CalcSkipProba */
  *skip_proba = p;
  *use_skip = p < 250;
  int size = 256;
  if (*use_skip) size += nb_skip * bit_cost(1, p) + (nmb - nb_skip) * bit_cost(0, p) + 8 * 256;
  return size;
}

int vp8h_pass_finish(vp8h_frame* fr, uint64_t size_p0) {
  if (fr->rd_opt == 0 && size_p0 == 0) return 0;   /* StatLoop gives up (frame_enc.c:645) */
  if (fr->max_i4_header_bits > 0 && size_p0 > VP8H_P0_LIMIT) {
    ++fr->pass_left;
    fr->max_i4_header_bits >>= 1;   /* strengthen the header bit limit and start over */
    return 1;
  }
  if (fr->is_last_pass) return 0;
  if (fr->do_search) compute_next_q(fr);
  return fr->pass_left > 0;
}

void vp8h_default_probas(uint8_t* coeffs) {   /* VP8DefaultCoeffProbas, tree_enc.c */
  memcpy(coeffs, &kVP8CoeffProba0[0][0][0][0], VP8G_NUM_SLOTS);
}

int vp8h_finalize_probas(const uint32_t* stats, uint8_t* coeffs, int* dirty) {
  const uint8_t* p0 = &kVP8CoeffProba0[0][0][0][0];
  const uint8_t* pu = &kVP8CoeffUpdateProba[0][0][0][0];
  int changed = 0, size = 0;
  for (int s = 0; s < VP8G_NUM_SLOTS; ++s) {
    const int nb = stats[s] & 0xffff, total = (stats[s] >> 16) & 0xffff;
    const int old_p = p0[s], upd = pu[s];
    const int new_p = nb ? (255 - nb * 255 / total) : 255;
    const int old_cost = nb * bit_cost(1, old_p) + (total - nb) * bit_cost(0, old_p) + bit_cost(0, upd);
    const int new_cost = nb * bit_cost(1, new_p) + (total - nb) * bit_cost(0, new_p) +
                         bit_cost(1, upd) + 8 * 256;
    const int use_new = old_cost > new_cost;
    size += bit_cost(use_new, upd);
    if (use_new) {
      coeffs[s] = (uint8_t)new_p;
      changed |= new_p != old_p;
      size += 8 * 256;
    } else {
      coeffs[s] = (uint8_t)old_p;
    }
  }
  *dirty = changed;
  return size;
}

double vp8h_pass_size_value(uint64_t finalize_cost, uint64_t token_bits, uint64_t size_p0) {
  uint64_t size = finalize_cost + token_bits;
  size = (size + size_p0 + 1024) >> 11;
  return (double)(size + HEADER_SIZE_ESTIMATE);
}

/* Sum of the per-MB header-bit estimates info.H (OneStatPass,
 * frame_enc.c:588-596) of MBs 0..nb-1 from their coded modes: an intra-16
 * MB's VP8FixedCostsI16[mode], an intra-4 MB's 211 plus each sub-block's
 * VP8FixedCostsI4[top][left][mode] (contexts from the neighbour MBs' modes, 0
 * outside the frame; an intra-16 MB lends its mode to all 16 contexts), plus
 * VP8FixedCostsUV[uv mode] (quant_enc.c:1002-1217). */
uint64_t vp8h_mode_header_bits(const uint8_t* mbinfo, int mbw, int nb) {
  uint64_t sum = 0;
  for (int mb = 0; mb < nb; ++mb) {
    const uint8_t* in = mbinfo + (size_t)mb * VP8G_MBINFO_BYTES;
    const uint8_t* m = in + 4;
    const int x = mb % mbw;
    uint32_t H;
    if (in[0]) {
      H = kVP8ModeCostI16[m[0]];
    } else {
      const uint8_t* top = mb >= mbw ? mbinfo + (size_t)(mb - mbw) * VP8G_MBINFO_BYTES + 4 : NULL;
      const uint8_t* left = x > 0 ? mbinfo + (size_t)(mb - 1) * VP8G_MBINFO_BYTES + 4 : NULL;
      H = 211;
      for (int i = 0; i < 16; ++i) {
        const int bx = i & 3, by = i >> 2;
        const int t = by > 0 ? m[i - 4] : top ? top[12 + bx] : 0;
        const int l = bx > 0 ? m[i - 1] : left ? left[4 * by + 3] : 0;
        H += kVP8ModeCostI4[t][l][m[i]];
      }
    }
    sum += H + kVP8ModeCostUV[in[1]];
  }
  return sum;
}

double vp8h_psnr(uint64_t mse, uint64_t count) {
  return (mse > 0 && count > 0) ? 10. * log10(255. * 255. * count / mse) : 99;
}

/* ------------------------------------------------------------------------ */
/* k-means segmentation: analysis_enc.c:28-216 */

static void smooth_map(uint8_t* seg, int w, int h) {
  uint8_t* tmp = (uint8_t*)malloc((size_t)w * h);
  if (!tmp) return;
  for (int y = 1; y < h - 1; ++y)
    for (int x = 1; x < w - 1; ++x) {
      const uint8_t* s = seg + x + w * y;
      int cnt[4] = {0, 0, 0, 0}, maj = s[0];
      cnt[s[-w - 1]]++; cnt[s[-w]]++; cnt[s[-w + 1]]++; cnt[s[-1]]++;
      cnt[s[1]]++; cnt[s[w - 1]]++; cnt[s[w]]++; cnt[s[w + 1]]++;
      for (int n = 0; n < 4; ++n)
        if (cnt[n] >= 5) { maj = n; break; }
      tmp[x + y * w] = (uint8_t)maj;
    }
  for (int y = 1; y < h - 1; ++y)
    for (int x = 1; x < w - 1; ++x) seg[x + w * y] = tmp[x + y * w];
  free(tmp);
}

static void kmeans_segments(vp8h_frame* fr, const uint8_t* mb_alpha, uint8_t* segmap) {
  const int nmb = fr->mbw * fr->mbh;
  const int nb = fr->num_segments < 4 ? fr->num_segments : 4;
  int alphas[256], map[256], centers[4], accum[4], dist[4];
  int n, k, wavg = 0;
  memset(alphas, 0, sizeof(alphas));
  memset(map, 0, sizeof(map));
  for (int i = 0; i < nmb; ++i) alphas[mb_alpha[i]]++;
  for (n = 0; n <= 255 && alphas[n] == 0; ++n) {}
  const int min_a = n;
  for (n = 255; n > min_a && alphas[n] == 0; --n) {}
  const int max_a = n;
  const int range = max_a - min_a;
  for (k = 0, n = 1; k < nb; ++k, n += 2) centers[k] = min_a + (n * range) / (2 * nb);
  for (k = 0; k < 6; ++k) {
    int tw = 0, moved = 0;
    for (n = 0; n < nb; ++n) accum[n] = dist[n] = 0;
    n = 0;
    for (int a = min_a; a <= max_a; ++a) {
      if (!alphas[a]) continue;
      while (n + 1 < nb && iabs(a - centers[n + 1]) < iabs(a - centers[n])) n++;
      map[a] = n;
      dist[n] += a * alphas[a];
      accum[n] += alphas[a];
    }
    wavg = 0;
    for (n = 0; n < nb; ++n) {
      if (!accum[n]) continue;
      const int c = (dist[n] + accum[n] / 2) / accum[n];
      moved += iabs(centers[n] - c);
      centers[n] = c;
      wavg += c * accum[n];
      tw += accum[n];
    }
    wavg = (wavg + tw / 2) / tw;
    if (moved < 5) break;
  }
  for (int i = 0; i < nmb; ++i) segmap[i] = (uint8_t)map[mb_alpha[i]];
  for (int a = 0; a < 256; ++a) fr->alpha_center[a] = (uint8_t)centers[map[a]];
  if (nb > 1 && (fr->preprocessing & 1)) smooth_map(segmap, fr->mbw, fr->mbh);
  int mn = centers[0], mx = centers[0];
  if (nb > 1)
    for (n = 0; n < nb; ++n) {
      if (mn > centers[n]) mn = centers[n];
      if (mx < centers[n]) mx = centers[n];
    }
  if (mx == mn) mx = mn + 1;
  for (n = 0; n < nb; ++n) {
    fr->seg_alpha[n] = clampi(255 * (centers[n] - wavg) / (mx - mn), -127, 127);
    fr->seg_beta[n] = clampi(255 * (centers[n] - mn) / (mx - mn), 0, 255);
  }
}

/* ------------------------------------------------------------------------ */
/* quant_enc.c:205-455 */

static int fill_matrix(vp8g_mtx* m, int type, int q_dc, int q_ac) {
  m->q[0] = (uint16_t)q_dc;
  m->q[1] = (uint16_t)q_ac;
  for (int i = 0; i < 2; ++i) {
    m->iq[i] = (uint16_t)((1 << QFIX) / m->q[i]);
    m->bias[i] = (uint32_t)kVP8BiasMtx[type][i > 0] << (QFIX - 8);
    m->zthresh[i] = ((1u << QFIX) - 1 - m->bias[i]) / m->iq[i];
  }
  for (int i = 2; i < 16; ++i) {
    m->q[i] = m->q[1]; m->iq[i] = m->iq[1];
    m->bias[i] = m->bias[1]; m->zthresh[i] = m->zthresh[1];
  }
  int sum = 0;
  for (int i = 0; i < 16; ++i) {
    m->sharpen[i] = (uint16_t)(type == 0 ? (kVP8FreqSharpen[i] * m->q[i]) >> 11 : 0);
    sum += m->q[i];
  }
  return (sum + 8) >> 4;
}

static double q_to_compression(double c) {
  const double lin = (c < 0.75) ? c * (2. / 3.) : 2. * c - 1.;
  return pow(lin, 1 / 3.);
}
static double q_to_jpeg_compression(double c, double alpha) {
  const double amin = 0.30, amax = 0.85, emin = 0.4, emax = 0.9;
  const double slope = (emin - emax) / (amax - amin);
  const double e = (alpha > amax) ? emin : (alpha < amin) ? emax : emax + slope * (alpha - amin);
  return pow(c, e);
}

static int get_proba(int a, int b) {
  const int t = a + b;
  return t == 0 ? 255 : (255 * a + t / 2) / t;
}

void vp8h_setup_segments(vp8h_frame* fr, const uint8_t* mb_alpha, const uint16_t* mb_uva,
                         uint8_t* segmap, vp8g_frame_params* P) {
  vp8h_analyze_segments(fr, mb_alpha, mb_uva, segmap);
  vp8h_set_loop_params(fr, fr->ps_q, segmap, P);
}

void vp8h_analyze_segments(vp8h_frame* fr, const uint8_t* mb_alpha, const uint16_t* mb_uva,
                           uint8_t* segmap) {
  const int nmb = fr->mbw * fr->mbh;
  /* VP8EncAnalyze tail (analysis_enc.c:422-482) */
  /* methods 0-1 also need the analysis' modes (analysis_enc.c:424-427) */
  const int do_seg = fr->emulate_jpeg_size || fr->num_segments > 1 || fr->method <= 1;
  if (do_seg) {
    long sa = 0, suva = 0;
    for (int i = 0; i < nmb; ++i) { sa += mb_alpha[i]; suva += mb_uva[i]; }
    fr->alpha = (int)(sa / nmb);
    fr->uv_alpha = (int)(suva / nmb);
    kmeans_segments(fr, mb_alpha, segmap);
  } else {
    memset(segmap, 0, (size_t)nmb);
    memset(fr->alpha_center, 0, sizeof(fr->alpha_center));
    fr->seg_alpha[0] = fr->seg_beta[0] = 0;
    fr->alpha = fr->uv_alpha = 0;
  }
}

void vp8h_set_loop_params(vp8h_frame* fr, float quality, uint8_t* segmap, vp8g_frame_params* P) {
  const int nmb = fr->mbw * fr->mbh;
  /* SetLoopParams: q clamped to [0, 100] */
  quality = quality < 0.f ? 0.f : quality > 100.f ? 100.f : quality;
  /* VP8SetSegmentParams */
  const int ns = fr->num_segments;
  const double amp = 0.9 * fr->sns_strength / 100. / 128.;
  const double Q = quality / 100.;
  const double cbase = fr->emulate_jpeg_size ? q_to_jpeg_compression(Q, fr->alpha / 255.)
                                             : q_to_compression(Q);
  for (int i = 0; i < ns; ++i) {
    const double expn = 1. - amp * fr->seg_alpha[i];
    fr->seg_quant[i] = clampi((int)(127. * (1. - pow(cbase, expn))), 0, 127);
  }
  fr->base_quant = fr->seg_quant[0];
  for (int i = ns; i < 4; ++i) fr->seg_quant[i] = fr->base_quant;
  int dq_uv_ac = (fr->uv_alpha - 64) * (6 - (-4)) / (100 - 30);
  dq_uv_ac = dq_uv_ac * fr->sns_strength / 100;
  fr->dq_uv_ac = clampi(dq_uv_ac, -4, 6);
  fr->dq_uv_dc = clampi(-4 * fr->sns_strength / 100, -15, 15);
  /* SetupFilterStrength: uses the header sharpness *before* it is set */
  const int level0 = 5 * fr->filter_strength;
  for (int i = 0; i < 4; ++i) {
    const int qstep = kVP8AcQ[clampi(fr->seg_quant[i], 0, 127)] >> 2;
    const int base = kVP8LevelsFromDelta[fr->f_sharpness][qstep < 64 ? qstep : 63];
    const int f = base * level0 / (256 + fr->seg_beta[i]);
    fr->seg_fstrength[i] = (f < 2) ? 0 : (f > 63) ? 63 : f;
  }
  fr->f_level = fr->seg_fstrength[0];
  fr->f_simple = (fr->filter_type == 0);
  fr->f_sharpness = fr->filter_sharpness;
  /* SimplifySegments */
  if (ns > 1) {
    int map[4] = {0, 1, 2, 3}, nfinal = 1;
    for (int s1 = 1; s1 < ns; ++s1) {
      int s2, found = 0;
      for (s2 = 0; s2 < nfinal; ++s2)
        if (fr->seg_quant[s1] == fr->seg_quant[s2] &&
            fr->seg_fstrength[s1] == fr->seg_fstrength[s2]) {
          found = 1;
          break;
        }
      map[s1] = s2;
      if (!found) {
        if (nfinal != s1) {
          fr->seg_quant[nfinal] = fr->seg_quant[s1];
          fr->seg_fstrength[nfinal] = fr->seg_fstrength[s1];
          fr->seg_alpha[nfinal] = fr->seg_alpha[s1];
          fr->seg_beta[nfinal] = fr->seg_beta[s1];
        }
        ++nfinal;
      }
    }
    if (nfinal < ns) {
      for (int i = 0; i < nmb; ++i) segmap[i] = (uint8_t)map[segmap[i]];
      fr->num_segments = nfinal;
      for (int i = nfinal; i < ns; ++i) {
        fr->seg_quant[i] = fr->seg_quant[nfinal - 1];
        fr->seg_fstrength[i] = fr->seg_fstrength[nfinal - 1];
        fr->seg_alpha[i] = fr->seg_alpha[nfinal - 1];
        fr->seg_beta[i] = fr->seg_beta[nfinal - 1];
      }
    }
  }
  /* SetupMatrices */
  memset(P, 0, sizeof(*P));
  const int tls = fr->method >= 4 ? fr->sns_strength : 0;
  for (int i = 0; i < fr->num_segments; ++i) {
    vp8g_seg* m = &P->seg[i];
    const int q = fr->seg_quant[i];
    const int q_i4 = fill_matrix(&m->y1, 0, kVP8DcQ[clampi(q, 0, 127)], kVP8AcQ[clampi(q, 0, 127)]);
    const int q_i16 = fill_matrix(&m->y2, 1, kVP8DcQ[clampi(q, 0, 127)] * 2,
                                  kVP8AcQ2[clampi(q, 0, 127)]);
    const int q_uv = fill_matrix(&m->uv, 2, kVP8DcQ[clampi(q + fr->dq_uv_dc, 0, 117)],
                                 kVP8AcQ[clampi(q + fr->dq_uv_ac, 0, 127)]);
#define AT_LEAST_1(v) ((v) < 1 ? 1 : (v))
    m->lambda_i4 = AT_LEAST_1((3 * q_i4 * q_i4) >> 7);
    m->lambda_i16 = AT_LEAST_1(3 * q_i16 * q_i16);
    m->lambda_uv = AT_LEAST_1((3 * q_uv * q_uv) >> 6);
    m->lambda_mode = AT_LEAST_1((1 * q_i4 * q_i4) >> 7);
    m->lambda_trellis_i4 = AT_LEAST_1((7 * q_i4 * q_i4) >> 3);
    m->lambda_trellis_i16 = AT_LEAST_1((q_i16 * q_i16) >> 2);
    m->lambda_trellis_uv = AT_LEAST_1((q_uv * q_uv) << 1);
    m->tlambda = AT_LEAST_1((tls * q_i4) >> 5);
    m->i4_penalty = 1000 * q_i4 * q_i4;
#undef AT_LEAST_1
    m->min_disto = 20 * m->y1.q[0];
    fr->seg_y2ac[i] = m->y2.q[1];
  }
  for (int i = fr->num_segments; i < 4; ++i) fr->seg_y2ac[i] = 0;
  /* SetSegmentProbas (frame_enc.c:198-231) */
  int p[4] = {0, 0, 0, 0};
  for (int i = 0; i < nmb; ++i) p[segmap[i]]++;
  for (int i = 0; i < 4; ++i) fr->segment_size[i] = p[i];
  if (fr->num_segments > 1) {
    uint8_t* pr = fr->seg_probas;
    pr[0] = (uint8_t)get_proba(p[0] + p[1], p[2] + p[3]);
    pr[1] = (uint8_t)get_proba(p[0], p[1]);
    pr[2] = (uint8_t)get_proba(p[2], p[3]);
    fr->update_map = (pr[0] != 255) || (pr[1] != 255) || (pr[2] != 255);
    if (!fr->update_map) memset(segmap, 0, (size_t)nmb);
    fr->seg_hdr_size = p[0] * (bit_cost(0, pr[0]) + bit_cost(0, pr[1])) +
                       p[1] * (bit_cost(0, pr[0]) + bit_cost(1, pr[1])) +
                       p[2] * (bit_cost(1, pr[0]) + bit_cost(0, pr[2])) +
                       p[3] * (bit_cost(1, pr[0]) + bit_cost(1, pr[2]));
  } else {
    fr->update_map = 0;
    fr->seg_hdr_size = 0;
  }
  P->max_i4_header_bits = fr->max_i4_header_bits;
  P->rd_opt = fr->rd_opt;
  P->method = fr->method;
  P->use_derr = fr->quality <= 98 || fr->cfg_pass > 1;   /* webp_enc.c:162-164 */
  P->max_count = (nmb >> 3) < 96 ? 96 : (nmb >> 3);
  /* RD_OPT_NONE (VP8EncLoop): no refreshes; StatLoop's probe size (:631-638)
   * and whether it reaches its finalisation (header estimate != 0, :645) */
  P->mb_header_limit = (int32_t)((int64_t)256 * 510 * 8 * 1024 / nmb);
  P->nb_stat = fr->method == 0 ? ((nmb > 200) ? nmb >> 2 : 50) : nmb;
  P->none_finalize = fr->seg_hdr_size != 0;
  P->skip_count = -1;
  if (fr->rd_opt == 0) P->max_count = 0x7fffffff;
}

/* ------------------------------------------------------------------------ */
/* Dithered RGB -> YUV import: webp_enc.c:357-365, picture_csp_enc.c:150-166,
 * 520-619, utils/random_utils.{h,c} */

float vp8h_import_dithering(const WebPConfig* cfg) {
  if (!(cfg->preprocessing & 2)) return 0.f;
  const float x = cfg->quality / 100.f;
  const float x2 = x * x;
  return 1.0f + (0.5f - 1.0f) * x2 * x2;   /* 1 at q 0 down to 0.5 at q 100 */
}

static const uint32_t kRandomTable[55] = {   /* random_utils.c:19-29 */
    0x0de15230, 0x03b31886, 0x775faccb, 0x1c88626a, 0x68385c55, 0x14b3b828, 0x4a85fef8,
    0x49ddb84b, 0x64fcf397, 0x5c550289, 0x4a290000, 0x0d7ec1da, 0x5940b7ab, 0x5492577d,
    0x4e19ca72, 0x38d38c69, 0x0c01ee65, 0x32a1755f, 0x5437f652, 0x5abb2c32, 0x0faa57b1,
    0x73f533e7, 0x685feeda, 0x7563cce2, 0x6e990e83, 0x4730a7ed, 0x4fc0d9c6, 0x496b153c,
    0x4f1403fa, 0x541afb0c, 0x73990b32, 0x26d7cb1c, 0x6fcc3706, 0x2cbb77d8, 0x75762f2a,
    0x6425ccdd, 0x24b35461, 0x0a7d8715, 0x220414a8, 0x141ebf67, 0x56b41583, 0x73e502e3,
    0x44cab16f, 0x28264d42, 0x73baaefb, 0x0a50ebed, 0x1d6ab6fb, 0x0d3ad40b, 0x35db3b68,
    0x2b081e83, 0x77ce6b95, 0x5181e5f0, 0x78853bbc, 0x009f9494, 0x27e5ed3c};

typedef struct {
  int i1, i2, amp;
  uint32_t tab[55];
} DitherRng;

static int rng_bits(DitherRng* rg, int num_bits) {   /* VP8RandomBits2 */
  int diff = (int)(rg->tab[rg->i1] - rg->tab[rg->i2]);
  if (diff < 0) diff = (int)((uint32_t)diff + (1u << 31));
  rg->tab[rg->i1] = (uint32_t)diff;
  if (++rg->i1 == 55) rg->i1 = 0;
  if (++rg->i2 == 55) rg->i2 = 0;
  diff = (int)((uint32_t)diff << 1) >> (32 - num_bits);   /* sign-extend, 0-center */
  diff = (diff * rg->amp) >> 8;
  return diff + (1 << (num_bits - 1));
}

void vp8h_dither_rounders(int w, int h, float dithering, uint16_t* ry, uint32_t* ruv) {
  DitherRng rg;
  memcpy(rg.tab, kRandomTable, sizeof(rg.tab));
  rg.i1 = 0;
  rg.i2 = 31;
  rg.amp = (dithering < 0.0) ? 0 : (dithering > 1.0) ? 256 : (int)(uint32_t)(256 * dithering);
  const int uvw = (w + 1) >> 1;
  /* the reference's order: two Y rows, then the U,V pairs of their chroma row */
  for (int y = 0; y < (h >> 1); ++y) {
    for (int r = 0; r < 2; ++r)
      for (int x = 0; x < w; ++x) ry[(size_t)(2 * y + r) * w + x] = (uint16_t)rng_bits(&rg, 16);
    for (int i = 0; i < uvw; ++i) {
      ruv[2 * ((size_t)y * uvw + i)] = (uint32_t)rng_bits(&rg, 18);
      ruv[2 * ((size_t)y * uvw + i) + 1] = (uint32_t)rng_bits(&rg, 18);
    }
  }
  if (h & 1) {
    const int y = h >> 1;
    for (int x = 0; x < w; ++x) ry[(size_t)(h - 1) * w + x] = (uint16_t)rng_bits(&rg, 16);
    for (int i = 0; i < uvw; ++i) {
      ruv[2 * ((size_t)y * uvw + i)] = (uint32_t)rng_bits(&rg, 18);
      ruv[2 * ((size_t)y * uvw + i) + 1] = (uint32_t)rng_bits(&rg, 18);
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Alpha level reduction: src/utils/quant_levels_utils.c:31-137 */

int vp8h_alpha_levels(int quality) {
  return (quality <= 70) ? (2 + quality / 5) : (16 + (quality - 70) * 8);
}

void vp8h_quantize_levels_map(const uint32_t hist[256], uint64_t count, int num_levels,
                              uint8_t map[256], uint64_t* sse) {
  int q_level[256] = {0};
  double inv_q_level[256] = {0};
  int min_s = 255, max_s = 0, num_levels_in = 0;
  double last_err = 1.e38, err = 0.;
  const double err_threshold = 1e-4 * (double)count;
  for (int s = 0; s < 256; ++s) {
    map[s] = (uint8_t)s;
    if (hist[s]) {
      ++num_levels_in;
      if (min_s > s) min_s = s;
      if (max_s < s) max_s = s;
    }
  }
  if (num_levels_in > num_levels) {
    for (int i = 0; i < num_levels; ++i)
      inv_q_level[i] = min_s + (double)(max_s - min_s) * i / (num_levels - 1);
    q_level[min_s] = 0;
    q_level[max_s] = num_levels - 1;
    for (int iter = 0; iter < 6; ++iter) {   /* k-means, MAX_ITER */
      double q_sum[256] = {0}, q_count[256] = {0};
      int slot = 0;
      for (int s = min_s; s <= max_s; ++s) {
        while (slot < num_levels - 1 && 2 * s > inv_q_level[slot] + inv_q_level[slot + 1]) ++slot;
        if (hist[s] > 0) {
          q_sum[slot] += s * (int)hist[s];
          q_count[slot] += (int)hist[s];
        }
        q_level[s] = slot;
      }
      if (num_levels > 2)
        for (slot = 1; slot < num_levels - 1; ++slot)
          if (q_count[slot] > 0.) inv_q_level[slot] = q_sum[slot] / q_count[slot];
      err = 0.;
      for (int s = min_s; s <= max_s; ++s) {
        const double e = s - inv_q_level[q_level[s]];
        err += (int)hist[s] * e * e;
      }
      if (last_err - err < err_threshold) break;
      last_err = err;
    }
    for (int s = min_s; s <= max_s; ++s) map[s] = (uint8_t)(inv_q_level[q_level[s]] + .5);
  }
  if (sse) *sse = (uint64_t)err;
}

/* ------------------------------------------------------------------------ */
/* Boolean coder: bit_writer_utils.c:26-179. Renormalisation shift is
 * 7 - floor(log2(range + 1)) (the kNorm / kNewRange tables). */

void vp8h_bw_init(vp8h_bw* bw, size_t expected) {
  memset(bw, 0, sizeof(*bw));
  bw->range = 254;
  bw->nb_bits = -8;
  if (expected) {
    bw->buf = (uint8_t*)malloc(expected);
    if (bw->buf) bw->cap = expected; else bw->error = 1;
  }
}

void vp8h_bw_free(vp8h_bw* bw) {
  if (bw->cap) free(bw->buf);   /* cap 0: the bytes are borrowed (K4's packed output) */
  bw->buf = NULL;
  bw->cap = bw->pos = 0;
}

static int bw_grow(vp8h_bw* bw, size_t extra) {
  if (bw->pos + extra <= bw->cap) return 1;
  size_t n = 2 * bw->cap;
  if (n < bw->pos + extra) n = bw->pos + extra;
  if (n < 1024) n = 1024;
  uint8_t* nb = (uint8_t*)realloc(bw->buf, n);
  if (!nb) { bw->error = 1; return 0; }
  bw->buf = nb;
  bw->cap = n;
  return 1;
}

static void bw_flush(vp8h_bw* bw) {
  const int s = 8 + bw->nb_bits;
  const int32_t bits = bw->value >> s;
  bw->value -= bits << s;
  bw->nb_bits -= 8;
  if ((bits & 0xff) != 0xff) {
    size_t pos = bw->pos;
    if (!bw_grow(bw, bw->run + 1)) return;
    if ((bits & 0x100) && pos > 0) bw->buf[pos - 1]++;
    const uint8_t fillv = (bits & 0x100) ? 0x00 : 0xff;
    for (; bw->run > 0; --bw->run) bw->buf[pos++] = fillv;
    bw->buf[pos++] = (uint8_t)(bits & 0xff);
    bw->pos = pos;
  } else {
    bw->run++;
  }
}

static inline int bw_put(vp8h_bw* bw, int bit, int prob) {
  const int split = (bw->range * prob) >> 8;
  if (bit) { bw->value += split + 1; bw->range -= split + 1; }
  else { bw->range = split; }
  if (bw->range < 127) {
    const int shift = __builtin_clz((unsigned)(bw->range + 1)) - 24;
    bw->range = ((bw->range + 1) << shift) - 1;
    bw->value <<= shift;
    bw->nb_bits += shift;
    if (bw->nb_bits > 0) bw_flush(bw);
  }
  return bit;
}

static inline int bw_put_uniform(vp8h_bw* bw, int bit) { return bw_put(bw, bit, 128); }

static void bw_put_bits(vp8h_bw* bw, uint32_t v, int n) {
  for (uint32_t m = 1u << (n - 1); m; m >>= 1) bw_put_uniform(bw, (v & m) != 0);
}

void vp8h_bw_finish(vp8h_bw* bw) {
  bw_put_bits(bw, 0, 9 - bw->nb_bits);
  bw->nb_bits = 0;
  bw_flush(bw);
}

void vp8h_emit_tokens(vp8h_bw* bw, const uint16_t* tok, size_t n, const uint8_t* probas) {
  /* hot loop: keep the coder state in registers, spill only to flush */
  int32_t range = bw->range, value = bw->value;
  int nb_bits = bw->nb_bits;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t t = tok[i];
    const int bit = (int)(t >> 15);
    const int p = (t & 0x4000) ? (int)(t & 0xff) : probas[t & 0x3fff];
    const int split = (range * p) >> 8;
    const int32_t one = split + 1;
    value += bit ? one : 0;
    range = bit ? range - one : split;
    if (range < 127) {
      const int shift = __builtin_clz((unsigned)(range + 1)) - 24;
      range = ((range + 1) << shift) - 1;
      value <<= shift;
      nb_bits += shift;
      if (nb_bits > 0) {
        bw->range = range; bw->value = value; bw->nb_bits = nb_bits;
        bw_flush(bw);
        value = bw->value; nb_bits = bw->nb_bits;
      }
    }
  }
  bw->range = range; bw->value = value; bw->nb_bits = nb_bits;
}

/* ------------------------------------------------------------------------ */
/* Partition 0 (syntax_enc.c:187-310, tree_enc.c:270-347,485-504) and the
 * RIFF container (syntax_enc.c:37-185,320-389). */

/* Partition-0 modes are coded in two steps per MB row: the row's decisions
 * become (bit << 8 | probability) tokens through path tables (no branches on
 * the modes), then one tight coder loop with a branch-free renormalisation
 * codes them; both branch-heavy tree walks of the direct form mispredicted on
 * nearly every decision. */
#define P0_MB_TOKENS 128   /* >= 2 + 1 + 16 * 7 + 3, plus 7 slack for the path writes */

/* intra4 mode tree (tree_enc.c:270-295): nodes visited and bits, per mode */
static const uint8_t kI4PathLen[10] = {1, 2, 3, 5, 6, 6, 5, 6, 7, 7};
static const uint8_t kI4PathNode[10][7] = {
    {0}, {0, 1}, {0, 1, 2}, {0, 1, 2, 3, 4}, {0, 1, 2, 3, 4, 5}, {0, 1, 2, 3, 4, 5},
    {0, 1, 2, 3, 6}, {0, 1, 2, 3, 6, 7}, {0, 1, 2, 3, 6, 7, 8}, {0, 1, 2, 3, 6, 7, 8}};
static const uint8_t kI4PathBit[10][7] = {
    {0}, {1, 0}, {1, 1, 0}, {1, 1, 1, 0, 0}, {1, 1, 1, 0, 1, 0}, {1, 1, 1, 0, 1, 1},
    {1, 1, 1, 1, 0}, {1, 1, 1, 1, 1, 0}, {1, 1, 1, 1, 1, 1, 0}, {1, 1, 1, 1, 1, 1, 1}};

static inline uint32_t p0_tok(int bit, int prob) { return ((uint32_t)bit << 8) | (uint32_t)prob; }

static void p0_code(vp8h_bw* bw, const uint16_t* tok, size_t n) {
  int32_t range = bw->range, value = bw->value;
  int nb_bits = bw->nb_bits;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t t = tok[i];
    const int split = (range * (int)(t & 0xff)) >> 8;
    const int bit = (int)(t >> 8);
    value += bit ? split + 1 : 0;
    range = bit ? range - split - 1 : split;
    const int shift = __builtin_clz((unsigned)(range + 1)) - 24;   /* 0 when range >= 127 */
    range = ((range + 1) << shift) - 1;
    value <<= shift;
    nb_bits += shift;
    if (nb_bits > 0) {
      bw->value = value; bw->nb_bits = nb_bits;
      bw_flush(bw);
      value = bw->value; nb_bits = bw->nb_bits;
    }
  }
  bw->range = range; bw->value = value; bw->nb_bits = nb_bits;
}

static void code_intra_modes(vp8h_bw* bw, const vp8h_frame* fr, const uint8_t* mbinfo,
                             int use_skip, int skip_proba) {
  const int mbw = fr->mbw;
  uint8_t* top_modes = (uint8_t*)calloc(4 * (size_t)mbw, 1);   /* B_DC_PRED border */
  uint16_t* tok = (uint16_t*)malloc((size_t)mbw * P0_MB_TOKENS * sizeof(uint16_t));
  if (!top_modes || !tok) { bw->error = 1; free(top_modes); free(tok); return; }
  const int upd = fr->update_map;
  const uint8_t* sp = fr->seg_probas;
  for (int y = 0; y < fr->mbh; ++y) {
    uint8_t left_modes[4] = {0, 0, 0, 0};
    size_t n = 0;
    for (int x = 0; x < mbw; ++x) {
      const uint8_t* info = mbinfo + ((size_t)y * mbw + x) * VP8G_MBINFO_BYTES;
      const uint8_t* modes = info + 4;
      if (upd) {   /* segment id tree */
        const int s = info[2];
        tok[n] = (uint16_t)p0_tok(s >= 2, sp[0]);
        tok[n + 1] = (uint16_t)p0_tok(s & 1, sp[1 + (s >= 2)]);
        n += 2;
      }
      if (use_skip) tok[n++] = (uint16_t)p0_tok(info[3] != 0, skip_proba);   /* tree_enc.c:323-325 */
      const int i16 = info[0] != 0;
      tok[n++] = (uint16_t)p0_tok(i16, 145);
      if (i16) {
        const int m = modes[0];
        const int b0 = m == 1 || m == 3;
        tok[n] = (uint16_t)p0_tok(b0, 156);
        tok[n + 1] = (uint16_t)(b0 ? p0_tok(m == 1, 128) : p0_tok(m == 2, 163));
        n += 2;
      } else {
        for (int yy = 0; yy < 4; ++yy) {
          int left = left_modes[yy];
          for (int xx = 0; xx < 4; ++xx) {
            const int top = yy == 0 ? top_modes[4 * x + xx] : modes[4 * (yy - 1) + xx];
            const uint8_t* pr = kVP8BModeProba[top][left];
            const int m = modes[4 * yy + xx];
            for (int k = 0; k < 7; ++k)   /* fixed trip count; the length advances n */
              tok[n + k] = (uint16_t)p0_tok(kI4PathBit[m][k], pr[kI4PathNode[m][k]]);
            n += kI4PathLen[m];
            left = m;
          }
        }
      }
      const int uvm = info[1];   /* uv mode tree: DC, then V / H / TM */
      tok[n] = (uint16_t)p0_tok(uvm != 0, 142);
      tok[n + 1] = (uint16_t)p0_tok(uvm != 2, 114);
      tok[n + 2] = (uint16_t)p0_tok(uvm != 3, 183);
      n += uvm == 0 ? 1 : uvm == 2 ? 2 : 3;
      for (int k = 0; k < 4; ++k) {
        top_modes[4 * x + k] = modes[12 + k];
        left_modes[k] = modes[4 * k + 3];
      }
    }
    p0_code(bw, tok, n);
  }
  free(top_modes);
  free(tok);
}

static void put_le32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* The frame header part of partition 0 (syntax_enc.c:187-245 PutSegmentHeader
 * .. PutQuant, tree_enc.c:485-504 VP8WriteProbas, the skip probability) as
 * fixed-probability K4 tokens (bit << 15 | 0x4000 | probability): coded here
 * by vp8h_build_p0, or appended to by k_p0_modes and coded by K4. */
typedef struct {
  uint16_t* t;
  int n, cap;
} p0_hdr;
static inline int hput(p0_hdr* h, int bit, int prob) {
  if (h->n < h->cap) h->t[h->n] = (uint16_t)((bit ? 0x8000u : 0u) | 0x4000u | (unsigned)prob);
  ++h->n;
  return bit;
}
static void hput_bits(p0_hdr* h, uint32_t v, int n) {   /* VP8PutBits */
  for (uint32_t m = 1u << (n - 1); m; m >>= 1) hput(h, (v & m) != 0, 128);
}
static void hput_signed(p0_hdr* h, int v, int n) {      /* VP8PutSignedBits */
  if (!hput(h, v != 0, 128)) return;
  if (v < 0) hput_bits(h, ((uint32_t)(-v) << 1) | 1, n + 1);
  else hput_bits(h, (uint32_t)v << 1, n + 1);
}

int vp8h_p0_header(vp8h_frame* fr, const vp8g_frame_result* res, uint16_t* tok, int cap,
                   int* hdr_bytes0) {
  /* VP8AdjustFilterStrength (filter_enc.c:194-233): with the autofilter the
   * engine has already set seg_fstrength from the SSIM statistics */
  if (!fr->autofilter && fr->filter_strength > 0) {
    int max_level = 0;
    for (int s = 0; s < 4; ++s) {
      const int delta = (res->max_edge[s] * fr->seg_y2ac[s]) >> 3;
      const int lvl = kVP8LevelsFromDelta[fr->f_sharpness][delta < 64 ? delta : 63];
      if (lvl > fr->seg_fstrength[s]) fr->seg_fstrength[s] = lvl;
      if (max_level < fr->seg_fstrength[s]) max_level = fr->seg_fstrength[s];
    }
    fr->f_level = max_level;
  }
  p0_hdr h = {tok, 0, cap}, *H = &h;
  hput(H, 0, 128);   /* colorspace */
  hput(H, 0, 128);   /* clamping type */
  if (hput(H, fr->num_segments > 1, 128)) {
    hput(H, fr->update_map, 128);
    hput(H, 1, 128);   /* update segment feature data */
    hput(H, 1, 128);   /* absolute values */
    for (int s = 0; s < 4; ++s) hput_signed(H, fr->seg_quant[s], 7);
    for (int s = 0; s < 4; ++s) hput_signed(H, fr->seg_fstrength[s], 6);
    if (fr->update_map)
      for (int s = 0; s < 3; ++s)
        if (hput(H, fr->seg_probas[s] != 255u, 128)) hput_bits(H, fr->seg_probas[s], 8);
  }
  hput(H, fr->f_simple, 128);
  hput_bits(H, (uint32_t)fr->f_level, 6);
  hput_bits(H, (uint32_t)fr->f_sharpness, 3);
  hput(H, 0, 128);          /* no loop-filter deltas */
  hput_bits(H, fr->num_parts == 8 ? 3 : fr->num_parts == 4 ? 2 : fr->num_parts == 2 ? 1 : 0,
            2);             /* token partitions (syntax_enc.c:283-285) */
  hput_bits(H, (uint32_t)fr->base_quant, 7);
  hput_signed(H, 0, 4);     /* dq_y1_dc */
  hput_signed(H, 0, 4);     /* dq_y2_dc */
  hput_signed(H, 0, 4);     /* dq_y2_ac */
  hput_signed(H, fr->dq_uv_dc, 4);
  hput_signed(H, fr->dq_uv_ac, 4);
  hput(H, 0, 128);          /* no probability refresh */
  const uint8_t* p0 = &kVP8CoeffProba0[0][0][0][0];
  const uint8_t* pu = &kVP8CoeffUpdateProba[0][0][0][0];
  for (int s = 0; s < VP8G_NUM_SLOTS; ++s) {
    const int v = res->probas[s];
    if (hput(H, v != p0[s], pu[s])) hput_bits(H, (uint32_t)v, 8);
  }
  /* skip probability (tree_enc.c:500-502): only the RD_OPT_NONE loop uses it */
  if (hput(H, res->use_skip != 0, 128)) hput_bits(H, (uint32_t)res->skip_proba, 8);
  if (h.n > cap) return -1;
  if (hdr_bytes0) {   /* the bytes the coder has written after the header (WebPAuxStats) */
    vp8h_bw bw;
    vp8h_bw_init(&bw, 2048);
    vp8h_emit_tokens(&bw, tok, (size_t)h.n, NULL);
    *hdr_bytes0 = bw.error ? 0 : (int)bw.pos;
    vp8h_bw_free(&bw);
  }
  return h.n;
}

void vp8h_p0_par(const vp8h_frame* fr, const vp8g_frame_result* res, int nhdr, vp8g_p0_par* p) {
  memset(p, 0, sizeof(*p));
  p->nhdr = nhdr < 0 ? 0xffffffffu : (uint32_t)nhdr;
  p->update_map = (uint8_t)(fr->update_map != 0);
  p->use_skip = (uint8_t)(res->use_skip != 0);
  p->skip_proba = (uint8_t)res->skip_proba;
  for (int s = 0; s < 3; ++s) p->seg_probas[s] = fr->seg_probas[s];
}

int vp8h_build_p0(vp8h_frame* fr, const vp8g_frame_result* res, const uint8_t* mbinfo,
                  vp8h_bw* out0, int* hdr_bytes) {
  uint16_t tok[VP8G_P0_HDR_CAP];
  vp8h_bw bw;
  vp8h_bw_init(&bw, (size_t)fr->mbw * fr->mbh * 7 / 8 + 1024);
  *out0 = bw;   /* handed back even on error so the caller can free it */
  const int nh = vp8h_p0_header(fr, res, tok, VP8G_P0_HDR_CAP, NULL);
  if (nh < 0) return VP8_ENC_ERROR_OUT_OF_MEMORY;
  vp8h_emit_tokens(&bw, tok, (size_t)nh, NULL);
  const size_t hdr_pos = bw.pos;
  code_intra_modes(&bw, fr, mbinfo, res->use_skip != 0, res->skip_proba);
  vp8h_bw_finish(&bw);
  *out0 = bw;
  if (hdr_bytes) { hdr_bytes[0] = (int)hdr_pos; hdr_bytes[1] = (int)(bw.pos - hdr_pos); }
  if (bw.error) return VP8_ENC_ERROR_OUT_OF_MEMORY;
  if (bw.pos >= (1u << 19)) return VP8_ENC_ERROR_PARTITION0_OVERFLOW;
  return VP8_ENC_OK;
}

size_t vp8h_write_riff(const vp8h_frame* fr, vp8h_bw* p0, const vp8h_bw* parts, int nparts,
                       const vp8h_alpha* alpha, uint8_t** out, size_t* cap, int* err) {
  /* VP8EncWrite + PutWebPHeaders (syntax_enc.c:149-185, 320-392): RIFF,
   * [VP8X + ALPH when the picture has alpha], 'VP8 ', frame header,
   * partition 0, the sizes of all token partitions but the last (3 bytes
   * each, EmitPartitionsSize :248-265), the token partitions, pad byte */
  vp8h_bw bw = *p0;
  memset(p0, 0, sizeof(*p0));
  size_t size1 = 0;
  for (int p = 0; p < nparts; ++p) {
    if (parts[p].error) {
      vp8h_bw_free(&bw);
      *err = VP8_ENC_ERROR_OUT_OF_MEMORY;
      return 0;
    }
    if (p < nparts - 1 && parts[p].pos >= (1u << 24)) {   /* VP8_MAX_PARTITION_SIZE */
      vp8h_bw_free(&bw);
      *err = VP8_ENC_ERROR_PARTITION_OVERFLOW;
      return 0;
    }
    size1 += parts[p].pos;
  }
  const size_t size0 = bw.pos, psz = 3 * (size_t)(nparts - 1);
  size_t vp8_size = 10 + size0 + psz + size1;
  const size_t pad = vp8_size & 1;
  vp8_size += pad;
  size_t riff_size = 4 + 8 + vp8_size;
  const size_t asize = alpha ? 1 + alpha->size : 0;   /* header byte + data */
  if (alpha) riff_size += 8 + 10 + 8 + asize + (asize & 1);   /* VP8X + ALPH chunks */
  if (riff_size > 0xfffffffeU) {
    vp8h_bw_free(&bw);
    *err = VP8_ENC_ERROR_FILE_TOO_BIG;
    return 0;
  }
  const size_t total = 8 + riff_size;
  uint8_t* o = cap && *out && *cap >= total ? *out : (uint8_t*)malloc(total);
  if (!o) {
    vp8h_bw_free(&bw);
    *err = VP8_ENC_ERROR_OUT_OF_MEMORY;
    return 0;
  }
  memcpy(o, "RIFF", 4);
  put_le32(o + 4, (uint32_t)riff_size);
  memcpy(o + 8, "WEBP", 4);
  uint8_t* q = o + 12;
  if (alpha) {
    memcpy(q, "VP8X", 4);
    put_le32(q + 4, 10);
    put_le32(q + 8, 0x10);   /* ALPHA_FLAG */
    q[12] = (uint8_t)(fr->w - 1); q[13] = (uint8_t)((fr->w - 1) >> 8);
    q[14] = (uint8_t)((fr->w - 1) >> 16);
    q[15] = (uint8_t)(fr->h - 1); q[16] = (uint8_t)((fr->h - 1) >> 8);
    q[17] = (uint8_t)((fr->h - 1) >> 16);
    q += 18;
    memcpy(q, "ALPH", 4);
    put_le32(q + 4, (uint32_t)asize);
    q[8] = alpha->header;
    if (alpha->size) memcpy(q + 9, alpha->data, alpha->size);
    q += 8 + asize;
    if (asize & 1) *q++ = 0;
  }
  memcpy(q, "VP8 ", 4);
  put_le32(q + 4, (uint32_t)vp8_size);
  const uint32_t bits = (uint32_t)(fr->profile << 1) | (1u << 4) | ((uint32_t)size0 << 5);
  uint8_t* fh = q + 8;
  fh[0] = (uint8_t)bits; fh[1] = (uint8_t)(bits >> 8); fh[2] = (uint8_t)(bits >> 16);
  fh[3] = 0x9d; fh[4] = 0x01; fh[5] = 0x2a;   /* VP8 keyframe signature */
  fh[6] = (uint8_t)(fr->w & 0xff); fh[7] = (uint8_t)(fr->w >> 8);
  fh[8] = (uint8_t)(fr->h & 0xff); fh[9] = (uint8_t)(fr->h >> 8);
  memcpy(fh + 10, bw.buf, size0);
  uint8_t* d = fh + 10 + size0;
  for (int p = 0; p < nparts - 1; ++p) {
    const size_t ps = parts[p].pos;
    d[0] = (uint8_t)ps; d[1] = (uint8_t)(ps >> 8); d[2] = (uint8_t)(ps >> 16);
    d += 3;
  }
  for (int p = 0; p < nparts; ++p) {
    if (parts[p].pos) memcpy(d, parts[p].buf, parts[p].pos);
    d += parts[p].pos;
  }
  if (pad) *d = 0;
  vp8h_bw_free(&bw);
  if (o != *out) {
    if (cap) {   /* the caller's buffer was too small: replace it */
      free(*out);
      *cap = total;
    }
    *out = o;
  }
  *err = VP8_ENC_OK;
  return total;
}

size_t vp8h_assemble(vp8h_frame* fr, const vp8g_frame_result* res, const uint8_t* mbinfo,
                     vp8h_bw* part1, uint8_t** out, int* err, int* hdr_bytes) {
  vp8h_bw p0;
  *err = vp8h_build_p0(fr, res, mbinfo, &p0, hdr_bytes);
  if (*err != VP8_ENC_OK) {
    vp8h_bw_free(&p0);
    return 0;
  }
  return vp8h_write_riff(fr, &p0, part1, 1, NULL, out, NULL, err);
}
