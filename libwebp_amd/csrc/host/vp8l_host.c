/* Host side of the lossless (VP8L) path: Huffman codes, the header bits and
 * the RIFF container. Every choice here is the one oracle/vp8l_model.py
 * states (same function names), so the GPU bitstream can be checked bit for
 * bit against the model; the format is the reference decoder's:
 *   header / transforms / cache / meta codes   src/dec/vp8l_dec.c:126-135, 1330-1380, 1455-1490, 364-420
 *   Huffman code reading                       src/dec/vp8l_dec.c:255-356
 * The code-length layout follows the reference writer's structure
 * (src/enc/vp8l_enc.c:476-643: storage order, simple codes, single-symbol
 * codes written with zero bits). */
#include "vp8l_host.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- writer */

void vp8l_bw_init(vp8l_bw* bw, size_t cap) {
  memset(bw, 0, sizeof(*bw));
  bw->buf = (uint8_t*)malloc(cap ? cap : 1);
  bw->cap = bw->buf ? cap : 0;
  bw->oom = bw->buf == NULL;
}

void vp8l_bw_free(vp8l_bw* bw) {
  free(bw->buf);
  memset(bw, 0, sizeof(*bw));
}

static void bw_byte(vp8l_bw* bw, uint8_t v) {
  if (bw->pos == bw->cap) {
    const size_t cap = bw->cap ? 2 * bw->cap : 1024;
    uint8_t* nb = (uint8_t*)realloc(bw->buf, cap);
    if (!nb) { bw->oom = 1; return; }
    bw->buf = nb;
    bw->cap = cap;
  }
  bw->buf[bw->pos++] = v;
}

void vp8l_bw_put(vp8l_bw* bw, uint32_t v, int nbits) {
  if (nbits <= 0) return;
  bw->acc |= (uint64_t)(v & (uint32_t)((1ull << nbits) - 1)) << bw->used;
  bw->used += nbits;
  bw->nbits += (uint64_t)nbits;
  while (bw->used >= 8) {
    bw_byte(bw, (uint8_t)bw->acc);
    bw->acc >>= 8;
    bw->used -= 8;
  }
}

size_t vp8l_bw_finish(vp8l_bw* bw) {
  if (bw->used) {
    bw_byte(bw, (uint8_t)bw->acc);
    bw->acc = 0;
    bw->used = 0;
  }
  return bw->pos;
}

/* ---------------------------------------------------------------- params */

static int sub_sample(int size, int bits) { return (size + (1 << bits) - 1) >> bits; }

int vp8l_histo_bits(int method, int w, int h) {
  int b = 7 - method;
  while (sub_sample(w, b) * sub_sample(h, b) > VP8L_MAX_HUFF_IMAGE) ++b;
  return b < 2 ? 2 : b > 9 ? 9 : b;
}

int vp8l_transform_bits(int method, int hb) {
  const int mx = method < 4 ? 6 : method > 4 ? 4 : 5;
  return hb > mx ? mx : hb;
}

static const uint8_t kCodeToPlane[120] = {
  0x18, 0x07, 0x17, 0x19, 0x28, 0x06, 0x27, 0x29, 0x16, 0x1a,
  0x26, 0x2a, 0x38, 0x05, 0x37, 0x39, 0x15, 0x1b, 0x36, 0x3a,
  0x25, 0x2b, 0x48, 0x04, 0x47, 0x49, 0x14, 0x1c, 0x35, 0x3b,
  0x46, 0x4a, 0x24, 0x2c, 0x58, 0x45, 0x4b, 0x34, 0x3c, 0x03,
  0x57, 0x59, 0x13, 0x1d, 0x56, 0x5a, 0x23, 0x2d, 0x44, 0x4c,
  0x55, 0x5b, 0x33, 0x3d, 0x68, 0x02, 0x67, 0x69, 0x12, 0x1e,
  0x66, 0x6a, 0x22, 0x2e, 0x54, 0x5c, 0x43, 0x4d, 0x65, 0x6b,
  0x32, 0x3e, 0x78, 0x01, 0x77, 0x79, 0x53, 0x5d, 0x11, 0x1f,
  0x64, 0x6c, 0x42, 0x4e, 0x76, 0x7a, 0x21, 0x2f, 0x75, 0x7b,
  0x31, 0x3f, 0x63, 0x6d, 0x52, 0x5e, 0x00, 0x74, 0x7c, 0x41,
  0x4f, 0x10, 0x20, 0x62, 0x6e, 0x30, 0x73, 0x7d, 0x51, 0x5f,
  0x40, 0x72, 0x7e, 0x61, 0x6f, 0x50, 0x71, 0x7f, 0x60, 0x70};

/* src/dec/vp8l_dec.c:176-186 */
static int plane_code_to_distance(int w, int code) {
  if (code > 120) return code - 120;
  const int dc = kCodeToPlane[code - 1];
  const int d = (dc >> 4) * w + 8 - (dc & 0xf);
  return d >= 1 ? d : 1;
}

static int distance_code(int w, int d) {
  for (int c = 1; c <= 120; ++c)
    if (plane_code_to_distance(w, c) == d) return c;
  return d + 120;
}

void vp8l_setup_params(vp8l_params* p, int w, int h, int n, int method, int alpha) {
  memset(p, 0, sizeof(*p));
  p->w = w; p->h = h; p->n = n;
  p->alpha = alpha != 0;
  p->exact = alpha != 0;   /* the ALPH encoder sets exact (alpha_enc.c:66-72) */
  p->low_effort = method == 0;   /* the ALPH encoder passes its effort as the method (alpha_enc.c:76) */
  p->cache_bits = alpha ? 0 : VP8L_MAX_CACHE_BITS;
  p->ow = w;
  p->hb = vp8l_histo_bits(method, w, h);
  p->tb = vp8l_transform_bits(method, p->hb);
  const int nht = sub_sample(w, p->hb) * sub_sample(h, p->hb);
  p->k = nht < VP8L_KMAX ? nht : VP8L_KMAX;
  const int cand[4] = {w, 1, w + 1, w - 1};
  int nc = 0;
  for (int i = 0; i < 4; ++i) {
    const int d = cand[i];
    int dup = d < 1;
    for (int j = 0; j < nc; ++j) dup |= p->dist[j] == d;
    if (dup) continue;
    p->dist[nc] = d;
    p->dcode[nc] = distance_code(w, d);
    ++nc;
  }
}

/* distance -> smallest plane code for every distance a plane code reaches
 * (model: distance_code); returns the table size (largest such distance + 1) */
int vp8l_plane_dcodes(int w, uint8_t* tab) {
  int nd = 0;
  for (int c = 1; c <= 120; ++c) {
    const int d = plane_code_to_distance(w, c);
    if (d + 1 > nd) nd = d + 1;
  }
  if (!tab) return nd;
  memset(tab, 0, (size_t)nd);
  for (int c = 1; c <= 120; ++c) {
    const int d = plane_code_to_distance(w, c);
    if (!tab[d]) tab[d] = (uint8_t)c;
  }
  return nd;
}

/* the shortest-path parse's candidate distances (model: dp_candidates): the
 * first VP8L_DP_NC distinct plane-code distances >= 1 for width w, each as
 * {distance, rows up, columns left, distance code} with the distance =
 * rows * w + columns and |columns| <= w / 2 (the kernel's source pixel is
 * the flat index p - distance, wrapping across a row end at most once).
 * Returns the count. */
int vp8l_dp_candidates(int w, int32_t* out) {
  int n = 0;
  for (int code = 1; code <= 120 && n < VP8L_DP_NC; ++code) {
    const int d = plane_code_to_distance(w, code);
    int dup = d < 1;
    for (int i = 0; i < n; ++i) dup |= out[4 * i] == d;
    if (dup) continue;
    const int dy = (d + w / 2) / w;
    out[4 * n + 0] = d;
    out[4 * n + 1] = dy;
    out[4 * n + 2] = d - dy * w;
    out[4 * n + 3] = distance_code(w, d);
    ++n;
  }
  return n;
}

/* the colour-indexing engine: coded width = bundled width, tile bits from
 * GetHistoBits with use_palette on the picture size (vp8l_enc.c:234-245) */
/* histogram bits of a picture whose colours fit a palette (GetHistoBits
 * with use_palette, src/enc/vp8l_enc.c:234-245): EncoderAnalyze sets them
 * (:295-300) whatever entropy mode the frame then takes */
int vp8l_histo_bits_palette(int method, int w, int h) {
  int b = 9 - method;
  while (sub_sample(w, b) * sub_sample(h, b) > VP8L_MAX_HUFF_IMAGE) ++b;
  return b < 2 ? 2 : b > 9 ? 9 : b;
}

/* the spatial / direct engine for frames whose colours fit a palette */
void vp8l_setup_params_palette_hb(vp8l_params* p, int w, int h, int n, int method, int alpha) {
  vp8l_setup_params(p, w, h, n, method, alpha);
  p->hb = vp8l_histo_bits_palette(method, w, h);
  p->tb = vp8l_transform_bits(method, p->hb);
  const int nht = sub_sample(w, p->hb) * sub_sample(h, p->hb);
  p->k = nht < VP8L_KMAX ? nht : VP8L_KMAX;
}

void vp8l_setup_palette_params(vp8l_params* p, int w, int h, int n, int method, int xbits,
                               int alpha) {
  const int pw = sub_sample(w, xbits);
  vp8l_setup_params(p, pw, h, n, method, alpha);
  p->palette = 1;
  p->xbits = xbits;
  p->ow = w;
  p->hb = vp8l_histo_bits_palette(method, w, h);
  p->tb = 2;   /* unused: no predictor */
  const int nht = sub_sample(pw, p->hb) * sub_sample(h, p->hb);
  /* at most VP8L_KMAX_PALETTE code groups (model: KMAX_PALETTE) */
  p->k = nht < VP8L_KMAX_PALETTE ? nht : VP8L_KMAX_PALETTE;
}

static int32_t g_nlogn[4097];
static int32_t g_flog2[1024];
static float g_ftabs[512];   /* VP8LFastSLog2 / log2 of 0..255 as the reference's float tables */
static pthread_once_t g_tab_once = PTHREAD_ONCE_INIT;
static void tables_init(void) {
  /* kSLog2Table / kLog2Table (src/dsp/lossless_enc.c:28-224) are the float
   * roundings of v log2 v and log2 v (tests/test_vp8l.py checks all 512) */
  for (int v = 0; v < 256; ++v) {
    g_ftabs[v] = v < 2 ? 0.f : (float)(v * log2((double)v));
    g_ftabs[256 + v] = v < 2 ? 0.f : (float)log2((double)v);
  }
  g_nlogn[0] = g_nlogn[1] = 0;
  for (int n = 2; n <= 4096; ++n) g_nlogn[n] = (int32_t)floor(n * log2((double)n) * 4096 + 0.5);
  for (int m = 0; m < 1024; ++m) g_flog2[m] = (int32_t)floor(4096 * log2(1 + m / 1024.0) + 0.5);
}
const int32_t* vp8l_nlogn_table(void) { pthread_once(&g_tab_once, tables_init); return g_nlogn; }
const int32_t* vp8l_flog2_table(void) { pthread_once(&g_tab_once, tables_init); return g_flog2; }
const float* vp8l_float_tables(void) { pthread_once(&g_tab_once, tables_init); return g_ftabs; }

/* ---------------------------------------------------------------- analysis */

/* model: flog2 -- log2(v) in 1/4096 bit, v >= 1 */
static int64_t flog2_fx(uint64_t v) {
  const int32_t* frac = vp8l_flog2_table();
  int e = 63 - __builtin_clzll(v);
  const uint64_t m = (e >= 10 ? (v >> (e - 10)) : (v << (10 - e))) & 1023;
  return ((int64_t)e << 12) + frac[m];
}

/* model: bits_entropy_fx (VP8LBitsEntropy in fixed point) */
int64_t vp8l_bits_entropy_fx(const uint32_t* h, int n) {
  uint64_t s = 0, mx = 0;
  int nz = 0;
  int64_t sl = 0;
  for (int i = 0; i < n; ++i) {
    if (!h[i]) continue;
    s += h[i]; ++nz;
    if (h[i] > mx) mx = h[i];
    if (h[i] > 1) sl += (int64_t)h[i] * flog2_fx(h[i]);
  }
  if (nz <= 1) return 0;
  const int64_t S = (int64_t)s;
  const int64_t ent = (s > 1 ? S * flog2_fx(s) : 0) - sl;
  if (nz == 2) return (99 * S * 4096 + ent) / 100;
  const int64_t mix = nz == 3 ? 950 : nz == 4 ? 700 : 627;
  int64_t ml = (2 * S - (int64_t)mx) * 4096;
  ml = (mix * ml + (1000 - mix) * ent) / 1000;
  return ent < ml ? ml : ent;
}

/* model: entropy_choice (AnalyzeEntropy's estimates, vp8l_enc.c:158-201) */
int vp8l_entropy_choice(const uint32_t* ehist, int npal, int ntiles) {
  if (npal > 0 && npal <= 16) return VP8L_MODE_PALETTE;
  int64_t e[13];
  for (int i = 0; i < 13; ++i) e[i] = vp8l_bits_entropy_fx(ehist + 256 * i, 256);
  int64_t ent[5];
  ent[0] = e[0] + e[4] + e[2] + e[6];
  ent[1] = e[1] + e[5] + e[3] + e[7] + (int64_t)ntiles * flog2_fx(14);
  ent[2] = e[0] + e[8] + e[2] + e[10];
  ent[3] = e[1] + e[9] + e[3] + e[11] + (int64_t)ntiles * flog2_fx(24);
  ent[4] = e[12] + (int64_t)npal * 8 * 4096;
  const int last = npal > 0 ? VP8L_MODE_PALETTE : VP8L_MODE_SPATIAL_SUBGREEN;
  int best = 0;
  for (int k = 1; k <= last; ++k)
    if (ent[best] > ent[k]) best = k;
  return best;
}

static uint32_t sub_pixels(uint32_t a, uint32_t b) {
  const uint32_t ag = (a | 0x00ff00ffu) - (b & 0xff00ff00u);
  const uint32_t rb = (a | 0xff00ff00u) - (b & 0x00ff00ffu);
  return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}

static int u32_cmp(const void* a, const void* b) {
  const uint32_t x = *(const uint32_t*)a, y = *(const uint32_t*)b;
  return x < y ? -1 : x > y;
}

static uint32_t comp_dist(uint32_t v) { return v <= 128 ? v : 256 - v; }

/* model: minimize_deltas -- sort ascending (GetColorPalette), then
 * PaletteSortMinimizeDeltas (src/utils/palette.c:155-207) in place */
void vp8l_palette_order(uint32_t* pal, int n) {
  qsort(pal, (size_t)n, sizeof(*pal), u32_cmp);
  uint32_t pred = 0;
  unsigned sign = 0;
  for (int i = 0; i < n; ++i) {
    const uint32_t d = sub_pixels(pal[i], pred);
    const uint32_t rd = (d >> 16) & 255, gd = (d >> 8) & 255, bd = d & 255;
    if (rd) sign |= rd < 0x80 ? 1 : 2;
    if (gd) sign |= gd < 0x80 ? 8 : 16;
    if (bd) sign |= bd < 0x80 ? 64 : 128;
    pred = pal[i];
  }
  if (!(sign & (sign << 1))) return;
  pred = 0;
  for (int i = 0; i < n; ++i) {
    int best_ix = i;
    uint32_t best = ~0u;
    for (int k = i; k < n; ++k) {
      const uint32_t d = sub_pixels(pal[k], pred);
      const uint32_t sc = 9 * (comp_dist(d & 255) + comp_dist((d >> 8) & 255) +
                               comp_dist((d >> 16) & 255)) + comp_dist(d >> 24);
      if (best > sc) { best = sc; best_ix = k; }
    }
    const uint32_t t = pal[best_ix]; pal[best_ix] = pal[i]; pal[i] = t;
    pred = pal[i];
  }
}

/* ---------------------------------------------------------------- Huffman */

/* leaves sorted by (weight, symbol): LSD radix sort of packed 64-bit keys
 * weight << 12 | symbol, one 8-bit digit per pass up to the largest weight
 * (the headers build ~200 codes per frame; qsort and its comparator calls
 * were most of the host header time) */
static void sort_keys(uint64_t* k, uint64_t* tmp, int n) {
  if (n <= 48) {   /* insertion sort: cheaper than 256-bucket passes here */
    for (int i = 1; i < n; ++i) {
      const uint64_t v = k[i];
      int j = i - 1;
      while (j >= 0 && k[j] > v) { k[j + 1] = k[j]; --j; }
      k[j + 1] = v;
    }
    return;
  }
  uint64_t mx = 0;
  for (int i = 0; i < n; ++i) mx |= k[i];
  for (int sh = 0; sh < 64 && (mx >> sh); sh += 8) {
    uint32_t cnt[257] = {0};
    for (int i = 0; i < n; ++i) cnt[((k[i] >> sh) & 255) + 1]++;
    if (cnt[((k[0] >> sh) & 255) + 1] == (uint32_t)n) continue;   /* one digit value: no-op */
    for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
    for (int i = 0; i < n; ++i) tmp[cnt[(k[i] >> sh) & 255]++] = k[i];
    memcpy(k, tmp, sizeof(uint64_t) * (size_t)n);
  }
}

#define HUFF_MAX_SYMS (VP8L_GS > 280 ? VP8L_GS : 280)

/* model: huffman_lengths -- two-queue Huffman on (max(count, count_min),
 * symbol)-sorted leaves, count_min doubling until the depth fits. */
static int huffman_lengths(const uint32_t* hist, int n, int limit, uint8_t* len) {
  memset(len, 0, (size_t)n);
  int nu = 0, last = -1;
  for (int s = 0; s < n; ++s)
    if (hist[s]) { ++nu; last = s; }
  if (nu == 0) return 1;
  if (nu == 1) { len[last] = 1; return 1; }
  if (n > HUFF_MAX_SYMS) return 0;
  uint64_t lv[HUFF_MAX_SYMS], tmp[HUFF_MAX_SYMS], iw[HUFF_MAX_SYMS];
  int lpar[HUFF_MAX_SYMS], ipar[HUFF_MAX_SYMS], idep[HUFF_MAX_SYMS];
  for (uint64_t cmin = 1;; cmin *= 2) {
    int k = 0;
    for (int s = 0; s < n; ++s)
      if (hist[s]) lv[k++] = ((hist[s] > cmin ? (uint64_t)hist[s] : cmin) << 12) | (uint64_t)s;
    sort_keys(lv, tmp, nu);
    int i1 = 0, i2 = 0, n2 = 0;
    while ((nu - i1) + (n2 - i2) > 1) {
      int node[2];
      uint64_t wsum = 0;
      for (int t = 0; t < 2; ++t) {
        if (i2 >= n2 || (i1 < nu && (lv[i1] >> 12) <= iw[i2])) {
          wsum += lv[i1] >> 12; node[t] = i1++;
        } else {
          wsum += iw[i2]; node[t] = -1 - i2++;
        }
      }
      for (int t = 0; t < 2; ++t) {
        if (node[t] >= 0) lpar[node[t]] = n2;
        else ipar[-1 - node[t]] = n2;
      }
      iw[n2++] = wsum;
    }
    idep[n2 - 1] = 0;
    for (int j = n2 - 2; j >= 0; --j) idep[j] = idep[ipar[j]] + 1;
    int mx = 0;
    for (int j = 0; j < nu; ++j) {
      const int d = idep[lpar[j]] + 1;
      len[lv[j] & 4095] = (uint8_t)d;
      if (d > mx) mx = d;
    }
    if (mx <= limit) break;
  }
  return 1;
}

static const uint8_t* rev8_table(void) {
  static uint8_t t[256];
  static int done = 0;
  if (!done) {   /* benign race: every thread writes the same bytes */
    for (int i = 0; i < 256; ++i) {
      int r = 0;
      for (int b = 0; b < 8; ++b) r |= ((i >> b) & 1) << (7 - b);
      t[i] = (uint8_t)r;
    }
    __atomic_store_n(&done, 1, __ATOMIC_RELEASE);
  }
  return t;
}

/* model: canonical_codes (deflate order, bit-reversed for LSB-first) */
static void canonical_codes(const uint8_t* len, int n, uint16_t* codes) {
  const uint8_t* rv = rev8_table();
  int bl[17] = {0}, next[17] = {0};
  for (int s = 0; s < n; ++s) bl[len[s]]++;
  bl[0] = 0;
  int code = 0;
  for (int b = 1; b <= 16; ++b) {
    code = (code + bl[b - 1]) << 1;
    next[b] = code;
  }
  for (int s = 0; s < n; ++s) {
    codes[s] = 0;
    if (!len[s]) continue;
    const uint32_t c = (uint32_t)next[len[s]]++;
    const uint32_t r16 = ((uint32_t)rv[c & 255] << 8) | rv[(c >> 8) & 255];
    codes[s] = (uint16_t)(r16 >> (16 - len[s]));
  }
}

#define MAX_ALPH VP8L_GS

typedef struct {
  int n;                 /* alphabet size */
  int nused, used0, used1;
  uint8_t len[MAX_ALPH];
  uint8_t wlen[MAX_ALPH];
  uint16_t codes[MAX_ALPH];
} Code;

/* model: Code.__init__ */
static int code_build(Code* c, const uint32_t* hist, int n) {
  c->n = n;
  c->nused = 0; c->used0 = c->used1 = 0;
  for (int s = 0; s < n; ++s)
    if (hist[s]) {
      if (c->nused == 0) c->used0 = s;
      else if (c->nused == 1) c->used1 = s;
      ++c->nused;
    }
  if (!huffman_lengths(hist, n, 15, c->len)) return 0;
  canonical_codes(c->len, n, c->codes);
  if (c->nused <= 1) memset(c->wlen, 0, (size_t)n);
  else memcpy(c->wlen, c->len, (size_t)n);
  return 1;
}

static const uint8_t kStorageOrder[19] = {17, 18, 0, 1, 2, 3, 4, 5, 16, 6, 7, 8, 9, 10, 11,
                                          12, 13, 14, 15};

/* model: code_length_tokens */
static int cl_tokens(const uint8_t* len, int n, uint8_t* tc, uint8_t* te) {
  int k = 0, i = 0;
  while (i < n) {
    const int v = len[i];
    int j = i;
    while (j < n && len[j] == v) ++j;
    int run = j - i;
    if (v == 0) {
      while (run > 0) {
        if (run < 3) {
          for (; run > 0; --run) { tc[k] = 0; te[k++] = 0; }
        } else if (run <= 10) {
          tc[k] = 17; te[k++] = (uint8_t)(run - 3); run = 0;
        } else {
          const int r = run < 138 ? run : 138;
          tc[k] = 18; te[k++] = (uint8_t)(r - 11); run -= r;
        }
      }
    } else {
      tc[k] = (uint8_t)v; te[k++] = 0; --run;
      while (run > 0) {
        if (run < 3) {
          for (; run > 0; --run) { tc[k] = (uint8_t)v; te[k++] = 0; }
        } else {
          const int r = run < 6 ? run : 6;
          tc[k] = 16; te[k++] = (uint8_t)(r - 3); run -= r;
        }
      }
    }
    i = j;
  }
  return k;
}

/* model: Code.store */
static void code_store(const Code* c, vp8l_bw* bw) {
  if (c->nused == 0) {
    vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, 0, 1); vp8l_bw_put(bw, 0, 1); vp8l_bw_put(bw, 0, 1);
    return;
  }
  const int maxu = c->nused == 1 ? c->used0 : c->used1;
  if (c->nused <= 2 && maxu < 256) {
    vp8l_bw_put(bw, 1, 1);
    vp8l_bw_put(bw, (uint32_t)(c->nused - 1), 1);
    if (c->used0 <= 1) { vp8l_bw_put(bw, 0, 1); vp8l_bw_put(bw, (uint32_t)c->used0, 1); }
    else { vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, (uint32_t)c->used0, 8); }
    if (c->nused == 2) vp8l_bw_put(bw, (uint32_t)c->used1, 8);
    return;
  }
  vp8l_bw_put(bw, 0, 1);
  uint8_t tc[MAX_ALPH], te[MAX_ALPH];
  const int nt = cl_tokens(c->len, c->n, tc, te);
  uint32_t th[19] = {0};
  for (int i = 0; i < nt; ++i) th[tc[i]]++;
  uint8_t cl[19];
  uint16_t cc[19];
  huffman_lengths(th, 19, 7, cl);
  canonical_codes(cl, 19, cc);
  int ncodes = 19;
  while (ncodes > 4 && cl[kStorageOrder[ncodes - 1]] == 0) --ncodes;
  vp8l_bw_put(bw, (uint32_t)(ncodes - 4), 4);
  for (int i = 0; i < ncodes; ++i) vp8l_bw_put(bw, cl[kStorageOrder[i]], 3);
  int nz = 0;
  for (int i = 0; i < 19; ++i) nz += cl[i] != 0;
  const int single = nz <= 1;
  vp8l_bw_put(bw, 0, 1);   /* no max_symbol */
  for (int i = 0; i < nt; ++i) {
    if (!single) vp8l_bw_put(bw, cc[tc[i]], cl[tc[i]]);
    if (tc[i] == 16) vp8l_bw_put(bw, te[i], 2);
    else if (tc[i] == 17) vp8l_bw_put(bw, te[i], 3);
    else if (tc[i] == 18) vp8l_bw_put(bw, te[i], 7);
  }
}

static void code_put(const Code* c, vp8l_bw* bw, int s) { vp8l_bw_put(bw, c->codes[s], c->wlen[s]); }

/* model: write_sub_image -- level > 0 image, no cache, literals only */
static int write_sub_image(vp8l_bw* bw, const uint32_t* pix, int n) {
  uint32_t* h = (uint32_t*)calloc(280 + 3 * 256 + 40, sizeof(uint32_t));
  Code* c = (Code*)malloc(5 * sizeof(Code));
  if (!h || !c) { free(h); free(c); return 0; }
  uint32_t* hg = h; uint32_t* hr = h + 280; uint32_t* hbl = hr + 256; uint32_t* ha = hbl + 256;
  uint32_t* hd = ha + 256;
  for (int i = 0; i < n; ++i) {
    hg[(pix[i] >> 8) & 255]++; hr[(pix[i] >> 16) & 255]++;
    hbl[pix[i] & 255]++; ha[pix[i] >> 24]++;
  }
  int ok = code_build(&c[0], hg, 280) && code_build(&c[1], hr, 256) &&
           code_build(&c[2], hbl, 256) && code_build(&c[3], ha, 256) && code_build(&c[4], hd, 40);
  if (ok) {
    vp8l_bw_put(bw, 0, 1);   /* no colour cache */
    for (int k = 0; k < 5; ++k) code_store(&c[k], bw);
    for (int i = 0; i < n; ++i) {
      code_put(&c[0], bw, (pix[i] >> 8) & 255); code_put(&c[1], bw, (pix[i] >> 16) & 255);
      code_put(&c[2], bw, pix[i] & 255); code_put(&c[3], bw, pix[i] >> 24);
    }
  }
  free(h); free(c);
  return ok;
}

/* ---------------------------------------------------------------- header */

static const int kAlphOff[5] = {0, VP8L_GS, VP8L_GS + 256, VP8L_GS + 512, VP8L_GS + 768};
static const int kAlphSize[5] = {VP8L_GS, 256, 256, 256, 40};

static uint64_t data_bits(const Code* g, const uint32_t* h) {
  uint64_t b = 0;
  for (int a = 0; a < 5; ++a)
    for (int s = 0; s < g[a].n; ++s) b += (uint64_t)h[kAlphOff[a] + s] * g[a].wlen[s];
  return b;
}

/* model: encode() from the cluster histograms on */
int vp8l_build_header(const vp8l_params* p, int has_alpha, int emode, int cache_bits,
                      const uint32_t* palette, int npal, const uint8_t* modes,
                      const uint32_t* mult, const uint32_t* hc, const uint8_t* assign,
                      vp8l_bw* bw, uint32_t* ctab, uint8_t* gtile) {
  const int W = p->w, H = p->h, tb = p->tb, hb = p->hb;
  const int ntt = p->palette ? (npal > 0 ? npal : 1) : sub_sample(W, tb) * sub_sample(H, tb);
  const int nht = sub_sample(W, hb) * sub_sample(H, hb);
  int ok = 1;
  int remap[VP8L_KMAX], used[VP8L_KMAX], ng = 0;
  for (int k = 0; k < VP8L_KMAX; ++k) remap[k] = -1;
  for (int t = 0; t < nht; ++t) remap[assign[t]] = 0;
  for (int k = 0; k < VP8L_KMAX; ++k)
    if (remap[k] == 0) { remap[k] = ng; used[ng++] = k; }
  uint32_t* tot = (uint32_t*)calloc(VP8L_NS, sizeof(uint32_t));
  uint32_t* pix = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(ntt > nht ? ntt : nht));
  if (p->palette && (npal < 1 || npal > VP8L_MAX_PALETTE || !palette)) ok = 0;
  Code* groups = (Code*)malloc(sizeof(Code) * 5 * (size_t)(ng + 1));
  if (!tot || !pix || !groups) { ok = 0; goto done; }
  for (int g = 0; g < ng; ++g)
    for (int i = 0; i < VP8L_NS; ++i) tot[i] += hc[(size_t)used[g] * VP8L_NS + i];
  /* the green alphabet has no cache symbols without a colour cache */
  int asize[5];
  for (int a = 0; a < 5; ++a) asize[a] = kAlphSize[a];
  asize[0] = 256 + 24 + (cache_bits ? 1 << cache_bits : 0);
  Code* single = groups + 5 * ng;
  for (int a = 0; a < 5; ++a) ok &= code_build(&single[a], tot + kAlphOff[a], asize[a]);
  for (int g = 0; g < ng; ++g)
    for (int a = 0; a < 5; ++a)
      ok &= code_build(&groups[5 * g + a], hc + (size_t)used[g] * VP8L_NS + kAlphOff[a],
                       asize[a]);
  if (!ok) goto done;
  for (int t = 0; t < nht; ++t) pix[t] = (uint32_t)remap[assign[t]] << 8;
  int meta = 0;
  if (ng > 1) {   /* model: cost(...) -- exact bits with headers */
    vp8l_bw tmp;
    vp8l_bw_init(&tmp, 1 << 16);
    vp8l_bw_put(&tmp, 1, 1); vp8l_bw_put(&tmp, (uint32_t)(hb - 2), 3);
    ok &= write_sub_image(&tmp, pix, nht);
    uint64_t cm = 0;
    for (int g = 0; g < ng; ++g) {
      for (int a = 0; a < 5; ++a) code_store(&groups[5 * g + a], &tmp);
      cm += data_bits(&groups[5 * g], hc + (size_t)used[g] * VP8L_NS);
    }
    cm += tmp.nbits;
    vp8l_bw_free(&tmp);
    vp8l_bw_init(&tmp, 1 << 14);
    for (int a = 0; a < 5; ++a) code_store(&single[a], &tmp);
    const uint64_t cs = tmp.nbits + data_bits(single, tot);
    ok &= !tmp.oom;
    vp8l_bw_free(&tmp);
    meta = cm < cs;
  }
  /* image header + transforms; the ALPH form has no image header */
  if (!p->alpha) {
    vp8l_bw_put(bw, 0x2f, 8);
    vp8l_bw_put(bw, (uint32_t)((p->palette ? p->ow : W) - 1), 14);
    vp8l_bw_put(bw, (uint32_t)(H - 1), 14);
    vp8l_bw_put(bw, has_alpha ? 1 : 0, 1);
    vp8l_bw_put(bw, 0, 3);
  }
  if (p->palette) {   /* COLOR_INDEXING, delta-coded palette (vp8l_enc.c:1412-1430) */
    vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, 3, 2); vp8l_bw_put(bw, (uint32_t)(npal - 1), 8);
    for (int i = npal - 1; i >= 1; --i) pix[i] = sub_pixels(palette[i], palette[i - 1]);
    pix[0] = palette[0];
    ok &= write_sub_image(bw, pix, npal);
  } else {
    if (emode & VP8L_MODE_SUBGREEN) { vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, 2, 2); }
    if (emode & VP8L_MODE_SPATIAL) {
      vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, 0, 2); vp8l_bw_put(bw, (uint32_t)(tb - 2), 3);
      for (int t = 0; t < ntt; ++t) pix[t] = 0xff000000u | ((uint32_t)modes[t] << 8);
      ok &= write_sub_image(bw, pix, ntt);
      if (!p->low_effort) {   /* no cross colour at method 0 (vp8l_enc.c:1525-1526) */
        vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, 1, 2); vp8l_bw_put(bw, (uint32_t)(tb - 2), 3);
        for (int t = 0; t < ntt; ++t) pix[t] = 0xff000000u | (mult[t] & 0xffffffu);
        ok &= write_sub_image(bw, pix, ntt);
      }
    }
  }
  vp8l_bw_put(bw, 0, 1);
  if (cache_bits) {
    vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, (uint32_t)cache_bits, 4);
  } else {
    vp8l_bw_put(bw, 0, 1);
  }
  if (meta) {
    vp8l_bw_put(bw, 1, 1); vp8l_bw_put(bw, (uint32_t)(hb - 2), 3);
    for (int t = 0; t < nht; ++t) pix[t] = (uint32_t)remap[assign[t]] << 8;
    ok &= write_sub_image(bw, pix, nht);
  } else {
    vp8l_bw_put(bw, 0, 1);
  }
  const int nout = meta ? ng : 1;
  for (int g = 0; g < nout; ++g) {
    const Code* gc = meta ? &groups[5 * g] : single;
    for (int a = 0; a < 5; ++a) {
      code_store(&gc[a], bw);
      for (int s = 0; s < asize[a]; ++s)
        ctab[(size_t)g * VP8L_NS + kAlphOff[a] + s] =
            (uint32_t)gc[a].codes[s] | ((uint32_t)gc[a].wlen[s] << 16);
    }
  }
  for (int t = 0; t < nht; ++t) gtile[t] = meta ? (uint8_t)remap[assign[t]] : 0;
  ok &= !bw->oom;
done:
  free(tot); free(pix); free(groups);
  return ok;
}

static void put_le32(uint8_t* d, uint32_t v) {
  d[0] = (uint8_t)v; d[1] = (uint8_t)(v >> 8); d[2] = (uint8_t)(v >> 16); d[3] = (uint8_t)(v >> 24);
}

void vp8l_riff_header(uint8_t out[20], size_t size) {
  const size_t pad = size & 1;
  memcpy(out, "RIFF", 4);
  put_le32(out + 4, (uint32_t)(4 + 8 + size + pad));
  memcpy(out + 8, "WEBPVP8L", 8);
  put_le32(out + 16, (uint32_t)size);
}
