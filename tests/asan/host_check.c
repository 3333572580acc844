/* Host-code sanitizer driver (-fsanitize=address,undefined
 * on the host C). Built by `make -C libwebp_amd/csrc asan` together with every
 * HIP-free host source of the product (picture_enc.c, picture_tools.c,
 * vp8_host.c, vp8l_host.c) and the oracle / own decoder, then run by
 * tests/test_asan.py. It walks the host paths over random sizes and
 * configurations: config presets and validation, picture allocation, copy,
 * view, crop, rescale, distortion, YUVA->ARGB, transparent-area cleanup and
 * alpha blending; frame setup, segment analysis and probability finalisation
 * of the lossy host code; VP8L parameters, headers and Huffman codes from
 * random statistics; the oracle encoder and the own decoder end to end.
 * Any sanitizer report aborts with a non-zero exit. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../libwebp_amd/csrc/host/vp8_host.h"
#include "../../libwebp_amd/csrc/host/vp8l_host.h"
#include "../../oracle/vp8_oracle.h"
#include "webp/encode.h"

int odec_info(const uint8_t* data, size_t size, int* w, int* h, int* has_alpha, int* lossless);
int odec_decode_rgba(const uint8_t* data, size_t size, uint8_t* out);
int odec_decode_yuv(const uint8_t* data, size_t size, uint8_t* y, uint8_t* u, uint8_t* v);

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd(void) {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return (uint32_t)(g_rng >> 11);
}
static int rnd_in(int lo, int hi) { return lo + (int)(rnd() % (uint32_t)(hi - lo + 1)); }

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      fprintf(stderr, "host_check: %s failed at line %d\n", #c, __LINE__); \
      exit(2);                                                           \
    }                                                                    \
  } while (0)

static void fill_argb(WebPPicture* p, int opaque) {
  for (int y = 0; y < p->height; ++y)
    for (int x = 0; x < p->width; ++x) {
      uint32_t v = rnd();
      if (opaque) v |= 0xff000000u;
      p->argb[y * p->argb_stride + x] = v;
    }
}

static void picture_paths(void) {
  for (int it = 0; it < 40; ++it) {
    WebPPicture a, b, v;
    CHECK(WebPPictureInitInternal(&a, WEBP_ENCODER_ABI_VERSION));
    CHECK(WebPPictureInitInternal(&b, WEBP_ENCODER_ABI_VERSION));
    CHECK(WebPPictureInitInternal(&v, WEBP_ENCODER_ABI_VERSION));
    a.width = rnd_in(1, 97);
    a.height = rnd_in(1, 83);
    a.use_argb = 1;
    CHECK(WebPPictureAlloc(&a));
    fill_argb(&a, it & 1);
    CHECK(WebPPictureCopy(&a, &b));
    const int cw = rnd_in(1, a.width), ch = rnd_in(1, a.height);
    const int cx = rnd_in(0, a.width - cw), cy = rnd_in(0, a.height - ch);
    CHECK(WebPPictureView(&a, cx, cy, cw, ch, &v));
    CHECK(WebPPictureIsView(&v));
    float d[5];
    CHECK(WebPPictureDistortion(&a, &b, it % 3, d));
    CHECK(WebPPictureCrop(&b, cx, cy, cw, ch));
    CHECK(WebPPictureRescale(&b, rnd_in(1, 120), rnd_in(1, 90)));
    WebPBlendAlpha(&b, rnd() & 0xffffff);
    WebPCleanupTransparentArea(&a);
    (void)WebPPictureHasTransparency(&a);
    /* YUVA container: rescale, cleanup and back to ARGB */
    WebPPicture y;
    CHECK(WebPPictureInitInternal(&y, WEBP_ENCODER_ABI_VERSION));
    y.width = a.width;
    y.height = a.height;
    y.colorspace = (it & 2) ? WEBP_YUV420A : WEBP_YUV420;
    CHECK(WebPPictureAlloc(&y));
    const int uvw = (y.width + 1) / 2, uvh = (y.height + 1) / 2;
    for (int j = 0; j < y.height; ++j)
      for (int i = 0; i < y.width; ++i) y.y[j * y.y_stride + i] = (uint8_t)rnd();
    for (int j = 0; j < uvh; ++j)
      for (int i = 0; i < uvw; ++i) {
        y.u[j * y.uv_stride + i] = (uint8_t)rnd();
        y.v[j * y.uv_stride + i] = (uint8_t)rnd();
      }
    if (y.a)
      for (int j = 0; j < y.height; ++j)
        for (int i = 0; i < y.width; ++i) y.a[j * y.a_stride + i] = (uint8_t)rnd();
    float dy[5];
    CHECK(WebPPictureDistortion(&y, &y, 0, dy));
    WebPCleanupTransparentArea(&y);
    CHECK(WebPPictureRescale(&y, rnd_in(1, 64), rnd_in(1, 64)));
    CHECK(WebPPictureYUVAToARGB(&y));
    WebPPictureFree(&y);
    WebPPictureFree(&v);
    WebPPictureFree(&b);
    WebPPictureFree(&a);
  }
  for (int preset = 0; preset <= WEBP_PRESET_TEXT; ++preset) {
    WebPConfig c;
    CHECK(WebPConfigInitInternal(&c, (WebPPreset)preset, (float)rnd_in(0, 100),
                                 WEBP_ENCODER_ABI_VERSION));
    CHECK(WebPValidateConfig(&c));
    CHECK(WebPConfigLosslessPreset(&c, rnd_in(0, 9)));
  }
  WebPMemoryWriter w;
  WebPMemoryWriterInit(&w);
  WebPPicture p;
  CHECK(WebPPictureInitInternal(&p, WEBP_ENCODER_ABI_VERSION));
  p.custom_ptr = &w;
  uint8_t chunk[3000];
  for (int i = 0; i < 50; ++i) CHECK(WebPMemoryWrite(chunk, (size_t)rnd_in(0, 3000), &p));
  WebPMemoryWriterClear(&w);
}

static void lossy_host_paths(void) {
  for (int it = 0; it < 30; ++it) {
    WebPConfig c;
    CHECK(WebPConfigInitInternal(&c, WEBP_PRESET_DEFAULT, (float)rnd_in(0, 100),
                                 WEBP_ENCODER_ABI_VERSION));
    c.method = rnd_in(0, 6);
    c.segments = rnd_in(1, 4);
    c.sns_strength = rnd_in(0, 100);
    c.filter_strength = rnd_in(0, 100);
    c.filter_sharpness = rnd_in(0, 7);
    c.preprocessing = rnd_in(0, 1);
    const int w = rnd_in(1, 300), h = rnd_in(1, 300);
    vp8h_frame fr;
    if (!vp8h_frame_init(&fr, &c, w, h)) continue;
    const int nmb = ((w + 15) >> 4) * ((h + 15) >> 4);
    uint8_t* alpha = (uint8_t*)malloc((size_t)nmb);
    uint16_t* uva = (uint16_t*)malloc((size_t)nmb * 2);
    uint8_t* segmap = (uint8_t*)malloc((size_t)nmb);
    for (int i = 0; i < nmb; ++i) {
      alpha[i] = (uint8_t)rnd();
      uva[i] = (uint16_t)rnd();
    }
    vp8g_frame_params params;
    vp8h_setup_segments(&fr, alpha, uva, segmap, &params);
    uint32_t stats[VP8G_NUM_SLOTS];
    uint8_t coeffs[VP8G_NUM_SLOTS];
    for (int i = 0; i < VP8G_NUM_SLOTS; ++i) {   /* (total << 16) | hits, hits <= total */
      const uint32_t total = rnd() % 0xffffu, hits = total ? rnd() % (total + 1) : 0;
      stats[i] = (total << 16) | hits;
    }
    int dirty = 0;
    (void)vp8h_finalize_probas(stats, coeffs, &dirty);
    free(alpha);
    free(uva);
    free(segmap);
  }
}

static void lossless_host_paths(void) {
  for (int it = 0; it < 24; ++it) {
    const int w = rnd_in(1, 200), h = rnd_in(1, 200);
    const int pal_engine = (it % 3) == 2;
    const int npal = rnd_in(1, VP8L_MAX_PALETTE);
    const int xb = npal <= 2 ? 3 : npal <= 4 ? 2 : npal <= 16 ? 1 : 0;
    vp8l_params p;
    if (pal_engine) vp8l_setup_palette_params(&p, w, h, 1, rnd_in(0, 6), xb, it & 1);
    else vp8l_setup_params(&p, w, h, 1, rnd_in(0, 6), it & 1);
    const int ntt = ((p.w + (1 << p.tb) - 1) >> p.tb) * ((h + (1 << p.tb) - 1) >> p.tb);
    const int nht = ((p.w + (1 << p.hb) - 1) >> p.hb) * ((h + (1 << p.hb) - 1) >> p.hb);
    uint8_t* modes = (uint8_t*)malloc((size_t)ntt);
    uint32_t* mult = (uint32_t*)malloc((size_t)ntt * 4);
    uint32_t* hc = (uint32_t*)calloc((size_t)VP8L_KMAX * VP8L_NS, 4);
    uint32_t* ctab = (uint32_t*)calloc((size_t)VP8L_KMAX * VP8L_NS, 4);
    uint8_t* assign = (uint8_t*)malloc((size_t)nht);
    uint8_t* gtile = (uint8_t*)malloc((size_t)nht);
    uint32_t pal[VP8L_MAX_PALETTE];
    uint32_t eh[VP8L_EHIST];
    for (int i = 0; i < npal; ++i) pal[i] = rnd() ^ ((uint32_t)i << 24);
    vp8l_palette_order(pal, npal);
    for (int i = 0; i < VP8L_EHIST; ++i) eh[i] = (rnd() & 3) ? 0 : rnd() & 0xfffff;
    const int emode = vp8l_entropy_choice(eh, (it & 4) ? npal : 0, ntt);
    CHECK(emode >= 0 && emode <= VP8L_MODE_PALETTE);
    const int k = rnd_in(1, VP8L_KMAX);
    const int cb = p.alpha ? 0 : rnd_in(0, VP8L_MAX_CACHE_BITS);   /* ALPH: no cache */
    for (int i = 0; i < ntt; ++i) { modes[i] = (uint8_t)rnd_in(0, 13); mult[i] = rnd() & 0xffffff; }
    for (int i = 0; i < nht; ++i) assign[i] = (uint8_t)rnd_in(0, k - 1);
    for (int i = 0; i < k * VP8L_NS; ++i) hc[i] = (rnd() & 7) ? 0 : rnd() & 0xffff;
    vp8l_bw bw;
    vp8l_bw_init(&bw, 1 << 12);
    CHECK(vp8l_build_header(&p, it & 2, pal_engine ? VP8L_MODE_PALETTE : rnd_in(0, 3), cb,
                            pal_engine ? pal : NULL, pal_engine ? npal : 0, modes, mult, hc,
                            assign, &bw, ctab, gtile));
    (void)vp8l_bw_finish(&bw);
    vp8l_bw_free(&bw);
    free(modes); free(mult); free(hc); free(ctab); free(assign); free(gtile);
  }
}

static void oracle_and_decoder(void) {
  for (int it = 0; it < 12; ++it) {
    const int w = rnd_in(1, 130), h = rnd_in(1, 130);
    uint8_t* rgba = (uint8_t*)malloc((size_t)w * h * 4);
    for (int i = 0; i < w * h; ++i) {
      const uint32_t v = rnd();
      memcpy(rgba + 4 * i, &v, 3);
      rgba[4 * i + 3] = 255;
    }
    vp8o_config cfg;
    vp8o_default_config(&cfg);
    cfg.quality = (float)rnd_in(0, 100);
    cfg.method = rnd_in(3, 6);
    cfg.segments = rnd_in(1, 4);
    cfg.filter_sharpness = rnd_in(0, 7);
    uint8_t* out = NULL;
    const size_t n = vp8o_encode_rgba(rgba, w, h, 4 * w, &cfg, &out);
    CHECK(n > 0 && out != NULL);
    int dw, dh, da, dl;
    CHECK(odec_info(out, n, &dw, &dh, &da, &dl) && dw == w && dh == h && !dl);
    uint8_t* dec = (uint8_t*)malloc((size_t)w * h * 4);
    CHECK(odec_decode_rgba(out, n, dec));
    uint8_t* yy = (uint8_t*)malloc((size_t)w * h);
    uint8_t* uu = (uint8_t*)malloc((size_t)((w + 1) / 2) * ((h + 1) / 2));
    uint8_t* vv = (uint8_t*)malloc((size_t)((w + 1) / 2) * ((h + 1) / 2));
    CHECK(odec_decode_yuv(out, n, yy, uu, vv));
    /* truncated and corrupted streams must fail or decode, never fault */
    (void)odec_decode_rgba(out, n / 2, dec);
    out[n / 3] ^= 0x5a;
    (void)odec_decode_rgba(out, n, dec);
    vp8o_free(out);
    free(dec); free(yy); free(uu); free(vv); free(rgba);
  }
}

int main(void) {
  picture_paths();
  lossy_host_paths();
  lossless_host_paths();
  oracle_and_decoder();
  printf("host_check: ok\n");
  return 0;
}
