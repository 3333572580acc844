/* Test infrastructure ONLY: a scalar CPU restatement of libwebp v1.3.2's
 * lossy (VP8) encode path, used by tests/ and bench.py's cpu_baseline leg as
 * the checker for the HIP product path. Never linked into libwebp_amd.
 * Every function in vp8_oracle.c cites the reference file:line it follows.
 * Pinned by the known-answer SHA-256s of SURVEY.md §8(d) and by the reference
 * build in oracle/_ref (tests/test_oracle.py). */
#ifndef VP8_ORACLE_H_
#define VP8_ORACLE_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  float quality;          /* 0..100 */
  int method;             /* 3..6 supported (token-buffer path) */
  int segments;           /* 1..4 */
  int sns_strength;       /* 0..100 */
  int filter_strength;    /* 0..100 */
  int filter_sharpness;   /* 0..7 */
  int filter_type;        /* 0 simple, 1 strong */
  int partition_limit;    /* 0..100 */
  int preprocessing;      /* bit0: segment smoothing */
  int emulate_jpeg_size;  /* 0/1 */
  int use_sharp_yuv;      /* 0/1: iterative RGB->YUV (sharp_oracle.c) */
  int pass;               /* 1..10 entropy passes */
  int target_size;        /* bytes, 0 = off */
  float target_PSNR;      /* dB, 0 = off */
  int qmin, qmax;         /* 0..100 */
  int autofilter;         /* 0/1: SSIM-driven per-segment filter levels */
  int low_memory;         /* 0/1: VP8EncLoop for methods 3-6 too */
  int partitions;         /* 0..3: 2^partitions token partitions (VP8EncLoop only) */
} vp8o_config;

/* per-macroblock decisions, for stage-by-stage comparison with the GPU */
typedef struct {
  uint8_t segment, type, uv_mode, skip;
  uint8_t modes[16];        /* i16: modes[0..15] all equal the i16 mode */
  uint8_t alpha;            /* analysis susceptibility (after k-means remap) */
  uint8_t pad[3];
  int16_t y_dc[16];
  int16_t y_ac[16][16];
  int16_t uv[8][16];
} vp8o_mb_trace;

void vp8o_default_config(vp8o_config* cfg);

/* RGBA -> YUV420 (ImportYUVAFromRGBA, opaque path). Returns 0 if the input
 * has non-opaque alpha (that path is not restated). */
int vp8o_import_rgba(const uint8_t* rgba, int w, int h, int stride,
                     uint8_t* y, uint8_t* u, uint8_t* v);

/* the dithered conversion (WebPPictureARGBToYUVADithered), opaque input */
int vp8o_import_rgba_dithered(const uint8_t* rgba, int w, int h, int stride, float dithering,
                              uint8_t* y, uint8_t* u, uint8_t* v);

/* Full lossy encode from YUV420 planes. Returns the .webp size (malloc'ed
 * into *out, free with vp8o_free) or 0 on error. trace may be NULL. */
size_t vp8o_encode_yuv(const uint8_t* y, const uint8_t* u, const uint8_t* v,
                       int w, int h, int y_stride, int uv_stride,
                       const vp8o_config* cfg, uint8_t** out,
                       vp8o_mb_trace* trace);

size_t vp8o_encode_rgba(const uint8_t* rgba, int w, int h, int stride,
                        const vp8o_config* cfg, uint8_t** out);

/* analysis only: per-MB alpha (pre-k-means) and the 256-bin histogram */
void vp8o_analyze(const uint8_t* y, const uint8_t* u, const uint8_t* v,
                  int w, int h, int y_stride, int uv_stride,
                  uint8_t* mb_alpha, int* uv_alpha_sum, int* histo256);

/* sharp (iterative) RGBA -> YUV420 (sharp_oracle.c; sharpyuv/sharpyuv.c).
 * Opaque input, width and height >= 4. */
int vp8o_sharp_import_rgba(const uint8_t* rgba, int w, int h, int stride,
                           uint8_t* y, uint8_t* u, uint8_t* v);
/* the sRGB gamma tables of the sharp path (either pointer may be NULL) */
void vp8o_sharp_tables(uint32_t g2l[1026], uint32_t l2g[514]);

void vp8o_free(void* p);
/* number of MB-loop passes of the last vp8o_encode_* call (> 1 when the
 * partition-0 overflow retry of frame_enc.c:869-876 ran) */
int vp8o_last_pass_count(void);
/* header-bit estimate of the last pass over the partition-0 limit */
double vp8o_last_p0_fraction(void);

#ifdef __cplusplus
}
#endif
#endif
