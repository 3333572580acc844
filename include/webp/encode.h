/* libwebp_amd -- libwebp-compatible encoder C ABI (encoder ABI 0x020f).
 *
 * Every declaration here replaces the one of the same name in the
 * reference's src/webp/encode.h (line numbers cited per item). Struct layouts
 * are byte-identical to the reference so that cwebp, img2webp, the mux
 * library and any other existing caller link against libwebp_amd.so without
 * recompiling; tests/test_abi.py checks sizes and offsets against the
 * reference build.
 *
 * Lossy encodes (config->lossless == 0, method 3..6) run on the MI355X: the
 * RGB->YUV import, macroblock analysis, rate-distortion mode search,
 * quantisation/reconstruction and token statistics are HIP kernels; the
 * boolean coder and bitstream assembly run in host C.
 * Unsupported configurations fail with VP8_ENC_ERROR_INVALID_CONFIGURATION.
 */
#ifndef WEBP_WEBP_ENCODE_H_
#define WEBP_WEBP_ENCODE_H_

#include "./types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define WEBP_ENCODER_ABI_VERSION 0x020f   /* ref encode.h:23 */

typedef struct WebPConfig WebPConfig;
typedef struct WebPPicture WebPPicture;
typedef struct WebPAuxStats WebPAuxStats;
typedef struct WebPMemoryWriter WebPMemoryWriter;

/* ref encode.h:38 -- (major << 16) | (minor << 8) | revision */
WEBP_EXTERN int WebPGetEncoderVersion(void);

/* One-shot lossy encoders, ref encode.h:46-57. Return the .webp size and a
 * WebPMalloc'ed buffer in *output (release with WebPFree), 0 on error. */
WEBP_EXTERN size_t WebPEncodeRGB(const uint8_t* rgb, int width, int height,
                                 int stride, float quality_factor,
                                 uint8_t** output);
WEBP_EXTERN size_t WebPEncodeBGR(const uint8_t* bgr, int width, int height,
                                 int stride, float quality_factor,
                                 uint8_t** output);
WEBP_EXTERN size_t WebPEncodeRGBA(const uint8_t* rgba, int width, int height,
                                  int stride, float quality_factor,
                                  uint8_t** output);
WEBP_EXTERN size_t WebPEncodeBGRA(const uint8_t* bgra, int width, int height,
                                  int stride, float quality_factor,
                                  uint8_t** output);

/* Lossless one-shot encoders, ref encode.h:67-78: the VP8L path is not part
 * of this build; these return 0. */
WEBP_EXTERN size_t WebPEncodeLosslessRGB(const uint8_t* rgb, int width,
                                         int height, int stride,
                                         uint8_t** output);
WEBP_EXTERN size_t WebPEncodeLosslessBGR(const uint8_t* bgr, int width,
                                         int height, int stride,
                                         uint8_t** output);
WEBP_EXTERN size_t WebPEncodeLosslessRGBA(const uint8_t* rgba, int width,
                                          int height, int stride,
                                          uint8_t** output);
WEBP_EXTERN size_t WebPEncodeLosslessBGRA(const uint8_t* bgra, int width,
                                          int height, int stride,
                                          uint8_t** output);

/* ref encode.h:86-92 */
typedef enum WebPImageHint {
  WEBP_HINT_DEFAULT = 0,
  WEBP_HINT_PICTURE,
  WEBP_HINT_PHOTO,
  WEBP_HINT_GRAPH,
  WEBP_HINT_LAST
} WebPImageHint;

/* Encoding parameters, ref encode.h:95-153 (field order is the ABI). */
struct WebPConfig {
  int lossless;           /* 0: lossy (VP8), 1: lossless (VP8L) */
  float quality;          /* [0..100] */
  int method;             /* speed/quality trade-off [0..6] */
  WebPImageHint image_hint;
  int target_size;        /* bytes; 0 = off */
  float target_PSNR;      /* dB; 0 = off */
  int segments;           /* [1..4] */
  int sns_strength;       /* spatial noise shaping [0..100] */
  int filter_strength;    /* [0..100] */
  int filter_sharpness;   /* [0..7] */
  int filter_type;        /* 0 simple, 1 strong */
  int autofilter;         /* 0/1 */
  int alpha_compression;
  int alpha_filtering;
  int alpha_quality;
  int pass;               /* entropy passes [1..10] */
  int show_compressed;
  int preprocessing;      /* bit0: segment smoothing, bit1: dithering */
  int partitions;         /* log2(token partitions) [0..3] */
  int partition_limit;    /* [0..100] */
  int emulate_jpeg_size;
  int thread_level;
  int low_memory;
  int near_lossless;
  int exact;
  int use_delta_palette;
  int use_sharp_yuv;
  int qmin;
  int qmax;
};

/* ref encode.h:157-164 */
typedef enum WebPPreset {
  WEBP_PRESET_DEFAULT = 0,
  WEBP_PRESET_PICTURE,
  WEBP_PRESET_PHOTO,
  WEBP_PRESET_DRAWING,
  WEBP_PRESET_ICON,
  WEBP_PRESET_TEXT
} WebPPreset;

/* ref encode.h:167 (internal; use the inline wrappers below) */
WEBP_EXTERN int WebPConfigInitInternal(WebPConfig*, WebPPreset, float, int);

/* ref encode.h:173-186 */
static WEBP_INLINE int WebPConfigInit(WebPConfig* config) {
  return WebPConfigInitInternal(config, WEBP_PRESET_DEFAULT, 75.f,
                                WEBP_ENCODER_ABI_VERSION);
}
static WEBP_INLINE int WebPConfigPreset(WebPConfig* config, WebPPreset preset,
                                 float quality) {
  return WebPConfigInitInternal(config, preset, quality,
                                WEBP_ENCODER_ABI_VERSION);
}

/* ref encode.h:194, :198 */
WEBP_EXTERN int WebPConfigLosslessPreset(WebPConfig* config, int level);
WEBP_EXTERN int WebPValidateConfig(const WebPConfig* config);

/* Encoder statistics, ref encode.h:204-232 (layout is the ABI). */
struct WebPAuxStats {
  int coded_size;
  float PSNR[5];              /* Y, U, V, all, alpha */
  int block_count[3];         /* intra4, intra16, skipped */
  int header_bytes[2];        /* partition-0 headers, modes */
  int residual_bytes[3][4];
  int segment_size[4];
  int segment_quant[4];
  int segment_level[4];
  int alpha_data_size;
  int layer_data_size;
  uint32_t lossless_features;
  int histogram_bits;
  int transform_bits;
  int cache_bits;
  int palette_size;
  int lossless_size;
  int lossless_hdr_size;
  int lossless_data_size;
  uint32_t pad[2];
};

/* ref encode.h:237-239 */
typedef int (*WebPWriterFunction)(const uint8_t* data, size_t data_size,
                                  const WebPPicture* picture);

/* Growable in-memory sink, ref encode.h:242-259. */
struct WebPMemoryWriter {
  uint8_t* mem;
  size_t size;
  size_t max_size;
  uint32_t pad[1];
};
WEBP_EXTERN void WebPMemoryWriterInit(WebPMemoryWriter* writer);
WEBP_EXTERN void WebPMemoryWriterClear(WebPMemoryWriter* writer);
WEBP_EXTERN int WebPMemoryWrite(const uint8_t* data, size_t data_size,
                                const WebPPicture* picture);

/* ref encode.h:264 */
typedef int (*WebPProgressHook)(int percent, const WebPPicture* picture);

/* ref encode.h:267-272 */
typedef enum WebPEncCSP {
  WEBP_YUV420 = 0,
  WEBP_YUV420A = 4,
  WEBP_CSP_UV_MASK = 3,
  WEBP_CSP_ALPHA_BIT = 4
} WebPEncCSP;

/* ref encode.h:276-289 */
typedef enum WebPEncodingError {
  VP8_ENC_OK = 0,
  VP8_ENC_ERROR_OUT_OF_MEMORY,
  VP8_ENC_ERROR_BITSTREAM_OUT_OF_MEMORY,
  VP8_ENC_ERROR_NULL_PARAMETER,
  VP8_ENC_ERROR_INVALID_CONFIGURATION,
  VP8_ENC_ERROR_BAD_DIMENSION,
  VP8_ENC_ERROR_PARTITION0_OVERFLOW,
  VP8_ENC_ERROR_PARTITION_OVERFLOW,
  VP8_ENC_ERROR_BAD_WRITE,
  VP8_ENC_ERROR_FILE_TOO_BIG,
  VP8_ENC_ERROR_USER_ABORT,
  VP8_ENC_ERROR_LAST
} WebPEncodingError;

#define WEBP_MAX_DIMENSION 16383   /* ref encode.h:292 */

/* Input picture, ref encode.h:300-364 (layout, padding included, is the
 * ABI; memory_ / memory_argb_ are private to the library). */
struct WebPPicture {
  int use_argb;
  WebPEncCSP colorspace;
  int width, height;
  uint8_t *y, *u, *v;
  int y_stride, uv_stride;
  uint8_t* a;
  int a_stride;
  uint32_t pad1[2];
  uint32_t* argb;
  int argb_stride;
  uint32_t pad2[3];
  WebPWriterFunction writer;
  void* custom_ptr;
  int extra_info_type;
  uint8_t* extra_info;
  WebPAuxStats* stats;
  WebPEncodingError error_code;
  WebPProgressHook progress_hook;
  void* user_data;
  uint32_t pad3[3];
  uint8_t *pad4, *pad5;
  uint32_t pad6[8];
  void* memory_;
  void* memory_argb_;
  void* pad7[2];
};

/* ref encode.h:367-375 */
WEBP_EXTERN int WebPPictureInitInternal(WebPPicture*, int);
static WEBP_INLINE int WebPPictureInit(WebPPicture* picture) {
  return WebPPictureInitInternal(picture, WEBP_ENCODER_ABI_VERSION);
}

/* Picture memory, ref encode.h:383-395 */
WEBP_EXTERN int WebPPictureAlloc(WebPPicture* picture);
WEBP_EXTERN void WebPPictureFree(WebPPicture* picture);
WEBP_EXTERN int WebPPictureCopy(const WebPPicture* src, WebPPicture* dst);

/* Import from packed 8-bit samples, ref encode.h:458-476. With
 * use_argb == 0 the RGB->YUV420 conversion runs on the GPU. */
WEBP_EXTERN int WebPPictureImportRGB(WebPPicture* picture, const uint8_t* rgb,
                                     int rgb_stride);
WEBP_EXTERN int WebPPictureImportRGBA(WebPPicture* picture,
                                      const uint8_t* rgba, int rgba_stride);
WEBP_EXTERN int WebPPictureImportRGBX(WebPPicture* picture,
                                      const uint8_t* rgbx, int rgbx_stride);
WEBP_EXTERN int WebPPictureImportBGR(WebPPicture* picture, const uint8_t* bgr,
                                     int bgr_stride);
WEBP_EXTERN int WebPPictureImportBGRA(WebPPicture* picture,
                                      const uint8_t* bgra, int bgra_stride);
WEBP_EXTERN int WebPPictureImportBGRX(WebPPicture* picture,
                                      const uint8_t* bgrx, int bgrx_stride);

/* ref encode.h:480-482, :508 */
WEBP_EXTERN int WebPPictureARGBToYUVA(WebPPicture* picture,
                                      WebPEncCSP colorspace);
/* ref encode.h:493-509: dithered (only dithering == 0 is accepted here) and
 * sharp (iterative, GPU kernels hip/vp8_sharp.hip) ARGB -> YUV420. */
WEBP_EXTERN int WebPPictureARGBToYUVADithered(WebPPicture* picture,
                                              WebPEncCSP colorspace,
                                              float dithering);
WEBP_EXTERN int WebPPictureSharpARGBToYUVA(WebPPicture* picture);
WEBP_EXTERN int WebPPictureSmartARGBToYUVA(WebPPicture* picture);
WEBP_EXTERN int WebPPictureHasTransparency(const WebPPicture* picture);

/* Picture utilities beside the encode path (host C, host buffers):
 * ref encode.h:377-456, 510-529. */
WEBP_EXTERN int WebPPlaneDistortion(const uint8_t* src, size_t src_stride,
                                    const uint8_t* ref, size_t ref_stride,
                                    int width, int height, size_t x_step,
                                    int type, float* distortion, float* result);
WEBP_EXTERN int WebPPictureDistortion(const WebPPicture* src,
                                      const WebPPicture* ref, int metric_type,
                                      float result[5]);
WEBP_EXTERN int WebPPictureCrop(WebPPicture* picture, int left, int top,
                                int width, int height);
WEBP_EXTERN int WebPPictureView(const WebPPicture* src, int left, int top,
                                int width, int height, WebPPicture* dst);
WEBP_EXTERN int WebPPictureIsView(const WebPPicture* picture);
WEBP_EXTERN int WebPPictureRescale(WebPPicture* picture, int width,
                                   int height);
WEBP_EXTERN int WebPPictureYUVAToARGB(WebPPicture* picture);
WEBP_EXTERN void WebPCleanupTransparentArea(WebPPicture* picture);
WEBP_EXTERN void WebPBlendAlpha(WebPPicture* picture, uint32_t background_rgb);

/* Main entry point, ref encode.h:544. Returns 0 on error, reason in
 * picture->error_code (first error wins). */
WEBP_EXTERN int WebPEncode(const WebPConfig* config, WebPPicture* picture);

#ifdef __cplusplus
}
#endif

#endif /* WEBP_WEBP_ENCODE_H_ */
