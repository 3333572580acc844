/* Host-side (C) parts of the VP8 lossy path that are per-frame and serial:
 * segment/quantiser setup between the analysis and RD kernels, and the
 * boolean-coder tail + bitstream assembly after them. */
#ifndef LIBWEBP_AMD_VP8_HOST_H_
#define LIBWEBP_AMD_VP8_HOST_H_

#include <stddef.h>
#include <stdint.h>

#include "../vp8_gpu.h"
#include "webp/encode.h"

#ifdef __cplusplus
extern "C" {
#endif

/* partition-0 limit on the header estimate (frame_enc.c:32) */
#define VP8H_P0_LIMIT ((((uint64_t)1 << 19) - 2048ULL) << 11)

/* Frame-level encoder state that lives on the host (a slice of the
 * reference's VP8Encoder, src/enc/vp8i_enc.h:346-413). */
typedef struct {
  int w, h, mbw, mbh;
  /* config-derived (webp_enc.c:95-123, 144-252) */
  int method, rd_opt, max_i4_header_bits, profile;
  float quality;
  int sns_strength, filter_strength, filter_sharpness, filter_type;
  int preprocessing, emulate_jpeg_size, cfg_segments;
  /* segment header + per-segment values */
  int num_segments, update_map, seg_hdr_size;
  int num_parts;   /* token partitions (1, 2, 4 or 8) */
  uint8_t seg_probas[3];
  int alpha, uv_alpha, base_quant, dq_uv_dc, dq_uv_ac;
  int seg_alpha[4], seg_beta[4], seg_quant[4], seg_fstrength[4], seg_y2ac[4];
  int segment_size[4];
  /* mb->alpha_ after AssignSegments (analysis_enc.c:202-207): the centre of
   * each raw analysis alpha's class, 0 without segmentation (extra_info 7) */
  uint8_t alpha_center[256];
  /* filter header */
  int f_simple, f_level, f_sharpness;
  /* multi-pass convergence (PassStats, frame_enc.c:38-80) */
  int lm_skip_proba;   /* low_memory: StatLoop's skip probability */
  int lm_nskip;        /* StatLoop search: the last pass's skip count */
  int lm_max_edge[4];  /* StatLoop at RD_OPT_BASIC: the last pass's StoreMaxDelta maxima
                          (SetupMatrices resets them per pass, quant_enc.c:283) */
  int autofilter;   /* segment filter levels from the GPU SSIM search (filter_enc.c:156-212) */
  int cfg_pass, pass_left, is_last_pass, npass, do_search, do_size_search, ps_is_first;
  float ps_dq, ps_q, ps_last_q, ps_qmin, ps_qmax;
  double ps_value, ps_last_value, ps_target;
} vp8h_frame;

/* Initialise from a validated config (lossy, method 3..6). Returns 0 if the
 * config is outside what the GPU path implements. */
/* sRGB gamma tables of the sharp-YUV import (sharpyuv/sharpyuv_gamma.c:33-78):
 * 1026 gamma->linear and 514 linear->gamma entries, double pow like the
 * reference. Thread-safe, computed once. */
void vp8h_sharp_tables(const uint32_t** g2l, const uint32_t** l2g);
/* whether an encode with this config on a w x h picture takes the sharp
 * import (use_sharp_yuv or preprocessing & 4, and both dimensions >= 4,
 * webp_enc.c:352-356, picture_csp_enc.c:493-496) */
int vp8h_use_sharp(const WebPConfig* cfg, int w, int h);

int vp8h_frame_init(vp8h_frame* fr, const WebPConfig* cfg, int w, int h);

/* Segment analysis + parameters (analysis_enc.c:76-216, quant_enc.c:205-455,
 * frame_enc.c:198-231). Inputs: per-MB analysis alphas from the GPU.
 * Outputs: final per-MB segment ids and the kernel parameter block. */
void vp8h_setup_segments(vp8h_frame* fr, const uint8_t* mb_alpha, const uint16_t* mb_uva,
                         uint8_t* segmap, vp8g_frame_params* params);
/* the two halves of vp8h_setup_segments: the k-means on the analysis alphas
 * (VP8EncAnalyze tail) once per frame, then SetLoopParams (frame_enc.c:563-572:
 * VP8SetSegmentParams + SetupMatrices + SetSegmentProbas) at the start of
 * every pass with that pass's quality */
void vp8h_analyze_segments(vp8h_frame* fr, const uint8_t* mb_alpha, const uint16_t* mb_uva,
                           uint8_t* segmap);
void vp8h_set_loop_params(vp8h_frame* fr, float q, uint8_t* segmap, vp8g_frame_params* params);

/* Pass loop of VP8EncTokenLoop (frame_enc.c:808-880), one frame:
 *   while (vp8h_pass_start(fr)) { SetLoopParams(fr->ps_q); K3;
 *                                 if (!vp8h_pass_finish(...)) break; }
 * vp8h_pass_start consumes a pass and sets fr->is_last_pass (K3 resets the
 * token statistics only on the last pass). vp8h_pass_finish takes the pass's
 * header estimate (K3 size_p0 + segment header) and its value (estimated
 * size in bytes or PSNR, vp8h_pass_value) and returns 1 when another pass
 * follows: partition-0 overflow retry (:869-876) or a search step
 * (ComputeNextQ, :60-80). */
int vp8h_pass_start(vp8h_frame* fr);
int vp8h_pass_finish(vp8h_frame* fr, uint64_t size_p0);
/* StatLoop's pass loop (VP8EncLoop with a size / PSNR search, frame_enc.c:
 * 614-672) with the same vp8h_pass_start; returns 1 when another pass
 * follows */
int vp8h_statloop_finish(vp8h_frame* fr, uint64_t size_p0);
/* FinalizeSkipProba (frame_enc.c:111-127): returns the size term */
int vp8h_finalize_skip(int nb_skip, int nmb, int* skip_proba, int* use_skip);
/* FinalizeTokenProbas (frame_enc.c:146-180) from the token statistics:
 * writes the probabilities, returns the proba-update header cost (1/256
 * bit); *dirty = some probability differs from the default table */
void vp8h_default_probas(uint8_t* coeffs);   /* the default coefficient probabilities */
int vp8h_finalize_probas(const uint32_t* stats, uint8_t* coeffs, int* dirty);
/* size of the pass in bytes (size search) from the finalize cost, the token
 * bit estimate (VP8EstimateTokenSize) and the header estimate */
double vp8h_pass_size_value(uint64_t finalize_cost, uint64_t token_bits, uint64_t size_p0);
double vp8h_psnr(uint64_t mse, uint64_t count);   /* GetPSNR, frame_enc.c:554-556 */
/* sum of the header-bit estimates info.H of MBs 0..nb-1 from their modes
 * (mbinfo rows of VP8G_MBINFO_BYTES): the probe's size_p0 before the
 * segment header */
uint64_t vp8h_mode_header_bits(const uint8_t* mbinfo, int mbw, int nb);

/* Dithered import (preprocessing & 2): the amplitude WebPEncode derives from
 * the quality (webp_enc.c:357-365, 0 when off), and the rounding terms the
 * VP8Random generator feeds RGBToY / RGBToU / RGBToV in the reference's
 * order (picture_csp_enc.c:150-166,520-619): ry[W*H], ruv[2*uvw*uvh] (U, V
 * interleaved per chroma sample). */
float vp8h_import_dithering(const WebPConfig* cfg);
void vp8h_dither_rounders(int w, int h, float dithering, uint16_t* ry, uint32_t* ruv);

/* QuantizeLevels (src/utils/quant_levels_utils.c:31-137) from the plane's
 * histogram: the symbol map to num_levels levels (identity when the plane has
 * no more levels than that) and the squared error it reports. */
void vp8h_quantize_levels_map(const uint32_t hist[256], uint64_t count, int num_levels,
                              uint8_t map[256], uint64_t* sse);
/* alpha_enc.c:346-347: levels for an alpha_quality < 100 */
int vp8h_alpha_levels(int quality);

/* Boolean coder (bit_writer_utils.c). */
typedef struct {
  int32_t range, value;
  int run, nb_bits;
  uint8_t* buf;
  size_t pos, cap;
  int error;
} vp8h_bw;

void vp8h_bw_init(vp8h_bw* bw, size_t expected);
void vp8h_bw_free(vp8h_bw* bw);
void vp8h_bw_finish(vp8h_bw* bw);

/* VP8EmitTokens (token_enc.c:200-223): replay the GPU token stream through
 * the boolean coder with the final probabilities. */
void vp8h_emit_tokens(vp8h_bw* bw, const uint16_t* tokens, size_t n, const uint8_t* probas);

/* Assemble the complete RIFF/WEBP/VP8 file (syntax_enc.c:269-389) into a
 * malloc'ed buffer. Applies VP8AdjustFilterStrength (filter_enc.c:194-233)
 * first. Returns the size, 0 on error (*err set). */
/* The two halves of vp8h_assemble: partition 0 (frame header + intra modes,
 * syntax_enc.c:183-245, tree_enc.c:378-411) needs only K3's outputs and can be
 * coded while K4 codes partition 1; the RIFF write joins them. */
int vp8h_build_p0(vp8h_frame* fr, const vp8g_frame_result* res, const uint8_t* mbinfo,
                  vp8h_bw* p0, int* hdr_bytes);
/* partition 0's frame header as fixed-probability tokens (at most cap; -1
 * if more), after VP8AdjustFilterStrength; *hdr_bytes0 (if not NULL): the
 * bytes a coder has written after them (WebPAuxStats header_bytes[0]) */
int vp8h_p0_header(vp8h_frame* fr, const vp8g_frame_result* res, uint16_t* tok, int cap,
                   int* hdr_bytes0);
/* what k_p0_modes needs of the frame (nhdr < 0: no stream) */
void vp8h_p0_par(const vp8h_frame* fr, const vp8g_frame_result* res, int nhdr, vp8g_p0_par* p);
/* ALPH chunk payload: header byte (compression | filter << 2 | levels << 4,
 * alpha_enc.c:168-170) and the data (bare VP8L stream or raw plane) */
typedef struct {
  uint8_t header;
  const uint8_t* data;
  size_t size;
} vp8h_alpha;
/* *out is reused when *cap (if cap != NULL) already holds the file, else
 * replaced by a fresh allocation (*cap updated) */
size_t vp8h_write_riff(const vp8h_frame* fr, vp8h_bw* p0, const vp8h_bw* parts, int nparts,
                       const vp8h_alpha* alpha, uint8_t** out, size_t* cap, int* err);
size_t vp8h_assemble(vp8h_frame* fr, const vp8g_frame_result* res, const uint8_t* mbinfo,
                     vp8h_bw* part1, uint8_t** out, int* err, int* hdr_bytes);

#ifdef __cplusplus
}
#endif
#endif
