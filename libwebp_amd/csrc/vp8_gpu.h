/* Data layouts shared by the host C engine and the HIP kernels.
 *
 * HBM layout per batch (N frames of W x H, mbw = ceil(W/16), mbh = ceil(H/16)):
 *   rgba      N x (row_stride * H)          caller-owned input
 *   yuv       N x (W*H + 2*uvw*uvh)         Y | U | V planes, the WebPPicture
 *                                           memory_ layout (picture_enc.c:104-162)
 *   mb_alpha  N x nmb  uint8                analysis susceptibility (K2)
 *   mb_uva    N x nmb  uint16               analysis uv susceptibility (K2)
 *   segmap    N x nmb  uint8                final segment per MB (host)
 *   params    N x vp8g_frame_params         quantisers / lambdas (host)
 *   tokens    N x tok_cap uint16            VP8 token stream (K3), the
 *                                           reference's token_t format
 *                                           (token_enc.c:31-35)
 *   mbinfo    N x nmb x VP8G_MBINFO_BYTES   modes for partition 0 (K3)
 *   results   N x vp8g_frame_result         final probas, stats (K3)
 */
#ifndef LIBWEBP_AMD_VP8_GPU_H_
#define LIBWEBP_AMD_VP8_GPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VP8G_NUM_SLOTS 1056        /* 4 types x 8 bands x 3 ctx x 11 probas */
#define VP8G_MBINFO_BYTES 20       /* type, uv_mode, segment, skip, modes[16] */
#define VP8G_MAX_TOKENS_PER_MB 7680 /* 25 blocks x 16 coeffs x 19 tokens + EOBs */
/* the frame error bit of a launch whose token rows ran out of room (the
 * host grows the rows and runs the pass again; see vp8g_rows) */
#define VP8G_ERR_ARENA 0x100

/* one quantiser matrix, src/enc/vp8i_enc.h:181-187 */
typedef struct {
  uint16_t q[16], iq[16];
  uint32_t bias[16], zthresh[16];
  uint16_t sharpen[16];
} vp8g_mtx;

/* per-segment parameters, src/enc/vp8i_enc.h:189-205 */
typedef struct {
  vp8g_mtx y1, y2, uv;
  int32_t lambda_i16, lambda_i4, lambda_uv, lambda_mode, tlambda, min_disto;
  int32_t lambda_trellis_i16, lambda_trellis_i4, lambda_trellis_uv;
  int32_t i4_penalty;    /* 1000 * q_i4^2, RD_OPT_NONE intra-4 start score (quant_enc.c:285) */
} vp8g_seg;

typedef struct {
  vp8g_seg seg[4];
  int32_t max_i4_header_bits;
  int32_t rd_opt;        /* 1 basic (m3/m4), 2 trellis-final (m5), 3 trellis-all (m6) */
  int32_t method;
  int32_t use_derr;      /* U/V DC error diffusion (quality <= 98) */
  int32_t max_count;     /* cost-refresh period (frame_enc.c:785,800) */
  int32_t pass_mode;     /* 0 first pass (default probabilities, zero statistics);
                            1 later pass starting from the previous pass's cost
                            state in rerun_state with the token statistics
                            reset (the last pass of frame_enc.c:808-880, and
                            the partition-0 re-run of :869-876); 3 the same but
                            the statistics continue from rerun_state (a
                            non-last pass); 2 frame already final: skip */
  uint64_t recon_addr;   /* device address of this frame's nmb x 512 B
                            reconstruction buffer (autofilter), or 0 */
  /* RD_OPT_NONE (methods 0-2, VP8EncLoop) */
  int32_t mb_header_limit;  /* webp_enc.c:109-110 */
  int32_t nb_stat;          /* MBs of the statistics pass (StatLoop's fast probe) */
  int32_t none_finalize;    /* the statistics pass finalises the probabilities */
  int32_t skip_count;       /* >= 0: FinalizeSkipProba's skip count, StatLoop having run as
                               K3 passes (a size / PSNR search); -1: the probe's own */
  /* WebPEncode progress / abort (iterator_enc.c:89-99): device address of two
     host-mapped words, or 0: [0] MB rows folded so far (K3 stores it in
     raster order), [1] non-zero = abort (the host sets it when the progress
     hook returns 0; K3 stops after the row it folds next, error site 6) */
  uint64_t progress_addr;
} vp8g_frame_params;

/* per-frame cost state K3 leaves for the next pass: the probabilities the
 * level-cost tables were last computed from, then the probabilities at the
 * end of the MB loop (before the final refresh), then the token statistics
 * (uint32 per slot, proba_t of src/enc/vp8i_enc.h:146). Between passes of a
 * size search the host replaces the probabilities by FinalizeTokenProbas'. */
#define VP8G_RERUN_STATE_BYTES (6 * VP8G_NUM_SLOTS)
#define VP8G_STATE_COEFFS (VP8G_NUM_SLOTS)       /* offset of the loop-end probabilities */
#define VP8G_STATE_STATS (2 * VP8G_NUM_SLOTS)    /* offset of the statistics */

typedef struct {
  uint32_t ntokens;
  uint32_t error;        /* nonzero: token buffer overflow */
  int32_t max_edge[4];
  uint64_t size_p0;      /* sum of per-MB header-bit estimates (frame_enc.c:839) */
  uint64_t sse[3];
  uint64_t distortion;   /* sum of the per-MB VP8ModeScore D (frame_enc.c:840) */
  uint64_t size_rh;      /* sum of the per-MB R + H (OneStatPass's size, frame_enc.c:593);
                            K3 only */
  int32_t block_count[3];
  int16_t use_skip, skip_proba;   /* RD_OPT_NONE: FinalizeSkipProba (frame_enc.c:111-127) */
  uint64_t stamps[8];    /* per-stage shader-clock cycles summed over MBs (profiling) */
  uint8_t probas[VP8G_NUM_SLOTS];   /* final coefficient probabilities */
} vp8g_frame_result;

/* first-error capture for diagnostics (host side, thread-local) */
void vp8g_set_error(const char* where, const char* what);

/* --- kernel launchers (HIP side, extern "C") --- */

/* RGB(A)->YUV420 for n frames. g2l/l2g are DEVICE pointers to the
 * host-computed gamma tables (picture_csp_enc.c:103-117). Sets
 * alpha_flags[f] bit 0 if frame f has a non-0xff alpha sample. */
int vp8g_launch_import(const uint8_t* rgba, size_t frame_stride, int row_stride,
                       int w, int h, int n, uint8_t* yuv, size_t yuv_frame_bytes,
                       uint32_t* alpha_flags, uint8_t* alpha_plane, const uint16_t* g2l_dev,
                       const int32_t* l2g_dev, const uint16_t* rnd_y, const uint32_t* rnd_uv,
                       void* stream);
/* (rnd_y, rnd_uv: DEVICE rounding terms of the dithered import, W*H and
 * 2 x uvw*uvh with U, V interleaved, from vp8h_dither_rounders; NULL = plain) */
/* alpha planes (n x w*h, stride w) of RGBA frames: all of them (aflags
 * NULL, the sharp-YUV path) or those with aflags[f] != 0 (after K1) */
int vp8g_launch_extract_alpha(const uint8_t* rgba, size_t frame_stride, int row_stride, int w,
                              int h, int n, const uint32_t* aflags, uint8_t* alpha_plane,
                              void* stream);
/* WebPCleanupTransparentArea on the YUV planes of the frames whose
 * alpha_flags are set (config->exact == 0) */
int vp8g_launch_cleanup_alpha(uint8_t* yuv, size_t yuv_frame_bytes, const uint8_t* alpha_plane,
                              const uint32_t* alpha_flags, int w, int h, int n, void* stream);

/* K2 (analysis_enc.c:230-333). fast_q >= 0 selects the methods 0-1
 * analysis (FastMBAnalyze with that integer quality); mb_amode (or NULL)
 * receives per MB the analysis UV mode (bit 0) and, for methods 0-1, the
 * intra-4 pick (bit 1), inputs of the RD_OPT_NONE encoder */
/* alpha level reduction (QuantizeLevels): per-frame 256-bin histograms of
 * the alpha planes of the frames with aflags set (hist zeroed here), and the
 * remap of those planes through maps[f * 256 + symbol] */
int vp8g_launch_alpha_hist(const uint8_t* aplane, size_t plane, const uint32_t* aflags, int n,
                           uint32_t* hist, void* stream);
int vp8g_launch_alpha_remap(uint8_t* aplane, size_t plane, const uint32_t* aflags, int n,
                            const uint8_t* maps, void* stream);

int vp8g_launch_analysis(const uint8_t* yuv, size_t yuv_frame_bytes, int w, int h,
                         int n, uint8_t* mb_alpha, uint16_t* mb_uva, int fast_q,
                         uint8_t* mb_amode, void* stream);

/* K3: RD search + tokens. Without rows, each frame's tokens end up as one
 * compact stream at the start of its tok_cap region (per-MB slots of
 * VP8G_MAX_TOKENS_PER_MB are used as scratch; mboff is scratch of n * nmb
 * uint32, each MB's offset in the compact stream). trellis != 0 reserves the
 * trellis LDS (method >= 5). recon (n x nmb x 512 bytes, or NULL) receives
 * each MB's reconstruction in the 32-byte-stride layout of the reference's
 * yuv_out_ (Y | U | V side by side, src/enc/vp8i_enc.h:72-78) for the
 * autofilter.
 * With rows (the token loop): every token is written once, where K4 reads
 * it -- MB row y of frame f at tokens + f * tok_cap + y * rowcap, its MBs'
 * tokens one after another in raster order (the row's owner knows its own
 * offsets; only the frame-wide stream offsets wait for the rows above, and
 * nothing needs them). The row's count goes to rowtok[f * mbh + y]; a row that
 * would pass rowcap writes nothing more and the frame reports VP8G_ERR_ARENA
 * (the host grows rowcap and runs the launch again). mboff is not written. */
typedef struct {
  uint32_t rowcap;           /* tokens per MB row (a multiple of 8) */
  uint32_t* rowtok;          /* n x mbh row token counts */
} vp8g_rows;

int vp8g_launch_encode(const uint8_t* yuv, size_t yuv_frame_bytes, int w, int h,
                       int n, const uint8_t* segmap,
                       const vp8g_frame_params* params, uint16_t* tokens,
                       size_t tok_cap, uint8_t* mbinfo, uint32_t* mboff, int trellis,
                       vp8g_frame_result* results, uint8_t* rerun_state, uint8_t* recon,
                       uint8_t* xsync, uint32_t* wsnap, const vp8g_rows* rows,
                       void* stream);

/* K3X: when a launch has few frames (n <= VP8G_XSPLIT_MAX_FRAMES) and xsync
 * is not NULL, each frame's MB rows are split over several workgroups (CUs)
 * that hand the wavefront boundary, the statistics fold and the cost epochs
 * to each other through xsync (n x vp8g_xsync_bytes(w, h), zeroed by the
 * launch). */
#define VP8G_XSPLIT_MAX_FRAMES 64
size_t vp8g_xsync_bytes(int w, int h);
/* wsnap (NULL: none): n x vp8g_wsnap_bytes(w, h), the statistics snapshots
 * of K3's row folds (each MB worker's pending deltas every 16 MBs of its row,
 * so the exact replay of a counter's halving starts near it); written before
 * they are read, no reset needed */
size_t vp8g_wsnap_bytes(int w, int h);

/* Autofilter (config->autofilter, filter_enc.c:156-212): per frame the
 * segment filter levels and the filter header fields used for the search */
typedef struct {
  uint8_t simple, sharpness, pad[2];
  uint8_t level0[4];   /* segment fstrength_ from SetupFilterStrength */
  uint8_t quant[4];    /* segment quant_ */
} vp8g_af_frame;
/* per MB (grid nmb x n): SSIM (GetMBSSIM) of the reconstruction unfiltered
 * and filtered at every candidate level of its segment (DoFilter) into
 * mbval[(f * nmb + mb) * 64 + level], 0 elsewhere; then per frame the
 * raster-order sums per segment and level and the best level per segment
 * (VP8AdjustFilterStrength) into level[4 * f + s]. src = the source YUV
 * planes (edge-replicated like VP8IteratorImport). */
int vp8g_launch_autofilter(const uint8_t* yuv, size_t yuv_frame_bytes, int w, int h, int n,
                           const uint8_t* mbinfo, const uint8_t* recon,
                           const vp8g_af_frame* afp, const uint8_t* active, double* mbval,
                           uint8_t* level, void* stream);

/* K3 for methods 0-2 (RD_OPT_NONE; VP8EncLoop, frame_enc.c:739-775): one
 * wavefront per frame in raster order, modes by prediction SSE
 * (RefineUsingDistortion, quant_enc.c:1248-1350), token statistics of the
 * first params->nb_stat MBs (StatLoop), final probabilities and skip
 * probability, then the tokens of skipped MBs dropped when the skip flag
 * pays. amode = K2's analysis modes; mboff scratch n x nmb. rerun_state:
 * statistics carried between passes (pass_mode 3). */
int vp8g_launch_encode_none(const uint8_t* yuv, size_t yuv_frame_bytes, int w, int h, int n,
                            const uint8_t* segmap, const uint8_t* amode,
                            const vp8g_frame_params* params, uint16_t* tokens, size_t tok_cap,
                            uint8_t* mbinfo, uint32_t* mboff, vp8g_frame_result* results,
                            uint8_t* rerun_state, void* stream);

/* low_memory on K3's compact stream (hip/vp8_emit.hip k_lowmem): mode 0
 * adds StatLoop's statistics of the first nb_stat[f] MBs to stats[f]
 * (NUM_SLOTS uint32) and counts their skipped MBs into nskip[f]; mode 1
 * drops the tokens of the skipped MBs and updates results[f].ntokens.
 * Frames with active[f] == 0 are left alone. */
int vp8g_launch_lowmem(uint16_t* tokens, size_t tok_cap, const uint32_t* mboff,
                       vp8g_frame_result* results, const uint8_t* mbinfo, int nmb, int n,
                       const int32_t* nb_stat, const uint8_t* active, int mode, uint32_t* stats,
                       int32_t* nskip, void* stream);

/* VP8EstimateTokenSize (token_enc.c:226-247) of each frame's token stream
 * (compact, or with rows != NULL in K3's token rows) under the probabilities
 * at state + f * VP8G_RERUN_STATE_BYTES + VP8G_STATE_COEFFS; frames with
 * active[f] == 0 are skipped. bits[f] (device, zeroed here) receives the sum
 * in 1/256 bit. */
int vp8g_launch_token_cost(const uint16_t* tokens, size_t tok_cap, const vp8g_rows* rows, int mbh,
                           int n,
                           const vp8g_frame_result* results, const uint8_t* state,
                           const uint8_t* active, unsigned long long* bits, void* stream);

/* K4: boolean coder for the token partitions, parallel inside each stream
 * (hip/vp8_emit.hip). A stream is one token partition of one frame (or its
 * partition 0): its tokens take their probabilities from results[frame] and
 * lie either compact at tokens + tok_off (a multiple of 8 tokens; nrows 0)
 * or in nrows token rows (vp8g_rows) from tokens + tok_off, rowcap apart,
 * their lengths in rowtok[frame * nrows ..]; the coded bytes go to tokens +
 * tok_off. The stream is cut into segments of at most VP8G_EMIT_SEG tokens
 * that never cross a row (k_emit_desc: vp8g_emit_desc per segment).
 * Per-stream bookkeeping: ntok, the segment count (an upper bound from the
 * host for row streams, set exactly on the device) and the first segment /
 * first N-array word of the stream (host), S and L (device). */
typedef struct {
  uint32_t ntok, nseg, seg_base, nb_base, S, L;
  uint32_t frame, nrows;
  uint64_t tok_off;
  uint32_t rowcap, pad;
} vp8g_emit_meta;
typedef struct {
  uint64_t off;    /* the segment's first token: tokens + off (a multiple of 8) */
  uint32_t len, pad;
} vp8g_emit_desc;
#define VP8G_MAX_PARTS 8   /* token partitions per frame (syntax_enc.c:283) */
typedef struct {
  uint32_t T;      /* bit offset of the segment's part of N */
  uint16_t S;      /* renormalisation shifts inside the segment */
  uint8_t rs;      /* true range at the segment start */
  uint8_t H;       /* bits of the segment's partial sum above its region */
} vp8g_emit_seg;
#define VP8G_EMIT_SEG 2048
/* n streams; out_size[s] = the byte count of stream s */
int vp8g_launch_emit(uint16_t* tokens, size_t tok_cap, int n,
                     const vp8g_frame_result* results, vp8g_emit_meta* meta,
                     const uint32_t* rowtok, uint32_t max_ntok, uint32_t max_seg, uint8_t* emap,
                     uint16_t* eshift, uint8_t* img, vp8g_emit_desc* desc, vp8g_emit_seg* segs,
                     uint32_t* nbuf, uint32_t* out_size, void* stream);

/* K4 alone on caller-given fixed-probability token streams (host memory in
 * and out; test hook, see hip/vp8_emit.hip) */
int vp8g_emit_streams(const uint16_t* host_tokens, const uint32_t* ntok, int n, uint8_t* host_out,
                      uint32_t out_stride, uint32_t* out_size);

/* Partition 0 as a K4 stream (syntax_enc.c:187-310, tree_enc.c:313-347,
 * 485-504): the host turns each frame's header (segment / filter / quant
 * headers, probability updates, skip probability) into fixed-probability
 * tokens (vp8h_p0_header, at most VP8G_P0_HDR_CAP), k_p0_modes appends the
 * per-MB segment ids, skip flags and intra modes from K3's mbinfo and K4
 * codes the stream beside the token partitions. vp8g_p0_par carries what
 * the MB part needs; the frame's p0 tokens start at tokens + tok_off of its
 * stream (room for vp8g_p0_cap(nmb) tokens), and k_p0_modes writes the
 * stream's ntok / nseg into its K4 meta. */
#define VP8G_P0_HDR_CAP 10240   /* >= 2 + 59 + 21 + 7 + 30 + 1 + 1056 * 9 + 9 header tokens */
typedef struct {
  uint32_t nhdr;                /* header tokens; 0xffffffff: no stream (frame failed) */
  uint8_t update_map, use_skip, skip_proba, pad;
  uint8_t seg_probas[3], pad2;
} vp8g_p0_par;
/* tokens of one frame's partition 0: header + <= 119 per MB (2 segment,
 * 1 skip, 1 + 16 x 7 luma, 3 chroma), + a K4 segment of slack, 8-aligned */
static inline size_t vp8g_p0_cap(int nmb) {
  return ((size_t)VP8G_P0_HDR_CAP + 119 * (size_t)nmb + VP8G_EMIT_SEG + 7) & ~(size_t)7;
}
/* n frames: frame f's stream is meta[meta_base + f], its header tokens at
 * hdr + f * VP8G_P0_HDR_CAP */
int vp8g_launch_p0_modes(const uint8_t* mbinfo, int mbw, int mbh, int n, const vp8g_p0_par* par,
                         const uint16_t* hdr, uint16_t* tokens, vp8g_emit_meta* meta,
                         int meta_base, void* stream);

/* K4 tail: copy each stream's bytes (size[s] bytes at tokens +
 * meta[s].tok_off) to dst + off[s]; off[s] must be 16-byte aligned. */
int vp8g_launch_pack(const uint16_t* tokens, const vp8g_emit_meta* meta, int n,
                     const uint64_t* off, const uint32_t* size, uint32_t max_size, uint8_t* dst,
                     void* stream);

/* Token partitions (VP8EncLoop, iterator_enc.c:48; methods 0-2 and
 * low_memory): per frame, gather the MB rows of the compact raster token
 * stream into nparts streams, row y into partition y & (nparts - 1), placed
 * from token round8(tok_cap / 2) of the frame's slab. Each MB's token count
 * comes from mboff: kind 0 = the count itself (K3N), kind 1 = compact-stream
 * offsets with the last MB ending at the frame's token count (K3 + k_lowmem);
 * MBs with the skip flag of a use_skip frame count 0. part[16 f + p] = start
 * of partition p (tokens from the frame slab), part[16 f + 8 + p] = its token
 * count; part[16 f] = 0xffffffff when the stream does not fit. */
int vp8g_launch_partition(uint16_t* tokens, size_t tok_cap, int n, const uint32_t* mboff,
                          const vp8g_frame_result* results, const uint8_t* mbinfo, int mbw,
                          int mbh, int kind, int nparts, uint32_t* part, void* stream);

/* Sharp (iterative) RGB->YUV420 for n frames (hip/vp8_sharp.hip), the
 * use_sharp_yuv import (sharpyuv/sharpyuv.c). scratch holds
 * vp8g_sharp_frame_bytes(w, h) per frame, state one entry per frame; g2l/l2g
 * are DEVICE copies of the sRGB tables (1026 + 514 entries, vp8h_sharp_tables).
 * w and h must be >= 4 (smaller pictures take vp8g_launch_import). */
typedef struct {
  unsigned long long prev_sum;
  int done, iters;
} vp8g_sharp_state;
size_t vp8g_sharp_frame_bytes(int w, int h);
int vp8g_launch_sharp(const uint8_t* rgba, size_t frame_stride, int row_stride, int w, int h,
                      int n, uint8_t* yuv, size_t yuv_frame_bytes, uint32_t* alpha_flags,
                      uint8_t* scratch, vp8g_sharp_state* state, const uint32_t* g2l_dev,
                      const uint32_t* l2g_dev, void* stream);

/* synthetic syn-v1 frames straight into device memory */
int vp8g_launch_synth(uint8_t* rgba, size_t frame_stride, int w, int h,
                      int first_frame, int n, int seed, void* stream);

#ifdef __cplusplus
}
#endif
#endif
