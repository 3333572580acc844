/* Internal: the lossless (VP8L) side of WebPGpuBatch (config->lossless). */
#ifndef LIBWEBP_AMD_VP8L_BATCH_H_
#define LIBWEBP_AMD_VP8L_BATCH_H_

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime_api.h>

#include "../vp8l_gpu.h"

struct WebPGpuBatch;

typedef struct vp8l_engine {
  hipEvent_t ev[5];            /* stage boundaries of the last call */
  vp8l_params p;               /* n = max_frames; per call a copy with n set */
  int max_frames, ntt, nht, nblk, method;
  size_t npix, hdr_cap, out_cap;
  /* the root engine decides per frame: its own slots take the spatial /
   * direct / subtract-green frames, palette engines (one per bundling,
   * created on demand) the colour-indexed ones; route_* map frame -> slot */
  struct vp8l_engine* sub[6];   /* [0..3] palette by bundling, [4] spatial / direct frames
                                   whose colours fit a palette (palette histogram bits),
                                   [5] repeat-heavy frames of more colours (p.lz) */
  struct vp8l_engine** route_eng;
  int* route_slot;
  /* device (HBM) */
  int32_t* d_tabs;             /* nlogn (4097) | log2 fraction (1024) */
  uint32_t* d_argb;
  uint32_t* d_ops;
  uint8_t* d_minb;             /* smallest cache size holding each pixel */
  uint32_t* d_cseg;            /* L2 segment cache tables (vp8l_gpu.h) */
  uint16_t* d_prov;            /* provisional parse */
  uint32_t* d_chist;           /* cache-size choice histograms */
  uint8_t* d_cbits;            /* chosen cache bits per slot */
  uint32_t* d_ehist;           /* L0 entropy histograms (root engine) */
  uint32_t* d_scan;            /* L0 colour sets (root engine) */
  uint32_t* d_rep;             /* L0b repeat test, 2 words per frame (root engine) */
  uint32_t* h_rep;
  int* d_fidx;                 /* input frame of each slot */
  uint8_t* d_fmode;            /* entropy mode of each slot */
  uint32_t* d_psort;           /* palette engine: sorted palette per slot */
  uint8_t* d_psidx;            /*   stored index of each sorted colour */
  int* d_npal;
  int nl_bits;                 /* near-lossless limit bits (0 = lossless) */
  uint8_t* d_nl[2];            /* near-lossless passes (max_frames x w*h*4), on demand */
  uint8_t* d_nlapply;          /* per slot: preprocess (1) or copy (0) */
  uint8_t* h_nlapply;
  uint8_t* d_modes;
  uint32_t* d_mult;
  uint32_t* d_aflag;
  uint32_t* d_pflag;           /* per slot: residuals from the serial pass (L1a) */
  uint8_t* d_pexact;           /* per slot: the reference's predictor choice (L1a) */
  uint8_t* h_pexact;
  int64_t* d_feat;
  uint32_t* d_tl;
  uint32_t* d_tn;
  uint32_t* d_hc;
  uint8_t* d_assign;
  uint32_t* d_ctab;
  uint8_t* d_gtile;
  uint64_t* d_start;
  uint64_t* d_end;
  uint32_t* d_bsum;
  uint64_t* d_boff;
  uint8_t* d_out;
  uint8_t* d_packed;           /* packed .webp files (k_vp8l_pack), grown on demand */
  size_t d_packed_cap;
  uint64_t* d_poff;
  uint32_t* d_hpack;           /* packed headers, grown on demand */
  size_t d_hpack_cap;
  uint64_t* d_hoff;
  uint32_t* d_hwords;
  /* host (pinned) */
  uint32_t* h_ehist;
  uint32_t* h_scan;
  int* h_fidx;
  uint8_t* h_fmode;
  uint8_t* h_cbits;
  uint32_t* h_psort;
  uint8_t* h_psidx;
  int* h_npal;
  uint32_t* h_pal;             /* palette in stored order per slot */
  uint8_t* h_modes;
  uint32_t* h_mult;
  uint32_t* h_aflag;
  uint32_t* h_hc;
  uint8_t* h_assign;
  uint32_t* h_ctab;
  uint8_t* h_gtile;
  uint64_t* h_start;
  uint64_t* h_end;
  uint8_t* h_hdr;              /* per frame hdr_cap bytes of header */
  uint8_t* h_out;              /* packed .webp files of the last call */
  uint64_t* h_poff;
  uint8_t* h_hpack;
  size_t h_hpack_cap;
  uint64_t* h_hoff;
  uint32_t* h_hwords;
  size_t h_out_cap;
  size_t* hdr_bytes;
  size_t* out_off;
  size_t* out_size;
  int* err;
  /* colour-indexed engines: the cost-model parse's buffers (vp8l_gpu.h) */
  vp8l_lz lz;
  uint8_t* d_dcodes;
  int32_t* d_dpcand;   /* shortest-path parse: VP8L_DP_NC x 4 candidate words */
  int dp_ncand;
  int32_t* d_dpcost;   /* max_frames x VP8L_DP_NCOST */
  int device;   /* the HIP device current at creation (host threads' NUMA node) */
} vp8l_engine;

#ifdef __cplusplus
extern "C" {
#endif
/* alpha != 0: ALPH-chunk engine, input = alpha planes (1 byte per pixel);
 * outputs are bare VP8L streams at vp8l_engine_output() */
vp8l_engine* vp8l_engine_new(int w, int h, int max_frames, int method, int alpha);
/* results of frame f of the last call (routed to the engine that coded it) */
const uint8_t* vp8l_engine_output(const vp8l_engine* l, int f);
size_t vp8l_engine_out_size(const vp8l_engine* l, int f);
int vp8l_engine_error(const vp8l_engine* l, int f);

/* WebPAuxStats' lossless fields of frame f of the last call
 * (src/enc/vp8l_enc.c:1628-1639): transforms used (1 predictor, 2 cross
 * colour, 4 subtract green, 8 palette), tile bits, colour-cache bits,
 * palette size, header bytes (image header + transforms + codes) and
 * pixel-data bytes */
typedef struct {
  int features, histogram_bits, transform_bits, cache_bits, palette_size;
  int hdr_bytes, data_bytes;
} vp8l_frame_info;
void vp8l_engine_frame_info(const vp8l_engine* l, int f, vp8l_frame_info* info);
void vp8l_engine_free(vp8l_engine* l);
/* config->near_lossless (0..100) for the next calls: frames coded without a
 * palette are first passed through VP8ApplyNearLossless (own choice for the
 * spatial modes, see oracle/vp8l_model.py:encode) */
void vp8l_engine_set_near_lossless(vp8l_engine* l, int quality);
/* WebPConfig::exact for the predictor's residuals (ALPH engines stay exact) */
void vp8l_engine_set_exact(vp8l_engine* l, int exact);
int vp8l_engine_run(struct WebPGpuBatch* b, const uint8_t* rgba, size_t fstride, int rstride,
                    int n);
/* one call on `stream` (hipStream_t) with `threads` host threads; stage
 * times (us) into timings[0..8] as WebPGpuBatchTimings documents */
int vp8l_engine_encode(vp8l_engine* l, void* stream, int threads, const uint8_t* in,
                       size_t fstride, int rstride, int n, double timings[10]);
#ifdef __cplusplus
}
#endif

#endif /* LIBWEBP_AMD_VP8L_BATCH_H_ */
