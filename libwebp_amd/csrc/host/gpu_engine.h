/* Internal: the batched GPU engine behind WebPGpuBatch and WebPEncode. */
#ifndef LIBWEBP_AMD_GPU_ENGINE_H_
#define LIBWEBP_AMD_GPU_ENGINE_H_

#include <pthread.h>
#include <stdatomic.h>

#include <hip/hip_runtime_api.h>

#include "../vp8_gpu.h"
#include "vp8_host.h"
#include "vp8l_batch.h"
#include "webp/encode.h"

/* host-thread placement on the GPU's NUMA node (host_cpus.c) */
int vp8g_thread_create(pthread_t* th, void* (*fn)(void*), void* arg, int device);
int vp8g_device_ncpu(int device);   /* CPUs of the device's share (0: not pinned) */
int vp8g_rank_threads(int device);  /* the rank's host-thread budget (quota / ranks, pinned CPUs) */
/* a host phase's n per-frame items on the rank's persistent thread pool
 * (host_cpus.c): submit queues the job (at most `width` pool threads on it at
 * once), join has the caller take items too and returns when all are done */
typedef struct vp8g_job {
  void (*fn)(void* ctx, int i);
  void* ctx;
  int n, width, active;
  atomic_int next, done;
  struct vp8g_job* link;
  void* pool;
} vp8g_job;
void vp8g_job_submit(int device, vp8g_job* j, void (*fn)(void*, int), void* ctx, int n, int width);
void vp8g_job_join(vp8g_job* j);

struct WebPGpuBatch {
  int device, w, h, max_frames, mbw, mbh, nmb, uvw, uvh, threads, last_n;
  /* WebPEncode's per-MB-row progress / abort (vp8g_frame_params::progress_addr):
     progress(ctx, rows_done, mbh) is polled while K3 runs on frame 0; a 0
     return stops K3 after its next row fold (VP8_ENC_ERROR_USER_ABORT) */
  int (*progress)(void* ctx, int rows_done, int rows_total);
  void* progress_ctx;
  uint32_t* h_prog;          /* 2 host-mapped words: rows done, abort */
  uint64_t d_prog;           /* their device address */
  WebPConfig cfg;
  size_t yfb, tok_cap, d_rgba_cap, h_tok_cap;
  hipStream_t stream;
  hipEvent_t ev[6];          /* K1 start, K2 end, K3 start, K3 end, K4 start, K4 end */
  int ev0_recorded;
  /* device (HBM) */
  uint8_t* d_rgba;
  /* the next batch's frames, uploaded while this one encodes
     (WebPGpuBatchEncodeRGBAHostPrefetch): a second RGBA buffer and the
     copy in flight into it */
  uint8_t* d_rgba2;
  size_t d_rgba2_cap;
  const uint8_t* pf_src;
  size_t pf_need, pf_fstride;
  int pf_rstride, pf_n, pf_busy;
  uint64_t pf_sig;
  uint16_t* d_g2l;   /* gamma tables: 256 x u16 then 33 x i32 */
  int32_t* d_l2g;
  uint8_t* d_yuv;
  uint32_t* d_aflags;
  uint8_t* d_aplane;         /* alpha planes, n x w*h (K1 / upload) */
  vp8l_engine* la;           /* ALPH-chunk VP8L engine, created on first use */
  uint8_t** araw;            /* raw alpha planes (alpha_compression 0 / fallback) */
  uint32_t* d_ahist;         /* alpha level reduction: histograms, maps (first use) */
  uint8_t* d_amaps;
  uint32_t* h_ahist;
  uint8_t* h_amaps;
  uint64_t* asse;            /* alpha squared error per frame (WebPAuxStats PSNR[4]) */
  uint8_t* d_alpha;
  uint8_t* d_amode;          /* K2 analysis modes (RD_OPT_NONE input) */
  uint16_t* d_uva;
  uint8_t* d_segmap;
  vp8g_frame_params* d_params;
  uint16_t* d_tokens;         /* per-frame compact streams, stride tok_cap tokens */
  /* token rows of the token loop (methods 3-6 without low_memory): K3
   * writes each MB's tokens once, row y of frame f at d_tokens + f * tok_cap
   * + y * rowcap, and K4 reads them there (vp8g_rows; grown when a row runs
   * out of room) */
  size_t rowcap;
  uint32_t* d_rowtok;        /* n x mbh row token counts */
  uint32_t* h_rowtok;
  int tiny_tokens;   /* WEBP_AMD_TEST_TINY_TOKENS=1 (tests): tiny initial token rows */
  uint8_t* d_rerun_snap;     /* d_rerun before a pass that re-reads it (regrow re-runs) */
  uint8_t* d_mbinfo;
  uint32_t* d_mboff;         /* K3 scratch: compact-stream offset per MB */
  uint8_t* d_rerun;          /* K3 cost state carried from pass to pass */
  uint8_t* d_xsync;          /* K3X cross-workgroup frame state (max_frames <= 64) */
  uint32_t* d_wsnap;         /* K3 row-fold statistics snapshots (vp8g_wsnap_bytes) */
  /* size search between passes (allocated on first use) */
  uint8_t* h_state;          /* pinned copy of d_rerun */
  uint8_t* d_active;         /* frames whose token bits are estimated */
  uint8_t* h_active;
  unsigned long long* d_tbits;
  unsigned long long* h_tbits;
  int* fin_cost;             /* FinalizeTokenProbas header cost per frame */
  uint32_t* d_lmstats;       /* low_memory: StatLoop statistics (first use) */
  uint32_t* h_lmstats;
  int32_t* d_lmi;            /* low_memory: probe MBs, then skips, per frame */
  int32_t* h_lmi;
  /* autofilter (allocated on first use) */
  uint8_t* d_recon;          /* reconstructed MBs, n x nmb x 512 */
  double* d_mbval;           /* per-MB SSIM per level, n x nmb x 64 */
  vp8g_af_frame* d_afp;
  vp8g_af_frame* h_afp;
  uint8_t* d_aflevel;        /* best level per frame and segment */
  uint8_t* h_aflevel;
  uint8_t* pass_act;         /* frames with a pass to run */
  vp8g_frame_result* d_results;
  uint32_t* d_psize;         /* partition-1 bytes per frame (K4) */
  vp8g_emit_meta* d_emeta;   /* K4 per-stream bookkeeping (nparts streams per frame) */
  int nparts;                /* token partitions per frame (1 << partitions for VP8EncLoop) */
  uint32_t* d_pinfo;         /* k_partition: 16 words per frame (starts, counts) */
  uint32_t* h_pinfo;
  vp8g_emit_meta* h_emeta;
  uint8_t* d_emap;           /* K4 scratch, grown on demand */
  vp8g_emit_desc* d_edesc;   /* K4 segment descriptors */
  uint16_t* d_eshift;
  uint8_t* d_eimg;           /* possible start ranges per segment (17 B each) */
  vp8g_emit_seg* d_esegs;
  uint32_t* d_nbuf;
  size_t emit_seg_cap, emit_word_cap;
  /* sharp-YUV import (allocated on first use) */
  int sharp;                 /* config asks for it and the frame is >= 4x4 */
  float dither, dither_built;   /* dithered K1 import (preprocessing & 2) */
  uint16_t* d_rnd_y;         /* its rounding terms (VP8Random), built on first use */
  uint32_t* d_rnd_uv;
  uint32_t* d_stabs;         /* 1026 gamma->linear + 514 linear->gamma */
  uint8_t* d_sharp;          /* per-frame W/RGB planes */
  vp8g_sharp_state* d_sstate;
  /* host (pinned) */
  uint32_t* h_aflags;
  uint8_t* h_alpha;
  uint16_t* h_uva;
  uint8_t* h_segmap;
  vp8g_frame_params* h_params;
  uint8_t* h_mbinfo;
  vp8g_frame_result* h_results;
  uint32_t* h_psize;
  uint8_t* h_part;           /* pinned partition-1 bytes of all frames */
  size_t h_part_cap;
  uint64_t* h_poff;          /* pinned: 16-byte aligned offset of each frame in h_part */
  uint64_t* d_poff;
  uint8_t* d_part;           /* packed partition-1 bytes (k_pack), grown on demand */
  size_t d_part_cap;
  vp8h_bw* p0;               /* partition 0 of each frame, coded while K4 runs */
  /* partition 0 as K4 streams (k_p0_modes; gpu_p0): the header tokens per
     frame (host-built, pinned) and k_p0_modes' parameters; the streams' tokens
     follow the frames' token slabs in d_tokens (p0_cap tokens per frame) */
  int gpu_p0;                /* 0 host, 1 device, -1 by the rank's thread budget */
  int p0_dev;                /* the last call put partition 0 on the device */
  int last_ns;               /* its token-partition streams (partition 0 follows) */
  size_t p0_cap;
  uint16_t* h_p0hdr;
  uint16_t* d_p0hdr;
  vp8g_p0_par* h_p0par;
  vp8g_p0_par* d_p0par;
  uint16_t* h_tokens;
  size_t* tok_off;
  vp8h_frame* frames;
  /* outputs of the last call */
  uint8_t** out;
  size_t* out_cap;     /* allocated bytes of out[f] (reused across batches) */
  size_t* out_size;
  int* err;
  int* hdr;
  double timings[10];
  int host_emit;             /* partition 1 coded on the host (A/B, WEBP_AMD_HOST_EMIT=1) */
  vp8l_engine* l;            /* config->lossless: the VP8L engine (lossy buffers unused) */
};

#ifdef __cplusplus
extern "C" {
#endif
int vp8g_engine_run_yuv(struct WebPGpuBatch* b, int n);
int vp8g_engine_upload_yuv(struct WebPGpuBatch* b, int f, const uint8_t* y, int ys,
                           const uint8_t* u, const uint8_t* v, int uvs, const uint8_t* a,
                           int as);
int vp8g_engine_import(struct WebPGpuBatch* b, const uint8_t* rgba, int stride, uint8_t* y,
                       uint8_t* u, uint8_t* v, uint8_t* a, int* has_alpha, int sharp,
                       float dither);
#ifdef __cplusplus
}
#endif
#endif
