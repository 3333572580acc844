/* Lossless (VP8L) batch: layouts shared by the host C engine
 * (host/vp8l_batch.c, host/vp8l_host.c) and the HIP kernels
 * (hip/vp8l_kernels.hip). The algorithm is stated in oracle/vp8l_model.py;
 * the format is the reference decoder's (src/dec/vp8l_dec.c).
 *
 * HBM layout per batch (N frames of W x H, npix = W*H):
 *   rgba      N x (row_stride * H)       caller-owned input
 *   argb      N x npix uint32            residual image after subtract-green,
 *                                        predictor and cross-colour (L1)
 *   modes     N x ntt  uint8             predictor mode per transform tile
 *   mult      N x ntt  uint32            g2r | g2b << 8 | r2b << 16
 *   hits      N x ceil(npix/64) uint64   colour-cache hit bit per pixel (L2)
 *   ops       N x npix uint32            parse: act | len << 2 | dist_code << 15 (L3)
 *   feat      N x nht  int64             histogram-tile entropy feature (L4)
 *   tl / tn   N x nht x tile_cap uint32  sparse tile histograms: symbol | count << 12,
 *             N x nht uint32             and their lengths (L4)
 *   hc        N x KMAX x NS uint32       cluster histograms (L5)
 *   assign    N x nht  uint8             cluster per histogram tile (L5)
 *   ctab      N x KMAX x NS uint32       code | bits << 16 per group/symbol (host)
 *   gtile     N x nht  uint8             code group per histogram tile (host)
 *   bsum/boff N x nblk                   per-1024-pixel-block bits / offsets (L6)
 *   out       N x out_cap bytes          VP8L payload: host header words, then
 *                                        the pixel data bits (L7)
 */
#ifndef LIBWEBP_AMD_VP8L_GPU_H_
#define LIBWEBP_AMD_VP8L_GPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VP8L_KMAX 16               /* max code groups (clusters) per frame */
#define VP8L_CACHE_BITS 8          /* colour cache size (fixed) */
#define VP8L_CLUSTER_ITERS 6
#define VP8L_MIN_COPY 3
#define VP8L_MAX_LENGTH 4096
#define VP8L_NUM_CAND 4            /* candidate distances: up, left, up-left, up-right */
#define VP8L_GS (256 + 24 + (1 << VP8L_CACHE_BITS))
#define VP8L_NS (VP8L_GS + 3 * 256 + 40)   /* G | R | B | A | D */
#define VP8L_BLOCK 1024            /* pixels per bit-writer block */
#define VP8L_MAX_HUFF_IMAGE 2600   /* MAX_HUFF_IMAGE_SIZE, src/enc/vp8l_enc.c */

/* entries of one sparse tile histogram: at most NS symbols, at most 4 per
 * pixel of a (1 << hb)^2 tile */
#define VP8L_TILE_CAP(hb) \
  ((((size_t)4 << (2 * (hb))) < (size_t)VP8L_NS) ? ((size_t)4 << (2 * (hb))) : (size_t)VP8L_NS)

typedef struct {
  int w, h, n;
  int tb, hb;                      /* transform / histogram tile bits */
  int k;                           /* clusters = min(KMAX, nht) */
  int dist[VP8L_NUM_CAND];         /* candidate distances (0 = unused) */
  int dcode[VP8L_NUM_CAND];        /* their distance codes */
  int alpha;                       /* ALPH mode: input is an alpha plane (1 B/px,
                                      coded as green), bare stream (no image
                                      header), no subtract green, no colour cache */
  int cache_bits;                  /* VP8L_CACHE_BITS, or 0 in ALPH mode */
} vp8l_params;

/* L1: subtract green + per-tile predictor + cross colour. rgba frames at
 * fstride bytes, rows at rstride bytes. alpha_flag[f] |= 1 if any alpha
 * != 255. */
int vp8l_launch_transform(const uint8_t* rgba, size_t fstride, int rstride,
                          const vp8l_params* p,
                          uint32_t* argb, uint8_t* modes, uint32_t* mult,
                          uint32_t* alpha_flag, void* stream);
/* L2..L5: cache hits, row parse, tile features, clustering. flog2: DEVICE
 * table (1024 entries) of the fraction of log2 in 1/4096 bit. */
int vp8l_launch_analyze(const uint32_t* argb, const vp8l_params* p,
                        const int32_t* flog2, uint64_t* hits, uint32_t* ops,
                        int64_t* feat, uint32_t* tl, uint32_t* tn, uint32_t* hc,
                        uint8_t* assign, void* stream);
/* L6/L7: per-block bit counts, per-frame scan from start_bit[f], and the
 * bit writer into out (n x out_cap bytes, zeroed except the header words the
 * host placed at the start). end_bit[f] = total payload bits. */
int vp8l_launch_write(const uint32_t* argb, const uint32_t* ops,
                      const vp8l_params* p, const uint32_t* ctab,
                      const uint8_t* gtile, const uint64_t* start_bit,
                      uint32_t* bsum, uint64_t* boff, uint64_t* end_bit,
                      uint8_t* out, size_t out_cap, void* stream);

/* staging: headers packed at 4-byte aligned offsets hoff (hwords words each)
 * into the slabs; payloads into one buffer at poff[f] + 20 (16-aligned). */
int vp8l_launch_put_headers(const uint32_t* hdr, const uint64_t* hoff,
                            const uint32_t* hwords, int n, uint8_t* out,
                            size_t out_cap, void* stream);
int vp8l_launch_pack(const uint8_t* out, size_t out_cap, const uint64_t* poff,
                     const uint64_t* end_bit, int n, uint8_t* packed, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* LIBWEBP_AMD_VP8L_GPU_H_ */
