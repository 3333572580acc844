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
 *   ehist     N x 13 x 256 uint32        AnalyzeEntropy histograms (L0)
 *   pal       N x VP8L_PAL_STRIDE uint32 colour count (257 = too many) + colours (L0)
 *   minb      N x npix uint8             smallest cache size holding the pixel (L2)
 *   cseg      N x CACHE_SEGS x CACHE_TAB uint32 pairs   per L2 segment: its last
 *                                        cache contents, then the contents at its start
 *   ops       N x npix uint32            parse: act | (len - 1) << 2 | dist_code << 14 (L3)
 *   prov      N x npix uint16            provisional parse: act | len << 2 (L3)
 *   chist     N x VP8L_CHIST uint32      cache-size choice histograms (L3)
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
#define VP8L_MAX_CACHE_BITS 9      /* largest colour cache (the size is chosen per frame) */
#define VP8L_NEVER_HIT (VP8L_MAX_CACHE_BITS + 1)
#define VP8L_CACHE_TAB ((2 << VP8L_MAX_CACHE_BITS) - 2)   /* entries of all 9 cache sizes */
#define VP8L_CACHE_SEGS 16         /* L2 walks a frame in up to this many segments at once */
#define VP8L_CACHE_PARTIAL 0x80    /* minb from L2: not settled below the size in bits 0-3 */
#define VP8L_CLUSTER_ITERS 6
#define VP8L_MIN_COPY 3
#define VP8L_MAX_LENGTH 4096
#define VP8L_NUM_CAND 4            /* candidate distances: up, left, up-left, up-right */
#define VP8L_GS (256 + 24 + (1 << VP8L_MAX_CACHE_BITS))
#define VP8L_NS (VP8L_GS + 3 * 256 + 40)   /* G | R | B | A | D */
#define VP8L_BLOCK 1024            /* pixels per bit-writer block */
#define VP8L_MAX_HUFF_IMAGE 2600   /* MAX_HUFF_IMAGE_SIZE, src/enc/vp8l_enc.c */
/* per frame: AnalyzeEntropy's 13 histograms (HistoIx order), then the
 * transform search's accumulated histograms: predictor-12 residuals of A, R,
 * G, B and of the sub-green R-G, B-G (VP8L_EH_ACC + 0..5), then the count of
 * fully transparent pixels over the whole picture (VP8L_EH_TRANSP: the
 * histograms skip pixels equal to their left or upper neighbour, so a
 * transparent area leaves no trace in them) */
#define VP8L_EH_ACC 13
#define VP8L_EH_TRANSP (19 * 256)
#define VP8L_EHIST (19 * 256 + 4)
#define VP8L_PAL_STRIDE 260        /* count + up to 256 colours (+ pad) */
#define VP8L_MAX_PALETTE 256
/* cache-size choice histograms per frame: literal channels G,R,B,A per
 * class c = minb (1..NEVER_HIT), cache keys (9 bits) per class 1..9, length
 * prefixes of the provisional copies */
#define VP8L_CH_LIT 0
#define VP8L_CH_KEY (VP8L_NEVER_HIT * 1024)
#define VP8L_CH_LEN (VP8L_CH_KEY + VP8L_MAX_CACHE_BITS * 512)
#define VP8L_CHIST (VP8L_CH_LEN + 24)
/* entropy modes (src/enc/vp8l_enc.c:38-46): bit 0 predictor + cross colour,
 * bit 1 subtract green; 4 = palette (colour indexing) */
#define VP8L_MODE_DIRECT 0
#define VP8L_MODE_SPATIAL 1
#define VP8L_MODE_SUBGREEN 2
#define VP8L_MODE_SPATIAL_SUBGREEN 3
#define VP8L_MODE_PALETTE 4
/* the shortest-path parse of frames without a predictor (direct / subtract
 * green; model: dp_parse): candidate distances, longest copy, cost table
 * (G with 2^MAX_CACHE_BITS cache symbols | R | B | A | D) per frame */
#define VP8L_DP_ENABLED 1   /* oracle/vp8l_model.py: DP_ENABLED */
#define VP8L_DP_NC 32
#define VP8L_DP_MAXK 64
#define VP8L_DP_NG (280 + (1 << VP8L_MAX_CACHE_BITS))
#define VP8L_DP_NCOST (VP8L_DP_NG + 3 * 256 + 40)

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
  int cache_bits;                  /* largest cache size tried (VP8L_MAX_CACHE_BITS),
                                      0 = no colour cache (ALPH mode) */
  int palette;                     /* colour-indexing engine: w = packed width */
  int xbits;                       /* palette bundling (0..3) */
  int ow;                          /* picture width (w is the coded width) */
  int exact;                       /* WebPConfig::exact: no alpha-0 clean-up in the
                                      predictor's residuals */
  int nlq_bits;                    /* predictor near-lossless quantisation
                                      (VP8LNearLosslessBits; 0 = off) */
  int low_effort;                  /* method 0: predictor 11 everywhere, no cross colour */
  int lz;                          /* non-palette engine of repeat-heavy frames: the
                                      cost-model parse over the hash chain, no cache */
} vp8l_params;

/* the engine's table block (tabs): nlogn 0..4096 (int, 1/4096 bit) | log2
 * fractions (1024 int) | VP8LFastSLog2 0..255 (float) | log2 0..255 (float) */
#define VP8L_TAB_FSLOG (4097 + 1024)
#define VP8L_TAB_WORDS (VP8L_TAB_FSLOG + 512)

/* L0: per frame (rgba frames at fstride bytes, rows at rstride) the 13
 * AnalyzeEntropy histograms into ehist (n x VP8L_EHIST, zeroed by the
 * caller) and the colour set into pal (n x VP8L_PAL_STRIDE: count, 257 when
 * it exceeds VP8L_MAX_PALETTE, then the colours in no particular order).
 * plane: the input is ALPH alpha planes (1 byte per pixel, coded as green). */
int vp8l_launch_scan(const uint8_t* rgba, size_t fstride, int rstride, int w, int h, int n,
                     int plane, uint32_t* ehist, uint32_t* pal, void* stream);
/* L0b: the repeat test (oracle/vp8l_model.py: repeat_stats) of n RGBA
 * frames: out[2f] busy sampled windows, out[2f + 1] repeats among them;
 * ystep from vp8l_repeat_ystep. Frames with more than 256 colours that pass
 * it (vp8l_repeat_heavy) take the cost-model parse over the hash chain
 * (vp8l_params::lz). */
#define VP8L_REP_MAX_SAMPLES 16384
#define VP8L_REP_MIN_BUSY 64
#define VP8L_REP_FRAC_DEN 10
int vp8l_launch_repeat(const uint8_t* rgba, size_t fstride, int rstride, int w, int h, int n,
                       int ystep, uint32_t* out, void* stream);
static inline int vp8l_repeat_ystep(int w, int h) {
  const long nx = w >= 8 ? (w - 8) / 16 + 1 : 0;
  int k = 1;
  while (nx * ((h + 4L * k - 1) / (4L * k)) > VP8L_REP_MAX_SAMPLES) ++k;
  return 4 * k;
}
static inline int vp8l_repeat_heavy(const uint32_t* rep) {
  return rep[0] >= VP8L_REP_MIN_BUSY && (uint64_t)VP8L_REP_FRAC_DEN * rep[1] >= rep[0];
}
/* L1: per slot f the input frame fidx[f] (NULL: f); entropy mode fmode[f]
 * (0..3): subtract green (mode & 2), per-tile predictor + cross colour
 * (mode & 1). The predictor: the reference's own choice (L1a) for slots with
 * pexact[f] (their residuals update the picture: near-lossless, alpha-0
 * clean-up) and at method 0, else the cross-entropy choice against the L0
 * histograms ehist of input frame efidx[f] (NULL: f), which also score the
 * cross colour; any_exact: some slot has pexact. tabs: the engine's table
 * block (VP8L_TAB_WORDS). sg_mask: bit 0 some slot without subtract green,
 * bit 1 some with. pflag (n words): per slot 1 when the residuals came from
 * the serial pass. alpha_flag[f] |= 1 if any alpha != 255. */
int vp8l_launch_transform(const uint8_t* rgba, size_t fstride, int rstride,
                          const vp8l_params* p, const int* fidx, const int* efidx,
                          const uint8_t* fmode, const uint32_t* ehist, const int32_t* tabs,
                          int sg_mask, uint32_t* argb, uint8_t* modes, const uint8_t* pexact,
                          int any_exact, uint32_t* pflag, uint32_t* mult, uint32_t* alpha_flag,
                          void* stream);
/* Near-lossless preprocessing (VP8ApplyNearLossless): passes at bits .. 1
 * from frame fidx[f] of rgba into slot f of buf0 / buf1 (n x w*h*4 each,
 * packed RGBA), slots with apply[f] == 0 copied; *out = the buffer holding
 * the last pass. */
int vp8l_launch_near_lossless(const uint8_t* rgba, size_t fstride, int rstride, const int* fidx,
                              const uint8_t* apply, int w, int h, int n, int bits,
                              uint8_t* buf0, uint8_t* buf1, const uint8_t** out, void* stream);
/* L1 (palette engine): colour indexing with bundling. sorted: per slot the
 * palette sorted ascending (VP8L_MAX_PALETTE entries), sidx: the index each
 * sorted colour has in the stored palette, npal: palette sizes. */
int vp8l_launch_palette_apply(const uint8_t* rgba, size_t fstride, int rstride,
                              const vp8l_params* p, const int* fidx, const uint32_t* sorted,
                              const uint8_t* sidx, const int* npal, uint32_t* argb,
                              uint32_t* alpha_flag, void* stream);
/* L2..L5: cache sizes, provisional parse, cache-size choice (cbits[f]),
 * row parse, tile features, clustering. tabs: DEVICE tables (nlogn 4097 |
 * log2 fraction 1024, in 1/4096 bit). */
/* Colour-indexed frames: at most this many code groups (model: KMAX_PALETTE) */
#define VP8L_KMAX_PALETTE 8
/* Colour-indexed frames: buffers of the cost-model parse (L3p kernels) */
#define VP8L_LZ_NCOST (280 + 3 * 256 + 40)
#define VP8L_LZ_HASH_SIZE (1 << 18)
typedef struct {
  uint16_t* runs;              /* n x npix: equal pixels from each position */
  int32_t* htab;               /* n x VP8L_LZ_HASH_SIZE: hash -> last position */
  int32_t* chain;              /* n x npix */
  uint32_t* hoff;              /* n x npix: the chain's best match */
  uint16_t* hlen;
  uint32_t* loff;              /* n x npix: the best of the 4 candidate distances */
  uint16_t* llen;
  int32_t* costs;              /* n x VP8L_LZ_NCOST symbol costs (1/256 bit) */
  int32_t* costs_row;          /* n x VP8L_LZ_NCOST: those of the greedy row parse */
  unsigned long long* est;     /* 2n: the two first parses' bits (row, chain) */
  const uint8_t* dcodes;       /* distance -> plane code for distances < nd (0: none) */
  int nd;
} vp8l_lz;

/* lz != NULL (colour-indexed engines): no colour cache, the greedy parse
 * feeds two rounds of the cost-model parse over the hash chain's and the
 * candidate distances' matches */
/* the shortest-path parse of frames without a predictor (k_vp8l_dp*): the
 * slots' entropy modes (NULL: none of them), VP8L_DP_NC x {distance, rows,
 * columns, code} candidates (host vp8l_dp_candidates) and n x VP8L_DP_NCOST
 * symbol costs of scratch */
typedef struct {
  const uint8_t* fmode;
  const int32_t* cand;
  int ncand;
  int32_t* costs;
} vp8l_dp;
int vp8l_launch_analyze(const uint32_t* argb, const vp8l_params* p, const int32_t* tabs,
                        uint8_t* minb, uint32_t* cseg, uint16_t* prov, uint32_t* chist,
                        uint8_t* cbits,
                        uint32_t* ops, int64_t* feat, uint32_t* tl, uint32_t* tn,
                        uint32_t* hc, uint8_t* assign, const vp8l_lz* lz, const vp8l_dp* dp,
                        void* stream);
/* L6/L7: per-block bit counts, per-frame scan from start_bit[f], and the
 * bit writer into out (n x out_cap bytes, zeroed except the header words the
 * host placed at the start). end_bit[f] = total payload bits. */
int vp8l_launch_write(const uint32_t* argb, const uint32_t* ops,
                      const vp8l_params* p, const uint8_t* cbits, const uint32_t* ctab,
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
