/* Host side of the lossless (VP8L) path: Huffman codes, the bitstream
 * header (transforms, colour cache, meta codes, code lengths) and the RIFF
 * container. The choices mirror oracle/vp8l_model.py; the format is the
 * reference decoder's (src/dec/vp8l_dec.c). */
#ifndef LIBWEBP_AMD_VP8L_HOST_H_
#define LIBWEBP_AMD_VP8L_HOST_H_

#include <stddef.h>
#include <stdint.h>

#include "../vp8l_gpu.h"

typedef struct {
  uint8_t* buf;
  size_t cap, pos;     /* bytes */
  uint64_t acc;
  int used;            /* bits in acc */
  uint64_t nbits;      /* total bits written */
  int oom;
} vp8l_bw;

void vp8l_bw_init(vp8l_bw* bw, size_t cap);
void vp8l_bw_free(vp8l_bw* bw);
void vp8l_bw_put(vp8l_bw* bw, uint32_t v, int nbits);
/* flush the partial byte (zero padded); returns the byte count */
size_t vp8l_bw_finish(vp8l_bw* bw);

/* GetHistoBits / GetTransformBits (src/enc/vp8l_enc.c:234-253), no palette */
int vp8l_histo_bits(int method, int w, int h);
int vp8l_transform_bits(int method, int histo_bits);
int vp8l_histo_bits_palette(int method, int w, int h);
void vp8l_setup_params_palette_hb(vp8l_params* p, int w, int h, int n, int method, int alpha);
/* candidate distances and their codes (model: candidate_distances,
 * distance_code); alpha != 0: the ALPH-chunk form (model: alpha_plane) */
void vp8l_setup_params(vp8l_params* p, int w, int h, int n, int method, int alpha);
/* the colour-indexing engine for w x h pictures bundled by xbits (alpha:
 * ALPH planes) */
void vp8l_setup_palette_params(vp8l_params* p, int w, int h, int n, int method, int xbits,
                               int alpha);

/* model: bits_entropy_fx / entropy_choice -- the entropy mode (0..4,
 * VP8L_MODE_*) from the 13 AnalyzeEntropy histograms; npal = colours when
 * they fit a palette, else 0; ntiles = transform tiles */
int64_t vp8l_bits_entropy_fx(const uint32_t* h, int n);
int vp8l_entropy_choice(const uint32_t* ehist, int npal, int ntiles);
/* model: minimize_deltas -- palette sorted, then reordered in place */
void vp8l_palette_order(uint32_t* pal, int n);

/* nlogn table (4097 entries, round(n log2 n * 4096)) and the log2 fraction
 * table (1024 entries) uploaded to the device */
const int32_t* vp8l_nlogn_table(void);
const int32_t* vp8l_flog2_table(void);
const float* vp8l_float_tables(void);   /* 512 floats: VP8LFastSLog2, log2 of 0..255 */

/* Per-frame header. Inputs: the entropy mode (transforms written), the
 * frame's colour-cache bits, the palette in stored order (palette engine);
 * from the device: predictor modes and colour multipliers per transform tile
 * (spatial modes), cluster histograms hc (KMAX x NS) and the cluster of each
 * histogram tile. Outputs: the header bits (bw), the code table ctab (KMAX x
 * NS: code | bits << 16) and the code group of each histogram tile (gtile).
 * Returns 0 on allocation failure. */
int vp8l_build_header(const vp8l_params* p, int has_alpha, int emode, int cache_bits,
                      const uint32_t* palette, int npal, const uint8_t* modes,
                      const uint32_t* mult, const uint32_t* hc, const uint8_t* assign,
                      vp8l_bw* bw, uint32_t* ctab, uint8_t* gtile);

/* distance -> smallest plane code table for width w (NULL: size only) */
int vp8l_plane_dcodes(int w, uint8_t* tab);
int vp8l_dp_candidates(int w, int32_t* out);   /* VP8L_DP_NC x {d, dy, dx, dcode} */

/* RIFF + "VP8L" chunk header for a payload of `size` bytes (20 bytes) */
void vp8l_riff_header(uint8_t out[20], size_t size);

#endif /* LIBWEBP_AMD_VP8L_HOST_H_ */
