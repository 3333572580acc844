// Lossless (VP8L) encoder kernels for gfx950. The decisions are stated in
// oracle/vp8l_model.py (same names); the bitstream format is the reference
// decoder's (src/dec/vp8l_dec.c, src/dsp/lossless.c). All integer work:
// HBM/LDS bound, no MFMA.
//
//   L0 k_vp8l_entropy    AnalyzeEntropy's 13 histograms per frame (row bands,
//                        LDS histograms, one global add per bin)
//      k_vp8l_palscan    one workgroup per frame: the colour set in an LDS hash
//                        table, out as soon as it exceeds 256 colours
//   L1a k_vp8l_predsel   one workgroup per frame: the reference's predictor
//                        choice exactly (serial over tiles, float entropy)
//      k_vp8l_resid_serial  one wave per frame: residuals where near-lossless
//                        / alpha-0 clean-up update the picture (wavefront)
//   L1 k_vp8l_transform  one workgroup per L1_TILES transform tiles: subtract
//                        green, the chosen predictor's residuals and the
//                        cross-colour multipliers (a descent over parallel
//                        candidate steps) scored by entropy against the
//                        frame's L0 histograms; residual ARGB to HBM -- or the
//                        plain (sub-green) pixels for the non-spatial modes
//      k_vp8l_palapply   colour indexing: binary search in the sorted palette,
//                        2^xbits indices bundled per packed pixel
//   L2 k_vp8l_cache      one wave per frame segment, 64 pixels per step: per
//                        pixel the smallest cache size (1..9 bits) holding it;
//                        same-key lanes found with one ballot per key bit, MSB
//                        first; k_vp8l_cache_start chains the segments
//   L3 k_vp8l_match      one wave per row: best candidate run per pixel (ballots)
//      k_vp8l_parse      one thread per row: greedy copy / cache / literal
//                        (once with every hit of the largest cache, then with
//                        the frame's chosen size)
//      k_vp8l_cachehist / k_vp8l_cachechoose  the cache size of each frame
//                        from the provisional parse
//   L4 k_vp8l_tilefeat   one workgroup per histogram tile: own entropy/pixel
//   L5 k_vp8l_cluster    one workgroup per frame: k-means of histogram tiles
//                        into <= KMAX code groups (histograms + costs in LDS)
//   L6 k_vp8l_bitcount / k_vp8l_scan   bits per 1024-pixel block, offsets
//   L7 k_vp8l_write      one workgroup per block: fields into LDS words,
//                        interior words stored, the two edge words OR-ed
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../vp8l_gpu.h"

#define HASH_MUL 0x1e35a7bdu

namespace {

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// histogram add with a fast path for the wave-uniform case (flat areas put
// every lane on one bin; LDS atomics on one address serialise)
__device__ __forceinline__ void hadd(uint32_t* h, uint32_t idx) {
  const uint64_t act = __ballot(1);
  const uint32_t first = __builtin_amdgcn_readfirstlane(idx);
  const uint64_t same = __ballot(idx == first);
  if (same == act) {
    if (lane_id() == __ffsll((long long)act) - 1) atomicAdd(&h[first], (uint32_t)__popcll(act));
  } else {
    atomicAdd(&h[idx], 1u);
  }
}

__device__ __forceinline__ uint32_t avg2(uint32_t a, uint32_t b) {
  return (((a ^ b) & 0xfefefefeu) >> 1) + (a & b);
}
__device__ __forceinline__ int clip255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }
__device__ __forceinline__ int ch(uint32_t v, int s) { return (int)((v >> s) & 255); }

// src/dsp/lossless.c:103-180
__device__ __forceinline__ uint32_t predict(int m, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
  switch (m) {
    case 0: return 0xff000000u;
    case 1: return L;
    case 2: return T;
    case 3: return TR;
    case 4: return TL;
    case 5: return avg2(avg2(L, TR), T);
    case 6: return avg2(L, TL);
    case 7: return avg2(L, T);
    case 8: return avg2(TL, T);
    case 9: return avg2(T, TR);
    case 10: return avg2(avg2(L, TL), avg2(T, TR));
    case 11: {
      int s = 0;
      for (int k = 0; k < 32; k += 8) s += abs(ch(L, k) - ch(TL, k)) - abs(ch(T, k) - ch(TL, k));
      return s <= 0 ? T : L;
    }
    case 12: {
      uint32_t o = 0;
      for (int k = 0; k < 32; k += 8)
        o |= (uint32_t)clip255(ch(L, k) + ch(T, k) - ch(TL, k)) << k;
      return o;
    }
    default: {
      const uint32_t a = avg2(L, T);
      uint32_t o = 0;
      for (int k = 0; k < 32; k += 8) {
        const int x = ch(a, k) - ch(TL, k);
        o |= (uint32_t)clip255(ch(a, k) + x / 2) << k;   // C division truncates
      }
      return o;
    }
  }
}

__device__ __forceinline__ uint32_t sub_pixels(uint32_t a, uint32_t b) {
  // per-channel (a - b) & 255
  const uint32_t ag = (a | 0x00ff00ffu) - (b & 0xff00ff00u);
  const uint32_t rb = (a | 0xff00ff00u) - (b & 0x00ff00ffu);
  return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}

// (A, R-G, G, B-G) of a pixel (subtract green, src/dsp/lossless_enc.c)
__device__ __forceinline__ uint32_t sub_green(uint32_t v) {
  const uint32_t g = (v >> 8) & 255;
  return (v & 0xff00ff00u) | ((((v >> 16) - g) & 255) << 16) | (((v & 255) - g) & 255);
}

__device__ __forceinline__ int s8(int v) { return (int)(int8_t)(uint8_t)v; }
__device__ __forceinline__ int ctd(int t, int c) { return (t * s8(c)) >> 5; }

// block-wide sums through LDS atomics (T threads, wave reductions first)
template <typename V>
__device__ __forceinline__ V wave_sum(V v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

}  // namespace

// Phase cycle accounting only in the diagnostic build (-DVP8L_PS_PROF,
// libwebp_amd_prof.so; vp8l_prof_phase_cycles): workgroup thread 0 adds the
// shader-clock delta of each phase to a device-global counter.
#ifdef VP8L_PS_PROF
__device__ unsigned long long g_vp8l_prof[16];
#define PS_STAMP(i)                                                          \
  do {                                                                      \
    if (threadIdx.x == 0) {                                                 \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();           \
      atomicAdd(&g_vp8l_prof[i], t_ - ps_t);                                \
      ps_t = t_;                                                            \
    }                                                                       \
  } while (0)
#define PS_STAMP_INIT unsigned long long ps_t = __builtin_amdgcn_s_memtime()
#define PS_PARAM , unsigned long long& ps_t
#define PS_ARG , ps_t
#else
#define PS_PARAM
#define PS_ARG
#define PS_STAMP(i) \
  do {              \
  } while (0)
#define PS_STAMP_INIT
#endif

// ------------------------------------------------------------------ L1

// The tile's residuals under the predictor L1a chose, then the cross-colour
// search (model: choose_cross_color, oracle/vp8l_model.py): every candidate
// is scored by
//   cost = 16 * sum_i t_i SP[i] - sum_{i: t_i > 0} [slog(t_i) + slog(t_i + G_i) - slog(G_i)]
// (1/4096 bit) over the tile's residual histograms t against the frame's
// accumulated histograms G (L0's residuals against the raster predecessor).
// SP: PredictionCostSpatial (src/enc/predictor_enc.c:35-46) per value.
__constant__ int8_t kSpCC[16] = {-77, -61, -37, -22, -13, -8, -5, -3, -2, -1, -1, 0, 0, 0, 0, 0};
__device__ __forceinline__ int sp_of(const int8_t* tab, int v) {
  const int k = v < 128 ? v : 256 - v;   // symmetric in +-k
  return k < 16 ? tab[k] : 0;
}

#define CC_ZERO_BONUS (3ll << 12)
#define L1_TILES 4   // transform tiles per workgroup (the per-frame setup is shared)

template <int T>
struct TransformSmem {
  union {
    uint32_t src[(T + 1) * (T + 2)];   // rows y0-1.., cols x0-1..x0+tw (until the residuals)
    uint32_t h9[8 * 128];              // colour search: up to 8 candidates, u16 counts
  } u;
  uint32_t first[T];                 // P(0, y) for the right-edge TR wrap
  uint32_t res[T * T];               // the chosen predictor's residuals
  int32_t frac[1024];                // log2 fraction table (model: FLOG2_FRAC)
  int32_t cost[2][8];                // colour-search step sums, alternate steps alternate rows
  int32_t ct[4][256];                // cross-entropy cost per channel and residual (model: ce_tables)
  int32_t slogt[T * T + 1];          // slog(t) for the counts a tile can have
  int32_t pcost[16];                 // the tile's cross-entropy cost per predictor
  uint32_t nsum[4];
  int best;
};

// log2(v) in 1/4096 bit for v >= 1 (model: flog2)
__device__ __forceinline__ int flog2_fx(const int32_t* frac, uint32_t v) {
  const int e = 31 - __clz((int)v);
  const uint32_t m = (e >= 10 ? (v >> (e - 10)) : (v << (10 - e))) & 1023;
  return (e << 12) + frac[m];
}

// v * log2(v) in 1/4096 bit, 0 for v <= 1 (model: slog2_fx)
__device__ __forceinline__ long long slog_fx(const int32_t* frac, uint32_t v) {
  if (v <= 1) return 0;
  const int e = 31 - __clz((int)v);
  const uint32_t m = (e >= 10 ? (v >> (e - 10)) : (v << (10 - e))) & 1023;
  return (long long)v * (((long long)e << 12) + frac[m]);
}

// block-wide sums of K values into cost[0..K) (zeroed beforehand)
template <int K>
__device__ __forceinline__ void reduce_costs(int32_t* cost, const int32_t (&v)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int32_t w = wave_sum(v[k]);
    if (lane_id() == 0) atomicAdd(&cost[k], w);
  }
}

// what thread b = value b brings to every candidate evaluation: the frame's
// R and B counts G, slog(G) and PredictionCostSpatial of the value
struct CcBin {
  uint32_t g[2];
  long long sg[2];
  int spv;
};

// The bin side of one candidate evaluation: thread b owns value b of each of
// the K histograms (u16 pairs in h) against channel ch (0: R, 1: B) of G, and
// zeroes the words it read for the next step (their other reader is the
// neighbouring lane of the same wave, whose reads are issued with these).
// Every term fits 32 bits (t <= 4096: slog(t) < 2^28, slog(t + g) - slog(g) ~
// t log2(t + g)), and so does a candidate's sum over the bins (< 2^29 at 4096
// pixels).
template <int K, int T>
__device__ __forceinline__ void bin_costs(TransformSmem<T>& S, uint32_t* h, int chn,
                                          const CcBin& cb, int32_t (&acc)[K]) {
  const int b = threadIdx.x;   // 256 threads = 256 values
  const uint32_t gv = cb.g[chn];
  const long long sg = cb.sg[chn];
  uint32_t w[K];
#pragma unroll
  for (int k = 0; k < K; ++k) w[k] = h[k * 128 + (b >> 1)];
#pragma unroll
  for (int k = 0; k < K; ++k) h[k * 128 + (b >> 1)] = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t t = (w[k] >> ((b & 1) * 16)) & 0xffffu;
    if (t)
      acc[k] += 16 * (int32_t)t * cb.spv - (S.slogt[t] + (int32_t)(slog_fx(S.frac, t + gv) - sg));
  }
}

__device__ __forceinline__ void hist_add(uint32_t* h, int v) {
  atomicAdd(&h[v >> 1], 1u << ((v & 1) * 16));
}

// register fields of the histogram counts (count_res below): five 11-bit
// fields (values -2..2) up to 32 x 32 tiles, four 13-bit ones (-1..2) for
// 64 x 64 -- wide enough for a whole wave's sum over a tile of one value
template <int T>
struct Hot {
  static constexpr int NH = T >= 64 ? 4 : 5, FB = T >= 64 ? 13 : 11, OFF = T >= 64 ? 1 : 2;
  static constexpr uint32_t MASK = (1u << FB) - 1;
  __device__ static int slot(int v) { return (v + OFF) & 255; }   // < NH: a register field
  __device__ static int value(int j) { return (j - OFF) & 255; }
};

// one colour-search step: the costs of KR green-to-red candidates r0[] and
// KB (green-to-blue, red-to-blue) candidates (b0[], b1[]) -- the two
// descents are independent (the blue one reads the untransformed red), so
// their steps share an evaluation
// Entry: S.u.h9 all zero, S.cost[par] zero; exit: the same for the next step
// (par ^ 1), after two block barriers.
template <int KR, int KB, int T>
__device__ void cc_eval(TransformSmem<T>& S, int np, const CcBin& cb, int& par,
                        const int (&r0)[KR > 0 ? KR : 1],
                        const int (&b0)[KB > 0 ? KB : 1], const int (&b1)[KB > 0 ? KB : 1],
                        long long (&outR)[KR > 0 ? KR : 1], long long (&outB)[KB > 0 ? KB : 1]
                        PS_PARAM) {
  constexpr int K = KR + KB;
  const int tid = threadIdx.x;
  PS_STAMP(11);
  // every thread takes every 256th pixel of the tile for all K candidates:
  // the values next to 0 -- most of a good multiplier's residuals -- counted
  // in packed register fields and summed over the wave once (lane k * NH + j
  // adds field j of candidate k), the rest by LDS atomics (same-bin atomics
  // of a wave serialise)
  uint64_t hot[K];
#pragma unroll
  for (int k = 0; k < K; ++k) hot[k] = 0;
  for (int i = tid; i < np; i += 256) {
    const uint32_t r = S.res[i];
    const int g = ch(r, 8), rr = ch(r, 16), bb = ch(r, 0);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int v = k >= KR ? (bb - ctd(b0[k - KR], g) - ctd(b1[k - KR], rr)) & 255
                            : (rr - ctd(r0[k], g)) & 255;
      const int q = Hot<T>::slot(v);
      hot[k] += q < Hot<T>::NH ? (1ull << (Hot<T>::FB * q)) : 0ull;
      if (q >= Hot<T>::NH) hist_add(S.u.h9 + k * 128, v);
    }
  }
  {
    const int lane = lane_id(), kk = lane / Hot<T>::NH, j = lane - kk * Hot<T>::NH;
    uint64_t mine = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t t = wave_sum(hot[k]);
      if (k == kk) mine = t;
    }
    if (kk < K) {
      const uint32_t t = (uint32_t)(mine >> (Hot<T>::FB * j)) & Hot<T>::MASK;
      const int v = Hot<T>::value(j);
      if (t) atomicAdd(&S.u.h9[kk * 128 + (v >> 1)], t << ((v & 1) * 16));
    }
  }
  __syncthreads();
  PS_STAMP(12);
  // the previous step's sums were read before the barrier above
  if (tid < 8) S.cost[par ^ 1][tid] = 0;
  int32_t acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0;
  if constexpr (KR > 0) {
    int32_t a[KR];
#pragma unroll
    for (int k = 0; k < KR; ++k) a[k] = 0;
    bin_costs<KR>(S, S.u.h9, 0, cb, a);
#pragma unroll
    for (int k = 0; k < KR; ++k) acc[k] = a[k];
  }
  if constexpr (KB > 0) {
    int32_t a[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) a[k] = 0;
    bin_costs<KB>(S, S.u.h9 + KR * 128, 1, cb, a);
#pragma unroll
    for (int k = 0; k < KB; ++k) acc[KR + k] = a[k];
  }
  reduce_costs<K>(S.cost[par], acc);
  __syncthreads();
  PS_STAMP(13);
#pragma unroll
  for (int k = 0; k < KR; ++k) outR[k] = (long long)S.cost[par][k] - CC_ZERO_BONUS * (r0[k] == 0);
#pragma unroll
  for (int k = 0; k < KB; ++k)
    outB[k] = (long long)S.cost[par][KR + k] - CC_ZERO_BONUS * ((b0[k] == 0) + (b1[k] == 0));
  par ^= 1;
}

// SG: the subtract-green instantiation; a launch of each covers every slot,
// the blocks of slots with the other flag leave at once (a runtime flag
// costs the spatial search registers and occupancy)
template <int T, bool SG>
__global__ __launch_bounds__(256) void k_vp8l_transform(const uint8_t* __restrict__ rgba,
                                                        size_t fstride, int rstride, vp8l_params p,
                                                        const int* __restrict__ fidx,
                                                        const int* __restrict__ efidx,
                                                        const uint8_t* __restrict__ fmode,
                                                        const uint32_t* __restrict__ ehist,
                                                        const int32_t* __restrict__ frac_tab,
                                                        uint8_t* __restrict__ modes,
                                                        const uint32_t* __restrict__ pflag,
                                                        const uint8_t* __restrict__ pexact,
                                                        uint32_t* __restrict__ argb_out,
                                                        uint32_t* __restrict__ mult,
                                                        uint32_t* __restrict__ alpha_flag) {
  __shared__ TransformSmem<T> S;
  const int tid = threadIdx.x, f = blockIdx.z;
  const int W = p.w, H = p.h;
  const uint8_t* img = rgba + (size_t)(fidx ? fidx[f] : f) * fstride;
  const int tiles_x = (W + T - 1) / T, tiles_y = (H + T - 1) / T, ntt = tiles_x * tiles_y;
  const int emode = fmode ? (int)fmode[f] : VP8L_MODE_SPATIAL;
  constexpr bool subgreen = SG;
  if (((emode & VP8L_MODE_SUBGREEN) != 0) != SG) return;
  const int tile0 = blockIdx.x * L1_TILES;

  if (!(emode & VP8L_MODE_SPATIAL)) {   // direct / subtract green only: no predictor
    bool any_alpha = false;
    uint32_t* out = argb_out + (size_t)f * W * H;
    for (int tile = tile0; tile < min(tile0 + L1_TILES, ntt); ++tile) {
      const int x0 = (tile % tiles_x) * T, y0 = (tile / tiles_x) * T;
      const int tw = min(T, W - x0), th = min(T, H - y0);
      for (int i = tid; i < tw * th; i += 256) {
        const int ly = i / tw, lx = i - ly * tw;
        uint32_t v;
        if (p.alpha) {   // ALPH: the alpha plane as green
          const uint32_t g = img[(size_t)(y0 + ly) * rstride + x0 + lx];
          v = subgreen ? (((0u - g) & 255) << 16) | (g << 8) | ((0u - g) & 255) : g << 8;
        } else {
          const uint8_t* q = img + (size_t)(y0 + ly) * rstride + 4 * (x0 + lx);
          const uint32_t r = q[0], g = q[1], b = q[2], a = q[3];
          any_alpha |= a != 255;
          v = subgreen ? (a << 24) | (((r - g) & 255) << 16) | (g << 8) | ((b - g) & 255)
                       : (a << 24) | (r << 16) | (g << 8) | b;
        }
        out[(size_t)(y0 + ly) * W + x0 + lx] = v;
      }
    }
    if (__any(any_alpha) && lane_id() == 0) atomicOr(&alpha_flag[f], 1u);
    return;
  }

  CcBin cb;   // thread tid = value tid of the colour search's histograms
  // per-frame setup: the accumulated histograms (L0's predictor-12 residual
  // histograms of the input frame, plain or sub-green) and their slog, the
  // log2 fraction table
  {
    const uint32_t* eh = ehist + (size_t)(efidx ? efidx[f] : f) * VP8L_EHIST;
    const int hix[4] = {VP8L_EH_ACC + 0, VP8L_EH_ACC + (SG ? 4 : 1), VP8L_EH_ACC + 2,
                        VP8L_EH_ACC + (SG ? 5 : 3)};
    for (int i = tid; i < 1024; i += 256) S.frac[i] = frac_tab[i];
    __syncthreads();
    for (int i = tid; i <= T * T; i += 256) S.slogt[i] = (int32_t)slog_fx(S.frac, (uint32_t)i);
    if (tid < 4) S.nsum[tid] = 0;
    __syncthreads();
    uint32_t gv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      gv[c] = eh[hix[c] * 256 + tid];
      if (c & 1) {
        cb.g[c >> 1] = gv[c];
        cb.sg[c >> 1] = slog_fx(S.frac, gv[c]);
      }
      const uint32_t t = wave_sum(gv[c]);
      if (lane_id() == 0) atomicAdd(&S.nsum[c], t);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c)   // model: ce_tables
      S.ct[c][tid] = flog2_fx(S.frac, 2 * S.nsum[c] + 256) - flog2_fx(S.frac, 2 * gv[c] + 1);
  }
  const bool own_pred = !p.low_effort && !(pexact && pexact[f]);   // else L1a's choice
  cb.spv = sp_of(kSpCC, tid);

  PS_STAMP_INIT;
  for (int tile = tile0; tile < min(tile0 + L1_TILES, ntt); ++tile) {
    const int x0 = (tile % tiles_x) * T, y0 = (tile / tiles_x) * T;
    const int tw = min(T, W - x0), th = min(T, H - y0);
    const int sw = tw + 2;   // LDS source row width (cols x0-1 .. x0+tw)
    __syncthreads();         // the previous tile is done with S
    // load sub-green pixels (A, R-G, G, B-G) with a 1-pixel border
    bool tile_alpha = false, opaque = true;   // opaque: every real pixel loaded has A 255
    for (int i = tid; i < (th + 1) * sw; i += 256) {
      const int ly = i / sw, lx = i - ly * sw;
      const int y = y0 - 1 + ly, x = x0 - 1 + lx;
      uint32_t v = 0;
      if (y >= 0 && x >= 0 && x < W) {
        if (p.alpha) {   // ALPH: the alpha plane as green
          const uint32_t g = img[(size_t)y * rstride + x];
          v = subgreen ? (((0u - g) & 255) << 16) | (g << 8) | ((0u - g) & 255) : g << 8;
        } else {
          const uint8_t* q = img + (size_t)y * rstride + 4 * x;
          const uint32_t r = q[0], g = q[1], b = q[2], a = q[3];
          v = subgreen ? (a << 24) | (((r - g) & 255) << 16) | (g << 8) | ((b - g) & 255)
                       : (a << 24) | (r << 16) | (g << 8) | b;
          if (a != 255 && ly > 0 && lx > 0 && lx <= tw) tile_alpha = true;
          opaque &= a == 255;
        }
      }
      if (p.alpha) opaque = false;
      S.u.src[i] = v;
    }
    if (x0 + tw == W) {
      for (int i = tid; i < th; i += 256) {
        const uint8_t* q = img + (size_t)(y0 + i) * rstride;
        if (p.alpha) {
          const uint32_t g = q[0];
          S.first[i] = subgreen ? (((0u - g) & 255) << 16) | (g << 8) | ((0u - g) & 255) : g << 8;
        } else {
          const uint32_t r = q[0], g = q[1], b = q[2], a = q[3];
          S.first[i] = subgreen ? (a << 24) | (((r - g) & 255) << 16) | (g << 8) | ((b - g) & 255)
                                : (a << 24) | (r << 16) | (g << 8) | b;
          opaque &= a == 255;
        }
      }
    }
    if (__any(tile_alpha) && lane_id() == 0) atomicOr(&alpha_flag[f], 1u);
    opaque = __syncthreads_and(opaque);
    PS_STAMP(6);

    auto at = [&](int lx, int ly) -> uint32_t { return S.u.src[(ly + 1) * sw + lx + 1]; };
    auto tr = [&](int lx, int ly) -> uint32_t {   // (y-1)*W + x + 1, linear
      return (x0 + lx + 1 < W) ? at(lx + 1, ly - 1) : S.first[ly];
    };
    const int np = tw * th;
    // fixed predictors: (0,0) black, row 0 left, column 0 top (lossless.c:219-239)
    auto fixed_mode = [&](int x, int y) -> int { return y == 0 ? (x == 0 ? 0 : 1) : (x == 0 ? 2 : -1); };
    // the tile's predictor (L1a, the reference's choice) and its residuals:
    // computed here, or, where GetResidual updated the picture (pflag), the
    // serial pass's
    int best;
    if (own_pred) {
      // the cross-entropy choice (model: choose_predictors_ce): every thread
      // sums the 14 predictors' costs over its pixels, then wave sums. The
      // fixed-predictor pixels (frame row 0 / column 0) add one cost to every
      // mode, which leaves the first minimum where it is: skipped. Where every
      // pixel is opaque, every residual alpha is 0: skipped likewise.
      if (tid < 16) S.pcost[tid] = 0;
      __syncthreads();   // pcost zeroed
      int32_t pc[14];
#pragma unroll
      for (int m = 0; m < 14; ++m) pc[m] = 0;
      auto ce_sum = [&](auto opq) {
        for (int i = tid; i < np; i += 256) {
          const int ly = i / tw, lx = i - ly * tw;
          if (fixed_mode(x0 + lx, y0 + ly) >= 0) continue;
          const uint32_t P = at(lx, ly), L = at(lx - 1, ly), T_ = at(lx, ly - 1);
          const uint32_t TL = at(lx - 1, ly - 1), TR = tr(lx, ly);
#pragma unroll
          for (int m = 0; m < 14; ++m) {
            const uint32_t r = sub_pixels(P, predict(m, L, T_, TL, TR));
            pc[m] += (decltype(opq)::value ? 0 : S.ct[0][r >> 24]) + S.ct[1][ch(r, 16)] +
                     S.ct[2][ch(r, 8)] + S.ct[3][ch(r, 0)];
          }
        }
      };
      if (opaque) ce_sum(std::true_type{});
      else ce_sum(std::false_type{});
#pragma unroll
      for (int m = 0; m < 14; ++m) {
        const int32_t t = wave_sum(pc[m]);
        if (lane_id() == 0) atomicAdd(&S.pcost[m], t);
      }
      __syncthreads();
      best = 0;
#pragma unroll
      for (int m = 1; m < 14; ++m)
        if (S.pcost[m] < S.pcost[best]) best = m;
      if (tid == 0) modes[(size_t)f * ntt + tile] = (uint8_t)best;
    } else {
      best = modes[(size_t)f * ntt + tile];
    }
    PS_STAMP(7);
    uint32_t* out = argb_out + (size_t)f * W * H;
    if (pflag[f]) {
      for (int i = tid; i < np; i += 256) {
        const int ly = i / tw, lx = i - ly * tw;
        S.res[i] = out[(size_t)(y0 + ly) * W + x0 + lx];
      }
    } else {
      for (int i = tid; i < np; i += 256) {
        const int ly = i / tw, lx = i - ly * tw;
        const int fm = fixed_mode(x0 + lx, y0 + ly);
        S.res[i] = sub_pixels(at(lx, ly), predict(fm >= 0 ? fm : best, at(lx - 1, ly),
                                                       at(lx, ly - 1), at(lx - 1, ly - 1), tr(lx, ly)));
      }
    }
    __syncthreads();   // every source pixel read before the colour search reuses its LDS
    PS_STAMP(8);
    int par = 0;
    if (!p.low_effort) {
      for (int i = tid; i < 8 * 128; i += 256) S.u.h9[i] = 0;
      if (tid < 8) S.cost[0][tid] = 0;
      __syncthreads();
    }
    // colour search (model: choose_cross_color); none at method 0 (vp8l_enc.c:1525-1526)
    int g2r = 0, g2b = 0, r2b = 0;
    if (!p.low_effort) {
      // green-to-red: start 0, then +-32, 16, .., 1 around the best;
      // (green-to-blue, red-to-blue): start (0, 0), then the 4 axis steps at
      // deltas 16, 16, 8, 4, 2, 2, 2 (stopping once a delta-2 step leaves
      // both at 0); step i of both in one evaluation
      const int ax0[4] = {0, 0, -1, 1}, ax1[4] = {-1, 1, 0, 0};
      const int bdel[7] = {16, 16, 8, 4, 2, 2, 2};
      long long bestr, bestb;
      {   // the starts and the first steps
        const int r0[3] = {0, -32, 32};
        int b0[5], b1[5];
        b0[0] = 0; b1[0] = 0;
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2) { b0[a2 + 1] = ax0[a2] * 16; b1[a2 + 1] = ax1[a2] * 16; }
        long long vr[3], vb[5];
        cc_eval<3, 5, T>(S, np, cb, par, r0, b0, b1, vr, vb PS_ARG);
        bestr = vr[0];
        int k = vr[2] < vr[1] ? 2 : 1;
        if (vr[k] < bestr) { bestr = vr[k]; g2r = r0[k]; }
        bestb = vb[0];
        k = 1;
#pragma unroll
        for (int a2 = 2; a2 < 5; ++a2)
          if (vb[a2] < vb[k]) k = a2;
        if (vb[k] < bestb) { bestb = vb[k]; g2b = b0[k]; r2b = b1[k]; }
      }
      bool blue_on = true;
      for (int it = 1; it < 7; ++it) {
        const int d = bdel[it], dr = 32 >> it;   // red deltas 16, 8, 4, 2, 1, then none
        int b0[4], b1[4];
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2) { b0[a2] = g2b + ax0[a2] * d; b1[a2] = r2b + ax1[a2] * d; }
        long long vb[4];
        if (dr > 0 && blue_on) {
          const int r0[2] = {g2r - dr, g2r + dr};
          long long vr[2];
          cc_eval<2, 4, T>(S, np, cb, par, r0, b0, b1, vr, vb PS_ARG);
          const int k = vr[1] < vr[0] ? 1 : 0;
          if (vr[k] < bestr) { bestr = vr[k]; g2r = r0[k]; }
        } else if (dr > 0) {
          const int r0[2] = {g2r - dr, g2r + dr}, z[1] = {0};
          long long vr[2], vz[1];
          cc_eval<2, 0, T>(S, np, cb, par, r0, z, z, vr, vz PS_ARG);
          const int k = vr[1] < vr[0] ? 1 : 0;
          if (vr[k] < bestr) { bestr = vr[k]; g2r = r0[k]; }
          continue;
        } else if (blue_on) {
          const int z[1] = {0};
          long long vz[1];
          cc_eval<0, 4, T>(S, np, cb, par, z, b0, b1, vz, vb PS_ARG);
        } else {
          break;
        }
        int k = 0;
#pragma unroll
        for (int a2 = 1; a2 < 4; ++a2)
          if (vb[a2] < vb[k]) k = a2;
        if (vb[k] < bestb) { bestb = vb[k]; g2b = b0[k]; r2b = b1[k]; }
        if (d == 2 && g2b == 0 && r2b == 0) blue_on = false;
      }
    }   // !low_effort
    PS_STAMP(9);
    // final residuals
    __syncthreads();   // every residual of the tile read before any is overwritten
    for (int i = tid; i < np; i += 256) {
      const int ly = i / tw, lx = i - ly * tw;
      const uint32_t r = S.res[i];
      const int g = ch(r, 8), rr = ch(r, 16), bb = ch(r, 0);
      const int nr = (rr - ctd(g2r, g)) & 255;
      const int nb = (bb - ctd(g2b, g) - ctd(r2b, rr)) & 255;
      out[(size_t)(y0 + ly) * W + x0 + lx] = (r & 0xff00ff00u) | ((uint32_t)nr << 16) | (uint32_t)nb;
    }
    if (tid == 0) {
      mult[(size_t)f * ntt + tile] =
          (uint32_t)(g2r & 255) | ((uint32_t)(g2b & 255) << 8) | ((uint32_t)(r2b & 255) << 16);
    }
    PS_STAMP(10);
  }
}

// ------------------------------------------------------------------ L1 (wave tiles)
// The same transform search with one wave per tile (T = 8, 16, 32): a
// workgroup's four waves share the frame's tables and each walks its own
// tiles, so no block barrier sits in the search. A lane owns the tile's
// pixels ln, ln + 64, .. (PX of them) and keeps their residuals in
// registers; every sum over the tile is a wave butterfly, which leaves the
// total in every lane. Same arithmetic and order of choices as
// k_vp8l_transform (model: choose_predictors_ce, choose_cross_color).
#define L1W_TPW 2   // tiles per wave
template <int T>
struct WaveTile {
  union {
    uint32_t src[(T + 1) * (T + 2)];   // rows y0-1.., cols x0-1..x0+tw (until the residuals)
    uint32_t h9[8 * 128];              // colour search: up to 8 candidates, u16 counts
  } u;
  uint32_t first[T];
};
template <int T>
struct TransformWSmem {
  int32_t frac[1024];
  int32_t ct[4][256];
  uint32_t g[2][256];                // the frame's accumulated R and B histograms
  long long slogg[2][256];           // and their slog
  uint32_t nsum[4];
  WaveTile<T> w[4];
};

// LDS written by some lanes of a wave, then read by others
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v log2 v in 1/4096 bit for the counts of a tile (v <= 4096: 32 bits)
__device__ __forceinline__ int32_t slog_small(const int32_t* frac, uint32_t v) {
  if (v <= 1) return 0;
  const int e = 31 - __clz((int)v);
  const uint32_t m = (e >= 10 ? (v >> (e - 10)) : (v << (10 - e))) & 1023;
  return (int32_t)v * ((e << 12) + frac[m]);
}

__device__ __forceinline__ uint32_t load_px(const uint8_t* img, int rstride, bool plane, int x,
                                            int y, bool sg, bool& opaque) {
  if (plane) {   // ALPH: the alpha plane as green
    const uint32_t g = img[(size_t)y * rstride + x];
    opaque = false;
    return sg ? (((0u - g) & 255) << 16) | (g << 8) | ((0u - g) & 255) : g << 8;
  }
  const uint32_t v = *reinterpret_cast<const uint32_t*>(img + (size_t)y * rstride + 4 * x);
  const uint32_t r = v & 255, g = (v >> 8) & 255, b = (v >> 16) & 255, a = v >> 24;
  opaque &= a == 255;
  return sg ? (a << 24) | (((r - g) & 255) << 16) | (g << 8) | ((b - g) & 255)
            : (a << 24) | (r << 16) | (g << 8) | b;
}

// one colour-search step of a wave's tile (cc_eval's arithmetic): h9 zero on
// entry and on exit
template <int KR, int KB, int T, int PX>
__device__ __forceinline__ void cc_eval_w(TransformWSmem<T>& S, uint32_t* h9, const uint32_t (&res)[PX], int np,
                          const int (&spv)[2], const int (&r0)[KR > 0 ? KR : 1],
                          const int (&b0)[KB > 0 ? KB : 1], const int (&b1)[KB > 0 ? KB : 1],
                          long long (&outR)[KR > 0 ? KR : 1], long long (&outB)[KB > 0 ? KB : 1]) {
  constexpr int K = KR + KB;
  const int ln = lane_id();
  uint64_t hot[K];
#pragma unroll
  for (int k = 0; k < K; ++k) hot[k] = 0;
#pragma unroll
  for (int j = 0; j < PX; ++j) {
    if (ln + 64 * j >= np) break;
    uint32_t r = res[j];
    asm volatile("" : "+v"(r));   // no channel values kept live across the steps: registers
    const int g = ch(r, 8), rr = ch(r, 16), bb = ch(r, 0);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int v = k >= KR ? (bb - ctd(b0[k - KR], g) - ctd(b1[k - KR], rr)) & 255
                            : (rr - ctd(r0[k], g)) & 255;
      const int q = Hot<T>::slot(v);
      hot[k] += q < Hot<T>::NH ? (1ull << (Hot<T>::FB * q)) : 0ull;
      if (q >= Hot<T>::NH) hist_add(h9 + k * 128, v);
    }
  }
  {
    const int kk = ln / Hot<T>::NH, j = ln - kk * Hot<T>::NH;
    uint64_t mine = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint64_t t = wave_sum(hot[k]);
      if (k == kk) mine = t;
    }
    if (kk < K) {
      const uint32_t t = (uint32_t)(mine >> (Hot<T>::FB * j)) & Hot<T>::MASK;
      const int v = Hot<T>::value(j);
      if (t) atomicAdd(&h9[kk * 128 + (v >> 1)], t << ((v & 1) * 16));
    }
  }
  wave_sync();
  // bins: lane ln owns values ln + 64 i; the words it reads are zeroed by
  // their two readers (neighbouring lanes) after the reads
  int32_t acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int b = ln + 64 * i;
    uint32_t w[K];
#pragma unroll
    for (int k = 0; k < K; ++k) w[k] = h9[k * 128 + (b >> 1)];
#pragma unroll
    for (int k = 0; k < K; ++k) h9[k * 128 + (b >> 1)] = 0;
    const int sp = i == 0 ? spv[0] : i == 3 ? spv[1] : 0;   // |value| >= 64 in between: 0
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t t = (w[k] >> ((b & 1) * 16)) & 0xffffu;
      if (t) {
        const int c = k < KR ? 0 : 1;   // R or B
        acc[k] += 16 * (int32_t)t * sp -
                  (slog_small(S.frac, t) + (int32_t)(slog_fx(S.frac, t + S.g[c][b]) - S.slogg[c][b]));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KR; ++k) outR[k] = (long long)wave_sum(acc[k]) - CC_ZERO_BONUS * (r0[k] == 0);
#pragma unroll
  for (int k = 0; k < KB; ++k)
    outB[k] = (long long)wave_sum(acc[KR + k]) - CC_ZERO_BONUS * ((b0[k] == 0) + (b1[k] == 0));
  wave_sync();
}

template <int T, bool SG>
__global__ __launch_bounds__(256) void k_vp8l_transform_w(const uint8_t* __restrict__ rgba,
                                                          size_t fstride, int rstride, vp8l_params p,
                                                          const int* __restrict__ fidx,
                                                          const int* __restrict__ efidx,
                                                          const uint8_t* __restrict__ fmode,
                                                          const uint32_t* __restrict__ ehist,
                                                          const int32_t* __restrict__ frac_tab,
                                                          uint8_t* __restrict__ modes,
                                                          const uint32_t* __restrict__ pflag,
                                                          const uint8_t* __restrict__ pexact,
                                                          uint32_t* __restrict__ argb_out,
                                                          uint32_t* __restrict__ mult,
                                                          uint32_t* __restrict__ alpha_flag) {
  constexpr int PX = T * T / 64;
  static_assert(PX >= 1, "one wave per tile needs >= 64 pixels");
  __shared__ TransformWSmem<T> S;
  const int tid = threadIdx.x, ln = lane_id(), wv = tid >> 6, f = blockIdx.z;
  const int W = p.w, H = p.h;
  const uint8_t* img = rgba + (size_t)(fidx ? fidx[f] : f) * fstride;
  const int tiles_x = (W + T - 1) / T, tiles_y = (H + T - 1) / T, ntt = tiles_x * tiles_y;
  const int emode = fmode ? (int)fmode[f] : VP8L_MODE_SPATIAL;
  if (((emode & VP8L_MODE_SUBGREEN) != 0) != SG) return;
  const int tile0 = blockIdx.x * 4 * L1W_TPW, tile1 = min(tile0 + 4 * L1W_TPW, ntt);
  const bool plane = p.alpha != 0;
  uint32_t* out = argb_out + (size_t)f * W * H;

  if (!(emode & VP8L_MODE_SPATIAL)) {   // direct / subtract green only: no predictor
    bool opaque = true;
    for (int tile = tile0 + wv; tile < tile1; tile += 4) {
      const int x0 = (tile % tiles_x) * T, y0 = (tile / tiles_x) * T;
      const int tw = min(T, W - x0), th = min(T, H - y0);
      for (int i = ln; i < tw * th; i += 64) {
        const int ly = i / tw, lx = i - ly * tw;
        out[(size_t)(y0 + ly) * W + x0 + lx] = load_px(img, rstride, plane, x0 + lx, y0 + ly, SG, opaque);
      }
    }
    if (!plane && !__all(opaque) && ln == 0) atomicOr(&alpha_flag[f], 1u);
    return;
  }

  // per-frame setup (as k_vp8l_transform)
  {
    const uint32_t* eh = ehist + (size_t)(efidx ? efidx[f] : f) * VP8L_EHIST;
    const int hix[4] = {VP8L_EH_ACC + 0, VP8L_EH_ACC + (SG ? 4 : 1), VP8L_EH_ACC + 2,
                        VP8L_EH_ACC + (SG ? 5 : 3)};
    for (int i = tid; i < 1024; i += 256) S.frac[i] = frac_tab[i];
    if (tid < 4) S.nsum[tid] = 0;
    __syncthreads();
    uint32_t gv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      gv[c] = eh[hix[c] * 256 + tid];
      if (c & 1) {
        S.g[c >> 1][tid] = gv[c];
        S.slogg[c >> 1][tid] = slog_fx(S.frac, gv[c]);
      }
      const uint32_t t = wave_sum(gv[c]);
      if (ln == 0) atomicAdd(&S.nsum[c], t);
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 4; ++c)   // model: ce_tables
      S.ct[c][tid] = flog2_fx(S.frac, 2 * S.nsum[c] + 256) - flog2_fx(S.frac, 2 * gv[c] + 1);
    __syncthreads();
  }
  const bool own_pred = !p.low_effort && !(pexact && pexact[f]);   // else L1a's choice
  const int spv[2] = {sp_of(kSpCC, ln), sp_of(kSpCC, ln + 192)};
  WaveTile<T>& Wt = S.w[wv];
  bool any_alpha = false;

  for (int tile = tile0 + wv; tile < tile1; tile += 4) {
    const int x0 = (tile % tiles_x) * T, y0 = (tile / tiles_x) * T;
    const int tw = min(T, W - x0), th = min(T, H - y0);
    const int sw = tw + 2, np = tw * th;
    // the tile (+ the row above and the column left) into LDS
    bool opaque = true;
    for (int i = ln; i < (th + 1) * sw; i += 64) {
      const int ly = i / sw, lx = i - ly * sw;
      const int y = y0 - 1 + ly, x = x0 - 1 + lx;
      uint32_t v = 0;
      if (y >= 0 && x >= 0 && x < W) {
        bool o = true;
        v = load_px(img, rstride, plane, x, y, SG, o);
        opaque &= o;
        if (!o && !plane && ly > 0 && lx > 0 && lx <= tw) any_alpha = true;
      }
      Wt.u.src[i] = v;
    }
    if (x0 + tw == W)
      for (int i = ln; i < th; i += 64) Wt.first[i] = load_px(img, rstride, plane, 0, y0 + i, SG, opaque);
    opaque = !plane && __all(opaque);
    wave_sync();

    auto at = [&](int lx, int ly) -> uint32_t { return Wt.u.src[(ly + 1) * sw + lx + 1]; };
    auto tr = [&](int lx, int ly) -> uint32_t {   // (y-1)*W + x + 1, linear
      return (x0 + lx + 1 < W) ? at(lx + 1, ly - 1) : Wt.first[ly];
    };
    auto fixed_mode = [&](int x, int y) -> int { return y == 0 ? (x == 0 ? 0 : 1) : (x == 0 ? 2 : -1); };
    int best;
    if (own_pred) {   // model: choose_predictors_ce (fixed-predictor pixels: one cost for all)
      int32_t pc[14];
#pragma unroll
      for (int m = 0; m < 14; ++m) pc[m] = 0;
      auto ce_sum = [&](auto opq) {
#pragma unroll
        for (int j = 0; j < PX; ++j) {
          const int i = ln + 64 * j;
          if (i >= np) break;
          const int ly = i / tw, lx = i - ly * tw;
          if (fixed_mode(x0 + lx, y0 + ly) >= 0) continue;
          const uint32_t P = at(lx, ly), L = at(lx - 1, ly), T_ = at(lx, ly - 1);
          const uint32_t TL = at(lx - 1, ly - 1), TR = tr(lx, ly);
#pragma unroll
          for (int m = 0; m < 14; ++m) {
            const uint32_t r = sub_pixels(P, predict(m, L, T_, TL, TR));
            pc[m] += (decltype(opq)::value ? 0 : S.ct[0][r >> 24]) + S.ct[1][ch(r, 16)] +
                     S.ct[2][ch(r, 8)] + S.ct[3][ch(r, 0)];
          }
        }
      };
      if (opaque) ce_sum(std::true_type{});
      else ce_sum(std::false_type{});
      best = 0;
      int32_t bv = wave_sum(pc[0]);
#pragma unroll
      for (int m = 1; m < 14; ++m) {
        const int32_t v = wave_sum(pc[m]);
        if (v < bv) { bv = v; best = m; }
      }
      if (ln == 0) modes[(size_t)f * ntt + tile] = (uint8_t)best;
    } else {
      best = modes[(size_t)f * ntt + tile];
    }
    // the chosen predictor's residuals (or the serial pass's, pflag), in registers
    uint32_t res[PX];
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int i = ln + 64 * j;
      res[j] = 0;
      if (i < np) {
        const int ly = i / tw, lx = i - ly * tw;
        if (pflag[f]) {
          res[j] = out[(size_t)(y0 + ly) * W + x0 + lx];
        } else {
          const int fm = fixed_mode(x0 + lx, y0 + ly);
          res[j] = sub_pixels(at(lx, ly), predict(fm >= 0 ? fm : best, at(lx - 1, ly), at(lx, ly - 1),
                                                  at(lx - 1, ly - 1), tr(lx, ly)));
        }
      }
    }
    wave_sync();   // every source pixel read before h9 reuses the LDS
    int g2r = 0, g2b = 0, r2b = 0;
    if (!p.low_effort) {   // model: choose_cross_color; none at method 0
      uint32_t* h9 = Wt.u.h9;
      for (int i = ln; i < 8 * 128; i += 64) h9[i] = 0;
      wave_sync();
      const int ax0[4] = {0, 0, -1, 1}, ax1[4] = {-1, 1, 0, 0};
      const int bdel[7] = {16, 16, 8, 4, 2, 2, 2};
      long long bestr, bestb;
      {
        const int r0[3] = {0, -32, 32};
        int b0[5], b1[5];
        b0[0] = 0; b1[0] = 0;
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2) { b0[a2 + 1] = ax0[a2] * 16; b1[a2 + 1] = ax1[a2] * 16; }
        long long vr[3], vb[5];
        cc_eval_w<3, 5, T, PX>(S, h9, res, np, spv, r0, b0, b1, vr, vb);
        bestr = vr[0];
        int k = vr[2] < vr[1] ? 2 : 1;
        if (vr[k] < bestr) { bestr = vr[k]; g2r = r0[k]; }
        bestb = vb[0];
        k = 1;
#pragma unroll
        for (int a2 = 2; a2 < 5; ++a2)
          if (vb[a2] < vb[k]) k = a2;
        if (vb[k] < bestb) { bestb = vb[k]; g2b = b0[k]; r2b = b1[k]; }
      }
      bool blue_on = true;
      for (int it = 1; it < 7; ++it) {
        const int d = bdel[it], dr = 32 >> it;
        int b0[4], b1[4];
#pragma unroll
        for (int a2 = 0; a2 < 4; ++a2) { b0[a2] = g2b + ax0[a2] * d; b1[a2] = r2b + ax1[a2] * d; }
        long long vb[4];
        if (dr > 0 && blue_on) {
          const int r0[2] = {g2r - dr, g2r + dr};
          long long vr[2];
          cc_eval_w<2, 4, T, PX>(S, h9, res, np, spv, r0, b0, b1, vr, vb);
          const int k = vr[1] < vr[0] ? 1 : 0;
          if (vr[k] < bestr) { bestr = vr[k]; g2r = r0[k]; }
        } else if (dr > 0) {
          const int r0[2] = {g2r - dr, g2r + dr}, z[1] = {0};
          long long vr[2], vz[1];
          cc_eval_w<2, 0, T, PX>(S, h9, res, np, spv, r0, z, z, vr, vz);
          const int k = vr[1] < vr[0] ? 1 : 0;
          if (vr[k] < bestr) { bestr = vr[k]; g2r = r0[k]; }
          continue;
        } else if (blue_on) {
          const int z[1] = {0};
          long long vz[1];
          cc_eval_w<0, 4, T, PX>(S, h9, res, np, spv, z, b0, b1, vz, vb);
        } else {
          break;
        }
        int k = 0;
#pragma unroll
        for (int a2 = 1; a2 < 4; ++a2)
          if (vb[a2] < vb[k]) k = a2;
        if (vb[k] < bestb) { bestb = vb[k]; g2b = b0[k]; r2b = b1[k]; }
        if (d == 2 && g2b == 0 && r2b == 0) blue_on = false;
      }
    }
    // final residuals
#pragma unroll
    for (int j = 0; j < PX; ++j) {
      const int i = ln + 64 * j;
      if (i >= np) break;
      const int ly = i / tw, lx = i - ly * tw;
      const uint32_t r = res[j];
      const int g = ch(r, 8), rr = ch(r, 16), bb = ch(r, 0);
      const int nr = (rr - ctd(g2r, g)) & 255;
      const int nb = (bb - ctd(g2b, g) - ctd(r2b, rr)) & 255;
      out[(size_t)(y0 + ly) * W + x0 + lx] = (r & 0xff00ff00u) | ((uint32_t)nr << 16) | (uint32_t)nb;
    }
    if (ln == 0)
      mult[(size_t)f * ntt + tile] =
          (uint32_t)(g2r & 255) | ((uint32_t)(g2b & 255) << 8) | ((uint32_t)(r2b & 255) << 16);
    wave_sync();   // the next tile's load reuses the LDS
  }
  if (__any(any_alpha) && ln == 0) atomicOr(&alpha_flag[f], 1u);
}

// ------------------------------------------------------------------ L1a
// VP8LResidualImage's predictor choice, exactly (model: residual_image;
// src/enc/predictor_enc.c:299-409,476-516). Serial over the frame's tiles in
// raster order -- each tile is scored against the histograms of the
// residuals its predecessors chose -- so one workgroup per frame:
//   1. the tile (+ border) into LDS; near-lossless max diffs (:121-146);
//   2. the 14 modes' residual histograms: all pixels at once, or, where
//      GetResidual updates the picture as it goes (near-lossless
//      quantisation, alpha-0 clean-up; :234-292), a wavefront per mode with
//      one lane per tile row (row r at column s - 2r in step s; the row
//      above comes in by a lane shuffle, one column ahead);
//   3. PredictionCostSpatialHistogram (:47-57) per mode: the subtrahends of
//      CombinedShannonEntropy (src/dsp/lossless_enc.c:403-422) computed in
//      parallel, then one lane per (mode, channel) subtracts them in the
//      reference's order -- float32 with no contraction, so the sums are the
//      reference's bit for bit; the first minimum wins.
// The float tables (VP8LFastSLog2 0..255, log2 0..255: tabs + 5121, + 5377)
// are the host's (float)(v log2 v), (float)log2 v, equal to the reference's
// literals (tests/test_vp8l.py checks them against its source).
#define PS_THREADS 1024
#define LOG_2_RECIPROCAL_D 1.44269504088896338700465094007086


// histogram / term rows padded by one word / one float4: the cost chains'
// lanes walk one row each, and unpadded rows would all start in one LDS bank
#define PS_HS 129
#define PS_TS 129
// T: tile size; NCH channels' cost terms at a time (all four up to T = 32,
// two at T = 64 where the tile itself takes more LDS)
template <int T>
struct PredSelSmem {
  static constexpr int NCH = T >= 64 ? 2 : 4;
  uint32_t src[(T + 2) * (T + 2)];   // rows y0-1..y1, cols x0-1..x1 (original)
  uint32_t first[T + 1];             // P(0, y) for y0-1 .. y1-1 (TR wrap)
  uint8_t maxd[T * T];
  uint32_t hist[14 * 4 * PS_HS];     // u16 pairs: [mode][channel][value], padded rows
  int32_t acc[4][256];
  float sacc[4][256];                // FastSLog2(acc)
  float4 terms[NCH][14][PS_TS];      // subtrahends in bin order: (t1, t2) of two bins
  float slog[256], log2t[256];
  float pcs[14][4], cse[14][4];
  int accsum[4];
  int best, serial, any_t;
};

__device__ __forceinline__ float ps_slog2(uint32_t v, const float* slog, const float* log2t) {
  if (v < 256) return slog[v];
  if (v < 65536) {   // FastSLog2Slow_C (src/dsp/lossless_enc.c:329-359)
    const int log_cnt = (31 - __clz((int)v)) - 7;
    const uint32_t y = 1u << log_cnt;
    const int corr = (int)((23 * (v & (y - 1))) >> 4);
    return __fadd_rn(__fmul_rn((float)v, __fadd_rn(log2t[v >> log_cnt], (float)log_cnt)),
                     (float)corr);
  }
  return (float)__dmul_rn(__dmul_rn(LOG_2_RECIPROCAL_D, (double)v), log((double)v));
}

__device__ __forceinline__ uint32_t add_pixels(uint32_t a, uint32_t b) {
  const uint32_t ag = (a & 0xff00ff00u) + (b & 0xff00ff00u);
  const uint32_t rb = (a & 0x00ff00ffu) + (b & 0x00ff00ffu);
  return (ag & 0xff00ff00u) | (rb & 0x00ff00ffu);
}

// NearLosslessComponent (src/enc/predictor_enc.c:151-179)
__device__ __forceinline__ int nl_component(int value, int pred, int boundary, int q) {
  const int residual = (value - pred) & 0xff;
  const int boundary_residual = (boundary - pred) & 0xff;
  const int lower = residual & ~(q - 1);
  const int upper = lower + q;
  const int bias = ((boundary - value) & 0xff) < boundary_residual;
  if (residual - lower < upper - residual + bias) {
    if (residual > boundary_residual && lower <= boundary_residual) return lower + (q >> 1);
    return lower;
  }
  if (residual <= boundary_residual && upper > boundary_residual) return lower + (q >> 1);
  return upper & 0xff;
}

// NearLossless (:190-227)
__device__ uint32_t nl_residual(uint32_t value, uint32_t pred, int max_q, int max_diff, bool sg) {
  if (max_diff <= 2) return sub_pixels(value, pred);
  int q = max_q;
  while (q >= max_diff) q >>= 1;
  const int va = (int)(value >> 24);
  const int a = (va == 0 || va == 0xff) ? (va - (int)(pred >> 24)) & 0xff
                                        : nl_component(va, (int)(pred >> 24), 0xff, q);
  const int g = nl_component(ch(value, 8), ch(pred, 8), 0xff, q);
  int new_green = 0, green_diff = 0;
  if (sg) {
    new_green = (ch(pred, 8) + g) & 0xff;
    green_diff = (new_green - ch(value, 8)) & 0xff;
  }
  const int r = nl_component((ch(value, 16) - green_diff) & 0xff, ch(pred, 16), 0xff - new_green, q);
  const int b = nl_component((ch(value, 0) - green_diff) & 0xff, ch(pred, 0), 0xff - new_green, q);
  return ((uint32_t)a << 24) | ((uint32_t)r << 16) | ((uint32_t)g << 8) | (uint32_t)b;
}

__device__ __forceinline__ uint32_t add_green(uint32_t v) {   // AddGreenToBlueAndRed (:113-119)
  const uint32_t g = (v >> 8) & 0xff;
  return (v & 0xff00ff00u) | (((v & 0x00ff00ffu) + ((g << 16) | g)) & 0x00ff00ffu);
}
__device__ __forceinline__ int max_diff_px(uint32_t a, uint32_t b) {
  int m = 0;
#pragma unroll
  for (int k = 0; k < 32; k += 8) m = max(m, abs(ch(a, k) - ch(b, k)));
  return m;
}

// one pixel of GetResidual's non-exact branch (:243-290): the residual, and
// the (possibly updated) pixel the later predictions read
__device__ __forceinline__ uint32_t resid_px(uint32_t cur, uint32_t pred, bool quant, int max_q,
                                             int md, bool sg, uint32_t& rec) {
  uint32_t res;
  if (!quant) {
    res = sub_pixels(cur, pred);
  } else {
    res = nl_residual(cur, pred, max_q, md, sg);
    cur = add_pixels(pred, res);
  }
  rec = cur;
  if ((cur >> 24) == 0) {
    res &= 0xff000000u;
    rec = pred & 0x00ffffffu;
  }
  return res;
}

// residual histogram counts with the most frequent values per channel (0 and
// its neighbours) kept in registers -- same-bin LDS atomics within a wave
// serialise, and those values are most of a good predictor's residuals --
// packed per channel into the fields of a u64: five 11-bit fields (values
// -2..2) up to 32 x 32 tiles, four 13-bit ones (-1..2) for 64 x 64, wide
// enough for a whole wave's sum over a tile of one value
template <int T>
__device__ __forceinline__ void count_res(uint32_t res, uint64_t (&hot)[4], uint32_t* h) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int v = ch(res, 24 - 8 * c);
    const int k = Hot<T>::slot(v);
    hot[c] += k < Hot<T>::NH ? (1ull << (Hot<T>::FB * k)) : 0ull;
    if (k >= Hot<T>::NH) hist_add(h + c * PS_HS, v);
  }
}
template <int T>
__device__ __forceinline__ void flush_hot(const uint64_t (&hot)[4], uint32_t* h) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int j = 0; j < Hot<T>::NH; ++j) {
      const uint32_t t = (uint32_t)(hot[c] >> (Hot<T>::FB * j)) & Hot<T>::MASK;
      const int v = Hot<T>::value(j);
      if (t) atomicAdd(&h[c * PS_HS + (v >> 1)], t << ((v & 1) * 16));
    }
}

// pixel of the input frame as the transform sees it (sub-green when SG)
template <bool SG>
__device__ __forceinline__ uint32_t in_px(const uint8_t* img, int rstride, bool plane, int x, int y) {
  if (plane) {
    const uint32_t g = img[(size_t)y * rstride + x];
    return SG ? (((0u - g) & 255) << 16) | (g << 8) | ((0u - g) & 255) : g << 8;
  }
  const uint32_t q = *reinterpret_cast<const uint32_t*>(img + (size_t)y * rstride + 4 * x);
  const uint32_t r = q & 255, g = (q >> 8) & 255, b = (q >> 16) & 255, a = q >> 24;
  return SG ? (a << 24) | (((r - g) & 255) << 16) | (g << 8) | ((b - g) & 255)
            : (a << 24) | (r << 16) | (g << 8) | b;
}

template <int T, bool SG>
__global__ __launch_bounds__(PS_THREADS) void k_vp8l_predsel(const uint8_t* __restrict__ rgba,
                                                             size_t fstride, int rstride,
                                                             vp8l_params p,
                                                             const int* __restrict__ fidx,
                                                             const uint8_t* __restrict__ fmode,
                                                             const uint8_t* __restrict__ pexact,
                                                             const float* __restrict__ ftabs,
                                                             uint8_t* __restrict__ modes,
                                                             uint32_t* __restrict__ pflag) {
  extern __shared__ __align__(16) uint8_t ps_smem[];
  using Smem = PredSelSmem<T>;
  Smem& S = *reinterpret_cast<Smem*>(ps_smem);
  const int tid = threadIdx.x, f = blockIdx.x;
  const int W = p.w, H = p.h;
  const int emode = fmode ? (int)fmode[f] : VP8L_MODE_SPATIAL;
  if (!(emode & VP8L_MODE_SPATIAL) || ((emode & VP8L_MODE_SUBGREEN) != 0) != SG) return;
  const uint8_t* img = rgba + (size_t)(fidx ? fidx[f] : f) * fstride;
  const int tiles_x = (W + T - 1) / T, tiles_y = (H + T - 1) / T, ntt = tiles_x * tiles_y;
  uint8_t* fm = modes + (size_t)f * ntt;
  const bool plane = p.alpha != 0;
  if (p.low_effort) {   // kPredLowEffort everywhere (:488-492), plain residuals
    for (int t = tid; t < ntt; t += PS_THREADS) fm[t] = 11;
    if (tid == 0) pflag[f] = 0;
    return;
  }
  if (!(pexact && pexact[f])) return;   // L1's cross-entropy choice
  const int max_q = 1 << p.nlq_bits;
  for (int i = tid; i < 256; i += PS_THREADS) { S.slog[i] = ftabs[i]; S.log2t[i] = ftabs[256 + i]; }
  for (int i = tid; i < 1024; i += PS_THREADS) {
    (&S.acc[0][0])[i] = 0;
    (&S.sacc[0][0])[i] = 0.f;
  }
  if (tid < 4) S.accsum[tid] = 0;
  if (tid == 0) S.any_t = 0;
  const float kBias = 15.f;   // kSpatialPredictorBias (:24)
  PS_STAMP_INIT;

  for (int tile = 0; tile < ntt; ++tile) {
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    const int x0 = tx * T, y0 = ty * T;
    const int tw = min(T, W - x0), th = min(T, H - y0);
    const int sw = tw + 2, np = tw * th;
    __syncthreads();   // the previous tile is done with S
    bool tr_alpha = false;
    for (int i = tid; i < (th + 2) * sw; i += PS_THREADS) {
      const int ly = i / sw, lx = i - ly * sw;
      const int y = y0 - 1 + ly, x = x0 - 1 + lx;
      uint32_t v = 0;
      if (y >= 0 && y < H && x >= 0 && x < W) v = in_px<SG>(img, rstride, plane, x, y);
      S.src[i] = v;
      if (ly >= 1 && ly <= th && lx >= 1 && lx <= tw && (v >> 24) == 0) tr_alpha = true;
    }
    for (int i = tid; i <= th; i += PS_THREADS) {
      const int y = y0 - 1 + i;
      S.first[i] = y >= 0 ? in_px<SG>(img, rstride, plane, 0, y) : 0u;
    }
    for (int i = tid; i < 14 * 4 * PS_HS; i += PS_THREADS) S.hist[i] = 0;
    if (tid == 0) S.serial = 0;
    __syncthreads();
    PS_STAMP(0);
    if (!p.exact && __any(tr_alpha) && lane_id() == 0) { S.serial = 1; S.any_t = 1; }
    if (!p.exact && max_q > 1) {
      if (tid == 0) S.serial = 1;
      for (int i = tid; i < np; i += PS_THREADS) {   // MaxDiffsForRow over the original
        const int ly = i / tw, lx = i - ly * tw;
        const int x = x0 + lx, y = y0 + ly;
        int md = 0;
        if (x >= 1 && x < W - 1 && y >= 1 && y < H - 1) {
          auto at = [&](int ax, int ay) -> uint32_t {
            const uint32_t v = S.src[(ay + 1) * sw + ax + 1];
            return SG ? add_green(v) : v;
          };
          const uint32_t c = at(lx, ly);
          md = max(max(max_diff_px(c, at(lx, ly - 1)), max_diff_px(c, at(lx, ly + 1))),
                   max(max_diff_px(c, at(lx - 1, ly)), max_diff_px(c, at(lx + 1, ly))));
        }
        S.maxd[i] = (uint8_t)min(md, 255);
      }
    }
    __syncthreads();
    PS_STAMP(1);
    auto at = [&](int lx, int ly) -> uint32_t { return S.src[(ly + 1) * sw + lx + 1]; };
    if (!S.serial) {
      // plain residuals: one wave per mode over the tile's pixels (fixed
      // modes on row 0 / column 0)
      const int m = tid >> 6;
      if (m < 14) {
        uint64_t hot[4] = {0, 0, 0, 0};
        uint32_t* h = S.hist + m * 4 * PS_HS;
        for (int k = lane_id(); k < np; k += 64) {
          const int ly = k / tw, lx = k - ly * tw;
          const int x = x0 + lx, y = y0 + ly;
          uint32_t pred;
          if (y == 0) pred = x == 0 ? 0xff000000u : at(lx - 1, ly);
          else if (x == 0) pred = at(lx, ly - 1);
          else pred = predict(m, at(lx - 1, ly), at(lx, ly - 1), at(lx - 1, ly - 1),
                              x + 1 < W ? at(lx + 1, ly - 1) : S.first[ly + 1]);
          count_res<T>(sub_pixels(at(lx, ly), pred), hot, h);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) hot[c] = wave_sum(hot[c]);
        if (lane_id() == 0) flush_hot<T>(hot, h);
      }
    } else {
      // wavefront: lane (m, r) takes tile row r; T lanes per mode, 64 / T modes per wave
      const int m = tid / T, r = tid - m * T;
      const bool live = m < 14 && r < th;
      const int y = y0 + r;
      const bool quant_row = max_q > 1 && m != 0 && y != 0 && y != H - 1;
      uint32_t out = live ? at(-1, r) : 0u;   // what the row below reads next: left context first
      uint32_t a = 0, b = 0, c = 0;           // the row above at x-1, x, x+1 (r > 0)
      uint32_t L = out, first_rec = 0;
      uint64_t hot[4] = {0, 0, 0, 0};
      uint32_t* h = S.hist + (m < 14 ? m : 0) * 4 * PS_HS;
      const int nsteps = tw + 2 * (th - 1);
      for (int s = 0; s < nsteps; ++s) {
        const uint32_t up = __shfl_up(out, 1);   // row r-1's newest pixel
        a = b; b = c; c = up;
        const int lx = s - 2 * r, x = x0 + lx;
        if (live && lx >= 0 && lx < tw) {
          uint32_t T_, TL, TR;
          if (r == 0) {
            T_ = at(lx, -1); TL = at(lx - 1, -1);
            TR = x + 1 < W ? at(lx + 1, -1) : S.first[1];
          } else {
            T_ = b; TL = a;
            TR = lx + 1 < tw ? c : (x + 1 < W ? at(lx + 1, r - 1) : 0u);
          }
          if (x + 1 >= W) TR = (x0 == 0) ? first_rec : S.first[r + 1];   // P(0, y), this row
          uint32_t pred;
          if (y == 0) pred = x == 0 ? 0xff000000u : L;
          else if (x == 0) pred = T_;
          else pred = predict(m, L, T_, TL, TR);
          const bool q = quant_row && x != 0 && x != W - 1;
          uint32_t rec;
          const uint32_t res = resid_px(at(lx, r), pred, q, max_q, q ? S.maxd[r * tw + lx] : 0,
                                        SG, rec);
          count_res<T>(res, hot, h);
          if (lx == 0) first_rec = rec;
          L = rec;
          out = rec;
        } else if (live && lx == tw) {
          out = x < W ? at(lx, r) : 0u;   // the right context, for the row below's last TR
        }
      }
      if (live) flush_hot<T>(hot, h);
    }
    __syncthreads();
    PS_STAMP(2);
    // costs, NCH channels at a time: the subtrahends in parallel, then one
    // lane per (mode, channel) subtracts them in bin order
    constexpr int NCH = Smem::NCH;
    for (int c0 = 0; c0 < 4; c0 += NCH) {
      for (int i = tid; i < NCH * 14 * 128; i += PS_THREADS) {
        const int cc = i / (14 * 128), rem = i - cc * 14 * 128;
        const int m = rem >> 7, v2 = rem & 127, c = c0 + cc;
        const uint32_t xx = S.hist[(m * 4 + c) * PS_HS + v2];   // bins 2 v2, 2 v2 + 1
        float4 t;
        {
          const uint32_t x = xx & 0xffffu, y = (uint32_t)S.acc[c][2 * v2];
          t.x = x ? ps_slog2(x, S.slog, S.log2t) : S.sacc[c][2 * v2];   // 0 when y == 0
          t.y = x ? ps_slog2(x + y, S.slog, S.log2t) : 0.f;
        }
        {
          const uint32_t x = xx >> 16, y = (uint32_t)S.acc[c][2 * v2 + 1];
          t.z = x ? ps_slog2(x, S.slog, S.log2t) : S.sacc[c][2 * v2 + 1];
          t.w = x ? ps_slog2(x + y, S.slog, S.log2t) : 0.f;
        }
        S.terms[cc][m][v2] = t;
      }
      __syncthreads();
      PS_STAMP(3);
      if (tid < NCH * 14) {
        const int cc = tid / 14, m = tid - cc * 14, c = c0 + cc;
        float rr = 0.f;
        const float4* tv = S.terms[cc][m];
#pragma unroll 16
        for (int v2 = 0; v2 < 128; ++v2) {
          const float4 t = tv[v2];
          rr = __fsub_rn(rr, t.x);
          rr = __fsub_rn(rr, t.y);
          rr = __fsub_rn(rr, t.z);
          rr = __fsub_rn(rr, t.w);
        }
        const float sxy = __fadd_rn(ps_slog2((uint32_t)np, S.slog, S.log2t),
                                    ps_slog2((uint32_t)(np + S.accsum[c]), S.slog, S.log2t));
        S.cse[m][c] = __fadd_rn(rr, sxy);
        // PredictionCostSpatial(counts, 1, 0.94f) (:34-45)
        auto cnt = [&](int v) -> int {
          return (int)((S.hist[(m * 4 + c) * PS_HS + (v >> 1)] >> ((v & 1) * 16)) & 0xffffu);
        };
        float bits = __fmul_rn(1.f, (float)cnt(0));
        float e = 0.94f;
#pragma unroll
        for (int i = 1; i < 16; ++i) {
          bits = __fadd_rn(bits, __fmul_rn(e, (float)(cnt(i) + cnt(256 - i))));
          e = __fmul_rn(e, 0.6f);
        }
        S.pcs[m][c] = (float)__dmul_rn(-0.1, (double)bits);
      }
      __syncthreads();
      PS_STAMP(4);
    }
    if (tid == 0) {
      const int left = tx > 0 ? fm[tile - 1] : 0xff, above = ty > 0 ? fm[tile - tiles_x] : 0xff;
      float best_diff = 1e30f;
      int best = 0;
      for (int m = 0; m < 14; ++m) {
        float cst = 0.f;
        for (int c = 0; c < 4; ++c) {
          cst = __fadd_rn(cst, S.pcs[m][c]);
          cst = __fadd_rn(cst, S.cse[m][c]);
        }
        if (m == left) cst = __fsub_rn(cst, kBias);
        if (m == above) cst = __fsub_rn(cst, kBias);
        if (cst < best_diff) { best_diff = cst; best = m; }
      }
      S.best = best;
      fm[tile] = (uint8_t)best;
    }
    __syncthreads();
    {   // accumulate the chosen histograms (:401-405)
      const int best = S.best;
      for (int i = tid; i < 1024; i += PS_THREADS) {
        const int c = i >> 8, v = i & 255;
        const uint32_t x = (S.hist[(best * 4 + c) * PS_HS + (v >> 1)] >> ((v & 1) * 16)) & 0xffffu;
        if (x) {
          const int nv = S.acc[c][v] + (int)x;
          S.acc[c][v] = nv;
          S.sacc[c][v] = ps_slog2((uint32_t)nv, S.slog, S.log2t);
        }
      }
      if (tid < 4) S.accsum[tid] += np;
    }
    PS_STAMP(5);
  }
  __syncthreads();
  if (tid == 0) pflag[f] = (!p.exact && (max_q > 1 || S.any_t)) ? 1u : 0u;
}

// CopyImageWithPrediction (:414-470) where GetResidual updates the picture
// (pflag[f]): one wave per frame, the rows in bands of 64 (one lane each),
// row r of a band at column s - 2r in step s; the row above comes from the
// lane above by a shuffle or, for the band's first row, from the previous
// band's last row (LDS, read before it is overwritten: lane 63 stores column
// x only at step x + 126). Residuals to argb (before the colour transform).
template <bool SG>
__global__ __launch_bounds__(64) void k_vp8l_resid_serial(const uint8_t* __restrict__ rgba,
                                                          size_t fstride, int rstride,
                                                          vp8l_params p,
                                                          const int* __restrict__ fidx,
                                                          const uint8_t* __restrict__ fmode,
                                                          const uint8_t* __restrict__ modes,
                                                          const uint32_t* __restrict__ pflag,
                                                          uint32_t* __restrict__ argb_out) {
  extern __shared__ __align__(16) uint32_t prev_row[];   // W pixels of the band above
  const int f = blockIdx.x, lane = threadIdx.x;
  const int emode = fmode ? (int)fmode[f] : VP8L_MODE_SPATIAL;
  if (!(emode & VP8L_MODE_SPATIAL) || ((emode & VP8L_MODE_SUBGREEN) != 0) != SG || !pflag[f]) return;
  const int W = p.w, H = p.h, tb = p.tb;
  const int tiles_x = (W + (1 << tb) - 1) >> tb;
  const uint8_t* img = rgba + (size_t)(fidx ? fidx[f] : f) * fstride;
  const uint8_t* fm = modes + (size_t)f * tiles_x * ((H + (1 << tb) - 1) >> tb);
  uint32_t* out = argb_out + (size_t)f * W * H;
  const bool plane = p.alpha != 0;
  const int max_q = 1 << p.nlq_bits;
  auto src = [&](int x, int y) -> uint32_t { return in_px<SG>(img, rstride, plane, x, y); };
  auto orig_g = [&](int x, int y) -> uint32_t {   // for the max diffs: sub-green undone
    const uint32_t v = src(x, y);
    return SG ? add_green(v) : v;
  };
  for (int yb = 0; yb < H; yb += 64) {
    const int r = lane, y = yb + r;
    const bool live = y < H;
    const bool quant_row = max_q > 1 && y != 0 && y != H - 1;
    uint32_t outv = 0, a = 0, b = 0, c = 0, L = 0, first_rec = 0;
    const int nrows = min(64, H - yb);
    const int nsteps = W + 2 * (nrows - 1);
    for (int s = 0; s < nsteps; ++s) {
      const uint32_t up = __shfl_up(outv, 1);
      a = b; b = c; c = up;
      const int x = s - 2 * r;
      if (live && x >= 0 && x < W) {
        uint32_t T_ = 0, TL = 0, TR = 0;
        if (y > 0) {
          if (r == 0) {
            T_ = prev_row[x];
            TL = x > 0 ? prev_row[x - 1] : 0u;
            TR = x + 1 < W ? prev_row[x + 1] : 0u;
          } else {
            T_ = b; TL = a; TR = c;
          }
        }
        if (x + 1 >= W) TR = first_rec;   // P(0, y), reconstructed
        const int m = fm[(y >> tb) * tiles_x + (x >> tb)];
        uint32_t pred;
        if (y == 0) pred = x == 0 ? 0xff000000u : L;
        else if (x == 0) pred = T_;
        else pred = predict(m, L, T_, TL, TR);
        const bool q = quant_row && m != 0 && x != 0 && x != W - 1;
        int md = 0;
        if (q) {
          const uint32_t cg = orig_g(x, y);
          md = max(max(max_diff_px(cg, orig_g(x, y - 1)), max_diff_px(cg, orig_g(x, y + 1))),
                   max(max_diff_px(cg, orig_g(x - 1, y)), max_diff_px(cg, orig_g(x + 1, y))));
        }
        uint32_t rec;
        out[(size_t)y * W + x] = resid_px(src(x, y), pred, q, max_q, md, SG, rec);
        if (x == 0) first_rec = rec;
        L = rec;
        outv = rec;
        if (r == 63 || y == H - 1) prev_row[x] = rec;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ L0

__device__ __forceinline__ uint32_t rgba_argb(const uint8_t* q) {
  // one dword load: R | G << 8 | B << 16 | A << 24 (RGBA rows are 4-byte aligned)
  const uint32_t v = *reinterpret_cast<const uint32_t*>(q);
  return (v & 0xff00ff00u) | ((v >> 16) & 0xffu) | ((v & 0xffu) << 16);
}
// pixel x of a row: RGBA bytes, or (plane) an ALPH alpha byte as green
// (WebPDispatchAlphaToGreen, src/enc/alpha_enc.c:73)
__device__ __forceinline__ uint32_t pix_at(const uint8_t* row, int x, bool plane) {
  return plane ? (uint32_t)row[x] << 8 : rgba_argb(row + 4 * x);
}

// AnalyzeEntropy's histograms (src/enc/vp8l_enc.c:87-141, HistoIx order
// A, A', G, G', R, R', B, B', R-G, (R-G)', B-G, (B-G)', palette hash) over
// one band of rows; pixels equal to their raster predecessor or to the pixel
// above are skipped as there. One global add per non-zero bin.
#define ENTROPY_BANDS 16
__global__ __launch_bounds__(256) void k_vp8l_entropy(const uint8_t* __restrict__ rgba,
                                                      size_t fstride, int rstride, int W, int H,
                                                      int plane, uint32_t* __restrict__ ehist) {
  __shared__ uint32_t h[VP8L_EHIST];
  const int tid = threadIdx.x, f = blockIdx.y;
  const uint8_t* img = rgba + (size_t)f * fstride;
  for (int i = tid; i < VP8L_EHIST; i += 256) h[i] = 0;
  __syncthreads();
  const int y0 = (int)((long long)H * blockIdx.x / ENTROPY_BANDS);
  const int y1 = (int)((long long)H * (blockIdx.x + 1) / ENTROPY_BANDS);
  const int n = (y1 - y0) * W;   // <= 2^31: a band of rows
  // a pixel, its raster predecessor, the pixels above and above-left, loaded
  // one iteration ahead of their use
  auto load = [&](int i, uint32_t (&o)[4]) {
    const int yy = i / W, x = i - yy * W, y = y0 + yy;
    const uint8_t* row = img + (size_t)y * rstride;
    o[0] = pix_at(row, x, plane);
    o[1] = x > 0 ? pix_at(row, x - 1, plane) : y > 0 ? pix_at(row - rstride, W - 1, plane) : o[0];
    o[2] = y > 0 ? pix_at(row - rstride, x, plane) : 0u;
    o[3] = (x > 0 && y > 0) ? pix_at(row - rstride, x - 1, plane) : 0u;
  };
  uint32_t nx[4] = {0, 0, 0, 0};
  if (tid < n) load(tid, nx);
  for (int i = tid; i < n; i += 256) {
    const uint32_t pix = nx[0], prev = nx[1], up = nx[2], ul = nx[3];
    if (i + 256 < n) load(i + 256, nx);
    const int yy = i / W, x = i - yy * W, y = y0 + yy;
    {   // transparent pixels, none skipped (VP8L_EH_TRANSP): one add per wave
      const uint64_t tr = __ballot(!plane && (pix >> 24) == 0);
      if (tr && (threadIdx.x & 63) == __builtin_ctzll(__ballot(1)))
        atomicAdd(&h[VP8L_EH_TRANSP], (uint32_t)__popcll(tr));
    }
    const uint32_t d = sub_pixels(pix, prev);
    if (d == 0) continue;
    if (y > 0 && up == pix) continue;
    const int g = (int)(pix >> 8), gd = (int)(d >> 8);
    // alpha is one value over most waves: the wave-uniform fast path
    hadd(h, 0 * 256 + (pix >> 24));
    hadd(h, 1 * 256 + (d >> 24));
    atomicAdd(&h[2 * 256 + (g & 255)], 1u);
    atomicAdd(&h[3 * 256 + (gd & 255)], 1u);
    atomicAdd(&h[4 * 256 + ((pix >> 16) & 255)], 1u);
    atomicAdd(&h[5 * 256 + ((d >> 16) & 255)], 1u);
    atomicAdd(&h[6 * 256 + (pix & 255)], 1u);
    atomicAdd(&h[7 * 256 + (d & 255)], 1u);
    atomicAdd(&h[8 * 256 + ((((int)pix >> 16) - g) & 255)], 1u);
    atomicAdd(&h[9 * 256 + ((((int)d >> 16) - gd) & 255)], 1u);
    atomicAdd(&h[10 * 256 + (((int)pix - g) & 255)], 1u);
    atomicAdd(&h[11 * 256 + (((int)d - gd) & 255)], 1u);
    const uint64_t hp = ((uint64_t)pix + (pix >> 19)) * 0x39c5fba7ull;   // HashPix :81-85
    atomicAdd(&h[12 * 256 + (uint32_t)((hp & 0xffffffffull) >> 24)], 1u);
    // the transform search's accumulated histograms (model:
    // accumulated_histograms): residuals of predictor 12, or of the fixed
    // modes on row 0 (left) and column 0 (top), plain and sub-green
    const uint32_t T_ = up;
    const uint32_t L = x > 0 ? prev : 0u;
    const uint32_t TL = ul;
    const int fm = y == 0 ? 1 : (x == 0 ? 2 : 12);
    const uint32_t r = sub_pixels(pix, predict(fm, L, T_, TL, 0u));
    const uint32_t rs = sub_pixels(sub_green(pix), predict(fm, sub_green(L), sub_green(T_),
                                                          sub_green(TL), 0u));
    hadd(h, (VP8L_EH_ACC + 0) * 256 + (r >> 24));
    atomicAdd(&h[(VP8L_EH_ACC + 1) * 256 + ((r >> 16) & 255)], 1u);
    atomicAdd(&h[(VP8L_EH_ACC + 2) * 256 + ((r >> 8) & 255)], 1u);
    atomicAdd(&h[(VP8L_EH_ACC + 3) * 256 + (r & 255)], 1u);
    atomicAdd(&h[(VP8L_EH_ACC + 4) * 256 + ((rs >> 16) & 255)], 1u);
    atomicAdd(&h[(VP8L_EH_ACC + 5) * 256 + (rs & 255)], 1u);
  }
  __syncthreads();
  uint32_t* out = ehist + (size_t)f * VP8L_EHIST;
  for (int i = tid; i < VP8L_EHIST; i += 256)
    if (h[i]) atomicAdd(&out[i], h[i]);
}

// The colour set of a frame (GetColorPalette, src/utils/palette.c:95-148):
// an LDS hash table with linear probing (colour 0 kept as a flag, the empty
// slot marker), abandoned by every thread once more than 256 colours are in.
// out: count (VP8L_MAX_PALETTE + 1 = too many) then the colours unordered.
__global__ __launch_bounds__(256) void k_vp8l_palscan(const uint8_t* __restrict__ rgba,
                                                      size_t fstride, int rstride, int W, int H,
                                                      int plane, uint32_t* __restrict__ pal) {
  __shared__ uint32_t keys[1024];
  __shared__ uint32_t cnt, zero, over, outn;
  const int tid = threadIdx.x, f = blockIdx.x;
  const uint8_t* img = rgba + (size_t)f * fstride;
  for (int i = tid; i < 1024; i += 256) keys[i] = 0;
  if (tid == 0) { cnt = 0; zero = 0; over = 0; outn = 0; }
  __syncthreads();
  const long long n = (long long)W * H;
  uint32_t last = 0;
  bool have_last = false;
  for (long long i = tid; i < n; i += 256) {
    if (*(volatile uint32_t*)&over) break;
    const int y = (int)(i / W), x = (int)(i % W);
    const uint32_t pix = pix_at(img + (size_t)y * rstride, x, plane);
    if (have_last && pix == last) continue;
    last = pix; have_last = true;
    if (pix == 0) {
      if (atomicExch(&zero, 1u) == 0 && atomicAdd(&cnt, 1u) + 1 > VP8L_MAX_PALETTE) over = 1;
      continue;
    }
    uint32_t k = (pix * 0x1e35a7bdu) >> 22;
    for (;;) {
      const uint32_t old = atomicCAS(&keys[k], 0u, pix);
      if (old == 0) {
        if (atomicAdd(&cnt, 1u) + 1 > VP8L_MAX_PALETTE) over = 1;
        break;
      }
      if (old == pix) break;
      k = (k + 1) & 1023;
    }
  }
  __syncthreads();
  uint32_t* o = pal + (size_t)f * VP8L_PAL_STRIDE;
  if (over || cnt > VP8L_MAX_PALETTE) {
    if (tid == 0) o[0] = VP8L_MAX_PALETTE + 1;
    return;
  }
  for (int i = tid; i < 1024; i += 256)
    if (keys[i]) o[1 + atomicAdd(&outn, 1u)] = keys[i];
  __syncthreads();
  if (tid == 0) {
    if (zero) o[1 + outn] = 0;
    o[0] = cnt;
  }
}

// Colour indexing + VP8LBundleColorMap (src/dsp/lossless_enc.c): packed
// pixel x of row y holds the indices of pixels (x << xbits) + j in green at
// bit 8 + j * (8 >> xbits); alpha 0xff. Index = position of the colour in the
// sorted palette (binary search, SearchColorNoIdx) mapped to the stored order.
__global__ __launch_bounds__(256) void k_vp8l_palapply(const uint8_t* __restrict__ rgba,
                                                       size_t fstride, int rstride, vp8l_params p,
                                                       const int* __restrict__ fidx,
                                                       const uint32_t* __restrict__ sorted,
                                                       const uint8_t* __restrict__ sidx,
                                                       const int* __restrict__ npal,
                                                       uint32_t* __restrict__ argb_out,
                                                       uint32_t* __restrict__ alpha_flag) {
  __shared__ uint32_t sp[VP8L_MAX_PALETTE];
  __shared__ uint8_t si[VP8L_MAX_PALETTE];
  const int tid = threadIdx.x, f = blockIdx.z, y = blockIdx.y;
  const int np = npal[f];
  for (int i = tid; i < np; i += 256) {
    sp[i] = sorted[(size_t)f * VP8L_MAX_PALETTE + i];
    si[i] = sidx[(size_t)f * VP8L_MAX_PALETTE + i];
  }
  __syncthreads();
  const int x = blockIdx.x * 256 + tid;
  if (x >= p.w) return;
  const uint8_t* row = rgba + (size_t)(fidx ? fidx[f] : f) * fstride + (size_t)y * rstride;
  const int xb = p.xbits, bd = 8 >> xb;
  uint32_t code = 0;
  bool a_any = false;
  for (int j = 0; j < (1 << xb); ++j) {
    const int sx = (x << xb) + j;
    if (sx >= p.ow) break;
    const uint32_t c = pix_at(row, sx, p.alpha != 0);
    a_any |= !p.alpha && (c >> 24) != 255;
    int lo = 0, hi = np;   // sp[lo] <= c < sp[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (sp[mid] <= c) lo = mid; else hi = mid;
    }
    code |= (uint32_t)si[lo] << (8 + bd * j);
  }
  argb_out[(size_t)f * p.w * p.h + (size_t)y * p.w + x] = 0xff000000u | code;
  if (__any(a_any) && lane_id() == 0) atomicOr(&alpha_flag[f], 1u);
}

// Near-lossless preprocessing, one pass (NearLossless,
// src/enc/near_lossless_enc.c:63-101): an interior pixel whose 4-neighbourhood
// is not smooth (some channel differs by >= 2^bits) snaps each channel to the
// closest multiple of 2^bits (FindClosestDiscretized :27-34); border rows and
// columns stay. in: frame fidx[f] (NULL: f) at fstride / rstride; out: slot f,
// packed RGBA. One thread per pixel: each pass reads only the previous one.
__device__ __forceinline__ uint32_t nl_snap(uint32_t a, int bits) {
  const uint32_t mask = (1u << bits) - 1;
  const uint32_t b = a + (mask >> 1) + ((a >> bits) & 1);
  return b > 255 ? 255 : (b & ~mask);
}
// apply: per slot, 0 = copy (model: near_lossless_applies)
__global__ __launch_bounds__(256) void k_vp8l_nearlossless(const uint8_t* __restrict__ in,
                                                           size_t fstride, int rstride,
                                                           const int* __restrict__ fidx, int W,
                                                           int H, int bits,
                                                           const uint8_t* __restrict__ apply,
                                                           uint8_t* __restrict__ out) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
  if (x >= W) return;
  const uint8_t* img = in + (size_t)(fidx ? fidx[f] : f) * fstride;
  const uint32_t c = *reinterpret_cast<const uint32_t*>(img + (size_t)y * rstride + 4 * x);
  uint32_t o = c;
  if (apply[f] && x > 0 && x < W - 1 && y > 0 && y < H - 1) {
    const uint32_t nb[4] = {
        *reinterpret_cast<const uint32_t*>(img + (size_t)y * rstride + 4 * (x - 1)),
        *reinterpret_cast<const uint32_t*>(img + (size_t)y * rstride + 4 * (x + 1)),
        *reinterpret_cast<const uint32_t*>(img + (size_t)(y - 1) * rstride + 4 * x),
        *reinterpret_cast<const uint32_t*>(img + (size_t)(y + 1) * rstride + 4 * x)};
    const int limit = 1 << bits;
    bool smooth = true;
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int sh = 0; sh < 32; sh += 8) {
        const int d = (int)((c >> sh) & 255) - (int)((nb[k] >> sh) & 255);
        smooth &= d < limit && d > -limit;
      }
    if (!smooth) {
      o = 0;
#pragma unroll
      for (int sh = 0; sh < 32; sh += 8) o |= nl_snap((c >> sh) & 255, bits) << sh;
    }
  }
  *reinterpret_cast<uint32_t*>(out + ((size_t)f * H + y) * W * 4 + 4 * x) = o;
}

// ------------------------------------------------------------------ L2

// A frame's pixels in stream order are cut into S segments of whole 64-pixel
// chunks, one wave each, walked at once. A wave keeps the decoder's colour
// caches of every size b = 1..9 in LDS (2 + 4 + ... + 512 entries). The keys
// of size b are the top b bits of one 9-bit key, so the lanes sharing a key
// of every size come from 9 ballots (most significant bit first, AND-ed). A
// lane's cache content is the value of its nearest lower same-key lane, else
// the table entry; the highest lane of each key group updates the table (the
// other lanes write a slot of their own, no branch). The nine sizes are
// independent: all lane exchanges, then all table reads, then all table
// writes, so their latencies overlap. Out: per pixel the smallest size whose
// cache holds it (hits are monotone in the size: the most recent same-key
// pixel at b is also the most recent one at b + 1), one byte store per lane.
//
// Segment 0 starts from the zeroed caches (VP8LColorCacheInit); a later
// segment does not know its start, so an entry it has not written yet is
// unknown. Unknown at b means no earlier same-key pixel in the segment, so
// it is unknown at b + 1 too: a pixel whose smallest known hit is not below
// its first unknown size u leaves VP8L_CACHE_PARTIAL | u, and the segment's
// final tables go to cseg. k_vp8l_cache_start turns those into each
// segment's start contents; k_vp8l_match settles the partial pixels there.
#define CACHE_BATCH 8
__device__ __forceinline__ int cache_seg_begin(int s, int S, int nchunk) {
  return (int)((long long)nchunk * s / S);
}
__device__ __forceinline__ int cache_seg_of(int c, int S, int nchunk) {   // begin(s) <= c < begin(s+1)
  return (int)(((long long)(c + 1) * S - 1) / nchunk);
}

__global__ __launch_bounds__(64) void k_vp8l_cache(const uint32_t* __restrict__ argb, int npix,
                                                   int S, uint8_t* __restrict__ minb,
                                                   uint2* __restrict__ cseg) {
  __shared__ uint2 tab[VP8L_CACHE_TAB + 64];   // (value, written); + one dump slot per lane
  const int s = blockIdx.x, f = blockIdx.y, ln = lane_id();
  const uint32_t* E = argb + (size_t)f * npix;
  const int nchunk = (npix + 63) >> 6;
  const int cb = cache_seg_begin(s, S, nchunk), ce = cache_seg_begin(s + 1, S, nchunk);
  uint8_t* out = minb + (size_t)f * npix;
  for (int i = ln; i < VP8L_CACHE_TAB; i += 64) tab[i] = make_uint2(0u, s == 0 ? 1u : 0u);
  __syncthreads();
  const uint64_t below = (1ull << ln) - 1ull;
  uint32_t cur[CACHE_BATCH], nxt[CACHE_BATCH];
#pragma unroll
  for (int k = 0; k < CACHE_BATCH; ++k) {
    const int q = ((cb + k) << 6) + ln;
    cur[k] = (cb + k < ce && q < npix) ? E[q] : 0;
  }
  for (int c0 = cb; c0 < ce; c0 += CACHE_BATCH) {
#pragma unroll
    for (int k = 0; k < CACHE_BATCH; ++k) {
      const int c = c0 + CACHE_BATCH + k, q = (c << 6) + ln;
      nxt[k] = (c < ce && q < npix) ? E[q] : 0;
    }
#pragma unroll
    for (int k = 0; k < CACHE_BATCH; ++k) {
      const int c = c0 + k;
      if (c >= ce) break;
      const int q = (c << 6) + ln;
      const bool valid = q < npix;
      const uint32_t v = cur[k];
      const uint32_t key9 = (v * HASH_MUL) >> (32 - VP8L_MAX_CACHE_BITS);
      uint64_t m[VP8L_MAX_CACHE_BITS];
      uint32_t pv[VP8L_MAX_CACHE_BITS];
      uint2 tv[VP8L_MAX_CACHE_BITS];
      uint64_t acc = __ballot(valid);
#pragma unroll
      for (int b = 1; b <= VP8L_MAX_CACHE_BITS; ++b) {
        const bool bit = (key9 >> (VP8L_MAX_CACHE_BITS - b)) & 1;
        const uint64_t bv = __ballot(valid && bit);
        acc &= bit ? bv : ~bv;
        m[b - 1] = acc;
      }
#pragma unroll
      for (int b = 1; b <= VP8L_MAX_CACHE_BITS; ++b) {
        const uint64_t lower = m[b - 1] & below;
        pv[b - 1] = __shfl(v, lower ? 63 - __clzll((long long)lower) : ln);
        tv[b - 1] = tab[(1 << b) - 2 + (key9 >> (VP8L_MAX_CACHE_BITS - b))];
      }
      uint32_t mb = VP8L_NEVER_HIT, u = VP8L_NEVER_HIT;
#pragma unroll
      for (int b = VP8L_MAX_CACHE_BITS; b >= 1; --b) {
        const bool low = (m[b - 1] & below) != 0;
        const uint32_t held = low ? pv[b - 1] : tv[b - 1].x;
        if (!low && !tv[b - 1].y) u = b;
        else if (held == v) mb = b;
      }
      if (mb == VP8L_NEVER_HIT && u < VP8L_NEVER_HIT) mb = VP8L_CACHE_PARTIAL | u;
      if (valid) out[q] = (uint8_t)mb;
      // LDS ops of a wave stay in order: every read above precedes these writes
#pragma unroll
      for (int b = 1; b <= VP8L_MAX_CACHE_BITS; ++b) {
        const bool top = valid && (m[b - 1] >> ln) == 1ull;
        tab[top ? (1 << b) - 2 + (key9 >> (VP8L_MAX_CACHE_BITS - b)) : VP8L_CACHE_TAB + ln] =
            make_uint2(v, 1u);
      }
    }
#pragma unroll
    for (int k = 0; k < CACHE_BATCH; ++k) cur[k] = nxt[k];
  }
  if (s + 1 < S) {
    __syncthreads();
    uint2* o = cseg + ((size_t)f * S + s) * VP8L_CACHE_TAB;
    for (int i = ln; i < VP8L_CACHE_TAB; i += 64) o[i] = tab[i];
  }
}

// per frame and cache entry, the segments' start contents in place: the
// value of the latest earlier segment that wrote the entry, else 0
__global__ __launch_bounds__(1024) void k_vp8l_cache_start(int S, uint2* __restrict__ cseg) {
  const int e = threadIdx.x, f = blockIdx.x;
  if (e >= VP8L_CACHE_TAB) return;
  uint2* t = cseg + (size_t)f * S * VP8L_CACHE_TAB + e;
  uint32_t cur = 0;
  for (int s = 0; s < S; ++s) {
    const uint2 w = s + 1 < S ? t[(size_t)s * VP8L_CACHE_TAB] : make_uint2(0u, 0u);
    t[(size_t)s * VP8L_CACHE_TAB] = make_uint2(cur, 1u);
    if (w.y) cur = w.x;
  }
}

// a partial pixel of L2: its sizes from u up hold the segment's start contents
__device__ __forceinline__ uint32_t cache_settle(uint32_t mb, uint32_t v, size_t q, int npix, int S,
                                                 const uint2* __restrict__ cstart) {
  const int nchunk = (npix + 63) >> 6;
  const uint2* t = cstart + (size_t)cache_seg_of((int)(q >> 6), S, nchunk) * VP8L_CACHE_TAB;
  const uint32_t key9 = (v * HASH_MUL) >> (32 - VP8L_MAX_CACHE_BITS);
  for (int b = (int)(mb & 15); b <= VP8L_MAX_CACHE_BITS; ++b)
    if (t[(1 << b) - 2 + (key9 >> (VP8L_MAX_CACHE_BITS - b))].x == v) return (uint32_t)b;
  return VP8L_NEVER_HIT;
}

// ------------------------------------------------------------------ L3

// One wave per row, chunks of 64 pixels right to left: for each candidate
// distance the run of equal pixels starting at every x (ballot of the 64
// comparisons; count trailing ones; a run reaching the chunk end continues
// with the run at the next chunk's start), the longest (first on ties,
// capped at MAX_LENGTH) and the smallest cache size holding the pixel (L2's,
// settled here where L2 left it partial), packed per pixel as
// len | cand << 13 | minb << 15 for the parse.
__global__ __launch_bounds__(64) void k_vp8l_match(const uint32_t* __restrict__ argb,
                                                   uint8_t* __restrict__ minb,
                                                   const uint2* __restrict__ cstart, int S,
                                                   vp8l_params p, uint32_t* __restrict__ bm) {
  // XCD-aware rows: the hardware deals consecutive workgroup ids to the 8
  // XCDs in turn, so row y-1 (the row above's candidates) would be read into
  // another XCD's L2; instead each XCD takes a contiguous run of (frame, row)
  // (k_vp8l_match read 20.3 GB per 1024-frame launch from HBM, 2.4x the frames)
  const unsigned total = gridDim.x * gridDim.y, id = blockIdx.x + gridDim.x * blockIdx.y;
  const unsigned xcd = id & 7u, chunk = total >> 3, rem = total & 7u;
  const unsigned g = xcd * chunk + min(xcd, rem) + (id >> 3);
  const int f = (int)(g / gridDim.x), y = (int)(g % gridDim.x), ln = lane_id();
  const int W = p.w;
  const size_t npix = (size_t)W * p.h;
  const uint32_t* E = argb + f * npix;
  uint8_t* MB = minb + (size_t)f * npix;
  uint32_t* O = bm + f * npix;
  const size_t row = (size_t)y * W;
  int carry[VP8L_NUM_CAND] = {0, 0, 0, 0};
  // chunk c's pixel, its 4 candidates and its cache size, loaded one chunk
  // ahead of their use (the walk is serial over the row's chunks)
  struct Ld { uint32_t e, cv[VP8L_NUM_CAND], mb; };
  auto load = [&](int c, Ld& o) {
    const int x = (c << 6) + ln;
    const bool valid = c >= 0 && x < W;
    const size_t q = row + (size_t)(valid ? x : 0);
    o.e = valid ? E[q] : 0u;
#pragma unroll
    for (int k = 0; k < VP8L_NUM_CAND; ++k) {
      const int d = p.dist[k];
      o.cv[k] = (valid && d > 0 && (size_t)d <= q) ? E[q - d] : ~o.e;   // ~e: never equal
    }
    o.mb = valid ? MB[q] : 0u;
  };
  Ld cur, nxt;
  load((W - 1) >> 6, cur);
  for (int c = (W - 1) >> 6; c >= 0; --c) {
    load(c - 1, nxt);
    const int x = (c << 6) + ln;
    const bool valid = x < W;
    const size_t q = row + (size_t)x;
    const uint32_t e = cur.e;
    int bn = 0, bk = 0;
#pragma unroll
    for (int k = 0; k < VP8L_NUM_CAND; ++k) {
      const bool ok = valid && cur.cv[k] == e;
      const uint64_t mask = __ballot(ok);
      const uint64_t miss = ~(mask >> ln);   // zero when all 64 lanes from lane 0 match:
      int run = miss ? (int)__builtin_ctzll(miss) : 64;   // ctz(0) is undefined (gives 31)
      if (run == 64 - ln) run += carry[k];
      carry[k] = __shfl(run, 0);
      const int n = min(run, VP8L_MAX_LENGTH);
      if (n > bn) { bn = n; bk = k; }
    }
    if (valid) {
      uint32_t mb = cur.mb;
      if (mb & VP8L_CACHE_PARTIAL) {   // settled here, and kept for the shortest-path parse
        mb = cache_settle(mb, e, q, (int)npix, S, cstart + (size_t)f * S * VP8L_CACHE_TAB);
        MB[q] = (uint8_t)mb;
      }
      O[q] = (uint32_t)bn | ((uint32_t)bk << 13) | (mb << 15);
    }
    cur = nxt;
  }
}

// Greedy copy / cache / literal over the packed match words (model: parse),
// each row on its own. A wave owns 64 rows (one per lane) and walks them in
// 64-pixel chunks staged through LDS: the chunk's 64 x 64 words are loaded
// row by row (coalesced), every lane parses its row up to the chunk end, the
// chunk goes back coalesced. Positions a copy from an earlier chunk covers
// are marked when their chunk is loaded (xs[] = each row's parse position).
// A hit is a pixel held by the cache of the frame's size. Provisional pass
// (cbits == NULL): every hit of the largest cache, act | (len - 1) << 2 into
// prov, the match words kept; final pass: the frame's size cbits[f], the
// match words rewritten in place as parse ops.
__global__ __launch_bounds__(64) void k_vp8l_parse(vp8l_params p, uint32_t* __restrict__ ops,
                                                   uint16_t* __restrict__ prov,
                                                   const uint8_t* __restrict__ cbits) {
  __shared__ uint32_t tile[64][65];
  __shared__ int xs[64];
  const int f = blockIdx.y, ln = lane_id();
  const int W = p.w, H = p.h, y0 = blockIdx.x * 64;
  const int nrows = min(64, H - y0);
  const size_t npix = (size_t)W * H;
  uint32_t* O = ops + f * npix + (size_t)y0 * W;
  const bool final_pass = cbits != nullptr;
  uint16_t* P = final_pass ? nullptr : prov + f * npix + (size_t)y0 * W;
  const uint32_t cb = final_pass ? cbits[f] : (uint32_t)p.cache_bits;
  int x = 0;   // this lane's row position
  xs[ln] = 0;
  for (int cx = 0; cx < W; cx += 64) {
    const int cw = min(64, W - cx);
    __syncthreads();
    // 16 rows' loads in flight at a time (a load behind the covered test
    // would wait for each row in turn)
    for (int r0 = 0; r0 < nrows; r0 += 16) {
      uint32_t v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        v[k] = (r0 + k < nrows && ln < cw) ? O[(size_t)(r0 + k) * W + cx + ln] : 0u;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (r0 + k < nrows && ln < cw)
          tile[r0 + k][ln] = cx + ln < xs[r0 + k] ? 0xffffffffu : v[k];   // covered: marker
    }
    __syncthreads();
    if (ln < nrows) {
      while (x < cx + cw) {
        const int i = x - cx;
        const uint32_t m = tile[ln][i];
        const int bn = (int)(m & 0x1fff), bk = (int)((m >> 13) & 3);
        const bool hit = cb > 0 && (m >> 15) <= cb;
        if (bn >= VP8L_MIN_COPY || (bn == 2 && !hit)) {
          tile[ln][i] = final_pass ? 2u | ((uint32_t)(bn - 1) << 2) | ((uint32_t)p.dcode[bk] << 14)
                                   : 2u | ((uint32_t)(bn - 1) << 2);
          const int e = min(x + bn, cx + cw);
          for (int j = i + 1; j < e - cx; ++j) tile[ln][j] = 3u;
          x += bn;
        } else {
          tile[ln][i] = hit ? 1u : 0u;
          ++x;
        }
      }
      xs[ln] = x;
    }
    __syncthreads();
    for (int r = 0; r < nrows; ++r) {
      if (ln < cw) {
        uint32_t v = tile[r][ln];
        if (v == 0xffffffffu) v = 3u;
        if (final_pass) O[(size_t)r * W + cx + ln] = v;
        else P[(size_t)r * W + cx + ln] = (uint16_t)v;
      }
    }
  }
}

// ------------------------------------------------------------------ symbols

namespace {

struct PixSym {
  int s[4];          // symbol in G|R|B|A|D space, -1 none (write order s0 x0 s1 x1 s2 s3)
  uint32_t xv[2];    // extra bits after s0 (length) and after s1 (distance)
  int xb[2];
};

__device__ __forceinline__ void prefix_enc(uint32_t v, int& sym, int& nb, uint32_t& ex) {
  const uint32_t d = v - 1;
  if (d < 4) { sym = (int)d; nb = 0; ex = 0; return; }
  const int h = 31 - __clz((int)d);
  sym = 2 * h + (int)((d >> (h - 1)) & 1);
  nb = h - 1;
  ex = d & ((1u << (h - 1)) - 1);
}

__device__ __forceinline__ void pix_symbols(uint32_t op, uint32_t a, int cb, PixSym& o) {
  const uint32_t act = op & 3;
  o.s[0] = o.s[1] = o.s[2] = o.s[3] = -1;
  o.xv[0] = o.xv[1] = 0; o.xb[0] = o.xb[1] = 0;
  if (act == 0) {
    o.s[0] = (int)((a >> 8) & 255);
    o.s[1] = VP8L_GS + (int)((a >> 16) & 255);
    o.s[2] = VP8L_GS + 256 + (int)(a & 255);
    o.s[3] = VP8L_GS + 512 + (int)(a >> 24);
  } else if (act == 1) {
    o.s[0] = 280 + (int)((a * HASH_MUL) >> (32 - cb));
  } else if (act == 2) {
    int sym, nb; uint32_t ex;
    prefix_enc(((op >> 2) & 0xfff) + 1, sym, nb, ex);
    o.s[0] = 256 + sym; o.xv[0] = ex; o.xb[0] = nb;
    prefix_enc(op >> 14, sym, nb, ex);
    o.s[1] = VP8L_GS + 768 + sym; o.xv[1] = ex; o.xb[1] = nb;
  }
}

// alphabet index of a symbol in the concatenated space
__device__ __forceinline__ int alph_of(int s) {
  return s < VP8L_GS ? 0 : s < VP8L_GS + 256 ? 1 : s < VP8L_GS + 512 ? 2 : s < VP8L_GS + 768 ? 3 : 4;
}
// alphabet sizes of a frame with a colour cache of cb bits (the green
// alphabet's cache part is 2^cb of the layout's 2^VP8L_MAX_CACHE_BITS)
__device__ __forceinline__ int alph_size(int a, int cb) {
  return a == 0 ? 280 + (cb ? 1 << cb : 0) : a == 4 ? 40 : 256;
}

__device__ __forceinline__ long long flog2_fx64(const int32_t* frac, unsigned long long v) {
  const int e = 63 - __clzll((long long)v);
  const unsigned long long m = (e >= 10 ? (v >> (e - 10)) : (v << (10 - e))) & 1023;
  return ((long long)e << 12) + frac[m];
}

}  // namespace

// ------------------------------------------------------------------ L3p
// Colour-indexed frames: the cost-model parse over long-range matches
// (model: palette_parse and the lz_* functions, oracle/vp8l_model.py; the
// reference's VP8LHashChainFill, backward_references_enc.c:259-452, and
// TraceBackwards, backward_references_cost_enc.c:569-795).

#define LZ_SEG 4096
#define LZ_MAX_LENGTH 4095
#define LZ_HASH_SIZE (1 << 18)
#define LZ_ITER_MAX (8 + (75 * 75) / 128)
#define LZ_WINDOW_CAP ((1 << 18) - 121)
#define LZ_NCOST (280 + 3 * 256 + 40)   // G+length | R | B | A | D
#define LZ_INF 0x7fffffff

__device__ __forceinline__ uint32_t lz_hash(uint32_t a, uint32_t b) {
  return (b * 0xc6a4a793u + a * 0x5bd1e996u) >> (32 - 18);
}

// R[q] = equal pixels starting at q, capped at LZ_MAX_LENGTH + 3 (model:
// lz_runs): one wave per frame, 64-pixel chunks from the end, a run reaching
// a chunk's end continues with the next chunk's first run.
// Runs of equal pixels (capped at LZ_MAX_LENGTH + 3), one wave per piece of
// LZ_RUN_PIECE positions: the walk goes backwards 64 positions at a time and
// starts LZ_RUN_LOOK positions past the piece with no carry. The run it has
// at the piece's last position is then the capped run of the whole-frame
// walk (a run reaching the walk's start is at least LZ_RUN_LOOK long there,
// past the cap), so every piece matches one backward walk over the frame.
#define LZ_RUN_PIECE 16384
#define LZ_RUN_LOOK 4160
static_assert(LZ_RUN_LOOK >= LZ_MAX_LENGTH + 4 && LZ_RUN_LOOK % 64 == 0 && LZ_RUN_PIECE % 64 == 0,
              "the look-ahead must cover the run cap");
__global__ __launch_bounds__(64) void k_lz_runs(const uint32_t* __restrict__ argb, int npix,
                                                uint16_t* __restrict__ runs) {
  const int f = blockIdx.y, ln = lane_id();
  const int p0 = blockIdx.x * LZ_RUN_PIECE;
  if (p0 >= npix) return;   // whole wave
  const int p1 = min(npix, p0 + LZ_RUN_PIECE), top = min(npix, p1 + LZ_RUN_LOOK);
  const uint32_t* E = argb + (size_t)f * npix;
  uint16_t* R = runs + (size_t)f * npix;
  int carry = 0;   // run at the first position of the chunk after this one
  for (int c = (top - 1) >> 6; c >= (p0 >> 6); --c) {
    const int q = (c << 6) + ln;
    const bool valid = q < npix;
    const bool eq = valid && q + 1 < npix && E[q] == E[q + 1];
    const uint64_t mask = __ballot(eq);
    const uint64_t miss = ~(mask >> ln);
    int run = (miss ? (int)__builtin_ctzll(miss) : 64) + 1;   // this pixel + equal followers
    if (run == 65 - ln) run += carry - 1 >= 0 ? carry - 1 : 0;
    if (run > LZ_MAX_LENGTH + 3) run = LZ_MAX_LENGTH + 3;
    if (valid && q < p1) R[q] = (uint16_t)run;
    carry = __shfl(run, 0);
  }
}

// The hash chain (model: lz_hash_chain): one wave per frame walks the
// positions 64 at a time; the lanes sharing a hash come from 18 ballots, a
// lane's link is its nearest lower inserting lane of the same hash, else the
// table entry, and the highest inserting lane of each hash updates the table
// (n x 2^18 words in HBM, -1 filled by the caller).
__global__ __launch_bounds__(64) void k_lz_chain(const uint32_t* __restrict__ argb, int npix,
                                                 const uint16_t* __restrict__ runs,
                                                 int32_t* __restrict__ htab,
                                                 int32_t* __restrict__ chain) {
  const int f = blockIdx.x, ln = lane_id();
  const uint32_t* E = argb + (size_t)f * npix;
  const uint16_t* R = runs + (size_t)f * npix;
  int32_t* T = htab + (size_t)f * LZ_HASH_SIZE;
  int32_t* C = chain + (size_t)f * npix;
  const uint64_t below = (1ull << ln) - 1ull;
  for (int c = 0; c < (npix + 63) >> 6; ++c) {
    const int q = (c << 6) + ln;
    const bool look0 = q <= npix - 2 && npix > 2;
    uint32_t key = 0;
    bool skip = false;
    if (look0) {
      const int r = R[q];
      if (r >= 3) {
        skip = r - 2 > LZ_MAX_LENGTH;
        key = lz_hash(E[q], (uint32_t)(r - 2));
      } else {
        key = lz_hash(E[q], E[q + 1]);
      }
    }
    const bool look = look0 && !skip;
    const bool ins = look && q <= npix - 3;
    uint64_t acc = __ballot(ins);
#pragma unroll
    for (int b = 17; b >= 0; --b) {
      const bool bit = (key >> b) & 1;
      const uint64_t bv = __ballot(ins && bit);
      acc &= bit ? bv : ~bv;
    }
    const uint64_t lower = acc & below;
    int32_t link = -1;
    if (look)
      link = lower ? (c << 6) + (63 - __clzll((long long)lower))
                   : __hip_atomic_load(&T[key], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (q < npix) C[q] = look ? link : -1;
    // every lane has read the table above before the writes below (one wave,
    // program order; the loads are waited for by the link store); table
    // reads and writes go to L2 (agent scope), so the next chunk's reads see
    // this chunk's writes
    if (ins && (acc >> ln) == 1ull)
      __hip_atomic_store(&T[key], (int32_t)q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Per position the chain's best match (model: lz_hash_search): one thread
// per position.
__global__ __launch_bounds__(256) void k_lz_search(const uint32_t* __restrict__ argb, int W,
                                                   int npix, const int32_t* __restrict__ chain,
                                                   uint32_t* __restrict__ hoff,
                                                   uint16_t* __restrict__ hlen) {
  const int f = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  const uint32_t* E = argb + (size_t)f * npix;
  const int32_t* C = chain + (size_t)f * npix;
  uint32_t bd = 0;
  int bl = 0;
  if (p >= 1 && p <= npix - 2) {
    const int seg_end = (p / LZ_SEG + 1) * LZ_SEG;
    const int max_len = min(min(npix - 1 - p, LZ_MAX_LENGTH), seg_end - p);
    auto mlen = [&](int a) {
      int k = 0;
      while (k < max_len && E[a + k] == E[p + k]) ++k;
      return k;
    };
    const int window = min(W << 8, LZ_WINDOW_CAP);
    const int min_pos = max(p - window, 0);
    const int length_max = min(max_len, 256);
    int it = LZ_ITER_MAX;
    int q = C[p];
    if (p >= W) {
      const int c = mlen(p - W);
      if (c > bl) { bl = c; bd = (uint32_t)W; }
      --it;
    }
    {
      const int c = mlen(p - 1);
      if (c > bl) { bl = c; bd = 1; }
      --it;
    }
    if (bl == LZ_MAX_LENGTH) q = min_pos - 1;
    while (q >= min_pos) {
      if (--it == 0) break;
      if (E[q + bl] == E[p + bl]) {
        const int c = mlen(q);
        if (c > bl) {
          bl = c; bd = (uint32_t)(p - q);
          if (bl >= length_max) break;
        }
      }
      q = C[q];
    }
  }
  hoff[(size_t)f * npix + p] = bd;
  hlen[(size_t)f * npix + p] = (uint16_t)bl;
}

// Per position the longest run against the 4 candidate distances within its
// segment (model: lz_local): one wave per segment, 64-pixel chunks from the
// segment end, ballots as in k_vp8l_match.
__global__ __launch_bounds__(64) void k_lz_local(const uint32_t* __restrict__ argb, vp8l_params p,
                                                 uint32_t* __restrict__ loff,
                                                 uint16_t* __restrict__ llen) {
  const int f = blockIdx.y, ln = lane_id();
  const int npix = p.w * p.h;
  const int s = blockIdx.x * LZ_SEG, e = min(npix, s + LZ_SEG);
  const uint32_t* E = argb + (size_t)f * npix;
  int carry[VP8L_NUM_CAND] = {0, 0, 0, 0};
  const int nch = (e - s + 63) >> 6;
  for (int c = nch - 1; c >= 0; --c) {
    const int q = s + (c << 6) + ln;
    const bool valid = q < e;
    const uint32_t v = valid ? E[q] : 0u;
    int bn = 0, bk = 0;
#pragma unroll
    for (int k = 0; k < VP8L_NUM_CAND; ++k) {
      const int d = p.dist[k];
      const bool ok = valid && d > 0 && d <= q && E[q - d] == v;
      const uint64_t mask = __ballot(ok);
      const uint64_t miss = ~(mask >> ln);
      int run = miss ? (int)__builtin_ctzll(miss) : 64;
      if (run == 64 - ln) run += carry[k];
      carry[k] = __shfl(run, 0);
      const int n = min(run, LZ_MAX_LENGTH);
      if (n > bn) { bn = n; bk = k; }
    }
    if (valid) {
      loff[(size_t)f * npix + q] = bn ? (uint32_t)p.dist[bk] : 0u;
      llen[(size_t)f * npix + q] = (uint16_t)bn;
    }
  }
}

// Symbol costs of a frame's parse (model: lz_costs / lz_pop_costs): one
// workgroup per frame, histograms in LDS, 1/256 bit per symbol. est (may be
// null): the parse's bits under those costs, extra bits included (model:
// lz_est_bits).
__global__ __launch_bounds__(1024) void k_lz_costs(const uint32_t* __restrict__ argb,
                                                   const uint32_t* __restrict__ ops, int npix,
                                                   const int32_t* __restrict__ frac,
                                                   int32_t* __restrict__ costs,
                                                   unsigned long long* __restrict__ est) {
  __shared__ uint32_t h[LZ_NCOST];
  __shared__ uint32_t tot[5], nz[5];
  __shared__ unsigned long long xbits, bits;
  const int f = blockIdx.x, tid = threadIdx.x;
  const uint32_t* E = argb + (size_t)f * npix;
  const uint32_t* O = ops + (size_t)f * npix;
  for (int i = tid; i < LZ_NCOST; i += 1024) h[i] = 0;
  if (tid < 5) { tot[tid] = 0; nz[tid] = 0; }
  if (tid == 0) { xbits = 0; bits = 0; }
  __syncthreads();
  uint32_t myx = 0;   // this thread's extra bits
  for (int q = tid; q < npix; q += 1024) {
    const uint32_t op = O[q], act = op & 3;
    if (act == 0) {
      const uint32_t a = E[q];
      atomicAdd(&h[(a >> 8) & 255], 1u);
      atomicAdd(&h[280 + ((a >> 16) & 255)], 1u);
      atomicAdd(&h[536 + (a & 255)], 1u);
      atomicAdd(&h[792 + (a >> 24)], 1u);
    } else if (act == 2) {
      int sym, nb; uint32_t ex;
      prefix_enc(((op >> 2) & 0xfff) + 1, sym, nb, ex);
      atomicAdd(&h[256 + sym], 1u);
      myx += (uint32_t)nb;
      prefix_enc(op >> 14, sym, nb, ex);
      atomicAdd(&h[1048 + sym], 1u);
      myx += (uint32_t)nb;
    }
  }
  if (est && myx) atomicAdd(&xbits, (unsigned long long)myx);
  __syncthreads();
  auto alph = [](int i) { return i < 280 ? 0 : i < 536 ? 1 : i < 792 ? 2 : i < 1048 ? 3 : 4; };
  for (int i = tid; i < LZ_NCOST; i += 1024)
    if (h[i]) { atomicAdd(&tot[alph(i)], h[i]); atomicAdd(&nz[alph(i)], 1u); }
  __syncthreads();
  int32_t* out = costs + (size_t)f * LZ_NCOST;
  unsigned long long mine = 0;
  for (int i = tid; i < LZ_NCOST; i += 1024) {
    const int a = alph(i);
    int32_t c = 0;
    if (nz[a] > 1)
      c = (flog2_fx(frac, tot[a]) - (h[i] ? flog2_fx(frac, h[i]) : 0)) >> 4;
    out[i] = c;
    mine += (unsigned long long)h[i] * (unsigned long long)c;
  }
  if (est) {
    if (mine) atomicAdd(&bits, mine);
    __syncthreads();
    if (tid == 0) est[f] = bits + 256ull * xbits;
  }
}

// The first parse of the cost-model route (model: palette_parse): per frame
// the cheaper of the two first parses' costs (the row parse on ties)
__global__ __launch_bounds__(256) void k_lz_pick(const unsigned long long* __restrict__ est_row,
                                                 const unsigned long long* __restrict__ est_chain,
                                                 const int32_t* __restrict__ costs_row,
                                                 int32_t* __restrict__ costs) {
  const int f = blockIdx.x;
  if (est_chain[f] < est_row[f]) return;   // costs hold the chain parse's already
  for (int i = threadIdx.x; i < LZ_NCOST; i += 256)
    costs[(size_t)f * LZ_NCOST + i] = costs_row[(size_t)f * LZ_NCOST + i];
}

// VP8L distance code of a distance (model: distance_code): the plane code
// table of the frame width for short distances (dcodes[d], 0 = none), else
// d + 120
__device__ __forceinline__ uint32_t lz_dcode(const uint8_t* dcodes, int nd, uint32_t d) {
  const uint32_t c = d < (uint32_t)nd ? dcodes[d] : 0u;
  return c ? c : d + 120;
}

// The first parse of the cost-model route (model: lz_greedy): per segment
// from its start, the longer of the chain match and the local match (the
// chain's on ties), cut at the segment end, when it is at least
// LZ_GREEDY_MIN long, else a literal. One wave per segment: the lengths
// staged in LDS, lane 0 walks them (a copy's distance is read at its start
// only), the wave writes the segment's ops.
#define LZ_GREEDY_MIN 3
__global__ __launch_bounds__(64) void k_lz_greedy(int npix, const uint32_t* __restrict__ hoff,
                                                  const uint16_t* __restrict__ hlen,
                                                  const uint32_t* __restrict__ loff,
                                                  const uint16_t* __restrict__ llen,
                                                  const uint8_t* __restrict__ dcodes, int nd,
                                                  uint32_t* __restrict__ ops) {
  __shared__ uint16_t hl[LZ_SEG], ll[LZ_SEG];
  __shared__ uint32_t op[LZ_SEG];
  const int f = blockIdx.y, ln = lane_id();
  const int s = blockIdx.x * LZ_SEG, m = min(npix, s + LZ_SEG) - s;
  const size_t base = (size_t)f * npix + s;
  for (int i = ln; i < m; i += 64) {
    hl[i] = hlen[base + i];
    ll[i] = llen[base + i];
    op[i] = 0u;
  }
  __syncthreads();
  if (ln == 0) {
    int j = 0;
    while (j < m) {
      const int a = min((int)hl[j], m - j), b = min((int)ll[j], m - j);
      const bool loc = b > a;
      const int L = loc ? b : a;
      if (L >= LZ_GREEDY_MIN) {
        const uint32_t d = loc ? loff[base + j] : hoff[base + j];
        op[j] = 2u | ((uint32_t)(L - 1) << 2) | (lz_dcode(dcodes, nd, d) << 14);
        for (int t = j + 1; t < j + L; ++t) op[t] = 3u;
        j += L;
      } else {
        ++j;
      }
    }
  }
  __syncthreads();
  for (int i = ln; i < m; i += 64) ops[base + i] = op[i];
}

// The cost-model parse of one segment (model: lz_dp): one wave per segment,
// the path costs / choices in LDS; per position the literal (lane 0), then
// the chain match and then the local match, each with one lane per length of
// LZ_LENGTHS (and one for the match's own length). Lanes of one match write
// distinct targets; the matches run one after the other (one wave: LDS ops
// in program order). Then lane 0 walks the choices back and the wave writes
// the segment's ops.
__constant__ int16_t kLzLengths[32] = {2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17,
                                       32, 33, 64, 65, 128, 129, 256, 257, 512, 513, 1024,
                                       1025, 2048, 2049, 0, 0};
#define LZ_NLEN 30
struct LzSmem {
  int32_t cost[LZ_SEG + 1];
  uint32_t cd[LZ_SEG + 1];   // choice ending here: length k (12 bits) | distance << 12 (18 bits)
  int32_t tab[LZ_NCOST];
};
static_assert(LZ_MAX_LENGTH < (1 << 12) && LZ_WINDOW_CAP < (1 << 18) && 16384 + 1 < (1 << 18),
              "LzSmem::cd packs a length and a distance (window, or a local one <= width + 1)");
__global__ __launch_bounds__(64) void k_lz_dp(const uint32_t* __restrict__ argb, int W, int npix,
                                              const int32_t* __restrict__ costs,
                                              const uint32_t* __restrict__ hoff,
                                              const uint16_t* __restrict__ hlen,
                                              const uint32_t* __restrict__ loff,
                                              const uint16_t* __restrict__ llen,
                                              const uint8_t* __restrict__ dcodes, int nd,
                                              uint32_t* __restrict__ ops) {
  __shared__ LzSmem S;
  const int f = blockIdx.y, ln = lane_id();
  const int s = blockIdx.x * LZ_SEG, e = min(npix, s + LZ_SEG), m = e - s;
  const uint32_t* E = argb + (size_t)f * npix;
  const size_t base = (size_t)f * npix;
  for (int i = ln; i < LZ_NCOST; i += 64) S.tab[i] = costs[(size_t)f * LZ_NCOST + i];
  for (int i = ln; i <= m; i += 64) { S.cost[i] = i ? LZ_INF : 0; S.cd[i] = 0; }
  __syncthreads();
  const int32_t* cG = S.tab;
  const int32_t* cR = S.tab + 280;
  const int32_t* cB = S.tab + 536;
  const int32_t* cA = S.tab + 792;
  const int32_t* cD = S.tab + 1048;
  const int myk = ln < LZ_NLEN ? kLzLengths[ln] : 0;
  int lcost_my = 0;   // this lane's listed length: its prefix cost (per frame)
  if (myk) {
    int sym, nb; uint32_t ex;
    prefix_enc((uint32_t)myk, sym, nb, ex);
    lcost_my = cG[256 + sym] + 256 * nb;
  }
  // Everything a position needs that does not depend on the path costs --
  // its literal cost, and per match the length L, the distance's cost, the
  // own-length lane's length and cost -- is worked out 64 positions at a
  // time, one position per lane, and read back with readlane in the serial
  // walk; the chunk's inputs are loaded a chunk ahead. (With the loads and
  // the distance-code lookup on the walk's path it waited ~1 us per
  // position: 175 ms per launch on 64 copied-tile 1080p frames,
  // profiles/r4/lzprof.)
  uint32_t pa = 0, ph = 0, pl = 0, phl = 0, pll = 0;
  auto fetch = [&](int j0) {
    const int q = j0 + ln;
    pa = ph = pl = phl = pll = 0;
    if (q < m) {
      const size_t i = base + s + q;
      pa = E[s + q]; ph = hoff[i]; pl = loff[i]; phl = hlen[i]; pll = llen[i];
    }
  };
  fetch(0);
  for (int j0 = 0; j0 < m; j0 += 64) {
    const uint32_t ca = pa, cd[2] = {ph, pl}, cl[2] = {phl, pll};
    if (j0 + 64 < m) fetch(j0 + 64);   // in flight during this chunk
    const int jn = min(64, m - j0);
    const int q = j0 + ln, rem = e - (s + q);   // positions left in the segment from q
    const int litc = ((cA[ca >> 24] + cR[(ca >> 16) & 255] + cG[(ca >> 8) & 255] + cB[ca & 255]) *
                      82) / 100;
    int mL[2], mdc[2], mok[2], mol[2];
#pragma unroll
    for (int mk = 0; mk < 2; ++mk) {
      const int L = q < m ? min((int)cl[mk], rem) : 0;
      mL[mk] = L;
      mdc[mk] = mok[mk] = mol[mk] = 0;
      if (L >= 2) {
        int sym, nb; uint32_t ex;
        prefix_enc(lz_dcode(dcodes, nd, cd[mk]), sym, nb, ex);
        mdc[mk] = cD[sym] + 256 * nb;
        bool own_listed = false;
#pragma unroll
        for (int t = 0; t < LZ_NLEN; ++t) own_listed |= kLzLengths[t] == L;
        if (!own_listed) {
          prefix_enc((uint32_t)L, sym, nb, ex);
          mok[mk] = L;
          mol[mk] = cG[256 + sym] + 256 * nb;
        }
      }
    }
    for (int jj = 0; jj < jn; ++jj) {
      const int j = j0 + jj;
      const int c = S.cost[j];
      if (ln == 0) {
        const int v = c + __builtin_amdgcn_readlane(litc, jj);
        if (v < S.cost[j + 1]) { S.cost[j + 1] = v; S.cd[j + 1] = 1; }
      }
#pragma unroll
      for (int mk = 0; mk < 2; ++mk) {
        const int L = __builtin_amdgcn_readlane(mL[mk], jj);
        if (L < 2) continue;   // wave-uniform
        const int dc = c + __builtin_amdgcn_readlane(mdc[mk], jj);
        // lane LZ_NLEN takes the match's own length when it is not in the list
        int k = myk, lc = lcost_my;
        if (ln == LZ_NLEN) {
          k = __builtin_amdgcn_readlane(mok[mk], jj);
          lc = __builtin_amdgcn_readlane(mol[mk], jj);
        }
        if (k >= 2 && k <= L) {
          const int v = dc + lc;
          if (v < S.cost[j + k]) {
            S.cost[j + k] = v;
            S.cd[j + k] = (uint32_t)k | ((uint32_t)__builtin_amdgcn_readlane((int)cd[mk], jj) << 12);
          }
        }
      }
    }
  }
  __syncthreads();
  // trace back: mark copy starts (ch value at the start position: 2 | k << 2
  // with the code), the rest literal or inside
  if (ln == 0) {
    int j = m;
    while (j > 0) {
      const uint32_t cdj = S.cd[j];
      const int k = (int)(cdj & 4095u);
      const int st = j - k;
      if (k >= 2) {
        S.cost[st] = (int32_t)(2u | ((uint32_t)(k - 1) << 2) | (lz_dcode(dcodes, nd, cdj >> 12) << 14));
        for (int t = st + 1; t < j; ++t) S.cost[t] = 3;
      } else {
        S.cost[st] = 0;
      }
      j = st;
    }
  }
  __syncthreads();
  for (int i = ln; i < m; i += 64) ops[base + s + i] = (uint32_t)S.cost[i];
}

// ------------------------------------------------------------------ L3b

// Cache-size choice, statistics (model: choose_cache_bits): one workgroup
// per frame over the provisional parse. A pixel coded as literal or cache hit
// with smallest holding size c goes to class c: its G, R, B, A bytes (the
// literal it is for every size < c) and its 9-bit key (the cache symbol it is
// for every size >= c); copies add their length prefix.
__global__ __launch_bounds__(1024) void k_vp8l_cachehist(const uint32_t* __restrict__ argb,
                                                         const uint32_t* __restrict__ match,
                                                         const uint16_t* __restrict__ prov,
                                                         int npix, uint32_t* __restrict__ chist) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  uint32_t* h = reinterpret_cast<uint32_t*>(smem_raw);
  const int tid = threadIdx.x, f = blockIdx.x;
  for (int i = tid; i < VP8L_CHIST; i += 1024) h[i] = 0;
  __syncthreads();
  const size_t base = (size_t)f * npix;
  // the three words of a pixel loaded one iteration ahead of their use
  uint32_t op_n = 0, v_n = 0, m_n = 0;
  if (tid < npix) { op_n = prov[base + tid]; v_n = argb[base + tid]; m_n = match[base + tid]; }
  for (int q = tid; q < npix; q += 1024) {
    const uint32_t op = op_n, v = v_n, mw = m_n;
    if (q + 1024 < npix) {
      op_n = prov[base + q + 1024]; v_n = argb[base + q + 1024]; m_n = match[base + q + 1024];
    }
    const uint32_t act = op & 3;
    if (act == 3) continue;
    if (act == 2) {
      int sym, nb; uint32_t ex;
      prefix_enc((op >> 2) + 1, sym, nb, ex);
      atomicAdd(&h[VP8L_CH_LEN + sym], 1u);
      continue;
    }
    const int c = (int)(mw >> 15);   // smallest cache size holding it
    const uint32_t L = VP8L_CH_LIT + (uint32_t)(c - 1) * 1024;   // lanes differ in class:
    hadd(h, L + ((v >> 8) & 255));                               // full index for hadd
    hadd(h, L + 256 + ((v >> 16) & 255));
    hadd(h, L + 512 + (v & 255));
    hadd(h, L + 768 + (v >> 24));
    if (c <= VP8L_MAX_CACHE_BITS)
      atomicAdd(&h[VP8L_CH_KEY + (c - 1) * 512 + ((v * HASH_MUL) >> (32 - VP8L_MAX_CACHE_BITS))], 1u);
  }
  __syncthreads();
  uint32_t* o = chist + (size_t)f * VP8L_CHIST;
  for (int i = tid; i < VP8L_CHIST; i += 1024) o[i] = h[i];
}

namespace {
// bits_entropy_fx of the model from (sum, nonzeros, max, sum of n log2 n)
__device__ long long bits_entropy_fx(const int32_t* frac, unsigned long long sum, int nonzeros,
                                     unsigned long long mx, long long sl) {
  if (nonzeros <= 1) return 0;
  const long long s = (long long)sum;
  const long long ent = (s > 1 ? s * flog2_fx64(frac, sum) : 0) - sl;
  if (nonzeros == 2) return (99 * s * 4096 + ent) / 100;
  const long long mix = nonzeros == 3 ? 950 : nonzeros == 4 ? 700 : 627;
  long long ml = (2 * s - (long long)mx) * 4096;
  ml = (mix * ml + (1000 - mix) * ent) / 1000;
  return ent < ml ? ml : ent;
}
}  // namespace

// Cache-size choice (model: choose_cache_bits): for every size b = 0..9 the
// four codes' estimates from the class histograms; the smallest (first on
// ties) becomes cbits[f].
__global__ __launch_bounds__(256) void k_vp8l_cachechoose(const uint32_t* __restrict__ chist,
                                                          const int32_t* __restrict__ frac,
                                                          int max_bits,
                                                          uint8_t* __restrict__ cbits) {
  __shared__ unsigned long long red[4][4][4];   // [wave][alphabet][sum, nz, max, slog]
  const int tid = threadIdx.x, f = blockIdx.x, wv = tid >> 6;
  const uint32_t* h = chist + (size_t)f * VP8L_CHIST;
  long long best = 0;
  int best_b = 0;
  for (int b = 0; b <= max_bits; ++b) {
    const int ng = 280 + (b ? 1 << b : 0);
    unsigned long long sum[4] = {0, 0, 0, 0}, mx[4] = {0, 0, 0, 0}, nz[4] = {0, 0, 0, 0};
    long long sl[4] = {0, 0, 0, 0};
    for (int i = tid; i < ng + 768; i += 256) {
      int a, ch = 0, bin = 0;
      uint32_t v = 0;
      if (i < ng) {
        a = 0;
        if (i < 256) { ch = 0; bin = i; }
        else if (i < 280) { v = h[VP8L_CH_LEN + i - 256]; ch = -1; }
        else {   // cache symbol k of size b: classes 1..b, keys k << (9 - b) ..
          const int k = i - 280, sh = VP8L_MAX_CACHE_BITS - b;
          for (int c = 1; c <= b; ++c)
            for (int j = 0; j < (1 << sh); ++j)
              v += h[VP8L_CH_KEY + (c - 1) * 512 + (k << sh) + j];
          ch = -1;
        }
      } else {
        a = 1 + (i - ng) / 256;            // R, B, A
        ch = a; bin = (i - ng) & 255;
      }
      if (ch >= 0)
        for (int c = b + 1; c <= VP8L_NEVER_HIT; ++c) v += h[VP8L_CH_LIT + (c - 1) * 1024 + ch * 256 + bin];
      if (v) {
        sum[a] += v; nz[a] += 1;
        if (v > mx[a]) mx[a] = v;
        if (v > 1) sl[a] += (long long)v * flog2_fx(frac, v);
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      sum[a] = wave_sum(sum[a]); nz[a] = wave_sum(nz[a]); sl[a] = wave_sum(sl[a]);
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long t = __shfl_xor(mx[a], o);
        mx[a] = t > mx[a] ? t : mx[a];
      }
    }
    __syncthreads();
    if (lane_id() == 0)
      for (int a = 0; a < 4; ++a) {
        red[wv][a][0] = sum[a]; red[wv][a][1] = nz[a]; red[wv][a][2] = mx[a];
        red[wv][a][3] = (unsigned long long)sl[a];
      }
    __syncthreads();
    if (tid == 0) {
      long long e = 0;
      for (int a = 0; a < 4; ++a) {
        unsigned long long S = 0, N = 0, X = 0;
        long long L = 0;
        for (int w = 0; w < 4; ++w) {
          S += red[w][a][0]; N += red[w][a][1];
          X = red[w][a][2] > X ? red[w][a][2] : X;
          L += (long long)red[w][a][3];
        }
        e += bits_entropy_fx(frac, S, (int)N, X, L);
      }
      if (b == 0 || e < best) { best = e; best_b = b; }
    }
  }
  if (tid == 0) cbits[f] = (uint8_t)best_b;
}

// ------------------------------------------------------------------ L4

// One workgroup per histogram tile: the tile's symbol histogram in LDS, its
// own entropy per pixel (the clustering's initial order), and the histogram
// as a sparse list (symbol | count << 12) for the clustering passes.
__global__ __launch_bounds__(256) void k_vp8l_tilefeat(const uint32_t* __restrict__ argb,
                                                       const uint32_t* __restrict__ ops,
                                                       vp8l_params p,
                                                       const uint8_t* __restrict__ cbits,
                                                       const int32_t* __restrict__ frac,
                                                       int64_t* __restrict__ feat,
                                                       uint32_t* __restrict__ tl,
                                                       uint32_t* __restrict__ tn) {
  __shared__ uint32_t h[VP8L_NS];
  __shared__ unsigned long long acc[6];
  __shared__ uint32_t nnz;
  const int tid = threadIdx.x, f = blockIdx.y, t = blockIdx.x;
  const int W = p.w, H = p.h, hb = p.hb;
  const int cb = cbits[f];
  const int tx_n = (W + (1 << hb) - 1) >> hb;
  const int tiles = tx_n * ((H + (1 << hb) - 1) >> hb);
  const int x0 = (t % tx_n) << hb, y0 = (t / tx_n) << hb;
  const int tw = min(1 << hb, W - x0), th = min(1 << hb, H - y0);
  const size_t npix = (size_t)W * H;
  for (int i = tid; i < VP8L_NS; i += 256) h[i] = 0;
  if (tid < 6) acc[tid] = 0;
  if (tid == 0) nnz = 0;
  __syncthreads();
  for (int i0 = tid; i0 < tw * th; i0 += 4 * 256) {   // 4 pixels' loads in flight
    uint32_t o4[4], a4[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 256 * u;
      o4[u] = a4[u] = 0;
      if (i < tw * th) {
        const int ly = i / tw, lx = i - ly * tw;
        const size_t q = f * npix + (size_t)(y0 + ly) * W + x0 + lx;
        o4[u] = ops[q];
        a4[u] = argb[q];
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + 256 * u >= tw * th) break;
      PixSym s;
      pix_symbols(o4[u], a4[u], cb, s);
      for (int k = 0; k < 4; ++k)
        if (s.s[k] >= 0) hadd(h, (uint32_t)s.s[k]);
    }
  }
  __syncthreads();
  // per alphabet: N, then own = sum_a N_a log N_a - sum h log h
  unsigned long long n[5] = {0, 0, 0, 0, 0};
  unsigned long long hl = 0;
  const size_t cap = VP8L_TILE_CAP(hb);
  uint32_t* out = tl + ((size_t)f * tiles + t) * cap;
  for (int i0 = 0; i0 < VP8L_NS; i0 += 256) {
    const int i = i0 + tid;
    const uint32_t c = i < VP8L_NS ? h[i] : 0u;
    if (i < VP8L_NS) n[alph_of(i)] += c;
    if (c > 1) hl += (unsigned long long)c * (unsigned long long)flog2_fx(frac, c);
    // the non-zero bins' slots: one LDS atomic per wave, a ballot prefix inside
    const uint64_t nzm = __ballot(c != 0);
    uint32_t base = 0;
    if (lane_id() == 0 && nzm) base = atomicAdd(&nnz, (uint32_t)__popcll(nzm));
    base = __shfl(base, 0);
    if (c) out[base + __popcll(nzm & ((1ull << lane_id()) - 1ull))] = (uint32_t)i | (c << 12);
  }
  for (int a = 0; a < 5; ++a) n[a] = wave_sum(n[a]);
  hl = wave_sum(hl);
  if (lane_id() == 0) {
    for (int a = 0; a < 5; ++a) atomicAdd(&acc[a], n[a]);
    atomicAdd(&acc[5], hl);
  }
  __syncthreads();
  if (tid == 0) {
    long long own = 0;
    for (int a = 0; a < 5; ++a)
      if (acc[a] > 1) own += (long long)acc[a] * flog2_fx64(frac, acc[a]);
    own -= (long long)acc[5];
    feat[(size_t)f * tiles + t] = own / (long long)(tw * th);
    tn[(size_t)f * tiles + t] = nnz;
  }
}

// ------------------------------------------------------------------ L5

struct ClusterSmem {
  uint32_t hc[VP8L_KMAX * VP8L_NS];
  union {
    uint16_t lc[VP8L_NS * VP8L_KMAX];   // per symbol the cost under each cluster (1/256 bit)
    long long feat[VP8L_MAX_HUFF_IMAGE];
  } u;
  uint8_t assign[VP8L_MAX_HUFF_IMAGE];
  uint32_t nsum[VP8L_KMAX * 5];
};

// The cluster of each tile: the cheapest under the per-symbol costs lc
// (symbol-major, 16 x u16). Narrow tiles (counts < 2^16, sums < 2^32): every
// pair of clusters is two dot2 steps of one cost word (v_dot2_u32_u16);
// wider ones sum in 64 bits, 8 clusters per pass over the tile's list. The
// tile's histogram then goes into its new cluster's (S.hc, zeroed by the
// caller once lc was built): the next iteration's accumulation done in the
// same pass over the lists, whose second read of the tile hits the cache
// (one pass over every frame's tile lists per iteration instead of two).
__device__ __forceinline__ void reassign_tiles(ClusterSmem& S, const uint32_t* __restrict__ TL,
                                               const uint32_t* __restrict__ TN, size_t cap, int nt,
                                               int K, bool narrow, int wv, int ln) {
  typedef unsigned short us2 __attribute__((ext_vector_type(2)));
  for (int t = wv; t < nt; t += 16) {
    const uint32_t* e = TL + (size_t)t * cap;
    const int m = (int)TN[t];
    int bc = 0;
    if (narrow) {
      uint32_t cost[VP8L_KMAX];
#pragma unroll
      for (int c = 0; c < VP8L_KMAX; ++c) cost[c] = 0;
      for (int i0 = ln; i0 < m; i0 += 256) {   // 4 loads in flight per lane
        uint32_t ev[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) ev[u] = i0 + 64 * u < m ? e[i0 + 64 * u] : 0u;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t v = ev[u];   // 0: past the list (count 0 adds nothing)
          const uint32_t cnt = v >> 12;
          const uint4* row = reinterpret_cast<const uint4*>(S.u.lc + (v & 4095) * VP8L_KMAX);
          const uint4 w0 = row[0], w1 = row[1];
          const uint32_t w[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
          const us2 lo = {(unsigned short)cnt, 0}, hi = {0, (unsigned short)cnt};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const us2 pr = __builtin_bit_cast(us2, w[j]);
            cost[2 * j] = __builtin_amdgcn_udot2(pr, lo, cost[2 * j], false);
            cost[2 * j + 1] = __builtin_amdgcn_udot2(pr, hi, cost[2 * j + 1], false);
          }
        }
      }
      uint32_t bv = ~0u;
#pragma unroll
      for (int c = 0; c < VP8L_KMAX; ++c) {
        const uint32_t v = wave_sum(cost[c]);
        if (c < K && v < bv) { bv = v; bc = c; }
      }
    } else {
      unsigned long long bv = ~0ull;
      for (int h = 0; h < 2; ++h) {
        unsigned long long cost[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) cost[c] = 0;
        for (int i = ln; i < m; i += 64) {
          const uint32_t v = e[i];
          const unsigned long long cnt = v >> 12;
          const uint4 w = reinterpret_cast<const uint4*>(S.u.lc + (v & 4095) * VP8L_KMAX)[h];
          const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            cost[2 * j] += cnt * (ww[j] & 0xffffu);
            cost[2 * j + 1] += cnt * (ww[j] >> 16);
          }
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const unsigned long long v = wave_sum(cost[c]);
          if (8 * h + c < K && v < bv) { bv = v; bc = 8 * h + c; }
        }
      }
    }
    if (ln == 0) S.assign[t] = (uint8_t)bc;
    uint32_t* hcc = S.hc + bc * VP8L_NS;
    for (int i = ln; i < m; i += 64) {
      const uint32_t v = e[i];
      if (v) atomicAdd(&hcc[v & 4095], v >> 12);
    }
  }
}

// One workgroup per frame (16 waves): k-means of the histogram tiles over
// their sparse histograms (model: cluster_tiles). A wave owns a tile at a
// time in both the accumulation and the reassignment passes.
__global__ __launch_bounds__(1024) void k_vp8l_cluster(vp8l_params p,
                                                       const uint8_t* __restrict__ cbits,
                                                       const int32_t* __restrict__ frac,
                                                       const int64_t* __restrict__ feat,
                                                       const uint32_t* __restrict__ tl,
                                                       const uint32_t* __restrict__ tn,
                                                       uint32_t* __restrict__ hc_out,
                                                       uint8_t* __restrict__ assign_out) {
  extern __shared__ __align__(16) unsigned char smem_raw[];
  ClusterSmem& S = *reinterpret_cast<ClusterSmem*>(smem_raw);
  const int tid = threadIdx.x, f = blockIdx.x, wv = tid >> 6, ln = lane_id();
  const int W = p.w, H = p.h, hb = p.hb, K = p.k;
  const int cb = cbits[f];
  const int tx_n = (W + (1 << hb) - 1) >> hb, ty_n = (H + (1 << hb) - 1) >> hb;
  const int nt = tx_n * ty_n;
  const size_t cap = VP8L_TILE_CAP(hb);
  const uint32_t* TL = tl + (size_t)f * nt * cap;
  const uint32_t* TN = tn + (size_t)f * nt;
  // a tile's counts fit 16 bits and its costs 32 (count sum <= 4 px, cost < 2^16)
  const bool narrow = (1 << (2 * hb)) <= 16384;

  // init: rank by (feature, tile), K quantiles
  for (int t = tid; t < nt; t += 1024) S.u.feat[t] = feat[(size_t)f * nt + t];
  __syncthreads();
  for (int t = tid; t < nt; t += 1024) {
    const long long ft = S.u.feat[t];
    int r = 0;
    for (int u = 0; u < nt; ++u) {
      const long long fu = S.u.feat[u];
      r += (fu < ft) || (fu == ft && u < t);
    }
    S.assign[t] = (uint8_t)((long long)r * K / nt);
  }
  __syncthreads();

  // accumulate the initial clusters' histograms; every iteration then
  // rebuilds them inside its reassignment pass
  for (int i = tid; i < K * VP8L_NS; i += 1024) S.hc[i] = 0;
  __syncthreads();
  for (int t = wv; t < nt; t += 16) {
    uint32_t* hcc = S.hc + S.assign[t] * VP8L_NS;
    const uint32_t* e = TL + (size_t)t * cap;
    const int m = (int)TN[t];
    for (int i0 = ln; i0 < m; i0 += 256) {   // 4 loads in flight per lane
      uint32_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = i0 + 64 * j < m ? e[i0 + 64 * j] : 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (v[j]) atomicAdd(&hcc[v[j] & 4095], v[j] >> 12);
    }
  }
  __syncthreads();
  for (int it = 0; it < VP8L_CLUSTER_ITERS; ++it) {
    // per-symbol costs (1/256 bit): log2((10 N + A) / (10 n + 1))
    for (int i = tid; i < K * 5; i += 1024) S.nsum[i] = 0;
    __syncthreads();
    for (int c = 0; c < K; ++c) {
      uint32_t n[5] = {0, 0, 0, 0, 0};
      for (int i = tid; i < VP8L_NS; i += 1024) n[alph_of(i)] += S.hc[c * VP8L_NS + i];
      for (int a = 0; a < 5; ++a) {
        n[a] = wave_sum(n[a]);
        if (ln == 0 && n[a]) atomicAdd(&S.nsum[c * 5 + a], n[a]);
      }
    }
    __syncthreads();
    // symbol-major, all 16 slots of a symbol in 32 bytes (unused clusters 0)
    for (int i = tid; i < VP8L_KMAX * VP8L_NS; i += 1024) {
      const int s = i >> 4, c = i & 15, a = alph_of(s);
      int v = 0;
      if (c < K)
        v = flog2_fx(frac, 10u * S.nsum[c * 5 + a] + (uint32_t)alph_size(a, cb)) -
            flog2_fx(frac, 10u * S.hc[c * VP8L_NS + s] + 1u);
      S.u.lc[i] = (uint16_t)(v >> 4);
    }
    __syncthreads();
    for (int i = tid; i < K * VP8L_NS; i += 1024) S.hc[i] = 0;
    __syncthreads();
    // reassign (one wave per tile) + the new clusters' histograms
    reassign_tiles(S, TL, TN, cap, nt, K, narrow, wv, ln);
    __syncthreads();
  }
  uint32_t* ho = hc_out + (size_t)f * VP8L_KMAX * VP8L_NS;
  for (int i = tid; i < K * VP8L_NS; i += 1024) ho[i] = S.hc[i];
  for (int t = tid; t < nt; t += 1024) assign_out[(size_t)f * nt + t] = S.assign[t];
}

// ------------------------------------------------------------------ L6/L7

namespace {
__device__ __forceinline__ int pix_bits(const PixSym& s, const uint32_t* ct) {
  int b = s.xb[0] + s.xb[1];
  for (int k = 0; k < 4; ++k)
    if (s.s[k] >= 0) b += (int)(ct[s.s[k]] >> 16);
  return b;
}
static_assert(VP8L_BLOCK == 4 * 256, "bit writer: 4 pixels per thread");
// words q0..q0+3 of a frame's array (one 16-byte load when all are inside
// and aligned: frames of npix % 4 == 0)
__device__ __forceinline__ void load4(const uint32_t* __restrict__ a, size_t q0, size_t npix,
                                      uint32_t (&o)[4]) {
  if (q0 + 4 <= npix && ((reinterpret_cast<uintptr_t>(a + q0) & 15) == 0)) {
    const uint4 v = *reinterpret_cast<const uint4*>(a + q0);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = q0 + k < npix ? a[q0 + k] : 0u;
  }
}
__device__ __forceinline__ const uint32_t* pixel_codes(const vp8l_params& p, const uint32_t* ctab,
                                                       const uint8_t* gtile, int f, size_t q) {
  const int W = p.w, hb = p.hb;
  const int tx_n = (W + (1 << hb) - 1) >> hb, ty_n = (p.h + (1 << hb) - 1) >> hb;
  const uint32_t qq = (uint32_t)q, y = qq / (uint32_t)W, x = qq - y * (uint32_t)W;
  const int g = gtile[(size_t)f * tx_n * ty_n + (y >> hb) * tx_n + (x >> hb)];
  return ctab + ((size_t)f * VP8L_KMAX + g) * VP8L_NS;
}
}  // namespace

__global__ __launch_bounds__(256) void k_vp8l_bitcount(const uint32_t* __restrict__ argb,
                                                       const uint32_t* __restrict__ ops,
                                                       vp8l_params p,
                                                       const uint8_t* __restrict__ cbits,
                                                       const uint32_t* __restrict__ ctab,
                                                       const uint8_t* __restrict__ gtile,
                                                       uint32_t* __restrict__ bsum) {
  __shared__ uint32_t tot;
  const int tid = threadIdx.x, f = blockIdx.y, blk = blockIdx.x;
  const size_t npix = (size_t)p.w * p.h;
  const int nblk = (int)((npix + VP8L_BLOCK - 1) / VP8L_BLOCK);
  if (tid == 0) tot = 0;
  __syncthreads();
  uint32_t b = 0;
  const size_t q0 = (size_t)blk * VP8L_BLOCK + tid * (VP8L_BLOCK / 256);
  const int cb = cbits[f];
  uint32_t op4[4], px4[4];
  load4(ops + f * npix, q0, npix, op4);
  load4(argb + f * npix, q0, npix, px4);
#pragma unroll
  for (int k = 0; k < VP8L_BLOCK / 256; ++k) {
    const size_t q = q0 + k;
    if (q >= npix) break;
    PixSym s;
    pix_symbols(op4[k], px4[k], cb, s);
    b += pix_bits(s, pixel_codes(p, ctab, gtile, f, q));
  }
  b = wave_sum(b);
  if (lane_id() == 0) atomicAdd(&tot, b);
  __syncthreads();
  if (tid == 0) bsum[(size_t)f * nblk + blk] = tot;
}

__global__ __launch_bounds__(1024) void k_vp8l_scan(const uint32_t* __restrict__ bsum, int nblk,
                                                    const uint64_t* __restrict__ start_bit,
                                                    uint64_t* __restrict__ boff,
                                                    uint64_t* __restrict__ end_bit) {
  __shared__ unsigned long long part[1024];
  const int tid = threadIdx.x, f = blockIdx.x;
  // each thread owns a contiguous range of blocks
  const int per = (nblk + 1023) / 1024;
  const int b0 = tid * per, b1 = min(nblk, b0 + per);
  unsigned long long s = 0;
  for (int b = b0; b < b1; ++b) s += bsum[(size_t)f * nblk + b];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {   // inclusive Hillis-Steele scan
    const unsigned long long v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  unsigned long long off = start_bit[f] + (tid ? part[tid - 1] : 0);
  for (int b = b0; b < b1; ++b) {
    boff[(size_t)f * nblk + b] = off;
    off += bsum[(size_t)f * nblk + b];
  }
  if (tid == 1023) end_bit[f] = start_bit[f] + part[1023];
}

__global__ __launch_bounds__(256) void k_vp8l_write(const uint32_t* __restrict__ argb,
                                                    const uint32_t* __restrict__ ops, vp8l_params p,
                                                    const uint8_t* __restrict__ cbits,
                                                    const uint32_t* __restrict__ ctab,
                                                    const uint8_t* __restrict__ gtile,
                                                    const uint32_t* __restrict__ bsum,
                                                    const uint64_t* __restrict__ boff,
                                                    uint8_t* __restrict__ out, size_t out_cap) {
  // block bits <= 1024 px * 4 symbols * 15 + 2 * 18 extra -> < 2^17; +2 words
  __shared__ uint32_t words[VP8L_BLOCK * 78 / 32 + 4];
  __shared__ uint32_t tsum[256];
  const int tid = threadIdx.x, f = blockIdx.y, blk = blockIdx.x;
  const size_t npix = (size_t)p.w * p.h;
  const int nblk = (int)((npix + VP8L_BLOCK - 1) / VP8L_BLOCK);
  const unsigned long long B0 = boff[(size_t)f * nblk + blk];
  const uint32_t Bn = bsum[(size_t)f * nblk + blk];
  if (Bn == 0) return;
  const unsigned long long w0 = B0 >> 5;
  const int nw = (int)(((B0 + Bn + 31) >> 5) - w0);
  for (int i = tid; i < nw; i += 256) words[i] = 0;
  PixSym s[VP8L_BLOCK / 256];
  const uint32_t* ct[VP8L_BLOCK / 256];
  uint32_t mine = 0;
  const size_t q0 = (size_t)blk * VP8L_BLOCK + tid * (VP8L_BLOCK / 256);
  const int cb = cbits[f];
  uint32_t op4[4], px4[4];
  load4(ops + f * npix, q0, npix, op4);
  load4(argb + f * npix, q0, npix, px4);
#pragma unroll
  for (int k = 0; k < VP8L_BLOCK / 256; ++k) {
    const size_t q = q0 + k;
    if (q < npix) {
      pix_symbols(op4[k], px4[k], cb, s[k]);
      ct[k] = pixel_codes(p, ctab, gtile, f, q);
      mine += pix_bits(s[k], ct[k]);
    } else {
      s[k].s[0] = s[k].s[1] = s[k].s[2] = s[k].s[3] = -1;
      s[k].xb[0] = s[k].xb[1] = 0;
      ct[k] = ctab;
    }
  }
  tsum[tid] = mine;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t v = tid >= o ? tsum[tid - o] : 0;
    __syncthreads();
    tsum[tid] += v;
    __syncthreads();
  }
  uint32_t pos = (uint32_t)(B0 & 31) + tsum[tid] - mine;   // bit position within words[]
  auto put = [&](uint32_t v, int nb) {
    if (nb == 0) return;
    const int wi = (int)(pos >> 5), sh = (int)(pos & 31);
    atomicOr(&words[wi], v << sh);
    if (sh + nb > 32) atomicOr(&words[wi + 1], v >> (32 - sh));
    pos += (uint32_t)nb;
  };
#pragma unroll
  for (int k = 0; k < VP8L_BLOCK / 256; ++k) {
    const PixSym& ps = s[k];
    const uint32_t* c = ct[k];
    if (ps.s[0] >= 0) put(c[ps.s[0]] & 0xffff, (int)(c[ps.s[0]] >> 16));
    put(ps.xv[0], ps.xb[0]);
    if (ps.s[1] >= 0) put(c[ps.s[1]] & 0xffff, (int)(c[ps.s[1]] >> 16));
    put(ps.xv[1], ps.xb[1]);
    if (ps.s[2] >= 0) put(c[ps.s[2]] & 0xffff, (int)(c[ps.s[2]] >> 16));
    if (ps.s[3] >= 0) put(c[ps.s[3]] & 0xffff, (int)(c[ps.s[3]] >> 16));
  }
  __syncthreads();
  uint32_t* O = reinterpret_cast<uint32_t*>(out + (size_t)f * out_cap);
  for (int i = tid; i < nw; i += 256) {
    const uint32_t v = words[i];
    if ((w0 + i + 1) * 4 > out_cap) break;   // overflow: the host reports it from end_bit
    if (i == 0 || i == nw - 1) {
      if (v) atomicOr(&O[w0 + i], v);
    } else {
      O[w0 + i] = v;
    }
  }
}

// ------------------------------------------------------------------ staging

// headers packed back to back (4-byte aligned offsets hoff[f], word counts
// hwords[f]) -> the start of each frame's output slab
__global__ __launch_bounds__(256) void k_vp8l_put_headers(const uint32_t* __restrict__ hdr,
                                                          const uint64_t* __restrict__ hoff,
                                                          const uint32_t* __restrict__ hwords,
                                                          uint8_t* __restrict__ out,
                                                          size_t out_cap) {
  const int f = blockIdx.y;
  const uint32_t n = hwords[f];
  const uint32_t* src = hdr + (hoff[f] >> 2);
  uint32_t* dst = reinterpret_cast<uint32_t*>(out + (size_t)f * out_cap);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) dst[i] = src[i];
}

// payloads (bytes[f]) -> one packed buffer at poff[f] + 20, 16-byte aligned
// frame starts, for a single device-to-host copy
__global__ __launch_bounds__(256) void k_vp8l_pack(const uint8_t* __restrict__ out, size_t out_cap,
                                                   const uint64_t* __restrict__ poff,
                                                   const uint64_t* __restrict__ end_bit,
                                                   uint8_t* __restrict__ packed) {
  const int f = blockIdx.y;
  if (poff[f + 1] == poff[f]) return;   // frame failed on the host: nothing to copy
  const size_t bytes = (size_t)((end_bit[f] + 7) >> 3);
  const size_t words = (bytes + 3) >> 2;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(out + (size_t)f * out_cap);
  uint32_t* dst = reinterpret_cast<uint32_t*>(packed + poff[f] + 20);   // poff 16-aligned
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < words; i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

// ------------------------------------------------------------------ launchers

static int check_launch() { return hipGetLastError() == hipSuccess; }
#define CHK_LAUNCH(x) \
  do {                \
    if ((x) != hipSuccess) return 0; \
  } while (0)

// L0b: the repeat test of a frame (oracle/vp8l_model.py: repeat_stats). One
// workgroup per frame: every sampled 8-pixel window (columns 0, 16, ..., rows
// 0, ystep, ...) that is busy (no pixel equal to its left neighbour) goes
// into an LDS hash set of its 32-bit key by linear probing; out[2f] = busy
// windows, out[2f + 1] = those whose key was already in the set. The set
// holds 2 x VP8L_REP_MAX_SAMPLES keys, so it never fills.
#define REP_SLOTS (2 * VP8L_REP_MAX_SAMPLES)
__global__ __launch_bounds__(1024) void k_vp8l_repeat(const uint8_t* __restrict__ rgba,
                                                      size_t fstride, int rstride, int w, int h,
                                                      int ystep, uint32_t* __restrict__ out) {
  extern __shared__ uint32_t rset[];   // REP_SLOTS keys, 0 = empty
  __shared__ uint32_t cnt[2];
  const int f = blockIdx.x, t = threadIdx.x;
  for (int i = t; i < REP_SLOTS; i += 1024) rset[i] = 0;
  if (t < 2) cnt[t] = 0;
  __syncthreads();
  const int nx = (w - 8) / 16 + 1, ny = (h + ystep - 1) / ystep;
  const uint8_t* F = rgba + (size_t)f * fstride;
  uint32_t nb = 0, nr = 0;
  for (int i = t; i < nx * ny; i += 1024) {
    const int y = (i / nx) * ystep, x = (i % nx) * 16;
    const uint8_t* q = F + (size_t)y * rstride + 4 * (size_t)x;
    uint32_t key = 0, prev = 0;
    bool busy = true;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t px = ((uint32_t)q[4 * k + 3] << 24) | ((uint32_t)q[4 * k] << 16) |
                          ((uint32_t)q[4 * k + 1] << 8) | q[4 * k + 2];
      if (k && px == prev) busy = false;
      prev = px;
      key = key * 0x9E3779B1u + px;
    }
    if (!busy) continue;
    ++nb;
    if (key == 0) key = 1;
    uint32_t slot = (key * 0x85EBCA6Bu) % REP_SLOTS;
    for (;;) {
      const uint32_t old = atomicCAS(&rset[slot], 0u, key);
      if (old == 0u) break;
      if (old == key) { ++nr; break; }
      slot = slot + 1 == REP_SLOTS ? 0 : slot + 1;
    }
  }
  atomicAdd(&cnt[0], nb);
  atomicAdd(&cnt[1], nr);
  __syncthreads();
  if (t < 2) out[2 * f + t] = cnt[t];
}

extern "C" int vp8l_launch_repeat(const uint8_t* rgba, size_t fstride, int rstride, int w, int h,
                                  int n, int ystep, uint32_t* out, void* stream) {
  if (w < 8 || h <= 0 || n <= 0 || ystep <= 0) return 0;
  if ((size_t)((w - 8) / 16 + 1) * (size_t)((h + ystep - 1) / ystep) > VP8L_REP_MAX_SAMPLES) return 0;
  static bool lds_ok = [] {
    return hipFuncSetAttribute((const void*)k_vp8l_repeat, hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)(REP_SLOTS * sizeof(uint32_t))) == hipSuccess;
  }();
  if (!lds_ok) return 0;
  hipLaunchKernelGGL(k_vp8l_repeat, dim3(n), dim3(1024), REP_SLOTS * sizeof(uint32_t),
                     (hipStream_t)stream, rgba, fstride, rstride, w, h, ystep, out);
  return check_launch();
}

extern "C" int vp8l_launch_scan(const uint8_t* rgba, size_t fstride, int rstride, int w, int h,
                                int n, int plane, uint32_t* ehist, uint32_t* pal, void* stream) {
  if (w <= 0 || h <= 0 || n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_vp8l_entropy, dim3(ENTROPY_BANDS, n), dim3(256), 0, st, rgba, fstride,
                     rstride, w, h, plane, ehist);
  hipLaunchKernelGGL(k_vp8l_palscan, dim3(n), dim3(256), 0, st, rgba, fstride, rstride, w, h, plane,
                     pal);
  return check_launch();
}

template <int T, bool SG>
static int launch_predsel(const uint8_t* rgba, size_t fstride, int rstride, const vp8l_params* p,
                          const int* fidx, const uint8_t* fmode, const uint8_t* pexact,
                          const float* ftabs, uint8_t* modes, uint32_t* pflag, uint32_t* argb,
                          hipStream_t st) {
  static bool lds_ok = [] {
    return hipFuncSetAttribute((const void*)k_vp8l_predsel<T, SG>,
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)sizeof(PredSelSmem<T>)) == hipSuccess;
  }();
  if (!lds_ok) return 0;
  hipLaunchKernelGGL((k_vp8l_predsel<T, SG>), dim3(p->n), dim3(PS_THREADS), sizeof(PredSelSmem<T>),
                     st, rgba, fstride, rstride, *p, fidx, fmode, pexact, ftabs, modes, pflag);
  if (!check_launch()) return 0;
  const size_t row_lds = (size_t)p->w * sizeof(uint32_t);
  static bool lds2_ok = [] {
    return hipFuncSetAttribute((const void*)k_vp8l_resid_serial<SG>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
  }();
  if (!lds2_ok || row_lds > 160 * 1024) return 0;
  hipLaunchKernelGGL((k_vp8l_resid_serial<SG>), dim3(p->n), dim3(64), row_lds, st, rgba, fstride,
                     rstride, *p, fidx, fmode, (const uint8_t*)modes, (const uint32_t*)pflag, argb);
  return check_launch();
}

extern "C" int vp8l_launch_transform(const uint8_t* rgba, size_t fstride, int rstride,
                                     const vp8l_params* p, const int* fidx, const int* efidx,
                                     const uint8_t* fmode, const uint32_t* ehist,
                                     const int32_t* tabs, int sg_mask, uint32_t* argb,
                                     uint8_t* modes, const uint8_t* pexact, int any_exact,
                                     uint32_t* pflag, uint32_t* mult, uint32_t* alpha_flag,
                                     void* stream) {
  if (p->tb < 2 || p->tb > 6 || p->w <= 0 || p->h <= 0 || p->n <= 0) return 0;
  if (!p->alpha && !fmode) return 0;
  if (!fmode) sg_mask = 1;
  const int ntt = ((p->w + (1 << p->tb) - 1) >> p->tb) * ((p->h + (1 << p->tb) - 1) >> p->tb);
  dim3 grid((ntt + L1_TILES - 1) / L1_TILES, 1, p->n);
  dim3 gridw((ntt + 4 * L1W_TPW - 1) / (4 * L1W_TPW), 1, p->n);
  hipStream_t st = (hipStream_t)stream;
  const int32_t* frac = tabs + 4097;
  const float* ftabs = reinterpret_cast<const float*>(tabs + VP8L_TAB_FSLOG);
  // L1a: the reference's predictor choice for the frames that need it
  // (pexact, or every frame at method 0), with the serial residuals
  CHK_LAUNCH(hipMemsetAsync(pflag, 0, (size_t)p->n * sizeof(uint32_t), st));
#define L1A(T, SG)                                                                                \
  if (!launch_predsel<T, SG>(rgba, fstride, rstride, p, fidx, fmode, pexact, ftabs, modes, pflag, \
                             argb, st))                                                           \
  return 0
  for (int sg = 0; sg < 2; ++sg) {
    if (!((sg_mask >> sg) & 1) || !(any_exact || p->low_effort)) continue;
    switch (p->tb) {
      case 2: if (sg) { L1A(4, true); } else { L1A(4, false); } break;
      case 3: if (sg) { L1A(8, true); } else { L1A(8, false); } break;
      case 4: if (sg) { L1A(16, true); } else { L1A(16, false); } break;
      case 5: if (sg) { L1A(32, true); } else { L1A(32, false); } break;
      default: if (sg) { L1A(64, true); } else { L1A(64, false); } break;
    }
  }
#undef L1A
#define L1(T, SG)                                                                             \
  hipLaunchKernelGGL((k_vp8l_transform<T, SG>), grid, dim3(256), 0, st, rgba, fstride, rstride, \
                     *p, fidx, efidx, fmode, ehist, frac, modes, (const uint32_t*)pflag, pexact, \
                     argb, mult, alpha_flag)
#define L1W(T, SG)                                                                               \
  hipLaunchKernelGGL((k_vp8l_transform_w<T, SG>), gridw, dim3(256), 0, st, rgba, fstride,         \
                     rstride, *p, fidx, efidx, fmode, ehist, frac, modes, (const uint32_t*)pflag, \
                     pexact, argb, mult, alpha_flag)
  for (int sg = 0; sg < 2; ++sg) {
    if (!((sg_mask >> sg) & 1)) continue;
    switch (p->tb) {
      case 2: if (sg) L1(4, true); else L1(4, false); break;
      case 3: if (sg) L1W(8, true); else L1W(8, false); break;
      case 4: if (sg) L1W(16, true); else L1W(16, false); break;
      case 5: if (sg) L1W(32, true); else L1W(32, false); break;
      default: if (sg) L1(64, true); else L1(64, false); break;
    }
  }
#undef L1
#undef L1W
  return check_launch();
}

extern "C" int vp8l_launch_near_lossless(const uint8_t* rgba, size_t fstride, int rstride,
                                         const int* fidx, const uint8_t* apply, int w, int h,
                                         int n, int bits, uint8_t* buf0, uint8_t* buf1,
                                         const uint8_t** out, void* stream) {
  if (w <= 0 || h <= 0 || n <= 0 || bits < 1 || bits > 5 || (rstride & 3) || (fstride & 3) ||
      ((uintptr_t)rgba & 3))
    return 0;   // the pass reads whole RGBA words
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((w + 255) / 256, h, n);
  uint8_t* bufs[2] = {buf0, buf1};
  hipLaunchKernelGGL(k_vp8l_nearlossless, grid, dim3(256), 0, st, rgba, fstride, rstride, fidx, w,
                     h, bits, apply, bufs[0]);
  int cur = 0;
  for (int i = bits - 1; i >= 1; --i, cur ^= 1)
    hipLaunchKernelGGL(k_vp8l_nearlossless, grid, dim3(256), 0, st, (const uint8_t*)bufs[cur],
                       (size_t)w * h * 4, w * 4, (const int*)nullptr, w, h, i, apply,
                       bufs[cur ^ 1]);
  *out = bufs[cur];
  return check_launch();
}

extern "C" int vp8l_launch_palette_apply(const uint8_t* rgba, size_t fstride, int rstride,
                                         const vp8l_params* p, const int* fidx,
                                         const uint32_t* sorted, const uint8_t* sidx,
                                         const int* npal, uint32_t* argb, uint32_t* alpha_flag,
                                         void* stream) {
  if (!p->palette || p->xbits < 0 || p->xbits > 3 || p->w <= 0 || p->h <= 0 || p->n <= 0 ||
      ((p->ow + (1 << p->xbits) - 1) >> p->xbits) != p->w)
    return 0;
  hipLaunchKernelGGL(k_vp8l_palapply, dim3((p->w + 255) / 256, p->h, p->n), dim3(256), 0,
                     (hipStream_t)stream, rgba, fstride, rstride, *p, fidx, sorted, sidx, npal,
                     argb, alpha_flag);
  return check_launch();
}

// ------------------------------------------------------------------ L3d
// Frames without a predictor (direct / subtract green): the shortest-path
// parse (model: dp_parse, oracle/vp8l_dp.c) over the first VP8L_DP_NC plane-
// code distances with the colour cache in the cost model, two rounds of
// symbol costs (k_vp8l_dpcost) -> backward DP per row (k_vp8l_dp) -> the
// forward walk into parse ops (k_vp8l_dpwalk). Reference idea:
// TraceBackwards, backward_references_cost_enc.c:569-795.

__device__ __forceinline__ bool dp_frame(const uint8_t* fmode, int f) {
  if (!fmode) return false;
  const int m = fmode[f];
  return m != VP8L_MODE_PALETTE && !(m & VP8L_MODE_SPATIAL);
}

// Symbol costs of a frame's parse with its colour cache (model: dp_costs):
// one workgroup per frame, histograms in LDS, 1/256 bit per symbol.
__global__ __launch_bounds__(1024) void k_vp8l_dpcost(const uint32_t* __restrict__ argb,
                                                      const uint32_t* __restrict__ ops, int npix,
                                                      const uint8_t* __restrict__ fmode,
                                                      const uint8_t* __restrict__ cbits,
                                                      const int32_t* __restrict__ frac,
                                                      int32_t* __restrict__ costs) {
  __shared__ uint32_t h[VP8L_DP_NCOST];
  __shared__ uint32_t tot[5], nz[5];
  const int f = blockIdx.x, tid = threadIdx.x;
  if (!dp_frame(fmode, f)) return;
  const uint32_t* E = argb + (size_t)f * npix;
  const uint32_t* O = ops + (size_t)f * npix;
  const int cb = cbits[f];
  const int oR = VP8L_DP_NG, oB = oR + 256, oA = oB + 256, oD = oA + 256;
  for (int i = tid; i < VP8L_DP_NCOST; i += 1024) h[i] = 0;
  if (tid < 5) { tot[tid] = 0; nz[tid] = 0; }
  __syncthreads();
  for (int q = tid; q < npix; q += 1024) {
    const uint32_t op = O[q], act = op & 3;
    if (act == 0) {
      const uint32_t a = E[q];
      atomicAdd(&h[(a >> 8) & 255], 1u);
      atomicAdd(&h[oR + ((a >> 16) & 255)], 1u);
      atomicAdd(&h[oB + (a & 255)], 1u);
      atomicAdd(&h[oA + (a >> 24)], 1u);
    } else if (act == 1) {
      atomicAdd(&h[280 + ((E[q] * HASH_MUL) >> (32 - cb))], 1u);
    } else if (act == 2) {
      int sym, nb; uint32_t ex;
      prefix_enc(((op >> 2) & 0xfff) + 1, sym, nb, ex);
      atomicAdd(&h[256 + sym], 1u);
      prefix_enc(op >> 14, sym, nb, ex);
      atomicAdd(&h[oD + sym], 1u);
    }
  }
  __syncthreads();
  auto alph = [&](int i) { return i < oR ? 0 : i < oB ? 1 : i < oA ? 2 : i < oD ? 3 : 4; };
  for (int i = tid; i < VP8L_DP_NCOST; i += 1024)
    if (h[i]) { atomicAdd(&tot[alph(i)], h[i]); atomicAdd(&nz[alph(i)], 1u); }
  __syncthreads();
  int32_t* out = costs + (size_t)f * VP8L_DP_NCOST;
  for (int i = tid; i < VP8L_DP_NCOST; i += 1024) {
    const int a = alph(i);
    int32_t c = 0;
    if (nz[a] > 1) c = (flog2_fx(frac, tot[a]) - (h[i] ? flog2_fx(frac, h[i]) : 0)) >> 4;
    out[i] = c;
  }
}

#define DP_XM 8                        // columns either side of a chunk in the tile
#define DP_MAXDY 8                     // rows above the block in the tile (+1 for a wrap)
#define DP_TR (64 + DP_MAXDY + 1)
#define DP_TW (64 + 2 * DP_XM)
#define DP_RING (VP8L_DP_MAXK + 1)
struct DpSmem {
  uint32_t tile[DP_TR][DP_TW];         // the block's rows (and DP_MAXDY + 1 above), chunk +- DP_XM
  int32_t ring[64][DP_RING + 1];       // per row: cost to the row end of the next 64 positions
  uint8_t runs[VP8L_DP_NC][64];        // per row: each candidate's run from the position on (<= 64)
  uint16_t ch[64][66];                 // the chunk's choices, row-major (k | candidate << 7)
  uint8_t mb[64][68];                  // the chunk's smallest cache sizes
  int32_t cost[VP8L_DP_NCOST];
  int32_t lcost[VP8L_DP_MAXK + 1];
  int32_t dcost[VP8L_DP_NC], ord[VP8L_DP_NC], cdy[VP8L_DP_NC], cdx[VP8L_DP_NC];
};

// Backward DP per row (model / oracle vp8l_dp_parse): one wave per 64 rows of
// a frame, one row per lane, the row walked right to left in 64-pixel chunks
// staged in LDS with the rows above the source candidates reach (a source
// outside the tile -- a wrap across a row end, or a far row -- is read from
// HBM). Per position: every candidate's run updated from the one to its
// right, then the literal / cache hit against copies of 2..min(run, 64) in
// increasing length, each length by the cheapest candidate covering it
// (candidates walked in (distance cost, index) order), strictly better only.
__global__ __launch_bounds__(64) void k_vp8l_dp(const uint32_t* __restrict__ argb,
                                                const uint8_t* __restrict__ minb, vp8l_params p,
                                                const uint8_t* __restrict__ fmode,
                                                const uint8_t* __restrict__ cbits,
                                                const int32_t* __restrict__ costs,
                                                const int4* __restrict__ cand, int ncand,
                                                uint16_t* __restrict__ choice) {
  __shared__ DpSmem S;
  const int f = blockIdx.y, ln = lane_id();
  if (!dp_frame(fmode, f)) return;   // whole wave
  const int W = p.w, H = p.h, r0 = blockIdx.x * 64, r = r0 + ln;
  const bool valid = r < H;
  const size_t npix = (size_t)W * H;
  const uint32_t* E = argb + (size_t)f * npix;
  const uint8_t* MB = minb + (size_t)f * npix;
  uint16_t* CH = choice + (size_t)f * npix;
  const int cb = cbits[f];
  const int oR = VP8L_DP_NG, oB = oR + 256, oA = oB + 256, oD = oA + 256;
  for (int i = ln; i < VP8L_DP_NCOST; i += 64) S.cost[i] = costs[(size_t)f * VP8L_DP_NCOST + i];
  __syncthreads();
  static_assert(VP8L_DP_MAXK <= 64, "one lane per copy length");
  if (ln < VP8L_DP_MAXK) {   // lengths 1..64 on lanes 0..63
    int sym, nb; uint32_t ex;
    prefix_enc((uint32_t)ln + 1u, sym, nb, ex);
    S.lcost[ln + 1] = S.cost[256 + sym] + 256 * nb;
  }
  int4 cv = make_int4(0, 0, 0, 0);
  if (ln < ncand) {
    cv = cand[ln];
    int sym, nb; uint32_t ex;
    prefix_enc((uint32_t)cv.w, sym, nb, ex);
    S.dcost[ln] = S.cost[oD + sym] + 256 * nb;
    S.cdy[ln] = cv.y;
    S.cdx[ln] = cv.z;
  }
  __syncthreads();
  if (ln < ncand) {   // rank by (distance cost, index)
    int rank = 0;
    for (int c = 0; c < ncand; ++c)
      rank += S.dcost[c] < S.dcost[ln] || (S.dcost[c] == S.dcost[ln] && c < ln);
    S.ord[rank] = ln;
  }
  for (int c = 0; c < ncand; ++c) S.runs[c][ln] = 0;
  S.ring[ln][W % DP_RING] = 0;
  __syncthreads();
  const int trow0 = r0 - DP_MAXDY - 1;   // the tile's first row
  for (int c0 = ((W - 1) >> 6) << 6; c0 >= 0; c0 -= 64) {
    const int tcol0 = c0 - DP_XM;
    __syncthreads();
    for (int i = ln; i < DP_TR * DP_TW; i += 64) {
      const int tr = i / DP_TW, tc = i - tr * DP_TW;
      const int rr = trow0 + tr, cc = tcol0 + tc;
      S.tile[tr][tc] = (rr >= 0 && rr < H && cc >= 0 && cc < W) ? E[(size_t)rr * W + cc] : 0u;
    }
    for (int rr = 0; rr < 64; ++rr)
      if (r0 + rr < H && c0 + ln < W) S.mb[rr][ln] = MB[(size_t)(r0 + rr) * W + c0 + ln];
    __syncthreads();
    const int jt = min(63, W - 1 - c0);
    for (int jj = jt; jj >= 0; --jj) {
      const int j = c0 + jj;
      if (valid) {
        const uint32_t e = S.tile[ln + DP_MAXDY + 1][jj + DP_XM];
        for (int c = 0; c < ncand; ++c) {
          int sc = j - S.cdx[c], sr = r - S.cdy[c];
          if (sc < 0) { sc += W; sr -= 1; }
          else if (sc >= W) { sc -= W; sr += 1; }
          bool eq = false;
          if (sr >= 0) {
            const int tr = sr - trow0, tc = sc - tcol0;
            eq = (tr >= 0 && tc >= 0 && tc < DP_TW) ? S.tile[tr][tc] == e
                                                    : E[(size_t)sr * W + sc] == e;
          }
          const int run = eq ? min((int)S.runs[c][ln] + 1, VP8L_DP_MAXK) : 0;
          S.runs[c][ln] = (uint8_t)run;
        }
        const int m = S.mb[ln][jj];
        int lit;
        if (cb > 0 && m <= cb)
          lit = S.cost[280 + (int)((e * HASH_MUL) >> (32 - cb))] * 68 / 100;
        else
          lit = (S.cost[(e >> 8) & 255] + S.cost[oR + ((e >> 16) & 255)] + S.cost[oB + (e & 255)] +
                 S.cost[oA + (e >> 24)]) * 82 / 100;
        int best = S.ring[ln][(j + 1) % DP_RING] + lit, bk = 1, bc = 0;
        const int kmax = min(VP8L_DP_MAXK, W - j);
        int maxl = 1;
        for (int i = 0; i < ncand; ++i) {
          const int c = S.ord[i];
          const int L = min((int)S.runs[c][ln], kmax);
          if (L <= maxl) continue;
          const int dc = S.dcost[c];
          for (int k = maxl + 1; k <= L; ++k) {
            const int v = S.ring[ln][(j + k) % DP_RING] + dc + S.lcost[k];
            if (v < best) { best = v; bk = k; bc = c; }
          }
          maxl = L;
        }
        S.ring[ln][j % DP_RING] = best;
        S.ch[ln][jj] = (uint16_t)(bk | (bc << 7));
      }
    }
    __syncthreads();
    for (int rr = 0; rr < 64; ++rr)
      if (r0 + rr < H && c0 + ln < W) CH[(size_t)(r0 + rr) * W + c0 + ln] = S.ch[rr][ln];
  }
}

// The forward walk of the DP choices into parse ops (the structure of
// k_vp8l_parse: a wave owns 64 rows, 64-pixel chunks staged through LDS,
// positions a copy from an earlier chunk covers marked on load).
__global__ __launch_bounds__(64) void k_vp8l_dpwalk(vp8l_params p, const uint8_t* __restrict__ fmode,
                                                    const uint16_t* __restrict__ choice,
                                                    const uint8_t* __restrict__ minb,
                                                    const uint8_t* __restrict__ cbits,
                                                    const int4* __restrict__ cand,
                                                    uint32_t* __restrict__ ops) {
  __shared__ uint32_t tile[64][65];
  __shared__ int xs[64];
  __shared__ int dcode[VP8L_DP_NC];
  const int f = blockIdx.y, ln = lane_id();
  if (!dp_frame(fmode, f)) return;
  const int W = p.w, H = p.h, y0 = blockIdx.x * 64;
  const int nrows = min(64, H - y0);
  const size_t npix = (size_t)W * H;
  uint32_t* O = ops + (size_t)f * npix + (size_t)y0 * W;
  const uint16_t* C = choice + (size_t)f * npix + (size_t)y0 * W;
  const uint8_t* MB = minb + (size_t)f * npix + (size_t)y0 * W;
  const int cb = cbits[f];
  if (ln < VP8L_DP_NC) dcode[ln] = cand[ln].w;
  int x = 0;
  xs[ln] = 0;
  for (int cx = 0; cx < W; cx += 64) {
    const int cw = min(64, W - cx);
    __syncthreads();
    for (int r = 0; r < nrows; ++r) {
      if (ln < cw) {
        const size_t q = (size_t)r * W + cx + ln;
        const uint32_t hit = cb > 0 && MB[q] <= cb;
        tile[r][ln] = cx + ln < xs[r] ? 0xffffffffu : ((uint32_t)C[q] | (hit << 16));
      }
    }
    __syncthreads();
    if (ln < nrows) {
      while (x < cx + cw) {
        const int i = x - cx;
        const uint32_t w = tile[ln][i];
        const int k = (int)(w & 127);
        if (k >= 2) {
          tile[ln][i] = 2u | ((uint32_t)(k - 1) << 2) | ((uint32_t)dcode[(w >> 7) & 31] << 14);
          const int e = min(x + k, cx + cw);
          for (int t = i + 1; t < e - cx; ++t) tile[ln][t] = 3u;
          x += k;
        } else {
          tile[ln][i] = (w >> 16) & 1u;
          ++x;
        }
      }
      xs[ln] = x;
    }
    __syncthreads();
    for (int r = 0; r < nrows; ++r) {
      if (ln < cw) {
        uint32_t v = tile[r][ln];
        if (v == 0xffffffffu) v = 3u;
        O[(size_t)r * W + cx + ln] = v;
      }
    }
  }
}

extern "C" int vp8l_launch_analyze(const uint32_t* argb, const vp8l_params* p,
                                   const int32_t* tabs, uint8_t* minb, uint32_t* cseg,
                                   uint16_t* prov,
                                   uint32_t* chist, uint8_t* cbits, uint32_t* ops, int64_t* feat,
                                   uint32_t* tl, uint32_t* tn, uint32_t* hc, uint8_t* assign,
                                   const vp8l_lz* lz, const vp8l_dp* dp, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int npix = p->w * p->h;
  const int32_t* flog2 = tabs + 4097;
  const int tx_n = (p->w + (1 << p->hb) - 1) >> p->hb, ty_n = (p->h + (1 << p->hb) - 1) >> p->hb;
  if (tx_n * ty_n > VP8L_MAX_HUFF_IMAGE || p->k < 1 || p->k > VP8L_KMAX) return 0;
  if (p->cache_bits < 0 || p->cache_bits > VP8L_MAX_CACHE_BITS) return 0;
  if (lz) {   // colour-indexed: cost-model parse (model: palette_parse), no cache
    if (hipMemsetAsync(minb, VP8L_NEVER_HIT, (size_t)p->n * npix, st) != hipSuccess ||
        hipMemsetAsync(cbits, 0, (size_t)p->n, st) != hipSuccess ||
        hipMemsetAsync(lz->htab, 0xff, (size_t)p->n * LZ_HASH_SIZE * sizeof(int32_t), st) !=
            hipSuccess)
      return 0;
    const int nseg = (npix + LZ_SEG - 1) / LZ_SEG;
    // first parse A: the greedy row parse over the 4 local candidates
    hipLaunchKernelGGL(k_vp8l_match, dim3(p->h, p->n), dim3(64), 0, st, argb, minb,
                       (const uint2*)nullptr, 1, *p, ops);
    hipLaunchKernelGGL(k_vp8l_parse, dim3((p->h + 63) / 64, p->n), dim3(64), 0, st, *p, ops, prov,
                       (const uint8_t*)cbits);
    hipLaunchKernelGGL(k_lz_costs, dim3(p->n), dim3(1024), 0, st, argb, (const uint32_t*)ops,
                       npix, flog2, lz->costs_row, lz->est);
    hipLaunchKernelGGL(k_lz_runs, dim3((npix + LZ_RUN_PIECE - 1) / LZ_RUN_PIECE, p->n), dim3(64), 0,
                       st, argb, npix, lz->runs);
    hipLaunchKernelGGL(k_lz_chain, dim3(p->n), dim3(64), 0, st, argb, npix,
                       (const uint16_t*)lz->runs, lz->htab, lz->chain);
    hipLaunchKernelGGL(k_lz_search, dim3((npix + 255) / 256, p->n), dim3(256), 0, st, argb, p->w,
                       npix, (const int32_t*)lz->chain, lz->hoff, lz->hlen);
    hipLaunchKernelGGL(k_lz_local, dim3(nseg, p->n), dim3(64), 0, st, argb, *p, lz->loff,
                       lz->llen);
    // first parse B: greedy over the chain and local matches; the cheaper
    // of A and B under their own costs seeds the first cost-model parse
    hipLaunchKernelGGL(k_lz_greedy, dim3(nseg, p->n), dim3(64), 0, st, npix,
                       (const uint32_t*)lz->hoff, (const uint16_t*)lz->hlen,
                       (const uint32_t*)lz->loff, (const uint16_t*)lz->llen, lz->dcodes, lz->nd,
                       ops);
    hipLaunchKernelGGL(k_lz_costs, dim3(p->n), dim3(1024), 0, st, argb, (const uint32_t*)ops,
                       npix, flog2, lz->costs, lz->est + p->n);
    hipLaunchKernelGGL(k_lz_pick, dim3(p->n), dim3(256), 0, st, (const unsigned long long*)lz->est,
                       (const unsigned long long*)lz->est + p->n, (const int32_t*)lz->costs_row,
                       lz->costs);
    for (int round = 0; round < 2; ++round) {
      if (round)
        hipLaunchKernelGGL(k_lz_costs, dim3(p->n), dim3(1024), 0, st, argb, (const uint32_t*)ops,
                           npix, flog2, lz->costs, (unsigned long long*)nullptr);
      hipLaunchKernelGGL(k_lz_dp, dim3(nseg, p->n), dim3(64), 0, st, argb, p->w, npix,
                         (const int32_t*)lz->costs, (const uint32_t*)lz->hoff,
                         (const uint16_t*)lz->hlen, (const uint32_t*)lz->loff,
                         (const uint16_t*)lz->llen, lz->dcodes, lz->nd, ops);
    }
  } else {
    // L2 segments: >= 256 chunks each, so few pixels are left partial
    const int S = p->cache_bits ? max(1, min(VP8L_CACHE_SEGS, ((npix + 63) >> 6) / 256)) : 1;
    if (p->cache_bits) {
      if (!cseg) return 0;
      hipLaunchKernelGGL(k_vp8l_cache, dim3(S, p->n), dim3(64), 0, st, argb, npix, S, minb,
                         (uint2*)cseg);
      if (S > 1)
        hipLaunchKernelGGL(k_vp8l_cache_start, dim3(p->n), dim3(1024), 0, st, S, (uint2*)cseg);
    } else if (hipMemsetAsync(minb, VP8L_NEVER_HIT, (size_t)p->n * npix, st) != hipSuccess) {
      return 0;
    }
    hipLaunchKernelGGL(k_vp8l_match, dim3(p->h, p->n), dim3(64), 0, st, argb, minb,
                       (const uint2*)cseg, S, *p, ops);
    if (p->cache_bits) {
      hipLaunchKernelGGL(k_vp8l_parse, dim3((p->h + 63) / 64, p->n), dim3(64), 0, st, *p, ops,
                         prov, (const uint8_t*)nullptr);   // provisional
      hipLaunchKernelGGL(k_vp8l_cachehist, dim3(p->n), dim3(1024), VP8L_CHIST * sizeof(uint32_t),
                         st, argb, (const uint32_t*)ops, prov, npix, chist);
      hipLaunchKernelGGL(k_vp8l_cachechoose, dim3(p->n), dim3(256), 0, st, chist, flog2,
                         p->cache_bits, cbits);
    } else if (hipMemsetAsync(cbits, 0, (size_t)p->n, st) != hipSuccess) {
      return 0;
    }
    hipLaunchKernelGGL(k_vp8l_parse, dim3((p->h + 63) / 64, p->n), dim3(64), 0, st, *p, ops, prov,
                       (const uint8_t*)cbits);
    if (dp && dp->fmode && dp->ncand > 0 && prov) {   // frames without a predictor
      for (int round = 0; round < 2; ++round) {
        hipLaunchKernelGGL(k_vp8l_dpcost, dim3(p->n), dim3(1024), 0, st, argb, (const uint32_t*)ops,
                           npix, dp->fmode, (const uint8_t*)cbits, flog2, dp->costs);
        hipLaunchKernelGGL(k_vp8l_dp, dim3((p->h + 63) / 64, p->n), dim3(64), 0, st, argb,
                           (const uint8_t*)minb, *p, dp->fmode, (const uint8_t*)cbits,
                           (const int32_t*)dp->costs, (const int4*)dp->cand, dp->ncand, prov);
        hipLaunchKernelGGL(k_vp8l_dpwalk, dim3((p->h + 63) / 64, p->n), dim3(64), 0, st, *p,
                           dp->fmode, (const uint16_t*)prov, (const uint8_t*)minb,
                           (const uint8_t*)cbits, (const int4*)dp->cand, ops);
      }
    }
  }
  hipLaunchKernelGGL(k_vp8l_tilefeat, dim3(tx_n * ty_n, p->n), dim3(256), 0, st, argb, ops, *p,
                     (const uint8_t*)cbits, flog2, feat, tl, tn);
  static int attr = 0;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_vp8l_cluster,
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(ClusterSmem)) != hipSuccess)
      return 0;
    attr = 1;
  }
  hipLaunchKernelGGL(k_vp8l_cluster, dim3(p->n), dim3(1024), sizeof(ClusterSmem), st, *p,
                     (const uint8_t*)cbits, flog2, feat, tl, tn, hc, assign);
  return check_launch();
}

extern "C" int vp8l_launch_write(const uint32_t* argb, const uint32_t* ops, const vp8l_params* p,
                                 const uint8_t* cbits, const uint32_t* ctab, const uint8_t* gtile,
                                 const uint64_t* start_bit, uint32_t* bsum, uint64_t* boff,
                                 uint64_t* end_bit, uint8_t* out, size_t out_cap, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t npix = (size_t)p->w * p->h;
  const int nblk = (int)((npix + VP8L_BLOCK - 1) / VP8L_BLOCK);
  if ((out_cap & 3) != 0) return 0;
  hipLaunchKernelGGL(k_vp8l_bitcount, dim3(nblk, p->n), dim3(256), 0, st, argb, ops, *p, cbits,
                     ctab, gtile, bsum);
  hipLaunchKernelGGL(k_vp8l_scan, dim3(p->n), dim3(1024), 0, st, bsum, nblk, start_bit, boff,
                     end_bit);
  hipLaunchKernelGGL(k_vp8l_write, dim3(nblk, p->n), dim3(256), 0, st, argb, ops, *p, cbits, ctab,
                     gtile, bsum, boff, out, out_cap);
  return check_launch();
}

extern "C" int vp8l_launch_put_headers(const uint32_t* hdr, const uint64_t* hoff,
                                       const uint32_t* hwords, int n, uint8_t* out,
                                       size_t out_cap, void* stream) {
  hipLaunchKernelGGL(k_vp8l_put_headers, dim3(8, n), dim3(256), 0, (hipStream_t)stream, hdr, hoff,
                     hwords, out, out_cap);
  return check_launch();
}

extern "C" int vp8l_launch_pack(const uint8_t* out, size_t out_cap, const uint64_t* poff,
                                const uint64_t* end_bit, int n, uint8_t* packed, void* stream) {
  hipLaunchKernelGGL(k_vp8l_pack, dim3(64, n), dim3(256), 0, (hipStream_t)stream, out, out_cap,
                     poff, end_bit, packed);
  return check_launch();
}

#ifdef VP8L_PS_PROF
// diagnostic build only: the phase cycle counters (L1a phases 0-5, L1 8-9)
extern "C" __attribute__((visibility("default"))) int vp8l_prof_phase_cycles(
    unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vp8l_prof), sizeof(g_vp8l_prof)) != hipSuccess) return 0;
  if (reset) {
    static const unsigned long long zero[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_vp8l_prof), zero, sizeof(zero)) != hipSuccess) return 0;
  }
  return 1;
}
#endif
