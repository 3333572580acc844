// Lossless (VP8L) encoder kernels for gfx950. The decisions are stated in
// oracle/vp8l_model.py (same names); the bitstream format is the reference
// decoder's (src/dec/vp8l_dec.c, src/dsp/lossless.c). All integer work:
// HBM/LDS bound, no MFMA.
//
//   L1 k_vp8l_transform  one workgroup per transform tile: subtract green,
//                        best of 14 predictors by a bit-length cost,
//                        cross-colour multipliers (least squares + 6
//                        candidates), residual ARGB to HBM
//   L2 k_vp8l_cache      one wave per frame, 64 pixels per step: colour-cache
//                        hit bits (same-key lanes found with CACHE_BITS ballots)
//   L3 k_vp8l_match      one wave per row: best candidate run per pixel (ballots)
//      k_vp8l_parse      one thread per row: greedy copy / cache / literal
//   L4 k_vp8l_tilefeat   one workgroup per histogram tile: own entropy/pixel
//   L5 k_vp8l_cluster    one workgroup per frame: k-means of histogram tiles
//                        into <= KMAX code groups (histograms + costs in LDS)
//   L6 k_vp8l_bitcount / k_vp8l_scan   bits per 1024-pixel block, offsets
//   L7 k_vp8l_write      one workgroup per block: fields into LDS words,
//                        interior words stored, the two edge words OR-ed
#include <hip/hip_runtime.h>
#include <stdint.h>

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
__device__ uint32_t predict(int m, uint32_t L, uint32_t T, uint32_t TL, uint32_t TR) {
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

__device__ __forceinline__ int s8(int v) { return (int)(int8_t)(uint8_t)v; }
__device__ __forceinline__ int ctd(int t, int c) { return (t * s8(c)) >> 5; }

// round(32 * sxy / sxx) half away from zero, clamped to int8 (model: ls_multiplier)
__device__ int ls_multiplier(long long sxy, long long sxx) {
  if (sxx == 0) return 0;
  const long long num = 32 * sxy;
  const long long an = num < 0 ? -num : num;
  long long q = (2 * an + sxx) / (2 * sxx);
  q = num >= 0 ? q : -q;
  return (int)(q < -128 ? -128 : q > 127 ? 127 : q);
}

__device__ __forceinline__ int clamp8(int v) { return v < -128 ? -128 : v > 127 ? 127 : v; }

// block-wide sums through LDS atomics (T threads, wave reductions first)
template <typename V>
__device__ __forceinline__ V wave_sum(V v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

}  // namespace

// ------------------------------------------------------------------ L1

// bits of |v| for the signed 8-bit view of each residual byte, summed over
// the bytes of a pixel (model: bitlen) -- the search cost, pure VALU
__device__ __forceinline__ int bitlen8(int b) { return 32 - __clz(abs(s8(b))); }
__device__ __forceinline__ int pixel_bits(uint32_t r) {
  return bitlen8(ch(r, 0)) + bitlen8(ch(r, 8)) + bitlen8(ch(r, 16)) + bitlen8(ch(r, 24));
}

template <int T>
struct TransformSmem {
  uint32_t src[(T + 1) * (T + 2)];   // rows y0-1.., cols x0-1..x0+tw
  uint32_t first[T];                 // P(0, y) for the right-edge TR wrap
  uint32_t res[T * T];
  int score[16];
  long long sums[4];
  int best;
};

template <int T>
__global__ __launch_bounds__(256) void k_vp8l_transform(const uint8_t* __restrict__ rgba,
                                                        size_t fstride, int rstride, vp8l_params p,
                                                        uint32_t* __restrict__ argb_out,
                                                        uint8_t* __restrict__ modes,
                                                        uint32_t* __restrict__ mult,
                                                        uint32_t* __restrict__ alpha_flag) {
  __shared__ TransformSmem<T> S;
  const int tid = threadIdx.x, f = blockIdx.z;
  const int W = p.w, H = p.h;
  const int x0 = blockIdx.x * T, y0 = blockIdx.y * T;
  const int tw = min(T, W - x0), th = min(T, H - y0);
  const int sw = tw + 2;   // LDS source row width (cols x0-1 .. x0+tw)
  const uint8_t* img = rgba + (size_t)f * fstride;
  const int tiles_x = (W + T - 1) / T;
  const int tile = blockIdx.y * tiles_x + blockIdx.x;

  // load sub-green pixels (A, R-G, G, B-G) with a 1-pixel border
  bool tile_alpha = false;
  for (int i = tid; i < (th + 1) * sw; i += 256) {
    const int ly = i / sw, lx = i - ly * sw;
    const int y = y0 - 1 + ly, x = x0 - 1 + lx;
    uint32_t v = 0;
    if (y >= 0 && x >= 0 && x < W) {
      if (p.alpha) {   // ALPH: the alpha plane as green, no subtract green
        v = (uint32_t)img[(size_t)y * rstride + x] << 8;
      } else {
        const uint8_t* q = img + (size_t)y * rstride + 4 * x;
        const uint32_t r = q[0], g = q[1], b = q[2], a = q[3];
        v = (a << 24) | (((r - g) & 255) << 16) | (g << 8) | ((b - g) & 255);
        if (a != 255 && ly > 0 && lx > 0 && lx <= tw) tile_alpha = true;
      }
    }
    S.src[i] = v;
  }
  if (x0 + tw == W) {
    for (int i = tid; i < th; i += 256) {
      const uint8_t* q = img + (size_t)(y0 + i) * rstride;
      if (p.alpha) {
        S.first[i] = (uint32_t)q[0] << 8;
      } else {
        const uint32_t r = q[0], g = q[1], b = q[2], a = q[3];
        S.first[i] = (a << 24) | (((r - g) & 255) << 16) | (g << 8) | ((b - g) & 255);
      }
    }
  }
  if (__any(tile_alpha) && lane_id() == 0) atomicOr(&alpha_flag[f], 1u);
  if (tid < 16) S.score[tid] = 0;
  __syncthreads();

  auto at = [&](int lx, int ly) -> uint32_t { return S.src[(ly + 1) * sw + lx + 1]; };
  auto tr = [&](int lx, int ly) -> uint32_t {   // (y-1)*W + x + 1, linear
    return (x0 + lx + 1 < W) ? at(lx + 1, ly - 1) : S.first[ly];
  };
  const int np = tw * th;
  // fixed predictors: (0,0) black, row 0 left, column 0 top (lossless.c:219-239)
  auto fixed_mode = [&](int x, int y) -> int { return y == 0 ? (x == 0 ? 0 : 1) : (x == 0 ? 2 : -1); };

  // cost of each of the 14 predictors over the tile (smallest wins, first on ties)
  {
    int sc[14];
#pragma unroll
    for (int m = 0; m < 14; ++m) sc[m] = 0;
    for (int i = tid; i < np; i += 256) {
      const int ly = i / tw, lx = i - ly * tw;
      const uint32_t P = at(lx, ly), L = at(lx - 1, ly), T_ = at(lx, ly - 1), TL = at(lx - 1, ly - 1);
      const uint32_t TR = tr(lx, ly);
      const int fm = fixed_mode(x0 + lx, y0 + ly);
#pragma unroll
      for (int m = 0; m < 14; ++m)
        sc[m] += pixel_bits(sub_pixels(P, predict(fm >= 0 ? fm : m, L, T_, TL, TR)));
    }
#pragma unroll
    for (int m = 0; m < 14; ++m) {
      const int v = wave_sum(sc[m]);
      if (lane_id() == 0) atomicAdd(&S.score[m], v);
    }
  }
  __syncthreads();
  if (tid == 0) {
    int best = 0;
    for (int m = 1; m < 14; ++m)
      if (S.score[m] < S.score[best]) best = m;
    S.best = best;
    S.sums[0] = S.sums[1] = S.sums[2] = S.sums[3] = 0;
  }
  __syncthreads();
  const int best = S.best;
  long long sgg = 0, sgr = 0, sgb = 0;
  for (int i = tid; i < np; i += 256) {
    const int ly = i / tw, lx = i - ly * tw;
    const int fm = fixed_mode(x0 + lx, y0 + ly);
    const uint32_t r = sub_pixels(at(lx, ly), predict(fm >= 0 ? fm : best, at(lx - 1, ly),
                                                      at(lx, ly - 1), at(lx - 1, ly - 1), tr(lx, ly)));
    S.res[i] = r;
    const int g = s8(ch(r, 8)), rr = s8(ch(r, 16)), bb = s8(ch(r, 0));
    sgg += g * g; sgr += g * rr; sgb += g * bb;
  }
  sgg = wave_sum(sgg); sgr = wave_sum(sgr); sgb = wave_sum(sgb);
  if (lane_id() == 0) {
    atomicAdd((unsigned long long*)&S.sums[0], (unsigned long long)sgg);
    atomicAdd((unsigned long long*)&S.sums[1], (unsigned long long)sgr);
    atomicAdd((unsigned long long*)&S.sums[2], (unsigned long long)sgb);
  }
  __syncthreads();
  // cross colour (model: choose_cross_color): three rounds, each the best of
  // 6 candidates {0, ls-2 .. ls+2} by the bitlen cost
  int g2r = 0, g2b = 0, r2b = 0;
  for (int round = 0; round < 3; ++round) {
    long long sxy, sxx;
    if (round == 0) { sxy = S.sums[1]; sxx = S.sums[0]; }
    else if (round == 1) { sxy = S.sums[2]; sxx = S.sums[0]; }
    else { sxy = S.sums[3]; sxx = S.sums[2]; }   // r2b sums, computed in round 1
    const int ls = ls_multiplier(sxy, sxx);
    int cand[6];
    cand[0] = 0;
#pragma unroll
    for (int c = 1; c < 6; ++c) cand[c] = clamp8(ls + c - 3);
    int cs[6] = {0, 0, 0, 0, 0, 0};
    for (int i = tid; i < np; i += 256) {
      const uint32_t r = S.res[i];
      const int g = ch(r, 8), rr = ch(r, 16), bb = ch(r, 0);
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        int v;
        if (round == 0) v = rr - ctd(cand[c], g);
        else if (round == 1) v = bb - ctd(cand[c], g);
        else v = (bb - ctd(g2b, g)) - ctd(cand[c], rr);
        cs[c] += bitlen8(v & 255);
      }
    }
    __syncthreads();   // everyone has read S.score / S.sums of the previous step
    if (tid < 6) S.score[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 6; ++c) {
      const int v = wave_sum(cs[c]);
      if (lane_id() == 0) atomicAdd(&S.score[c], v);
    }
    __syncthreads();
    int bc = 0;
    for (int c = 1; c < 6; ++c)
      if (S.score[c] < S.score[bc]) bc = c;
    const int chosen = cand[bc];
    if (round == 0) g2r = chosen;
    else if (round == 1) {
      g2b = chosen;
      // sums for r2b: srr = sum r^2, srb = sum r * s8(b - ctd(g2b, g))
      long long srr = 0, srb = 0;
      for (int i = tid; i < np; i += 256) {
        const uint32_t r = S.res[i];
        const int rr = s8(ch(r, 16));
        const int bq = s8((ch(r, 0) - ctd(g2b, ch(r, 8))) & 255);
        srr += rr * rr; srb += rr * bq;
      }
      srr = wave_sum(srr); srb = wave_sum(srb);
      __syncthreads();
      if (tid == 0) { S.sums[2] = 0; S.sums[3] = 0; }
      __syncthreads();
      if (lane_id() == 0) {
        atomicAdd((unsigned long long*)&S.sums[2], (unsigned long long)srr);
        atomicAdd((unsigned long long*)&S.sums[3], (unsigned long long)srb);
      }
    } else {
      r2b = chosen;
    }
    __syncthreads();
  }
  // final residuals
  uint32_t* out = argb_out + (size_t)f * W * H;
  for (int i = tid; i < np; i += 256) {
    const int ly = i / tw, lx = i - ly * tw;
    const uint32_t r = S.res[i];
    const int g = ch(r, 8), rr = ch(r, 16), bb = ch(r, 0);
    const int nr = (rr - ctd(g2r, g)) & 255;
    const int nb = (bb - ctd(g2b, g) - ctd(r2b, rr)) & 255;
    out[(size_t)(y0 + ly) * W + x0 + lx] = (r & 0xff00ff00u) | ((uint32_t)nr << 16) | (uint32_t)nb;
  }
  if (tid == 0) {
    const int ntt = tiles_x * ((H + T - 1) / T);
    modes[(size_t)f * ntt + tile] = (uint8_t)best;
    mult[(size_t)f * ntt + tile] =
        (uint32_t)(g2r & 255) | ((uint32_t)(g2b & 255) << 8) | ((uint32_t)(r2b & 255) << 16);
  }
}

// ------------------------------------------------------------------ L2

// One wave per frame walks the pixels in stream order, 64 at a time, keeping
// the decoder's colour cache in LDS (zero-initialised like
// VP8LColorCacheInit). Lanes with the same key find each other with one
// ballot per key bit; a lane's cache content is the value of its nearest
// lower same-key lane, else the table entry; the highest lane of each key
// group updates the table.
#define CACHE_BATCH 16
__global__ __launch_bounds__(64) void k_vp8l_cache(const uint32_t* __restrict__ argb, int npix,
                                                   uint64_t* __restrict__ hits) {
  __shared__ uint32_t tab[1 << VP8L_CACHE_BITS];
  const int f = blockIdx.x, ln = lane_id();
  const uint32_t* E = argb + (size_t)f * npix;
  uint64_t* out = hits + (size_t)f * ((npix + 63) >> 6);
  for (int i = ln; i < (1 << VP8L_CACHE_BITS); i += 64) tab[i] = 0;
  __syncthreads();
  const int nchunk = (npix + 63) >> 6;
  uint32_t cur[CACHE_BATCH], nxt[CACHE_BATCH];
#pragma unroll
  for (int k = 0; k < CACHE_BATCH; ++k) {
    const int q = (k << 6) + ln;
    cur[k] = q < npix ? E[q] : 0;
  }
  for (int c0 = 0; c0 < nchunk; c0 += CACHE_BATCH) {
#pragma unroll
    for (int k = 0; k < CACHE_BATCH; ++k) {
      const int q = ((c0 + CACHE_BATCH + k) << 6) + ln;
      nxt[k] = q < npix ? E[q] : 0;
    }
#pragma unroll
    for (int k = 0; k < CACHE_BATCH; ++k) {
      const int c = c0 + k;
      if (c >= nchunk) break;
      const int q = (c << 6) + ln;
      const bool valid = q < npix;
      const uint32_t v = cur[k];
      const uint32_t key = (v * HASH_MUL) >> (32 - VP8L_CACHE_BITS);
      uint64_t m = __ballot(valid);
#pragma unroll
      for (int b = 0; b < VP8L_CACHE_BITS; ++b) {
        const bool bit = (key >> b) & 1;
        const uint64_t bv = __ballot(valid && bit);
        m &= bit ? bv : ~bv;
      }
      const uint64_t lower = m & ((1ull << ln) - 1ull);
      const int j = lower ? 63 - __clzll((long long)lower) : ln;
      const uint32_t pv = __shfl(v, j);
      const uint32_t held = lower ? pv : tab[key];
      const uint64_t hm = __ballot(valid && held == v);
      if (ln == 0) out[c] = hm;
      if (valid && (m >> ln) == 1ull) tab[key] = v;   // LDS ops of a wave stay in order
    }
#pragma unroll
    for (int k = 0; k < CACHE_BATCH; ++k) cur[k] = nxt[k];
  }
}

// ------------------------------------------------------------------ L3

// One wave per row, chunks of 64 pixels right to left: for each candidate
// distance the run of equal pixels starting at every x (ballot of the 64
// comparisons; count trailing ones; a run reaching the chunk end continues
// with the run at the next chunk's start), the longest (first on ties,
// capped at MAX_LENGTH) and the cache-hit bit, packed per pixel as
// len | cand << 13 | hit << 15 for the parse.
__global__ __launch_bounds__(64) void k_vp8l_match(const uint32_t* __restrict__ argb,
                                                   const uint64_t* __restrict__ hits, vp8l_params p,
                                                   uint32_t* __restrict__ bm) {
  const int f = blockIdx.y, y = blockIdx.x, ln = lane_id();
  const int W = p.w;
  const size_t npix = (size_t)W * p.h;
  const uint32_t* E = argb + f * npix;
  const uint64_t* hb = hits + (size_t)f * ((npix + 63) >> 6);
  uint32_t* O = bm + f * npix;
  const size_t row = (size_t)y * W;
  int carry[VP8L_NUM_CAND] = {0, 0, 0, 0};
  for (int c = (W - 1) >> 6; c >= 0; --c) {
    const int x = (c << 6) + ln;
    const bool valid = x < W;
    const size_t q = row + (size_t)x;
    const uint32_t e = valid ? E[q] : 0u;
    int bn = 0, bk = 0;
#pragma unroll
    for (int k = 0; k < VP8L_NUM_CAND; ++k) {
      const int d = p.dist[k];
      const bool ok = valid && d > 0 && (size_t)d <= q && E[q - d] == e;
      const uint64_t mask = __ballot(ok);
      int run = (int)__builtin_ctzll(~(mask >> ln));
      if (run == 64 - ln) run += carry[k];
      carry[k] = __shfl(run, 0);
      const int n = min(run, VP8L_MAX_LENGTH);
      if (n > bn) { bn = n; bk = k; }
    }
    if (valid) {
      const uint32_t hit = (uint32_t)((hb[q >> 6] >> (q & 63)) & 1);
      O[q] = (uint32_t)bn | ((uint32_t)bk << 13) | (hit << 15);
    }
  }
}

// One thread per row: greedy copy / cache / literal over the packed match
// words (model: parse), rewriting them in place as parse ops.
__global__ __launch_bounds__(64) void k_vp8l_parse(vp8l_params p, uint32_t* __restrict__ ops) {
  const int f = blockIdx.y, y = blockIdx.x * 64 + threadIdx.x;
  const int W = p.w, H = p.h;
  if (y >= H) return;
  const size_t npix = (size_t)W * H;
  uint32_t* O = ops + f * npix + (size_t)y * W;
  int x = 0;
  while (x < W) {
    const uint32_t m = O[x];
    const int bn = (int)(m & 0x1fff), bk = (int)((m >> 13) & 3);
    const bool hit = (m >> 15) & 1;
    if (bn >= VP8L_MIN_COPY || (bn == 2 && !hit)) {
      O[x] = 2u | ((uint32_t)bn << 2) | ((uint32_t)p.dcode[bk] << 15);
      for (int i = 1; i < bn; ++i) O[x + i] = 3u;
      x += bn;
    } else {
      O[x] = hit ? 1u : 0u;
      ++x;
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

__device__ __forceinline__ void pix_symbols(uint32_t op, uint32_t a, PixSym& o) {
  const uint32_t act = op & 3;
  o.s[0] = o.s[1] = o.s[2] = o.s[3] = -1;
  o.xv[0] = o.xv[1] = 0; o.xb[0] = o.xb[1] = 0;
  if (act == 0) {
    o.s[0] = (int)((a >> 8) & 255);
    o.s[1] = VP8L_GS + (int)((a >> 16) & 255);
    o.s[2] = VP8L_GS + 256 + (int)(a & 255);
    o.s[3] = VP8L_GS + 512 + (int)(a >> 24);
  } else if (act == 1) {
    o.s[0] = 280 + (int)((a * HASH_MUL) >> (32 - VP8L_CACHE_BITS));
  } else if (act == 2) {
    int sym, nb; uint32_t ex;
    prefix_enc((op >> 2) & 0x1fff, sym, nb, ex);
    o.s[0] = 256 + sym; o.xv[0] = ex; o.xb[0] = nb;
    prefix_enc(op >> 15, sym, nb, ex);
    o.s[1] = VP8L_GS + 768 + sym; o.xv[1] = ex; o.xb[1] = nb;
  }
}

// alphabet index of a symbol in the concatenated space
__device__ __forceinline__ int alph_of(int s) {
  return s < VP8L_GS ? 0 : s < VP8L_GS + 256 ? 1 : s < VP8L_GS + 512 ? 2 : s < VP8L_GS + 768 ? 3 : 4;
}
__device__ __forceinline__ int alph_size(int a) { return a == 0 ? VP8L_GS : a == 4 ? 40 : 256; }

__device__ __forceinline__ int flog2_fx(const int32_t* frac, uint32_t v) {
  // log2(v) in 1/4096 bit, v >= 1 (model: flog2)
  const int e = 31 - __clz((int)v);
  const uint32_t m = (e >= 10 ? (v >> (e - 10)) : (v << (10 - e))) & 1023;
  return (e << 12) + frac[m];
}
__device__ __forceinline__ long long flog2_fx64(const int32_t* frac, unsigned long long v) {
  const int e = 63 - __clzll((long long)v);
  const unsigned long long m = (e >= 10 ? (v >> (e - 10)) : (v << (10 - e))) & 1023;
  return ((long long)e << 12) + frac[m];
}

}  // namespace

// ------------------------------------------------------------------ L4

// One workgroup per histogram tile: the tile's symbol histogram in LDS, its
// own entropy per pixel (the clustering's initial order), and the histogram
// as a sparse list (symbol | count << 12) for the clustering passes.
__global__ __launch_bounds__(256) void k_vp8l_tilefeat(const uint32_t* __restrict__ argb,
                                                       const uint32_t* __restrict__ ops,
                                                       vp8l_params p,
                                                       const int32_t* __restrict__ frac,
                                                       int64_t* __restrict__ feat,
                                                       uint32_t* __restrict__ tl,
                                                       uint32_t* __restrict__ tn) {
  __shared__ uint32_t h[VP8L_NS];
  __shared__ unsigned long long acc[6];
  __shared__ uint32_t nnz;
  const int tid = threadIdx.x, f = blockIdx.y, t = blockIdx.x;
  const int W = p.w, H = p.h, hb = p.hb;
  const int tx_n = (W + (1 << hb) - 1) >> hb;
  const int tiles = tx_n * ((H + (1 << hb) - 1) >> hb);
  const int x0 = (t % tx_n) << hb, y0 = (t / tx_n) << hb;
  const int tw = min(1 << hb, W - x0), th = min(1 << hb, H - y0);
  const size_t npix = (size_t)W * H;
  for (int i = tid; i < VP8L_NS; i += 256) h[i] = 0;
  if (tid < 6) acc[tid] = 0;
  if (tid == 0) nnz = 0;
  __syncthreads();
  for (int i = tid; i < tw * th; i += 256) {
    const int ly = i / tw, lx = i - ly * tw;
    const size_t q = f * npix + (size_t)(y0 + ly) * W + x0 + lx;
    PixSym s;
    pix_symbols(ops[q], argb[q], s);
    for (int k = 0; k < 4; ++k)
      if (s.s[k] >= 0) hadd(h, (uint32_t)s.s[k]);
  }
  __syncthreads();
  // per alphabet: N, then own = sum_a N_a log N_a - sum h log h
  unsigned long long n[5] = {0, 0, 0, 0, 0};
  unsigned long long hl = 0;
  const size_t cap = VP8L_TILE_CAP(hb);
  uint32_t* out = tl + ((size_t)f * tiles + t) * cap;
  for (int i = tid; i < VP8L_NS; i += 256) {
    const uint32_t c = h[i];
    n[alph_of(i)] += c;
    if (c > 1) hl += (unsigned long long)c * (unsigned long long)flog2_fx(frac, c);
    if (c) out[atomicAdd(&nnz, 1u)] = (uint32_t)i | (c << 12);
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
    uint16_t lc[VP8L_KMAX * VP8L_NS];
    long long feat[VP8L_MAX_HUFF_IMAGE];
  } u;
  uint8_t assign[VP8L_MAX_HUFF_IMAGE];
  uint32_t nsum[VP8L_KMAX * 5];
};

// One workgroup per frame (16 waves): k-means of the histogram tiles over
// their sparse histograms (model: cluster_tiles). A wave owns a tile at a
// time in both the accumulation and the reassignment passes.
__global__ __launch_bounds__(1024) void k_vp8l_cluster(vp8l_params p,
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
  const int tx_n = (W + (1 << hb) - 1) >> hb, ty_n = (H + (1 << hb) - 1) >> hb;
  const int nt = tx_n * ty_n;
  const size_t cap = VP8L_TILE_CAP(hb);
  const uint32_t* TL = tl + (size_t)f * nt * cap;
  const uint32_t* TN = tn + (size_t)f * nt;

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

  for (int it = 0; it <= VP8L_CLUSTER_ITERS; ++it) {
    // accumulate cluster histograms
    for (int i = tid; i < K * VP8L_NS; i += 1024) S.hc[i] = 0;
    __syncthreads();
    for (int t = wv; t < nt; t += 16) {
      uint32_t* hcc = S.hc + S.assign[t] * VP8L_NS;
      const uint32_t* e = TL + (size_t)t * cap;
      const int m = (int)TN[t];
      for (int i = ln; i < m; i += 64) {
        const uint32_t v = e[i];
        atomicAdd(&hcc[v & 4095], v >> 12);
      }
    }
    __syncthreads();
    if (it == VP8L_CLUSTER_ITERS) break;
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
    for (int i = tid; i < K * VP8L_NS; i += 1024) {
      const int c = i / VP8L_NS, s = i - c * VP8L_NS, a = alph_of(s);
      const uint32_t N = S.nsum[c * 5 + a];
      const int v = flog2_fx(frac, 10u * N + (uint32_t)alph_size(a)) -
                    flog2_fx(frac, 10u * S.hc[i] + 1u);
      S.u.lc[i] = (uint16_t)(v >> 4);
    }
    __syncthreads();
    // reassign: one wave per tile
    for (int t = wv; t < nt; t += 16) {
      const uint32_t* e = TL + (size_t)t * cap;
      const int m = (int)TN[t];
      unsigned long long cost[VP8L_KMAX];
#pragma unroll
      for (int c = 0; c < VP8L_KMAX; ++c) cost[c] = 0;
      for (int i = ln; i < m; i += 64) {
        const uint32_t v = e[i];
        const int sym = (int)(v & 4095);
        const uint32_t cnt = v >> 12;
#pragma unroll
        for (int c = 0; c < VP8L_KMAX; ++c)
          if (c < K) cost[c] += (unsigned long long)cnt * S.u.lc[c * VP8L_NS + sym];
      }
      int bc = 0;
      unsigned long long bv = ~0ull;
#pragma unroll
      for (int c = 0; c < VP8L_KMAX; ++c) {
        const unsigned long long v = wave_sum(cost[c]);
        if (c < K && v < bv) { bv = v; bc = c; }
      }
      if (ln == 0) S.assign[t] = (uint8_t)bc;
    }
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
  for (int k = 0; k < VP8L_BLOCK / 256; ++k) {
    const size_t q = (size_t)blk * VP8L_BLOCK + tid * (VP8L_BLOCK / 256) + k;
    if (q >= npix) break;
    PixSym s;
    pix_symbols(ops[f * npix + q], argb[f * npix + q], s);
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
#pragma unroll
  for (int k = 0; k < VP8L_BLOCK / 256; ++k) {
    const size_t q = (size_t)blk * VP8L_BLOCK + tid * (VP8L_BLOCK / 256) + k;
    if (q < npix) {
      pix_symbols(ops[f * npix + q], argb[f * npix + q], s[k]);
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

extern "C" int vp8l_launch_transform(const uint8_t* rgba, size_t fstride, int rstride,
                                     const vp8l_params* p, uint32_t* argb,
                                     uint8_t* modes, uint32_t* mult, uint32_t* alpha_flag,
                                     void* stream) {
  if (p->tb < 2 || p->tb > 6 || p->w <= 0 || p->h <= 0 || p->n <= 0) return 0;
  dim3 grid((p->w + (1 << p->tb) - 1) >> p->tb, (p->h + (1 << p->tb) - 1) >> p->tb, p->n);
  hipStream_t st = (hipStream_t)stream;
#define L1(T)                                                                              \
  hipLaunchKernelGGL(k_vp8l_transform<T>, grid, dim3(256), 0, st, rgba, fstride, rstride, *p, \
                     argb, modes, mult, alpha_flag)
  switch (p->tb) {
    case 2: L1(4); break;
    case 3: L1(8); break;
    case 4: L1(16); break;
    case 5: L1(32); break;
    default: L1(64); break;
  }
#undef L1
  return check_launch();
}

extern "C" int vp8l_launch_analyze(const uint32_t* argb, const vp8l_params* p,
                                   const int32_t* flog2, uint64_t* hits, uint32_t* ops,
                                   int64_t* feat, uint32_t* tl, uint32_t* tn, uint32_t* hc,
                                   uint8_t* assign, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int npix = p->w * p->h;
  const int tx_n = (p->w + (1 << p->hb) - 1) >> p->hb, ty_n = (p->h + (1 << p->hb) - 1) >> p->hb;
  if (tx_n * ty_n > VP8L_MAX_HUFF_IMAGE || p->k < 1 || p->k > VP8L_KMAX) return 0;
  if (p->cache_bits) {
    hipLaunchKernelGGL(k_vp8l_cache, dim3(p->n), dim3(64), 0, st, argb, npix, hits);
  } else if (hipMemsetAsync(hits, 0, (size_t)p->n * ((npix + 63) >> 6) * sizeof(uint64_t), st) !=
             hipSuccess) {
    return 0;
  }
  hipLaunchKernelGGL(k_vp8l_match, dim3(p->h, p->n), dim3(64), 0, st, argb, hits, *p, ops);
  hipLaunchKernelGGL(k_vp8l_parse, dim3((p->h + 63) / 64, p->n), dim3(64), 0, st, *p, ops);
  hipLaunchKernelGGL(k_vp8l_tilefeat, dim3(tx_n * ty_n, p->n), dim3(256), 0, st, argb, ops, *p,
                     flog2, feat, tl, tn);
  static int attr = 0;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)k_vp8l_cluster,
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)sizeof(ClusterSmem)) != hipSuccess)
      return 0;
    attr = 1;
  }
  hipLaunchKernelGGL(k_vp8l_cluster, dim3(p->n), dim3(1024), sizeof(ClusterSmem), st, *p, flog2,
                     feat, tl, tn, hc, assign);
  return check_launch();
}

extern "C" int vp8l_launch_write(const uint32_t* argb, const uint32_t* ops, const vp8l_params* p,
                                 const uint32_t* ctab, const uint8_t* gtile,
                                 const uint64_t* start_bit, uint32_t* bsum, uint64_t* boff,
                                 uint64_t* end_bit, uint8_t* out, size_t out_cap, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const size_t npix = (size_t)p->w * p->h;
  const int nblk = (int)((npix + VP8L_BLOCK - 1) / VP8L_BLOCK);
  if ((out_cap & 3) != 0) return 0;
  hipLaunchKernelGGL(k_vp8l_bitcount, dim3(nblk, p->n), dim3(256), 0, st, argb, ops, *p, ctab,
                     gtile, bsum);
  hipLaunchKernelGGL(k_vp8l_scan, dim3(p->n), dim3(1024), 0, st, bsum, nblk, start_bit, boff,
                     end_bit);
  hipLaunchKernelGGL(k_vp8l_write, dim3(nblk, p->n), dim3(256), 0, st, argb, ops, *p, ctab, gtile,
                     bsum, boff, out, out_cap);
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
