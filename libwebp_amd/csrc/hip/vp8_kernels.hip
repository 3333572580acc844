// HIP/CDNA4 kernels for the batched VP8 lossy encoder (gfx950).
//
//   K1 k_import    RGBA -> YUV420 with gamma-linear chroma averaging
//                  (picture_csp_enc.c:375-619; yuv.h:186-204). One thread per
//                  2x2 luma quad, coalesced 8-byte RGBA reads. HBM-bound.
//   K2 k_analyze   per-macroblock susceptibility (analysis_enc.c:230-333):
//                  one wavefront per MB, 48 4x4 DCTs on 48 lanes, LDS
//                  histograms.
//   K3 k_encode    the raster-order RD macroblock loop of VP8EncTokenLoop
//                  (frame_enc.c:783-894): one wavefront owns one frame and
//                  walks its MBs in order (the only exact order for the
//                  token statistics / cost-refresh epochs); inside an MB the
//                  I16 (4 modes x 16 blocks = 64 lanes), I4 (10 modes) and
//                  UV (4 modes x 8 blocks) candidates run lane-parallel out
//                  of LDS, then the MB's tokens are generated 25 blocks
//                  in parallel and folded into exact saturating statistics.
//
// No MFMA: there is no dense contraction on this path.
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "vp8_dev.h"

// ---------------------------------------------------------------------------
// K1: RGBA -> YUV420

__device__ __forceinline__ int lin_to_gamma(const int* l2g, uint32_t sum, int shift) {
  const int v = (int)(sum << shift);
  const int pos = v >> 9, frac = v & 511;
  return (l2g[pos + 1] * frac + l2g[pos] * (512 - frac) + 64) >> 7;
}
// VP8RGBToY / VP8ClipUV (src/dsp/yuv.h:186-204) with the rounding term:
// YUV_HALF (<< 2 for chroma), or the dithered one of VP8RandomBits
// (picture_csp_enc.c:153-166) when the import dithers
__device__ __forceinline__ int rgb_to_y(int r, int g, int b, int rnd = 1 << 15) {
  return (16839 * r + 33059 * g + 6420 * b + rnd + (16 << 16)) >> 16;
}
__device__ __forceinline__ int clip_uv(int v, int rnd = 1 << 17) {
  v = (v + rnd + (128 << 18)) >> 18;
  return (v & ~0xff) == 0 ? v : (v < 0 ? 0 : 255);
}

__global__ __launch_bounds__(256) void k_import(const uint8_t* __restrict__ rgba,
                                                size_t fstride, int rstride, int w, int h,
                                                uint8_t* __restrict__ yuv, size_t yfb,
                                                uint32_t* __restrict__ aflags,
                                                uint8_t* __restrict__ aplane,
                                                const uint16_t* __restrict__ g_g2l,
                                                const int32_t* __restrict__ g_l2g,
                                                const uint16_t* __restrict__ rnd_y,
                                                const uint32_t* __restrict__ rnd_uv) {
  __shared__ uint16_t g2l[256];
  __shared__ int l2g[33];
  const int t = threadIdx.x;
  g2l[t] = g_g2l[t];
  if (t < 33) l2g[t] = g_l2g[t];
  __syncthreads();
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  const int i = blockIdx.x * blockDim.x + t;   // chroma column
  const int j = blockIdx.y;                    // chroma row
  const int f = blockIdx.z;
  if (i >= uvw) return;
  const uint8_t* src = rgba + f * fstride;
  uint8_t* Y = yuv + f * yfb;
  uint8_t* U = Y + (size_t)w * h;
  uint8_t* V = U + (size_t)uvw * uvh;
  const int x0 = 2 * i, y0 = 2 * j;
  const bool two_cols = x0 + 1 < w, two_rows = y0 + 1 < h;
  const uint8_t* r0 = src + (size_t)y0 * rstride + 4 * x0;
  const uint8_t* r1 = two_rows ? r0 + rstride : r0;
  uint8_t p[2][2][4];
  if (two_cols && ((rstride | (int)((uintptr_t)src & 7)) & 7) == 0) {   // 8-byte loads
    const uint2 a = *reinterpret_cast<const uint2*>(r0);
    const uint2 b = *reinterpret_cast<const uint2*>(r1);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p[0][0][k] = (uint8_t)(a.x >> (8 * k)); p[0][1][k] = (uint8_t)(a.y >> (8 * k));
      p[1][0][k] = (uint8_t)(b.x >> (8 * k)); p[1][1][k] = (uint8_t)(b.y >> (8 * k));
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      p[0][0][k] = r0[k];
      p[1][0][k] = r1[k];
      p[0][1][k] = two_cols ? r0[4 + k] : 0;
      p[1][1][k] = two_cols ? r1[4 + k] : 0;
    }
  }
  const bool pair16 = two_cols && !(w & 1);   // 16-bit stores of the pixel pairs
  uint32_t alpha_bad = (p[0][0][3] != 0xff) | (p[1][0][3] != 0xff);
  if (two_cols) alpha_bad |= (p[0][1][3] != 0xff) | (p[1][1][3] != 0xff);
  // the WebPPicture alpha plane (WebPExtractAlpha) is not written here: an
  // opaque frame never reads it, and k_extract_alpha copies it afterwards for
  // the frames this kernel flags (0.5 GB of writes per 256 x 1080p batch saved)
  if (alpha_bad) atomicOr(aflags + f, 1u);
  uint8_t* yrow = Y + (size_t)y0 * w + x0;
  const size_t yo = (size_t)y0 * w + x0;
  const int ry00 = rnd_y ? rnd_y[yo] : 1 << 15;
  const int ry01 = rnd_y && two_cols ? rnd_y[yo + 1] : 1 << 15;
  const int ry10 = rnd_y && two_rows ? rnd_y[yo + w] : 1 << 15;
  const int ry11 = rnd_y && two_rows && two_cols ? rnd_y[yo + w + 1] : 1 << 15;
  {
    const int y00 = rgb_to_y(p[0][0][0], p[0][0][1], p[0][0][2], ry00);
    const int y01 = rgb_to_y(p[0][1][0], p[0][1][1], p[0][1][2], ry01);
    const int y10 = rgb_to_y(p[1][0][0], p[1][0][1], p[1][0][2], ry10);
    const int y11 = rgb_to_y(p[1][1][0], p[1][1][1], p[1][1][2], ry11);
    if (pair16) {
      *reinterpret_cast<uint16_t*>(yrow) = (uint16_t)(y00 | (y01 << 8));
      if (two_rows) *reinterpret_cast<uint16_t*>(yrow + w) = (uint16_t)(y10 | (y11 << 8));
    } else {
      yrow[0] = (uint8_t)y00;
      if (two_cols) yrow[1] = (uint8_t)y01;
      if (two_rows) {
        yrow[w] = (uint8_t)y10;
        if (two_cols) yrow[w + 1] = (uint8_t)y11;
      }
    }
  }
  // AccumulateRGBA (picture_csp_enc.c:388-424): 2x2 blocks with partial
  // alpha average in linear light weighted by alpha, divided through
  // kInvAlpha[a] = 2^19 / a (LinearToGammaWeighted, :359-373); opaque and
  // fully transparent blocks take the plain average (AccumulateRGB)
  const uint32_t asum = two_cols ? (uint32_t)p[0][0][3] + p[1][0][3] + p[0][1][3] + p[1][1][3]
                                 : 2u * ((uint32_t)p[0][0][3] + p[1][0][3]);
  const bool weighted = asum != 0 && asum != 4 * 0xff;
  int c[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (weighted) {
      uint64_t sum;
      if (two_cols) {
        sum = (uint64_t)p[0][0][3] * g2l[p[0][0][k]] + (uint64_t)p[0][1][3] * g2l[p[0][1][k]] +
              (uint64_t)p[1][0][3] * g2l[p[1][0][k]] + (uint64_t)p[1][1][3] * g2l[p[1][1][k]];
      } else {
        sum = 2 * ((uint64_t)p[0][0][3] * g2l[p[0][0][k]] + (uint64_t)p[1][0][3] * g2l[p[1][0][k]]);
      }
      const uint32_t inv = (1u << 19) / asum;
      c[k] = lin_to_gamma(l2g, (uint32_t)((sum * inv) >> 17), 0);
    } else if (two_cols) {
      c[k] = lin_to_gamma(l2g, (uint32_t)g2l[p[0][0][k]] + g2l[p[0][1][k]] + g2l[p[1][0][k]] +
                                   g2l[p[1][1][k]], 0);
    } else {
      c[k] = lin_to_gamma(l2g, (uint32_t)g2l[p[0][0][k]] + g2l[p[1][0][k]], 1);
    }
  }
  const size_t uo = (size_t)j * uvw + i;
  const int ru = rnd_uv ? (int)rnd_uv[2 * uo] : 1 << 17;
  const int rv = rnd_uv ? (int)rnd_uv[2 * uo + 1] : 1 << 17;
  U[uo] = clip_uv(-9719 * c[0] - 19081 * c[1] + 28800 * c[2], ru);
  V[uo] = clip_uv(28800 * c[0] - 24116 * c[1] - 4684 * c[2], rv);
}

// alpha plane (WebPExtractAlpha): every frame (the sharp-YUV path, aflags
// NULL) or only the frames K1 flagged as not opaque
__global__ __launch_bounds__(256) void k_extract_alpha(const uint8_t* __restrict__ rgba,
                                                       size_t fstride, int rstride, int w, int h,
                                                       const uint32_t* __restrict__ aflags,
                                                       uint8_t* __restrict__ aplane) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, f = blockIdx.z;
  if (x >= w || (aflags && !aflags[f])) return;
  aplane[(size_t)f * w * h + (size_t)y * w + x] = rgba[f * fstride + (size_t)y * rstride + 4 * x + 3];
}

// WebPCleanupTransparentArea for YUVA (picture_tools_enc.c:99-168), frames
// with alpha only. One workgroup per 8-row strip: 8x8 blocks with some
// transparent pixels get those pixels' luma set to the average of the
// visible ones (SmoothenBlock :53-84); fully transparent blocks of a full
// strip are flattened to the Y/U/V values of the first block of their run
// (`need_reset`), which no thread changes (its own flatten rewrites the same
// values), so the runs resolve in parallel.
__global__ __launch_bounds__(256) void k_cleanup_alpha(uint8_t* __restrict__ yuv, size_t yfb,
                                                       const uint8_t* __restrict__ aplane,
                                                       const uint32_t* __restrict__ aflags,
                                                       int w, int h) {
  __shared__ uint8_t transparent[16384 / 8 + 1];
  const int f = blockIdx.y, y0 = blockIdx.x * 8, t = threadIdx.x;
  if (!aflags[f]) return;
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  uint8_t* Y = yuv + (size_t)f * yfb;
  uint8_t* U = Y + (size_t)w * h;
  uint8_t* V = U + (size_t)uvw * uvh;
  const uint8_t* A = aplane + (size_t)f * w * h;
  const int bh = min(8, h - y0);
  const int nfull = w / 8, nb = (w + 7) / 8;
  for (int b = t; b < nb; b += 256) {
    const int x0 = b * 8, bw = min(8, w - x0);
    int sum = 0, count = 0;
    for (int y = 0; y < bh; ++y)
      for (int x = 0; x < bw; ++x)
        if (A[(size_t)(y0 + y) * w + x0 + x] != 0) {
          ++count;
          sum += Y[(size_t)(y0 + y) * w + x0 + x];
        }
    if (count > 0 && count < bw * bh) {
      const uint8_t avg = (uint8_t)(sum / count);
      for (int y = 0; y < bh; ++y)
        for (int x = 0; x < bw; ++x)
          if (A[(size_t)(y0 + y) * w + x0 + x] == 0) Y[(size_t)(y0 + y) * w + x0 + x] = avg;
    }
    transparent[b] = (count == 0 && bh == 8 && b < nfull);
  }
  __syncthreads();
  if (bh != 8) return;   // the partial last strip is only smoothed
  for (int b = t; b < nfull; b += 256) {
    if (!transparent[b]) continue;
    int s0 = b;
    while (s0 > 0 && transparent[s0 - 1]) --s0;
    const uint8_t vy = Y[(size_t)y0 * w + 8 * s0];
    const uint8_t vu = U[(size_t)(y0 >> 1) * uvw + 4 * s0];
    const uint8_t vv = V[(size_t)(y0 >> 1) * uvw + 4 * s0];
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) Y[(size_t)(y0 + y) * w + 8 * b + x] = vy;
    for (int y = 0; y < 4; ++y)
      for (int x = 0; x < 4; ++x) {
        U[(size_t)((y0 >> 1) + y) * uvw + 4 * b + x] = vu;
        V[(size_t)((y0 >> 1) + y) * uvw + 4 * b + x] = vv;
      }
  }
}

// ---------------------------------------------------------------------------
// K2: analysis (analysis_enc.c:230-333, iterator_enc.c:147-173; histogram
// dsp/enc.c:46-81). A 256-thread workgroup takes a strip of K2_STRIP MBs of
// one MB row: the strip's Y/U/V pixels plus the row above and the column to
// the left are staged in LDS with coalesced loads (edge replication by
// clamping to the picture, which is iterator_enc.c's import), then each
// wavefront analyses K2_STRIP / 4 of the MBs from LDS.

#define K2_STRIP 8
#define K2_YW (16 * K2_STRIP + 4)   // Y tile row: column -1 .. 16*K2_STRIP-1 (+pad)
#define K2_CW (8 * K2_STRIP + 4)    // U/V tile row: column -1 .. 8*K2_STRIP-1 (+pad)

struct K2Wave {
  uint8_t yl[17], ul[9], vl[9];
  uint8_t top[32];
  int dc3[3];   // the DC predictions of Y, U, V
  int hist[4][32];
};

__global__ __launch_bounds__(256) void k_analyze(const uint8_t* __restrict__ yuv, size_t yfb,
                                                 int w, int h, int nmb,
                                                 uint8_t* __restrict__ mb_alpha,
                                                 uint16_t* __restrict__ mb_uva, int fast_q,
                                                 uint8_t* __restrict__ mb_amode) {
  __shared__ uint8_t ty[17 * K2_YW];       // row 0 = the row above the strip
  __shared__ uint8_t tuv[2 * 9 * K2_CW];   // U tile, then V tile
  uint8_t* const tu = tuv;
  uint8_t* const tv = tuv + 9 * K2_CW;
  __shared__ K2Wave S[4];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  const int f = blockIdx.z, y = blockIdx.y, x0 = blockIdx.x * K2_STRIP;
  const int mbw = (w + 15) >> 4;
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  const uint8_t* Yp = yuv + f * yfb;
  const uint8_t* Up = Yp + (size_t)w * h;
  const uint8_t* Vp = Up + (size_t)uvw * uvh;
  // ---- strip tiles: tile (r, c) = picture (16y - 1 + r, 16x0 - 1 + c), clamped.
  // Every byte a thread loads is fetched before any goes to LDS, so the
  // loads are in flight together (a load / wait / store loop made the strip
  // 14 HBM round trips long: K2 4.5 ms per 256 x 1080p batch).
  constexpr int NY = 17 * (16 * K2_STRIP + 1), NYI = (NY + 255) / 256;
  constexpr int NC = 2 * 9 * (8 * K2_STRIP + 1), NCI = (NC + 255) / 256;
  uint8_t vy[NYI], vc[NCI];
  int oy[NYI], oc[NCI];
#pragma unroll
  for (int i = 0; i < NYI; ++i) {   // no branches here: a thread past the tile reloads its last byte
    const int k0 = tid + 256 * i, k = min(k0, NY - 1);
    const int r = k / (16 * K2_STRIP + 1), c = k % (16 * K2_STRIP + 1);
    const int gy = min(max(16 * y - 1 + r, 0), h - 1), gx = min(max(16 * x0 - 1 + c, 0), w - 1);
    vy[i] = Yp[(size_t)gy * w + gx];
    oy[i] = k0 < NY ? r * K2_YW + c : -1;
  }
#pragma unroll
  for (int i = 0; i < NCI; ++i) {
    const int k0 = tid + 256 * i, k = min(k0, NC - 1);
    const int pl = k / (9 * (8 * K2_STRIP + 1)), kk = k % (9 * (8 * K2_STRIP + 1));
    const int r = kk / (8 * K2_STRIP + 1), c = kk % (8 * K2_STRIP + 1);
    const int gy = min(max(8 * y - 1 + r, 0), uvh - 1), gx = min(max(8 * x0 - 1 + c, 0), uvw - 1);
    vc[i] = (pl ? Vp : Up)[(size_t)gy * uvw + gx];
    oc[i] = k0 < NC ? pl * (9 * K2_CW) + r * K2_CW + c : -1;   // tu and tv back to back
  }
#pragma unroll
  for (int i = 0; i < NYI; ++i)
    if (oy[i] >= 0) ty[oy[i]] = vy[i];
#pragma unroll
  for (int i = 0; i < NCI; ++i)
    if (oc[i] >= 0) tuv[oc[i]] = vc[i];
  __syncthreads();
  K2Wave& L = S[wave];
  for (int it = 0; it < K2_STRIP / 4; ++it) {   // uniform trip count: the barriers below
    const int xl = wave + 4 * it, x = x0 + xl;
    const bool valid = x < mbw;
    const int mb = y * mbw + x;
    // this MB's pixels in the tiles: Y at (1, 1 + 16 xl), U/V at (1, 1 + 8 xl)
    const uint8_t* yin = ty + K2_YW + 1 + 16 * xl;
    const uint8_t* uin = tu + K2_CW + 1 + 8 * xl;
    const uint8_t* vin = tv + K2_CW + 1 + 8 * xl;
    uint8_t* yl = L.yl + 1;
    uint8_t* ul = L.ul + 1;
    uint8_t* vl = L.vl + 1;
    if (lane < 32) {   // source boundary (iterator_enc.c:147-173)
      const int i = lane;
      if (x == 0) {
        if (i < 16) yl[i] = 129;
        if (i < 8) { ul[i] = 129; vl[i] = 129; }
        if (i == 0) yl[-1] = ul[-1] = vl[-1] = (y > 0) ? 129 : 127;
      } else {
        if (i < 16) yl[i] = yin[i * K2_YW - 1];
        if (i < 8) { ul[i] = uin[i * K2_CW - 1]; vl[i] = vin[i * K2_CW - 1]; }
        if (i == 0) {
          if (y == 0) {
            yl[-1] = ul[-1] = vl[-1] = 127;
          } else {
            yl[-1] = yin[-K2_YW - 1]; ul[-1] = uin[-K2_CW - 1]; vl[-1] = vin[-K2_CW - 1];
          }
        }
      }
      if (y == 0) L.top[i] = 127;
      else if (i < 16) L.top[i] = yin[i - K2_YW];
      else L.top[i] = (i < 24 ? uin : vin)[(i & 7) - K2_CW];
    }
    if (lane >= 32 && lane < 35) {   // DC predictions straight from the tiles (dc_value)
      const int c = lane - 32, n = c ? 8 : 16, stride = c ? K2_CW : K2_YW;
      const uint8_t* in = c == 0 ? yin : c == 1 ? uin : vin;
      int dc = 0;
      if (y > 0) {
        for (int jj = 0; jj < n; ++jj) dc += in[jj - stride];
        if (x > 0) { for (int jj = 0; jj < n; ++jj) dc += in[jj * stride - 1]; }
        else dc += dc;
        dc = (dc + n) >> (c ? 4 : 5);
      } else if (x > 0) {
        for (int jj = 0; jj < n; ++jj) dc += in[jj * stride - 1];
        dc += dc;
        dc = (dc + n) >> (c ? 4 : 5);
      } else {
        dc = 0x80;
      }
      L.dc3[c] = dc;
    }
    for (int k = lane; k < 4 * 32; k += 64) (&L.hist[0][0])[k] = 0;
    __syncthreads();
    const bool hl = x > 0, ht = y > 0;
    if (lane < 48) {   // DC / TM residual of one 4x4 block, predicted on the fly
      int coeffs[16], hsel, d[16];
      const uint8_t* src;
      int ss, m, px0, py0, n;
      const uint8_t *left, *top;
      if (lane < 32) {
        m = lane >> 4;
        const int b = lane & 15;
        px0 = (b & 3) * 4; py0 = (b >> 2) * 4;
        src = yin + py0 * K2_YW + px0; ss = K2_YW;
        left = yl; top = L.top; n = 16;
        hsel = m;
      } else {
        m = (lane - 32) >> 3;
        const int b = lane & 7, c = b >> 2, k = b & 3;
        px0 = (k & 1) * 4; py0 = (k >> 1) * 4;
        src = (c ? vin : uin) + py0 * K2_CW + px0; ss = K2_CW;
        left = c ? vl : ul; top = L.top + 16 + 8 * c; n = 8;
        hsel = 2 + m;
      }
      const int dcv = m == 0 ? L.dc3[lane < 32 ? 0 : 1 + ((lane & 7) >> 2)] : 0;
#pragma unroll
      for (int i = 0; i < 16; ++i)
        d[i] = src[(i >> 2) * ss + (i & 3)] -
               pred_sample(m, n, px0 + (i & 3), py0 + (i >> 2), left, top, hl, ht, dcv);
      fdct4_res(d, coeffs);
      // bins 0..7 counted in 16-bit fields of two registers, summed over the
      // block group's lanes (16 for Y, 8 for U/V) with shuffles; the rarer
      // bins 8..31 by LDS atomics
      uint64_t c0 = 0, c1 = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int v = min(iabs_(coeffs[k]) >> 3, 31);
        const uint64_t one = 1ull << (16 * (v & 3));
        c0 += v < 4 ? one : 0ull;
        c1 += (v >= 4 && v < 8) ? one : 0ull;
#ifndef K2_NO_ATOMIC   // (timing A/B only: drops bins 8..31)
        if (v >= 8) atomicAdd(&L.hist[hsel][v], 1);
#endif
      }
      const int gsz = lane < 32 ? 16 : 8;
      for (int o = 1; o < gsz; o <<= 1) {
        c0 += __shfl_xor(c0, o);
        c1 += __shfl_xor(c1, o);
      }
      if ((lane & (gsz - 1)) < 8) {   // 8 lanes per group store the 8 bins
        const int bin = lane & 7;
        const uint64_t c = bin < 4 ? c0 : c1;
        L.hist[hsel][bin] = (int)((c >> (16 * (bin & 3))) & 0xffff);
      }
    }
    uint32_t dcs = 0;   // VP8Mean16x4 block sums (dsp/enc.c:594-608), lanes 0..15
    if (fast_q >= 0 && lane < 16)
      for (int k = 0; k < 16; ++k)
        dcs += yin[(4 * (lane >> 2) + (k >> 2)) * K2_YW + 4 * (lane & 3) + (k & 3)];
    __syncthreads();
    // alpha of each histogram (dsp/enc.c:46-81): max count and last non-empty
    // bin, one bin per lane, half a wave per histogram, two rounds
    int alpha[4];
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int hh = (lane >> 5) + 2 * pass;
      const int v = L.hist[hh][lane & 31];
      int mx = v;
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
      const uint64_t nz = __ballot(v > 0);
      const uint32_t half = (uint32_t)(nz >> (lane & 32));
      const int last = half ? 31 - __builtin_clz(half) : 1;
      const int al = mx > 1 ? 510 * last / mx : 0;
      alpha[2 * pass] = __shfl(al, 0);
      alpha[2 * pass + 1] = __shfl(al, 32);
    }
    uint32_t dsum = dcs, dsq = dcs * dcs;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) { dsum += __shfl_xor(dsum, o); dsq += __shfl_xor(dsq, o); }
    if (lane == 0 && valid) {
      int best = -1;
      if (alpha[0] > best) best = alpha[0];
      if (alpha[1] > best) best = alpha[1];
      int best_uv = -1;
      if (alpha[2] > best_uv) best_uv = alpha[2];
      if (alpha[3] > best_uv) best_uv = alpha[3];
      // analysis modes for the RD_OPT_NONE encoder (methods 0-2): the UV mode
      // of smallest alpha (analysis_enc.c:278-305) and, for methods 0-1,
      // FastMBAnalyze's intra-16 / intra-4 pick with susceptibility 0 (:255-276)
      int i4 = 0;
      if (fast_q >= 0) {
        const uint32_t thr = 8 + (17 - 8) * fast_q / 100;
        i4 = !(thr * dsq < dsum * dsum);
        best = 0;
      }
      if (mb_amode != nullptr)
        mb_amode[(size_t)f * nmb + mb] = (uint8_t)((alpha[3] < alpha[2] ? 1 : 0) | (i4 << 1));
      int a = (3 * best + best_uv + 2) >> 2;
      a = 255 - a;
      a = a < 0 ? 0 : a > 255 ? 255 : a;
      mb_alpha[(size_t)f * nmb + mb] = (uint8_t)a;
      mb_uva[(size_t)f * nmb + mb] = (uint16_t)best_uv;
    }
    __syncthreads();   // this wave's LDS is reused by its next MB
  }
}

// ---------------------------------------------------------------------------
// K3: RD search + tokens + statistics, one wavefront per frame.

struct K3Lds {
  uint32_t stats[NSLOT];
  uint32_t delta[NSLOT];
  uint16_t lcost[96][MAX_VLEVEL + 1];  // [type*24 + band*3 + ctx][level], incl. fixed cost
  uint16_t ecost[256];            // kVP8EntropyCost
  uint16_t mcost4[1000];          // kVP8ModeCostI4[top][left][mode]
  P4Op p4[160];                   // kP4
  uint8_t coeffs[NSLOT];
  uint32_t mark[33];
  vp8g_seg seg[4];
  uint8_t yin[16 * BPS];
  uint8_t yout[16 * BPS];
  uint8_t p16[4][256];
  uint8_t puv[4][128];
  uint8_t rec16[4][256];
  uint8_t recuv[4][128];
  alignas(16) int16_t lv16[4][16][16];
  alignas(16) int16_t lvdc[4][16];
  int16_t whtq[4][16];
  int16_t dcs[4][16];
  alignas(16) int16_t lvuv[4][8][16];
  int16_t uvdc[4][8];
  int8_t uvderr[4][2][3];
  alignas(16) int16_t fin_dc[16];
  alignas(16) int16_t fin_ac[16][16];
  alignas(16) int16_t fin_uv[8][16];
  uint8_t modes[16];
  uint8_t canvas[17][24];
  uint8_t edges[16];
  uint8_t pred4[10][16];
  alignas(16) int16_t lv4[10][16];
  uint8_t rec4[10][16];
  int32_t r4[10][8];
  alignas(16) int16_t acc_ac[16][16];
  uint8_t acc_out[256];          // I4 reconstruction, stride 16
  int32_t mres[4][4];
  int32_t blkinfo[32];            // per token block: type | first<<4 | ctx<<8
  uint32_t trnz[4];               // per-mode trellis nz bits (I16 anti-diagonals)
  uint32_t tnodes[64][32];        // per-lane trellis node scratch
  int32_t max_edge[4];
  uint8_t yl_mem[17], ul_mem[9], vl_mem[9];
  uint8_t predleft[4];
  int8_t lderr[2][2];
};

// I16 candidates: lane = mode*16 + block (quant_enc.c:772-822,
// cost_enc.c:232-256). Fills rec16 / lv16 / lvdc and
// mres[m] = {SSE, texture distortion, rate, nz (ac bits | dc << 24)}.
// With trellis (m6 search, m5 final pass) the AC blocks are trellis-quantised
// in anti-diagonal waves so each block sees its top/left neighbours' nz.
template <bool TRELLIS>
__device__ void eval_i16(K3Lds& L, const vp8g_seg& S, const MBCtx& ctx, int lane) {
  constexpr bool trellis = TRELLIS;
  const int m = lane >> 4, b = lane & 15, bx = b & 3, by = b >> 2;
  int c[16];
  const uint8_t* src = L.yin + by * 4 * BPS + bx * 4;
  const uint8_t* ref = L.p16[m] + by * 64 + bx * 4;
  fdct4(src, BPS, ref, 16, c);
  L.dcs[m][b] = (int16_t)c[0];
  if (lane < 4) L.trnz[lane] = 0;
  wsync();
  {   // WHT coefficient b of mode m, quantised with y2 (natural index b)
    const int16_t* d = L.dcs[m];
    const int r = b >> 2, col = b & 3;
    int t0[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int a0 = d[4 * rr + 0] + d[4 * rr + 2], a1 = d[4 * rr + 1] + d[4 * rr + 3];
      const int a2 = d[4 * rr + 1] - d[4 * rr + 3], a3 = d[4 * rr + 0] - d[4 * rr + 2];
      t0[rr] = col == 0 ? a0 + a1 : col == 1 ? a3 + a2 : col == 2 ? a3 - a2 : a0 - a1;
    }
    const int a0 = t0[0] + t0[2], a1 = t0[1] + t0[3], a2 = t0[1] - t0[3], a3 = t0[0] - t0[2];
    int v = r == 0 ? a0 + a1 : r == 1 ? a3 + a2 : r == 2 ? a3 - a2 : a0 - a1;
    v = (int16_t)(v >> 1);
    const vp8g_mtx& M = S.y2;
    const int neg = v < 0;
    const uint32_t coeff = (uint32_t)(neg ? -v : v) + M.sharpen[b];
    int level = 0;
    if (coeff > M.zthresh[b]) {
      level = (int)((coeff * M.iq[b] + M.bias[b]) >> QFIX);
      if (level > MAX_LEVEL) level = MAX_LEVEL;
      if (neg) level = -level;
    }
    L.lvdc[m][zz_inv(b)] = (int16_t)level;
    L.whtq[m][b] = (int16_t)(level * (int)M.q[b]);
  }
  int nzb = 0;
  int lvr[16];
  if constexpr (trellis) {   // quant_enc.c:790-803
    for (int st = 0; st < 7; ++st) {
      if (bx + by == st) {
        const uint32_t tm = L.trnz[m];
        const int tc = by == 0 ? ctx.top(bx) : (int)((tm >> (b - 4)) & 1);
        const int lc = bx == 0 ? ctx.left(by) : (int)((tm >> (b - 1)) & 1);
        nzb = trellis_quant(L, L.tnodes[lane], c, L.lv16[m][b], tc + lc, 0, &S.y1,
                            S.lambda_trellis_i16);
        L.lv16[m][b][0] = 0;
        if (nzb) atomicOr(&L.trnz[m], 1u << b);
      }
      wsync();
    }
    load_lv(L.lv16[m][b], lvr);
  } else {         // quant_enc.c:805-812: DC position zeroed first
    c[0] = 0;
    nzb = quantize_block(c, L.lv16[m][b], &S.y1, lvr);
  }
  // rate of the AC levels while they are still in registers (nz contexts of
  // the neighbouring blocks of the same mode from a ballot)
  const uint64_t nzmask_all = __ballot(nzb);
  const uint32_t nzm = (uint32_t)(nzmask_all >> (16 * m)) & 0xffff;
  int r;
  {
    const int tctx = by == 0 ? ctx.top(bx) : (int)((nzm >> (b - 4)) & 1);
    const int lctx = bx == 0 ? ctx.left(by) : (int)((nzm >> (b - 1)) & 1);
    r = residual_cost_r(L, tctx + lctx, 0, 1, lvr);
  }
  wsync();
  {   // inverse WHT -> DC of block b (dec.c:137-162)
    const int16_t* q = L.whtq[m];
    const int r = b >> 2, col = b & 3;
    int t[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int a0 = q[i] + q[12 + i], a1 = q[4 + i] + q[8 + i];
      const int a2 = q[4 + i] - q[8 + i], a3 = q[i] - q[12 + i];
      t[i] = r == 0 ? a0 + a1 : r == 1 ? a3 + a2 : r == 2 ? a0 - a1 : a3 - a2;
    }
    const int dd = t[0] + 3;
    const int a0 = dd + t[3], a1 = t[1] + t[2], a2 = t[1] - t[2], a3 = dd - t[3];
    c[0] = (int16_t)((col == 0 ? a0 + a1 : col == 1 ? a3 + a2 : col == 2 ? a0 - a1 : a3 - a2) >> 3);
  }
  idct4(ref, 16, c, L.rec16[m] + by * 64 + bx * 4, 16);
  wsync();
  const uint8_t* rec = L.rec16[m] + by * 64 + bx * 4;
  int d = sse4(src, BPS, rec, 16);
  int td = iabs_(hadamard_w(rec, 16) - hadamard_w(src, BPS)) >> 5;
  int dcl[16];
  load_lv(L.lvdc[m], dcl);
  int dcnz = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) dcnz |= dcl[k];
  if (b == 0) r += residual_cost_r(L, ctx.top(8) + ctx.left(8), 1, 0, dcl);
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1) {
    d += __shfl_xor(d, off, 16);
    td += __shfl_xor(td, off, 16);
    r += __shfl_xor(r, off, 16);
  }
  if (b == 0) {
    L.mres[m][0] = d;
    L.mres[m][1] = td;
    L.mres[m][2] = r;
    L.mres[m][3] = (int)(nzm | (dcnz ? (1u << 24) : 0u));
  }
  wsync();
}

// UV candidates: lane = mode*8 + block, lanes 0..31 (quant_enc.c:875-969,
// cost_enc.c:258-278). Fills recuv / lvuv / uvderr and
// mres[m] = {SSE, rate, non-zero AC count, nz bits}.
__device__ void eval_uv(K3Lds& L, const vp8g_seg& S, const MBCtx& ctx, int lane, int x,
                        const int8_t* topderr, int use_derr) {
  int d = 0, r = 0, flatc = 0, nzb = 0;
  int lvr[16];
  const int m = lane >> 3, b = lane & 7;
  int c[16];
  const int ch = b >> 2, k4 = b & 3;
  const uint8_t* src = L.yin + 16 + 8 * ch + (k4 >> 1) * 4 * BPS + (k4 & 1) * 4;
  const uint8_t* ref = L.puv[m & 3] + 8 * ch + (k4 >> 1) * 64 + (k4 & 1) * 4;
  if (lane < 32) {
    fdct4(src, BPS, ref, 16, c);
    L.uvdc[m][b] = (int16_t)c[0];
  }
  wsync();
  if (use_derr && lane < 8) {   // CorrectDCValues per (mode, channel)
    const int mm = lane >> 1, cch = lane & 1;
    const vp8g_mtx& M = S.uv;
    const int8_t* top = topderr + 4 * x + 2 * cch;
    const int8_t* left = L.lderr[cch];
    int16_t* cc = &L.uvdc[mm][4 * cch];
    int err[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int add;
      if (k == 0) add = (7 * top[0] + 8 * left[0]) >> 3;
      else if (k == 1) add = (7 * top[1] + 8 * err[0]) >> 3;
      else if (k == 2) add = (7 * err[0] + 8 * left[1]) >> 3;
      else add = (7 * err[1] + 8 * err[2]) >> 3;
      int V = (int16_t)(cc[k] + add);
      const int neg = V < 0;
      if (neg) V = -V;
      if (V > (int)M.zthresh[0]) {
        const int qV = (int)(((uint32_t)V * M.iq[0] + M.bias[0]) >> QFIX) * M.q[0];
        const int e = V - qV;
        cc[k] = (int16_t)(neg ? -qV : qV);
        err[k] = (neg ? -e : e) >> 1;
      } else {
        cc[k] = 0;
        err[k] = (neg ? -V : V) >> 1;
      }
    }
    L.uvderr[mm][cch][0] = (int8_t)err[1];
    L.uvderr[mm][cch][1] = (int8_t)err[2];
    L.uvderr[mm][cch][2] = (int8_t)err[3];
  }
  wsync();
  if (lane < 32) {
    c[0] = L.uvdc[m][b];
    nzb = quantize_block(c, L.lvuv[m][b], &S.uv, lvr);
    idct4(ref, 16, c, L.recuv[m] + 8 * ch + (k4 >> 1) * 64 + (k4 & 1) * 4, 16);
  }
  wsync();
  const uint64_t nzall = __ballot(lane < 32 && nzb);
  if (lane < 32) {
    const uint8_t* rec = L.recuv[m] + 8 * ch + (k4 >> 1) * 64 + (k4 & 1) * 4;
    d = sse4(src, BPS, rec, 16);
    const uint32_t nzm = (uint32_t)(nzall >> (8 * m)) & 0xff;
    const int bxx = k4 & 1, byy = k4 >> 1;
    const int tctx = byy == 0 ? ctx.top(4 + 2 * ch + bxx) : (int)((nzm >> (b - 2)) & 1);
    const int lctx = bxx == 0 ? ctx.left(4 + 2 * ch + byy) : (int)((nzm >> (b - 1)) & 1);
    r = residual_cost_r(L, tctx + lctx, 2, 0, lvr);
#pragma unroll
    for (int i = 1; i < 16; ++i) flatc += lvr[i] != 0;
#pragma unroll
    for (int off = 4; off >= 1; off >>= 1) {
      d += __shfl_xor(d, off, 8);
      r += __shfl_xor(r, off, 8);
      flatc += __shfl_xor(flatc, off, 8);
    }
    if (b == 0) {
      L.mres[m][0] = d; L.mres[m][1] = r; L.mres[m][2] = flatc; L.mres[m][3] = (int)nzm;
    }
  }
  wsync();
}

struct I4Result {
  int ok;
  score_t H, score;
  uint32_t nz;
};

// Intra4 sub-block loop (quant_enc.c:1072-1165). search: RD mode choice with
// the reference's early-outs; !search: the m5 SimpleQuantize pass over the
// already chosen L.modes (quant_enc.c:1230-1240), whose trellis contexts are
// the macroblock-boundary flags only (the reference never updates them
// inside that loop). Reconstruction lands in acc_out, levels in acc_ac.
template <bool TRELLIS>
// search: 0 = reconstruct L.modes; 1 = RD search (PickBestIntra4,
// quant_enc.c:1072-1165); 2 = distortion search of RD_OPT_NONE
// (RefineUsingDistortion, :1287-1320): prediction SSE + fixed mode cost,
// running score from the segment's i4_penalty, abort against rd_score (the
// intra-16 distortion score) or max_bits
__device__ I4Result run_i4(K3Lds& L, const vp8g_seg& S, const MBCtx& ctx, int lane, int x,
                           int mbw, const uint8_t* predtop, const uint8_t* yl,
                           const uint8_t* yt, int search, score_t rd_score, int max_bits) {
  constexpr bool trellis = TRELLIS;
  for (int k = lane; k < 21; k += 64) {
    uint8_t v;
    if (k == 0) v = yl[-1];
    else if (k <= 16) v = yt[k - 1];
    else v = (x < mbw - 1) ? yt[16 + k - 17] : yt[15];
    L.canvas[0][k] = v;
  }
  if (lane < 16) L.canvas[1 + lane][0] = yl[lane];
  uint32_t tnz = ctx.t & 0xf, lnz = ctx.l & 0xf;
  score_t accD = 0, accSD = 0, accR = 0, accH = 211;
  score_t acc_score = search == 2 ? (score_t)S.i4_penalty : accH * S.lambda_mode;
  uint32_t acc_nz = 0;
  int total_hdr = 0;
  I4Result res;
  res.ok = 1;
  wsync();
  for (int i4 = 0; i4 < 16; ++i4) {
    const int bx = i4 & 3, by = i4 >> 2;
    const int left_m = bx == 0 ? L.predleft[by] : L.modes[i4 - 1];
    const int top_m = by == 0 ? predtop[4 * x + bx] : L.modes[i4 - 4];
    if (lane < 13) {   // edges e[0..12] = L K J I X A..D E..H
      const int r = 4 * by, cc = 4 * bx;
      uint8_t v;
      if (lane < 4) v = L.canvas[r + 4 - lane][cc];
      else if (lane == 4) v = L.canvas[r][cc];
      else if (lane < 9) v = L.canvas[r][cc + 1 + (lane - 5)];
      else v = (by > 0 && bx == 3) ? L.canvas[0][17 + lane - 9] : L.canvas[r][cc + 5 + lane - 9];
      L.edges[lane] = v;
    }
    wsync();
    for (int k = lane; k < 160; k += 64) {
      const int m = k >> 4, p = k & 15;
      const P4Op op = L.p4[k];
      const uint8_t* e = L.edges;
      int v;
      if (op.kind == 0) v = (e[op.a] + 2 * e[op.b] + e[op.c] + 2) >> 2;
      else if (op.kind == 1) v = (e[op.a] + e[op.b] + 1) >> 1;
      else if (op.kind == 2) v = e[op.a];
      else if (op.kind == 3) v = clip8(e[5 + (p & 3)] + e[3 - (p >> 2)] - e[4]);
      else v = (4 + e[0] + e[1] + e[2] + e[3] + e[5] + e[6] + e[7] + e[8]) >> 3;
      L.pred4[m][p] = (uint8_t)v;
    }
    wsync();
    if (lane < 10) {
      const int m = lane;
      const uint8_t* src = L.yin + by * 4 * BPS + bx * 4;
      int c[16];
      fdct4(src, BPS, L.pred4[m], 4, c);
      const int ctx4 = (int)((tnz >> bx) & 1) + (int)((lnz >> by) & 1);
      int nz;
      int lvr[16];
      if constexpr (trellis) {
        nz = trellis_quant(L, L.tnodes[lane], c, L.lv4[m], ctx4, 3, &S.y1, S.lambda_trellis_i4);
        load_lv(L.lv4[m], lvr);
      } else {
        nz = quantize_block(c, L.lv4[m], &S.y1, lvr);
      }
      idct4(L.pred4[m], 4, c, L.rec4[m], 4);
      if (search == 2) L.r4[m][6] = sse4(src, BPS, L.pred4[m], 4);
      if (search == 1) {
        const int D = sse4(src, BPS, L.rec4[m], 4);
        const int SD = S.tlambda ? (S.tlambda * (iabs_(hadamard_w(L.rec4[m], 4) -
                                                        hadamard_w(src, BPS)) >> 5) + 128) >> 8
                                 : 0;
        int cntnz = 0;
#pragma unroll
        for (int i = 1; i < 16; ++i) cntnz += lvr[i] != 0;
        const int R0 = (m > 0 && cntnz <= 3) ? 140 : 0;
        const int Rc = residual_cost_r(L, ctx4, 3, 0, lvr);
        L.r4[m][0] = D; L.r4[m][1] = SD; L.r4[m][2] = L.mcost4[(top_m * 10 + left_m) * 10 + m];
        L.r4[m][3] = R0; L.r4[m][4] = Rc;
      }
      L.r4[m][5] = nz;
    }
    wsync();
    int bm;
    int bnz;
    if (search == 2) {
      bm = -1;
      score_t bscore = MAX_COST;
      for (int m = 0; m < 10; ++m) {
        const score_t sc = (score_t)L.r4[m][6] * 256 + L.mcost4[(top_m * 10 + left_m) * 10 + m] * 11;
        if (sc < bscore) { bm = m; bscore = sc; }
      }
      total_hdr += L.mcost4[(top_m * 10 + left_m) * 10 + bm];
      acc_score += bscore;
      if (lane == 0) L.modes[i4] = (uint8_t)bm;
      if (acc_score >= rd_score || total_hdr > max_bits) { res.ok = 0; break; }
      bnz = L.r4[bm][5];
      acc_nz |= (uint32_t)(bnz ? 1 : 0) << i4;
    } else if (search) {
      bm = -1;
      score_t bscore = MAX_COST, bD = 0, bSD = 0, bR = 0, bH = 0;
      bnz = 0;
      for (int m = 0; m < 10; ++m) {
        const score_t D = L.r4[m][0], SD = L.r4[m][1], H = L.r4[m][2];
        score_t R = L.r4[m][3];
        score_t sc = (R + H) * S.lambda_i4 + 256 * (D + SD);
        if (bm >= 0 && sc >= bscore) continue;
        R += L.r4[m][4];
        sc = (R + H) * S.lambda_i4 + 256 * (D + SD);
        if (bm < 0 || sc < bscore) {
          bm = m; bscore = sc; bD = D; bSD = SD; bR = R; bH = H; bnz = L.r4[m][5];
        }
      }
      const score_t bsm = (bR + bH) * S.lambda_mode + 256 * (bD + bSD);
      accD += bD; accSD += bSD; accR += bR; accH += bH; acc_score += bsm;
      acc_nz |= (uint32_t)(bnz ? 1 : 0) << i4;
      if (acc_score >= rd_score) { res.ok = 0; break; }
      total_hdr += (int)bH;
      if (total_hdr > max_bits) { res.ok = 0; break; }
    } else {
      bm = L.modes[i4];
      bnz = L.r4[bm][5];
      acc_nz |= (uint32_t)(bnz ? 1 : 0) << i4;
    }
    if (lane < 16) {
      const int py = lane >> 2, px = lane & 3;
      const uint8_t v = L.rec4[bm][lane];
      L.canvas[4 * by + 1 + py][4 * bx + 1 + px] = v;
      L.acc_out[(4 * by + py) * 16 + 4 * bx + px] = v;
      L.acc_ac[i4][lane] = L.lv4[bm][lane];
    }
    if (search == 1) {
      if (lane == 0) L.modes[i4] = (uint8_t)bm;
      tnz = (tnz & ~(1u << bx)) | ((bnz ? 1u : 0u) << bx);
      lnz = (lnz & ~(1u << by)) | ((bnz ? 1u : 0u) << by);
    }
    wsync();
  }
  wsync();
  res.H = accH;
  res.score = acc_score;
  res.nz = acc_nz;
  (void)accD; (void)accSD; (void)accR;
  return res;
}

// per-stage cycle accounting (s_memtime, uniform -> SGPRs); ~40 cycles each
#define K3_STAMP(i)                                   \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    stamps[i] += t_ - stamp_last;                     \
    stamp_last = t_;                                  \
  } while (0)

struct K3ArgsW1 {
  const uint8_t* yuv;
  size_t yfb;
  int w, h, mbw, mbh;
  const uint8_t* segmap;
  const vp8g_frame_params* params;
  uint16_t* tokens;
  size_t tok_cap;
  uint8_t* mbinfo;
  vp8g_frame_result* results;
  // RD_OPT_NONE (methods 0-2) only
  const uint8_t* amode;   // K2 analysis modes
  uint32_t* mboff;        // per-MB token offsets (skip compaction)
  uint8_t* rerun;         // statistics carried between passes
};

// NONE: the methods 0-2 encoder (RefineUsingDistortion, VP8EncLoop); else the
// single-wavefront diagnostic twin of K3 (WEBP_AMD_K3=1)
template <bool NONE>
__global__ __launch_bounds__(64) void k_encode_w1(K3ArgsW1 a) {
  extern __shared__ __align__(16) uint8_t smem[];
  K3Lds& L = *reinterpret_cast<K3Lds*>(smem);
  const int mbw = a.mbw, mbh = a.mbh, nmb = mbw * mbh;
  uint8_t* ytop = smem + sizeof(K3Lds);          // 16*mbw + 4
  uint8_t* uvtop = ytop + 16 * mbw + 16;         // 16*mbw
  uint32_t* nzw = reinterpret_cast<uint32_t*>(uvtop + 16 * mbw) + 1;   // [-1..mbw-1]
  uint8_t* predtop = reinterpret_cast<uint8_t*>(nzw + mbw);           // 4*mbw
  int8_t* topderr = reinterpret_cast<int8_t*>(predtop + 4 * mbw);     // 4*mbw

  const int f = blockIdx.x;
  const int lane = threadIdx.x;
  const int w = a.w, h = a.h;
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  const uint8_t* Yp = a.yuv + f * a.yfb;
  const uint8_t* Up = Yp + (size_t)w * h;
  const uint8_t* Vp = Up + (size_t)uvw * uvh;
  const vp8g_frame_params* P = a.params + f;
  const uint8_t* segmap = a.segmap + (size_t)f * nmb;
  uint16_t* tok_base = a.tokens + f * a.tok_cap;
  uint8_t* mbinfo = a.mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES;
  // this single-wavefront diagnostic kernel keeps no re-run state: it skips
  // final frames and refuses a partition-0 re-run (error 3)
  if (P->pass_mode == 2) return;
  if (P->pass_mode != 0 && !(NONE && P->pass_mode == 3)) {
    if (lane == 0) a.results[f].error = 3;
    return;
  }
  uint32_t* rstats =
      NONE ? reinterpret_cast<uint32_t*>(a.rerun + (size_t)f * VP8G_RERUN_STATE_BYTES +
                                         VP8G_STATE_STATS)
           : nullptr;

  // ---- frame init
  for (int s = lane; s < NSLOT; s += 64) {
    L.stats[s] = (NONE && P->pass_mode == 3) ? rstats[s] : 0u;   // StatLoop keeps them
    L.delta[s] = 0;
    L.coeffs[s] = (&kVP8CoeffProba0[0][0][0][0])[s];
  }
  for (int k = lane; k < 33; k += 64) L.mark[k] = 0;
  for (int k = lane; k < 256; k += 64) L.ecost[k] = kVP8EntropyCost[k];
  for (int k = lane; k < 1000; k += 64) L.mcost4[k] = (&kVP8ModeCostI4[0][0][0])[k];
  for (int k = lane; k < 160; k += 64) L.p4[k] = (&kP4[0][0])[k];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(P->seg);
    uint32_t* dst = reinterpret_cast<uint32_t*>(L.seg);
    for (int k = lane; k < (int)(sizeof(L.seg) / 4); k += 64) dst[k] = src[k];
  }
  for (int k = lane; k < 16 * mbw + 16; k += 64) ytop[k] = 127;
  for (int k = lane; k < 16 * mbw; k += 64) uvtop[k] = 127;
  for (int k = lane - 1; k < mbw; k += 64) nzw[k] = 0;
  for (int k = lane; k < 4 * mbw; k += 64) { predtop[k] = 0; topderr[k] = 0; }
  wsync();
  level_costs(L, lane);

  const int rd_opt = P->rd_opt;
  const int max_i4_bits = P->max_i4_header_bits;
  const int use_derr = P->use_derr;
  const int max_count = P->max_count;
  int cnt = max_count;
  if (lane < 4) L.max_edge[lane] = 0;
  uint64_t size_p0 = 0, sse_acc[3] = {0, 0, 0};
  int nb_i4 = 0, nb_i16 = 0, nb_skip = 0, nb_skip_stat = 0;
  uint32_t ntok = 0;
  int tok_err = 0;
  int left_dc = 0;
  uint64_t stamps[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t stamp_last = __builtin_amdgcn_s_memtime();
  uint8_t* yl = L.yl_mem + 1;
  uint8_t* ul = L.ul_mem + 1;
  uint8_t* vl = L.vl_mem + 1;

  for (int mb = 0; mb < nmb; ++mb) {
    const int x = mb % mbw, y = mb / mbw;
    if (x == 0) {   // InitLeft (iterator_enc.c:22-32)
      if (lane < 16) yl[lane] = 129;
      if (lane < 8) { ul[lane] = 129; vl[lane] = 129; }
      if (lane == 0) {
        yl[-1] = ul[-1] = vl[-1] = (y > 0) ? 129 : 127;
        L.lderr[0][0] = L.lderr[0][1] = L.lderr[1][0] = L.lderr[1][1] = 0;
      }
      if (lane < 4) L.predleft[lane] = 0;
      left_dc = 0;
    }
    load_mb(Yp, Up, Vp, w, h, x, y, L.yin, lane, 64);
    if (!NONE && --cnt < 0) {   // StatLoop never refreshes the probabilities
      if (finalize_probas(L, lane)) level_costs(L, lane);
      cnt = max_count;
    }
    wsync();
    const int segid = segmap[mb];
    const vp8g_seg& S = L.seg[segid];
    const bool hl = x > 0, ht = y > 0;
    const uint8_t* yt = ytop + 16 * x;
    const uint8_t* uvt = uvtop + 16 * x;
    MBCtx ctx;
    nz_flags(nzw[x], nzw[x - 1], left_dc, ctx);

    // ---- predictions (quant_enc.c:469-479)
    {
      const int dcy = dc_value(yl, yt, hl, ht, 16, 5);
      for (int k = lane; k < 1024; k += 64) {
        const int m = k >> 8, p = k & 255;
        L.p16[m][p] = pred_sample(m, 16, p & 15, p >> 4, yl, yt, hl, ht, dcy);
      }
      const int dcu = dc_value(ul, uvt, hl, ht, 8, 4);
      const int dcv = dc_value(vl, uvt + 8, hl, ht, 8, 4);
      for (int k = lane; k < 512; k += 64) {
        const int m = k >> 7, p = k & 127, px = p & 15, py = p >> 4, c = px >> 3;
        L.puv[m][p] = pred_sample(m, 8, px & 7, py, c ? vl : ul, uvt + 8 * c, hl, ht, c ? dcv : dcu);
      }
    }
    wsync();

    K3_STAMP(0);
    int is_i16 = 1, bu = 0, best16 = 0;
    uint32_t rd_nz = 0;
    score_t rdH = 0;
    if constexpr (NONE) {
      // ---- RefineUsingDistortion (quant_enc.c:1248-1350): modes by
      // prediction SSE + fixed mode costs, then the chosen modes' reconstruction
      const uint8_t am = a.amode[(size_t)f * nmb + mb];
      int try_both = P->method >= 2;
      const int refine_uv = P->method >= 1;
      const score_t bit_limit = try_both ? (score_t)P->mb_header_limit : MAX_COST;
      score_t best_score = MAX_COST;
      is_i16 = try_both || !(am & 2);
      if (is_i16) {
        int best_mode = -1;
        for (int mm = 0; mm < 4; ++mm) {
          int sq = 0;
          for (int k = lane; k < 256; k += 64) {
            const int d = L.yin[(k >> 4) * BPS + (k & 15)] - L.p16[mm][k];
            sq += d * d;
          }
          for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
          const score_t sc = (score_t)sq * 256 + kVP8ModeCostI16[mm] * 106;
          if (mm > 0 && kVP8ModeCostI16[mm] > bit_limit) continue;
          if (sc < best_score) { best_mode = mm; best_score = sc; }
        }
        if (x == 0 || y == 0) {   // IsFlatSource16: avoid a border checkerboard (bug #432)
          int same = 1;
          const int v0 = L.yin[0];
          for (int k = lane; k < 256; k += 64) same &= (L.yin[(k >> 4) * BPS + (k & 15)] == v0);
          if (__all(same)) { best_mode = (x == 0) ? 0 : 2; try_both = 0; }
        }
        best16 = best_mode;
        if (lane < 16) L.modes[lane] = best16;
        wsync();
      }
      if (try_both || !is_i16) {
        is_i16 = 0;
        const I4Result r4 = run_i4<false>(L, S, ctx, lane, x, mbw, predtop, yl, yt, 2, best_score,
                                          bit_limit > 0x7fffffff ? 0x7fffffff : (int)bit_limit);
        if (r4.ok) {
          rd_nz = r4.nz;
          for (int k = lane; k < 256; k += 64) {
            L.yout[(k >> 4) * BPS + (k & 15)] = L.acc_out[k];
            (&L.fin_ac[0][0])[k] = (&L.acc_ac[0][0])[k];
          }
        } else {
          is_i16 = 1;
          if (lane < 16) L.modes[lane] = best16;
        }
        wsync();
      }
      if (is_i16) {   // ReconstructIntra16 of the chosen mode
        eval_i16<false>(L, S, ctx, lane);
        for (int k = lane; k < 256; k += 64) {
          L.yout[(k >> 4) * BPS + (k & 15)] = L.rec16[best16][k];
          (&L.fin_ac[0][0])[k] = (&L.lv16[best16][0][0])[k];
        }
        if (lane < 16) L.fin_dc[lane] = L.lvdc[best16][lane];
        rd_nz = (uint32_t)L.mres[best16][3];
      }
      wsync();
      if (refine_uv) {
        score_t best_uv = MAX_COST;
        for (int mm = 0; mm < 4; ++mm) {
          int sq = 0;
          for (int k = lane; k < 128; k += 64) {
            const int d = L.yin[(k >> 4) * BPS + 16 + (k & 15)] - L.puv[mm][k];
            sq += d * d;
          }
          for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
          const score_t sc = (score_t)sq * 256 + kVP8ModeCostUV[mm] * 120;
          if (sc < best_uv) { bu = mm; best_uv = sc; }
        }
      } else {
        bu = (am & 1) | ((am >> 1) & 2);   // method 0 keeps the preset UV mode (bits 0, 2)
      }
      // ReconstructUV: the DC error diffusion reads errors that RD_OPT_NONE
      // never stores (StoreDiffusionErrors is PickBestUV's), i.e. zeros
      eval_uv(L, S, ctx, lane, x, topderr, use_derr);
      for (int k = lane; k < 128; k += 64) {
        L.yout[(k >> 4) * BPS + 16 + (k & 15)] = L.recuv[bu][k];
        (&L.fin_uv[0][0])[k] = (&L.lvuv[bu][0][0])[k];
      }
      rd_nz |= (uint32_t)L.mres[bu][3] << 16;
      wsync();
    } else {
      score_t rd_score = 0;
      // ---- Intra16 (quant_enc.c:1002-1058)
      const bool trellis_all = rd_opt >= 3;
      if (trellis_all) eval_i16<true>(L, S, ctx, lane);
      else eval_i16<false>(L, S, ctx, lane);
      score_t best16_score = 0;
      uint32_t nz16 = 0;
      score_t D16 = 0, SD16 = 0, H16 = 0, R16 = 0;
      {
        int same = 1;
        const int v0 = L.yin[0];
        for (int k = lane; k < 256; k += 64) same &= (L.yin[(k >> 4) * BPS + (k & 15)] == v0);
        int flat = __all(same);
        for (int mm = 0; mm < 4; ++mm) {
          score_t Dm = L.mres[mm][0];
          score_t SDm = S.tlambda ? (score_t)((S.tlambda * L.mres[mm][1] + 128) >> 8) : 0;
          const score_t Hm = kVP8ModeCostI16[mm];
          const score_t Rm = L.mres[mm][2];
          if (flat) {
            flat = (L.mres[mm][3] & 0xffff) == 0;
            if (flat) { Dm *= 2; SDm *= 2; }
          }
          const score_t sc = (Rm + Hm) * S.lambda_i16 + 256 * (Dm + SDm);
          if (mm == 0 || sc < best16_score) {
            best16_score = sc; best16 = mm;
            D16 = Dm; SD16 = SDm; H16 = Hm; R16 = Rm;
            nz16 = (uint32_t)L.mres[mm][3];
          }
        }
      }
      // commit I16 as current best
      for (int k = lane; k < 256; k += 64) L.yout[(k >> 4) * BPS + (k & 15)] = L.rec16[best16][k];
      for (int k = lane; k < 256; k += 64) (&L.fin_ac[0][0])[k] = (&L.lv16[best16][0][0])[k];
      if (lane < 16) { L.fin_dc[lane] = L.lvdc[best16][lane]; L.modes[lane] = best16; }
      rd_score = (R16 + H16) * S.lambda_mode + 256 * (D16 + SD16);
      rdH = H16;
      rd_nz = nz16;
      is_i16 = 1;
      if ((rd_nz & 0x100ffff) == 0x1000000 && D16 > S.min_disto) {
        int mv = iabs_(L.lvdc[best16][1]);
        mv = max(mv, iabs_(L.lvdc[best16][2]));
        mv = max(mv, iabs_(L.lvdc[best16][4]));
        if (lane == 0 && mv > L.max_edge[segid]) L.max_edge[segid] = mv;
      }
      wsync();

      K3_STAMP(1);
      // ---- Intra4 (quant_enc.c:1072-1165)
      if (max_i4_bits > 0) {
        I4Result r4 = trellis_all ? run_i4<true>(L, S, ctx, lane, x, mbw, predtop, yl, yt, true,
                                                 rd_score, max_i4_bits)
                                  : run_i4<false>(L, S, ctx, lane, x, mbw, predtop, yl, yt, true,
                                                  rd_score, max_i4_bits);
        if (r4.ok) {
          is_i16 = 0;
          rdH = r4.H;
          rd_score = r4.score;
          rd_nz = r4.nz;
          for (int k = lane; k < 256; k += 64) {
            L.yout[(k >> 4) * BPS + (k & 15)] = L.acc_out[k];
            (&L.fin_ac[0][0])[k] = (&L.acc_ac[0][0])[k];
          }
        } else {
          if (lane < 16) L.modes[lane] = best16;   // the aborted search wrote some
        }
        wsync();
      }

      K3_STAMP(2);
      // ---- UV (quant_enc.c:1169-1217)
      {
        eval_uv(L, S, ctx, lane, x, topderr, use_derr);
        score_t bsc = 0, bH = 0;
        for (int mm = 0; mm < 4; ++mm) {
          const score_t Dm = L.mres[mm][0], Hm = kVP8ModeCostUV[mm];
          score_t Rm = L.mres[mm][1];
          if (mm > 0 && L.mres[mm][2] <= 2) Rm += 140 * 8;
          const score_t sc = (Rm + Hm) * S.lambda_uv + 256 * Dm;
          if (mm == 0 || sc < bsc) { bsc = sc; bu = mm; bH = Hm; }
        }
        rdH += bH;
        rd_score += bsc;
        rd_nz |= (uint32_t)L.mres[bu][3] << 16;
        for (int k = lane; k < 128; k += 64) {
          L.yout[(k >> 4) * BPS + 16 + (k & 15)] = L.recuv[bu][k];
          (&L.fin_uv[0][0])[k] = (&L.lvuv[bu][0][0])[k];
        }
        if (use_derr && lane < 2) {   // StoreDiffusionErrors (quant_enc.c:909-920)
          const int cch = lane;
          int8_t* top = topderr + 4 * x + 2 * cch;
          int8_t* left = L.lderr[cch];
          const int8_t* e = L.uvderr[bu][cch];
          left[0] = e[0];
          left[1] = (int8_t)(3 * e[2] >> 2);
          top[0] = e[1];
          top[1] = (int8_t)(e[2] - left[1]);
        }
        wsync();
      }

      // ---- m5: final re-quantisation of the chosen modes with trellis
      // (SimpleQuantize, quant_enc.c:1222-1245; RD_OPT_TRELLIS, :1384-1387)
      if (rd_opt == 2) {
        uint32_t nzq = 0;
        if (is_i16) {
          eval_i16<true>(L, S, ctx, lane);
          for (int k = lane; k < 256; k += 64) {
            L.yout[(k >> 4) * BPS + (k & 15)] = L.rec16[best16][k];
            (&L.fin_ac[0][0])[k] = (&L.lv16[best16][0][0])[k];
          }
          if (lane < 16) L.fin_dc[lane] = L.lvdc[best16][lane];
          nzq = (uint32_t)L.mres[best16][3];
        } else {
          I4Result r4 = run_i4<true>(L, S, ctx, lane, x, mbw, predtop, yl, yt, false, 0, 0);
          for (int k = lane; k < 256; k += 64) {
            L.yout[(k >> 4) * BPS + (k & 15)] = L.acc_out[k];
            (&L.fin_ac[0][0])[k] = (&L.acc_ac[0][0])[k];
          }
          nzq = r4.nz;
        }
        wsync();
        eval_uv(L, S, ctx, lane, x, topderr, use_derr);   // derr state already updated
        for (int k = lane; k < 128; k += 64) {
          L.yout[(k >> 4) * BPS + 16 + (k & 15)] = L.recuv[bu][k];
          (&L.fin_uv[0][0])[k] = (&L.lvuv[bu][0][0])[k];
        }
        rd_nz = nzq | ((uint32_t)L.mres[bu][3] << 16);
        wsync();
      }
      (void)rd_score;
    }
    K3_STAMP(3);
    {

      // ---- per-MB info + stats side info
      const int skip = rd_nz == 0;
      if (lane == 0) {
        uint8_t* info = mbinfo + (size_t)mb * VP8G_MBINFO_BYTES;
        info[0] = is_i16; info[1] = bu; info[2] = segid; info[3] = skip;
        if (is_i16) ++nb_i16; else ++nb_i4;
        if (skip) ++nb_skip;
        if (NONE && skip && mb < P->nb_stat) ++nb_skip_stat;
        if (NONE) a.mboff[(size_t)f * nmb + mb] = ntok;
      }
      if (NONE && P->recon_addr != 0) {   // autofilter input (filter_enc.c:179)
        for (int k = lane; k < 128; k += 64)
          reinterpret_cast<uint32_t*>(P->recon_addr + ((size_t)mb << 9))[k] =
              reinterpret_cast<const uint32_t*>(L.yout)[k];
        size_p0 += rdH;
      }
      if (lane < 16) mbinfo[(size_t)mb * VP8G_MBINFO_BYTES + 4 + lane] = L.modes[lane];
    }
    // SSE for WebPAuxStats (frame_enc.c:480-489)
    {
      int sy = 0, su = 0, sv = 0;
      for (int k = lane; k < 256; k += 64) {
        const int o = (k >> 4) * BPS + (k & 15);
        const int dd = L.yin[o] - L.yout[o];
        sy += dd * dd;
      }
      {
        const int o = (lane >> 3) * BPS + 16 + (lane & 7);
        const int du = L.yin[o] - L.yout[o], dv = L.yin[o + 8] - L.yout[o + 8];
        su = du * du; sv = dv * dv;
      }
      for (int off = 32; off >= 1; off >>= 1) {
        sy += __shfl_xor(sy, off);
        su += __shfl_xor(su, off);
        sv += __shfl_xor(sv, off);
      }
      sse_acc[0] += sy; sse_acc[1] += su; sse_acc[2] += sv;
    }

    K3_STAMP(4);
    // ---- tokens + exact statistics (frame_enc.c:411-453, token_enc.c:113-193)
    {
      // per-block nz flags from final levels -> contexts
      const int first_blk = is_i16 ? 0 : 1;
      int my_ctx = 0, my_type = 0, my_first = 0;
      const int k = lane;                    // block index 0..24
      const bool active = k >= first_blk && k < 25;
      int nzk = 0;
      if (active) {
        const int16_t* lv = blk_levels(L, k);
        for (int i = 0; i < 16; ++i) nzk |= lv[i];
      }
      const uint64_t nzb = __ballot(active && nzk != 0);
      if (active) {
        if (k == 0) {
          my_type = 1; my_first = 0; my_ctx = ctx.top(8) + ctx.left(8);
        } else if (k <= 16) {
          const int b = k - 1, bx = b & 3, by = b >> 2;
          my_type = is_i16 ? 0 : 3; my_first = is_i16 ? 1 : 0;
          const int t = by == 0 ? ctx.top(bx) : (int)((nzb >> (k - 4)) & 1);
          const int l = bx == 0 ? ctx.left(by) : (int)((nzb >> (k - 1)) & 1);
          my_ctx = t + l;
        } else {
          const int b = k - 17, ch = b >> 2, k4 = b & 3, bx = k4 & 1, by = k4 >> 1;
          my_type = 2; my_first = 0;
          const int t = by == 0 ? ctx.top(4 + 2 * ch + bx) : (int)((nzb >> (k - 2)) & 1);
          const int l = bx == 0 ? ctx.left(4 + 2 * ch + by) : (int)((nzb >> (k - 1)) & 1);
          my_ctx = t + l;
        }
      }
      if (active) L.blkinfo[k] = my_type | (my_first << 4) | (my_ctx << 8);
      int nzdummy;
      const int mycount = active ? gen_tokens<0, K3Lds, NONE>(L, blk_levels(L, k), my_type,
                                                              my_first, my_ctx, nullptr, &nzdummy)
                                 : 0;
      // exclusive prefix sum over lanes
      int incl = mycount;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
      }
      const int total = __shfl(incl, 63);
      const int excl = incl - mycount;
      if (ntok + (uint32_t)total > a.tok_cap) tok_err = 1;
      if (!tok_err && active)
        gen_tokens<1, K3Lds, NONE>(L, blk_levels(L, k), my_type, my_first, my_ctx,
                                   tok_base + ntok + excl, &nzdummy);
      if (!tok_err) ntok += total;
      wsync();
      K3_STAMP(5);
      // fold deltas into the statistics; slots that cross the halving
      // threshold inside this MB are replayed in token order.
      int any_mark = 0;
      // RD_OPT_NONE: only StatLoop's MBs count (frame_enc.c:631-638)
      const bool stat_on = !NONE || mb < P->nb_stat;
      for (int s = lane; s < NSLOT; s += 64) {
        const uint32_t dlt = stat_on ? L.delta[s] : 0u;
        if (!stat_on) L.delta[s] = 0;
        if (dlt) {
          const uint32_t p = L.stats[s];
          if ((p >> 16) + (dlt >> 16) < 0xffffu) {
            L.stats[s] = p + dlt;
          } else {
            atomicOr(&L.mark[s >> 5], 1u << (s & 31));
            any_mark = 1;
          }
          L.delta[s] = 0;
        }
      }
      wsync();
      if (__any(any_mark)) {
        if (lane == 0) {
          for (int kk = first_blk; kk < 25; ++kk) {
            const int bi = L.blkinfo[kk];
            gen_tokens<2, K3Lds, NONE>(L, blk_levels(L, kk), bi & 15, (bi >> 4) & 15, bi >> 8,
                                       nullptr, &nzdummy);
          }
        }
        wsync();
        for (int kk = lane; kk < 33; kk += 64) L.mark[kk] = 0;
        wsync();
      }
      K3_STAMP(6);
      // update nz context (iterator_enc.c:267-283) and the left DC flag
      {
        int tn[9], ln[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) { tn[i] = ctx.top(i); ln[i] = ctx.left(i); }
        if (is_i16) { tn[8] = ln[8] = (int)(nzb & 1); }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tn[i] = (int)((nzb >> (1 + 12 + i)) & 1);      // block (i, 3)
          ln[i] = (int)((nzb >> (1 + 4 * i + 3)) & 1);   // block (3, i)
        }
#pragma unroll
        for (int ch = 0; ch < 2; ++ch)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            tn[4 + 2 * ch + i] = (int)((nzb >> (17 + 4 * ch + 2 + i)) & 1);
            ln[4 + 2 * ch + i] = (int)((nzb >> (17 + 4 * ch + 2 * i + 1)) & 1);
          }
        uint32_t word = 0;
        word |= (tn[0] << 12) | (tn[1] << 13) | (tn[2] << 14) | (tn[3] << 15) |
                (tn[4] << 18) | (tn[5] << 19) | (tn[6] << 22) | (tn[7] << 23) | (tn[8] << 24);
        word |= (ln[0] << 3) | (ln[1] << 7) | (ln[2] << 11) | (ln[4] << 17) | (ln[6] << 21);
        left_dc = ln[8];
        wsync();
        if (lane == 0) nzw[x] = word;
      }
    }

    // ---- boundary save (iterator_enc.c:290-313) + mode context
    wsync();
    if (x < mbw - 1) {
      if (lane < 16) yl[lane] = L.yout[15 + lane * BPS];
      if (lane < 8) { ul[lane] = L.yout[16 + 7 + lane * BPS]; vl[lane] = L.yout[24 + 7 + lane * BPS]; }
      if (lane == 0) { yl[-1] = yt[15]; ul[-1] = uvt[7]; vl[-1] = uvt[15]; }
    }
    wsync();
    if (y < mbh - 1) {
      if (lane < 16) {
        ytop[16 * x + lane] = L.yout[15 * BPS + lane];
        uvtop[16 * x + lane] = L.yout[7 * BPS + 16 + lane];
      }
    }
    if (lane < 4) {
      predtop[4 * x + lane] = L.modes[12 + lane];
      L.predleft[lane] = L.modes[4 * lane + 3];
    }
    wsync();
    K3_STAMP(7);
  }

  // ---- frame epilogue: final probabilities and side results
  vp8g_frame_result* R = a.results + f;
  int use_skip = 0, skip_proba = 255;
  if constexpr (NONE) {
    wsync();
    for (int s = lane; s < NSLOT; s += 64) rstats[s] = L.stats[s];
    // StatLoop gives up before FinalizeSkipProba / FinalizeTokenProbas when
    // its header estimate is 0 (frame_enc.c:645-646): default probabilities
    if (P->none_finalize) {
      finalize_probas(L, lane);
      const int nbs = __shfl(nb_skip_stat, 0);   // counted by lane 0 only
      skip_proba = (int)((uint64_t)(nmb - nbs) * 255 / nmb);   // CalcSkipProba
      use_skip = skip_proba < 250;
    }
    if (use_skip && !tok_err) {
      // VP8EncLoop codes no residuals for skipped MBs: drop their tokens
      // (forward compaction, each 64-token chunk read before it is written)
      uint32_t dst = 0;
      for (int m = 0; m < nmb; ++m) {
        const uint32_t b0 = a.mboff[(size_t)f * nmb + m];
        const uint32_t b1 = m + 1 < nmb ? a.mboff[(size_t)f * nmb + m + 1] : ntok;
        if (mbinfo[(size_t)m * VP8G_MBINFO_BYTES + 3]) continue;
        if (dst != b0)
          for (uint32_t i = 0; i < b1 - b0; i += 64) {
            const bool in = i + lane < b1 - b0;
            const uint16_t t = in ? tok_base[b0 + i + lane] : 0;
            __builtin_amdgcn_wave_barrier();
            if (in) tok_base[dst + i + lane] = t;
            __builtin_amdgcn_wave_barrier();
          }
        dst += b1 - b0;
      }
      ntok = dst;
    }
  } else {
    finalize_probas(L, lane);
  }
  for (int s = lane; s < NSLOT; s += 64) R->probas[s] = L.coeffs[s];
  if (lane == 0) {
    R->use_skip = (int16_t)use_skip;
    R->skip_proba = (int16_t)skip_proba;
    R->ntokens = ntok;
    R->error = tok_err;
    for (int s = 0; s < 4; ++s) R->max_edge[s] = L.max_edge[s];
    R->size_p0 = size_p0;
    R->sse[0] = sse_acc[0]; R->sse[1] = sse_acc[1]; R->sse[2] = sse_acc[2];
    R->block_count[0] = nb_i4; R->block_count[1] = nb_i16; R->block_count[2] = nb_skip;
    for (int i = 0; i < 8; ++i) R->stamps[i] = stamps[i];
  }
}

// ---------------------------------------------------------------------------
// syn-v1 generator for benchmarks: counter-based, so any
// frame is produced directly in HBM.

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_synth(uint8_t* rgba, size_t fstride, int w, int h, int f0, int seed) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  const int f = f0 + blockIdx.z;
  if (x >= w) return;
  const uint64_t hh = splitmix64(((uint64_t)seed << 48) ^ ((uint64_t)f << 32) ^
                                 ((uint64_t)y << 16) ^ (uint64_t)x);
  const int region = ((x >> 5) ^ (y >> 5) ^ f) & 3;
  const int n = (int)(hh & 31) - 16;
  const int gx = w > 1 ? x * 255 / (w - 1) : 0, gy = h > 1 ? y * 255 / (h - 1) : 0;
  int r, g, b;
  if (region == 0) { r = g = b = (f * 37 + 64) & 255; }
  else if (region == 1) { r = gx + n; g = gy + n; b = (x ^ y) & 255; }
  else if (region == 2) { r = (hh >> 8) & 255; g = (hh >> 16) & 255; b = (hh >> 24) & 255; }
  else { r = g = b = (((x + y + f) >> 2) & 1) ? 235 : 20; }
  uint8_t* p = rgba + blockIdx.z * fstride + ((size_t)y * w + x) * 4;
  p[0] = min(max(r, 0), 255); p[1] = min(max(g, 0), 255); p[2] = min(max(b, 0), 255); p[3] = 255;
}

// ---------------------------------------------------------------------------
// launchers


// ---------------------------------------------------------------------------
// K3N: the methods 0-2 encoder (RD_OPT_NONE, VP8EncLoop) with NW MB workers
// of one wavefront per frame. The decisions depend only on the reconstructed
// neighbours (no rate, no statistics feedback), so rows are dealt to the
// waves round-robin and run as a wavefront (row y starts MB x once row y-1
// has finished x+1: top-right dependency, iterator_enc.c:290-313); boundary
// rows live in shared LDS like K3's. Each MB's tokens go to its own slot;
// after the loop the workgroup replays StatLoop's statistics in raster order
// (exact saturation), finalises, and compacts the slots into the frame's
// stream (dropping skipped MBs when the skip flag pays).
struct K3NShared {
  int32_t nb[4];               // i4, i16, skip, skip among the statistics MBs
  unsigned long long sse[3];
  int32_t any_mark;
  int32_t use_skip, skip_proba;
  uint32_t ntok;
};

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_encode_none(K3ArgsW1 a) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, tid = threadIdx.x;
  K3Lds& L = reinterpret_cast<K3Lds*>(smem)[wv];
  K3Lds& L0 = reinterpret_cast<K3Lds*>(smem)[0];
  const int mbw = a.mbw, mbh = a.mbh, nmb = mbw * mbh;
  K3NShared& G = *reinterpret_cast<K3NShared*>(smem + NW * sizeof(K3Lds));
  uint8_t* ytop = smem + NW * sizeof(K3Lds) + sizeof(K3NShared);   // 16*mbw + 16
  uint8_t* uvtop = ytop + 16 * mbw + 16;                             // 16*mbw
  uint32_t* nzw = reinterpret_cast<uint32_t*>(uvtop + 16 * mbw) + 1; // [-1..mbw-1]
  uint8_t* predtop = reinterpret_cast<uint8_t*>(nzw + mbw);         // 4*mbw
  int8_t* topderr = reinterpret_cast<int8_t*>(predtop + 4 * mbw);   // 4*mbw, stays 0
  int32_t* rowdone = reinterpret_cast<int32_t*>(topderr + 4 * mbw + 4 - ((4 * mbw) & 3));

  const int f = blockIdx.x;
  const int w = a.w, h = a.h;
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  const uint8_t* Yp = a.yuv + f * a.yfb;
  const uint8_t* Up = Yp + (size_t)w * h;
  const uint8_t* Vp = Up + (size_t)uvw * uvh;
  const vp8g_frame_params* P = a.params + f;
  const uint8_t* segmap = a.segmap + (size_t)f * nmb;
  uint16_t* tok_base = a.tokens + f * a.tok_cap;
  uint8_t* mbinfo = a.mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES;
  uint32_t* mbcnt = a.mboff + (size_t)f * nmb;   // tokens of each MB's slot
  if (P->pass_mode == 2) return;
  if (P->pass_mode != 0 && P->pass_mode != 3) {
    if (tid == 0) a.results[f].error = 3;
    return;
  }
  uint32_t* rstats =
      reinterpret_cast<uint32_t*>(a.rerun + (size_t)f * VP8G_RERUN_STATE_BYTES + VP8G_STATE_STATS);

  // ---- frame init
  for (int k = lane; k < 1000; k += 64) L.mcost4[k] = (&kVP8ModeCostI4[0][0][0])[k];
  for (int k = lane; k < 160; k += 64) L.p4[k] = (&kP4[0][0])[k];
  for (int k = lane; k < 256; k += 64) L.ecost[k] = kVP8EntropyCost[k];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(P->seg);
    uint32_t* dst = reinterpret_cast<uint32_t*>(L.seg);
    for (int k = lane; k < (int)(sizeof(L.seg) / 4); k += 64) dst[k] = src[k];
  }
  for (int k = tid; k < 16 * mbw + 16; k += NW * 64) ytop[k] = 127;
  for (int k = tid; k < 16 * mbw; k += NW * 64) uvtop[k] = 127;
  for (int k = tid - 1; k < mbw; k += NW * 64) nzw[k] = 0;
  for (int k = tid; k < 4 * mbw; k += NW * 64) { predtop[k] = 0; topderr[k] = 0; }
  for (int k = tid; k < mbh; k += NW * 64) rowdone[k] = 0;
  if (tid < 4) G.nb[tid] = 0;
  if (tid < 3) G.sse[tid] = 0;
  if (tid == 0) { G.any_mark = 0; G.ntok = 0; }
  __syncthreads();
  // the level-cost tables only feed rates RD_OPT_NONE never looks at

  const int use_derr = P->use_derr;
  uint8_t* yl = L.yl_mem + 1;
  uint8_t* ul = L.ul_mem + 1;
  uint8_t* vl = L.vl_mem + 1;

  for (int y = wv; y < mbh; y += NW) {
    if (lane < 16) yl[lane] = 129;   // InitLeft (iterator_enc.c:22-32)
    if (lane < 8) { ul[lane] = 129; vl[lane] = 129; }
    if (lane == 0) {
      yl[-1] = ul[-1] = vl[-1] = (y > 0) ? 129 : 127;
      L.lderr[0][0] = L.lderr[0][1] = L.lderr[1][0] = L.lderr[1][1] = 0;
    }
    if (lane < 4) L.predleft[lane] = 0;
    int left_dc = 0;
    wsync();
    for (int x = 0; x < mbw; ++x) {
      const int mb = y * mbw + x;
      if (y > 0) {   // row y-1 has finished MB x+1 (top-right samples)
        const int need = min(x + 2, mbw);
        if (lane == 0)
          while (__hip_atomic_load(&rowdone[y - 1], __ATOMIC_ACQUIRE,
                                   __HIP_MEMORY_SCOPE_WORKGROUP) < need)
            __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        wsync();
      }
      load_mb(Yp, Up, Vp, w, h, x, y, L.yin, lane, 64);
      wsync();
      const int segid = segmap[mb];
      const vp8g_seg& S = L.seg[segid];
      const bool hl = x > 0, ht = y > 0;
      const uint8_t* yt = ytop + 16 * x;
      const uint8_t* uvt = uvtop + 16 * x;
      MBCtx ctx;
      nz_flags(nzw[x], nzw[x - 1], left_dc, ctx);
      {   // predictions (quant_enc.c:469-479)
        const int dcy = dc_value(yl, yt, hl, ht, 16, 5);
        for (int k = lane; k < 1024; k += 64) {
          const int m = k >> 8, p = k & 255;
          L.p16[m][p] = pred_sample(m, 16, p & 15, p >> 4, yl, yt, hl, ht, dcy);
        }
        const int dcu = dc_value(ul, uvt, hl, ht, 8, 4);
        const int dcv = dc_value(vl, uvt + 8, hl, ht, 8, 4);
        for (int k = lane; k < 512; k += 64) {
          const int m = k >> 7, p = k & 127, px = p & 15, py = p >> 4, c = px >> 3;
          L.puv[m][p] = pred_sample(m, 8, px & 7, py, c ? vl : ul, uvt + 8 * c, hl, ht,
                                    c ? dcv : dcu);
        }
      }
      wsync();
      int is_i16 = 1, bu = 0, best16 = 0;
      uint32_t rd_nz = 0;
      {
      // ---- RefineUsingDistortion (quant_enc.c:1248-1350): modes by
      // prediction SSE + fixed mode costs, then the chosen modes' reconstruction
      const uint8_t am = a.amode[(size_t)f * nmb + mb];
      int try_both = P->method >= 2;
      const int refine_uv = P->method >= 1;
      const score_t bit_limit = try_both ? (score_t)P->mb_header_limit : MAX_COST;
      score_t best_score = MAX_COST;
      is_i16 = try_both || !(am & 2);
      if (is_i16) {
        int best_mode = -1;
        for (int mm = 0; mm < 4; ++mm) {
          int sq = 0;
          for (int k = lane; k < 256; k += 64) {
            const int d = L.yin[(k >> 4) * BPS + (k & 15)] - L.p16[mm][k];
            sq += d * d;
          }
          for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
          const score_t sc = (score_t)sq * 256 + kVP8ModeCostI16[mm] * 106;
          if (mm > 0 && kVP8ModeCostI16[mm] > bit_limit) continue;
          if (sc < best_score) { best_mode = mm; best_score = sc; }
        }
        if (x == 0 || y == 0) {   // IsFlatSource16: avoid a border checkerboard (bug #432)
          int same = 1;
          const int v0 = L.yin[0];
          for (int k = lane; k < 256; k += 64) same &= (L.yin[(k >> 4) * BPS + (k & 15)] == v0);
          if (__all(same)) { best_mode = (x == 0) ? 0 : 2; try_both = 0; }
        }
        best16 = best_mode;
        if (lane < 16) L.modes[lane] = best16;
        wsync();
      }
      if (try_both || !is_i16) {
        is_i16 = 0;
        const I4Result r4 = run_i4<false>(L, S, ctx, lane, x, mbw, predtop, yl, yt, 2, best_score,
                                          bit_limit > 0x7fffffff ? 0x7fffffff : (int)bit_limit);
        if (r4.ok) {
          rd_nz = r4.nz;
          for (int k = lane; k < 256; k += 64) {
            L.yout[(k >> 4) * BPS + (k & 15)] = L.acc_out[k];
            (&L.fin_ac[0][0])[k] = (&L.acc_ac[0][0])[k];
          }
        } else {
          is_i16 = 1;
          if (lane < 16) L.modes[lane] = best16;
        }
        wsync();
      }
      if (is_i16) {   // ReconstructIntra16 of the chosen mode
        eval_i16<false>(L, S, ctx, lane);
        for (int k = lane; k < 256; k += 64) {
          L.yout[(k >> 4) * BPS + (k & 15)] = L.rec16[best16][k];
          (&L.fin_ac[0][0])[k] = (&L.lv16[best16][0][0])[k];
        }
        if (lane < 16) L.fin_dc[lane] = L.lvdc[best16][lane];
        rd_nz = (uint32_t)L.mres[best16][3];
      }
      wsync();
      if (refine_uv) {
        score_t best_uv = MAX_COST;
        for (int mm = 0; mm < 4; ++mm) {
          int sq = 0;
          for (int k = lane; k < 128; k += 64) {
            const int d = L.yin[(k >> 4) * BPS + 16 + (k & 15)] - L.puv[mm][k];
            sq += d * d;
          }
          for (int off = 32; off >= 1; off >>= 1) sq += __shfl_xor(sq, off);
          const score_t sc = (score_t)sq * 256 + kVP8ModeCostUV[mm] * 120;
          if (sc < best_uv) { bu = mm; best_uv = sc; }
        }
      } else {
        bu = (am & 1) | ((am >> 1) & 2);   // method 0 keeps the preset UV mode (bits 0, 2)
      }
      // ReconstructUV: the DC error diffusion reads errors that RD_OPT_NONE
      // never stores (StoreDiffusionErrors is PickBestUV's), i.e. zeros
      eval_uv(L, S, ctx, lane, x, topderr, use_derr);
      for (int k = lane; k < 128; k += 64) {
        L.yout[(k >> 4) * BPS + 16 + (k & 15)] = L.recuv[bu][k];
        (&L.fin_uv[0][0])[k] = (&L.lvuv[bu][0][0])[k];
      }
      rd_nz |= (uint32_t)L.mres[bu][3] << 16;
      wsync();
      }
      // ---- per-MB info + side statistics
      const int skip = rd_nz == 0;
      if (lane == 0) {
        uint8_t* info = mbinfo + (size_t)mb * VP8G_MBINFO_BYTES;
        info[0] = is_i16; info[1] = bu; info[2] = segid; info[3] = skip;
        atomicAdd(&G.nb[is_i16 ? 1 : 0], 1);
        if (skip) atomicAdd(&G.nb[2], 1);
        if (skip && mb < P->nb_stat) atomicAdd(&G.nb[3], 1);
      }
      if (lane < 16) mbinfo[(size_t)mb * VP8G_MBINFO_BYTES + 4 + lane] = L.modes[lane];
      if (P->recon_addr != 0)   // autofilter input (filter_enc.c:179)
        for (int k = lane; k < 128; k += 64)
          reinterpret_cast<uint32_t*>(P->recon_addr + ((size_t)mb << 9))[k] =
              reinterpret_cast<const uint32_t*>(L.yout)[k];
      {   // SSE for WebPAuxStats (frame_enc.c:480-489)
        int sy = 0, su = 0, sv = 0;
        for (int k = lane; k < 256; k += 64) {
          const int o = (k >> 4) * BPS + (k & 15);
          const int dd = L.yin[o] - L.yout[o];
          sy += dd * dd;
        }
        {
          const int o = (lane >> 3) * BPS + 16 + (lane & 7);
          const int du = L.yin[o] - L.yout[o], dv = L.yin[o + 8] - L.yout[o + 8];
          su = du * du; sv = dv * dv;
        }
        for (int off = 32; off >= 1; off >>= 1) {
          sy += __shfl_xor(sy, off);
          su += __shfl_xor(su, off);
          sv += __shfl_xor(sv, off);
        }
        if (lane == 0) {
          atomicAdd(&G.sse[0], (unsigned long long)sy);
          atomicAdd(&G.sse[1], (unsigned long long)su);
          atomicAdd(&G.sse[2], (unsigned long long)sv);
        }
      }
      // ---- tokens (token_enc.c:113-193) into this MB's slot
      {
        const int first_blk = is_i16 ? 0 : 1;
        int my_ctx = 0, my_type = 0, my_first = 0;
        const int k = lane;   // block index 0..24
        const bool active = k >= first_blk && k < 25;
        int nzk = 0;
        if (active) {
          const int16_t* lv = blk_levels(L, k);
          for (int i = 0; i < 16; ++i) nzk |= lv[i];
        }
        const uint64_t nzb = __ballot(active && nzk != 0);
        if (active) {
          if (k == 0) {
            my_type = 1; my_first = 0; my_ctx = ctx.top(8) + ctx.left(8);
          } else if (k <= 16) {
            const int b = k - 1, bx = b & 3, by = b >> 2;
            my_type = is_i16 ? 0 : 3; my_first = is_i16 ? 1 : 0;
            const int t = by == 0 ? ctx.top(bx) : (int)((nzb >> (k - 4)) & 1);
            const int l = bx == 0 ? ctx.left(by) : (int)((nzb >> (k - 1)) & 1);
            my_ctx = t + l;
          } else {
            const int b = k - 17, ch = b >> 2, k4 = b & 3, bx = k4 & 1, by = k4 >> 1;
            my_type = 2; my_first = 0;
            const int t = by == 0 ? ctx.top(4 + 2 * ch + bx) : (int)((nzb >> (k - 2)) & 1);
            const int l = bx == 0 ? ctx.left(4 + 2 * ch + by) : (int)((nzb >> (k - 1)) & 1);
            my_ctx = t + l;
          }
        }
        int nzdummy;
        const int mycount = active ? gen_tokens<0, K3Lds, true>(L, blk_levels(L, k), my_type,
                                                                my_first, my_ctx, nullptr, &nzdummy)
                                   : 0;
        int incl = mycount;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int v = __shfl_up(incl, off);
          if (lane >= off) incl += v;
        }
        const int total = __shfl(incl, 63);
        const int excl = incl - mycount;
        uint16_t* slot = tok_base + (size_t)mb * VP8G_MAX_TOKENS_PER_MB;
        if (active)
          gen_tokens<1, K3Lds, true>(L, blk_levels(L, k), my_type, my_first, my_ctx, slot + excl,
                                     &nzdummy);
        if (lane == 0) mbcnt[mb] = (uint32_t)total;
        // nz contexts (iterator_enc.c:267-283) and the left DC flag
        int tn[9], ln[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) { tn[i] = ctx.top(i); ln[i] = ctx.left(i); }
        if (is_i16) { tn[8] = ln[8] = (int)(nzb & 1); }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tn[i] = (int)((nzb >> (1 + 12 + i)) & 1);
          ln[i] = (int)((nzb >> (1 + 4 * i + 3)) & 1);
        }
#pragma unroll
        for (int ch = 0; ch < 2; ++ch)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            tn[4 + 2 * ch + i] = (int)((nzb >> (17 + 4 * ch + 2 + i)) & 1);
            ln[4 + 2 * ch + i] = (int)((nzb >> (17 + 4 * ch + 2 * i + 1)) & 1);
          }
        uint32_t word = 0;
        word |= (tn[0] << 12) | (tn[1] << 13) | (tn[2] << 14) | (tn[3] << 15) |
                (tn[4] << 18) | (tn[5] << 19) | (tn[6] << 22) | (tn[7] << 23) | (tn[8] << 24);
        word |= (ln[0] << 3) | (ln[1] << 7) | (ln[2] << 11) | (ln[4] << 17) | (ln[6] << 21);
        left_dc = ln[8];
        wsync();
        if (lane == 0) nzw[x] = word;
      }
      // ---- boundary save (iterator_enc.c:290-313) + mode context
      wsync();
      if (x < mbw - 1) {
        if (lane < 16) yl[lane] = L.yout[15 + lane * BPS];
        if (lane < 8) { ul[lane] = L.yout[16 + 7 + lane * BPS]; vl[lane] = L.yout[24 + 7 + lane * BPS]; }
        if (lane == 0) { yl[-1] = yt[15]; ul[-1] = uvt[7]; vl[-1] = uvt[15]; }
      }
      wsync();
      if (y < mbh - 1 && lane < 16) {
        ytop[16 * x + lane] = L.yout[15 * BPS + lane];
        uvtop[16 * x + lane] = L.yout[7 * BPS + 16 + lane];
      }
      if (lane < 4) {
        predtop[4 * x + lane] = L.modes[12 + lane];
        L.predleft[lane] = L.modes[4 * lane + 3];
      }
      wsync();
      if (lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __hip_atomic_store(&rowdone[y], x + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
  }
  __threadfence_block();
  __syncthreads();

  // ---- StatLoop's statistics: the probe MBs' tokens in raster order, per
  // slot delta + exact in-order replay of the slots reaching the halving
  // point (VP8RecordStats, cost_enc.h:45-56). RecordCoeffs puts every
  // dynamic token's statistic in its probability slot (gen_tokens RC).
  for (int s = tid; s < NSLOT; s += NW * 64) {
    L0.stats[s] = P->pass_mode == 3 ? rstats[s] : 0u;
    L0.delta[s] = 0;
  }
  for (int k = tid; k < 33; k += NW * 64) L0.mark[k] = 0;
  __syncthreads();
  const int nb_stat = min(P->nb_stat, nmb);
  for (int m = 0; m < nb_stat; ++m) {
    const uint16_t* T = tok_base + (size_t)m * VP8G_MAX_TOKENS_PER_MB;
    const uint32_t n = mbcnt[m];
    for (uint32_t i = tid; i < n; i += NW * 64) {
      const uint32_t tk = T[i];
      if (!(tk & 0x4000u)) atomicAdd(&L0.delta[tk & 0x3fffu], 0x10000u + (tk >> 15));
    }
    __syncthreads();
    for (int s = tid; s < NSLOT; s += NW * 64) {
      const uint32_t d = L0.delta[s];
      if (d) {
        const uint32_t p = L0.stats[s];
        if ((p >> 16) + (d >> 16) < 0xffffu) {
          L0.stats[s] = p + d;
        } else {
          atomicOr(&L0.mark[s >> 5], 1u << (s & 31));
          G.any_mark = 1;
        }
        L0.delta[s] = 0;
      }
    }
    __syncthreads();
    if (G.any_mark) {
      if (tid == 0) {
        for (uint32_t i = 0; i < n; ++i) {
          const uint32_t tk = T[i];
          const uint32_t sl = tk & 0x3fffu;
          if (!(tk & 0x4000u) && (L0.mark[sl >> 5] & (1u << (sl & 31))))
            record_stat(&L0.stats[sl], (int)(tk >> 15));
        }
      }
      __syncthreads();
      for (int k = tid; k < 33; k += NW * 64) L0.mark[k] = 0;
      if (tid == 0) G.any_mark = 0;
      __syncthreads();
    }
  }
  for (int s = tid; s < NSLOT; s += NW * 64) rstats[s] = L0.stats[s];
  if (wv == 0) {
    for (int s = lane; s < NSLOT; s += 64) L0.coeffs[s] = (&kVP8CoeffProba0[0][0][0][0])[s];
    for (int k = lane; k < 256; k += 64) L0.ecost[k] = kVP8EntropyCost[k];
    wsync();
    int use_skip = 0, skip_proba = 255;
    // StatLoop gives up before FinalizeSkipProba / FinalizeTokenProbas when
    // its header estimate is 0 (frame_enc.c:645-646): default probabilities
    if (P->none_finalize) {
      finalize_probas(L0, lane);
      const int nsk = P->skip_count >= 0 ? P->skip_count : G.nb[3];
      skip_proba = (int)((uint64_t)(nmb - nsk) * 255 / nmb);   // CalcSkipProba
      use_skip = skip_proba < 250;
    }
    if (lane == 0) { G.use_skip = use_skip; G.skip_proba = skip_proba; }
  }
  __syncthreads();
  // ---- the frame's token stream in raster order; VP8EncLoop codes no
  // residuals for skipped MBs when the skip flag is used
  uint32_t dst = 0;
  for (int m = 0; m < nmb; ++m) {
    if (G.use_skip && mbinfo[(size_t)m * VP8G_MBINFO_BYTES + 3]) continue;
    const uint32_t n = mbcnt[m];
    const uint16_t* src = tok_base + (size_t)m * VP8G_MAX_TOKENS_PER_MB;
    if ((size_t)dst != (size_t)m * VP8G_MAX_TOKENS_PER_MB) {
      for (uint32_t i = 0; i < n; i += NW * 64) {
        const bool in = i + tid < n;
        const uint16_t t = in ? src[i + tid] : 0;
        __syncthreads();
        if (in) tok_base[dst + i + tid] = t;
        __threadfence_block();
        __syncthreads();
      }
    }
    dst += n;
  }
  vp8g_frame_result* R = a.results + f;
  for (int s = tid; s < NSLOT; s += NW * 64) R->probas[s] = L0.coeffs[s];
  if (tid == 0) {
    R->use_skip = (int16_t)G.use_skip;
    R->skip_proba = (int16_t)G.skip_proba;
    R->ntokens = dst;
    R->error = 0;
    for (int s = 0; s < 4; ++s) R->max_edge[s] = 0;   // StoreMaxDelta is PickBestIntra16's
    R->size_p0 = 0;                                   // RD_OPT_NONE has no header estimate
    R->distortion = 0;
    R->sse[0] = G.sse[0]; R->sse[1] = G.sse[1]; R->sse[2] = G.sse[2];
    R->block_count[0] = G.nb[0]; R->block_count[1] = G.nb[1]; R->block_count[2] = G.nb[2];
    for (int i = 0; i < 8; ++i) R->stamps[i] = 0;
  }
}

static size_t k3_lds_bytes(int mbw) {
  return sizeof(K3Lds) + (16 * mbw + 16) + 16 * mbw + 4 * (mbw + 1) + 4 * mbw + 4 * mbw + 16;
}

static int g_sync_mode = -1;
extern "C" int vp8g_launch_check(const char* what);
static int launch_check(const char* what) { return vp8g_launch_check(what); }
extern "C" int vp8g_launch_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    if (g_sync_mode < 0) {
      const char* v = getenv("WEBP_AMD_SYNC");
      g_sync_mode = (v && v[0] == '1') ? 1 : 0;
    }
    if (g_sync_mode) e = hipDeviceSynchronize();
  }
  if (e != hipSuccess) {
    vp8g_set_error(what, hipGetErrorString(e));
    return 0;
  }
  return 1;
}

// Alpha level reduction (alpha_quality < 100; QuantizeLevels,
// src/utils/quant_levels_utils.c:31-137): per-frame 256-bin histogram of the
// alpha plane here, the k-means over the 256 symbols on the host (doubles,
// the reference's own order), then the symbol map applied here.
__global__ __launch_bounds__(256) void k_alpha_hist(const uint8_t* __restrict__ aplane,
                                                    size_t plane, const uint32_t* aflags,
                                                    uint32_t* __restrict__ hist) {
  const int f = blockIdx.y;
  if (!aflags[f]) return;
  __shared__ uint32_t hs[256];
  hs[threadIdx.x] = 0;
  __syncthreads();
  const uint8_t* a = aplane + (size_t)f * plane;
  const size_t n16 = plane >> 4;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const uint4 v = reinterpret_cast<const uint4*>(a)[i];
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) atomicAdd(&hs[(w4[k >> 2] >> (8 * (k & 3))) & 255], 1u);
  }
  if (blockIdx.x == 0)
    for (size_t i = (n16 << 4) + threadIdx.x; i < plane; i += 256) atomicAdd(&hs[a[i]], 1u);
  __syncthreads();
  if (hs[threadIdx.x]) atomicAdd(&hist[(size_t)f * 256 + threadIdx.x], hs[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_alpha_remap(uint8_t* __restrict__ aplane, size_t plane,
                                                     const uint32_t* aflags,
                                                     const uint8_t* __restrict__ maps) {
  const int f = blockIdx.y;
  if (!aflags[f]) return;
  __shared__ uint8_t m[256];
  m[threadIdx.x] = maps[(size_t)f * 256 + threadIdx.x];
  __syncthreads();
  uint8_t* a = aplane + (size_t)f * plane;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < plane; i += (size_t)gridDim.x * 256)
    a[i] = m[a[i]];
}

extern "C" {

int vp8g_launch_import(const uint8_t* rgba, size_t fstride, int rstride, int w, int h, int n,
                       uint8_t* yuv, size_t yfb, uint32_t* aflags, uint8_t* aplane,
                       const uint16_t g2l[256], const int32_t l2g[33], const uint16_t* rnd_y,
                       const uint32_t* rnd_uv, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  dim3 grid((uvw + 255) / 256, uvh, n);
  hipLaunchKernelGGL(k_import, grid, dim3(256), 0, st, rgba, fstride, rstride, w, h, yuv, yfb,
                     aflags, aplane, g2l, l2g, rnd_y, rnd_uv);
  return launch_check("k_import");
}

int vp8g_launch_extract_alpha(const uint8_t* rgba, size_t fstride, int rstride, int w, int h,
                              int n, const uint32_t* aflags, uint8_t* aplane, void* stream) {
  dim3 grid((w + 255) / 256, h, n);
  hipLaunchKernelGGL(k_extract_alpha, grid, dim3(256), 0, (hipStream_t)stream, rgba, fstride,
                     rstride, w, h, aflags, aplane);
  return launch_check("k_extract_alpha");
}

int vp8g_launch_cleanup_alpha(uint8_t* yuv, size_t yfb, const uint8_t* aplane,
                              const uint32_t* aflags, int w, int h, int n, void* stream) {
  dim3 grid((h + 7) / 8, n);
  hipLaunchKernelGGL(k_cleanup_alpha, grid, dim3(256), 0, (hipStream_t)stream, yuv, yfb, aplane,
                     aflags, w, h);
  return launch_check("k_cleanup_alpha");
}

int vp8g_launch_alpha_hist(const uint8_t* aplane, size_t plane, const uint32_t* aflags, int n,
                           uint32_t* hist, void* stream) {
  if (hipMemsetAsync(hist, 0, (size_t)n * 256 * sizeof(uint32_t), (hipStream_t)stream) !=
      hipSuccess)
    return launch_check("k_alpha_hist memset");
  dim3 grid((unsigned)min((size_t)64, (plane + 4095) / 4096 + 1), n);
  hipLaunchKernelGGL(k_alpha_hist, grid, dim3(256), 0, (hipStream_t)stream, aplane, plane, aflags,
                     hist);
  return launch_check("k_alpha_hist");
}

int vp8g_launch_alpha_remap(uint8_t* aplane, size_t plane, const uint32_t* aflags, int n,
                            const uint8_t* maps, void* stream) {
  dim3 grid((unsigned)min((size_t)256, (plane + 255) / 256), n);
  hipLaunchKernelGGL(k_alpha_remap, grid, dim3(256), 0, (hipStream_t)stream, aplane, plane, aflags,
                     maps);
  return launch_check("k_alpha_remap");
}

int vp8g_launch_analysis(const uint8_t* yuv, size_t yfb, int w, int h, int n, uint8_t* mb_alpha,
                         uint16_t* mb_uva, int fast_q, uint8_t* mb_amode, void* stream) {
  const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4, nmb = mbw * mbh;
  dim3 grid((mbw + K2_STRIP - 1) / K2_STRIP, mbh, n);
  hipLaunchKernelGGL(k_analyze, grid, dim3(256), 0, (hipStream_t)stream, yuv, yfb, w, h, nmb,
                     mb_alpha, mb_uva, fast_q, mb_amode);
  return launch_check("k_analyze");
}

#ifdef WEBP_AMD_DIAG   // the single-wavefront twin of K3 (WEBP_AMD_K3=1, libwebp_amd_diag.so)
int vp8g_launch_encode_w1(const uint8_t* yuv, size_t yfb, int w, int h, int n,
                       const uint8_t* segmap, const vp8g_frame_params* params, uint16_t* tokens,
                       size_t tok_cap, uint8_t* mbinfo, vp8g_frame_result* results,
                       void* stream) {
  K3ArgsW1 a;
  a.yuv = yuv; a.yfb = yfb; a.w = w; a.h = h;
  a.mbw = (w + 15) >> 4; a.mbh = (h + 15) >> 4;
  a.segmap = segmap; a.params = params; a.tokens = tokens; a.tok_cap = tok_cap;
  a.mbinfo = mbinfo; a.results = results;
  const size_t lds = k3_lds_bytes(a.mbw);
  if (lds > 160 * 1024) {
    vp8g_set_error("k_encode", "frame too wide for the LDS budget");
    return 0;
  }
  a.amode = nullptr; a.mboff = nullptr; a.rerun = nullptr;
  static int attr_done = 0;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)k_encode_w1<false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_done = 1;
  }
  hipLaunchKernelGGL(k_encode_w1<false>, dim3(n), dim3(64), lds, (hipStream_t)stream, a);
  return launch_check("k_encode_w1");
}

#endif

int vp8g_launch_encode_none(const uint8_t* yuv, size_t yfb, int w, int h, int n,
                            const uint8_t* segmap, const uint8_t* amode,
                            const vp8g_frame_params* params, uint16_t* tokens, size_t tok_cap,
                            uint8_t* mbinfo, uint32_t* mboff, vp8g_frame_result* results,
                            uint8_t* rerun_state, void* stream) {
  K3ArgsW1 a;
  a.yuv = yuv; a.yfb = yfb; a.w = w; a.h = h;
  a.mbw = (w + 15) >> 4; a.mbh = (h + 15) >> 4;
  a.segmap = segmap; a.params = params; a.tokens = tokens; a.tok_cap = tok_cap;
  a.mbinfo = mbinfo; a.results = results;
  a.amode = amode; a.mboff = mboff; a.rerun = rerun_state;
  constexpr int NW = 3;   // MB workers (one wavefront each) per frame
  const size_t lds = NW * sizeof(K3Lds) + sizeof(K3NShared) + (16 * a.mbw + 16) + 16 * a.mbw +
                     4 * (a.mbw + 1) + 4 * a.mbw + 4 * a.mbw + 8 + 4 * (size_t)a.mbh + 16;
  if (lds > 160 * 1024) {
    vp8g_set_error("k_encode_none", "frame too wide for the LDS budget");
    return 0;
  }
  static int attr_done = 0;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)k_encode_none<NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_done = 1;
  }
  hipLaunchKernelGGL(k_encode_none<NW>, dim3(n), dim3(NW * 64), lds, (hipStream_t)stream, a);
  return launch_check("k_encode_none");
}

int vp8g_launch_synth(uint8_t* rgba, size_t fstride, int w, int h, int f0, int n, int seed,
                      void* stream) {
  dim3 grid((w + 255) / 256, h, n);
  hipLaunchKernelGGL(k_synth, grid, dim3(256), 0, (hipStream_t)stream, rgba, fstride, w, h, f0,
                     seed);
  return launch_check("k_synth");
}

}  // extern "C"
