// Autofilter (config->autofilter, cwebp -af): the SSIM-driven choice of each
// segment's loop-filter level (src/enc/filter_enc.c:156-212).
//
// The reference, for every MB of the last pass except skipped intra-16 ones,
// adds to lf_stats[segment][level] the SSIM (GetMBSSIM, :112-132) between the
// source MB and its reconstruction, unfiltered (level 0) and filtered with the
// inner-edge loop filter (DoFilter, :85-107; src/dsp/dec.c:484-692) at every
// level0 + d, d in [-quant, quant] step 4 (or 1); then picks per segment the
// level whose sum beats 1.00001 x the unfiltered one the most.
//
// Nothing here depends on MB order except the double sums, so:
//   A1 k_af_mb      one workgroup per MB: the 4 waves take the candidate
//                   levels round-robin; per level, filter a private copy of
//                   the reconstruction in LDS (rows, then columns, one lane
//                   per row/column of an edge), SSIM of its 172 windows (one
//                   lane per window), and the window sum in the reference's
//                   order by one lane -> mbval[mb][level] (0 for levels not
//                   tried, which leaves the later sums unchanged)
//   A2 k_af_reduce  per frame: one thread per (segment, level) adds the MBs'
//                   values in raster order (the reference's order of double
//                   additions), then the argmax per segment
// Doubles are IEEE (division correctly rounded) and contraction is off, so
// the sums are bit-identical to the reference's.
#include "vp8_dev.h"

#define AF_BPS 32
#define AF_NWIN 172   // 10 x 10 luma windows + 2 x 6 x 6 chroma windows

namespace {

__device__ __forceinline__ int sclip1(int v) { return min(max(v, -128), 127); }   // VP8ksclip1
__device__ __forceinline__ int sclip2(int v) { return min(max(v, -16), 15); }     // VP8ksclip2
__device__ __forceinline__ int uclip1(int v) { return min(max(v, 0), 255); }      // VP8kclip1

// DoFilter2_C / DoFilter4_C with the NeedsFilter(2) and Hev tests, one edge
// position (p points at q0, step across the edge)
__device__ void lf_simple(uint8_t* p, int step, int t2) {
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  if (4 * abs(p0 - q0) + abs(p1 - q1) > t2) return;
  const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
  const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
  p[-step] = (uint8_t)uclip1(p0 + a2);
  p[0] = (uint8_t)uclip1(q0 - a1);
}

__device__ void lf_inner(uint8_t* p, int step, int t2, int it, int hev) {   // FilterLoop24_C
  const int p3 = p[-4 * step], p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
  const int q0 = p[0], q1 = p[step], q2 = p[2 * step], q3 = p[3 * step];
  if (4 * abs(p0 - q0) + abs(p1 - q1) > t2) return;
  if (abs(p3 - p2) > it || abs(p2 - p1) > it || abs(p1 - p0) > it || abs(q3 - q2) > it ||
      abs(q2 - q1) > it || abs(q1 - q0) > it)
    return;
  if (abs(p1 - p0) > hev || abs(q1 - q0) > hev) {   // DoFilter2
    const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
    const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3);
    p[-step] = (uint8_t)uclip1(p0 + a2);
    p[0] = (uint8_t)uclip1(q0 - a1);
  } else {                                           // DoFilter4
    const int a = 3 * (q0 - p0);
    const int a1 = sclip2((a + 4) >> 3), a2 = sclip2((a + 3) >> 3), a3 = (a1 + 1) >> 1;
    p[-2 * step] = (uint8_t)uclip1(p1 + a3);
    p[-step] = (uint8_t)uclip1(p0 + a2);
    p[0] = (uint8_t)uclip1(q0 - a1);
    p[step] = (uint8_t)uclip1(q1 - a3);
  }
}

// window i of GetMBSSIM's order: luma rows 3..12 x columns 3..12, then for
// x = 1..6, y = 1..6 the U then the V window
__device__ __forceinline__ void af_window(int i, int& off, int& xo, int& yo, int& n) {
  if (i < 100) {
    off = 0; yo = 3 + i / 10; xo = 3 + i % 10; n = 16;
  } else {
    const int j = i - 100, pr = j >> 1;
    off = (j & 1) ? 24 : 16; xo = 1 + pr / 6; yo = 1 + pr % 6; n = 8;
  }
}

// VP8SSIMGetClipped (ssim.c:73-99) + SSIMCalculation (ssim.c:28-52)
__device__ double af_ssim(const uint8_t* s1, const uint8_t* s2, int xo, int yo, int n) {
#pragma clang fp contract(off)
  const int ymin = max(yo - 3, 0), ymax = min(yo + 3, n - 1);
  const int xmin = max(xo - 3, 0), xmax = min(xo + 3, n - 1);
  uint32_t w = 0, xm = 0, ym = 0, xxm = 0, xym = 0, yym = 0;
  for (int y = ymin; y <= ymax; ++y) {
    const uint32_t wy = 4 - abs(y - yo);
    for (int x = xmin; x <= xmax; ++x) {
      const uint32_t wt = (4 - abs(x - xo)) * wy;   // kWeight = 1 2 3 4 3 2 1
      const uint32_t a = s1[y * AF_BPS + x], b = s2[y * AF_BPS + x];
      w += wt; xm += wt * a; ym += wt * b;
      xxm += wt * a * a; xym += wt * a * b; yym += wt * b * b;
    }
  }
  const uint32_t N = w, w2 = N * N;
  const uint32_t C1 = 20 * w2, C2 = 60 * w2, C3 = 8 * 8 * w2;
  const uint64_t xmxm = (uint64_t)xm * xm, ymym = (uint64_t)ym * ym;
  if (xmxm + ymym < C3) return 1.;
  const int64_t xmym = (int64_t)xm * ym;
  const int64_t sxy = (int64_t)xym * N - xmym;
  const uint64_t sxx = (uint64_t)xxm * N - xmxm, syy = (uint64_t)yym * N - ymym;
  const uint64_t num_S = (2 * (uint64_t)(sxy < 0 ? 0 : sxy) + C2) >> 8;
  const uint64_t den_S = (sxx + syy + C2) >> 8;
  const uint64_t fnum = (2 * xmym + C1) * num_S;
  const uint64_t fden = (xmxm + ymym + C1) * den_S;
  return (double)fnum / (double)fden;
}

}  // namespace

__global__ __launch_bounds__(256) void k_af_mb(const uint8_t* __restrict__ yuv, size_t yfb,
                                               int w, int h, const uint8_t* __restrict__ mbinfo,
                                               const uint8_t* __restrict__ recon,
                                               const vp8g_af_frame* __restrict__ afp,
                                               const uint8_t* __restrict__ active,
                                               double* __restrict__ mbval) {
#pragma clang fp contract(off)
  const int f = blockIdx.y, mb = blockIdx.x, t = threadIdx.x, wv = t >> 6, lane = t & 63;
  const int mbw = (w + 15) >> 4, nmb = mbw * ((h + 15) >> 4);
  if (!active[f]) return;
  __shared__ uint8_t src[16 * AF_BPS];
  __shared__ uint32_t rec[4 * AF_BPS];
  __shared__ uint8_t work[4][16 * AF_BPS];
  __shared__ double win[4][AF_NWIN];
  __shared__ double res[64];
  const size_t gmb = (size_t)f * nmb + mb;
  const uint8_t* info = mbinfo + gmb * VP8G_MBINFO_BYTES;
  const int is_i16 = info[0], seg = info[2], skip = info[3];
  if (t < 64) res[t] = 0.;
  if (!(is_i16 && skip)) {   // skipped intra-16 MBs add nothing (filter_enc.c:176)
    // source MB with the edge replication of VP8IteratorImport (iterator_enc.c:107-147)
    const int mx = mb % mbw, my = mb / mbw;
    const uint8_t* Yp = yuv + (size_t)f * yfb;
    const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
    const uint8_t* Up = Yp + (size_t)w * h;
    const uint8_t* Vp = Up + (size_t)uvw * uvh;
    {
      const int x = t & 15, y = t >> 4;
      const int sx = min(mx * 16 + x, w - 1), sy = min(my * 16 + y, h - 1);
      src[y * AF_BPS + x] = Yp[(size_t)sy * w + sx];
    }
    if (t < 128) {
      const int x = t & 7, y = (t >> 3) & 7, pl = t >> 6;
      const int sx = min(mx * 8 + x, uvw - 1), sy = min(my * 8 + y, uvh - 1);
      src[y * AF_BPS + 16 + 8 * pl + x] = (pl ? Vp : Up)[(size_t)sy * uvw + sx];
    }
    if (t < 128) rec[t] = reinterpret_cast<const uint32_t*>(recon + gmb * 512)[t];
  }
  __syncthreads();
  if (is_i16 && skip) {
    if (t < 64) mbval[gmb * 64 + t] = 0.;
    return;
  }
  const vp8g_af_frame P = afp[f];
  const int level0 = P.level0[seg], q = P.quant[seg];
  const int step = (2 * q >= 4) ? 4 : 1;
  const int ncand = 1 + (2 * q) / step + 1;   // level 0, then d = -q, -q + step, ... <= q
  const uint8_t* recb = reinterpret_cast<const uint8_t*>(rec);
  uint8_t* wk = work[wv];
  for (int base = 0; base < ncand; base += 4) {
    const int c = base + wv;
    int level = 0;
    bool on = c < ncand;
    if (on && c > 0) {
      level = level0 - q + (c - 1) * step;
      on = level > 0 && level < 64;
    }
    if (on) {
      for (int k = lane; k < 4 * AF_BPS; k += 64)
        reinterpret_cast<uint32_t*>(wk)[k] = rec[k];
    }
    __syncthreads();
    if (on && level > 0) {   // DoFilter: the inner edges, rows first, then columns
      int ilevel = level;
      if (P.sharpness > 0) {   // GetILevel (filter_enc.c:70-83)
        ilevel >>= (P.sharpness > 4) ? 2 : 1;
        if (ilevel > 9 - P.sharpness) ilevel = 9 - P.sharpness;
      }
      if (ilevel < 1) ilevel = 1;
      const int t2 = 2 * (2 * level + ilevel) + 1;
      const int hev = (level >= 40) ? 2 : (level >= 15) ? 1 : 0;
      for (int dir = 0; dir < 2; ++dir) {   // 0: vertical edges (HFilter), 1: horizontal
        const int hs = dir ? AF_BPS : 1, vs = dir ? 1 : AF_BPS;
        for (int k = 1; k <= 3; ++k) {
          if (lane < 16) {
            uint8_t* p = wk + 4 * k * hs + lane * vs;
            if (P.simple) lf_simple(p, hs, t2);
            else lf_inner(p, hs, t2, ilevel, hev);
          } else if (k == 1 && lane < 32 && !P.simple) {   // HFilter8i / VFilter8i: U, V
            const int r = lane & 7, pl = (lane >> 3) & 1;
            uint8_t* p = wk + 16 + 8 * pl + 4 * hs + r * vs;
            lf_inner(p, hs, t2, ilevel, hev);
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
    }
    if (on) {
      for (int i = lane; i < AF_NWIN; i += 64) {
        int off, xo, yo, n;
        af_window(i, off, xo, yo, n);
        win[wv][i] = af_ssim(src + off, wk + off, xo, yo, n);
      }
    }
    __syncthreads();
    if (on && lane == 0) {   // GetMBSSIM's order of additions
      double sum = 0.;
      for (int i = 0; i < AF_NWIN; ++i) sum += win[wv][i];
      res[level] = sum;
    }
    __syncthreads();
  }
  if (t < 64) mbval[gmb * 64 + t] = res[t];
}

__global__ __launch_bounds__(256) void k_af_reduce(int nmb, const uint8_t* __restrict__ mbinfo,
                                                   const double* __restrict__ mbval,
                                                   const uint8_t* __restrict__ active,
                                                   uint8_t* __restrict__ level) {
#pragma clang fp contract(off)
  const int f = blockIdx.x, t = threadIdx.x, s = t >> 6, lv = t & 63;
  if (!active[f]) return;
  __shared__ double lf[4][64];
  const uint8_t* info = mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES;
  const double* v = mbval + (size_t)f * nmb * 64;
  double acc = 0.;
  for (int mb = 0; mb < nmb; ++mb)   // lf_stats_[s][level] += ..., raster order
    if (info[(size_t)mb * VP8G_MBINFO_BYTES + 2] == s) acc += v[(size_t)mb * 64 + lv];
  lf[s][lv] = acc;
  __syncthreads();
  if (t < 4) {   // VP8AdjustFilterStrength (filter_enc.c:197-212)
    int best = 0;
    double best_v = 1.00001 * lf[t][0];
    for (int i = 1; i < 64; ++i)
      if (lf[t][i] > best_v) { best_v = lf[t][i]; best = i; }
    level[4 * f + t] = (uint8_t)best;
  }
}

extern "C" int vp8g_launch_check(const char* what);

extern "C" int vp8g_launch_autofilter(const uint8_t* yuv, size_t yfb, int w, int h, int n,
                                      const uint8_t* mbinfo, const uint8_t* recon,
                                      const vp8g_af_frame* afp, const uint8_t* active,
                                      double* mbval, uint8_t* level, void* stream) {
  if (n <= 0) return 1;
  const int nmb = ((w + 15) >> 4) * ((h + 15) >> 4);
  hipLaunchKernelGGL(k_af_mb, dim3(nmb, n), dim3(256), 0, (hipStream_t)stream, yuv, yfb, w, h,
                     mbinfo, recon, afp, active, mbval);
  if (!vp8g_launch_check("k_af_mb")) return 0;
  hipLaunchKernelGGL(k_af_reduce, dim3(n), dim3(256), 0, (hipStream_t)stream, nmb, mbinfo, mbval,
                     active, level);
  return vp8g_launch_check("k_af_reduce");
}
