// Device-side building blocks shared by the HIP kernels (tables, 4x4
// transforms, quantiser, predictors, rate/statistics helpers).
#ifndef LIBWEBP_AMD_VP8_DEV_H_
#define LIBWEBP_AMD_VP8_DEV_H_
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "../vp8_gpu.h"

#define VP8T_DECL static __constant__ const
#include "../vp8_tables.h"

#define BPS 32
#define QFIX 17
#define MAX_LEVEL 2047
#define MAX_VLEVEL 67
#define NSLOT VP8G_NUM_SLOTS
#define MAX_COST ((long long)0x7fffffffffffffLL)

typedef long long score_t;

// zigzag scan as constexpr functions so unrolled loops index registers
// statically (a __constant__ table would force private arrays to scratch)
__device__ __forceinline__ constexpr int zz(int n) {
  return n == 0 ? 0 : n == 1 ? 1 : n == 2 ? 4 : n == 3 ? 8 : n == 4 ? 5 : n == 5 ? 2 :
         n == 6 ? 3 : n == 7 ? 6 : n == 8 ? 9 : n == 9 ? 12 : n == 10 ? 13 : n == 11 ? 10 :
         n == 12 ? 7 : n == 13 ? 11 : n == 14 ? 14 : 15;
}
// inverse zigzag and VP8EncBands (src/enc/cost_enc.c:...; kZigzag inverse)
// as 4-bit fields of 64-bit immediates: register-only lookups, no memory
__device__ __forceinline__ int zz_inv(int b) {
  return (int)((0xfea9db83c7426510ull >> (4 * b)) & 15);
}
__device__ __forceinline__ int band_of(int n) {   // n in 0..16, band(16) = 0
  return n >= 16 ? 0 : (int)((0x7666666665463210ull >> (4 * n)) & 15);
}

// 4x4 intra predictor as data: pred[m][p] = f(edges e[0..12]) with
// e = L K J I X A B C D E F G H (src/dsp/enc.c:351-512). kind: 0 AVG3(a,b,c)
// 1 AVG2(a,b) 2 copy(a) 3 TM clip(e[5+x] + e[3-y] - X) 4 DC.
struct P4Op { uint8_t kind, a, b, c; };
#define A3(a, b, c) {0, a, b, c}
#define A2(a, b) {1, a, b, 0}
#define CP(a) {2, a, 0, 0}
enum { eL = 0, eK, eJ, eI, eX, eA, eB, eC, eD, eE, eF, eG, eH };
static __constant__ const P4Op kP4[10][16] = {
  // DC
  {{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},
   {4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0},{4,0,0,0}},
  // TM
  {{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},
   {3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0},{3,0,0,0}},
  // VE
  {A3(eX,eA,eB),A3(eA,eB,eC),A3(eB,eC,eD),A3(eC,eD,eE), A3(eX,eA,eB),A3(eA,eB,eC),A3(eB,eC,eD),A3(eC,eD,eE),
   A3(eX,eA,eB),A3(eA,eB,eC),A3(eB,eC,eD),A3(eC,eD,eE), A3(eX,eA,eB),A3(eA,eB,eC),A3(eB,eC,eD),A3(eC,eD,eE)},
  // HE
  {A3(eX,eI,eJ),A3(eX,eI,eJ),A3(eX,eI,eJ),A3(eX,eI,eJ), A3(eI,eJ,eK),A3(eI,eJ,eK),A3(eI,eJ,eK),A3(eI,eJ,eK),
   A3(eJ,eK,eL),A3(eJ,eK,eL),A3(eJ,eK,eL),A3(eJ,eK,eL), A3(eK,eL,eL),A3(eK,eL,eL),A3(eK,eL,eL),A3(eK,eL,eL)},
  // RD
  {A3(eA,eX,eI),A3(eB,eA,eX),A3(eC,eB,eA),A3(eD,eC,eB), A3(eX,eI,eJ),A3(eA,eX,eI),A3(eB,eA,eX),A3(eC,eB,eA),
   A3(eI,eJ,eK),A3(eX,eI,eJ),A3(eA,eX,eI),A3(eB,eA,eX), A3(eJ,eK,eL),A3(eI,eJ,eK),A3(eX,eI,eJ),A3(eA,eX,eI)},
  // VR
  {A2(eX,eA),A2(eA,eB),A2(eB,eC),A2(eC,eD), A3(eI,eX,eA),A3(eX,eA,eB),A3(eA,eB,eC),A3(eB,eC,eD),
   A3(eJ,eI,eX),A2(eX,eA),A2(eA,eB),A2(eB,eC), A3(eK,eJ,eI),A3(eI,eX,eA),A3(eX,eA,eB),A3(eA,eB,eC)},
  // LD
  {A3(eA,eB,eC),A3(eB,eC,eD),A3(eC,eD,eE),A3(eD,eE,eF), A3(eB,eC,eD),A3(eC,eD,eE),A3(eD,eE,eF),A3(eE,eF,eG),
   A3(eC,eD,eE),A3(eD,eE,eF),A3(eE,eF,eG),A3(eF,eG,eH), A3(eD,eE,eF),A3(eE,eF,eG),A3(eF,eG,eH),A3(eG,eH,eH)},
  // VL
  {A2(eA,eB),A2(eB,eC),A2(eC,eD),A2(eD,eE), A3(eA,eB,eC),A3(eB,eC,eD),A3(eC,eD,eE),A3(eD,eE,eF),
   A2(eB,eC),A2(eC,eD),A2(eD,eE),A3(eE,eF,eG), A3(eB,eC,eD),A3(eC,eD,eE),A3(eD,eE,eF),A3(eF,eG,eH)},
  // HD
  {A2(eI,eX),A3(eI,eX,eA),A3(eX,eA,eB),A3(eA,eB,eC), A2(eJ,eI),A3(eJ,eI,eX),A2(eI,eX),A3(eI,eX,eA),
   A2(eK,eJ),A3(eK,eJ,eI),A2(eJ,eI),A3(eJ,eI,eX), A2(eL,eK),A3(eL,eK,eJ),A2(eK,eJ),A3(eK,eJ,eI)},
  // HU
  {A2(eI,eJ),A3(eI,eJ,eK),A2(eJ,eK),A3(eJ,eK,eL), A2(eJ,eK),A3(eJ,eK,eL),A2(eK,eL),A3(eK,eL,eL),
   A2(eK,eL),A3(eK,eL,eL),CP(eL),CP(eL), CP(eL),CP(eL),CP(eL),CP(eL)},
};
#undef A3
#undef A2
#undef CP

__device__ __forceinline__ int clip8(int v) { return (v & ~0xff) == 0 ? v : (v < 0 ? 0 : 255); }
__device__ __forceinline__ int iabs_(int v) { return v < 0 ? -v : v; }
// VP8BitCost (cost_enc.h:59-61) from the LDS copy of kVP8EntropyCost
__device__ __forceinline__ int bit_cost(const uint16_t* ec, int bit, int p) {
  return ec[bit ? 255 - p : p];
}

// ---------------------------------------------------------------------------
// 4x4 transforms (src/dsp/enc.c:112-222, src/dsp/dec.c:137-162)

__device__ __forceinline__ void fdct4(const uint8_t* src, int ss, const uint8_t* ref, int rs,
                                      int out[16]) {
  int t[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d0 = src[i * ss + 0] - ref[i * rs + 0];
    const int d1 = src[i * ss + 1] - ref[i * rs + 1];
    const int d2 = src[i * ss + 2] - ref[i * rs + 2];
    const int d3 = src[i * ss + 3] - ref[i * rs + 3];
    const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
    t[4 * i + 0] = (a0 + a1) * 8;
    t[4 * i + 1] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
    t[4 * i + 2] = (a0 - a1) * 8;
    t[4 * i + 3] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int a0 = t[i] + t[12 + i], a1 = t[4 + i] + t[8 + i];
    const int a2 = t[4 + i] - t[8 + i], a3 = t[i] - t[12 + i];
    out[i] = (int16_t)((a0 + a1 + 7) >> 4);
    out[4 + i] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
    out[8 + i] = (int16_t)((a0 - a1 + 7) >> 4);
    out[12 + i] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
  }
}

// the same transform of a residual block d (row-major 4x4)
__device__ __forceinline__ void fdct4_res(const int d[16], int out[16]) {
  int t[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int d0 = d[4 * i], d1 = d[4 * i + 1], d2 = d[4 * i + 2], d3 = d[4 * i + 3];
    const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
    t[4 * i + 0] = (a0 + a1) * 8;
    t[4 * i + 1] = (a2 * 2217 + a3 * 5352 + 1812) >> 9;
    t[4 * i + 2] = (a0 - a1) * 8;
    t[4 * i + 3] = (a3 * 2217 - a2 * 5352 + 937) >> 9;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int a0 = t[i] + t[12 + i], a1 = t[4 + i] + t[8 + i];
    const int a2 = t[4 + i] - t[8 + i], a3 = t[i] - t[12 + i];
    out[i] = (int16_t)((a0 + a1 + 7) >> 4);
    out[4 + i] = (int16_t)(((a2 * 2217 + a3 * 5352 + 12000) >> 16) + (a3 != 0));
    out[8 + i] = (int16_t)((a0 - a1 + 7) >> 4);
    out[12 + i] = (int16_t)((a3 * 2217 - a2 * 5352 + 51000) >> 16);
  }
}

#define IMUL(a, b) (((a) * (b)) >> 16)
__device__ __forceinline__ void idct4(const uint8_t* ref, int rs, const int in[16], uint8_t* dst,
                                      int ds) {
  const int c1 = 20091 + (1 << 16), c2 = 35468;
  int t[16];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int a = in[i] + in[8 + i], b = in[i] - in[8 + i];
    const int c = IMUL(in[4 + i], c2) - IMUL(in[12 + i], c1);
    const int d = IMUL(in[4 + i], c1) + IMUL(in[12 + i], c2);
    t[4 * i + 0] = a + d; t[4 * i + 1] = b + c;
    t[4 * i + 2] = b - c; t[4 * i + 3] = a - d;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int dc = t[i] + 4;
    const int a = dc + t[8 + i], b = dc - t[8 + i];
    const int c = IMUL(t[4 + i], c2) - IMUL(t[12 + i], c1);
    const int d = IMUL(t[4 + i], c1) + IMUL(t[12 + i], c2);
    dst[i * ds + 0] = clip8(ref[i * rs + 0] + ((a + d) >> 3));
    dst[i * ds + 1] = clip8(ref[i * rs + 1] + ((b + c) >> 3));
    dst[i * ds + 2] = clip8(ref[i * rs + 2] + ((b - c) >> 3));
    dst[i * ds + 3] = clip8(ref[i * rs + 3] + ((a - d) >> 3));
  }
}

// Hadamard texture measure (src/dsp/enc.c:590-622)
__device__ __forceinline__ int hadamard_w(const uint8_t* in, int st) {
  int t[16], sum = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint8_t* p = in + i * st;
    const int a0 = p[0] + p[2], a1 = p[1] + p[3], a2 = p[1] - p[3], a3 = p[0] - p[2];
    t[4 * i + 0] = a0 + a1; t[4 * i + 1] = a3 + a2;
    t[4 * i + 2] = a3 - a2; t[4 * i + 3] = a0 - a1;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int a0 = t[i] + t[8 + i], a1 = t[4 + i] + t[12 + i];
    const int a2 = t[4 + i] - t[12 + i], a3 = t[i] - t[8 + i];
    sum += kVP8WeightY[i] * iabs_(a0 + a1) + kVP8WeightY[4 + i] * iabs_(a3 + a2) +
           kVP8WeightY[8 + i] * iabs_(a3 - a2) + kVP8WeightY[12 + i] * iabs_(a0 - a1);
  }
  return sum;
}

__device__ __forceinline__ int sse4(const uint8_t* a, int as, const uint8_t* b, int bs) {
  int s = 0;
#pragma unroll
  for (int y = 0; y < 4; ++y)
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int d = a[y * as + x] - b[y * bs + x];
      s += d * d;
    }
  return s;
}

// QuantizeBlock_C on natural-order coefficients c[] (int16 semantics),
// writes zigzag-order levels to lv[] (LDS), dequantises c[] in place.
__device__ __forceinline__ int quantize_block(int c[16], int16_t* lv, const vp8g_mtx* m,
                                              int lvr[16]) {
  int nz = 0;
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    const int j = zz(n);
    const int neg = c[j] < 0;
    const uint32_t coeff = (uint32_t)(neg ? -c[j] : c[j]) + m->sharpen[j];
    int level = 0;
    if (coeff > m->zthresh[j]) {
      level = (int)((coeff * m->iq[j] + m->bias[j]) >> QFIX);
      if (level > MAX_LEVEL) level = MAX_LEVEL;
      if (neg) level = -level;
    }
    c[j] = (int16_t)(level * (int)m->q[j]);
    lv[n] = (int16_t)level;
    lvr[n] = level;
    nz |= level;
  }
  return nz != 0;
}

// ---------------------------------------------------------------------------
// Shared MB helpers: cache import with edge replication (iterator_enc.c:107-145)

// Loads the 16x16 Y / 8x8 U / 8x8 V block of MB (x,y) into a BPS=32 cache
// (Y at col 0, U at col 16, V at col 24), replicating right/bottom edges.
__device__ __forceinline__ void load_mb(const uint8_t* Yp, const uint8_t* Up, const uint8_t* Vp,
                                        int w, int h, int x, int y, uint8_t* cache, int lane,
                                        int nlanes) {
  const int uvw = (w + 1) >> 1;
  const int bw = min(w - 16 * x, 16), bh = min(h - 16 * y, 16);
  const int cw = (bw + 1) >> 1, ch = (bh + 1) >> 1;
  for (int k = lane; k < 16 * 16 + 2 * 64; k += nlanes) {
    if (k < 256) {
      const int r = k >> 4, c = k & 15;
      const int rr = min(r, bh - 1), cc = min(c, bw - 1);
      cache[r * BPS + c] = Yp[(size_t)(16 * y + rr) * w + 16 * x + cc];
    } else {
      const int kk = k - 256, pl = kk >> 6, r = (kk >> 3) & 7, c = kk & 7;
      const int rr = min(r, ch - 1), cc = min(c, cw - 1);
      const uint8_t* P = pl ? Vp : Up;
      cache[r * BPS + 16 + 8 * pl + c] = P[(size_t)(8 * y + rr) * uvw + 8 * x + cc];
    }
  }
}

// load_mb for a 256-thread worker in two steps, so the global loads of the
// next MB can be in flight while the current one finishes: fetch_mb256 puts
// MB (x, y)'s Y byte of this thread (and a U or V byte for threads < 128)
// into one register (Y in bits 0-7, U or V in bits 8-15), put_mb256 stores
// them into the cache.
__device__ __forceinline__ uint32_t fetch_mb256(const uint8_t* Yp, const uint8_t* Up,
                                                const uint8_t* Vp, int w, int h, int x, int y,
                                                int t) {
  const int uvw = (w + 1) >> 1;
  const int bw = min(w - 16 * x, 16), bh = min(h - 16 * y, 16);
  const int cw = (bw + 1) >> 1, ch = (bh + 1) >> 1;
  uint32_t v;
  {
    const int r = t >> 4, c = t & 15;
    const int rr = min(r, bh - 1), cc = min(c, bw - 1);
    v = Yp[(size_t)(16 * y + rr) * w + 16 * x + cc];
  }
  if (t < 128) {
    const int pl = t >> 6, r = (t >> 3) & 7, c = t & 7;
    const int rr = min(r, ch - 1), cc = min(c, cw - 1);
    const uint8_t* P = pl ? Vp : Up;
    v |= (uint32_t)P[(size_t)(8 * y + rr) * uvw + 8 * x + cc] << 8;
  }
  return v;
}
__device__ __forceinline__ void put_mb256(uint32_t v, uint8_t* cache, int t) {
  cache[(t >> 4) * BPS + (t & 15)] = (uint8_t)v;
  if (t < 128) cache[((t >> 3) & 7) * BPS + 16 + 8 * (t >> 6) + (t & 7)] = (uint8_t)(v >> 8);
}

// 16x16 / 8x8 predictor sample (src/dsp/enc.c:238-342). left/top arrays with
// index -1 = corner; has_left/has_top select the 127/129 fall-backs.
__device__ __forceinline__ int pred_sample(int mode, int n, int px, int py, const uint8_t* left,
                                           const uint8_t* top, bool hl, bool ht, int dc) {
  switch (mode) {
    case 0: return dc;
    case 1:  // TM
      if (hl && ht) return clip8(top[px] + left[py] - left[-1]);
      if (hl) return left[py];
      if (ht) return top[px];
      return 129;
    case 2: return ht ? top[px] : 127;   // VE
    default: return hl ? left[py] : 129; // HE
  }
}
__device__ __forceinline__ int dc_value(const uint8_t* left, const uint8_t* top, bool hl, bool ht,
                                        int n, int shift) {
  int dc = 0;
  if (ht) {
    for (int j = 0; j < n; ++j) dc += top[j];
    if (hl) { for (int j = 0; j < n; ++j) dc += left[j]; }
    else dc += dc;
    return (dc + n) >> shift;
  }
  if (hl) {
    for (int j = 0; j < n; ++j) dc += left[j];
    dc += dc;
    return (dc + n) >> shift;
  }
  return 0x80;
}

// ---------------------------------------------------------------------------
// K3 helpers, generic over the LDS layout of the kernel using them
// per-MB non-zero context (iterator_enc.c:234-265) as bit masks:
// bit i of t = top_nz[i], bit i of l = left_nz[i]
struct MBCtx {
  uint32_t t, l;
  __device__ __forceinline__ int top(int i) const { return (t >> i) & 1; }
  __device__ __forceinline__ int left(int i) const { return (l >> i) & 1; }
};

// VP8LevelCost (cost_enc.h:63-66). The LDS rows already include
// kVP8LevelFixedCost[v] for v <= MAX_VLEVEL (folded in level_costs()), so
// only the rare v > 67 touches the global table.
__device__ __forceinline__ int level_cost(const uint16_t* tab, int v) {
  return v <= MAX_VLEVEL ? tab[v]
                         : tab[MAX_VLEVEL] - kVP8LevelFixedCost[MAX_VLEVEL] + kVP8LevelFixedCost[v];
}

// 16 zigzag levels from LDS into registers (two 16-byte reads)
__device__ __forceinline__ void load_lv(const int16_t* p, int r[16]) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint4 b = *reinterpret_cast<const uint4*>(p + 8);
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r[2 * i] = (int)(int16_t)(w[i] & 0xffff);
    r[2 * i + 1] = (int)(int16_t)(w[i] >> 16);
  }
}

// GetResidualCost_C (src/dsp/cost.c:322-355) on register-resident levels:
// each position's context is the previous level, already in a register, so
// all the LDS table reads are independent and overlap instead of chaining.
template <class LDS>
__device__ __forceinline__ int residual_cost_r(const LDS& L, int ctx0, int type, int first,
                                               const int lv[16]) {
  int last = -1;
#pragma unroll
  for (int n = 0; n < 16; ++n)
    if (n >= first && lv[n] != 0) last = n;
  const int p0 = L.coeffs[((type * 8 + first) * 3 + ctx0) * 11];   // band(first) == first
  if (last < 0) return bit_cost(L.ecost, 0, p0);
  int cost = ctx0 == 0 ? bit_cost(L.ecost, 1, p0) : 0;
  int prev = ctx0;
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    if (n >= first && n <= last) {
      const int v = iabs_(lv[n]);
      cost += level_cost(L.lcost[type * 24 + band_of(n) * 3 + prev], v);
      prev = v >= 2 ? 2 : v;
    }
  }
  if (last < 15)
    cost += bit_cost(L.ecost, 0, L.coeffs[((type * 8 + band_of(last + 1)) * 3 + prev) * 11]);
  return cost;
}

// TrellisQuantizeBlock (quant_enc.c:593-763). c[]: natural-order DCT
// coefficients (int16 semantics), dequantised in place; lv: zigzag levels.
// nodes: 32 words of LDS scratch owned by the calling lane. The position
// loops are fully unrolled so c[zz(n)] stays in registers.
template <class LDS>
__device__ __noinline__ int trellis_quant(const LDS& L, uint32_t* nodes, int c[16],
                                          int16_t* lv, int ctx0, int type,
                                          const vp8g_mtx* m, int lambda) {
  const int first = type == 0 ? 1 : 0;
  const int thresh = m->q[1] * m->q[1] / 4;
  const int last_proba = L.coeffs[((type * 8 + first) * 3 + ctx0) * 11];
  int last = first - 1;
#pragma unroll
  for (int n = 0; n < 16; ++n)
    if (n >= first && c[zz(n)] * c[zz(n)] > thresh) last = n;
  if (last < 15) ++last;
  score_t best_score = (score_t)bit_cost(L.ecost, 0, last_proba) * lambda;
  score_t sp0, sp1;
  int tp0, tp1;   // lcost row index of each predecessor node
  sp0 = sp1 = (score_t)(ctx0 == 0 ? bit_cost(L.ecost, 1, last_proba) : 0) * lambda;
  tp0 = tp1 = type * 24 + first * 3 + ctx0;
  int bp_n = -1, bp_k = 0, bp_prev = 0;
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    if (n >= first && n <= last) {
      const int j = zz(n);
      const uint32_t Q = m->q[j], iQ = m->iq[j];
      const int neg = c[j] < 0;
      const uint32_t coeff0 = (uint32_t)(neg ? -c[j] : c[j]) + m->sharpen[j];
      int level0 = (int)((coeff0 * iQ) >> QFIX);
      int thr = (int)((coeff0 * iQ + (0x80u << (QFIX - 8))) >> QFIX);
      if (thr > MAX_LEVEL) thr = MAX_LEVEL;
      if (level0 > MAX_LEVEL) level0 = MAX_LEVEL;
      const int band = band_of(n + 1);
      score_t sc0 = MAX_COST, sc1 = MAX_COST;
      int tc0 = 0, tc1 = 0;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int level = level0 + k;
        const int ctx = level > 2 ? 2 : level;
        const int tc = type * 24 + band * 3 + ctx;
        score_t cur = MAX_COST;
        if (level <= thr) {
          const int new_err = (int)coeff0 - level * (int)Q;
          const int delta = kVP8WeightTrellis[j] * (new_err * new_err - (int)(coeff0 * coeff0));
          score_t best = sp0 + (score_t)level_cost(L.lcost[tp0], level) * lambda;
          int bprev = 0;
          const score_t s1 = sp1 + (score_t)level_cost(L.lcost[tp1], level) * lambda;
          if (s1 < best) { best = s1; bprev = 1; }
          best += (score_t)256 * delta;
          nodes[2 * n + k] = (uint32_t)level | ((uint32_t)neg << 16) | ((uint32_t)bprev << 17);
          cur = best;
          if (level != 0 && best < best_score) {
            const score_t lc =
                (n < 15) ? bit_cost(L.ecost, 0, L.coeffs[((type * 8 + band) * 3 + ctx) * 11]) : 0;
            const score_t sc = best + lc * lambda;
            if (sc < best_score) { best_score = sc; bp_n = n; bp_k = k; bp_prev = bprev; }
          }
        }
        if (k == 0) { sc0 = cur; tc0 = tc; } else { sc1 = cur; tc1 = tc; }
      }
      sp0 = sc0; sp1 = sc1; tp0 = tc0; tp1 = tc1;
    }
  }
#pragma unroll
  for (int n = 0; n < 16; ++n) {
    if (n >= first) { c[zz(n)] = 0; lv[n] = 0; }
  }
  if (bp_n < 0) return 0;
  nodes[2 * bp_n + bp_k] = (nodes[2 * bp_n + bp_k] & ~(1u << 17)) | ((uint32_t)bp_prev << 17);
  int nz = 0, node = bp_k;
#pragma unroll
  for (int n = 15; n >= 0; --n) {
    if (n <= bp_n && n >= first) {
      const uint32_t nd = nodes[2 * n + node];
      const int level = (int)(nd & 0xffff);
      const int v = (nd >> 16) & 1 ? -level : level;
      lv[n] = (int16_t)v;
      nz |= level;
      c[zz(n)] = (int16_t)(v * (int)m->q[zz(n)]);
      node = (nd >> 17) & 1;
    }
  }
  return nz != 0;
}

// Barrier of a one-wavefront worker: orders its LDS traffic across lanes
// (the w1 / K3N kernels run one MB per wavefront, several per workgroup)
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// FinalizeTokenProbas (frame_enc.c:146-180): returns "changed" (dirty)
template <class LDS>
__device__ int finalize_probas(LDS& L, int lane) {
  int changed = 0;
  for (int s = lane; s < NSLOT; s += 64) {
    const uint32_t st = L.stats[s];
    const int nb = st & 0xffff, total = (st >> 16) & 0xffff;
    const int upd = (&kVP8CoeffUpdateProba[0][0][0][0])[s];
    const int old_p = (&kVP8CoeffProba0[0][0][0][0])[s];
    const int new_p = nb ? (255 - nb * 255 / total) : 255;
    const int old_cost = nb * bit_cost(L.ecost, 1, old_p) + (total - nb) * bit_cost(L.ecost, 0, old_p) + bit_cost(L.ecost, 0, upd);
    const int new_cost =
        nb * bit_cost(L.ecost, 1, new_p) + (total - nb) * bit_cost(L.ecost, 0, new_p) + bit_cost(L.ecost, 1, upd) + 8 * 256;
    if (old_cost > new_cost) {
      L.coeffs[s] = new_p;
      changed |= (new_p != old_p);
    } else {
      L.coeffs[s] = old_p;
    }
  }
  wsync();
  return __any(changed);
}

// VP8CalculateLevelCosts (cost_enc.c:42-90)
template <class LDS>
__device__ void level_costs(LDS& L, int lane, int nthr = 64) {
  for (int k = lane; k < 96 * (MAX_VLEVEL + 1); k += nthr) {
    const int tbc = k / (MAX_VLEVEL + 1), v = k % (MAX_VLEVEL + 1);
    const uint8_t* p = L.coeffs + tbc * 11;
    const int ctx = tbc % 3;
    const int c0 = ctx > 0 ? bit_cost(L.ecost, 1, p[0]) : 0;
    int cost;
    if (v == 0) {
      cost = bit_cost(L.ecost, 0, p[1]) + c0;
    } else {
      cost = bit_cost(L.ecost, 1, p[1]) + c0;
      int pat = kVP8LevelCodes[v - 1][0], bits = kVP8LevelCodes[v - 1][1];
      for (int i = 2; pat; ++i, pat >>= 1, bits >>= 1)
        if (pat & 1) cost += bit_cost(L.ecost, bits & 1, p[i]);
    }
    L.lcost[tbc][v] = (uint16_t)(cost + kVP8LevelFixedCost[v]);
  }
  wsync();
}

// VP8RecordStats (cost_enc.h:45-56)
__device__ __forceinline__ void record_stat(uint32_t* s, int bit) {
  uint32_t p = *s;
  if (p >= 0xfffe0000u) p = ((p + 1u) >> 1) & 0x7fff7fffu;
  *s = p + 0x00010000u + bit;
}

// Token generation for one block (token_enc.c:113-193). mode 0: count only;
// 1: write tokens + accumulate LDS stat deltas; 2: replay stats for marked
// slots (exact saturation order). RC: statistics with VP8RecordCoeffs' slots
// (cost_enc.c:289-340, the statistics pass of methods 0-2), which put the
// second category bit of cat5/cat6 in slot 10 where the token recorder uses 9.
template <int MODE, class LDS, bool RC = false>
__device__ int gen_tokens(LDS& L, const int16_t* lv, int type, int first, int ctx,
                          uint16_t* out, int* nz_out) {
  int last = -1;
  for (int n = 15; n >= first; --n)
    if (lv[n]) { last = n; break; }
  int count = 0;
  auto dyn = [&](int bit, int pid, int sid) -> int {
    if (MODE == 1) {
      out[count] = (uint16_t)((bit << 15) | pid);
      atomicAdd(&L.delta[sid], 0x10000u + bit);
    } else if (MODE == 2) {
      if (L.mark[sid >> 5] & (1u << (sid & 31))) record_stat(&L.stats[sid], bit);
    }
    ++count;
    return bit;
  };
  auto fix = [&](int bit, int proba) {
    if (MODE == 1) out[count] = (uint16_t)((bit << 15) | (1 << 14) | proba);
    ++count;
  };
  int n = first;
  int base = 11 * (ctx + 3 * (band_of(n) + 8 * type));
  *nz_out = last >= 0;
  if (!dyn(last >= 0, base + 0, base + 0)) return count;
  while (n < 16) {
    const int c = lv[n++];
    const int neg = c < 0;
    const uint32_t v = neg ? -c : c;
    if (!dyn(v != 0, base + 1, base + 1)) {
      base = 11 * (0 + 3 * (band_of(n) + 8 * type));
      continue;
    }
    if (!dyn(v > 1, base + 2, base + 2)) {
      base = 11 * (1 + 3 * (band_of(n) + 8 * type));
    } else {
      if (!dyn(v > 4, base + 3, base + 3)) {
        if (dyn(v != 2, base + 4, base + 4)) dyn(v == 4, base + 5, base + 5);
      } else if (!dyn(v > 10, base + 6, base + 6)) {
        if (!dyn(v > 6, base + 7, base + 7)) {
          fix(v == 6, 159);
        } else {
          fix(v >= 9, 165);
          fix(!(v & 1), 145);
        }
      } else {
        const uint8_t* tab;
        int mask;
        uint32_t res = v - 3;
        if (res < (8 << 1)) {
          dyn(0, base + 8, base + 8); dyn(0, base + 9, base + 9);
          res -= 8 << 0; mask = 1 << 2; tab = kVP8Cat3;
        } else if (res < (8 << 2)) {
          dyn(0, base + 8, base + 8); dyn(1, base + 9, base + 9);
          res -= 8 << 1; mask = 1 << 3; tab = kVP8Cat4;
        } else if (res < (8 << 3)) {
          dyn(1, base + 8, base + 8); dyn(0, base + 10, base + (RC ? 10 : 9));  // token_enc.c:168
          res -= 8 << 2; mask = 1 << 4; tab = kVP8Cat5;
        } else {
          dyn(1, base + 8, base + 8); dyn(1, base + 10, base + (RC ? 10 : 9));
          res -= 8 << 3; mask = 1 << 10; tab = kVP8Cat6;
        }
        for (; mask; mask >>= 1) fix((res & mask) != 0, *tab++);
      }
      base = 11 * (2 + 3 * (band_of(n) + 8 * type));
    }
    fix(neg, 128);
    if (n == 16 || !dyn(n <= last, base + 0, base + 0)) return count;
  }
  return count;
}

__device__ __forceinline__ void nz_flags(uint32_t t, uint32_t l, int left_dc, MBCtx& c) {
  c.t = ((t >> 12) & 0xf) | (((t >> 18) & 3) << 4) | (((t >> 22) & 3) << 6) | (((t >> 24) & 1) << 8);
  c.l = ((l >> 3) & 1) | (((l >> 7) & 1) << 1) | (((l >> 11) & 1) << 2) | (((l >> 15) & 1) << 3) |
        (((l >> 17) & 1) << 4) | (((l >> 19) & 1) << 5) | (((l >> 21) & 1) << 6) |
        (((l >> 23) & 1) << 7) | ((uint32_t)left_dc << 8);
}

// Block list of an MB for token order (frame_enc.c:411-453):
// idx 0 = I16 DC (only if i16), 1..16 = Y raster, 17..20 = U, 21..24 = V.
template <class LDS>
__device__ __forceinline__ const int16_t* blk_levels(const LDS& L, int k) {
  return k == 0 ? L.fin_dc : (k <= 16 ? L.fin_ac[k - 1] : L.fin_uv[k - 17]);
}

#endif
