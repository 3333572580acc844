// Sharp (iterative) RGB -> YUV420 on gfx950: the conversion libwebp applies
// for use_sharp_yuv / preprocessing & 4 (src/enc/webp_enc.c:352-356 ->
// picture_csp_enc.c:176-186 -> sharpyuv/sharpyuv.c:297-430, 8-bit RGB in,
// 8-bit YUV out, WebP matrix, sRGB transfer). Bit-exact with the reference.
//
// The algorithm works on 10-bit "W/RGB" planes: best_y (W per pixel) and
// best_uv (R-W, G-W, B-W per 2x2 block), refined up to 4 times against the
// targets computed from the source. Inside one iteration the row pairs are
// *sequential*: best_uv is updated in place, so row pair j interpolates with
// the already-updated row j-1 (sharpyuv.c:354-406). Columns are independent.
//
//   k_sharp_init   one thread per 2x2 block, whole grid: targets + initial
//                  W/RGB planes (sharpyuv.c:318-346), opaque check.
//   k_sharp_iter   one workgroup per frame, one launch per iteration: walks
//                  the row pairs top to bottom with one thread per chroma
//                  column; the updated previous chroma row is exchanged in
//                  LDS (double-buffered, one barrier per row pair). best_uv
//                  is double-buffered in HBM across launches (iteration k
//                  reads buffer k&1, writes (k+1)&1), so every HBM value a
//                  thread reads from another thread was written by an earlier
//                  launch. The frame's exit test (sum of |dY| against
//                  3*w*h and the previous iteration, :407-413) is evaluated by
//                  the workgroup and stored in the frame's state; later
//                  launches of a finished frame return at once.
//   k_sharp_final  one thread per 2x2 block: ConvertWRGBToYUV (:221-268)
//                  into the WebPPicture YUV420 layout.
//
// Integer byte/word work, HBM/latency bound; no MFMA.
#include <hip/hip_runtime.h>

#include "../vp8_gpu.h"

namespace {

struct Tabs {
  uint32_t g2l[1026];
  uint32_t l2g[514];
};

__device__ __forceinline__ void load_tabs(Tabs& t, const uint32_t* g2l, const uint32_t* l2g) {
  for (int i = threadIdx.x; i < 1026; i += blockDim.x) t.g2l[i] = g2l[i];
  for (int i = threadIdx.x; i < 514; i += blockDim.x) t.l2g[i] = l2g[i];
}

// sharpyuv_gamma.c:84-99,109-114 at 10 bits: linear (16-bit) -> gamma
__device__ __forceinline__ int to_gamma(const Tabs& t, uint32_t v) {
  const uint32_t pos = v >> 7, x = v & 127;
  const uint32_t v0 = t.l2g[pos] >> 6, v1 = t.l2g[pos + 1] >> 6;
  return (int)(v0 + (((v1 - v0) * x + 64) >> 7));
}
// sharpyuv.c:67-70 (inputs < 2^16: the sum fits 32 unsigned bits)
__device__ __forceinline__ int gray(uint32_t r, uint32_t g, uint32_t b) {
  return (int)((13933u * r + 46871u * g + 4732u * b + 32768u) >> 16);
}
__device__ __forceinline__ int clip10(int v) { return min(max(v, 0), 1023); }

struct Px {
  int c[4][3];   // 2x2 block (row-major), 10-bit R,G,B
};

// W of each pixel (UpdateW :85-101) and the block's chroma (UpdateChroma +
// ScaleDown :72-83,103-128); the linearised samples are shared.
__device__ __forceinline__ void w_and_chroma(const Tabs& t, const Px& p, int wv[4], int uv[3]) {
  uint32_t lin[4][3];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 3; ++k) lin[q][k] = t.g2l[p.c[q][k]];
#pragma unroll
  for (int q = 0; q < 4; ++q) wv[q] = to_gamma(t, (uint32_t)gray(lin[q][0], lin[q][1], lin[q][2]));
  int c[3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
    c[k] = to_gamma(t, (lin[0][k] + lin[1][k] + lin[2][k] + lin[3][k] + 2) >> 2);
  const int W = gray(c[0], c[1], c[2]);
#pragma unroll
  for (int k = 0; k < 3; ++k) uv[k] = (int)(int16_t)(c[k] - W);
}

struct Planes {   // per-frame scratch views
  uint16_t* by;   // best_y   [2*uvh][2*uvw]
  uint16_t* ty;   // target_y [2*uvh][2*uvw]
  int16_t* buv0;  // best_uv, buffer 0 [uvh][3][uvw]
  int16_t* buv1;  // best_uv, buffer 1
  int16_t* tuv;   // target_uv [uvh][3][uvw]
};

__device__ __forceinline__ Planes planes(uint8_t* scratch, size_t fbytes, int f, int uvw,
                                         int uvh) {
  Planes p;
  const size_t ny = (size_t)4 * uvw * uvh, nuv = (size_t)3 * uvw * uvh;
  uint8_t* b = scratch + (size_t)f * fbytes;
  p.by = (uint16_t*)b;
  p.ty = p.by + ny;
  p.buv0 = (int16_t*)(p.ty + ny);
  p.buv1 = p.buv0 + nuv;
  p.tuv = p.buv1 + nuv;
  return p;
}

}  // namespace

__global__ __launch_bounds__(256) void k_sharp_init(const uint8_t* __restrict__ rgba,
                                                    size_t fstride, int rstride, int width,
                                                    int height, uint8_t* __restrict__ scratch,
                                                    size_t fbytes, vp8g_sharp_state* state,
                                                    uint32_t* __restrict__ aflags,
                                                    const uint32_t* __restrict__ g2l,
                                                    const uint32_t* __restrict__ l2g) {
  __shared__ Tabs t;
  load_tabs(t, g2l, l2g);
  __syncthreads();
  const int uvw = (width + 1) >> 1, uvh = (height + 1) >> 1, w2 = 2 * uvw;
  const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y, f = blockIdx.z;
  if (i == 0 && j == 0) {
    state[f].prev_sum = ~0ull;
    state[f].done = 0;
    state[f].iters = 0;
  }
  if (i >= uvw) return;
  const Planes P = planes(scratch, fbytes, f, uvw, uvh);
  const uint8_t* src = rgba + f * fstride;
  // ImportOneRow (:152-180): x4, replicate the last column / row
  Px p;
  uint32_t bad = 0;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int yy = min(2 * j + r, height - 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int xx = min(2 * i + s, width - 1);
      const uint8_t* q = src + (size_t)yy * rstride + 4 * xx;   // any row stride
      p.c[2 * r + s][0] = q[0] << 2;
      p.c[2 * r + s][1] = q[1] << 2;
      p.c[2 * r + s][2] = q[2] << 2;
      bad |= q[3] != 0xff;
    }
  }
  if (bad) atomicOr(aflags + f, 1u);
  int wv[4], uv[3];
  w_and_chroma(t, p, wv, uv);
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const size_t o = (size_t)(2 * j + r) * w2 + 2 * i;
    const int g0 = gray(p.c[2 * r][0], p.c[2 * r][1], p.c[2 * r][2]);        // StoreGray
    const int g1 = gray(p.c[2 * r + 1][0], p.c[2 * r + 1][1], p.c[2 * r + 1][2]);
    *(uint32_t*)(P.by + o) = (uint32_t)g0 | ((uint32_t)g1 << 16);
    *(uint32_t*)(P.ty + o) = (uint32_t)wv[2 * r] | ((uint32_t)wv[2 * r + 1] << 16);
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const size_t o = ((size_t)j * 3 + k) * uvw + i;
    P.tuv[o] = (int16_t)uv[k];
    P.buv0[o] = (int16_t)uv[k];
  }
}

// one iteration of sharpyuv.c:349-418 for each frame (blockIdx.x)
__global__ __launch_bounds__(1024) void k_sharp_iter(int iter, int width, int height,
                                                     uint8_t* __restrict__ scratch,
                                                     size_t fbytes, vp8g_sharp_state* state,
                                                     const uint32_t* __restrict__ g2l,
                                                     const uint32_t* __restrict__ l2g) {
  __shared__ Tabs t;
  __shared__ unsigned long long red[16];
  extern __shared__ int16_t rows[];   // 2 slots x [3][uvw]: updated previous row
  const int f = blockIdx.x;
  if (state[f].done) return;
  load_tabs(t, g2l, l2g);
  const int uvw = (width + 1) >> 1, uvh = (height + 1) >> 1, w2 = 2 * uvw;
  const Planes P = planes(scratch, fbytes, f, uvw, uvh);
  const int16_t* __restrict__ src = (iter & 1) ? P.buv1 : P.buv0;
  int16_t* __restrict__ dst = (iter & 1) ? P.buv0 : P.buv1;
  __syncthreads();
  unsigned long long sum = 0;
  for (int j = 0; j < uvh; ++j) {
    const int16_t* cur = src + (size_t)j * 3 * uvw;
    const int16_t* nxt = src + (size_t)min(j + 1, uvh - 1) * 3 * uvw;
    // prev: the updated row j-1 (LDS slot (j-1)&1), or row 0 itself at j=0
    const int16_t* prv = j ? rows + ((j - 1) & 1) * 3 * uvw : cur;
    int16_t* out = rows + (j & 1) * 3 * uvw;
    for (int i = threadIdx.x; i < uvw; i += blockDim.x) {
      const int il = max(i - 1, 0), ir = min(i + 1, uvw - 1);
      Px p;
      const size_t o0 = (size_t)(2 * j) * w2 + 2 * i, o1 = o0 + w2;
      const uint32_t by0 = *(const uint32_t*)(P.by + o0), by1 = *(const uint32_t*)(P.by + o1);
      const int byv[4] = {(int)(by0 & 0xffff), (int)(by0 >> 16), (int)(by1 & 0xffff),
                          (int)(by1 >> 16)};
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int a = cur[k * uvw + i], al = cur[k * uvw + il], ar = cur[k * uvw + ir];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const int16_t* B = r ? nxt : prv;
          const int b = B[k * uvw + i], bl = B[k * uvw + il], br = B[k * uvw + ir];
          // even pixel x=2i: v1 of filter index i-1, or Filter2 at x=0;
          // odd pixel x=2i+1: v0 of filter index i, or Filter2 at x=w-1
          // (InterpolateTwoRows :182-219, SharpYuvFilterRow_C dsp:53-65)
          const int e2 = (a * 3 + b + 2) >> 2;
          const int ve = i == 0 ? e2 : (a * 9 + al * 3 + b * 3 + bl + 8) >> 4;
          const int vo = i == uvw - 1 ? e2 : (a * 9 + ar * 3 + b * 3 + br + 8) >> 4;
          p.c[2 * r][k] = clip10(byv[2 * r] + ve);
          p.c[2 * r + 1][k] = clip10(byv[2 * r + 1] + vo);
        }
      }
      int wv[4], uv[3];
      w_and_chroma(t, p, wv, uv);
      // SharpYuvUpdateY_C (dsp:28-41) on the block's 4 pixels
      const uint32_t ty0 = *(const uint32_t*)(P.ty + o0), ty1 = *(const uint32_t*)(P.ty + o1);
      const int tyv[4] = {(int)(ty0 & 0xffff), (int)(ty0 >> 16), (int)(ty1 & 0xffff),
                          (int)(ty1 >> 16)};
      int ny[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int d = tyv[q] - wv[q];
        ny[q] = clip10(byv[q] + d);
        sum += (unsigned)abs(d);
      }
      *(uint32_t*)(P.by + o0) = (uint32_t)ny[0] | ((uint32_t)ny[1] << 16);
      *(uint32_t*)(P.by + o1) = (uint32_t)ny[2] | ((uint32_t)ny[3] << 16);
      // SharpYuvUpdateRGB_C (dsp:43-51)
      const int16_t* tu = P.tuv + (size_t)j * 3 * uvw;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int16_t v = (int16_t)(cur[k * uvw + i] + tu[k * uvw + i] - uv[k]);
        out[k * uvw + i] = v;
        dst[(size_t)j * 3 * uvw + k * uvw + i] = v;
      }
    }
    __syncthreads();
  }
  // frame-wide sum of |dY| and the exit test (:407-413)
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (int q = 0; q < (int)(blockDim.x >> 6); ++q) s += red[q];
    const unsigned long long thresh =
        (unsigned long long)(3.0 * (double)w2 * (double)(2 * uvh));
    vp8g_sharp_state st = state[f];
    st.iters = iter + 1;
    if (iter > 0 && (s < thresh || s > st.prev_sum)) st.done = 1;
    st.prev_sum = s;
    state[f] = st;
  }
}

__global__ __launch_bounds__(256) void k_sharp_final(int width, int height,
                                                     const uint8_t* __restrict__ scratch,
                                                     size_t fbytes,
                                                     const vp8g_sharp_state* state,
                                                     uint8_t* __restrict__ yuv, size_t yfb) {
  const int uvw = (width + 1) >> 1, uvh = (height + 1) >> 1, w2 = 2 * uvw;
  const int i = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y, f = blockIdx.z;
  if (i >= uvw) return;
  const Planes P = planes((uint8_t*)scratch, fbytes, f, uvw, uvh);
  const int16_t* buv = ((state[f].iters & 1) ? P.buv1 : P.buv0) + (size_t)j * 3 * uvw;
  const int r = buv[i], g = buv[uvw + i], b = buv[2 * uvw + i];
  uint8_t* Y = yuv + (size_t)f * yfb;
  uint8_t* U = Y + (size_t)width * height;
  uint8_t* V = U + (size_t)uvw * uvh;
  // RGBToYUVComponent with the WebP matrix, sfix = 2 (:195-202, :221-268);
  // clip_8b sees the value as int16 (:56-58)
  auto clip8 = [](int v) -> uint8_t {
    const int s = (int16_t)v;
    return (uint8_t)((s & ~0xff) == 0 ? s : (s < 0 ? 0 : 255));
  };
#pragma unroll
  for (int rr = 0; rr < 2; ++rr) {
    const int y = 2 * j + rr;
    if (y >= height) break;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int x = 2 * i + s;
      if (x >= width) break;
      const int W = P.by[(size_t)y * w2 + x];
      Y[(size_t)y * width + x] = clip8(
          (16839 * (r + W) + 33059 * (g + W) + 6420 * (b + W) + (16 << 18) + (1 << 17)) >> 18);
    }
  }
  U[(size_t)j * uvw + i] = clip8((-9719 * r - 19081 * g + 28800 * b + (128 << 18) + (1 << 17)) >> 18);
  V[(size_t)j * uvw + i] = clip8((28800 * r - 24116 * g - 4684 * b + (128 << 18) + (1 << 17)) >> 18);
}

extern "C" int vp8g_launch_check(const char* what);

extern "C" size_t vp8g_sharp_frame_bytes(int w, int h) {
  const size_t uvw = (size_t)((w + 1) >> 1), uvh = (size_t)((h + 1) >> 1);
  return (34 * uvw * uvh + 255) & ~(size_t)255;
}

extern "C" int vp8g_launch_sharp(const uint8_t* rgba, size_t fstride, int rstride, int w, int h,
                                 int n, uint8_t* yuv, size_t yfb, uint32_t* aflags,
                                 uint8_t* scratch, vp8g_sharp_state* state,
                                 const uint32_t* g2l, const uint32_t* l2g, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  const size_t fbytes = vp8g_sharp_frame_bytes(w, h);
  const size_t lds = (size_t)2 * 3 * uvw * sizeof(int16_t);
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_sharp_iter,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) {
      vp8g_set_error("k_sharp_iter (dynamic LDS)", hipGetErrorString(e));
      return 0;
    }
  }
  dim3 grid((uvw + 255) / 256, uvh, n);
  hipLaunchKernelGGL(k_sharp_init, grid, dim3(256), 0, st, rgba, fstride, rstride, w, h, scratch,
                     fbytes, state, aflags, g2l, l2g);
  if (!vp8g_launch_check("k_sharp_init")) return 0;
  for (int it = 0; it < 4; ++it) {   // kNumIterations, sharpyuv.c:36
    hipLaunchKernelGGL(k_sharp_iter, dim3(n), dim3(1024), lds, st, it, w, h, scratch, fbytes,
                       state, g2l, l2g);
    if (!vp8g_launch_check("k_sharp_iter")) return 0;
  }
  hipLaunchKernelGGL(k_sharp_final, grid, dim3(256), 0, st, w, h, scratch, fbytes, state, yuv,
                     yfb);
  return vp8g_launch_check("k_sharp_final");
}
