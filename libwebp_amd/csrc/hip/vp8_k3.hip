// K3 k_encode: the raster-order RD macroblock loop of VP8EncTokenLoop
// (src/enc/frame_enc.c:783-894) for CDNA4, one 256-thread workgroup
// (4 wavefronts, one per SIMD of a CU) per frame.
//
// The MB order is the reference's raster order: it is the only order that
// reproduces the token statistics, the cost-refresh epochs and the U/V DC
// error diffusion bit-exactly. Parallelism inside an MB is per COEFFICIENT:
// a 4x4 block lives on 16 lanes (lane = natural coefficient index), its
// forward/inverse transforms are two 4-lane butterfly passes exchanged with
// cross-lane shuffles, quantisation is one coefficient per lane, and the rate
// (GetResidualCost_C) is one table term per lane plus a 16-lane reduction.
//
//   I16  wave = prediction mode, 4 passes of 4 blocks x 16 coefficients
//   UV   wave = prediction mode, 2 passes of 4 blocks x 16 coefficients
//   I4   160 lanes = 10 modes x 16 coefficients, 16 dependent sub-blocks
//   tokens / statistics / contexts: wave 0 (25 blocks in parallel)
//
// Trellis quantisation (m5 final pass, m6 everywhere; quant_enc.c:593-763)
// stays one lane per block: the Viterbi over 16 positions is inherently
// sequential; the other lanes hand it their coefficients through LDS.
#include "vp8_dev.h"

#include <stdio.h>

#include <atomic>
#include <mutex>

#define K3T 256

// a cross-worker wait that has not been satisfied after this long (100 MHz
// s_memrealtime ticks, 30 s) is a bug: the frame is aborted with an error
// instead of hanging the GPU
#ifndef K3_WAIT_TICKS
#define K3_WAIT_TICKS (30ull * 100000000ull)
#endif

// LDS shared by all of a frame's workers: cost tables of the current epoch,
// token statistics, quantiser/segment parameters and frame-level counters.
struct alignas(16) K3G {
  uint32_t stats[NSLOT];
  uint16_t lcost[96][MAX_VLEVEL + 1];  // [type*24 + band*3 + ctx][level], incl. fixed cost
  uint16_t ecost[256];
  uint16_t mcost4[1000];
  P4Op p4[160];
  uint16_t wy[16];
  uint16_t hc[96][2];              // VP8BitCost(0/1, proba[type][band][ctx][0]) of this epoch
  uint8_t coeffs[NSLOT];
  uint32_t mark[33];
  vp8g_seg seg[4];
  int32_t max_edge[4];
  struct {
    unsigned long long size_p0, sse[3], dist;
    unsigned long long size_rh;    // sum of the per-MB R + H (OneStatPass, frame_enc.c:593)
    int32_t nb[3];
  } fs;                            // per-frame side statistics (frame_enc.c:480-489, :839)
  int32_t dirty;                   // FinalizeTokenProbas result
  int32_t flag_mark;               // some statistics slot needs the in-order replay
  uint32_t fold_ptr;               // raster MBs whose tokens are folded into stats
  uint32_t ntok;                   // tokens in the frame's compact stream
  int32_t tok_err;
  int32_t epoch;                   // cost-table epochs published
  int32_t abort;                   // a cross-worker wait timed out (bug guard)
};

static_assert(offsetof(K3G, coeffs) % 4 == 0, "K3X moves the probabilities as words");

// LDS private to one worker (4 wavefronts) and the MB it is encoding.
struct K3S {
  uint8_t yin[16 * BPS];
  uint8_t yout[16 * BPS];
  uint8_t p16[4][256];
  uint8_t puv[4][128];
  uint8_t rec16[4][256];
  uint8_t recuv[4][128];
  alignas(16) int16_t lv16[4][16][16];   // zigzag levels per mode/block
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
  alignas(8) unsigned long long best4[3];   // intra4 argmin key (score << 4 | mode), 3 buffers
  alignas(8) score_t sm4[2][10];   // intra4 candidate scores with lambda_mode (by sub-block parity)
  int32_t r4[2][10][4];            // H, nz, R, D (by sub-block parity)
  uint8_t rec4[2][10][16];         // every candidate's reconstruction (by sub-block parity)
  int32_t nzsel;                   // the m5 pass: nz of the sub-block's given mode
  int32_t lead;                    // the worker's place in the row wavefront (issue priority)
  int32_t hsrc[16];                // sum_j w_j |Hadamard(src block)_j| per luma block
  alignas(16) int16_t acc_ac[16][16];
  uint8_t acc_out[256];
  int32_t mres[4][4];
  int32_t blkinfo[32];
  int32_t blast[32];               // last non-zero zigzag position per token block
  int32_t wsum[2][4];              // per-wave token-count totals (scan)
  int32_t redw[4];                 // per-wave reduction slots
  uint32_t fold_total;             // tokens of the MBs being folded
  uint32_t fold_base;              // their first compact-stream offset
  int32_t epseen;                  // G.epoch as one lane read it before the last worker barrier
  uint32_t bar;                    // worker barrier counter
  int32_t myabort;
  int32_t flag_ldc;                // left DC nz flag hand-off from wave 0
  int32_t mdist;                   // VP8ModeScore D of the MB (thread 0 only)
  int32_t d4acc;                   // intra4 D of the blocks chosen so far (thread 0 only)
  int32_t r4acc;                   // intra4 R of the blocks chosen so far (thread 0 only)
  int32_t ry16;                    // R of the best intra16 mode
  uint32_t mark_any;
  uint8_t yl_mem[17], ul_mem[9], vl_mem[9];
  uint8_t predleft[4];
  int8_t lderr[2][2];
  // statistics of this worker's tokens not folded yet (counted as they are
  // written), and the token count of each MB of its current row
  uint32_t rdelta[NSLOT];
  uint16_t rowcnt[1024];           // mbw <= 1024 (width <= 16383)
  // token rows (K3Args::rowtok): tokens this worker's current row has
  // written so far, and where in the row each of its MBs put them
  uint32_t rowfill;
  uint32_t rowpos[1024];
#ifdef K3_TRACE
  unsigned long long trace[16];    // diagnostic build: per-worker cycle / event counts (K3TR_*)
#endif
#ifdef K3_CHECK
  uint32_t ck_nmb, ck_cap;         // check build: the frame's MBs, a token row's room
  int32_t ck_y, ck_x;              // the MB the worker is at (the hang record)
  uint32_t ck_rowdone;             // LDS offset of rowdone[0]
#endif
};

// Index checks (-DK3_CHECK, diagnostic build libwebp_amd_check.so): every
// global address k_encode computes from LDS state (token row positions,
// per-MB token counts and positions, compact-stream offsets, MB indices) is
// checked before the access; a failing check records the first failure
// (site, workgroup, worker, MB, value, bound) and counts the rest, and the
// access is skipped, so a bad index shows up as a record instead of a GPU
// fault. vp8g_k3_check reads the record back (tools/k3_trace.py).
#ifdef K3_CHECK
__device__ unsigned long long g_k3check[8];
__device__ __noinline__ void k3ck_fail(int site, unsigned long long v, unsigned long long bound,
                                       unsigned mb) {
  if (atomicAdd(&g_k3check[0], 1ull) == 0) {
    g_k3check[1] = (unsigned long long)site;
    g_k3check[2] = blockIdx.x;
    g_k3check[3] = threadIdx.x;
    g_k3check[4] = mb;
    g_k3check[5] = v;
    g_k3check[6] = bound;
  }
}
#define K3CK(cond, site, v, bound, mb) \
  ((cond) ? true : (k3ck_fail((site), (unsigned long long)(v), (unsigned long long)(bound), (mb)), false))
// a cross-worker wait that gives up (timeout or another worker's abort)
// records, per workgroup and worker: site, the waited word's LDS offset, the
// value waited for, the value seen, the worker's MB (y, x), its barrier count
__device__ uint32_t g_k3hang[1024][4][10];
#define CK_NMB(L, dflt) (L).ck_nmb
#define CK_CAP(L, dflt) (unsigned long long)(L).ck_cap
#else
#define K3CK(cond, site, v, bound, mb) true
#define CK_NMB(L, dflt) (dflt)
#define CK_CAP(L, dflt) (dflt)
#endif

// Barrier over the 4 wavefronts of one worker (s_barrier would stop the whole
// workgroup, i.e. every worker). Arrivals count up an LDS word; a wave
// waits for the next multiple of 4. Called in worker-uniform control flow.
// The poll loop is deliberately bare: ~40 of these barriers sit on each MB's
// dependent chain, and every variant with a time or iteration bound inside
// the loop measured 3-7% slower K3 launches. A worker
// barrier can only wait forever if a wave of the worker never arrives: all
// waves of a worker take the same path, and every cross-worker wait that can
// fail (wait_ge / wait_gx, bounded by K3_WAIT_TICKS) releases its worker's
// waiting waves by setting bit 31 of the counter (WBAR_RELEASE), so they
// fall through, the worker leaves its row loop and the frame reports an error.
#define WBAR_RELEASE 0x80000000u
#ifndef K3_WBAR_SLEEP
#define K3_WBAR_SLEEP 0   // s_sleep units between polls (0 / 1 / 2: 124.0 / 124.3 / 124.9 ms, profiles/r3/ab13_*)
#endif
// The synchronisation words are handled without any compiler-visible
// lane-masked region: this compiler's register
// allocator places live-range-split copies and spill stores of wave-wide
// values at the end of a divergent region, BEFORE the instruction that
// restores the exec mask -- after a poll loop's exit (no lanes enabled),
// inside the lane-0 branch of a barrier arrival, in the else arm of an
// if / else -- so some or all lanes keep stale registers (the row index, the
// row-wavefront word's address, the thread id). Four diagnostic builds
// stalled, faulted or leaked token-arena chunks that way; tools/isa_lane0_check.py
// finds the pattern in every one of them and checks every shipped code
// object (build() fails on it). Hence: the arrival is one asm statement that
// switches to lane 0 and back itself, and every poll loop tests a
// wave-uniform (readfirstlane) value, i.e. is a scalar loop. The last wave to
// arrive (its add returned 3 mod 4) does not poll: the count it completed is
// the release.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ uint32_t lane0_add(uint32_t* p, uint32_t v) {
  uint32_t old;
  uint64_t saved;
  asm volatile(
      "s_mov_b64 %1, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_add_rtn_u32 %0, %2, %3\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 exec, %1"
      : "=&v"(old), "=&s"(saved)
      : "v"(lds_addr(p)), "v"(v)
      : "memory");
  return (uint32_t)__builtin_amdgcn_readlane((int)old, 0);
}
template <typename T>
__device__ __forceinline__ T ld_uni(const T* p, int order = __ATOMIC_RELAXED) {
  const T v = order == __ATOMIC_ACQUIRE ? __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)
                                        : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return (T)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ void wbar(K3S& L) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  const uint32_t old = lane0_add(&L.bar, 1u);
  const uint32_t target = (old & ~3u) + 4u;
#ifndef K3_NOSKIP
  if ((old & 3u) != 3u)
#endif
    while (ld_uni(&L.bar) < target) __builtin_amdgcn_s_sleep(K3_WBAR_SLEEP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
#ifdef K3_BARCHECK
// diagnostic build (-DK3_CHECK -DK3_BARCHECK): a worker barrier that has not
// completed after K3_BAR_TICKS records, per workgroup / worker / wave, the
// source line of the barrier, the counter before the arrival, the target and
// the counter seen, the worker's MB; then the worker gives up (its barriers
// release, its row loop ends) so the launch drains and the records come back
#ifndef K3_BAR_TICKS
#define K3_BAR_TICKS (5ull * 100000000ull)
#endif
__device__ uint32_t g_k3bar[1024][4][4][8];
__device__ __noinline__ void wbar_late(K3S& L, uint32_t old, uint32_t target, int line) {
  const uint32_t lane = threadIdx.x & 63, wv = (threadIdx.x >> 6) & 3, wk = (threadIdx.x >> 8) & 3;
  const uint32_t seen = ld_uni(&L.bar);
  uint32_t v = 0x80000000u;
  v = lane == 0 ? (uint32_t)line : v;
  v = lane == 1 ? old : v;
  v = lane == 2 ? target : v;
  v = lane == 3 ? seen : v;
  v = lane == 4 ? (uint32_t)L.ck_y : v;
  v = lane == 5 ? (uint32_t)L.ck_x : v;
  v = lane == 6 ? 0u : v;
  if (blockIdx.x < 1024 && lane < 8) g_k3bar[blockIdx.x][wk][wv][lane] = v;
  L.myabort = 1;
  atomicOr(&L.bar, WBAR_RELEASE);
}
__device__ __forceinline__ void wbar_at(K3S& L, int line) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  const uint32_t old = lane0_add(&L.bar, 1u);
  const uint32_t target = (old & ~3u) + 4u;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  if ((old & 3u) != 3u)
    while (ld_uni(&L.bar) < target) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > K3_BAR_TICKS) {
        wbar_late(L, old, target, line);
        break;
      }
      __builtin_amdgcn_s_sleep(K3_WBAR_SLEEP);
    }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
#define wbar(L) wbar_at(L, __LINE__)
#endif
#define WB() wbar(L)

// all-threads AND over the worker
__device__ __forceinline__ int wbar_and(K3S& L, int v) {
  // wave-uniform throughout: every lane stores its wave's vote (same value,
  // same word: no lane mask), the result goes through readfirstlane, so a
  // branch on it is a scalar branch
  const int all = __all(v);
  L.redw[(__builtin_amdgcn_readfirstlane(threadIdx.x) >> 6) & 3] = all;
  wbar(L);
  return __builtin_amdgcn_readfirstlane(L.redw[0] & L.redw[1] & L.redw[2] & L.redw[3]);
}

// ---------------------------------------------------------------------------
// 16-lane block primitives. g = first lane of the block's group in the wave,
// j = natural coefficient / pixel index (x = j & 3, y = j >> 2).

__device__ __forceinline__ int zz_rt(int n) {   // kZigzag[n] for a runtime n
  return (int)((0xfeb7adc963258410ull >> (4 * n)) & 15);
}

// Cross-lane exchange inside a 16-lane group with DPP (no LDS round trip):
// quad_perm broadcasts lane k of each 4-lane row of the block, row_ror:4/8/12
// fetch the same column from the other three rows.
template <int C>
__device__ __forceinline__ int dpp(int v) {
  return __builtin_amdgcn_mov_dpp(v, C, 0xf, 0xf, false);
}
// DPP reads for the trellis whose result is pinned where it is written: a
// DPP whose value feeds only one arm of a select may otherwise be sunk into
// a branch, where the lanes of the other arm are masked off and the source
// lanes among them hand over stale registers (seen on gfx950: lane first + 1
// read its own initial value instead of lane first's score). `old` is what a
// lane with no source lane in its row (row_shr at lane 0, row_shl at 15) gets.
template <int C>
__device__ __forceinline__ int dpp_pin(int old, int v) {
  int r = __builtin_amdgcn_update_dpp(old, v, C, 0xf, 0xf, false);
  asm volatile("" : "+v"(r));
  return r;
}
#define DPP_QB(k) ((k) | ((k) << 2) | ((k) << 4) | ((k) << 6))
#define DPP_ROR(n) (0x120 + (n))   // lane i reads lane (i - n) mod 16

// MUL of ITransformOne with a 24-bit multiply: |a| < 2^23 and the constants
// are 17-bit, and v_mul_i32_i24 returns the low 32 bits of the product, as
// the reference's int arithmetic does
#define IMUL24(a, b) (__mul24((a), (b)) >> 16)

// the 4 values of this lane's 4-lane row, in x order
__device__ __forceinline__ void row4(int v, int& r0, int& r1, int& r2, int& r3) {
  r0 = dpp<DPP_QB(0)>(v);
  r1 = dpp<DPP_QB(1)>(v);
  r2 = dpp<DPP_QB(2)>(v);
  r3 = dpp<DPP_QB(3)>(v);
}
// the 4 values of this lane's column, ROTATED: u_s = row (y - s) & 3
__device__ __forceinline__ void colrot(int v, int& u0, int& u1, int& u2, int& u3) {
  u0 = v;
  u1 = dpp<DPP_ROR(4)>(v);
  u2 = dpp<DPP_ROR(8)>(v);
  u3 = dpp<DPP_ROR(12)>(v);
}

// An optimisation barrier on a per-lane value: constants derived from it are
// rebuilt where they are used instead of being hoisted out of the MB loop and
// held in registers (and spilled) across the whole kernel.
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

#define K_C1 (20091 + (1 << 16))
#define K_C2 35468

// FTransform_C (src/dsp/enc.c:157-191): lane holds the residual of pixel
// (x, y); returns output coefficient j (int16 like the reference's out[]).
// Row pass over the lane's row in natural order (row4), column pass over the
// column rotated by the lane's row (colrot: u_s = row (y - s) & 3), both as
// the reference's butterflies with the lane picking its output:
//   row    x = 0, 2: (a0 +- a1) * 8        x = 1, 3: (a2 2217 + a3 5352 + 1812) >> 9,
//                                                    (a3 2217 - a2 5352 +  937) >> 9
//   column y = 0, 2: (a0 +- a1 + 7) >> 4   y = 1, 3: the same pair with 12000 / 51000,
//                                                    >> 16, + (a3 != 0) on row 1
// where in the rotated column a0 + a1 = u0 + u1 + u2 + u3 (y = 0),
// a0 - a1 = u2 + u3 - u0 - u1 (y = 2), (a2, a3) = (u0 - u3, u1 - u2) (y = 1)
// and (u2 - u1, u3 - u0) (y = 3).
__device__ __forceinline__ int fdct_lane(int d, int j) {
  const int x = j & 3, y = j >> 2;
  int d0, d1, d2, d3;
  row4(d, d0, d1, d2, d3);
  const int a0 = d0 + d3, a1 = d1 + d2, a2 = d1 - d2, a3 = d0 - d3;
  const bool x1 = x == 1;
  const int P = x1 ? a2 : a3, Q = x1 ? a3 : -a2;
  const int todd = (__mul24(P, 2217) + __mul24(Q, 5352) + (x1 ? 1812 : 937)) >> 9;
  const int tev = (x == 0 ? a0 + a1 : a0 - a1) * 8;
  const int t = (x & 1) ? todd : tev;
  int u0, u1, u2, u3;
  colrot(t, u0, u1, u2, u3);
  const int S = u0 + u1, T = u2 + u3;
  const int oev = ((y == 0 ? S + T : T - S) + 7) >> 4;
  const bool y1 = y == 1;
  const int b2 = y1 ? u0 - u3 : u2 - u1, b3 = y1 ? u1 - u2 : u3 - u0;
  const int P2 = y1 ? b2 : b3, Q2 = y1 ? b3 : -b2;
  const int oodd = ((__mul24(P2, 2217) + __mul24(Q2, 5352) + (y1 ? 12000 : 51000)) >> 16) +
                   (y1 && b3 != 0);
  return (int16_t)((y & 1) ? oodd : oev);
}

// ITransformOne (src/dsp/enc.c:116-147): lane holds dequantised coefficient
// j and the prediction sample of pixel (x, y); returns the reconstruction.
// Vertical pass (output y of column x) over the rotated column u_s:
// with (p, q, r, s) = (u0, u2, MUL(u1, kC2), MUL(u3, kC1)) for even y and
// (u1, u3, MUL(u0, kC2), MUL(u2, kC1)) for odd y, the reference's a + d,
// b + c, b - c, a - d are (p + q) + (r + s), (p - q) + (r - s),
// -((p - q) + (r - s)), (p + q) - (r + s) for y = 0..3.
__device__ __forceinline__ int idct_lane(int c, int pr, int j) {
  const int y = j >> 2;
  int u0, u1, u2, u3;
  colrot(c, u0, u1, u2, u3);
  const bool yo = y & 1;
  const int p = yo ? u1 : u0, q = yo ? u3 : u2, mA = yo ? u0 : u1, mB = yo ? u2 : u3;
  const int r = IMUL24(mA, K_C2), s = IMUL24(mB, K_C1);
  const bool e = ((y + 1) & 2) == 0;   // y = 0 or 3
  const int A = e ? p + q : p - q, B = e ? r + s : r - s;
  int t = y == 3 ? A - B : A + B;   // tmp[4x + y]
  t = y == 2 ? -t : t;
  int t0, t1, t2, t3;
  row4(t, t0, t1, t2, t3);
  // horizontal pass (:134-146): a = dc + t2, b = dc - t2 (dc = t0 + 4),
  // d = MUL(t1, kC1) + MUL(t3, kC2), c = MUL(t1, kC2) - MUL(t3, kC1);
  // x = 0..3 takes a + d, b + c, b - c, a - d
  const int x = j & 3;
  const bool xo = ((x + 1) & 2) == 0;   // x = 0 or 3
  const int P = t0 + 4 + (xo ? t2 : -t2);
  const int m1 = IMUL24(t1, xo ? K_C1 : K_C2), m3 = IMUL24(t3, xo ? K_C2 : K_C1);
  const int Q = xo ? m1 + m3 : m1 - m3;
  const int v = x < 2 ? P + Q : P - Q;
  return clip8(pr + (v >> 3));
}

// One lane's term of TTransform (src/dsp/enc.c:590-622): weighted |Hadamard
// coefficient j| of the 4x4 samples p, as butterflies without per-lane
// constants. Only |coefficient| is used, so each lane may compute its
// coefficient up to a sign: a sign that depends on the lane's column x
// alone flips all four row-pass values a column-pass lane combines, and the
// column pass is free to flip its own result. With those freedoms the row
// pass of column x is a0 + a1 | a3 + a2 | a3 - a2 | a0 - a1 (x = 0..3) over
// a0 = i0 + i2, a1 = i1 + i3, a2 = i1 - i3, a3 = i0 - i2, and the column
// pass over the rotated rows u_s (colrot) is (u0 + u1) + (u2 + u3) (y = 0),
// (u0 + u1) - (u2 + u3) (y = 1, 2), (u0 - u1) + (u2 - u3) (y = 3).
__device__ __forceinline__ int ttrans_lane(int p, int j, int wj) {
  const int x = j & 3, y = j >> 2;
  int i0, i1, i2, i3;
  row4(p, i0, i1, i2, i3);
  const int a0 = i0 + i2, a1 = i1 + i3, a2 = i1 - i3, a3 = i0 - i2;
  const bool xo = ((x + 1) & 2) == 0;   // x = 0 or 3
  const int pu = xo ? a0 : a3, pv = xo ? a1 : a2;
  const int t = x < 2 ? pu + pv : pu - pv;
  int u0, u1, u2, u3;
  colrot(t, u0, u1, u2, u3);
  const bool y3 = y == 3;
  const int A = y3 ? u0 - u1 : u0 + u1;
  const int B = y3 ? u2 - u3 : u2 + u3;
  const int o = (y == 1 || y == 2) ? A - B : A + B;
  return __mul24(wj, iabs_(o));
}

__device__ __forceinline__ int sum16(int v) {
  v += dpp<DPP_ROR(8)>(v);
  v += dpp<DPP_ROR(4)>(v);
  v += dpp<DPP_ROR(2)>(v);
  v += dpp<DPP_ROR(1)>(v);
  return v;
}
__device__ __forceinline__ int max16(int v) {
  v = max(v, dpp<DPP_ROR(8)>(v));
  v = max(v, dpp<DPP_ROR(4)>(v));
  v = max(v, dpp<DPP_ROR(2)>(v));
  v = max(v, dpp<DPP_ROR(1)>(v));
  return v;
}
// wave total (uniform): 16-lane sums, then the four row results
__device__ __forceinline__ int sum64(int v) {
  v = sum16(v);
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
         __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

// QuantizeBlock_C for coefficient j (src/dsp/enc.c:653-677)
__device__ __forceinline__ int quant_lane(int cv, int j, const vp8g_mtx& M, int& dq) {
  const int neg = cv < 0;
  const uint32_t coeff = (uint32_t)(neg ? -cv : cv) + M.sharpen[j];
  int level = min((int)((__umul24(coeff, M.iq[j]) + M.bias[j]) >> QFIX), MAX_LEVEL);
  level = coeff > M.zthresh[j] ? level : 0;
  level = neg ? -level : level;
  dq = (int16_t)__mul24(level, (int)M.q[j]);
  return level;
}

// GetResidualCost_C (src/dsp/cost.c:322-355) with one zigzag position per
// lane: the context of position n is the previous position's level (one
// bpermute), every lane does its table reads unconditionally (no divergent
// branches) and a 16-lane reduction sums the terms.
// The level at the previous zigzag position, from its lane of the same
// 16-lane block: natural index j reads j-1, j-3, j-4 or j+3 (DPP row shifts,
// no LDS round trip). Lane j = 0 (zigzag 0) has no predecessor.
__device__ __forceinline__ int zz_prev(int v, int j) {
  const int m1 = dpp_pin<0x111>(0, v);   // row_shr:1
  const int m3 = dpp_pin<0x113>(0, v);   // row_shr:3
  const int m4 = dpp_pin<0x114>(0, v);   // row_shr:4
  const int p3 = dpp_pin<0x103>(0, v);   // row_shl:3
  const uint32_t bit = 1u << j;
  return (bit & 0xA00Au) ? m1 : (bit & 0x5250u) ? m3 : (bit & 0x0900u) ? m4 : p3;
}

__device__ __forceinline__ int rate_lane(const K3G& G, int level, int j, int g, int ctx0, int type,
                                         int first) {
  const int n = zz_inv(j);
  const int v = iabs_(level);
  const int last = max16((v != 0 && n >= first) ? n : -1);
  const int vprev = iabs_(zz_prev(level, j));
  const int ctxp = n == first ? ctx0 : min(vprev, 2);
  int cost = G.lcost[type * 24 + band_of(n) * 3 + ctxp][min(v, MAX_VLEVEL)];
  if (v > MAX_VLEVEL)   // rare: beyond the LDS rows
    cost += kVP8LevelFixedCost[v] - kVP8LevelFixedCost[MAX_VLEVEL];
  const int eob = G.hc[type * 24 + band_of(n + 1) * 3 + min(v, 2)][0];
  cost += (n == last && n < 15) ? eob : 0;
  cost = (n >= first && n <= last) ? cost : 0;
  const int t0 = type * 24 + first * 3 + ctx0;   // band(first) == first
  const int h0 = G.hc[t0][0], h1 = G.hc[t0][1];
  const int hdr = last < 0 ? h0 : (ctx0 == 0 ? h1 : 0);
  cost += j == 0 ? hdr : 0;
  return sum16(cost);
}

// ---------------------------------------------------------------------------
// Lane-parallel TrellisQuantizeBlock (quant_enc.c:593-763) on the 16-lane
// groups of a wave, one block per group (group-uniform `act`, `ctx0`).
//
// The reference walks zigzag positions n = first..last keeping two nodes
// (level0 and level0 + 1) with their best score. Everything but the scores
// is known up front: a node's level, its distortion change and the cost row
// of each predecessor (that row depends only on the predecessor's level,
// level0(n - 1) + p, not on the path). So lane n of the group (zigzag
// order; the coefficients arrive by one bpermute) computes its levels,
// distortion terms and the four transition costs in parallel, and only the
// min-plus recursion over n stays sequential: round r hands every lane its
// predecessor's two scores by DPP row_shr:1, and lane n holds its final
// scores after n - first + 1 rounds -- the same int64 additions and the same
// comparisons (predecessor 0 first, 1 only if strictly smaller) as the
// reference, so the result is bit-exact. The best terminal node (first
// minimum over (n, m) in the reference's order, against the skip score) is a
// 16-lane minimum plus a ballot; the path is unwound by row_shl:1 rounds.
// Rounds run to the wave's longest group only.
struct Trellis16 {
  int level;   // quantised level of this lane's coefficient (natural index j)
  int dq;      // level * q[j] (reconstruction input)
  int lvz;     // the level at zigzag position lane & 15
  int nz;      // the group's block has a non-zero level (group-uniform)
};

template <int C>
__device__ __forceinline__ long long dpp64(long long old, long long v) {
  const int lo = dpp_pin<C>((int)(old & 0xffffffff), (int)(v & 0xffffffff));
  const int hi = dpp_pin<C>((int)(old >> 32), (int)(v >> 32));
  return (long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int wtrellis(int j) {   // kWeightTrellis[j] (quant_enc.c)
  const unsigned long long t = j < 8 ? 0x0a11181b0b131b1eull : 0x06080a0b080c1113ull;
  return (int)((t >> (8 * (j & 7))) & 0xff);
}

template <bool DBG = false>
__device__ Trellis16 trellis16(const K3G& G, int c, bool act, int ctx0, int type,
                               const vp8g_mtx& M, int lambda, long long* dbg = nullptr) {
  const int lane = threadIdx.x & 63, g = lane & 48, n = lane & 15;
  const int first = type == 0 ? 1 : 0;
  const int jn = zz_rt(n);   // natural index of zigzag position n
  const int cin = __shfl(c, g + jn);
  // the last position worth inspecting (+1)
  const int thresh2 = (int)M.q[1] * (int)M.q[1] / 4;
  int last = max16((n >= first && cin * cin > thresh2) ? n : first - 1);
  if (last < 15) ++last;
  // this position's two nodes
  const uint32_t Q = M.q[jn], iQ = M.iq[jn];
  const int sign = cin < 0;
  const uint32_t coeff0 = (uint32_t)(sign ? -cin : cin) + M.sharpen[jn];
  const int level0 = min((int)((coeff0 * iQ) >> QFIX), MAX_LEVEL);
  const int thr = min((int)((coeff0 * iQ + (0x80u << (QFIX - 8))) >> QFIX), MAX_LEVEL);
  const int wt = wtrellis(jn);
  const int e0 = (int)coeff0 - level0 * (int)Q, e1 = e0 - (int)Q;
  const int cc = (int)(coeff0 * coeff0);
  // delta_error in the reference's uint32 arithmetic, then as int
  const score_t base0 = (score_t)256 * (int)((uint32_t)wt * ((uint32_t)(e0 * e0) - (uint32_t)cc));
  const score_t base1 = (score_t)256 * (int)((uint32_t)wt * ((uint32_t)(e1 * e1) - (uint32_t)cc));
  const bool live1 = level0 + 1 <= thr;   // level0 itself never exceeds thr
  // cost rows of the two predecessors (position n - 1's nodes)
  const int lp0 = dpp_pin<0x111>(0, level0);   // row_shr:1: level0 of position n - 1
  const int rfirst = type * 24 + first * 3 + ctx0;
  const int rb = type * 24 + band_of(n) * 3;
  const int row0 = n == first ? rfirst : rb + min(lp0, 2);
  const int row1 = n == first ? rfirst : rb + min(lp0 + 1, 2);
  const score_t t00 = (score_t)level_cost(G.lcost[row0], level0) * lambda;
  const score_t t01 = (score_t)level_cost(G.lcost[row1], level0) * lambda;
  const int l1 = min(level0 + 1, MAX_LEVEL);   // (a node beyond MAX_LEVEL is dead anyway)
  const score_t t10 = (score_t)level_cost(G.lcost[row0], l1) * lambda;
  const score_t t11 = (score_t)level_cost(G.lcost[row1], l1) * lambda;
  // the source node and the skip score
  const int lastp = G.coeffs[((type * 8 + first) * 3 + ctx0) * 11];
  const score_t s_init = (score_t)(ctx0 == 0 ? bit_cost(G.ecost, 1, lastp) : 0) * lambda;
  const score_t skip = (score_t)bit_cost(G.ecost, 0, lastp) * lambda;
  // min-plus recursion: R rounds, R = the longest group of the wave
  const int span = act ? last - first + 1 : 0;
  int R = span;
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) R = max(R, __shfl_xor(R, o));
  R = __builtin_amdgcn_readfirstlane(R);
  // the source node reaches position `first` as its predecessor: through the
  // DPP's `old` at lane 0 (first = 0), from lane 0 held at s_init (first = 1)
  const bool src = n < first;
  score_t S0 = src ? s_init : MAX_COST, S1 = S0;
  int pv = 0;   // best predecessor of node 0 (bit 0) and node 1 (bit 1)
  for (int r = 0; r < R; ++r) {
    const score_t p0 = dpp64<0x111>(s_init, S0);
    const score_t p1 = dpp64<0x111>(s_init, S1);
    const score_t a0 = p0 + t00, b0 = p1 + t01;
    const score_t a1 = p0 + t10, b1 = p1 + t11;
    const bool q0 = b0 < a0, q1 = b1 < a1;
    const score_t n0 = (q0 ? b0 : a0) + base0;
    const score_t n1 = live1 ? (q1 ? b1 : a1) + base1 : MAX_COST;
    S0 = src ? s_init : n0;
    S1 = src ? s_init : n1;
    pv = (int)q0 | ((int)q1 << 1);
  }
  // best terminal node: sc = S + last-position cost, first minimum in (n, m)
  const bool in = act && n >= first && n <= last;
  const int ctx1 = min(level0 + 1, 2);
  const int bnext = type * 8 + band_of(n + 1);
  const int lpc0 = n < 15 ? bit_cost(G.ecost, 0, G.coeffs[(bnext * 3 + min(level0, 2)) * 11]) : 0;
  const int lpc1 = n < 15 ? bit_cost(G.ecost, 0, G.coeffs[(bnext * 3 + ctx1) * 11]) : 0;
  const bool v0 = in && level0 != 0, v1 = in && live1;
  const score_t sc0 = S0 + (score_t)lpc0 * lambda, sc1 = S1 + (score_t)lpc1 * lambda;
  const bool take1 = v1 && (!v0 || sc1 < sc0);
  const score_t NONE = 0x7fffffffffffffffLL;
  const score_t cand = take1 ? sc1 : v0 ? sc0 : NONE;
  score_t mn = cand;
  mn = min(mn, dpp64<DPP_ROR(8)>(mn, mn));
  mn = min(mn, dpp64<DPP_ROR(4)>(mn, mn));
  mn = min(mn, dpp64<DPP_ROR(2)>(mn, mn));
  mn = min(mn, dpp64<DPP_ROR(1)>(mn, mn));
  const bool path = mn < skip;   // group-uniform
  const uint64_t hit = __ballot(cand == mn && (v0 || v1));
  const int nstar = path ? __builtin_ctzll((hit >> g) & 0xffff) : -1;
  const int mstar = __shfl((int)take1, g + max(nstar, 0));
  // unwind the path: node(n) = predecessor bit of node(n + 1) at n + 1
  int B = path && act ? nstar - first + 1 : 0;
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) B = max(B, __shfl_xor(B, o));
  B = __builtin_amdgcn_readfirstlane(B);
  int nd = mstar;
  for (int r = 0; r < B; ++r) {
    const int t = dpp_pin<0x101>(0, (pv >> nd) & 1);   // row_shl:1: lane n + 1's predecessor bit
    nd = n == nstar ? mstar : t;
  }
  if constexpr (DBG) {
    long long* d = dbg + 16 * lane;
    d[0] = S0; d[1] = S1; d[2] = pv; d[3] = level0; d[4] = live1; d[5] = t00; d[6] = t01;
    d[7] = t10; d[8] = t11; d[9] = base0; d[10] = base1; d[11] = nstar; d[12] = mstar;
    d[13] = nd; d[14] = cand; d[15] = ((long long)R << 32) | (uint32_t)B;
  }
  Trellis16 res;
  const int lvl = level0 + nd;
  res.lvz = (path && act && n >= first && n <= nstar) ? (sign ? -lvl : lvl) : 0;
  res.nz = ((__ballot(res.lvz != 0) >> g) & 0xffff) != 0;
  const int j = lane & 15;
  res.level = __shfl(res.lvz, g + zz_inv(j));
  res.dq = (int16_t)(res.level * (int)M.q[j]);   // in[j] = out[n] * q_[j] (int16_t)
  return res;
}

// ---------------------------------------------------------------------------
// Intra16 candidates (quant_enc.c:772-822 ReconstructIntra16, cost_enc.c:232-256
// VP8GetCostLuma16). Wave m = mode m. Fills rec16/lv16/lvdc and
// mres[m] = {SSE, texture distortion, rate, nz (ac bits | dc << 24)}.

template <bool TRELLIS>
__device__ void eval_i16(const K3G& G, K3S& L, const vp8g_seg& S,
                         const MBCtx& ctx, int tid, K3S& B) {
  const int m = tid >> 6, lane = tid & 63, g = lane & 48, j = lane & 15, x = j & 3, y = j >> 2;
  const int bsub = lane >> 4;
  int co[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int b = 4 * p + bsub, px = 4 * (b & 3) + x, py = 4 * (b >> 2) + y;
    const int d = L.yin[py * BPS + px] - L.p16[m][py * 16 + px];
    co[p] = fdct_lane(d, j);
    if (j == 0) L.dcs[m][b] = (int16_t)co[p];
  }
  wsync();   // the DC terms of this mode: written and read by its own wave
  if (lane < 16) {   // FTransformWHT + y2 quantisation, coefficient b = lane
    const int16_t* d = L.dcs[m];
    const int b = lane, r = b >> 2, col = b & 3;
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
    int dq;
    const int level = quant_lane(v, b, S.y2, dq);
    L.lvdc[m][zz_inv(b)] = (int16_t)level;
    L.whtq[m][b] = (int16_t)dq;
  }
  int lv[4], dq[4];
  if constexpr (TRELLIS) {
    // quant_enc.c:790-803: the 16 blocks in anti-diagonal order, each
    // block's context from the trellis results of the blocks above and to
    // its left. Step st: group bx (= bsub) takes block (bx, st - bx) -- up to
    // four blocks at once, one per 16-lane group of the mode's wave; the nz
    // bits stay in a wave-uniform mask (no worker barrier)
    uint32_t tnz = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) { lv[p] = 0; dq[p] = 0; }
    for (int st = 0; st < 7; ++st) {
      const int bx = bsub, by = st - bsub;
      const bool on = by >= 0 && by < 4;
      const int byc = on ? by : 0;
      const int cst = byc == 0 ? co[0] : byc == 1 ? co[1] : byc == 2 ? co[2] : co[3];
      const int tc = byc == 0 ? ctx.top(bx) : (int)((tnz >> (4 * (byc - 1) + bx)) & 1);
      const int lc = bx == 0 ? ctx.left(byc) : (int)((tnz >> (4 * byc + bx - 1)) & 1);
      const Trellis16 t = trellis16(G, j == 0 ? 0 : cst, on, tc + lc, 0, S.y1,
                                    S.lambda_trellis_i16);
      const uint64_t bal = __ballot(on && t.nz && j == 0);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if ((bal >> (16 * q)) & 1) tnz |= 1u << (4 * (st - q) + q);
      if (on) L.lv16[m][4 * byc + bx][j] = (int16_t)t.lvz;   // zigzag order (lane & 15 = n)
#pragma unroll
      for (int p = 0; p < 4; ++p)
        if (on && byc == p) { lv[p] = j == 0 ? 0 : t.level; dq[p] = j == 0 ? 0 : t.dq; }
    }
  } else {   // quant_enc.c:805-812: DC position zeroed before QuantizeBlock
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int b = 4 * p + bsub;
      lv[p] = quant_lane(j == 0 ? 0 : co[p], j, S.y1, dq[p]);
      L.lv16[m][b][zz_inv(j)] = (int16_t)lv[p];
    }
  }
  // nz bit per block of this mode
  uint32_t nzm = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint64_t bal = __ballot(lv[p] != 0);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      nzm |= (((bal >> (16 * q)) & 0xffff) ? 1u : 0u) << (4 * p + q);
  }
  // AC rate while the levels are in registers
  int rate = 0;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int b = 4 * p + bsub, bx = b & 3, by = b >> 2;
    const int tctx = by == 0 ? ctx.top(bx) : (int)((nzm >> (b - 4)) & 1);
    const int lctx = bx == 0 ? ctx.left(by) : (int)((nzm >> (b - 1)) & 1);
    const int r = rate_lane(G, lv[p], j, g, tctx + lctx, 0, 1);
    if (j == 0) rate += r;
  }
  wsync();   // whtq complete (this mode's wave only)
  // inverse WHT (dec.c:137-162): lane b < 16 of the mode's wave computes the
  // DC of block b once; each block's coefficient-0 lane takes it by a shuffle
  {
    int dcv = 0;
    if (lane < 16) {
      const int16_t* q = L.whtq[m];
      const int b = lane, r = b >> 2, col = b & 3;
      int t[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int a0 = q[i] + q[12 + i], a1 = q[4 + i] + q[8 + i];
        const int a2 = q[4 + i] - q[8 + i], a3 = q[i] - q[12 + i];
        t[i] = r == 0 ? a0 + a1 : r == 1 ? a3 + a2 : r == 2 ? a0 - a1 : a3 - a2;
      }
      const int dd = t[0] + 3;
      const int a0 = dd + t[3], a1 = t[1] + t[2], a2 = t[1] - t[2], a3 = dd - t[3];
      dcv = (int16_t)((col == 0 ? a0 + a1 : col == 1 ? a3 + a2 : col == 2 ? a0 - a1 : a3 - a2) >> 3);
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int v = __shfl(dcv, 4 * p + bsub);
      if (j == 0) dq[p] = v;
    }
  }
  // reconstruction, SSE, texture distortion
  int sse = 0, tds = 0;
  const int wj = G.wy[j];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int b = 4 * p + bsub, px = 4 * (b & 3) + x, py = 4 * (b >> 2) + y;
    const int pr = L.p16[m][py * 16 + px];
    const int src = L.yin[py * BPS + px];
    const int rec = idct_lane(dq[p], pr, j);
    L.rec16[m][py * 16 + px] = (uint8_t)rec;
    sse += (src - rec) * (src - rec);
    const int td = sum16(ttrans_lane(rec, j, wj)) - L.hsrc[b];
    if (j == 0) tds += iabs_(td) >> 5;
  }
  sse = sum64(sse);
  tds = sum64(tds);
  rate = sum64(rate);
  // DC block rate: lanes 0..15 hold the WHT levels in natural order
  int dcl = 0;
  if (lane < 16) dcl = L.lvdc[m][zz_inv(lane)];
  const int dcnz = __ballot(lane < 16 && dcl != 0) != 0;
  const int rdc = rate_lane(G, dcl, lane & 15, 0, ctx.top(8) + ctx.left(8), 1, 0);
  if (lane == 0) {
    L.mres[m][0] = sse;
    L.mres[m][1] = tds;
    L.mres[m][2] = rate + rdc;
    L.mres[m][3] = (int)(nzm | (dcnz ? (1u << 24) : 0u));
  }
  wbar(B);   // (B: the worker running this, L: the MB state it evaluates)
}

// ---------------------------------------------------------------------------
// Chroma candidates (quant_enc.c:875-969 ReconstructUV + CorrectDCValues,
// cost_enc.c:258-278 VP8GetCostUV). Wave m = mode m, 8 blocks in 2 passes.
// mres[m] = {SSE, rate, non-zero AC count, nz bits}.

__device__ void eval_uv(const K3G& G, K3S& L, const vp8g_seg& S, const MBCtx& ctx, int tid, int x0,
                        const int8_t* topderr, int use_derr, K3S& B) {
  const int m = tid >> 6, lane = tid & 63, g = lane & 48, j = lane & 15, x = j & 3, y = j >> 2;
  const int bsub = lane >> 4;
  int co[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int b = 4 * p + bsub, ch = b >> 2, k4 = b & 3;
    const int px = 8 * ch + 4 * (k4 & 1) + x, py = 4 * (k4 >> 1) + y;
    const int d = L.yin[py * BPS + 16 + px] - L.puv[m][py * 16 + px];
    co[p] = fdct_lane(d, j);
    if (j == 0) L.uvdc[m][b] = (int16_t)co[p];
  }
  wsync();   // uvdc of this mode: its own wave
  if (use_derr && lane < 2) {   // CorrectDCValues (quant_enc.c:875-906)
    const int cch = lane;
    const vp8g_mtx& M = S.uv;
    const int8_t* top = topderr + 4 * x0 + 2 * cch;
    const int8_t* left = L.lderr[cch];
    int16_t* cc = &L.uvdc[m][4 * cch];
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
    L.uvderr[m][cch][0] = (int8_t)err[1];
    L.uvderr[m][cch][1] = (int8_t)err[2];
    L.uvderr[m][cch][2] = (int8_t)err[3];
  }
  wsync();   // CorrectDCValues results: this mode's wave
  int lv[2], dq[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int b = 4 * p + bsub;
    const int cv = j == 0 ? L.uvdc[m][b] : co[p];
    lv[p] = quant_lane(cv, j, S.uv, dq[p]);
    L.lvuv[m][b][zz_inv(j)] = (int16_t)lv[p];
  }
  uint32_t nzm = 0;
  int flatc = 0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const uint64_t bal = __ballot(lv[p] != 0);
    const uint64_t bac = __ballot(lv[p] != 0 && j != 0);
    flatc += __popcll(bac);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      nzm |= (((bal >> (16 * q)) & 0xffff) ? 1u : 0u) << (4 * p + q);
  }
  int rate = 0, sse = 0;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int b = 4 * p + bsub, ch = b >> 2, k4 = b & 3, bx = k4 & 1, by = k4 >> 1;
    const int tctx = by == 0 ? ctx.top(4 + 2 * ch + bx) : (int)((nzm >> (b - 2)) & 1);
    const int lctx = bx == 0 ? ctx.left(4 + 2 * ch + by) : (int)((nzm >> (b - 1)) & 1);
    const int r = rate_lane(G, lv[p], j, g, tctx + lctx, 2, 0);
    if (j == 0) rate += r;
    const int px = 8 * ch + 4 * bx + x, py = 4 * by + y;
    const int pr = L.puv[m][py * 16 + px];
    const int src = L.yin[py * BPS + 16 + px];
    const int rec = idct_lane(dq[p], pr, j);
    L.recuv[m][py * 16 + px] = (uint8_t)rec;
    sse += (src - rec) * (src - rec);
  }
  sse = sum64(sse);
  rate = sum64(rate);
  if (lane == 0) {
    L.mres[m][0] = sse;
    L.mres[m][1] = rate;
    L.mres[m][2] = flatc;
    L.mres[m][3] = (int)nzm;
  }
  wbar(B);
}

// ---------------------------------------------------------------------------
// Intra4 (quant_enc.c:1072-1165 PickBestIntra4; ReconstructIntra4 :825-858).
// Threads 0..159 = 10 modes x 16 coefficients. search: RD choice; the
// reference's early-skip inside the mode loop never changes the winner
// (the skipped score only grows), so the choice is an argmin with ties to
// the lower mode. !search: the m5 SimpleQuantize pass over L.modes
// (quant_enc.c:1230-1240), with trellis contexts from the MB boundary only,
// as in the reference. Reconstruction lands in acc_out, levels in acc_ac.

// Diagnostic build only (-DK3_SUBPROF): cycle split of the intra4 loop; a
// stamp waits for outstanding LDS ops, so that build's total runs slower.
#ifdef K3_SUBPROF
__device__ __forceinline__ uint64_t k3_clock() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define SUBST(i)                      \
  do {                                \
    const uint64_t t_ = k3_clock();   \
    sp[i] += t_ - sp_last;            \
    sp_last = t_;                     \
  } while (0)
#else
#define SUBST(i) \
  do {           \
  } while (0)
#endif

constexpr score_t kI4NoBound = (score_t)0x7fffffffffffffffll;

// a search's result is the same in every lane; read back through
// readfirstlane, branches on it are scalar
__device__ __forceinline__ score_t uni64(score_t v) {
  const uint64_t u = (uint64_t)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
  return (score_t)(((uint64_t)hi << 32) | lo);
}

struct I4Result {
  int ok;
  score_t H, score;
  uint32_t nz;
};


// Branch-free 4x4 intra predictor sample (src/dsp/enc.c:351-512) for this
// lane's (mode, pixel): pred = clip((wa*ea + wb*eb + wc*ec + rnd) >> sh) over
// edge samples e = L K J I X A B C D E F G H read straight from the canvas;
// DC averages 8 edges.
struct P4Lane {
  int8_t ia, ib, ic, wa, wb, wc, rnd, sh;
  int dc;
};
__device__ __forceinline__ P4Lane p4_lane(const P4Op& op, int x, int y) {
  P4Lane r;
  r.dc = op.kind == 4;
  if (op.kind == 0) {        // AVG3(a, b, c) = (a + 2b + c + 2) >> 2
    r.ia = op.a; r.ib = op.b; r.ic = op.c; r.wa = 1; r.wb = 2; r.wc = 1; r.rnd = 2; r.sh = 2;
  } else if (op.kind == 1) { // AVG2(a, b) = (a + b + 1) >> 1
    r.ia = op.a; r.ib = op.b; r.ic = 0; r.wa = 1; r.wb = 1; r.wc = 0; r.rnd = 1; r.sh = 1;
  } else if (op.kind == 2) { // copy
    r.ia = op.a; r.ib = 0; r.ic = 0; r.wa = 1; r.wb = 0; r.wc = 0; r.rnd = 0; r.sh = 0;
  } else if (op.kind == 3) { // TM: clip(top[x] + left[y] - corner)
    r.ia = 5 + x; r.ib = 3 - y; r.ic = 4; r.wa = 1; r.wb = 1; r.wc = -1; r.rnd = 0; r.sh = 0;
  } else {                   // DC
    r.ia = 0; r.ib = 0; r.ic = 0; r.wa = 0; r.wb = 0; r.wc = 0; r.rnd = 0; r.sh = 0;
  }
  return r;
}
// canvas byte offset of edge k (L K J I X A B C D E F G H) from the base of
// its sub-block (row 4 by, column 4 bx): rows of 24 bytes, row 0 = the row
// above the MB, column 0 = the column left of it. Left edges are the column
// before the sub-block, the others the row above it (incl. the top-right
// samples, which run_i4 places beside rows 4 / 8 / 12 for bx = 3).
__device__ __forceinline__ int edge_off0(int k) {
  // arithmetic select: as a ternary the compiler emitted a divergent if / else
  // per call, a place where it then parked register copies
  const int m = -(int)(k < 4);
  return (((4 - k) * 24) & m) | ((k - 4) & ~m);
}

// HPB (K3X helper pairs): the search starts without the intra-16 bound and
// takes it (*bound) once *bound_flag >= bound_at, i.e. once the helper has
// published its intra-16 choice: from then on it ends early like the
// sequential search (the same choice: the running score only grows). The
// flag is read by wave 0 before a sub-block's barrier and handed to the
// other waves through L.redw[2 + parity] (two slots: wave 0 can store the
// next sub-block's reading before a slower wave has read this one's), so
// all waves switch together.
template <bool TRELLIS, bool HPB = false>
__device__ I4Result run_i4(const K3G& G, K3S& L, const vp8g_seg& S,
                           const MBCtx& ctx, int tid, int x0,
                           int mbw, const uint8_t* predtop, const uint8_t* yl,
                           const uint8_t* yt, bool search, score_t rd_score, int max_bits,
                           uint64_t* sp, const int32_t* bound_flag = nullptr,
                           int32_t bound_at = 0, const score_t* bound = nullptr) {
#ifdef K3_SUBPROF
  uint64_t sp_last = k3_clock();
#endif
  for (int k = tid; k < 21; k += K3T) {
    uint8_t v;
    if (k == 0) v = yl[-1];
    else if (k <= 16) v = yt[k - 1];
    else v = (x0 < mbw - 1) ? yt[16 + k - 17] : yt[15];
    L.canvas[0][k] = v;
  }
  if (tid < 16) L.canvas[1 + tid][0] = yl[tid];
  // the top-right samples of the right column's sub-blocks (bx = 3, by > 0)
  // are the MB above-right's (row 0, columns 17..20): copied to rows 4, 8,
  // 12 so that every edge sample sits at sub-block base + a fixed offset
  if (tid >= 64 && tid < 76) {
    const int k = tid - 64;
    L.canvas[4 * (1 + (k >> 2))][17 + (k & 3)] = (x0 < mbw - 1) ? yt[16 + (k & 3)] : yt[15];
  }
  const int m = tid >> 4, j = tid & 15, g = (tid & 63) & 48, x = j & 3, y = j >> 2;
  const bool act = tid < 160;
  const int wj = G.wy[j];
  const P4Lane pl = p4_lane(G.p4[act ? tid : 0], x, y);
  const int offa = edge_off0(pl.ia), offb = edge_off0(pl.ib), offc = edge_off0(pl.ic);
  // left-edge samples (L K J I = column 3 of the sub-block to the left, rows
  // 3..0): during the search they come from the winning candidate's row of
  // rec4 -- the sub-block to the left was decided by the barrier just passed,
  // its winner's commit to the canvas is not ordered before this read
  const int la = pl.ia < 4 ? 4 * (3 - pl.ia) + 3 : -1;
  const int lb = pl.ib < 4 ? 4 * (3 - pl.ib) + 3 : -1;
  const int lc = pl.ic < 4 ? 4 * (3 - pl.ic) + 3 : -1;
  // this lane's y1 quantiser entries, once per MB
  const vp8g_mtx& M = S.y1;
  const uint32_t q_sh = M.sharpen[j], q_zt = M.zthresh[j], q_iq = M.iq[j], q_bias = M.bias[j];
  const int q_q = M.q[j];
  const uint8_t* cv = &L.canvas[0][0];
  uint32_t tnz = ctx.t & 0xf, lnz = ctx.l & 0xf;
  score_t acc_score = (score_t)211 * S.lambda_mode, accH = 211;
  uint32_t acc_nz = 0;
  int total_hdr = 0;
  I4Result res;
  res.ok = 1;
  if (tid == 0) { L.best4[0] = ~0ull; L.best4[1] = ~0ull; L.d4acc = 0; L.r4acc = 0; }
  WB();
  int prev_bm = 0;   // the mode chosen for the previous sub-block (worker-uniform)
  for (int i4 = 0; i4 < 16; ++i4) {
    const int bx = i4 & 3, by = i4 >> 2, par = i4 & 1;
    const int left_m = bx == 0 ? L.predleft[by] : search ? prev_bm : L.modes[i4 - 1];
    const int top_m = by == 0 ? predtop[4 * x0 + bx] : L.modes[i4 - 4];
    const int ctx4 = (int)((tnz >> bx) & 1) + (int)((lnz >> by) & 1);
    // the worker's 4th wave (rtid 192..255) holds no mode: it skips straight
    // to the barrier, leaving its SIMD's issue slots to the other workers
    const bool busy = (tid >> 6) != 3;   // wave-uniform
    const int src = L.yin[(4 * by + y) * BPS + 4 * bx + x];
    int pr = 0, rec = 0, nzb = 0;
    int level = 0, dq = 0;
    if (busy) {
    {
      const uint8_t* cb = cv + 96 * by + 4 * bx;   // sub-block base (worker-uniform)
      const bool lft = search && bx > 0;          // worker-uniform
      const uint8_t* rl = &L.rec4[par ^ 1][prev_bm][0];
      const int ea = *(lft && la >= 0 ? rl + la : cb + offa);
      const int eb = *(lft && lb >= 0 ? rl + lb : cb + offb);
      const int ec = *(lft && lc >= 0 ? rl + lc : cb + offc);
      pr = clip8((pl.wa * ea + pl.wb * eb + pl.wc * ec + pl.rnd) >> pl.sh);
      if (pl.dc) {
        int s4 = 4;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          s4 += *(lft ? rl + 4 * (3 - k) + 3 : cb + edge_off0(k)) + cb[edge_off0(5 + k)];
        pr = s4 >> 3;
      }
    }
    SUBST(0);
    const int c = fdct_lane(src - pr, j);
    SUBST(1);
    if constexpr (TRELLIS) {   // one mode per 16-lane group, no worker barrier
      const Trellis16 t = trellis16(G, c, act, ctx4, 3, S.y1, S.lambda_trellis_i4);
      level = t.level;
      dq = t.dq;
    } else {   // QuantizeBlock_C (src/dsp/enc.c:653-677)
      const int neg = c < 0;
      const uint32_t coeff = (uint32_t)(neg ? -c : c) + q_sh;
      level = min((int)((__umul24(coeff, q_iq) + q_bias) >> QFIX), MAX_LEVEL);
      level = coeff > q_zt ? level : 0;
      level = neg ? -level : level;
      dq = (int16_t)__mul24(level, q_q);
    }
    SUBST(2);
    rec = idct_lane(dq, pr, j);
    const uint64_t bnz = __ballot(act && level != 0);
    const uint64_t bac = __ballot(act && level != 0 && j != 0);
    nzb = ((bnz >> g) & 0xffff) != 0;
    SUBST(3);
    if (search) {
      const int D = sum16((src - rec) * (src - rec));
      int SD = 0;
      if (S.tlambda) {
        const int td = sum16(ttrans_lane(rec, j, wj)) - L.hsrc[i4];
        SD = (S.tlambda * (iabs_(td) >> 5) + 128) >> 8;
      }
      SUBST(4);
      const int cntnz = __popcll((bac >> g) & 0xffff);
      const int R0 = (m > 0 && cntnz <= 3) ? 140 : 0;
      const int Rc = rate_lane(G, level, j, g, ctx4, 3, 0);
      if (act) L.rec4[par][m][j] = (uint8_t)rec;
      if (act && j == 0) {
        const int H = G.mcost4[(top_m * 10 + left_m) * 10 + m];
        const score_t dist = 256 * (score_t)(D + SD);
        const score_t sc = (score_t)(R0 + Rc + H) * S.lambda_i4 + dist;
        atomicMin(&L.best4[i4 % 3], ((unsigned long long)sc << 4) | (unsigned)m);
        L.sm4[par][m] = (score_t)(R0 + Rc + H) * S.lambda_mode + dist;
        L.r4[par][m][0] = H;
        L.r4[par][m][1] = nzb;
        L.r4[par][m][2] = R0 + Rc;
        L.r4[par][m][3] = D;
      }
    }
    }   // busy
    SUBST(5);
    bool hpb_have = false;
    if constexpr (HPB) {
      hpb_have = rd_score != kI4NoBound;
      if (!hpb_have && tid < 64)   // (a whole wave: a lone-lane store here spills)
        L.redw[2 + (i4 & 1)] =
            __hip_atomic_load(bound_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= bound_at;
    }
    WB();
    if constexpr (HPB) {
      if (!hpb_have && __builtin_amdgcn_readfirstlane(L.redw[2 + (i4 & 1)])) rd_score = *bound;
    }
    int bm;
    if (search) {
      // argmin, ties to the lower mode. The slot read here was last written
      // before this barrier; the one reset here (used two sub-blocks on) was
      // last read before it (three slots, so no second barrier is needed)
      bm = (int)(L.best4[i4 % 3] & 15);
      if (tid == 0) {
        L.best4[(i4 + 2) % 3] = ~0ull;
        L.d4acc += L.r4[par][bm][3];
        L.r4acc += L.r4[par][bm][2];
      }
      const int H = L.r4[par][bm][0], bnzv = L.r4[par][bm][1];
      accH += H;
      acc_score += L.sm4[par][bm];
      acc_nz |= (uint32_t)bnzv << i4;
      if (acc_score >= rd_score) { res.ok = 0; break; }
      total_hdr += H;
      if (total_hdr > max_bits) { res.ok = 0; break; }
      tnz = (tnz & ~(1u << bx)) | ((uint32_t)bnzv << bx);
      lnz = (lnz & ~(1u << by)) | ((uint32_t)bnzv << by);
    } else {
      bm = L.modes[i4];
    }
    SUBST(6);
    if (act && m == bm) {   // the winning mode's lanes commit their own results
      L.canvas[4 * by + 1 + y][4 * bx + 1 + x] = (uint8_t)rec;
      L.acc_out[(4 * by + y) * 16 + 4 * bx + x] = (uint8_t)rec;
      L.acc_ac[i4][zz_inv(j)] = (int16_t)level;
      if (!search && j == 0) L.nzsel = nzb;
    }
    if (search && tid == 0) L.modes[i4] = (uint8_t)bm;
    prev_bm = bm;
    // the search needs no second barrier: the next sub-block reads its left
    // edge from rec4 (above), every other canvas sample it reads was committed
    // before an earlier barrier, and L.modes[i4] is read 4 sub-blocks on
    if (!search) {
      WB();
      acc_nz |= (uint32_t)L.nzsel << i4;
    }
    SUBST(7);
  }
  WB();
  res.H = accH;
  res.score = acc_score;
  res.nz = acc_nz;
  return res;
}

// ---------------------------------------------------------------------------

// The tokens of zigzag position n of one block (VP8RecordCoeffTokens,
// token_enc.c:113-193, restated per position): the "more coefficients"
// check (only at the first position and after a non-zero level), the zero
// check and, for a non-zero level, its value tokens and sign. The context of
// position n is the previous level. Returns the token count; EMIT writes the
// tokens and adds their statistics to the worker's pending deltas.
template <bool EMIT>
__device__ __forceinline__ int pos_tokens(int type, int first, int ctx0, int n, int c,
                                          int cprev, int last, uint16_t* out, uint32_t* delta) {
  if (n < first) return 0;
  const int vprev = iabs_(cprev);
  if (n > first && vprev == 0 && n > last) return 0;
  const int ctx = n == first ? ctx0 : (vprev >= 2 ? 2 : vprev);
  const int base = 11 * (ctx + 3 * (band_of(n) + 8 * type));
  int count = 0;
  auto dyn = [&](int bit, int pid, int sid) -> int {
    if (EMIT) {
      out[count] = (uint16_t)((bit << 15) | pid);
      atomicAdd(&delta[sid], 0x10000u + (uint32_t)bit);   // folded in raster order later
    }
    ++count;
    return bit;
  };
  auto fix = [&](int bit, int proba) {
    if (EMIT) out[count] = (uint16_t)((bit << 15) | (1 << 14) | proba);
    ++count;
  };
  if (n == first || vprev != 0) {
    if (!dyn(n <= last, base + 0, base + 0)) return count;
  }
  const int neg = c < 0;
  const uint32_t v = neg ? -c : c;
  if (!dyn(v != 0, base + 1, base + 1)) return count;
  if (!dyn(v > 1, base + 2, base + 2)) {
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
        dyn(1, base + 8, base + 8); dyn(0, base + 10, base + 9);  // token_enc.c:168
        res -= 8 << 2; mask = 1 << 4; tab = kVP8Cat5;
      } else {
        dyn(1, base + 8, base + 8); dyn(1, base + 10, base + 9);
        res -= 8 << 3; mask = 1 << 10; tab = kVP8Cat6;
      }
      for (; mask; mask >>= 1) fix((res & mask) != 0, *tab++);
    }
  }
  fix(neg, 128);
  return count;
}

// pos_tokens' token count without its branches (selects only): the header
// token (first position or after a non-zero level; alone when n > last), the
// zero check, and for a non-zero level the v > 1 check, the value tokens of
// its range (2..4: 2 + (v != 2); 5..10: 3 + (v <= 6 ? 1 : 2); 11+: 4 + the
// category's extra bits 3 / 4 / 5 / 11) and the sign
__device__ __forceinline__ int pos_count(int first, int n, int c, int cprev, int last) {
  const int vprev = iabs_(cprev), v = iabs_(c);
  const int none = (n < first) | ((n > first) & (vprev == 0) & (n > last));
  const int hdr = (n == first) | (vprev != 0);
  const int res = v - 3;
  const int nextra = res < 16 ? 3 : res < 32 ? 4 : res < 64 ? 5 : 11;
  const int big = v <= 4 ? 2 + (v != 2) : v <= 10 ? 3 + 1 + (v > 6) : 4 + nextra;
  const int body = 1 + (v != 0 ? 2 + (v > 1 ? big : 0) : 0);
  const int cnt = (hdr & (n > last)) ? 1 : hdr + body;
  return none ? 0 : cnt;
}

// FinalizeTokenProbas (frame_enc.c:146-180) over the workgroup; returns the
// reference's "dirty" flag (some probability differs from the default).
__device__ int finalize_probas_wg(K3G& G, K3S& L, int tid) {
  if (tid == 0) G.dirty = 0;
  WB();
  int changed = 0;
  for (int s = tid; s < NSLOT; s += K3T) {
    const uint32_t st = G.stats[s];
    const int nb = st & 0xffff, total = (st >> 16) & 0xffff;
    const int upd = (&kVP8CoeffUpdateProba[0][0][0][0])[s];
    const int old_p = (&kVP8CoeffProba0[0][0][0][0])[s];
    const int new_p = nb ? (255 - nb * 255 / total) : 255;
    const int old_cost = nb * bit_cost(G.ecost, 1, old_p) + (total - nb) * bit_cost(G.ecost, 0, old_p) +
                         bit_cost(G.ecost, 0, upd);
    const int new_cost = nb * bit_cost(G.ecost, 1, new_p) + (total - nb) * bit_cost(G.ecost, 0, new_p) +
                         bit_cost(G.ecost, 1, upd) + 8 * 256;
    if (old_cost > new_cost) {
      G.coeffs[s] = new_p;
      changed |= (new_p != old_p);
    } else {
      G.coeffs[s] = old_p;
    }
  }
  if (changed) G.dirty = 1;
  WB();
  return G.dirty;
}

// bit costs of the first probability of every (type, band, ctx): read by
// rate_lane for the block-header and end-of-block bits; refreshed at every
// FinalizeTokenProbas since the probabilities change even when the level
// cost tables are not recomputed
__device__ __forceinline__ void refresh_hc(K3G& G, int tid) {
  for (int k = tid; k < 96; k += K3T) {
    const int p = G.coeffs[k * 11];
    G.hc[k][0] = bit_cost(G.ecost, 0, p);
    G.hc[k][1] = bit_cost(G.ecost, 1, p);
  }
}

// Stage cycle accounting only in the diagnostic builds (-DK3_STAMPS for the
// coarse stages, -DK3_SUBPROF for the intra4 split): the production kernel
// keeps no timers live across the MB loop.
#ifdef K3_STAMPS
#define K3_STAMP(i)                                   \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    stamps[i] += t_ - stamp_last;                     \
    stamp_last = t_;                                  \
  } while (0)
#else
#define K3_STAMP(i) \
  do {              \
  } while (0)
#endif

// Wait / stage accounting per worker (-DK3_TRACE, diagnostic build only; the
// product kernel has none of it): shader-clock cycles and event counts kept
// by each worker's thread 0 in LDS and written to g_k3trace at frame end
// (vp8g_k3_trace reads them back)
enum {
  K3TR_REFR_WAIT = 0,   // the refresher waiting for every earlier MB folded (site 1)
  K3TR_EPOCH_WAIT,      // other workers waiting for the epoch (site 2)
  K3TR_ROW_WAIT,        // the top-right wavefront wait (site 3)
  K3TR_FOLD_WAIT,       // row end: waiting for the rows above folded (site 4)
  K3TR_FOLD,            // fold_rows (row ends and epoch refreshes)
  K3TR_REPLAY,          // of which the in-order replay of marked counters
  K3TR_NREPLAY,         // marked counters replayed
  K3TR_REFRESH,         // FinalizeTokenProbas + level costs + header costs
  K3TR_MB,              // MB work (after the waits, to the MB's publish)
  K3TR_I4,              // intra-4 search
  K3TR_I16,             // intra-16 candidates
  K3TR_NMB,             // MBs
  K3TR_TOTAL,           // the worker's whole lifetime
  K3TR_NROWWAIT,        // wavefront waits that found the row above behind
  K3TR_TOK,             // per-MB info, SSE and tokens
  K3TR_UV,              // chroma candidates (+ the m5 re-quantisation)
  K3TR_N
};
#ifdef K3_TRACE
#define K3TR_MAXB 1024
static_assert(K3TR_N == 16, "L.trace[16]");
__device__ unsigned long long g_k3trace[K3TR_MAXB][4][K3TR_N];
#define TR_NOW() __builtin_amdgcn_s_memtime()
// (the worker's first wave adds, every lane the same value: a wave-uniform
// branch, no lane-masked region -- DESIGN.md section 9)
#define TR_ADD(slot, v)                                                          \
  do {                                                                           \
    if ((__builtin_amdgcn_readfirstlane(threadIdx.x) % K3T) < 64) L.trace[slot] += (v); \
  } while (0)
#define TR_SINCE(slot, t0) TR_ADD(slot, TR_NOW() - (t0))
#else
#define TR_NOW() 0ull
#define TR_ADD(slot, v) \
  do {                  \
  } while (0)
#define TR_SINCE(slot, t0) \
  do {                     \
  } while (0)
#endif

// ---------------------------------------------------------------------------
// Frame-level machinery: several workers encode MBs of different rows at the
// same time (a wavefront: row y may encode MB x once row y-1 has finished
// MB x+1, exactly the data the reference's iterator carries down: top,
// top-right, nz, I4 modes, U/V DC errors). The cost tables only change at the
// refresh points of VP8EncTokenLoop (frame_enc.c:785-832), so inside an
// epoch the wavefront reproduces the raster loop bit for bit; at an epoch
// boundary everything before it is finished and folded first. Token
// statistics are folded strictly in raster order (the saturating counters
// are order dependent) by the owner of each row at its row end, which also
// moves the row's tokens from per-MB slots to the compact stream.

// VP8CalculateLevelCosts (cost_enc.c:42-90) over one worker, no barrier
// from the probabilities src (G.coeffs, or the K3X copy of the last dirty epoch's)
__device__ void level_costs_w(K3G& G, const uint8_t* src, int tid) {
  for (int k = tid; k < 96 * (MAX_VLEVEL + 1); k += K3T) {
    const int tbc = k / (MAX_VLEVEL + 1), v = k % (MAX_VLEVEL + 1);
    const uint8_t* p = src + tbc * 11;
    const int ctx = tbc % 3;
    const int c0 = ctx > 0 ? bit_cost(G.ecost, 1, p[0]) : 0;
    int cost;
    if (v == 0) {
      cost = bit_cost(G.ecost, 0, p[1]) + c0;
    } else {
      cost = bit_cost(G.ecost, 1, p[1]) + c0;
      int pat = kVP8LevelCodes[v - 1][0], bits = kVP8LevelCodes[v - 1][1];
      for (int i = 2; pat; ++i, pat >>= 1, bits >>= 1)
        if (pat & 1) cost += bit_cost(G.ecost, bits & 1, p[i]);
    }
    G.lcost[tbc][v] = (uint16_t)(cost + kVP8LevelFixedCost[v]);
  }
}

// statistics slot of a dynamic token: its probability slot, except the
// second bit of the cat5/cat6 prefix, coded with probability base+10 but
// counted at base+9 (token_enc.c:168)
__device__ __forceinline__ int tok_stat_slot(uint32_t t) {
  const int id = (int)(t & 0x3fff);
  return (id % 11 == 10) ? id - 1 : id;
}

// worker-uniform wait until *p >= v (another worker of this workgroup publishes *p)
// (SL: s_sleep units between polls)
template <int SL = 2>
__device__ bool wait_ge(K3G& G, K3S& L, const int32_t* p, int32_t v, int site) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_uni(p, __ATOMIC_ACQUIRE) < v) {
    if (ld_uni(&G.abort) ||
        __builtin_amdgcn_s_memrealtime() - t0 > K3_WAIT_TICKS) {
#ifdef K3_CHECK
      if ((threadIdx.x & 255) == 0 && blockIdx.x < 1024) {
        uint32_t* hr = g_k3hang[blockIdx.x][(threadIdx.x >> 8) & 3];
        extern __shared__ __align__(16) uint8_t smem[];
        hr[0] = (uint32_t)site;
        hr[1] = (uint32_t)((uintptr_t)p - (uintptr_t)smem);
        hr[2] = (uint32_t)v;
        hr[3] = (uint32_t)__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        hr[4] = (uint32_t)L.ck_y;
        hr[5] = (uint32_t)L.ck_x;
        hr[6] = L.bar;
        hr[7] = 0x80000000u | (uint32_t)G.abort;
        hr[8] = L.ck_rowdone;
        hr[9] = (uint32_t)((uintptr_t)&G.fold_ptr - (uintptr_t)smem);
      }
#endif
      L.myabort = 1;
      atomicOr(&L.bar, WBAR_RELEASE);   // no wave of this worker waits at a barrier now
      if (!G.abort) G.abort = site;     // the wait that gave up (in the result's error)
      break;
    }
    __builtin_amdgcn_s_sleep(SL);
  }
  wbar(L);
  return L.myabort == 0;
}

// ---------------------------------------------------------------------------
// K3X: one frame over several workgroups. Everything handed from one
// workgroup to another goes through the frame's xsync block in HBM with
// write-through (sc1) stores and L1-bypassing (sc1) loads, drained by the
// storing wave before the flag that publishes it (the hand-off form of the
// microarchitecture guide's inter-workgroup visibility table, row 1):
//   rowdone[y]  MB columns of row y finished; rec[y][x] its boundary record
//               (bottom Y row, bottom U|V rows, nz word, I4 modes, DC errors)
//   fold_ptr    raster MBs whose statistics are folded; stats/ntok with it
//   epoch       cost-table epochs published; coeffs (current probabilities)
//               and lcoeffs/lcver (those of the last level-cost recompute)
struct XHdr {
  int32_t fold_ptr, epoch, abort, lcver;
  uint32_t ntok;
  int32_t tok_err, uabort, pad;   // uabort: the progress hook asked to stop
  unsigned long long size_p0, sse[3], dist, size_rh;
  int32_t nb[3], max_edge[4], pad2;
};
#define XS_HDR 128
static_assert(sizeof(XHdr) <= XS_HDR, "XHdr outgrew its slot");
#define XS_STATS XS_HDR
#define XS_COEFFS (XS_STATS + 4 * NSLOT)
#define XS_LCOEFFS (XS_COEFFS + NSLOT)
#define XS_ROWDONE (XS_LCOEFFS + NSLOT)
#define XS_REC_WORDS 12
#define XS_PULL_COLS 16   // boundary records one row-above wait may pull
static_assert(sizeof(XHdr) <= XS_HDR, "xsync header");
static_assert(NSLOT % 4 == 0, "probabilities move as words");

__host__ __device__ inline size_t xs_rec_off(int mbh) {
  return ((size_t)XS_ROWDONE + 4 * (size_t)mbh + 15) & ~(size_t)15;
}
// per row, every XS_SNAP_MBS MBs: the worker's pending statistics deltas
// (count << 16 | ones per slot, cumulative since the row's last fold point),
// so that a fold's replay finds the block holding a counter's halving point
// without scanning the row's tokens up to it
#ifndef K3_DFULL   // (a test build lowers it so that the early folds run)
#define K3_DFULL 0xc000u
#endif
#ifndef K3_DFULL_EVERY   // columns between two checks (a multiple of XS_SNAP_MBS)
#define K3_DFULL_EVERY 32
#endif
#ifndef XS_SNAP_MBS
#define XS_SNAP_MBS 16
#endif
static_assert(K3_DFULL + K3_DFULL_EVERY * 288 < 0x10000u, "pending deltas stay 16-bit");
static_assert(K3_DFULL_EVERY % XS_SNAP_MBS == 0, "checked at snapshot columns");
__host__ __device__ inline int xs_snaps_per_row(int mbw) { return (mbw + XS_SNAP_MBS - 1) / XS_SNAP_MBS; }
__host__ __device__ inline size_t xs_snap_off(int mbw, int mbh) {
  return (xs_rec_off(mbh) + 4 * XS_REC_WORDS * (size_t)mbw * mbh + 255) & ~(size_t)255;
}
__device__ __forceinline__ uint32_t* xs_snap_row(uint8_t* xs, int mbw, int mbh, int y) {
  return reinterpret_cast<uint32_t*>(xs + xs_snap_off(mbw, mbh)) +
         (size_t)y * xs_snaps_per_row(mbw) * NSLOT;
}
extern "C" size_t vp8g_wsnap_bytes(int w, int h) {
  (void)h;   // one row's snapshots per MB worker (at most 4 per frame)
  return 4 * 4 * (size_t)NSLOT * xs_snaps_per_row((w + 15) >> 4);
}
extern "C" size_t vp8g_xsync_bytes(int w, int h) {
  const int mbw = (w + 15) >> 4, mbh = (h + 15) >> 4;
  return (xs_snap_off(mbw, mbh) + 4 * (size_t)NSLOT * xs_snaps_per_row(mbw) * mbh + 255) &
         ~(size_t)255;
}

// LDS of one K3X workgroup beyond the K3 layout: the boundary of the row
// above its worker 0 (pulled from rec[]) and its level-cost bookkeeping
struct K3XL {
  uint8_t lcoeffs[NSLOT];
  int32_t lcver;    // lcver of the level costs in G.lcost
  int32_t claim;    // highest epoch some worker of this workgroup refreshes to
  // helper pairs (k_encode<.., HP>): worker 1 evaluates each MB's intra-16
  // and chroma candidates in worker 0's MB state while worker 0 runs the
  // intra-4 search; MBs handed over / finished (raster index + 1), the MB's
  // context, and the helper's two decisions
  int32_t hp_go, hp_done;
  int32_t hp_i16;            // MBs whose intra-16 choice (hp_rd16) is out (raster index + 1)
  int32_t hp_nseg;           // the segment of the MB whose source is in the helper's yin
  int32_t hp_pre;            // the MB whose source the helper has loaded into its yin (+ 1)
  int32_t hp_bnd;            // MBs whose boundary (ytop, uvtop, nzw, predtop, topderr) is out
  int32_t hp_tokgo, hp_tok;  // MBs handed to / tokenized by the helper (+ 1)
  uint32_t tk_ctx_t, tk_ctx_l;
  int32_t tk_first, tk_pad;  // the handed MB's context and first block (0: intra-16)
  uint32_t dk_ctx_t, dk_ctx_l;   // the same, of an MB whose tokens the helper put off
  int32_t dk_first, dk_pad;
  // intra-4 pairs (k_encode<3, .., HP, P3>): the partner's go (MB + 1) and
  // skip, the pair barrier, the decided sub-blocks' nz bits, the stop flags
  int32_t p_go, p_skip;
  uint32_t p_bar, p_pad;
  int32_t p_nz[16];
  int32_t p_stop[2];
  int32_t xseen[4];   // the main worker's waves' polls of the row above (wait_gx_seen)
  uint32_t hp_ctx_t, hp_ctx_l;
  int32_t hp_seg, hp_best16, hp_bu, hp_pad;
  uint32_t hp_nz16, hp_pad2;
  score_t hp_D16, hp_SD16, hp_H16, hp_R16, hp_bH, hp_bsc;
  score_t hp_rd16;   // the intra-16 choice's score with lambda_mode (the intra-4 bound)
};

__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ld_sc1(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// worker-uniform wait until the xsync word *p >= v; every wave polls it
// itself, so each wave's later sc1 loads follow its own matching poll
__device__ bool wait_gx(K3G& G, K3S& L, const int32_t* p, int32_t v, XHdr* XH) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_readfirstlane(ld_sc1(p)) < v) {
    if (ld_uni(&G.abort) || __builtin_amdgcn_readfirstlane(ld_sc1(&XH->abort)) ||
        __builtin_amdgcn_s_memrealtime() - t0 > K3_WAIT_TICKS) {
      L.myabort = 1;
      atomicOr(&L.bar, WBAR_RELEASE);
      G.abort = 1;
      st_sc1(&XH->abort, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  wbar(L);
  return L.myabort == 0;
}

// wait_gx that also hands back how far *p had got: the smallest of the
// waves' last polls (each >= v), so each wave's later sc1 loads of what that
// value covers still follow its own matching poll; slot: one word per wave
__device__ bool wait_gx_seen(K3G& G, K3S& L, const int32_t* p, int32_t v, XHdr* XH, int32_t* slot,
                             int tid, int32_t& seen) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  int32_t o;
  while ((o = __builtin_amdgcn_readfirstlane(ld_sc1(p))) < v) {
    if (ld_uni(&G.abort) || __builtin_amdgcn_readfirstlane(ld_sc1(&XH->abort)) ||
        __builtin_amdgcn_s_memrealtime() - t0 > K3_WAIT_TICKS) {
      L.myabort = 1;
      atomicOr(&L.bar, WBAR_RELEASE);
      G.abort = 1;
      st_sc1(&XH->abort, 1);
      break;
    }
    __builtin_amdgcn_s_sleep(4);
  }
  if ((tid & 63) == 0) slot[tid >> 6] = o;
  wbar(L);
  int32_t m = slot[0];
#pragma unroll
  for (int k = 1; k < K3T / 64; ++k) m = min(m, slot[k]);
  seen = __builtin_amdgcn_readfirstlane(m);
  return L.myabort == 0;
}

// probabilities between LDS and xsync, as words
__device__ __forceinline__ void probas_to_x(const uint8_t* src, uint8_t* xdst, int tid) {
  for (int k = tid; k < NSLOT / 4; k += K3T)
    st_sc1(reinterpret_cast<uint32_t*>(xdst) + k, reinterpret_cast<const uint32_t*>(src)[k]);
}
__device__ __forceinline__ void probas_from_x(uint8_t* dst, const uint8_t* xsrc, int tid) {
  for (int k = tid; k < NSLOT / 4; k += K3T)
    reinterpret_cast<uint32_t*>(dst)[k] = ld_sc1(reinterpret_cast<const uint32_t*>(xsrc) + k);
}

// the four 16x16 and four chroma predictions of an MB (quant_enc.c:469-479)
__device__ __forceinline__ void predict_mb(K3S& L, const uint8_t* yl, const uint8_t* ul,
                                           const uint8_t* vl, const uint8_t* yt, const uint8_t* uvt,
                                           bool hl, bool ht, int tid) {
  const int dcy = dc_value(yl, yt, hl, ht, 16, 5);
  for (int k = tid; k < 1024; k += K3T) {
    const int m = k >> 8, p = k & 255;
    L.p16[m][p] = pred_sample(m, 16, p & 15, p >> 4, yl, yt, hl, ht, dcy);
  }
  const int dcu = dc_value(ul, uvt, hl, ht, 8, 4);
  const int dcv = dc_value(vl, uvt + 8, hl, ht, 8, 4);
  for (int k = tid; k < 512; k += K3T) {
    const int m = k >> 7, p = k & 127, px = p & 15, py = p >> 4, c = px >> 3;
    L.puv[m][p] = pred_sample(m, 8, px & 7, py, c ? vl : ul, uvt + 8 * c, hl, ht, c ? dcv : dcu);
  }
}

__device__ __forceinline__ void publish(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// barrier of an intra-4 pair (the main and the partner worker: 8 waves),
// the worker barrier's form (wbar) with 8 arrivals per generation
__device__ __forceinline__ void pbar(uint32_t* ctr) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  const uint32_t old = lane0_add(ctr, 1u);
  const uint32_t target = (old & ~7u) + 8u;
  if ((old & 7u) != 7u)
    while (ld_uni(ctr) < target) __builtin_amdgcn_s_sleep(K3_WBAR_SLEEP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The intra-4 search of a helper pair with a partner worker (k_encode<3, ..,
// HP, P3>): the 16 sub-blocks in the wavefront order t = bx + 2 by, 10 steps,
// steps 2-7 holding two sub-blocks (kI4Pair: role 0 = the main worker, role 1
// = the partner). A sub-block's candidates depend only on the sub-blocks to
// its left, top, top-left and top-right, all decided at earlier steps, so
// every choice is the sequential search's (quant_enc.c:1072-1165); the
// running score, header bits and distortion / rate sums are the same sums in
// another order, and the search ends (i16 wins) exactly when the sequential
// one would, since those sums only grow. Per step: each worker evaluates its
// sub-block's 10 candidates (the canvas is complete: a second pair barrier
// after the commits), a pair barrier, both read the choices, the owners
// commit to the main's canvas / acc_out / acc_ac / modes, the main
// accumulates both and sets the stop flag, a second pair barrier.
__constant__ int8_t kI4Pair[10][2] = {{0, -1}, {1, -1}, {2, 4},  {3, 5},   {6, 8},
                                      {7, 9},  {10, 12}, {11, 13}, {14, -1}, {15, -1}};
template <bool TRELLIS>
__device__ I4Result run_i4_pair(const K3G& G, K3S& W, K3S& Lm, K3S& Lp, K3XL& XL, int role,
                                const vp8g_seg& S, const MBCtx& ctx, int tid, int x0, int mbw,
                                const uint8_t* predtop, const uint8_t* yl, const uint8_t* yt,
                                score_t rd_score, int max_bits, const int32_t* bound_flag,
                                int32_t bound_at, const score_t* bound) {
  if (role == 0) {   // the canvas (as run_i4), then the partner may start
    for (int k = tid; k < 21; k += K3T) {
      uint8_t v;
      if (k == 0) v = yl[-1];
      else if (k <= 16) v = yt[k - 1];
      else v = (x0 < mbw - 1) ? yt[16 + k - 17] : yt[15];
      Lm.canvas[0][k] = v;
    }
    if (tid < 16) Lm.canvas[1 + tid][0] = yl[tid];
    if (tid >= 64 && tid < 76) {
      const int k = tid - 64;
      Lm.canvas[4 * (1 + (k >> 2))][17 + (k & 3)] = (x0 < mbw - 1) ? yt[16 + (k & 3)] : yt[15];
    }
    if (tid == 0) { Lm.d4acc = 0; Lm.r4acc = 0; XL.p_stop[0] = 0; XL.p_stop[1] = 0; }
  }
  if (tid == 0) { W.best4[0] = ~0ull; W.best4[1] = ~0ull; W.best4[2] = ~0ull; }
  pbar(&XL.p_bar);
  const int m = tid >> 4, j = tid & 15, g = (tid & 63) & 48, x = j & 3, y = j >> 2;
  const bool act = tid < 160;
  const int wj = G.wy[j];
  const P4Lane pl = p4_lane(G.p4[act ? tid : 0], x, y);
  const int offa = edge_off0(pl.ia), offb = edge_off0(pl.ib), offc = edge_off0(pl.ic);
  const vp8g_mtx& M = S.y1;
  const uint32_t q_sh = M.sharpen[j], q_zt = M.zthresh[j], q_iq = M.iq[j], q_bias = M.bias[j];
  const int q_q = M.q[j];
  const uint8_t* cv = &Lm.canvas[0][0];
  score_t acc_score = (score_t)211 * S.lambda_mode, accH = 211;
  uint32_t acc_nz = 0;
  int total_hdr = 0;
  I4Result res;
  res.ok = 1;
  for (int t = 0; t < 10; ++t) {
    const int b = kI4Pair[t][role];   // worker-uniform
    const int par = t & 1;
    int rec = 0, level = 0, nzb = 0;
    if (b >= 0 && (tid >> 6) != 3) {   // (the 4th wave holds no mode)
      const int bx = b & 3, by = b >> 2;
      const int left_m = bx == 0 ? Lm.predleft[by] : Lm.modes[b - 1];
      const int top_m = by == 0 ? predtop[4 * x0 + bx] : Lm.modes[b - 4];
      const int tn = by == 0 ? (int)((ctx.t >> bx) & 1) : XL.p_nz[b - 4];
      const int ln = bx == 0 ? (int)((ctx.l >> by) & 1) : XL.p_nz[b - 1];
      const int ctx4 = tn + ln;
      const int src = Lm.yin[(4 * by + y) * BPS + 4 * bx + x];
      const uint8_t* cb = cv + 96 * by + 4 * bx;
      int pr = clip8((pl.wa * cb[offa] + pl.wb * cb[offb] + pl.wc * cb[offc] + pl.rnd) >> pl.sh);
      if (pl.dc) {
        int s4 = 4;
#pragma unroll
        for (int k = 0; k < 4; ++k) s4 += cb[edge_off0(k)] + cb[edge_off0(5 + k)];
        pr = s4 >> 3;
      }
      const int c = fdct_lane(src - pr, j);
      int dq;
      if constexpr (TRELLIS) {
        const Trellis16 tr = trellis16(G, c, act, ctx4, 3, S.y1, S.lambda_trellis_i4);
        level = tr.level;
        dq = tr.dq;
      } else {
        const int neg = c < 0;
        const uint32_t coeff = (uint32_t)(neg ? -c : c) + q_sh;
        level = min((int)((__umul24(coeff, q_iq) + q_bias) >> QFIX), MAX_LEVEL);
        level = coeff > q_zt ? level : 0;
        level = neg ? -level : level;
        dq = (int16_t)__mul24(level, q_q);
      }
      rec = idct_lane(dq, pr, j);
      const uint64_t bnz = __ballot(act && level != 0);
      const uint64_t bac = __ballot(act && level != 0 && j != 0);
      nzb = ((bnz >> g) & 0xffff) != 0;
      const int D = sum16((src - rec) * (src - rec));
      int SD = 0;
      if (S.tlambda) {
        const int td = sum16(ttrans_lane(rec, j, wj)) - Lm.hsrc[b];
        SD = (S.tlambda * (iabs_(td) >> 5) + 128) >> 8;
      }
      const int cntnz = __popcll((bac >> g) & 0xffff);
      const int R0 = (m > 0 && cntnz <= 3) ? 140 : 0;
      const int Rc = rate_lane(G, level, j, g, ctx4, 3, 0);
      if (act && j == 0) {
        const int H = G.mcost4[(top_m * 10 + left_m) * 10 + m];
        const score_t dist = 256 * (score_t)(D + SD);
        const score_t sc = (score_t)(R0 + Rc + H) * S.lambda_i4 + dist;
        atomicMin(&W.best4[t % 3], ((unsigned long long)sc << 4) | (unsigned)m);
        W.sm4[par][m] = (score_t)(R0 + Rc + H) * S.lambda_mode + dist;
        W.r4[par][m][0] = H;
        W.r4[par][m][1] = nzb;
        W.r4[par][m][2] = R0 + Rc;
        W.r4[par][m][3] = D;
      }
    }
    bool have = true;
    if (role == 0) {   // the intra-16 bound, as run_i4<.., HPB>
      have = rd_score != kI4NoBound;
      if (!have && tid < 64)
        Lm.redw[2 + par] =
            __hip_atomic_load(bound_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= bound_at;
    }
    pbar(&XL.p_bar);
    if (role == 0 && !have && __builtin_amdgcn_readfirstlane(Lm.redw[2 + par])) rd_score = *bound;
    if (b >= 0) {
      const int bm = (int)(W.best4[t % 3] & 15);
      const int bx = b & 3, by = b >> 2;
      if (act && m == bm) {   // the winning mode's lanes commit their own results
        Lm.canvas[4 * by + 1 + y][4 * bx + 1 + x] = (uint8_t)rec;
        Lm.acc_out[(4 * by + y) * 16 + 4 * bx + x] = (uint8_t)rec;
        Lm.acc_ac[b][zz_inv(j)] = (int16_t)level;
      }
      if (tid == 0) {
        Lm.modes[b] = (uint8_t)bm;
        XL.p_nz[b] = W.r4[par][bm][1];
        W.best4[(t + 2) % 3] = ~0ull;
      }
    }
    if (role == 0) {   // the main worker accumulates both sub-blocks, in block order
      bool stop = false;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int bb = kI4Pair[t][r];
        if (bb < 0) continue;
        const K3S& O = r == 0 ? W : Lp;
        const int bm = (int)(O.best4[t % 3] & 15);
        const int H = O.r4[par][bm][0], bnzv = O.r4[par][bm][1];
        if (tid == 0) {
          Lm.d4acc += O.r4[par][bm][3];
          Lm.r4acc += O.r4[par][bm][2];
        }
        accH += H;
        acc_score += O.sm4[par][bm];
        acc_nz |= (uint32_t)bnzv << bb;
        total_hdr += H;
      }
      stop = acc_score >= rd_score || total_hdr > max_bits;
      if (tid < 64) XL.p_stop[par] = stop;
    }
    pbar(&XL.p_bar);
    if (__builtin_amdgcn_readfirstlane(XL.p_stop[par])) { res.ok = 0; break; }
  }
  res.H = accH;
  res.score = acc_score;
  res.nz = acc_nz;
  return res;
}

// Fold MBs [i0, i1) into the statistics in raster order: each MB's tokens
// move from its slot to the compact stream while their statistics deltas
// accumulate; counters that would cross the halving threshold inside the MB
// are replayed token by token (VP8RecordStats, cost_enc.h:45-56).
// RD: 64-token chunks per replay step (K3X: 16, the batch kernels: 4, where
// deeper steps cost registers in the MB loop and the replay is ~2% anyway)
#ifndef K3_RD_X
#define K3_RD_X 8    // (config 4: 8 404 ms, 16 406, 32 518; r5s26)
#endif
#ifndef K3_RD_BATCH
#define K3_RD_BATCH 8   // (batch K3: 4 99.05 ms, 8 98.4; r5s26)
#endif
// The statistics fold is inlined into the MB loop (round 6): as an
// out-of-line call (b59c671 .. round 5) the worker's LDS state went to it as
// flat pointers and the caller saved its live registers to scratch around
// the call, and builds with that call faulted (illegal address) or hung
// depending on the code around it; inlined it also
// needs less scratch (headline kernel 120 -> 80 B/lane). -DK3_FOLD_CALL
// restores the call (A/B).
#ifdef K3_FOLD_CALL
#define K3_FOLD_ATTR __device__
#else
#define K3_FOLD_ATTR __device__ __forceinline__
#endif
template <int RD>
K3_FOLD_ATTR void fold_mbs(K3G& G, K3S& L, int tid, uint32_t i0, uint32_t i1, uint32_t row0,
                         uint16_t* tok_base, uint32_t* mboff, const uint16_t* rowbase,
                         const uint32_t* snap = nullptr) {
  const bool rows = rowbase != nullptr;   // token rows: this row's tokens at rowbase
  // MBs [i0, i1) of this worker's row (first MB row0): their token count
  // (and, in the slot layout, where their tokens go in the frame's compact
  // stream, moved there at frame end by compact_tokens), then their
  // statistics added in one step.
  // Called once every earlier MB is folded (G.fold_ptr == i0).
  const uint32_t base = G.ntok;
  const uint32_t ln = (uint32_t)tid & 63;
  if (tid < 64) {   // compact-stream offsets: a wave scan over the MBs, 64 at a time
    uint32_t off = base;
    for (uint32_t c = i0; c < i1; c += 64) {
      const uint32_t i = c + ln;
      const uint32_t v = i < i1 ? L.rowcnt[i - row0] : 0u;
      uint32_t incl = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o);
        if (ln >= (uint32_t)o) incl += u;
      }
      if (!rows && i < i1 && K3CK(i < CK_NMB(L, i + 1), 10, i, 0, i)) mboff[i] = off + incl - v;
      off += __shfl(incl, 63);
    }
    if (ln == 0) { L.fold_total = off - base; L.fold_base = base; L.mark_any = 0; }
  }
  wbar(L);
  const uint32_t total = L.fold_total;
  // statistics: one add per counter unless it would reach the halving point
  // (VP8RecordStats, cost_enc.h:50-57), then an in-order replay of that counter
  for (int s = tid; s < NSLOT; s += K3T) {
    const uint32_t dlt = L.rdelta[s];
    if (dlt) {
      const uint32_t p = G.stats[s];
      if ((p >> 16) + (dlt >> 16) < 0xffffu) {
        G.stats[s] = p + dlt;
        L.rdelta[s] = 0;
      } else {   // the delta stays for the replay below
        atomicOr(&G.mark[s >> 5], 1u << (s & 31));
        L.mark_any = 1;
      }
    }
  }
  wbar(L);
  if (L.mark_any) {
#ifdef K3_TRACE
    const uint64_t tr_rp = TR_NOW();
    {   // (every lane counts: no lane-masked region in the trace build)
      int nm = 0;
      for (int wd = 0; wd < 33; ++wd) nm += __popc(G.mark[wd]);
      TR_ADD(K3TR_NREPLAY, nm);
    }
#endif
    // exact in-order replay of each marked counter by one wave: its tokens only
    // matter up to the points where the counter halves, so the row's tokens
    // are scanned (four 64-token chunks per load step) with the counter's
    // count / ones of each chunk taken by ballots, the chunk holding a halving
    // point applied token by token, and everything after the last halving
    // point added at once from the row's delta
    {   // the marked counters are independent: dealt round-robin to the 4 waves
      const int wv = tid >> 6;
      int j = 0;
      for (int wd = 0; wd < 33; ++wd) {
        uint32_t bits = G.mark[wd];
        while (bits) {
          const int ss = wd * 32 + __builtin_ctz(bits);
          bits &= bits - 1;
          if ((j++ & 3) != wv) continue;
          uint32_t p = G.stats[ss];
          const uint32_t dlt = L.rdelta[ss];
          uint32_t n = dlt >> 16, k = dlt & 0xffffu;   // the row's tokens of ss not applied yet
          // the token ids counted in slot ss (tok_stat_slot: id, and id + 1
          // when that is the 11th, cat-bit token of its (type, band, ctx))
          const uint32_t alt = (ss % 11 == 9) ? (uint32_t)ss + 1u : 0xffffu;
          uint32_t istart = i0;
          if (snap) {
            // the row's snapshots at MB boundaries b in (i0, i1) hold the
            // counts since i0 (i0 is a fold point); counts only grow, so the
            // boundaries reached before the halving point are a prefix of
            // the lanes: their last one is added at once and the walk starts
            // there
            const uint32_t c0 = i0 - row0, c1 = i1 - row0;
            const uint32_t b = (c0 / XS_SNAP_MBS + 1 + ln) * XS_SNAP_MBS;
            const bool valid = b < c1;
            const uint32_t v = valid ? ld_sc1(reinterpret_cast<const int32_t*>(snap) +
                                              (size_t)(b / XS_SNAP_MBS - 1) * NSLOT + ss)
                                     : 0u;
            const int nok = __popcll(__ballot(valid && (p >> 16) + (v >> 16) < 0xfffeu));
            if (nok > 0) {
              const uint32_t vb = (uint32_t)__builtin_amdgcn_readlane((int)v, nok - 1);
              p += vb;
              n -= vb >> 16;
              k -= vb & 0xffffu;
              istart = row0 + (c0 / XS_SNAP_MBS + (uint32_t)nok) * XS_SNAP_MBS;
            }
          }
          // (a frame whose token rows overflowed is encoded again: no walk
          // through tokens that were never written)
          for (uint32_t i = istart; i < i1 && n && !(G.tok_err & VP8G_ERR_ARENA); ++i) {
            const uint32_t nt = L.rowcnt[i - row0];
            const uint16_t* tk = rows ? rowbase + L.rowpos[i - row0]
                                      : tok_base + (size_t)i * VP8G_MAX_TOKENS_PER_MB;
            if (rows && !K3CK((unsigned long long)L.rowpos[i - row0] + nt <= CK_CAP(L, ~0u), 11,
                              L.rowpos[i - row0], nt, i))
              break;
            // RD 64-token chunks per step, all loads issued before the first
            // ballot, and the step's count / ones of ss taken first from
            // independent ballots: only the step holding the halving point
            // goes chunk by chunk (K3X's row fold at q90 m6, ~750 K tokens
            // per 4096-wide row, was 99% replay, a serial chain per chunk)
            for (uint32_t k4 = 0; k4 < nt && n; k4 += 64 * RD) {
              if ((p >> 16) + n < 0xfffeu) break;   // no halving left in the row
              uint32_t tq[RD];
#pragma unroll
              for (int q = 0; q < RD; ++q) {
                const uint32_t kk = k4 + 64 * q + ln;
                tq[q] = kk < nt ? tk[kk] : 0x4000u;
              }
              uint32_t scnt = 0, sone = 0;
#pragma unroll
              for (int q = 0; q < RD; ++q) {
                // (bit 14, the fixed-probability flag, keeps fixed tokens and
                // the padding off ss / alt, both < 0x4000)
                const uint32_t id = tq[q] & 0x7fffu;
                const bool mine = id == (uint32_t)ss || id == alt;
                scnt += (uint32_t)__popcll(__ballot(mine));
                sone += (uint32_t)__popcll(__ballot(mine && (tq[q] >> 15)));
              }
              if ((p >> 16) + scnt < 0xfffeu) {   // no halving point in this step
                p += (scnt << 16) + sone;
                n -= scnt;
                k -= sone;
                continue;
              }
#pragma unroll
              for (int q = 0; q < RD; ++q) {
                const uint32_t t = tq[q], id = t & 0x7fffu;
                const bool mine = id == (uint32_t)ss || id == alt;
                const uint64_t mm = __ballot(mine);
                const uint64_t ones = __ballot(mine && (t >> 15));
                const uint32_t cnt = (uint32_t)__popcll(mm);
                if ((p >> 16) + cnt < 0xfffeu) {
                  p += (cnt << 16) + (uint32_t)__popcll(ones);
                } else {
                  for (uint64_t bm = mm; bm; bm &= bm - 1) {
                    if (p >= 0xfffe0000u) p = ((p + 1u) >> 1) & 0x7fff7fffu;
                    p += 0x00010000u + (uint32_t)((ones >> __builtin_ctzll(bm)) & 1u);
                  }
                }
                n -= cnt;
                k -= (uint32_t)__popcll(ones);
              }
            }
          }
          p += (n << 16) + k;   // the rest of the row: no halving point left
          if (ln == 0) {
            G.stats[ss] = p;
            L.rdelta[ss] = 0;
          }
        }
      }
    }
    wbar(L);
    for (int k = tid; k < 33; k += K3T) G.mark[k] = 0;
    wbar(L);
    TR_SINCE(K3TR_REPLAY, tr_rp);
  }
  if (tid == 0) {
    G.ntok = base + total;
    publish((int32_t*)&G.fold_ptr, (int32_t)i1);
  }
}

// WebPEncode progress: MB rows folded (folds run in raster order, so the
// stored value only grows), a system-scope store to the host-mapped word; the
// word after it is the hook's stop request, taken up here as an abort the
// other workers see at their next wait (the worker's loop ends on myabort)
template <bool X>
__device__ __forceinline__ void report_rows(K3G& G, K3S& L, const vp8g_frame_params* P, int tid,
                                            uint32_t i1, int mbw, XHdr* XH) {
  if (P->progress_addr && tid == 0) {
    uint32_t* w = reinterpret_cast<uint32_t*>(P->progress_addr);
    __hip_atomic_store(w, i1 / (uint32_t)mbw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (__hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
      L.myabort = 1;
      G.abort = 6;
      if constexpr (X) { st_sc1(&XH->uabort, 1); st_sc1(&XH->abort, 1); }
    }
  }
}

// fold_mbs for the worker's own workgroup (X = false) or, in K3X, with the
// frame's statistics and stream length taken from xsync before and handed
// back after, then the fold pointer published (folds are serialised in
// raster order by fold_ptr, so one worker of the frame folds at a time)
template <bool X>
K3_FOLD_ATTR void fold_rows(K3G& G, K3S& L, int tid, uint32_t i0, uint32_t i1, uint32_t row0,
                          uint16_t* tok_base, uint32_t* mboff, uint8_t* xs,
                          const uint16_t* rowbase, const uint32_t* snap = nullptr) {
#ifdef K3_NO_SNAP
  snap = nullptr;
#endif
  if constexpr (X) {
    XHdr* XH = reinterpret_cast<XHdr*>(xs);
    uint32_t* xstats = reinterpret_cast<uint32_t*>(xs + XS_STATS);
    if (i0 != 0) {   // before the frame's first fold the workgroup's LDS holds the start state
      for (int s = tid; s < NSLOT; s += K3T) G.stats[s] = ld_sc1(xstats + s);
      if (tid == 0) G.ntok = ld_sc1(&XH->ntok);
      wbar(L);
    }
    fold_mbs<K3_RD_X>(G, L, tid, i0, i1, row0, tok_base, mboff, rowbase, snap);
    wbar(L);
    for (int s = tid; s < NSLOT; s += K3T) st_sc1(xstats + s, G.stats[s]);
    if (tid == 0) st_sc1(&XH->ntok, G.ntok);
    vm_drain();
    wbar(L);
    if (tid == 0) st_sc1(&XH->fold_ptr, (int32_t)i1);
  } else {
    fold_mbs<K3_RD_BATCH>(G, L, tid, i0, i1, row0, tok_base, mboff, rowbase, snap);
  }
}

// Frame end: move every MB's tokens from its VP8G_MAX_TOKENS_PER_MB slot to
// its offset in the compact stream (mboff, raster order), with the whole
// workgroup. A destination never lies above its own source, but it may
// overlap an EARLIER MB's slot, so MBs go in windows [i0, i1) whose
// destinations all lie below slot i0: inside a window every copy is
// independent. An MB whose destination reaches into its own slot is moved
// alone, chunk by chunk (each chunk read before it is written; writes stay
// below the next chunk). The windows grow geometrically (a handful per frame).
__device__ void compact_tokens(K3G& G, uint16_t* tok_base, const uint32_t* mboff, int nmb) {
  const int T = blockDim.x, t = threadIdx.x, wv = t >> 6, nwv = T >> 6, ln = t & 63;
  const uint32_t total = G.ntok;
  uint32_t i0 = 1;   // MB 0 is already in place
  while (i0 < (uint32_t)nmb) {
    if (t == 0) {    // largest i1 with end(i1 - 1) <= slot(i0)
      const uint64_t lim = (uint64_t)i0 * VP8G_MAX_TOKENS_PER_MB;
      uint32_t lo = i0, hi = (uint32_t)nmb;   // end(k - 1) = mboff[k] (or total)
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        const uint64_t e = mid < (uint32_t)nmb ? mboff[mid] : total;
        if (e <= lim) lo = mid; else hi = mid - 1;
      }
      G.mark[0] = lo;
    }
    __syncthreads();
    const uint32_t i1 = G.mark[0];
    __syncthreads();
    if (i1 > i0) {
      for (uint32_t i = i0 + wv; i < i1; i += nwv) {
        const uint32_t d = mboff[i];
        const uint32_t n = (i + 1 < (uint32_t)nmb ? mboff[i + 1] : total) - d;
        const uint16_t* src = tok_base + (size_t)i * VP8G_MAX_TOKENS_PER_MB;
        uint16_t* dst = tok_base + d;
        if (dst == src) continue;
        uint32_t c = ln;
        for (; c + 192 < n; c += 256) {
          const uint16_t t0 = src[c], t1 = src[c + 64], t2 = src[c + 128], t3 = src[c + 192];
          dst[c] = t0; dst[c + 64] = t1; dst[c + 128] = t2; dst[c + 192] = t3;
        }
        for (; c < n; c += 64) dst[c] = src[c];
      }
      i0 = i1;
    } else {
      const uint32_t d = mboff[i0];
      const uint32_t n = (i0 + 1 < (uint32_t)nmb ? mboff[i0 + 1] : total) - d;
      const uint16_t* src = tok_base + (size_t)i0 * VP8G_MAX_TOKENS_PER_MB;
      uint16_t* dst = tok_base + d;
      if (dst != src) {
        for (uint32_t c0 = 0; c0 < n; c0 += (uint32_t)T) {
          const uint32_t c = c0 + (uint32_t)t;
          const uint16_t v = c < n ? src[c] : (uint16_t)0;
          __syncthreads();
          if (c < n) dst[c] = v;
        }
      }
      i0 += 1;
    }
    __syncthreads();
  }
  if (t == 0) G.mark[0] = 0;
}

struct K3Args {
  const uint8_t* yuv;
  size_t yfb;
  int w, h, mbw, mbh;
  const uint8_t* segmap;
  const vp8g_frame_params* params;
  uint16_t* tokens;
  size_t tok_cap;
  uint8_t* mbinfo;
  uint32_t* mboff;   // n x nmb: compact-stream offset of each MB's tokens
  vp8g_frame_result* results;
  uint8_t* rerun;   // n x VP8G_RERUN_STATE_BYTES
  uint8_t* xs;      // K3X: n x xs_fb bytes of cross-workgroup frame state
  size_t xs_fb;
  int nwg;          // K3X: workgroups per frame
  uint32_t* wsnap;  // K3 (not K3X: xs holds its snapshots): n x vp8g_wsnap_bytes, or NULL
  // token rows (vp8g_rows; NULL: the per-MB slot layout, compacted at frame
  // end): MB row y's tokens at tok_base + y * rowcap in raster order, the
  // row's count to rowtok[f * mbh + y]; a row past rowcap writes nothing
  // more and the frame reports VP8G_ERR_ARENA
  uint32_t rowcap;
  uint32_t* rowtok;
};

// TR: the method >= 5 instantiation carries the trellis paths; m3/m4 frames
// run a kernel without them (smaller register footprint).
// AF: also store each MB's reconstruction for the autofilter
// X: K3X, the frame's rows are dealt to a.nwg workgroups (blocks of NW rows
// round-robin); k_encode_xtail finishes the frame
// HP: K3X helper pairs (NW = 2): each workgroup runs one row at a time, worker
// 0 the MB loop and worker 1 each MB's intra-16 and chroma evaluation beside
// worker 0's intra-4 search (K3XL::hp_*)
template <int NW, bool TR, bool AF = false, bool X = false, int WPE = 1, int PAD = 0,
          bool HP = false, bool P3 = false>
__global__ __launch_bounds__(NW * K3T) __attribute__((amdgpu_waves_per_eu(WPE))) void k_encode(K3Args a) {
  extern __shared__ __align__(16) uint8_t smem[];
  const int mbw = a.mbw, mbh = a.mbh, nmb = mbw * mbh;
  K3G& G = *reinterpret_cast<K3G*>(smem);
  const int wk = threadIdx.x / K3T;        // worker
  const int tid_k = threadIdx.x % K3T;     // thread within the worker
  const int tid = tid_k;
  K3S& L = reinterpret_cast<K3S*>(smem + sizeof(K3G) + PAD)[wk];
  uint8_t* ytop = smem + sizeof(K3G) + PAD + NW * sizeof(K3S);   // 16*mbw + 16
  uint8_t* uvtop = ytop + 16 * mbw + 16;                      // 16*mbw
  uint32_t* nzw = reinterpret_cast<uint32_t*>(uvtop + 16 * mbw) + 1;   // [-1..mbw-1]
  uint8_t* predtop = reinterpret_cast<uint8_t*>(nzw + mbw);           // 4*mbw
  int8_t* topderr = reinterpret_cast<int8_t*>(predtop + 4 * mbw);     // 4*mbw
  int32_t* rowdone = reinterpret_cast<int32_t*>(topderr + 4 * mbw);   // mbh
  // K3X: the row above worker 0 comes from another workgroup, pulled into
  // these copies of the boundary arrays (same layout); every worker still
  // writes its own row's boundary into the shared arrays
  uint8_t* xbase = reinterpret_cast<uint8_t*>(((uintptr_t)(rowdone + mbh) + 15) & ~(uintptr_t)15);
  K3XL& XL = *reinterpret_cast<K3XL*>(xbase);
  uint8_t* xytop = xbase + ((sizeof(K3XL) + 15) & ~(size_t)15);
  uint8_t* xuvtop = xytop + 16 * mbw + 16;
  uint32_t* xnzw = reinterpret_cast<uint32_t*>(xuvtop + 16 * mbw);
  uint8_t* xpredtop = reinterpret_cast<uint8_t*>(xnzw + mbw);
  int8_t* xtopderr = reinterpret_cast<int8_t*>(xpredtop + 4 * mbw);
  const bool xr = X && wk == 0;   // this worker reads the x copies
  static_assert(!HP || (X && NW == (P3 ? 3 : 2) && !AF),
                "helper pairs: K3X, one main, one helper (and an intra-4 partner) worker");
  constexpr int RW = HP ? 1 : NW;  // rows a workgroup runs at once

  const int nwg = X ? a.nwg : 1;
  const int f = X ? (int)blockIdx.x / nwg : (int)blockIdx.x;
  const int blk = X ? (int)blockIdx.x % nwg : 0;
  uint8_t* xs = X ? a.xs + (size_t)f * a.xs_fb : nullptr;
  // the statistics snapshots of row y's folds (fold_mbs): K3X per row in
  // xsync, K3 per worker (its row is folded before it starts the next)
  auto snap_of = [&](int y) -> uint32_t* {
    if constexpr (X) return xs_snap_row(xs, mbw, mbh, y);
    else return a.wsnap ? a.wsnap + ((size_t)f * 4 + wk) * xs_snaps_per_row(mbw) * NSLOT : nullptr;
  };
  XHdr* XH = reinterpret_cast<XHdr*>(xs);
  int32_t* xrowdone = reinterpret_cast<int32_t*>(xs + XS_ROWDONE);
  uint32_t* xrec = reinterpret_cast<uint32_t*>(xs + xs_rec_off(mbh));
  const int gt = threadIdx.x;
  // thread id rotated by one wave per worker: stages that leave a wave idle
  // (intra4's 160 lanes, the token tail, wave-0 bookkeeping) put the idle wave
  // on a different SIMD for each worker
  const int rtid_k = (tid + 64 * (wk & 3)) & (K3T - 1);
  const int w = a.w, h = a.h;
  const int uvw = (w + 1) >> 1, uvh = (h + 1) >> 1;
  const uint8_t* Yp = a.yuv + f * a.yfb;
  const uint8_t* Up = Yp + (size_t)w * h;
  const uint8_t* Vp = Up + (size_t)uvw * uvh;
  const vp8g_frame_params* P = a.params + f;
  const uint8_t* segmap = a.segmap + (size_t)f * nmb;
  uint16_t* tok_base = a.tokens + f * a.tok_cap;
  const bool rows = a.rowtok != nullptr;   // token rows (else per-MB slots)
  auto rowbase_of = [&](int y) -> const uint16_t* {
    return rows ? tok_base + (size_t)y * a.rowcap : nullptr;
  };
  uint8_t* mbinfo = a.mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES;
  uint32_t* mboff = a.mboff + (size_t)f * nmb;

  // partition-0 re-run (frame_enc.c:869-876): only the frames that overflowed
  // run again, from the cost state their previous pass ended with
  if (P->pass_mode == 2) return;
  const bool rerun = P->pass_mode == 1 || P->pass_mode == 3;
  uint8_t* rstate = a.rerun + (size_t)f * VP8G_RERUN_STATE_BYTES;
  uint32_t* rstats = reinterpret_cast<uint32_t*>(rstate + VP8G_STATE_STATS);

  // ---- frame init (whole workgroup); a non-last pass (mode 3) keeps the
  // token statistics of the passes before it (frame_enc.c:820-823)
  for (int s = gt; s < NSLOT; s += NW * K3T) {
    G.stats[s] = P->pass_mode == 3 ? rstats[s] : 0u;
    G.coeffs[s] = rerun ? rstate[s] : (&kVP8CoeffProba0[0][0][0][0])[s];
  }
  for (int s = tid; s < NSLOT; s += K3T) L.rdelta[s] = 0;
  for (int k = gt; k < 33; k += NW * K3T) G.mark[k] = 0;
  for (int k = gt; k < 256; k += NW * K3T) G.ecost[k] = kVP8EntropyCost[k];
  for (int k = gt; k < 1000; k += NW * K3T) G.mcost4[k] = (&kVP8ModeCostI4[0][0][0])[k];
  for (int k = gt; k < 160; k += NW * K3T) G.p4[k] = (&kP4[0][0])[k];
  if (gt < 16) G.wy[gt] = kVP8WeightY[gt];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(P->seg);
    uint32_t* dst = reinterpret_cast<uint32_t*>(G.seg);
    for (int k = gt; k < (int)(sizeof(G.seg) / 4); k += NW * K3T) dst[k] = src[k];
  }
  for (int k = gt; k < 16 * mbw + 16; k += NW * K3T) ytop[k] = 127;
  for (int k = gt; k < 16 * mbw; k += NW * K3T) uvtop[k] = 127;
  for (int k = gt - 1; k < mbw; k += NW * K3T) nzw[k] = 0;
  for (int k = gt; k < 4 * mbw; k += NW * K3T) { predtop[k] = 0; topderr[k] = 0; }
  for (int k = gt; k < mbh; k += NW * K3T) rowdone[k] = 0;
  if constexpr (X) {
    for (int k = gt; k < 16 * mbw + 16; k += NW * K3T) xytop[k] = 127;
    for (int k = gt; k < 16 * mbw; k += NW * K3T) xuvtop[k] = 127;
    for (int k = gt; k < mbw; k += NW * K3T) xnzw[k] = 0;
    for (int k = gt; k < 4 * mbw; k += NW * K3T) { xpredtop[k] = 0; xtopderr[k] = 0; }
    if (gt == 0) {
      XL.lcver = 0; XL.claim = 0;
      XL.hp_go = 0; XL.hp_done = 0; XL.hp_i16 = 0; XL.hp_pre = 0; XL.hp_bnd = 0;
      XL.hp_tokgo = 0; XL.hp_tok = 0;
      XL.p_go = 0; XL.p_skip = 0; XL.p_bar = 0;
    }
  }
  if (gt < 4) G.max_edge[gt] = 0;
  if (gt == 0) {
    G.fs.size_p0 = 0; G.fs.sse[0] = G.fs.sse[1] = G.fs.sse[2] = 0; G.fs.dist = 0;
    G.fs.size_rh = 0;
    G.fs.nb[0] = G.fs.nb[1] = G.fs.nb[2] = 0;
    G.fold_ptr = 0; G.ntok = 0; G.tok_err = 0; G.epoch = 0; G.abort = 0;
  }
  if (tid == 0) { L.bar = 0; L.myabort = 0; L.rowfill = 0; }
#ifdef K3_CHECK
  if (tid == 0) {
    L.ck_nmb = (uint32_t)nmb; L.ck_cap = a.rowcap;
    L.ck_rowdone = (uint32_t)((uintptr_t)rowdone - (uintptr_t)smem);
    L.ck_y = -1; L.ck_x = 0;
  }
#endif
  __syncthreads();
  if (wk == 0) level_costs_w(G, G.coeffs, tid);
  __syncthreads();
  if (rerun) {   // the level costs came from rstate[0..]; the probabilities are the loop-end ones
    for (int s = gt; s < NSLOT; s += NW * K3T) G.coeffs[s] = rstate[NSLOT + s];
    __syncthreads();
  } else if (blk == 0) {   // first pass: the level costs are those of the default probabilities
    for (int s = gt; s < NSLOT; s += NW * K3T) rstate[s] = G.coeffs[s];
  }
  if (wk == 0) refresh_hc(G, tid);
  __syncthreads();

  const int rd_opt = P->rd_opt;
#ifdef K3_NO_I4   // (timing build only, wrong output: no intra-4 search)
  const int max_i4_bits = 0;
#else
  const int max_i4_bits = P->max_i4_header_bits;
#endif
  const int use_derr = P->use_derr;
  const int max_count = P->max_count;
  const bool trellis_all = TR && rd_opt >= 3;
#ifdef K3_SUBPROF
  uint64_t subacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t* substamps = subacc;
#else
  uint64_t* substamps = nullptr;
#endif
#ifdef K3_STAMPS
  uint64_t stamps[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t stamp_last = __builtin_amdgcn_s_memtime();
#endif
  uint8_t* yl = L.yl_mem + 1;
  uint8_t* ul = L.ul_mem + 1;
  uint8_t* vl = L.vl_mem + 1;
#ifdef K3_TRACE
  if (__builtin_amdgcn_readfirstlane(tid) < 64) L.trace[tid & (K3TR_N - 1)] = 0;
  const uint64_t tr_start = TR_NOW();
#endif

#ifndef K3X_HELPER_SLEEP   // s_sleep units between a helper's / partner's polls (single
#define K3X_HELPER_SLEEP 2    // 1080p 30.3-30.5 ms at 2, 30.6-30.7 at 0, 30.55 at 10 vs 30.26
#endif                        // at 2 on another box; profiles/r6/k3x/sleep)
#ifndef K3X_MAIN_PRIO
#define K3X_MAIN_PRIO 2
#endif
  if constexpr (HP) {
    // each SIMD runs one wave of every worker: the main worker's (and the
    // intra-4 partner's) waves, on the MB's critical path, win the SIMD's
    // issue arbitration over the helper's, which fills the gaps (config 4
    // 149.5 -> 141.1 ms; the helper raised to 3 while its intra-16 bound is
    // pending instead: 148.1 ms, single 1080p 30.6 -> 31.1 ms; profiles/r6/k3x/prio)
    if (wk != 1) __builtin_amdgcn_s_setprio(K3X_MAIN_PRIO);
  }
  if constexpr (HP) {
    if (wk == 1) {
      // the helper: for every MB of the main worker's rows, once the main has
      // published it (predictions and source measure in M), the intra-16
      // candidates and choice (quant_enc.c:1002-1058, StoreMaxDelta) and the
      // chroma candidates and choice with StoreDiffusionErrors
      // (quant_enc.c:1169-1217); its own barriers (L), M's data
      K3S& M = reinterpret_cast<K3S*>(smem + sizeof(K3G) + PAD)[0];
      const int8_t* derrx = xtopderr;   // the row above's DC errors, pulled by the main
      for (int y = blk; y < mbh && !L.myabort; y += nwg) {
        bool dk_pending = false;   // the previous MB's tokens are still to write
        for (int x = 0; x < mbw; ++x) {
          const int tid = opaque(tid_k), lane = tid & 63;
          const uint32_t mb = (uint32_t)y * mbw + x;
          // one MB's tokens and their statistics into the main's pending
          // deltas (levels from Lv: the main's, or this worker's copy)
          auto mb_tokens = [&](const K3S& Lv, int xx, uint32_t mbx, uint32_t tct, uint32_t tcl,
                               int tfirst) {
            const int rtid = opaque(rtid_k);
            const int first_blk = __builtin_amdgcn_readfirstlane(tfirst);
            const bool is_i16 = first_blk == 0;
            MBCtx tc;
            tc.t = __builtin_amdgcn_readfirstlane(tct);
            tc.l = __builtin_amdgcn_readfirstlane(tcl);
            const uint32_t rfill = rows ? M.rowfill : 0u;
            int lvi[2], lvp[2], cnt[2], bi[2], last[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int item = rtid + K3T * q, k = item >> 4, n = item & 15;
              int v = 0, vp = 0;
              if (k < 25 && k >= first_blk) {
                const int16_t* lvb = blk_levels(Lv, k);
                v = lvb[n];
                vp = n > 0 ? lvb[n - 1] : 0;
              }
              lvi[q] = v;
              lvp[q] = vp;
              const int lq = max16(v != 0 ? n : -1);
              if (n == 0 && k < 32) L.blast[k] = lq;
            }
            wbar(L);
            const uint64_t nzb = __ballot(lane >= first_blk && lane < 25 && L.blast[lane] >= 0);
            auto blk_param = [&](int k) -> int {
              if (k < first_blk || k >= 25) return -1;
              if (k == 0) return 1 | ((tc.top(8) + tc.left(8)) << 8);
              if (k <= 16) {
                const int b = k - 1, bx = b & 3, by = b >> 2;
                const int t = by == 0 ? tc.top(bx) : (int)((nzb >> (k - 4)) & 1);
                const int l = bx == 0 ? tc.left(by) : (int)((nzb >> (k - 1)) & 1);
                return (is_i16 ? 0 | (1 << 4) : 3) | ((t + l) << 8);
              }
              const int b = k - 17, ch = b >> 2, k4 = b & 3, bx = k4 & 1, by = k4 >> 1;
              const int t = by == 0 ? tc.top(4 + 2 * ch + bx) : (int)((nzb >> (k - 2)) & 1);
              const int l = bx == 0 ? tc.left(4 + 2 * ch + by) : (int)((nzb >> (k - 1)) & 1);
              return 2 | ((t + l) << 8);
            };
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int item = rtid + K3T * q, k = item >> 4, n = item & 15;
              bi[q] = blk_param(k);
              last[q] = k < 25 ? L.blast[k] : -1;
              cnt[q] = bi[q] < 0 ? 0 : pos_count((bi[q] >> 4) & 15, n, lvi[q], lvp[q], last[q]);
            }
            int inc0 = cnt[0], inc1 = cnt[1];
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
              const int v0 = __shfl_up(inc0, off), v1 = __shfl_up(inc1, off);
              if (lane >= off) { inc0 += v0; inc1 += v1; }
            }
            const int wv = rtid >> 6;
            if (lane == 63) { L.wsum[0][wv] = inc0; L.wsum[1][wv] = inc1; }
            wbar(L);
            int pre0 = 0, pre1 = 0, tot0 = 0, tot1 = 0;
#pragma unroll
            for (int w2 = 0; w2 < 4; ++w2) {
              const int s0 = L.wsum[0][w2], s1 = L.wsum[1][w2];
              if (w2 < wv) { pre0 += s0; pre1 += s1; }
              tot0 += s0; tot1 += s1;
            }
            uint16_t* slot = rows ? tok_base + (size_t)y * a.rowcap + rfill
                                  : tok_base + (size_t)mbx * VP8G_MAX_TOKENS_PER_MB;
            const int off0 = pre0 + inc0 - cnt[0];
            const int off1 = tot0 + pre1 + inc1 - cnt[1];
            const bool over = rows && rfill + (uint32_t)(tot0 + tot1) > a.rowcap;
            if (over) { cnt[0] = 0; cnt[1] = 0; }
            if (cnt[0])
              pos_tokens<true>(bi[0] & 15, (bi[0] >> 4) & 15, bi[0] >> 8, rtid & 15, lvi[0], lvp[0],
                               last[0], slot + off0, M.rdelta);
            if (cnt[1])
              pos_tokens<true>(bi[1] & 15, (bi[1] >> 4) & 15, bi[1] >> 8, rtid & 15, lvi[1], lvp[1],
                               last[1], slot + off1, M.rdelta);
            if (rtid == 0) {
              M.rowcnt[xx] = (uint16_t)(tot0 + tot1);
              if (rows) {
                M.rowpos[xx] = rfill;
                M.rowfill = rfill + (uint32_t)(tot0 + tot1);
                if (over) atomicOr(&G.tok_err, VP8G_ERR_ARENA);
              }
            }
            wbar(L);
            if (tid == 0) publish(&XL.hp_tok, (int32_t)mbx + 1);
          };
          const uint64_t tr_w = TR_NOW();
          if (!wait_ge<K3X_HELPER_SLEEP>(G, L, &XL.hp_go, (int32_t)mb + 1, 8)) break;
          const uint64_t tr_e = TR_NOW();
          TR_ADD(K3TR_ROW_WAIT, tr_e - tr_w);   // (helper: waiting for the main)
          TR_ADD(K3TR_NMB, 1);
          const int segid = __builtin_amdgcn_readfirstlane(XL.hp_seg);
          const vp8g_seg& S = G.seg[segid];
          MBCtx ctx;
          ctx.t = __builtin_amdgcn_readfirstlane(XL.hp_ctx_t);
          ctx.l = __builtin_amdgcn_readfirstlane(XL.hp_ctx_l);
          // the 16x16 and chroma predictions from the main's edges (its left
          // samples and the row above it pulled, unchanged until this MB is done)
          predict_mb(M, M.yl_mem + 1, M.ul_mem + 1, M.vl_mem + 1, xytop + 16 * x, xuvtop + 16 * x,
                     x > 0, y > 0, tid);
          wbar(L);
          if constexpr (TR) {
            if (__builtin_amdgcn_readfirstlane((int)trellis_all))   // (a scalar branch)
              eval_i16<true>(G, M, S, ctx, tid, L);
            else
              eval_i16<false>(G, M, S, ctx, tid, L);
          } else {
            eval_i16<false>(G, M, S, ctx, tid, L);
          }
          int best16 = 0;
          uint32_t nz16 = 0;
          score_t D16 = 0, SD16 = 0, H16 = 0, R16 = 0;
          {
            const int v0 = M.yin[0];
            int same = 1;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int p = lane + 64 * q;
              same &= M.yin[(p >> 4) * BPS + (p & 15)] == v0;
            }
            int flat = __all(same);
            score_t best16_score = 0;
            for (int mm = 0; mm < 4; ++mm) {
              score_t Dm = M.mres[mm][0];
              score_t SDm = S.tlambda ? (score_t)((S.tlambda * M.mres[mm][1] + 128) >> 8) : 0;
              const score_t Hm = kVP8ModeCostI16[mm];
              const score_t Rm = M.mres[mm][2];
              if (flat) {
                flat = (M.mres[mm][3] & 0xffff) == 0;
                if (flat) { Dm *= 2; SDm *= 2; }
              }
              const score_t sc = (Rm + Hm) * S.lambda_i16 + 256 * (Dm + SDm);
              if (mm == 0 || sc < best16_score) {
                best16_score = sc; best16 = mm;
                D16 = Dm; SD16 = SDm; H16 = Hm; R16 = Rm;
                nz16 = (uint32_t)M.mres[mm][3];
              }
            }
          }
          if (tid < 64) {   // (a whole wave)
            XL.hp_best16 = best16; XL.hp_nz16 = nz16;
            XL.hp_D16 = D16; XL.hp_SD16 = SD16; XL.hp_H16 = H16; XL.hp_R16 = R16;
            XL.hp_rd16 = (R16 + H16) * S.lambda_mode + 256 * (D16 + SD16);
          }
          if ((nz16 & 0x100ffff) == 0x1000000 && D16 > S.min_disto) {   // StoreMaxDelta
            int mv = iabs_(M.lvdc[best16][1]);
            mv = max(mv, iabs_(M.lvdc[best16][2]));
            mv = max(mv, iabs_(M.lvdc[best16][4]));
            if (tid == 0) atomicMax(&G.max_edge[segid], mv);
          }
          // the chroma candidates overwrite M.mres: every wave has read it;
          // the intra-16 score goes out now (the search's bound)
          wbar(L);
          if (tid == 0) publish(&XL.hp_i16, (int32_t)mb + 1);
          eval_uv(G, M, S, ctx, tid, x, derrx, use_derr, L);
          int bu = 0;
          score_t bsc = 0, bH = 0;
          for (int mm = 0; mm < 4; ++mm) {
            const score_t Dm = M.mres[mm][0], Hm = kVP8ModeCostUV[mm];
            score_t Rm = M.mres[mm][1];
            if (mm > 0 && M.mres[mm][2] <= 2) Rm += 140 * 8;
            const score_t sc = (Rm + Hm) * S.lambda_uv + 256 * Dm;
            if (mm == 0 || sc < bsc) { bsc = sc; bu = mm; bH = Hm; }
          }
          if (tid < 64) { XL.hp_bu = bu; XL.hp_bH = bH; XL.hp_bsc = bsc; }
          if (use_derr && tid < 2) {   // StoreDiffusionErrors (quant_enc.c:909-920)
            const int cch = tid;
            int8_t* top = topderr + 4 * x + 2 * cch;
            int8_t* left = M.lderr[cch];
            const int8_t* e = M.uvderr[bu][cch];
            left[0] = e[0];
            left[1] = (int8_t)(3 * e[2] >> 2);
            top[0] = e[1];
            top[1] = (int8_t)(e[2] - left[1]);
          }
          wbar(L);
          if (tid == 0) publish(&XL.hp_done, (int32_t)mb + 1);
          TR_SINCE(K3TR_I16, tr_e);   // (helper: intra-16 + chroma)
          // the next MB's source into this worker's yin (the main copies it
          // from LDS instead of waiting for its own global loads)
          if (x + 1 < mbw) {
            const int nseg = segmap[mb + 1];
            load_mb(Yp, Up, Vp, w, h, x + 1, y, L.yin, tid, K3T);
            if (tid == 0) XL.hp_nseg = nseg;
            wbar(L);
            {   // and its texture measure (see the main worker's)
              const int b = tid >> 4, j = tid & 15;
              const int src = L.yin[(4 * (b >> 2) + (j >> 2)) * BPS + 4 * (b & 3) + (j & 3)];
              const int hs = sum16(ttrans_lane(src, j, G.wy[j]));
              if (j == 0) L.hsrc[b] = hs;
            }
            wbar(L);
            if (tid == 0) publish(&XL.hp_pre, (int32_t)mb + 2);
          }
          // the previous MB's tokens, when they were put off (below): after
          // this MB's intra-16 bound, chroma choice and the next source are
          // out, from the levels copied then
          if (x > 0 && dk_pending) {
            mb_tokens(L, x - 1, mb - 1, XL.dk_ctx_t, XL.dk_ctx_l, XL.dk_first);
            dk_pending = false;
          }
          // ---- this MB's tokens (token_enc.c:113-193) into its row slot, off
          // the main worker's path, once the main has committed the MB: now,
          // when the main waits for them before its next MB (a statistics
          // snapshot column, the row's end, an epoch refresh next), else put
          // off until the next MB's intra-16 bound, chroma choice and source
          // are out (the main's search takes the bound sooner), from a copy of
          // the levels (the main overwrites its own once it has that bound)
          {
            if (!wait_ge<K3X_HELPER_SLEEP>(G, L, &XL.hp_tokgo, (int32_t)mb + 1, 11)) break;
            const int nx = (int)mb + 1;
            const bool now = x == mbw - 1 || ((x + 1) % XS_SNAP_MBS == 0) ||
                             (nx >= max_count && (nx - max_count) % (max_count + 1) == 0);
            if (now) {
              mb_tokens(M, x, mb, XL.tk_ctx_t, XL.tk_ctx_l, XL.tk_first);
            } else {
              if (tid < 8)
                reinterpret_cast<uint32_t*>(L.fin_dc)[tid] = reinterpret_cast<const uint32_t*>(M.fin_dc)[tid];
              else if (tid < 8 + 128)
                reinterpret_cast<uint32_t*>(&L.fin_ac[0][0])[tid - 8] =
                    reinterpret_cast<const uint32_t*>(&M.fin_ac[0][0])[tid - 8];
              else if (tid < 8 + 128 + 64)
                reinterpret_cast<uint32_t*>(&L.fin_uv[0][0])[tid - 136] =
                    reinterpret_cast<const uint32_t*>(&M.fin_uv[0][0])[tid - 136];
              if (tid == 0) {
                XL.dk_ctx_t = XL.tk_ctx_t; XL.dk_ctx_l = XL.tk_ctx_l; XL.dk_first = XL.tk_first;
              }
              wbar(L);
              dk_pending = true;
            }
          }
          // column x's boundary record for the next row's workgroup, off the
          // main worker's path (the stores' drain)
          if (y < mbh - 1) {
            if (!wait_ge<K3X_HELPER_SLEEP>(G, L, &XL.hp_bnd, (int32_t)mb + 1, 9)) break;
            if (tid < 64) {
              if (tid < 11) {
                uint32_t v;
                if (tid < 4) v = reinterpret_cast<const uint32_t*>(ytop + 16 * x)[tid];
                else if (tid < 8) v = reinterpret_cast<const uint32_t*>(uvtop + 16 * x)[tid - 4];
                else if (tid == 8) v = nzw[x];
                else if (tid == 9) v = reinterpret_cast<const uint32_t*>(predtop + 4 * x)[0];
                else v = reinterpret_cast<const uint32_t*>(topderr + 4 * x)[0];
                st_sc1(xrec + ((size_t)y * mbw + x) * XS_REC_WORDS + tid, v);
              }
              vm_drain();
              if (tid == 0) st_sc1(&xrowdone[y], x + 1);
            }
          }
        }
      }
    }
  }
  if constexpr (P3) {
    if (wk == 2) {
      // the intra-4 partner: its half of each MB's search (run_i4_pair)
      K3S& M = reinterpret_cast<K3S*>(smem + sizeof(K3G) + PAD)[0];
      for (int y = blk; y < mbh && !L.myabort; y += nwg) {
        for (int x = 0; x < mbw; ++x) {
          const int rtid = opaque(rtid_k);
          const uint32_t mb = (uint32_t)y * mbw + x;
          if (!wait_ge<K3X_HELPER_SLEEP>(G, L, &XL.p_go, (int32_t)mb + 1, 12)) break;
          if (__builtin_amdgcn_readfirstlane(XL.p_skip)) continue;
          const int segid = __builtin_amdgcn_readfirstlane(XL.hp_seg);
          const vp8g_seg& S = G.seg[segid];
          MBCtx ctx;
          ctx.t = __builtin_amdgcn_readfirstlane(XL.hp_ctx_t);
          ctx.l = __builtin_amdgcn_readfirstlane(XL.hp_ctx_l);
          if (__builtin_amdgcn_readfirstlane((int)trellis_all))   // (a scalar branch)
            (void)run_i4_pair<true>(G, L, M, L, XL, 1, S, ctx, rtid, x, mbw, xpredtop,
                                    M.yl_mem + 1, xytop + 16 * x, kI4NoBound, max_i4_bits,
                                    &XL.hp_i16, (int32_t)mb + 1, &XL.hp_rd16);
          else
            (void)run_i4_pair<false>(G, L, M, L, XL, 1, S, ctx, rtid, x, mbw, xpredtop,
                                     M.yl_mem + 1, xytop + 16 * x, kI4NoBound, max_i4_bits,
                                     &XL.hp_i16, (int32_t)mb + 1, &XL.hp_rd16);
        }
      }
    }
  }
  for (int y = blk * RW + (HP ? 0 : wk); (!HP || wk == 0) && y < mbh && !L.myabort;
       y += RW * nwg) {
    // InitLeft (iterator_enc.c:22-32)
    if (tid < 16) yl[tid] = 129;
    if (tid < 8) { ul[tid] = 129; vl[tid] = 129; }
    if (tid == 0) {
      L.rowfill = 0;
      yl[-1] = ul[-1] = vl[-1] = (y > 0) ? 129 : 127;
      L.lderr[0][0] = L.lderr[0][1] = L.lderr[1][0] = L.lderr[1][1] = 0;
    }
    if (tid < 4) L.predleft[tid] = 0;
    if (tid == 0)
      L.epseen = __hip_atomic_load(&G.epoch, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    int left_dc = 0;
    uint32_t fold_from = (uint32_t)y * mbw;   // first MB of this row not folded yet
    int xpc = 0;   // K3X: columns of the row above pulled so far
#ifdef K3_PF   // (A/B) each MB fetches the next one's source during its token stage
    uint32_t pf = K3T == 256 ? fetch_mb256(Yp, Up, Vp, w, h, 0, y, tid) : 0u;
#endif
    wbar(L);
    for (int x = 0; x < mbw; ++x) {
      // per-lane ids re-derived every MB (opaque): values computed from them
      // stay next to their uses instead of being hoisted out of the MB loop
      // and held in registers across it
      const int tid = opaque(tid_k), rtid = opaque(rtid_k), lane = tid & 63;
      const bool w0 = rtid < 64;
      const uint32_t mb = (uint32_t)y * mbw + x;
#ifdef K3_CHECK
      if (tid == 0) { L.ck_y = y; L.ck_x = -1 - x; }   // (negative: before the MB's waits)
#endif
      // ---- cost-table epoch (frame_enc.c:828-832): refresh before MB k with
      // k = max_count + e * (max_count + 1)
      const int ep = (int)mb < max_count ? 0 : ((int)mb - max_count) / (max_count + 1) + 1;
      // The decision is the worker's, from one lane's read of G.epoch taken
      // before the barrier that ended the previous MB (L.epseen): every wave
      // of the worker takes the same branch and so the same barriers. (Each
      // wave reading G.epoch itself let the waves of a waiting worker split
      // when the refresher published between their reads: some entered the
      // wait with its barrier, some skipped it, and the worker's barrier
      // generations went out of step -- a hang at the frame's end.) A stale
      // value only sends the worker through a wait that returns at once.
      if (ep > L.epseen) {
        const bool refresher = (int)mb == max_count + (ep - 1) * (max_count + 1);
        if (refresher) {
          // everything before this MB: rows above folded by their owners,
          // this row's earlier MBs folded here
          const uint64_t tr_w = TR_NOW();
          if constexpr (X) {
            if (tid == 0) atomicMax(&XL.claim, ep);
            if (!wait_gx(G, L, &XH->fold_ptr, (int32_t)fold_from, XH)) break;
          } else {
            if (!wait_ge(G, L, (const int32_t*)&G.fold_ptr, (int32_t)fold_from, 1)) break;
          }
          if constexpr (HP) {   // the helper's tokens of this row's MBs before this one
            if (x > 0 && !wait_ge(G, L, &XL.hp_tok, (int32_t)mb, 11)) break;
          }
          const uint64_t tr_f = TR_NOW();
          TR_ADD(K3TR_REFR_WAIT, tr_f - tr_w);
          fold_rows<X>(G, L, tid, fold_from, mb, (uint32_t)y * mbw, tok_base, mboff, xs, rowbase_of(y),
                       snap_of(y));
          fold_from = mb;
          wbar(L);
          const uint64_t tr_r = TR_NOW();
          TR_ADD(K3TR_FOLD, tr_r - tr_f);
          const int dirty = finalize_probas_wg(G, L, tid);
          if constexpr (X) {
            // level costs: recomputed when dirty, else those of the frame's
            // last dirty epoch (this workgroup may have skipped that epoch)
            if (dirty) {
              level_costs_w(G, G.coeffs, tid);
              probas_to_x(G.coeffs, xs + XS_LCOEFFS, tid);
              if (tid == 0) XL.lcver = ep;
            } else {
              const int32_t lv = ld_sc1(&XH->lcver);
              if (lv != XL.lcver) {
                probas_from_x(XL.lcoeffs, xs + XS_LCOEFFS, tid);
                wbar(L);
                level_costs_w(G, XL.lcoeffs, tid);
                if (tid == 0) XL.lcver = lv;
              }
            }
            probas_to_x(G.coeffs, xs + XS_COEFFS, tid);
            vm_drain();
          } else {
            if (dirty) {
              level_costs_w(G, G.coeffs, tid);
              for (int s = tid; s < NSLOT; s += K3T) rstate[s] = G.coeffs[s];
            }
          }
          refresh_hc(G, tid);
          wbar(L);
          if constexpr (X) {
            if (tid == 0) {
              if (dirty) { st_sc1(&XH->lcver, ep); vm_drain(); }
              st_sc1(&XH->epoch, ep);
            }
          }
          if (tid == 0) publish(&G.epoch, ep);
          TR_SINCE(K3TR_REFRESH, tr_r);
        } else if (X) {
          // the frame's refresher published epoch ep; the first worker of this
          // workgroup to need it copies the probabilities (and, if they
          // changed, recomputes the level costs) for the whole workgroup
          const uint64_t tr_w = TR_NOW();
          if (!wait_gx(G, L, &XH->epoch, ep, XH)) break;
          TR_SINCE(K3TR_EPOCH_WAIT, tr_w);
          const uint64_t tr_r = TR_NOW();
          if (tid == 0) L.redw[0] = atomicMax(&XL.claim, ep) < ep;
          wbar(L);
          const int mine = L.redw[0];
          wbar(L);
          if (mine) {
            const int32_t lv = ld_sc1(&XH->lcver);
            if (lv != XL.lcver) {
              probas_from_x(XL.lcoeffs, xs + XS_LCOEFFS, tid);
              wbar(L);
              level_costs_w(G, XL.lcoeffs, tid);
              if (tid == 0) XL.lcver = lv;
            }
            probas_from_x(G.coeffs, xs + XS_COEFFS, tid);
            wbar(L);
            refresh_hc(G, tid);
            wbar(L);
            if (tid == 0) publish(&G.epoch, ep);
          } else {
            if (!wait_ge(G, L, &G.epoch, ep, 2)) break;
          }
          TR_SINCE(K3TR_REFRESH, tr_r);
        } else {
          const uint64_t tr_w = TR_NOW();
          if (!wait_ge(G, L, &G.epoch, ep, 2)) break;
          TR_SINCE(K3TR_EPOCH_WAIT, tr_w);
        }
      }
      // ---- wavefront dependency: MB x+1 of the row above (top-right) is done
#ifndef K3_NO_PRIO
      // place in the row wavefront (issue priority below), taken by one lane
      // before the wait so the wait's barrier hands every wave the same value
      if constexpr (!X) {
        if (tid == 0) {
          int ld = 0;
#ifdef K3_PRIO4   // A/B: one level per row above still running (3 = leads)
          if (y == 0 || __hip_atomic_load(&rowdone[y - 1], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP) >= mbw)
            ld = 3;
          else if (y == 1 || __hip_atomic_load(&rowdone[y - 2], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP) >= mbw)
            ld = 2;
          else if (y == 2 || __hip_atomic_load(&rowdone[y - 3], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP) >= mbw)
            ld = 1;
#else
          if (y == 0 || __hip_atomic_load(&rowdone[y - 1], __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP) >= mbw)
            ld = 2;
          else if (y == 1 || __hip_atomic_load(&rowdone[y - 2], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP) >= mbw)
            ld = 1;
#endif
          L.lead = ld;
        }
        if (y == 0) wbar(L);   // (rows > 0 pass the wait's barrier)
      }
#endif
      if (xr) {
        if (y > 0) {
#ifdef K3_TRACE
          const uint64_t tr_w = TR_NOW();
          TR_ADD(K3TR_NROWWAIT, ld_sc1(&xrowdone[y - 1]) < min(x + 2, mbw) ? 1 : 0);
#endif
          // MB x needs columns x and x + 1 of the row above; every column
          // that row has published by the time of the wait is pulled at once
          // (up to XS_PULL_COLS), so while it runs ahead the next MBs skip
          // the poll and the record loads
          const int need = min(x + 2, mbw);
          int32_t seen = xpc;
          if (xpc < need &&
              !wait_gx_seen(G, L, &xrowdone[y - 1], need, XH, XL.xseen, tid, seen)) break;
          TR_SINCE(K3TR_ROW_WAIT, tr_w);
          const int c0 = xpc;
          const int nc = min(min((int)seen, mbw), c0 + XS_PULL_COLS) - c0;
          xpc = c0 + max(nc, 0);
          if (tid < XS_REC_WORDS * nc) {
            const int c = c0 + tid / XS_REC_WORDS, k = tid % XS_REC_WORDS;
            const uint32_t v = ld_sc1(xrec + ((size_t)(y - 1) * mbw + c) * XS_REC_WORDS + k);
            if (k < 4) reinterpret_cast<uint32_t*>(xytop + 16 * c)[k] = v;
            else if (k < 8) reinterpret_cast<uint32_t*>(xuvtop + 16 * c)[k - 4] = v;
            else if (k == 8) xnzw[c] = v;
            else if (k == 9) reinterpret_cast<uint32_t*>(xpredtop + 4 * c)[0] = v;
            else if (k == 10) reinterpret_cast<uint32_t*>(xtopderr + 4 * c)[0] = v;
          }
        }
      } else if (y > 0) {
#ifdef K3_TRACE
        const uint64_t tr_w = TR_NOW();
        TR_ADD(K3TR_NROWWAIT, ld_uni(&rowdone[y - 1]) < min(x + 2, mbw) ? 1 : 0);
#endif
        if (!wait_ge(G, L, &rowdone[y - 1], min(x + 2, mbw), 3)) break;
        TR_SINCE(K3TR_ROW_WAIT, tr_w);
      }
#ifndef K3_NO_PRIO   // K3 124.5 -> 118.1 ms (profiles/r3/ab16_*)
      if constexpr (!X) {
        // issue priority by place in the row wavefront: a worker whose row
        // above is finished leads and gates the others (they wait on its
        // progress), so its waves win the SIMDs' issue arbitration
        int lead = __builtin_amdgcn_readfirstlane(L.lead);
#ifndef K3_NO_EPRIO   // before a cost-epoch boundary K every row above K's row
                      // must finish first: the row right above leads, the
                      // rows below wait anyway (K3 105.8 -> 102.7 ms, r5s19)
        {
          const int K = max_count + ep * (max_count + 1);
          const int d = __builtin_amdgcn_readfirstlane(K / mbw - y);
#if defined(K3_EPRIO2)   // (A/B) three levels above the boundary row, over the usual lead
          if (d >= 1 && d <= 3) lead = 4 - d;
          else if (d == 0) lead = 0;
#elif defined(K3_EPRIO3)   // (A/B) both rows right above lead
          if (d >= 1 && d <= 2) lead = 2;
          else if (d == 3) lead = 1;
          else if (d == 0) lead = 0;
#elif defined(K3_EPRIO4)   // (A/B) the refresher's row also gives way to the usual lead
          if (d >= 1 && d <= 2) lead = 3 - d;
          else if (d == 3) lead = 0;
#else
          if (d >= 1 && d <= 2) lead = 3 - d;
          else if (d == 3 || d == 0) lead = 0;
#endif
        }
#endif
#ifndef K3_PRIO_LEAD
#define K3_PRIO_LEAD 2
#endif
#ifdef K3_PRIO4
        if (lead == 3) __builtin_amdgcn_s_setprio(3);
        else if (lead == 2) __builtin_amdgcn_s_setprio(2);
        else if (lead == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
#else
        if (lead == 3) __builtin_amdgcn_s_setprio(3);
        else if (lead == 2) __builtin_amdgcn_s_setprio(K3_PRIO_LEAD);
        else if (lead == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
#endif
      }
#endif
      K3_STAMP(0);
#ifdef K3_CHECK
      if (tid == 0) { L.ck_y = y; L.ck_x = x; }
#endif
      const uint64_t tr_mb = TR_NOW();
      TR_ADD(K3TR_NMB, 1);

#ifdef K3_PF
      put_mb256(pf, L.yin, tid);
#else
      if (HP && x > 0) {   // the source the helper loaded (LDS to LDS)
        if (!wait_ge(G, L, &XL.hp_pre, (int32_t)mb + 1, 10)) break;
        const K3S& Hs = reinterpret_cast<const K3S*>(smem + sizeof(K3G) + PAD)[1];
        if (tid < 16 * BPS / 4)
          reinterpret_cast<uint32_t*>(L.yin)[tid] = reinterpret_cast<const uint32_t*>(Hs.yin)[tid];
        else if (tid < 16 * BPS / 4 + 16)
          L.hsrc[tid - 16 * BPS / 4] = Hs.hsrc[tid - 16 * BPS / 4];
      } else {
        load_mb(Yp, Up, Vp, w, h, x, y, L.yin, tid, K3T);
      }
#endif
      wbar(L);
      int segid = HP && x > 0 ? XL.hp_nseg : segmap[mb];   // (HP: read with the source)
      if (!K3CK(segid >= 0 && segid < 4, 13, segid, 4, mb)) segid = 0;
      const vp8g_seg& S = G.seg[segid];
      const bool hl = x > 0, ht = y > 0;
      const uint8_t* yt = (xr ? xytop : ytop) + 16 * x;
      const uint8_t* uvt = (xr ? xuvtop : uvtop) + 16 * x;
      const uint8_t* predrd = xr ? xpredtop : predtop;   // the row above's I4 modes
      const int8_t* derrrd = xr ? xtopderr : topderr;     // and its DC errors
      MBCtx ctx;
      nz_flags(xr ? xnzw[x] : nzw[x], nzw[x - 1], left_dc, ctx);

      // ---- predictions (quant_enc.c:469-479; a helper pair's helper makes
      // them, the main worker's intra-4 search does not read them)
      if (!(HP && x > 0)) {   // (a pair's helper made the measure with the source)
        if (!HP) predict_mb(L, yl, ul, vl, yt, uvt, hl, ht, tid);
        // texture (Hadamard) measure of the 16 source blocks, shared by the
        // intra16 and intra4 distortions (VP8TDisto4x4 / 16x16)
        const int b = tid >> 4, j = tid & 15;
        const int src = L.yin[(4 * (b >> 2) + (j >> 2)) * BPS + 4 * (b & 3) + (j & 3)];
        const int hs = sum16(ttrans_lane(src, j, G.wy[j]));
        if (j == 0) L.hsrc[b] = hs;
        wbar(L);
      }
      K3_STAMP(1);

      int best16 = 0, is_i16 = 1, bu = 0;
      uint64_t tr_uv = 0;
      score_t rd_score = 0, rdH = 0;
      uint32_t rd_nz = 0;
      if constexpr (HP) {
        // hand the MB to the helper, run the intra-4 search without the
        // intra-16 bound (the bound only ends early a search whose score, which
        // only grows, would lose anyway: the same choice), then take the
        // helper's intra-16 and chroma results
        if (tid == 0) {
          XL.hp_ctx_t = ctx.t; XL.hp_ctx_l = ctx.l; XL.hp_seg = segid;
          publish(&XL.hp_go, (int32_t)mb + 1);
        }
        TR_SINCE(K3TR_I16, tr_mb);   // (main worker of a pair: load + predictions)
        K3_STAMP(2);
        const uint64_t tr_i4 = TR_NOW();
        I4Result r4;
        r4.ok = 0; r4.H = 0; r4.score = 0; r4.nz = 0;
        if constexpr (P3) {   // the partner's go (or skip)
          if (tid == 0) {
            XL.p_skip = max_i4_bits <= 0;
            publish(&XL.p_go, (int32_t)mb + 1);
          }
        }
        if (P3 && max_i4_bits > 0) {
          K3S& Lp = reinterpret_cast<K3S*>(smem + sizeof(K3G) + PAD)[2 % NW];
          const int32_t at = (int32_t)mb + 1;
          if (__builtin_amdgcn_readfirstlane((int)trellis_all))   // (a scalar branch)
            r4 = run_i4_pair<true>(G, L, L, Lp, XL, 0, S, ctx, rtid, x, mbw, predrd, yl, yt,
                                   kI4NoBound, max_i4_bits, &XL.hp_i16, at, &XL.hp_rd16);
          else
            r4 = run_i4_pair<false>(G, L, L, Lp, XL, 0, S, ctx, rtid, x, mbw, predrd, yl, yt,
                                    kI4NoBound, max_i4_bits, &XL.hp_i16, at, &XL.hp_rd16);
          // (the result is the same in every lane: scalar branches on it)
          r4.ok = __builtin_amdgcn_readfirstlane(r4.ok);
          r4.nz = (uint32_t)__builtin_amdgcn_readfirstlane((int)r4.nz);
          r4.H = uni64(r4.H);
          r4.score = uni64(r4.score);
        } else if (max_i4_bits > 0) {
          const int32_t at = (int32_t)mb + 1;
          if constexpr (TR) {
            r4 = trellis_all ? run_i4<true, true>(G, L, S, ctx, rtid, x, mbw, predrd, yl, yt, true,
                                                  kI4NoBound, max_i4_bits, substamps, &XL.hp_i16,
                                                  at, &XL.hp_rd16)
                             : run_i4<false, true>(G, L, S, ctx, rtid, x, mbw, predrd, yl, yt, true,
                                                   kI4NoBound, max_i4_bits, substamps, &XL.hp_i16,
                                                   at, &XL.hp_rd16);
          } else {
            r4 = run_i4<false, true>(G, L, S, ctx, rtid, x, mbw, predrd, yl, yt, true, kI4NoBound,
                                     max_i4_bits, substamps, &XL.hp_i16, at, &XL.hp_rd16);
          }
        }
        tr_uv = TR_NOW();
        TR_ADD(K3TR_I4, tr_uv - tr_i4);
        // the luma choice as soon as the intra-16 one is out (the chroma one
        // may still be running)
        if (!wait_ge(G, L, &XL.hp_i16, (int32_t)mb + 1, 7)) break;
        K3_STAMP(3);
        best16 = __builtin_amdgcn_readfirstlane(XL.hp_best16);
        const score_t D16 = XL.hp_D16, SD16 = XL.hp_SD16, H16 = XL.hp_H16, R16 = XL.hp_R16;
        const uint32_t nz16 = __builtin_amdgcn_readfirstlane(XL.hp_nz16);
        // (worker-uniform, through readfirstlane: the branches on the choice are scalar)
        const score_t rd16 = uni64((R16 + H16) * S.lambda_mode + 256 * (D16 + SD16));
        if (tid < 64) {   // whole wave 0: a lone-lane store here spills
          L.mdist = (int32_t)D16;
          L.ry16 = (int32_t)R16;
        }
        if (r4.ok && r4.score < rd16) {
          is_i16 = 0;
          if (tid == 0) L.mdist = L.d4acc;
          rdH = r4.H;
          rd_score = r4.score;
          rd_nz = r4.nz;
          L.yout[(tid >> 4) * BPS + (tid & 15)] = L.acc_out[tid];
          (&L.fin_ac[0][0])[tid] = (&L.acc_ac[0][0])[tid];
        } else {
          rdH = H16;
          rd_score = rd16;
          rd_nz = nz16;
          L.yout[(tid >> 4) * BPS + (tid & 15)] = L.rec16[best16][tid];
          (&L.fin_ac[0][0])[tid] = (&L.lv16[best16][0][0])[tid];
          if (tid < 16) { L.fin_dc[tid] = L.lvdc[best16][tid]; L.modes[tid] = best16; }
        }
        if (!wait_ge(G, L, &XL.hp_done, (int32_t)mb + 1, 7)) break;
        bu = __builtin_amdgcn_readfirstlane(XL.hp_bu);
        rdH += XL.hp_bH;
        rd_score += XL.hp_bsc;
        if (tid == 0) L.mdist += L.mres[bu][0];
        rd_nz |= (uint32_t)L.mres[bu][3] << 16;
        if (tid < 128) {
          L.yout[(tid >> 4) * BPS + 16 + (tid & 15)] = L.recuv[bu][tid];
          (&L.fin_uv[0][0])[tid] = (&L.lvuv[bu][0][0])[tid];
        }
        wbar(L);
      } else {
      // ---- Intra16 (quant_enc.c:1002-1058)
      const uint64_t tr_i16 = TR_NOW();
      if constexpr (TR) {
        if (trellis_all) eval_i16<true>(G, L, S, ctx, tid, L);
        else eval_i16<false>(G, L, S, ctx, tid, L);
      } else {
        eval_i16<false>(G, L, S, ctx, tid, L);
      }
      TR_SINCE(K3TR_I16, tr_i16);
      uint32_t nz16 = 0;
      score_t D16 = 0, SD16 = 0, H16 = 0, R16 = 0;
      {
        // IsFlatSource16 per wave (each lane checks 4 of the 256 samples): no barrier
        const int v0 = L.yin[0];
        int same = 1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int p = lane + 64 * q;
          same &= L.yin[(p >> 4) * BPS + (p & 15)] == v0;
        }
        int flat = __all(same);
        score_t best16_score = 0;
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
      L.yout[(tid >> 4) * BPS + (tid & 15)] = L.rec16[best16][tid];
      (&L.fin_ac[0][0])[tid] = (&L.lv16[best16][0][0])[tid];
      if (tid < 16) { L.fin_dc[tid] = L.lvdc[best16][tid]; L.modes[tid] = best16; }
      rd_score = (R16 + H16) * S.lambda_mode + 256 * (D16 + SD16);
      rdH = H16;
      rd_nz = nz16;
      is_i16 = 1;
      if (tid < 64) {   // whole wave 0: a lone-lane store here spills
        L.mdist = (int32_t)D16;
        L.ry16 = (int32_t)R16;
      }
      if ((rd_nz & 0x100ffff) == 0x1000000 && D16 > S.min_disto) {   // StoreMaxDelta
        int mv = iabs_(L.lvdc[best16][1]);
        mv = max(mv, iabs_(L.lvdc[best16][2]));
        mv = max(mv, iabs_(L.lvdc[best16][4]));
        if (tid == 0) atomicMax(&G.max_edge[segid], mv);
      }
      // the intra-4 search opens with a worker barrier, which orders the
      // commit above before anything reads it
      if (max_i4_bits <= 0) wbar(L);
      K3_STAMP(2);

      // ---- Intra4 (quant_enc.c:1072-1165)
      const uint64_t tr_i4 = TR_NOW();
      if (max_i4_bits > 0) {
        I4Result r4;
        if constexpr (TR) {
          r4 = trellis_all ? run_i4<true>(G, L, S, ctx, rtid, x, mbw, predrd, yl, yt, true,
                                          rd_score, max_i4_bits, substamps)
                           : run_i4<false>(G, L, S, ctx, rtid, x, mbw, predrd, yl, yt, true,
                                           rd_score, max_i4_bits, substamps);
        } else {
          r4 = run_i4<false>(G, L, S, ctx, rtid, x, mbw, predrd, yl, yt, true, rd_score,
                             max_i4_bits, substamps);
        }
        if (r4.ok) {
          is_i16 = 0;
          if (tid == 0) L.mdist = L.d4acc;
          rdH = r4.H;
          rd_score = r4.score;
          rd_nz = r4.nz;
          L.yout[(tid >> 4) * BPS + (tid & 15)] = L.acc_out[tid];
          (&L.fin_ac[0][0])[tid] = (&L.acc_ac[0][0])[tid];
        } else {
          if (tid < 16) L.modes[tid] = best16;   // the aborted search wrote some
        }
        // (no barrier: the chroma search reads none of this, and its own
        // barriers order it before the readers -- info, SSE, tokens)
      }
      K3_STAMP(3);
      tr_uv = TR_NOW();
      TR_ADD(K3TR_I4, tr_uv - tr_i4);

      // ---- UV (quant_enc.c:1169-1217)
      {
        eval_uv(G, L, S, ctx, tid, x, derrrd, use_derr, L);
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
        if (tid == 0) L.mdist += L.mres[bu][0];
        rd_nz |= (uint32_t)L.mres[bu][3] << 16;
        if (tid < 128) {
          L.yout[(tid >> 4) * BPS + 16 + (tid & 15)] = L.recuv[bu][tid];
          (&L.fin_uv[0][0])[tid] = (&L.lvuv[bu][0][0])[tid];
        }
        if (use_derr && tid < 2) {   // StoreDiffusionErrors (quant_enc.c:909-920)
          const int cch = tid;
          int8_t* top = topderr + 4 * x + 2 * cch;
          int8_t* left = L.lderr[cch];
          const int8_t* e = L.uvderr[bu][cch];
          left[0] = e[0];
          left[1] = (int8_t)(3 * e[2] >> 2);
          top[0] = e[1];
          top[1] = (int8_t)(e[2] - left[1]);
        }
        wbar(L);
      }
      }   // (!HP)

      // ---- m5: final re-quantisation of the chosen modes with trellis
      // (SimpleQuantize, quant_enc.c:1222-1245; RD_OPT_TRELLIS, :1384-1387)
      if (TR && rd_opt == 2) {
        uint32_t nzq = 0;
        if constexpr (!TR) {
        } else if (__builtin_amdgcn_readfirstlane((int)is_i16)) {   // (a scalar branch)
          eval_i16<true>(G, L, S, ctx, tid, L);
          L.yout[(tid >> 4) * BPS + (tid & 15)] = L.rec16[best16][tid];
          (&L.fin_ac[0][0])[tid] = (&L.lv16[best16][0][0])[tid];
          if (tid < 16) L.fin_dc[tid] = L.lvdc[best16][tid];
          nzq = (uint32_t)L.mres[best16][3];
        } else {
          I4Result r4 = run_i4<true>(G, L, S, ctx, rtid, x, mbw, predrd, yl, yt, false, 0, 0,
                                     substamps);
          L.yout[(tid >> 4) * BPS + (tid & 15)] = L.acc_out[tid];
          (&L.fin_ac[0][0])[tid] = (&L.acc_ac[0][0])[tid];
          nzq = r4.nz;
        }
        wbar(L);
        eval_uv(G, L, S, ctx, tid, x, topderr, use_derr, L);   // derr state already updated
        if (tid < 128) {
          L.yout[(tid >> 4) * BPS + 16 + (tid & 15)] = L.recuv[bu][tid];
          (&L.fin_uv[0][0])[tid] = (&L.lvuv[bu][0][0])[tid];
        }
        rd_nz = nzq | ((uint32_t)L.mres[bu][3] << 16);
        wbar(L);
      }
      (void)rd_score;
      K3_STAMP(4);
      const uint64_t tr_tok = TR_NOW();
      TR_ADD(K3TR_UV, tr_tok - tr_uv);

      // ---- per-MB info + side statistics
      const int skip = rd_nz == 0;
      if (tid == 0) {
        (void)K3CK(mb < (uint32_t)nmb, 14, mb, nmb, mb);
        uint8_t* info = mbinfo + (size_t)mb * VP8G_MBINFO_BYTES;
        info[0] = is_i16; info[1] = bu; info[2] = segid; info[3] = skip;
        atomicAdd(&G.fs.nb[is_i16 ? 1 : 0], 1);
        if (skip) atomicAdd(&G.fs.nb[2], 1);
        atomicAdd(&G.fs.size_p0, (unsigned long long)rdH);
        if constexpr (!TR) {   // R of the chosen luma modes + the chosen UV mode's R
          // with its flatness penalty (StatLoop passes run RD_OPT_BASIC, never TR)
          const int ruv = L.mres[bu][1] + ((bu > 0 && L.mres[bu][2] <= 2) ? 140 * 8 : 0);
          atomicAdd(&G.fs.size_rh,
                    (unsigned long long)(rdH + (is_i16 ? L.ry16 : L.r4acc) + ruv));
        }
        atomicAdd(&G.fs.dist, (unsigned long long)L.mdist);
      }
      if (tid < 16) mbinfo[(size_t)mb * VP8G_MBINFO_BYTES + 4 + tid] = L.modes[tid];
      if constexpr (AF) {   // VP8StoreFilterStats input (filter_enc.c:179)
        // (a separate instantiation: any extra store here makes the default
        // kernel spill at its 168-VGPR budget)
        if (tid < 128)
          reinterpret_cast<uint32_t*>(P->recon_addr + ((size_t)mb << 9))[tid] =
              reinterpret_cast<const uint32_t*>(L.yout)[tid];
      }
      if (w0) {   // SSE for WebPAuxStats (frame_enc.c:480-489)
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
        sy = sum64(sy); su = sum64(su); sv = sum64(sv);
        if (lane == 0) {
          atomicAdd(&G.fs.sse[0], (unsigned long long)sy);
          atomicAdd(&G.fs.sse[1], (unsigned long long)su);
          atomicAdd(&G.fs.sse[2], (unsigned long long)sv);
        }
      }

#ifdef K3_PF
      if (x + 1 < mbw) pf = fetch_mb256(Yp, Up, Vp, w, h, x + 1, y, tid);
#endif
      // ---- tokens (token_enc.c:113-193) into this MB's slot; one (block,
      // zigzag position) item per thread, counts + scan + writes in parallel
      const int first_blk = is_i16 ? 0 : 1;
      // this MB's place in its row: read before the scan barrier below, after
      // which one thread moves the row's fill on
      const uint32_t rfill = rows ? L.rowfill : 0u;
      uint64_t nzb = 0;
      int lvi[2], lvp[2];
      if constexpr (HP) {
        // the helper writes the tokens (see there); the blocks' nz bits come
        // from the decision's (rd_nz: luma blocks 0-15 -- AC only for
        // intra-16 --, chroma << 16, the intra-16 DC block << 24), in token
        // block order (0 = Y2, 1-16 luma, 17-24 chroma)
        nzb = ((uint64_t)(rd_nz & 0xffffu) << 1) | ((uint64_t)((rd_nz >> 16) & 0xffu) << 17) |
              (is_i16 ? (uint64_t)((rd_nz >> 24) & 1u) : 0ull);
        if (tid == 0) {
          XL.tk_ctx_t = ctx.t; XL.tk_ctx_l = ctx.l; XL.tk_first = first_blk;
          publish(&XL.hp_tokgo, (int32_t)mb + 1);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) {   // items rtid and rtid + 256 = block*16 + pos
          const int item = rtid + K3T * q, k = item >> 4, n = item & 15;
          int v = 0, vp = 0;
          if (k < 25 && k >= first_blk) {
            const int16_t* lvb = blk_levels(L, k);
            v = lvb[n];
            vp = n > 0 ? lvb[n - 1] : 0;
          }
          lvi[q] = v;
          lvp[q] = vp;
          const int last = max16(v != 0 ? n : -1);
          if (n == 0 && k < 32) L.blast[k] = last;
        }
        wbar(L);
        // every wave derives the blocks' nz bits and its items' block
        // parameters itself (no second barrier): type | first << 4 | ctx << 8
        nzb = __ballot(lane >= first_blk && lane < 25 && L.blast[lane] >= 0);
      }
      auto blk_param = [&](int k) -> int {
        if (k < first_blk || k >= 25) return -1;
        if (k == 0) return 1 | ((ctx.top(8) + ctx.left(8)) << 8);
        if (k <= 16) {
          const int b = k - 1, bx = b & 3, by = b >> 2;
          const int t = by == 0 ? ctx.top(bx) : (int)((nzb >> (k - 4)) & 1);
          const int l = bx == 0 ? ctx.left(by) : (int)((nzb >> (k - 1)) & 1);
          return (is_i16 ? 0 | (1 << 4) : 3) | ((t + l) << 8);
        }
        const int b = k - 17, ch = b >> 2, k4 = b & 3, bx = k4 & 1, by = k4 >> 1;
        const int t = by == 0 ? ctx.top(4 + 2 * ch + bx) : (int)((nzb >> (k - 2)) & 1);
        const int l = bx == 0 ? ctx.left(4 + 2 * ch + by) : (int)((nzb >> (k - 1)) & 1);
        return 2 | ((t + l) << 8);
      };
      if constexpr (!HP) {
        int cnt[2], bi[2], last[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int item = rtid + K3T * q, k = item >> 4, n = item & 15;
          bi[q] = blk_param(k);
          last[q] = k < 25 ? L.blast[k] : -1;
#ifndef K3_NO_CNT   // (branch-free count: 105.8 -> 105.1 ms, r5s19)
          cnt[q] = bi[q] < 0 ? 0 : pos_count((bi[q] >> 4) & 15, n, lvi[q], lvp[q], last[q]);
#else
          cnt[q] = bi[q] < 0 ? 0
                             : pos_tokens<false>(bi[q] & 15, (bi[q] >> 4) & 15, bi[q] >> 8, n,
                                                 lvi[q], lvp[q], last[q], nullptr, nullptr);
#endif
        }
        int inc0 = cnt[0], inc1 = cnt[1];
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int v0 = __shfl_up(inc0, off), v1 = __shfl_up(inc1, off);
          if (lane >= off) { inc0 += v0; inc1 += v1; }
        }
        const int wv = rtid >> 6;
        if (lane == 63) { L.wsum[0][wv] = inc0; L.wsum[1][wv] = inc1; }
        wbar(L);
        int pre0 = 0, pre1 = 0, tot0 = 0, tot1 = 0;
#pragma unroll
        for (int w2 = 0; w2 < 4; ++w2) {
          const int s0 = L.wsum[0][w2], s1 = L.wsum[1][w2];
          if (w2 < wv) { pre0 += s0; pre1 += s1; }
          tot0 += s0; tot1 += s1;
        }
        uint16_t* slot = rows ? tok_base + (size_t)y * a.rowcap + rfill
                              : tok_base + (size_t)mb * VP8G_MAX_TOKENS_PER_MB;
        const int off0 = pre0 + inc0 - cnt[0];
        const int off1 = tot0 + pre1 + inc1 - cnt[1];
        // a row that would pass its room writes nothing more: the frame is
        // encoded again with wider rows (VP8G_ERR_ARENA; worker-uniform)
        const bool over = rows && rfill + (uint32_t)(tot0 + tot1) > a.rowcap;
        if (over) { cnt[0] = 0; cnt[1] = 0; }
#ifdef K3_CHECK
        if (rows) {
          const unsigned long long top = (unsigned long long)rfill + tot0 + tot1;
          if (!over && !K3CK(top <= CK_CAP(L, ~0u) && tot0 + tot1 <= VP8G_MAX_TOKENS_PER_MB, 15,
                             rfill, tot0 + tot1, mb)) {
            cnt[0] = 0; cnt[1] = 0;
          }
        }
#endif
        if (cnt[0])
          pos_tokens<true>(bi[0] & 15, (bi[0] >> 4) & 15, bi[0] >> 8, rtid & 15, lvi[0], lvp[0],
                           last[0], slot + off0, L.rdelta);
        if (cnt[1])
          pos_tokens<true>(bi[1] & 15, (bi[1] >> 4) & 15, bi[1] >> 8, rtid & 15, lvi[1], lvp[1],
                           last[1], slot + off1, L.rdelta);
        if (rtid == 0) {
          L.rowcnt[x] = (uint16_t)(tot0 + tot1);
          if (rows) {
            L.rowpos[x] = rfill;
            L.rowfill = rfill + (uint32_t)(tot0 + tot1);   // read by the next MB after the barriers
            if (over) atomicOr(&G.tok_err, VP8G_ERR_ARENA);
          }
        }
      }
      K3_STAMP(5);
      TR_SINCE(K3TR_TOK, tr_tok);
      // update nz context (iterator_enc.c:267-283) and the left DC flag
      if (rtid == 0) {
        int tn9[9], ln[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) { tn9[i] = ctx.top(i); ln[i] = ctx.left(i); }
        if (is_i16) { tn9[8] = ln[8] = (int)(nzb & 1); }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tn9[i] = (int)((nzb >> (1 + 12 + i)) & 1);      // block (i, 3)
          ln[i] = (int)((nzb >> (1 + 4 * i + 3)) & 1);    // block (3, i)
        }
#pragma unroll
        for (int ch = 0; ch < 2; ++ch)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            tn9[4 + 2 * ch + i] = (int)((nzb >> (17 + 4 * ch + 2 + i)) & 1);
            ln[4 + 2 * ch + i] = (int)((nzb >> (17 + 4 * ch + 2 * i + 1)) & 1);
          }
        uint32_t word = 0;
        word |= (tn9[0] << 12) | (tn9[1] << 13) | (tn9[2] << 14) | (tn9[3] << 15) |
                (tn9[4] << 18) | (tn9[5] << 19) | (tn9[6] << 22) | (tn9[7] << 23) | (tn9[8] << 24);
        word |= (ln[0] << 3) | (ln[1] << 7) | (ln[2] << 11) | (ln[4] << 17) | (ln[6] << 21);
        nzw[x] = word;
        L.flag_ldc = ln[8];
      }

      // ---- boundary save (iterator_enc.c:290-313) + mode context, in the
      // same phase as the nz words: the left corners (yl[-1], ul[-1], vl[-1]
      // = the row above's samples at columns 15 / 7 / 15 of this MB) are read
      // by the threads that then overwrite those samples in ytop / uvtop
      if (x < mbw - 1) {
        if (tid < 16) yl[tid] = L.yout[15 + tid * BPS];
        if (tid < 8) { ul[tid] = L.yout[16 + 7 + tid * BPS]; vl[tid] = L.yout[24 + 7 + tid * BPS]; }
        if (tid == 15) { yl[-1] = yt[15]; vl[-1] = uvt[15]; }
        if (tid == 7) ul[-1] = uvt[7];
      }
      if (y < mbh - 1) {
        if (tid < 16) {
          ytop[16 * x + tid] = L.yout[15 * BPS + tid];
          uvtop[16 * x + tid] = L.yout[7 * BPS + 16 + tid];
        }
      }
      if (tid < 4) {
        predtop[4 * x + tid] = L.modes[12 + tid];
        L.predleft[tid] = L.modes[4 * tid + 3];
      }
      if (tid == 0)
        L.epseen = __hip_atomic_load(&G.epoch, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      wbar(L);
      left_dc = L.flag_ldc;
      if (tid == 0) publish(&rowdone[y], x + 1);
      if constexpr (X) {
        // the last worker's row feeds worker 0 of the next workgroup: its
        // boundary record for column x, drained, then the column count
        const uint64_t tr_x = TR_NOW();
        if (HP) {   // the helper publishes the record
          if (tid == 0) publish(&XL.hp_bnd, (int32_t)mb + 1);
        } else if (wk == NW - 1 && y < mbh - 1 && tid < 64) {
          if (tid < 11) {
            uint32_t v;
            if (tid < 4) v = reinterpret_cast<const uint32_t*>(ytop + 16 * x)[tid];
            else if (tid < 8) v = reinterpret_cast<const uint32_t*>(uvtop + 16 * x)[tid - 4];
            else if (tid == 8) v = nzw[x];
            else if (tid == 9) v = reinterpret_cast<const uint32_t*>(predtop + 4 * x)[0];
            else v = reinterpret_cast<const uint32_t*>(topderr + 4 * x)[0];
            st_sc1(xrec + ((size_t)y * mbw + x) * XS_REC_WORDS + tid, v);
          }
          vm_drain();
          if (tid == 0) st_sc1(&xrowdone[y], x + 1);
        }
        TR_SINCE(K3TR_REPLAY, tr_x);   // (K3X: the boundary record's publish)
      }
      if ((x + 1) % XS_SNAP_MBS == 0 && x + 1 < mbw) {
        if constexpr (HP) {   // the helper's tokens (and their pending deltas) up to here
          if (!wait_ge(G, L, &XL.hp_tok, (int32_t)mb + 1, 11)) break;
        }
        // every XS_SNAP_MBS-th column: the statistics snapshot (see fold_mbs);
        // every K3_DFULL_EVERY-th the 16-bit count / ones of the row's pending
        // deltas checked: an MB adds at most 288 to one slot (9 positions of a
        // band, 2 counted tokens each, 16 blocks), so a pending field past
        // K3_DFULL folds the row's MBs so far now, before it could wrap (a
        // very wide, noisy picture at high quality)
        uint32_t* sr = snap_of(y);
#ifdef K3_NO_SNAP
        sr = nullptr;
#endif
        if (sr) sr += (size_t)((x + 1) / XS_SNAP_MBS - 1) * NSLOT;
        uint32_t big = 0;
        for (int s = tid; s < NSLOT; s += K3T) {
          const uint32_t d = L.rdelta[s];
          if (sr) st_sc1(sr + s, d);
          big |= (uint32_t)((d >> 16) >= K3_DFULL) | (uint32_t)((d & 0xffffu) >= K3_DFULL);
        }
        if (sr) vm_drain();
#ifdef K3_NO_DFULL   // (A/B) without the check
        big = 0;
        if (false) {
#else
        if ((x + 1) % K3_DFULL_EVERY == 0 &&
            !wbar_and(L, big == 0)) {   // (a wave-uniform result: a scalar branch)
#endif
          const uint32_t mb1 = mb + 1;
          if constexpr (X) {
            if (!wait_gx(G, L, &XH->fold_ptr, (int32_t)fold_from, XH)) break;
          } else {
            if (!wait_ge(G, L, (const int32_t*)&G.fold_ptr, (int32_t)fold_from, 4)) break;
          }
          fold_rows<X>(G, L, tid, fold_from, mb1, (uint32_t)y * mbw, tok_base, mboff, xs, rowbase_of(y),
                       snap_of(y));
          fold_from = mb1;
          wbar(L);
        }
      }
      K3_STAMP(6);
      TR_SINCE(K3TR_MB, tr_mb);
    }
    if (L.myabort) break;
    if constexpr (HP) {   // the helper's tokens of the whole row
      if (!wait_ge(G, L, &XL.hp_tok, (int32_t)(y + 1) * mbw, 11)) break;
    }
    // row end: fold this row's remaining MBs once the rows above are folded
    const uint64_t tr_fw = TR_NOW();
    if constexpr (X) {
      if (!wait_gx(G, L, &XH->fold_ptr, (int32_t)fold_from, XH)) break;
    } else {
      if (!wait_ge(G, L, (const int32_t*)&G.fold_ptr, (int32_t)fold_from, 4)) break;
    }
    const uint64_t tr_ff = TR_NOW();
    TR_ADD(K3TR_FOLD_WAIT, tr_ff - tr_fw);
    fold_rows<X>(G, L, tid, fold_from, (uint32_t)(y + 1) * mbw, (uint32_t)y * mbw, tok_base,
                 mboff, xs, rowbase_of(y), snap_of(y));
    TR_SINCE(K3TR_FOLD, tr_ff);
    report_rows<X>(G, L, P, tid, (uint32_t)(y + 1) * mbw, mbw, XH);
    if (rows && tid == 0) a.rowtok[(size_t)f * mbh + y] = L.rowfill;   // K4's row length
    wbar(L);
    K3_STAMP(7);
  }

  // ---- frame epilogue: final probabilities and side results
#ifdef K3_TRACE
  TR_SINCE(K3TR_TOTAL, tr_start);
  if (tid < K3TR_N && blockIdx.x < K3TR_MAXB) g_k3trace[blockIdx.x][wk & 3][tid] = L.trace[tid];
#endif
  __syncthreads();
  if constexpr (X) {   // this workgroup's share of the side statistics; k_encode_xtail finishes
    if (gt == 0) {
      atomicAdd(&XH->size_p0, G.fs.size_p0);
      atomicAdd(&XH->size_rh, G.fs.size_rh);
      for (int c = 0; c < 3; ++c) {
        atomicAdd(&XH->sse[c], G.fs.sse[c]);
        atomicAdd(&XH->nb[c], G.fs.nb[c]);
      }
      atomicAdd(&XH->dist, G.fs.dist);
      for (int c = 0; c < 4; ++c) atomicMax(&XH->max_edge[c], G.max_edge[c]);
      if (G.tok_err) atomicOr(&XH->tok_err, G.tok_err);
      if (G.abort) atomicOr(&XH->abort, 1);
#ifdef K3_SUBPROF   // row 0's main worker's intra-4 split (k_encode_xtail keeps it)
      if (blk == 0)
        for (int i = 0; i < 8; ++i) a.results[f].stamps[i] = subacc[i];
#endif
    }
    return;
  }
  if (!rows && !G.abort && !G.tok_err) compact_tokens(G, tok_base, mboff, nmb);
  __syncthreads();
  if (wk == 0) {
    for (int s = tid; s < NSLOT && !(G.tok_err & VP8G_ERR_ARENA); s += K3T) {
      rstate[NSLOT + s] = G.coeffs[s];
      rstats[s] = G.stats[s];
    }
    finalize_probas_wg(G, L, tid);
    vp8g_frame_result* R = a.results + f;
    for (int s = tid; s < NSLOT; s += K3T) R->probas[s] = G.coeffs[s];
    if (tid == 0) {
      R->ntokens = G.ntok;
      R->error = G.abort ? 2 | (G.abort << 4) : G.tok_err;
      for (int s = 0; s < 4; ++s) R->max_edge[s] = G.max_edge[s];
      R->size_p0 = G.fs.size_p0;
      R->size_rh = G.fs.size_rh;
      R->sse[0] = G.fs.sse[0]; R->sse[1] = G.fs.sse[1]; R->sse[2] = G.fs.sse[2];
      R->distortion = G.fs.dist;
      R->use_skip = 0;     // the token loop never uses the skip flag (frame_enc.c:805)
      R->skip_proba = 255;
      R->block_count[0] = G.fs.nb[0]; R->block_count[1] = G.fs.nb[1];
      R->block_count[2] = G.fs.nb[2];
#if defined(K3_STAMPS)
      for (int i = 0; i < 8; ++i) R->stamps[i] = stamps[i];   // worker 0, wave 0
#elif defined(K3_SUBPROF)
      for (int i = 0; i < 8; ++i) R->stamps[i] = subacc[i];
#else
      for (int i = 0; i < 8; ++i) R->stamps[i] = 0;
#endif
    }
  }
}


// K3X frame end, one 256-thread workgroup per frame after k_encode<.., X>:
// the compact token stream, the state a later pass starts from, the final
// probabilities and the side results, all from the frame's xsync block (the
// k_encode epilogue, with the workgroups' shares merged)
__global__ __launch_bounds__(K3T) void k_encode_xtail(K3Args a) {
  extern __shared__ __align__(16) uint8_t smem[];
  K3G& G = *reinterpret_cast<K3G*>(smem);
  K3S& L = *reinterpret_cast<K3S*>(smem + sizeof(K3G));
  const int f = blockIdx.x, tid = threadIdx.x, nmb = a.mbw * a.mbh;
  const vp8g_frame_params* P = a.params + f;
  if (P->pass_mode == 2) return;
  const bool rerun = P->pass_mode == 1 || P->pass_mode == 3;
  uint8_t* rstate = a.rerun + (size_t)f * VP8G_RERUN_STATE_BYTES;
  uint32_t* rstats = reinterpret_cast<uint32_t*>(rstate + VP8G_STATE_STATS);
  const uint8_t* xs = a.xs + (size_t)f * a.xs_fb;
  const XHdr* XH = reinterpret_cast<const XHdr*>(xs);
  const uint32_t* xstats = reinterpret_cast<const uint32_t*>(xs + XS_STATS);
  uint16_t* tok_base = a.tokens + f * a.tok_cap;
  const uint32_t* mboff = a.mboff + (size_t)f * nmb;
  const int32_t ep = XH->epoch, lcver = XH->lcver;
  for (int s = tid; s < NSLOT; s += K3T) {
    G.stats[s] = xstats[s];
    // the loop-end probabilities: the last epoch's, else the start state's
    G.coeffs[s] = ep > 0 ? xs[XS_COEFFS + s]
                         : (rerun ? rstate[NSLOT + s] : (&kVP8CoeffProba0[0][0][0][0])[s]);
  }
  for (int k = tid; k < 256; k += K3T) G.ecost[k] = kVP8EntropyCost[k];
  if (tid == 0) {
    L.bar = 0; L.myabort = 0;
    G.ntok = XH->ntok;
    G.mark[0] = 0;
  }
  __syncthreads();
  const int err = XH->uabort ? 2 | (6 << 4) : XH->abort ? 2 : XH->tok_err;
  if (!err && !a.rowtok) compact_tokens(G, tok_base, mboff, nmb);
  __syncthreads();
  for (int s = tid; s < NSLOT && !(XH->tok_err & VP8G_ERR_ARENA); s += K3T) {
    if (lcver > 0) rstate[s] = xs[XS_LCOEFFS + s];   // the level costs' probabilities
    rstate[NSLOT + s] = G.coeffs[s];
    rstats[s] = G.stats[s];
  }
  finalize_probas_wg(G, L, tid);
  vp8g_frame_result* R = a.results + f;
  for (int s = tid; s < NSLOT; s += K3T) R->probas[s] = G.coeffs[s];
  if (tid == 0) {
    R->ntokens = G.ntok;
    R->error = err;
    for (int s = 0; s < 4; ++s) R->max_edge[s] = XH->max_edge[s];
    R->size_p0 = XH->size_p0;
    R->size_rh = XH->size_rh;
    R->sse[0] = XH->sse[0]; R->sse[1] = XH->sse[1]; R->sse[2] = XH->sse[2];
    R->distortion = XH->dist;
    R->use_skip = 0;
    R->skip_proba = 255;
    R->block_count[0] = XH->nb[0]; R->block_count[1] = XH->nb[1];
    R->block_count[2] = XH->nb[2];
#if !defined(K3_SUBPROF)   // (that build: row 0's main worker's, from k_encode)
    for (int i = 0; i < 8; ++i) R->stamps[i] = 0;
#endif
  }
}
// ---------------------------------------------------------------------------

template <int NW>
static size_t k3_lds_bytes(int mbw, int mbh, bool trellis, size_t pad = 0) {
  (void)trellis;   // (the trellis keeps its nodes in registers: no LDS of its own)
  return sizeof(K3G) + pad + NW * sizeof(K3S) + (16 * mbw + 16) + 16 * mbw + 4 * (mbw + 1) + 4 * mbw +
         4 * mbw + 4 * mbh + 16;
}

#ifdef WEBP_AMD_DIAG
extern "C" int vp8g_launch_encode_w1(const uint8_t* yuv, size_t yfb, int w, int h, int n,
                                     const uint8_t* segmap, const vp8g_frame_params* params,
                                     uint16_t* tokens, size_t tok_cap, uint8_t* mbinfo,
                                     vp8g_frame_result* results, void* stream);
#endif
extern "C" int vp8g_launch_check(const char* what);

template <int NW, bool TR, bool AF = false, int WPE = 1, int PAD = 0>
static int launch_k3_t(const K3Args& a, int n, bool trellis, void* stream) {
  const size_t lds = k3_lds_bytes<NW>(a.mbw, a.mbh, trellis, PAD);
  if (lds > 160 * 1024) {
    vp8g_set_error("k_encode", "frame too wide for the LDS budget");
    return 0;
  }
  if (lds > 64 * 1024) {   // beyond the default dynamic-LDS limit: opt in
    // once, to the whole 160 KB: engines on other host threads launch this
    // kernel concurrently, and a smaller opt-in landing after a larger one
    // would lower the limit under the other launch
    static std::once_flag once;
    static hipError_t attr_err = hipSuccess;
    std::call_once(once, [] {
      attr_err = hipFuncSetAttribute((const void*)k_encode<NW, TR, AF, false, WPE, PAD>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    });
    if (attr_err != hipSuccess) {
      vp8g_set_error("k_encode dynamic LDS opt-in", hipGetErrorString(attr_err));
      return 0;
    }
  }
  hipLaunchKernelGGL((k_encode<NW, TR, AF, false, WPE, PAD>), dim3(n), dim3(NW * K3T), lds,
                     (hipStream_t)stream, a);
  // WEBP_AMD_SYNC_K3=1: wait for K3 (fault localisation)
  static const bool sync_each = getenv("WEBP_AMD_SYNC_K3") != nullptr;
  if (sync_each) {
    const hipError_t e = hipStreamSynchronize((hipStream_t)stream);
    if (e != hipSuccess) {
      vp8g_set_error("k_encode (synchronised)", hipGetErrorString(e));
      return 0;
    }
  }
  return vp8g_launch_check("k_encode");
}

#ifdef WEBP_AMD_DIAG
template <int NW>
static int launch_k3(const K3Args& a, int n, bool trellis, void* stream) {
  return trellis ? launch_k3_t<NW, true>(a, n, true, stream)
                 : launch_k3_t<NW, false>(a, n, false, stream);
}
#endif

static std::atomic<int> g_x_free{-1};   // K3X workgroup budget (k3x_take)

static void k3x_release(void* p) { g_x_free.fetch_add((int)(intptr_t)p); }

// K3X: grid n * nwg main workgroups, then the per-frame tail
static size_t k3x_lds_extra(int mbw) {
  return ((sizeof(K3XL) + 15) & ~(size_t)15) + 44 * (size_t)mbw + 32;
}

template <int NW, bool TR, bool HP = false, bool P3 = false>
static int launch_k3x(K3Args a, int n, int nwg, void* stream) {
  const size_t lds = k3_lds_bytes<NW>(a.mbw, a.mbh, TR) + k3x_lds_extra(a.mbw);
  const size_t lds_tail = sizeof(K3G) + sizeof(K3S);
  if (lds > 160 * 1024) {
    vp8g_set_error("k_encode (K3X)", "frame too wide for the LDS budget");
    return 0;
  }
  // one opt-in to the whole 160 KB per kernel (see launch_k3_t)
  static std::once_flag once;
  static hipError_t attr_err = hipSuccess;
  std::call_once(once, [] {
    attr_err = hipFuncSetAttribute((const void*)k_encode<NW, TR, false, true, 1, 0, HP, P3>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr_err == hipSuccess)
      attr_err = hipFuncSetAttribute((const void*)k_encode_xtail,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  });
  if (attr_err != hipSuccess) {
    vp8g_set_error("k_encode (K3X) dynamic LDS opt-in", hipGetErrorString(attr_err));
    return 0;
  }
  (void)lds_tail;
  a.nwg = nwg;
  if (hipMemsetAsync(a.xs, 0, (size_t)n * a.xs_fb, (hipStream_t)stream) != hipSuccess) {
    vp8g_set_error("k_encode (K3X)", "xsync reset failed");
    return 0;
  }
  hipLaunchKernelGGL((k_encode<NW, TR, false, true, 1, 0, HP, P3>), dim3(n * nwg), dim3(NW * K3T), lds,
                     (hipStream_t)stream, a);
  if (!vp8g_launch_check("k_encode (K3X)")) return 0;
  hipLaunchKernelGGL(k_encode_xtail, dim3(n), dim3(K3T), lds_tail, (hipStream_t)stream, a);
  return vp8g_launch_check("k_encode_xtail");
}

template <int NW, bool TR, bool HP = false, bool P3 = false>
static int launch_k3x_budget(const K3Args& a, int n, int nwg, void* stream) {
  const int ok = launch_k3x<NW, TR, HP, P3>(a, n, nwg, stream);
  // give the workgroups back once the stream has passed the kernels (at once
  // if they never got enqueued)
  if (!ok || hipLaunchHostFunc((hipStream_t)stream, k3x_release,
                               (void*)(intptr_t)(n * nwg)) != hipSuccess) {
    if (ok) (void)hipStreamSynchronize((hipStream_t)stream);
    k3x_release((void*)(intptr_t)(n * nwg));
  }
  return ok;
}

// K3X workgroups wait on each other, so every workgroup of a launch must be
// resident at once. Launches from several engines (concurrent WebPEncode
// callers on their own streams) share one process-wide budget of one
// workgroup per CU: a launch takes what it uses before it is enqueued and a
// host callback on its stream gives it back when its kernels have finished.

// workgroups per frame for K3X: fill the free CUs with the frames' MB rows
// (NW rows per workgroup), taken from the budget; 1 = the one-workgroup kernel
static int k3x_take(int n, int mbh, int nw) {
  static const int mode = [] {   // WEBP_AMD_K3X=0 turns the split off (A/B)
    const char* v = getenv("WEBP_AMD_K3X");
    return (v && v[0] == '0') ? 0 : 1;
  }();
  if (!mode || n > VP8G_XSPLIT_MAX_FRAMES) return 1;
  int cur = g_x_free.load();
  if (cur < 0) {   // first use: one workgroup per CU of the device
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
      cus = 256;
    int expect = -1;
    g_x_free.compare_exchange_strong(expect, cus);
    cur = g_x_free.load();
  }
  const int rows = (mbh + nw - 1) / nw;
  for (;;) {
    const int nwg = min(cur / n, rows);
    if (nwg < 2) return 1;
    if (g_x_free.compare_exchange_weak(cur, cur - n * nwg)) return nwg;
  }
}

// default: 4 MB workers for m3/m4 frames (a 1,024-thread workgroup held to
// 128 VGPRs, 120 B/lane of scratch: 16 waves per CU hide more of each MB's
// dependency latency than 12 waves with 168 VGPRs -- K3 116.9 -> 105.4 ms,
// profiles/r4/nw4a_*), 2 when the trellis paths are in the kernel, 3 for the
// autofilter instantiation
static int launch_k3_default(const K3Args& a, int n, bool trellis, bool af, void* stream) {
  if (af)
    return trellis ? launch_k3_t<2, true, true>(a, n, true, stream)
                   : launch_k3_t<3, false, true>(a, n, false, stream);
  return trellis ? launch_k3_t<2, true>(a, n, true, stream)
                 : launch_k3_t<4, false>(a, n, false, stream);
}

#ifdef K3_CHECK
// check build: the index-check record (count, site, workgroup, thread, MB,
// value, bound) since the last call, then cleared
extern "C" __attribute__((visibility("default"))) int vp8g_k3_check(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k3check), 7 * sizeof(unsigned long long), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  unsigned long long z[8] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_k3check), z, sizeof(z), 0, hipMemcpyHostToDevice) ==
         hipSuccess;
}
#ifdef K3_BARCHECK
extern "C" __attribute__((visibility("default"))) int vp8g_k3_bar(uint32_t* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k3bar), sizeof(g_k3bar), 0,
                             hipMemcpyDeviceToHost) == hipSuccess;
}
#endif
// check build: the hang records [1024][4][8] (see g_k3hang), then cleared
extern "C" __attribute__((visibility("default"))) int vp8g_k3_hang(uint32_t* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k3hang), sizeof(g_k3hang), 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return 1;
}
#endif

#ifdef K3_TRACE
// diagnostic build: trellis16 against the serial trellis_quant on random
// blocks (one wave; its 4 groups take 4 blocks per iteration) with random
// cost tables. out[0] = mismatching blocks, out[1] = blocks, out[2..] = the
// first mismatch (type, ctx0, lambda, coefficients, both level vectors).
__global__ __launch_bounds__(64) void k_trellis_selftest(int iters, uint32_t seed, int* out) {
  __shared__ K3G G;
  __shared__ uint32_t nodes[4][32];
  __shared__ int16_t lvs[4][16];
  __shared__ int cs[4][16];
  __shared__ long long dbg[64 * 16];
  const int lane = threadIdx.x, g = lane & 48, j = lane & 15, grp = lane >> 4;
  auto rnd = [](uint32_t& st) {
    st ^= st << 13; st ^= st >> 17; st ^= st << 5;
    return st;
  };
  uint32_t st = seed * 747796405u + lane * 2891336453u + 1u;
  for (int k = lane; k < 256; k += 64) G.ecost[k] = kVP8EntropyCost[k];
  for (int it = 0; it < iters; ++it) {
    // fresh tables every 64 iterations: level costs, probabilities, matrix
    if ((it & 63) == 0) {
      for (int k = lane; k < 96 * (MAX_VLEVEL + 1); k += 64)
        (&G.lcost[0][0])[k] = (uint16_t)(rnd(st) % 3000);
      for (int k = lane; k < NSLOT; k += 64) G.coeffs[k] = (uint8_t)(1 + rnd(st) % 255);
      if (lane < 16) {
        const int q = 4 + (int)(rnd(st) % 120);
        G.seg[0].y1.q[lane] = (uint16_t)q;
        G.seg[0].y1.iq[lane] = (uint16_t)((1 << QFIX) / q);
        G.seg[0].y1.sharpen[lane] = (uint16_t)(rnd(st) % 16);
      }
      __syncthreads();
    }
    const vp8g_mtx& M = G.seg[0].y1;
    const uint32_t ru = __shfl(rnd(st), g);
    const int type = (int)((ru >> 3) & 3), ctx0 = (int)(ru % 3);
    const int lambda = 1 + (int)((ru >> 8) % 4000);
    const int mag = 1 << (2 + (ru >> 20) % 10);
    const uint32_t r2 = rnd(st);
    int c = (r2 & 1) ? (int)(r2 % (2 * mag)) - mag : 0;
    c = max(-2048, min(2047, c));
    cs[grp][j] = c;
    __syncthreads();
    const Trellis16 t = trellis16<true>(G, c, true, ctx0, type, M, lambda, dbg);
    int ref_lv = 0;
    if (j == 0) {
      int cc[16];
      for (int k = 0; k < 16; ++k) cc[k] = cs[grp][k];
      trellis_quant(G, nodes[grp], cc, lvs[grp], ctx0, type, &M, lambda);
    }
    __syncthreads();
    ref_lv = lvs[grp][j];
    if (type == 0 && j == 0) ref_lv = 0;   // position 0 is left to the caller
    const uint64_t bad = __ballot(ref_lv != t.lvz);
    __shared__ int first_bad;
    if (lane == 0) {
      first_bad = -1;
      for (int q = 0; q < 4; ++q) {
        atomicAdd(&out[1], 1);
        if ((bad >> (16 * q)) & 0xffff) {
          if (atomicAdd(&out[0], 1) == 0) {
            out[2] = q; out[3] = type; out[4] = ctx0; out[5] = lambda; out[6] = it;
            first_bad = q;
          }
        }
      }
    }
    __syncthreads();
    if (grp == first_bad) {
      out[8 + j] = c; out[24 + j] = ref_lv; out[40 + j] = t.lvz;
      out[56 + j] = G.seg[0].y1.q[j]; out[72 + j] = G.seg[0].y1.sharpen[j];
      for (int k = 0; k < 32; k += 1) out[96 + 32 * 0 + k] = (int)nodes[grp][k];   // same for all lanes
      long long* o = (long long*)(out + 128);
      for (int k = 0; k < 16; ++k) o[16 * j + k] = dbg[16 * lane + k];
    }
    __syncthreads();
  }
}

extern "C" __attribute__((visibility("default"))) int vp8g_trellis_selftest(int iters,
                                                                            unsigned seed,
                                                                            int* host_out) {
  int* d = nullptr;
  if (hipMalloc(&d, 1024 * sizeof(int)) != hipSuccess) return 0;
  (void)hipMemset(d, 0, 1024 * sizeof(int));
  hipLaunchKernelGGL(k_trellis_selftest, dim3(1), dim3(64), 0, 0, iters, seed, d);
  const int ok = hipMemcpy(host_out, d, 1024 * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess;
  (void)hipFree(d);
  return ok;
}


// diagnostic build: the per-worker K3TR_* counters of the last launch,
// out[block][worker][slot] for the first nblocks workgroups
extern "C" __attribute__((visibility("default"))) int vp8g_k3_trace(unsigned long long* out,
                                                                    int nblocks) {
  if (nblocks > K3TR_MAXB) nblocks = K3TR_MAXB;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k3trace),
                             (size_t)nblocks * 4 * K3TR_N * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess
             ? nblocks
             : 0;
}
#endif

extern "C" int vp8g_launch_encode(const uint8_t* yuv, size_t yfb, int w, int h, int n,
                                  const uint8_t* segmap, const vp8g_frame_params* params,
                                  uint16_t* tokens, size_t tok_cap, uint8_t* mbinfo,
                                  uint32_t* mboff, int trellis, vp8g_frame_result* results,
                                  uint8_t* rerun_state, uint8_t* recon, uint8_t* xsync,
                                  uint32_t* wsnap, const vp8g_rows* rows, void* stream) {
#ifdef WEBP_AMD_DIAG
  // diagnostic build only (make diag -> libwebp_amd_diag.so; the product
  // library has no switch): WEBP_AMD_K3 = 1 single-wavefront twin,
  // 2/3/5 = 1/2/3 MB workers per frame, 4 = the 4-worker build, 6 = 3 workers
  // held to 128 VGPRs, 7 / 8 = 3 / 2 workers with their state moved 40 KB /
  // 64 KB up the LDS
  static const int variant = [] {
    const char* v = getenv("WEBP_AMD_K3");
    return (v && v[0] >= '1' && v[0] <= '8') ? v[0] - '0' : 0;
  }();
#else
  constexpr int variant = 0;
#endif
  // recon != NULL selects the autofilter instantiation; each frame's buffer
  // address travels in vp8g_frame_params::recon_addr
  if (recon != nullptr && variant != 0) {
    vp8g_set_error("k_encode", "the autofilter runs on the default K3 variant only");
    return 0;
  }
#ifdef WEBP_AMD_DIAG
  if (variant == 1)
    return vp8g_launch_encode_w1(yuv, yfb, w, h, n, segmap, params, tokens, tok_cap, mbinfo,
                                 results, stream);
#endif
  K3Args a;
  a.yuv = yuv; a.yfb = yfb; a.w = w; a.h = h;
  a.mbw = (w + 15) >> 4; a.mbh = (h + 15) >> 4;
  a.segmap = segmap; a.params = params; a.tokens = tokens; a.tok_cap = tok_cap;
  a.mbinfo = mbinfo; a.mboff = mboff; a.results = results; a.rerun = rerun_state;
  a.xs = xsync; a.xs_fb = vp8g_xsync_bytes(w, h); a.nwg = 1;
  a.wsnap = wsnap;
  a.rowcap = rows ? rows->rowcap : 0u;
  a.rowtok = rows ? rows->rowtok : nullptr;
  if (xsync != nullptr && recon == nullptr && variant == 0) {
    // K3X workgroups, one MB row each, every row on a CU of its own: a
    // helper pair (the MB loop + a helper for intra-16, chroma, tokens,
    // source and boundary hand-offs; m3/m4) or, for the trellis methods
    // (m5/m6), a helper pair plus an intra-4 partner taking the second
    // sub-block of the 10-step wavefront (config 4 158 -> 147 ms; at m4 the
    // pair barriers cost more than the steps save: 30.8 -> 31.7 ms,
    // profiles/r6/k3x/partner). A/B: WEBP_AMD_K3X_NW=h / p all frames one
    // way, =1 one worker (262 -> 233 / 43.2 -> 40.9 ms against 2), =2 two
    // workers with rows handed over in LDS
    static const int xnw = [] {
      const char* v = getenv("WEBP_AMD_K3X_NW");
      return (v && v[0] == '2') ? 2 : (v && v[0] == '1') ? 1 : (v && v[0] == 'p') ? 4
             : (v && v[0] == 'h') ? 3 : 0;
    }();
    const int nwg = k3x_take(n, a.mbh, xnw == 2 ? 2 : 1);
    if (nwg > 1) {
      if (xnw == 4 || (xnw == 0 && trellis))
        return trellis ? launch_k3x_budget<3, true, true, true>(a, n, nwg, stream)
                       : launch_k3x_budget<3, false, true, true>(a, n, nwg, stream);
      if (xnw == 0) return launch_k3x_budget<2, false, true>(a, n, nwg, stream);
      if (xnw == 3)
        return trellis ? launch_k3x_budget<2, true, true>(a, n, nwg, stream)
                       : launch_k3x_budget<2, false, true>(a, n, nwg, stream);
      if (xnw == 1)
        return trellis ? launch_k3x_budget<1, true>(a, n, nwg, stream)
                       : launch_k3x_budget<1, false>(a, n, nwg, stream);
      return trellis ? launch_k3x_budget<2, true>(a, n, nwg, stream)
                     : launch_k3x_budget<2, false>(a, n, nwg, stream);
    }
  }
#ifdef WEBP_AMD_DIAG
  if (variant == 2) return launch_k3<1>(a, n, trellis != 0, stream);
  if (variant == 3) return launch_k3<2>(a, n, trellis != 0, stream);
  if (variant == 4) return launch_k3<4>(a, n, trellis != 0, stream);
  if (variant == 5) return launch_k3<3>(a, n, trellis != 0, stream);
  if (variant == 6 && !trellis) return launch_k3_t<3, false, false, 4>(a, n, false, stream);
  if (variant == 7 && !trellis) return launch_k3_t<3, false, false, 1, 40960>(a, n, false, stream);
  if (variant == 8 && !trellis) return launch_k3_t<2, false, false, 1, 65536>(a, n, false, stream);
#endif
  return launch_k3_default(a, n, trellis != 0, recon != nullptr, stream);
}
