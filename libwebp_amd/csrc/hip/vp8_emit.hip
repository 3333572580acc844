// K4: the VP8 boolean coder for the token partition on the GPU, parallel
// INSIDE each frame (VP8EmitTokens, src/enc/token_enc.c:200-223; VP8PutBit /
// Flush / VP8BitWriterFinish, src/utils/bit_writer_utils.c:55-124,199-206).
//
// The coder's only serial state that matters is the 8-bit range (the "low"
// register is linear): the output bytes are exactly the big-endian bytes of
// N >> 1 on L = (S + 7) / 8 bytes, where N = sum_i c_i * 2^(E_i), c_i is the
// amount token i adds to the low register (split + 1 for a 1 bit, else 0),
// E_i the number of renormalisation shifts from token i (inclusive) to the
// end of the stream including the finishing pad bits, and S the total shift
// count. (Checked against the reference coder; tests/test_emit_model.py.)
// So a stream's tokens are cut into segments (k_emit_desc: every
// EMIT_SEG tokens of a compact stream, or of each of K3's token rows, where
// the tokens were written once; a segment never crosses a row) and:
//   (tokens are resolved to (bit, probability) under the frame's final
//   probabilities by each kernel below as it stages them in LDS)
//   E1 k_emit_img      per segment, the few ranges it can start with (the end
//                      states of the previous segment's last 256 tokens run
//                      from all 128 ranges; typically 4-10 survive)
//      k_emit_maps     per segment, the end range and shift count from each
//                      of those start ranges (the group's (segment, start)
//                      pairs packed densely onto the lanes)
//   E2 k_emit_compose  per frame, chain the segment maps: every segment's true
//                      start range and bit offset, pad bits, S and L
//   E3 k_emit_seg      per segment (one lane each): one forward pass with the
//                      true start range places every c_i at bit E_i of N, most
//                      significant first (a 64-bit window sliding down a word
//                      at a time); its low S_s bits tile N exactly (plain
//                      stores inside, atomicOr on the two shared boundary
//                      words), the <= 8 bits above go to H_s
//   E4 k_emit_carry    adds every H_s at its segment's top with atomicAdd and
//                      ripple carry (additions commute, so order is free)
//   E5 k_emit_bytes    output byte k = bits [1 + 8(L-1-k), +8) of N, written
//                      over the frame's (consumed) token buffer
#include <stdlib.h>

#include "vp8_dev.h"

#define EMIT_SEG VP8G_EMIT_SEG   // tokens per segment

namespace {

__device__ __forceinline__ int renorm(int& r) {   // range_ in [0, 254] -> [127, 254]
  const int sh = __builtin_clz((unsigned)r + 1u) - 24;   // r + 1 > 0: no clz(0) clamp
  r = ((r + 1) << sh) - 1;
  return sh;
}

}  // namespace

// One range-chain step: returns the renormalisation shift.
__device__ __forceinline__ int chain_step(int& r, uint32_t pb) {
  const int split = (int)(__umul24((unsigned)r, pb & 0xff) >> 8);   // full-rate 24-bit multiply
  r = (pb >> 8) ? r - split - 1 : split;
  return renorm(r);
}

// A recorded token (bit << 15 | fixed << 14 | probability or slot) as
// (bit << 8 | probability) under the frame's final probabilities (prob in
// LDS): the consumers resolve tokens as they stage them.
__device__ __forceinline__ uint32_t resolve_tok(uint32_t t, const uint8_t* prob) {
  const uint32_t p = (t & 0x4000) ? (t & 0xff) : prob[t & 0x3fff & 2047];
  return ((t >> 15) << 8) | p;
}
__device__ __forceinline__ uint32_t resolve_pair(uint32_t w, const uint8_t* prob) {
  return resolve_tok(w & 0xffff, prob) | (resolve_tok(w >> 16, prob) << 16);
}
__device__ __forceinline__ uint4 resolve_quad(uint4 q, const uint8_t* prob) {
  return make_uint4(resolve_pair(q.x, prob), resolve_pair(q.y, prob), resolve_pair(q.z, prob),
                    resolve_pair(q.w, prob));
}
__device__ __forceinline__ void load_probas(uint8_t* prob, const vp8g_frame_result* results,
                                            const vp8g_emit_meta& M, int t, int nt) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(results[M.frame].probas);
  for (int k = t; k < VP8G_NUM_SLOTS / 4; k += nt) reinterpret_cast<uint32_t*>(prob)[k] = src[k];
}

// E1a: the range a segment can start with is the end state of the previous
// segment, whatever state that one was in EMIT_IMG tokens before its end:
// push the set of all 128 ranges through those last tokens and keep the end
// set (a handful: the chains merge quickly). Only the set matters, so it is
// carried as distinct values: a wavefront takes IMG_G segments, runs the
// (segment, range) pairs of the current sets packed onto its lanes for one
// phase of tokens, collects the images in per-segment 128-bit maps and
// repacks the (by then far fewer) distinct ranges for the next phase.
// Segment 0 starts at 254.
#ifndef EMIT_IMG   // (overridable for the K4 A/B builds, tools/emit_ab.sh)
#define EMIT_IMG 256
#endif
#define EMIT_SLOTS 16
#define IMG_G 16                     // segments per wavefront (4 lanes each for the maps)
#define IMG_ROW (EMIT_IMG + 8)       // u16; +16 B per row: conflict-free b128 reads
__global__ __launch_bounds__(64) void k_emit_img(const uint16_t* __restrict__ tokens,
                                                 size_t tok_cap,
                                                 const vp8g_frame_result* __restrict__ results,
                                                 const vp8g_emit_meta* __restrict__ meta,
                                                 const vp8g_emit_desc* __restrict__ desc,
                                                 uint8_t* __restrict__ img) {
  __shared__ __align__(16) uint16_t tk[IMG_G * IMG_ROW];
  __shared__ __align__(4) uint8_t prob[VP8G_NUM_SLOTS];
  __shared__ uint32_t bm[IMG_G * 4];
  __shared__ uint16_t pairs[IMG_G * 128];   // (segment << 7) | (range - 127)
  const int f = blockIdx.y, lane = threadIdx.x;
  const vp8g_emit_meta M = meta[f];
  const uint32_t sbase = blockIdx.x * IMG_G;
  if (sbase >= M.nseg) return;   // whole wave
  const vp8g_emit_desc* D = desc + M.seg_base;
  load_probas(prob, results, M, lane, 64);
  __syncthreads();
#pragma unroll
  for (int t = 0; t < IMG_G * EMIT_IMG / 8 / 64; ++t) {   // every segment's last-tokens window
    const int q = lane + 64 * t, sg = q / (EMIT_IMG / 8), part = q % (EMIT_IMG / 8);
    const uint32_t s = sbase + sg;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (s > 0 && s < M.nseg) {
      // the EMIT_IMG tokens before the segment in stream order: the previous
      // segment's last ones -- token by token when it is a row's last segment
      // (its end is off the 8-token grid) -- reaching back into the segment
      // before it when that one is shorter (a row's short last segment)
      const vp8g_emit_desc d1 = D[s - 1];
      if (d1.len >= EMIT_IMG) {
        const uint64_t b = d1.off + d1.len - EMIT_IMG + 8 * part;
        uint4 raw;
        if ((b & 7) == 0) {
          raw = *reinterpret_cast<const uint4*>(tokens + b);
        } else {
          const uint16_t* pt = tokens + b;
          raw = make_uint4(pt[0] | ((uint32_t)pt[1] << 16), pt[2] | ((uint32_t)pt[3] << 16),
                           pt[4] | ((uint32_t)pt[5] << 16), pt[6] | ((uint32_t)pt[7] << 16));
        }
        v = resolve_quad(raw, prob);
      } else if (s >= 2) {
        const vp8g_emit_desc d2 = D[s - 2];
        if (d1.len + d2.len >= EMIT_IMG) {
          uint32_t w[4];
#pragma unroll
          for (int k = 0; k < 8; k += 2) {
            uint32_t pr[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint32_t back = EMIT_IMG - (8 * part + k + h);   // 1..256 before the start
              pr[h] = back <= d1.len ? tokens[d1.off + d1.len - back]
                                     : tokens[d2.off + d2.len - (back - d1.len)];
            }
            w[k >> 1] = pr[0] | (pr[1] << 16);
          }
          v = resolve_quad(make_uint4(w[0], w[1], w[2], w[3]), prob);
        }
      }
    }
    *reinterpret_cast<uint4*>(&tk[sg * IMG_ROW + 8 * part]) = v;
  }
  // this lane's piece of the maps: segment mg, word mw
  const int mg = lane >> 2, mw = lane & 3;
  const uint32_t ms = sbase + mg;
  const bool mact = ms > 0 && ms < M.nseg;
  int np = IMG_G * 128;   // phase 0: pair p = (segment p >> 7, range 127 + (p & 127))
  int cnt = 0, wofs = 0;
  for (int ph = 0, t0 = 0; t0 < EMIT_IMG; ++ph) {
    const int t1 = ph == 0 ? 8 : 2 * t0;   // phases [0,8) [8,16) [16,32) ... [128,256)
    bm[lane] = 0;
    __syncthreads();   // tokens / pairs / cleared maps visible
    for (int p0 = 0; p0 < np; p0 += 64) {
      const int p = p0 + lane;
      if (p < np) {
        const int pr = ph == 0 ? p : pairs[p];
        const int g = pr >> 7;
        const uint32_t s = sbase + g;
        if (s > 0 && s < M.nseg) {
          int r = 127 + (pr & 127);
          const uint16_t* row = tk + g * IMG_ROW;
          for (int i = t0; i < t1; i += 8) {
            const uint4 q = *reinterpret_cast<const uint4*>(row + i);
            const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int k = 0; k < 8; ++k) chain_step(r, (w[k >> 1] >> (16 * (k & 1))) & 0xffff);
          }
          atomicOr(&bm[g * 4 + ((r - 127) >> 5)], 1u << ((r - 127) & 31));
        }
      }
    }
    __syncthreads();   // the maps are complete
    // repack: this lane's map word -> pairs[offset of its segment + earlier words]
    const uint32_t word = bm[lane];
    const int pc = __popc(word);
    int incl = pc;   // inclusive scan over all 64 words = segment-major order
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    np = __shfl(incl, 63);
    const int gfirst = __shfl(incl - pc, lane & ~3);   // the segment's first pair
    cnt = __shfl(incl, lane | 3) - gfirst;
    wofs = incl - pc - gfirst;
    t0 = t1;
    if (t0 < EMIT_IMG) {
      int k = incl - pc;
      for (uint32_t m = word; m; m &= m - 1)
        pairs[k++] = (uint16_t)((mg << 7) | (32 * mw + __ffs(m) - 1));
    }
  }
  // output: the end set of each segment (lanes of segment mg, word mw)
  if (ms >= M.nseg) return;
  uint8_t* out = img + ((size_t)M.seg_base + ms) * (EMIT_SLOTS + 1);
  if (!mact) {   // segment 0
    if (mw == 0) { out[0] = 1; out[1] = 254; }
    return;
  }
  if (D[ms - 1].len < EMIT_IMG && (ms < 2 || D[ms - 1].len + D[ms - 2].len < EMIT_IMG)) {
    if (mw == 0) out[0] = 0xff;   // fewer than EMIT_IMG tokens to look back on: all 128 ranges
    return;
  }
  if (cnt > EMIT_SLOTS) {   // too many: the map kernel covers all 128 ranges
    if (mw == 0) out[0] = 0xff;
    return;
  }
  if (mw == 0) out[0] = (uint8_t)cnt;
  int k = 1 + wofs;
  for (uint32_t m = bm[lane]; m; m &= m - 1) out[k++] = (uint8_t)(127 + 32 * mw + __ffs(m) - 1);
}

// E1b: per segment, the end range and shift count from each possible start
// range. A wavefront takes MAP_G consecutive segments and packs their
// (segment, start range) pairs densely onto its 64 lanes (a segment has ~4
// start ranges, so a fixed 16 lanes per segment would leave most lanes idle);
// more than 64 pairs take further rounds. The group's tokens go through LDS
// MAP_CH per segment at a time (the next chunk is loaded into registers while
// this one runs), so the chains read LDS broadcasts instead of global loads.
#ifndef MAP_G
#define MAP_G 8
#endif
#define MAP_CH 256
#define MAP_ROW (MAP_CH + 8)   // u16; +16 B per row: the 16 rows' b128 reads hit distinct banks
#define MAP_PIECES (MAP_G * MAP_CH / 8 / 64)   // 16-byte pieces per lane per chunk
__global__ __launch_bounds__(64) void k_emit_maps(const uint16_t* __restrict__ tokens,
                                                  size_t tok_cap,
                                                  const vp8g_frame_result* __restrict__ results,
                                                  const vp8g_emit_meta* __restrict__ meta,
                                                  const vp8g_emit_desc* __restrict__ desc,
                                                  const uint8_t* __restrict__ img,
                                                  uint8_t* __restrict__ emap,
                                                  uint16_t* __restrict__ eshift) {
  __shared__ __align__(16) uint16_t stage[MAP_G * MAP_ROW];
  __shared__ __align__(4) uint8_t prob[VP8G_NUM_SLOTS];
  __shared__ vp8g_emit_desc ld[MAP_G];
  const int f = blockIdx.y, lane = threadIdx.x;
  const vp8g_emit_meta M = meta[f];
  const uint32_t sbase = blockIdx.x * MAP_G;
  if (sbase >= M.nseg) return;   // whole wave
  // pair counts of the group's segments (lanes 0..MAP_G-1), inclusive scan
  int nk = 0;
  if (lane < MAP_G && sbase + lane < M.nseg) {
    const int ni = img[((size_t)M.seg_base + sbase + lane) * (EMIT_SLOTS + 1)];
    nk = ni == 0xff ? 128 : ni;
  }
  int incl = nk;
  for (int o = 1; o < MAP_G; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  const int total = __shfl(incl, MAP_G - 1);
  if (lane < MAP_G && sbase + lane < M.nseg) ld[lane] = desc[M.seg_base + sbase + lane];
  load_probas(prob, results, M, lane, 64);
  __syncthreads();
  uint64_t pofs[MAP_PIECES];   // the descriptor of each of the lane's pieces, in registers
  uint32_t plen[MAP_PIECES];
#pragma unroll
  for (int t = 0; t < MAP_PIECES; ++t) {
    const int sg = (lane + 64 * t) / (MAP_CH / 8);
    const bool in = sbase + sg < M.nseg;
    pofs[t] = in ? ld[sg].off : 0;
    plen[t] = in ? ld[sg].len : 0u;
  }
  auto load = [&](uint32_t c0, uint4* v) {
#pragma unroll
    for (int t = 0; t < MAP_PIECES; ++t) {
      const int part = (lane + 64 * t) % (MAP_CH / 8);
      const uint32_t i = c0 + 8 * part;
      v[t] = make_uint4(0, 0, 0, 0);
      if (i < plen[t]) v[t] = *reinterpret_cast<const uint4*>(tokens + pofs[t] + i);
    }
  };
  for (int p0 = 0; p0 < total; p0 += 64) {
    const int p = p0 + lane;   // this lane's pair
    int g = 0, excl = 0;
#pragma unroll
    for (int j = 0; j < MAP_G; ++j) {
      const int ij = __shfl(incl, j);
      if (p >= ij) { g = j + 1; excl = ij; }
    }
    const bool live = p < total;
    const uint32_t s = sbase + (live ? g : 0);
    const uint8_t* im = img + ((size_t)M.seg_base + s) * (EMIT_SLOTS + 1);
    const int k = p - excl;
    const int r0 = !live ? 127 : im[0] == 0xff ? 127 + k : im[1 + k];
    const uint32_t cnt = live ? ld[g].len : 0u;
    const uint16_t* st = stage + (live ? g : 0) * MAP_ROW;
    int r = r0;
    uint32_t S = 0;
    uint4 nv[MAP_PIECES];
    load(0, nv);
    for (uint32_t c0 = 0; c0 < EMIT_SEG; c0 += MAP_CH) {
      __syncthreads();   // the previous chunk's reads are done
#pragma unroll
      for (int t = 0; t < MAP_PIECES; ++t) {
        const int q = lane + 64 * t, sg = q / (MAP_CH / 8), part = q % (MAP_CH / 8);
        *reinterpret_cast<uint4*>(&stage[sg * MAP_ROW + 8 * part]) = resolve_quad(nv[t], prob);
      }
      __syncthreads();
      if (c0 + MAP_CH < EMIT_SEG) load(c0 + MAP_CH, nv);   // in flight during the chain
      const uint32_t n = cnt > c0 ? min((uint32_t)MAP_CH, cnt - c0) : 0u;
      if (n == MAP_CH) {
        for (int i = 0; i < MAP_CH; i += 8) {
          const uint4 q = *reinterpret_cast<const uint4*>(st + i);
          const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) S += chain_step(r, (w[kk >> 1] >> (16 * (kk & 1))) & 0xffff);
        }
      } else {
        for (uint32_t i = 0; i < n; ++i) S += chain_step(r, st[i]);   // a row's / stream's last segment
      }
    }
    if (live) {
      const size_t o = ((size_t)M.seg_base + s) * 128 + (r0 - 127);
      emap[o] = (uint8_t)r;
      eshift[o] = (uint16_t)S;
    }
  }
}

// E2: one wavefront per frame. The segment maps are staged through LDS 64
// segments at a time (coalesced 16-byte loads of the whole 128-entry maps),
// so the serial walk along the true range chain reads LDS, not dependent
// global loads; the walk's per-segment (rs, S, T) go out coalesced.
#define CMP_SEGS 64
#define CMP_T 256   // threads: a chunk's maps load as 2 + 4 16-byte pieces per thread
__global__ __launch_bounds__(CMP_T) void k_emit_compose(vp8g_emit_meta* __restrict__ meta,
                                                        const uint8_t* __restrict__ emap,
                                                        const uint16_t* __restrict__ eshift,
                                                        vp8g_emit_seg* __restrict__ segs,
                                                        uint32_t* __restrict__ out_size) {
  // two chunk buffers: the next chunk's maps load while lane 0 walks this one
  // (a serial load -> store per piece cost one memory latency each: 456 us
  // for one 1080p frame's ~650 segments)
  __shared__ __align__(16) uint8_t lmap[2][CMP_SEGS * 128];
  __shared__ __align__(16) uint16_t lsh[2][CMP_SEGS * 128];
  __shared__ vp8g_emit_seg lseg[CMP_SEGS];
  __shared__ uint32_t lS;
  const int f = blockIdx.x, t = threadIdx.x;
  vp8g_emit_meta M = meta[f];
  int r = 254;        // thread 0's walk state
  uint32_t cum = 0;
  uint4 pm[2], ps[4];
  auto fetch = [&](uint32_t c) {   // chunk c's maps into registers (all issued at once)
    const uint32_t m = min((uint32_t)CMP_SEGS, M.nseg - c);
    const uint4* gm = reinterpret_cast<const uint4*>(emap + ((size_t)M.seg_base + c) * 128);
    const uint4* gs = reinterpret_cast<const uint4*>(eshift + ((size_t)M.seg_base + c) * 128);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t q = t + CMP_T * k;
      pm[k] = q < m * 8 ? gm[q] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t q = t + CMP_T * k;
      ps[k] = q < m * 16 ? gs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  auto stage = [&](int b) {
#pragma unroll
    for (int k = 0; k < 2; ++k) reinterpret_cast<uint4*>(lmap[b])[t + CMP_T * k] = pm[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) reinterpret_cast<uint4*>(lsh[b])[t + CMP_T * k] = ps[k];
  };
  if (M.nseg) fetch(0);
  for (uint32_t c = 0, b = 0; c < M.nseg; c += CMP_SEGS, b ^= 1) {
    const uint32_t m = min((uint32_t)CMP_SEGS, M.nseg - c);
    stage(b);
    __syncthreads();   // chunk c staged; the previous chunk's lseg written out
    if (c + CMP_SEGS < M.nseg) fetch(c + CMP_SEGS);   // in flight during the walk
    if (t == 0) {
      for (uint32_t j = 0; j < m; ++j) {
        const uint32_t o = j * 128 + (r - 127);
        const uint32_t Ss = lsh[b][o];
        lseg[j] = vp8g_emit_seg{cum, (uint16_t)Ss, (uint8_t)r, 0};   // T: shifts BEFORE the segment
        cum += Ss;
        r = lmap[b][o];
      }
    }
    __syncthreads();
    if ((uint32_t)t < m) segs[M.seg_base + c + t] = lseg[t];
  }
  if (t == 0) {
    // VP8BitWriterFinish pads 9 - nb_bits zero bits at probability 1/2, where
    // nb_bits is what the flushes left after cum shifts from -8
    const int tt = (int)cum - 8;
    const int nb = tt <= 0 ? tt : tt - 8 * ((tt + 7) / 8);
    uint32_t spad = 0;
    for (int k = 0; k < 9 - nb; ++k) {
      r = (r * 128) >> 8;
      spad += renorm(r);
    }
    M.S = cum + spad;
    M.L = (M.S + 7) / 8;
    meta[f] = M;
    out_size[f] = M.L;
    lS = M.S;
  }
  __syncthreads();
  const uint32_t St = lS;
  for (uint32_t s = t; s < M.nseg; s += CMP_T) {   // T_s = bit offset of the segment's bottom in N
    vp8g_emit_seg& g = segs[M.seg_base + s];
    g.T = St - (g.T + g.S);
  }
}

// One wave = 64 segments, one lane each. The segments' tokens are staged
// through LDS 64 tokens at a time: the wave loads a chunk of all 64 segments
// with 128-byte runs per segment (a lane-per-segment walk would touch 64
// lines 4 KB apart per load), each lane then walks its own row.
#define SEG_CH 64                   // tokens per segment per chunk
#define SEG_ROW (SEG_CH / 2 + 1)    // LDS row in dwords, +1: conflict-free rows

// a chunk of 64 segments x SEG_CH tokens in two steps: global -> registers (issued early, so the
// loads fly while the previous chunk is processed), registers -> LDS
// (pofs / plen: the segment descriptor of each of the lane's 8 pieces, held
// in registers for the whole kernel: the fetch is address arithmetic only)
__device__ __forceinline__ void seg_chunk_fetch(uint4 v[8], const uint16_t* tokens,
                                                const uint64_t pofs[8], const uint32_t plen[8],
                                                uint32_t c0, int lane) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const uint32_t i = c0 + 8 * (lane & 7);
    v[t] = make_uint4(0, 0, 0, 0);
    if (i < plen[t]) v[t] = *reinterpret_cast<const uint4*>(tokens + pofs[t] + i);
  }
}
__device__ __forceinline__ void seg_chunk_put(uint32_t* lds, const uint4 v[8], int lane) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int q = lane + 64 * t, sg = q >> 3, part = q & 7;
    uint32_t* d = lds + sg * SEG_ROW + 4 * part;
    d[0] = v[t].x; d[1] = v[t].y; d[2] = v[t].z; d[3] = v[t].w;
  }
}

// The segment's bits of N, most significant first. Token i's c_i lands at
// bit E_i = top - P_i (P_i: the segment's shifts before token i), so with the
// true start range one forward pass places every c: the lane keeps the bits
// [B, B + 64) of the sum in a 64-bit window with p - B in [0, 39] (p the bit
// the next c lands on). Once p - B <= 7 every later c lies below B + 15, so
// the window's upper word can only change by a carry out of the lower one: it
// is staged (LDS, one column per lane) and the window slides down 32 bits.
// A carry out of the window needs the >= 17 bits between the current byte and
// the window top all ones (the coder's carries themselves are frequent: with
// no headroom above p + 8 this kernel ran 60x slower); it ripples into the
// words already written. Bits at or above top go to H_s, the word that
// straddles top is kept in a register until the end (the segment above ORs its
// low bits into the same word), the word that straddles T is ORed.
struct seg_sink {
  uint32_t* W;
  int T, top;
  uint32_t topw, H;
};
__device__ __forceinline__ void seg_put(seg_sink& o, int wp, uint32_t v) {
  if (!v) return;   // the words start zeroed
  if (wp + 32 <= o.top) {
    if (wp >= o.T) o.W[wp >> 5] = v;
    else atomicOr(o.W + (wp >> 5), v);   // the bottom word, shared with the segment below
  } else if (wp < o.top) {
    const int k = o.top - wp;
    o.topw += v & ((1u << k) - 1u);
    o.H += v >> k;
  } else if (wp - o.top < 32) {
    o.H += v << (wp - o.top);
  }
}
__device__ __noinline__ void seg_carry(seg_sink& o, int q) {   // +1 at bit q (> T)
  __threadfence();   // the words this lane stored before
  for (;;) {
    const int wp = q & ~31;
    if (q >= o.top) { o.H += 1u << (q - o.top); return; }
    if (wp + 32 > o.top) {
      const int k = o.top - wp;
      o.topw += 1u << (q - wp);
      if (o.topw >> k) { o.topw -= 1u << k; o.H += 1; }
      return;
    }
    const uint32_t add = 1u << (q & 31);
    const uint32_t old = atomicAdd(o.W + (wp >> 5), add);
    if (old + add >= old) return;
    q = wp + 32;
  }
}
#define SEG_STG 16   // staged words per lane: a chunk shifts at most 7 * SEG_CH bits
__device__ __forceinline__ void seg_unstage(seg_sink& o, const uint32_t* stg, int& nst, int B,
                                            int lane) {
  // staged word i sits at B + 64 + 32 (nst - 1 - i)
  for (int i = 0; i < nst; ++i) seg_put(o, B + 64 + 32 * (nst - 1 - i), stg[i * 64 + lane]);
  nst = 0;
}

__global__ __launch_bounds__(64) void k_emit_seg(const uint16_t* __restrict__ tokens, size_t tok_cap,
                                                 const vp8g_frame_result* __restrict__ results,
                                                 const vp8g_emit_meta* __restrict__ meta,
                                                 const vp8g_emit_desc* __restrict__ desc,
                                                 vp8g_emit_seg* __restrict__ segs,
                                                 uint32_t* __restrict__ nbuf) {
  __shared__ uint32_t lds[64 * SEG_ROW];
  __shared__ vp8g_emit_desc ld[64];
  __shared__ uint32_t stg[SEG_STG * 64];
  __shared__ __align__(4) uint8_t prob[VP8G_NUM_SLOTS];
  const int f = blockIdx.y, lane = threadIdx.x;
  const uint32_t s0 = blockIdx.x * 64, s = s0 + lane;
  const vp8g_emit_meta M = meta[f];
  if (s0 >= M.nseg) return;   // whole wave
  const bool valid = s < M.nseg;
  const vp8g_emit_seg g = valid ? segs[M.seg_base + s] : vp8g_emit_seg{0, 0, 254, 0};
  const vp8g_emit_desc dd = valid ? desc[M.seg_base + s] : vp8g_emit_desc{0, 0, 0};
  ld[lane] = dd;
  const uint32_t cnt = dd.len;
  const uint32_t* row = lds + lane * SEG_ROW;
  // the chunks this wave needs: up to its longest segment
  uint32_t span = cnt;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) span = max(span, (uint32_t)__shfl_xor((int)span, o));
  seg_sink o{nbuf + M.nb_base, (int)g.T, (int)(g.T + g.S), 0u, 0u};
  int p = o.top;                 // the bit the next c lands on
  int B = (o.top - 7) & ~31;     // window [B, B + 64); top - B in [7, 38]
  uint64_t acc = 0;
  int nst = 0;
  load_probas(prob, results, M, lane, 64);
  int r = g.rs;
  uint4 nv[8];
  __syncthreads();   // the wave's descriptors in LDS
  uint64_t pofs[8];
  uint32_t plen[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {   // piece t of this lane: segment (lane + 64 t) >> 3, part lane & 7
    const int sg = (lane + 64 * t) >> 3;
    const bool in = s0 + sg < M.nseg;
    pofs[t] = in ? ld[sg].off : 0;
    plen[t] = in ? ld[sg].len : 0u;
  }
  seg_chunk_fetch(nv, tokens, pofs, plen, 0, lane);
  for (uint32_t c0 = 0; c0 < span; c0 += SEG_CH) {
    seg_chunk_put(lds, nv, lane);
    __syncthreads();
    if (c0 + SEG_CH < span) seg_chunk_fetch(nv, tokens, pofs, plen, c0 + SEG_CH, lane);
#pragma unroll 2
    for (int k = 0; k < SEG_CH / 2; ++k) {
      const uint32_t w = resolve_pair(row[k], prob);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t pb = (w >> (16 * h)) & 0xffff;
        const int split = (int)(__umul24((unsigned)r, pb & 0xff) >> 8);   // full-rate 24-bit multiply
        const int bit = (pb >> 8) & 1;
        const uint32_t c = bit ? (uint32_t)split + 1u : 0u;
        int rr = bit ? r - split - 1 : split;
        const int sh = renorm(rr);
        if (c0 + 2 * k + h < cnt) {
          r = rr;
          const uint64_t na = acc + ((uint64_t)c << (p - B));   // p - B in [0, 39]
          if (na < acc) {   // carry out of the window
            seg_unstage(o, stg, nst, B, lane);
            seg_carry(o, B + 64);
          }
          acc = na;
          p -= sh;
          if (p - B <= 7) {   // the upper word is final but for carries
            stg[nst * 64 + lane] = (uint32_t)(acc >> 32);
            ++nst;
            acc <<= 32;
            B -= 32;
          }
        }
      }
    }
    if (nst) seg_unstage(o, stg, nst, B, lane);
    __syncthreads();
  }
  if (!valid) return;
  seg_put(o, B + 32, (uint32_t)(acc >> 32));
  seg_put(o, B, (uint32_t)acc);
  if ((o.top & 31) && o.topw) atomicOr(o.W + (o.top >> 5), o.topw);
  segs[M.seg_base + s].H = (uint8_t)o.H;
}

// big-number add of h at bit b (h < 256) with ripple carry, via atomics
__device__ __forceinline__ void big_add(uint32_t* W, uint32_t b, uint32_t h) {
  const uint64_t v = (uint64_t)h << (b & 31);
  uint32_t w = b >> 5;
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  uint32_t old = atomicAdd(W + w, lo);
  uint32_t carry = (old + lo) < old;
  ++w;
  uint32_t add = hi + carry;   // hi < 256, no overflow
  while (add) {
    old = atomicAdd(W + w, add);
    add = (old + add) < old;
    ++w;
  }
}

__global__ __launch_bounds__(64) void k_emit_carry(const vp8g_emit_meta* __restrict__ meta,
                                                   const vp8g_emit_seg* __restrict__ segs,
                                                   uint32_t* __restrict__ nbuf) {
  const int f = blockIdx.y;
  const uint32_t s = blockIdx.x * 64 + threadIdx.x;
  const vp8g_emit_meta M = meta[f];
  if (s >= M.nseg) return;
  const vp8g_emit_seg g = segs[M.seg_base + s];
  if (g.H) big_add(nbuf + M.nb_base, g.T + g.S, g.H);
}

__global__ __launch_bounds__(256) void k_emit_bytes(uint16_t* __restrict__ tokens, size_t tok_cap,
                                                    const vp8g_emit_meta* __restrict__ meta,
                                                    const uint32_t* __restrict__ nbuf) {
  const int f = blockIdx.y;
  const vp8g_emit_meta M = meta[f];
  const uint32_t k0 = 4 * (blockIdx.x * 256 + threadIdx.x);   // output bytes k0 .. k0 + 3
  if (k0 >= M.L) return;
  const uint32_t* W = nbuf + M.nb_base;
  uint8_t* out = reinterpret_cast<uint8_t*>(tokens + M.tok_off);
  if (k0 + 3 < M.L) {   // bits [b, b + 32) of N, byte k0 the most significant
    const uint32_t b = 1 + 8 * (M.L - 1 - (k0 + 3));
    const uint64_t two = (uint64_t)W[b >> 5] | ((uint64_t)W[(b >> 5) + 1] << 32);
    *reinterpret_cast<uint32_t*>(out + k0) = __builtin_bswap32((uint32_t)(two >> (b & 31)));
  } else {
    for (uint32_t k = k0; k < M.L; ++k) {
      const uint32_t b = 1 + 8 * (M.L - 1 - k);   // lowest bit of output byte k
      const uint64_t two = (uint64_t)W[b >> 5] | ((uint64_t)W[(b >> 5) + 1] << 32);
      out[k] = (uint8_t)(two >> (b & 31));
    }
  }
}

// E0: the segments. A compact stream is cut every EMIT_SEG tokens; a row
// stream (K3's token rows: the tokens stay where K3 wrote them) every
// EMIT_SEG tokens of each row, so a segment never crosses a row and every
// segment starts at a multiple of 8 tokens. One workgroup per stream; a row
// stream's exact segment count replaces the host's bound in its meta.
#define DESC_T 256
__global__ __launch_bounds__(DESC_T) void k_emit_desc(vp8g_emit_meta* __restrict__ meta,
                                                      const uint32_t* __restrict__ rowtok,
                                                      vp8g_emit_desc* __restrict__ desc) {
  const int st = blockIdx.x, t = threadIdx.x;
  const vp8g_emit_meta M = meta[st];
  vp8g_emit_desc* D = desc + M.seg_base;
  if (M.nrows == 0) {
    const uint32_t nseg = (M.ntok + EMIT_SEG - 1) / EMIT_SEG;
    for (uint32_t s = t; s < nseg; s += DESC_T)
      D[s] = vp8g_emit_desc{M.tok_off + (uint64_t)s * EMIT_SEG,
                            min((uint32_t)EMIT_SEG, M.ntok - s * EMIT_SEG), 0u};
    if (t == 0) meta[st].nseg = nseg;
    return;
  }
  const uint32_t* rt = rowtok + (size_t)M.frame * M.nrows;
  const uint32_t per = (M.nrows + DESC_T - 1) / DESC_T;
  const uint32_t r0 = min(t * per, M.nrows), r1 = min(r0 + per, M.nrows);
  uint32_t cnt = 0;
  for (uint32_t r = r0; r < r1; ++r) cnt += (rt[r] + EMIT_SEG - 1) / EMIT_SEG;
  __shared__ uint32_t wsum[DESC_T / 64];
  const int lane = t & 63, wv = t >> 6;
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t s = incl - cnt, total = 0;
#pragma unroll
  for (int k = 0; k < DESC_T / 64; ++k) {
    s += k < wv ? wsum[k] : 0u;
    total += wsum[k];
  }
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t n = rt[r];
    for (uint32_t k = 0; k < n; k += EMIT_SEG)
      D[s++] = vp8g_emit_desc{M.tok_off + (uint64_t)r * M.rowcap + k, min((uint32_t)EMIT_SEG, n - k),
                              0u};
  }
  if (t == 0) meta[st].nseg = total;
}

extern "C" int vp8g_launch_check(const char* what);

extern "C" int vp8g_launch_emit(uint16_t* tokens, size_t tok_cap, int n,
                                const vp8g_frame_result* results, vp8g_emit_meta* meta,
                                const uint32_t* rowtok, uint32_t max_ntok, uint32_t max_seg,
                                uint8_t* emap, uint16_t* eshift, uint8_t* img, vp8g_emit_desc* desc,
                                vp8g_emit_seg* segs, uint32_t* nbuf, uint32_t* out_size,
                                void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (n <= 0) return 1;
  (void)max_ntok;   // the token consumers resolve the probabilities themselves
  hipLaunchKernelGGL(k_emit_desc, dim3(n), dim3(DESC_T), 0, st, meta, rowtok, desc);
  if (!vp8g_launch_check("k_emit_desc")) return 0;
  if (max_seg) {
    hipLaunchKernelGGL(k_emit_img, dim3((max_seg + IMG_G - 1) / IMG_G, n), dim3(64), 0, st,
                       (const uint16_t*)tokens, tok_cap, results, (const vp8g_emit_meta*)meta,
                       (const vp8g_emit_desc*)desc, img);
    if (!vp8g_launch_check("k_emit_img")) return 0;
    hipLaunchKernelGGL(k_emit_maps, dim3((max_seg + MAP_G - 1) / MAP_G, n), dim3(64), 0, st,
                       (const uint16_t*)tokens, tok_cap, results, (const vp8g_emit_meta*)meta,
                       (const vp8g_emit_desc*)desc, (const uint8_t*)img, emap, eshift);
    if (!vp8g_launch_check("k_emit_maps")) return 0;
  }
  hipLaunchKernelGGL(k_emit_compose, dim3(n), dim3(CMP_T), 0, st, meta, (const uint8_t*)emap,
                     (const uint16_t*)eshift, segs, out_size);
  if (!vp8g_launch_check("k_emit_compose")) return 0;
  const uint32_t sb = (max_seg + 63) / 64;
  if (sb) {
    hipLaunchKernelGGL(k_emit_seg, dim3(sb, n), dim3(64), 0, st, tokens, tok_cap, results,
                       (const vp8g_emit_meta*)meta, (const vp8g_emit_desc*)desc, segs, nbuf);
    if (!vp8g_launch_check("k_emit_seg")) return 0;
    hipLaunchKernelGGL(k_emit_carry, dim3(sb, n), dim3(64), 0, st, (const vp8g_emit_meta*)meta,
                       (const vp8g_emit_seg*)segs, nbuf);
    if (!vp8g_launch_check("k_emit_carry")) return 0;
  }
  // output bytes: at most (7 * ntok + 40) / 8 + 1 per frame
  const uint32_t maxL = (7u * max_ntok + 48) / 8 + 2;
  hipLaunchKernelGGL(k_emit_bytes, dim3((maxL + 1023) / 1024, n), dim3(256), 0, st, tokens, tok_cap,
                     (const vp8g_emit_meta*)meta, (const uint32_t*)nbuf);
  return vp8g_launch_check("k_emit_bytes");
}

// K4 on caller-given token streams (fixed-probability tokens: bit << 15 |
// 1 << 14 | probability), for tests that drive the coder with streams the
// encoder rarely makes (long all-ones runs: the carry paths). Streams are
// concatenated in host_tokens; stream s's bytes go to host_out + s * out_stride,
// its size to out_size[s]. Returns 0 on any HIP error or a too small stride.
// rowlen > 0: each stream is laid out as K3's token rows are -- rows of
// rowlen tokens (the last one shorter) rowcap = round8(rowlen) + 8 apart --
// and coded as a row stream (vp8g_emit_rows)
static int emit_streams(const uint16_t* host_tokens, const uint32_t* ntok, int n, uint32_t rowlen,
                        uint8_t* host_out, uint32_t out_stride, uint32_t* out_size) {
  if (n <= 0) return 1;
  vp8g_emit_meta* meta = (vp8g_emit_meta*)calloc((size_t)n, sizeof(vp8g_emit_meta));
  if (!meta) return 0;
  const uint32_t rowcap = rowlen ? ((rowlen + 7) & ~7u) + 8 : 0;
  size_t off = 0, segs = 0, words = 0, src = 0;
  uint32_t max_ntok = 0, max_seg = 0, nrt = 0;   // nrt: rows of every row stream (the rest empty)
  for (int s = 0; s < n && rowlen; ++s) nrt = max(nrt, (ntok[s] + rowlen - 1) / rowlen);
  for (int s = 0; s < n; ++s) {
    vp8g_emit_meta& m = meta[s];
    m.ntok = ntok[s];
    m.frame = (uint32_t)s;
    m.tok_off = off;
    m.nrows = rowlen ? nrt : 0;
    m.rowcap = rowcap;
    m.nseg = (m.ntok + EMIT_SEG - 1) / EMIT_SEG + m.nrows;
    m.seg_base = (uint32_t)segs;
    m.nb_base = (uint32_t)words;
    segs += m.nseg;
    words += (7 * (size_t)m.ntok + 17 + 8 + 63) / 32 + 4;
    const size_t room = rowlen ? (size_t)m.nrows * rowcap : (size_t)m.ntok;
    off += (room + 64 + 7) & ~(size_t)7;   // room for the bytes of a short stream
    max_ntok = m.ntok > max_ntok ? m.ntok : max_ntok;
    max_seg = m.nseg > max_seg ? m.nseg : max_seg;
    if ((7ull * m.ntok + 48) / 8 + 2 > out_stride) { free(meta); return 0; }
  }
  uint16_t* d_tok = nullptr; vp8g_frame_result* d_res = nullptr; vp8g_emit_meta* d_meta = nullptr;
  uint8_t *d_emap = nullptr, *d_img = nullptr; uint16_t* d_eshift = nullptr;
  vp8g_emit_seg* d_segs = nullptr; uint32_t *d_nbuf = nullptr, *d_size = nullptr, *d_rt = nullptr;
  vp8g_emit_desc* d_desc = nullptr;
  const size_t cs = segs + 1;
  bool ok = hipMalloc((void**)&d_tok, off * 2) == hipSuccess &&
            hipMalloc((void**)&d_res, (size_t)n * sizeof(vp8g_frame_result)) == hipSuccess &&
            hipMalloc((void**)&d_meta, (size_t)n * sizeof(vp8g_emit_meta)) == hipSuccess &&
            hipMalloc((void**)&d_emap, cs * 128) == hipSuccess &&
            hipMalloc((void**)&d_eshift, cs * 128 * sizeof(uint16_t)) == hipSuccess &&
            hipMalloc((void**)&d_img, cs * 17) == hipSuccess &&
            hipMalloc((void**)&d_desc, cs * sizeof(vp8g_emit_desc)) == hipSuccess &&
            hipMalloc((void**)&d_segs, cs * sizeof(vp8g_emit_seg)) == hipSuccess &&
            hipMalloc((void**)&d_nbuf, (words + 1) * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc((void**)&d_rt, ((size_t)n * nrt + 1) * sizeof(uint32_t)) == hipSuccess &&
            hipMalloc((void**)&d_size, (size_t)n * sizeof(uint32_t)) == hipSuccess;
  ok = ok && hipMemset(d_res, 0, (size_t)n * sizeof(vp8g_frame_result)) == hipSuccess &&
       hipMemset(d_nbuf, 0, (words + 1) * sizeof(uint32_t)) == hipSuccess &&
       hipMemset(d_rt, 0, ((size_t)n * nrt + 1) * sizeof(uint32_t)) == hipSuccess &&
       hipMemset(d_tok, 0, off * 2) == hipSuccess;
  for (int s = 0; ok && s < n; ++s) {
    if (!rowlen) {
      if (meta[s].ntok)
        ok = hipMemcpy(d_tok + meta[s].tok_off, host_tokens + src, meta[s].ntok * 2,
                       hipMemcpyHostToDevice) == hipSuccess;
    } else {   // row r of stream s: tokens [r * rowlen, ...) at tok_off + r * rowcap
      for (uint32_t r = 0; ok && r * rowlen < meta[s].ntok; ++r) {
        const uint32_t len = min(rowlen, meta[s].ntok - r * rowlen);
        ok = hipMemcpy(d_tok + meta[s].tok_off + (size_t)r * rowcap, host_tokens + src + (size_t)r * rowlen,
                       len * 2, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(d_rt + (size_t)s * meta[s].nrows + r, &len, 4, hipMemcpyHostToDevice) == hipSuccess;
      }
    }
    src += meta[s].ntok;
  }
  ok = ok && hipMemcpy(d_meta, meta, (size_t)n * sizeof(vp8g_emit_meta), hipMemcpyHostToDevice) == hipSuccess;
  ok = ok && vp8g_launch_emit(d_tok, off, n, d_res, d_meta, d_rt, max_ntok, max_seg, d_emap,
                              d_eshift, d_img, d_desc, d_segs, d_nbuf, d_size, 0);
  ok = ok && hipDeviceSynchronize() == hipSuccess &&
       hipMemcpy(out_size, d_size, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess;
  for (int s = 0; ok && s < n; ++s) {
    if (out_size[s] > out_stride) { ok = false; break; }
    if (out_size[s])
      ok = hipMemcpy(host_out + (size_t)s * out_stride, d_tok + meta[s].tok_off, out_size[s],
                     hipMemcpyDeviceToHost) == hipSuccess;
  }
  void* bufs[] = {d_tok, d_res, d_meta, d_emap, d_eshift, d_img, d_desc, d_segs, d_nbuf, d_rt, d_size};
  for (void* b : bufs) (void)hipFree(b);
  free(meta);
  return ok ? 1 : 0;
}

extern "C" __attribute__((visibility("default"))) int vp8g_emit_streams(
    const uint16_t* host_tokens, const uint32_t* ntok, int n, uint8_t* host_out,
    uint32_t out_stride, uint32_t* out_size) {
  return emit_streams(host_tokens, ntok, n, 0, host_out, out_stride, out_size);
}

// the same streams laid out and coded as K3's token rows of rowlen tokens
extern "C" __attribute__((visibility("default"))) int vp8g_emit_rows(
    const uint16_t* host_tokens, const uint32_t* ntok, int n, uint32_t rowlen, uint8_t* host_out,
    uint32_t out_stride, uint32_t* out_size) {
  if (rowlen == 0) return 0;
  return emit_streams(host_tokens, ntok, n, rowlen, host_out, out_stride, out_size);
}

// Gather every stream's bytes (at its token offset) into one packed buffer at
// 16-byte aligned offsets, so the host pulls the whole batch back with a
// single DMA instead of one copy per stream.
__global__ __launch_bounds__(256) void k_pack(const uint16_t* __restrict__ tokens,
                                              const vp8g_emit_meta* __restrict__ meta,
                                              const uint64_t* __restrict__ off,
                                              const uint32_t* __restrict__ size,
                                              uint8_t* __restrict__ dst) {
  const int f = blockIdx.y;
  const uint32_t n16 = (size[f] + 15) >> 4;
  const uint4* s4 = reinterpret_cast<const uint4*>(tokens + meta[f].tok_off);
  uint4* d4 = reinterpret_cast<uint4*>(dst + off[f]);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n16; i += gridDim.x * 256) d4[i] = s4[i];
}

extern "C" int vp8g_launch_pack(const uint16_t* tokens, const vp8g_emit_meta* meta, int n,
                                const uint64_t* off, const uint32_t* size, uint32_t max_size,
                                uint8_t* dst, void* stream) {
  if (n <= 0 || max_size == 0) return 1;
  uint32_t gx = (max_size + 16 * 256 - 1) / (16 * 256);
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(k_pack, dim3(gx, n), dim3(256), 0, (hipStream_t)stream, tokens, meta, off,
                     size, dst);
  return vp8g_launch_check("k_pack");
}

// Token partitions (VP8EncLoop writes MB row y into parts_[y & (P - 1)],
// iterator_enc.c:48): one workgroup per frame. Row token counts from the
// per-MB counts, raster row starts in the compact stream, then each
// partition's rows are copied, in order, to its own region in the upper half
// of the frame's slab (disjoint from the compact stream in the lower half).
// Each region holds at least the partition's coded bytes, so K4's output at a
// region's head never reaches the next one.
#define PART_MAX_ROWS 1024   // mbh <= 1024 (height <= 16383)
__device__ __forceinline__ uint32_t part_region(uint32_t ntok) {
  const uint32_t bytes = (7u * ntok + 48) / 8 + 2;   // K4's output bound
  const uint32_t need = max(ntok, (bytes + 1) / 2);
  return (need + 7u) & ~7u;
}

__global__ __launch_bounds__(256) void k_partition(uint16_t* __restrict__ tokens, size_t tok_cap,
                                                   const uint32_t* __restrict__ mboff,
                                                   const vp8g_frame_result* __restrict__ results,
                                                   const uint8_t* __restrict__ mbinfo, int mbw,
                                                   int mbh, int kind, int nparts,
                                                   uint32_t* __restrict__ part) {
  __shared__ uint32_t rowlen[PART_MAX_ROWS], rowsrc[PART_MAX_ROWS], rowdst[PART_MAX_ROWS];
  __shared__ uint32_t poff[VP8G_MAX_PARTS], plen[VP8G_MAX_PARTS];
  __shared__ uint32_t lastfix;
  __shared__ int bad;
  const int f = blockIdx.x, tid = threadIdx.x;
  const int nmb = mbw * mbh;
  const vp8g_frame_result& R = results[f];
  uint32_t* P = part + 16 * (size_t)f;
  if (R.error) {
    if (tid < 16) P[tid] = 0;
    return;
  }
  const uint32_t* cnt = mboff + (size_t)f * nmb;
  const uint8_t* info = mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES;
  const bool drop = R.use_skip != 0;
  const uint32_t ntok = R.ntokens;
  auto mb_count = [&](int m) -> uint32_t {   // the last MB of kind 1 is fixed up below
    if (drop && info[(size_t)m * VP8G_MBINFO_BYTES + 3]) return 0u;
    if (kind == 0) return cnt[m];
    return m + 1 < nmb ? cnt[m + 1] - cnt[m] : 0u;
  };
  for (int y = tid; y < mbh; y += 256) {
    uint32_t sum = 0;
    for (int x = 0; x < mbw; ++x) sum += mb_count(y * mbw + x);
    rowlen[y] = sum;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0;
    for (int y = 0; y < mbh; ++y) acc += rowlen[y];
    lastfix = 0;
    if (kind == 1 && !(drop && info[(size_t)(nmb - 1) * VP8G_MBINFO_BYTES + 3]))
      lastfix = ntok - acc;   // the last MB ends at the frame's token count
    rowlen[mbh - 1] += lastfix;
    uint32_t src = 0;
    for (int p = 0; p < VP8G_MAX_PARTS; ++p) plen[p] = 0;
    for (int y = 0; y < mbh; ++y) {
      rowsrc[y] = src;
      src += rowlen[y];
      plen[y & (nparts - 1)] += rowlen[y];
    }
    uint32_t o = (uint32_t)(((tok_cap / 2) + 7) & ~(size_t)7);
    bad = src != ntok || (size_t)ntok > tok_cap / 2;
    for (int p = 0; p < nparts; ++p) {
      poff[p] = o;
      o += part_region(plen[p]);
    }
    bad |= (size_t)o > tok_cap;
    uint32_t at[VP8G_MAX_PARTS];
    for (int p = 0; p < nparts; ++p) at[p] = poff[p];
    for (int y = 0; y < mbh; ++y) {
      rowdst[y] = at[y & (nparts - 1)];
      at[y & (nparts - 1)] += rowlen[y];
    }
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) P[0] = 0xffffffffu;
    return;
  }
  uint16_t* T = tokens + (size_t)f * tok_cap;
  const int wv = tid >> 6, ln = tid & 63;
  for (int y = wv; y < mbh; y += 4) {
    const uint16_t* s = T + rowsrc[y];
    uint16_t* d = T + rowdst[y];
    for (uint32_t i = ln; i < rowlen[y]; i += 64) d[i] = s[i];
  }
  if (tid < nparts) {
    P[tid] = poff[tid];
    P[8 + tid] = plen[tid];
  }
}

extern "C" int vp8g_launch_partition(uint16_t* tokens, size_t tok_cap, int n,
                                     const uint32_t* mboff, const vp8g_frame_result* results,
                                     const uint8_t* mbinfo, int mbw, int mbh, int kind,
                                     int nparts, uint32_t* part, void* stream) {
  if (n <= 0) return 1;
  if (mbh > PART_MAX_ROWS || nparts < 1 || nparts > VP8G_MAX_PARTS || (nparts & (nparts - 1))) {
    vp8g_set_error("k_partition", "unsupported frame height or partition count");
    return 0;
  }
  hipLaunchKernelGGL(k_partition, dim3(n), dim3(256), 0, (hipStream_t)stream, tokens, tok_cap,
                     mboff, results, mbinfo, mbw, mbh, kind, nparts, part);
  return vp8g_launch_check("k_partition");
}

// Partition 0's MB part (tree_enc.c:313-347: segment id, skip flag, intra-16
// or the 16 intra-4 modes, chroma mode) as fixed-probability tokens behind
// the frame's header tokens (vp8h_p0_header), for K4 to code as one more
// stream. The host's code_intra_modes (host/vp8_host.c) is the same walk.
// G 1,024-thread workgroups per frame, each a chunk of <= 1,024 raster MBs
// (one frame on one CU took 334 us at 1080p, on the latency path of a single
// picture): a workgroup counts the tokens of the MBs before its chunk (a
// block sum), a thread takes a run of consecutive MBs of the chunk, counts
// them, a block scan places the runs, then every thread writes its MBs' tokens. The intra-4 contexts are read from mbinfo
// directly: left = the previous MB of the row, top = the MB above, B_DC_PRED
// (0) across the picture edges; an intra-16 MB's mode fills its 16 entries.
#define P0T 1024
__constant__ uint8_t kP0PathLen[10] = {1, 2, 3, 5, 6, 6, 5, 6, 7, 7};
// intra-4 mode tree (tree_enc.c:270-295): nodes and bits along each mode's path
__constant__ uint8_t kP0PathNode[10][7] = {
    {0}, {0, 1}, {0, 1, 2}, {0, 1, 2, 3, 4}, {0, 1, 2, 3, 4, 5}, {0, 1, 2, 3, 4, 5},
    {0, 1, 2, 3, 6}, {0, 1, 2, 3, 6, 7}, {0, 1, 2, 3, 6, 7, 8}, {0, 1, 2, 3, 6, 7, 8}};
__constant__ uint8_t kP0PathBit[10][7] = {
    {0}, {1, 0}, {1, 1, 0}, {1, 1, 1, 0, 0}, {1, 1, 1, 0, 1, 0}, {1, 1, 1, 0, 1, 1},
    {1, 1, 1, 1, 0}, {1, 1, 1, 1, 1, 0}, {1, 1, 1, 1, 1, 1, 0}, {1, 1, 1, 1, 1, 1, 1}};

__device__ __forceinline__ uint16_t p0t(int bit, int prob) {
  return (uint16_t)((bit ? 0x8000u : 0u) | 0x4000u | (unsigned)prob);
}
__device__ __forceinline__ uint32_t p0_mb_count(const uint8_t* info, int upd, int use_skip) {
  uint32_t n = (upd ? 2u : 0u) + (use_skip ? 1u : 0u) + 1u;
  if (info[0]) {
    n += 2;
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) n += kP0PathLen[info[4 + k] < 10 ? info[4 + k] : 0];
  }
  const int uvm = info[1];
  return n + (uvm == 0 ? 1u : uvm == 2 ? 2u : 3u);
}

__global__ __launch_bounds__(P0T) void k_p0_modes(const uint8_t* __restrict__ mbinfo, int mbw,
                                                 int mbh, const vp8g_p0_par* __restrict__ par,
                                                 const uint16_t* __restrict__ hdr,
                                                 uint16_t* __restrict__ tokens,
                                                 vp8g_emit_meta* __restrict__ meta, int meta_base,
                                                 int G) {
  const int f = blockIdx.x / G, g = blockIdx.x % G, t = threadIdx.x, nmb = mbw * mbh;
  const vp8g_p0_par P = par[f];
  vp8g_emit_meta* M = meta + meta_base + f;
  if (P.nhdr == 0xffffffffu) {   // the frame failed: an empty stream
    if (g == 0 && t == 0) { M->ntok = 0; M->nseg = 0; }
    return;
  }
  uint16_t* out = tokens + M->tok_off;
  if (g == 0) {
    const uint16_t* h = hdr + (size_t)f * VP8G_P0_HDR_CAP;
    for (uint32_t k = t; k < P.nhdr; k += P0T) out[k] = h[k];
  }
  const uint8_t* info = mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES;
  const int lane = t & 63, wv = t >> 6;
  __shared__ uint32_t wsum[P0T / 64];
  // the tokens of the MBs before this workgroup's chunk
  const int chunk = (nmb + G - 1) / G;
  const int c0 = min(g * chunk, nmb), c1 = min(c0 + chunk, nmb);
  uint32_t prior = 0;
  for (int m = t; m < c0; m += P0T)
    prior += p0_mb_count(info + (size_t)m * VP8G_MBINFO_BYTES, P.update_map, P.use_skip);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) prior += __shfl_xor(prior, o);
  if (lane == 0) wsum[wv] = prior;
  __syncthreads();
  prior = 0;
#pragma unroll
  for (int k = 0; k < P0T / 64; ++k) prior += wsum[k];
  __syncthreads();   // wsum is reused by the scan below
  const int per = (c1 - c0 + P0T - 1) / P0T;
  const int m0 = min(c0 + t * per, c1), m1 = min(m0 + per, c1);
  uint32_t cnt = 0;
  for (int m = m0; m < m1; ++m)
    cnt += p0_mb_count(info + (size_t)m * VP8G_MBINFO_BYTES, P.update_map, P.use_skip);
  // exclusive scan of the runs' counts over the workgroup
  uint32_t incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int k = 0; k < P0T / 64; ++k) {
    const uint32_t v = wsum[k];
    before += k < wv ? v : 0u;
    total += v;
  }
  uint32_t pos = P.nhdr + prior + before + incl - cnt;
  for (int m = m0; m < m1; ++m) {
    const int x = m % mbw, y = m / mbw;
    const uint8_t* in = info + (size_t)m * VP8G_MBINFO_BYTES;
    const uint8_t* modes = in + 4;
    if (P.update_map) {   // segment id tree (tree_enc.c:313-321)
      const int sg = in[2];
      out[pos] = p0t(sg >= 2, P.seg_probas[0]);
      out[pos + 1] = p0t(sg & 1, P.seg_probas[1 + (sg >= 2)]);
      pos += 2;
    }
    if (P.use_skip) out[pos++] = p0t(in[3] != 0, P.skip_proba);   // :323-325
    const int i16 = in[0] != 0;
    out[pos++] = p0t(i16, 145);
    if (i16) {   // PutI16Mode (:257-266): DC 0, TM 1, V 2, H 3
      const int md = modes[0];
      const int b0 = md == 1 || md == 3;
      out[pos] = p0t(b0, 156);
      out[pos + 1] = b0 ? p0t(md == 1, 128) : p0t(md == 2, 163);
      pos += 2;
    } else {     // PutI4Mode (:268-295) with the neighbours' modes as context
      const uint8_t* above = y > 0 ? in - (size_t)mbw * VP8G_MBINFO_BYTES + 4 + 12 : nullptr;
      const uint8_t* leftm = x > 0 ? in - VP8G_MBINFO_BYTES + 4 : nullptr;
      for (int yy = 0; yy < 4; ++yy) {
        int left = leftm ? leftm[4 * yy + 3] : 0;
        for (int xx = 0; xx < 4; ++xx) {
          const int top = yy == 0 ? (above ? above[xx] : 0) : modes[4 * (yy - 1) + xx];
          const uint8_t* pr = kVP8BModeProba[top < 10 ? top : 0][left < 10 ? left : 0];
          const int md = modes[4 * yy + xx] < 10 ? modes[4 * yy + xx] : 0;
          const int len = kP0PathLen[md];
          for (int k = 0; k < len; ++k) out[pos + k] = p0t(kP0PathBit[md][k], pr[kP0PathNode[md][k]]);
          pos += len;
          left = md;
        }
      }
    }
    const int uvm = in[1];   // PutUVMode (:297-303): DC, then V / H / TM
    out[pos++] = p0t(uvm != 0, 142);
    if (uvm != 0) {
      out[pos++] = p0t(uvm != 2, 114);
      if (uvm != 2) out[pos++] = p0t(uvm != 3, 183);
    }
  }
  if (g == G - 1 && t == 0) {   // the last chunk ends the stream
    const uint32_t ntok = P.nhdr + prior + total;
    M->ntok = ntok;
    M->nseg = (ntok + EMIT_SEG - 1) / EMIT_SEG;
  }
}

extern "C" int vp8g_launch_p0_modes(const uint8_t* mbinfo, int mbw, int mbh, int n,
                                    const vp8g_p0_par* par, const uint16_t* hdr, uint16_t* tokens,
                                    vp8g_emit_meta* meta, int meta_base, void* stream) {
  if (n <= 0) return 1;
  const int G = (mbw * mbh + P0T - 1) / P0T;   // chunks of <= P0T MBs per frame
  hipLaunchKernelGGL(k_p0_modes, dim3(n * G), dim3(P0T), 0, (hipStream_t)stream, mbinfo, mbw, mbh,
                     par, hdr, tokens, meta, meta_base, G);
  return vp8g_launch_check("k_p0_modes");
}

// VP8EstimateTokenSize (token_enc.c:226-247) between the passes of a size
// search: sum of VP8BitCost(bit, p) over a frame's compact token stream, p the
// fixed probability of the token or the frame's probability table entry.
// Grid (chunks, n); probability and entropy tables staged in LDS; one
// 64-bit atomic per workgroup.
__global__ __launch_bounds__(256) void k_token_cost(const uint16_t* __restrict__ tokens,
                                                    size_t tok_cap, uint32_t rowcap,
                                                    const uint32_t* __restrict__ rowtok, int mbh,
                                                    const vp8g_frame_result* __restrict__ res,
                                                    const uint8_t* __restrict__ state,
                                                    const uint8_t* __restrict__ active,
                                                    unsigned long long* __restrict__ bits) {
  const int f = blockIdx.y;
  if (!active[f] || res[f].error) return;
  __shared__ uint8_t prob[VP8G_NUM_SLOTS];
  __shared__ uint16_t ecost[256];
  __shared__ unsigned long long wsum[4];
  const uint8_t* coeffs = state + (size_t)f * VP8G_RERUN_STATE_BYTES + VP8G_STATE_COEFFS;
  for (int s = threadIdx.x; s < VP8G_NUM_SLOTS; s += 256) prob[s] = coeffs[s];
  ecost[threadIdx.x] = kVP8EntropyCost[threadIdx.x];
  __syncthreads();
  const uint16_t* t = tokens + (size_t)f * tok_cap;
  uint32_t acc = 0;   // < 2^32: a chunk of the grid stride holds few tokens per thread
  // the compact stream, or K3's token rows one after another
  const int nr = rowtok ? mbh : 1;
  for (int y = 0; y < nr; ++y) {
    const uint32_t nt = rowtok ? rowtok[(size_t)f * mbh + y] : res[f].ntokens;
    const uint16_t* tr = t + (size_t)y * rowcap;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nt; i += gridDim.x * 256) {
      const uint32_t tk = tr[i];
      const int p = (tk & 0x4000u) ? (int)(tk & 0xffu) : (int)prob[tk & 0x3fffu];
      acc += (tk & 0x8000u) ? ecost[255 - p] : ecost[p];
    }
  }
  unsigned long long v = acc;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(&bits[f], wsum[0] + wsum[1] + wsum[2] + wsum[3]);
}

extern "C" int vp8g_launch_token_cost(const uint16_t* tokens, size_t tok_cap, const vp8g_rows* rows,
                                      int mbh, int n,
                                      const vp8g_frame_result* results, const uint8_t* state,
                                      const uint8_t* active, unsigned long long* bits,
                                      void* stream) {
  if (n <= 0) return 1;
  if (hipMemsetAsync(bits, 0, (size_t)n * sizeof(*bits), (hipStream_t)stream) != hipSuccess)
    return vp8g_launch_check("k_token_cost memset");
  // 128 chunks per frame: 7.6 M tokens at 1080p -> ~230 per thread, and
  // each token costs < 2^12, so the 32-bit per-thread sum cannot wrap below
  // 2^20 tokens per thread (2.7e10 tokens per frame)
  hipLaunchKernelGGL(k_token_cost, dim3(128, n), dim3(256), 0, (hipStream_t)stream, tokens,
                     tok_cap, rows ? rows->rowcap : 0u, rows ? rows->rowtok : nullptr, mbh, results,
                     state, active, bits);
  return vp8g_launch_check("k_token_cost");
}

// low_memory (VP8EncLoop for methods 3-6, frame_enc.c:614-775) on K3's
// compact token stream (MB m's tokens at [mboff[m], mboff[m+1])), one
// workgroup per frame:
//   mode 0: StatLoop's statistics — the dynamic tokens of the first
//           nb_stat[f] MBs replayed in raster order into stats[f] (kept
//           across passes; VP8RecordCoeffs puts each statistic in its
//           probability slot; exact in-order replay of the counters that reach
//           the halving point, cost_enc.h:45-56), and the skip count of those
//           MBs into nskip[f]
//   mode 1: drop the tokens of skipped MBs (use_skip[f]), update ntokens
__global__ __launch_bounds__(256) void k_lowmem(uint16_t* __restrict__ tokens, size_t tok_cap,
                                                const uint32_t* __restrict__ mboff,
                                                vp8g_frame_result* __restrict__ res,
                                                const uint8_t* __restrict__ mbinfo, int nmb,
                                                const int32_t* __restrict__ nb_stat,
                                                const uint8_t* __restrict__ active, int mode,
                                                uint32_t* __restrict__ stats,
                                                int32_t* __restrict__ nskip) {
  const int f = blockIdx.x, tid = threadIdx.x;
  if (!active[f]) return;
  __shared__ uint32_t st[VP8G_NUM_SLOTS], dl[VP8G_NUM_SLOTS], mark[33];
  __shared__ int any, cnt;
  uint16_t* T = tokens + (size_t)f * tok_cap;
  const uint32_t* off = mboff + (size_t)f * nmb;
  const uint8_t* info = mbinfo + (size_t)f * nmb * VP8G_MBINFO_BYTES;
  const uint32_t ntok = res[f].ntokens;
  if (mode == 0) {
    uint32_t* S = stats + (size_t)f * VP8G_NUM_SLOTS;
    for (int s = tid; s < VP8G_NUM_SLOTS; s += 256) { st[s] = S[s]; dl[s] = 0; }
    if (tid < 33) mark[tid] = 0;
    if (tid == 0) { any = 0; cnt = 0; }
    __syncthreads();
    const int nb = min(nb_stat[f], nmb);
    for (int m = 0; m < nb; ++m) {
      const uint32_t b0 = off[m], b1 = m + 1 < nmb ? off[m + 1] : ntok;
      if (tid == 0 && info[(size_t)m * VP8G_MBINFO_BYTES + 3]) ++cnt;
      for (uint32_t i = b0 + tid; i < b1; i += 256) {
        const uint32_t tk = T[i];
        if (!(tk & 0x4000u)) atomicAdd(&dl[tk & 0x3fffu], 0x10000u + (tk >> 15));
      }
      __syncthreads();
      for (int s = tid; s < VP8G_NUM_SLOTS; s += 256) {
        const uint32_t d = dl[s];
        if (d) {
          if ((st[s] >> 16) + (d >> 16) < 0xffffu) {
            st[s] += d;
          } else {
            atomicOr(&mark[s >> 5], 1u << (s & 31));
            any = 1;
          }
          dl[s] = 0;
        }
      }
      __syncthreads();
      if (any) {
        if (tid == 0)
          for (uint32_t i = b0; i < b1; ++i) {
            const uint32_t tk = T[i], sl = tk & 0x3fffu;
            if (!(tk & 0x4000u) && (mark[sl >> 5] & (1u << (sl & 31)))) {
              uint32_t p = st[sl];
              if (p >= 0xfffe0000u) p = ((p + 1u) >> 1) & 0x7fff7fffu;
              st[sl] = p + 0x00010000u + (tk >> 15);
            }
          }
        __syncthreads();
        if (tid < 33) mark[tid] = 0;
        if (tid == 0) any = 0;
        __syncthreads();
      }
    }
    for (int s = tid; s < VP8G_NUM_SLOTS; s += 256) S[s] = st[s];
    if (tid == 0) nskip[f] = cnt;
  } else {
    uint32_t dst = 0;
    for (int m = 0; m < nmb; ++m) {
      const uint32_t b0 = off[m], b1 = m + 1 < nmb ? off[m + 1] : ntok;
      if (info[(size_t)m * VP8G_MBINFO_BYTES + 3]) continue;
      if (dst != b0)
        for (uint32_t i = 0; i < b1 - b0; i += 256) {
          const bool in = i + tid < b1 - b0;
          const uint16_t t = in ? T[b0 + i + tid] : 0;
          __syncthreads();
          if (in) T[dst + i + tid] = t;
          __threadfence_block();
          __syncthreads();
        }
      dst += b1 - b0;
    }
    if (tid == 0) res[f].ntokens = dst;
  }
}

extern "C" int vp8g_launch_lowmem(uint16_t* tokens, size_t tok_cap, const uint32_t* mboff,
                                  vp8g_frame_result* results, const uint8_t* mbinfo, int nmb,
                                  int n, const int32_t* nb_stat, const uint8_t* active, int mode,
                                  uint32_t* stats, int32_t* nskip, void* stream) {
  if (n <= 0) return 1;
  hipLaunchKernelGGL(k_lowmem, dim3(n), dim3(256), 0, (hipStream_t)stream, tokens, tok_cap, mboff,
                     results, mbinfo, nmb, nb_stat, active, mode, stats, nskip);
  return vp8g_launch_check("k_lowmem");
}
