/* Test infrastructure only: the restatement of libwebp_amd's lossless
 * shortest-path parse for frames without a spatial predictor (oracle/
 * vp8l_model.py: dp_parse), in C because it walks every pixel. Reference
 * counterpart: TraceBackwards / BackwardReferencesHashChainDistanceOnly
 * (src/enc/backward_references_cost_enc.c:569-795): literal costs x 0.82,
 * colour-cache hits x 0.68, copies = length + distance prefix symbols and
 * their extra bits. Here each image row is parsed on its own, backwards
 * (cost_to_end[j] = the cheapest coding of pixels j..W-1), over the
 * candidate distances the caller passes (the first plane codes), copy
 * lengths 2..min(run, VP8L_DP_MAXK); ties keep the literal / cache hit,
 * then the shorter copy, then the earlier candidate. Costs are integers in
 * 1/256 bit. */
#include <stdint.h>
#include <stdlib.h>

#define VP8L_DP_MAXK 64

static void dp_prefix(uint32_t v, int* sym, int* nb) {
  const uint32_t d = v - 1;
  if (d < 4) { *sym = (int)d; *nb = 0; return; }
  const int h = 31 - __builtin_clz(d);
  *sym = 2 * h + (int)((d >> (h - 1)) & 1);
  *nb = h - 1;
}

/* runs: ncand x H*W (the run of argb[p + i] == argb[p + i - d_c] from p on
 * inside the row); hit: colour-cache hit per pixel (cache of the frame's
 * size); keys: its cache key; G has 280 + 2^cache_bits entries. Output in
 * the model's layout: act (0 literal, 1 cache, 2 copy start, 3 inside),
 * clen, ccode per pixel. */
void vp8l_dp_parse(int H, int W, const uint32_t* argb, const uint8_t* hit, const int32_t* keys,
                   int ncand, const int32_t* runs, const int32_t* dcodes, const int32_t* G,
                   const int32_t* R, const int32_t* B, const int32_t* A, const int32_t* D,
                   int64_t* act, int64_t* clen, int64_t* ccode) {
  int64_t* cost = (int64_t*)malloc(sizeof(int64_t) * (size_t)(W + 1));
  int16_t* chk = (int16_t*)malloc(sizeof(int16_t) * (size_t)(W + 1));
  int8_t* chc = (int8_t*)malloc((size_t)(W + 1));
  int dcost[64];
  int lcost[VP8L_DP_MAXK + 1];
  for (int c = 0; c < ncand && c < 64; ++c) {
    int s, nb;
    dp_prefix((uint32_t)dcodes[c], &s, &nb);
    dcost[c] = D[s] + 256 * nb;
  }
  for (int k = 1; k <= VP8L_DP_MAXK; ++k) {
    int s, nb;
    dp_prefix((uint32_t)k, &s, &nb);
    lcost[k] = G[256 + s] + 256 * nb;
  }
  for (int y = 0; y < H; ++y) {
    const size_t r0 = (size_t)y * W;
    cost[W] = 0;
    for (int j = W - 1; j >= 0; --j) {
      const size_t q = r0 + (size_t)j;
      const uint32_t a = argb[q];
      int64_t best = hit[q] ? cost[j + 1] + (int64_t)G[280 + keys[q]] * 68 / 100
                            : cost[j + 1] + (int64_t)(G[(a >> 8) & 255] + R[(a >> 16) & 255] +
                                                      B[a & 255] + A[a >> 24]) * 82 / 100;
      int bk = 1, bc = 0;
      for (int k = 2; k <= VP8L_DP_MAXK && j + k <= W; ++k) {
        /* the cheapest candidate whose run covers k */
        int dc = -1, cc = 0;
        for (int c = 0; c < ncand; ++c)
          if (runs[(size_t)c * H * W + q] >= k && (dc < 0 || dcost[c] < dc)) { dc = dcost[c]; cc = c; }
        if (dc < 0) break;   /* runs only shrink as k grows */
        const int64_t v = cost[j + k] + dc + lcost[k];
        if (v < best) { best = v; bk = k; bc = cc; }
      }
      cost[j] = best;
      chk[j] = (int16_t)bk;
      chc[j] = (int8_t)bc;
    }
    for (int j = 0; j < W;) {
      const size_t q = r0 + (size_t)j;
      const int k = chk[j];
      if (k >= 2) {
        act[q] = 2; clen[q] = k; ccode[q] = dcodes[chc[j]];
        for (int t = 1; t < k; ++t) { act[q + t] = 3; clen[q + t] = 0; ccode[q + t] = 0; }
        j += k;
      } else {
        act[q] = hit[q] ? 1 : 0; clen[q] = 0; ccode[q] = 0;
        j += 1;
      }
    }
  }
  free(cost); free(chk); free(chc);
}
