// Loss epilogues over an LDS tile of logits (whole rows, N <= 32), shared by
// the grouped GEMM (FWD_LOSS) and the fused MLP tail kernel.
//   C    : fp32 logits [BM][LDC]; replaced by dL/dz * inv_valid (train) in place
//   Ys   : fp32 targets [BM][BN]
//   srow : < 0 marks rows outside the batch (zero gradient, no loss)
// Only p.N, p.act, p.loss, p.nmet, p.met, p.Y (non-null = targets present),
// p.pred/p.sPred/p.ldp/p.chunk/p.B (prediction output) are read from `p`.
#pragma once
#include "common.h"

namespace ea {

// Fused softmax + (sparse) categorical cross-entropy over a GEMM tile holding
// whole rows (N <= 32): one quad (4 lanes) per row, the row's logits/targets in
// registers (NV = ceil(N/4) statically unrolled slots per lane) and DPP quad
// reductions -- no LDS round trips inside the row math, 64 rows per pass.
// Same math as row_loss's logits path (keras backend.categorical_crossentropy
// with from_logits): loss = -sum y (z - lse), dL/dz = softmax(z) * sum(y) - y.
// Other loss/activation/metric combinations use loss_tile_lds.
__device__ __forceinline__ bool softmax_cce_fast(const Prob& p) {
  if (p.act != ACT_SOFTMAX || !(p.loss == LOSS_CCE || p.loss == LOSS_SPARSE_CCE) || !p.Y || p.N > 32) return false;
  bool ok = true;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (q < p.nmet)
      ok = ok && (p.met[q] == MET_ACC_CAT || p.met[q] == MET_ACC_SPARSE || p.met[q] == LOSS_CCE ||
                  p.met[q] == LOSS_SPARSE_CCE);
  return ok;
}

template <int NV, int BM, int LDC, int BN>
__device__ __forceinline__ void loss_tile_cce(const Prob& p, int r, int m0, float* C, const float* Ys, const int* srow,
                                              bool train, float inv_valid, float (&sums)[6]) {
  constexpr int W = 4;
  const int lane = threadIdx.x & 3, grp = threadIdx.x >> 2;
  const int N = p.N;
  const bool sparse = p.loss == LOSS_SPARSE_CCE;
  for (int row = grp; row < BM; row += 64) {
    float* zrow = C + row * LDC;
    const float* yrow = Ys + row * BN;
    float z[NV], y[NV];
    const int ycls = sparse ? (int)yrow[0] : -1;
#pragma unroll
    for (int i = 0; i < NV; ++i) {  // in-bounds of the LDS tile even past N
      const int j = lane + i * W;
      z[i] = zrow[j];
      y[i] = sparse ? (j == ycls ? 1.f : 0.f) : yrow[j];
    }
    if (srow[row] < 0) {
      if (train) {
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if (lane + i * W < N) zrow[lane + i * W] = 0.f;
      }
      continue;
    }
    float zmax = -INFINITY;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (lane + i * W < N) zmax = fmaxf(zmax, z[i]);
    zmax = row_max<W>(zmax);
    float se = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if (lane + i * W < N) se += __expf(z[i] - zmax);
    se = row_sum<W>(se);
    const float lse = zmax + logf(se);
    float l = 0.f, ysum = 0.f, bp = -INFINITY, by = -INFINITY, pr[NV];
    int ip = 0x7fffffff, iy = 0x7fffffff;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int j = lane + i * W;
      pr[i] = __expf(z[i] - lse);
      if (j < N) {
        l += -y[i] * (z[i] - lse);
        ysum += y[i];
        if (pr[i] > bp) { bp = pr[i]; ip = j; }
        if (y[i] > by) { by = y[i]; iy = j; }
      }
    }
    l = row_sum<W>(l);
    ysum = row_sum<W>(ysum);
    row_argmax<W>(bp, ip);
    row_argmax<W>(by, iy);
    if (sparse) iy = ycls;
    const float acc = ip == iy ? 1.f : 0.f;
    if (p.pred) {
      float* prow = p.pred + (long long)r * p.sPred + (p.chunk * p.B + m0 + row) * p.ldp;
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if (lane + i * W < N) prow[lane + i * W] = pr[i];
    }
    if (train) {
#pragma unroll
      for (int i = 0; i < NV; ++i)
        if (lane + i * W < N) zrow[lane + i * W] = (pr[i] * ysum - y[i]) * inv_valid;
    }
    if (lane == 0) {
      sums[0] += l;
      sums[1] += 1.f;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < p.nmet) sums[2 + q] += (p.met[q] == MET_ACC_CAT || p.met[q] == MET_ACC_SPARSE) ? acc : l;
    }
  }
}

// Generic fused loss (any loss/activation/metrics): 16 lanes per row, values
// read from the LDS tile in runtime loops (keeps code size bounded).
template <int BM, int LDC, int BN>
__device__ __forceinline__ void loss_tile_lds(const Prob& p, int r, int m0, float* C, const float* Ys, const int* srow,
                                              bool train, float inv_valid, float (&sums)[6]) {
  constexpr int W = 16;
  const int lane = threadIdx.x % W, grp = threadIdx.x / W;
  for (int row = grp; row < BM; row += 256 / W) {
    float* zrow = C + row * LDC;
    const float* yrow = Ys + row * BN;
    if (srow[row] < 0) {
      if (train)
        for (int j = lane; j < p.N; j += W) zrow[j] = 0.f;
      continue;
    }
    float* prow = p.pred ? p.pred + (long long)r * p.sPred + (p.chunk * p.B + m0 + row) * p.ldp : nullptr;
    auto zat = [&](int, int j) { return zrow[j]; };
    auto pout = [&](int, int j, float v) { prow[j] = v; };
    if (!p.Y) {
      if (prow) row_predict<W, 0>(lane, p.N, p.act, zat, pout);
      continue;
    }
    RowOut ro;
    ro.loss = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) ro.metric[q] = 0.f;
    row_loss<W, 0>(lane, p.N, p.act, p.loss, p.met, p.nmet, zat, [&](int, int j) { return yrow[j]; }, yrow[0],
                   train, [&](int, int j, float v) { zrow[j] = v * inv_valid; }, prow != nullptr, pout, ro);
    if (lane == 0) {
      sums[0] += ro.loss;
      sums[1] += 1.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) sums[2 + q] += ro.metric[q];
    }
  }
}

}  // namespace ea
