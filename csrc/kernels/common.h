// Shared device-side definitions for the elephas_amd CDNA4 (gfx950) kernels.
//
// Design notes (MI355X-first, see docs/ARCHITECTURE.md):
//  * wave64 everywhere; every block is 256 threads = 4 waves.
//  * GEMM-shaped work runs on MFMA: bf16 operands use v_mfma_f32_16x16x32_bf16,
//    fp32 operands use the exact-f32 v_mfma_f32_16x16x4_f32 (no xf32 on gfx950).
//  * Activation / dropout / loss / optimizer math is fused into GEMM epilogues.
//  * Dropout masks are counter-based (a hash of seed/replica/layer/iteration/
//    row/column) so backward regenerates them instead of storing them.
//
// Semantics mirror tf.keras 2.10 as used by the reference
// (reference: elephas/worker.py:41-42 model.fit, tests/conftest.py:8-40 layer set).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "args.h"

namespace ea {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr float KERAS_EPS = 1e-7f;

// -------------------------------------------------------------- bf16 I/O ----
template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<__bf16>(__bf16 v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __bf16 from_f<__bf16>(float v) { return (__bf16)v; }

// ---------------------------------------------------------------- dropout
// keep iff u >= rate (tf.nn.dropout semantics), kept values scaled by 1/(1-rate).
// Dropout keep-uniforms as a pure function of (seed, replica, layer, iteration,
// batch row, column), so forward and backward (and the grouped and fused
// kernels) regenerate identical masks without storing them. One murmur3 fmix32
// (2 quarter-rate multiplies) per column PAIR yields two 16-bit uniforms --
// ~6x cheaper than a Philox4x32-7 call per 4 columns; keep-probability error
// < 2^-16. The per-(replica, layer, iteration) base is hoisted by the caller.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t dropout_base(uint64_t seed, int replica, int layer, long long iter) {
  return fmix32((uint32_t)seed ^ fmix32((uint32_t)iter * 0x9E3779B1u ^ (uint32_t)((unsigned long long)iter >> 32) ^
                                        ((uint32_t)layer << 24) ^ (uint32_t)replica * 0x27D4EB2Fu ^
                                        (uint32_t)(seed >> 32)));
}
// uniforms for columns c0 .. c0+7 (c0 % 8 == 0) of batch row `row` (< 65536)
__device__ __forceinline__ void dropout_u8(uint32_t base, int row, int c0, float (&u)[8]) {
  constexpr float s = 1.0f / 65536.0f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t h = fmix32(base ^ (((uint32_t)row << 16) | (uint32_t)((c0 >> 1) + j)));
    u[2 * j] = (float)(h & 0xFFFFu) * s;
    u[2 * j + 1] = (float)(h >> 16) * s;
  }
}

// ----------------------------------------------------------- activations ----
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float softplusf_(float x) {
  // log(1+exp(x)), stable
  return fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x)));
}

__device__ __forceinline__ float act_fwd(int act, float z) {
  switch (act) {
    case ACT_RELU: return fmaxf(z, 0.f);
    case ACT_SIGMOID: return sigmoidf_(z);
    case ACT_TANH: return tanhf(z);
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    case ACT_SELU: return 1.0507009873554805f * (z > 0.f ? z : 1.6732632423543772f * expm1f(z));
    case ACT_SOFTPLUS: return softplusf_(z);
    case ACT_SOFTSIGN: return z / (fabsf(z) + 1.f);
    case ACT_EXPONENTIAL: return __expf(z);
    case ACT_HARD_SIGMOID: return fminf(fmaxf(0.2f * z + 0.5f, 0.f), 1.f);
    case ACT_SWISH: return z * sigmoidf_(z);
    case ACT_GELU: return 0.5f * z * (1.f + erff(z * 0.7071067811865476f));
    case ACT_RELU6: return fminf(fmaxf(z, 0.f), 6.f);
    default: return z;  // linear (softmax handled row-wise)
  }
}

// d act / d z evaluated at z
__device__ __forceinline__ float act_grad(int act, float z) {
  switch (act) {
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    case ACT_SIGMOID: { float s = sigmoidf_(z); return s * (1.f - s); }
    case ACT_TANH: { float t = tanhf(z); return 1.f - t * t; }
    case ACT_ELU: return z > 0.f ? 1.f : __expf(z);
    case ACT_SELU: return 1.0507009873554805f * (z > 0.f ? 1.f : 1.6732632423543772f * __expf(z));
    case ACT_SOFTPLUS: return sigmoidf_(z);
    case ACT_SOFTSIGN: { float d = fabsf(z) + 1.f; return 1.f / (d * d); }
    case ACT_EXPONENTIAL: return __expf(z);
    case ACT_HARD_SIGMOID: return (z > -2.5f && z < 2.5f) ? 0.2f : 0.f;
    case ACT_SWISH: { float s = sigmoidf_(z); return s + z * s * (1.f - s); }
    case ACT_GELU: {
      const float c = 0.3989422804014327f;  // 1/sqrt(2pi)
      return 0.5f * (1.f + erff(z * 0.7071067811865476f)) + z * c * __expf(-0.5f * z * z);
    }
    case ACT_RELU6: return (z > 0.f && z < 6.f) ? 1.f : 0.f;
    default: return 1.f;
  }
}

// Vector forms: the activation is uniform per layer, so dispatch ONCE and run a
// compact per-case loop. Inlining the scalar switch per element (8-32 copies)
// made kernels 0.3-1.3 MB and their executed path instruction-fetch bound.
#define EA_ACTS(X)                                                                                   \
  X(ACT_RELU, fmaxf(x, 0.f), (x > 0.f ? 1.f : 0.f))                                                  \
  X(ACT_SIGMOID, sigmoidf_(x), (sigmoidf_(x) * (1.f - sigmoidf_(x))))                                \
  X(ACT_TANH, tanhf(x), (1.f - tanhf(x) * tanhf(x)))                                                 \
  X(ACT_ELU, (x > 0.f ? x : expm1f(x)), (x > 0.f ? 1.f : __expf(x)))                                 \
  X(ACT_SELU, 1.0507009873554805f * (x > 0.f ? x : 1.6732632423543772f * expm1f(x)),                  \
    1.0507009873554805f * (x > 0.f ? 1.f : 1.6732632423543772f * __expf(x)))                          \
  X(ACT_SOFTPLUS, softplusf_(x), sigmoidf_(x))                                                       \
  X(ACT_SOFTSIGN, x / (fabsf(x) + 1.f), 1.f / ((fabsf(x) + 1.f) * (fabsf(x) + 1.f)))                 \
  X(ACT_EXPONENTIAL, __expf(x), __expf(x))                                                            \
  X(ACT_HARD_SIGMOID, fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f), ((x > -2.5f && x < 2.5f) ? 0.2f : 0.f)) \
  X(ACT_SWISH, x * sigmoidf_(x), (sigmoidf_(x) + x * sigmoidf_(x) * (1.f - sigmoidf_(x))))          \
  X(ACT_GELU, 0.5f * x * (1.f + erff(x * 0.7071067811865476f)),                                       \
    0.5f * (1.f + erff(x * 0.7071067811865476f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x))   \
  X(ACT_RELU6, fminf(fmaxf(x, 0.f), 6.f), ((x > 0.f && x < 6.f) ? 1.f : 0.f))

template <int NV>
__device__ __forceinline__ void act_fg_v(int act, const float (&z)[NV], float (&o)[NV], float (&g)[NV]) {
#define EA_CASE_FG(ID, F, G) \
  case ID:                   \
    _Pragma("unroll") for (int q = 0; q < NV; ++q) { const float x = z[q]; o[q] = (F); g[q] = (G); } break;
  switch (act) {
    EA_ACTS(EA_CASE_FG)
    default:
      _Pragma("unroll") for (int q = 0; q < NV; ++q) { o[q] = z[q]; g[q] = 1.f; }
  }
#undef EA_CASE_FG
}
template <int NV>
__device__ __forceinline__ void act_f_v(int act, const float (&z)[NV], float (&o)[NV]) {
#define EA_CASE_F(ID, F, G) \
  case ID:                  \
    _Pragma("unroll") for (int q = 0; q < NV; ++q) { const float x = z[q]; o[q] = (F); } break;
  switch (act) {
    EA_ACTS(EA_CASE_F)
    default:
      _Pragma("unroll") for (int q = 0; q < NV; ++q) o[q] = z[q];
  }
#undef EA_CASE_F
}
template <int NV>
__device__ __forceinline__ void act_g_v(int act, const float (&z)[NV], float (&g)[NV]) {
#define EA_CASE_G(ID, F, G) \
  case ID:                  \
    _Pragma("unroll") for (int q = 0; q < NV; ++q) { const float x = z[q]; g[q] = (G); } break;
  switch (act) {
    EA_ACTS(EA_CASE_G)
    default:
      _Pragma("unroll") for (int q = 0; q < NV; ++q) g[q] = 1.f;
  }
#undef EA_CASE_G
}

// --------------------------------------------------------- row reductions ----
// W = 1: a single thread owns the row.  W = 64: a whole wave owns the row.
// lane-group reductions. W == 4 (quads) uses DPP quad_perm moves (no LDS
// round trip); wider groups use ds_bpermute via __shfl_xor.
__device__ __forceinline__ float quad_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_xor2(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
}
__device__ __forceinline__ int quad_xor1(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int quad_xor2(int v) { return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false); }

template <int W> __device__ __forceinline__ float row_sum(float v) {
  if constexpr (W == 1) return v;
  if constexpr (W == 4) { v += quad_xor1(v); return v + quad_xor2(v); }
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, W);
  return v;
}
template <int W> __device__ __forceinline__ float row_max(float v) {
  if constexpr (W == 1) return v;
  if constexpr (W == 4) { v = fmaxf(v, quad_xor1(v)); return fmaxf(v, quad_xor2(v)); }
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, W));
  return v;
}
// argmax with first-index tie-break (np.argmax / tf.argmax semantics)
template <int W> __device__ __forceinline__ void row_argmax(float& v, int& i) {
  if constexpr (W == 1) return;
  if constexpr (W == 4) {
    float ov = quad_xor1(v); int oi = quad_xor1(i);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
    ov = quad_xor2(v); oi = quad_xor2(i);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
    return;
  }
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) {
    float ov = __shfl_xor(v, o, W);
    int oi = __shfl_xor(i, o, W);
    if (ov > v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

// ------------------------------------------------- per-row loss & metrics ----
// Computes, for one row of logits z[0..N) with targets y, the per-row loss value
// (keras per-sample loss, before the batch mean), optional per-row metric
// values, and optionally dL/dz (per-row, NOT yet divided by batch size) and/or
// the activated prediction p.
//
// z:  pointer to the row's pre-activation values (fp32) (read-only)
// y:  pointer to the row's targets (fp32); sparse labels: y[0] = class id
// Softmax+CCE and sigmoid+BCE take tf.keras's logits path
// (keras/backend.py categorical_crossentropy: output._keras_logits); every other
// pairing uses the clipped probability formula and a chain rule through act.
struct RowOut {
  float loss;
  float metric[4];
};

template <int W>
__device__ __forceinline__ float loss_elem_value(int loss, float p, float y, float z, bool logit_path) {
  const float eps = KERAS_EPS;
  switch (loss) {
    case LOSS_MSE: { float d = p - y; return d * d; }
    case LOSS_MAE: return fabsf(p - y);
    case LOSS_MAPE: return 100.f * fabsf((y - p) / fmaxf(fabsf(y), eps));
    case LOSS_MSLE: { float a = log1pf(fmaxf(p, eps)) - log1pf(fmaxf(y, eps)); return a * a; }
    case LOSS_LOGCOSH: { float x = p - y; return x + softplusf_(-2.f * x) - 0.6931471805599453f; }
    case LOSS_HINGE: return fmaxf(1.f - y * p, 0.f);
    case LOSS_SQ_HINGE: { float h = fmaxf(1.f - y * p, 0.f); return h * h; }
    case LOSS_POISSON: return p - y * logf(p + eps);
    case LOSS_BCE: {
      if (logit_path) return fmaxf(z, 0.f) - z * y + log1pf(__expf(-fabsf(z)));
      float pc = fminf(fmaxf(p, eps), 1.f - eps);
      return -(y * logf(pc + eps) + (1.f - y) * logf(1.f - pc + eps));
    }
    case LOSS_KLD: {
      float yt = fminf(fmaxf(y, eps), 1.f), pp = fminf(fmaxf(p, eps), 1.f);
      return yt * logf(yt / pp);
    }
    default: return 0.f;
  }
}

// derivative of the elementwise loss term wrt p
__device__ __forceinline__ float loss_elem_grad(int loss, float p, float y) {
  const float eps = KERAS_EPS;
  switch (loss) {
    case LOSS_MSE: return 2.f * (p - y);
    case LOSS_MAE: return (p > y) ? 1.f : ((p < y) ? -1.f : 0.f);
    case LOSS_MAPE: { float s = (p > y) ? 1.f : ((p < y) ? -1.f : 0.f); return 100.f * s / fmaxf(fabsf(y), eps); }
    case LOSS_MSLE: {
      float a = log1pf(fmaxf(p, eps)) - log1pf(fmaxf(y, eps));
      return (p > eps) ? 2.f * a / (1.f + p) : 0.f;
    }
    case LOSS_LOGCOSH: return tanhf(p - y);
    case LOSS_HINGE: return (1.f - y * p > 0.f) ? -y : 0.f;
    case LOSS_SQ_HINGE: { float h = 1.f - y * p; return h > 0.f ? -2.f * y * h : 0.f; }
    case LOSS_POISSON: return 1.f - y / (p + eps);
    case LOSS_BCE: {
      if (p <= eps || p >= 1.f - eps) return 0.f;  // clip_by_value grad
      return -(y / (p + eps)) + (1.f - y) / (1.f - p + eps);
    }
    case LOSS_KLD: { float yt = fminf(fmaxf(y, eps), 1.f); return (p > eps && p < 1.f) ? -yt / p : 0.f; }
    default: return 0.f;
  }
}

__device__ __forceinline__ bool loss_is_mean_over_last_axis(int loss) {
  return !(loss == LOSS_CCE || loss == LOSS_SPARSE_CCE || loss == LOSS_KLD || loss == LOSS_COSINE ||
           loss == LOSS_CAT_HINGE);
}

// Generic per-row evaluation. Element j is visited by lane `lane` for j = lane, lane+W, ...
//   dz_out(j, v) is called with the per-row gradient dL_row/dz_j (if want_grad)
//   p_out(j, v) is called with the prediction p_j (if want_pred)
// Column loop over this lane's elements j = lane, lane+W, ... (< N).
// NV > 0: fully unrolled over NV register slots (i_ is a compile-time index, so
// accessors may index register arrays); NV == 0: runtime loop (wide rows).
#define EA_FORJ(...)                                                         \
  if constexpr (NV > 0) {                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < (NV > 0 ? NV : 1); ++i_) {       \
      const int j = lane + i_ * W;                                           \
      if (j < N) { __VA_ARGS__ }                                             \
    }                                                                        \
  } else {                                                                   \
    for (int j = lane, i_ = 0; j < N; j += W, ++i_) { __VA_ARGS__ }          \
  }

template <int W, int NV, typename ZF, typename YF, typename GF, typename PF>
__device__ __forceinline__ void row_loss(int lane, int N, int act, int loss, const int* metrics, int nmetrics,
                         ZF zat, YF yat, float y0, bool want_grad, GF dz_out, bool want_pred, PF p_out,
                         RowOut& out) {
  // y0: the row's first target value (the class id for sparse labels)
  const bool sparse = (loss == LOSS_SPARSE_CCE);
  const int ycls = sparse ? (int)y0 : -1;
  auto Y = [&](int i, int j) -> float { return sparse ? (j == ycls ? 1.f : 0.f) : yat(i, j); };
  // softmax statistics
  float zmax = -INFINITY, sumexp = 0.f;
  if (act == ACT_SOFTMAX) {
    EA_FORJ(zmax = fmaxf(zmax, zat(i_, j));)
    zmax = row_max<W>(zmax);
    EA_FORJ(sumexp += __expf(zat(i_, j) - zmax);)
    sumexp = row_sum<W>(sumexp);
  }
  const float lse = zmax + logf(sumexp);
  auto P = [&](int i, int j) -> float {
    float z = zat(i, j);
    return act == ACT_SOFTMAX ? __expf(z - lse) : act_fwd(act, z);
  };
  const bool cce_like = (loss == LOSS_CCE || loss == LOSS_SPARSE_CCE);
  const bool logit_cce = cce_like && act == ACT_SOFTMAX;
  const bool logit_bce = (loss == LOSS_BCE) && act == ACT_SIGMOID;
  const float invN = 1.f / (float)N;

  // ---- loss value
  float lsum = 0.f, psum = 0.f, ysum = 0.f;
  if (cce_like && !logit_cce) {
    EA_FORJ(psum += P(i_, j);)
    psum = row_sum<W>(psum);
  }
  float ynorm = 0.f, pnorm = 0.f, yp = 0.f;  // cosine
  float cat_pos = 0.f, cat_neg = -INFINITY;  // categorical hinge
  EA_FORJ(float z = zat(i_, j), y = Y(i_, j), p = P(i_, j);
    if (logit_cce) lsum += -y * (z - lse);
    else if (cce_like) {
      float pn = fminf(fmaxf(p / psum, KERAS_EPS), 1.f - KERAS_EPS);
      lsum += -y * logf(pn);
    } else if (loss == LOSS_COSINE) { ynorm += y * y; pnorm += p * p; yp += y * p; }
    else if (loss == LOSS_CAT_HINGE) { cat_pos += y * p; cat_neg = fmaxf(cat_neg, (1.f - y) * p); }
    else lsum += loss_elem_value<W>(loss, p, y, z, logit_bce);
    ysum += y;)
  lsum = row_sum<W>(lsum);
  ysum = row_sum<W>(ysum);
  float rl;
  if (loss == LOSS_COSINE) {
    ynorm = row_sum<W>(ynorm); pnorm = row_sum<W>(pnorm); yp = row_sum<W>(yp);
    float ny = rsqrtf(fmaxf(ynorm, 1e-12f)), np_ = rsqrtf(fmaxf(pnorm, 1e-12f));
    rl = -yp * ny * np_;
  } else if (loss == LOSS_CAT_HINGE) {
    cat_pos = row_sum<W>(cat_pos); cat_neg = row_max<W>(cat_neg);
    rl = fmaxf(cat_neg - cat_pos + 1.f, 0.f);
  } else {
    rl = loss_is_mean_over_last_axis(loss) ? lsum * invN : lsum;
  }
  out.loss = rl;

  // ---- metrics (static indices only: no scratch copies of the metric list)
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    if (mi >= nmetrics) break;
    const int m = metrics[mi];
    float mv = 0.f;
    if (m == MET_ACC_CAT || m == MET_ACC_SPARSE) {
      float bp = -INFINITY; int ip = 0x7fffffff;
      float by = -INFINITY; int iy = 0x7fffffff;
      EA_FORJ(float p = P(i_, j);
        if (p > bp) { bp = p; ip = j; }
        float yv = Y(i_, j);
        if (yv > by) { by = yv; iy = j; })
      row_argmax<W>(bp, ip);
      row_argmax<W>(by, iy);
      if (m == MET_ACC_SPARSE) iy = ycls;
      mv = (ip == iy) ? 1.f : 0.f;
    } else if (m == MET_ACC_BIN) {
      float s = 0.f;
      EA_FORJ(s += ((P(i_, j) > 0.5f ? 1.f : 0.f) == Y(i_, j)) ? 1.f : 0.f;)
      mv = row_sum<W>(s) * invN;
    } else if (m == LOSS_CCE || m == LOSS_SPARSE_CCE) {
      float s = 0.f;
      EA_FORJ(s += (act == ACT_SOFTMAX) ? -Y(i_, j) * (zat(i_, j) - lse)
                                                                  : -Y(i_, j) * logf(fminf(fmaxf(P(i_, j), KERAS_EPS), 1.f - KERAS_EPS));)
      mv = row_sum<W>(s);
    } else if (m == LOSS_COSINE) {
      float a = 0.f, b = 0.f, c = 0.f;
      EA_FORJ(float p = P(i_, j), y = Y(i_, j); a += y * y; b += p * p; c += y * p;)
      a = row_sum<W>(a); b = row_sum<W>(b); c = row_sum<W>(c);
      mv = c * rsqrtf(fmaxf(a, 1e-12f)) * rsqrtf(fmaxf(b, 1e-12f));  // keras metric: +cos
    } else {
      float s = 0.f;
      EA_FORJ(s += loss_elem_value<W>(m, P(i_, j), Y(i_, j), zat(i_, j), m == LOSS_BCE && act == ACT_SIGMOID);)
      s = row_sum<W>(s);
      mv = loss_is_mean_over_last_axis(m) ? s * invN : s;
    }
    out.metric[mi] = mv;
  }

  // ---- prediction
  if (want_pred)
    EA_FORJ(p_out(i_, j, P(i_, j));)

  // ---- gradient wrt z (per row)
  if (want_grad) {
    if (logit_cce) {
      EA_FORJ(dz_out(i_, j, __expf(zat(i_, j) - lse) * ysum - Y(i_, j));)
    } else if (logit_bce) {
      EA_FORJ(dz_out(i_, j, (sigmoidf_(zat(i_, j)) - Y(i_, j)) * invN);)
    } else {
      // g_j = dL/dp_j
      auto G = [&](int i, int j) -> float {
        float p = P(i, j), y = Y(i, j);
        if (cce_like) {
          float pn = p / psum;
          if (pn <= KERAS_EPS || pn >= 1.f - KERAS_EPS) return 0.f;
          // d/dp_j of -sum_k y_k log(p_k/psum) = -y_j/p_j + ysum/psum
          return -y / p + ysum / psum;
        }
        if (loss == LOSS_COSINE) {
          float ny = rsqrtf(fmaxf(ynorm, 1e-12f)), np_ = rsqrtf(fmaxf(pnorm, 1e-12f));
          // d/dp (-(y.p) ny np)
          return -(y * ny * np_ - yp * ny * np_ * np_ * np_ * p);
        }
        if (loss == LOSS_CAT_HINGE) {
          float h = cat_neg - cat_pos + 1.f;
          if (h <= 0.f) return 0.f;
          float g = -y;
          if ((1.f - y) * p == cat_neg) g += (1.f - y);
          return g;
        }
        float g = loss_elem_grad(loss, p, y);
        return loss_is_mean_over_last_axis(loss) ? g * invN : g;
      };
      if (act == ACT_SOFTMAX) {
        float gp = 0.f;
        EA_FORJ(gp += G(i_, j) * P(i_, j);)
        gp = row_sum<W>(gp);
        EA_FORJ(dz_out(i_, j, P(i_, j) * (G(i_, j) - gp));)
      } else {
        EA_FORJ(dz_out(i_, j, G(i_, j) * act_grad(act, zat(i_, j)));)
      }
    }
  }
}


// ---------------------------------------------------------- optimizer math
// Keras 2.10 optimizer_v2 update rules (keras/optimizers/optimizer_v2/{gradient_descent,
// rmsprop,adam,adagrad,adamax}.py); decayed lr = lr / (1 + decay * iterations).
__device__ __forceinline__ float opt_update(const OptParams& p, float w, float g, float* S, long long si,
                                            long long iter) {
  const float lr = p.lr / (1.f + p.decay * (float)iter);
  switch (p.opt) {
    case OPT_SGD: {
      if (p.mom == 0.f) return w - lr * g;
      float v = p.mom * S[si] - lr * g;
      S[si] = v;
      return p.nesterov ? w + p.mom * v - lr * g : w + v;
    }
    case OPT_RMSPROP: {
      float ms = p.rho * S[si] + (1.f - p.rho) * g * g;
      S[si] = ms;
      if (p.mom > 0.f) {  // tf ApplyRMSProp: epsilon inside the square root
        float m = p.mom * S[si + p.s_plane] + lr * g / sqrtf(ms + p.eps);
        S[si + p.s_plane] = m;
        return w - m;
      }
      return w - lr * g / (sqrtf(ms) + p.eps);
    }
    case OPT_ADAM: {
      const float t = (float)(iter + 1);
      const float b1t = powf(p.b1, t), b2t = powf(p.b2, t);
      const float lrt = lr * sqrtf(1.f - b2t) / (1.f - b1t);
      float m = p.b1 * S[si] + (1.f - p.b1) * g;
      float v = p.b2 * S[si + p.s_plane] + (1.f - p.b2) * g * g;
      S[si] = m;
      S[si + p.s_plane] = v;
      return w - lrt * m / (sqrtf(v) + p.eps);
    }
    case OPT_ADAGRAD: {
      float a = S[si] + g * g;
      S[si] = a;
      return w - lr * g / (sqrtf(a) + p.eps);
    }
    case OPT_ADAMAX: {
      const float t = (float)(iter + 1);
      const float lrt = lr / (1.f - powf(p.b1, t));
      float m = p.b1 * S[si] + (1.f - p.b1) * g;
      float u = fmaxf(p.b2 * S[si + p.s_plane], fabsf(g));
      S[si] = m;
      S[si + p.s_plane] = u;
      return w - lrt * m / (u + p.eps);
    }
  }
  return w;
}

template <int W, int NV, typename ZF, typename PF>
__device__ __forceinline__ void row_predict(int lane, int N, int act, ZF zat, PF p_out) {
  if (act == ACT_SOFTMAX) {
    float zmax = -INFINITY, s = 0.f;
    EA_FORJ(zmax = fmaxf(zmax, zat(i_, j));)
    zmax = row_max<W>(zmax);
    EA_FORJ(s += __expf(zat(i_, j) - zmax);)
    s = row_sum<W>(s);
    const float inv = 1.f / s;
    EA_FORJ(p_out(i_, j, __expf(zat(i_, j) - zmax) * inv);)
  } else {
    EA_FORJ(p_out(i_, j, act_fwd(act, zat(i_, j)));)
  }
}

// number of optimizer state planes a rule reads/writes
__device__ __forceinline__ int opt_planes(const OptParams& p) {
  switch (p.opt) {
    case OPT_SGD: return p.mom != 0.f ? 1 : 0;
    case OPT_RMSPROP: return p.mom > 0.f ? 2 : 1;
    case OPT_ADAGRAD: return 1;
    default: return 2;  // adam, adamax
  }
}

// same rules as opt_update with the state held in registers

// Vector form: one dispatch on the optimizer, per-step scalars (decayed lr,
// Adam/Adamax bias corrections) computed once, compact per-case loops.
template <int NV>
__device__ __forceinline__ void opt_update_v(const OptParams& p, float (&w)[NV], const float (&g)[NV],
                                             float (&s0)[NV], float (&s1)[NV], long long iter) {
  const float lr = p.lr / (1.f + p.decay * (float)iter);
  switch (p.opt) {
    case OPT_SGD:
      if (p.mom == 0.f) {
        _Pragma("unroll") for (int q = 0; q < NV; ++q) w[q] -= lr * g[q];
      } else {
        _Pragma("unroll") for (int q = 0; q < NV; ++q) {
          const float v = p.mom * s0[q] - lr * g[q];
          s0[q] = v;
          w[q] = p.nesterov ? w[q] + p.mom * v - lr * g[q] : w[q] + v;
        }
      }
      break;
    case OPT_RMSPROP:
      _Pragma("unroll") for (int q = 0; q < NV; ++q) {
        const float ms = p.rho * s0[q] + (1.f - p.rho) * g[q] * g[q];
        s0[q] = ms;
        if (p.mom > 0.f) {  // tf ApplyRMSProp: epsilon inside the square root
          const float m = p.mom * s1[q] + lr * g[q] / sqrtf(ms + p.eps);
          s1[q] = m;
          w[q] -= m;
        } else {
          w[q] -= lr * g[q] / (sqrtf(ms) + p.eps);
        }
      }
      break;
    case OPT_ADAM: {
      const float t = (float)(iter + 1);
      const float lrt = lr * sqrtf(1.f - powf(p.b2, t)) / (1.f - powf(p.b1, t));
      _Pragma("unroll") for (int q = 0; q < NV; ++q) {
        const float m = p.b1 * s0[q] + (1.f - p.b1) * g[q];
        const float v = p.b2 * s1[q] + (1.f - p.b2) * g[q] * g[q];
        s0[q] = m;
        s1[q] = v;
        w[q] -= lrt * m / (sqrtf(v) + p.eps);
      }
      break;
    }
    case OPT_ADAGRAD:
      _Pragma("unroll") for (int q = 0; q < NV; ++q) {
        const float a = s0[q] + g[q] * g[q];
        s0[q] = a;
        w[q] -= lr * g[q] / (sqrtf(a) + p.eps);
      }
      break;
    case OPT_ADAMAX: {
      const float lrt = lr / (1.f - powf(p.b1, (float)(iter + 1)));
      _Pragma("unroll") for (int q = 0; q < NV; ++q) {
        const float m = p.b1 * s0[q] + (1.f - p.b1) * g[q];
        const float u = fmaxf(p.b2 * s1[q], fabsf(g[q]));
        s0[q] = m;
        s1[q] = u;
        w[q] -= lrt * m / (u + p.eps);
      }
      break;
    }
  }
}

// ------------------------------------------------------------ step counters
// Uniform reads of launch-invariant device words (step counters, per-replica row
// counts): through the constant address space they are scalar loads (the cache is
// invalidated at every dispatch, as for kernel arguments), issued together at the
// top of the kernel instead of as vector loads, each waited for on its own.
// Only for words nothing in the reading kernel writes.
template <typename T> __device__ __forceinline__ T ld_inv(const T* p) {
  // the address is forced into SGPRs: hipcc otherwise sometimes forms it on the
  // vector ALU (e.g. from a copy of the workgroup id) and emits a vector load
  const unsigned long long u = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return *(const __attribute__((address_space(4))) T*)(((unsigned long long)hi << 32) | lo);
}

// a whole launch-invariant struct, dword by dword (unused words are dropped)
template <typename T> __device__ __forceinline__ T ld_inv_struct(const T* p) {
  static_assert(sizeof(T) % 4 == 0, "dword-sized struct");
  T out;
  const __attribute__((address_space(4))) unsigned* src =
      (const __attribute__((address_space(4))) unsigned*)(unsigned long long)p;
  unsigned* dst = reinterpret_cast<unsigned*>(&out);
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 4); ++i) dst[i] = src[i];
  return out;
}

// see GroupArgs::step_off (args.h)
__device__ __forceinline__ long long iter_at(const long long* ctr, const int* ntrain, int B, int r, long long s0,
                                             int off) {
  const long long nb = ((long long)ld_inv(ntrain + r) + B - 1) / B;
  long long d = nb - s0;
  d = d < 0 ? 0 : (d > off ? off : d);
  return ld_inv(ctr + 2 + r) + d;
}

}  // namespace ea
