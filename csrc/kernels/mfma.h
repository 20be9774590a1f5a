// MFMA fragment helpers shared by the grouped GEMM and the fused MLP kernels.
//
// 16x16 output tiles; per lane: A/B fragment = 16 bytes of one row (A) or one
// column (B^T row) at k = (lane >> 4) * EPL .. +EPL, C/D = 4 floats at
// row (lane >> 4) * 4 + q, col lane & 15.
//   bf16: v_mfma_f32_16x16x32_bf16, EPL 8, KC (k per step) 32
//   f32 : 4x v_mfma_f32_16x16x4f32,  EPL 4, KC 16 (lane group g holds k = 4g..4g+3;
//         MFMA t consumes element t, so each MFMA covers a strided k subset and the
//         four together cover the 16-deep chunk)
#pragma once
#include "common.h"

namespace ea {

template <typename T> struct KT;
template <> struct KT<__bf16> { static constexpr int EPL = 8, KC = 32; };
template <> struct KT<float> { static constexpr int EPL = 4, KC = 16; };

template <typename T>
__device__ __forceinline__ void mma16(f32x4& acc, const uint4& a, const uint4& b) {
  if constexpr (sizeof(T) == 2) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  } else {
    // lane group g holds k = 4g..4g+3 of this 16-deep chunk; MFMA t consumes element t.
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
}

template <typename T> __device__ __forceinline__ uint4 ones_frag() {
  if constexpr (sizeof(T) == 2) {
    const unsigned o = 0x3F803F80u;  // two bf16 1.0
    return make_uint4(o, o, o, o);
  } else {
    const unsigned o = 0x3F800000u;
    return make_uint4(o, o, o, o);
  }
}


}  // namespace ea
