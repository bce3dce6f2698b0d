// Device-side helpers shared by the gfx950 kernel translation units.
#pragma once
#include <hip/hip_runtime.h>

namespace vox {

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  return __builtin_bit_cast(bf16x8, u);
}
__device__ __forceinline__ f32x4 ld16(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}

template <typename F> __device__ __forceinline__ F zero_frag() { return F{}; }

// Elementwise helpers on fragments (in fp32).
__device__ __forceinline__ bf16x8 frag_add(bf16x8 a, bf16x8 b) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (bf16_t)((float)a[e] + (float)b[e]);
  return r;
}
__device__ __forceinline__ f32x4 frag_add(f32x4 a, f32x4 b) { return a + b; }

// ReLU on bf16 bit patterns: every negative value (and -0) has the sign bit
// set, i.e. is a negative int16, so a packed int16 max with 0 is ReLU.  bf16
// rounding is monotone and keeps the sign, so relu(bf16(x)) == bf16(relu(x))
// bit for bit; one v_pk_max_i16 per two channels instead of two v_max_f32.
__device__ __forceinline__ bf16x4 relu_bf16(bf16x4 v) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const s16x4 s = __builtin_elementwise_max(__builtin_bit_cast(s16x4, v), (s16x4){0, 0, 0, 0});
  return __builtin_bit_cast(bf16x4, s);
}
__device__ __forceinline__ bf16x8 relu_bf16(bf16x8 v) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 s = __builtin_elementwise_max(__builtin_bit_cast(s16x8, v),
                                            (s16x8){0, 0, 0, 0, 0, 0, 0, 0});
  return __builtin_bit_cast(bf16x8, s);
}

__device__ __forceinline__ f32x4 mfma_step(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

}  // namespace vox
