// rwconv.hpp -- helpers of the resident-weight conv kernels (l1block.hip,
// l2conv.hip): weights held in AGPRs for a whole launch, so the MFMAs that read
// them are inline asm (hipcc only places MFMA A/B operands in VGPRs); packed
// bf16 conversion and ReLU; compile-time loops.
#pragma once
#include <utility>

#include "common.hpp"

namespace sad {

typedef unsigned int l1b_v4 __attribute__((ext_vector_type(4)));
typedef unsigned int l1b_v2 __attribute__((ext_vector_type(2)));
// acc (VGPR) [+]= w (AGPR) . b (VGPR).  hipcc places MFMA A/B operands only
// in VGPRs, and the 288 weight registers of both convs do not fit there next
// to the accumulators: the weights live in AGPRs, the MFMA is inline asm.
__device__ __forceinline__ void l1b_mfma_a0(f32x4& acc, const l1b_v4& w, const uint4& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "a"(w), "v"(__builtin_bit_cast(l1b_v4, b)));
}
__device__ __forceinline__ void l1b_mfma_a(f32x4& acc, const l1b_v4& w, const uint4& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(__builtin_bit_cast(l1b_v4, b)));
}
// acc = c + w . b (the first K-step: C = the bias)
__device__ __forceinline__ void l1b_mfma_ac(f32x4& acc, const l1b_v4& w, const uint4& b, const f32x4& c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %3"
               : "=&v"(acc)
               : "a"(w), "v"(__builtin_bit_cast(l1b_v4, b)), "v"(c));
}
// the same with the weights in VGPRs (the AGPR file holds 256 of the 288)
__device__ __forceinline__ void l1b_mfma_v0(f32x4& acc, const l1b_v4& w, const uint4& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(w), "v"(__builtin_bit_cast(l1b_v4, b)));
}
__device__ __forceinline__ void l1b_mfma_v(f32x4& acc, const l1b_v4& w, const uint4& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(w), "v"(__builtin_bit_cast(l1b_v4, b)));
}
// two floats -> packed bf16 pair (RNE), one v_cvt_pk_bf16_f32
typedef __bf16 l1b_bf2 __attribute__((ext_vector_type(2)));
typedef float l1b_f2 __attribute__((ext_vector_type(2)));
// relu of an asm MFMA result (fmaxf would first canonicalise it: one more VALU)
__device__ __forceinline__ float l1b_relu(float x) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
  return r;
}
// ReLU of a packed bf16 pair: as int16, negative bf16 values (and -0) are
// negative, so max(x, 0) per half is relu (= relu before the rounding)
__device__ __forceinline__ uint32_t l1b_relu2(uint32_t x) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t l1b_pk(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((l1b_f2){lo, hi}, l1b_bf2));
}

template <typename F, int... I>
__device__ __forceinline__ void l1b_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void l1b_for(F&& f) {
  l1b_for_impl(f, std::make_integer_sequence<int, N>{});
}


}  // namespace sad
