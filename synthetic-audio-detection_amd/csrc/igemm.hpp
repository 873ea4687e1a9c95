// igemm.hpp -- device helpers shared by the implicit-GEMM kernels (gfx950).
#pragma once
#include "common.hpp"

namespace sad {

template <typename T>
struct DT;
template <>
struct DT<u16> {
  static constexpr int EPC = 8;  // elements per 16-B chunk
};
template <>
struct DT<float> {
  static constexpr int EPC = 4;
};

__device__ __forceinline__ int swz(int row, int chunk) { return (chunk ^ ((row >> 1) & 7)); }

// Same, M0 declared clobbered instead of saved/restored (2 fewer SALU per DMA;
// hipcc re-materialises M0 where it needs it, which in these kernels is nowhere
// inside the main loop).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16_m0(__amdgpu_buffer_rsrc_t rsrc, int voff, unsigned lds_base) {
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %2, 0 offen lds"
      :
      : "v"(voff), "s"(__builtin_amdgcn_readfirstlane(lds_base)), "s"(rsrc)
      : "memory", "m0");
}
#pragma clang diagnostic pop

// One LDS-DMA wave-instruction: 16 B per lane from buffer offset `voff` to LDS
// [lds_base + 16*lane].  M0 (compiler-reserved) is saved/restored inside the
// statement; offsets past the buffer's num_records load zeros.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, int voff, unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(__builtin_amdgcn_readfirstlane(lds_base)), "s"(rsrc)
      : "memory");
}

template <typename T>
__device__ __forceinline__ void mfma_chunk(const uint4& a, const uint4& b, f32x4& acc);

template <>
__device__ __forceinline__ void mfma_chunk<u16>(const uint4& a, const uint4& b, f32x4& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mfma_chunk<float>(const uint4& a, const uint4& b, f32x4& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}

}  // namespace sad
