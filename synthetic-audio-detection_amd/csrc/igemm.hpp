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

// Sum over the 16 lanes of a DPP row (all 16 receive the total).
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true));  // row_ror:8
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, true));  // row_ror:4
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));   // quad [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));   // quad [1,0,3,2]
  return v;
}

// Training BatchNorm statistics fused into a conv epilogue (the trainer's
// train-mode convs, submodel_trainer.py:250-255): lane (fr, fg) holds channels
// i*16 + fg*4 + r (i < TC, r < 4) of pixel fr.  Per tile, the lane's sums of v
// and v^2 over its pixels are reduced across the 16 fr lanes, and value
// m = (i*4 + r)*2 + {0: sum, 1: sum of squares} is parked in register m / 16 of
// lane m % 16 -- TC/2 registers per lane instead of 8*TC.
template <int TC>
struct StatAcc {
  static_assert(TC % 2 == 0, "fused BN statistics need an even channel-fragment count");
  float r[TC / 2];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < TC / 2; ++k) r[k] = 0.f;
  }
  __device__ __forceinline__ void add(int i, int rr, float s, float q, int fr) {
    s = row16_sum(s);
    q = row16_sum(q);
    const int m = (i * 4 + rr) * 2;
    r[m >> 4] += fr == (m & 15) ? s : 0.f;
    r[(m + 1) >> 4] += fr == ((m + 1) & 15) ? q : 0.f;
  }
  // s_red[slot][2][bc] (floats) <- this lane's parked values; cbase = the
  // wave's first channel within the bc-wide tile
  __device__ __forceinline__ void park(float* s_red, int slot, int bc, int cbase, int fr, int fg) const {
#pragma unroll
    for (int k = 0; k < TC / 2; ++k) {
      const int m = 16 * k + fr, i = m >> 3, rr = (m >> 1) & 3, sq = m & 1;
      s_red[(slot * 2 + sq) * bc + cbase + i * 16 + fg * 4 + rr] = r[k];
    }
  }
};

// Same statistics with full per-lane sums (8*TC registers) and the cross-lane
// reduction deferred to the end of the kernel: for kernels with registers to
// spare, whose epilogue sits on the critical path (the halo kernels).
template <int TC>
struct StatLane {
  float s[TC][4], q[TC][4];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[i][r] = q[i][r] = 0.f;
  }
  __device__ __forceinline__ void add(int i, int r, float v) {
    s[i][r] += v;
    q[i][r] += v * v;
  }
  // reduce over the 16 fr lanes and store: s_red[slot][2][bc]
  __device__ __forceinline__ void park(float* s_red, int slot, int bc, int cbase, int fr, int fg) {
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float a = row16_sum(s[i][r]), b = row16_sum(q[i][r]);
        if (fr == 0) {
          s_red[(slot * 2 + 0) * bc + cbase + i * 16 + fg * 4 + r] = a;
          s_red[(slot * 2 + 1) * bc + cbase + i * 16 + fg * 4 + r] = b;
        }
      }
  }
};

// part[row][2][C] at channels c0 .. c0+bc <- sum over nslot of s_red[slot][2][bc]
__device__ __forceinline__ void stat_rows_write(const float* s_red, int nslot, int bc, float* part, int row, int C,
                                                int c0, int tid, int nt) {
  for (int c = tid; c < 2 * bc; c += nt) {
    float v = 0.f;
    for (int sl = 0; sl < nslot; ++sl) v += s_red[sl * 2 * bc + c];
    part[((int64_t)row * 2 + c / bc) * C + c0 + c % bc] = v;
  }
}
__device__ __forceinline__ void stat_rows_zero(int bc, float* part, int row, int C, int c0, int tid, int nt) {
  for (int c = tid; c < 2 * bc; c += nt) part[((int64_t)row * 2 + c / bc) * C + c0 + c % bc] = 0.f;
}

}  // namespace sad
