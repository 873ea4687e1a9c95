// common.hpp -- shared helpers for libsad (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <string>

#include "../../include/sad.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

namespace sad {

// thread-local last error (sad_last_error)
void set_error(const std::string& msg);

#define SAD_CHECK_HIP(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      ::sad::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));         \
      return SAD_ERR_HIP;                                                          \
    }                                                                              \
  } while (0)

#define SAD_REQUIRE(cond, msg)                                                     \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      ::sad::set_error(std::string("argument check failed: ") + (msg));            \
      return SAD_ERR_ARG;                                                          \
    }                                                                              \
  } while (0)

// host fp32 -> bf16 round-to-nearest-even (no NaN inputs on this path)
inline u16 f2bf_host(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (u16)(u >> 16);
}

__device__ __forceinline__ u16 f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32, RNE
  return __builtin_bit_cast(u16, b);
}
__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float(((uint32_t)h) << 16); }

// Bijective XCD-aware block remap (cdna_hip_programming.md 5, T1): consecutive
// logical tiles land on the same XCD (blocks b, b+8, ... share one).
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

}  // namespace sad
