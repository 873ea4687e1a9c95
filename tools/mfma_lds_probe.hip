// Issue cost of LDS fragment reads between MFMAs at ONE wave per SIMD (the
// resident-weight kernels' regime: l1block.hip, l2conv.hip), all in inline asm
// so no address VALU or compiler waits enter the loop:
//   mode 0: 16 x v_mfma_f32_16x16x32_bf16, no reads
//   mode 1: 16 x 16x16x32, one ds_read_b128 per 2 MFMAs (the kernels' density)
//   mode 2: 16 x 16x16x32, one ds_read_b128 per MFMA
//   mode 3: 8 x v_mfma_f32_32x32x16_bf16, no reads
//   mode 4: 8 x 32x32x16, one ds_read_b128 per MFMA (same bytes per FLOP as 1)
//   mode 5: 8 x 32x32x16, two ds_read_b128 per MFMA
//   mode 6: 16 x 16x16x32 + one buffer_load_dwordx4 ... lds (a 1-KB DMA piece) per 16 MFMAs
// Reads use fixed address registers + immediate offsets (conflict-free
// image) and land in registers no MFMA reads, with up to 4 (6) in flight
// (counted lgkmcnt): the pure issue cost.  Prints cycles (s_memtime) per MFMA.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_lds_probe.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned int v4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256, 1) void probe(float* out, unsigned long long* cyc, int iters,
                                                 const float* src) {
  __shared__ __attribute__((aligned(16))) char sm[65536];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16384; i += 256) ((float*)sm)[i] = 1e-3f * (float)(i & 255);
  __syncthreads();
  v4 w = {0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u};
  v4 b0 = {0x3c003c00u, 0x3c003c00u, 0x3c003c00u, 0x3c003c00u}, b1 = b0, b2 = b0, b3 = b0;
  f4 a0 = {}, a1 = {}, a2 = {}, a3 = {};
  f16v c0 = {}, c1 = {};
  const unsigned ad = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)sm + lane * 16;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, 1 << 20, 0x00020000);
  const unsigned lds_dma = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)sm + 32768;
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0 || MODE == 1 || MODE == 2 || MODE == 6) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        // reads land in b1 / b2 (never consumed: pure issue cost with up to 4 in flight)
        if constexpr (MODE == 1) {
          if ((k & 1) == 0) {
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(b1) : "v"(ad), "i"((k & 7) * 1024));
            asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
          }
        }
        if constexpr (MODE == 2) {
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(b1) : "v"(ad), "i"((k & 7) * 1024));
          asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
        }
        if constexpr (MODE == 6) {
          if (k == 0)
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(
                             __builtin_amdgcn_readfirstlane(lds_dma)),
                         "v"(lane * 16), "s"(rs)
                         : "memory", "m0");
        }
        if (k & 1)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(a1) : "v"(w), "v"(b0));
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(a0) : "v"(w), "v"(b0));
      }
      if constexpr (MODE == 6) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if constexpr (MODE == 4 || MODE == 5) {
          asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(b1) : "v"(ad), "i"((k & 7) * 1024));
          if constexpr (MODE == 5)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(b2) : "v"(ad), "i"((k & 7) * 1024 + 16384));
          asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(MODE == 5 ? 6 : 4) : "memory");
        }
        if (k & 1)
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c1) : "v"(w), "v"(b0));
        else
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c0) : "v"(w), "v"(b0));
      }
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)\n\ts_nop 15" ::: "memory");
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (lane == 0 && (threadIdx.x >> 6) == 0) cyc[blockIdx.x] = t1 - t0;
  float s = a0[0] + a1[1] + a2[2] + a3[3] + c0[0] + c1[5] + (float)b1[0] + (float)b2[0] + (float)b3[1];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  float *out, *src;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&src, 1 << 20);
  hipMemset(src, 0, 1 << 20);
  hipMalloc(&cyc, 256 * 8);
  const int iters = 4000;
  const char* what[7] = {"16x16x32, no reads", "16x16x32, 1 read / 2 MFMA", "16x16x32, 1 read / MFMA",
                         "32x32x16, no reads", "32x32x16, 1 read / MFMA", "32x32x16, 2 reads / MFMA",
                         "16x16x32, 1 DMA piece / 16 MFMA"};
  for (int rep = 0; rep < 2; ++rep)
    for (int m = 0; m < 7; ++m) {
      switch (m) {
        case 0: hipLaunchKernelGGL(probe<0>, dim3(256), dim3(256), 0, 0, out, cyc, iters, src); break;
        case 1: hipLaunchKernelGGL(probe<1>, dim3(256), dim3(256), 0, 0, out, cyc, iters, src); break;
        case 2: hipLaunchKernelGGL(probe<2>, dim3(256), dim3(256), 0, 0, out, cyc, iters, src); break;
        case 3: hipLaunchKernelGGL(probe<3>, dim3(256), dim3(256), 0, 0, out, cyc, iters, src); break;
        case 4: hipLaunchKernelGGL(probe<4>, dim3(256), dim3(256), 0, 0, out, cyc, iters, src); break;
        case 5: hipLaunchKernelGGL(probe<5>, dim3(256), dim3(256), 0, 0, out, cyc, iters, src); break;
        case 6: hipLaunchKernelGGL(probe<6>, dim3(256), dim3(256), 0, 0, out, cyc, iters, src); break;
      }
      hipDeviceSynchronize();
      unsigned long long h[256];
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double s = 0;
      for (int i = 0; i < 256; ++i) s += (double)h[i];
      const double n_mfma = (double)iters * (m >= 3 && m <= 5 ? 8 : 16);
      const double per16 = s / 256 / n_mfma / (m >= 3 && m <= 5 ? 2.0 : 1.0);  // per 16x16x32-equivalent
      if (rep == 1) printf("mode %d (%s): %.2f cycles per MFMA, %.2f per 16x16x32-equivalent\n", m, what[m],
                           s / 256 / n_mfma, per16);
    }
  return 0;
}
