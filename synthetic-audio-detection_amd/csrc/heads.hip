// heads.hip -- last head layer (Linear 256->2) for N heads + ensemble merge.
//
// Replaces head[10] of BinaryClassifier (inference_runner.py:47) and
// ModularMultiHeadClassifier.forward (inference_runner.py:62-73):
//   logits[b, h, :] = W3_h . y2[b, h*256 : (h+1)*256] + b3_h   ([Real, Synthetic])
//   merged[b, :N]   = logits[b, :, 1];  merged[b, N] = mean_h logits[b, h, 0]
// The two wide head layers (512->512, 512->256, BN1d folded, ReLU) run on the
// f32 MFMA implicit-GEMM kernel as 1x1 "convolutions" (api.hip).
// One wave per segment; a head's 256-term dots are split over the 64 lanes.
#include "common.hpp"
#include "kernels.hpp"

namespace sad {

__global__ __launch_bounds__(256) void heads_final_kernel(const float* __restrict__ y2, int64_t B,
                                                          int n_heads, const float* __restrict__ w3,
                                                          const float* __restrict__ b3,
                                                          float* __restrict__ logits,
                                                          float* __restrict__ merged) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;  // wave-uniform
  const float* y = y2 + b * (int64_t)n_heads * 256;
  float real_sum = 0.f;
  for (int h = 0; h < n_heads; ++h) {
    const float4 yv = *(const float4*)(y + h * 256 + lane * 4);
    const float4 w0 = *(const float4*)(w3 + (h * 2 + 0) * 256 + lane * 4);
    const float4 w1 = *(const float4*)(w3 + (h * 2 + 1) * 256 + lane * 4);
    float s0 = yv.x * w0.x + yv.y * w0.y + yv.z * w0.z + yv.w * w0.w;
    float s1 = yv.x * w1.x + yv.y * w1.y + yv.z * w1.z + yv.w * w1.w;
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o, 64);
      s1 += __shfl_xor(s1, o, 64);
    }
    const float z0 = s0 + b3[h * 2 + 0], z1 = s1 + b3[h * 2 + 1];
    if (lane == 0) {
      if (logits) {
        logits[(b * n_heads + h) * 2 + 0] = z0;
        logits[(b * n_heads + h) * 2 + 1] = z1;
      }
      merged[b * (n_heads + 1) + h] = z1;
    }
    real_sum += z0;
  }
  if (lane == 0) merged[b * (n_heads + 1) + n_heads] = real_sum / (float)n_heads;
}

int launch_heads_final(const float* y2, int64_t B, int n_heads, const float* w3, const float* b3,
                       float* logits, float* merged, hipStream_t s) {
  if (B == 0) return SAD_OK;
  hipLaunchKernelGGL(heads_final_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, y2, B, n_heads,
                     w3, b3, logits, merged);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

}  // namespace sad
