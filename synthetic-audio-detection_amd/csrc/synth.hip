// synth.hip -- on-device deterministic synthetic PCM.
// Same counter-based hash as sad/synth.py so a 1 M-segment shard is generated
// in HBM without a host round trip.  One thread per sample.
#include <math.h>

#include "common.hpp"

namespace sad {

constexpr uint64_t GOLD = 0x9E3779B97F4A7C15ull;
constexpr uint64_t GOLD2 = 0xD1B54A32D192ED03ull;

__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void synth_kernel(uint64_t seed, int64_t first_seg, int n, int16_t* __restrict__ pcm) {
  const int64_t seg = first_seg + blockIdx.y;
  const uint64_t key = mix64(mix64(seed) + (uint64_t)seg * GOLD);
  __shared__ double s_tone[3][3];
  __shared__ int s_k;
  if (threadIdx.x == 0) {
    const uint64_t hs = mix64(key ^ 0x5EED5EED5EED5EEDull);
    const int k = 1 + (int)(hs % 3);
    s_k = k;
    for (int i = 0; i < k; ++i) {
      const uint64_t hi = mix64(hs + (uint64_t)(i + 1) * GOLD2);
      s_tone[i][0] = 100.0 + ((double)(hi & 0xFFFF) / 65536.0) * 10900.0;
      s_tone[i][1] = (0.05 + ((double)((hi >> 16) & 0xFFFF) / 65536.0) * 0.25) * 32767.0;
      s_tone[i][2] = ((double)((hi >> 32) & 0xFFFF) / 65536.0) * 2.0 * M_PI;
    }
  }
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t r = mix64(key + (uint64_t)(j + 1) * GOLD2);
  const int64_t s4 = (int64_t)(r & 0xFFFF) + (int64_t)((r >> 16) & 0xFFFF) + (int64_t)((r >> 32) & 0xFFFF) +
                     (int64_t)((r >> 48) & 0xFFFF) - 131070;
  const int64_t num = s4 * 5675;
  const int64_t noise = num >= 0 ? (num >> 16) : -((-num + 65535) >> 16);  // floor division
  double tone = 0.0;
  for (int i = 0; i < s_k; ++i) {
    const double w = 2.0 * M_PI * s_tone[i][0] / 32000.0;
    tone += s_tone[i][1] * sin(w * (double)j + s_tone[i][2]);
  }
  int64_t x = noise + (int64_t)rint(tone);
  x = x < -32768 ? -32768 : (x > 32767 ? 32767 : x);
  pcm[(int64_t)blockIdx.y * n + j] = (int16_t)x;
}

}  // namespace sad

extern "C" int sad_synth_pcm(uint64_t seed, int64_t first_seg, int64_t count, int32_t n_samples,
                             int16_t* pcm, void* stream) {
  SAD_REQUIRE(n_samples > 0 && count >= 0, "bad sizes");
  int64_t done = 0;
  while (done < count) {
    const int64_t chunk = std::min<int64_t>(65535, count - done);
    hipLaunchKernelGGL(sad::synth_kernel, dim3((n_samples + 255) / 256, (unsigned)chunk), dim3(256), 0,
                       (hipStream_t)stream, seed, first_seg + done, n_samples, pcm + done * n_samples);
    SAD_CHECK_HIP(hipGetLastError());
    done += chunk;
  }
  return SAD_OK;
}
