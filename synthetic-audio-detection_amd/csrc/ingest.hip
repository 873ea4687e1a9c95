// ingest.hip -- the ingestion edge of the inference path on the device
// (SURVEY 8(f) row 1): a long file's PCM goes to HBM once, compact (int16 as
// it sits in the WAV), and everything from there on runs on the GPU:
//
//   interleaved PCM -> fp32 mono (+ zero pad)        sad_pcm_mono_run
//     preprocess_waveform, inference_runner.py:144-155 (torchaudio.load
//     normalize=True scaling, waveform.mean(dim=0), the pad to one window)
//   -> 32 kHz, torchaudio sinc_interp_hann           sad_resample_run
//     torchaudio.transforms.Resample(sr, 32000) at inference_runner.py:148
//     (lowpass_filter_width 6, rolloff 0.99; the polyphase kernel table is
//     built on the host in float64 and rounded once to fp32, as torchaudio does)
//   -> per-window max |x| for the silence skip       sad_window_absmax_run
//     slice_waveform, inference_runner.py:176-190 (piece.abs().max() < thr)
//   -> the front end reads the kept windows in place by sample offset
//     (sad_frontend_run_windows, frontend.hip): overlapping windows are never
//     copied, and nothing goes back to the host but one float per window.
//
// The mono / window kernels are HBM streaming work; the resampler is fp32-FMA
// work (K = 2 width + orig taps per output, 459 for 44.1 kHz): register-blocked
// over frames with the inputs staged in LDS (resample_wide_kernel).  No MFMA:
// a polyphase FIR is not GEMM-shaped enough to pay for one at fp32.
#include <math.h>

#include <vector>

#include "common.hpp"

namespace sad {

// ---- interleaved PCM [frames][channels] -> mono fp32 [out_len] -------------
// out[i] = (sum_c x[i][c]) / C for i < frames, 0 for frames <= i < out_len.
// The reference's waveform.mean(dim=0) runs on the CPU, where ATen's mean is
// sum(dim).div_(C): channels summed in order, then a true fp32 division (not a
// multiply by 1/C, which differs by an ulp for C = 3, 5, 6, ...); int16 is
// scaled by 1/32768 first (torchaudio.load normalize=True).  Bit-exact with
// the host for every channel count.
template <typename IT>
__global__ __launch_bounds__(256) void pcm_mono_kernel(const IT* __restrict__ x, int64_t frames, int channels,
                                                       float fc, float* __restrict__ out, int64_t out_len) {
  const float scale = sizeof(IT) == 2 ? (1.0f / 32768.0f) : 1.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < out_len;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (i < frames) {
      const IT* p = x + i * channels;
      float s = (float)p[0] * scale;
      for (int c = 1; c < channels; ++c) s += (float)p[c] * scale;
      v = channels == 1 ? s : s / fc;
    }
    out[i] = v;
  }
}

// ---- polyphase windowed-sinc resampler --------------------------------------
// torchaudio.functional.resample with orig/new reduced by their gcd:
//   xp = pad(x, (width, width + orig));  y = conv1d(xp, kernel[new][K], stride orig)
// so output m = j*new + p is  sum_k x[j*orig + k - width] * kernel[p][k]
// (x = 0 outside [0, n_in)), truncated to ceil(new * n_in / orig) samples.
// The table is stored transposed, kt[k][p], so the lanes of a wave (consecutive
// p of one j) read consecutive words, and x[j*orig + k - width] is one
// broadcast address per j.
__global__ __launch_bounds__(256) void resample_kernel(const float* __restrict__ x, int64_t n_in,
                                                       const float* __restrict__ kt, int orig, int nw, int width,
                                                       int K, float* __restrict__ y, int64_t n_out, int64_t y_len) {
  for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < y_len; m += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
    if (m < n_out) {
      const int64_t j = m / nw;
      const int p = (int)(m - j * nw);
      const int64_t base = j * orig - width;  // x index of tap k = 0
      const int k0 = base < 0 ? (int)-base : 0;
      const int64_t kend = n_in - base;
      const int k1 = kend < K ? (int)kend : K;
      const float* xp = x + base;
      const float* kp = kt + p;
      for (int k = k0; k < k1; ++k) acc = fmaf(xp[k], kp[(int64_t)k * nw], acc);
    }
    y[m] = acc;
  }
}

// Many phases (nw >= 64: 44.1 / 22.05 kHz -> 32 kHz, nw = 320 / 640, K = 459 /
// 455): lanes own 64 consecutive phases p, a wave owns RS_R consecutive frames
// j (RS_R accumulators per lane), and K is walked in chunks of RS_KC taps: the
// chunk's input samples for the wave's frames are staged in LDS as xs[k][r]
// (frame-fastest, so one tap's RS_R inputs are 4 broadcast ds_read_b128), the
// tap's coefficient kt[k][p] is one coalesced load (the table stays in L2), and
// each tap costs RS_R FMAs per lane.  The sum runs over k in the same order as
// resample_kernel, so the two give identical results.
constexpr int RS_R = 16, RS_KC = 64, RS_WAVES = 4;
__global__ __launch_bounds__(256) void resample_wide_kernel(const float* __restrict__ x, int64_t n_in,
                                                            const float* __restrict__ kt, int orig, int nw, int width,
                                                            int K, float* __restrict__ y, int64_t n_out) {
  __shared__ __attribute__((aligned(16))) float xs[RS_WAVES][RS_KC][RS_R];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int p = blockIdx.y * 64 + lane;
  const bool pok = p < nw;
  const int64_t j0 = ((int64_t)blockIdx.x * RS_WAVES + wave) * RS_R;  // this wave's first frame
  float acc[RS_R];
#pragma unroll
  for (int r = 0; r < RS_R; ++r) acc[r] = 0.f;
  for (int kc = 0; kc < K; kc += RS_KC) {
    __syncthreads();  // the previous chunk's reads are done
#pragma unroll 4
    for (int e = lane; e < RS_KC * RS_R; e += 64) {
      const int r = e % RS_R, k = e / RS_R;
      const int64_t i = (j0 + r) * orig + kc + k - width;
      xs[wave][k][r] = (kc + k < K && i >= 0 && i < n_in) ? x[i] : 0.f;
    }
    __syncthreads();
    const int kn = K - kc < RS_KC ? K - kc : RS_KC;
    const float* kp = kt + (int64_t)kc * nw + p;
#pragma unroll 4
    for (int k = 0; k < kn; ++k) {
      const float w = pok ? kp[(int64_t)k * nw] : 0.f;
      const float4* xr = (const float4*)&xs[wave][k][0];
#pragma unroll
      for (int q = 0; q < RS_R / 4; ++q) {
        const float4 v = xr[q];
        acc[4 * q + 0] = fmaf(v.x, w, acc[4 * q + 0]);
        acc[4 * q + 1] = fmaf(v.y, w, acc[4 * q + 1]);
        acc[4 * q + 2] = fmaf(v.z, w, acc[4 * q + 2]);
        acc[4 * q + 3] = fmaf(v.w, w, acc[4 * q + 3]);
      }
    }
  }
  if (pok) {
#pragma unroll
    for (int r = 0; r < RS_R; ++r) {
      const int64_t m = (j0 + r) * nw + p;
      if (m < n_out) y[m] = acc[r];
    }
  }
}

// ---- max |x| over each window [w*hop, w*hop + window) -------------------------
// torch.max propagates NaN, so a NaN sample makes the window's maximum NaN
// (and `NaN < thr` keeps the window, as in the reference)
__device__ __forceinline__ float nanmax(float a, float b) { return (b > a || b != b) ? b : a; }

__global__ __launch_bounds__(256) void window_absmax_kernel(const float* __restrict__ x, int64_t n, int64_t window,
                                                            int64_t hop, float* __restrict__ out) {
  __shared__ float red[4];
  const int64_t w = blockIdx.x;
  const int64_t b = w * hop;
  const int64_t e = b + window < n ? b + window : n;
  float m = 0.f;  // |x| >= 0: 0 is the identity (an empty window reports 0)
  for (int64_t i = b + threadIdx.x; i < e; i += blockDim.x) m = nanmax(m, fabsf(x[i]));
  for (int o = 32; o > 0; o >>= 1) m = nanmax(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[w] = nanmax(nanmax(red[0], red[1]), nanmax(red[2], red[3]));
}

static unsigned grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

}  // namespace sad

using namespace sad;

struct sad_resample_plan {
  int32_t orig_freq = 0, new_freq = 0;
  int orig = 1, nw = 1, width = 0, K = 0;  // reduced by the gcd
  float* d_kt = nullptr;                    // [K][nw] fp32
  int device = 0;
};

static int64_t gcd64(int64_t a, int64_t b) {
  while (b) {
    const int64_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}

extern "C" int sad_pcm_mono_run(const void* pcm, int32_t format, int64_t frames, int32_t channels, float* out,
                                int64_t out_len, void* stream) {
  SAD_REQUIRE(format == SAD_PCM_I16 || format == SAD_PCM_F32, "format must be SAD_PCM_I16 or SAD_PCM_F32");
  SAD_REQUIRE(frames >= 0 && channels >= 1 && channels <= 64, "frames / channels");
  SAD_REQUIRE(out_len >= frames, "out_len < frames");
  if (out_len == 0) return SAD_OK;
  SAD_REQUIRE(out && (pcm || frames == 0), "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const float fc = (float)channels;
  if (format == SAD_PCM_I16)
    hipLaunchKernelGGL(pcm_mono_kernel<int16_t>, dim3(grid_for(out_len)), dim3(256), 0, s, (const int16_t*)pcm,
                       frames, channels, fc, out, out_len);
  else
    hipLaunchKernelGGL(pcm_mono_kernel<float>, dim3(grid_for(out_len)), dim3(256), 0, s, (const float*)pcm, frames,
                       channels, fc, out, out_len);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_resample_plan_create(int32_t orig_freq, int32_t new_freq, sad_resample_plan** out) {
  SAD_REQUIRE(out, "null out");
  SAD_REQUIRE(orig_freq > 0 && new_freq > 0, "sample rates must be positive");
  const int64_t g = gcd64(orig_freq, new_freq);
  const int orig = (int)(orig_freq / g), nw = (int)(new_freq / g);
  // torchaudio _get_sinc_resample_kernel (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99), float64
  const int lpw = 6;
  const double rolloff = 0.99;
  const double base = (double)(orig < nw ? orig : nw) * rolloff;
  const int width = (int)ceil(lpw * (double)orig / base);
  const int K = 2 * width + orig;
  SAD_REQUIRE((int64_t)K * nw * 4 <= (256ll << 20),
              "resample ratio too irregular: the polyphase table would exceed 256 MiB");
  std::vector<float> kt((size_t)K * nw);
  const double scale = base / orig;
  for (int p = 0; p < nw; ++p) {
    for (int k = 0; k < K; ++k) {
      // idx = arange(-width, width + orig, float64) / orig; t = arange(0, -new, -1) / new + idx, where
      // the integer arange / new is a default-dtype (fp32) division, promoted to float64 by the add
      const float ph = (float)(-p) / (float)nw;
      double t = ((double)ph + (double)(k - width) / orig) * base;
      t = t < -lpw ? -lpw : (t > lpw ? lpw : t);
      const double c = cos(t * M_PI / lpw / 2);
      const double window = c * c;
      t *= M_PI;
      const double v = (t == 0.0 ? 1.0 : sin(t) / t) * (window * scale);  // kernels *= window * scale
      kt[(size_t)k * nw + p] = (float)v;
    }
  }
  auto* pl = new sad_resample_plan();
  pl->orig_freq = orig_freq;
  pl->new_freq = new_freq;
  pl->orig = orig;
  pl->nw = nw;
  pl->width = width;
  pl->K = K;
  (void)hipGetDevice(&pl->device);
  if (hipMalloc((void**)&pl->d_kt, kt.size() * 4) != hipSuccess ||
      hipMemcpy(pl->d_kt, kt.data(), kt.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(pl->d_kt);
    delete pl;
    set_error("sad_resample_plan_create: device allocation / upload failed");
    return SAD_ERR_NOMEM;
  }
  *out = pl;
  return SAD_OK;
}

extern "C" int sad_resample_plan_destroy(sad_resample_plan* p) {
  if (!p) return SAD_OK;
  (void)hipFree(p->d_kt);
  delete p;
  return SAD_OK;
}

extern "C" int sad_resample_out_len(const sad_resample_plan* p, int64_t n_in, int64_t* n_out) {
  SAD_REQUIRE(p && n_out && n_in >= 0, "null plan / n_out, or n_in < 0");
  SAD_REQUIRE(n_in <= (INT64_MAX - p->orig) / p->nw, "n_in too large");
  *n_out = (p->nw * n_in + p->orig - 1) / p->orig;  // ceil(new * length / orig)
  return SAD_OK;
}

extern "C" int sad_resample_run(const sad_resample_plan* p, const float* x, int64_t n_in, float* y, int64_t y_len,
                                void* stream) {
  int64_t n_out = 0;
  if (int rc = sad_resample_out_len(p, n_in, &n_out)) return rc;
  SAD_REQUIRE(y_len >= n_out, "y_len < the resampled length (sad_resample_out_len)");
  if (y_len == 0) return SAD_OK;
  SAD_REQUIRE(y && (x || n_in == 0), "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (p->nw >= 64 && n_out > 0) {
    const int64_t frames = (n_out + p->nw - 1) / p->nw;
    const int64_t gx = (frames + RS_WAVES * RS_R - 1) / (RS_WAVES * RS_R);
    SAD_REQUIRE(gx < (1ll << 31), "input too long for one launch");
    hipLaunchKernelGGL(resample_wide_kernel, dim3((unsigned)gx, (unsigned)((p->nw + 63) / 64)), dim3(256), 0, s, x,
                       n_in, p->d_kt, p->orig, p->nw, p->width, p->K, y, n_out);
    SAD_CHECK_HIP(hipGetLastError());
    if (y_len > n_out) SAD_CHECK_HIP(hipMemsetAsync(y + n_out, 0, (size_t)(y_len - n_out) * 4, s));
    return SAD_OK;
  }
  hipLaunchKernelGGL(resample_kernel, dim3(grid_for(y_len)), dim3(256), 0, s, x, n_in, p->d_kt, p->orig, p->nw,
                     p->width, p->K, y, n_out, y_len);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_window_absmax_run(const float* wav, int64_t n, int64_t window, int64_t hop, int64_t n_windows,
                                     float* out, void* stream) {
  SAD_REQUIRE(n >= 0 && window > 0 && hop > 0 && n_windows >= 0, "n / window / hop / n_windows");
  SAD_REQUIRE(n_windows == 0 || (n_windows - 1) * hop < n, "window start past the end of the waveform");
  SAD_REQUIRE(n_windows <= 0x7FFFFFFF, "too many windows for one launch");
  if (n_windows == 0) return SAD_OK;
  SAD_REQUIRE(wav && out, "null pointer");
  hipLaunchKernelGGL(window_absmax_kernel, dim3((unsigned)n_windows), dim3(256), 0, (hipStream_t)stream, wav, n,
                     window, hop, out);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}
