// train.hip -- training-mode kernels for the submodel_trainer.py hot path
//  on gfx950.
//
// The reference trains a timm ResNet-18 with model.train() (every BatchNorm2d
// normalises with BATCH statistics and updates its running stats, momentum 0.1)
// on pooled features fed to CrossEntropyLoss (quirk C1), back-propagates into
// layer4 (and, from epoch epochs//3, layer3: quirk C4), clips the gradient norm
// to 0.5 and steps AdamW (submodel_trainer.py:241-302,606-660).  Inference
// folds BN into the convs; training cannot, so a train-mode conv is
//   raw conv (conv_igemm_kernel, bias 0)  ->  bn_stats  ->  bn_apply(+res, ReLU)
// and the backward pass is
//   bn_backward (reduce + finalize + apply)  ->  dgrad (the forward conv kernels
//   on flipped, transposed weights; stride 2: a pixel-axis GEMM + col2im)  ->
//   wgrad (the pixel-axis GEMM, wgrad.hip).
//
// Kernels here are HBM-bound elementwise / reduction passes over NHWC
// activations (8 channels = 16 B (bf16) per thread, coalesced); the dense
// contractions are hand-written MFMA kernels: the conv kernels (conv.hip,
// block.hip, halo.hip) and kouter_bf16_kernel (wgrad.hip) for the weight
// gradient and the stride-2 input gradient.  No BLAS library is linked.
#include <math.h>

#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace sad {

// ------------------------------------------------------------ load/store --
template <typename T>
__device__ __forceinline__ void load8(const T* p, float v[8]);
template <>
__device__ __forceinline__ void load8<float>(const float* p, float v[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <>
__device__ __forceinline__ void load8<u16>(const u16* p, float v[8]) {
  const uint4 q = *(const uint4*)p;
  const u16* h = (const u16*)&q;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(h[e]);
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float v[8]);
template <>
__device__ __forceinline__ void store8<float>(float* p, const float v[8]) {
  *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
  *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
template <>
__device__ __forceinline__ void store8<u16>(u16* p, const float v[8]) {
  uint4 q;
  u16* h = (u16*)&q;
#pragma unroll
  for (int e = 0; e < 8; ++e) h[e] = f2bf(v[e]);
  *(uint4*)p = q;
}
template <typename T>
__device__ __forceinline__ float ld1(const T* p) {
  if constexpr (sizeof(T) == 2)
    return bf2f(*(const u16*)p);
  else
    return *p;
}
template <typename T>
__device__ __forceinline__ void st1(T* p, float v) {
  if constexpr (sizeof(T) == 2)
    *(u16*)p = f2bf(v);
  else
    *p = v;
}

__device__ double block_sum_d1024(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

// ------------------------------------------------------------ front end --
// SpecAugment + per-spectrogram standardisation (submodel_trainer.py:107-114,
// 195-199): torchaudio FrequencyMasking / TimeMasking fill [f0,f1) rows and
// [t0,t1) columns of the (top-db clamped) dB map with 0.0, then
// (x - mean) / (std_unbiased + 1e-6).  One workgroup per segment; float64 sums.
__global__ __launch_bounds__(1024) void specaug_norm_kernel(const float* __restrict__ db, int n_mels, int n_frames,
                                                           const int* __restrict__ masks, float* __restrict__ out) {
  __shared__ double red[16];
  const int64_t seg = blockIdx.x;
  const int count = n_mels * n_frames;
  const float* x = db + seg * count;
  float* y = out + seg * count;
  int f0 = 0, f1 = 0, t0 = 0, t1 = 0;
  if (masks) {
    f0 = masks[seg * 4 + 0];
    f1 = masks[seg * 4 + 1];
    t0 = masks[seg * 4 + 2];
    t1 = masks[seg * 4 + 3];
  }
  auto val = [&](int i) {
    const int m = i / n_frames, t = i - m * n_frames;
    return ((m >= f0 && m < f1) || (t >= t0 && t < t1)) ? 0.f : x[i];
  };
  double s = 0.0;
  for (int i = threadIdx.x; i < count; i += blockDim.x) s += (double)val(i);
  const double mean = block_sum_d1024(s, red) / count;
  double ss = 0.0;
  for (int i = threadIdx.x; i < count; i += blockDim.x) {
    const double d = (double)val(i) - mean;
    ss += d * d;
  }
  const double var = block_sum_d1024(ss, red) / (count - 1);
  const float mean_f = (float)mean, denom = (float)sqrt(var) + 1e-6f;
  for (int i = threadIdx.x; i < count; i += blockDim.x) y[i] = (val(i) - mean_f) / denom;
}

// torchvision bilinear sample (align_corners=False, source index clamped at 0;
// the antialias filter reduces to this for upsampling) of an ih x iw plane at
// output pixel o of an `on`-long axis: (i0, i1, weight of i1).
__device__ __forceinline__ void bl_axis(int o, int in, int on, int& i0, int& i1, float& l) {
  const float sc = (float)in / on;
  float f = sc * (o + 0.5f) - 0.5f;
  f = f < 0.f ? 0.f : f;
  i0 = min((int)floorf(f), in - 1);
  i1 = min(i0 + 1, in - 1);
  l = fminf(fmaxf(f - i0, 0.f), 1.f);
}

// Resize((512,512)) of the standardised map (submodel_trainer.py:200), then the
// train transform RandomResizedCrop(512, scale=(0.8,1)) = resized_crop(i,j,h,w)
// back to out x out (:466), composed exactly: each output pixel interpolates 4
// crop pixels, each of which interpolates 4 map pixels.  The reference's 3
// identical channels (:203) are one plane here.
// One workgroup per output row: the row's two crop rows (bi + cy0, bi + cy1)
// are evaluated once over the box's columns into LDS (each 512-image pixel =
// 4 map gathers), then every output pixel is one 2x2 lerp from LDS -- half the
// gathers of the per-pixel form and no repeated bl_axis work.
template <typename OT>
__global__ __launch_bounds__(256) void crop_resize_kernel(const float* __restrict__ map, int mh, int mw,
                                                          const int* __restrict__ boxes, int out_hw,
                                                          OT* __restrict__ img) {
  constexpr int R = 512;  // the reference's Resize((512,512))
  __shared__ float rows[2][R];
  const int oy = blockIdx.x;
  const int64_t n = blockIdx.y;
  int bi = 0, bj = 0, bh = R, bw = R;
  if (boxes) {
    bi = boxes[n * 4 + 0];
    bj = boxes[n * 4 + 1];
    bh = boxes[n * 4 + 2];
    bw = min(boxes[n * 4 + 3], R);  // a valid box lies inside the 512 x 512 image
  }
  const float* p = map + n * mh * mw;
  int cy0, cy1;
  float ly;
  bl_axis(oy, bh, out_hw, cy0, cy1, ly);
  // crop columns [0, bw) of crop rows cy0, cy1 (bw <= 512)
  for (int e = threadIdx.x; e < 2 * bw; e += blockDim.x) {
    const int r = e >= bw, cx = e - r * bw;
    const int iy = bi + (r ? cy1 : cy0), ix = bj + cx;
    int y0, y1, x0, x1;
    float a, b;
    bl_axis(iy, mh, R, y0, y1, a);
    bl_axis(ix, mw, R, x0, x1, b);
    rows[r][cx] = (1.f - a) * ((1.f - b) * p[y0 * mw + x0] + b * p[y0 * mw + x1]) +
                  a * ((1.f - b) * p[y1 * mw + x0] + b * p[y1 * mw + x1]);
  }
  __syncthreads();
  OT* o = img + ((int64_t)n * out_hw + oy) * out_hw;
  for (int ox = threadIdx.x; ox < out_hw; ox += blockDim.x) {
    int cx0, cx1;
    float lx;
    bl_axis(ox, bw, out_hw, cx0, cx1, lx);
    const float v00 = rows[0][cx0], v01 = rows[0][cx1], v10 = rows[1][cx0], v11 = rows[1][cx1];
    st1(o + ox, (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11));
  }
}

// conv1 7x7/2/p3 of the one-plane image as im2col rows: col[p][k] for
// k = ky*7+kx < 49, 0 for k in [49, 64).  Thread = one pixel x 8 k.
template <typename T>
__global__ void stem_im2col_kernel(const T* __restrict__ img, int ih, int iw, int oh, int ow, T* __restrict__ col,
                                   int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int kc = (int)(idx & 7);
  const int64_t pix = idx >> 3;
  const int ox = (int)(pix % ow), oy = (int)((pix / ow) % oh);
  const int64_t n = pix / ((int64_t)ow * oh);
  const T* p = img + n * ih * iw;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = kc * 8 + e;
    const int ky = k / 7, kx = k - ky * 7;
    const int iy = oy * 2 - 3 + ky, ix = ox * 2 - 3 + kx;
    v[e] = (k < 49 && iy >= 0 && iy < ih && ix >= 0 && ix < iw) ? ld1(p + iy * iw + ix) : 0.f;
  }
  store8(col + pix * 64 + kc * 8, v);
}

// ------------------------------------------------------------ weights --
// fp32 OIHW master weights -> compute layouts:
//   0: [Cout][k][k][Cin]                   (forward conv kernel)
//   1: [Cin][k][k][Cout], taps flipped     (stride-1 dgrad = conv of dy)
//   2: [Cout][64], k = ky*7+kx, channels summed (stem, the 3 input planes are identical)
//   3: [Cout][Cin][k][k]                   (dtype convert; strided dgrad GEMM)
//   4: [Cout][64], k = ky*8+kx (7x7 in an 8x8 grid), channels summed (bf16 training stem)
template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ w, int cout, int cin, int k, int mode,
                                   T* __restrict__ out, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int kk = k * k;
  float v;
  if (mode == 0) {  // idx = ((co*k + ky)*k + kx)*cin + ci
    const int ci = (int)(idx % cin);
    const int t = (int)((idx / cin) % kk);
    const int co = (int)(idx / ((int64_t)cin * kk));
    v = w[((int64_t)co * cin + ci) * kk + t];
  } else if (mode == 1) {  // idx = ((ci*k + ky)*k + kx)*cout + co
    const int co = (int)(idx % cout);
    const int t = (int)((idx / cout) % kk);
    const int ci = (int)(idx / ((int64_t)cout * kk));
    v = w[((int64_t)co * cin + ci) * kk + (kk - 1 - t)];
  } else if (mode == 2) {  // idx = co*64 + kpos
    const int kp = (int)(idx & 63), co = (int)(idx >> 6);
    v = 0.f;
    if (kp < kk)
      for (int c = 0; c < cin; ++c) v += w[((int64_t)co * cin + c) * kk + kp];
  } else if (mode == 4) {  // idx = co*64 + ky*8 + kx
    const int ky = (int)((idx >> 3) & 7), kx = (int)(idx & 7), co = (int)(idx >> 6);
    v = 0.f;
    if (ky < k && kx < k)
      for (int c = 0; c < cin; ++c) v += w[((int64_t)co * cin + c) * kk + ky * k + kx];
  } else {
    v = w[idx];
  }
  st1(out + idx, v);
}

// ------------------------------------------------------------ BatchNorm --
// Per-channel partial sums over an NHWC [P][C] tensor.  Thread = 8 channels of
// one row; a workgroup covers R = 256/(C/8) rows per pass, rows strided over
// the grid.  part[b][0][c] = sum, part[b][1][c] = sum of squares (mode 0), or
// for the backward pass (mode 1) sum dz, sum dz*xhat with dz = dy * [y > 0]
// (dy either a tensor or the avg-pool gradient dpool[n][c] / hw).
template <typename T, int MODE>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const T* __restrict__ x, int64_t P, int C,
                                                        const T* __restrict__ dy, const float* __restrict__ dpool,
                                                        int pool_hw, const T* __restrict__ y,
                                                        const float* __restrict__ stats, T* __restrict__ dz_out,
                                                        float* __restrict__ part) {
  __shared__ float red[2][256][9];
  const int G = C >> 3, R = 256 / G;
  const int g = threadIdx.x % G, r = threadIdx.x / G;
  const int c0 = g * 8;
  float s[8] = {}, q[8] = {};
  float mean[8], istd[8];
  if (MODE == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mean[e] = stats[c0 + e];
      istd[e] = stats[C + c0 + e];
    }
  }
  if (r < R) {
    for (int64_t row = (int64_t)blockIdx.x * R + r; row < P; row += (int64_t)gridDim.x * R) {
      float v[8];
      load8(x + row * C + c0, v);
      if (MODE == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s[e] += v[e];
          q[e] += v[e] * v[e];
        }
      } else {
        float d[8];
        if (dpool) {
          const float* dp = dpool + (row / pool_hw) * C + c0;
          const float inv = 1.f / pool_hw;
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = dp[e] * inv;
        } else {
          load8(dy + row * C + c0, d);
        }
        if (y) {
          float yy[8];
          load8(y + row * C + c0, yy);
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] = yy[e] > 0.f ? d[e] : 0.f;
        }
        if (dz_out) store8(dz_out + row * C + c0, d);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s[e] += d[e];
          q[e] += d[e] * ((v[e] - mean[e]) * istd[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][threadIdx.x][e] = s[e];
    red[1][threadIdx.x][e] = q[e];
  }
  __syncthreads();
  if (threadIdx.x < G) {
    float ts[8] = {}, tq[8] = {};
    for (int rr = 0; rr < R; ++rr) {
      const int t = rr * G + threadIdx.x;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ts[e] += red[0][t][e];
        tq[e] += red[1][t][e];
      }
    }
    float* pb = part + (int64_t)blockIdx.x * 2 * C;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pb[c0 + e] = ts[e];
      pb[C + c0 + e] = tq[e];
    }
  }
}

// Sum of the nb per-workgroup partials of channel c (one 256-thread workgroup
// per channel, float64 tree reduction).
__device__ __forceinline__ void channel_partials(const float* __restrict__ part, int nb, int C, int c, double& s,
                                                 double& q) {
  __shared__ double red[2][4];
  s = 0.0;
  q = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    s += part[(int64_t)b * 2 * C + c];
    q += part[(int64_t)b * 2 * C + C + c];
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = q;
  }
  __syncthreads();
  s = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
  q = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
}

// Forward finalize: batch mean / biased var (normalisation) and the running
// stats update with the unbiased var (torch BatchNorm2d train mode).
// stats = [mean | invstd | scale | shift], each [C].  Grid = C x 256 threads.
__global__ __launch_bounds__(256) void bn_finalize_fwd_kernel(const float* __restrict__ part, int nb, int64_t P,
                                                              int C, const float* __restrict__ gamma,
                                                              const float* __restrict__ beta, float eps,
                                                              float momentum, float* __restrict__ rmean,
                                                              float* __restrict__ rvar, float* __restrict__ stats) {
  const int c = blockIdx.x;
  double s, q;
  channel_partials(part, nb, C, c, s, q);
  if (threadIdx.x != 0) return;
  const double mean = s / (double)P;
  double var = q / (double)P - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  const double istd = 1.0 / sqrt(var + (double)eps);
  const double sc = (double)gamma[c] * istd;
  stats[c] = (float)mean;
  stats[C + c] = (float)istd;
  stats[2 * C + c] = (float)sc;
  stats[3 * C + c] = (float)((double)beta[c] - mean * sc);
  if (rmean) {
    const double unb = P > 1 ? var * (double)P / (double)(P - 1) : var;
    rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * mean);
    rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * unb);
  }
}

// Backward finalize: dbeta = sum dz, dgamma = sum dz*xhat (written, or added for
// the never-zeroed layer3 grads of quirk C4); coef = [gamma*istd | sum dz / P |
// sum dz*xhat / P].  Grid = C x 256 threads.
__global__ __launch_bounds__(256) void bn_finalize_bwd_kernel(const float* __restrict__ part, int nb, int64_t P,
                                                              int C, const float* __restrict__ gamma,
                                                              const float* __restrict__ stats,
                                                              float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                              int accumulate, float* __restrict__ coef) {
  const int c = blockIdx.x;
  double s, q;
  channel_partials(part, nb, C, c, s, q);
  if (threadIdx.x != 0) return;
  if (dgamma) dgamma[c] = (float)(accumulate ? (double)dgamma[c] + q : q);
  if (dbeta) dbeta[c] = (float)(accumulate ? (double)dbeta[c] + s : s);
  coef[c] = gamma[c] * stats[C + c];
  coef[C + c] = (float)(s / (double)P);
  coef[2 * C + c] = (float)(q / (double)P);
}

// The training stem's bn1 + ReLU on the sign(gamma)-max-pooled raw conv
// (conv.hip stem_bf16_kernel<false, true>): out = relu(|scale| * m' + shift).
__global__ void pooled_bn_relu_kernel(const u16* __restrict__ m, int64_t P, int C, const float* __restrict__ stats,
                                      u16* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int G = C >> 3;
  if (idx >= P * G) return;
  const int c0 = (int)(idx % G) * 8;
  float v[8];
  load8(m + idx * 8, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = fmaxf(fabsf(stats[2 * C + c0 + e]) * v[e] + stats[3 * C + c0 + e], 0.f);
  store8(out + idx * 8, v);
}

// y = act(x*scale + shift [+ res | + res*rscale + rshift]); thread = 8 channels.
template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ x, int64_t P, int C, const float* __restrict__ stats,
                                const T* __restrict__ res, const float* __restrict__ rstats, int relu,
                                T* __restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int G = C >> 3;
  if (idx >= P * G) return;
  const int c0 = (int)(idx % G) * 8;
  const int64_t off = (idx / G) * C + c0;
  float v[8];
  load8(x + off, v);
  const float* sc = stats + 2 * C + c0;
  const float* sh = stats + 3 * C + c0;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = v[e] * sc[e] + sh[e];
  if (res) {
    float r[8];
    load8(res + off, r);
    if (rstats) {
#pragma unroll
      for (int e = 0; e < 8; ++e) r[e] = r[e] * rstats[2 * C + c0 + e] + rstats[3 * C + c0 + e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  }
  if (relu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  store8(out + off, v);
}

// bn1 + ReLU + maxpool 3x3/2/p1 of the stem (timm resnet18 conv1 -> bn1 -> act1
// -> maxpool), NHWC, thread = one pooled pixel x 8 channels.
template <typename T>
__global__ void bn_relu_maxpool_kernel(const T* __restrict__ x, int H, int W, int C, const float* __restrict__ stats,
                                       int Ho, int Wo, T* __restrict__ out, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int G = C >> 3;
  const int c0 = (int)(idx % G) * 8;
  const int64_t pix = idx / G;
  const int ox = (int)(pix % Wo), oy = (int)((pix / Wo) % Ho);
  const int64_t n = pix / ((int64_t)Wo * Ho);
  const float* sc = stats + 2 * C + c0;
  const float* sh = stats + 3 * C + c0;
  float m[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) m[e] = 0.f;  // every window has a valid tap and ReLU output >= 0
  for (int dy = 0; dy < 3; ++dy) {
    const int iy = oy * 2 - 1 + dy;
    if (iy < 0 || iy >= H) continue;
    for (int dx = 0; dx < 3; ++dx) {
      const int ix = ox * 2 - 1 + dx;
      if (ix < 0 || ix >= W) continue;
      float v[8];
      load8(x + ((n * H + iy) * W + ix) * C + c0, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], v[e] * sc[e] + sh[e]);
    }
  }
  store8(out + pix * C + c0, m);
}

// dx = gamma*istd * (dz - mean(dz) - xhat * mean(dz*xhat)); dz from a stored
// tensor or recomputed from (dy | dpool) * [y > 0].
template <typename T>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ x, int64_t P, int C, const T* __restrict__ dz,
                                    const T* __restrict__ dy, const float* __restrict__ dpool, int pool_hw,
                                    const T* __restrict__ y, const float* __restrict__ stats,
                                    const float* __restrict__ coef, T* __restrict__ dx) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int G = C >> 3;
  if (idx >= P * G) return;
  const int c0 = (int)(idx % G) * 8;
  const int64_t row = idx / G, off = row * C + c0;
  float v[8], d[8];
  load8(x + off, v);
  if (dz) {
    load8(dz + off, d);
  } else {
    if (dpool) {
      const float* dp = dpool + (row / pool_hw) * C + c0;
      const float inv = 1.f / pool_hw;
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = dp[e] * inv;
    } else {
      load8(dy + off, d);
    }
    if (y) {
      float yy[8];
      load8(y + off, yy);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = yy[e] > 0.f ? d[e] : 0.f;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c0 + e;
    const float xh = (v[e] - stats[c]) * stats[C + c];
    d[e] = coef[c] * (d[e] - coef[C + c] - xh * coef[2 * C + c]);
  }
  store8(dx + off, d);
}

// ------------------------------------------------------------ loss --
// CrossEntropyLoss over the pooled features used as logits (quirk C1,
// submodel_trainer.py:262-263,281): one workgroup; wave per row, lane per 8
// logits.  dlogits = (softmax - onehot) * scale; out[0] = sum of row losses,
// out[1] = number of rows whose argmax (first max) equals the target.
__global__ __launch_bounds__(1024) void ce_kernel(const float* __restrict__ z, const int64_t* __restrict__ target,
                                                  int B, int C, float scale, float* __restrict__ dz,
                                                  float* __restrict__ out, int* __restrict__ pred) {
  __shared__ double sl[16];
  __shared__ int sc[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  double loss = 0.0;
  int correct = 0;
  for (int b = wave; b < B; b += nw) {
    const float* zr = z + (int64_t)b * C;
    float mx = -INFINITY;
    int am = 0x7fffffff;
    for (int j = lane; j < C; j += 64) {
      const float v = zr[j];
      if (v > mx) {  // first index within the lane's strided set
        mx = v;
        am = j;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(mx, o, 64);
      const int oa = __shfl_xor(am, o, 64);
      if (om > mx || (om == mx && oa < am)) {
        mx = om;
        am = oa;
      }
    }
    float se = 0.f;
    for (int j = lane; j < C; j += 64) se += expf(zr[j] - mx);
    for (int o = 32; o > 0; o >>= 1) se += __shfl_xor(se, o, 64);
    const float lse = mx + logf(se);
    const int t = (int)target[b];
    if (lane == 0) {
      loss += (double)(lse - zr[t]);
      correct += (am == t);
      if (pred) pred[b] = am;
    }
    for (int j = lane; j < C; j += 64) dz[(int64_t)b * C + j] = (expf(zr[j] - lse) - (j == t ? 1.f : 0.f)) * scale;
  }
  if (lane == 0) {
    sl[wave] = loss;
    sc[wave] = correct;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double L = 0.0;
    int K = 0;
    for (int i = 0; i < nw; ++i) {
      L += sl[i];
      K += sc[i];
    }
    out[0] = (float)L;
    out[1] = (float)K;
  }
}

// ------------------------------------------------------------ col2im --
// Gather form of col2im (deterministic): dx[n,iy,ix,ci] (+)= sum over taps with
// (iy + pad - ky) % s == 0 of dcol[n,oy,ox][ci*k*k + ky*k + kx].
template <typename T>
__global__ void col2im_kernel(const float* __restrict__ dcol, int H, int W, int C, int k, int s, int pad, int Ho,
                              int Wo, int accumulate, T* __restrict__ dx, int64_t total) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int ci = (int)(idx % C);
  const int64_t pix = idx / C;
  const int ix = (int)(pix % W), iy = (int)((pix / W) % H);
  const int64_t n = pix / ((int64_t)W * H);
  const int kk = k * k;
  float acc = accumulate ? ld1(dx + idx) : 0.f;
  for (int ky = 0; ky < k; ++ky) {
    const int ty = iy + pad - ky;
    if (ty < 0 || ty % s) continue;
    const int oy = ty / s;
    if (oy >= Ho) continue;
    for (int kx = 0; kx < k; ++kx) {
      const int tx = ix + pad - kx;
      if (tx < 0 || tx % s) continue;
      const int ox = tx / s;
      if (ox >= Wo) continue;
      acc += dcol[((n * Ho + oy) * Wo + ox) * ((int64_t)C * kk) + (int64_t)ci * kk + ky * k + kx];
    }
  }
  st1(dx + idx, acc);
}

// ------------------------------------------------------------ optimizer --
// torch.nn.utils.clip_grad_norm_(max_norm) (submodel_trainer.py:276) over one
// flat fp32 gradient buffer: partial sums of squares, then
// coef = min(max_norm / (||g|| + 1e-6), 1) and g *= coef.
__global__ __launch_bounds__(256) void sqnorm_kernel(const float* __restrict__ g, int64_t n, double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double v = g[i];
    s += v * v;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void clip_coef_kernel(const double* __restrict__ part, int nb, float max_norm,
                                                        float* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) s += part[b];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x != 0) return;
  s = (red[0] + red[1]) + (red[2] + red[3]);
  const float norm = (float)sqrt(s);
  const float coef = max_norm / (norm + 1e-6f);
  out[0] = norm;
  out[1] = coef < 1.f ? coef : 1.f;
}

__global__ void scale_kernel(float* __restrict__ g, int64_t n, const float* __restrict__ coef) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) g[i] *= coef[1];
}

// torch.optim.AdamW single-tensor step (submodel_trainer.py:648-652,278):
// p *= 1 - lr*wd; m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                             float bc1, float bc2_sqrt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i];
  float pi = p[i] * (1.f - lr * wd);
  const float mi = m[i] + (gi - m[i]) * (1.f - b1);
  const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  pi -= (lr / bc1) * (mi / denom);
  p[i] = pi;
  m[i] = mi;
  v[i] = vi;
}

static inline unsigned nblk(int64_t total, int t = 256) { return (unsigned)((total + t - 1) / t); }
static inline size_t ES(int dtype) { return dtype == SAD_BF16 ? 2 : 4; }

int launch_col2im(const float* dcol, int64_t N, int H, int W, int C, int k, int stride, int pad, int Ho, int Wo,
                  int accumulate, void* dx, int dtype, hipStream_t s) {
  const int64_t total = N * H * W * (int64_t)C;
  if (!total) return SAD_OK;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(col2im_kernel<u16>, dim3(nblk(total)), dim3(256), 0, s, dcol, H, W, C, k, stride, pad, Ho, Wo,
                       accumulate, (u16*)dx, total);
  else
    hipLaunchKernelGGL(col2im_kernel<float>, dim3(nblk(total)), dim3(256), 0, s, dcol, H, W, C, k, stride, pad, Ho,
                       Wo, accumulate, (float*)dx, total);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

}  // namespace sad

using namespace sad;

extern "C" int sad_specaug_norm_run(const float* db, int64_t n, int32_t n_mels, int32_t n_frames, const int32_t* masks,
                                    float* out_map, void* stream) {
  SAD_REQUIRE(db && out_map && n >= 0 && n_mels > 0 && n_frames > 0, "bad args");
  for (int64_t i = 0; i < n; i += 65535) {
    const int64_t c = std::min<int64_t>(65535, n - i);
    const int64_t off = i * n_mels * n_frames;
    hipLaunchKernelGGL(specaug_norm_kernel, dim3((unsigned)c), dim3(1024), 0, (hipStream_t)stream, db + off, n_mels,
                       n_frames, masks ? masks + i * 4 : nullptr, out_map + off);
    SAD_CHECK_HIP(hipGetLastError());
  }
  return SAD_OK;
}

extern "C" int sad_crop_resize_run(const float* map, int64_t n, int32_t h, int32_t w, const int32_t* boxes,
                                   int32_t out_hw, int32_t dtype, void* img, void* stream) {
  SAD_REQUIRE(map && img && n >= 0 && h > 0 && w > 0 && out_hw > 0, "bad args");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  SAD_REQUIRE(n <= 65535, "crop_resize: n > 65535");
  if (!n) return SAD_OK;
  const dim3 grid((unsigned)out_hw, (unsigned)n);
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(crop_resize_kernel<u16>, grid, dim3(256), 0, (hipStream_t)stream, map, h, w, boxes, out_hw,
                       (u16*)img);
  else
    hipLaunchKernelGGL(crop_resize_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, map, h, w, boxes, out_hw,
                       (float*)img);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_pack_conv_weight_run(const float* w, int32_t cout, int32_t cin, int32_t k, int32_t mode,
                                        int32_t dtype, void* out, void* stream) {
  SAD_REQUIRE(w && out && cout > 0 && cin > 0 && k > 0 && mode >= 0 && mode <= 4, "bad args");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  SAD_REQUIRE(mode != 2 || k * k <= 64, "stem pack needs k*k <= 64");
  SAD_REQUIRE(mode != 4 || k <= 8, "8x8-grid stem pack needs k <= 8");
  const int64_t total = mode == 2 || mode == 4 ? (int64_t)cout * 64 : (int64_t)cout * cin * k * k;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(pack_weight_kernel<u16>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, w, cout, cin, k,
                       mode, (u16*)out, total);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, w, cout, cin,
                       k, mode, (float*)out, total);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_stem_conv_run(const void* img, int64_t n, int32_t ih, int32_t iw, const void* w_packed,
                                 void* col_ws, size_t ws_bytes, void* out, int32_t dtype, void* stream) {
  SAD_REQUIRE(img && w_packed && col_ws && out && n >= 0 && ih > 0 && iw > 0, "bad args");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  const int oh = (ih + 6 - 7) / 2 + 1, ow = (iw + 6 - 7) / 2 + 1;
  const int64_t pix = n * oh * ow;
  SAD_REQUIRE(ws_bytes >= (size_t)pix * 64 * ES(dtype), "stem col workspace too small");
  if (!pix) return SAD_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(stem_im2col_kernel<u16>, dim3(nblk(pix * 8)), dim3(256), 0, s, (const u16*)img, ih, iw, oh, ow,
                       (u16*)col_ws, pix * 8);
  else
    hipLaunchKernelGGL(stem_im2col_kernel<float>, dim3(nblk(pix * 8)), dim3(256), 0, s, (const float*)img, ih, iw, oh,
                       ow, (float*)col_ws, pix * 8);
  SAD_CHECK_HIP(hipGetLastError());
  static float* zero_bias[64] = {};
  int dev = 0;
  SAD_CHECK_HIP(hipGetDevice(&dev));
  if (!zero_bias[dev]) {
    SAD_CHECK_HIP(hipMalloc((void**)&zero_bias[dev], 512 * sizeof(float)));
    SAD_CHECK_HIP(hipMemset(zero_bias[dev], 0, 512 * sizeof(float)));
  }
  SAD_REQUIRE(pix < (1ll << 31), "stem: too many pixels");
  BlockConvArgs a{};
  a.in0 = col_ws;
  a.in0_pstride = 64;
  a.N = 1;
  a.H = 1;
  a.W = (int)pix;
  a.Cin = 64;
  a.KH = a.KW = 1;
  a.stride = 1;
  a.pad = 0;
  a.wt = w_packed;
  a.wt_ld = 64;
  a.bias = zero_bias[dev];
  a.out = out;
  a.out_pstride = 64;
  a.Ho = 1;
  a.Wo = (int)pix;
  a.Cout = 64;
  a.M = pix;
  return launch_block_conv(a, dtype, s);
}

static int bn_nblocks(int64_t P, int C) {
  const int R = 256 / (C / 8);
  const int64_t want = (P + R * 16 - 1) / (R * 16);  // >= 16 rows per thread
  return (int)std::max<int64_t>(1, std::min<int64_t>(1024, want));
}

// Zero conv bias (the trainer's convs are bias-free; the conv kernels add one)
static const float* device_zero_bias() {
  static float* zb[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!zb[dev]) {
    if (hipMalloc((void**)&zb[dev], 2048 * sizeof(float)) != hipSuccess) return nullptr;
    if (hipMemset(zb[dev], 0, 2048 * sizeof(float)) != hipSuccess) return nullptr;
  }
  return zb[dev];
}

extern "C" int sad_stem_train_workspace_size(int64_t n, size_t* bytes) {
  SAD_REQUIRE(bytes && n >= 0, "bad args");
  *bytes = (size_t)n * 128 * 128 * 64 * 2 + (size_t)n * STEM_TRAIN_PARTS * 128 * sizeof(float);
  return SAD_OK;
}

extern "C" int sad_stem_train_run(const void* img, int64_t n, const void* w_packed, const float* gamma,
                                  const float* beta, float eps, float momentum, float* running_mean,
                                  float* running_var, float* stats, void* out, void* ws, size_t ws_bytes,
                                  void* stream) {
  SAD_REQUIRE(img && w_packed && gamma && beta && stats && out && ws && n >= 0, "bad args");
  SAD_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "running stats: both or neither");
  size_t need = 0;
  sad_stem_train_workspace_size(n, &need);
  SAD_REQUIRE(ws_bytes >= need, "stem workspace too small (sad_stem_train_workspace_size)");
  if (n == 0) return SAD_OK;
  hipStream_t s = (hipStream_t)stream;
  u16* pooled = (u16*)ws;
  float* part = (float*)((char*)ws + (size_t)n * 128 * 128 * 64 * 2);
  StemArgs a{};
  a.img16 = (const u16*)img;
  a.w = w_packed;
  a.bias = gamma;
  a.out = pooled;
  a.part = part;
  a.B = n;
  int rc = launch_stem_train(a, s);
  if (rc) return rc;
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(64), dim3(256), 0, s, part, (int)(n * STEM_TRAIN_PARTS),
                     n * 256 * 256, 64, gamma, beta, eps, momentum, running_mean, running_var, stats);
  SAD_CHECK_HIP(hipGetLastError());
  const int64_t P = n * 128 * 128;
  hipLaunchKernelGGL(pooled_bn_relu_kernel, dim3(nblk(P * 8)), dim3(256), 0, s, pooled, P, 64, stats, (u16*)out);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}


// conv -> raw NHWC output + train-mode BatchNorm statistics.  bf16: the
// statistics are summed in the conv kernels' epilogues (variants 13, 15, 20,
// 25: StatAcc, one partial row per pixel-group workgroup), so the raw output is
// never re-read; other shapes / fp32: conv, then the bn_reduce pass.
static constexpr int kStatRowsMax = 512;  // >= the workgroup rows of any variant (256 x occupancy)

extern "C" int sad_conv_bn_train_workspace_size(int64_t N, int32_t H, int32_t W, int32_t Cout, int32_t k,
                                                int32_t stride, int32_t pad, size_t* bytes) {
  SAD_REQUIRE(bytes && N >= 0 && H > 0 && W > 0 && Cout > 0 && k > 0 && stride > 0 && pad >= 0, "bad args");
  const int64_t P = N * ((H + 2 * pad - k) / stride + 1) * ((W + 2 * pad - k) / stride + 1);
  const size_t fused = (size_t)kStatRowsMax * 2 * Cout * sizeof(float) + 3 * (size_t)Cout * sizeof(float);
  const size_t unfused = (size_t)bn_nblocks(P, Cout) * 2 * Cout * sizeof(float) + 3 * (size_t)Cout * sizeof(float);
  *bytes = std::max(fused, unfused);
  return SAD_OK;
}

// SAD_TRAIN_L2_RW (default 1): the trainer's layer2 raw convs on the
// resident-weight variants with fused statistics (round 4): 128 -> 128 on
// variant 41, the stride-2 64 -> 128 on variant 43; 0 = variants 20 / 15
static bool train_l2_rw() {
  static const bool v = [] {
    const char* e = getenv("SAD_TRAIN_L2_RW");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}

extern "C" int sad_conv_bn_train_run(const void* x, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* w_packed,
                                     int32_t Cout, int32_t k, int32_t stride, int32_t pad, int32_t dtype,
                                     const float* gamma, const float* beta, float eps, float momentum,
                                     float* running_mean, float* running_var, float* stats, void* out, float* ws,
                                     size_t ws_bytes, int32_t* fused_out, void* stream) {
  SAD_REQUIRE(x && w_packed && gamma && beta && stats && out && ws, "null tensor");
  SAD_REQUIRE(N > 0 && H > 0 && W > 0 && Cin > 0 && k > 0 && stride > 0 && pad >= 0, "bad shape");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  SAD_REQUIRE(Cout % 8 == 0 && Cout >= 8 && Cout <= 2048, "Cout must be a multiple of 8 in [8, 2048]");
  SAD_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "running stats: both or neither");
  size_t need = 0;
  sad_conv_bn_train_workspace_size(N, H, W, Cout, k, stride, pad, &need);
  SAD_REQUIRE(ws_bytes >= need, "workspace too small (sad_conv_bn_train_workspace_size)");
  hipStream_t s = (hipStream_t)stream;
  const float* zb = device_zero_bias();
  SAD_REQUIRE(zb != nullptr, "zero bias allocation");
  BlockConvArgs a{};
  a.in0 = x;
  a.in0_pstride = Cin;
  a.N = (int)N;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.KH = a.KW = k;
  a.stride = stride;
  a.pad = pad;
  a.wt = w_packed;
  a.bias = zb;
  a.out = out;
  a.out_pstride = Cout;
  a.Ho = (H + 2 * pad - k) / stride + 1;
  a.Wo = (W + 2 * pad - k) / stride + 1;
  a.Cout = Cout;
  a.M = N * a.Ho * a.Wo;
  const int64_t P = a.M;
  int v = default_block_variant(a, dtype);
  // The fused statistics need ONE launch (one partial row per workgroup).  A
  // batch whose operands pass the kernels' 32-bit buffer range (e.g. a
  // Bottleneck's 256-channel 128^2 layer1 maps at ~256 images) is split by
  // launch_block_conv into image-range launches, so it takes the unfused path:
  // plain conv launches, then bn_reduce over the stored output.
  const int64_t es = dtype == SAD_F32 ? 4 : 2, lim = (1ll << 31) - 65536;
  const bool one_launch = N * H * W * Cin * es < lim && a.M * Cout * es < lim;
  // the patch-resident kernels (30, 31, 32) sum no statistics; their
  // implicit-GEMM counterparts (13 / 15) do
  // (variant 43 sums them, layer2.0's stride-2 conv1; SAD_TRAIN_L2_RW=0 keeps the implicit GEMM there)
  if ((v == 30 || v == 31 || v == 32 || (v == 43 && !train_l2_rw())) && dtype == SAD_BF16 && one_launch)
    v = gemm_block_variant(a);
  // variant 41 sums them in its plain form (no shortcut / residual: the
  // trainer's raw convs of layer2's 128 -> 128 convs); SAD_TRAIN_L2_RW=0 keeps
  // the weight-ring halo kernel (variant 20) there
  if (v == 41 && dtype == SAD_BF16 && one_launch && (a.in1 || a.res || !train_l2_rw())) v = 20;
  const bool fused = dtype == SAD_BF16 && one_launch && (v == 13 || v == 15 || v == 20 || v == 25 || v == 41 || v == 43);
  int rows = 0;
  if (fused) {
    a.st_part = ws;
    a.st_rows = &rows;
  }
  int rc = launch_block_conv(a, dtype, s, v);
  if (rc) return rc;
  if (fused_out) *fused_out = fused;
  if (!fused) {
    const int nb = bn_nblocks(P, Cout);
    if (dtype == SAD_BF16)
      hipLaunchKernelGGL((bn_reduce_kernel<u16, 0>), dim3(nb), dim3(256), 0, s, (const u16*)out, P, Cout, nullptr,
                         nullptr, 1, nullptr, nullptr, nullptr, ws);
    else
      hipLaunchKernelGGL((bn_reduce_kernel<float, 0>), dim3(nb), dim3(256), 0, s, (const float*)out, P, Cout,
                         nullptr, nullptr, 1, nullptr, nullptr, nullptr, ws);
    SAD_CHECK_HIP(hipGetLastError());
    rows = nb;
  }
  SAD_REQUIRE(rows > 0 && rows <= (fused ? kStatRowsMax : 1024), "statistic partial rows");
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(Cout), dim3(256), 0, s, ws, rows, P, Cout, gamma, beta, eps,
                     momentum, running_mean, running_var, stats);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_bn_workspace_size(int64_t P, int32_t C, size_t* bytes) {
  SAD_REQUIRE(bytes && C > 0, "bad args");
  *bytes = (size_t)bn_nblocks(P, C) * 2 * C * sizeof(float) + 3 * (size_t)C * sizeof(float);
  return SAD_OK;
}

extern "C" int sad_bn_stats_run(const void* x, int64_t P, int32_t C, int32_t dtype, const float* gamma,
                                const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                                float* stats, float* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(x && gamma && beta && stats && ws && P > 0, "bad args");
  SAD_REQUIRE(C % 8 == 0 && C >= 8 && C <= 2048, "C must be a multiple of 8 in [8, 2048]");
  SAD_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "running stats: both or neither");
  size_t need = 0;
  sad_bn_workspace_size(P, C, &need);
  SAD_REQUIRE(ws_bytes >= need, "bn workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int nb = bn_nblocks(P, C);
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL((bn_reduce_kernel<u16, 0>), dim3(nb), dim3(256), 0, s, (const u16*)x, P, C, nullptr, nullptr, 1,
                       nullptr, nullptr, nullptr, ws);
  else
    hipLaunchKernelGGL((bn_reduce_kernel<float, 0>), dim3(nb), dim3(256), 0, s, (const float*)x, P, C, nullptr,
                       nullptr, 1, nullptr, nullptr, nullptr, ws);
  SAD_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(bn_finalize_fwd_kernel, dim3(C), dim3(256), 0, s, ws, nb, P, C, gamma, beta, eps,
                     momentum, running_mean, running_var, stats);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_bn_apply_run(const void* x, int64_t P, int32_t C, int32_t dtype, const float* stats,
                                const void* res, const float* res_stats, int32_t relu, void* out, void* stream) {
  SAD_REQUIRE(x && stats && out && P >= 0 && C % 8 == 0, "bad args");
  const int64_t total = P * (C / 8);
  if (!total) return SAD_OK;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<u16>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, (const u16*)x, P, C,
                       stats, (const u16*)res, res_stats, relu, (u16*)out);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream, (const float*)x, P,
                       C, stats, (const float*)res, res_stats, relu, (float*)out);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_bn_relu_maxpool_run(const void* x, int64_t n, int32_t H, int32_t W, int32_t C, int32_t dtype,
                                       const float* stats, void* out, void* stream) {
  SAD_REQUIRE(x && stats && out && n >= 0 && H > 0 && W > 0 && C % 8 == 0, "bad args");
  const int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  const int64_t total = n * Ho * Wo * (C / 8);
  if (!total) return SAD_OK;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<u16>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream,
                       (const u16*)x, H, W, C, stats, Ho, Wo, (u16*)out, total);
  else
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<float>, dim3(nblk(total)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, H, W, C, stats, Ho, Wo, (float*)out, total);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_ce_loss_run(const float* logits, const int64_t* target, int64_t B, int32_t C, float scale,
                               float* dlogits, float* out, int32_t* pred, void* stream) {
  SAD_REQUIRE(logits && target && dlogits && out && B >= 0 && C > 0, "bad args");
  SAD_REQUIRE(B < (1 << 30), "B too large");
  hipLaunchKernelGGL(ce_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, logits, target, (int)B, C, scale, dlogits,
                     out, pred);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_bn_backward_run(const void* x, int64_t P, int32_t C, int32_t dtype, const float* stats,
                                   const float* gamma, const void* dy, const float* dpool, int32_t pool_hw,
                                   const void* y, float* dgamma, float* dbeta, int32_t accumulate, void* dz_out,
                                   void* dx, float* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(x && stats && gamma && dx && ws && P > 0, "bad args");
  SAD_REQUIRE((dy != nullptr) != (dpool != nullptr), "exactly one of dy / dpool");
  SAD_REQUIRE(!dpool || (pool_hw > 0 && P % pool_hw == 0), "pool_hw");
  SAD_REQUIRE(C % 8 == 0 && C >= 8 && C <= 2048, "C must be a multiple of 8 in [8, 2048]");
  size_t need = 0;
  sad_bn_workspace_size(P, C, &need);
  SAD_REQUIRE(ws_bytes >= need, "bn workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int nb = bn_nblocks(P, C);
  float* coef = ws + (size_t)nb * 2 * C;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL((bn_reduce_kernel<u16, 1>), dim3(nb), dim3(256), 0, s, (const u16*)x, P, C, (const u16*)dy,
                       dpool, pool_hw > 0 ? pool_hw : 1, (const u16*)y, stats, (u16*)dz_out, ws);
  else
    hipLaunchKernelGGL((bn_reduce_kernel<float, 1>), dim3(nb), dim3(256), 0, s, (const float*)x, P, C,
                       (const float*)dy, dpool, pool_hw > 0 ? pool_hw : 1, (const float*)y, stats, (float*)dz_out, ws);
  SAD_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(bn_finalize_bwd_kernel, dim3(C), dim3(256), 0, s, ws, nb, P, C, gamma, stats,
                     dgamma, dbeta, accumulate, coef);
  SAD_CHECK_HIP(hipGetLastError());
  const int64_t total = P * (C / 8);
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<u16>, dim3(nblk(total)), dim3(256), 0, s, (const u16*)x, P, C,
                       (const u16*)dz_out, (const u16*)dy, dpool, pool_hw > 0 ? pool_hw : 1, (const u16*)y, stats,
                       coef, (u16*)dx);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<float>, dim3(nblk(total)), dim3(256), 0, s, (const float*)x, P, C,
                       (const float*)dz_out, (const float*)dy, dpool, pool_hw > 0 ? pool_hw : 1, (const float*)y,
                       stats, coef, (float*)dx);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_clip_grad_norm_run(float* g, int64_t n, float max_norm, float* norm_coef, void* ws, size_t ws_bytes,
                                      void* stream) {
  SAD_REQUIRE(g && norm_coef && ws && n >= 0, "bad args");
  SAD_REQUIRE(ws_bytes >= 1024 * sizeof(double), "clip workspace must hold 1024 doubles");
  hipStream_t s = (hipStream_t)stream;
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (n + 4095) / 4096));
  hipLaunchKernelGGL(sqnorm_kernel, dim3(nb), dim3(256), 0, s, g, n, (double*)ws);
  SAD_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, s, (const double*)ws, nb, max_norm, norm_coef);
  SAD_CHECK_HIP(hipGetLastError());
  if (n) {
    hipLaunchKernelGGL(scale_kernel, dim3(nblk(n)), dim3(256), 0, s, g, n, (const float*)norm_coef);
    SAD_CHECK_HIP(hipGetLastError());
  }
  return SAD_OK;
}

__global__ void axpy_kernel(float* __restrict__ y, const float* __restrict__ x, int64_t n, float alpha) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] += alpha * x[i];
}

extern "C" int sad_axpy_run(float* y, const float* x, int64_t n, float alpha, void* stream) {
  SAD_REQUIRE(y && x && n >= 0, "bad args");
  if (!n) return SAD_OK;
  hipLaunchKernelGGL(axpy_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, y, x, n, alpha);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

// 8 elements per thread: fp32 -> bf16 (one v_cvt_pk_bf16_f32 per pair) or bf16 -> fp32
template <bool TO_BF16>
__global__ void cast_kernel(const void* __restrict__ src, void* __restrict__ dst, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  if constexpr (TO_BF16) {
    const float* s = (const float*)src + i;
    u16* d = (u16*)dst + i;
    if (i + 8 <= n) {
      const float4 a = *(const float4*)s, b = *(const float4*)(s + 4);
      *(uint4*)d = make_uint4((uint32_t)f2bf(a.x) | ((uint32_t)f2bf(a.y) << 16),
                              (uint32_t)f2bf(a.z) | ((uint32_t)f2bf(a.w) << 16),
                              (uint32_t)f2bf(b.x) | ((uint32_t)f2bf(b.y) << 16),
                              (uint32_t)f2bf(b.z) | ((uint32_t)f2bf(b.w) << 16));
    } else {
      for (int64_t k = i; k < n; ++k) ((u16*)dst)[k] = f2bf(((const float*)src)[k]);
    }
  } else {
    const u16* s = (const u16*)src + i;
    float* d = (float*)dst + i;
    if (i + 8 <= n) {
      const uint4 q = *(const uint4*)s;
      *(float4*)d = make_float4(bf2f((u16)(q.x & 0xFFFF)), bf2f((u16)(q.x >> 16)), bf2f((u16)(q.y & 0xFFFF)),
                                bf2f((u16)(q.y >> 16)));
      *(float4*)(d + 4) = make_float4(bf2f((u16)(q.z & 0xFFFF)), bf2f((u16)(q.z >> 16)), bf2f((u16)(q.w & 0xFFFF)),
                                      bf2f((u16)(q.w >> 16)));
    } else {
      for (int64_t k = i; k < n; ++k) ((float*)dst)[k] = bf2f(((const u16*)src)[k]);
    }
  }
}

extern "C" int sad_cast_run(const void* src, int32_t src_dtype, void* dst, int32_t dst_dtype, int64_t n, void* stream) {
  SAD_REQUIRE(src && dst && n >= 0, "bad args");
  SAD_REQUIRE((src_dtype == SAD_F32 && dst_dtype == SAD_BF16) || (src_dtype == SAD_BF16 && dst_dtype == SAD_F32),
              "cast: fp32 <-> bf16 only");
  SAD_REQUIRE(((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0, "cast: 16-B aligned buffers");
  if (!n) return SAD_OK;
  const int64_t th = (n + 7) / 8;
  const dim3 grid((unsigned)((th + 255) / 256));
  if (src_dtype == SAD_F32)
    hipLaunchKernelGGL(cast_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, src, dst, n);
  else
    hipLaunchKernelGGL(cast_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, src, dst, n);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_avgpool_run(const void* x, int64_t B, int32_t hw, int32_t C, int32_t dtype, float* out,
                               void* stream) {
  SAD_REQUIRE(x && out && B >= 0 && hw > 0 && C % 64 == 0, "bad args (C must be a multiple of 64)");
  return launch_avgpool(x, B, hw, C, out, dtype, (hipStream_t)stream);
}

// AdamW + re-pack of the updated conv weights into their cached compute
// layouts (pack modes 0 and 1), so the next forward / backward needs no pack
// launches.  Segment search is per thread over <= 16 (wave-uniform) entries.
struct PackSegs {
  sad_pack_seg s[16];
  int n;
};
template <typename T>
__global__ void adamw_pack_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                  float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                                  float bc1, float bc2_sqrt, PackSegs segs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i];
  float pi = p[i] * (1.f - lr * wd);
  const float mi = m[i] + (gi - m[i]) * (1.f - b1);
  const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  pi -= (lr / bc1) * (mi / denom);
  p[i] = pi;
  m[i] = mi;
  v[i] = vi;
  for (int k = 0; k < segs.n; ++k) {
    const sad_pack_seg& sg = segs.s[k];
    const int kk = sg.k * sg.k;
    const int64_t loc = i - sg.offset;
    if (loc < 0 || loc >= (int64_t)sg.cout * sg.cin * kk) continue;
    const int t = (int)(loc % kk), ci = (int)((loc / kk) % sg.cin), co = (int)(loc / ((int64_t)kk * sg.cin));
    if (sg.mode0) st1((T*)sg.mode0 + ((int64_t)co * kk + t) * sg.cin + ci, pi);
    if (sg.mode1) st1((T*)sg.mode1 + ((int64_t)ci * kk + (kk - 1 - t)) * sg.cout + co, pi);
  }
}

extern "C" int sad_adamw_pack_run(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                                  float beta2, float eps, float weight_decay, int64_t step, const sad_pack_seg* segs,
                                  int32_t nseg, int32_t dtype, void* stream) {
  SAD_REQUIRE(p && g && m && v && n >= 0 && step >= 1, "bad args");
  SAD_REQUIRE(nseg >= 0 && nseg <= 16 && (nseg == 0 || segs), "at most 16 pack segments");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  PackSegs ps{};
  ps.n = nseg;
  for (int k = 0; k < nseg; ++k) {
    ps.s[k] = segs[k];
    SAD_REQUIRE(segs[k].offset >= 0 && segs[k].cout > 0 && segs[k].cin > 0 && segs[k].k > 0 &&
                    segs[k].offset + (int64_t)segs[k].cout * segs[k].cin * segs[k].k * segs[k].k <= n,
                "pack segment outside the parameter range");
  }
  if (!n) return SAD_OK;
  const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(adamw_pack_kernel<u16>, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr,
                       beta1, beta2, eps, weight_decay, bc1, bc2s, ps);
  else
    hipLaunchKernelGGL(adamw_pack_kernel<float>, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr,
                       beta1, beta2, eps, weight_decay, bc1, bc2s, ps);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_adamw_run(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                             float beta2, float eps, float weight_decay, int64_t step, void* stream) {
  SAD_REQUIRE(p && g && m && v && n >= 0 && step >= 1, "bad args");
  if (!n) return SAD_OK;
  const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  const float bc2s = (float)sqrt(1.0 - pow((double)beta2, (double)step));
  hipLaunchKernelGGL(adamw_kernel, dim3(nblk(n)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, lr, beta1, beta2,
                     eps, weight_decay, bc1, bc2s);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}
