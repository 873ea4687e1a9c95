// conv.hip -- ResNet-18 conv kernels for gfx950 (CDNA4).
//
// Replaces the timm ResNet-18 forward_features (cuDNN/MIOpen conv + BN + ReLU +
// residual add + maxpool) behind inference_runner.py:49-51, and its head's
// AdaptiveAvgPool2d (inference_runner.py:37).
//
// conv_igemm_kernel<T, WM, WN>: implicit GEMM, NHWC activations,
//   out[m, n] = act( sum_k A[m, k] * W[n, k] + bias[n] (+ res[m, n]) )
//   m = (b, oy, ox), n = output channel, k = (ky, kx, ci); BN is folded into W
//   and bias at plan time.  Tile BM x BN = 64*WM x 64*WN, 4 waves of 64x64,
//   each wave 4x4 MFMA 16x16 tiles.  One K-step = one filter tap x 128 bytes of
//   input channels (64 bf16 / 32 f32): every A row of a K-step is ONE
//   contiguous 128-B NHWC span, loaded as 8 x 16 B per pixel (coalesced, zero
//   for padding taps).  Tiles are register-staged into a double-buffered LDS
//   ring (one barrier per K-step, loads for step k+1 in flight under the MFMAs
//   of step k) with an XOR swizzle (chunk ^ ((row>>1)&7)) that makes both the
//   16-B staging writes and the 16-B fragment reads bank-conflict free.
//   T = bf16: v_mfma_f32_16x16x32_bf16; T = float: v_mfma_f32_16x16x4_f32
//   (parity mode; exact fp32 FMA chains).  Both fragment maps read the same
//   16-B chunk per lane (k order permuted identically for A and B).
//   Epilogue: accumulators -> LDS -> 16-B/lane rows: + bias, + residual, ReLU,
//   convert, coalesced store.  Grid = M/BM x N/BN tiles, XCD-remapped so the
//   N-tiles of one M-tile share an L2.
//
// stem_kernel<T>: fused bilinear resize (map 128x251 -> 512x512, torchvision
//   Resize semantics) + conv1 7x7/2 (3 identical input channels folded into
//   the weights) + bn1 + ReLU + maxpool 3x3/2/p1.  One workgroup = one pooled
//   output row (128 x 64): it builds the 11 x 517 image band in LDS, computes
//   the three conv rows 2py-1..2py+1 as [256 px x 64 k(49 used)] x [64 x 64]
//   MFMA GEMMs, keeps the vertical max in registers, and pools horizontally
//   through LDS.  The 512x512 image and the 256x256x64 conv1 map never reach
//   HBM.
#include "common.hpp"
#include "kernels.hpp"

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

template <int WM, int WN>
constexpr int conv_smem_bytes() {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int main_b = 2 * (BM + BN) * 128;
  constexpr int epi_b = BM * (BN + 4) * 4;
  return main_b > epi_b ? main_b : epi_b;
}

template <typename T, int WM, int WN>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(ConvArgs a) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int EPC = DT<T>::EPC;
  constexpr int BK = 8 * EPC;
  constexpr int A_PER_T = BM / 32, B_PER_T = BN / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int n_tn = a.Cout / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = wg % n_tn, tm = wg / n_tn;
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;

  const T* __restrict__ in = (const T*)a.in;
  const T* __restrict__ wt = (const T*)a.wt;
  const int ch = tid & 7, rbase = tid >> 3;
  const int HoWo = a.Ho * a.Wo;

  // per-thread A rows: base pointer at tap (0,0), input origin, validity
  const T* arow[A_PER_T];
  int aiy[A_PER_T], aix[A_PER_T];
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int64_t m = m0 + rbase + 32 * i;
    if (m < a.M) {
      const int b = (int)(m / HoWo);
      const int rem = (int)(m - (int64_t)b * HoWo);
      const int oy = rem / a.Wo, ox = rem - (rem / a.Wo) * a.Wo;
      aiy[i] = oy * a.stride - a.pad;
      aix[i] = ox * a.stride - a.pad;
      arow[i] = in + (((int64_t)b * a.H + aiy[i]) * a.W + aix[i]) * a.in_pstride + ch * EPC;
    } else {
      aiy[i] = -100000;
      aix[i] = -100000;
      arow[i] = in;
    }
  }
  const int64_t Ktot = (int64_t)a.KH * a.KW * a.Cin;
  const T* brow = wt + (int64_t)(n0 + rbase) * Ktot + ch * EPC;
  const int cpt = a.Cin / BK;
  const int nk = a.KH * a.KW * cpt;

  uint4 ra[A_PER_T], rb[B_PER_T];
  auto gload = [&](int ks) {
    const int tap = ks / cpt;
    const int ci0 = (ks - tap * cpt) * BK;
    const int ky = tap / a.KW, kx = tap - (tap / a.KW) * a.KW;
    const int64_t toff = ((int64_t)ky * a.W + kx) * a.in_pstride + ci0;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int iy = aiy[i] + ky, ix = aix[i] + kx;
      const bool ok = ((unsigned)iy < (unsigned)a.H) && ((unsigned)ix < (unsigned)a.W);
      ra[i] = ok ? *(const uint4*)(arow[i] + toff) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) rb[i] = *(const uint4*)(brow + (int64_t)32 * i * Ktot + (int64_t)ks * BK);
  };
  auto sstore = [&](int buf) {
    char* base = smem + buf * (BM + BN) * 128;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int r = rbase + 32 * i;
      *(uint4*)(base + r * 128 + (swz(r, ch) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int r = BM + rbase + 32 * i;
      *(uint4*)(base + r * 128 + (swz(r, ch) << 4)) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  gload(0);
  sstore(0);
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < nk) gload(ks + 1);
    const char* base = smem + cur * (BM + BN) * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 af[4], bfr[4];
      const int c = fg + 4 * s;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wm * 64 + i * 16 + fr;
        af[i] = *(const uint4*)(base + r * 128 + (swz(r, c) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = BM + wn * 64 + j * 16 + fr;
        bfr[j] = *(const uint4*)(base + r * 128 + (swz(r, c) << 4));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_chunk<T>(af[i], bfr[j], acc[i][j]);
    }
    if (ks + 1 < nk) sstore(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: acc -> LDS [BM][BN+4] f32 -> bias/residual/relu -> store
  float* ep = (float*)smem;
  constexpr int LDE = BN + 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        ep[(wm * 64 + i * 16 + fg * 4 + r) * LDE + wn * 64 + j * 16 + fr] = acc[i][j][r];
  __syncthreads();
  constexpr int TPR = BN / 8;          // threads per output row (8 values each)
  constexpr int RPP = 256 / TPR;       // rows per pass
  const int c8 = (tid % TPR) * 8;
  const float4 bias0 = *(const float4*)(a.bias + n0 + c8);
  const float4 bias1 = *(const float4*)(a.bias + n0 + c8 + 4);
  const T* __restrict__ res = (const T*)a.res;
  T* __restrict__ out = (T*)a.out;
  for (int row = tid / TPR; row < BM; row += RPP) {
    const int64_t m = m0 + row;
    if (m >= a.M) break;
    const float4 v0 = *(const float4*)(ep + row * LDE + c8);
    const float4 v1 = *(const float4*)(ep + row * LDE + c8 + 4);
    float v[8] = {v0.x + bias0.x, v0.y + bias0.y, v0.z + bias0.z, v0.w + bias0.w,
                  v1.x + bias1.x, v1.y + bias1.y, v1.z + bias1.z, v1.w + bias1.w};
    if (res) {
      const T* rp = res + m * a.res_pstride + n0 + c8;
      if constexpr (sizeof(T) == 2) {
        const uint4 q = *(const uint4*)rp;
        const u16* h = (const u16*)&q;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bf2f(h[e]);
      } else {
        const float4 q0 = *(const float4*)rp, q1 = *(const float4*)(rp + 4);
        v[0] += q0.x; v[1] += q0.y; v[2] += q0.z; v[3] += q0.w;
        v[4] += q1.x; v[5] += q1.y; v[6] += q1.z; v[7] += q1.w;
      }
    }
    if (a.relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    T* op = out + m * a.out_pstride + n0 + c8;
    if constexpr (sizeof(T) == 2) {
      uint4 q;
      u16* h = (u16*)&q;
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = f2bf(v[e]);
      *(uint4*)op = q;
    } else {
      *(float4*)op = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(op + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
  }
}

// ------------------------------------------------------------------- stem --
constexpr int STEM_IMG_ROWS = 11;
constexpr int STEM_IMG_PITCH = 520;  // >= 517 columns (ix + 3 in [0, 517))

template <typename T>
__global__ __launch_bounds__(256) void stem_kernel(StemArgs a) {
  // LDS: image band f32 [11][520] | weights [64 co][64 k] (+pad) | pool [256][64] T
  constexpr int WPITCH = (64 * sizeof(T) + 16) / sizeof(T);  // elements
  __shared__ __attribute__((aligned(16))) float s_img[STEM_IMG_ROWS * STEM_IMG_PITCH];
  __shared__ __attribute__((aligned(16))) T s_w[64 * WPITCH];
  __shared__ __attribute__((aligned(16))) T s_pool[256 * 64];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int py = blockIdx.x;          // pooled row 0..127
  const int64_t b = blockIdx.y;       // image
  const float* __restrict__ map = a.map + b * a.mh * a.mw;

  // weights -> LDS (already in the per-dtype k order, see plan)
  for (int i = tid; i < 64 * 64; i += 256) s_w[(i >> 6) * WPITCH + (i & 63)] = ((const T*)a.w)[i];
  // image band rows iy = 4py-5 .. 4py+5, cols ix = -3 .. 513 (zero outside 512x512)
  const float sh = (float)a.mh / 512.f, sw = (float)a.mw / 512.f;
  for (int i = tid; i < STEM_IMG_ROWS * 517; i += 256) {
    const int tr = i / 517, tc = i - tr * 517;
    const int iy = 4 * py - 5 + tr, ix = tc - 3;
    float v = 0.f;
    if ((unsigned)iy < 512u && (unsigned)ix < 512u) {
      float fy = sh * (iy + 0.5f) - 0.5f;
      fy = fy < 0.f ? 0.f : fy;
      float fx = sw * (ix + 0.5f) - 0.5f;
      fx = fx < 0.f ? 0.f : fx;
      const int y0 = min((int)floorf(fy), a.mh - 1), x0 = min((int)floorf(fx), a.mw - 1);
      const int y1 = min(y0 + 1, a.mh - 1), x1 = min(x0 + 1, a.mw - 1);
      const float ly = fminf(fmaxf(fy - y0, 0.f), 1.f), lx = fminf(fmaxf(fx - x0, 0.f), 1.f);
      v = (1.f - ly) * ((1.f - lx) * map[y0 * a.mw + x0] + lx * map[y0 * a.mw + x1]) +
          ly * ((1.f - lx) * map[y1 * a.mw + x0] + lx * map[y1 * a.mw + x1]);
      if constexpr (sizeof(T) == 2) v = bf2f(f2bf(v));  // the bf16 path's image is bf16
    }
    s_img[tr * STEM_IMG_PITCH + tc] = v;
  }
  __syncthreads();

  // per-lane tap offsets (16 k values per lane, in the MFMA operand order)
  const int fr = lane & 15, fg = lane >> 4;
  int toff[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    int k;
    if constexpr (sizeof(T) == 2)
      k = 32 * (t >> 3) + 8 * fg + (t & 7);   // bf16 16x16x32: s = t>>3, j = t&7
    else
      k = 4 * t + fg;                        // f32 16x16x4: MFMA q = t
    toff[t] = k < 49 ? (k / 7) * STEM_IMG_PITCH + (k % 7) : -1;
  }
  // B fragments (weights), fixed for the whole workgroup
  uint4 bw[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const T* wr = s_w + (j * 16 + fr) * WPITCH;
    if constexpr (sizeof(T) == 2) {
      bw[j][0] = *(const uint4*)(wr + 8 * fg);
      bw[j][1] = *(const uint4*)(wr + 32 + 8 * fg);
    } else {
      bw[j][0] = *(const uint4*)(wr + 16 * fg);      // f32: plan stores k = 4q+g at g*16+q
      bw[j][1] = *(const uint4*)(wr + 16 * fg + 4);
    }
  }
  uint4 bw2[4][2];  // f32 only: elements 8..15 of the lane's 16
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const T* wr = s_w + (j * 16 + fr) * WPITCH;
      bw2[j][0] = *(const uint4*)(wr + 16 * fg + 8);
      bw2[j][1] = *(const uint4*)(wr + 16 * fg + 12);
    }
  }

  f32x4 vmax[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) vmax[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};  // ReLU output >= 0

  for (int d = -1; d <= 1; ++d) {
    const int cr = 2 * py + d;
    if (cr < 0 || cr >= 256) continue;  // block-uniform
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cx = wave * 64 + i * 16 + fr;
      const float* ib = s_img + (2 * d + 2) * STEM_IMG_PITCH + 2 * cx;
      float av[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) av[t] = toff[t] >= 0 ? ib[toff[t]] : 0.f;
      if constexpr (sizeof(T) == 2) {
        uint4 a0, a1;
        u16* h0 = (u16*)&a0;
        u16* h1 = (u16*)&a1;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          h0[t] = f2bf(av[t]);
          h1[t] = f2bf(av[8 + t]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          mfma_chunk<u16>(a0, bw[j][0], acc[i][j]);
          mfma_chunk<u16>(a1, bw[j][1], acc[i][j]);
        }
      } else {
        const uint4 a0 = make_uint4(__float_as_uint(av[0]), __float_as_uint(av[1]), __float_as_uint(av[2]), __float_as_uint(av[3]));
        const uint4 a1 = make_uint4(__float_as_uint(av[4]), __float_as_uint(av[5]), __float_as_uint(av[6]), __float_as_uint(av[7]));
        const uint4 a2 = make_uint4(__float_as_uint(av[8]), __float_as_uint(av[9]), __float_as_uint(av[10]), __float_as_uint(av[11]));
        const uint4 a3 = make_uint4(__float_as_uint(av[12]), __float_as_uint(av[13]), __float_as_uint(av[14]), __float_as_uint(av[15]));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          mfma_chunk<float>(a0, bw[j][0], acc[i][j]);
          mfma_chunk<float>(a1, bw[j][1], acc[i][j]);
          mfma_chunk<float>(a2, bw2[j][0], acc[i][j]);
          mfma_chunk<float>(a3, bw2[j][1], acc[i][j]);
        }
      }
    }
    // bias + ReLU + vertical max
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bj = a.bias[j * 16 + fr];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = fmaxf(acc[i][j][r] + bj, 0.f);
          if constexpr (sizeof(T) == 2) v = bf2f(f2bf(v));
          vmax[i][j][r] = fmaxf(vmax[i][j][r], v);
        }
    }
  }
  // vertical-max rows -> LDS [256 px][64 co]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int px = wave * 64 + i * 16 + fg * 4 + r;
        const float v = vmax[i][j][r];
        if constexpr (sizeof(T) == 2)
          s_pool[px * 64 + j * 16 + fr] = f2bf(v);
        else
          s_pool[px * 64 + j * 16 + fr] = v;
      }
  __syncthreads();
  // horizontal 3-wide stride-2 max, pooled q in [0,128), 8 channels per item
  T* __restrict__ out = (T*)a.out + ((b * 128 + py) * 128) * 64;
  for (int it = tid; it < 128 * 8; it += 256) {
    const int q = it >> 3, c0 = (it & 7) * 8;
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = 0.f;
    for (int px = 2 * q - 1; px <= 2 * q + 1; ++px) {
      if (px < 0 || px >= 256) continue;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v;
        if constexpr (sizeof(T) == 2)
          v = bf2f(s_pool[px * 64 + c0 + e]);
        else
          v = s_pool[px * 64 + c0 + e];
        m[e] = fmaxf(m[e], v);
      }
    }
    if constexpr (sizeof(T) == 2) {
      uint4 qv;
      u16* h = (u16*)&qv;
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = f2bf(m[e]);
      *(uint4*)(out + q * 64 + c0) = qv;
    } else {
      *(float4*)(out + q * 64 + c0) = make_float4(m[0], m[1], m[2], m[3]);
      *(float4*)(out + q * 64 + c0 + 4) = make_float4(m[4], m[5], m[6], m[7]);
    }
  }
}

// --------------------------------------------------------------- avgpool --
// [B, HW, C] (NHWC, dtype T) -> [B, C] fp32 mean over HW.
template <typename T>
__global__ __launch_bounds__(256) void avgpool_kernel(const T* __restrict__ in, int hw, int c,
                                                      float* __restrict__ out) {
  const int64_t b = blockIdx.x;
  for (int ch = threadIdx.x; ch < c; ch += blockDim.x) {
    float s = 0.f;
    const T* p = in + b * hw * c + ch;
    for (int i = 0; i < hw; ++i) {
      if constexpr (sizeof(T) == 2)
        s += bf2f(p[(int64_t)i * c]);
      else
        s += p[(int64_t)i * c];
    }
    out[b * c + ch] = s / (float)hw;
  }
}

// ---------------------------------------------------------------- launch --
template <typename T, int WM, int WN>
static int launch_conv_t(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int smem = conv_smem_bytes<WM, WN>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_igemm_kernel<T, WM, WN>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const int64_t tiles_m = (a.M + BM - 1) / BM;
  const int64_t nwg = tiles_m * (a.Cout / BN);
  SAD_REQUIRE(nwg < (1ll << 31), "grid too large");
  hipLaunchKernelGGL((conv_igemm_kernel<T, WM, WN>), dim3((unsigned)nwg), dim3(256), smem, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

int launch_conv(const ConvArgs& a, int dtype, hipStream_t s) {
  const int EPC = dtype == SAD_BF16 ? 8 : 4;
  SAD_REQUIRE(a.Cin % (8 * EPC) == 0, "Cin must be a multiple of the K-step");
  SAD_REQUIRE(a.Cout % 64 == 0, "Cout must be a multiple of 64");
  SAD_REQUIRE(a.in_pstride % EPC == 0 && a.out_pstride % 8 == 0, "pixel strides must keep 16-B alignment");
  // tile choice: 128x128 when Cout allows, else 256x64
  const bool wide = a.Cout % 128 == 0;
  if (dtype == SAD_BF16)
    return wide ? launch_conv_t<u16, 2, 2>(a, s) : launch_conv_t<u16, 4, 1>(a, s);
  return wide ? launch_conv_t<float, 2, 2>(a, s) : launch_conv_t<float, 4, 1>(a, s);
}

int launch_stem(const StemArgs& a, int dtype, hipStream_t s) {
  SAD_REQUIRE(a.B <= 65535, "stem: B > 65535");
  if (a.B == 0) return SAD_OK;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(stem_kernel<u16>, dim3(128, (unsigned)a.B), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(stem_kernel<float>, dim3(128, (unsigned)a.B), dim3(256), 0, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

int launch_avgpool(const void* in, int64_t B, int hw, int c, float* out, int dtype, hipStream_t s) {
  if (B == 0) return SAD_OK;
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(avgpool_kernel<u16>, dim3((unsigned)B), dim3(256), 0, s, (const u16*)in, hw, c, out);
  else
    hipLaunchKernelGGL(avgpool_kernel<float>, dim3((unsigned)B), dim3(256), 0, s, (const float*)in, hw, c, out);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

}  // namespace sad
