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
#include "igemm.hpp"

namespace sad {

template <int WM, int WN, int S>
constexpr int conv_smem_bytes() {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int main_b = S * (BM + BN) * 128;
  constexpr int epi_b = BM * (BN + 4) * 4;
  return main_b > epi_b ? main_b : epi_b;
}

// S = LDS ring stages (prefetch depth S-1): 3 at one workgroup per CU, 2 when
// two workgroups share a CU.
template <typename T, int WM, int WN, int S>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv_igemm_kernel(ConvArgs a) {
  static_assert(S == 2 || S == 3, "ring depth");
  constexpr int NW = WM * WN;               // waves per workgroup
  constexpr int NT = 64 * NW;               // threads
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int ES = sizeof(T);
  if (blockIdx.y > 0) {  // grouped launch: this group's operands (uniform)
    const int g = blockIdx.y;
    a.in = (const T*)a.in + g * a.in_gstride;
    a.wt = (const T*)a.wt + g * a.wt_gstride;
    a.bias = a.bias + g * a.bias_gstride;
    a.out = (T*)a.out + g * a.out_gstride;
  }
  constexpr int STAGE = (BM + BN) * 128;    // bytes per ring stage
  constexpr int QA = BM / 8 / NW;           // A LDS-DMA wave-instructions per wave per K-step
  constexpr int QB = BN / 8 / NW;           // B ...
  static_assert(QA * 8 * NW == BM && QB * 8 * NW == BN, "tile/wave mismatch");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int n_tn = a.Cout / BN;
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = wg % n_tn, tm = wg / n_tn;
  const int64_t m0 = (int64_t)tm * BM;
  const int n0 = tn * BN;
  const int HoWo = a.Ho * a.Wo;

  // Buffer resources: 32-bit byte offsets; an offset past num_records reads 0,
  // which implements the conv zero padding without branches.
  const __amdgpu_buffer_rsrc_t rin =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in, (short)0, (int)a.in_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwt =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int pstride_b = (int)a.in_pstride * ES;

  // LDS-DMA writes lane-linearly (dest = wave base + 16*lane), so the XOR
  // swizzle is applied on the SOURCE: lane L of the wave-instruction that fills
  // rows 8q..8q+7 loads chunk (L&7) ^ swzkey(row) of row 8q + (L>>3).
  const int lrow = lane >> 3;
  // A rows of this lane: q = wave + NW*i, row = 8q + lrow
  int aoff[QA], aiy[QA], aix[QA];
#pragma unroll
  for (int i = 0; i < QA; ++i) {
    const int r = 8 * (wave + NW * i) + lrow;
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int64_t m = m0 + r;
    if (m < a.M) {
      const int b = (int)(m / HoWo);
      const int rem = (int)(m - (int64_t)b * HoWo);
      const int oy = rem / a.Wo, ox = rem - oy * a.Wo;
      aiy[i] = oy * a.stride - a.pad;
      aix[i] = ox * a.stride - a.pad;
      aoff[i] = ((b * a.H + aiy[i]) * a.W + aix[i]) * pstride_b + c * 16;
    } else {
      aiy[i] = -0x4000;
      aix[i] = -0x4000;
      aoff[i] = 0;
    }
  }
  const int ktot_b = a.KH * a.KW * a.Cin * ES;
  int boff[QB];
#pragma unroll
  for (int i = 0; i < QB; ++i) {
    const int r = 8 * (wave + NW * i) + lrow;           // row within the B tile
    const int c = (lane & 7) ^ (((r + BM) >> 1) & 7);   // swizzle key of LDS row BM + r
    boff[i] = (n0 + r) * ktot_b + c * 16;
  }
  const int cpt = a.Cin / (128 / ES);
  const int nk = a.KH * a.KW * cpt;

  // LDS byte address of the ring (M0 operand of the DMA)
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // Issue the LDS-DMA for K-step ks into ring stage st.  Inline asm keeps the
  // DMA out of hipcc's vmcnt bookkeeping (which would otherwise drain it with
  // vmcnt(0) before the next ds_read); the loop counts vmcnt by hand.
  auto issue = [&](int ks, int st) __attribute__((always_inline)) {
    const int tap = ks / cpt;
    const int ci0 = ks - tap * cpt;
    const int ky = tap / a.KW, kx = tap - ky * a.KW;
    const int toff = (ky * a.W + kx) * pstride_b + ci0 * 128;
    const unsigned sb = lds0 + st * STAGE;
#pragma unroll
    for (int i = 0; i < QA; ++i) {
      const int iy = aiy[i] + ky, ix = aix[i] + kx;
      const bool ok = ((unsigned)iy < (unsigned)a.H) && ((unsigned)ix < (unsigned)a.W);
      dma16(rin, ok ? aoff[i] + toff : 0x7FFFFFF0, sb + (wave + NW * i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < QB; ++i) dma16(rwt, boff[i] + ks * 128, sb + BM * 128 + (wave + NW * i) * 1024);
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  issue(0, 0);
  if (S == 3 && nk > 1) issue(1, 1);
  int st = 0;
  for (int ks = 0; ks < nk; ++ks) {
    // retire this wave's DMA for step ks (with S = 3, step ks+1's stays in
    // flight), then the barrier publishes every wave's step-ks DMA and frees
    // the stage the next issue overwrites (read by step ks-1)
    if (S == 3 && ks + 1 < nk)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QA + QB) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (ks + S - 1 < nk) issue(ks + S - 1, S == 3 ? (st == 0 ? 2 : st - 1) : (st ^ 1));
    const char* base = smem + st * STAGE;
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
    st = st + 1 == S ? 0 : st + 1;
  }
  __syncthreads();

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
  constexpr int RPP = NT / TPR;        // rows per pass
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
// torchvision Resize((512,512)) sample (bilinear, align_corners=False; the
// antialias filter is a no-op for this upsample) of an mh x mw map at (iy, ix).
__device__ __forceinline__ float bilinear512(const float* __restrict__ map, int mh, int mw, float sh, float sw,
                                            int iy, int ix) {
  float fy = sh * (iy + 0.5f) - 0.5f;
  fy = fy < 0.f ? 0.f : fy;
  float fx = sw * (ix + 0.5f) - 0.5f;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = min((int)floorf(fy), mh - 1), x0 = min((int)floorf(fx), mw - 1);
  const int y1 = min(y0 + 1, mh - 1), x1 = min(x0 + 1, mw - 1);
  const float ly = fminf(fmaxf(fy - y0, 0.f), 1.f), lx = fminf(fmaxf(fx - x0, 0.f), 1.f);
  return (1.f - ly) * ((1.f - lx) * map[y0 * mw + x0] + lx * map[y0 * mw + x1]) +
         ly * ((1.f - lx) * map[y1 * mw + x0] + lx * map[y1 * mw + x1]);
}

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
  const float* __restrict__ map = a.img ? nullptr : a.map + b * a.mh * a.mw;

  // weights -> LDS (already in the per-dtype k order, see plan)
  for (int i = tid; i < 64 * 64; i += 256) s_w[(i >> 6) * WPITCH + (i & 63)] = ((const T*)a.w)[i];
  // image band rows iy = 4py-5 .. 4py+5, cols ix = -3 .. 513 (zero outside 512x512)
  const float sh = (float)a.mh / 512.f, sw = (float)a.mw / 512.f;
  for (int i = tid; i < STEM_IMG_ROWS * 517; i += 256) {
    const int tr = i / 517, tc = i - tr * 517;
    const int iy = 4 * py - 5 + tr, ix = tc - 3;
    float v = 0.f;
    if ((unsigned)iy < 512u && (unsigned)ix < 512u) {
      v = a.img ? a.img[(b * 512 + iy) * 512 + ix] : bilinear512(map, a.mh, a.mw, sh, sw, iy, ix);
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

// ------------------------------------------------------------ stem, bf16 --
// Throughput-mode stem: conv1 7x7/2 (BN folded, 3 identical input channels
// folded into one) -> ReLU -> maxpool 3x3/2, one launch (inference_runner.py:
// 49-51 via timm resnet18 conv1/bn1/act1/maxpool).
//
// K is laid out (ky, kx) on an 8 x 8 grid (ky = 7 and kx = 7 carry zero
// weights), so the 8 consecutive k of one MFMA fragment are 8 consecutive
// image pixels of ONE row: 4 x ds_read_b32 from a bf16 image band (row pitch
// 272 dwords = 16 banks mod 32: conflict-free).  Operands are swapped
// (C = W . img^T): a lane holds 4 consecutive channels of one conv pixel.
//
// A workgroup produces STEM_P pooled rows (conv rows 2*py0-1 .. 2*(py0+P)-1).
// Max-pool runs on the raw accumulators -- bias and ReLU are monotonic, so
// relu(max(x) + b) == max(relu(x + b)) and rounding once to bf16 after the
// pool equals rounding before it: vertical max in registers, horizontal max by
// DPP row shifts (lane fr <- fr +- 1 within a 16-pixel block, block edges by
// row_shl:15, wave edges through LDS).  The resize is separable: map rows are
// x-interpolated once per workgroup into LDS, then each band pixel is one
// y-lerp (same arithmetic as bilinear512).
constexpr int STEM_P = 8;
constexpr int STEM_BAND_ROWS = 4 * STEM_P + 8;  // 4P+7 with non-zero weights
constexpr int STEM_BPITCH = 544;                 // bf16 elements per band row (>= 518)
constexpr int STEM_HROWS = 12;                   // x-interpolated map rows kept in LDS (>= 4P+8 image rows at 128/512)
constexpr int STEM_UPITCH = 520;                 // floats per x-interpolated row, indexed by band column
                                                 // (>= 518 read; zero outside the image)
constexpr int STEM_OPITCH = 128;                 // staging bytes per pooled pixel (64 ch bf16), 16-B
                                                 // chunk c of pixel q at c ^ stem_oswz(q)
constexpr int STEM_WPITCH = 80;                  // bf16 per weight row in LDS (64 + pad): the
                                                 // fragment reads are conflict-free (72: 2-way)
// pooled-row staging swizzle (bf16 stems): chunk c of pixel q at c ^ g(q), g =
// 0, 4, 2, 6 for q mod 4 -- the b32 stores of a 32-lane group (4 pixels x 2
// chunks) and the b128 row copy-out are both conflict-free (a padded pitch
// cannot do both: 160 B gave 3-way reads)
__device__ __forceinline__ int stem_oswz(int q) { return ((q & 1) << 2) | (q & 2); }

// two floats -> packed bf16 pair (RNE): one v_cvt_pk_bf16_f32
typedef __bf16 stem_bf2 __attribute__((ext_vector_type(2)));
typedef float stem_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t stem_pk(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((stem_f2){lo, hi}, stem_bf2));
}
// ReLU of a packed bf16 pair (as int16 negative bf16 values are negative)
__device__ __forceinline__ uint32_t stem_relu2(uint32_t x) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
  return r;
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
}

// X3 (split-bf16 parity mode, SAD_BF16X3): the band is kept as hi and lo bf16
// planes, the weights as hi and lo, each product is W_hi.X_hi + W_lo.X_hi +
// W_hi.X_lo, and the pooled output is stored split ([hi 32 | lo 32] per 32
// channels; one workgroup per CU for the larger LDS footprint).  X4 adds
// W_lo.X_lo (the deep Bottleneck plans, resnet.hip).
constexpr int STEM_OPITCH_X3 = 288;  // 128 bf16 (64 ch hi + lo) + pad: 72 dwords -> 4 rows on disjoint bank sets
// s_u holds, while the band is built, the x-interpolated rows + a zero row +
// the [NBR] row table; afterwards the pooled-row staging + the wave-edge exchange
constexpr int stem_u_build_floats() { return (STEM_HROWS + 1) * STEM_UPITCH + 4 * STEM_BAND_ROWS; }
template <bool X3>
constexpr int stem_u_floats() {
  return (X3 ? 128 * STEM_OPITCH_X3 / 4 : 128 * STEM_OPITCH / 4) + 256 > stem_u_build_floats()
             ? (X3 ? 128 * STEM_OPITCH_X3 / 4 : 128 * STEM_OPITCH / 4) + 256
             : stem_u_build_floats();
}

// TRAIN (the trainer's bf16 stem, submodel_trainer.py:250-255 in model.train()):
// bn1 normalises with the BATCH statistics of the raw conv, so nothing can be
// folded before the pass.  The kernel reads the bf16 training image, computes
// the raw conv y, and max-pools y' = sign(gamma_c) * y (bias and ReLU skipped):
// with scale = gamma * invstd, sign(gamma) * scale >= 0, so maxpool(relu(bn(y)))
// == relu(|scale| * maxpool(y') + shift) exactly, applied afterwards by
// pooled_bn_relu_kernel (train.hip).  Alongside, every conv row this workgroup
// owns (2*py0 .. 2*py0 + 2P - 1; the carry-in row belongs to the previous one)
// feeds per-channel sums of y and y^2 -> a.part[workgroup][2][64] (the
// bn_reduce_kernel partial format) for the batch statistics.
template <bool X3, bool TRAIN = false, bool X4 = false>
__global__ __launch_bounds__(256, X3 ? 1 : 2) void stem_bf16_kernel(StemArgs a) {
  static_assert(!(X3 && TRAIN), "the training stem is bf16");
  static_assert(!X4 || X3, "X4: the split stem's fourth product");
  constexpr int OPITCH = X3 ? STEM_OPITCH_X3 : STEM_OPITCH;
  __shared__ __attribute__((aligned(16))) u16 s_img[STEM_BAND_ROWS * STEM_BPITCH];
  __shared__ __attribute__((aligned(16))) u16 s_imgl[X3 ? STEM_BAND_ROWS * STEM_BPITCH : 8];
  __shared__ __attribute__((aligned(16))) u16 s_w[64 * STEM_WPITCH];
  __shared__ __attribute__((aligned(16))) u16 s_wl[X3 ? 64 * STEM_WPITCH : 8];
  __shared__ __attribute__((aligned(16))) float s_bias[64];
  // x-interpolated map rows while the band is built; afterwards the pooled-row
  // staging [128 q][64 ch] bf16 (X3: hi + lo) and the wave-edge exchange [4][64] fp32
  __shared__ __attribute__((aligned(16))) float s_u[stem_u_floats<X3>()];
  char* s_out = (char*)s_u;                  // pooled row staging, [128 q][OPITCH B]
  float* s_edge = s_u + 128 * OPITCH / 4;    // [4 waves][64 ch]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int py0 = blockIdx.x * STEM_P;
  const int64_t b = blockIdx.y;
  for (int i = tid; i < 64 * 8; i += 256) {  // [64 co][64 k] bf16 -> pitch STEM_WPITCH
    const int co = i >> 3, c8 = (i & 7) * 8;
    uint4 wv = *(const uint4*)((const u16*)a.w + co * 64 + c8);
    if (TRAIN && a.bias[co] < 0.f) wv ^= make_uint4(0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u);  // y' = -y
    *(uint4*)(s_w + co * STEM_WPITCH + c8) = wv;
    if constexpr (X3)
      *(uint4*)(s_wl + co * STEM_WPITCH + c8) = *(const uint4*)((const u16*)a.w + 64 * 64 + co * 64 + c8);
  }
  // band element store: bf16, or the hi/lo pair
  auto put = [&](int i, float v) __attribute__((always_inline)) {
    const u16 h = f2bf(v);
    s_img[i] = h;
    if constexpr (X3) s_imgl[i] = f2bf(v - bf2f(h));
  };
  if (tid < 64) s_bias[tid] = TRAIN ? (a.bias[tid] < 0.f ? -1.f : 1.f) : a.bias[tid];
  // ---- image band: rows iy = 4*py0 - 5 + tr, cols ix = tc - 3 (zero outside 512x512)
  // every band row a fragment reads, incl. the zero-weight tap row ky = 7
  // (uninitialised LDS could hold NaN, and NaN * 0 is NaN)
  constexpr int NBR = STEM_BAND_ROWS;
  if (TRAIN) {
    for (int i = tid; i < NBR * STEM_BPITCH; i += 256) {
      const int tr = i / STEM_BPITCH, tc = i - tr * STEM_BPITCH;
      const int iy = 4 * py0 - 5 + tr, ix = tc - 3;
      u16 v = 0;
      if ((unsigned)iy < 512u && (unsigned)ix < 512u) v = a.img16[(b * 512 + iy) * 512 + ix];
      s_img[i] = v;
    }
  } else if (a.img) {
    for (int i = tid; i < NBR * STEM_BPITCH; i += 256) {
      const int tr = i / STEM_BPITCH, tc = i - tr * STEM_BPITCH;
      const int iy = 4 * py0 - 5 + tr, ix = tc - 3;
      float v = 0.f;
      if ((unsigned)iy < 512u && (unsigned)ix < 512u) v = a.img[(b * 512 + iy) * 512 + ix];
      put(i, v);
    }
  } else {
    const float* __restrict__ map = a.map + b * a.mh * a.mw;
    const float sh = (float)a.mh / 512.f, sw = (float)a.mw / 512.f;
    auto src_row = [&](int iy, int& y0, int& y1, float& ly) {
      float fy = sh * (iy + 0.5f) - 0.5f;
      fy = fy < 0.f ? 0.f : fy;
      y0 = min((int)floorf(fy), a.mh - 1);
      y1 = min(y0 + 1, a.mh - 1);
      ly = fminf(fmaxf(fy - y0, 0.f), 1.f);
    };
    const int iy_lo = max(4 * py0 - 5, 0), iy_hi = min(4 * py0 - 5 + NBR - 1, 511);
    int ylo, yhi, t0, t1;
    float tl;
    src_row(iy_lo, ylo, t0, tl);
    src_row(iy_hi, t1, yhi, tl);
    const int nh = yhi - ylo + 1;
    if (nh <= STEM_HROWS) {
      // separable resize in two vector passes.  (1) x-lerp of map rows
      // ylo..yhi into s_u, indexed by BAND column tc = ix + 3 (zero outside
      // the image): a thread owns image columns tid and tid + 256 and issues
      // all its rows' gathers before the first use (one memory latency per
      // workgroup).  (2) y-lerp of 4 band columns per item from a per-row table
      // (source-row offsets and weights; rows outside the image point at a zero
      // row), so the band costs 2 ds_read_b128 + 8 VALU + one 8-B store per 4
      // pixels instead of the per-pixel index arithmetic
      constexpr int UP = STEM_UPITCH;
      float* s_zero = s_u + STEM_HROWS * UP;
      int4* s_rt = (int4*)(s_u + (STEM_HROWS + 1) * UP);
      int x0[2], x1[2];
      float lx[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int ix = tid + 256 * c;
        float fx = sw * (ix + 0.5f) - 0.5f;
        fx = fx < 0.f ? 0.f : fx;
        x0[c] = min((int)floorf(fx), a.mw - 1);
        x1[c] = min(x0[c] + 1, a.mw - 1);
        lx[c] = fminf(fmaxf(fx - x0[c], 0.f), 1.f);
      }
      float g0[STEM_HROWS][2], g1[STEM_HROWS][2];
#pragma unroll
      for (int r = 0; r < STEM_HROWS; ++r) {
        const float* mr = map + (ylo + min(r, nh - 1)) * a.mw;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          g0[r][c] = mr[x0[c]];
          g1[r][c] = mr[x1[c]];
        }
      }
#pragma unroll
      for (int r = 0; r < STEM_HROWS; ++r)
        if (r < nh) {
#pragma unroll
          for (int c = 0; c < 2; ++c) s_u[r * UP + 3 + tid + 256 * c] = (1.f - lx[c]) * g0[r][c] + lx[c] * g1[r][c];
        }
      // band columns outside the image (tc 0..2 and 515..519) of every row, the zero row
      if (tid < STEM_HROWS * 8) {
        const int r = tid >> 3, k = tid & 7;
        s_u[r * UP + (k < 3 ? k : 512 + k)] = 0.f;
      }
      for (int i = tid; i < UP; i += 256) s_zero[i] = 0.f;
      if (tid < NBR) {
        const int iy = 4 * py0 - 5 + tid;
        int4 rt = make_int4(STEM_HROWS * UP, STEM_HROWS * UP, __float_as_int(1.f), __float_as_int(0.f));
        if ((unsigned)iy < 512u) {
          int y0, y1;
          float ly;
          src_row(iy, y0, y1, ly);
          rt = make_int4((y0 - ylo) * UP, (y1 - ylo) * UP, __float_as_int(1.f - ly), __float_as_int(ly));
        }
        s_rt[tid] = rt;
      }
      __syncthreads();
      constexpr int QPR = (2 * 255 + 8 + 3) / 4;  // 4-column quads per band row that fragments read (tc < 518)
      static_assert(4 * QPR <= UP && 4 * QPR <= STEM_BPITCH, "band quads");
#pragma unroll 2
      for (int it = tid; it < NBR * QPR; it += 256) {
        const int tr = it / QPR, q = it - tr * QPR;
        const int4 rt = s_rt[tr];
        const float w0 = __int_as_float(rt.z), w1 = __int_as_float(rt.w);
        const float4 u0 = *(const float4*)(s_u + rt.x + 4 * q);
        const float4 u1 = *(const float4*)(s_u + rt.y + 4 * q);
        const float v[4] = {w0 * u0.x + w1 * u1.x, w0 * u0.y + w1 * u1.y, w0 * u0.z + w1 * u1.z,
                            w0 * u0.w + w1 * u1.w};
        u16 h[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) h[e] = f2bf(v[e]);
        const int o = tr * STEM_BPITCH + 4 * q;
        *(uint2*)(s_img + o) = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
        if constexpr (X3) {
          u16 l[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) l[e] = f2bf(v[e] - bf2f(h[e]));
          *(uint2*)(s_imgl + o) =
              make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
        }
      }
    } else {  // very tall maps: direct bilinear per pixel
      for (int i = tid; i < NBR * STEM_BPITCH; i += 256) {
        const int tr = i / STEM_BPITCH, tc = i - tr * STEM_BPITCH;
        const int iy = 4 * py0 - 5 + tr, ix = tc - 3;
        float v = 0.f;
        if ((unsigned)iy < 512u && (unsigned)ix < 512u) v = bilinear512(map, a.mh, a.mw, sh, sw, iy, ix);
        put(i, v);
      }
    }
  }
  __syncthreads();  // band complete; s_u is free from here on

  const int fr = lane & 15, fg = lane >> 4;

  // raw conv row cr for this wave's 64 conv columns: r[i][j] = C[ch j*16+fg*4+e][px 64w+16i+fr]
  // (cr >= 0: only the first workgroup's carry-in row, conv row -1, lies above
  // the image; the caller fills it with -inf, which never wins the max)
  auto conv_row = [&](int cr, f32x4 (&r)[4][4]) __attribute__((always_inline)) {
    // accumulators start at zero (the MFMA's inline-constant C operand: no
    // register copies); the bias goes in after the max-pool (relu(max(x) + b)
    // == max(relu(x + b)))
    const f32x4 init[4] = {};
    const int rb = 2 * (cr - 2 * py0) + 2;
    uint4 bw[4][2];  // weight fragments (LDS-resident; re-read per row keeps VGPRs for the pool)
    uint4 bwl[X3 ? 4 : 1][2];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bw[j][s] = *(const uint4*)(s_w + (j * 16 + fr) * STEM_WPITCH + 32 * s + 8 * fg);
        if constexpr (X3) bwl[j][s] = *(const uint4*)(s_wl + (j * 16 + fr) * STEM_WPITCH + 32 * s + 8 * fg);
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cx = wave * 64 + i * 16 + fr;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int o = (rb + 4 * s + fg) * STEM_BPITCH + 2 * cx;
        const u16* p = s_img + o;
        uint4 av;
        av.x = *(const uint32_t*)(p + 0);
        av.y = *(const uint32_t*)(p + 2);
        av.z = *(const uint32_t*)(p + 4);
        av.w = *(const uint32_t*)(p + 6);
#pragma unroll
        for (int j = 0; j < 4; ++j)  // C[px][ch]
          r[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                            __builtin_bit_cast(bf16x8, bw[j][s]),
                                                            s == 0 ? init[j] : r[i][j], 0, 0, 0);
        if constexpr (X3) {
          const u16* pl = s_imgl + o;
          uint4 al;
          al.x = *(const uint32_t*)(pl + 0);
          al.y = *(const uint32_t*)(pl + 2);
          al.z = *(const uint32_t*)(pl + 4);
          al.w = *(const uint32_t*)(pl + 6);
          // product-outer: 4 independent accumulators between dependent MFMAs
#pragma unroll
          for (int j = 0; j < 4; ++j) mfma_chunk<u16>(av, bwl[j][s], r[i][j]);  // X_hi . W_lo
#pragma unroll
          for (int j = 0; j < 4; ++j) mfma_chunk<u16>(al, bw[j][s], r[i][j]);   // X_lo . W_hi
          if constexpr (X4) {
#pragma unroll
            for (int j = 0; j < 4; ++j) mfma_chunk<u16>(al, bwl[j][s], r[i][j]);  // X_lo . W_lo
          }
        }
      }
    }
  };

  // TRAIN: the conv rows of the image (y', sign folded into s_w) feed the statistics
  float st_s[4] = {0.f, 0.f, 0.f, 0.f}, st_q[4] = {0.f, 0.f, 0.f, 0.f};
  auto train_row = [&](const f32x4 (&r)[4][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          st_s[j] += r[i][j][e];
          st_q[j] += r[i][j][e] * r[i][j][e];
        }
  };
  // conv row 2py+1 is the next pooled row's first: two carry sets alternate
  // (pooled rows in pairs), so the carried row needs no register copies
  f32x4 ca[4][4], cb[4][4], cur[4][4];
  if (py0 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) ca[i][j] = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  } else {
    conv_row(2 * py0 - 1, ca);
  }
  // the vertical max as one v_med3_f32 (x, y, +inf) = max(x, y): fmaxf would
  // first canonicalise each MFMA result (two more VALU per value), and an
  // inline-asm v_max would escape the compiler's MFMA result-hazard waits; no
  // NaN reaches it.  (The training stem keeps fmaxf: with its statistics the
  // med3 form spills.)
  auto vmax = [](float x, float y) __attribute__((always_inline)) {
    if constexpr (TRAIN) return fmaxf(x, y);
    return __builtin_amdgcn_fmed3f(x, y, INFINITY);
  };
  auto pooled_row = [&](int pi, f32x4 (&carry)[4][4], f32x4 (&next)[4][4]) __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);  // the two rows of a pair do not interleave (register pressure)
    const int py = py0 + pi;
    // vertical max over conv rows 2py-1 (carry), 2py, 2py+1 (next)
    conv_row(2 * py, cur);
    if (TRAIN) train_row(cur);
    // max with the carried row BEFORE the next row's MFMAs, so the carried row
    // is dead during them (a fused 3-way max after them kept all three rows
    // live: 254 VGPRs and register copies)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int e = 0; e < 4; ++e) cur[i][j][e] = vmax(carry[i][j][e], cur[i][j][e]);
      }
    conv_row(2 * py + 1, next);
    if (TRAIN) train_row(next);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) cur[i][j][e] = vmax(cur[i][j][e], next[i][j][e]);
    // wave edge: conv column 64w-1 comes from wave w-1 (tile 3, lanes fg = 3, element 3)
    if (fg == 3) {
#pragma unroll
      for (int j = 0; j < 4; ++j) s_edge[wave * 64 + j * 16 + fr] = cur[3][j][3];
    }
    __syncthreads();
    // horizontal max, window 3 stride 2.  Lane (fr, fg) of tile i holds conv
    // columns 64w+16i+4fg+e of channel 16j+fr (C[px][ch] layout), so its pooled
    // outputs q = 32w+8i+2fg (columns 4fg-1..4fg+1) and q+1 (4fg+1..4fg+3) are
    // in-lane except column 4fg-1: element 3 of lane (fr, fg-1), or of tile
    // i-1's lane (fr, 3), or of wave w-1 -- one bpermute rotating the wave by
    // 16 lanes.  Then bias, ReLU, and channel pairs (fr, fr+1) packed by a DPP
    // row shift: even lanes write pooled q, odd lanes q+1, as b32.
    float bias[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bias[j] = s_bias[j * 16 + fr];
    const bool even = (fr & 1) == 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 x = cur[i][j];
        const float send = fg == 3 ? (i > 0 ? cur[i - 1][j][3] : 0.f) : x[3];
        float left = __int_as_float(__builtin_amdgcn_ds_bpermute(((lane + 48) & 63) << 2, __float_as_int(send)));
        if (i == 0 && fg == 0) left = wave > 0 ? s_edge[(wave - 1) * 64 + j * 16 + fr] : -INFINITY;
        if constexpr (!X3 && !TRAIN) {
          // pooled pixels q0 = 32w+8i+2fg and q0 + 1 of channel c = 16j + fr,
          // plus the bias, packed as one bf16 pair, ReLU on the
          // pair (int16 max), then lanes (c, c^1) trade pairs (one DPP) and a
          // byte permute forms (c0, c0+1) of q0 (even lanes) / q0+1 (odd)
          const uint32_t pq = stem_relu2(stem_pk(fmaxf(fmaxf(left, x[0]), x[1]) + bias[j],
                                                 fmaxf(fmaxf(x[1], x[2]), x[3]) + bias[j]));
          const uint32_t pn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pq, 0xB1, 0xF, 0xF, true);  // quad_perm 1,0,3,2
          const uint32_t w = __builtin_amdgcn_perm(pn, pq, even ? 0x05040100u : 0x03020706u);
          const int q = wave * 32 + i * 8 + 2 * fg + (even ? 0 : 1);
          const int bo = (j * 16 + (fr & ~1)) * 2;  // byte in the pixel: chunk j * 2 + (fr >> 3)
          *(uint32_t*)(s_out + q * OPITCH + ((((bo >> 4) ^ stem_oswz(q)) << 4) | (bo & 15))) = w;
          continue;
        }
        const float oa = TRAIN ? fmaxf(fmaxf(left, x[0]), x[1]) : fmaxf(fmaxf(fmaxf(left, x[0]), x[1]) + bias[j], 0.f);
        const float ob = TRAIN ? fmaxf(fmaxf(x[1], x[2]), x[3]) : fmaxf(fmaxf(fmaxf(x[1], x[2]), x[3]) + bias[j], 0.f);
        const float oa_next = dppf<0x101>(oa);  // row_shl:1 (fr + 1)
        const float ob_prev = dppf<0x111>(ob);  // row_shr:1 (fr - 1)
        // c0 = channel fr & ~1 (value v0), c0 + 1 (value v1) of pooled pixel q
        const float v0 = even ? oa : ob_prev, v1 = even ? oa_next : ob;
        const int q = wave * 32 + i * 8 + 2 * fg + (even ? 0 : 1);
        const int c0 = j * 16 + (fr & ~1);
        const u16 h0 = f2bf(v0), h1 = f2bf(v1);
        if constexpr (X3) {
          const int pc = ((c0 >> 5) << 6) + (c0 & 31);
          *(uint32_t*)(s_out + q * OPITCH + pc * 2) = (uint32_t)h0 | ((uint32_t)h1 << 16);
          *(uint32_t*)(s_out + q * OPITCH + pc * 2 + 64) =
              (uint32_t)f2bf(v0 - bf2f(h0)) | ((uint32_t)f2bf(v1 - bf2f(h1)) << 16);
        } else {
          const int bo = c0 * 2;
          *(uint32_t*)(s_out + q * OPITCH + ((((bo >> 4) ^ stem_oswz(q)) << 4) | (bo & 15))) =
              (uint32_t)h0 | ((uint32_t)h1 << 16);
        }
      }
    }
    __syncthreads();
    constexpr int PXE = X3 ? 128 : 64;  // bf16 elements per pooled pixel
    u16* __restrict__ out = (u16*)a.out + ((b * 128 + py) * 128) * PXE;
#pragma unroll
    for (int k = 0; k < PXE / 16; ++k) {
      const int idx = (k * 256 + tid) * 8;  // 16 (X3: 32) KB row, 16 B per thread per k
      const int px = idx / PXE, c = (idx % PXE) / 8;  // pooled pixel, 16-B chunk
      *(uint4*)(out + idx) = *(const uint4*)(s_out + px * OPITCH + ((X3 ? c : c ^ stem_oswz(px)) << 4));
    }
    __syncthreads();
  };
  static_assert(STEM_P % 2 == 0, "pooled rows in pairs");
  if constexpr (TRAIN) {  // (the statistics' registers: one row per iteration, the carry copied)
    for (int pi = 0; pi < STEM_P; ++pi) {
      pooled_row(pi, ca, cb);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) ca[i][j] = cb[i][j];
    }
  } else {
    for (int pi = 0; pi < STEM_P; pi += 2) {
      pooled_row(pi, ca, cb);
      pooled_row(pi + 1, cb, ca);
    }
  }
  if constexpr (TRAIN) {
    // lanes (fr, fg = 0..3) share channels 16j + fr: fold fg, then the 4 waves
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      st_s[j] += __shfl_xor(st_s[j], 16, 64);
      st_s[j] += __shfl_xor(st_s[j], 32, 64);
      st_q[j] += __shfl_xor(st_q[j], 16, 64);
      st_q[j] += __shfl_xor(st_q[j], 32, 64);
    }
    float* red = s_u;  // [4 waves][2][64]
    if (fg == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        red[wave * 128 + j * 16 + fr] = st_s[j];
        red[wave * 128 + 64 + j * 16 + fr] = st_q[j];
      }
    }
    __syncthreads();
    if (tid < 128) {
      const float v = (red[tid] + red[128 + tid]) + (red[256 + tid] + red[384 + tid]);
      // sums of y = sign * y' (the sign is its own inverse); squares are sign-free
      a.part[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 128 + tid] = tid < 64 ? v * s_bias[tid] : v;
    }
  }
}

// ------------------------------------------------- stem, distinct channels --
// conv1 7x7/2 p3 over 3 DISTINCT input channels (BN scale folded) + bias +
// ReLU + maxpool 3x3/2 p1, fp32 arithmetic, output in the plan dtype.  The
// reference's model accepts any [B,3,512,512] tensor (its load-time check feeds
// torch.randn(2,3,512,512), inference_runner.py:119-122, model_merger.py:
// 148-151); the spectrogram path's three channels are identical and take the
// folded MFMA stems above.  Not the hot path: one workgroup per pooled row,
// one thread per pooled pixel, weights broadcast from LDS.
// OUT: 0 fp32, 1 bf16, 2 split-bf16 ([hi 32 | lo 32] per 32 channels)
constexpr int STEM3_PITCH = 520;  // band columns ix + 5 in [0, 519)
template <int OUT>
__global__ __launch_bounds__(128) void stem3_kernel(StemArgs a) {
  __shared__ float s_band[3 * STEM_IMG_ROWS * STEM3_PITCH];
  __shared__ __attribute__((aligned(16))) float s_w[64 * 148];
  const int tid = threadIdx.x;
  const int py = blockIdx.x;
  const int64_t b = blockIdx.y;
  for (int i = tid; i < 64 * 147; i += 128) s_w[(i / 147) * 148 + i % 147] = a.w3[i];
  const float* img = a.img3 + b * 3 * 512 * 512;
  for (int i = tid; i < 3 * STEM_IMG_ROWS * STEM3_PITCH; i += 128) {
    const int c = i / (STEM_IMG_ROWS * STEM3_PITCH), r = i % (STEM_IMG_ROWS * STEM3_PITCH);
    const int tr = r / STEM3_PITCH, tc = r % STEM3_PITCH;
    const int iy = 4 * py - 5 + tr, ix = tc - 5;
    s_band[i] = ((unsigned)iy < 512u && (unsigned)ix < 512u) ? img[((int64_t)c * 512 + iy) * 512 + ix] : 0.f;
  }
  __syncthreads();
  const int px = tid;
  float pooled[64];
#pragma unroll
  for (int j = 0; j < 64; ++j) pooled[j] = 0.f;  // ReLU outputs are >= 0
  for (int g = 0; g < 4; ++g) {
    float best[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) best[j] = 0.f;
    for (int dy = -1; dy <= 1; ++dy) {
      const int cy = 2 * py + dy;
      if (cy < 0 || cy >= 256) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int cx = 2 * px + dx;
        if (cx < 0 || cx >= 256) continue;
        float acc[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = a.bias[g * 16 + j];
        for (int c = 0; c < 3; ++c)
          for (int ky = 0; ky < 7; ++ky) {
            // band row of image row 2cy - 3 + ky; column 2cx - 3 + kx (+5)
            const float* br = s_band + (c * STEM_IMG_ROWS + (2 * cy - 3 + ky) - (4 * py - 5)) * STEM3_PITCH + 2 * cx + 2;
            for (int kx = 0; kx < 7; ++kx) {
              const float v = br[kx];
              const float* wr = s_w + (g * 16) * 148 + c * 49 + ky * 7 + kx;
#pragma unroll
              for (int j = 0; j < 16; ++j) acc[j] = fmaf(v, wr[j * 148], acc[j]);
            }
          }
#pragma unroll
        for (int j = 0; j < 16; ++j) best[j] = fmaxf(best[j], acc[j]);  // relu folded into the 0 init
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) pooled[g * 16 + j] = best[j];
  }
  const int64_t pix = (b * 128 + py) * 128 + px;
  if constexpr (OUT == 0) {
    float* o = (float*)a.out + pix * 64;
#pragma unroll
    for (int j = 0; j < 64; j += 4) *(float4*)(o + j) = make_float4(pooled[j], pooled[j + 1], pooled[j + 2], pooled[j + 3]);
  } else if constexpr (OUT == 1) {
    u16* o = (u16*)a.out + pix * 64;
#pragma unroll
    for (int j = 0; j < 64; ++j) o[j] = f2bf(pooled[j]);
  } else {
    u16* o = (u16*)a.out + pix * 128;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const u16 h = f2bf(pooled[j]);
      o[(j >> 5) * 64 + (j & 31)] = h;
      o[(j >> 5) * 64 + 32 + (j & 31)] = f2bf(pooled[j] - bf2f(h));
    }
  }
}

// --------------------------------------------------------------- avgpool --
// [B, HW, C] (NHWC, dtype T) -> [B, C] fp32 mean over HW.  Workgroup = one
// segment x 64 channels; 4 waves split the pixels, LDS combine.
// X3: split-bf16 input ([hi 32 | lo 32] per 32 channels, 2c bf16 per pixel).
template <typename T, bool X3 = false>
__global__ __launch_bounds__(256) void avgpool_kernel(const T* __restrict__ in, int hw, int c,
                                                      float* __restrict__ out) {
  __shared__ float part[4][64];
  const int64_t b = blockIdx.x;
  const int ch = blockIdx.y * 64 + (threadIdx.x & 63), g = threadIdx.x >> 6;
  const int pc = X3 ? ((ch >> 5) << 6) + (ch & 31) : ch;
  const int ps = X3 ? 2 * c : c;
  const T* p = in + b * hw * ps + pc;
  float s = 0.f;
  for (int i = g; i < hw; i += 4) {
    if constexpr (X3)
      s += bf2f(p[(int64_t)i * ps]) + bf2f(p[(int64_t)i * ps + 32]);
    else if constexpr (sizeof(T) == 2)
      s += bf2f(p[(int64_t)i * c]);
    else
      s += p[(int64_t)i * c];
  }
  part[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0) {
    const int t = threadIdx.x;
    out[b * c + ch] = ((part[0][t] + part[1][t]) + (part[2][t] + part[3][t])) / (float)hw;
  }
}

// ---------------------------------------------------------------- launch --
template <typename T, int WM, int WN, int S>
static int launch_conv_t(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = 64 * WM, BN = 64 * WN;
  constexpr int smem = conv_smem_bytes<WM, WN, S>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_igemm_kernel<T, WM, WN, S>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  SAD_REQUIRE(a.Cout % BN == 0, "Cout must be a multiple of the tile width");
  const int64_t tiles_m = (a.M + BM - 1) / BM;
  const int64_t nwg = tiles_m * (a.Cout / BN);
  SAD_REQUIRE(nwg < (1ll << 31), "grid too large");
  SAD_REQUIRE(a.groups <= 1 || !a.res, "grouped conv: no residual");
  hipLaunchKernelGGL((conv_igemm_kernel<T, WM, WN, S>), dim3((unsigned)nwg, (unsigned)std::max(a.groups, 1)),
                     dim3(64 * WM * WN), smem, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

// Tile variants (BM x BN, waves, ring stages, LDS):
//  1: 256x64  4w S3 120 KB      2: 256x64  4w S2  80 KB (2 WG/CU)
//  3: 256x128 8w S3 144 KB      4: 128x128 4w S3  96 KB
//  5: 128x128 4w S2  64 KB      6: 512x64  8w S2 144 KB
//  7: 128x64  2w S3  72 KB      8: 256x128 8w S2  96 KB
template <typename T>
static int launch_conv_v(const ConvArgs& a, int v, hipStream_t s) {
  switch (v) {
    case 1: return launch_conv_t<T, 4, 1, 3>(a, s);
    case 2: return launch_conv_t<T, 4, 1, 2>(a, s);
    case 3: return launch_conv_t<T, 4, 2, 3>(a, s);
    case 4: return launch_conv_t<T, 2, 2, 3>(a, s);
    case 5: return launch_conv_t<T, 2, 2, 2>(a, s);
    case 6: return launch_conv_t<T, 8, 1, 2>(a, s);
    case 7: return launch_conv_t<T, 2, 1, 3>(a, s);
    case 8: return launch_conv_t<T, 4, 2, 2>(a, s);
  }
  set_error("unknown conv variant");
  return SAD_ERR_ARG;
}

int default_conv_variant(const ConvArgs& a) { return a.Cout % 128 == 0 ? 5 : 2; }

int launch_conv(const ConvArgs& a_in, int dtype, hipStream_t s, int variant) {
  const int EPC = dtype == SAD_BF16 ? 8 : 4;
  const int ES = dtype == SAD_BF16 ? 2 : 4;
  ConvArgs a = a_in;
  a.in_bytes = (((int64_t)a.N * a.H * a.W - 1) * a.in_pstride + a.Cin) * ES;
  a.wt_bytes = (int64_t)a.Cout * a.KH * a.KW * a.Cin * ES;
  SAD_REQUIRE(a.in_bytes < (1ll << 31) - 64 && a.wt_bytes < (1ll << 31),
              "conv operand exceeds the 2 GiB buffer range (lower the micro-batch)");
  SAD_REQUIRE(a.Cin % (8 * EPC) == 0, "Cin must be a multiple of the K-step");
  SAD_REQUIRE(a.Cout % 64 == 0, "Cout must be a multiple of 64");
  SAD_REQUIRE(a.in_pstride % EPC == 0 && a.out_pstride % 8 == 0, "pixel strides must keep 16-B alignment");
  if (a.M == 0) return SAD_OK;
  const int v = variant > 0 ? variant : default_conv_variant(a);
  return dtype == SAD_BF16 ? launch_conv_v<u16>(a, v, s) : launch_conv_v<float>(a, v, s);
}

int launch_stem(const StemArgs& a, int dtype, hipStream_t s) {
  SAD_REQUIRE(a.B <= 65535, "stem: B > 65535");
  if (a.B == 0) return SAD_OK;
  if (a.img3) {
    SAD_REQUIRE(a.w3 && a.bias, "distinct-channel stem: weights");
    if (dtype == SAD_F32)
      hipLaunchKernelGGL(stem3_kernel<0>, dim3(128, (unsigned)a.B), dim3(128), 0, s, a);
    else if (dtype == SAD_BF16)
      hipLaunchKernelGGL(stem3_kernel<1>, dim3(128, (unsigned)a.B), dim3(128), 0, s, a);
    else
      hipLaunchKernelGGL(stem3_kernel<2>, dim3(128, (unsigned)a.B), dim3(128), 0, s, a);
    SAD_CHECK_HIP(hipGetLastError());
    return SAD_OK;
  }
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(stem_bf16_kernel<false>, dim3(128 / STEM_P, (unsigned)a.B), dim3(256), 0, s, a);
  else if (dtype == SAD_BF16X3 && a.x4)
    hipLaunchKernelGGL((stem_bf16_kernel<true, false, true>), dim3(128 / STEM_P, (unsigned)a.B), dim3(256), 0, s, a);
  else if (dtype == SAD_BF16X3)
    hipLaunchKernelGGL(stem_bf16_kernel<true>, dim3(128 / STEM_P, (unsigned)a.B), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(stem_kernel<float>, dim3(128, (unsigned)a.B), dim3(256), 0, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

int launch_stem_train(const StemArgs& a, hipStream_t s) {
  SAD_REQUIRE(a.B <= 65535, "stem: B > 65535");
  SAD_REQUIRE(a.img16 && a.w && a.bias && a.out && a.part, "training stem: null argument");
  if (a.B == 0) return SAD_OK;
  hipLaunchKernelGGL((stem_bf16_kernel<false, true>), dim3(128 / STEM_P, (unsigned)a.B), dim3(256), 0, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

int launch_avgpool(const void* in, int64_t B, int hw, int c, float* out, int dtype, hipStream_t s) {
  if (B == 0) return SAD_OK;
  if (dtype == SAD_BF16X3)
    hipLaunchKernelGGL((avgpool_kernel<u16, true>), dim3((unsigned)B, c / 64), dim3(256), 0, s, (const u16*)in, hw, c,
                       out);
  else if (dtype == SAD_BF16)
    hipLaunchKernelGGL(avgpool_kernel<u16>, dim3((unsigned)B, c / 64), dim3(256), 0, s, (const u16*)in, hw, c, out);
  else
    hipLaunchKernelGGL(avgpool_kernel<float>, dim3((unsigned)B, c / 64), dim3(256), 0, s, (const float*)in, hw, c, out);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

}  // namespace sad
