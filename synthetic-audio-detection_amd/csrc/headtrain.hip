// headtrain.hip -- the trainer's BinaryClassifier head in train mode, for the
// optional --head-loss flag of submodel_trainer.py.
//
// The reference builds model.head (submodel_trainer.py:613-625)
//   AdaptiveAvgPool2d(1), Flatten, Linear(nf, 512), BatchNorm1d(512), ReLU,
//   Dropout(0.5), Linear(512, 256), BatchNorm1d(256), ReLU, Dropout(0.3),
//   Linear(256, 2)
// and puts its parameters in the optimizer (:648-652), but never calls it: the
// loss runs on the pooled features (quirk C1, reproduced by default).  With
// --head-loss the pooled features go through this head, CrossEntropy runs on
// its two logits (sad_ce_loss_run), and the backward returns d(features) for
// the backbone and the head's parameter gradients.
//
// Sizes are small (B x 512 x nf per GEMM, nf = 512 or 2048), so everything is
// fp32 on the vector ALU: one tiled GEMM kernel with strided operands serves
// the forward Linear, the data gradient and the weight gradient; one kernel
// per BatchNorm1d layer does batch statistics + affine + ReLU + dropout
// (forward) or the BN / ReLU / dropout backward (one thread per channel, the
// batch walked in order: deterministic, no atomics).  Dropout masks come from
// a counter hash of (seed, layer, row, channel), so the backward regenerates
// the forward's mask (tests restate the hash in numpy).
#include "common.hpp"

namespace sad {

// ---- C[M, N] = sum_k A(m, k) B(k, n) (+ bias[n]); A(m, k) = A[m*sam + k*sak]
// Split-K (blockIdx.z = split s of S): split s sums k in [s*kc, (s+1)*kc) and
// writes its partial tile to C + s*M*ldc (S > 1: a workspace, reduced in split
// order by hsplit_reduce_kernel -- deterministic).  The next K-step's operands
// are loaded into registers while the current one computes.
constexpr int HG_T = 64, HG_K = 16;
__global__ __launch_bounds__(256) void hgemm_kernel(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                    const float* __restrict__ Bm, int64_t sbk, int64_t sbn,
                                                    const float* __restrict__ bias, float* __restrict__ C,
                                                    int64_t ldc, int M, int N, int K, int kc) {
  __shared__ float sA[HG_K][HG_T + 4];
  __shared__ float sB[HG_K][HG_T + 4];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int m0 = blockIdx.y * HG_T, n0 = blockIdx.x * HG_T;
  const int kb = blockIdx.z * kc, ke = min(K, kb + kc);
  C += (int64_t)blockIdx.z * M * ldc;
  float acc[4][4] = {};
  float ra[4], rb[4];
  // consecutive threads walk each operand's unit-stride axis
  auto fetch = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      const int am = sak == 1 ? e >> 4 : e & 63, ak = sak == 1 ? e & 15 : e >> 6;
      const int bn = sbn == 1 ? e & 63 : e >> 4, bk = sbn == 1 ? e >> 6 : e & 15;
      const int gm = m0 + am, gk = k0 + ak, gn = n0 + bn, gk2 = k0 + bk;
      ra[r] = (gm < M && gk < ke) ? A[gm * sam + gk * sak] : 0.f;
      rb[r] = (gn < N && gk2 < ke) ? Bm[gk2 * sbk + gn * sbn] : 0.f;
    }
  };
  fetch(kb);
  for (int k0 = kb; k0 < ke; k0 += HG_K) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      const int am = sak == 1 ? e >> 4 : e & 63, ak = sak == 1 ? e & 15 : e >> 6;
      const int bn = sbn == 1 ? e & 63 : e >> 4, bk = sbn == 1 ? e >> 6 : e & 15;
      sA[ak][am] = ra[r];
      sB[bk][bn] = rb[r];
    }
    __syncthreads();
    if (k0 + HG_K < ke) fetch(k0 + HG_K);
#pragma unroll
    for (int kk = 0; kk < HG_K; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = sA[kk][ty * 4 + i];
        b[i] = sB[kk][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + ty * 4 + i;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + tx * 4 + j;
      if (n < N) C[m * ldc + n] = acc[i][j] + (bias ? bias[n] : 0.f);
    }
  }
}

// C[m, n] = sum_s P[s][m][n] (+ bias[n]), splits in order
__global__ void hsplit_reduce_kernel(const float* __restrict__ P, int S, int M, int N,
                                     const float* __restrict__ bias, float* __restrict__ C, int64_t ldc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int m = (int)(i / N), n = (int)(i % N);
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += P[(int64_t)s * M * N + i];
  C[m * ldc + n] = v + (bias ? bias[n] : 0.f);
}

// dropout keep test: u(seed, layer, idx) in [0, 1) from a splitmix64 finaliser
__device__ __forceinline__ bool hkeep(uint64_t seed, int layer, int64_t idx, float p) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(idx + 1) + ((uint64_t)layer << 56);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f) >= p;
}

// BatchNorm1d (train: batch statistics, running stats updated with the
// unbiased variance; eval: running stats) -> ReLU -> Dropout(p) (train only).
// x, y [B, C]; stats [2C] = mean | invstd (saved for the backward)
__global__ __launch_bounds__(256) void hbn_fwd_kernel(const float* __restrict__ x, int B, int C,
                                                      const float* __restrict__ g, const float* __restrict__ be,
                                                      float* __restrict__ rm, float* __restrict__ rv, float eps,
                                                      float mom, int train, float p, uint64_t seed, int layer,
                                                      float* __restrict__ y, float* __restrict__ stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean, invstd;
  if (train) {
    double s = 0.0;
    for (int b = 0; b < B; ++b) s += x[(int64_t)b * C + c];
    const double mu = s / B;
    double q = 0.0;
    for (int b = 0; b < B; ++b) {
      const double d = x[(int64_t)b * C + c] - mu;
      q += d * d;
    }
    const double var = q / B;
    mean = (float)mu;
    invstd = (float)(1.0 / sqrt(var + eps));
    rm[c] = (1.f - mom) * rm[c] + mom * mean;
    rv[c] = (1.f - mom) * rv[c] + mom * (float)(B > 1 ? q / (B - 1) : var);
  } else {
    mean = rm[c];
    invstd = 1.f / sqrtf(rv[c] + eps);
  }
  const float sc = g[c] * invstd, sh = be[c] - mean * sc, keep = 1.f / (1.f - p);
  const bool drop = train && p > 0.f;
  for (int b = 0; b < B; ++b) {
    const int64_t i = (int64_t)b * C + c;
    float a = fmaxf(fmaf(x[i], sc, sh), 0.f);
    if (drop) a = hkeep(seed, layer, i, p) ? a * keep : 0.f;
    y[i] = a;
  }
  stats[c] = mean;
  stats[C + c] = invstd;
}

// the backward of hbn_fwd in train mode: dz = dy * dropout mask / (1 - p) *
// [bn output > 0]; dbeta = sum dz, dgamma = sum dz * xhat; dx = gamma * invstd *
// (dz - mean dz - xhat * mean(dz xhat)); dlin = sum dx (the preceding
// Linear's bias gradient)
__global__ __launch_bounds__(256) void hbn_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                                      int B, int C, const float* __restrict__ g,
                                                      const float* __restrict__ be, const float* __restrict__ stats,
                                                      float p, uint64_t seed, int layer, float* __restrict__ dx,
                                                      float* __restrict__ dg, float* __restrict__ dbe,
                                                      float* __restrict__ dlin) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mean = stats[c], invstd = stats[C + c], gc = g[c], bc = be[c];
  const float keep = 1.f / (1.f - p);
  const bool drop = p > 0.f;
  auto dz_of = [&](int64_t i, float& xh) {
    xh = (x[i] - mean) * invstd;
    const float z = fmaf(xh, gc, bc);
    float d = z > 0.f ? dy[i] : 0.f;
    if (drop) d = hkeep(seed, layer, i, p) ? d * keep : 0.f;
    return d;
  };
  float s1 = 0.f, s2 = 0.f;
  for (int b = 0; b < B; ++b) {
    float xh;
    const float d = dz_of((int64_t)b * C + c, xh);
    s1 += d;
    s2 += d * xh;
  }
  dbe[c] = s1;
  dg[c] = s2;
  const float m1 = s1 / B, m2 = s2 / B, k = gc * invstd;
  float sdx = 0.f;
  for (int b = 0; b < B; ++b) {
    const int64_t i = (int64_t)b * C + c;
    float xh;
    const float d = dz_of(i, xh);
    const float v = k * (d - m1 - xh * m2);
    dx[i] = v;
    sdx += v;
  }
  dlin[c] = sdx;
}

// out[n] = sum_m x[m, n] (the last Linear's bias gradient), batch in order
__global__ void hcolsum_kernel(const float* __restrict__ x, int M, int N, float* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int m = 0; m < M; ++m) s += x[(int64_t)m * N + n];
  out[n] = s;
}

constexpr int HG_SPLITS = 8;  // at most; the workspace holds HG_SPLITS x the largest B x N partial

static int hgemm(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                 const float* bias, float* C, int64_t ldc, int M, int N, int K, hipStream_t s,
                 float* part = nullptr, size_t part_floats = 0) {
  if (M == 0 || N == 0) return SAD_OK;
  const int tiles = ((N + HG_T - 1) / HG_T) * ((M + HG_T - 1) / HG_T);
  // split K when the tiles alone leave the chip idle and each split keeps >= 64 of K
  int S = 1;
  while (S < HG_SPLITS && tiles * S < 256 && K / (2 * S) >= 64 && part &&
         (size_t)(2 * S) * M * N <= part_floats)
    S *= 2;
  const int kc = (K + S - 1) / S;
  dim3 grid((N + HG_T - 1) / HG_T, (M + HG_T - 1) / HG_T, S);
  SAD_REQUIRE(grid.y <= 65535, "head GEMM: too many rows");
  if (S == 1) {
    hipLaunchKernelGGL(hgemm_kernel, grid, dim3(256), 0, s, A, sam, sak, B, sbk, sbn, bias, C, ldc, M, N, K, kc);
  } else {
    hipLaunchKernelGGL(hgemm_kernel, grid, dim3(256), 0, s, A, sam, sak, B, sbk, sbn, nullptr, part, (int64_t)N, M,
                       N, K, kc);
    SAD_CHECK_HIP(hipGetLastError());
    const int64_t n = (int64_t)M * N;
    hipLaunchKernelGGL(hsplit_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, S, M, N, bias,
                       C, ldc);
  }
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

constexpr int H1 = 512, H2 = 256, HO = 2;

// workspace layout (floats): h1, a1 [B, 512]; h2, a2 [B, 256]; stats3 [1024];
// stats7 [512]; backward scratch da2, dh2 [B, 256]; da1, dh1 [B, 512]; the
// split-K partials of the B-row GEMMs [HG_SPLITS][B][max(nf, 512)]
struct HeadWs {
  float *h1, *a1, *h2, *a2, *st3, *st7, *da2, *dh2, *da1, *dh1, *part;
  size_t part_floats;
};
static size_t head_part_floats(int64_t B, int nf) { return (size_t)HG_SPLITS * B * (nf > H1 ? nf : H1); }
static size_t head_ws_floats(int64_t B, int nf) {
  return (size_t)B * (2 * H1 + 2 * H2) * 2 + 2 * H1 + 2 * H2 + head_part_floats(B, nf);
}
static HeadWs head_ws(void* ws, int64_t B, int nf) {
  float* f = (float*)ws;
  HeadWs w;
  w.h1 = f;
  w.a1 = w.h1 + B * H1;
  w.h2 = w.a1 + B * H1;
  w.a2 = w.h2 + B * H2;
  w.st3 = w.a2 + B * H2;
  w.st7 = w.st3 + 2 * H1;
  w.da2 = w.st7 + 2 * H2;
  w.dh2 = w.da2 + B * H2;
  w.da1 = w.dh2 + B * H2;
  w.dh1 = w.da1 + B * H1;
  w.part = w.dh1 + B * H1;
  w.part_floats = head_part_floats(B, nf);
  return w;
}

}  // namespace sad

using namespace sad;

extern "C" int sad_head_workspace_size(int64_t B, int32_t in_features, size_t* bytes) {
  SAD_REQUIRE(bytes && B >= 0 && in_features > 0, "bad args");
  *bytes = head_ws_floats(B, in_features) * sizeof(float);
  return SAD_OK;
}

static int head_check(const sad_head_params* h, const float* feats, int64_t B, void* ws, size_t ws_bytes) {
  SAD_REQUIRE(h && feats && ws, "null argument");
  SAD_REQUIRE(h->w2 && h->b2 && h->g3 && h->be3 && h->w6 && h->b6 && h->g7 && h->be7 && h->w10 && h->b10,
              "null head parameter");
  SAD_REQUIRE(h->rm3 && h->rv3 && h->rm7 && h->rv7, "null running statistics");
  SAD_REQUIRE(h->in_features > 0 && B > 0 && B < (1 << 24), "bad shape");
  SAD_REQUIRE(h->p1 >= 0.f && h->p1 < 1.f && h->p2 >= 0.f && h->p2 < 1.f, "dropout rate outside [0, 1)");
  SAD_REQUIRE(ws_bytes >= head_ws_floats(B, h->in_features) * sizeof(float),
              "head workspace too small (sad_head_workspace_size)");
  return SAD_OK;
}

extern "C" int sad_head_train_forward_run(const sad_head_params* h, const float* feats, int64_t B, int32_t train,
                                          uint64_t seed, float* logits, void* ws, size_t ws_bytes, void* stream) {
  if (int rc = head_check(h, feats, B, ws, ws_bytes)) return rc;
  SAD_REQUIRE(logits, "null logits");
  SAD_REQUIRE(train || B > 0, "bad args");
  hipStream_t s = (hipStream_t)stream;
  const int nf = h->in_features, Bi = (int)B;
  const HeadWs w = head_ws(ws, B, nf);
  int rc;
  // Linear(nf, 512): h1 = feats . W2^T + b2
  if ((rc = hgemm(feats, nf, 1, h->w2, 1, nf, h->b2, w.h1, H1, Bi, H1, nf, s, w.part, w.part_floats))) return rc;
  hipLaunchKernelGGL(hbn_fwd_kernel, dim3((H1 + 255) / 256), dim3(256), 0, s, w.h1, Bi, H1, h->g3, h->be3, h->rm3,
                     h->rv3, h->eps, h->momentum, train, h->p1, seed, 1, w.a1, w.st3);
  SAD_CHECK_HIP(hipGetLastError());
  // Linear(512, 256)
  if ((rc = hgemm(w.a1, H1, 1, h->w6, 1, H1, h->b6, w.h2, H2, Bi, H2, H1, s, w.part, w.part_floats))) return rc;
  hipLaunchKernelGGL(hbn_fwd_kernel, dim3((H2 + 255) / 256), dim3(256), 0, s, w.h2, Bi, H2, h->g7, h->be7, h->rm7,
                     h->rv7, h->eps, h->momentum, train, h->p2, seed, 2, w.a2, w.st7);
  SAD_CHECK_HIP(hipGetLastError());
  // Linear(256, 2)
  return hgemm(w.a2, H2, 1, h->w10, 1, H2, h->b10, logits, HO, Bi, HO, H2, s);
}

extern "C" int sad_head_train_backward_run(const sad_head_params* h, const float* feats, int64_t B, uint64_t seed,
                                           const float* dlogits, float* dfeats, float* grads, void* ws,
                                           size_t ws_bytes, void* stream) {
  if (int rc = head_check(h, feats, B, ws, ws_bytes)) return rc;
  SAD_REQUIRE(dlogits && dfeats && grads, "null output");
  hipStream_t s = (hipStream_t)stream;
  const int nf = h->in_features, Bi = (int)B;
  const HeadWs w = head_ws(ws, B, nf);
  // gradient layout = the parameters' order: 2.w, 2.b, 3.w, 3.b, 6.w, 6.b, 7.w, 7.b, 10.w, 10.b
  float* g_w2 = grads;
  float* g_b2 = g_w2 + (int64_t)H1 * nf;
  float* g_g3 = g_b2 + H1;
  float* g_be3 = g_g3 + H1;
  float* g_w6 = g_be3 + H1;
  float* g_b6 = g_w6 + H2 * H1;
  float* g_g7 = g_b6 + H2;
  float* g_be7 = g_g7 + H2;
  float* g_w10 = g_be7 + H2;
  float* g_b10 = g_w10 + HO * H2;
  int rc;
  // Linear(256, 2): dW10 = dlogits^T a2, db10 = sum dlogits, da2 = dlogits . W10
  if ((rc = hgemm(dlogits, 1, HO, w.a2, H2, 1, nullptr, g_w10, H2, HO, H2, Bi, s))) return rc;
  hipLaunchKernelGGL(hcolsum_kernel, dim3(1), dim3(64), 0, s, dlogits, Bi, HO, g_b10);
  SAD_CHECK_HIP(hipGetLastError());
  if ((rc = hgemm(dlogits, HO, 1, h->w10, H2, 1, nullptr, w.da2, H2, Bi, H2, HO, s))) return rc;
  // Dropout(0.3) / ReLU / BatchNorm1d(256) -> dh2 (+ db6 = sum dh2)
  hipLaunchKernelGGL(hbn_bwd_kernel, dim3((H2 + 255) / 256), dim3(256), 0, s, w.h2, w.da2, Bi, H2, h->g7, h->be7,
                     w.st7, h->p2, seed, 2, w.dh2, g_g7, g_be7, g_b6);
  SAD_CHECK_HIP(hipGetLastError());
  // Linear(512, 256): dW6 = dh2^T a1, da1 = dh2 . W6
  if ((rc = hgemm(w.dh2, 1, H2, w.a1, H1, 1, nullptr, g_w6, H1, H2, H1, Bi, s))) return rc;
  if ((rc = hgemm(w.dh2, H2, 1, h->w6, H1, 1, nullptr, w.da1, H1, Bi, H1, H2, s, w.part, w.part_floats))) return rc;
  hipLaunchKernelGGL(hbn_bwd_kernel, dim3((H1 + 255) / 256), dim3(256), 0, s, w.h1, w.da1, Bi, H1, h->g3, h->be3,
                     w.st3, h->p1, seed, 1, w.dh1, g_g3, g_be3, g_b2);
  SAD_CHECK_HIP(hipGetLastError());
  // Linear(nf, 512): dW2 = dh1^T feats, dfeats = dh1 . W2
  if ((rc = hgemm(w.dh1, 1, H1, feats, nf, 1, nullptr, g_w2, nf, H1, nf, Bi, s))) return rc;
  return hgemm(w.dh1, H1, 1, h->w2, nf, 1, nullptr, dfeats, nf, Bi, nf, H1, s, w.part, w.part_floats);
}
