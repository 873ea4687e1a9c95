// wgrad.hip -- the trainer's two pixel-axis contractions on the MFMA cores
// (gfx950): the conv weight gradient and the strided conv input gradient of
// submodel_trainer.py's loss.backward() (:273-275, layer4 and, from epoch
// epochs//3, layer3: quirk C4).
//
//   wgrad:  dW[co][ci][ky][kx] = sum_p dy[p][co] * x[src(p, ky, kx)][ci]
//   dgrad:  dcol[p][j]          = sum_co dy[p][co] * W[co][j]    (+ col2im)
//
// Both are C[m][n] = sum_k A[k][m] * B[k][n] with the reduction over the
// OUTER (row) index of both operands: NHWC rows of dy and x for wgrad, OIHW
// rows of W and (transposed) dy for dgrad.  Tiles arrive from HBM row-major
// (coalesced 256/512-B rows) and are consumed column-wise: bf16 fragments come
// out of LDS with the transposing ds_read_b64_tr_b16 (cdna_hip_programming.md
// T10), fp32 fragments are single dwords per lane, which the 16x16x4 f32 MFMA
// takes k-major anyway.  No im2col: the wgrad B operand is gathered per tap
// straight from the NHWC activation (zero rows for the padding).
//
// Work split: 128x128 output tiles x taps x split-K over the pixels; each
// split writes fp32 partials [split][tap][M][N] that a deterministic reduce
// folds into the OIHW gradient (beta*dW + sum).  256 threads = 2x2 waves of
// 64x64; one 16-KB tile per operand per K-step (64 bf16 / 32 fp32 rows),
// register-staged into a 2-stage LDS ring, one barrier per K-step.
#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"

namespace sad {

struct KoArgs {
  const void* a;  // A[k][m] at a + k*lda + m (elements)
  int64_t lda;
  const void* b;  // B row k = source row src(k) of b (ldb elements per row)
  int64_t ldb;
  int M, N, K;
  // B gather: row k -> pixel (n, oy, ox) of an [Ho][Wo] map; source pixel
  // (oy*stride - pad + ky, ox*stride - pad + kx) of an [H][W] map, zero outside.
  int H, W, Ho, Wo, ksz, stride, pad;
  int kchunk;  // rows per split (multiple of the K-step)
  float* out;  // [split][ksz*ksz][M][N]
  // bf16 kernel: buffer sizes (bytes, < 2 GiB) and k -> (n, oy, ox) divisors
  int64_t a_bytes, b_bytes;
  uint32_t hw_m, hw_s, wo_m, wo_s;
};

// q = k / d for k < 2^31 by multiply-high (d > 1: p = 31 + ceil(log2 d),
// m = ceil(2^p / d), q = umulhi(k, m) >> (p - 32); d == 1: m = 0 marks identity)
static void fast_div(uint32_t d, uint32_t* m, uint32_t* sh) {
  if (d <= 1) {
    *m = 0;
    *sh = 0;
    return;
  }
  int l = 0;
  while ((1ull << l) < d) ++l;
  const int p = 31 + l;
  *m = (uint32_t)(((1ull << p) + d - 1) / d);
  *sh = (uint32_t)(p - 32);
}
__device__ __forceinline__ uint32_t fdiv(uint32_t k, uint32_t m, uint32_t sh) {
  return m ? (__umulhi(k, m) >> sh) : k;
}

template <typename T>
struct KO;
template <>
struct KO<u16> {
  static constexpr int KS = 64, CPR = 16;  // rows per K-step, 16-B chunks per 128-element row
};
template <>
struct KO<float> {
  static constexpr int KS = 32, CPR = 32;
};

// Byte offset of 16-B chunk `ch` of tile row `r`.  bf16: 256-B rows with the
// (b) XOR image of T10, conflict-free for the 16x16x32 transposed reads (a
// 32-lane half reads two 4-row blocks 8 rows apart).  fp32: 512-B rows with
// bit 2 of the row flipping the 64-B half-bank group, so the two 16-lane
// groups of a half (rows 4 apart) hit disjoint banks.
template <typename T>
__device__ __forceinline__ int ko_off(int r, int ch) {
  if constexpr (sizeof(T) == 2)
    return 256 * r + 16 * (ch ^ (((r & 3) << 2) | ((r >> 2) & 3)));
  else
    return 512 * r + 16 * (ch ^ (r & 4));
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// A/B fragment of one 16x16x32 bf16 MFMA from a k-major tile: lane l gets
// column c0 + (l & 15), rows kb + 8*(l >> 4) + 0..7.  Lane 4q+p of a 16-lane
// group supplies row (block row 0 + q), columns 4p..4p+3 of its group's block.
__device__ __forceinline__ uint4 tr_frag(const char* tile, int kb, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int ch = (c0 >> 3) + (p >> 1);
  const int r = kb + 8 * g + q;
  const char* p0 = tile + ko_off<u16>(r, ch) + 8 * (p & 1);
  const char* p1 = tile + ko_off<u16>(r + 4, ch) + 8 * (p & 1);
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p0);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)p1);
  uint4 f;
  f.x = (uint32_t)(uint16_t)lo.x | ((uint32_t)(uint16_t)lo.y << 16);
  f.y = (uint32_t)(uint16_t)lo.z | ((uint32_t)(uint16_t)lo.w << 16);
  f.z = (uint32_t)(uint16_t)hi.x | ((uint32_t)(uint16_t)hi.y << 16);
  f.w = (uint32_t)(uint16_t)hi.z | ((uint32_t)(uint16_t)hi.w << 16);
  return f;
}

// fp32: lane l gets column c0 + (l & 15), rows kb + 4*(l >> 4) + 0..3 (one
// per chained 16x16x4 MFMA of mfma_chunk<float>).
__device__ __forceinline__ uint4 f32_frag(const char* tile, int kb, int c0, int lane) {
  const int c = c0 + (lane & 15), r = kb + 4 * (lane >> 4);
  uint4 f;
  f.x = *(const uint32_t*)(tile + ko_off<float>(r + 0, c >> 2) + 4 * (c & 3));
  f.y = *(const uint32_t*)(tile + ko_off<float>(r + 1, c >> 2) + 4 * (c & 3));
  f.z = *(const uint32_t*)(tile + ko_off<float>(r + 2, c >> 2) + 4 * (c & 3));
  f.w = *(const uint32_t*)(tile + ko_off<float>(r + 3, c >> 2) + 4 * (c & 3));
  return f;
}

template <typename T>
__global__ __launch_bounds__(256) void kouter_gemm_kernel(KoArgs g) {
  constexpr int KS = KO<T>::KS, CPR = KO<T>::CPR, EPC = DT<T>::EPC, RSTEP = 256 / CPR;
  constexpr int TILE = 16384;
  __shared__ uint4 lds[4 * TILE / 16];  // [stage][A | B]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_m = (g.M + 127) >> 7;
  const int m0 = (blockIdx.x % tiles_m) * 128, n0 = (blockIdx.x / tiles_m) * 128;
  const int tap = blockIdx.y, ky = tap / g.ksz, kx = tap - ky * g.ksz;
  const int k_lo = blockIdx.z * g.kchunk;
  const int k_hi = min(g.K, k_lo + g.kchunk);
  const T* A = (const T*)g.a;
  const T* B = (const T*)g.b;
  const int ch = t % CPR, r0 = t / CPR;
  const int am = m0 + ch * EPC, bn = n0 + ch * EPC;
  const bool a_ok = am < g.M, b_ok = bn < g.N;
  const int hw = g.Ho * g.Wo;

  uint4 ra[4], rb[4];
  auto load = [&](int kb) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = kb + r0 + i * RSTEP;
      ra[i] = make_uint4(0, 0, 0, 0);
      rb[i] = make_uint4(0, 0, 0, 0);
      if (k < k_hi) {
        if (a_ok) ra[i] = *(const uint4*)(A + (int64_t)k * g.lda + am);
        const int n = k / hw, rem = k - n * hw;
        const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
        const int iy = oy * g.stride - g.pad + ky, ix = ox * g.stride - g.pad + kx;
        if (b_ok && iy >= 0 && iy < g.H && ix >= 0 && ix < g.W)
          rb[i] = *(const uint4*)(B + ((int64_t)(n * g.H + iy) * g.W + ix) * g.ldb + bn);
      }
    }
  };
  auto store = [&](int st) {
    char* base = (char*)lds + st * 2 * TILE;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = ko_off<T>(r0 + i * RSTEP, ch);
      *(uint4*)(base + off) = ra[i];
      *(uint4*)(base + TILE + off) = rb[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  load(k_lo);
  store(0);
  __syncthreads();
  int st = 0;
  for (int kb = k_lo; kb < k_hi; kb += KS) {
    const bool more = kb + KS < k_hi;
    if (more) load(kb + KS);
    const char* ta = (const char*)lds + st * 2 * TILE;
    const char* tb = ta + TILE;
#pragma unroll
    for (int kk = 0; kk < KS; kk += (sizeof(T) == 2 ? 32 : 16)) {
      uint4 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (sizeof(T) == 2) {
          fa[i] = tr_frag(ta, kk, wm * 64 + i * 16, lane);
          fb[i] = tr_frag(tb, kk, wn * 64 + i * 16, lane);
        } else {
          fa[i] = f32_frag(ta, kk, wm * 64 + i * 16, lane);
          fb[i] = f32_frag(tb, kk, wn * 64 + i * 16, lane);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_chunk<T>(fa[i], fb[j], acc[i][j]);
    }
    if (more) store(st ^ 1);
    __syncthreads();
    st ^= 1;
  }

  // D[m][n]: lane l, register r -> row 4*(l >> 4) + r, column l & 15
  float* out = g.out + ((int64_t)blockIdx.z * gridDim.y + tap) * (int64_t)g.M * g.N;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        if (m < g.M && n < g.N) out[(int64_t)m * g.N + n] = acc[i][j][r];
      }
    }
}

// bf16, LDS-DMA fed: BM x BN output tile, WM x WN waves, K-step of 32 rows,
// a 4-stage ring (3 steps of DMA in flight).  Each operand tile is stored as
// 128-column halves of 32 rows x 256 B in the T10 (b) XOR image; one
// buffer_load...lds instruction fills 4 rows of a half (lane-linear in LDS,
// so the XOR is applied to the GLOBAL chunk each lane fetches).  Rows past the
// split's K range, padding taps and columns past M / N load zeros (offset past
// num_records).  Products are formed as B^T A so each lane holds 4 consecutive
// n of one m and the fp32 partial tile leaves as float4 rows.
template <int BM, int BN, int WM, int WN>
constexpr int kouter_smem_bytes() {
  return 4 * (BM / 128 + BN / 128) * 32 * 256;
}

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void kouter_bf16_kernel(KoArgs g) {
  constexpr int NW = WM * WN, KS = 32, S = 4;
  constexpr int HA = BM / 128, HB = BN / 128;
  constexpr int HALF = KS * 256, STAGE = (HA + HB) * HALF;
  constexpr int GPH = KS / 4;               // DMA instructions per half
  constexpr int NI = (HA + HB) * GPH;       // per K-step
  static_assert(NI % NW == 0, "DMA pieces must split evenly over the waves");
  constexpr int QI = NI / NW;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_m = (g.M + BM - 1) / BM;
  const int m0 = (blockIdx.x % tiles_m) * BM, n0 = (blockIdx.x / tiles_m) * BN;
  const int tap = blockIdx.y, ky = tap / g.ksz, kx = tap - ky * g.ksz;
  const int k_lo = blockIdx.z * g.kchunk;
  const int k_hi = min(g.K, k_lo + g.kchunk);
  const int nsteps = k_hi > k_lo ? (k_hi - k_lo + KS - 1) / KS : 0;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)g.a, (short)0, (int)g.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)g.b, (short)0, (int)g.b_bytes, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  constexpr int BAD = 0x7FFFFFF0;

  // this wave's DMA pieces: operand, LDS offset in a stage, row, column (bytes)
  bool isb[QI], colok[QI];
  int dst[QI], row[QI], colb[QI];
#pragma unroll
  for (int i = 0; i < QI; ++i) {
    const int q = wave + NW * i;
    isb[i] = q >= HA * GPH;
    const int qq = isb[i] ? q - HA * GPH : q;
    const int half = qq / GPH, grp = qq % GPH;
    dst[i] = (isb[i] ? HA * HALF : 0) + half * HALF + grp * 1024;
    const int r = grp * 4 + (lane >> 4), pos = lane & 15;
    row[i] = r;
    const int ch = pos ^ (((r & 3) << 2) | ((r >> 2) & 3));
    const int col = (isb[i] ? n0 : m0) + half * 128 + ch * 8;
    colok[i] = col < (isb[i] ? g.N : g.M);
    colb[i] = col * 2;
  }
  const int hw = g.Ho * g.Wo;
  auto issue = [&](int step) __attribute__((always_inline)) {
    const unsigned sb = lds0 + (step % S) * STAGE;
    const int kb = k_lo + step * KS;
#pragma unroll
    for (int i = 0; i < QI; ++i) {
      const int k = kb + row[i];
      int voff = BAD;
      if (!isb[i]) {
        if (k < k_hi && colok[i]) voff = (int)((int64_t)k * g.lda * 2) + colb[i];
        dma16_m0(ra, voff, sb + dst[i]);
      } else {
        const int n = (int)fdiv((uint32_t)k, g.hw_m, g.hw_s), rem = k - n * hw;
        const int oy = (int)fdiv((uint32_t)rem, g.wo_m, g.wo_s), ox = rem - oy * g.Wo;
        const int iy = oy * g.stride - g.pad + ky, ix = ox * g.stride - g.pad + kx;
        if (k < k_hi && colok[i] && (unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
          voff = (int)(((int64_t)(n * g.H + iy) * g.W + ix) * g.ldb * 2) + colb[i];
        dma16_m0(rb, voff, sb + dst[i]);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int p = 0; p < S - 1 && p < nsteps; ++p) issue(p);
  for (int step = 0; step < nsteps; ++step) {
    // this wave's pieces of `step` landed (later steps may stay in flight),
    // then the barrier publishes everyone's and frees stage (step - 1) % S
    if (step + 2 < nsteps)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * QI) : "memory");
    else if (step + 1 < nsteps)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QI) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (step + S - 1 < nsteps) issue(step + S - 1);
    const char* ta = smem + (step % S) * STAGE;
    const char* tb = ta + HA * HALF;
    uint4 fa[TM], fb[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int c = wm * (BM / WM) + i * 16;
      fa[i] = tr_frag(ta + (c >> 7) * HALF, 0, c & 127, lane);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = wn * (BN / WN) + j * 16;
      fb[j] = tr_frag(tb + (c >> 7) * HALF, 0, c & 127, lane);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma_chunk<u16>(fb[j], fa[i], acc[i][j]);
  }

  // D'[n][m]: lane l, register r -> n = 4*(l >> 4) + r, m = l & 15
  float* out = g.out + ((int64_t)blockIdx.z * gridDim.y + tap) * (int64_t)g.M * g.N;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
      if (m < g.M && n < g.N)
        *(float4*)(out + (int64_t)m * g.N + n) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
}

// dW[co][ci0 .. ci0+255][tap] = beta*dW + sum_s part[s][tap][co][ci] (fixed
// order: deterministic).  Block = one co x 256 ci: partial rows are read as
// float4 per tap, transposed through LDS, and written as one contiguous
// 256*taps-float run of the OIHW gradient.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int taps,
                                                           int M, int N, float beta, float* __restrict__ dw) {
  __shared__ float sm[256 * 9];
  const int co = blockIdx.y, ci0 = blockIdx.x * 256;
  const int c4 = threadIdx.x & 63, tg = threadIdx.x >> 6;
  const int64_t plane = (int64_t)M * N;
  const int nci = min(256, N - ci0);
  for (int t = tg; t < taps; t += 4) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (4 * c4 < nci)
      for (int z = 0; z < splits; ++z) {
        const float4 v = *(const float4*)(part + ((int64_t)z * taps + t) * plane + (int64_t)co * N + ci0 + 4 * c4);
        s.x += v.x;
        s.y += v.y;
        s.z += v.z;
        s.w += v.w;
      }
    sm[(4 * c4 + 0) * taps + t] = s.x;
    sm[(4 * c4 + 1) * taps + t] = s.y;
    sm[(4 * c4 + 2) * taps + t] = s.z;
    sm[(4 * c4 + 3) * taps + t] = s.w;
  }
  __syncthreads();
  float* o = dw + ((int64_t)co * N + ci0) * taps;
  for (int e = threadIdx.x; e < nci * taps; e += 256) o[e] = beta != 0.f ? beta * o[e] + sm[e] : sm[e];
}

// out[c][p] = in[p][c] (64x64 tiles through LDS)
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(const T* __restrict__ in, int64_t P, int C,
                                                        T* __restrict__ out) {
  __shared__ T tile[64][65];
  const int64_t p0 = (int64_t)blockIdx.x * 64;
  const int c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int64_t p = p0 + r;
    if (p < P && c0 + tx < C) tile[r][tx] = in[p * C + c0 + tx];
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r;
    if (c < C && p0 + tx < P) out[(int64_t)c * P + p0 + tx] = tile[tx][r];
  }
}

// Split count: minimise the modelled time = (waves of resident blocks) x
// (K-steps per block) x (one block K-step at half the MFMA peak) + the fp32
// partial tiles written and re-read by the reduce (4 TB/s), over splits that
// leave >= 4 K-steps per block.
static int choose_splits(int64_t tiles, int64_t K, int ks, int slots, double step_us, double split_bytes) {
  int best = 1;
  double best_cost = 1e30;
  for (int s = 1; s <= 64; ++s) {
    if (s > 1 && K / s < 4 * ks) break;
    const int64_t steps = ((K + s - 1) / s + ks - 1) / ks;
    const double cost = (double)((tiles * s + slots - 1) / slots) * steps * step_us + s * split_bytes * 2 / 4e6;
    if (cost < best_cost * 0.999) {
      best_cost = cost;
      best = s;
    }
  }
  return best;
}

static int device_cus() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev]) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus[dev] = c;
  }
  return cus[dev];
}

// Kernel configuration of one contraction: bf16 uses the DMA-fed kernel with
// 256x256 tiles (8 waves, one block per CU) when both output dims reach 256,
// else 128x128 (4 waves, two blocks per CU); fp32 the register-staged kernel.
struct KoCfg {
  int bm, bn, ks, per_cu;
  double step_us;  // one K-step of every resident block of a CU at half the MFMA peak
};
static KoCfg ko_cfg(int M, int N, int dtype) {
  if (dtype != SAD_BF16) return {128, 128, KO<float>::KS, 2, 2.0 * 2 * 128 * 128 * 32 / (157e12 / 256 * 0.5) * 1e6};
  if (M >= 256 && N >= 256) return {256, 256, 32, 1, 2.0 * 256 * 256 * 32 / (2.5e15 / 256 * 0.5) * 1e6};
  return {128, 128, 32, 2, 2 * 2.0 * 128 * 128 * 32 / (2.5e15 / 256 * 0.5) * 1e6};
}

struct WgradPlan {
  int Ho, Wo, taps, splits, kchunk;
  int64_t P;
  size_t ws;
};

static WgradPlan wgrad_plan(int64_t N, int H, int W, int Cin, int Cout, int k, int stride, int pad, int dtype) {
  WgradPlan p{};
  p.Ho = (H + 2 * pad - k) / stride + 1;
  p.Wo = (W + 2 * pad - k) / stride + 1;
  p.P = N * p.Ho * p.Wo;
  p.taps = k * k;
  const KoCfg c = ko_cfg(Cout, Cin, dtype);
  const int64_t tiles = (int64_t)((Cout + c.bm - 1) / c.bm) * ((Cin + c.bn - 1) / c.bn) * p.taps;
  p.splits = p.P > 0 ? choose_splits(tiles, p.P, c.ks, c.per_cu * device_cus(), c.step_us,
                                     (double)p.taps * Cout * Cin * sizeof(float))
                     : 1;
  p.kchunk = (int)(((p.P + p.splits - 1) / p.splits + c.ks - 1) / c.ks * c.ks);
  p.ws = (size_t)p.splits * p.taps * Cout * Cin * sizeof(float);
  return p;
}

static inline unsigned nblk(int64_t total, int t = 256) { return (unsigned)((total + t - 1) / t); }

template <int BM, int BN, int WM, int WN>
static int launch_kouter_bf16(const KoArgs& a, int taps, int splits, hipStream_t s) {
  constexpr int smem = kouter_smem_bytes<BM, BN, WM, WN>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kouter_bf16_kernel<BM, BN, WM, WN>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr = true;
  }
  const dim3 grid((unsigned)(((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN)), (unsigned)taps, (unsigned)splits);
  hipLaunchKernelGGL((kouter_bf16_kernel<BM, BN, WM, WN>), grid, dim3(WM * WN * 64), smem, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

int launch_kouter(KoArgs a, int taps, int splits, int dtype, hipStream_t s) {
  if (dtype == SAD_BF16) {
    SAD_REQUIRE(a.a_bytes < (1ll << 31) - 64 && a.b_bytes < (1ll << 31) - 64,
                "contraction operands must stay below 2 GiB (32-bit buffer offsets)");
    fast_div((uint32_t)(a.Ho * a.Wo), &a.hw_m, &a.hw_s);
    fast_div((uint32_t)a.Wo, &a.wo_m, &a.wo_s);
    const KoCfg c = ko_cfg(a.M, a.N, dtype);
    if (c.bm == 256) return launch_kouter_bf16<256, 256, 2, 4>(a, taps, splits, s);
    return launch_kouter_bf16<128, 128, 2, 2>(a, taps, splits, s);
  }
  const dim3 grid((unsigned)(((a.M + 127) / 128) * ((a.N + 127) / 128)), (unsigned)taps, (unsigned)splits);
  hipLaunchKernelGGL(kouter_gemm_kernel<float>, grid, dim3(256), 0, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

}  // namespace sad

using namespace sad;

extern "C" int sad_conv_wgrad_workspace_size(int64_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t k,
                                             int32_t stride, int32_t pad, int32_t dtype, size_t* bytes) {
  SAD_REQUIRE(bytes && N >= 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && k > 0 && stride > 0 && pad >= 0, "bad args");
  *bytes = wgrad_plan(N, H, W, Cin, Cout, k, stride, pad, dtype).ws;
  return SAD_OK;
}

extern "C" int sad_conv_wgrad_run(const void* x, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* dy,
                                  int32_t Cout, int32_t k, int32_t stride, int32_t pad, int32_t dtype, float beta,
                                  float* dw, void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(x && dy && dw && N >= 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0 && k > 0 && stride > 0 && pad >= 0,
              "bad args");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  const int epc = dtype == SAD_BF16 ? 8 : 4;
  SAD_REQUIRE(Cin % epc == 0 && Cout % epc == 0, "wgrad: Cin and Cout must be multiples of 16 bytes");
  const WgradPlan p = wgrad_plan(N, H, W, Cin, Cout, k, stride, pad, dtype);
  SAD_REQUIRE(p.Ho > 0 && p.Wo > 0 && p.P < (1ll << 31) - 256, "wgrad: bad or too large output map");
  hipStream_t s = (hipStream_t)stream;
  SAD_REQUIRE(p.taps <= 9, "wgrad: k <= 3");
  const dim3 rgrid((unsigned)((Cin + 255) / 256), (unsigned)Cout);
  if (p.P == 0) {  // empty batch: dW = beta*dW
    hipLaunchKernelGGL(wgrad_reduce_kernel, rgrid, dim3(256), 0, s, (const float*)nullptr, 0, p.taps, Cout, Cin, beta,
                       dw);
    SAD_CHECK_HIP(hipGetLastError());
    return SAD_OK;
  }
  SAD_REQUIRE(ws && ws_bytes >= p.ws, "wgrad workspace too small (sad_conv_wgrad_workspace_size)");
  KoArgs a{};
  a.a = dy;
  a.lda = Cout;
  a.b = x;
  a.ldb = Cin;
  a.M = Cout;
  a.N = Cin;
  a.K = (int)p.P;
  a.H = H;
  a.W = W;
  a.Ho = p.Ho;
  a.Wo = p.Wo;
  a.ksz = k;
  a.stride = stride;
  a.pad = pad;
  a.kchunk = p.kchunk;
  a.out = (float*)ws;
  a.a_bytes = p.P * Cout * (dtype == SAD_BF16 ? 2 : 4);
  a.b_bytes = N * H * W * (int64_t)Cin * (dtype == SAD_BF16 ? 2 : 4);
  int rc = launch_kouter(a, p.taps, p.splits, dtype, s);
  if (rc) return rc;
  hipLaunchKernelGGL(wgrad_reduce_kernel, rgrid, dim3(256), 0, s, (const float*)ws, p.splits, p.taps, Cout, Cin,
                     beta, dw);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

extern "C" int sad_conv_dgrad_workspace_size(int64_t N, int32_t Ho, int32_t Wo, int32_t Cout, int32_t Cin, int32_t k,
                                             int32_t dtype, size_t* bytes) {
  SAD_REQUIRE(bytes && N >= 0 && Ho > 0 && Wo > 0 && Cout > 0 && Cin > 0 && k > 0, "bad args");
  const int64_t P = N * Ho * Wo;
  const size_t es = dtype == SAD_BF16 ? 2 : 4;
  const size_t dyt = ((size_t)P * Cout * es + 255) / 256 * 256;
  *bytes = dyt + (size_t)P * Cin * k * k * sizeof(float);
  return SAD_OK;
}

extern "C" int sad_conv_dgrad_run(const void* dy, int64_t N, int32_t Ho, int32_t Wo, int32_t Cout, const void* w_oihw,
                                  int32_t Cin, int32_t H, int32_t W, int32_t k, int32_t stride, int32_t pad,
                                  int32_t dtype, int32_t accumulate, void* dx, void* ws, size_t ws_bytes,
                                  void* stream) {
  SAD_REQUIRE(dy && w_oihw && dx && ws && N >= 0 && Cin > 0 && Cout > 0 && k > 0 && stride > 0, "bad args");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  SAD_REQUIRE((H + 2 * pad - k) / stride + 1 == Ho && (W + 2 * pad - k) / stride + 1 == Wo, "shape mismatch");
  const int64_t P = N * Ho * Wo, J = (int64_t)Cin * k * k;
  const int epc = dtype == SAD_BF16 ? 8 : 4;
  SAD_REQUIRE(P % epc == 0 && J % epc == 0, "dgrad: N*Ho*Wo and Cin*k*k must be multiples of 16 bytes");
  SAD_REQUIRE(P < (1ll << 31) && J < (1ll << 31), "dgrad too large");
  size_t need = 0;
  sad_conv_dgrad_workspace_size(N, Ho, Wo, Cout, Cin, k, dtype, &need);
  SAD_REQUIRE(ws_bytes >= need, "dgrad workspace too small (sad_conv_dgrad_workspace_size)");
  if (P == 0) return SAD_OK;
  hipStream_t s = (hipStream_t)stream;
  const size_t es = dtype == SAD_BF16 ? 2 : 4;
  void* dyt = ws;
  float* dcol = (float*)((char*)ws + ((size_t)P * Cout * es + 255) / 256 * 256);
  const dim3 tg(nblk(P, 64), (unsigned)((Cout + 63) / 64));
  if (dtype == SAD_BF16)
    hipLaunchKernelGGL(transpose_kernel<u16>, tg, dim3(256), 0, s, (const u16*)dy, P, Cout, (u16*)dyt);
  else
    hipLaunchKernelGGL(transpose_kernel<float>, tg, dim3(256), 0, s, (const float*)dy, P, Cout, (float*)dyt);
  SAD_CHECK_HIP(hipGetLastError());
  // dcol[p][j] = sum_co dyT[co][p] * W[co][j]: B rows are W's rows (identity gather)
  KoArgs a{};
  a.a = dyt;
  a.lda = P;
  a.b = w_oihw;
  a.ldb = J;
  a.M = (int)P;
  a.N = (int)J;
  a.K = Cout;
  a.H = a.W = a.Ho = a.Wo = 1;
  a.ksz = 1;
  a.stride = 1;
  a.pad = 0;
  a.kchunk = Cout;
  a.out = dcol;
  a.a_bytes = P * Cout * (int64_t)es;
  a.b_bytes = J * Cout * (int64_t)es;
  int rc = launch_kouter(a, 1, 1, dtype, s);
  if (rc) return rc;
  return launch_col2im(dcol, N, H, W, Cin, k, stride, pad, Ho, Wo, accumulate, dx, dtype, s);
}
