// halo256r.hip -- variant 31: patch-resident 256 x 256 block conv with the
// weights streamed straight into registers (bf16, gfx950).
//
// Replaces the same timm BasicBlock halves as variants 13 / 30 (conv -> bn
// [-> + shortcut] -> relu, inference_runner.py:49-51 via timm resnet18
// forward_features) for the layer3 / layer4 convs with stride 1:
//   out[px, co] = act( sum_{tap, ci} X0[px + tap; ci] W0[co, tap, ci]
//                    + sum_{k1} X1[px * ss1; k1] W1[co, k1] + bias[co] )
//
// Why a third form.  Variants 13 and 30 stage BOTH operands in LDS and so need
// a workgroup barrier per 64-deep K-step (the weight stage of step g+1 is
// filled by DMA while step g reads the other one).  Their stamps put a K-step
// at ~3,600 cycles for 2,048 cycles of MFMA per SIMD: after every barrier both
// waves of a SIMD read fragments and issue DMA at the same time, so the matrix
// pipe idles ~1,000 cycles per step, and a DMA burst stalls the issuing wave.
// Here each of the 8 waves owns 32 output channels x all 256 pixels of the
// 16 x 16 tile:
//  * its weight fragments (2 channel tiles x 2 K-halves, 16 B per lane each)
//    are read from global memory (L2) straight into VGPRs, one K-step ahead,
//    with a counted wait -- no LDS, no barrier, no redundancy (the waves own
//    disjoint channels);
//  * the pixel operand is the 18 x 18 input patch of a 64-channel chunk in LDS
//    (variant 30's column-keyed swizzle: a fragment is a lane constant + an
//    immediate row offset), DMA'd during the previous chunk, one piece per
//    wave per tap;
//  * so the only barrier is per chunk (every 9 K-steps): within a chunk the
//    two waves of a SIMD drift freely and one's fragment reads overlap the
//    other's MFMAs.
// Per K-step and wave: 4 x 16-B weight loads, 32 ds_read_b128 (LDS ~50 % busy
// at the MFMA rate), 64 MFMA 16x16x32.  Accumulators 128 VGPRs (2 x 16 tiles).
// Epilogue: register-only (bias, ReLU, bf16, 8-B stores) or the fused average
// pool (a wave holds all 256 pixels of its channels: no cross-wave reduction).
//
// BC = 128 (layer2's 128-channel stride-1 convs): the 8 waves are 4 channel
// groups x 2 pixel halves (rows 0-7 / 8-15 of the tile), so a wave keeps the
// same 2 MFMAs per fragment read and the same weight-load count per K-step;
// the two pixel halves of a channel group load the same weights (from L2).
#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"
#include "rwconv.hpp"

namespace sad {

namespace h31 {
constexpr int NW = 8, TC = 2;           // waves; per wave 2 x 16 channels
constexpr int TW = 16, TH = 16, PW = TW + 2, PR = PW * (TH + 2);
constexpr int NDP = (PR + 7) / 8;       // 41 pieces per conv chunk
constexpr int SCR = PW * TH;            // shortcut chunk: slots ty * 18 + tx
constexpr int NDS = SCR / 8;            // 36 pieces per shortcut chunk
constexpr int PATCH = NDP * 1024;
constexpr int ROWB = PW * 128;
constexpr int SMEM = 2 * PATCH;
constexpr int BAD = 0x7FFFFFF0;
constexpr uint64_t KEY = 0xd92dad912240ull;  // variant 30's column key {0,0,1,1,2,2,4,4,5,5,6,6,2,2,6,6,0,0}
static_assert(SMEM <= 160 * 1024, "LDS budget");
}  // namespace h31

__device__ __forceinline__ int h31_key(int px) { return (int)((h31::KEY >> (3 * px)) & 7); }

typedef unsigned int h31_v4 __attribute__((ext_vector_type(4)));
typedef __bf16 h31_bf2 __attribute__((ext_vector_type(2)));
typedef float h31_f2 __attribute__((ext_vector_type(2)));
// two floats -> packed bf16 pair (RNE): one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t h31_pk(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((h31_f2){lo, hi}, h31_bf2));
}
// ReLU of a packed bf16 pair: as int16, negative bf16 values (and -0) are
// negative, so max(x, 0) per half is relu (= relu before the rounding)
__device__ __forceinline__ uint32_t h31_relu2(uint32_t x) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
  return r;
}

// BC channels per workgroup (256 or 128): NCG channel groups of 32 x NPG pixel
// groups of TP tile rows.
// X3: split-bf16 parity mode (block.hip's layout: a 128-B chunk holds 32 logical
// channels, bytes 0-63 hi = bf16(v), 64-127 lo = bf16(v - hi), for pixels and
// weights alike).  A K-step's two halves then run W_hi.X_hi + W_lo.X_hi (half 0,
// both weight halves on the hi fragment) + W_hi.X_lo (half 1): 96 MFMAs per
// K-step and wave on the same operand reads and weight loads as bf16's 64; the
// epilogue splits the fp32 result into hi / lo again.
template <int BC, bool POOL, bool X3 = false>
__global__ __launch_bounds__(512, 1) void halo256r_kernel(BlockConvArgs a) {
  using namespace h31;
  constexpr int NCG = BC / 32, NPG = NW / NCG, TP = 16 / NPG;
  static_assert(NCG * NPG == NW && (!POOL || NPG == 1), "wave split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int n_tc = a.Cout / BC;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = w % n_tc;  // both channel tiles of a pixel range share an XCD
  const int gp = gridDim.x / n_tc, wi = w / n_tc;
  const int tiles_x = a.W / TW, tiles_img = tiles_x * (a.H / TH);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)wi * tiles_p / gp), tp_end = (int)((int64_t)(wi + 1) * tiles_p / gp);
  const int c0 = tc * BC;
  if (tp_begin >= tp_end) return;  // whole workgroup (uniform)
  const int cgrp = wave % NCG, pgrp = wave / NCG;
  const int cw = c0 + cgrp * 16 * TC;  // this wave's first output channel
  const int r0w = pgrp * TP;           // this wave's first tile row

  const int cinb = a.Cin * 2;
  const int nc0 = cinb / 128;                    // conv chunks (9 taps each)
  const int nk1 = a.in1 ? a.Cin1 * 2 / 128 : 0;  // shortcut chunks (1 step each)
  const int nch = nc0 + nk1;

  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.in1 ? a.in1 : a.in0), (short)0, (int)a.in1_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps0 = (int)a.in0_pstride * 2, ps1 = (int)a.in1_pstride * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int lrow = lane >> 3;
  const int ab = a.ablate;  // timing ablations (wrong results): 1 no loads / DMA in the loop, 2 no patch DMA,
                            // 4 no weight loads, 8 no epilogue, 128 no epilogue stores

  // ---- weights: lane (fr, fg) of fragment (i, h) = row cw + i*16 + fr, K bytes
  // kb + h*64 + fg*16 of the step (kb = tap * cinb + chunk * 128)
  const int wrow = a.wt_ld * 2;
  const int wlane = (cw + fr) * wrow + fg * 16;
  auto load_w = [&](int kb, h31_v4 (&wv)[TC][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        wv[i][h] = __builtin_amdgcn_raw_buffer_load_b128(rw, wlane + i * 16 * wrow + kb + h * 64, 0, 0);
  };
  auto kb_of = [&](int c, int tap) __attribute__((always_inline)) {
    return c < nc0 ? tap * cinb + c * 128 : 9 * cinb + (c - nc0) * 128;
  };

  // ---- patch pieces of chunk c of tile t into buffer buf: piece q = wave + 8k
  // (k = -1: all of this wave's pieces); the tile origin is wave-uniform and
  // decoded once per chunk (TileO), not per piece
  struct TileO {
    int b, oy0, ox0;
    bool ok;
  };
  auto tile_o = [&](int t) __attribute__((always_inline)) {
    const int tt = __builtin_amdgcn_readfirstlane(t);
    const int b = tt / tiles_img, rem = tt - b * tiles_img;
    const int ty = rem / tiles_x;
    return TileO{b, ty * TH, (rem - ty * tiles_x) * TW, tt < tp_end};
  };
  auto issue_patch = [&](const TileO& to, int c, int buf, int k_only) __attribute__((always_inline)) {
    if (!to.ok) return;
    const int b = to.b, oy0 = to.oy0, ox0 = to.ox0;
    int lr;  // opaque lane row: keeps the per-piece (py, px) from being hoisted into registers
    asm volatile("v_mov_b32 %0, %1" : "=v"(lr) : "v"(lrow));
    const unsigned dst = lds0 + buf * PATCH;
    if (c < nc0) {
      const int base = ((b * a.H + oy0 - 1) * a.W + ox0 - 1) * ps0 + c * 128;
#pragma unroll
      for (int k = 0; k < (NDP + NW - 1) / NW; ++k) {
        const int q = wave + NW * k;
        if ((k_only < 0 || k == k_only) && q < NDP) {
          const int s = 8 * q + lr, py = s / PW, px = s - py * PW;
          const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
          const int off = (s < PR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                              ? base + (py * a.W + px) * ps0 + (((lane & 7) ^ h31_key(px)) << 4)
                              : BAD;
          dma16_m0(r0, off, dst + q * 1024);
        }
      }
    } else {
      const int base = ((b * a.H1 + oy0 * a.ss1) * a.W1 + ox0 * a.ss1) * ps1 + (c - nc0) * 128;
#pragma unroll
      for (int k = 0; k < (NDS + NW - 1) / NW; ++k) {
        const int q = wave + NW * k;
        if ((k_only < 0 || k == k_only) && q < NDS) {
          const int s = 8 * q + lr, ty = s / PW, tx = s - ty * PW;
          const int off = tx < TW ? base + (ty * a.W1 + tx) * (a.ss1 * ps1) + (((lane & 7) ^ h31_key(tx)) << 4)
                                  : BAD;
          dma16_m0(r1, off, dst + q * 1024);
        }
      }
    }
  };

  // ---- prologue loads: the first chunk's patch, step 0's weights, the bias of
  // this lane's channels (every tile's accumulators start at the bias: the
  // epilogue adds nothing)
  issue_patch(tile_o(tp_begin), 0, 0, -1);
  f32x4 biasv[TC];
#pragma unroll
  for (int i = 0; i < TC; ++i) biasv[i] = *(const f32x4*)(a.bias + cw + i * 16 + fg * 4);
  // wnxt: the weights in flight (loaded one step ahead); wcur: this step's,
  // copied from wnxt only after the step's wait
  h31_v4 wcur[TC][2], wnxt[TC][2];
  load_w(0, wnxt);

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = biasv[i];

  // this step's weights: the copy from wnxt is where the compiler waits for
  // the loads (weights are compiler-tracked buffer loads; the patch DMA pieces,
  // inline asm, are not tracked, so each such wait also covers the pieces
  // issued before it -- conservative, never short).  An inline-asm load with a
  // hand-counted vmcnt gave wrong results: the register allocator may copy an
  // asm output before the data has landed.
  auto take_w = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) wcur[i][h] = wnxt[i][h];
  };

  // ---- one K-step: 64 MFMAs; the pixel fragment of output row j, half h is at
  // patch row j + ky, column kx + fr (shortcut chunks: ky = kx = 0)
  auto step = [&](int pbuf, int ky, int kx) __attribute__((always_inline)) {
    const int pbase = pbuf * PATCH + (ky + r0w) * ROWB;
    const int o0 = (kx + fr) * 128 + ((fg ^ h31_key(kx + fr)) << 4);
    const int o1 = (kx + fr) * 128 + (((fg + 4) ^ h31_key(kx + fr)) << 4);
    const char* pb0 = smem + pbase + o0;
    const char* pb1 = smem + pbase + o1;
    auto half = [&](auto hc) __attribute__((always_inline)) {
      constexpr int h = decltype(hc)::value;
      // bf16: W_h.X_h.  Split-bf16, half 0 (the hi fragment): W_hi.X_hi and
      // W_lo.X_hi; half 1 (the lo fragment): W_hi.X_lo.
      constexpr int NM = X3 && h == 0 ? 2 : 1;  // weight halves per fragment
      const char* pb = h ? pb1 : pb0;
      uint4 bf[TP];
#pragma unroll
      for (int j = 0; j < TP; ++j) bf[j] = *(const uint4*)(pb + j * ROWB);
#pragma unroll
      for (int j = 0; j < TP; ++j)
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
          for (int i = 0; i < TC; ++i)
            mfma_chunk<u16>(__builtin_bit_cast(uint4, wcur[i][X3 ? m : h]), bf[j], acc[i][j]);
      // reads run 4 fragments ahead of the MFMAs that consume them
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int j = 0; j < TP - 4; ++j) {
        __builtin_amdgcn_sched_group_barrier(0x008, NM * TC, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * NM * TC, 0);
    };
    half(std::integral_constant<int, 0>{});
    half(std::integral_constant<int, 1>{});
  };

  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int oy0 = (rem / tiles_x) * TH, ox0 = (rem - (rem / tiles_x) * tiles_x) * TW;
    if constexpr (POOL) {
      // the wave holds all 256 pixels of its channels: relu(acc) (the bias is
      // in acc) summed over its 16 row fragments, then over the 16 lanes of a
      // row (DPP)
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        float ps[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = 0.f;
#pragma unroll
          for (int j = 0; j < TP; ++j) v += fmaxf(acc[i][j][r], 0.f);
          ps[r] = row16_sum(v);
        }
        if (fr == 0)
          *(float4*)(a.pool_out + (int64_t)b * a.Cout + cw + i * 16 + fg * 4) =
              make_float4(ps[0] * (1.f / 256), ps[1] * (1.f / 256), ps[2] * (1.f / 256), ps[3] * (1.f / 256));
      }
    } else {
      // 16-B stores (the store tail is issue-bound): for fragment rows j, j+1
      // one v_permlane16_swap per dword pairs lane row fg's 4 channels with its
      // neighbour row's, so lane rows 0/2 hold 8 channels of pixel row j and
      // rows 1/3 of row j + 1 (cdna_hip_programming.md T21, 16-lane form)
      u16* __restrict__ out = (u16*)a.out;
#pragma unroll
      for (int j = 0; j < TP; j += 2) {
        const int64_t px = (int64_t)(b * a.H + oy0 + r0w + j + (fg & 1)) * a.W + ox0 + fr;
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          if constexpr (X3) {
            // ReLU in fp32, then hi = bf16(v), lo = bf16(v - hi) (block.hip's
            // split); hi and lo go to the two 32-channel halves of the wave's
            // 128-B output chunk (cw is a multiple of 32)
            float v[2][4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[0][r] = a.relu ? fmaxf(acc[i][j][r], 0.f) : acc[i][j][r];
              v[1][r] = a.relu ? fmaxf(acc[i][j + 1][r], 0.f) : acc[i][j + 1][r];
            }
            uint32_t qh[4], ql[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float x0 = v[e >> 1][2 * (e & 1)], x1 = v[e >> 1][2 * (e & 1) + 1];
              qh[e] = h31_pk(x0, x1);
              ql[e] = h31_pk(x0 - __uint_as_float(qh[e] << 16), x1 - __uint_as_float(qh[e] & 0xFFFF0000u));
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const auto rh = __builtin_amdgcn_permlane16_swap(qh[e], qh[e + 2], false, false);
              qh[e] = rh[0];
              qh[e + 2] = rh[1];
              const auto rl = __builtin_amdgcn_permlane16_swap(ql[e], ql[e + 2], false, false);
              ql[e] = rl[0];
              ql[e + 2] = rl[1];
            }
            u16* op = out + px * a.out_pstride + 2 * cw + i * 16 + (fg >> 1) * 8;
            *(uint4*)op = make_uint4(qh[0], qh[1], qh[2], qh[3]);
            *(uint4*)(op + 32) = make_uint4(ql[0], ql[1], ql[2], ql[3]);
            continue;
          }
          const int co = cw + i * 16 + (fg >> 1) * 8;
          uint32_t q[4] = {h31_pk(acc[i][j][0], acc[i][j][1]), h31_pk(acc[i][j][2], acc[i][j][3]),
                           h31_pk(acc[i][j + 1][0], acc[i][j + 1][1]), h31_pk(acc[i][j + 1][2], acc[i][j + 1][3])};
          if (a.relu)
#pragma unroll
            for (int e = 0; e < 4; ++e) q[e] = h31_relu2(q[e]);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const auto r = __builtin_amdgcn_permlane16_swap(q[e], q[e + 2], false, false);
            q[e] = r[0];
            q[e + 2] = r[1];
          }
          if (ab & 128) {  // timing: conversion + permutes kept, no store
            asm volatile("" ::"v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[3]));
          } else {
            *(uint4*)(out + px * a.out_pstride + co) = make_uint4(q[0], q[1], q[2], q[3]);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = biasv[i];
  };

  // ---- the K loop: tiles -> chunks -> steps.  Per step: wait for its weights;
  // at a chunk start also the barrier that publishes the chunk's patch (and
  // frees the other buffer); then this step's patch piece for the next chunk
  // (conv taps 1..6: one piece per wave; a shortcut chunk: all of them), the
  // next step's weights, and the MFMAs.
  int u = 0;  // chunk counter (patch buffer parity)
  bool post_epi = false;
  for (int t = tp_begin; t < tp_end; ++t) {
    for (int c = 0; c < nch; ++c) {
      const bool sc = c >= nc0;
      const int nsteps = sc ? 1 : 9;
      const int nt = c + 1 < nch ? t : t + 1, ncn = c + 1 < nch ? c + 1 : 0;  // next chunk
      const TileO nto = tile_o(nt);
      const int pbuf = u & 1;
      for (int tap = 0; tap < nsteps; ++tap) {
        if (tap == 0) {
          // the chunk's patch pieces (this wave's); after a tile's epilogue its
          // stores (the youngest operations) may stay in flight
          if (post_epi)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(POOL ? 0 : (X3 ? 2 : 1) * TC * TP / 2) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          post_epi = false;
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");  // LDS changed behind the barrier
        }
        take_w();
        if (!(ab & 1)) {
          // the next step's weights (after the last step: a harmless reload of
          // step 0's, so the wait counts stay uniform)
          const int kbn = tap + 1 < nsteps ? kb_of(c, tap + 1) : kb_of(ncn, 0);
          if (!(ab & 4)) load_w(kbn, wnxt);
          if (ab & 2) {
          } else if (sc) {
            issue_patch(nto, ncn, pbuf ^ 1, -1);  // waited for at the next step (a chunk start)
          } else if (tap >= 1 && tap <= 6) {
            issue_patch(nto, ncn, pbuf ^ 1, tap - 1);
          }
        }
        const int ky = sc ? 0 : tap / 3, kx = sc ? 0 : tap - 3 * (tap / 3);
        step(pbuf, ky, kx);
      }
      ++u;
    }
    if (!(ab & 8)) epilogue(t);
    post_epi = true;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BC, bool POOL, bool X3>
static int launch_halo256r_t(const BlockConvArgs& a, hipStream_t s) {
  using namespace h31;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)halo256r_kernel<BC, POOL, X3>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, SMEM);
    attr = true;
  }
  const int n_tc = a.Cout / BC;
  const int64_t tiles_p = (int64_t)a.N * (a.H / TH) * (a.W / TW);
  int64_t g = std::min<int64_t>(tiles_p * n_tc, 256);
  g = std::max<int64_t>(n_tc, g / n_tc * n_tc);
  hipLaunchKernelGGL((halo256r_kernel<BC, POOL, X3>), dim3((unsigned)g), dim3(512), SMEM, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

// (a: the kernel's bf16 channel counts and strides, as launch_block_conv passes
// them; x3: the split-bf16 layout, Cin / Cin1 / strides / wt_ld already doubled,
// Cout and the bias logical)
int launch_halo256r(const BlockConvArgs& a, hipStream_t s, bool x3) {
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1, "variant 31: 3x3, stride 1, pad 1");
  SAD_REQUIRE(!a.res && !a.st_part, "variant 31: no epilogue residual / fused statistics (shortcut as in1)");
  SAD_REQUIRE(a.Cout % 128 == 0, "variant 31: Cout must be a multiple of 128");
  SAD_REQUIRE(a.H % 16 == 0 && a.W % 16 == 0 && a.Ho == a.H && a.Wo == a.W, "variant 31: image must tile by 16 x 16");
  SAD_REQUIRE((a.Cin * 2) % 128 == 0 && (!a.in1 || (a.Cin1 * 2) % 128 == 0), "variant 31: whole 128-B chunks");
  SAD_REQUIRE(!a.in1 || ((a.Ho - 1) * a.ss1 < a.H1 && (a.Wo - 1) * a.ss1 < a.W1), "variant 31: shortcut source");
  SAD_REQUIRE(a.wt_ld >= 9 * a.Cin + (a.in1 ? a.Cin1 : 0) && (a.wt_ld * 2) % 16 == 0, "variant 31: weight rows");
  SAD_REQUIRE(a.out_pstride % 8 == 0 && a.in0_pstride % 8 == 0 && (!a.in1 || a.in1_pstride % 8 == 0),
              "variant 31: pixel strides");
  SAD_REQUIRE(a.out || a.pool_out, "null output");
  SAD_REQUIRE(a.M == (int64_t)a.N * a.H * a.W, "variant 31: M = N H W");
  if (a.pool_out) {
    SAD_REQUIRE(a.H == 16 && a.W == 16 && a.Cout % 256 == 0,
                "variant 31 fused average pool: a 16 x 16 tile must be one image, Cout % 256");
    return x3 ? launch_halo256r_t<256, true, true>(a, s) : launch_halo256r_t<256, true, false>(a, s);
  }
  if (x3)
    return a.Cout % 256 == 0 ? launch_halo256r_t<256, false, true>(a, s) : launch_halo256r_t<128, false, true>(a, s);
  return a.Cout % 256 == 0 ? launch_halo256r_t<256, false, false>(a, s) : launch_halo256r_t<128, false, false>(a, s);
}

}  // namespace sad
