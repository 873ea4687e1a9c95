// block.hip -- persistent implicit-GEMM conv with the shortcut inside the GEMM.
//
// Replaces one timm BasicBlock half (conv -> bn [-> + shortcut] -> relu,
// inference_runner.py:49-51 via timm resnet18) as ONE GEMM over a concatenated
// K axis:
//   out[px, co] = act( sum_{k0} X0[px; k0] W0[co, k0]          3x3 conv, BN folded
//                    + sum_{k1} X1[px*ss1; k1] W1[co, k1]      shortcut (optional)
//                    + bias[co] )
// The shortcut is either the identity (W1 = I, exact in bf16: the residual add
// becomes MFMA work, +Cin/(9 Cin) MACs) or the 1x1/2 downsample conv + its BN
// (W1 = folded downsample weights).  So a block needs two launches instead of
// three, and no epilogue ever reads the residual tensor.
//
// Structure (gfx950):
//  * operands swapped: C^T[co, px] = W . X^T, so each lane's 16x16 MFMA
//    accumulator holds 4 CONSECUTIVE output channels of one pixel -> the
//    epilogue is register-only (bias, ReLU, bf16 pack, one 8-B store per
//    16x16 tile per lane): no LDS staging, no barrier.
//  * persistent workgroups: grid = CUs x occupancy; workgroup w owns channel
//    tile w % n_tc (so its weights' DMA offsets and its bias registers are
//    fixed) and a contiguous run of pixel tiles (neighbouring tiles share input
//    rows through the XCD's L2).  The LDS-DMA ring (S stages, inline-asm
//    buffer_load...lds, counted vmcnt) runs continuously ACROSS tile
//    boundaries, so a tile's first K-steps are in flight while the previous
//    tile finishes and stores.
//  * one K-step = one filter tap (or shortcut chunk) x 128 B of channels
//    (64 bf16 / 32 f32), 8 x 16-B chunks per pixel row, XOR-swizzled through
//    the DMA source address (LDS-DMA writes lane-linearly).
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"

#ifndef SAD_STAMPS
#define SAD_STAMPS 0
#endif

namespace sad {

// diagnostic build (-DSAD_STAMPS=1): s_memtime of one wave at a point of the
// K loop (cdna_hip_programming.md 7, in-kernel stamps); never in a product build
#define SAD_STAMP(slot)                                                                          \
  do {                                                                                           \
    if constexpr (SAD_STAMPS) {                                                                  \
      if (stamp_on) {                                                                            \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        uint64_t t_;                                                                             \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        if (lane == 0) a.stamps[(size_t)stamp_wave * 4096 + (size_t)g * 4 + (slot)] = t_;        \
      }                                                                                          \
    }                                                                                            \
  } while (0)

// WC x WP waves; each wave owns (16*TC) channels x (16*TP) pixels (TC, TP 16x16
// MFMA tiles); OCC = workgroups per CU the LDS budget admits.
template <int WC, int WP, int TC, int TP, int S>
constexpr int block_ring_bytes() {
  return S * (16 * TP * WP + 16 * TC * WC) * 128;
}
// the tile's bias rides behind the ring when OCC workgroups still fit a CU
template <int WC, int WP, int TC, int TP, int S, int OCC>
constexpr bool block_lds_bias() {
  return (block_ring_bytes<WC, WP, TC, TP, S>() + 16 * TC * WC * 4) * OCC <= 160 * 1024;
}
// the fused average pool needs a [WP][BC] fp32 partial-sum area behind the bias
// (one-workgroup-per-CU 8-wave variants)
template <int WC, int WP, int TC, int TP, int S, int OCC>
constexpr bool block_can_pool() {
  return block_lds_bias<WC, WP, TC, TP, S, OCC>() && WC * WP == 8 &&
         (block_ring_bytes<WC, WP, TC, TP, S>() + 16 * TC * WC * 4 * (1 + WP)) * OCC <= 160 * 1024;
}
template <int WC, int WP, int TC, int TP, int S, int OCC>
constexpr int block_smem_bytes() {
  return block_ring_bytes<WC, WP, TC, TP, S>() + (block_lds_bias<WC, WP, TC, TP, S, OCC>() ? 16 * TC * WC * 4 : 0) +
         (block_can_pool<WC, WP, TC, TP, S, OCC>() ? 16 * TC * WC * 4 * WP : 0);
}
// ST instantiations: + the fused BN statistics, fp32 [WP][2][BC] behind the rest
template <int WC, int WP, int TC, int TP, int S, int OCC>
constexpr int block_smem_bytes_st() {
  return block_smem_bytes<WC, WP, TC, TP, S, OCC>() + WP * 2 * 16 * TC * WC * 4;
}

// RES: the epilogue adds a residual tensor (a Bottleneck's identity shortcut,
// resnet.hip) -- its own instantiation, so the ResNet-18 kernels' register
// allocation does not carry its loads
// X3: split-bf16 parity mode (SAD_BF16X3).  Every tensor stores a logical fp32
// value v as hi = bf16(v), lo = bf16(v - hi), channels interleaved in groups of
// 32: [hi c0..31 | lo c0..31 | hi c32..63 | ...], so one 128-B K-step holds 32
// logical channels, half 0 = hi, half 1 = lo, for pixels and weights alike.  A
// K-step then runs three MFMA sets, W_hi.X_hi + W_lo.X_hi + W_hi.X_lo (the
// dropped W_lo.X_lo is ~2^-18 relative), accumulated in fp32; the epilogue
// splits the fp32 result again.  An identity shortcut (W_hi = I, W_lo = 0)
// adds X_hi + X_lo exactly.
// ST: training forward (bf16) -- the epilogue also sums the conv output and its
// square per channel (StatAcc), one [2][BC] row per pixel-group workgroup wi.
// X4 (with X3): the fourth product W_lo.X_lo too -- the deep Bottleneck plans'
// parity mode (resnet.hip: resnet50's 53 convs accumulate the dropped term past
// 1e-3 on the logits, tools/deep_x3_budget.py), +33 % MFMA work.
template <typename T, int WC, int WP, int TC, int TP, int S, int OCC, bool RES, bool X3 = false, bool ST = false,
          bool X4 = false>
__global__ __launch_bounds__(64 * WC * WP, OCC * WC * WP / 4) void block_conv_kernel(BlockConvArgs a) {
  static_assert(S == 2 || S == 3, "ring depth");
  static_assert(!X3 || sizeof(T) == 2, "split-bf16 operands are bf16");
  static_assert(!X4 || (X3 && !ST), "X4 is the split-bf16 inference form's fourth product");
  constexpr int NW = WC * WP;
  constexpr int BC = 16 * TC * WC, BP = 16 * TP * WP;  // channels x pixels per tile
  constexpr int ES = sizeof(T);
  constexpr int STAGE = (BP + BC) * 128;     // rows [0,BP): pixels, [BP,BP+BC): weights
  constexpr int QP = BP / 8 / NW, QW = BC / 8 / NW;
  static_assert(QP * 8 * NW == BP && QW * 8 * NW == BC, "tile/wave mismatch");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave / WP, wp = wave % WP;
  SAD_CLOCK_STAMP(0);
  const int n_tc = a.Cout / BC;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  // channel tile tc = w % n_tc: both channel tiles share an XCD's pixel tiles.
  // (Channel tiles by contiguous w ranges -- one tile's weights per XCD L2 --
  // measured 3-4 % slower on layer4.)
  const int tc = w % n_tc;
  const int gp = gridDim.x / n_tc, wi = w / n_tc;
  // 32-bit tile/pixel arithmetic (the launcher checks M + BP and the step count
  // fit): the per-tile pixel decomposition is 2 x QP 32-bit divisions
  const int M = (int)a.M;
  const int tiles_p = (M + BP - 1) / BP;
  const int tp_begin = (int)((int64_t)wi * tiles_p / gp), tp_end = (int)((int64_t)(wi + 1) * tiles_p / gp);
  const int c0 = tc * BC;
  if (tp_begin >= tp_end) {  // whole workgroup (uniform)
    if constexpr (ST) stat_rows_zero(BC, a.st_part, wi, a.Cout, c0, tid, 64 * NW);
    return;
  }

  const int nk0 = a.KH * a.KW * a.Cin * ES / 128;
  const int nk1 = a.in1 ? a.Cin1 * ES / 128 : 0;
  const int nk = nk0 + nk1;
  const int total = (tp_end - tp_begin) * nk;

  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.in1 ? a.in1 : a.in0), (short)0, (int)a.in1_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps0 = (int)a.in0_pstride * ES, ps1 = (int)a.in1_pstride * ES;
  const int HoWo = a.Ho * a.Wo;
  const int lrow = lane >> 3;

  // weights: fixed for the workgroup (channel tile tc)
  const int ktot_b = a.wt_ld * ES;
  int woff[QW];
#pragma unroll
  for (int i = 0; i < QW; ++i) {
    const int r = 8 * (wave + NW * i) + lrow;               // weight row (channel) in the tile
    const int c = (lane & 7) ^ (((BP + r) >> 1) & 7);       // swizzle key of LDS row BP + r
    woff[i] = (c0 + r) * ktot_b + c * 16;
  }

  // ---- issue-side state: pixel-row metadata of the tile being DMA'd
  // LEAN (8 pixel pieces per wave: variants 16, 19): per piece one row offset
  // and a tap-validity mask (bit ky*KW + kx) instead of the source row/column
  // and the shortcut offset (recomputed on its few K-steps), 16 VGPRs fewer
  constexpr bool LEAN = QP > 4;
  int poff0[QP], poff1[LEAN ? 1 : QP], piy[LEAN ? 1 : QP], pix[LEAN ? 1 : QP];
  unsigned pmask[LEAN ? QP : 1];
  int itile = tp_begin;
  // K cursor of the next DMA, kept incrementally (no scalar divisions per step):
  // step iks = (ky * KW + kx) * kpt + ci of the conv taps, then the shortcut.
  // (Channel-chunk-outer order -- consecutive steps re-reading one 64-channel
  // slice shifted by a tap -- measured 2-4 % slower on layer3/4.)
  int iks = 0, ici = 0, ikx = 0, iky = 0, itoff = 0, itap = 0;
  const int kpt = a.Cin * ES / 128;  // K-steps per tap
  auto set_tile = [&](int tp) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < QP; ++i) {
      const int r = 8 * (wave + NW * i) + lrow;
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int m = tp * BP + r;
      if (m < M) {
        const int b = (int)((unsigned)m / (unsigned)HoWo);
        const int rem = m - b * HoWo;
        const int oy = (int)((unsigned)rem / (unsigned)a.Wo), ox = rem - oy * a.Wo;
        const int iy0 = oy * a.stride - a.pad, ix0 = ox * a.stride - a.pad;
        poff0[i] = ((b * a.H + iy0) * a.W + ix0) * ps0 + c * 16;
        if constexpr (LEAN) {
          unsigned mk = 0;
          for (int ky = 0; ky < a.KH; ++ky)
            for (int kx = 0; kx < a.KW; ++kx)
              if ((unsigned)(iy0 + ky) < (unsigned)a.H && (unsigned)(ix0 + kx) < (unsigned)a.W)
                mk |= 1u << (ky * a.KW + kx);
          pmask[i] = mk;
        } else {
          piy[i] = iy0;
          pix[i] = ix0;
          poff1[i] = ((b * a.H1 + oy * a.ss1) * a.W1 + ox * a.ss1) * ps1 + c * 16;
        }
      } else {
        poff0[i] = 0;
        if constexpr (LEAN) {
          pmask[i] = 0;
        } else {
          piy[i] = -0x4000;
          pix[i] = -0x4000;
          poff1[i] = 0x7FFF0000;  // + K offset (< 64 KB) stays past num_records
        }
      }
    }
  };
  // LEAN: the shortcut source offset of piece k of tile tp
  auto shortcut_off = [&](int tp, int k) __attribute__((always_inline)) {
    const int r = 8 * (wave + NW * k) + lrow;
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int m = tp * BP + r;
    if (m >= M) return 0x7FFF0000;
    const int b = (int)((unsigned)m / (unsigned)HoWo);
    const int rem = m - b * HoWo;
    const int oy = (int)((unsigned)rem / (unsigned)a.Wo), ox = rem - oy * a.Wo;
    return ((b * a.H1 + oy * a.ss1) * a.W1 + ox * a.ss1) * ps1 + c * 16;
  };
  set_tile(itile);
  // the tile's bias, behind the ring stages (published by the first barrier);
  // epilogues read it from LDS: a global load there would put a vmcnt wait on
  // whatever reuses its registers in the next K-step
  constexpr bool LDS_BIAS = block_lds_bias<WC, WP, TC, TP, S, OCC>();
  constexpr bool POOL_OK = block_can_pool<WC, WP, TC, TP, S, OCC>();
  const float* s_bias = LDS_BIAS ? (const float*)(smem + S * STAGE) : a.bias + c0;
  if (LDS_BIAS && tid < BC / 4) *(float4*)(smem + S * STAGE + 16 * tid) = *(const float4*)(a.bias + c0 + 4 * tid);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  // one DMA piece k of K-step `iks` into stage st: k < QP pixel rows, else weight rows
  auto issue_piece = [&](int st, int k) __attribute__((always_inline)) {
    const unsigned sb = lds0 + st * STAGE;
    if (k < QP) {
      if (iks < nk0) {
        bool ok;
        if constexpr (LEAN) {
          ok = (pmask[k] >> itap) & 1u;
        } else {
          const int iy = piy[k] + iky, ix = pix[k] + ikx;
          ok = ((unsigned)iy < (unsigned)a.H) && ((unsigned)ix < (unsigned)a.W);
        }
        dma16_m0(r0, ok ? poff0[k] + itoff : 0x7FFFFFF0, sb + (wave + NW * k) * 1024);
      } else {
        const int o1 = LEAN ? shortcut_off(itile, k) : poff1[LEAN ? 0 : k];
        dma16_m0(r1, o1 + (iks - nk0) * 128, sb + (wave + NW * k) * 1024);
      }
    } else {
      dma16_m0(rw, woff[k - QP] + iks * 128, sb + BP * 128 + (wave + NW * (k - QP)) * 1024);
    }
  };
  // advance the K cursor past step iks (and to the next tile)
  auto issue_advance = [&]() __attribute__((always_inline)) {
    if (iks < nk0) {
      itoff += 128;
      if (++ici == kpt) {
        ici = 0;
        ++itap;
        itoff += ps0 - kpt * 128;
        if (++ikx == a.KW) {
          ikx = 0;
          itoff += (a.W - a.KW) * ps0;
          ++iky;
        }
      }
    }
    if (++iks == nk) {
      iks = ici = ikx = iky = itoff = itap = 0;
      if (++itile < tp_end) set_tile(itile);
    }
  };
  auto issue = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < QP + QW; ++k) issue_piece(st, k);
    issue_advance();
  };

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // ST: [WP][2][BC] fp32 statistics in LDS (register-parked sums spill here)
  float* s_stat = (float*)(smem + block_smem_bytes<WC, WP, TC, TP, S, OCC>());
  if constexpr (ST)
    for (int c = tid; c < WP * 2 * BC; c += 64 * NW) s_stat[c] = 0.f;

  const int fr = lane & 15, fg = lane >> 4;
  issue(0);
  if (S == 3 && total > 1) issue(1);
  int st = 0, cks = 0;
  int ctile = tp_begin;
  T* __restrict__ out = (T*)a.out;
  // stamps: workgroup 0, waves 0 and NW/2 (the two waves of SIMD 0's pair), steps < 1024
  const bool stamp_on0 = SAD_STAMPS && a.stamps && blockIdx.x == 0 && (wave == 0 || wave == NW / 2);
  const int stamp_wave = wave == 0 ? 0 : 1;
  for (int g = 0; g < total; ++g) {
    const bool stamp_on = stamp_on0 && g < 1024;
    SAD_STAMP(0);
    // retire this wave's DMA for step g (S = 3: step g+1's stays in flight;
    // epilogue stores issued since are waited for conservatively), then the
    // barrier publishes every wave's step-g data and frees the stage the next
    // issue overwrites.
    if (!(a.ablate & 2)) {
      if (S == 3 && g + 1 < total)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(QP + QW) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (!(a.ablate & 4)) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    SAD_STAMP(1);
    const bool do_issue = g + S - 1 < total && !(a.ablate & 1);
    const int ist = S == 3 ? (st == 0 ? 2 : st - 1) : (st ^ 1);
    const char* base = smem + st * STAGE;
    if constexpr (TC * TP > 16) {
      // 128x64 wave tiles: 128 accumulator VGPRs leave room for one K-half's
      // fragments plus half 1's pixel fragments (two waves per SIMD).  Half 1's
      // weight fragment i is read into the registers weight fragment i of half 0
      // frees after its TP MFMAs (rolling prefetch), so only half 0's reads,
      // right after the barrier, expose LDS latency.  The ring's DMA issue goes
      // after those reads and overlaps their latency.
      uint4 wf[TC], pf[TP], pg[TP];
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int r = BP + wc * 16 * TC + i * 16 + fr;
        wf[i] = *(const uint4*)(base + r * 128 + (swz(r, fg) << 4));
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = wp * 16 * TP + j * 16 + fr;
        pf[j] = *(const uint4*)(base + r * 128 + (swz(r, fg) << 4));
      }
      // SIMD partners split in time: waves 0..NW/2-1 issue the ring's DMA
      // pieces before their MFMAs, waves NW/2.. after weight row SR of half 0,
      // so one wave's DMA issue (~100 cycles a piece, in-kernel stamps) overlaps
      // its partner's MFMAs instead of both idling the SIMD's matrix pipe.
      // Same-box A/B (bench, 3 rounds): bf16 SR = 8: layer3/4 launches -3.5 %,
      // +0.6 % end to end (SR = 4: +0.4 %, 2: -0.1 %); split-bf16 SR = 2: +1 %
      // (SR = 8 spills: 1443 vs 600 us)
      const bool dma_late = wave >= NW / 2;
      if (do_issue && !dma_late) issue(ist);
      __builtin_amdgcn_sched_barrier(0);
      SAD_STAMP(2);
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = wp * 16 * TP + j * 16 + fr;
        pg[j] = *(const uint4*)(base + r * 128 + (swz(r, fg + 4) << 4));
      }
      // half 0: per weight row i its TP (X3: 2 TP) MFMAs, then the read of its
      // half-1 fragment into the freed registers; the late waves' DMA goes in
      // after row SR
      constexpr int SR = X3 ? 2 : TC;
      auto half0_row = [&](int i) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[i], pf[j], acc[i][j]);
        if constexpr (X3) {  // W_hi . X_lo while W_hi is still in registers
#pragma unroll
          for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[i], pg[j], acc[i][j]);
        }
        const int r = BP + wc * 16 * TC + i * 16 + fr;
        wf[i] = *(const uint4*)(base + r * 128 + (swz(r, fg + 4) << 4));
      };
#pragma unroll
      for (int i = 0; i < SR; ++i) half0_row(i);
      // order: half 1's pixel reads, then per row its MFMAs and its read
      __builtin_amdgcn_sched_group_barrier(0x100, TP, 0);
#pragma unroll
      for (int i = 0; i < SR; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, X3 ? 2 * TP : TP, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (do_issue && dma_late) issue(ist);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (SR < TC) {
#pragma unroll
        for (int i = SR; i < TC; ++i) half0_row(i);
#pragma unroll
        for (int i = SR; i < TC; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, X3 ? 2 * TP : TP, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[i], X3 ? pf[j] : pg[j], acc[i][j]);  // X3: W_lo . X_hi
      if constexpr (X4) {  // W_lo . X_lo
#pragma unroll
        for (int i = 0; i < TC; ++i)
#pragma unroll
          for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[i], pg[j], acc[i][j]);
      }
      SAD_STAMP(3);
    } else {
    if (do_issue) issue(ist);
    // both K-halves' fragments in registers; half 1's reads are issued between
    // half 0's MFMAs (sched_group_barrier), so only half 0's read latency is
    // exposed per K-step (the co-resident wave covers it)
    uint4 wf[2][TC], pf[2][TP];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = fg + 4 * s;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int r = BP + wc * 16 * TC + i * 16 + fr;
        wf[s][i] = *(const uint4*)(base + r * 128 + (swz(r, c) << 4));
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = wp * 16 * TP + j * 16 + fr;
        pf[s][j] = *(const uint4*)(base + r * 128 + (swz(r, c) << 4));
      }
    }
if constexpr (X3) {
      static_assert(!X3 || TC * TP >= TC + TP, "X3 schedule needs TC*TP >= TC+TP");
      // W_hi.X_hi first (half 0 only), then W_lo.X_hi and W_hi.X_lo
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[0][i], pf[0][j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[1][i], pf[0][j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[0][i], pf[1][j], acc[i][j]);
      if constexpr (X4) {
#pragma unroll
        for (int i = 0; i < TC; ++i)
#pragma unroll
          for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[1][i], pf[1][j], acc[i][j]);
      }
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<T>(wf[s][i], pf[s][j], acc[i][j]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, TC + TP, 0);
#pragma unroll
    for (int k = 0; k < TC + TP; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, (X4 ? 4 : X3 ? 3 : 2) * TC * TP - (TC + TP), 0);
    }
    st = st + 1 == S ? 0 : st + 1;
    if (++cks == nk) {
      // ---- register epilogue: lane holds channels co..co+3 of pixel px
      cks = 0;
      // bias of this lane's channels c0 + wc*16*TC + i*16 + fg*4 + r, re-read per
      // tile from LDS rather than held in 4*TC registers through the loop
      float4 bias[TC];
#pragma unroll
      for (int i = 0; i < TC; ++i) bias[i] = *(const float4*)(s_bias + wc * 16 * TC + i * 16 + fg * 4);
      if constexpr (ST) {
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float sv = 0.f, qv = 0.f;
#pragma unroll
            for (int j = 0; j < TP; ++j) {
              const int px = ctile * BP + wp * 16 * TP + j * 16 + fr;
              const float v = px < M ? acc[i][j][r] + bb[r] : 0.f;
              sv += v;
              qv += v * v;
            }
            sv = row16_sum(sv);
            qv = row16_sum(qv);
            if (fr == 0) {
              const int cl = wc * 16 * TC + i * 16 + fg * 4 + r;
              s_stat[(wp * 2 + 0) * BC + cl] += sv;
              s_stat[(wp * 2 + 1) * BC + cl] += qv;
            }
          }
        }
      }
      if constexpr (POOL_OK) {
        if (a.pool_out) {
          // fused global average pool (the backbone's last conv; a tile = one
          // image): relu(acc + bias) summed over the wave's pixels -- its TP
          // fragments, then the 16 lanes of a row by DPP rotations -- then over
          // the WP pixel waves through LDS, in a fixed order (deterministic)
          float* s_pool = (float*)(smem + S * STAGE + BC * 4);
#pragma unroll
          for (int i = 0; i < TC; ++i) {
            const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
            float ps[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = 0.f;
#pragma unroll
              for (int j = 0; j < TP; ++j) v += fmaxf(acc[i][j][r] + bb[r], 0.f);
              v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, true));
              v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, true));
              v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, true));
              v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, true));
              ps[r] = v;
            }
            if (fr == 0)
              *(float4*)(s_pool + wp * BC + wc * 16 * TC + i * 16 + fg * 4) = make_float4(ps[0], ps[1], ps[2], ps[3]);
          }
          __syncthreads();
          if (tid < BC) {
            float sum = 0.f;
#pragma unroll
            for (int w2 = 0; w2 < WP; ++w2) sum += s_pool[w2 * BC + tid];
            a.pool_out[(int64_t)ctile * a.Cout + c0 + tid] = sum * (1.f / BP);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int px = ctile * BP + wp * 16 * TP + j * 16 + fr;
        if (out != nullptr && px < M && !(a.ablate & 8)) {
          // epilogue residual (a Bottleneck's identity shortcut): the pixel's TC
          // 4-channel groups are loaded together, before any of its stores (the
          // compiler cannot move a load above a store that may alias it, so
          // interleaved loads would each wait for the stores before them)
          using RV = typename std::conditional<sizeof(T) == 2, uint2, float4>::type;
          RV rres[RES ? TC : 1], rlo[RES && X3 ? TC : 1];
          if constexpr (RES) {
            const T* rp = (const T*)a.res + (int64_t)px * a.res_pstride;
#pragma unroll
            for (int i = 0; i < TC; ++i) {
              const int co = c0 + wc * 16 * TC + i * 16 + fg * 4;
              const int pc = X3 ? ((co >> 5) << 6) + (co & 31) : co;  // split layout: hi at pc, lo at pc + 32
              rres[i] = *(const RV*)(rp + pc);
              if constexpr (X3) rlo[i] = *(const RV*)(rp + pc + 32);
            }
          }
#pragma unroll
          for (int i = 0; i < TC; ++i) {
            const int co = c0 + wc * 16 * TC + i * 16 + fg * 4;
            float v[4];
            const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] = acc[i][j][r] + bb[r];
              if constexpr (!RES) {
                if (a.relu) v[r] = fmaxf(v[r], 0.f);
              }
            }
            if constexpr (RES) {
              if constexpr (sizeof(T) == 2) {
                const uint2 q = rres[i];
                if constexpr (X3) {
                  const uint2 l = rlo[i];
                  v[0] += bf2f((u16)(q.x & 0xFFFF)) + bf2f((u16)(l.x & 0xFFFF));
                  v[1] += bf2f((u16)(q.x >> 16)) + bf2f((u16)(l.x >> 16));
                  v[2] += bf2f((u16)(q.y & 0xFFFF)) + bf2f((u16)(l.y & 0xFFFF));
                  v[3] += bf2f((u16)(q.y >> 16)) + bf2f((u16)(l.y >> 16));
                } else {
                  v[0] += bf2f((u16)(q.x & 0xFFFF));
                  v[1] += bf2f((u16)(q.x >> 16));
                  v[2] += bf2f((u16)(q.y & 0xFFFF));
                  v[3] += bf2f((u16)(q.y >> 16));
                }
              } else {
                const float4 q = rres[i];
                v[0] += q.x;
                v[1] += q.y;
                v[2] += q.z;
                v[3] += q.w;
              }
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (a.relu) v[r] = fmaxf(v[r], 0.f);
            }
            if constexpr (X3) {
              T* op = out + (int64_t)px * a.out_pstride + ((co >> 5) << 6) + (co & 31);
              u16 h[4], l[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                h[r] = f2bf(v[r]);
                l[r] = f2bf(v[r] - bf2f(h[r]));
              }
              *(uint2*)op = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
              *(uint2*)(op + 32) =
                  make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
              continue;
            }
            T* op = out + (int64_t)px * a.out_pstride + co;
            if constexpr (sizeof(T) == 2) {
              uint2 q;
              q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
              q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
              *(uint2*)op = q;
            } else {
              *(float4*)op = make_float4(v[0], v[1], v[2], v[3]);
            }
          }
        }
      }
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      ++ctile;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SAD_CLOCK_STAMP(1);
  if constexpr (ST) {  // fold the WP pixel waves of each channel
    __syncthreads();
    stat_rows_write(s_stat, WP, BC, a.st_part, wi, a.Cout, c0, tid, 64 * NW);
  }
}

template <typename T, int WC, int WP, int TC, int TP, int S, int OCC, bool RES_OK = false, bool X3 = false,
          bool ST_OK = false, bool X4 = false>
static int launch_block_t(const BlockConvArgs& a, hipStream_t s) {
  constexpr int smem0 = block_smem_bytes<WC, WP, TC, TP, S, OCC>();
  static_assert(smem0 * OCC <= 160 * 1024, "LDS budget");
  static_assert(!ST_OK || block_smem_bytes_st<WC, WP, TC, TP, S, OCC>() * OCC <= 160 * 1024, "LDS budget (ST)");
  const int smem = a.st_part ? block_smem_bytes_st<WC, WP, TC, TP, S, OCC>() : smem0;
  SAD_REQUIRE(RES_OK || !a.res, "this block-conv variant has no epilogue residual (variants 13, 20, 21, 25 do)");
  SAD_REQUIRE(16 * TP * WP / 8 / (WC * WP) <= 4 || a.KH * a.KW <= 32, "variants 16 / 19: at most 32 filter taps");
  static_assert(!(ST_OK && X4), "no fused statistics in the four-product form");
  const void* kfn = (const void*)block_conv_kernel<T, WC, WP, TC, TP, S, OCC, false, X3, false, X4>;
  if constexpr (RES_OK) {
    if (a.res) kfn = (const void*)block_conv_kernel<T, WC, WP, TC, TP, S, OCC, true, X3, false, X4>;
  }
  if constexpr (ST_OK) {
    if (a.st_part) kfn = (const void*)block_conv_kernel<T, WC, WP, TC, TP, S, OCC, false, X3, true>;
  }
  SAD_REQUIRE(!a.st_part || (ST_OK && !a.res && !a.pool_out && a.st_rows),
              "fused BN statistics: variants 13 / 15 (bf16), no residual or pool, st_rows set");
  static bool attr[3] = {false, false, false};
  const int ak = a.st_part ? 2 : a.res != nullptr;
  if (!attr[ak]) {
    (void)hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr[ak] = true;
  }
  constexpr int BC = 16 * TC * WC, BP = 16 * TP * WP;
  const int occupancy = OCC;
  if (a.pool_out) {
    SAD_REQUIRE((block_can_pool<WC, WP, TC, TP, S, OCC>()), "fused average pool: variant has no LDS for it");
    SAD_REQUIRE(a.Ho * a.Wo == BP && a.M % BP == 0 && !a.res, "fused average pool: a pixel tile must be one image");
  }
  SAD_REQUIRE(a.out || a.pool_out, "null output");
  SAD_REQUIRE(a.Cout % BC == 0, "Cout must be a multiple of the channel tile");
  const int n_tc = a.Cout / BC;
  const int64_t tiles_p = (a.M + BP - 1) / BP;
  int64_t g = std::min<int64_t>(tiles_p * n_tc, (int64_t)256 * occupancy);
  g = std::max<int64_t>(n_tc, g / n_tc * n_tc);
  const int64_t nk = (int64_t)a.KH * a.KW * a.Cin * sizeof(T) / 128 + (a.in1 ? a.Cin1 * sizeof(T) / 128 : 0);
  SAD_REQUIRE(a.M + BP < (1ll << 31) && (tiles_p / (g / n_tc) + 1) * nk < (1ll << 31),
              "block conv: too many pixels for one launch (lower the micro-batch)");
  if constexpr (ST_OK) {
    if (a.st_part) {
      *a.st_rows = (int)(g / n_tc);
      hipLaunchKernelGGL((block_conv_kernel<T, WC, WP, TC, TP, S, OCC, false, X3, true>), dim3((unsigned)g),
                         dim3(64 * WC * WP), smem, s, a);
      SAD_CHECK_HIP(hipGetLastError());
      return SAD_OK;
    }
  }
  if constexpr (RES_OK) {
    if (a.res) {
      hipLaunchKernelGGL((block_conv_kernel<T, WC, WP, TC, TP, S, OCC, true, X3, false, X4>), dim3((unsigned)g),
                         dim3(64 * WC * WP), smem, s, a);
      SAD_CHECK_HIP(hipGetLastError());
      return SAD_OK;
    }
  }
  hipLaunchKernelGGL((block_conv_kernel<T, WC, WP, TC, TP, S, OCC, false, X3, false, X4>), dim3((unsigned)g),
                     dim3(64 * WC * WP),
                     smem, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

// Variants (channels x pixels tile, waves, wave tile, ring stages, LDS, workgroups/CU):
//  9: 64x256  4w 64x64  S2  80 KB 2     10: 128x128 4w 64x64  S2  64 KB 2
// 11: 64x256  4w 64x64  S3 120 KB 1     12: 128x128 4w 64x64  S3  96 KB 1
// 13: 256x256 8w 128x64 S2 128 KB 1     14: 128x256 8w 64x64  S2  96 KB 1
// 15: 128x256 8w 64x64  S3 144 KB 1     16: 64x512  8w 64x64  S2 144 KB 1
// 17: 256x128 4w 128x64 S2  96 KB 1     18: 128x256 4w 64x128 S2  96 KB 1
// 19: 128x512 8w 128x64 S2 160 KB 1 (Cout 128: the 256x256 kernel's wave tile and
//     LDS fill per FLOP within 20 %; the bias is read from global, no LDS left)
template <typename T, bool X3 = false>
static int launch_block_v(const BlockConvArgs& a, int v, hipStream_t s) {
  switch (v) {
    case 9: return launch_block_t<T, 1, 4, 4, 4, 2, 2, false, X3>(a, s);
    case 10: return launch_block_t<T, 2, 2, 4, 4, 2, 2, false, X3>(a, s);
    case 11: return launch_block_t<T, 1, 4, 4, 4, 3, 1, false, X3>(a, s);
    case 12: return launch_block_t<T, 2, 2, 4, 4, 3, 1, false, X3>(a, s);
    case 13: return launch_block_t<T, 2, 4, 8, 4, 2, 1, true, X3, sizeof(T) == 2 && !X3>(a, s);
    case 14: return launch_block_t<T, 2, 4, 4, 4, 2, 1, false, X3>(a, s);
    case 15: return launch_block_t<T, 2, 4, 4, 4, 3, 1, false, X3, sizeof(T) == 2 && !X3>(a, s);
    case 16: return launch_block_t<T, 1, 8, 4, 4, 2, 1, false, X3>(a, s);
    case 17: return launch_block_t<T, 2, 2, 8, 4, 2, 1, false, X3>(a, s);
    case 18: return launch_block_t<T, 2, 2, 4, 8, 2, 1, false, X3>(a, s);
    case 19: return launch_block_t<T, 1, 8, 8, 4, 2, 1, false, X3>(a, s);
  }
  set_error("unknown block-conv variant");
  return SAD_ERR_ARG;
}
// the four-product split-bf16 form (BlockConvArgs.x4): the implicit-GEMM
// variants gemm_block_variant picks (Cout 64, 128, multiples of 256)
static int launch_block_x4(const BlockConvArgs& a, int v, hipStream_t s) {
  switch (v) {
    case 9: return launch_block_t<u16, 1, 4, 4, 4, 2, 2, false, true, false, true>(a, s);
    case 13: return launch_block_t<u16, 2, 4, 8, 4, 2, 1, true, true, false, true>(a, s);
    case 15: return launch_block_t<u16, 2, 4, 4, 4, 3, 1, false, true, false, true>(a, s);
  }
  set_error("four-product split-bf16 convs run on the implicit-GEMM variants 9, 13, 15");
  return SAD_ERR_ARG;
}

int launch_halo_v(const BlockConvArgs& a, int v, hipStream_t s, bool x3 = false);
int launch_halo256(const BlockConvArgs& a, hipStream_t s, bool x3);
int launch_halo256r(const BlockConvArgs& a, hipStream_t s, bool x3);
bool halo256_ok(const BlockConvArgs& a);
int launch_halo_rw(const BlockConvArgs& a, hipStream_t s);
int launch_l2conv(const BlockConvArgs& a, hipStream_t s, bool x3 = false);
int launch_halo256s2(const BlockConvArgs& a, hipStream_t s);
bool halo256s2_ok(const BlockConvArgs& a);
int launch_halo_rw_x3(const BlockConvArgs& a, hipStream_t s);
int launch_l2s2conv(const BlockConvArgs& a, hipStream_t s);
int launch_halo256rs2(const BlockConvArgs& a, hipStream_t s, bool x3);
bool halo256rs2_ok(const BlockConvArgs& a);

// halo kernel (variant 20): bf16 stride-1 3x3 with Cout <= 128 (layer1, layer2's
// second block), where the implicit GEMM is L2->LDS-fill bound (convbench,
// mb 128: layer1 c2 261 vs 350 us, layer2 c1 187 vs 218 us); for Cout >= 256
// the patch would be re-loaded per 64-channel tile.  It is also the only
// kernel taking `res`.
// (split-bf16: logical channels; the kernel sees 2 Cin bf16 channels)
static bool halo_ok(const BlockConvArgs& a, int dtype) {
  return (dtype == SAD_BF16 || dtype == SAD_BF16X3) && a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 &&
         !a.in1 && a.Cin % (dtype == SAD_BF16X3 ? 32 : 64) == 0 && a.Cout % 64 == 0 && a.W % 16 == 0 &&
         a.H % 16 == 0;
}
// SAD_L2_HALO=0 runs layer2's second block on the implicit-GEMM kernel (identity
// shortcut as MFMA columns) instead of the halo kernel (A/B switch)
// SAD_L2_V31=1 runs layer2's stride-1 convs on variant 31 with 128-channel
// tiles (4 channel groups x 2 pixel halves; identity / downsample as shortcut
// columns) instead of the halo kernel (variant 20, identity as an epilogue
// residual) and the implicit GEMM (variant 15, conv2 + downsample).  Measured
// 2.2-2.7 % slower end to end (same box, 3 rounds: 52.4k vs 53.7k seg/s): at
// 128 channels a K-step is half the MFMAs for the same per-step weight loads,
// waits and chunk barriers.  Off by default; tested (test_gpu_blockconv.py).
bool layer2_v31() {
  static const bool v = [] {
    const char* e = getenv("SAD_L2_V31");
    return e ? atoi(e) != 0 : false;
  }();
  return v;
}
// variant 31's contract (either tile width): 3x3/s1/p1, 16 x 16 tiles, whole
// 128-B chunks, no epilogue residual / statistics
static bool halo31_ok(const BlockConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Cout % 128 == 0 && a.H % 16 == 0 &&
         a.W % 16 == 0 && a.Ho == a.H && a.Wo == a.W && !a.res && !a.st_part && a.Cin % 64 == 0 &&
         (!a.in1 || a.Cin1 % 64 == 0) && (!a.pool_out || (a.H == 16 && a.W == 16 && a.Cout % 256 == 0));
}
// SAD_X3_L2_V31 (split-bf16): layer2's stride-1 convs (layer2.0's conv2 +
// downsample, layer2.1's two; identity / downsample as shortcut columns) on
// variant 31's split form with 128-channel tiles instead of the weight-ring
// halo kernel (variant 20) and the implicit GEMM (variant 15)
bool x3_layer2_v31() {
  static const bool v = [] {
    const char* e = getenv("SAD_X3_L2_V31");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}
// SAD_L2_RW=0 runs layer2's second block on the weight-ring halo kernel
// (variant 20) instead of the resident-weight conv (variant 41; A/B switch)
static bool l2_rw() {
  static const bool v = [] {
    const char* e = getenv("SAD_L2_RW");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}
// SAD_L2_DS_RW=0 runs layer2.0's conv2 + downsample on the implicit GEMM
// (variant 15) instead of variant 41's downsample form (A/B switch)
static bool l2_ds_rw() {
  static const bool v = [] {
    const char* e = getenv("SAD_L2_DS_RW");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}
// variant 41's downsample form: 128 -> 128 3x3/s1/p1 + 1x1/2 of a 64-channel
// input at twice the size
static bool l2conv_ds_ok(const BlockConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Cin == 128 && a.Cout == 128 && a.H % 16 == 0 &&
         a.W % 16 == 0 && a.Ho == a.H && a.Wo == a.W && a.in1 && a.Cin1 == 64 && a.ss1 == 2 && a.H1 == 2 * a.H &&
         a.W1 == 2 * a.W && !a.res && !a.pool_out && !a.st_part;
}
// SAD_S2_PATCH (default 1 since round 4; 0 = the implicit GEMM, variants 13 /
// 15) runs the stride-2 3x3 convs that variant 43 does not take (layer3/4's
// first conv, bf16) on the patch-resident variant 32 (halo256s2.hip).  Round 3
// measured it slower at micro-batch 512 (l2.c1 644 vs 523 us, l3.c1 344 vs
// 328, l4.c1 284 vs 276, -1.6 % end to end, with layer2's conv1 on it too; its
// ablations put 29-35 % of its time in the patch DMA and 17-25 % in the
// epilogue).  At the round-4 micro-batch of 2,048 with layer2's conv1 on
// variant 43 it is +0.2 % end to end, 3 of 3 same-box rounds
// (profiles/r04_s2patch_ab.log).  Tested (test_gpu_blockconv.py).
// Round 5: variant 44 (SAD_S2_PATCH=2, the default since round 5;
// halo256rs2.hip: 64-channel chunks, whole 128-B lines per DMA piece, the
// 33 x 33 patch single-buffered as four parity planes) reads the input once:
// 1.20 vs 1.98 GB per bench launch (rocprof).  Its first form was slower (841 vs
// 773 us per launch); with the tile decode hoisted out of the DMA issue and the
// tap tables as SALU immediates: convbench mb 1,024 l3.c1 630 vs 682 us, l4.c1
// 552 vs 553; end to end +0.2 % (2 of 3 same-box rounds,
// profiles/r05_s2_ab.log).  SAD_S2_PATCH=1 keeps variant 32.
static int s2_patch() {
  static const int v = [] {
    const char* e = getenv("SAD_S2_PATCH");
    return e ? atoi(e) : 2;
  }();
  return v;
}
// SAD_X3_S2 (split-bf16): 44 (default) runs layer3/4's stride-2 convs on
// variant 44's split form, 0 on the split implicit GEMM (variants 13 / 15).
// Convbench mb 512: l3.c1 692 vs 741 us, l4.c1 610 vs 617; layer2's conv1
// (Cout 128) ties (1,071 vs 1,066) and stays on the GEMM; end to end neutral
// (profiles/r05_s2_ab.log), kept for the bytes (1.2 vs 1.8-1.9 GB per launch).
static int x3_s2_variant() {
  static const int v = [] {
    const char* e = getenv("SAD_X3_S2");
    return e ? atoi(e) : 44;
  }();
  return v;
}
// SAD_L2S2_RW=0 runs layer2.0's stride-2 conv1 (64 -> 128) on the implicit
// GEMM (variant 15) instead of the resident-weight stride-2 conv (variant 43,
// l2s2conv.hip; A/B switch)
static bool l2s2_rw() {
  static const bool v = [] {
    const char* e = getenv("SAD_L2S2_RW");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}
// variant 43's contract: 64 -> 128 3x3/s2/p1, output tiles 16 x 16, input
// exactly twice the output, no shortcut / residual / pool
// (the trainer's raw conv may add fused statistics: launch_l2s2conv checks them)
static bool l2s2_ok(const BlockConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.stride == 2 && a.pad == 1 && a.Cin == 64 && a.Cout == 128 && a.Ho % 16 == 0 &&
         a.Wo % 16 == 0 && a.H == 2 * a.Ho && a.W == 2 * a.Wo && !a.in1 && !a.res && !a.pool_out;
}
bool layer2_halo() {
  static const bool v = [] {
    const char* e = getenv("SAD_L2_HALO");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}
// SAD_C128_VARIANT: block-conv variant for Cout = 128 GEMM convs (layer2's first
// block; A/B switch).  15 (128x256, 8 waves, 3 stages) over 10 (128x128, 4
// waves, 2 workgroups/CU): l2.c1 580 -> 473 us in isolation at mb 512, +0.5 %
// end-to-end same-box (gpurun_out/ab_c128.log)
static int c128_variant() {
  static const int v = [] {
    const char* e = getenv("SAD_C128_VARIANT");
    return e ? atoi(e) : 15;
  }();
  return v;
}
// SAD_HALO_C128: halo variant for the Cout = 128 stride-1 convs (layer2's second
// block): 20 (64-channel tiles, two workgroups per tile) or 22 (128-channel
// tiles, 64 x 64 wave tiles, register epilogue); A/B switch
static int halo_c128_variant() {
  static const int v = [] {
    const char* e = getenv("SAD_HALO_C128");
    return e ? atoi(e) : 20;
  }();
  return v;
}
// SAD_X3_L1 (split-bf16 layer1, A/B): 42 = the resident-weight conv of layer2's
// bf16 kernel in its split form (l2conv.hip: 288 weight registers per wave, all
// 64 logical channels per workgroup, 3 MFMAs per fragment read), 26 = round 2's
// half-the-channels kernel (weights in LDS)
static int x3_l1_variant() {
  static const int v = [] {
    const char* e = getenv("SAD_X3_L1");
    return e ? atoi(e) : 42;
  }();
  return v;
}
// SAD_X3_RW=0 runs split-bf16 layer1 on the weight-ring halo kernel (variant 20) instead of variant 26 (A/B)
static bool x3_rw() {
  static const bool v = [] {
    const char* e = getenv("SAD_X3_RW");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}
// The stride-1 3x3 convs with Cout % 256 == 0 (layer3/4): bf16 runs the
// patch-resident variant 31 (weights streamed into registers, one barrier per
// 64-channel chunk; 6-10 % faster than variant 13 per launch, +3 % end to end
// same-box); split-bf16 variant 30's split form (below).  SAD_HALO256 (A/B
// switch): 0 = variant 13 for both, 1 = variant 30 for both, 2 = the default.
// SAD_X3_HALO256: the split-bf16 parity mode's layer3/4 stride-1 convs on
// variant 30 (default since round 4: its split form is +1.2 % end to end in the
// parity mode over variant 31's, same box, 2 rounds, profiles/
// r04_x3_halo256_ab.log) or 31; SAD_HALO256=0 still puts both modes on variant 13
static int x3_halo256_variant() {
  static const int v = [] {
    const char* e = getenv("SAD_X3_HALO256");
    return e ? atoi(e) : 30;
  }();
  return v;
}
static int halo256_mode() {
  static const int v = [] {
    const char* e = getenv("SAD_HALO256");
    return e ? atoi(e) : 2;
  }();
  return v;
}
static int block_device_cus() {
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
int default_block_variant(const BlockConvArgs& a, int dtype) {
  // split-bf16: the halo kernel for the stride-1 convs of layer1 (Cout 64) and
  // layer2 (Cout 128), whose implicit GEMM is L2->LDS-fill bound
  if (dtype == SAD_BF16X3) {
    // layer1 (64 -> 64): the resident-weight split-bf16 kernel (half the channels per workgroup)
    if (halo_ok(a, dtype) && a.Cin == 64 && a.Cout == 64 && x3_l1_variant() == 42) return 42;
    if (halo_ok(a, dtype) && a.Cin == 64 && a.Cout == 64 && x3_rw()) return 26;
    if (x3_layer2_v31() && a.Cout == 128 && halo31_ok(a)) return 31;
    // layer3/4 stride-1 convs: variant 30's split form (or 31's; chosen
    // whatever the grid size: their K orders differ from variant 13's)
    if (halo256_mode() != 0 && (halo256_mode() == 1 || x3_halo256_variant() == 30) && halo256_ok(a)) return 30;
    if (halo256_mode() == 2 && x3_halo256_variant() == 31 && a.Cout % 256 == 0 && halo31_ok(a)) return 31;
    // the stride-2 convs (layer2/3/4's conv1): variant 44's split form (chosen
    // whatever the grid size: its K order differs from the implicit GEMM's)
    if (x3_s2_variant() == 44 && halo256rs2_ok(a) && a.Cout % 256 == 0) return 44;
    return halo_ok(a, dtype) && a.Cout <= 128 ? 20 : (a.Cout % 256 == 0 ? 13 : (a.Cout % 128 == 0 ? c128_variant() : 9));
  }
  if (halo_ok(a, dtype) && a.Cin == 64 && a.Cout == 64) return 25;  // layer1: resident weights
  // layer2's second block (128 -> 128, stride 1, identity as an epilogue
  // residual): the resident-weight conv (variant 41)
  if (dtype == SAD_BF16 && l2_rw() && halo_ok(a, dtype) && a.Cin == 128 && a.Cout == 128 && !a.st_part) return 41;
  // layer2's first block, conv2 + the downsample (its 1x1/2 of the 64-channel
  // block input as two more K-steps): the same kernel
  if (dtype == SAD_BF16 && l2_ds_rw() && l2conv_ds_ok(a)) return 41;
  // layer2's 128-channel stride-1 convs (incl. conv2 + downsample / identity as
  // shortcut columns): variant 31 with 128-channel tiles
  if (dtype == SAD_BF16 && layer2_v31() && a.Cout == 128 && halo31_ok(a)) return 31;
  if (halo_ok(a, dtype) && (a.res || (a.Cout <= 128 && layer2_halo())))
    return a.Cout == 128 && !a.res && halo_c128_variant() == 22 ? 22 : 20;
  // layer3/4 stride-1 convs: the patch-resident kernels (bf16 only: the fp32
  // parity path stays on the implicit GEMM), chosen whatever the grid size: variants 30/31 sum K in a different order than
  // 13/15, and a batch-size-dependent switch would make results depend on the
  // micro-batch (a 1-rank and a 2-rank run of the same segments must agree
  // bit for bit)
  if (dtype == SAD_BF16 && halo256_mode() != 0 && halo256_ok(a)) return halo256_mode() == 2 ? 31 : 30;
  // layer2's stride-2 conv1 (64 -> 128): resident weights (variant 43; chosen
  // whatever the grid size: its K order differs from variant 15's)
  if (dtype == SAD_BF16 && l2s2_rw() && l2s2_ok(a)) return 43;
  // the stride-2 3x3 convs: the patch-resident variant 32 (chosen whatever the
  // grid size, as above)
  if (dtype == SAD_BF16 && s2_patch() == 2 && halo256rs2_ok(a)) return 44;
  if (dtype == SAD_BF16 && s2_patch() == 1 && halo256s2_ok(a)) return 32;
  return gemm_block_variant(a);
}
// the implicit-GEMM choice (also the fused-statistics path's: 30/31 sum no
// statistics).  Small maps (the trainer's 64-segment layer4: M = 16384): 256x256
// tiles would leave CUs idle (one workgroup per CU), so split the channel tile
// (variant 15, 128x256).  Both keep the 256-pixel tile and the same K order, so
// the results (incl. the fused average pool) do not depend on the choice.
int gemm_block_variant(const BlockConvArgs& a) {
  if (a.Cout % 256 == 0)
    return a.res || (a.M + 255) / 256 * (a.Cout / 256) >= block_device_cus() ? 13 : 15;  // 13: residual epilogue
  return a.Cout % 128 == 0 ? c128_variant() : 9;
}
// pixel tile of the variants that can fuse the average pool (0: cannot)
static int pool_tile(int v) {
  switch (v) {
    case 13: case 14: case 15: case 30: case 31: return 256;
    case 16: return 512;
  }
  return 0;
}
bool block_conv_can_pool(const BlockConvArgs& a, int dtype) {
  const int v = default_block_variant(a, dtype);
  const int bp = pool_tile(v);
  return bp > 0 && a.Ho * a.Wo == bp && !a.res && a.M % bp == 0 && (v != 31 || a.Cout % 256 == 0);
}
static bool variant_fits(int v, int cout) {
  if (v == 26 || v == 42) return cout == 64;
  if (v == 30) return cout % 256 == 0;
  if (v == 31 || v == 32 || v == 44) return cout % 128 == 0;
  const int bc[] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 64, 128, 64, 128, 256, 128, 128, 64, 256, 128, 128};
  if (v == 20 || v == 21) return cout % 64 == 0;
  if (v == 22) return cout % 128 == 0;
  if (v == 25) return cout == 64;
  if (v == 41 || v == 43) return cout == 128;
  return v >= 9 && v <= 19 && cout % bc[v] == 0;
}

#if SAD_STAMPS
// diagnostic build: stamp the launch, synchronise, print the per-step phase
// averages (cycles) of wave 0 and wave NW/2 of workgroup 0 to stderr
constexpr size_t kStampWords = SAD_CLOCK_BASE + 4 * SAD_CLOCK_WGS;
// SAD_STAMP_EVERY=n: stamp only every n-th launch of a stamped variant (the
// others run unstamped and unsynchronised, so a loop keeps the chip loaded)
static bool stamp_this_launch(int which) {  // counted per stamped variant
  static const int every = [] {
    const char* e = getenv("SAD_STAMP_EVERY");
    return e ? std::max(1, atoi(e)) : 1;
  }();
  static long count[2] = {0, 0};
  return count[which]++ % every == every - 1;
}
static int stamp_report(const BlockConvArgs& a, hipStream_t s) {
  std::vector<uint64_t> h(kStampWords);
  SAD_CHECK_HIP(hipStreamSynchronize(s));
  SAD_CHECK_HIP(hipMemcpy(h.data(), a.stamps, h.size() * 8, hipMemcpyDeviceToHost));
  {  // in-kernel clock over workgroups; ramp and tail from the 100 MHz clock
    std::vector<double> clk, dur, xcd[8];
    uint64_t r0 = ~0ull, r0max = 0, r1min = ~0ull, r1 = 0;
    for (int g = 0; g < SAD_CLOCK_WGS; ++g) {
      const uint64_t* c = &h[SAD_CLOCK_BASE + 4 * g];
      if (!c[0] || !c[2] || c[3] <= c[1]) continue;
      clk.push_back((double)(c[2] - c[0]) / (double)(c[3] - c[1]) * 100.0);  // MHz
      xcd[g % 8].push_back(clk.back());  // workgroups go round-robin over the 8 XCDs
      dur.push_back((double)(c[3] - c[1]) / 100.0);                          // us
      r0 = std::min(r0, c[1]); r0max = std::max(r0max, c[1]);
      r1min = std::min(r1min, c[3]); r1 = std::max(r1, c[3]);
    }
    if (!clk.empty()) {
      std::sort(clk.begin(), clk.end());
      std::sort(dur.begin(), dur.end());
      fprintf(stderr, "clock M=%lld Cout=%d: %zu workgroups, in-kernel clock median %.0f MHz (min %.0f, max %.0f); "
              "span %.1f us, workgroup time median %.1f us (min %.1f, max %.1f), starts spread %.1f us, "
              "ends spread %.1f us\n", (long long)a.M, a.Cout, clk.size(), clk[clk.size() / 2], clk.front(),
              clk.back(), (r1 - r0) / 100.0, dur[dur.size() / 2], dur.front(), dur.back(), (r0max - r0) / 100.0,
              (r1 - r1min) / 100.0);
      fprintf(stderr, "clock per XCD (median MHz):");
      for (auto& x : xcd) {
        if (x.empty()) continue;
        std::sort(x.begin(), x.end());
        fprintf(stderr, " %.0f", x[x.size() / 2]);
      }
      fprintf(stderr, "\n");
    }
  }
  for (int w = 0; w < 2; ++w) {
    double ph[4] = {0, 0, 0, 0};
    int n = 0;
    for (int g = a.N <= 64 ? 1 : 8; g + 1 < 1024; ++g) {  // small launches: skip only the first step
      const uint64_t* t = &h[w * 4096 + g * 4];
      const uint64_t t0n = h[w * 4096 + (g + 1) * 4];
      if (!t[0] || !t[3] || !t0n || t0n < t[3]) break;
      ph[0] += (double)(t[1] - t[0]);
      ph[1] += (double)(t[2] - t[1]);
      ph[2] += (double)(t[3] - t[2]);
      ph[3] += (double)(t0n - t[3]);
      ++n;
    }
    if (n)
      fprintf(stderr, "stamps M=%lld Cout=%d K=%d wave %d: %d steps, cycles/step phases 0-1 %.0f | 1-2 %.0f | "
              "2-3 %.0f | 3-next %.0f | total %.0f\n", (long long)a.M, a.Cout, a.KH * a.KW * a.Cin, w, n,
              ph[0] / n, ph[1] / n, ph[2] / n, ph[3] / n, (ph[0] + ph[1] + ph[2] + ph[3]) / n);
  }
  return SAD_OK;
}
#endif

// per host thread: a launch from another thread inside a caller's
// before/after bracket (sad_profile_*) must not land in that caller's count
static thread_local int64_t g_block_conv_kernels = 0;
int64_t block_conv_kernel_launches() { return g_block_conv_kernels; }

int launch_block_conv(const BlockConvArgs& a_in, int dtype, hipStream_t s, int variant) {
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16 || dtype == SAD_BF16X3, "dtype");
  const int ES = dtype == SAD_F32 ? 4 : 2;
  BlockConvArgs a = a_in;
  if (dtype == SAD_BF16X3) {
    // callers count logical channels; the kernel sees the split layout's bf16
    // channels (2 per logical channel, hi/lo interleaved in groups of 32)
    SAD_REQUIRE(a.Cin % 32 == 0 && a.Cin1 % 32 == 0, "split-bf16: channels must be multiples of 32");
    a.Cin *= 2;
    a.Cin1 *= 2;
    a.in0_pstride *= 2;
    a.in1_pstride *= 2;
    a.out_pstride *= 2;
    a.res_pstride *= 2;
    a.wt_ld *= 2;
  }
  a.in0_bytes = (((int64_t)a.N * a.H * a.W - 1) * a.in0_pstride + a.Cin) * ES;
  a.in1_bytes = a.in1 ? (((int64_t)a.N * a.H1 * a.W1 - 1) * a.in1_pstride + a.Cin1) * ES : 0;
  if (a.wt_ld == 0) a.wt_ld = a.KH * a.KW * a.Cin + (a.in1 ? a.Cin1 : 0);
  SAD_REQUIRE(a.wt_ld >= a.KH * a.KW * a.Cin + (a.in1 ? a.Cin1 : 0) && (a.wt_ld * ES) % 16 == 0, "weight row length");
  a.wt_bytes = (int64_t)a.Cout * a.wt_ld * ES;
  // (split-bf16: a pixel's residual is 2 Cout bf16, hi and lo -- Cout stays logical)
  a.res_bytes = a.res ? (a.M - 1) * a.res_pstride * ES + (dtype == SAD_BF16X3 ? 2 : 1) * a.Cout * ES : 0;
  // The kernels address their operands through 32-bit buffer offsets.  A batch
  // whose operands exceed that range runs as consecutive launches over image
  // ranges (every conv here is independent per image, so the results are the
  // single launch's, bit for bit); the fused-statistics launch, whose
  // per-workgroup rows would collide, is not split.
  const int64_t lim = (1ll << 31) - 65536;
  // (the output too: variants 31 / 41 check it against the same range)
  const int64_t out_bytes = a.out ? ((a.M - 1) * a.out_pstride + a.Cout) * ES : 0;
  if ((a.in0_bytes >= lim || a.in1_bytes >= lim || a.res_bytes >= lim || out_bytes >= lim) && a.N > 1 &&
      a.M == (int64_t)a.N * a.Ho * a.Wo && !a.st_part) {
    const int64_t img0 = (int64_t)a.H * a.W * a.in0_pstride * ES;
    const int64_t img1 = a.in1 ? (int64_t)a.H1 * a.W1 * a.in1_pstride * ES : 0;
    const int64_t imgr = a.res ? (int64_t)a.Ho * a.Wo * a.res_pstride * ES : 0;
    const int64_t imgo = (int64_t)a.Ho * a.Wo * a.out_pstride * ES;
    const int64_t per = std::max(std::max(img0, imgo), std::max(img1, imgr));
    const int64_t ncap = (lim - 65536) / per;
    SAD_REQUIRE(ncap >= 1, "one image exceeds the 2 GiB buffer range");
    // equal ranges (1,024 images at 2 GiB + a bit: 512 + 512, not 1,023 + a
    // 1-image launch whose grid is almost empty)
    const int64_t nl = (a.N + ncap - 1) / ncap, nc = (a.N + nl - 1) / nl;
    for (int64_t n0 = 0; n0 < a.N; n0 += nc) {
      const int n = (int)std::min<int64_t>(nc, a.N - n0);
      BlockConvArgs c = a_in;  // logical channel counts (split-bf16 doubles them again)
      c.N = n;
      c.M = (int64_t)n * a.Ho * a.Wo;
      c.in0 = (const char*)a.in0 + n0 * img0;
      if (a.in1) c.in1 = (const char*)a.in1 + n0 * img1;
      if (a.res) c.res = (const char*)a.res + n0 * imgr;
      if (a.out) c.out = (char*)a.out + n0 * imgo;
      if (a.pool_out) c.pool_out = a.pool_out + n0 * a.Cout;
      if (int rc = launch_block_conv(c, dtype, s, variant)) return rc;
    }
    return SAD_OK;
  }
  SAD_REQUIRE(a.in0_bytes < (1ll << 31) - 65536 && a.in1_bytes < (1ll << 31) - 65536 && a.wt_bytes < (1ll << 31) &&
                  a.res_bytes < (1ll << 31) - 65536,
              "block conv operand exceeds the 2 GiB buffer range (lower the micro-batch)");
  SAD_REQUIRE((a.Cin * ES) % 128 == 0 && (!a.in1 || (a.Cin1 * ES) % 128 == 0),
              "channels must fill whole 128-B K-steps");
  SAD_REQUIRE(a.Cout % 64 == 0 && a.out_pstride % 4 == 0, "Cout / output stride");
  SAD_REQUIRE(a.in0_pstride % (16 / ES) == 0 && (!a.in1 || a.in1_pstride % (16 / ES) == 0), "input strides");
  if (a.M == 0) return SAD_OK;
  // x4 (the deep Bottleneck plans' parity mode): every conv on the implicit GEMM
  const int v = variant > 0 ? variant : a.x4 ? gemm_block_variant(a_in) : default_block_variant(a_in, dtype);
  SAD_REQUIRE(variant_fits(v, a.Cout), "variant's channel tile does not divide Cout");
  SAD_REQUIRE(!a.x4 || (dtype == SAD_BF16X3 && !a.st_part && !a.pool_out && (v == 9 || v == 13 || v == 15)),
              "four-product convs: split-bf16 inference on variants 9 / 13 / 15, no fused statistics or pool");
  ++g_block_conv_kernels;
  if (v == 30) {
    SAD_REQUIRE(dtype != SAD_F32 && halo256_ok(a_in), "variant 30: bf16 / split-bf16 3x3/s1/p1, Cout % 256, 16 x 16 tiles");
#if SAD_STAMPS
    static uint64_t* stamp_buf30 = nullptr;
    if (!stamp_this_launch(1)) return launch_halo256(a, s, dtype == SAD_BF16X3);
    if (!stamp_buf30) SAD_CHECK_HIP(hipMalloc(&stamp_buf30, kStampWords * 8));
    SAD_CHECK_HIP(hipMemsetAsync(stamp_buf30, 0, kStampWords * 8, s));
    a.stamps = stamp_buf30;
    const int rc30 = launch_halo256(a, s, dtype == SAD_BF16X3);
    return rc30 == SAD_OK ? stamp_report(a, s) : rc30;
#else
    return launch_halo256(a, s, dtype == SAD_BF16X3);
#endif
  }
  if (v == 31) {
    SAD_REQUIRE((dtype == SAD_BF16 || dtype == SAD_BF16X3) && halo31_ok(a_in),
                "variant 31: bf16 / split-bf16 3x3/s1/p1, Cout % 128, 16 x 16 tiles");
    return launch_halo256r(a, s, dtype == SAD_BF16X3);
  }
  if (v == 32) {
    SAD_REQUIRE(dtype == SAD_BF16, "variant 32: bf16");
    return launch_halo256s2(a, s);
  }
  if (v == 44) {
    SAD_REQUIRE((dtype == SAD_BF16 || dtype == SAD_BF16X3) && halo256rs2_ok(a_in),
                "variant 44: bf16 / split-bf16 3x3/s2/p1, Cin % 64, Cout % 128, 16 x 16 output tiles");
    return launch_halo256rs2(a, s, dtype == SAD_BF16X3);
  }
  if (v == 41) {
    SAD_REQUIRE(dtype == SAD_BF16 && (halo_ok(a_in, dtype) || l2conv_ds_ok(a_in)), "variant 41: bf16 3x3/s1/p1, H, W % 16");
    return launch_l2conv(a, s);
  }
  if (v == 43) {
    SAD_REQUIRE(dtype == SAD_BF16 && l2s2_ok(a_in), "variant 43: bf16 64 -> 128 3x3/s2/p1, output H, W % 16");
    return launch_l2s2conv(a, s);
  }
  if (v == 42) {
    SAD_REQUIRE(dtype == SAD_BF16X3 && halo_ok(a_in, dtype) && a_in.Cin == 64 && a_in.Cout == 64,
                "variant 42: split-bf16 64 -> 64 3x3/s1/p1, H, W % 16");
    return launch_l2conv(a, s, true);
  }
  if (dtype == SAD_BF16X3 && v == 26) {
    SAD_REQUIRE(halo_ok(a_in, dtype), "split-bf16 halo conv: 3x3/s1/p1, H, W % 16");
    return launch_halo_rw_x3(a, s);
  }
  if (dtype == SAD_BF16X3 && (v == 20 || v == 21)) {
    SAD_REQUIRE(v == 20 && halo_ok(a_in, dtype), "split-bf16 halo conv: variant 20, 3x3/s1/p1, H, W % 16");
    return launch_halo_v(a, v, s, true);
  }
  if (v == 25) {
    SAD_REQUIRE(halo_ok(a, dtype), "halo conv (variant 25): bf16, 3x3/s1/p1, no GEMM shortcut, H, W % 16");
#if SAD_STAMPS
    static uint64_t* stamp_buf25 = nullptr;
    if (!stamp_this_launch(0)) return launch_halo_rw(a, s);
    if (!stamp_buf25) SAD_CHECK_HIP(hipMalloc(&stamp_buf25, kStampWords * 8));
    SAD_CHECK_HIP(hipMemsetAsync(stamp_buf25, 0, kStampWords * 8, s));
    a.stamps = stamp_buf25;
    const int rc25 = launch_halo_rw(a, s);
    return rc25 == SAD_OK ? stamp_report(a, s) : rc25;
#else
    return launch_halo_rw(a, s);
#endif
  }
  if (v == 20 || v == 21 || v == 22) {
    SAD_REQUIRE(halo_ok(a, dtype), "halo conv (variants 20-22): bf16, 3x3/s1/p1, no GEMM shortcut, H, W % 16");
    return launch_halo_v(a, v, s);
  }
  SAD_REQUIRE(!a.res || a.res_pstride % 4 == 0, "residual pixel stride must keep 4-channel alignment");
#if SAD_STAMPS
  static uint64_t* stamp_buf = nullptr;
  if (v == 13 && stamp_this_launch(1)) {
    if (!stamp_buf) SAD_CHECK_HIP(hipMalloc(&stamp_buf, kStampWords * 8));
    SAD_CHECK_HIP(hipMemsetAsync(stamp_buf, 0, kStampWords * 8, s));
    a.stamps = stamp_buf;
  }
#endif
  int rc;
  if (dtype == SAD_BF16X3 && a.x4) {
    rc = launch_block_x4(a, v, s);
  } else if (dtype == SAD_BF16X3) {
    SAD_REQUIRE(v >= 9 && v <= 19, "split-bf16 runs on the implicit-GEMM variants 9..19");
    rc = launch_block_v<u16, true>(a, v, s);
  } else {
    rc = dtype == SAD_BF16 ? launch_block_v<u16>(a, v, s) : launch_block_v<float>(a, v, s);
  }
#if SAD_STAMPS
  if (rc == SAD_OK && a.stamps) rc = stamp_report(a, s);
#endif
  return rc;
}

}  // namespace sad
