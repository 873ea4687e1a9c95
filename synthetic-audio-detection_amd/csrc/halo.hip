// halo.hip -- persistent halo-tile direct conv for layer1's stride-1 3x3 convs
// (bf16, gfx950).
//
// Contract: BlockConvArgs with KH = KW = 3, stride 1, pad 1, no in1; the
// optional identity shortcut comes in as `res` and is added in the epilogue:
//   out = act(conv3x3(in0) + bias [+ res])
// These are timm BasicBlock conv1 / conv2(+identity) of layer1
// (inference_runner.py:49-51 -> timm resnet18).
//
// Why a second kernel: block.hip's implicit GEMM DMAs every input pixel row
// once per filter tap, and for Cout = 64 that stream (≈52 FLOP per DMA byte)
// caps it at the CU's L2->LDS fill rate (≈70 GB/s/CU, MI355X_MICROARCH
// "gather into LDS"), i.e. ~1/3 of MFMA peak.  Here a workgroup owns a TH x TW
// output tile and DMAs the (TH+2) x (TW+2) input patch of each 64-channel
// chunk ONCE, serving all 9 taps from it; the identity shortcut costs an
// epilogue add instead of a 10th K-step.
//
// Pipeline -- one barrier per K-step, two wave roles (one of each per SIMD):
//  * weight waves (0 .. NW/2-1): DMA the BC x 64 weight slice of step g+4 into
//    a 5-stage ring during step g (counted vmcnt): an LDS-DMA takes ~1 us from
//    issue to landing even from L2, longer than a step, so one step of lead
//    time made the step time the DMA latency;
//  * patch waves (NW/2 .. NW-1): during taps 0-3 of chunk u, DMA the patch of
//    chunk u+1 (double buffer) and, in a tile's last chunk, during taps 2-5 the
//    tile's residual rows; they wait only before the first step of the next
//    chunk -- first-touch (HBM / MALL) data gets >= 4 steps of cover;
//  * the epilogue of tile t runs right after the barrier of tile t+1's first
//    step (its residual rows are published by that barrier): every wave adds
//    bias [+ residual], applies the activation and writes bf16 in place over
//    the residual rows; after the next barrier the patch waves store the tile
//    as full 128-B pixel rows (1 KB per wave-instruction).  Only patch waves
//    store, so the weight waves' counted waits see DMAs only.
//  * operands swapped (C = W . X^T): each lane holds 4 consecutive output
//    channels of one pixel.
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"

#ifndef SAD_STAMPS
#define SAD_STAMPS 0
#endif

namespace sad {

// f(std::integral_constant<int, I>) for I = 0 .. N-1, unrolled at compile time
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// LDS chunk swizzle of the halo kernel: chunk c of row r sits at c ^ (r & 6).
// Conflict-free for ds_read_b128 fragment reads of 16 consecutive rows at ANY
// row offset (the kx taps shift a fragment by one row); igemm.hpp's swz is
// conflict-free only for even offsets (exhaustive check over the b128 lane
// groups of MI355X_MICROARCH.md "LDS").
__device__ __forceinline__ int hswz(int row, int chunk) { return chunk ^ (row & 6); }

template <int WC, int WP, int TC, int TP, int TW, bool X3 = false>
struct HaloGeo {
  static constexpr int NW = WC * WP;
  static constexpr int NL = NW / 2;             // waves per role
  static constexpr int BC = 16 * TC * WC;       // channels per tile
  static constexpr int BP = 16 * TP * WP;       // pixels per tile
  static constexpr int TH = BP / TW;
  static constexpr int PW = TW + 2, PH = TH + 2;
  static constexpr int PR = PW * PH;            // patch rows (pixels)
  static constexpr int NDP = (PR + 7) / 8;      // DMA wave-instructions per patch
  static constexpr int QP = (NDP + NL - 1) / NL;  // per patch wave
  static constexpr int NDR = BP / 8;            // residual DMAs per tile
  static constexpr int QR = NDR / NL;
  static constexpr int QW = BC / 8 / NL;        // weight DMAs per weight wave per step
  static constexpr int PATCH = NDP * 1024;
  static constexpr int RES = BP * 128;
  static constexpr int WST = BC * 128;
  // channel tiles wider than 64 (variant 22: 128) keep the residual and the
  // outputs in registers (the X3 epilogue shape; the 128-B staging rows hold
  // 64 channels) and run a 4-stage weight ring to fit beside the patches
  static constexpr bool REG = X3 || BC > 64;
  static constexpr int NWS = BC > 64 ? 4 : 5;   // weight ring stages (NWS-1 steps ahead)
  // patch pieces of the next chunk go out over taps [0, PT) (<= 3 per wave and
  // step), the tile's residual rows over taps [2, 2 + RT)
  static constexpr int PT = QP <= 12 ? 4 : 7;
  static constexpr int RT = 4;
  // X3 (split-bf16): no LDS staging -- the residual comes into registers and
  // the epilogue stores hi/lo straight from them (the staging rows would be
  // 256 B per pixel and not fit beside the ring)
  static constexpr int OFF_RES = 2 * PATCH, OFF_W = 2 * PATCH + (REG ? 0 : RES);
  static constexpr int SMEM = OFF_W + NWS * WST;
  static_assert(TW == 16, "a 16-pixel fragment is one tile row");
  static_assert(BP % TW == 0 && NW % 2 == 0, "tile shape");
  static_assert(NDR % NL == 0 && BC % (8 * NL) == 0, "DMA split");
  static_assert(QP <= 3 * PT && PT <= 8, "patch pieces must be issued before the next chunk's last tap");
};

// X3: split-bf16 parity mode (block.hip): channels [hi 32 | lo 32] per 64-bf16
// chunk, so a K-step's halves are hi and lo; three MFMA sets per step; the
// epilogue adds the residual (hi + lo, loaded into registers during the
// tile's last chunk) and stores hi/lo from registers.
// ST: training forward -- fused BN statistics of the conv output (StatAcc),
// one [2][BC] row per pixel-group workgroup
template <int WC, int WP, int TC, int TP, int TW, bool RES, bool RELU, bool X3 = false, bool ST = false>
__global__ __launch_bounds__(64 * WC * WP, WC * WP / 4) void halo_conv_kernel(BlockConvArgs a) {
  using G = HaloGeo<WC, WP, TC, TP, TW, X3>;
  constexpr int NL = G::NL, BC = G::BC, TH = G::TH, PW = G::PW, PR = G::PR;
  constexpr int QP = G::QP, QR = G::QR, QW = G::QW, NDP = G::NDP, NWS = G::NWS;
  constexpr bool REG = G::REG;  // register epilogue (X3, or a channel tile > 64)
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool wloader = wave < NL;  // weight wave, else patch wave
  const int lw = wloader ? wave : wave - NL;
  const int wc = wave / WP, wp = wave % WP;
  const int n_tc = a.Cout / BC;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = w % n_tc;
  const int gp = gridDim.x / n_tc, wi = w / n_tc;
  const int tiles_x = a.W / TW, tiles_img = tiles_x * (a.H / TH);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)wi * tiles_p / gp), tp_end = (int)((int64_t)(wi + 1) * tiles_p / gp);
  const int c0 = tc * BC;
  if (tp_begin >= tp_end) {
    if constexpr (ST) stat_rows_zero(BC, a.st_part, wi, a.Cout, c0, tid, 64 * WC * WP);
    return;
  }
  const int nc0 = a.Cin / 64;  // 64-channel chunks, 9 taps each

  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps0 = (int)a.in0_pstride * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- weight waves: their rows of the (fixed) channel tile; K cursor of the next DMA
  int woff[QW];
#pragma unroll
  for (int i = 0; i < QW; ++i) {
    const int r = 8 * (lw + NL * i) + (lane >> 3);
    woff[i] = (c0 + r) * (a.wt_ld * 2) + ((lane & 7) ^ (r & 6)) * 16;
  }
  int wtap = 0, wch = 0, wsi = 0;
  auto load_weights = [&]() __attribute__((always_inline)) {
    const int kb = (wtap * nc0 + wch) * 128;
#pragma unroll
    for (int i = 0; i < QW; ++i) dma16_m0(rw, woff[i] + kb, lds0 + G::OFF_W + wsi * G::WST + (lw + NL * i) * 1024);
    if (++wtap == 9) {
      wtap = 0;
      if (++wch == nc0) wch = 0;
    }
    wsi = wsi + 1 == NWS ? 0 : wsi + 1;
  };

  // ---- patch waves: per piece k, the source offset of the (tile, chunk) being loaded
  int poff[QP];
  int ltile = tp_begin, lch = 0;
  auto prep_patch = [&]() __attribute__((always_inline)) {
    const bool live = ltile < tp_end;  // past the WG's last tile: all-zero pieces
    const int b = ltile / tiles_img, rem = ltile - b * tiles_img;
    const int oy0 = (rem / tiles_x) * TH, ox0 = (rem % tiles_x) * TW;
#pragma unroll
    for (int k = 0; k < QP; ++k) {
      const int pr = 8 * (lw + NL * k) + (lane >> 3);
      const int py = pr / PW, px = pr - py * PW;
      const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
      poff[k] = (live && pr < PR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                    ? ((b * a.H + iy) * a.W + ix) * ps0 + lch * 128 + ((lane & 7) ^ (pr & 6)) * 16
                    : 0x7FFFFFF0;  // padding / past the patch: zeros
    }
  };
  auto advance_patch = [&]() __attribute__((always_inline)) {
    if (++lch == nc0) {
      lch = 0;
      ++ltile;
    }
    prep_patch();
  };
  auto res_pieces = [&](int t, int tap) __attribute__((always_inline)) {
    if constexpr (RES && !REG) {
      const __amdgpu_buffer_rsrc_t rr =
          __builtin_amdgcn_make_buffer_rsrc((void*)a.res, (short)0, (int)a.res_bytes, 0x00020000);
      const int b = t / tiles_img, rem = t - b * tiles_img;
      const int oy0 = (rem / tiles_x) * TH, ox0 = (rem % tiles_x) * TW;
#pragma unroll
      for (int k = 0; k < QR; ++k) {
        if (k % G::RT != tap - 2) continue;
        const int q = lw + NL * k;
        const int p = 8 * q + (lane >> 3);
        const int ty = p / TW, tx = p - ty * TW;
        const int off = ((b * a.H + oy0 + ty) * a.W + ox0 + tx) * (int)a.res_pstride * 2 +
                        (c0 / 8 + ((lane & 7) ^ (p & 6))) * 16;
        dma16_m0(rr, off, lds0 + G::OFF_RES + q * 1024);
      }
    }
  };

  float bias[TC][4];
#pragma unroll
  for (int i = 0; i < TC; ++i) {
    const float4 b4 = *(const float4*)(a.bias + c0 + wc * 16 * TC + i * 16 + (lane >> 4) * 4);
    bias[i][0] = b4.x;
    bias[i][1] = b4.y;
    bias[i][2] = b4.z;
    bias[i][3] = b4.w;
  }
  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  StatLane<ST ? TC : 1> stat;
  stat.zero();
  // fragment j of this wave = tile row ty = wp*TP + j, pixels fr = 0..15
  // epilogue, part 1 (every wave, tap 0 of the next tile): bias [+ residual],
  // activation, bf16 -> the tile's LDS staging rows (in place over the
  // residual rows: each lane writes exactly the bytes it read)
  // X3: residual (hi, lo) of the tile in registers, loaded during its last chunk
  uint2 xres[REG && RES ? TP : 1][REG && RES ? TC : 1][X3 ? 2 : 1];
  auto x3_pix = [&](int t, int j) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int oy = (rem / tiles_x) * TH + wp * TP + j, ox = (rem % tiles_x) * TW + (lane & 15);
    return (int64_t)(b * a.Ho + oy) * a.Wo + ox;
  };
  auto x3_load_res = [&](int t, int j) __attribute__((always_inline)) {
    if constexpr (REG && RES) {
      const u16* rp = (const u16*)a.res + x3_pix(t, j) * a.res_pstride;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int co = c0 + wc * 16 * TC + i * 16 + (lane >> 4) * 4;
        if constexpr (X3) {
          const int pc = ((co >> 5) << 6) + (co & 31);
          xres[j][i][0] = *(const uint2*)(rp + pc);
          xres[j][i][X3 ? 1 : 0] = *(const uint2*)(rp + pc + 32);
        } else {
          xres[j][i][0] = *(const uint2*)(rp + co);
        }
      }
    }
  };
  auto x3_epilogue = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      u16* op = (u16*)a.out + x3_pix(t, j) * a.out_pstride;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int co = c0 + wc * 16 * TC + i * 16 + (lane >> 4) * 4;
        const int pc = ((co >> 5) << 6) + (co & 31);
        float v[4];
        if constexpr (X3) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[i][r];
        } else {  // variant 22: the bias is re-read here (L1) instead of held in 16 VGPRs
          const float4 bb = *(const float4*)(a.bias + co);
          v[0] = acc[i][j][0] + bb.x;
          v[1] = acc[i][j][1] + bb.y;
          v[2] = acc[i][j][2] + bb.z;
          v[3] = acc[i][j][3] + bb.w;
        }
        if constexpr (RES && X3) {
          const uint2 h = xres[j][i][0], l = xres[j][i][X3 ? 1 : 0];
          v[0] += __uint_as_float(h.x << 16) + __uint_as_float(l.x << 16);
          v[1] += __uint_as_float(h.x & 0xFFFF0000u) + __uint_as_float(l.x & 0xFFFF0000u);
          v[2] += __uint_as_float(h.y << 16) + __uint_as_float(l.y << 16);
          v[3] += __uint_as_float(h.y & 0xFFFF0000u) + __uint_as_float(l.y & 0xFFFF0000u);
        } else if constexpr (RES) {
          const uint2 h = xres[j][i][0];
          v[0] += __uint_as_float(h.x << 16);
          v[1] += __uint_as_float(h.x & 0xFFFF0000u);
          v[2] += __uint_as_float(h.y << 16);
          v[3] += __uint_as_float(h.y & 0xFFFF0000u);
        }
        if constexpr (RELU)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        if constexpr (!X3) {  // plain bf16 (variant 22): one 8-B store per lane
          *(uint2*)(op + co) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                          (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        u16 hh[4], ll[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          hh[r] = f2bf(v[r]);
          ll[r] = f2bf(v[r] - bf2f(hh[r]));
        }
        *(uint2*)(op + pc) =
            make_uint2((uint32_t)hh[0] | ((uint32_t)hh[1] << 16), (uint32_t)hh[2] | ((uint32_t)hh[3] << 16));
        *(uint2*)(op + pc + 32) =
            make_uint2((uint32_t)ll[0] | ((uint32_t)ll[1] << 16), (uint32_t)ll[2] | ((uint32_t)ll[3] << 16));
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  auto epilogue = [&]() __attribute__((always_inline)) {
    if constexpr (ST) {  // statistics of the conv output (bias added, before any residual)
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < TP; ++j) stat.add(i, r, acc[i][j][r] + bias[i][r]);
    }
    // every residual read issued before the first in-place write (the compiler
    // cannot prove the lanes' read and write addresses disjoint across (i, j))
    uint2 rvs[TP][TC];
    if constexpr (RES) {
#pragma unroll
      for (int j = 0; j < TP; ++j)
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const int p = (wp * TP + j) * TW + fr;
          const int cl = wc * 16 * TC + i * 16 + fg * 4;
          rvs[j][i] = *(const uint2*)(smem + G::OFF_RES + p * 128 + (hswz(p, cl >> 3) << 4) + (cl & 7) * 2);
        }
    }
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int p = (wp * TP + j) * TW + fr;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int cl = wc * 16 * TC + i * 16 + fg * 4;
        uint2* sp = (uint2*)(smem + G::OFF_RES + p * 128 + (hswz(p, cl >> 3) << 4) + (cl & 7) * 2);
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[i][r];
        if constexpr (RES) {
          const uint2 rv = rvs[j][i];
          v[0] += __uint_as_float(rv.x << 16);
          v[1] += __uint_as_float(rv.x & 0xFFFF0000u);
          v[2] += __uint_as_float(rv.y << 16);
          v[3] += __uint_as_float(rv.y & 0xFFFF0000u);
        }
        if constexpr (RELU)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        uint2 qv;
        qv.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        qv.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *sp = qv;
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };
  // epilogue, part 2 (patch waves, tap 1, after a barrier): staging rows ->
  // global, 8 pixels x 128 B per wave-instruction (full lines)
  auto store_tile = [&](int t) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int oy0 = (rem / tiles_x) * TH, ox0 = (rem % tiles_x) * TW;
    u16* __restrict__ out = (u16*)a.out + ((int64_t)(b * a.Ho + oy0) * a.Wo + ox0) * a.out_pstride + c0;
#pragma unroll
    for (int k = 0; k < QR; ++k) {
      const int p = 8 * (lw + NL * k) + (lane >> 3), c = lane & 7;
      const uint4 v = *(const uint4*)(smem + G::OFF_RES + p * 128 + (hswz(p, c) << 4));
      const int ty = p / TW, tx = p - ty * TW;
      *(uint4*)(out + (ty * a.Wo + tx) * (int)a.out_pstride + c * 8) = v;
    }
  };

  // ---- one K-step from LDS: two K-halves (s = 0, 1); half 1's reads are
  // issued between half 0's MFMAs
  auto compute_step = [&](int tap, int wst, int pbuf) __attribute__((always_inline)) {
    const char* pb = smem + pbuf * G::PATCH;
    const char* wb = smem + G::OFF_W + wst * G::WST;
    const int ky = tap / 3, kx = tap - ky * 3;
    uint4 w[2][TC], p[2][TP];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = fg + 4 * s;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int r = wc * 16 * TC + i * 16 + fr;
        w[s][i] = *(const uint4*)(wb + r * 128 + (hswz(r, c) << 4));
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = (wp * TP + j + ky) * PW + kx + fr;
        p[s][j] = *(const uint4*)(pb + r * 128 + (hswz(r, c) << 4));
      }
    }
    if constexpr (X3) {  // W_hi.X_hi (half 0 only), then W_lo.X_hi and W_hi.X_lo
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<u16>(w[0][i], p[0][j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<u16>(w[1][i], p[0][j], acc[i][j]);
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<u16>(w[0][i], p[1][j], acc[i][j]);
    } else {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<u16>(w[s][i], p[s][j], acc[i][j]);
    }
    // schedule: half 0's reads, then its MFMAs interleaved with half 1's reads
    __builtin_amdgcn_sched_group_barrier(0x100, TC + TP, 0);
#pragma unroll
    for (int k = 0; k < TC + TP; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, (X3 ? 3 : 2) * TC * TP - (TC + TP), 0);
  };

  // ---- prologue: patch of the first chunk, weights of the first NWS-1 steps,
  // fragments of step 0
  if (wloader) {
#pragma unroll
    for (int k = 0; k < NWS - 1; ++k) load_weights();
  } else {
    prep_patch();
#pragma unroll
    for (int k = 0; k < QP; ++k)
      if (NDP % NL == 0 || lw + NL * k < NDP) dma16_m0(r0, poff[k], lds0 + (lw + NL * k) * 1024);
    advance_patch();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // One chunk = 9 K-steps (taps) of tile t, channel chunk ch, unrolled so every
  // tap-dependent decision is static.  Each step: wait -> barrier -> DMA issue
  // -> [epilogue of the previous tile] -> step g from LDS.  Past the last step the weight waves keep issuing
  // (wrapped K cursor) and the patch waves issue all-zero pieces, so the
  // counted waits never change shape; nothing reads those stages.
  int t = tp_begin, ch = 0, wsc = 0, pbuf = 0;
  const int ab = a.ablate;
  auto chunk = [&]() __attribute__((always_inline)) {
    const bool after_tile = t > tp_begin && ch == 0;   // tile t-1's epilogue stores go out at tap 0
    const bool last_chunk = ch + 1 == nc0;
    static_for<9>([&](auto tap_c) __attribute__((always_inline)) {
      constexpr int tap = decltype(tap_c)::value;
      if (!(ab & 2)) {
        if (wloader) {
          // w(g) was issued at step g-(NWS-1); younger: w(g+1..g+NWS-2) (weight waves store nothing)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NWS - 2) * QW) : "memory");
        } else if (tap == 0) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // next chunk's patch + this tile's residual
        }
      }
      if constexpr (tap == 1 && !REG) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // staging rows written
      if (!(ab & 4)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (!(ab & 1)) {
        if (wloader) {
          if (!(ab & 16)) load_weights();
        } else if (!(ab & 32)) {
          if constexpr (tap < G::PT) {
#pragma unroll
            for (int k = tap; k < QP; k += G::PT)
              if (NDP % NL == 0 || lw + NL * k < NDP)
                dma16_m0(r0, poff[k], lds0 + (pbuf ^ 1) * G::PATCH + (lw + NL * k) * 1024);
            if constexpr (tap == G::PT - 1) advance_patch();
          }
          if constexpr (tap == 1 && !REG)
            if (after_tile) store_tile(t - 1);
          if constexpr (RES && tap >= 2 && tap < 2 + G::RT)
            if (last_chunk) res_pieces(t, tap);
        }
      }
      if constexpr (REG && RES && tap >= 2 && tap < 2 + TP)
        if (last_chunk) x3_load_res(t, tap - 2);
      if constexpr (tap == 0)
        if (after_tile && !(ab & 8)) {
          if constexpr (REG)
            x3_epilogue(t - 1);
          else
            epilogue();
        }
      compute_step(tap, wsc, pbuf);
      wsc = wsc + 1 == NWS ? 0 : wsc + 1;
    });
    pbuf ^= 1;
    if (++ch == nc0) {
      ch = 0;
      ++t;
    }
  };
  const int nchunks = (tp_end - tp_begin) * nc0;
  for (int c = 0; c < nchunks; ++c) chunk();
  // last tile: its residual rows were issued in its last chunk; publish, then store
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (REG) {
    x3_epilogue(tp_end - 1);
    return;
  }
  __builtin_amdgcn_s_barrier();
  epilogue();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (!wloader) store_tile(tp_end - 1);
  if constexpr (ST) {  // patch buffer 0 is free: fold the WP pixel waves of each channel
    float* s_red = (float*)smem;
    stat.park(s_red, wp, BC, wc * 16 * TC, fr, fg);
    __syncthreads();
    stat_rows_write(s_red, WP, BC, a.st_part, wi, a.Cout, c0, tid, 64 * WC * WP);
  }
}


// ---------------------------------------------------------------------------
// Resident-weight halo conv (variant 25): Cin = Cout = 64 (layer1).
//
// All 9 taps' weights (64 x 576 bf16 = 72 KB) are DMA'd into LDS once per
// workgroup, so a tile's 9 K-steps need no weight ring and no barrier: the
// only synchronisation is ONE barrier per 16x16 tile, which publishes the
// next tile's (double-buffered) input patch.  Within a tile, tap k+1's
// fragments are read while tap k's MFMAs run (no barrier in between).  The
// residual comes straight from global memory into registers (prefetched during
// the tile) and the epilogue stores from registers (8 B per lane), so LDS holds
// only weights + 2 patches (72 + 2 x 41 KB).
//
// The epilogue is staggered across the two waves of each SIMD (waves w, w+4):
// waves 0-3 run theirs before the tile barrier, waves 4-7 after it, so one
// wave's VALU epilogue overlaps its partner's MFMAs instead of idling the
// SIMD's matrix pipe.
template <bool RES, bool RELU, bool ST = false>
__global__ __launch_bounds__(512, 1) void halo_rw_kernel(BlockConvArgs a) {
  constexpr int NW = 8, TC = 4, TP = 2, TW = 16, TH = 16;
  constexpr int PW = TW + 2, PR = PW * (TH + 2);  // 18 x 18 patch rows
  constexpr int NDP = (PR + 7) / 8;               // 41 DMA pieces per patch
  constexpr int QP = (NDP + NW - 1) / NW;         // <= 6 per wave
  constexpr int WBYTES = 9 * 64 * 128;            // resident weights
  constexpr int PATCH = NDP * 1024;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool early = wave < 4;  // epilogue before the tile barrier
  const int wp = wave;          // tile rows 2wp, 2wp+1; all 64 channels
  SAD_CLOCK_STAMP(0);
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_x = a.W / TW, tiles_img = tiles_x * (a.H / TH);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)w * tiles_p / gridDim.x), tp_end = (int)((int64_t)(w + 1) * tiles_p / gridDim.x);
  if (tp_begin >= tp_end) {
    if constexpr (ST) stat_rows_zero(64, a.st_part, w, 64, 0, tid, 512);
    return;
  }

  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps0 = (int)a.in0_pstride * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- patch pieces of tile `pt` into buffer `pb` (piece q = wave + 8k, rows 8q..8q+7)
  int poff[QP];
  auto prep_patch = [&](int pt) __attribute__((always_inline)) {
    const int b = pt / tiles_img, rem = pt - b * tiles_img;
    const int oy0 = (rem / tiles_x) * TH, ox0 = (rem % tiles_x) * TW;
#pragma unroll
    for (int k = 0; k < QP; ++k) {
      const int pr = 8 * (wave + NW * k) + (lane >> 3);
      const int py = pr / PW, px = pr - py * PW;
      const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
      poff[k] = (pr < PR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                    ? ((b * a.H + iy) * a.W + ix) * ps0 + ((lane & 7) ^ (pr & 6)) * 16
                    : 0x7FFFFFF0;
    }
  };
  auto patch_piece = [&](int k, int pb) __attribute__((always_inline)) {
    if (NDP % NW == 0 || wave + NW * k < NDP)
      dma16_m0(r0, poff[k], lds0 + WBYTES + pb * PATCH + (wave + NW * k) * 1024);
  };

  // ---- prologue: resident weights (72 pieces, 9 per wave) + the first patch
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int q = wave + NW * i;  // tap q / 8, rows 8 (q % 8) + lane / 8
    const int tap = q >> 3, co = 8 * (q & 7) + (lane >> 3);
    dma16_m0(rw, co * (a.wt_ld * 2) + tap * 128 + ((lane & 7) ^ (co & 6)) * 16, lds0 + tap * 8192 + (q & 7) * 1024);
  }
  prep_patch(tp_begin);
#pragma unroll
  for (int k = 0; k < QP; ++k) patch_piece(k, 0);
  if (tp_begin + 1 < tp_end) prep_patch(tp_begin + 1);

  float bias[TC][4];
#pragma unroll
  for (int i = 0; i < TC; ++i) {
    const float4 b4 = *(const float4*)(a.bias + i * 16 + (lane >> 4) * 4);
    bias[i][0] = b4.x; bias[i][1] = b4.y; bias[i][2] = b4.z; bias[i][3] = b4.w;
  }
  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint2 resv[TC][TP];

  const int fr = lane & 15, fg = lane >> 4;
  StatLane<ST ? TC : 1> stat;
  stat.zero();
  // lane's pixel of fragment j: tile row 2wp + j, column fr; channels i*16 + fg*4 .. +3.
  // The tile's first pixel is wave-uniform (64-bit scalar math); the lane's
  // offset from it is a 32-bit VGPR product, so the per-j addresses cost no
  // 64-bit vector multiplies
  auto tile_pix = [&](int t) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int oy0 = (rem / tiles_x) * TH, ox0 = (rem % tiles_x) * TW;
    return (int64_t)(b * a.Ho + oy0) * a.Wo + ox0;
  };
  auto lane_pix = [&](int j) __attribute__((always_inline)) { return (2 * wp + j) * a.Wo + fr; };
  auto load_res = [&](int t, int j) __attribute__((always_inline)) {
    if constexpr (RES) {
      const u16* rp = (const u16*)a.res + tile_pix(t) * a.res_pstride + (lane_pix(j) * (int)a.res_pstride + fg * 4);
#pragma unroll
      for (int i = 0; i < TC; ++i) resv[i][j] = *(const uint2*)(rp + i * 16);
    }
  };
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    if constexpr (ST) {  // statistics of the conv output (bias added, before any residual)
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < TP; ++j) stat.add(i, r, acc[i][j][r] + bias[i][r]);
    }
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      u16* op = (u16*)a.out + tile_pix(t) * a.out_pstride + (lane_pix(j) * (int)a.out_pstride + fg * 4);
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[i][r];
        if constexpr (RES) {
          v[0] += __uint_as_float(resv[i][j].x << 16);
          v[1] += __uint_as_float(resv[i][j].x & 0xFFFF0000u);
          v[2] += __uint_as_float(resv[i][j].y << 16);
          v[3] += __uint_as_float(resv[i][j].y & 0xFFFF0000u);
        }
        if constexpr (RELU)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        uint2 q;
        q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *(uint2*)(op + i * 16) = q;  // (tap 0 of the next tile restarts acc from zero)
      }
    }
  };

  // fragments of tap k (both K-halves) from resident weights + patch buffer pb
  auto read_tap = [&](uint4 (&wf)[2][TC], uint4 (&pf)[2][TP], int k, int pb) __attribute__((always_inline)) {
    const char* wb = smem + k * 8192;
    const char* pbuf = smem + WBYTES + pb * PATCH;
    const int ky = k / 3, kx = k - ky * 3;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = fg + 4 * s;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int r = i * 16 + fr;
        wf[s][i] = *(const uint4*)(wb + r * 128 + (hswz(r, c) << 4));
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = (2 * wp + j + ky) * PW + kx + fr;
        pf[s][j] = *(const uint4*)(pbuf + r * 128 + (hswz(r, c) << 4));
      }
    }
  };
  // tap 0's first K-half starts each accumulator from an inline zero (no
  // per-tile v_mov zeroing of the 32 accumulator registers)
  auto mma_tap = [&](const uint4 (&wf)[2][TC], const uint4 (&pf)[2][TP], auto first) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) {
          if constexpr (decltype(first)::value) {
            if (s == 0) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wf[0][i]),
                                                                  __builtin_bit_cast(bf16x8, pf[0][j]),
                                                                  f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
              continue;
            }
          }
          mfma_chunk<u16>(wf[s][i], pf[s][j], acc[i][j]);
        }
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();

  uint4 wf[2][2][TC], pf[2][2][TP];
  int pb = 0;
  // diagnostic build (-DSAD_STAMPS=1): s_memtime of waves 0 and 4 of workgroup 0
  // per tile -- 0 tile start, 1 taps issued, 2 before the tile barrier, 3 after it
  const bool stamp_on = SAD_STAMPS && a.stamps && blockIdx.x == 0 && (wave == 0 || wave == 4);
  auto stamp = [&](int g, int slot) __attribute__((always_inline)) {
    if constexpr (SAD_STAMPS) {
      if (stamp_on && g < 1024) {
        __builtin_amdgcn_sched_barrier(0);
        uint64_t t_;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        if (lane == 0) a.stamps[(size_t)(wave == 0 ? 0 : 1) * 4096 + (size_t)g * 4 + slot] = t_;
      }
    }
  };
  for (int t = tp_begin; t < tp_end; ++t) {
    const bool has_next = t + 1 < tp_end;
    stamp(t - tp_begin, 0);
    read_tap(wf[0], pf[0], 0, pb);
    static_for<9>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      __builtin_amdgcn_sched_barrier(0);
      // next tile's patch: one piece per tap over taps 0..QP-1; this tile's
      // residual: fragment j at tap j
      // the next tile's patch, all pieces at tap 0: the stamps showed the
      // early waves waiting ~1.1k cycles for pieces issued at taps 0..5
      if constexpr (k == 0)
        if (has_next) {
#pragma unroll
          for (int kk = 0; kk < QP; ++kk) patch_piece(kk, pb ^ 1);
        }
      if constexpr (k < TP) load_res(t, k);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (k < 8) {
        read_tap(wf[(k + 1) & 1], pf[(k + 1) & 1], k + 1, pb);
        mma_tap(wf[k & 1], pf[k & 1], std::integral_constant<bool, k == 0>{});
        // the next tap's 12 reads spread over this tap's 16 MFMAs
#pragma unroll
        for (int q = 0; q < 2 * (TC + TP); ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * TC * TP - 2 * (TC + TP), 0);
      } else {
        mma_tap(wf[k & 1], pf[k & 1], std::integral_constant<bool, false>{});
      }
    });
    __builtin_amdgcn_sched_barrier(0);
    stamp(t - tp_begin, 1);
    if (has_next) prep_patch(t + 2 < tp_end ? t + 2 : t + 1);
    // early waves: epilogue, then wait for their DMAs/loads (the stores, youngest, may stay in flight)
    if (early) {
      epilogue(t);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(TC * TP) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    stamp(t - tp_begin, 2);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    stamp(t - tp_begin, 3);
    if (!early) epilogue(t);
    pb ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SAD_CLOCK_STAMP(1);
  if constexpr (ST) {  // the resident weights are done: fold the 8 pixel waves
    __syncthreads();
    float* s_red = (float*)smem;
    stat.park(s_red, wp, 64, 0, fr, fg);
    __syncthreads();
    stat_rows_write(s_red, NW, 64, a.st_part, w, 64, 0, tid, 512);
  }
}

template <bool RES, bool RELU, bool ST = false>
static int launch_halo_rw_t(const BlockConvArgs& a, hipStream_t s) {
  constexpr int smem = 9 * 64 * 128 + 2 * 41 * 1024;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)halo_rw_kernel<RES, RELU, ST>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem);
    attr = true;
  }
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && !a.in1,
              "halo conv: 3x3, stride 1, pad 1, no GEMM shortcut");
  SAD_REQUIRE(a.Cin == 64 && a.Cout == 64, "resident-weight halo conv (variant 25): Cin = Cout = 64");
  SAD_REQUIRE(a.W % 16 == 0 && a.H % 16 == 0 && a.Ho == a.H && a.Wo == a.W, "image must tile exactly");
  SAD_REQUIRE(a.wt_ld >= 9 * a.Cin && (a.wt_ld * 2) % 16 == 0, "weight row length");
  SAD_REQUIRE(!a.res || a.res_pstride >= a.Cout, "residual pixel stride");
  SAD_REQUIRE(a.out_pstride % 4 == 0 && (!a.res || a.res_pstride % 4 == 0), "8-B aligned pixel rows");
  const int64_t tiles_p = (int64_t)a.N * (a.H / 16) * (a.W / 16);
  SAD_REQUIRE(tiles_p < (1ll << 31) && (int64_t)a.N * a.H * a.W * a.in0_pstride * 2 < (1ll << 31),
              "too large for one launch");
  const int64_t g = std::min<int64_t>(tiles_p, 256);
  if (ST) *a.st_rows = (int)g;
  hipLaunchKernelGGL((halo_rw_kernel<RES, RELU, ST>), dim3((unsigned)g), dim3(512), smem, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

int launch_halo_rw(const BlockConvArgs& a, hipStream_t s) {
  if (a.st_part) {
    SAD_REQUIRE(!a.res && !a.relu && a.st_rows, "fused BN statistics: raw conv (no residual / ReLU), st_rows set");
    return launch_halo_rw_t<false, false, true>(a, s);
  }
  if (a.res) return a.relu ? launch_halo_rw_t<true, true>(a, s) : launch_halo_rw_t<true, false>(a, s);
  return a.relu ? launch_halo_rw_t<false, true>(a, s) : launch_halo_rw_t<false, false>(a, s);
}

// ---------------------------------------------------------------------------
// Split-bf16 (X3) resident-weight layer1 conv (variant 26): logical Cin = Cout
// = 64, i.e. 128 bf16 input channels ([hi 32 | lo 32] x 2 chunks).
//
// The hi/lo weights of all 64 output channels (144 KB) do not fit beside the
// patches, so a workgroup owns HALF the output channels (32: 72 KB resident,
// [tap][chunk][32 co][128 B]) and the two halves of a 16x16 tile run as
// neighbouring workgroups (one XCD: the second patch read hits L2).  The patch
// has two 64-bf16-channel chunks, one LDS buffer each (2 x 41 KB), ping-ponged:
// while chunk 0 of tile t is computed, chunk 1 of t is DMA'd; while chunk 1
// is computed, chunk 0 of tile t+1 -- every DMA has 9 taps of cover, and a
// tile needs two barriers (vs one per tap on the weight-ring kernel 20).
// Each tap: W_hi.X_hi + W_lo.X_hi + W_hi.X_lo (12 MFMAs per wave); the
// next tap's fragments are read between this tap's MFMAs.  8 waves, each 32
// channels x 2 tile rows; the epilogue adds bias [+ residual hi + lo] and
// stores hi/lo from registers.
template <bool RES, bool RELU>
__global__ __launch_bounds__(512, 1) void halo_rw_x3_kernel(BlockConvArgs a) {
  constexpr int NW = 8, TC = 2, TP = 2, TW = 16, TH = 16;
  constexpr int PW = TW + 2, PR = PW * (TH + 2);  // 18 x 18 patch rows
  constexpr int NDP = (PR + 7) / 8;               // 41 DMA pieces per chunk
  constexpr int QP = (NDP + NW - 1) / NW;         // <= 6 per wave
  constexpr int WBLK = 32 * 128;                  // one (tap, chunk) weight block
  constexpr int WBYTES = 18 * WBLK;               // resident weights
  constexpr int PATCH = NDP * 1024;
  constexpr int BAD = 0x7FFFFFF0;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wp = wave;  // tile rows 2wp, 2wp+1; the workgroup's 32 channels
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int half = w & 1, grp = w >> 1, ngrp = gridDim.x >> 1;
  const int tiles_x = a.W / TW, tiles_img = tiles_x * (a.H / TH);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)grp * tiles_p / ngrp), tp_end = (int)((int64_t)(grp + 1) * tiles_p / ngrp);
  if (tp_begin >= tp_end) return;

  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps0 = (int)a.in0_pstride * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // patch pieces of tile pt (chunk offset added at issue; padding stays past num_records)
  auto prep_patch = [&](int pt, int (&po)[QP]) __attribute__((always_inline)) {
    const int b = pt / tiles_img, rem = pt - b * tiles_img;
    const int oy0 = (rem / tiles_x) * TH, ox0 = (rem % tiles_x) * TW;
#pragma unroll
    for (int k = 0; k < QP; ++k) {
      const int pr = 8 * (wave + NW * k) + (lane >> 3);
      const int py = pr / PW, px = pr - py * PW;
      const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
      po[k] = (pr < PR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                  ? ((b * a.H + iy) * a.W + ix) * ps0 + ((lane & 7) ^ (pr & 6)) * 16
                  : BAD;
    }
  };
  auto patch_piece = [&](const int (&po)[QP], int k, int ch) __attribute__((always_inline)) {
    if (NDP % NW == 0 || wave + NW * k < NDP)
      dma16_m0(r0, po[k] == BAD ? BAD : po[k] + ch * 128, lds0 + WBYTES + ch * PATCH + (wave + NW * k) * 1024);
  };

  // ---- prologue: this half's weights (72 pieces, 9 per wave) + chunk 0 of the first tile
  const int wrow = (int)a.wt_ld * 2;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int q = wave + NW * i;  // block q / 4 = tap * 2 + chunk, rows 8 (q % 4) + lane / 8
    const int blk = q >> 2, col = 8 * (q & 3) + (lane >> 3);
    dma16_m0(rw, (32 * half + col) * wrow + blk * 128 + ((lane & 7) ^ (col & 6)) * 16,
             lds0 + blk * WBLK + (q & 3) * 1024);
  }
  int pcur[QP], pnext[QP];
  prep_patch(tp_begin, pcur);
#pragma unroll
  for (int k = 0; k < QP; ++k) patch_piece(pcur, k, 0);

  const int fr = lane & 15, fg = lane >> 4;
  float bias[TC][4];
#pragma unroll
  for (int i = 0; i < TC; ++i) {
    const float4 b4 = *(const float4*)(a.bias + 32 * half + i * 16 + fg * 4);
    bias[i][0] = b4.x;
    bias[i][1] = b4.y;
    bias[i][2] = b4.z;
    bias[i][3] = b4.w;
  }
  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint2 resv[TC][TP][2];

  auto pix_index = [&](int t, int j) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int oy = (rem / tiles_x) * TH + 2 * wp + j, ox = (rem % tiles_x) * TW + fr;
    return (int64_t)(b * a.Ho + oy) * a.Wo + ox;
  };
  // logical channel 32*half + i*16 + fg*4 (+0..3) -> split column 64*half + i*16 + fg*4 (hi), +32 (lo)
  const int pc0 = 64 * half + fg * 4;
  auto load_res = [&](int t, int j) __attribute__((always_inline)) {
    if constexpr (RES) {
      const u16* rp = (const u16*)a.res + pix_index(t, j) * a.res_pstride + pc0;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        resv[i][j][0] = *(const uint2*)(rp + i * 16);
        resv[i][j][1] = *(const uint2*)(rp + i * 16 + 32);
      }
    }
  };
  auto epilogue = [&](int t) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      u16* op = (u16*)a.out + pix_index(t, j) * a.out_pstride + pc0;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[i][r];
        if constexpr (RES) {
          const uint2 h = resv[i][j][0], l = resv[i][j][1];
          v[0] += __uint_as_float(h.x << 16) + __uint_as_float(l.x << 16);
          v[1] += __uint_as_float(h.x & 0xFFFF0000u) + __uint_as_float(l.x & 0xFFFF0000u);
          v[2] += __uint_as_float(h.y << 16) + __uint_as_float(l.y << 16);
          v[3] += __uint_as_float(h.y & 0xFFFF0000u) + __uint_as_float(l.y & 0xFFFF0000u);
        }
        if constexpr (RELU)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
        u16 hh[4], ll[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          hh[r] = f2bf(v[r]);
          ll[r] = f2bf(v[r] - bf2f(hh[r]));
        }
        *(uint2*)(op + i * 16) =
            make_uint2((uint32_t)hh[0] | ((uint32_t)hh[1] << 16), (uint32_t)hh[2] | ((uint32_t)hh[3] << 16));
        *(uint2*)(op + i * 16 + 32) =
            make_uint2((uint32_t)ll[0] | ((uint32_t)ll[1] << 16), (uint32_t)ll[2] | ((uint32_t)ll[3] << 16));
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  // fragments of (tap k, chunk ch): weights [half s][i], pixels [half s][j]; s = 0 hi, 1 lo
  auto read_tap = [&](uint4 (&wf)[2][TC], uint4 (&pf)[2][TP], int k, int ch) __attribute__((always_inline)) {
    const char* wb = smem + (k * 2 + ch) * WBLK;
    const char* pbuf = smem + WBYTES + ch * PATCH;
    const int ky = k / 3, kx = k - ky * 3;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = fg + 4 * s;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int r = i * 16 + fr;
        wf[s][i] = *(const uint4*)(wb + r * 128 + (hswz(r, c) << 4));
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = (2 * wp + j + ky) * PW + kx + fr;
        pf[s][j] = *(const uint4*)(pbuf + r * 128 + (hswz(r, c) << 4));
      }
    }
  };
  auto mma_tap = [&](const uint4 (&wf)[2][TC], const uint4 (&pf)[2][TP]) __attribute__((always_inline)) {
    // product-outer: a product's TC*TP MFMAs go to independent accumulators, so
    // dependent MFMAs (same accumulator) are TC*TP issues apart, not back to back
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int i = 0; i < TC; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j)
          mfma_chunk<u16>(wf[p == 1 ? 1 : 0][i], pf[p == 2 ? 1 : 0][j], acc[i][j]);  // hi.hi, lo.hi, hi.lo
  };
  // 9 taps of chunk ch; during taps k < QP the wave issues piece k of `issue`
  // (chunk ich of the pieces in po) -- the other chunk buffer is free
  uint4 wf[2][2][TC], pf[2][2][TP];
  auto chunk = [&](int ch, bool issue, const int (&po)[QP], int ich, int res_t) __attribute__((always_inline)) {
    read_tap(wf[0], pf[0], 0, ch);
    static_for<9>([&](auto kc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value;
      __builtin_amdgcn_sched_barrier(0);
      // the other chunk's pieces all at tap 0 (as variant 25: a piece issued at
      // tap 5 had too little of the chunk left to land)
      if constexpr (k == 0)
        if (issue) {
#pragma unroll
          for (int kk = 0; kk < QP; ++kk) patch_piece(po, kk, ich);
        }
      if constexpr (RES && k >= QP && k < QP + TP)
        if (res_t >= 0) load_res(res_t, k - QP);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (k < 8) {
        read_tap(wf[(k + 1) & 1], pf[(k + 1) & 1], k + 1, ch);
        mma_tap(wf[k & 1], pf[k & 1]);
#pragma unroll
        for (int q = 0; q < 2 * (TC + TP); ++q) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 3 * TC * TP - 2 * (TC + TP), 0);
      } else {
        mma_tap(wf[k & 1], pf[k & 1]);
      }
    });
    __builtin_amdgcn_sched_barrier(0);
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int t = tp_begin; t < tp_end; ++t) {
    const bool has_next = t + 1 < tp_end;
    // chunk 0 of t from buffer 0; chunk 1 of t goes into buffer 1
    // (this tile's residual goes out at taps QP.. of chunk 0, the youngest loads:
    // the wait below leaves them in flight, so they get chunk 1 as cover)
    chunk(0, true, pcur, 1, t);
    if constexpr (RES)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * TC * TP) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // chunk 1 published, buffer 0 free
    if (has_next) prep_patch(t + 1, pnext);
    // chunk 1 of t from buffer 1; chunk 0 of t+1 goes into buffer 0
    chunk(1, has_next, pnext, 0, -1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    epilogue(t);
    __builtin_amdgcn_s_barrier();  // chunk 0 of t+1 published, buffer 1 free
#pragma unroll
    for (int k = 0; k < QP; ++k) pcur[k] = pnext[k];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool RES, bool RELU>
static int launch_halo_rw_x3_t(const BlockConvArgs& a, hipStream_t s) {
  constexpr int smem = 18 * 32 * 128 + 2 * 41 * 1024;
  static_assert(smem <= 160 * 1024, "LDS budget");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)halo_rw_x3_kernel<RES, RELU>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              smem);
    attr = true;
  }
  const int64_t tiles_p = (int64_t)a.N * (a.H / 16) * (a.W / 16);
  const int64_t g = std::min<int64_t>(tiles_p, 128) * 2;
  hipLaunchKernelGGL((halo_rw_x3_kernel<RES, RELU>), dim3((unsigned)g), dim3(512), smem, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

// (a: the split layout's bf16 channel counts / strides, as launch_block_conv passes them)
int launch_halo_rw_x3(const BlockConvArgs& a, hipStream_t s) {
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && !a.in1,
              "halo conv: 3x3, stride 1, pad 1, no GEMM shortcut");
  SAD_REQUIRE(a.Cin == 128 && a.Cout == 64, "split-bf16 resident-weight halo conv (variant 26): 64 -> 64 logical");
  SAD_REQUIRE(a.W % 16 == 0 && a.H % 16 == 0 && a.Ho == a.H && a.Wo == a.W, "image must tile exactly");
  SAD_REQUIRE(a.wt_ld >= 9 * a.Cin && (a.wt_ld * 2) % 16 == 0, "weight row length");
  SAD_REQUIRE(a.out_pstride % 64 == 0 && (!a.res || a.res_pstride % 64 == 0), "split-bf16 pixel strides");
  SAD_REQUIRE(!a.st_part, "fused BN statistics: not on the split-bf16 kernels");
  const int64_t tiles_p = (int64_t)a.N * (a.H / 16) * (a.W / 16);
  SAD_REQUIRE(tiles_p < (1ll << 30) && (int64_t)a.N * a.H * a.W * a.in0_pstride * 2 < (1ll << 31),
              "too large for one launch");
  if (a.res) return a.relu ? launch_halo_rw_x3_t<true, true>(a, s) : launch_halo_rw_x3_t<true, false>(a, s);
  return a.relu ? launch_halo_rw_x3_t<false, true>(a, s) : launch_halo_rw_x3_t<false, false>(a, s);
}

template <int WC, int WP, int TC, int TP, int TW, bool RES, bool RELU, bool X3, bool ST = false>
static int launch_halo_t(const BlockConvArgs& a, hipStream_t s) {
  using G = HaloGeo<WC, WP, TC, TP, TW, X3>;
  static_assert(G::SMEM <= 160 * 1024, "LDS budget");
  static_assert(!ST || 2 * G::BC * WP * 4 <= 2 * G::PATCH, "statistics fold area");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)halo_conv_kernel<WC, WP, TC, TP, TW, RES, RELU, X3, ST>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, G::SMEM);
    attr = true;
  }
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && !a.in1,
              "halo conv: 3x3, stride 1, pad 1, no GEMM shortcut");
  SAD_REQUIRE(a.Cin % 64 == 0 && a.Cout % G::BC == 0, "halo conv: Cin % 64, Cout % channel tile");
  SAD_REQUIRE(a.W % TW == 0 && a.H % G::TH == 0 && a.Ho == a.H && a.Wo == a.W, "image must tile exactly");
  SAD_REQUIRE(a.wt_ld >= 9 * a.Cin && (a.wt_ld * 2) % 16 == 0, "weight row length");
  SAD_REQUIRE(!a.res || a.res_pstride >= a.Cout, "residual pixel stride");
  SAD_REQUIRE(a.out_pstride * 2 * (int64_t)a.M < (1ll << 40), "output too large");
  const int n_tc = a.Cout / G::BC;
  const int64_t tiles_p = (int64_t)a.N * (a.H / G::TH) * (a.W / TW);
  SAD_REQUIRE(tiles_p * 9 * (a.Cin / 64) < (1ll << 31), "too many tiles for one launch");
  int64_t g = std::min<int64_t>(tiles_p * n_tc, 256);
  g = std::max<int64_t>(n_tc, g / n_tc * n_tc);
  if (X3) SAD_REQUIRE(a.out_pstride % 64 == 0 && (!a.res || a.res_pstride % 64 == 0), "split-bf16 pixel strides");
  if (ST) *a.st_rows = (int)(g / n_tc);
  hipLaunchKernelGGL((halo_conv_kernel<WC, WP, TC, TP, TW, RES, RELU, X3, ST>), dim3((unsigned)g), dim3(64 * WC * WP),
                     G::SMEM, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

template <int WC, int WP, int TC, int TP, int TW, bool X3 = false>
static int launch_halo_g(const BlockConvArgs& a, hipStream_t s) {
  if (a.res) return a.relu ? launch_halo_t<WC, WP, TC, TP, TW, true, true, X3>(a, s)
                           : launch_halo_t<WC, WP, TC, TP, TW, true, false, X3>(a, s);
  return a.relu ? launch_halo_t<WC, WP, TC, TP, TW, false, true, X3>(a, s)
                : launch_halo_t<WC, WP, TC, TP, TW, false, false, X3>(a, s);
}

// Variants (channels x tile (TH x TW), waves, wave tile, LDS; one WG per CU):
//  20: 64 x 16x16  8w  64x32  154 KB
//  21: 64 x 16x16  4w  64x64  156 KB (one wave per SIMD: half the LDS fragment reads per MFMA)
//  22: 128 x 16x16 8w  64x64  146 KB (Cout 128: one patch read per tile instead of two, a
//      third fewer LDS fragment reads per MFMA than 20; 4-stage weight ring, register epilogue)
int launch_halo_v(const BlockConvArgs& a, int v, hipStream_t s, bool x3) {
  if (x3) {
    SAD_REQUIRE(v == 20, "split-bf16 halo conv: variant 20");
    return launch_halo_g<1, 8, 4, 2, 16, true>(a, s);
  }
  if (a.st_part) {
    SAD_REQUIRE(v == 20 && !a.res && !a.relu && a.st_rows,
                "fused BN statistics: halo variant 20, raw conv (no residual / ReLU), st_rows set");
    return launch_halo_t<1, 8, 4, 2, 16, false, false, false, true>(a, s);
  }
  switch (v) {
    case 20: return launch_halo_g<1, 8, 4, 2, 16>(a, s);
    case 21: return launch_halo_g<1, 4, 4, 4, 16>(a, s);
    case 22: return launch_halo_g<2, 4, 4, 4, 16>(a, s);
  }
  set_error("unknown halo-conv variant");
  return SAD_ERR_ARG;
}

}  // namespace sad
