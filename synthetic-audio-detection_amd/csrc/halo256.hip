// halo256.hip -- variant 30: patch-resident 256 x 256 block conv for the
// stride-1 3x3 convs of layer3 / layer4 (bf16 and split-bf16, gfx950).
//
// Replaces the same timm BasicBlock halves as block.hip's variant 13
// (conv -> bn [-> + shortcut] -> relu, inference_runner.py:49-51 via timm
// resnet18 forward_features) for the convs with stride 1:
//   out[px, co] = act( sum_{tap, ci} X0[px + tap; ci] W0[co, tap, ci]      3x3 conv, BN folded
//                    + sum_{k1} X1[px * ss1; k1] W1[co, k1]               shortcut (identity or 1x1/2)
//                    + bias[co] )
//
// Why: variant 13 DMAs every input pixel row once per filter tap.  Its stamps
//  put a K-step at ~3,600 cycles for 2,048 cycles of MFMA per
// SIMD, and its operand fill (64 KB per K-step through the CU's LDS-DMA path,
// ~18 B/clk/CU) is what sets the step.  Here a workgroup owns a 16 x 16 output
// tile x 256 output channels and DMAs the 18 x 18 input patch of each
// 64-channel chunk ONCE for all 9 taps, so a K-step moves 32 KB of weights +
// ~4.6 KB of patch instead of 64 KB.
//
// Pipeline (one barrier per K-step; two wave roles, one of each per SIMD):
//  * K-step = (channel chunk, tap) for the 3x3 conv -- 9 per chunk, the patch
//    buffer fixed, the pixel fragments shifted by the tap -- then the
//    shortcut chunks (1 step each, 256 gathered pixel rows of in1 at stride
//    ss1 in a patch buffer; W1 = I for an identity shortcut, exact in bf16).
//  * weight waves (0-3): the 32 KB weight slice of step g+1 into a 2-stage
//    ring right after the barrier of step g (counted vmcnt at the next top);
//  * patch waves (4-7): the next chunk's patch into the other buffer, spread
//    over taps 0-3 of the current chunk (>= 5 steps of cover; a 1-step chunk
//    issues the next chunk's data at once), after their half-0 MFMAs so the
//    issue overlaps the partner wave's MFMAs;
//  * compute as variant 13: operands swapped (C = W . X^T), 128 x 64 wave
//    tiles, half 1's weight fragments read into the registers half 0 frees
//    (rolling prefetch), register epilogue (bias, ReLU, bf16, 8-B stores) or
//    the fused global average pool (layer4's last conv: a tile = one image).
//  * LDS: 2 x 32 KB weights + 2 x 41 KB patches + bias + pool area = 151 KB.
#include <type_traits>
#include <utility>

#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"

#ifndef SAD_STAMPS
#define SAD_STAMPS 0
#endif

namespace sad {

namespace h256 {
constexpr int WC = 2, WP = 4, TC = 8, TP = 4;
constexpr int BC = 16 * TC * WC, BP = 16 * TP * WP;  // 256 channels x 256 pixels
constexpr int TW = 16, TH = 16, PW = TW + 2, PR = PW * (TH + 2);  // 18 x 18 patch
constexpr int NDP = (PR + 7) / 8;  // 41 DMA pieces (8 patch slots of 128 B) per conv chunk
constexpr int SCR = PW * TH;       // a shortcut chunk: 16 x 16 pixels at slots ty * 18 + tx
constexpr int NDS = SCR / 8;       // 36 pieces per shortcut chunk
constexpr int QP = (NDP + 3) / 4;  // <= 11 per patch wave
constexpr int QS = NDS / 4;        // 9 per patch wave
constexpr int QW = BC / 8 / 4;     // 8 weight pieces per weight wave and step
constexpr int WST = BC * 128;      // one weight stage
constexpr int PATCH = NDP * 1024;
constexpr int ROWB = PW * 128;     // bytes per patch row (18 slots)
constexpr int OFF_P = 2 * WST;
constexpr int OFF_BIAS = OFF_P + 2 * PATCH;
constexpr int OFF_POOL = OFF_BIAS + BC * 4;
constexpr int SMEM = OFF_POOL + WP * BC * 4;
constexpr int BAD = 0x7FFFFFF0;  // past num_records: the DMA loads zeros (padding)
// Patch swizzle: chunk c of a slot in patch column px (0..17) lands in 16-B
// slot c ^ key(px), key = 3-bit entries of KEY.  A fragment's 16 lanes read 16
// consecutive columns kx..kx+15 of one patch row; this table (found by a
// search over the ds_read_b128 lane groups) is conflict-free for kx = 0, 1, 2
// and both K-halves, and it depends on the column only, so a fragment's address
// moves by a constant 18 x 128 B per patch row: each lane needs 6 addresses
// (kx x half) for the whole kernel, and a tap's 4 row fragments are immediate
// offsets.  (The previous key, on the slot index, cost ~40 VALU per K-step in
// per-fragment address arithmetic: SQ_INSTS_VALU +49 % over variant 13.)
constexpr uint64_t KEY = 0xd92dad912240ull;  // {0,0,1,1,2,2,4,4,5,5,6,6,2,2,6,6,0,0}
static_assert(SMEM <= 160 * 1024, "LDS budget");
}  // namespace h256

__device__ __forceinline__ int h256_key(int px) { return (int)((h256::KEY >> (3 * px)) & 7); }
// byte offset of lane (fr, fg)'s half-h fragment at patch column kx + fr of a patch row
__device__ __forceinline__ int h256_po(int kx, int h, int fr, int fg) {
  return (kx + fr) * 128 + (((fg + 4 * h) ^ h256_key(kx + fr)) << 4);
}

// X3: split-bf16 parity mode (block.hip): [hi 32 | lo 32] per 128-B chunk,
// three MFMA sets per K-step (W_hi.X_hi + W_lo.X_hi + W_hi.X_lo), hi/lo stores.
// POOL: the fused global average pool (no map stored).
template <bool X3, bool POOL>
__global__ __launch_bounds__(512, 2) void halo256_kernel(BlockConvArgs a) {
  using namespace h256;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool wloader = wave < 4;  // weight wave, else patch wave
  const int lw = wave & 3;
  const int wc = wave / WP, wp = wave % WP;
  const int n_tc = a.Cout / BC;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = w % n_tc;  // both channel tiles of a pixel range share an XCD
  const int gp = gridDim.x / n_tc, wi = w / n_tc;
  const int tiles_x = a.W / TW, tiles_img = tiles_x * (a.H / TH);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)wi * tiles_p / gp), tp_end = (int)((int64_t)(wi + 1) * tiles_p / gp);
  const int c0 = tc * BC;
  if (tp_begin >= tp_end) return;  // whole workgroup (uniform)
  SAD_CLOCK_STAMP(0);

  const int cinb = a.Cin * 2;         // bytes of one pixel's conv channels
  const int nc0 = cinb / 128;         // 64-bf16-channel chunks, 9 taps each
  const int nk1 = a.in1 ? a.Cin1 * 2 / 128 : 0;  // shortcut chunks, 1 step each
  const int nk = 9 * nc0 + nk1;       // K-steps per tile
  const int total = (tp_end - tp_begin) * nk;

  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t r1 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.in1 ? a.in1 : a.in0), (short)0, (int)a.in1_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps0 = (int)a.in0_pstride * 2, ps1 = (int)a.in1_pstride * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int lrow = lane >> 3;

  // ---- weight waves: the 256 weight rows of a K-step; row r's chunk c in slot
  // c ^ (r & 6) (conflict-free for the fragments' 16 consecutive rows), and
  // r & 6 = lrow & 6 for every piece (pieces start at 8-row bounds)
  const int wrow = a.wt_ld * 2;
  const int wlane = (c0 + lrow) * wrow + (((lane & 7) ^ (lrow & 6)) << 4);
  auto issue_weights = [&](int kb, int stage) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < QW; ++i) {
      const int q = lw + 4 * i;
      dma16_m0(rw, wlane + q * 8 * wrow + kb, lds0 + stage * WST + q * 1024);
    }
  };

  // ---- patch waves: the pieces of a chunk (conv chunk: the 18 x 18 patch of
  // 64 channels; shortcut chunk: the 16 x 16 gathered pixels at slots ty*18+tx)
  auto tile_origin = [&](int t, int& b, int& oy0, int& ox0) __attribute__((always_inline)) {
    b = t / tiles_img;
    const int rem = t - b * tiles_img;
    oy0 = (rem / tiles_x) * TH;
    ox0 = (rem - (rem / tiles_x) * tiles_x) * TW;
  };
  struct Chunk {
    int t, c;  // tile; conv chunk (c < nc0) or shortcut chunk nc0 + s
  };
  auto next_chunk = [&](Chunk x) __attribute__((always_inline)) {
    if (++x.c == nc0 + nk1) {
      x.c = 0;
      ++x.t;
    }
    return x;
  };
  // pieces k = tap, tap + 4, ... of chunk x (all of them when tap < 0) into
  // buffer buf.  The tile origin is wave-uniform, computed once per call
  // (recomputed per piece, the patch waves' issue was VALU-bound).
  auto issue_chunk = [&](Chunk x, int buf, int tap) __attribute__((always_inline)) {
    if (x.t >= tp_end) return;
    int b, oy0, ox0;
    tile_origin(__builtin_amdgcn_readfirstlane(x.t), b, oy0, ox0);
    b = __builtin_amdgcn_readfirstlane(b);
    oy0 = __builtin_amdgcn_readfirstlane(oy0);
    ox0 = __builtin_amdgcn_readfirstlane(ox0);
    // lane slot through an opaque move: the compiler would otherwise hoist every
    // piece's (py, px) out of the K loop into registers and spill
    int lr;
    asm volatile("v_mov_b32 %0, %1" : "=v"(lr) : "v"(lrow));
    const unsigned dst = lds0 + OFF_P + buf * PATCH;
    if (x.c < nc0) {
      // slot py*18 + px holds input pixel (oy0 - 1 + py, ox0 - 1 + px)
      const int base = ((b * a.H + oy0 - 1) * a.W + ox0 - 1) * ps0 + x.c * 128;
#pragma unroll
      for (int k = 0; k < QP; ++k) {
        const int q = lw + 4 * k;
        if ((tap < 0 || k % 4 == tap) && q < NDP) {
          const int s = 8 * q + lr, py = s / PW, px = s - py * PW;
          const int iy = oy0 - 1 + py, ix = ox0 - 1 + px;
          const int off = (s < PR && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W)
                              ? base + (py * a.W + px) * ps0 + (((lane & 7) ^ h256_key(px)) << 4)
                              : BAD;
          dma16_m0(r0, off, dst + q * 1024);
        }
      }
    } else {
      // slot ty*18 + tx (tx < 16) holds shortcut pixel ((oy0 + ty) ss1, (ox0 + tx) ss1)
      const int base = ((b * a.H1 + oy0 * a.ss1) * a.W1 + ox0 * a.ss1) * ps1 + (x.c - nc0) * 128;
#pragma unroll
      for (int k = 0; k < QS; ++k) {
        const int q = lw + 4 * k;
        if (tap < 0 || k % 4 == tap) {
          const int s = 8 * q + lr, ty = s / PW, tx = s - ty * PW;
          const int off = tx < TW ? base + (ty * a.W1 + tx) * (a.ss1 * ps1) + (((lane & 7) ^ h256_key(tx)) << 4)
                                  : BAD;
          dma16_m0(r1, off, dst + q * 1024);
        }
      }
    }
  };

  // ---- bias into LDS (published by the first barrier)
  float* s_bias = (float*)(smem + OFF_BIAS);
  if (tid < BC / 4) *(float4*)(smem + OFF_BIAS + 16 * tid) = *(const float4*)(a.bias + c0 + 4 * tid);

  // ---- prologue: weights of step 0 (K offset 0), patch of the first chunk
  if (wloader)
    issue_weights(0, 0);
  else
    issue_chunk(Chunk{tp_begin, 0}, 0, -1);

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  int g = 0, u = 0;  // K-step, chunk counters of the workgroup
  // diagnostic build (-DSAD_STAMPS=1): s_memtime of waves 0 (weight) and 4
  // (patch, its SIMD partner) of workgroup 0 at 4 points of each K-step < 1024
  const bool stamp_on = SAD_STAMPS && a.stamps && blockIdx.x == 0 && (wave == 0 || wave == 4);
  auto stamp = [&](int slot) __attribute__((always_inline)) {
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
  const int ab = a.ablate;  // timing ablations (wrong results): 1 no DMA in the loop, 2 no waits,
                            // 4 no barrier, 8 no epilogue, 16 no weight DMA, 32 no patch DMA;
                            // 64: the patch pieces after the half-0 MFMAs, 128: the weight
                            // pieces after the half-0 MFMAs (same results)
  // weight fragment rows wc*128 + i*16 + fr: slot = chunk ^ (fr & 6)
  const int wsl0 = (fg ^ (fr & 6)) << 4, wsl1 = ((fg + 4) ^ (fr & 6)) << 4;
  const int wrow0 = (wc * 16 * TC + fr) * 128;

  int kb_next = 0;  // K byte offset of the next step's weights (set by the loop)
  // ---- one K-step: weight fragments from stage `ws`; pixel fragment j of
  // half h at patch row wp*4 + ky + j, column kx + fr of buffer pbuf.  The
  // weight waves issue the next step's weights after their half-0 fragment
  // reads (overlapping their latency); the patch waves' pieces (`late`) go at
  // the top of the step, ahead of the weight burst in the CU's DMA queue
  // (after their half-0 MFMAs they waited behind it: l4.c2 +5-15 %)
  auto compute = [&](int ws, int pbuf, int ky, int kx, auto late) __attribute__((always_inline)) {
    if (!wloader && !(ab & 64) && !(ab & 33)) late();
    __builtin_amdgcn_sched_barrier(0);
    const char* wb = smem + ws * WST + wrow0;
    const int pbase = OFF_P + pbuf * PATCH + (wp * TP + ky) * ROWB;  // uniform
    // (computed per step, ~12 VALU: a select among 6 precomputed offsets
    // became a lookup table in scratch)
    const int o0 = h256_po(kx, 0, fr, fg), o1 = h256_po(kx, 1, fr, fg);
    const char* pb0 = smem + pbase + o0;
    const char* pb1 = smem + pbase + o1;
    uint4 wf[TC], pf[TP], pg[TP];
#pragma unroll
    for (int i = 0; i < TC; ++i) wf[i] = *(const uint4*)(wb + i * 16 * 128 + wsl0);
#pragma unroll
    for (int j = 0; j < TP; ++j) pf[j] = *(const uint4*)(pb0 + j * ROWB);
    if (wloader && g + 1 < total && !(ab & 17) && !(ab & 128)) issue_weights(kb_next, (g + 1) & 1);
    __builtin_amdgcn_sched_barrier(0);
    stamp(2);
#pragma unroll
    for (int j = 0; j < TP; ++j) pg[j] = *(const uint4*)(pb1 + j * ROWB);
    // half 0: per weight row i its TP (X3: 2 TP) MFMAs, then the read of its
    // half-1 fragment into the freed registers (rolling prefetch, as variant 13)
    constexpr int SR = X3 ? 2 : TC;
    auto half0_row = [&](int i) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < TP; ++j) mfma_chunk<u16>(wf[i], pf[j], acc[i][j]);
      if constexpr (X3) {  // W_hi . X_lo while W_hi is still in registers
#pragma unroll
        for (int j = 0; j < TP; ++j) mfma_chunk<u16>(wf[i], pg[j], acc[i][j]);
      }
      wf[i] = *(const uint4*)(wb + i * 16 * 128 + wsl1);
    };
#pragma unroll
    for (int i = 0; i < SR; ++i) half0_row(i);
    __builtin_amdgcn_sched_group_barrier(0x100, TP, 0);
#pragma unroll
    for (int i = 0; i < SR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, X3 ? 2 * TP : TP, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (!wloader && (ab & 64) && !(ab & 33)) late();
    // ablate bit 128 (A/B): the weight waves issue after their half-0 MFMAs,
    // so their DMA stall overlaps the patch waves' MFMAs
    if (wloader && g + 1 < total && !(ab & 17) && (ab & 128)) issue_weights(kb_next, (g + 1) & 1);
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
      for (int j = 0; j < TP; ++j) mfma_chunk<u16>(wf[i], X3 ? pf[j] : pg[j], acc[i][j]);  // X3: W_lo . X_hi
  };

  // ---- register epilogue of tile t: lane holds channels co..co+3 of pixel (ty, fr)
  auto epilogue = [&](int t) __attribute__((always_inline)) {
    int b, oy0, ox0;
    tile_origin(t, b, oy0, ox0);
    float4 bias[TC];
#pragma unroll
    for (int i = 0; i < TC; ++i) bias[i] = *(const float4*)(s_bias + wc * 16 * TC + i * 16 + fg * 4);
    if constexpr (POOL) {
      // relu(acc + bias) summed over the wave's pixels (its TP fragments, then
      // the 16 lanes of a row by DPP), then over the WP pixel waves in a fixed
      // order through LDS (deterministic); the tile is the whole image
      float* s_pool = (float*)(smem + OFF_POOL);
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const float bb[4] = {bias[i].x, bias[i].y, bias[i].z, bias[i].w};
        float ps[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = 0.f;
#pragma unroll
          for (int j = 0; j < TP; ++j) v += fmaxf(acc[i][j][r] + bb[r], 0.f);
          ps[r] = row16_sum(v);
        }
        if (fr == 0)
          *(float4*)(s_pool + wp * BC + wc * 16 * TC + i * 16 + fg * 4) = make_float4(ps[0], ps[1], ps[2], ps[3]);
      }
      __syncthreads();
      if (tid < BC) {
        float sum = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < WP; ++w2) sum += s_pool[w2 * BC + tid];
        a.pool_out[(int64_t)b * a.Cout + c0 + tid] = sum * (1.f / BP);
      }
    } else {
      u16* __restrict__ out = (u16*)a.out;
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int64_t px = (int64_t)(b * a.H + oy0 + wp * TP + j) * a.W + ox0 + fr;
#pragma unroll
        for (int i = 0; i < TC; ++i) {
          const int co = c0 + wc * 16 * TC + i * 16 + fg * 4;
          float v[4] = {acc[i][j][0] + bias[i].x, acc[i][j][1] + bias[i].y, acc[i][j][2] + bias[i].z,
                        acc[i][j][3] + bias[i].w};
          if (a.relu)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
          if constexpr (X3) {
            u16* op = out + px * a.out_pstride + ((co >> 5) << 6) + (co & 31);
            u16 h[4], l[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              h[r] = f2bf(v[r]);
              l[r] = f2bf(v[r] - bf2f(h[r]));
            }
            *(uint2*)op = make_uint2((uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16));
            *(uint2*)(op + 32) =
                make_uint2((uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16));
          } else {
            uint2 q;
            q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            *(uint2*)(out + px * a.out_pstride + co) = q;
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // ---- the K loop.  Top of every step: the weight waves retire their DMA of
  // this step's weights (issued one step earlier); the patch waves, at a
  // chunk's first step, that chunk's pieces.  After a tile's epilogue the 32
  // 8-B stores per lane are the youngest operations and may stay in flight
  // (bf16 maps); split-bf16 (64 stores) and the pool wait for everything.
  constexpr int NST = (X3 || POOL) ? 0 : TC * TP;
  bool post_epi = false;
  auto top = [&](bool first_of_chunk) __attribute__((always_inline)) {
    stamp(0);
    if ((wloader || first_of_chunk) && !(ab & 2)) {
      if (post_epi)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    post_epi = false;
    if (!(ab & 4)) __builtin_amdgcn_s_barrier();
    // compiler memory fence: LDS changed behind this barrier (fragment loads
    // from the same addresses must not be merged across steps)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    stamp(1);
  };

  // ---- the K loop, nested: tiles -> chunks (nc0 conv chunks of 9 taps, then
  // nk1 shortcut chunks of 1 step) -> steps, with ONE inlined step body (two
  // inlined copies, conv and shortcut, made the register allocator spill)
  for (int t = tp_begin; t < tp_end; ++t) {
    for (int c = 0; c < nc0 + nk1; ++c) {
      const Chunk nx = next_chunk(Chunk{t, c});
      const int pbuf = u & 1;
      const bool sc = c >= nc0;
      const int nsteps = sc ? 1 : 9;
      // K byte offset of the first step of the next chunk (or next tile)
      const int kb_chunk_next = c + 1 < nc0 ? (c + 1) * 128 : (c + 1 < nc0 + nk1 ? 9 * cinb + (c + 1 - nc0) * 128 : 0);
      for (int tap = 0; tap < nsteps; ++tap) {
        const int ky = tap / 3, kx = tap - 3 * ky;
        kb_next = tap + 1 < nsteps ? (tap + 1) * cinb + c * 128 : kb_chunk_next;
        top(tap == 0);
        // a shortcut chunk's pixels sit at the conv tap (0, 0) positions
        compute(g & 1, pbuf, ky, kx, [&]() __attribute__((always_inline)) {
          if (sc)
            issue_chunk(nx, pbuf ^ 1, -1);
          else if (tap < 4)
            issue_chunk(nx, pbuf ^ 1, tap);
        });
        stamp(3);
        ++g;
      }
      ++u;
    }
    if (!(ab & 8)) epilogue(t);
    post_epi = true;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SAD_CLOCK_STAMP(1);
}

template <bool X3, bool POOL>
static int launch_halo256_t(const BlockConvArgs& a, hipStream_t s) {
  using namespace h256;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)halo256_kernel<X3, POOL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              SMEM);
    attr = true;
  }
  const int n_tc = a.Cout / BC;
  const int64_t tiles_p = (int64_t)a.N * (a.H / TH) * (a.W / TW);
  int64_t g = std::min<int64_t>(tiles_p * n_tc, 256);
  g = std::max<int64_t>(n_tc, g / n_tc * n_tc);
  hipLaunchKernelGGL((halo256_kernel<X3, POOL>), dim3((unsigned)g), dim3(512), SMEM, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

bool halo256_ok(const BlockConvArgs& a) {
  // a: logical channel counts (split-bf16 doubles them in launch_block_conv)
  return a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && a.Cout % h256::BC == 0 && a.H % 16 == 0 &&
         a.W % 16 == 0 && a.Ho == a.H && a.Wo == a.W && !a.res && !a.st_part && a.Cin % 64 == 0 &&
         (!a.in1 || a.Cin1 % 64 == 0) && (!a.pool_out || (a.H == 16 && a.W == 16));
}

// (a: the kernel's bf16 channel counts and strides, as launch_block_conv passes them)
int launch_halo256(const BlockConvArgs& a, hipStream_t s, bool x3) {
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1, "variant 30: 3x3, stride 1, pad 1");
  SAD_REQUIRE(!a.res && !a.st_part, "variant 30: no epilogue residual / fused statistics (shortcut as in1)");
  SAD_REQUIRE(a.Cout % h256::BC == 0, "variant 30: Cout must be a multiple of 256");
  SAD_REQUIRE(a.H % 16 == 0 && a.W % 16 == 0 && a.Ho == a.H && a.Wo == a.W, "variant 30: image must tile by 16 x 16");
  SAD_REQUIRE((a.Cin * 2) % 128 == 0 && (!a.in1 || (a.Cin1 * 2) % 128 == 0), "variant 30: whole 128-B chunks");
  SAD_REQUIRE(!a.in1 || ((a.Ho - 1) * a.ss1 < a.H1 && (a.Wo - 1) * a.ss1 < a.W1), "variant 30: shortcut source");
  SAD_REQUIRE(a.wt_ld >= 9 * a.Cin + (a.in1 ? a.Cin1 : 0) && (a.wt_ld * 2) % 16 == 0, "variant 30: weight rows");
  SAD_REQUIRE(a.out_pstride % 4 == 0 && a.in0_pstride % 8 == 0 && (!a.in1 || a.in1_pstride % 8 == 0),
              "variant 30: pixel strides");
  SAD_REQUIRE(a.out || a.pool_out, "null output");
  SAD_REQUIRE(a.M == (int64_t)a.N * a.H * a.W, "variant 30: M = N H W");
  if (x3) SAD_REQUIRE(a.out_pstride % 64 == 0 || a.pool_out, "split-bf16 pixel strides");
  if (a.pool_out) {
    SAD_REQUIRE(a.H == 16 && a.W == 16, "variant 30 fused average pool: a 16 x 16 tile must be one image");
    return x3 ? launch_halo256_t<true, true>(a, s) : launch_halo256_t<false, true>(a, s);
  }
  return x3 ? launch_halo256_t<true, false>(a, s) : launch_halo256_t<false, false>(a, s);
}

}  // namespace sad
