// l2s2conv.hip -- variant 43: resident-weight, patch-resident stride-2 3x3 conv
// for Cin = 64 -> Cout = 128 (bf16, gfx950): layer2's first conv,
//   out[oy, ox, co] = relu( sum_{ky, kx, ci} X[2 oy + ky - 1, 2 ox + kx - 1; ci] W[co, ky, kx, ci] + b[co] )
// (inference_runner.py:49-51 via timm resnet18 forward_features: layer2.0
// conv1 -> bn1 -> act1, BN folded into W and b).
//
// The implicit GEMM (variant 15) ran this conv at 0.25 of the MFMA peak: each
// 64-deep K-step re-fetched its im2col rows through L2 into LDS behind a
// barrier, and its weights streamed through LDS too.  Variant 41's scheme
// (l2conv.hip) fits it with room to spare: a wave owning 32 output channels
// holds 32 x 576 K x 2 B / 64 lanes = 144 weight registers (AGPRs, read by
// inline-asm MFMAs), so the whole launch moves no weight bytes, and the pixel
// operand is the tile's input patch, DMA'd to LDS once:
//  * a workgroup owns a 16 x 16 output tile x 128 channels, 4 waves x 32
//    channels; the tile runs as two row-half "chunks" (output rows 0-7, 8-15),
//    each over its 17 x 33 input patch x 64 channels (71.8 KB), double-buffered:
//    chunk 0's patch in buffer 0, chunk 1's in buffer 1, the other buffer's
//    next patch DMA'd during a chunk, one barrier per chunk;
//  * per chunk a wave runs 9 taps x 2 K-halves x 8 fragments (output rows):
//    one ds_read_b128 and 2 MFMA 16x16x32 per unit, 288 MFMAs, then the epilogue
//    of its 8 rows (bias in the accumulators, ReLU on packed bf16, 16-B stores
//    paired by v_permlane16_swap as in variant 41);
//  * the patch is de-interleaved by row and column parity, so a fragment's 16
//    pixels (input columns 2 ox + kx) are 16 consecutive pixel slots: rows
//    0, 2, .., 16 first, then 1, .., 15 (a tap's rows 2 j + ky are rows j + ky/2
//    of the even plane or row j of the odd one); per row the 17 even columns,
//    then the 16 odd ones, 128 B each (kx = 0 -> even slot fr, 1 -> odd slot
//    fr, 2 -> even slot fr + 1); 16-B chunk c of plane column x' at c ^ key(x')
//    (key by search: every ds_read_b128 lane group of every tap and K-half hits
//    16 distinct bank slots, tests/test_rwconv_layout.py);
//  * a DMA piece is 1 KB of that layout (8 pixels x 8 chunks, 8 lanes per
//    pixel: whole 128-B lines), the lanes gathering their source pixels; pad
//    and out-of-image pixels read as zero.  71 pieces per chunk, issued one
//    per 8 units (16 MFMAs) by each wave.
#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"
#include "rwconv.hpp"

namespace sad {

namespace l2s {
constexpr int NW = 4;
constexpr int PRR = 17, PCW = 33;                // patch rows per chunk, patch columns
constexpr int NEV = 9;                           // even patch rows (first), then 8 odd ones
constexpr int PXB = 128;                         // bytes per pixel (64 channels)
constexpr int ROWB = PCW * PXB;                  // 4,224 B per patch row
constexpr int ODDC = 17 * PXB;                   // the odd-column plane within a row
constexpr int NPX = PRR * PCW;                   // 561 pixels
constexpr int NDP = (NPX * PXB + 1023) / 1024;   // 71 DMA pieces per chunk
constexpr int PATCH = NDP * 1024;                // 72,704 B
constexpr int QP = (NDP + NW - 1) / NW;          // 18 pieces per wave per chunk
constexpr int OFF_BIAS = 2 * PATCH;
constexpr int SMEM = OFF_BIAS + 512;
constexpr int NS = 18;                           // K-steps: 9 taps x 2 halves of 32 channels
constexpr int TP = 8;                            // fragments (output rows) per chunk
constexpr int NUC = 9 * 2 * TP;                  // 144 units per chunk
constexpr int DQ = 8;                            // fragment reads in flight
// units between a wave's DMA pieces: spread over the chunk (all at its start
// measured 4 % faster in isolation, neutral end to end)
constexpr int PDIV = 8;
constexpr int BAD = 0x7FFFFFF0;
constexpr uint64_t KEY = 0x7929284ef1797ull;     // 3-bit chunk key per plane column 0..16
static_assert(SMEM <= 160 * 1024, "LDS budget");
static_assert(NUC / PDIV >= QP, "pieces fit the chunk's units");
static_assert(NW - 1 + NW * (QP - 2) < NDP, "only the last piece index can pass the patch");
static_assert(8 * ROWB + ODDC + 16 * PXB <= 65535, "fragment offsets are ds_read immediates");
}  // namespace l2s

__device__ __forceinline__ int l2s_key(int x) { return (int)((l2s::KEY >> (3 * x)) & 7); }

// ST (the trainer's raw conv): also the fused BN statistics, fp32 sums of the
// accumulators and their squares per channel, one row of a.st_part
// ([rows][2][128]) per workgroup
template <bool ST = false>
__global__ __launch_bounds__(256, 1) void l2s2conv_kernel(BlockConvArgs a) {
  using namespace l2s;
  const int ab = a.ablate;  // timing ablations (wrong results): 32 no patch DMA in the loop, 8 no epilogue stores
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int cw = wave * 32;  // this wave's first output channel
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_x = a.Wo / 16, tiles_img = tiles_x * (a.Ho / 16);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)w * tiles_p / gridDim.x), tp_end = (int)((int64_t)(w + 1) * tiles_p / gridDim.x);
  if (tp_begin >= tp_end) {  // whole workgroup (uniform); its statistics row is zero
    if constexpr (ST) a.st_part[(int64_t)w * 256 + tid] = 0.f;
    return;
  }

  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.out, (short)0, (int)a.out_bytes, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int ps = (int)a.in0_pstride * 2;  // bytes per input pixel

  struct TileO {
    int base, b, oy0, ox0;
  };
  // tile t: output origin (oy0, ox0); base = the offset of input pixel
  // (2 oy0, 2 ox0), patch pixel (1, 1) of row-half 0
  auto tile_o = [&](int t) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int ty = rem / tiles_x;
    TileO o;
    o.b = b;
    o.oy0 = ty * 16;
    o.ox0 = (rem - ty * tiles_x) * 16;
    o.base = ((b * a.H + 2 * o.oy0) * a.W + 2 * o.ox0) * ps;
    return o;
  };
  // DMA piece k of a wave (q = wave + 4k) writes LDS bytes q * 1024 + 16 ln of
  // the layout above: pixel slot u = 8q + ln / 8 (patch row r = u / 33 ->
  // input row Y; plane column -> input column X), chunk slot ln % 8.  Its source
  // offset from the tile's base is tile-invariant (row-half 1: + 16 input rows),
  // so it is computed once per lane and piece, with three flags in its low bits
  // (offsets are multiples of 16): 1 = patch row 0 (above the image on the first
  // tile row), 2 = patch column 0 (left of it on the first tile column), 4 = past
  // the patch.  The right and bottom edges are never crossed: the input is
  // exactly twice the output.
  int prel[QP];
#pragma unroll
  for (int k = 0; k < QP; ++k) {
    const int u = 8 * (wave + NW * k) + (lane >> 3);
    const int r = (u * 1986) >> 16;  // u / 33 exactly for u < 568
    const int cu = u - PCW * r;
    const int Y = r < NEV ? 2 * r : 2 * (r - NEV) + 1;
    const bool odd = cu >= 17;
    const int xp = odd ? cu - 17 : cu;
    const int X = 2 * xp + (odd ? 1 : 0);
    const int c = (lane & 7) ^ l2s_key(xp);
    prel[k] = (((Y - 1) * a.W + (X - 1)) * ps + (c << 4)) | (Y == 0 ? 1 : 0) | (X == 0 ? 2 : 0) | (u >= NPX ? 4 : 0);
  }
  const int hstep = 16 * a.W * ps;  // row-half 1's patch: 16 input rows down
  auto issue_piece = [&](int k, const TileO& o, int h) __attribute__((always_inline)) {
    const int q = wave + NW * k;
    if (k == QP - 1 && q >= NDP) return;  // uniform (pieces k < QP - 1 always exist)
    const int mask = 4 | (h == 0 && o.oy0 == 0 ? 1 : 0) | (o.ox0 == 0 ? 2 : 0);  // uniform
    const int e = prel[k];
    const int off = o.base + h * hstep + (e & ~15);
    dma16_m0(rx, (e & mask) ? BAD : off, lds0 + h * PATCH + q * 1024);
  };

  // ---- weights into registers: K-step s = (tap, K-half kh) -> lane (fr, fg)
  // holds channels kh * 32 + fg * 8 .. +7 of tap `tap` for output channel
  // cw + 16 i + fr
  l1b_v4 wr[2][NS];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < NS; ++s)
      wr[i][s] = *(const l1b_v4*)((const u16*)a.wt + (size_t)(cw + 16 * i + fr) * a.wt_ld + (s >> 1) * 64 +
                                  (s & 1) * 32 + fg * 8);
  // the bias (the accumulators' start value) behind the LDS buffers
  if (tid < 32) *(float4*)(smem + OFF_BIAS + 16 * tid) = *(const float4*)(a.bias + 4 * tid);
  auto biasv = [&](int i) __attribute__((always_inline)) {
    return *(const f32x4*)(smem + OFF_BIAS + (cw + 16 * i + fg * 4) * 4);
  };
  {
    const TileO o0 = tile_o(tp_begin);
#pragma unroll
    for (int k = 0; k < QP; ++k) issue_piece(k, o0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 acc[2][TP];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const f32x4 b0 = biasv(i);
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = b0;
  }

  // the lane's fragment offsets within a patch row: kx = 0 -> even column
  // slot fr, 1 -> odd slot fr, 2 -> even slot fr + 1
  int L[3][2];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) {
    const int xp = fr + (kx == 2 ? 1 : 0);
    const int key = l2s_key(xp);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh) L[kx][kh] = (kx == 1 ? ODDC : 0) + xp * PXB + (((4 * kh + fg) ^ key) << 4);
  }

  // ST: per-lane partial sums of channels cw + 16 i + 4 fg + e over this
  // workgroup's pixels, then across the 16 pixel lanes at the end
  float st_s[2][4] = {}, st_q[2][4] = {};
  for (int t = tp_begin; t < tp_end; ++t) {
    const TileO o = tile_o(t);
    const TileO onext = tile_o(t + 1 < tp_end ? t + 1 : t);
    const int frt = fr, fgt = fg;
    const int obase = ((o.b * a.Ho + o.oy0) * a.Wo + o.ox0) * (int)(a.out_pstride * 2);  // uniform

    l1b_for<2>([&](auto hc) __attribute__((always_inline)) {
      constexpr int h = decltype(hc)::value;
      // this chunk's patch (this wave's pieces; the previous chunk's 8 stores,
      // youngest, may stay in flight) is published by the barrier
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // bases per (kx, kh, row plane): the buffer and the odd-row plane in the
      // base, so the row offsets stay ds_read immediates
      int B[3][2][2];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int p = 0; p < 2; ++p) B[kx][kh][p] = L[kx][kh] + h * PATCH + p * NEV * ROWB;
      // unit u: tap u / 16, K-half (u / 8) % 2, fragment (output row) u % 8
      auto rd = [&](auto uc) __attribute__((always_inline)) -> uint4 {
        constexpr int u = decltype(uc)::value;
        constexpr int tap = u / 16, ky = tap / 3, kx = tap % 3, kh = (u / 8) & 1, j = u % 8;
        constexpr int p = ky == 1 ? 1 : 0, row = ky == 1 ? j : j + ky / 2;
        return *(const uint4*)(smem + B[kx][kh][p] + row * ROWB);
      };
      uint4 bq[DQ];
      l1b_for<DQ>([&](auto uc) __attribute__((always_inline)) { bq[decltype(uc)::value] = rd(uc); });
      l1b_for<NUC>([&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        constexpr int s = 2 * (u / 16) + ((u / 8) & 1), j = u % 8;
        const uint4 bf = bq[u % DQ];
        if constexpr (u + DQ < NUC) bq[u % DQ] = rd(std::integral_constant<int, u + DQ>{});
        // DMA: row-half 0 carries this tile's row-half-1 patch, row-half 1 the
        // next tile's row-half-0 patch (the last tile's own again: harmless)
        if constexpr (u % PDIV == 0 && u / PDIV < QP) {
          if (ab & 32) {
          } else if constexpr (h == 0)
            issue_piece(u / PDIV, o, 1);
          else
            issue_piece(u / PDIV, onext, 0);
        }
        l1b_mfma_a(acc[0][j], wr[0][s], bf);
        l1b_mfma_a(acc[1][j], wr[1][s], bf);
      });
      // asm MFMA results read by compiler code: 12 wait states (8-pass XDL)
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 11" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);

      // ---- epilogue of output rows 8h .. 8h + 7: ReLU on packed bf16 -> 16-B
      // stores; for rows j, j + 1 one v_permlane16_swap per dword pairs lane row
      // fg with its neighbour row, so lane rows 0/2 hold 8 channels of pixel row
      // j, 1/3 of j + 1
#pragma unroll
      for (int j = 0; j < TP; j += 2) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const f32x4 v0 = acc[i][j], v1 = acc[i][j + 1];
          if constexpr (ST) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              st_s[i][e] += v0[e];
              st_s[i][e] += v1[e];
              st_q[i][e] = fmaf(v0[e], v0[e], st_q[i][e]);
              st_q[i][e] = fmaf(v1[e], v1[e], st_q[i][e]);
            }
          }
          uint32_t q[4] = {l1b_pk(v0[0], v0[1]), l1b_pk(v0[2], v0[3]), l1b_pk(v1[0], v1[1]), l1b_pk(v1[2], v1[3])};
          if (a.relu)
#pragma unroll
            for (int e = 0; e < 4; ++e) q[e] = l1b_relu2(q[e]);
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const auto r = __builtin_amdgcn_permlane16_swap(q[e], q[e + 2], false, false);
            q[e] = r[0];
            q[e + 2] = r[1];
          }
          const int px = (8 * h + j + (fgt & 1)) * a.Wo + frt;
          const int co = cw + 16 * i + (fgt >> 1) * 8;
          if (!(ab & 8))
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(l1b_v4, make_uint4(q[0], q[1], q[2], q[3])),
                                                   ro, px * (int)(a.out_pstride * 2) + co * 2, obase, 0);
          const f32x4 b0 = biasv(i);
          acc[i][j] = b0;
          acc[i][j + 1] = b0;
        }
      }
    });
  }
  if constexpr (ST) {
    // across the 16 lanes (pixel columns) of each channel group, fixed order
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int off = 1; off < 16; off <<= 1) {
          st_s[i][e] += __shfl_xor(st_s[i][e], off, 64);
          st_q[i][e] += __shfl_xor(st_q[i][e], off, 64);
        }
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = cw + 16 * i + 4 * fg + e;
          a.st_part[(int64_t)w * 256 + c] = st_s[i][e];
          a.st_part[(int64_t)w * 256 + 128 + c] = st_q[i][e];
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int launch_l2s2conv(const BlockConvArgs& a, hipStream_t s) {
  using namespace l2s;
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 2 && a.pad == 1 && !a.in1 && !a.res && !a.pool_out,
              "variant 43: 3x3/s2/p1, no shortcut, residual or pool");
  SAD_REQUIRE(!a.st_part || (!a.relu && a.st_rows), "variant 43 statistics: the raw conv (no ReLU), st_rows set");
  SAD_REQUIRE(a.Cin == 64 && a.Cout == 128, "variant 43: Cin 64, Cout 128");
  SAD_REQUIRE(a.Ho % 16 == 0 && a.Wo % 16 == 0 && a.H == 2 * a.Ho && a.W == 2 * a.Wo,
              "variant 43: output must tile by 16 x 16, input twice its size");
  SAD_REQUIRE(a.wt_ld >= 9 * 64 && a.wt_ld % 8 == 0, "variant 43: weight rows");
  SAD_REQUIRE(a.in0_pstride % 8 == 0 && a.in0_pstride >= 64 && a.out_pstride % 8 == 0 && a.out_pstride >= 128 && a.out,
              "variant 43: 16-B aligned pixel strides, an output");
  const int64_t tiles = (int64_t)a.N * (a.Ho / 16) * (a.Wo / 16);
  if (tiles == 0) return SAD_OK;
  const int64_t g = std::min<int64_t>(tiles, 256);
  BlockConvArgs b = a;
  b.out_bytes = ((int64_t)a.N * a.Ho * a.Wo - 1) * a.out_pstride * 2 + 256;
  SAD_REQUIRE(b.out_bytes < (1ll << 31) - 65536, "variant 43: output passes the 32-bit buffer range");
  if (a.st_part) {
    static bool attr = false;
    if (!attr) {
      SAD_CHECK_HIP(hipFuncSetAttribute((const void*)l2s2conv_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
      attr = true;
    }
    hipLaunchKernelGGL(l2s2conv_kernel<true>, dim3((unsigned)g), dim3(256), SMEM, s, b);
    *a.st_rows = (int)g;
  } else {
    static bool attr = false;
    if (!attr) {
      SAD_CHECK_HIP(hipFuncSetAttribute((const void*)l2s2conv_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
      attr = true;
    }
    hipLaunchKernelGGL(l2s2conv_kernel<false>, dim3((unsigned)g), dim3(256), SMEM, s, b);
  }
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

}  // namespace sad
