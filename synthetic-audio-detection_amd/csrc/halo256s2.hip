// halo256s2.hip -- variant 32: patch-resident stride-2 3x3 block conv with the
// weights streamed straight into registers (bf16, gfx950).
//
// The first conv of layer2/3/4's first BasicBlock (conv1 3x3/2 -> bn -> relu,
// inference_runner.py:49-51 via timm resnet18 forward_features):
//   out[oy, ox, co] = relu( sum_{ky, kx, ci} X[2 oy + ky - 1, 2 ox + kx - 1; ci] W[co, ky, kx, ci] + bias[co] )
// run on the implicit GEMM (variants 13 / 15: each 64-deep K-step re-fetches
// its im2col rows through L2 into LDS behind a workgroup barrier).  Here, as in variant 31 (halo256r.hip), a workgroup owns a
// 16 x 16 output tile x BC channels, each wave 32 channels, the weights are
// read from L2 into VGPRs one K-step ahead, and the pixel operand is the
// tile's input patch in LDS, one barrier per channel chunk:
//  * the patch of a 16 x 16 output tile at stride 2 is 33 x 33 input pixels,
//    so a chunk is 32 channels (64 B per pixel; 2 x 76.8 KB double-buffered)
//    and a K-step is one tap x 32 channels (one 16x16x32 MFMA deep);
//  * the patch is stored de-interleaved by column parity: per patch row, the
//    17 even input columns at slots 0..16, the 16 odd ones at 20..35 (row
//    pitch 36 slots = 9 x 256 B), so the 16 pixels of a fragment (output
//    columns ox..ox+15 -> input columns 2 ox + kx) are 16 consecutive slots:
//    kx = 0 -> even slots fr, kx = 1 -> odd slots 20 + fr, kx = 2 -> even
//    slots fr + 1;
//  * 16-B chunk g of the pixel in plane column c sits at position g ^ key(c)
//    (key 2 at plane columns 4, 9..15, else 0): every ds_read_b128 lane group
//    (4 x 16 lanes) hits 16 distinct 16-B bank slots for all three kx;
//  * the DMA writes 16 consecutive slots (1 KB) per wave instruction, the
//    lanes gathering their source pixels (2 columns apart) and 16-B chunks;
//    pad slots 17..19 and out-of-image pixels read as zero.
// Per K-step and wave (BC = 256): 2 x 16-B weight loads, 16 ds_read_b128, 32
// MFMA 16x16x32; 2 patch pieces in each of the chunk's first 5 steps.
// BC = 128 (layer2's 64 -> 128): 4 channel groups x 2 pixel halves, as variant 31.
// The weights are loaded two steps ahead by inline asm and waited for by hand
// (below), so the patch pieces are not waited for one step after their issue.
//
// Status: correct (test_gpu_blockconv.py) but not faster than the implicit
// GEMM on the ResNet-18 shapes (same box, mb 512: l2.c1 644 vs 523 us, l3.c1
// 344 vs 328, l4.c1 284 vs 276), so off by default (SAD_S2_PATCH=1 selects
// it).  Timing ablations (l2.c1 / l3.c1): no patch DMA -35 / -29 %, no weight
// loads -13 / -13 %, no epilogue -25 / -17 %: the gathered DMA (75 pieces per
// 32-channel chunk, twice variant 31's per K) and the synchronous store burst
// at each tile's end are what it would have to shed.
#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"
#include "rwconv.hpp"

namespace sad {

namespace h32 {
constexpr int NW = 8, TC = 2;          // waves; per wave 2 x 16 channels
constexpr int PRH = 33, PRW = 36;      // patch rows; slots per patch row
constexpr int ODD = 20;                // first odd-column slot
constexpr int NSLOT = PRH * PRW;       // 1188 pixel slots
constexpr int NDP = (NSLOT + 15) / 16;  // 75 DMA pieces (16 slots) per chunk
constexpr int PATCH = NDP * 1024;      // 76,800 B (a multiple of 256 B)
constexpr int ROWB = PRW * 64;
constexpr int JUNK = 2 * PATCH;       // 1-KB slot for the pieces past the patch
constexpr int SMEM = 2 * PATCH + 1024;
constexpr int KPW = (NDP + NW - 1) / NW;  // 10 pieces per wave
constexpr int BAD = 0x7FFFFFF0;
constexpr unsigned KEYM = 0xFE10u;     // plane columns with chunk key 2
static_assert(SMEM <= 160 * 1024, "LDS budget");
static_assert(KPW <= 10, "pieces are issued 2 per step over the first 5 steps");
}  // namespace h32

__device__ __forceinline__ int h32_key(int c) { return (int)((h32::KEYM >> c) & 1u) << 1; }

typedef unsigned int h32_v4 __attribute__((ext_vector_type(4)));
typedef __bf16 h32_bf2 __attribute__((ext_vector_type(2)));
typedef float h32_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t h32_pk(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((h32_f2){lo, hi}, h32_bf2));
}
__device__ __forceinline__ uint32_t h32_relu2(uint32_t x) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
  return r;
}

template <int BC>
__global__ __launch_bounds__(512, 1) void halo256s2_kernel(BlockConvArgs a) {
  using namespace h32;
  constexpr int NCG = BC / 32, NPG = NW / NCG, TP = 16 / NPG;
  static_assert(NCG * NPG == NW, "wave split");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int n_tc = a.Cout / BC;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tc = w % n_tc;  // both channel tiles of a pixel range share an XCD
  const int gp = gridDim.x / n_tc, wi = w / n_tc;
  const int tiles_x = a.Wo / 16, tiles_img = tiles_x * (a.Ho / 16);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)wi * tiles_p / gp), tp_end = (int)((int64_t)(wi + 1) * tiles_p / gp);
  if (tp_begin >= tp_end) return;  // whole workgroup (uniform)
  const int cgrp = wave % NCG, pgrp = wave / NCG;
  const int cw = tc * BC + cgrp * 16 * TC;  // this wave's first output channel
  const int r0w = pgrp * TP;                // this wave's first tile row

  const int ab = a.ablate;  // timing ablations (wrong results): 2 no patch DMA, 4 no weight loads, 8 no epilogue
  const int cinb = a.Cin * 2;
  const int nch = cinb / 64;  // 32-channel chunks (9 taps each)

  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps0 = (int)a.in0_pstride * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- weights: lane (fr, fg) of fragment i = row cw + i*16 + fr, K bytes
  // kb + fg*16 of the step (kb = tap * cinb + chunk * 64)
  const int wrow = a.wt_ld * 2;
  const int wlane = (cw + fr) * wrow + fg * 16;
  // The weight loads are inline asm, outside the compiler's wait counting, and
  // waited for by hand: a compiler-tracked load would make the compiler's wait
  // for it (vmcnt(0): it does not count the asm DMA pieces issued after it)
  // also wait for those pieces, one step after their issue.  Each load's
  // registers are tied through the wait (a "+v" operand) into the MFMAs, so nothing
  // reads them before the data has landed.
  auto load_w = [&](int kb, h32_v4 (&wv)[TC]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TC; ++i)
      asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                   : "=v"(wv[i])
                   : "v"(wlane + i * 16 * wrow), "s"(rw), "s"(__builtin_amdgcn_readfirstlane(kb))
                   : "memory");
  };

  // ---- patch pieces k in [k0, k1) of chunk c of tile t into buffer buf: piece
  // q = wave + 8k covers slots 16q..16q+15 (lane: slot 16q + lane/4, 16-B
  // position lane & 3)
  // Every call issues exactly k1 - k0 DMA instructions (the hand-counted waits
  // rely on it): a piece past the patch (q >= 75) or past the last tile loads
  // zeros into a 1-KB junk slot behind the buffers.
  auto issue_patch = [&](int t, int c, int buf, int k0, int k1) __attribute__((always_inline)) {
    const bool live = t < tp_end;  // uniform
    const int tt = __builtin_amdgcn_readfirstlane(live ? t : tp_begin);
    const int b = tt / tiles_img, rem = tt - b * tiles_img;
    const int oy0 = (rem / tiles_x) * 16, ox0 = (rem - (rem / tiles_x) * tiles_x) * 16;
    const int iy0 = 2 * oy0 - 1, ix0 = 2 * ox0 - 1;
    int ln;  // opaque lane id: keeps the per-piece slot math from being hoisted into registers
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int base = ((b * a.H + iy0) * a.W + ix0) * ps0 + c * 64;
    const unsigned dst = lds0 + buf * PATCH;
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
      if (kk >= k1 - k0) break;  // uniform
      const int q = __builtin_amdgcn_readfirstlane(wave + NW * (k0 + kk));
      const bool qv = live && q < NDP;  // uniform
      const int s = 16 * q + (ln >> 2);
      const int row = s / PRW, col = s - PRW * row;
      const bool odd = col >= ODD;
      const int lc = odd ? col - ODD : col;
      const int x = 2 * lc + (odd ? 1 : 0);
      const bool ok = qv && s < NSLOT && (odd || col <= 16) && (unsigned)(iy0 + row) < (unsigned)a.H &&
                      (unsigned)(ix0 + x) < (unsigned)a.W;
      const int off = base + (row * a.W + x) * ps0 + (((ln & 3) ^ h32_key(lc)) << 4);
      dma16_m0(r0, ok ? off : BAD, qv ? dst + q * 1024 : lds0 + JUNK);
    }
  };

  // weights ring: step s (tap within the chunk) uses wr[s % 3], loaded two
  // steps ahead (9 % 3 == 0: the ring continues across chunks)
  h32_v4 wr[3][TC];
  issue_patch(tp_begin, 0, 0, 0, KPW);
  load_w(0, wr[0]);
  load_w(cinb, wr[1]);
  f32x4 biasv[TC];
#pragma unroll
  for (int i = 0; i < TC; ++i) biasv[i] = *(const f32x4*)(a.bias + cw + i * 16 + fg * 4);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[1][0]), "+v"(wr[1][1])::"memory");

  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = biasv[i];


  // ---- one K-step: the pixel fragment of output row j is patch row
  // 2 (r0w + j) + ky, slots (plane column) as above
  auto step = [&](int pbuf, int ky, int kx, const h32_v4 (&wcur)[TC]) __attribute__((always_inline)) {
    int ln;  // opaque lane id: the 9 steps' read bases are not all kept live
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int lc = (ln & 15) + (kx == 2 ? 1 : 0);
    const int slot = (kx == 1 ? ODD : 0) + lc;
    const char* pb = smem + pbuf * PATCH + (2 * r0w + ky) * ROWB + slot * 64 + (((ln >> 4) ^ h32_key(lc)) << 4);
    uint4 bf[TP];
#pragma unroll
    for (int j = 0; j < TP; ++j) bf[j] = *(const uint4*)(pb + 2 * j * ROWB);
#pragma unroll
    for (int j = 0; j < TP; ++j)
#pragma unroll
      for (int i = 0; i < TC; ++i) mfma_chunk<u16>(__builtin_bit_cast(uint4, wcur[i]), bf[j], acc[i][j]);
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int j = 0; j < TP - 4; ++j) {
      __builtin_amdgcn_sched_group_barrier(0x008, TC, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 4 * TC, 0);
  };

  auto epilogue = [&](int t) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int oy0 = (rem / tiles_x) * 16, ox0 = (rem - (rem / tiles_x) * tiles_x) * 16;
    // 16-B stores: v_permlane16_swap pairs fragment rows j, j + 1 (as variant 31)
    u16* __restrict__ out = (u16*)a.out;
#pragma unroll
    for (int j = 0; j < TP; j += 2) {
      const int64_t px = (int64_t)(b * a.Ho + oy0 + r0w + j + (fg & 1)) * a.Wo + ox0 + fr;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        const int co = cw + i * 16 + (fg >> 1) * 8;
        uint32_t q[4] = {h32_pk(acc[i][j][0], acc[i][j][1]), h32_pk(acc[i][j][2], acc[i][j][3]),
                         h32_pk(acc[i][j + 1][0], acc[i][j + 1][1]), h32_pk(acc[i][j + 1][2], acc[i][j + 1][3])};
        if (a.relu)
#pragma unroll
          for (int e = 0; e < 4; ++e) q[e] = h32_relu2(q[e]);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const auto r = __builtin_amdgcn_permlane16_swap(q[e], q[e + 2], false, false);
          q[e] = r[0];
          q[e + 2] = r[1];
        }
        *(uint4*)(out + px * a.out_pstride + co) = make_uint4(q[0], q[1], q[2], q[3]);
      }
    }
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = biasv[i];
  };

  // ---- tiles -> chunks -> taps.  A chunk starts with the barrier that
  // publishes its patch (every wave waited for its pieces at the end of the
  // previous chunk) and frees the other buffer; step s loads step s + 2's
  // weights, steps 0..4 issue the next chunk's pieces (2 per wave each), and
  // step s >= 2 waits for its weights with everything issued after them
  // (weights of s + 1, s + 2, the pieces of s - 2 .. s) left in flight.
  // Steps 0, 1 use weights the previous chunk's final wait covered.
  int u = 0;
  for (int t = tp_begin; t < tp_end; ++t) {
    for (int c = 0; c < nch; ++c) {
      const int nt = c + 1 < nch ? t : t + 1, ncn = c + 1 < nch ? c + 1 : 0;
      const int pbuf = u & 1;
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // the 9 taps unrolled (straight-line code: no phi copies of registers
      // whose loads are still in flight); ring slot = tap % 3
      l1b_for<9>([&](auto tc_) __attribute__((always_inline)) {
        constexpr int tap = decltype(tc_)::value;
        constexpr int r = tap % 3, rn = (tap + 2) % 3;
        const int kbn = tap + 2 < 9 ? (tap + 2) * cinb + c * 64 : (tap + 2 - 9) * cinb + ncn * 64;
        if (!(ab & 4)) load_w(kbn, wr[rn]);
        if constexpr (tap < 5)
          if (!(ab & 2)) issue_patch(nt, ncn, pbuf ^ 1, 2 * tap, 2 * tap + 2);
        if constexpr (tap >= 2) {
          // everything issued after this step's weights stays in flight:
          // pieces P(s) = 2 for s < 5, so P(s-2) + TC + P(s-1) + TC + P(s)
          constexpr int P2 = tap - 2 < 5 ? 2 : 0, P1 = tap - 1 < 5 ? 2 : 0, P0 = tap < 5 ? 2 : 0;
          asm volatile("s_waitcnt vmcnt(%2)" : "+v"(wr[r][0]), "+v"(wr[r][1]) : "n"(P2 + TC + P1 + TC + P0) : "memory");
        }
        step(pbuf, tap / 3, tap % 3, wr[r]);
        __builtin_amdgcn_sched_barrier(0);  // no fragment reads hoisted across steps
      });
      ++u;
      // the next chunk's patch pieces and first two steps' weights (and the
      // previous tile's stores); last in the body, before any copy at the loop
      // latch
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(wr[0][0]), "+v"(wr[0][1]), "+v"(wr[1][0]), "+v"(wr[1][1])::"memory");
    }
    if (!(ab & 8)) epilogue(t);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BC>
static int launch_halo256s2_t(const BlockConvArgs& a, hipStream_t s) {
  using namespace h32;
  static bool attr = false;
  if (!attr) {
    SAD_CHECK_HIP(
        hipFuncSetAttribute((const void*)halo256s2_kernel<BC>, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int n_tc = a.Cout / BC;
  const int64_t tiles_p = (int64_t)a.N * (a.Ho / 16) * (a.Wo / 16);
  int64_t g = std::min<int64_t>(tiles_p * n_tc, 256);
  g = std::max<int64_t>(n_tc, g / n_tc * n_tc);
  hipLaunchKernelGGL((halo256s2_kernel<BC>), dim3((unsigned)g), dim3(512), SMEM, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

bool halo256s2_ok(const BlockConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.stride == 2 && a.pad == 1 && !a.in1 && !a.res && !a.st_part && !a.pool_out &&
         a.Cin % 32 == 0 && a.Cout % 128 == 0 && a.Ho % 16 == 0 && a.Wo % 16 == 0 && a.H == 2 * a.Ho &&
         a.W == 2 * a.Wo;
}

// (a: the kernel's bf16 channel counts and strides, as launch_block_conv passes them)
int launch_halo256s2(const BlockConvArgs& a, hipStream_t s) {
  SAD_REQUIRE(halo256s2_ok(a), "variant 32: 3x3/2 pad 1, no shortcut / residual / pool / statistics, "
                               "Cin % 32, Cout % 128, 16 x 16 output tiles");
  SAD_REQUIRE(a.wt_ld >= 9 * a.Cin && (a.wt_ld * 2) % 16 == 0, "variant 32: weight rows");
  SAD_REQUIRE(a.out_pstride % 8 == 0 && a.in0_pstride % 8 == 0, "variant 32: pixel strides");
  SAD_REQUIRE(a.out != nullptr, "null output");
  SAD_REQUIRE(a.M == (int64_t)a.N * a.Ho * a.Wo, "variant 32: M = N Ho Wo");
  return a.Cout % 256 == 0 ? launch_halo256s2_t<256>(a, s) : launch_halo256s2_t<128>(a, s);
}

}  // namespace sad
