// l2conv.hip -- variant 41: resident-weight, patch-resident 3x3 conv for
// Cin = Cout = 128, stride 1 (bf16, gfx950): layer2's second BasicBlock,
//   out = act(conv3x3(x; W) + b [+ res])
// (inference_runner.py:49-51 via timm resnet18 forward_features; conv1 ->
// bn1 -> act1 with res = 0, conv2 -> bn2 -> + identity -> act2 with res = the
// block input).
//
// The register-resident weight scheme of the fused layer1 block (variant 40,
// l1block.hip) fits one 128-channel conv exactly: a wave owning 32 output
// channels holds 32 x 1,152 K x 2 B / 64 lanes = 288 registers of weights
// (256 in AGPRs, read by inline-asm MFMAs; 32 in VGPRs).  4 waves, one per
// SIMD, each 32 channels x all 256 pixels of a 16 x 16 tile (2 x 16 MFMA
// fragments, 128 accumulator VGPRs starting at the bias); per K-step of 32
// channels a wave reads 16 pixel fragments from LDS and issues 32 MFMAs: no
// weight traffic and no weight ring.
//
// LDS: the 18 x 18 input patch of each 64-channel chunk (variant 30's column
// swizzle: fragment addresses are lane constants + immediates), double-
// buffered by chunk -- chunk 0 of a tile in buffer 0, chunk 1 in buffer 1, the
// next chunk's patch DMA'd while the current one is computed, one barrier per
// chunk -- plus, with a residual, the tile's 16 x 16 x 128 residual (DMA'd in
// chunk 0, read by the epilogue; 16-B chunks XOR-swizzled by pixel column so the
// epilogue's 8-B reads are conflict-free).  149.5 KB.
// Epilogue: bias already in the accumulators, + residual, ReLU on packed bf16,
// 16-B stores (v_permlane16_swap pairs fragment rows j, j + 1).
//
// DS (layer2's first block, conv2 + downsample): the 1x1/2 downsample of the
// 64-channel block input is two more K-steps after the conv's 36 (its weights
// the 64 K columns behind the taps, 16 more VGPRs per wave), over a 16 x 16
// pixel patch of the input at stride 2 DMA'd to LDS during chunk 0 (16-B chunk
// c of pixel p at c ^ ((p >> 1) & 7): conflict-free fragment reads).
//
// X3 (variant 42, round 4): the split-bf16 parity mode's layer1 convs, logical
// Cin = Cout = 64 = 128 bf16 input channels ([hi 32 | lo 32] x 2 chunks, the
// same 2 x 128-B chunks per pixel as the bf16 128-channel conv): the same 288
// resident weight registers per wave then hold 32 logical output channels'
// hi and lo weights, so the 4 waves are 2 channel groups x 2 pixel halves (8
// fragments each).  Per fragment and tap the hi fragment feeds W_hi.X_hi and
// W_lo.X_hi, the lo fragment W_hi.X_lo: 3 MFMAs per fragment read (bf16: 2).
// The identity residual (hi + lo, 256 B per pixel) has the 128-channel conv's
// LDS tile layout; the epilogue splits relu(acc + res) into hi / lo again.
#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"
#include "rwconv.hpp"

namespace sad {

namespace l2c {
constexpr int NW = 4;
constexpr int PW = 18, PR = PW * PW;           // 18 x 18 patch per 64-channel chunk
constexpr int NDP = (PR + 7) / 8;              // 41 DMA pieces of 8 pixel rows
constexpr int PATCH = NDP * 1024;
constexpr int ROWB = PW * 128;
constexpr int QP = (NDP + NW - 1) / NW;        // 11 pieces per wave per chunk
constexpr int RESB = 256 * 256;                // residual tile: 256 pixels x 128 ch bf16
constexpr int NRP = RESB / 1024 / NW;          // 16 residual pieces per wave
constexpr int NDS = 256 * 128 / 1024 / NW;     // 8 downsample pieces per wave
constexpr int OFF_RES = 2 * PATCH;
constexpr int SMEM_RES = OFF_RES + RESB;
constexpr int NS = 36;                         // K-steps: 2 chunks x 9 taps x 2 halves of 32 channels
constexpr int NSC = 18;                        // per chunk
constexpr int DQ = 4;                          // fragment reads in flight
constexpr int WV = 8;                          // K-steps of channel tile 1 whose weights sit in VGPRs
constexpr int BAD = 0x7FFFFFF0;
constexpr uint64_t KEY = 0xd92dad912240ull;    // variant 30's column key
static_assert(SMEM_RES + 512 <= 160 * 1024, "LDS budget");
}  // namespace l2c

__device__ __forceinline__ int l2c_key(int x) { return (int)((l2c::KEY >> (3 * x)) & 7); }

// ST (the trainer's raw conv, bf16 plain form): also the fused BN statistics,
// fp32 sums of the accumulators and their squares per channel, one row of
// a.st_part ([rows][2][128]) per workgroup
template <bool RES, bool DS, bool X3 = false, bool ST = false>
__global__ __launch_bounds__(256, 1) void l2conv_kernel(BlockConvArgs a) {
  static_assert(!(RES && DS) && !(X3 && DS), "one shortcut form");
  static_assert(!ST || (!RES && !DS && !X3), "statistics: the plain bf16 form");
  using namespace l2c;
  constexpr int TP = X3 ? 8 : 16;       // fragments (tile rows) per wave
  constexpr int UPT = 2 * TP;           // units per tap: (fragment, K-half)
  constexpr int NUC = 9 * UPT;          // units per chunk
  constexpr int PDIV = X3 ? 8 : 16;     // units between patch DMA pieces
  constexpr int DQ = X3 ? 8 : l2c::DQ;  // fragment reads in flight (X3: 143 VGPRs leave room)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  // this wave's first output channel (logical) and first tile row
  const int cw = X3 ? (wave & 1) * 32 : wave * 32;
  const int r0w = X3 ? (wave >> 1) * 8 : 0;
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_x = a.W / 16, tiles_img = tiles_x * (a.H / 16);
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)w * tiles_p / gridDim.x), tp_end = (int)((int64_t)(w + 1) * tiles_p / gridDim.x);
  if (tp_begin >= tp_end) {  // whole workgroup (uniform); its statistics row is zero
    if constexpr (ST) a.st_part[(int64_t)w * 256 + tid] = 0.f;
    return;
  }

  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(RES ? a.res : DS ? a.in1 : a.in0), (short)0, (int)(RES ? a.res_bytes : DS ? a.in1_bytes : 16), 0x00020000);
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.out, (short)0, (int)a.out_bytes, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;
  const int ps = (int)a.in0_pstride * 2;  // bytes per input pixel

  // ---- patch pieces: piece k of this wave is q = wave + 4k (rows 8q..8q+7 of
  // the 18 x 18 patch); the lane's patch pixel and source offset from the tile
  // origin are tile-independent
  struct TileO {
    int base, oy0, ox0, b;
  };
  auto tile_o = [&](int t) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int ty = rem / tiles_x;
    TileO o;
    o.b = b;
    o.oy0 = ty * 16;
    o.ox0 = (rem - ty * tiles_x) * 16;
    o.base = ((b * a.H + o.oy0) * a.W + o.ox0) * ps;
    return o;
  };
  // piece k of chunk c of tile o into buffer c (branch-free bounds test)
  auto issue_piece = [&](int k, const TileO& o, int c) __attribute__((always_inline)) {
    if (wave + NW * k >= NDP) return;  // uniform
    // the lane's patch pixel and source offset, computed at the issue (VALU in
    // the MFMA shadow instead of registers next to the resident weights)
    int ln;  // opaque lane id: keeps these tile-invariant values from being hoisted
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int r = 8 * (wave + NW * k) + (ln >> 3);
    const int Y = (r * 3641) >> 16, X = r - PW * Y;  // r / 18 exactly for r < 330
    const bool ok = r < PR && (unsigned)(o.oy0 - 1 + Y) < (unsigned)a.H && (unsigned)(o.ox0 - 1 + X) < (unsigned)a.W;
    const int off = o.base + ((Y - 1) * a.W + (X - 1)) * ps + c * 128 + (((ln & 7) ^ l2c_key(X)) << 4);
    dma16_m0(rx, ok ? off : BAD, lds0 + c * PATCH + (wave + NW * k) * 1024);
  };
  // residual piece k (q = wave + 4k: pixels 4q..4q+3 of the tile, 256 B each,
  // 16-B chunk p of pixel px at position p ^ (px & 15))
  auto issue_res = [&](int k, const TileO& o) __attribute__((always_inline)) {
    const int q = wave + NW * k;
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int px = 4 * q + (ln >> 4), pos = ln & 15;
    const int chunk = pos ^ (px & 15);
    const int off = ((o.b * a.H + o.oy0 + (px >> 4)) * a.W + o.ox0 + (px & 15)) * (int)(a.res_pstride * 2) + chunk * 16;
    dma16_m0(rr, off, lds0 + OFF_RES + q * 1024);
  };

  // downsample piece k (q = wave + 4k: pixels 8q..8q+7 of the tile, 128 B
  // each, source pixel (2 oy, 2 ox) of the 64-channel block input)
  auto issue_ds = [&](int k, const TileO& o) __attribute__((always_inline)) {
    const int q = wave + NW * k;
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int px = 8 * q + (ln >> 3), pos = ln & 7;
    const int chunk = pos ^ ((px >> 1) & 7);
    const int off = ((o.b * a.H1 + (o.oy0 + (px >> 4)) * a.ss1) * a.W1 + (o.ox0 + (px & 15)) * a.ss1) *
                        (int)(a.in1_pstride * 2) + chunk * 16;
    dma16_m0(rr, off, lds0 + OFF_RES + q * 1024);
  };
  // the downsample's weights: K-steps h = 0, 1 (channels (fg + 4h)*8..+7)
  l1b_v4 wds[2][2];
  if constexpr (DS) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        wds[i][h] = *(const l1b_v4*)((const u16*)a.wt + (size_t)(cw + 16 * i + fr) * a.wt_ld + 9 * 128 + (fg + 4 * h) * 8);
  }

  // ---- weights into registers: K-step s = (chunk c, tap, half h) -> lane
  // (fr, fg) holds channels c*64 + (fg + 4h)*8 .. +7 of tap `tap` for output
  // channel cw + 16 i + fr
  l1b_v4 wr[2][NS];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int c = s / NSC, tap = (s % NSC) >> 1, h = s & 1;
      wr[i][s] = *(const l1b_v4*)((const u16*)a.wt + (size_t)(cw + 16 * i + fr) * a.wt_ld + tap * 128 + c * 64 +
                                  (fg + 4 * h) * 8);
    }
  // the bias (the accumulators' start value) behind the LDS buffers
  if (tid < (X3 ? 16 : 32))
    *(float4*)(smem + (RES || DS ? SMEM_RES : OFF_RES) + 16 * tid) = *(const float4*)(a.bias + 4 * tid);
  auto biasv = [&](int i) __attribute__((always_inline)) {
    return *(const f32x4*)(smem + (RES || DS ? SMEM_RES : OFF_RES) + (cw + 16 * i + fg * 4) * 4);
  };
  {
    const TileO o0 = tile_o(tp_begin);
#pragma unroll
    for (int k = 0; k < QP; ++k) issue_piece(k, o0, 0);
  }

  // the first patch has landed before the first barrier (the loop's chunk-0
  // wait lets 16 younger operations, the previous tile's stores, stay in
  // flight); the bias is visible after it
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  f32x4 acc[2][TP];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const f32x4 b0 = biasv(i);
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = b0;
  }

  // ST: per-lane partial sums of channels cw + 16 i + 4 fg + e over this
  // workgroup's pixels (column fr of every tile row), then across fr at the end
  float st_s[2][4] = {}, st_q[2][4] = {};
  for (int t = tp_begin; t < tp_end; ++t) {
    const TileO o = tile_o(t);
    const TileO onext = tile_o(t + 1 < tp_end ? t + 1 : t);
    // lane constants per tile from an opaque lane id (hoisted out of the tile
    // loop they would crowd the 288 weight registers)
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int frt = ln & 15, fgt = ln >> 4;
    int I2[3][2];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int h = 0; h < 2; ++h) I2[kx][h] = ((frt + kx) * 128 + ((fgt ^ l2c_key(frt + kx)) << 4)) ^ (h << 6);

    l1b_for<2>([&](auto cc) __attribute__((always_inline)) {
      constexpr int c = decltype(cc)::value;
      // the chunk's patch (this wave's pieces; the tile's stores, youngest, may
      // stay in flight) is published by the barrier
      if constexpr (c == 0)
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // this chunk's buffer in the bases, so the immediates stay < 64 KB
      int I2c[3][2];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int h = 0; h < 2; ++h) I2c[kx][h] = I2[kx][h] + c * PATCH;
      // unit u of the chunk: tap u / UPT; bf16: K-half h = (u % UPT) / 16,
      // fragment j = u % 16 (K-half-outer, as round 3); X3: fragment
      // j = (u % UPT) / 2, h = u % 2 (the hi fragment, then the lo one)
      auto rd = [&](auto uc) __attribute__((always_inline)) -> uint4 {
        constexpr int u = decltype(uc)::value;
        constexpr int tap = u / UPT, ky = tap / 3, kx = tap % 3;
        constexpr int j = X3 ? (u % UPT) / 2 : u % 16, h = X3 ? u % 2 : (u % UPT) / 16;
        return *(const uint4*)(smem + I2c[kx][h] + (r0w + j + ky) * ROWB);
      };
      uint4 bq[DQ];
      l1b_for<DQ>([&](auto uc) __attribute__((always_inline)) { bq[decltype(uc)::value] = rd(uc); });
      l1b_for<NUC>([&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        constexpr int tap = u / UPT;
        constexpr int j = X3 ? (u % UPT) / 2 : u % 16, h = X3 ? u % 2 : (u % UPT) / 16;
        constexpr int s = c * NSC + 2 * tap + h;   // this fragment's K-step (bf16; X3: its hi / lo weights)
        constexpr int s_hi = c * NSC + 2 * tap, s_lo = s_hi + 1;
        const uint4 bf = bq[u % DQ];
        if constexpr (u + DQ < NUC) bq[u % DQ] = rd(std::integral_constant<int, u + DQ>{});
        // DMA: chunk 0 carries this tile's chunk-1 patch and residual; chunk 1
        // the next tile's chunk-0 patch
        if constexpr (u % PDIV == 0 && u / PDIV < QP)
          if (!(a.ablate & 32)) issue_piece(u / PDIV, c == 0 ? o : onext, c ^ 1);
        if constexpr (RES && c == 0 && u % PDIV == PDIV / 2 && u / PDIV < NRP) issue_res(u / PDIV, o);
        if constexpr (DS && c == 0 && u % 32 == 8 && u / 32 < NDS) issue_ds(u / 32, o);
        auto mm = [&](auto ic, auto sc) __attribute__((always_inline)) {
          constexpr int i = decltype(ic)::value, ss = decltype(sc)::value;
          if constexpr (i == 1 && ss >= NS - WV)
            l1b_mfma_v(acc[i][j], wr[i][ss], bf);
          else
            l1b_mfma_a(acc[i][j], wr[i][ss], bf);
        };
        if constexpr (!X3) {
          mm(std::integral_constant<int, 0>{}, std::integral_constant<int, s>{});
          mm(std::integral_constant<int, 1>{}, std::integral_constant<int, s>{});
        } else if constexpr (u == NUC - 2) {
          // the chunk's last fragment (both its units) as ONE asm statement
          // ending in the 8-pass XDL result wait: hipcc does not pad for asm
          // MFMAs, and around the chunk end its register allocator moves
          // accumulators (v_mov) -- inside one statement it cannot, and after
          // it the results are complete (tools/asm_hazards.py audits this)
          const uint4 xl = bq[(u + 1) % DQ];
          static_assert(j == TP - 1 && h == 0, "last fragment");
          if constexpr (s_hi >= NS - WV)
            asm volatile(
                "v_mfma_f32_16x16x32_bf16 %0, %2, %6, %0\n\t"
                "v_mfma_f32_16x16x32_bf16 %1, %3, %6, %1\n\t"
                "v_mfma_f32_16x16x32_bf16 %0, %4, %6, %0\n\t"
                "v_mfma_f32_16x16x32_bf16 %1, %5, %6, %1\n\t"
                "v_mfma_f32_16x16x32_bf16 %0, %2, %7, %0\n\t"
                "v_mfma_f32_16x16x32_bf16 %1, %3, %7, %1\n\t"
                "s_nop 11"
                : "+v"(acc[0][j]), "+v"(acc[1][j])
                : "a"(wr[0][s_hi]), "v"(wr[1][s_hi]), "a"(wr[0][s_lo]), "v"(wr[1][s_lo]),
                  "v"(__builtin_bit_cast(l1b_v4, bf)), "v"(__builtin_bit_cast(l1b_v4, xl)));
          else
            asm volatile(
                "v_mfma_f32_16x16x32_bf16 %0, %2, %6, %0\n\t"
                "v_mfma_f32_16x16x32_bf16 %1, %3, %6, %1\n\t"
                "v_mfma_f32_16x16x32_bf16 %0, %4, %6, %0\n\t"
                "v_mfma_f32_16x16x32_bf16 %1, %5, %6, %1\n\t"
                "v_mfma_f32_16x16x32_bf16 %0, %2, %7, %0\n\t"
                "v_mfma_f32_16x16x32_bf16 %1, %3, %7, %1\n\t"
                "s_nop 11"
                : "+v"(acc[0][j]), "+v"(acc[1][j])
                : "a"(wr[0][s_hi]), "a"(wr[1][s_hi]), "a"(wr[0][s_lo]), "a"(wr[1][s_lo]),
                  "v"(__builtin_bit_cast(l1b_v4, bf)), "v"(__builtin_bit_cast(l1b_v4, xl)));
        } else if constexpr (u == NUC - 1) {
          // (issued with the previous unit)
        } else if constexpr (h == 0) {  // the hi fragment: W_hi.X_hi, W_lo.X_hi
          mm(std::integral_constant<int, 0>{}, std::integral_constant<int, s_hi>{});
          mm(std::integral_constant<int, 1>{}, std::integral_constant<int, s_hi>{});
          mm(std::integral_constant<int, 0>{}, std::integral_constant<int, s_lo>{});
          mm(std::integral_constant<int, 1>{}, std::integral_constant<int, s_lo>{});
        } else {  // the lo fragment: W_hi.X_lo
          mm(std::integral_constant<int, 0>{}, std::integral_constant<int, s_hi>{});
          mm(std::integral_constant<int, 1>{}, std::integral_constant<int, s_hi>{});
        }
      });
    });
    if constexpr (DS) {
      // the downsample: 2 K-steps over the stride-2 input patch (published by
      // the chunk-1 barrier, whose wait covered its pieces)
      int ln;
      asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
      const int frd = ln & 15, fgd = ln >> 4;
      const int dbase = OFF_RES + frd * 128;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int dofs = dbase + ((((fgd + 4 * h) ^ ((frd >> 1) & 7))) << 4);
        uint4 bd[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) bd[j] = *(const uint4*)(smem + dofs + j * 16 * 128);
#pragma unroll
        for (int j = 0; j < 16; ++j)
#pragma unroll
          for (int i = 0; i < 2; ++i) l1b_mfma_v(acc[i][j], wds[i][h], bd[j]);
      }
    }
    // asm MFMA results read by compiler code: 12 wait states (8-pass XDL)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 11" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);

    // ---- epilogue: (+ residual) -> ReLU on packed bf16 -> 16-B stores: for
    // rows j, j + 1 one v_permlane16_swap per dword pairs lane row fg with its
    // neighbour row, so lane rows 0/2 hold 8 channels of pixel row j, 1/3 of j+1
    const int obase = ((o.b * a.H + o.oy0) * a.W + o.ox0) * (int)(a.out_pstride * 2);  // uniform
#pragma unroll
    for (int j = 0; j < TP; j += 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        f32x4 v0 = acc[i][j], v1 = acc[i][j + 1];
        if constexpr (X3) {
          // residual hi + lo of logical channels cw + 16 i + 4 fgt .. +3: split
          // columns 64 (cw / 32) + 16 i + 4 fgt (hi) and + 32 (lo) -- 16-B chunk
          // ch (hi) / ch + 4 (lo), 8-B half fgt & 1; then ReLU in fp32, hi =
          // bf16(v), lo = bf16(v - hi), 16-B stores of rows (j, j + 1) paired by
          // v_permlane16_swap
          if constexpr (RES) {
            const int ch = 8 * (cw >> 5) + 2 * i + (fgt >> 1);
            const int pa = (r0w + j) * 16 + frt;
            const char* rb0 = smem + OFF_RES + pa * 256 + (fgt & 1) * 8;
            const char* rb1 = rb0 + 16 * 256;
            const uint2 h0 = *(const uint2*)(rb0 + ((ch ^ (pa & 15)) << 4));
            const uint2 l0 = *(const uint2*)(rb0 + (((ch + 4) ^ (pa & 15)) << 4));
            const uint2 h1 = *(const uint2*)(rb1 + ((ch ^ (pa & 15)) << 4));
            const uint2 l1 = *(const uint2*)(rb1 + (((ch + 4) ^ (pa & 15)) << 4));
            v0[0] += __uint_as_float(h0.x << 16) + __uint_as_float(l0.x << 16);
            v0[1] += __uint_as_float(h0.x & 0xFFFF0000u) + __uint_as_float(l0.x & 0xFFFF0000u);
            v0[2] += __uint_as_float(h0.y << 16) + __uint_as_float(l0.y << 16);
            v0[3] += __uint_as_float(h0.y & 0xFFFF0000u) + __uint_as_float(l0.y & 0xFFFF0000u);
            v1[0] += __uint_as_float(h1.x << 16) + __uint_as_float(l1.x << 16);
            v1[1] += __uint_as_float(h1.x & 0xFFFF0000u) + __uint_as_float(l1.x & 0xFFFF0000u);
            v1[2] += __uint_as_float(h1.y << 16) + __uint_as_float(l1.y << 16);
            v1[3] += __uint_as_float(h1.y & 0xFFFF0000u) + __uint_as_float(l1.y & 0xFFFF0000u);
          }
          if (a.relu)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v0[r] = fmaxf(v0[r], 0.f);
              v1[r] = fmaxf(v1[r], 0.f);
            }
          uint32_t qh[4] = {l1b_pk(v0[0], v0[1]), l1b_pk(v0[2], v0[3]), l1b_pk(v1[0], v1[1]), l1b_pk(v1[2], v1[3])};
          const float vv[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
          uint32_t ql[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            ql[e] = l1b_pk(vv[2 * e] - __uint_as_float(qh[e] << 16), vv[2 * e + 1] - __uint_as_float(qh[e] & 0xFFFF0000u));
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const auto rh = __builtin_amdgcn_permlane16_swap(qh[e], qh[e + 2], false, false);
            qh[e] = rh[0];
            qh[e + 2] = rh[1];
            const auto rl = __builtin_amdgcn_permlane16_swap(ql[e], ql[e + 2], false, false);
            ql[e] = rl[0];
            ql[e + 2] = rl[1];
          }
          const int px = (r0w + j + (fgt & 1)) * a.W + frt;
          const int pc = 64 * (cw >> 5) + 16 * i + (fgt >> 1) * 8;  // split column of the hi half
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(l1b_v4, make_uint4(qh[0], qh[1], qh[2], qh[3])), ro,
                                                 px * (int)(a.out_pstride * 2) + pc * 2, obase, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(l1b_v4, make_uint4(ql[0], ql[1], ql[2], ql[3])), ro,
                                                 px * (int)(a.out_pstride * 2) + (pc + 32) * 2, obase, 0);
          const f32x4 b0 = biasv(i);
          acc[i][j] = b0;
          acc[i][j + 1] = b0;
          continue;
        }
        if constexpr (RES) {
          // residual of channels cw + 16 i + 4 fgt .. +3 of pixels (j, frt), (j + 1, frt)
          const int ch = (cw >> 3) + 2 * i + (fgt >> 1);
          const int pa = j * 16 + frt;
          const uint2 r0 = *(const uint2*)(smem + OFF_RES + pa * 256 + ((ch ^ (pa & 15)) << 4) + (fgt & 1) * 8);
          const uint2 r1 = *(const uint2*)(smem + OFF_RES + (pa + 16) * 256 + ((ch ^ (pa & 15)) << 4) + (fgt & 1) * 8);
          v0[0] += __uint_as_float(r0.x << 16);
          v0[1] += __uint_as_float(r0.x & 0xFFFF0000u);
          v0[2] += __uint_as_float(r0.y << 16);
          v0[3] += __uint_as_float(r0.y & 0xFFFF0000u);
          v1[0] += __uint_as_float(r1.x << 16);
          v1[1] += __uint_as_float(r1.x & 0xFFFF0000u);
          v1[2] += __uint_as_float(r1.y << 16);
          v1[3] += __uint_as_float(r1.y & 0xFFFF0000u);
        }
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
        const int px = (j + (fgt & 1)) * a.W + frt;
        const int co = cw + 16 * i + (fgt >> 1) * 8;
        if (!(a.ablate & 8))  // timing ablations (wrong results): 8 no output stores, 32 no patch DMA
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(l1b_v4, make_uint4(q[0], q[1], q[2], q[3])), ro,
                                               px * (int)(a.out_pstride * 2) + co * 2, obase, 0);
        const f32x4 b0 = biasv(i);
        acc[i][j] = b0;
        acc[i][j + 1] = b0;
      }
    }
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

// (x3: the split layout's bf16 channel counts / strides, as launch_block_conv
// passes them: Cin 128 = 64 logical, Cout and the bias logical 64)
int launch_l2conv(const BlockConvArgs& a, hipStream_t s, bool x3) {
  using namespace l2c;
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad == 1 && !a.pool_out,
              "variant 41/42: 3x3/s1/p1, no pool");
  SAD_REQUIRE(!a.st_part || (!x3 && !a.in1 && !a.res && !a.relu && a.st_rows),
              "variant 41 statistics: the plain bf16 raw conv (no shortcut / residual / ReLU), st_rows set");
  if (x3) {
    SAD_REQUIRE(!a.in1 && a.Cin == 128 && a.Cout == 64 && a.H % 16 == 0 && a.W % 16 == 0 && a.Ho == a.H &&
                    a.Wo == a.W && a.wt_ld >= 9 * 128 && a.wt_ld % 8 == 0 && a.in0_pstride % 64 == 0 &&
                    a.in0_pstride >= 128 && a.out_pstride % 64 == 0 && a.out_pstride >= 128 &&
                    (!a.res || (a.res_pstride % 64 == 0 && a.res_pstride >= 128)) && a.out,
                "variant 42: split-bf16 64 -> 64 logical 3x3/s1/p1 (layer1), 16 x 16 tiles");
    const int64_t tiles = (int64_t)a.N * (a.H / 16) * (a.W / 16);
    if (tiles == 0) return SAD_OK;
    const int64_t g = std::min<int64_t>(tiles, 256);
    BlockConvArgs b = a;
    b.out_bytes = ((int64_t)a.N * a.H * a.W - 1) * a.out_pstride * 2 + 256;
    SAD_REQUIRE(b.out_bytes < (1ll << 31) - 65536, "variant 42: output passes the 32-bit buffer range");
    static bool attr[2] = {false, false};
    const void* kfn = a.res ? (const void*)l2conv_kernel<true, false, true> : (const void*)l2conv_kernel<false, false, true>;
    const int smem = (a.res ? SMEM_RES : OFF_RES) + 512;
    if (!attr[a.res ? 1 : 0]) {
      SAD_CHECK_HIP(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, smem));
      attr[a.res ? 1 : 0] = true;
    }
    if (a.res)
      hipLaunchKernelGGL((l2conv_kernel<true, false, true>), dim3((unsigned)g), dim3(256), smem, s, b);
    else
      hipLaunchKernelGGL((l2conv_kernel<false, false, true>), dim3((unsigned)g), dim3(256), smem, s, b);
    SAD_CHECK_HIP(hipGetLastError());
    return SAD_OK;
  }
  SAD_REQUIRE(!a.in1 || (!a.res && a.Cin1 == 64 && a.ss1 == 2 && a.H1 == 2 * a.H && a.W1 == 2 * a.W &&
                         a.in1_pstride % 8 == 0 && a.wt_ld >= 9 * 128 + 64),
              "variant 41: the shortcut is a 1x1/2 downsample of a 64-channel input at twice the size");
  SAD_REQUIRE(a.Cin == 128 && a.Cout == 128, "variant 41: Cin = Cout = 128");
  SAD_REQUIRE(a.H % 16 == 0 && a.W % 16 == 0 && a.Ho == a.H && a.Wo == a.W, "variant 41: image must tile by 16 x 16");
  SAD_REQUIRE(a.wt_ld >= 9 * 128 && a.wt_ld % 8 == 0, "variant 41: weight rows");
  SAD_REQUIRE(a.in0_pstride % 8 == 0 && a.out_pstride % 8 == 0 && (!a.res || a.res_pstride % 8 == 0) &&
                  a.in0_pstride >= 128 && a.out_pstride >= 128 && (!a.res || a.res_pstride >= 128),
              "variant 41: 16-B aligned pixel strides");
  SAD_REQUIRE(a.out, "null output");
  const int64_t tiles = (int64_t)a.N * (a.H / 16) * (a.W / 16);
  if (tiles == 0) return SAD_OK;
  const int64_t g = std::min<int64_t>(tiles, 256);
  BlockConvArgs b = a;
  b.out_bytes = ((int64_t)a.N * a.H * a.W - 1) * a.out_pstride * 2 + 256;
  SAD_REQUIRE(b.out_bytes < (1ll << 31) - 65536, "variant 41: output passes the 32-bit buffer range");
  if (a.res) {
    static bool attr = false;
    if (!attr) {
      SAD_CHECK_HIP(hipFuncSetAttribute((const void*)l2conv_kernel<true, false>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_RES + 512));
      attr = true;
    }
    hipLaunchKernelGGL((l2conv_kernel<true, false>), dim3((unsigned)g), dim3(256), SMEM_RES + 512, s, b);
  } else if (a.in1) {
    static bool attr = false;
    if (!attr) {
      SAD_CHECK_HIP(hipFuncSetAttribute((const void*)l2conv_kernel<false, true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, SMEM_RES + 512));
      attr = true;
    }
    hipLaunchKernelGGL((l2conv_kernel<false, true>), dim3((unsigned)g), dim3(256), SMEM_RES + 512, s, b);
  } else if (a.st_part) {
    static bool attr = false;
    if (!attr) {
      SAD_CHECK_HIP(hipFuncSetAttribute((const void*)l2conv_kernel<false, false, false, true>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, OFF_RES + 512));
      attr = true;
    }
    hipLaunchKernelGGL((l2conv_kernel<false, false, false, true>), dim3((unsigned)g), dim3(256), OFF_RES + 512, s, b);
    *a.st_rows = (int)g;
  } else {
    static bool attr = false;
    if (!attr) {
      SAD_CHECK_HIP(hipFuncSetAttribute((const void*)l2conv_kernel<false, false>,
                                        hipFuncAttributeMaxDynamicSharedMemorySize, OFF_RES + 512));
      attr = true;
    }
    hipLaunchKernelGGL((l2conv_kernel<false, false>), dim3((unsigned)g), dim3(256), OFF_RES + 512, s, b);
  }
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

}  // namespace sad
