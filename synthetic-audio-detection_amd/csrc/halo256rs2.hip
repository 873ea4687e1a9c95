// halo256rs2.hip -- variant 44: patch-resident stride-2 3x3 conv, weights
// streamed straight into registers, the input patch moved in whole 128-B lines
// (bf16 and split-bf16, gfx950).
//
// The first conv of layer2/3/4's first BasicBlock (conv1 3x3/2 -> bn -> relu,
// inference_runner.py:49-51 via timm resnet18 forward_features):
//   out[oy, ox, co] = relu( sum_{ky, kx, ci} X[2 oy + ky - 1, 2 ox + kx - 1; ci] W[co, ky, kx, ci] + bias[co] )
//
// Why.  Variant 32 (halo256s2.hip) runs these convs with 32-channel chunks: a
// 16 x 16 output tile needs the 33 x 33 input patch, which at 64 B per pixel is
// the most two buffers of LDS hold.  A 32-channel chunk is HALF of every 128-B
// line of a 256-B (layer3) or 512-B (layer4) pixel, so each line is fetched in
// two chunk passes ~9 K-steps apart, and in between the rest of the XCD's
// streaming evicts it: rocprof puts variant 32's reads at 1.93x the input
// (profiles/r04_pmc_traffic.json).  Here a chunk is 64 channels = one whole
// 128-B line per pixel, and the 33 x 33 patch (139 KB) is single-buffered as
// FOUR planes by row and column parity (input pixel (2r + pr, 2x + pc) of the
// patch at plane (pr, pc), row r, column x):
//   EE (17 x 17): taps (0,0) (0,2) (2,0) (2,2)    EO (17 x 16): taps (0,1) (2,1)
//   OE (16 x 17): taps (1,0) (1,2)                OO (16 x 16): tap (1,1)
// so a stride-2 fragment (16 output columns -> input columns 2 ox + kx) is 16
// consecutive pixels of one plane row, and the chunk's 9 taps run plane by
// plane.  A plane is free once its taps are done: its next chunk is DMA'd
// while the other planes' taps run (each plane has 5-8 of the chunk's 9 taps
// to land), one barrier per plane (4 per chunk).  A DMA piece is 8 pixels x
// 128 B (1 KB): 8 whole lines, the lanes gathering their source pixels.
//
// Work split as variant 31 (halo256r.hip): 8 waves, each 32 output channels x
// all 256 pixels of the tile (BC = 256; BC = 128: 4 channel groups x 2 pixel
// halves), weights read from L2 straight into VGPRs one K-step ahead (compiler-
// tracked loads), 16-B chunk c of plane column x at c ^ key(x) (variant 43's
// key: conflict-free for every tap, tests/test_rwconv_layout.py).
// Per K-step and wave: 4 x 16-B weight loads, 32 ds_read_b128, 64 MFMA
// 16x16x32 (split-bf16: 96), 2 DMA pieces.
// X3: the split-bf16 parity mode (block.hip's layout, as variant 31: a 128-B
// chunk holds 32 logical channels, hi then lo; half 0 runs W_hi.X_hi and
// W_lo.X_hi on the hi fragment, half 1 W_hi.X_lo on the lo one).
#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"
#include "rwconv.hpp"

namespace sad {

namespace h44 {
constexpr int NW = 8, TC = 2;
// planes EE, EO, OE, OO, each stored 17 pixel slots wide (the odd-column
// planes' slot 16 unused), so every plane row is PITCH bytes and a fragment's
// row offset is a ds_read immediate whatever the tap: rows, valid columns, DMA
// pieces (8 slots each), LDS offset
constexpr int PW = 17, PITCH = PW * 128;
constexpr int NR[4] = {17, 17, 16, 16};
constexpr int NCV[4] = {17, 16, 17, 16};
constexpr int NP[4] = {37, 37, 34, 34};
constexpr int OFF[4] = {0, 37 * 1024, 74 * 1024, 108 * 1024};
constexpr int SMEM = 142 * 1024;  // 145,408 B
constexpr int BAD = 0x7FFFFFF0;
constexpr uint64_t KEY = 0x7929284ef1797ull;  // variant 43's 3-bit chunk key per plane column 0..16
static_assert(SMEM <= 160 * 1024, "LDS budget");
static_assert(16 * PITCH < 65536, "fragment row offsets are ds_read immediates");
// the chunk's tap sequence T = 0..8: plane, row / column offset inside it, tap index 3 ky + kx
constexpr int TPL[9] = {0, 0, 0, 0, 1, 1, 2, 2, 3};
constexpr int TRO[9] = {0, 0, 1, 1, 0, 1, 0, 0, 0};
constexpr int TCO[9] = {0, 1, 0, 1, 0, 0, 0, 1, 0};
constexpr int TAP[9] = {0, 2, 6, 8, 1, 7, 3, 5, 4};
// DMA pieces issued at tap T (up to 3): plane | next chunk << 2 | k << 3, -1 none
constexpr int SCH[9][3] = {
    {1 | 3 << 3, 2 | 1 << 3, -1}, {1 | 4 << 3, 2 | 2 << 3, -1}, {2 | 3 << 3, 3 | 0 << 3, -1},
    {2 | 4 << 3, 3 | 1 << 3, -1}, {0 | 4 | 0 << 3, 3 | 2 << 3, -1}, {0 | 4 | 1 << 3, 3 | 3 << 3, -1},
    {0 | 4 | 2 << 3, 1 | 4 | 0 << 3, 3 | 4 << 3}, {0 | 4 | 3 << 3, 1 | 4 | 1 << 3, -1},
    {0 | 4 | 4 << 3, 1 | 4 | 2 << 3, 2 | 4 | 0 << 3}};
// the tables above packed into 64-bit immediates, decoded by shifts of the
// uniform tap index (SALU) instead of loads from a constant table
constexpr uint64_t pack_sch(int e) {
  uint64_t v = 0;
  for (int T = 0; T < 9; ++T) v |= (uint64_t)(SCH[T][e] < 0 ? 0x7F : SCH[T][e]) << (7 * T);
  return v;
}
constexpr uint64_t SCHP0 = pack_sch(0), SCHP1 = pack_sch(1), SCHP2 = pack_sch(2);
constexpr uint64_t pack_step() {  // plane 2 bits | row offset 1 | column offset 1, per T
  uint64_t v = 0;
  for (int T = 0; T < 9; ++T) v |= (uint64_t)(TPL[T] | TRO[T] << 2 | TCO[T] << 3) << (4 * T);
  return v;
}
constexpr uint64_t STEPP = pack_step();
constexpr uint64_t pack_tap() {  // the next tap's index 3 ky + kx, per T < 8
  uint64_t v = 0;
  for (int T = 0; T < 8; ++T) v |= (uint64_t)TAP[T + 1] << (4 * T);
  return v;
}
constexpr uint64_t TAPP = pack_tap();
}  // namespace h44

__device__ __forceinline__ int h44_key(int x) { return (int)((h44::KEY >> (3 * x)) & 7); }

typedef unsigned int h44_v4 __attribute__((ext_vector_type(4)));
typedef __bf16 h44_bf2 __attribute__((ext_vector_type(2)));
typedef float h44_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t h44_pk(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((h44_f2){lo, hi}, h44_bf2));
}
__device__ __forceinline__ uint32_t h44_relu2(uint32_t x) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(x));
  return r;
}

template <int BC, bool X3>
__global__ __launch_bounds__(512, 1) void halo256rs2_kernel(BlockConvArgs a) {
  using namespace h44;
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
  const int ab = a.ablate;  // timing ablations (wrong results): 2 no patch DMA in the loop, 4 no weight loads, 8 no epilogue,
                            // 16 no per-plane wait + barrier

  const int cinb = a.Cin * 2;
  const int nch = cinb / 128;  // 64-channel (128-B) chunks, 9 taps each
  const __amdgpu_buffer_rsrc_t r0 =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.in0, (short)0, (int)a.in0_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rw =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.wt, (short)0, (int)a.wt_bytes, 0x00020000);
  const int ps = (int)a.in0_pstride * 2;
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- weights: lane (fr, fg) of fragment (i, h) = row cw + i*16 + fr, K bytes
  // kb + h*64 + fg*16 of the step (kb = (3 ky + kx) * cinb + chunk * 128: the
  // wave-uniform part, in the load's SGPR offset)
  const int wrow = a.wt_ld * 2;
  const int wlane = (cw + fr) * wrow + fg * 16;
  auto load_w = [&](int kb, h44_v4 (&wv)[TC][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        wv[i][h] = __builtin_amdgcn_raw_buffer_load_b128(rw, wlane + i * 16 * wrow + h * 64,
                                                         __builtin_amdgcn_readfirstlane(kb), 0);
  };

  // ---- DMA piece k of this wave (q = wave + 8k) of plane P (runtime, uniform)
  // of chunk c of tile t: plane slot u = 8q + lane / 8 (row u / 17, column u %
  // 17) <- input pixel (2 oy0 - 1 + 2 row + pr, 2 ox0 - 1 + 2 col + pc), chunk
  // position lane % 8 <- source chunk (lane % 8) ^ key(col).  Slots past the
  // plane's pixels (an odd-column plane's column 16, the last piece's tail) and
  // pixels above / left of the image (the first patch row / column of a tile on
  // the image's top / left edge) load zeros; the right and bottom edges are
  // never crossed (the input is exactly twice the output).
  // a tile's image and input origin (decoded once per chunk, not per piece)
  struct TileO {
    int b, iy0, ix0;  // image, input row / column of the patch's slot (0, 0) minus the parity
    bool ok;
  };
  auto tile_o = [&](int t) __attribute__((always_inline)) {
    const int tt = __builtin_amdgcn_readfirstlane(t);
    const int b = tt / tiles_img, rem = tt - b * tiles_img;
    const int ty = rem / tiles_x;
    return TileO{b, 32 * ty - 1, 32 * (rem - ty * tiles_x) - 1, tt < tp_end};
  };
  auto issue = [&](int P, const TileO& to, int c, int k) __attribute__((always_inline)) {
    const int q = wave + NW * k;
    const int np = P < 2 ? 37 : 34, nr = P < 2 ? 17 : 16, ncv = (P & 1) ? 16 : 17;
    if (q >= np || !to.ok) return;  // uniform
    int ln;  // opaque lane id: the per-piece slot math is not hoisted into registers
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int u = 8 * q + (ln >> 3);
    const int r = (u * 3856) >> 16;  // u / 17, exact for u < 2000
    const int x = u - PW * r;
    const int iy = to.iy0 + 2 * r + (P >> 1), ix = to.ix0 + 2 * x + (P & 1);
    const bool ok = r < nr && x < ncv && iy >= 0 && ix >= 0;
    const int off = ((to.b * a.H + iy) * a.W + ix) * ps + c * 128 + (((ln & 7) ^ h44_key(x)) << 4);
    const int poff = P == 0 ? OFF[0] : P == 1 ? OFF[1] : P == 2 ? OFF[2] : OFF[3];
    dma16_m0(r0, ok ? off : BAD, lds0 + poff + q * 1024);
  };

  // ---- prologue: the first chunk's planes as the previous chunk's taps 4-8
  // would have issued them (EE whole, EO pieces 0-2, OE piece 0); the loop
  // issues the rest while it runs
  {
    const TileO t0 = tile_o(tp_begin);
    for (int k = 0; k < 5; ++k) issue(0, t0, 0, k);
    for (int k = 0; k < 3; ++k) issue(1, t0, 0, k);
    issue(2, t0, 0, 0);
  }
  f32x4 biasv[TC];
#pragma unroll
  for (int i = 0; i < TC; ++i) biasv[i] = *(const f32x4*)(a.bias + cw + i * 16 + fg * 4);
  h44_v4 wcur[TC][2], wnxt[TC][2];
  load_w(0, wnxt);
  f32x4 acc[TC][TP];
#pragma unroll
  for (int i = 0; i < TC; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = biasv[i];
  auto take_w = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TC; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) wcur[i][h] = wnxt[i][h];
  };

  // the lane's fragment offsets for column offset co = 0 / 1 and K-half h:
  // plane column fr + co, chunk (4 h + fg) at its key position, plus this
  // wave's first row
  int lofs[2][2];
#pragma unroll
  for (int co = 0; co < 2; ++co)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      lofs[co][h] = r0w * PITCH + (fr + co) * 128 + (((4 * h + fg) ^ h44_key(fr + co)) << 4);

  // ---- one K-step (tap T of the sequence): the fragment of output row j, half
  // h is plane TPL[T]'s row TRO[T] + r0w + j, column TCO[T] + fr
  auto step = [&](int pbase, int co) __attribute__((always_inline)) {
    auto half = [&](auto hc) __attribute__((always_inline)) {
      constexpr int h = decltype(hc)::value;
      constexpr int NM = X3 && h == 0 ? 2 : 1;  // weight halves per fragment
      const char* pb = smem + pbase + (co ? lofs[1][h] : lofs[0][h]);
      uint4 bf[TP];
#pragma unroll
      for (int j = 0; j < TP; ++j) bf[j] = *(const uint4*)(pb + j * PITCH);
#pragma unroll
      for (int j = 0; j < TP; ++j)
#pragma unroll
        for (int m = 0; m < NM; ++m)
#pragma unroll
          for (int i = 0; i < TC; ++i)
            mfma_chunk<u16>(__builtin_bit_cast(uint4, wcur[i][X3 ? m : h]), bf[j], acc[i][j]);
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
    const int oy0 = (rem / tiles_x) * 16, ox0 = (rem - (rem / tiles_x) * tiles_x) * 16;
    u16* __restrict__ out = (u16*)a.out;
#pragma unroll
    for (int j = 0; j < TP; j += 2) {
      const int64_t px = (int64_t)(b * a.Ho + oy0 + r0w + j + (fg & 1)) * a.Wo + ox0 + fr;
#pragma unroll
      for (int i = 0; i < TC; ++i) {
        if constexpr (X3) {
          // ReLU in fp32, then hi = bf16(v), lo = bf16(v - hi) to the two
          // 32-channel halves of the wave's 128-B output chunk
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
            qh[e] = h44_pk(x0, x1);
            ql[e] = h44_pk(x0 - __uint_as_float(qh[e] << 16), x1 - __uint_as_float(qh[e] & 0xFFFF0000u));
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
        // 16-B stores: v_permlane16_swap pairs fragment rows j, j + 1 (variant 31)
        const int co = cw + i * 16 + (fg >> 1) * 8;
        uint32_t q[4] = {h44_pk(acc[i][j][0], acc[i][j][1]), h44_pk(acc[i][j][2], acc[i][j][3]),
                         h44_pk(acc[i][j + 1][0], acc[i][j + 1][1]), h44_pk(acc[i][j + 1][2], acc[i][j + 1][3])};
        if (a.relu)
#pragma unroll
          for (int e = 0; e < 4; ++e) q[e] = h44_relu2(q[e]);
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

  // ---- tiles -> chunks -> the 9 taps, plane by plane.  A barrier opens each
  // plane's taps (T = 0, 4, 6, 8): every wave has waited for its pieces of that
  // plane, and every wave is done with the plane before it, whose next chunk
  // may now be DMA'd.  Piece issue per tap (SCH; k = the wave's piece index,
  // cur = this chunk, nxt = the next one, of this tile or the next):
  //   T0 EO cur 3, OE cur 1   T1 EO cur 4, OE cur 2   T2 OE cur 3, OO cur 0
  //   T3 OE cur 4, OO cur 1   T4 EE nxt 0, OO cur 2   T5 EE nxt 1, OO cur 3
  //   T6 EE nxt 2, EO nxt 0, OO cur 4   T7 EE nxt 3, EO nxt 1   T8 EE nxt 4, EO nxt 2, OE nxt 0
  bool post_epi = false;
  for (int t = tp_begin; t < tp_end; ++t) {
    const TileO tcur = tile_o(t), tnext = tile_o(t + 1);
    for (int c = 0; c < nch; ++c) {
      const int ncn = c + 1 < nch ? c + 1 : 0;  // the next chunk
      const TileO& tn = c + 1 < nch ? tcur : tnext;
#pragma unroll 1
      for (int T = 0; T < 9; ++T) {
        if ((T == 0 || T == 4 || T == 6 || T == 8) && !(ab & 16)) {  // uniform
          if (T == 0 && post_epi)  // the previous tile's stores (youngest) may stay in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"((X3 ? 2 : 1) * TC * TP / 2) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          post_epi = false;
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");  // LDS changed behind the barrier
        }
        take_w();
        // the next step's weights (after the last tap: the next chunk's tap (0, 0))
        const int kbn = T < 8 ? (int)((TAPP >> (4 * T)) & 15) * cinb + c * 128 : ncn * 128;
        if (!(ab & 4)) load_w(kbn, wnxt);
        if (!(ab & 2)) {
#pragma unroll
          for (int e = 0; e < 3; ++e) {
            const uint64_t sp = e == 0 ? SCHP0 : e == 1 ? SCHP1 : SCHP2;
            const int d = (int)((sp >> (7 * T)) & 0x7F);
            if (d != 0x7F) {  // uniform
              const bool nx = (d >> 2) & 1;
              issue(d & 3, nx ? tn : tcur, nx ? ncn : c, d >> 3);
            }
          }
        }
        const int sd = (int)((STEPP >> (4 * T)) & 15), pl = sd & 3;
        int co;  // opaque: a known 0/1 index turns step()'s select into a scratch-array load
        asm volatile("s_lshr_b32 %0, %1, 3" : "=s"(co) : "s"(sd));
        step(1024 * (37 * pl - (pl == 3 ? 3 : 0)) + ((sd >> 2) & 1) * PITCH, co);
      }
    }
    if (!(ab & 8)) epilogue(t);
    post_epi = true;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BC, bool X3>
static int launch_halo256rs2_t(const BlockConvArgs& a, hipStream_t s) {
  using namespace h44;
  static bool attr = false;
  if (!attr) {
    SAD_CHECK_HIP(hipFuncSetAttribute((const void*)halo256rs2_kernel<BC, X3>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  const int n_tc = a.Cout / BC;
  const int64_t tiles_p = (int64_t)a.N * (a.Ho / 16) * (a.Wo / 16);
  int64_t g = std::min<int64_t>(tiles_p * n_tc, 256);
  g = std::max<int64_t>(n_tc, g / n_tc * n_tc);
  hipLaunchKernelGGL((halo256rs2_kernel<BC, X3>), dim3((unsigned)g), dim3(512), SMEM, s, a);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}

// (logical channel counts, as default_block_variant sees them)
bool halo256rs2_ok(const BlockConvArgs& a) {
  return a.KH == 3 && a.KW == 3 && a.stride == 2 && a.pad == 1 && !a.in1 && !a.res && !a.st_part && !a.pool_out &&
         a.Cin % 64 == 0 && a.Cout % 128 == 0 && a.Ho % 16 == 0 && a.Wo % 16 == 0 && a.H == 2 * a.Ho &&
         a.W == 2 * a.Wo;
}

// (a: the kernel's bf16 channel counts and strides, as launch_block_conv passes
// them; x3: the split-bf16 layout, Cin / strides / wt_ld already doubled, Cout
// and the bias logical)
int launch_halo256rs2(const BlockConvArgs& a, hipStream_t s, bool x3) {
  SAD_REQUIRE(a.KH == 3 && a.KW == 3 && a.stride == 2 && a.pad == 1 && !a.in1 && !a.res && !a.st_part &&
                  !a.pool_out,
              "variant 44: 3x3/s2/p1, no shortcut / residual / pool / statistics");
  SAD_REQUIRE((a.Cin * 2) % 128 == 0 && a.Cout % 128 == 0, "variant 44: whole 128-B chunks, Cout % 128");
  SAD_REQUIRE(a.Ho % 16 == 0 && a.Wo % 16 == 0 && a.H == 2 * a.Ho && a.W == 2 * a.Wo,
              "variant 44: 16 x 16 output tiles, input exactly twice the output");
  SAD_REQUIRE(a.wt_ld >= 9 * a.Cin && (a.wt_ld * 2) % 16 == 0, "variant 44: weight rows");
  SAD_REQUIRE(a.out_pstride % 8 == 0 && a.in0_pstride % 8 == 0, "variant 44: pixel strides");
  SAD_REQUIRE(a.out != nullptr, "null output");
  SAD_REQUIRE(a.M == (int64_t)a.N * a.Ho * a.Wo, "variant 44: M = N Ho Wo");
  SAD_REQUIRE(((int64_t)a.N * a.H * a.W - 1) * a.in0_pstride * 2 + 2 * a.Cin < (1ll << 31) - 65536,
              "variant 44: input passes the 32-bit buffer range");
  if (x3)
    return a.Cout % 256 == 0 ? launch_halo256rs2_t<256, true>(a, s) : launch_halo256rs2_t<128, true>(a, s);
  return a.Cout % 256 == 0 ? launch_halo256rs2_t<256, false>(a, s) : launch_halo256rs2_t<128, false>(a, s);
}

}  // namespace sad
