// l1block.hip -- fused layer1 BasicBlock (variant 40, bf16, gfx950).
//
// One timm BasicBlock of layer1 with its BatchNorms folded (the reference runs
// timm resnet18's forward_features, inference_runner.py:49-51):
//   mid = relu(conv3x3(x; W1) + b1)
//   out = relu(conv3x3(mid; W2) + b2 + x)          Cin = Cout = 64, stride 1
// as ONE kernel: the 64-channel intermediate never leaves LDS, and the
// identity shortcut is read from the input patch the first conv already holds.
// Per 16 x 16 output tile the HBM traffic is the 20 x 20 input patch (50 KB,
// L2/MALL-shared halo) + the 32 KB output, against 41 + 32 + 41 + 32 + 32 KB for
// the two unfused convs (variant 25).
//
// Work split: 4 waves, ONE per SIMD; wave w owns 32 output channels
// (cg = w & 1) of both convs and half the pixels (pg = w >> 1).  A wave's
// weights for both convs (2 channel tiles x 18 K-steps x 2 convs x 16 B per
// lane = 288 registers) are loaded ONCE into registers, so the tile loop reads
// only pixel fragments from LDS (one ds_read_b128 per two MFMAs: half the LDS
// array's rate) and needs no weight traffic, no weight ring and no per-tap
// barrier: two barriers per tile (intermediate published; intermediate and
// patch free again).
//
// conv1 computes the 18 x 18 intermediate (1-pixel halo for conv2) in
// fragments of 16 pixels: row-aligned ones (row y, columns 0-15) and
// "leftover" ones holding columns 16-17 (pixel (y0 + fr/2, 16 + (fr & 1))).
// A workgroup walks its tiles down column strips (ty fastest), so a tile that
// continues a strip takes intermediate rows 0, 1 and patch rows 2, 3 from the
// tile above (LDS-to-LDS copies of its rows 16, 17 and 18, 19) and computes
// rows 2-17 only: wave pg takes rows 2+8pg .. 9+8pg (8 aligned + 1 leftover
// fragment), 18 fragments per tile (16 without the halo), and its patch needs
// 40 DMA pieces instead of 50.  The first tile of a strip also computes rows
// 0, 1 (3 more fragments).  At 8 tiles per strip (128 x 128 maps) conv1 runs
// 1.15x its halo-free MFMA work (21 fragments: 1.31x).
//
// LDS (142 KB): 2 x input patch [20 x 20 pixels][128 B] (the next tile's patch
// is DMA'd during this tile's conv1, one piece per 5 units), the intermediate
// [18 rows][18 x 128 B + 16 B pad] and the biases.  Swizzles (16-B chunk c of a
// pixel):
//  * intermediate pixel (y, x): position c ^ key(x) -- a column key that is
//    conflict-free for row-aligned fragment reads at every tap column (conv2's
//    fragment address is a lane constant + an immediate row offset) and takes
//    each value twice over columns 0-15 (conv1's aligned 8-B stores: 2-way);
//    the 16-B row pad staggers the 8 rows of a leftover fragment's stores over
//    the bank space (2-way; 8-way without it);
//  * patch row (Y, X): position c ^ key(X) ^ 2 (Y & 3) -- the row term is
//    uniform over an aligned fragment (an XOR with a scalar keeps it
//    conflict-free) and spreads the leftover fragments' 4 rows per column
//    over 4 positions (conflict-free too; exhaustive check in
//    tests/test_l1block_layout.py).
// Zero padding: patch pixels outside the image are DMA'd as zeros (offset
// past num_records); intermediate pixels outside the image are written as 0
// (conv2 pads the block's intermediate, not relu(b1)).
#include "common.hpp"
#include "igemm.hpp"
#include "kernels.hpp"
#include "rwconv.hpp"

#include <stdio.h>

#include <utility>
#include <vector>

#ifndef SAD_STAMPS
#define SAD_STAMPS 0
#endif

namespace sad {

namespace l1b {
constexpr int NW = 4;                      // waves: one per SIMD
constexpr int PWD = 20, PR = PWD * PWD;    // input patch 20 x 20 (halo 2)
constexpr int IWD = 18;                       // intermediate 18 x 18 (halo 1)
constexpr int PATCH = PR * 128;            // 51,200 B
// intermediate row pitch: 18 pixels + 16 B, so consecutive rows start 16 B
// apart in the bank space (the leftover fragments' stores span 8 rows)
constexpr int PROW = PWD * 128, IROW = IWD * 128 + 16;
constexpr int OFF_I = 2 * PATCH;           // patches double-buffered
constexpr int OFF_B = OFF_I + IWD * IROW;  // b1 [64], b2 [64] fp32
constexpr int SMEM = OFF_B + 2 * 64 * 4;
constexpr int NDP = PR / 8;                // 50 DMA pieces of 8 pixel rows
constexpr int QP = (NDP + NW - 1) / NW;    // 13 per wave (waves 2, 3: 12)
constexpr int NA = 8;                      // row-aligned conv1 fragments per wave (rows 2 + 8 pg + k)
constexpr int NF = NA + 1;                 // + 1 leftover fragment (columns 16, 17 of those rows)
constexpr int QSKIP = 10;                  // pieces 0-9 = patch rows 0-3: a continuation tile needs no
                                           // rows 0, 1 and copies rows 2, 3 from the previous patch
constexpr int NS = 18;                     // K-steps per conv: 9 taps x 2 halves of 32 channels
constexpr int NU1 = NS * NF;               // conv1 (read, 2 MFMA) units per wave
constexpr int NU2 = NS * 8;                // conv2 units per wave
constexpr int DQ = 10;                     // fragment reads in flight ahead of their MFMAs (round 4: 6 -> 10)
constexpr int SA = 6;                      // conv1 K-steps run K-step-outer (the rest fragment-outer)
constexpr int NB1 = NS - SA;
constexpr int W2V = 8;                     // conv2 K-steps of channel tile 1 whose weights sit in VGPRs
constexpr int BAD = 0x7FFFFFF0;
// column key {0,0,1,1,2,3,4,4,5,5,6,7,2,3,6,7,0,0} (columns 18, 19: 0): every
// fragment read conflict-free (as variant 30's key), and over columns 0-15
// each value exactly twice, so conv1's aligned 8-B intermediate stores are
// 2-way (the ds_write_b64 minimum for 128-B pixels; variant 30's key: 4-way)
constexpr uint64_t KEY = 0xf9afad91a240ull;
static_assert(SMEM <= 160 * 1024, "LDS budget");
static_assert(NDP % 2 == 0, "pieces");
// conv1 unit u -> (K-step, fragment): phase A K-step-outer, phase B fragment-outer
constexpr int l1b_s1(int u) { return u < SA * NF ? u / NF : SA + (u - SA * NF) % NB1; }
constexpr int l1b_k1(int u) { return u < SA * NF ? u % NF : (u - SA * NF) / NB1; }
}  // namespace l1b

__device__ __forceinline__ int l1b_key(int x) { return (int)((l1b::KEY >> (3 * x)) & 7); }

__global__ __launch_bounds__(256, 1) void l1block_kernel(L1BlockArgs a) {
  using namespace l1b;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fg = lane >> 4;
  const int cg = wave & 1, pg = wave >> 1;
  // timing ablations (wrong results; tools/l1bench.py --ablate): 1 no next-tile
  // patch DMA, 2 no intermediate stores, 4 no output stores
  const int ab = a.ablate;
  const int cw = cg * 32;  // this wave's first channel (both convs)
  const int w = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_y = a.H / 16, tiles_img = (a.W / 16) * tiles_y;
  const int tiles_p = a.N * tiles_img;
  const int tp_begin = (int)((int64_t)w * tiles_p / gridDim.x), tp_end = (int)((int64_t)(w + 1) * tiles_p / gridDim.x);
  if (tp_begin >= tp_end) return;  // whole workgroup (uniform)

  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.x, (short)0, (int)a.x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ro =
      __builtin_amdgcn_make_buffer_rsrc((void*)a.out, (short)0, (int)a.x_bytes, 0x00020000);
  const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)smem;

  // ---- patch piece k of this wave (q = wave + 4k: rows 8q .. 8q+7): the
  // lane's patch pixel (Y, X) and its source offset from the tile origin are
  // tile-independent (computed once)
  int DREL[QP], DYX[QP];
#pragma unroll
  for (int k = 0; k < QP; ++k) {
    const int r = 8 * (wave + NW * k) + (lane >> 3);
    const int Y = (r * 205) >> 12, X = r - 20 * Y;  // r / 20 exactly for r < 400
    const int c = (lane & 7) ^ l1b_key(X) ^ ((Y & 3) << 1);
    DREL[k] = ((Y - 2) * a.W + (X - 2)) * 128 + (c << 4);
    DYX[k] = Y | (X << 16);
  }
  // tile t's origin: image byte offset, (oy0, ox0), interior flag (uniform)
  struct TileO {
    int base, oy0, ox0;
  };
  // tiles run down column strips (ty fastest), so a tile's top halo is the
  // previous tile's bottom rows
  auto tile_o = [&](int t) __attribute__((always_inline)) {
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int tx = rem / tiles_y;
    TileO o;
    o.oy0 = (rem - tx * tiles_y) * 16;
    o.ox0 = tx * 16;
    o.base = ((b * a.H + o.oy0) * a.W + o.ox0) * 128;
    return o;
  };
  // (branch-free: the bounds test is VALU in the MFMA shadow; only the piece
  // count per wave is a uniform branch)
  auto issue_piece = [&](int k, const TileO& o, int buf, bool cont) __attribute__((always_inline)) {
    if (wave + NW * k >= NDP || (cont && wave + NW * k < QSKIP)) return;  // uniform
    const int Y = DYX[k] & 0xFFFF, X = DYX[k] >> 16;
    const bool ok = (unsigned)(o.oy0 - 2 + Y) < (unsigned)a.H && (unsigned)(o.ox0 - 2 + X) < (unsigned)a.W;
    dma16_m0(rx, ok ? o.base + DREL[k] : BAD, lds0 + buf * PATCH + (wave + NW * k) * 1024);
  };

  // ---- weights of both convs into registers: lane (fr, fg) of K-step s =
  // (tap, h) holds channels (fg + 4h) * 8 .. +7 of tap `tap` for output
  // channel cw + 16 i + fr
  l1b_v4 w1r[2][NS];
  l1b_v4 w2r[2][NS];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int tap = s >> 1, h = s & 1;
      w1r[i][s] = *(const l1b_v4*)(a.w1 + (size_t)(cw + 16 * i + fr) * a.w1_ld + tap * 64 + (fg + 4 * h) * 8);
      w2r[i][s] = *(const l1b_v4*)(a.w2 + (size_t)(cw + 16 * i + fr) * a.w2_ld + tap * 64 + (fg + 4 * h) * 8);
    }
  if (tid < 32) {
    const float* src = tid < 16 ? a.b1 + 4 * tid : a.b2 + 4 * (tid - 16);
    *(float4*)(smem + OFF_B + 16 * tid) = *(const float4*)src;
  }
#pragma unroll
  for (int k = 0; k < QP; ++k) issue_piece(k, tile_o(tp_begin), 0, false);

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");


  // diagnostic build (-DSAD_STAMPS=1): s_memtime of waves 0 and 2 of
  // workgroup 0 per tile -- 0 tile start, 1 conv1 issued, 2 after the
  // intermediate barrier, 3 conv2 issued, 4 after the tile barrier
  const bool stamp_on = SAD_STAMPS && a.stamps && blockIdx.x == 0 && (wave == 0 || wave == 2);
  auto stamp = [&](int g, int slot) __attribute__((always_inline)) {
    if constexpr (SAD_STAMPS) {
      if (stamp_on && g < 1024) {
        __builtin_amdgcn_sched_barrier(0);
        uint64_t t_;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
        __builtin_amdgcn_sched_barrier(0);
        if (lane == 0) a.stamps[(size_t)(wave >> 1) * 8192 + (size_t)g * 8 + slot] = t_;
      }
    }
  };
  int pb = 0;
  for (int t = tp_begin; t < tp_end; ++t) {
    stamp(t - tp_begin, 0);
    const bool has_next = t + 1 < tp_end;
    // the next tile's patch (after the last tile: this tile's again, into the
    // free buffer, which nothing reads -- no branch around the DMA)
    const TileO onext = tile_o(has_next ? t + 1 : t);
    const int b = t / tiles_img, rem = t - b * tiles_img;
    const int tx = rem / tiles_y, ty = rem - tx * tiles_y;
    const int oy0 = ty * 16, ox0 = tx * 16;
    // continuation tile (uniform): the previous tile is the one above it, so
    // intermediate rows 0, 1 and patch rows 2, 3 are copies of its rows 16, 17
    // and 18, 19 (LDS to LDS), and conv1 computes rows 2-17 only: 18 fragments
    // instead of 21, 40 patch pieces instead of 50
    const bool cont = t > tp_begin && ty > 0;
    const bool next_cont = has_next && onext.oy0 > 0;
    const int pbo = pb * PATCH;
    const int pboa = pbo + (2 + 8 * pg) * PROW;  // aligned fragments: rows 2 + 8pg + k
    // Lane constants, derived per tile from an opaque copy of the lane id:
    // the fragment addresses are tile-invariant, and hoisted out of the tile
    // loop they would take registers next to the 288 of resident weights.
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int frt = ln & 15, fgt = ln >> 4, et = ln & 1;
    // aligned fragment, patch column frt + kx: pixel row + chunk position of channel group fgt
    int LAt[3], KXt[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) {
      LAt[kx] = (frt + kx) * 128 + ((fgt ^ l1b_key(frt + kx)) << 4);
      KXt[kx] = fgt ^ l1b_key(16 + et + kx);
    }
    // the leftover fragment: pixel (LYt, 16 + et), rows 2 + 8pg .. 9 + 8pg
    const int LYt = 2 + 8 * pg + (frt >> 1);
    // per-tile read bases: aligned (+ the patch buffer and the wave's row
    // block), leftover (+ buffer) and the leftover row terms per tap row
    int LAp[3], LYG[3];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx) LAp[kx] = LAt[kx] + pboa;
    const int LRb = (LYt * PWD + 16 + et) * 128 + pbo;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) LYG[ky] = ((LYt + ky) & 3) << 1;

    // ---------------- conv1: 18 x 18 intermediate ----------------
    // Unit = one fragment read + its two MFMAs (channel tiles i = 0, 1).
    // Phase A (K-steps s < SA) runs K-step-outer over the 11 fragments and
    // carries the next tile's patch DMA; phase B runs fragment-outer over the
    // remaining K-steps, so fragments complete one by one and fragment k-1's
    // epilogue (ReLU, bf16, 0 outside the image, intermediate store) is issued
    // among fragment k's MFMAs instead of after all of them (one wave per
    // SIMD: VALU work only hides in the MFMA shadow).  The bias is the first
    // MFMA's C operand.
    auto rd1 = [&](auto uc) __attribute__((always_inline)) -> uint4 {
      constexpr int u = decltype(uc)::value;
      constexpr int s = l1b_s1(u), k = l1b_k1(u);
      constexpr int tap = s >> 1, h = s & 1, ky = tap / 3, kx = tap % 3;
      if constexpr (k < NA) {
        // patch row Y = 2 + 8pg + k + ky: Y & 3 is a constant
        constexpr int sg = (((2 + k + ky) & 3) << 5) ^ (h << 6);  // 2 (Y & 3) and the K-half, as chunk bits
        // (pboa is a multiple of 128, so it commutes with the XOR on bits 4-6)
        return *(const uint4*)(smem + (LAp[kx] ^ sg) + (k + ky) * PROW);
      } else {
        const int pos = KXt[kx] ^ LYG[ky] ^ (h << 2);
        return *(const uint4*)(smem + (LRb + (pos << 4)) + (ky * PWD + kx) * 128);
      }
    };
    f32x4 b1v[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) b1v[i] = *(const f32x4*)(smem + OFF_B + (cw + 16 * i + fgt * 4) * 4);
    // column masks of this tile's intermediate pixels (0: outside the image):
    // aligned fragments x = frt, leftovers x = 16 + et
    const uint32_t cma = (unsigned)(ox0 - 1 + frt) < (unsigned)a.W ? 0xFFFFFFFFu : 0u;
    const uint32_t cml = (unsigned)(ox0 + 15 + et) < (unsigned)a.W ? 0xFFFFFFFFu : 0u;
    f32x4 acc[2][NF];
    // epilogue of fragment k in 4 parts (channel tile i = part / 2; first or
    // second half of the 4 values), so it can be spread between MFMAs
    uint32_t e1_inm = 0, e1_qx = 0;
    int e1_addr = 0, e1_addr1 = 0;
    auto epi1 = [&](auto kc, auto pc) __attribute__((always_inline)) {
      constexpr int k = decltype(kc)::value, part = decltype(pc)::value, i = part >> 1;
      if constexpr (part == 0) {
        int y, x;
        if constexpr (k < NA) {
          y = 2 + 8 * pg + k;
          x = frt;
          e1_inm = (unsigned)(oy0 - 1 + y) < (unsigned)a.H ? cma : 0u;  // row test uniform
        } else {
          y = LYt;
          x = 16 + et;
          e1_inm = (unsigned)(oy0 - 1 + y) < (unsigned)a.H ? cml : 0u;
        }
        // channel tile 1 is chunk + 2: position (c + 2) ^ key = (c ^ key) ^ 2 (c
        // even); the XOR stays inside the pixel (the padded row pitch is not a
        // multiple of 64 B)
        const int pix = OFF_I + y * IROW + x * 128;
        const int pos = (((cw >> 3) + (fgt >> 1)) ^ l1b_key(x)) * 16 + (fgt & 1) * 8;
        e1_addr = pix + pos;
        e1_addr1 = pix + (pos ^ 32);
      }
      if constexpr ((part & 1) == 0) {
        e1_qx = l1b_relu2(l1b_pk(acc[i][k][0], acc[i][k][1])) & e1_inm;
      } else {
        uint2 q;
        q.x = e1_qx;
        q.y = l1b_relu2(l1b_pk(acc[i][k][2], acc[i][k][3])) & e1_inm;
        if (!(ab & 2)) *(uint2*)(smem + (i ? e1_addr1 : e1_addr)) = q;
      }
    };
    if (cont) {
      // intermediate rows 16, 17 of the tile above -> rows 0, 1: each pg = 1
      // wave copies its own channel half (those waves write rows 16, 17 later
      // in this conv1, and one wave's LDS operations complete in order)
      if (pg == 1) {
        // 144 16-B chunks (2 rows x 18 pixels x 4 chunks), 3 per lane
        auto off = [&](int r) __attribute__((always_inline)) {
          const int i = min(ln + 64 * r, 143), row = i >= 72, rem = i - 72 * row, x = rem >> 2;
          return row * IROW + x * 128 + ((((cw >> 3) + (rem & 3)) ^ l1b_key(x)) << 4);
        };
        const int o0 = off(0), o1 = off(1), o2 = off(2);
        const uint4 v0 = *(const uint4*)(smem + OFF_I + 16 * IROW + o0);
        const uint4 v1 = *(const uint4*)(smem + OFF_I + 16 * IROW + o1);
        const uint4 v2 = *(const uint4*)(smem + OFF_I + 16 * IROW + o2);
        *(uint4*)(smem + OFF_I + o0) = v0;
        *(uint4*)(smem + OFF_I + o1) = v1;
        *(uint4*)(smem + OFF_I + o2) = v2;
      }
    } else {
      // first tile of a strip (or of this workgroup's range): intermediate
      // rows 0, 1 as extra fragments -- wave pg computes row pg (columns
      // 0-15), the pg = 0 waves also columns 16, 17 of both rows (lane frt:
      // pixel ((frt >> 1) & 1, 16 + et); lanes 4-15 duplicate lanes 0-3)
      auto prefix = [&](bool left) __attribute__((always_inline)) {
        const int y = left ? (frt >> 1) & 1 : pg;
        f32x4 pa[2];
        auto rdp = [&](int st) __attribute__((always_inline)) {
          const int tap = st >> 1, h = st & 1, ky = tap / 3, kx = tap % 3;
          const int Y = y + ky;
          const int ad = left ? pbo + (Y * PWD + 16 + et + kx) * 128 +
                                    ((KXt[kx] ^ ((Y & 3) << 1) ^ (h << 2)) << 4)
                              : pbo + (LAt[kx] ^ (((Y & 3) << 5) ^ (h << 6))) + Y * PROW;
          return *(const uint4*)(smem + ad);
        };
        // 4 fragment reads in flight (a read per 2 dependent MFMAs would
        // otherwise wait out the LDS latency every K-step)
        uint4 pq[4];
#pragma unroll
        for (int st = 0; st < 4; ++st) pq[st] = rdp(st);
#pragma unroll
        for (int st = 0; st < NS; ++st) {
          const uint4 bf = pq[st & 3];
          if (st + 4 < NS) pq[st & 3] = rdp(st + 4);
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            if (st == 0)
              l1b_mfma_ac(pa[i], w1r[i][st], bf, b1v[i]);
            else
              l1b_mfma_a(pa[i], w1r[i][st], bf);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 11" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        const int x = left ? 16 + et : frt;
        const uint32_t inm = (unsigned)(oy0 - 1 + y) < (unsigned)a.H ? (left ? cml : cma) : 0u;
        const int pix = OFF_I + y * IROW + x * 128;
        const int pos = (((cw >> 3) + (fgt >> 1)) ^ l1b_key(x)) * 16 + (fgt & 1) * 8;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          uint2 q;
          q.x = l1b_relu2(l1b_pk(pa[i][0], pa[i][1])) & inm;
          q.y = l1b_relu2(l1b_pk(pa[i][2], pa[i][3])) & inm;
          *(uint2*)(smem + pix + (i ? pos ^ 32 : pos)) = q;
        }
      };
      prefix(false);
      if (pg == 0) prefix(true);
    }
    uint4 bq[DQ];
    l1b_for<DQ>([&](auto uc) __attribute__((always_inline)) { bq[decltype(uc)::value] = rd1(uc); });
    l1b_for<NU1>([&](auto uc) __attribute__((always_inline)) {
      constexpr int u = decltype(uc)::value;
      constexpr int s = l1b_s1(u), k = l1b_k1(u);
      const uint4 bf = bq[u % DQ];
      if constexpr (u + DQ < NU1) bq[u % DQ] = rd1(std::integral_constant<int, u + DQ>{});
      if constexpr (u % 5 == 0 && u / 5 < QP)
        if (!(ab & 1)) issue_piece(u / 5, onext, pb ^ 1, next_cont);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        if constexpr (s == 0)
          l1b_mfma_ac(acc[i][k], w1r[i][s], bf, b1v[i]);
        else
          l1b_mfma_a(acc[i][k], w1r[i][s], bf);
      }
      // fragment k-1 is complete: its epilogue parts go after units 2, 4, 6, 8
      // of fragment k (>= 6 MFMAs after its last one: the XDL -> VALU read
      // distance; the asm MFMAs keep compiler code from moving across them)
      if constexpr (u >= SA * NF && k >= 1) {
        constexpr int q = (u - SA * NF) % NB1;
        if constexpr (q >= 2 && q <= 8 && q % 2 == 0) {
          // pinned between the MFMAs: the asm MFMAs' results have no hazard
          // tracking, so the scheduler must not hoist these reads of acc
          // toward the MFMA that wrote it
          __builtin_amdgcn_sched_barrier(0);
          epi1(std::integral_constant<int, k - 1>{}, std::integral_constant<int, q / 2 - 1>{});
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    });
    stamp(t - tp_begin, 1);
    // the last fragment: asm MFMA results read by compiler code need 12 wait
    // states (8-pass XDL), which hipcc does not pad for asm
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 11" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    l1b_for<4>([&](auto pc) __attribute__((always_inline)) { epi1(std::integral_constant<int, NF - 1>{}, pc); });

    // conv2's accumulators start at b2 + x (the identity): residual of output
    // row 8pg + jj, channels cw + 16 i + 4 fg2, from the patch centre
    int ln2;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln2) : "v"(lane));
    const int fr2 = ln2 & 15, fg2 = ln2 >> 4;
    int LRr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      LRr[i] = (fr2 + 2) * 128 + ((((cw >> 3) + 2 * i + (fg2 >> 1)) ^ l1b_key(fr2 + 2)) << 4) + (fg2 & 1) * 8;
    f32x4 acc2[2][8];
    // in two halves: the bias and residual reads are issued a few units before
    // the adds that consume them, so the wait for them is not a wait for the
    // youngest LDS read (lgkmcnt(0) would drain the fragment reads in flight)
    f32x4 i2b[2];
    uint2 i2r[2];
    auto init2_rd = [&](auto jc, auto ic) __attribute__((always_inline)) {
      constexpr int jj = decltype(jc)::value, i = decltype(ic)::value;
      i2b[i] = *(const f32x4*)(smem + OFF_B + 256 + (cw + 16 * i + fg2 * 4) * 4);
      i2r[i] = *(const uint2*)(smem + ((LRr[i] ^ (((jj + 2) & 3) << 5)) + pbo + pg * 8 * PROW) + (jj + 2) * PROW);
    };
    auto init2_add = [&](auto jc, auto ic) __attribute__((always_inline)) {
      constexpr int jj = decltype(jc)::value, i = decltype(ic)::value;
      acc2[i][jj][0] = i2b[i][0] + __uint_as_float(i2r[i].x << 16);
      acc2[i][jj][1] = i2b[i][1] + __uint_as_float(i2r[i].x & 0xFFFF0000u);
      acc2[i][jj][2] = i2b[i][2] + __uint_as_float(i2r[i].y << 16);
      acc2[i][jj][3] = i2b[i][3] + __uint_as_float(i2r[i].y & 0xFFFF0000u);
    };
    auto init2 = [&](auto jc, auto ic) __attribute__((always_inline)) {
      init2_rd(jc, ic);
      init2_add(jc, ic);
    };
    init2(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    init2(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    stamp(t - tp_begin, 2);
    // ---------------- conv2 + identity ----------------
    // Fragment-outer throughout: fragment jj-1's epilogue (ReLU, bf16, 8-B
    // stores) and fragment jj+1's accumulator init go among fragment jj's MFMAs.
    // conv2: intermediate fragments of output rows 8pg + jj
    int I2[3][2];
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        I2[kx][h] = OFF_I + pg * 8 * IROW + (((fr2 + kx) * 128 + ((fg2 ^ l1b_key(fr2 + kx)) << 4)) ^ (h << 6));
    auto rd2 = [&](auto uc) __attribute__((always_inline)) -> uint4 {
      constexpr int u = decltype(uc)::value;
      constexpr int s = u % NS, jj = u / NS;
      constexpr int tap = s >> 1, h = s & 1, ky = tap / 3, kx = tap % 3;
      return *(const uint4*)(smem + I2[kx][h] + (jj + ky) * IROW);
    };
    const int obase = ((b * a.H + oy0 + 8 * pg) * a.W + ox0) * 128;  // uniform
    // epilogue of fragment jj in 4 parts, as conv1's
    uint32_t e2_qx = 0;
    auto epi2 = [&](auto jc, auto pc) __attribute__((always_inline)) {
      constexpr int jj = decltype(jc)::value, part = decltype(pc)::value, i = part >> 1;
      if constexpr ((part & 1) == 0) {
        e2_qx = l1b_relu2(l1b_pk(acc2[i][jj][0], acc2[i][jj][1]));
      } else {
        uint2 q;
        q.x = e2_qx;
        q.y = l1b_relu2(l1b_pk(acc2[i][jj][2], acc2[i][jj][3]));
        if (!(ab & 4))
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(l1b_v2, q), ro,
                                                (jj * a.W + fr2) * 128 + (cw + 16 * i + 4 * fg2) * 2, obase, 0);
      }
    };
    // the next tile continues this strip: its patch rows 2, 3 are this patch's
    // rows 18, 19 (same swizzle: Y & 3 and X agree), copied now -- buffer
    // pb ^ 1 is free and its DMA pieces cover rows 4-19 only; 320 16-B chunks
    const int pci1 = min(tid + 256, 319);
    uint4 pcv0 = {0, 0, 0, 0}, pcv1 = {0, 0, 0, 0};
    if (next_cont) {
      pcv0 = *(const uint4*)(smem + pbo + 360 * 128 + tid * 16);
      pcv1 = *(const uint4*)(smem + pbo + 360 * 128 + pci1 * 16);
    }
    l1b_for<DQ>([&](auto uc) __attribute__((always_inline)) { bq[decltype(uc)::value] = rd2(uc); });
    l1b_for<NU2>([&](auto uc) __attribute__((always_inline)) {
      constexpr int u = decltype(uc)::value;
      constexpr int s = u % NS, jj = u / NS;
      const uint4 bf = bq[u % DQ];
      if constexpr (u + DQ < NU2) bq[u % DQ] = rd2(std::integral_constant<int, u + DQ>{});
      if constexpr (u == 3) {
        if (next_cont) {
          *(uint4*)(smem + (pb ^ 1) * PATCH + 40 * 128 + tid * 16) = pcv0;
          *(uint4*)(smem + (pb ^ 1) * PATCH + 40 * 128 + pci1 * 16) = pcv1;
        }
      }
      l1b_for<2>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        // the last K-steps' weights of channel tile 1 sit in VGPRs
        if constexpr (i == 1 && s >= NS - W2V)
          l1b_mfma_v(acc2[i][jj], w2r[i][s], bf);
        else
          l1b_mfma_a(acc2[i][jj], w2r[i][s], bf);
      });
      // fragment jj-1's epilogue parts after units 2, 4, 6, 8 of fragment jj,
      // fragment jj+1's accumulator init: its reads after units 5 and 7, the
      // adds after units 11 and 13 (pinned between the MFMAs, as conv1's
      // epilogue parts)
      if constexpr (jj >= 1 && s >= 2 && s <= 8 && s % 2 == 0) {
        __builtin_amdgcn_sched_barrier(0);
        epi2(std::integral_constant<int, jj - 1>{}, std::integral_constant<int, s / 2 - 1>{});
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (jj + 1 < 8 && (s == 5 || s == 7)) {
        __builtin_amdgcn_sched_barrier(0);
        init2_rd(std::integral_constant<int, jj + 1>{}, std::integral_constant<int, (s - 5) / 2>{});
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (jj + 1 < 8 && (s == 11 || s == 13)) {
        __builtin_amdgcn_sched_barrier(0);
        init2_add(std::integral_constant<int, jj + 1>{}, std::integral_constant<int, (s - 11) / 2>{});
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    stamp(t - tp_begin, 3);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 11" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    l1b_for<4>([&](auto pc) __attribute__((always_inline)) { epi2(std::integral_constant<int, 7>{}, pc); });

    // this wave's patch pieces of the next tile (issued in conv1) have landed
    // -- the 16 output stores, younger, may stay in flight; then the
    // intermediate and patch pb are free and patch pb ^ 1 is published
    asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    stamp(t - tp_begin, 4);
    pb ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int launch_l1block(const L1BlockArgs& a_in, hipStream_t s) {
  using namespace l1b;
  SAD_REQUIRE(a_in.x && a_in.out && a_in.w1 && a_in.w2 && a_in.b1 && a_in.b2, "null tensor");
  SAD_REQUIRE(a_in.N >= 0 && a_in.H % 16 == 0 && a_in.W % 16 == 0 && a_in.H > 0 && a_in.W > 0,
              "fused layer1 block: H, W multiples of 16");
  SAD_REQUIRE(a_in.w1_ld >= 576 && a_in.w2_ld >= 576 && a_in.w1_ld % 8 == 0 && a_in.w2_ld % 8 == 0,
              "fused layer1 block: weight rows of >= 576 bf16, 16-B aligned");
  if (a_in.N == 0) return SAD_OK;
  static bool attr = false;
  if (!attr) {
    SAD_CHECK_HIP(hipFuncSetAttribute((const void*)l1block_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, SMEM));
    attr = true;
  }
  // the patch DMA addresses the input through 32-bit buffer offsets: split a
  // batch past that range into image ranges (every image is independent)
  const int64_t img = (int64_t)a_in.H * a_in.W * 128;
  const int64_t per = std::max<int64_t>(1, ((1ll << 31) - 65536) / img);
  for (int64_t n0 = 0; n0 < a_in.N; n0 += per) {
    L1BlockArgs a = a_in;
    a.N = (int)std::min<int64_t>(per, a_in.N - n0);
    a.x = a_in.x + n0 * img / 2;
    a.out = a_in.out + n0 * img / 2;
    a.x_bytes = a.N * img;
    const int64_t tiles = (int64_t)a.N * (a.H / 16) * (a.W / 16);
    const int64_t g = std::min<int64_t>(tiles, 256);
#if SAD_STAMPS
    static uint64_t* sbuf = nullptr;
    if (!sbuf) SAD_CHECK_HIP(hipMalloc(&sbuf, 2 * 8192 * 8));
    SAD_CHECK_HIP(hipMemsetAsync(sbuf, 0, 2 * 8192 * 8, s));
    a.stamps = sbuf;
#endif
    hipLaunchKernelGGL(l1block_kernel, dim3((unsigned)g), dim3(256), SMEM, s, a);
    SAD_CHECK_HIP(hipGetLastError());
#if SAD_STAMPS
    {  // per-tile phase averages of waves 0 and 2 of workgroup 0 (skipping the first tile)
      std::vector<uint64_t> h(2 * 8192);
      SAD_CHECK_HIP(hipStreamSynchronize(s));
      SAD_CHECK_HIP(hipMemcpy(h.data(), sbuf, h.size() * 8, hipMemcpyDeviceToHost));
      for (int wv = 0; wv < 2; ++wv) {
        double ph[5] = {0, 0, 0, 0, 0};
        int n = 0;
        for (int t = 1; t + 1 < 1024; ++t) {
          const uint64_t* c = &h[(size_t)wv * 8192 + (size_t)t * 8];
          const uint64_t nxt = h[(size_t)wv * 8192 + (size_t)(t + 1) * 8];
          if (!c[0] || !c[4] || !nxt) break;
          for (int k = 0; k < 4; ++k) ph[k] += (double)(c[k + 1] - c[k]);
          ph[4] += (double)(nxt - c[4]);
          ++n;
        }
        if (n)
          fprintf(stderr, "l1block stamps N=%d wave %d: %d tiles, cycles conv1 %.0f | epi1+B1 %.0f | conv2 %.0f | "
                  "epi2+B2 %.0f | loop %.0f | total %.0f\n", a.N, 2 * wv, n, ph[0] / n, ph[1] / n, ph[2] / n,
                  ph[3] / n, ph[4] / n, (ph[0] + ph[1] + ph[2] + ph[3] + ph[4]) / n);
      }
    }
#endif
  }
  return SAD_OK;
}

}  // namespace sad
