// kernels.hpp -- launch interfaces shared by the kernel translation units.
#pragma once
#include <vector>

#include "common.hpp"

namespace sad {

// Diagnostic builds (-DSAD_STAMPS=1): wave 0 of every workgroup records
// (s_memtime, s_memrealtime) at kernel entry (slot 0) and exit (slot 1) in
// a.stamps[SAD_CLOCK_BASE + 4 * blockIdx.x + 2 * slot ..]: the in-kernel clock
// (MI355X_MICROARCH.md 'DVFS give-back' item 6) and the launch's ramp and tail.
#define SAD_CLOCK_BASE 8192
#define SAD_CLOCK_WGS 4096
#define SAD_CLOCK_STAMP(slot)                                                                      \
  do {                                                                                             \
    if constexpr (SAD_STAMPS) {                                                                    \
      if (a.stamps && wave == 0 && blockIdx.x < SAD_CLOCK_WGS) {                                   \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();                                          \
        const uint64_t r_ = __builtin_amdgcn_s_memrealtime();                                      \
        if (lane == 0) {                                                                           \
          a.stamps[SAD_CLOCK_BASE + 4 * blockIdx.x + 2 * (slot)] = t_;                             \
          a.stamps[SAD_CLOCK_BASE + 4 * blockIdx.x + 2 * (slot) + 1] = r_;                         \
        }                                                                                          \
      }                                                                                            \
    }                                                                                              \
  } while (0)

struct ConvArgs {
  const void* in;        // NHWC [N, H, W, *] with pixel stride in_pstride (elements)
  int64_t in_pstride;
  int N, H, W, Cin;
  const void* wt;        // [Cout][KH][KW][Cin], BN folded
  const float* bias;     // [Cout], BN folded
  const void* res;       // optional residual, [M, *] pixel stride res_pstride
  int64_t res_pstride;
  void* out;             // [M, *] pixel stride out_pstride
  int64_t out_pstride;
  int Ho, Wo, Cout, KH, KW, stride, pad;
  int relu;
  int64_t M;             // N * Ho * Wo
  int64_t in_bytes;      // set by launch_conv: addressable input span (buffer range)
  int64_t wt_bytes;      // set by launch_conv
  // optional grouped launch (grid.y = groups): group g reads in + g*in_gstride,
  // wt + g*wt_gstride, bias + g*bias_gstride and writes out + g*out_gstride
  // (elements) -- e.g. the N heads' Linear(512, 256) GEMMs as one launch
  int groups;
  int64_t in_gstride, wt_gstride, bias_gstride, out_gstride;
};

// One GEMM = 3x3 (or 1x1) conv of source 0 + optional 1x1 shortcut of source 1
// (identity or downsample), BN folded, K axis concatenated (block.hip).
struct BlockConvArgs {
  const void* in0;       // NHWC [N, H, W, *], pixel stride in0_pstride (elements)
  int64_t in0_pstride;
  int N, H, W, Cin, KH, KW, stride, pad;
  const void* in1;       // optional shortcut source NHWC [N, H1, W1, *]; pixel (oy*ss1, ox*ss1)
  int64_t in1_pstride;
  int H1, W1, Cin1, ss1;
  const void* wt;        // [Cout][wt_ld] (dtype): KH*KW*Cin conv taps, then Cin1 shortcut columns
  int wt_ld;             // elements per weight row; 0 = KH*KW*Cin + Cin1
  const float* bias;     // [Cout]
  const void* res;       // optional residual added before the activation, NHWC [M, *] (halo kernel only)
  int64_t res_pstride;
  void* out;             // [M, *] pixel stride out_pstride
  int64_t out_pstride;
  int Ho, Wo, Cout, relu;
  int64_t M;
  int64_t in0_bytes, in1_bytes, wt_bytes, res_bytes;  // set by launch_block_conv
  int64_t out_bytes;     // (variant 41 sets it)
  int ablate;            // timing ablations (wrong results): 1 no DMA in loop, 2 no vmcnt wait, 4 no barrier,
                         // 8 no epilogue, 16 no weight DMA, 32 no patch DMA (halo)
  float* pool_out;       // optional fused global average pool, fp32 [N, Cout] (the variant's pixel tile
                         // must be one image: block_conv_can_pool); out may then be null
  uint64_t* stamps;      // diagnostic builds only (-DSAD_STAMPS): s_memtime stamps per K-step
  float* st_part;        // training (bf16): fused BN statistics, fp32 [rows][2][Cout] sums of the
                         // conv output and its square per workgroup row (variants 13, 15, 20, 25)
  int* st_rows;          // host out: rows written to st_part by the launch
  int x4;                // split-bf16: also the fourth product W_lo.X_lo (the deep Bottleneck plans,
                         // resnet.hip); runs on the implicit-GEMM variants
};

// Fused layer1 BasicBlock (l1block.hip, variant 40): bf16 NHWC, 64 channels,
// pixel stride 64; out = relu(conv(relu(conv(x; w1) + b1); w2) + b2 + x)
struct L1BlockArgs {
  const u16* x;          // [N, H, W, 64]
  u16* out;              // [N, H, W, 64] (must not alias x)
  int N, H, W;
  const u16* w1;         // [64][w1_ld]: k = tap * 64 + ci (BN folded)
  int w1_ld;
  const float* b1;       // [64]
  const u16* w2;
  int w2_ld;
  const float* b2;
  int64_t x_bytes;       // set by launch_l1block
  int ablate;            // timing ablations (wrong results): 1 no patch DMA, 2 no intermediate stores, 4 no output stores
  uint64_t* stamps;      // diagnostic builds only (-DSAD_STAMPS): s_memtime per tile phase
};
int launch_l1block(const L1BlockArgs& a, hipStream_t s);
int64_t block_conv_kernel_launches();  // kernels dispatched by launch_block_conv on this host thread so far (image-range launches each count)
bool l1_fused();  // SAD_L1_FUSED (default 1): bf16 layer1 BasicBlocks on the fused kernel (ResNet-18 and the generic plan)

struct StemArgs {
  const float* map;      // [B, mh, mw] standardised maps (bilinearly resized in-kernel), or
  const float* img;      // [B, 512, 512] fp32 image (one channel of the reference's 3 identical
                         // channels) when non-null
  int mh, mw;
  const void* w;         // [64 co][64 k] folded conv1; bf16: k = ky*8+kx (7x7 in an 8x8 grid),
                         // f32: k = ky*7+kx (zero for k >= 49),
                         // f32 variant permuted: position g*16+q holds k = 4q+g
  const float* bias;     // [64]
  void* out;             // NHWC [B, 128, 128, 64]
  int64_t B;
  const float* img3;     // [B, 3, 512, 512] fp32 images with DISTINCT channels (stem3 kernel), or null
  const float* w3;       // [64][3][49] fp32 conv1 with bn1's scale folded (the stem3 kernel's weights)
  const u16* img16;      // training stem: [B, 512, 512] bf16 image (bias = bn1 gamma, w unfolded)
  float* part;           // training stem: per-workgroup [2][64] sums of y, y^2
  int x4;                // split-bf16: also the fourth product W_lo.X_lo (resnet.hip's Bottleneck plans)
};

int launch_conv(const ConvArgs& a, int dtype, hipStream_t s, int variant = 0);
int default_conv_variant(const ConvArgs& a);
int launch_stem(const StemArgs& a, int dtype, hipStream_t s);
// training stem (bf16): raw conv1 -> sign(gamma)-pooled raw maps + statistic partials
int launch_stem_train(const StemArgs& a, hipStream_t s);
constexpr int STEM_TRAIN_PARTS = 16;  // statistic partials per image (128 pooled rows / STEM_P)
int launch_block_conv(const BlockConvArgs& a, int dtype, hipStream_t s, int variant = 0);
int default_block_variant(const BlockConvArgs& a, int dtype);
int gemm_block_variant(const BlockConvArgs& a);  // default_block_variant without 30/31 (bf16)
bool layer2_halo();
bool x3_layer2_v31();  // SAD_X3_L2_V31 (default 1): split-bf16 layer2 stride-1 convs on variant 31 (128-channel tiles)
bool layer2_v31();  // SAD_L2_V31 (default 0; 1: measured 2.2-2.7 % slower): layer2's stride-1 convs on variant 31 (128-channel tiles)
bool block_conv_can_pool(const BlockConvArgs& a, int dtype);  // default variant pools Ho x Wo tiles  // SAD_L2_HALO (default 1): layer2's identity blocks on the halo kernel
// dx (+)= col2im(dcol) (train.hip; the strided dgrad of wgrad.hip)
int launch_col2im(const float* dcol, int64_t N, int H, int W, int C, int k, int stride, int pad, int Ho, int Wo,
                  int accumulate, void* dx, int dtype, hipStream_t s);
int launch_avgpool(const void* in, int64_t B, int hw, int c, float* out, int dtype, hipStream_t s);
int launch_heads_final(const float* y2, int64_t B, int n_heads, const float* w3, const float* b3,
                       float* logits, float* merged, hipStream_t s);

// ---- host-side plan helpers (api.hip)
template <typename V>
int upload(void** dst, const std::vector<V>& v) {
  SAD_CHECK_HIP(hipMalloc(dst, v.size() * sizeof(V)));
  SAD_CHECK_HIP(hipMemcpy(*dst, v.data(), v.size() * sizeof(V), hipMemcpyHostToDevice));
  return SAD_OK;
}
// BN (eval) as a per-channel affine: scale = g / sqrt(var + 1e-5), shift = beta - mu * scale
void fold_bn(const float* g, const float* beta, const float* mu, const float* var, int c,
             std::vector<double>& scale, std::vector<double>& shift);
// fp32, bf16 (RNE) or split-bf16 (row_len: K per weight row, hi/lo interleaved per 32)
int upload_typed(void** dst, const std::vector<double>& v, int dtype, int64_t row_len = 0);
// timm conv1 + bn1 (5 arrays) -> the stem kernel's weight layout and bias, and
// (w3_out) the per-channel fp32 weights of the 3-distinct-channel stem
int fold_stem(const float* const* params, int dtype, void** w_out, float** b_out, float** w3_out);

}  // namespace sad
