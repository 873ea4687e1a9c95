// resnet.hip -- deeper timm ResNets (resnet34 BasicBlocks; resnet50/101/152
// Bottlenecks) on the backbone's kernels.  SURVEY.md 8(f) row 4; the
// reference selects the backbone by name (timm.create_model(model_name) at
// submodel_trainer.py:606, model_merger.py:24, inference_runner.py:35 with
// backbone_name at :77).  Declarations: include/sad.h (sad_resnet_*).
//
// Launch plan per micro-batch (NHWC activations in the plan dtype):
//   fused resize + stem (conv1 7x7/2 + bn1 + relu + maxpool)  -> X [128,128,64]
//   BasicBlock:  T1 = relu(conv3x3/s(X))
//                Y  = relu(conv3x3(T1) + shortcut)   the folded 1x1/s downsample
//                     as extra K columns over X; the identity as an epilogue
//                     residual where the halo / resident-weight kernels run
//                     (else identity K columns); bf16 layer1 blocks as one
//                     fused kernel (variant 40), as ResNet-18's plan
//   Bottleneck:  T1 = relu(conv1x1(X));  T2 = relu(conv3x3/s(T1))
//                downsample block: Y = relu(conv1x1(T2) + ds(X)) as one GEMM
//                (K = width + cin, shortcut pixels (oy*s, ox*s) of X)
//                identity block:   Y = relu(conv1x1(T2) + X), X added in the
//                     block-conv epilogue (block_conv_kernel<..., RES = true>;
//                     identity columns would add 4*width K per pixel: +94 % of
//                     the block's FLOPs)
//   global average pool -> feats [B, num_features] fp32
// Every conv is one launch of launch_block_conv (tile variant picked by
// default_block_variant: the resident-weight / halo kernels for the 3x3/s1
// convs that qualify); BN is folded into weights and bias.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

using namespace sad;

namespace {

struct ConvW {
  int cin = 0, cout = 0, k = 0;
  void* w = nullptr;  // [cout][k*k*cin (+ shortcut columns)] plan dtype
  float* b = nullptr;
  int ld = 0;         // elements per weight row
};

struct Block {
  int cin, width, cout, stride;
  bool has_ds;
  ConvW c1, c2, c3;  // Basic: c1, c2 (+ shortcut columns); Bottleneck: c1, c2, c3 (+ ds columns)
};

int fold_conv(const float* const* q, int cout, int cin, int k, int dtype, ConvW& out,
              const float* const* ds = nullptr, int ds_cin = 0, bool identity = false) {
  std::vector<double> sc, sh, scd, shd;
  fold_bn(q[1], q[2], q[3], q[4], cout, sc, sh);
  if (ds) fold_bn(ds[1], ds[2], ds[3], ds[4], cout, scd, shd);
  const int kk = k * k * cin;
  const int extra = ds ? ds_cin : (identity ? cout : 0);
  const int ld = kk + extra;
  std::vector<double> w((size_t)cout * ld, 0.0);
  std::vector<float> b(cout);
  const float* W = q[0];
  for (int o = 0; o < cout; ++o) {
    for (int c = 0; c < cin; ++c)
      for (int t = 0; t < k * k; ++t)  // timm [Cout][Cin][KH][KW] -> [Cout][KH][KW][Cin]
        w[(size_t)o * ld + (size_t)t * cin + c] = (double)W[((size_t)o * cin + c) * k * k + t] * sc[o];
    double bias = sh[o];
    if (ds) {
      for (int c = 0; c < ds_cin; ++c) w[(size_t)o * ld + kk + c] = (double)ds[0][(size_t)o * ds_cin + c] * scd[o];
      bias += shd[o];
    } else if (identity) {
      w[(size_t)o * ld + kk + o] = 1.0;  // exact in bf16
    }
    b[o] = (float)bias;
  }
  out.cin = cin;
  out.cout = cout;
  out.k = k;
  out.ld = ld;
  int rc;
  if ((rc = upload_typed(&out.w, w, dtype, ld))) return rc;
  return upload((void**)&out.b, b);
}

bool deep_x4() {
  static const bool on = [] {
    const char* e = getenv("SAD_DEEP_X4");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

void free_conv(ConvW& c) {
  (void)hipFree(c.w);
  (void)hipFree(c.b);
  c.w = nullptr;
  c.b = nullptr;
}

}  // namespace

struct sad_resnet_plan {
  int dtype, mh, mw, block, num_features;
  // split-bf16 Bottleneck plans: the fourth product W_lo.X_lo in every conv
  // (all on the implicit GEMM) -- resnet50's 53 convs otherwise accumulate the
  // dropped term to ~1.05e-3 on the logits (tools/deep_x3_budget.py: 6.8e-4
  // with it).  SAD_DEEP_X4=0 keeps the three-product form.
  int x4 = 0;
  void* stem_w = nullptr;
  float* stem_b = nullptr;
  float* stem_w3 = nullptr;  // distinct-channel stem (sad_resnet_run_img3)
  std::vector<Block> blocks;
  int64_t max_elems = 0;  // largest activation per segment (elements)
};

extern "C" int sad_resnet_plan_destroy(sad_resnet_plan* p) {
  if (!p) return SAD_OK;
  (void)hipFree(p->stem_w);
  (void)hipFree(p->stem_b);
  (void)hipFree(p->stem_w3);
  for (auto& b : p->blocks) {
    free_conv(b.c1);
    free_conv(b.c2);
    free_conv(b.c3);
  }
  delete p;
  return SAD_OK;
}

extern "C" int sad_resnet_plan_create(const float* const* params, int32_t n_params, int32_t block,
                                      const int32_t* layers, int32_t dtype, int32_t map_h, int32_t map_w,
                                      sad_resnet_plan** out) {
  SAD_REQUIRE(params && layers && out, "null args");
  SAD_REQUIRE(block == SAD_BASIC_BLOCK || block == SAD_BOTTLENECK, "block must be SAD_BASIC_BLOCK or SAD_BOTTLENECK");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16 || dtype == SAD_BF16X3, "dtype");
  SAD_REQUIRE(map_h > 0 && map_w > 0, "map shape");
  const int exp = block == SAD_BOTTLENECK ? 4 : 1;
  const int per_block = block == SAD_BOTTLENECK ? 3 : 2;
  int need = 1, inp = 64;
  const int planes[4] = {64, 128, 256, 512};
  for (int li = 0; li < 4; ++li) {
    SAD_REQUIRE(layers[li] > 0 && layers[li] <= 64, "layers[i] must be in 1..64");
    for (int b = 0; b < layers[li]; ++b) {
      const int s = (b == 0 && li > 0) ? 2 : 1;
      need += per_block + ((b == 0 && (s != 1 || inp != planes[li] * exp)) ? 1 : 0);
      inp = planes[li] * exp;
    }
  }
  SAD_REQUIRE(n_params == 5 * need, "n_params must be 5 x (number of conv+BN groups) of this architecture");
  for (int i = 0; i < n_params; ++i) SAD_REQUIRE(params[i] != nullptr, "null parameter pointer");
  auto* p = new sad_resnet_plan();
  p->dtype = dtype;
  p->mh = map_h;
  p->mw = map_w;
  p->block = block;
  p->num_features = 512 * exp;
  p->x4 = dtype == SAD_BF16X3 && block == SAD_BOTTLENECK && deep_x4();
  int rc;
  if ((rc = fold_stem(params, dtype, &p->stem_w, &p->stem_b, &p->stem_w3))) {
    sad_resnet_plan_destroy(p);
    return rc;
  }
  int gi = 1, H = 128;
  inp = 64;
  p->max_elems = (int64_t)H * H * 64;
  for (int li = 0; li < 4; ++li) {
    for (int b = 0; b < layers[li]; ++b) {
      Block blk{};
      blk.stride = (b == 0 && li > 0) ? 2 : 1;
      blk.cin = inp;
      blk.width = planes[li];
      blk.cout = planes[li] * exp;
      blk.has_ds = b == 0 && (blk.stride != 1 || inp != blk.cout);
      const float* const* q1 = params + 5 * gi++;
      const float* const* q2 = params + 5 * gi++;
      const float* const* q3 = block == SAD_BOTTLENECK ? params + 5 * gi++ : nullptr;
      const float* const* qd = blk.has_ds ? params + 5 * gi++ : nullptr;
      const int Ho = H / blk.stride;
      if (block == SAD_BASIC_BLOCK) {
        if ((rc = fold_conv(q1, blk.cout, inp, 3, dtype, blk.c1)) ||
            (rc = fold_conv(q2, blk.cout, blk.cout, 3, dtype, blk.c2, qd, inp, !blk.has_ds))) {
          p->blocks.push_back(blk);
          sad_resnet_plan_destroy(p);
          return rc;
        }
        p->max_elems = std::max<int64_t>(p->max_elems, (int64_t)Ho * Ho * blk.cout);
      } else {
        if ((rc = fold_conv(q1, blk.width, inp, 1, dtype, blk.c1)) ||
            (rc = fold_conv(q2, blk.width, blk.width, 3, dtype, blk.c2)) ||
            (rc = fold_conv(q3, blk.cout, blk.width, 1, dtype, blk.c3, qd, inp, false))) {
          p->blocks.push_back(blk);
          sad_resnet_plan_destroy(p);
          return rc;
        }
        p->max_elems = std::max<int64_t>(p->max_elems, (int64_t)H * H * blk.width);
        p->max_elems = std::max<int64_t>(p->max_elems, (int64_t)Ho * Ho * blk.cout);
      }
      p->blocks.push_back(blk);
      inp = blk.cout;
      H = Ho;
    }
  }
  *out = p;
  return SAD_OK;
}

extern "C" int sad_resnet_num_features(const sad_resnet_plan* p, int32_t* n) {
  SAD_REQUIRE(p && n, "null args");
  *n = p->num_features;
  return SAD_OK;
}

static size_t rn_act_bytes(const sad_resnet_plan* p, int64_t mb) {
  const size_t es = p->dtype == SAD_BF16 ? 2 : 4;
  return ((size_t)mb * p->max_elems * es + 255) & ~(size_t)255;
}

extern "C" int sad_resnet_workspace_size(const sad_resnet_plan* p, int64_t mb, size_t* bytes) {
  SAD_REQUIRE(p && bytes && mb > 0, "bad args");
  *bytes = 4 * rn_act_bytes(p, mb);
  return SAD_OK;
}

// one conv (+ optional GEMM shortcut of `sc`) on the block-conv kernels
static int rn_block_conv(const sad_resnet_plan* p, const ConvW& c, const void* x, int64_t n, int H, int stride,
                         const void* sc, int Hs, int sc_cin, int sc_stride, void* y, hipStream_t s,
                         const void* res = nullptr) {
  const int pad = c.k / 2;
  const int Ho = (H + 2 * pad - c.k) / stride + 1;
  BlockConvArgs a{};
  a.in0 = x;
  a.in0_pstride = c.cin;
  a.N = (int)n;
  a.H = a.W = H;
  a.Cin = c.cin;
  a.KH = a.KW = c.k;
  a.stride = stride;
  a.pad = pad;
  if (sc) {
    a.in1 = sc;
    a.in1_pstride = sc_cin;
    a.H1 = a.W1 = Hs;
    a.Cin1 = sc_cin;
    a.ss1 = sc_stride;
  }
  a.wt = c.w;
  a.wt_ld = c.ld;
  a.bias = c.b;
  a.res = res;  // epilogue residual (NHWC, c.cout channels)
  a.res_pstride = c.cout;
  a.out = y;
  a.out_pstride = c.cout;
  a.Ho = a.Wo = Ho;
  a.Cout = c.cout;
  a.relu = 1;
  a.M = n * Ho * Ho;
  a.x4 = p->x4;
  return launch_block_conv(a, p->dtype, s);
}

// BasicBlock conv2 whose identity shortcut goes in as an epilogue residual
// (ResNet-18's plan, api.hip run_blocks): stride 1, no downsample, 16 x 16
// tiles, Cout <= 64, or Cout <= 128 where layer2 runs the halo / resident-weight
// kernels (the split-bf16 mode's variant 31 takes the identity as K columns)
static bool identity_epilogue(const sad_resnet_plan* p, const Block& b, int Ho) {
  const int dtype = p->dtype;
  if (p->x4 || !(dtype == SAD_BF16 || dtype == SAD_BF16X3) || b.stride != 1 || b.has_ds || Ho % 16 != 0) return false;
  return b.cout <= 64 || (b.cout <= 128 && layer2_halo() && !(dtype == SAD_BF16 && layer2_v31()) &&
                          !(dtype == SAD_BF16X3 && x3_layer2_v31()));
}

static int rn_chunk(const sad_resnet_plan* p, const float* map, const float* img, int64_t n, float* feats, char* ws,
                    hipStream_t s, const float* img3 = nullptr) {
  const size_t ab = rn_act_bytes(p, n);
  void* X = ws;
  void* Y = ws + ab;
  void* T1 = ws + 2 * ab;
  void* T2 = ws + 3 * ab;
  int rc;
  StemArgs st{map, img, p->mh, p->mw, p->stem_w, p->stem_b, X, n, img3, p->stem_w3};
  st.x4 = p->x4;
  if ((rc = launch_stem(st, p->dtype, s))) return rc;
  int H = 128, C = 64;
  for (const Block& b : p->blocks) {
    const int Ho = H / b.stride;
    if (p->block == SAD_BASIC_BLOCK) {
      if (p->dtype == SAD_BF16 && b.stride == 1 && !b.has_ds && b.cin == 64 && b.cout == 64 && H % 16 == 0 &&
          l1_fused()) {
        // layer1: the whole BasicBlock as one kernel (variant 40), as ResNet-18's plan
        L1BlockArgs f{};
        f.x = (const u16*)X;
        f.out = (u16*)Y;
        f.N = (int)n;
        f.H = f.W = H;
        f.w1 = (const u16*)b.c1.w;
        f.w1_ld = b.c1.ld;
        f.b1 = b.c1.b;
        f.w2 = (const u16*)b.c2.w;
        f.w2_ld = b.c2.ld;  // 576 + the identity's 64 K columns (not read: the residual is the patch centre)
        f.b2 = b.c2.b;
        if ((rc = launch_l1block(f, s))) return rc;
      } else {
        if ((rc = rn_block_conv(p, b.c1, X, n, H, b.stride, nullptr, 0, 0, 1, T1, s))) return rc;
        if (identity_epilogue(p, b, Ho)) {
          // identity blocks of layer1/2: the shortcut as an epilogue add on the
          // halo / resident-weight kernels (as ResNet-18's plan), not as identity
          // K columns on the implicit GEMM
          if ((rc = rn_block_conv(p, b.c2, T1, n, Ho, 1, nullptr, 0, 0, 1, Y, s, X))) return rc;
        } else {
          if ((rc = rn_block_conv(p, b.c2, T1, n, Ho, 1, X, H, C, b.stride, Y, s))) return rc;
        }
      }
    } else {
      if ((rc = rn_block_conv(p, b.c1, X, n, H, 1, nullptr, 0, 0, 1, T1, s))) return rc;
      if ((rc = rn_block_conv(p, b.c2, T1, n, H, b.stride, nullptr, 0, 0, 1, T2, s))) return rc;
      if (b.has_ds) {
        if ((rc = rn_block_conv(p, b.c3, T2, n, Ho, 1, X, H, C, b.stride, Y, s))) return rc;
      } else {
        if ((rc = rn_block_conv(p, b.c3, T2, n, Ho, 1, nullptr, 0, 0, 1, Y, s, X))) return rc;
      }
    }
    std::swap(X, Y);
    H = Ho;
    C = b.cout;
  }
  return launch_avgpool(X, n, H * H, C, feats, p->dtype, s);
}

static int rn_run(const sad_resnet_plan* p, const float* map, const float* img, int64_t B, int64_t mb, float* feats,
                  void* ws, size_t ws_bytes, hipStream_t s, const float* img3 = nullptr) {
  SAD_REQUIRE(p && (map || img || img3) && feats && ws, "null args");
  SAD_REQUIRE(B >= 0 && mb > 0, "bad batch");
  size_t need = 0;
  sad_resnet_workspace_size(p, mb, &need);
  if (ws_bytes < need) {
    set_error("workspace too small");
    return SAD_ERR_NOMEM;
  }
  const int64_t plane = img ? 512 * 512 : (int64_t)p->mh * p->mw;
  for (int64_t i = 0; i < B; i += mb) {
    const int64_t n = std::min(mb, B - i);
    int rc = rn_chunk(p, map ? map + i * plane : nullptr, img ? img + i * plane : nullptr, n,
                      feats + i * p->num_features, (char*)ws, s, img3 ? img3 + i * 3 * 512 * 512 : nullptr);
    if (rc) return rc;
  }
  return SAD_OK;
}

extern "C" int sad_resnet_run(const sad_resnet_plan* p, const float* map, int64_t B, int64_t mb, float* feats,
                              void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(map, "null map");
  return rn_run(p, map, nullptr, B, mb, feats, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int sad_resnet_run_img(const sad_resnet_plan* p, const float* img, int64_t B, int64_t mb, float* feats,
                                  void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(img, "null img");
  return rn_run(p, nullptr, img, B, mb, feats, ws, ws_bytes, (hipStream_t)stream);
}

extern "C" int sad_resnet_run_img3(const sad_resnet_plan* p, const float* img3, int64_t B, int64_t mb, float* feats,
                                   void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(img3, "null img3");
  return rn_run(p, nullptr, nullptr, B, mb, feats, ws, ws_bytes, (hipStream_t)stream, img3);
}
