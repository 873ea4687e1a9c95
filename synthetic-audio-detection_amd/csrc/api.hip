// api.hip -- C ABI of libsad.so: runtime, backbone and heads plans.
// Declarations and the reference interfaces each entry replaces: include/sad.h.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <string>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace sad {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// ResNet-18 conv table in timm state-dict order.
struct ConvSpec {
  int cin, cout, k, stride, pad;
};
static std::vector<ConvSpec> resnet18_specs() {
  std::vector<ConvSpec> v;
  v.push_back({3, 64, 7, 2, 3});  // conv1
  int inp = 64;
  const int planes[4] = {64, 128, 256, 512};
  for (int li = 0; li < 4; ++li) {
    for (int b = 0; b < 2; ++b) {
      const int s = (b == 0 && li > 0) ? 2 : 1;
      v.push_back({inp, planes[li], 3, s, 1});          // conv1
      v.push_back({planes[li], planes[li], 3, 1, 1});   // conv2
      if (b == 0 && (s != 1 || inp != planes[li])) v.push_back({inp, planes[li], 1, s, 0});  // downsample
      inp = planes[li];
    }
  }
  return v;
}

struct DevConv {
  ConvSpec spec;
  void* w = nullptr;      // [cout][k][k][cin] dtype
  float* bias = nullptr;  // [cout]
};

}  // namespace sad

using namespace sad;

struct DevBlock {           // one BasicBlock on the block-conv path
  int cin, cout, stride;
  void* w1 = nullptr;        // conv1: [cout][9*cin]
  float* b1 = nullptr;
  void* w2 = nullptr;        // conv2 + shortcut: [cout][9*cout + cin_sc] (identity or downsample)
  float* b2 = nullptr;
  int cin_sc;
};

struct sad_backbone_plan {
  int dtype;
  int mh, mw;
  int device;
  bool block_path;           // true: persistent block-conv kernels (shortcut in GEMM)
  void* stem_w = nullptr;
  float* stem_b = nullptr;
  float* stem_w3 = nullptr;    // distinct-channel stem (sad_backbone_run_img3)
  std::vector<DevConv> convs;  // index 1.. of the spec table (igemm path)
  std::vector<DevBlock> blocks;
};

struct sad_heads_plan {
  int n_heads, n_feat;
  int feat_dim;                    // backbone feature width (512: ResNet-18/34; 2048: Bottleneck ResNets)
  int device;
  std::vector<int> feat_index;
  std::vector<int> group_of;      // head -> group (== feat index order of appearance)
  std::vector<int> y1_col;        // head -> column offset in Y1
  std::vector<std::vector<int>> groups;  // feat -> heads
  std::vector<float*> w1;          // per group: [512*G][512] folded
  std::vector<float*> b1;          // per group: [512*G]
  float* w2 = nullptr;             // [N][256][512] folded
  float* b2 = nullptr;             // [N][256]
  float* w3 = nullptr;             // [N][2][256]
  float* b3 = nullptr;             // [N][2]
};

extern "C" const char* sad_last_error(void) { return g_err.c_str(); }
extern "C" const char* sad_version(void) { return "libsad 0.1 gfx950 (" __DATE__ " " __TIME__ ")"; }

extern "C" int sad_init(int device) {
  int n = 0;
  SAD_CHECK_HIP(hipGetDeviceCount(&n));
  SAD_REQUIRE(device >= 0 && device < n, "device index out of range");
  SAD_CHECK_HIP(hipSetDevice(device));
  return SAD_OK;
}

// ------------------------------------------------------------- folding ----
namespace sad {
void fold_bn(const float* g, const float* beta, const float* mu, const float* var, int c,
             std::vector<double>& scale, std::vector<double>& shift) {
  scale.resize(c);
  shift.resize(c);
  for (int i = 0; i < c; ++i) {
    scale[i] = (double)g[i] / sqrt((double)var[i] + 1e-5);
    shift[i] = (double)beta[i] - (double)mu[i] * scale[i];
  }
}

int upload_typed(void** dst, const std::vector<double>& v, int dtype, int64_t row_len) {
  if (dtype == SAD_BF16X3) {
    // split-bf16: each row's K axis in groups of 32 -> [hi 32 | lo 32] (the
    // activations' channel interleave, so one 128-B K-step pairs them up)
    if (row_len <= 0 || row_len % 32 != 0 || v.size() % (size_t)row_len != 0) {
      set_error("split-bf16 weights need rows of a multiple of 32 elements");
      return SAD_ERR_ARG;
    }
    std::vector<u16> h(2 * v.size());
    for (size_t i = 0; i < v.size(); ++i) {
      const float x = (float)v[i];
      const u16 hi = f2bf_host(x);
      float hf;
      const uint32_t hb = (uint32_t)hi << 16;
      memcpy(&hf, &hb, 4);
      const size_t g = i / 32, e = i % 32;
      h[g * 64 + e] = hi;
      h[g * 64 + 32 + e] = f2bf_host(x - hf);
    }
    return upload(dst, h);
  }
  if (dtype == SAD_BF16) {
    std::vector<u16> h(v.size());
    for (size_t i = 0; i < v.size(); ++i) h[i] = f2bf_host((float)v[i]);
    return upload(dst, h);
  }
  std::vector<float> h(v.size());
  for (size_t i = 0; i < v.size(); ++i) h[i] = (float)v[i];
  return upload(dst, h);
}

// conv1 7x7/2 + bn1 folded for the stem kernel, the 3 identical input channels
// summed; k = ky*7+kx padded to 64 (params: conv weight, BN weight/bias/mean/var)
int fold_stem(const float* const* params, int dtype, void** w_out, float** b_out, float** w3_out) {
  const float* W = params[0];
  std::vector<double> sc, sh;
  fold_bn(params[1], params[2], params[3], params[4], 64, sc, sh);
  std::vector<double> w(64 * 64, 0.0);
  const int wdt = dtype == SAD_BF16X3 ? SAD_BF16 : dtype;  // split stem: bf16 layout, hi then lo
  std::vector<float> b(64);
  for (int co = 0; co < 64; ++co) {
    for (int k = 0; k < 49; ++k) {
      double s = 0.0;
      for (int c = 0; c < 3; ++c) s += (double)W[(co * 3 + c) * 49 + k];
      // bf16 stem: (ky, kx) on an 8x8 grid; f32 stem: k = ky*7+kx, k=4q+g at g*16+q
      const int pos = wdt == SAD_BF16 ? (k / 7) * 8 + (k % 7) : ((k & 3) * 16 + (k >> 2));
      w[co * 64 + pos] = s * sc[co];
    }
    b[co] = (float)sh[co];
  }
  int rc;
  {  // [64 co][3 c][49 k] fp32, BN scale folded (distinct-channel stem)
    std::vector<float> w3(64 * 3 * 49);
    for (int co = 0; co < 64; ++co)
      for (int i = 0; i < 3 * 49; ++i) w3[co * 147 + i] = (float)((double)W[co * 147 + i] * sc[co]);
    if ((rc = upload((void**)w3_out, w3))) return rc;
  }
  if (dtype == SAD_BF16X3) {  // [64 co][64 k] hi, then [64][64] lo
    std::vector<u16> h(2 * 64 * 64);
    for (int i = 0; i < 64 * 64; ++i) {
      const float x = (float)w[i];
      h[i] = f2bf_host(x);
      float hf;
      const uint32_t hb = (uint32_t)h[i] << 16;
      memcpy(&hf, &hb, 4);
      h[64 * 64 + i] = f2bf_host(x - hf);
    }
    if ((rc = upload(w_out, h))) return rc;
  } else if ((rc = upload_typed(w_out, w, dtype))) {
    return rc;
  }
  return upload((void**)b_out, b);
}
}  // namespace sad

extern "C" int sad_backbone_plan_create(const float* const* params, int32_t n_params, int32_t dtype,
                                        int32_t map_h, int32_t map_w, sad_backbone_plan** out) {
  const std::vector<ConvSpec> specs = resnet18_specs();
  SAD_REQUIRE(params && out, "null params/out");
  SAD_REQUIRE(n_params == (int)specs.size() * 5, "n_params must be 100 (20 conv+BN groups)");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16 || dtype == SAD_BF16X3, "dtype");
  SAD_REQUIRE(map_h > 0 && map_w > 0, "map shape");
  for (int i = 0; i < n_params; ++i) SAD_REQUIRE(params[i] != nullptr, "null parameter pointer");
  auto* p = new sad_backbone_plan();
  p->dtype = dtype;
  p->mh = map_h;
  p->mw = map_w;
  (void)hipGetDevice(&p->device);
  std::vector<double> sc, sh;
  int rc;
  if ((rc = fold_stem(params, dtype, &p->stem_w, &p->stem_b, &p->stem_w3))) return rc;
  // first-generation per-conv weights (SAD_BACKBONE_PATH=igemm; fp32 / bf16 only)
  for (size_t ci = 1; ci < specs.size() && dtype != SAD_BF16X3; ++ci) {
    const ConvSpec& s = specs[ci];
    const float* W = params[ci * 5];
    fold_bn(params[ci * 5 + 1], params[ci * 5 + 2], params[ci * 5 + 3], params[ci * 5 + 4], s.cout, sc, sh);
    std::vector<double> w((size_t)s.cout * s.k * s.k * s.cin);
    for (int co = 0; co < s.cout; ++co)
      for (int c = 0; c < s.cin; ++c)
        for (int ky = 0; ky < s.k; ++ky)
          for (int kx = 0; kx < s.k; ++kx)
            w[(((size_t)co * s.k + ky) * s.k + kx) * s.cin + c] =
                (double)W[(((size_t)co * s.cin + c) * s.k + ky) * s.k + kx] * sc[co];
    DevConv d;
    d.spec = s;
    if ((rc = upload_typed(&d.w, w, dtype))) return rc;
    std::vector<float> bf(sh.begin(), sh.end());
    if ((rc = upload((void**)&d.bias, bf))) return rc;
    p->convs.push_back(d);
  }
  // block path: conv2 and the shortcut (identity or folded downsample) share one
  // GEMM with a concatenated K axis; biases add.
  {
    const char* env = getenv("SAD_BACKBONE_PATH");
    p->block_path = !(env && strcmp(env, "igemm") == 0) || dtype == SAD_BF16X3;
    size_t ci = 1;
    int inp = 64;
    const int planes[4] = {64, 128, 256, 512};
    for (int li = 0; li < 4; ++li) {
      for (int b = 0; b < 2; ++b) {
        const size_t i1 = ci++, i2 = ci++;
        const bool has_ds = (b == 0 && li > 0);
        const size_t ids = has_ds ? ci++ : 0;
        const int co = planes[li];
        DevBlock blk;
        blk.cin = inp;
        blk.cout = co;
        blk.stride = has_ds ? 2 : 1;
        blk.cin_sc = inp;
        std::vector<double> sc1, sh1, sc2, sh2, scd, shd;
        fold_bn(params[i1 * 5 + 1], params[i1 * 5 + 2], params[i1 * 5 + 3], params[i1 * 5 + 4], co, sc1, sh1);
        fold_bn(params[i2 * 5 + 1], params[i2 * 5 + 2], params[i2 * 5 + 3], params[i2 * 5 + 4], co, sc2, sh2);
        if (has_ds) fold_bn(params[ids * 5 + 1], params[ids * 5 + 2], params[ids * 5 + 3], params[ids * 5 + 4], co, scd, shd);
        const int k1 = 9 * inp, k2 = 9 * co + inp;
        std::vector<double> w1((size_t)co * k1), w2((size_t)co * k2, 0.0), b2(co);
        const float* W1 = params[i1 * 5];
        const float* W2 = params[i2 * 5];
        for (int o = 0; o < co; ++o) {
          for (int c = 0; c < inp; ++c)
            for (int t = 0; t < 9; ++t) w1[(size_t)o * k1 + t * inp + c] = (double)W1[((size_t)o * inp + c) * 9 + t] * sc1[o];
          for (int c = 0; c < co; ++c)
            for (int t = 0; t < 9; ++t) w2[(size_t)o * k2 + t * co + c] = (double)W2[((size_t)o * co + c) * 9 + t] * sc2[o];
          if (has_ds) {
            const float* Wd = params[ids * 5];
            for (int c = 0; c < inp; ++c) w2[(size_t)o * k2 + 9 * co + c] = (double)Wd[(size_t)o * inp + c] * scd[o];
            b2[o] = sh2[o] + shd[o];
          } else {
            w2[(size_t)o * k2 + 9 * co + o] = 1.0;  // identity shortcut (exact in bf16)
            b2[o] = sh2[o];
          }
        }
        if ((rc = upload_typed(&blk.w1, w1, dtype, k1))) return rc;
        if ((rc = upload_typed(&blk.w2, w2, dtype, k2))) return rc;
        std::vector<float> b1f(sh1.begin(), sh1.end()), b2f(b2.begin(), b2.end());
        if ((rc = upload((void**)&blk.b1, b1f))) return rc;
        if ((rc = upload((void**)&blk.b2, b2f))) return rc;
        p->blocks.push_back(blk);
        inp = co;
      }
    }
  }
  *out = p;
  return SAD_OK;
}

extern "C" int sad_backbone_plan_destroy(sad_backbone_plan* p) {
  if (!p) return SAD_OK;
  (void)hipFree(p->stem_w);
  (void)hipFree(p->stem_b);
  (void)hipFree(p->stem_w3);
  for (auto& c : p->convs) {
    (void)hipFree(c.w);
    (void)hipFree(c.bias);
  }
  for (auto& b : p->blocks) {
    (void)hipFree(b.w1);
    (void)hipFree(b.b1);
    (void)hipFree(b.w2);
    (void)hipFree(b.b2);
  }
  delete p;
  return SAD_OK;
}

static constexpr int64_t kMaxActElems = 128ll * 128 * 64;  // per segment, layer1 map
static size_t act_bytes(const sad_backbone_plan* p, int64_t mb) {
  const size_t es = p->dtype == SAD_BF16 ? 2 : 4;  // fp32 and split-bf16: 4 B per value
  return ((size_t)mb * kMaxActElems * es + 255) & ~(size_t)255;
}

extern "C" int sad_backbone_workspace_size(const sad_backbone_plan* p, int64_t mb, size_t* bytes) {
  SAD_REQUIRE(p && bytes && mb > 0, "bad args");
  *bytes = 4 * act_bytes(p, mb);
  return SAD_OK;
}

// ---- launch timing of the block-conv kernels (sad_profile_*): HIP events on
// the launch stream around each launch, keyed by tile variant, with the
// launch's algorithmic FLOPs (the identity shortcut's K columns excluded).
struct ProfRec {
  int variant;
  double flops;
  hipEvent_t e0, e1;
  int64_t kernels;  // kernel launches inside the bracket (image-range splits each count)
};
static std::mutex g_prof_mu;
static bool g_prof_on = false;
static std::vector<ProfRec> g_prof;

static int timed_block_conv(const BlockConvArgs& a, int dtype, hipStream_t s, double flops) {
  if (!g_prof_on) return launch_block_conv(a, dtype, s);
  ProfRec r{default_block_variant(a, dtype), flops, nullptr, nullptr, 0};
  SAD_CHECK_HIP(hipEventCreate(&r.e0));
  SAD_CHECK_HIP(hipEventCreate(&r.e1));
  SAD_CHECK_HIP(hipEventRecord(r.e0, s));
  const int64_t k0 = block_conv_kernel_launches();
  int rc = launch_block_conv(a, dtype, s);
  r.kernels = block_conv_kernel_launches() - k0;
  SAD_CHECK_HIP(hipEventRecord(r.e1, s));
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof.push_back(r);
  return rc;
}

// SAD_L1_FUSED=0 runs layer1's blocks as two convs each (variant 25) instead of
// the fused BasicBlock kernel (variant 40; A/B switch).  Same box, 2 rounds:
// fused with 128-segment front sub-batches 52.5k seg/s vs 51.5k unfused at 32
bool sad::l1_fused() {
  static const bool v = [] {
    const char* e = getenv("SAD_L1_FUSED");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}
static int timed_l1block(const L1BlockArgs& a, hipStream_t s, double flops) {
  if (!g_prof_on) return launch_l1block(a, s);
  ProfRec r{40, flops, nullptr, nullptr, 1};
  SAD_CHECK_HIP(hipEventCreate(&r.e0));
  SAD_CHECK_HIP(hipEventCreate(&r.e1));
  SAD_CHECK_HIP(hipEventRecord(r.e0, s));
  int rc = launch_l1block(a, s);
  SAD_CHECK_HIP(hipEventRecord(r.e1, s));
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof.push_back(r);
  return rc;
}

extern "C" int sad_profile_begin(void) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& r : g_prof) {
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  g_prof.clear();
  g_prof_on = true;
  return SAD_OK;
}

// sad_shutdown: release what the library itself holds (the launch-timing
// events of an unfinished sad_profile_begin) after the device has drained.
// Plans are caller-owned and destroyed by their *_destroy calls.
extern "C" int sad_shutdown(void) {
  SAD_CHECK_HIP(hipDeviceSynchronize());
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& r : g_prof) {
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  g_prof.clear();
  g_prof_on = false;
  return SAD_OK;
}

extern "C" int sad_profile_end(int32_t variant, double* total_ms, int64_t* launches, double* flops) {
  SAD_REQUIRE(total_ms && launches && flops, "null outputs");
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof_on = false;
  double ms = 0.0, fl = 0.0;
  int64_t n = 0;
  for (auto& r : g_prof) {
    if (variant == 0 || r.variant == variant) {
      SAD_CHECK_HIP(hipEventSynchronize(r.e1));
      float t = 0.f;
      SAD_CHECK_HIP(hipEventElapsedTime(&t, r.e0, r.e1));
      ms += t;
      fl += r.flops;
      n += r.kernels;
    }
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  g_prof.clear();
  *total_ms = ms;
  *launches = n;
  *flops = fl;
  return SAD_OK;
}

// Blocks [b0, b1) of the block path on n segments: *in (NHWC, H x H x C) ->
// *in (the last output; the buffers *in, *alt, tmp rotate).
// pool_out (optional): fuse the global average pool into the last block's conv2
// when its kernel can (*pooled says whether it did; its NHWC output is not written)
static int run_blocks(const sad_backbone_plan* p, size_t b0, size_t b1, int64_t n, void** in, void** alt, void* tmp,
                      int& H, int& C, hipStream_t s, float* pool_out = nullptr, bool* pooled = nullptr) {
  int rc;
  void* bufA = *in;
  void* bufB = *alt;
  void* bufT = tmp;
  const int64_t mb = n;
  {
    for (size_t bi = b0; bi < b1; ++bi) {
      const DevBlock& blk = p->blocks[bi];
      const int Ho = H / blk.stride;
      if (p->dtype == SAD_BF16 && blk.stride == 1 && blk.cout == 64 && C == 64 && blk.cin == 64 && H % 16 == 0 &&
          l1_fused()) {
        // layer1: the whole BasicBlock as one kernel (variant 40)
        L1BlockArgs f{};
        f.x = (const u16*)bufA;
        f.out = (u16*)bufB;
        f.N = (int)mb;
        f.H = f.W = H;
        f.w1 = (const u16*)blk.w1;
        f.w1_ld = 9 * 64;
        f.b1 = blk.b1;
        f.w2 = (const u16*)blk.w2;
        f.w2_ld = 9 * 64 + blk.cin_sc;  // (the identity's K columns are not read)
        f.b2 = blk.b2;
        if ((rc = timed_l1block(f, s, 2.0 * 2.0 * mb * H * H * 64 * 576.0))) return rc;
        std::swap(bufA, bufB);
        continue;
      }
      BlockConvArgs a{};
      a.in0 = bufA;
      a.in0_pstride = C;
      a.N = (int)mb;
      a.H = a.W = H;
      a.Cin = C;
      a.KH = a.KW = 3;
      a.stride = blk.stride;
      a.pad = 1;
      a.wt = blk.w1;
      a.bias = blk.b1;
      a.out = bufT;
      a.out_pstride = blk.cout;
      a.Ho = a.Wo = Ho;
      a.Cout = blk.cout;
      a.relu = 1;
      a.M = mb * Ho * Ho;
      if ((rc = timed_block_conv(a, p->dtype, s, 2.0 * a.M * a.Cout * 9.0 * C))) return rc;
      BlockConvArgs b2 = a;
      b2.in0 = bufT;
      b2.in0_pstride = blk.cout;
      b2.H = b2.W = Ho;
      b2.Cin = blk.cout;
      b2.stride = 1;
      b2.wt_ld = 9 * blk.cout + blk.cin_sc;
      if ((p->dtype == SAD_BF16 || p->dtype == SAD_BF16X3) && blk.stride == 1 && Ho % 16 == 0 &&
          (blk.cout <= 64 || (blk.cout <= 128 && layer2_halo() && !(p->dtype == SAD_BF16 && layer2_v31()) &&
                            !(p->dtype == SAD_BF16X3 && x3_layer2_v31())))) {
        // identity blocks of layer1/2: the shortcut is an epilogue add on the halo kernel
        b2.res = bufA;
        b2.res_pstride = C;
      } else {
        b2.in1 = bufA;
        b2.in1_pstride = C;
        b2.H1 = b2.W1 = H;
        b2.Cin1 = C;
        b2.ss1 = blk.stride;
      }
      b2.wt = blk.w2;
      b2.bias = blk.b2;
      b2.out = bufB;
      // algorithmic work: conv2, plus the 1x1 downsample when there is one (not the identity)
      if (pool_out && bi + 1 == b1 && block_conv_can_pool(b2, p->dtype)) {
        b2.pool_out = pool_out;
        b2.out = nullptr;
        *pooled = true;
      }
      const double fl2 = 2.0 * b2.M * b2.Cout * (9.0 * blk.cout + (blk.stride != 1 ? (double)C : 0.0));
      if ((rc = timed_block_conv(b2, p->dtype, s, fl2))) return rc;
      std::swap(bufA, bufB);
      H = Ho;
      C = blk.cout;
    }
  }
  *in = bufA;
  *alt = bufB;
  return SAD_OK;
}

// Segments per sub-chunk for the stem and layer1 on the block path
// (SAD_FRONT_MB; 0 = the whole micro-batch).  At 32 segments a layer1
// activation is 64 MiB (bf16), so a conv's input, output and residual can stay
// in the 256 MiB Infinity Cache; layers 2-4 run on the whole micro-batch (their
// grids need the pixels, and bigger launches amortise the persistent kernels'
// ramp and tail).  Same-box sweeps (round 2, "front:micro-batch"):
// 32:512 46.9k seg/s vs 0:128 45.9k, 0:512 44.4-46.4k, 64:512 45.4k; 16 is 7%
// slower (layer2's grids underfill).  At 32:128 one box measured -1.1%.
// Round 2 at micro-batch 1024: 40 is 0.9 % and 48 1.4 % slower than 32 (same
// box, 3 rounds; profiles/r02s3_frontmb_ab.log).
// With layer1 fused (bf16, variant 40) only the block inputs/outputs pass
// through memory and the fused kernel's per-workgroup weight prologue wants
// more tiles: 128 segments (+1.8-2.1 % end to end vs fused at 32, same box;
// 64: +1.7-2 %).  With layer2 on variant 41 (round 3): 256 is +0.4-3 % over 128
// (same box, 3 rounds, tools/r03_sweep2.sh: 59.0-59.1k vs 57.3-58.9k seg/s;
// 512 with micro-batch 2048 within 0.2 % of 256).
static int front_sub_batch(int dtype) {
  static int v = [] {
    const char* e = getenv("SAD_FRONT_MB");
    return e ? atoi(e) : -1;
  }();
  if (v >= 0) return v;
  // split-bf16 (layer1 on variant 42): 64, +0.8 % over 32 in the parity mode
  // (same box, 2 rounds; 128 and the whole micro-batch are slower,
  // profiles/r04_x3_frontmb_ab.log)
  return dtype == SAD_BF16 && l1_fused() ? 256 : dtype == SAD_BF16X3 ? 64 : 32;
}

static int run_chunk(const sad_backbone_plan* p, const float* map, const float* img, int64_t mb, float* feats,
                     void* layer4_out, char* ws, hipStream_t s, const float* img3 = nullptr) {
  const size_t ab = act_bytes(p, mb);
  void* bufA = ws;
  void* bufB = ws + ab;
  void* bufT = ws + 2 * ab;
  void* bufD = ws + 3 * ab;
  int rc;
  int H = 128, C = 64;
  bool pooled = false;  // the last conv wrote the pooled features itself
  if (p->block_path) {
    const size_t es = p->dtype == SAD_BF16 ? 2 : 4;
    const int64_t f = front_sub_batch(p->dtype) > 0 ? std::min<int64_t>(front_sub_batch(p->dtype), mb) : mb;
    // stem + layer1 per sub-chunk of f segments (Infinity-Cache-sized); layer1's
    // output ([f, 128, 128, 64] per sub-chunk) is gathered in bufD, then layers
    // 2-4 run on the whole micro-batch (layer2's halo grids underfill at f = 32:
    // its two convs took 218 + 201 vs 197 + 185 us per 128 segments).
    const size_t l1_elems = 128 * 128 * 64;
    for (int64_t i = 0; i < mb; i += f) {
      const int64_t n = std::min(f, mb - i);
      void* a0 = bufA;
      void* a1 = bufB;
      StemArgs st{map ? map + i * p->mh * p->mw : nullptr, img ? img + i * 512 * 512 : nullptr, p->mh, p->mw,
                  p->stem_w, p->stem_b, a0, n, img3 ? img3 + i * 3 * 512 * 512 : nullptr, p->stem_w3};
      if ((rc = launch_stem(st, p->dtype, s))) return rc;
      H = 128;
      C = 64;
      if ((rc = run_blocks(p, 0, 1, n, &a0, &a1, bufT, H, C, s))) return rc;
      // layer1's second block writes straight into its slot of bufD
      void* slot = (char*)bufD + (size_t)i * l1_elems * es;
      void* dst = slot;
      void* src = a0;
      if ((rc = run_blocks(p, 1, 2, n, &src, &dst, bufT, H, C, s))) return rc;
      if (src != slot) {
        set_error("internal: layer1 output not in its bufD slot");
        return SAD_ERR_STATE;
      }
    }
    void* a0 = bufD;
    void* a1 = bufA;
    if ((rc = run_blocks(p, 2, p->blocks.size(), mb, &a0, &a1, bufB, H, C, s, layer4_out ? nullptr : feats,
                         &pooled)))
      return rc;
    bufA = a0;
  } else {
    StemArgs st{map, img, p->mh, p->mw, p->stem_w, p->stem_b, bufA, mb, img3, p->stem_w3};
    if ((rc = launch_stem(st, p->dtype, s))) return rc;
  }
  size_t ci = 0;
  for (int li = 0; li < 4 && !p->block_path; ++li) {
    for (int b = 0; b < 2; ++b) {
      const DevConv& c1 = p->convs[ci++];
      const DevConv& c2 = p->convs[ci++];
      const DevConv* ds = nullptr;
      if (b == 0 && li > 0) ds = &p->convs[ci++];
      const int Ho = H / c1.spec.stride;
      ConvArgs a{};
      a.in = bufA;
      a.in_pstride = C;
      a.N = (int)mb;
      a.H = H;
      a.W = H;
      a.Cin = C;
      a.wt = c1.w;
      a.bias = c1.bias;
      a.res = nullptr;
      a.out = bufT;
      a.out_pstride = c1.spec.cout;
      a.Ho = Ho;
      a.Wo = Ho;
      a.Cout = c1.spec.cout;
      a.KH = a.KW = c1.spec.k;
      a.stride = c1.spec.stride;
      a.pad = c1.spec.pad;
      a.relu = 1;
      a.M = mb * Ho * Ho;
      if ((rc = launch_conv(a, p->dtype, s))) return rc;
      const void* res = bufA;
      if (ds) {
        ConvArgs d = a;
        d.wt = ds->w;
        d.bias = ds->bias;
        d.out = bufD;
        d.KH = d.KW = 1;
        d.pad = 0;
        d.relu = 0;
        if ((rc = launch_conv(d, p->dtype, s))) return rc;
        res = bufD;
      }
      ConvArgs a2{};
      a2.in = bufT;
      a2.in_pstride = c2.spec.cin;
      a2.N = (int)mb;
      a2.H = Ho;
      a2.W = Ho;
      a2.Cin = c2.spec.cin;
      a2.wt = c2.w;
      a2.bias = c2.bias;
      a2.res = res;
      a2.res_pstride = c2.spec.cout;
      a2.out = bufB;
      a2.out_pstride = c2.spec.cout;
      a2.Ho = Ho;
      a2.Wo = Ho;
      a2.Cout = c2.spec.cout;
      a2.KH = a2.KW = 3;
      a2.stride = 1;
      a2.pad = 1;
      a2.relu = 1;
      a2.M = mb * Ho * Ho;
      if ((rc = launch_conv(a2, p->dtype, s))) return rc;
      std::swap(bufA, bufB);
      H = Ho;
      C = c2.spec.cout;
    }
  }
  if (layer4_out) {
    const size_t es = p->dtype == SAD_BF16 ? 2 : 4;
    SAD_CHECK_HIP(hipMemcpyAsync(layer4_out, bufA, (size_t)mb * H * H * C * es, hipMemcpyDeviceToDevice, s));
  }
  if (pooled) return SAD_OK;
  return launch_avgpool(bufA, mb, H * H, C, feats, p->dtype, s);
}

extern "C" int sad_backbone_run(const sad_backbone_plan* p, const float* map, int64_t B, int64_t mb,
                                float* feats, void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(p && feats && ws, "null args");
  SAD_REQUIRE(B >= 0 && mb > 0, "bad batch");
  size_t need = 0;
  sad_backbone_workspace_size(p, mb, &need);
  if (ws_bytes < need) {
    set_error("workspace too small");
    return SAD_ERR_NOMEM;
  }
  const int64_t plane = (int64_t)p->mh * p->mw;
  for (int64_t i = 0; i < B; i += mb) {
    const int64_t n = std::min(mb, B - i);
    int rc = run_chunk(p, map + i * plane, nullptr, n, feats + i * 512, nullptr, (char*)ws, (hipStream_t)stream);
    if (rc) return rc;
  }
  return SAD_OK;
}

extern "C" int sad_backbone_run_debug(const sad_backbone_plan* p, const float* map, int64_t B, float* feats,
                                      void* layer4_out, void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(p && feats && ws && layer4_out && B > 0, "null args");
  size_t need = 0;
  sad_backbone_workspace_size(p, B, &need);
  if (ws_bytes < need) {
    set_error("workspace too small (debug run needs micro_batch = B)");
    return SAD_ERR_NOMEM;
  }
  return run_chunk(p, map, nullptr, B, feats, layer4_out, (char*)ws, (hipStream_t)stream);
}

extern "C" int sad_backbone_stem_run(const sad_backbone_plan* p, const float* map, int64_t B, void* out,
                                     void* stream) {
  SAD_REQUIRE(p && map && out && B >= 0, "null args");
  StemArgs st{map, nullptr, p->mh, p->mw, p->stem_w, p->stem_b, out, B};
  return launch_stem(st, p->dtype, (hipStream_t)stream);
}

extern "C" int sad_backbone_run_img(const sad_backbone_plan* p, const float* img, int64_t B, int64_t mb,
                                    float* feats, void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(p && img && feats && ws, "null args");
  SAD_REQUIRE(B >= 0 && mb > 0, "bad batch");
  size_t need = 0;
  sad_backbone_workspace_size(p, mb, &need);
  if (ws_bytes < need) {
    set_error("workspace too small");
    return SAD_ERR_NOMEM;
  }
  for (int64_t i = 0; i < B; i += mb) {
    const int64_t n = std::min(mb, B - i);
    int rc = run_chunk(p, nullptr, img + i * 512 * 512, n, feats + i * 512, nullptr, (char*)ws, (hipStream_t)stream);
    if (rc) return rc;
  }
  return SAD_OK;
}

extern "C" int sad_backbone_run_img3(const sad_backbone_plan* p, const float* img3, int64_t B, int64_t mb,
                                     float* feats, void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(p && img3 && feats && ws, "null args");
  SAD_REQUIRE(B >= 0 && mb > 0, "bad batch");
  size_t need = 0;
  sad_backbone_workspace_size(p, mb, &need);
  if (ws_bytes < need) {
    set_error("workspace too small");
    return SAD_ERR_NOMEM;
  }
  for (int64_t i = 0; i < B; i += mb) {
    const int64_t n = std::min(mb, B - i);
    int rc = run_chunk(p, nullptr, nullptr, n, feats + i * 512, nullptr, (char*)ws, (hipStream_t)stream,
                       img3 + i * 3 * 512 * 512);
    if (rc) return rc;
  }
  return SAD_OK;
}

// ---------------------------------------------------------------- heads ----
extern "C" int sad_heads_plan_create(const float* const* params, int32_t n_heads, const int32_t* feat_index,
                                     int32_t n_feat, sad_heads_plan** out) {
  return sad_heads_plan_create_dim(params, n_heads, feat_index, n_feat, 512, out);
}

extern "C" int sad_heads_plan_create_dim(const float* const* params, int32_t n_heads, const int32_t* feat_index,
                                         int32_t n_feat, int32_t feat_dim, sad_heads_plan** out) {
  SAD_REQUIRE(params && out && n_heads > 0 && n_feat > 0, "bad args");
  SAD_REQUIRE(feat_dim > 0 && feat_dim % 64 == 0, "feat_dim must be a positive multiple of 64");
  for (int i = 0; i < n_heads * 14; ++i) SAD_REQUIRE(params[i], "null head parameter");
  auto* p = new sad_heads_plan();
  p->n_heads = n_heads;
  p->n_feat = n_feat;
  p->feat_dim = feat_dim;
  const int D = feat_dim;
  (void)hipGetDevice(&p->device);
  p->groups.assign(n_feat, {});
  for (int h = 0; h < n_heads; ++h) {
    const int f = feat_index ? feat_index[h] : 0;
    SAD_REQUIRE(f >= 0 && f < n_feat, "feat_index out of range");
    p->feat_index.push_back(f);
    p->groups[f].push_back(h);
  }
  p->y1_col.assign(n_heads, 0);
  int col = 0, rc;
  std::vector<double> sc, sh;
  for (int f = 0; f < n_feat; ++f) {
    const auto& g = p->groups[f];
    std::vector<float> w1((size_t)g.size() * 512 * D), b1(g.size() * 512);
    for (size_t gi = 0; gi < g.size(); ++gi) {
      const float* const* hp = params + g[gi] * 14;
      fold_bn(hp[2], hp[3], hp[4], hp[5], 512, sc, sh);
      for (int o = 0; o < 512; ++o) {
        for (int i = 0; i < D; ++i)
          w1[(gi * 512 + o) * D + i] = (float)((double)hp[0][(size_t)o * D + i] * sc[o]);
        b1[gi * 512 + o] = (float)((double)hp[1][o] * sc[o] + sh[o]);
      }
      p->y1_col[g[gi]] = col;
      col += 512;
    }
    void* dw = nullptr;
    void* db = nullptr;
    if (!g.empty()) {
      if ((rc = upload(&dw, w1))) return rc;
      if ((rc = upload(&db, b1))) return rc;
    }
    p->w1.push_back((float*)dw);
    p->b1.push_back((float*)db);
  }
  std::vector<float> w2((size_t)n_heads * 256 * 512), b2(n_heads * 256), w3(n_heads * 512), b3(n_heads * 2);
  for (int h = 0; h < n_heads; ++h) {
    const float* const* hp = params + h * 14;
    fold_bn(hp[8], hp[9], hp[10], hp[11], 256, sc, sh);
    for (int o = 0; o < 256; ++o) {
      for (int i = 0; i < 512; ++i) w2[((size_t)h * 256 + o) * 512 + i] = (float)((double)hp[6][o * 512 + i] * sc[o]);
      b2[h * 256 + o] = (float)((double)hp[7][o] * sc[o] + sh[o]);
    }
    memcpy(&w3[h * 512], hp[12], 512 * sizeof(float));
    memcpy(&b3[h * 2], hp[13], 2 * sizeof(float));
  }
  if ((rc = upload((void**)&p->w2, w2))) return rc;
  if ((rc = upload((void**)&p->b2, b2))) return rc;
  if ((rc = upload((void**)&p->w3, w3))) return rc;
  if ((rc = upload((void**)&p->b3, b3))) return rc;
  *out = p;
  return SAD_OK;
}

extern "C" int sad_heads_plan_destroy(sad_heads_plan* p) {
  if (!p) return SAD_OK;
  for (auto* w : p->w1) (void)hipFree(w);
  for (auto* b : p->b1) (void)hipFree(b);
  (void)hipFree(p->w2);
  (void)hipFree(p->b2);
  (void)hipFree(p->w3);
  (void)hipFree(p->b3);
  delete p;
  return SAD_OK;
}

extern "C" int sad_heads_workspace_size(const sad_heads_plan* p, int64_t B, size_t* bytes) {
  SAD_REQUIRE(p && bytes && B >= 0, "bad args");
  *bytes = (size_t)B * p->n_heads * (512 + 256) * sizeof(float) + 256;
  return SAD_OK;
}

extern "C" int sad_heads_merge_run(const sad_heads_plan* p, const float* const* feats, int64_t B, float* logits,
                                   float* merged, void* ws, size_t ws_bytes, void* stream) {
  SAD_REQUIRE(p && feats && merged && ws, "null args");
  size_t need = 0;
  sad_heads_workspace_size(p, B, &need);
  if (ws_bytes < need) {
    set_error("heads workspace too small");
    return SAD_ERR_NOMEM;
  }
  if (B == 0) return SAD_OK;
  hipStream_t s = (hipStream_t)stream;
  const int N = p->n_heads;
  float* y1 = (float*)ws;
  float* y2 = y1 + (size_t)B * N * 512;
  int rc, col = 0;
  for (int f = 0; f < p->n_feat; ++f) {
    const int G = (int)p->groups[f].size();
    if (!G) continue;
    SAD_REQUIRE(feats[f], "null feature pointer");
    ConvArgs a{};
    a.in = feats[f];
    a.in_pstride = p->feat_dim;
    a.N = (int)B;
    a.H = a.W = 1;
    a.Cin = p->feat_dim;
    a.wt = p->w1[f];
    a.bias = p->b1[f];
    a.out = y1 + col;
    a.out_pstride = (int64_t)N * 512;
    a.Ho = a.Wo = 1;
    a.Cout = 512 * G;
    a.KH = a.KW = 1;
    a.stride = 1;
    a.pad = 0;
    a.relu = 1;
    a.M = B;
    if ((rc = launch_conv(a, SAD_F32, s))) return rc;
    col += 512 * G;
  }
  // the N heads' Linear(512, 256) + BN1d + ReLU: one grouped launch when the
  // heads' hidden columns are in head order (always for a shared backbone)
  bool regular = true;
  for (int h = 0; h < N; ++h) regular = regular && p->y1_col[h] == h * 512;
  for (int h = 0; h < (regular ? 1 : N); ++h) {
    ConvArgs a{};
    if (regular && N > 1) {
      a.groups = N;
      a.in_gstride = 512;
      a.wt_gstride = (int64_t)256 * 512;
      a.bias_gstride = 256;
      a.out_gstride = 256;
    }
    a.in = y1 + p->y1_col[h];
    a.in_pstride = (int64_t)N * 512;
    a.N = (int)B;
    a.H = a.W = 1;
    a.Cin = 512;
    a.wt = p->w2 + (size_t)h * 256 * 512;
    a.bias = p->b2 + h * 256;
    a.out = y2 + h * 256;
    a.out_pstride = (int64_t)N * 256;
    a.Ho = a.Wo = 1;
    a.Cout = 256;
    a.KH = a.KW = 1;
    a.stride = 1;
    a.pad = 0;
    a.relu = 1;
    a.M = B;
    if ((rc = launch_conv(a, SAD_F32, s))) return rc;
  }
  return launch_heads_final(y2, B, N, p->w3, p->b3, logits, merged, s);
}

// ------------------------------------------------------------- operators ----
extern "C" int sad_conv2d_run(const void* in, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* wt,
                              const float* bias, const void* res, void* out, int32_t Cout, int32_t k,
                              int32_t stride, int32_t pad, int32_t relu, int32_t dtype, int32_t variant,
                              void* stream) {
  SAD_REQUIRE(in && wt && bias && out, "null tensor");
  SAD_REQUIRE(N >= 0 && H > 0 && W > 0 && k > 0 && stride > 0 && pad >= 0, "bad shape");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  ConvArgs a{};
  a.in = in;
  a.in_pstride = Cin;
  a.N = (int)N;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.wt = wt;
  a.bias = bias;
  a.res = res;
  a.res_pstride = Cout;
  a.out = out;
  a.out_pstride = Cout;
  a.Ho = (H + 2 * pad - k) / stride + 1;
  a.Wo = (W + 2 * pad - k) / stride + 1;
  a.Cout = Cout;
  a.KH = a.KW = k;
  a.stride = stride;
  a.pad = pad;
  a.relu = relu;
  a.M = N * a.Ho * a.Wo;
  return launch_conv(a, dtype, (hipStream_t)stream, variant);
}

extern "C" int sad_l1_block_run(const void* x, int64_t N, int32_t H, int32_t W, const void* w1, int32_t w1_ld,
                                const float* b1, const void* w2, int32_t w2_ld, const float* b2, void* out,
                                int32_t ablate, void* stream) {
  SAD_REQUIRE(x && w1 && b1 && w2 && b2 && out, "null tensor");
  SAD_REQUIRE(N >= 0 && N < (1ll << 31) && H > 0 && W > 0, "bad shape");
  const int64_t bytes = N * H * W * 128;
  SAD_REQUIRE((const char*)out + bytes <= (const char*)x || (const char*)x + bytes <= (const char*)out,
              "fused layer1 block: out must not overlap x");
  L1BlockArgs a{};
  a.x = (const u16*)x;
  a.out = (u16*)out;
  a.N = (int)N;
  a.H = H;
  a.W = W;
  a.w1 = (const u16*)w1;
  a.w1_ld = w1_ld;
  a.b1 = b1;
  a.w2 = (const u16*)w2;
  a.w2_ld = w2_ld;
  a.b2 = b2;
  a.ablate = ablate;
  return launch_l1block(a, (hipStream_t)stream);
}

extern "C" int sad_block_conv_run(const void* in0, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* in1,
                                  int32_t H1, int32_t W1, int32_t Cin1, int32_t ss1, const void* wt,
                                  int32_t wt_ld, const float* bias, const void* res, void* out, int32_t Cout,
                                  int32_t k, int32_t stride, int32_t pad, int32_t relu, int32_t dtype,
                                  int32_t variant, void* stream) {
  SAD_REQUIRE(in0 && wt && bias && out, "null tensor");
  SAD_REQUIRE(N >= 0 && H > 0 && W > 0 && k > 0 && stride > 0 && pad >= 0, "bad shape");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16 || dtype == SAD_BF16X3, "dtype");
  BlockConvArgs a{};
  a.in0 = in0;
  a.in0_pstride = Cin;
  a.N = (int)N;
  a.H = H;
  a.W = W;
  a.Cin = Cin;
  a.KH = a.KW = k;
  a.stride = stride;
  a.pad = pad;
  a.in1 = in1;
  a.in1_pstride = Cin1;
  a.H1 = H1;
  a.W1 = W1;
  a.Cin1 = in1 ? Cin1 : 0;
  a.ss1 = ss1;
  a.wt = wt;
  a.wt_ld = wt_ld;
  a.bias = bias;
  a.res = res;
  a.res_pstride = Cout;
  a.out = out;
  a.out_pstride = Cout;
  a.Ho = (H + 2 * pad - k) / stride + 1;
  a.Wo = (W + 2 * pad - k) / stride + 1;
  if (in1) SAD_REQUIRE((a.Ho - 1) * ss1 < H1 && (a.Wo - 1) * ss1 < W1, "shortcut source too small");
  a.Cout = Cout;
  a.relu = relu;
  a.M = N * a.Ho * a.Wo;
  a.ablate = (variant >> 8) & 255;  // timing-only ablation bits (tools/convbench.py --ablate)
  a.x4 = (variant & SAD_CONV_FOUR_PRODUCTS) != 0;
  return launch_block_conv(a, dtype, (hipStream_t)stream, variant & 255);
}
