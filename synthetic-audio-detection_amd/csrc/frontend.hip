// frontend.hip -- fused int16 PCM -> Hann -> rFFT(2048) -> |X|^2 -> mel -> dB
// -> per-segment top-db clamp + standardisation, for gfx950.
//
// Replaces torchaudio MelSpectrogram + AmplitudeToDB + the (x-mean)/(std+1e-6)
// step of inference_runner.py:157-171 (semantics: SURVEY.md Appendix A).
//
// Kernel 1 (fe_mel_db): one workgroup = 4 waves = one segment x a block of 32
//   STFT frames; each wave owns one frame at a time.  A 2048-point real frame
//   is packed as a 1024-point complex sequence z[m] = y[2m] + i*y[2m+1] and
//   transformed by a four-step 16 x 64 FFT: 16-point DFTs in registers, ONE
//   swizzled transpose through the wave's LDS slot, 16-point DFTs in registers
//   plus a 4-point DFT across each lane quad (DPP); per-lane twiddles
//   (float64-accurate table values) are held in registers for all frames.  The real
//   spectrum is recovered for the bins the mel bank touches (2..768), powered,
//   projected on the CSR mel bank (1515 nnz) and converted to dB.
//   PCM reads: the FFT input z is loaded straight from HBM, lane-
//   consecutive int16 pairs (coalesced); reflect padding is index arithmetic.
// Kernel 2 (fe_normalize): one workgroup per segment: max -> top-db clamp ->
//   float64 mean / unbiased variance -> standardise (32,128 values).
// Fused form (round 5, SAD_FE_FUSED=1/2, off by default: measured 1.7-2.2x
//   slower): fe_mel_db's workgroups publish their block's dB tile
//   and maximum, and the LAST workgroup of a segment to finish (a per-segment
//   counter; 1: agent-scope release / acquire fences, 2: agent-scope stores and
//   loads) standardises the whole segment -- fe_normalize's arithmetic in the
//   same order, so the maps are bit-identical.  SAD_FE_XCD_MAP=1 orders the 1-D
//   grid so a segment's 8 frame blocks share an XCD (neutral).
#include <math.h>

#include <algorithm>
#include <functional>
#include <type_traits>
#include <vector>

#include "common.hpp"

namespace sad {

constexpr int FE_NFFT = 2048;
constexpr int FE_NC = 1024;         // complex FFT length
constexpr int FE_FRAMES_PER_WG = 32;
constexpr int FE_WAVES = 4;

struct FrontendPlan {
  sad_frontend_cfg cfg;
  int n_frames;
  int bin_lo, bin_hi;         // mel bank nonzero bin range [lo, hi]
  int nnz = 0;                // packed mel weights
  float2* d_tw1024 = nullptr;  // e^{-2 pi i m / 1024}, m < 1024
  float2* d_tw2048 = nullptr;  // e^{-2 pi i k / 2048}, k <= 1024
  float* d_window = nullptr;   // periodic Hann(2048)
  float* d_window_s16 = nullptr;  // the same times 2^-15 (int16 PCM: torchaudio.load's 1/32768, folded)
  float2* d_rtw = nullptr;     // [FE_NC + 1] real-spectrum recovery twiddle of bin k (fe_rtw_kernel)
  int* d_mel_start = nullptr;  // [n_mels] first bin
  int* d_mel_len = nullptr;    // [n_mels]
  int* d_mel_off = nullptr;    // [n_mels] offset into d_mel_w
  float* d_mel_w = nullptr;    // packed nonzero weights
  // staged mel projection by lane (n_mels <= FE_STAGE_MELS): lane l sums mel
  // rows lane_tab[l] (q = 0) and lane_tab[64 + l] (q = 1; -1: none) from bins
  // bin_lo + lane_tab[128 + q * 64 + l] .. + ml[q] - 1, weights [ml0 + ml1][64]
  // zero past the row's filter (null: the CSR loop)
  int* d_lane_tab = nullptr;
  float* d_lane_w = nullptr;
  int ml0 = 0, ml1 = 0;
  // fused normalisation (staged plans): per-segment arrival counters (left at
  // zero by every launch) and per-block maxima, for one launch chunk
  unsigned* d_seg_cnt = nullptr;
  float* d_seg_bmax = nullptr;
  int device = 0;
};

constexpr int FE_CHUNK = 65535;  // segments per launch (the non-fused grid's y limit)
constexpr int kNormRegs = 32;    // normalisation: values per thread of 1,024 (maps up to 32,768 values)

__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// e^{-2 pi i k / 2048} of the real-spectrum recovery, k = 0..1024: the
// 1024-point table at k / 2, times e^{-2 pi i / 2048} for odd k (the per-bin
// arithmetic fe_mel_db_kernel ran per frame until round 6, now once per plan)
__device__ __forceinline__ float2 fe_rtw(const float2* tw1024, int k) {
  float2 w2 = tw1024[(k >> 1) & (FE_NC - 1)];
  if (k == FE_NC) w2 = make_float2(-1.f, 0.f);
  if (k & 1) w2 = cmul(w2, make_float2(0.99999529380957619f, -0.0030679567629659761f));
  return w2;
}
__global__ void fe_rtw_kernel(const float2* __restrict__ tw1024, float2* __restrict__ rtw) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k <= FE_NC) rtw[k] = fe_rtw(tw1024, k);
}

// ---- four-step 1024-point FFT building blocks (one wave per frame) ----------
// 4-point forward DFT in place: (x0, x1, x2, x3) -> (X0, X1, X2, X3)
__device__ __forceinline__ void dft4(float2& a, float2& b, float2& c, float2& d) {
  const float2 s02 = make_float2(a.x + c.x, a.y + c.y), d02 = make_float2(a.x - c.x, a.y - c.y);
  const float2 s13 = make_float2(b.x + d.x, b.y + d.y), d13 = make_float2(b.x - d.x, b.y - d.y);
  a = make_float2(s02.x + s13.x, s02.y + s13.y);
  b = make_float2(d02.x + d13.y, d02.y - d13.x);  // x0 - i x1 - x2 + i x3
  c = make_float2(s02.x - s13.x, s02.y - s13.y);
  d = make_float2(d02.x - d13.y, d02.y + d13.x);  // x0 + i x1 - x2 - i x3
}
// W16^j = e^{-2 pi i j / 16}
__device__ constexpr float W16R[10] = {1.f, 0.92387953251128674f, 0.70710678118654757f, 0.38268343236508978f, 0.f,
                                       -0.38268343236508978f, -0.70710678118654757f, -0.92387953251128674f, -1.f,
                                       -0.92387953251128674f};
__device__ constexpr float W16I[10] = {0.f, -0.38268343236508978f, -0.70710678118654757f, -0.92387953251128674f, -1.f,
                                       -0.92387953251128674f, -0.70710678118654757f, -0.38268343236508978f, 0.f,
                                       0.38268343236508978f};
// 16-point forward DFT in registers: t = 4 t1 + t2, k = k1 + 4 k2 (4-point DFTs
// over t1, twiddles W16^{t2 k1}, 4-point DFTs over t2).  In: x[t]; out: X[k] at
// x[fe_p16(k)].
__device__ __forceinline__ constexpr int fe_p16(int k) { return 4 * (k & 3) + (k >> 2); }
__device__ __forceinline__ void dft16(float2 (&x)[16]) {
#pragma unroll
  for (int t2 = 0; t2 < 4; ++t2) dft4(x[t2], x[4 + t2], x[8 + t2], x[12 + t2]);
#pragma unroll
  for (int k1 = 1; k1 < 4; ++k1)
#pragma unroll
    for (int t2 = 1; t2 < 4; ++t2) x[4 * k1 + t2] = cmul(x[4 * k1 + t2], make_float2(W16R[t2 * k1], W16I[t2 * k1]));
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) dft4(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3]);
}
// spectrum slot of bin k in the wave's buffer: 4 pad slots per 256 bins make the
// final scatter (k = k1 + 16 k2a + 256 br(q)) bank-conflict-free
// (one pad slot per 64 bins: the scatter's lane groups land on the same banks as
// with four per 256, and bins k + 64 are always 65 slots on, so the recovery
// walks its two spectrum reads by constant strides)
__device__ __forceinline__ int fe_zslot(int k) { return k + (k >> 6); }

// LDS exchange between the lanes of ONE wave: the wave's LDS operations
// complete in order, so a compiler fence at wavefront scope is all that is
// needed (no workgroup barrier: the four waves run independent frames).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr int FE_STAGE_MELS = 128;  // dB rows staged in LDS for coalesced stores
constexpr int FE_POW = 800;         // power bins per wave in LDS (the reference's bank: 767)
constexpr int FE_PWPAD = 8;         // zero slots before bin_lo (the mel windows' shifted starts)
constexpr int FE_ZBUF = FE_NC + 16;  // spectrum slots per wave (fe_zslot padding)
constexpr int FE_RTWN = 784;         // recovery twiddles held in LDS (the reference's bank: 767 bins)
// LDS: recovery twiddles 6.1 KB + 4 FFT buffers 32.5 KB + power 12.5 KB + dB
// staging 16.5 KB = 68 KB: two workgroups per CU (the frame-major form, without
// the staging: 52 KB, three).  (The mel weights are read from the lane
// table in global memory, L1-resident: 11.5 KB for the reference's bank.)

// The fused form's tail: the segment's last workgroup standardises it.  The
// values are visited as fe_normalize_kernel's 1,024 threads visit them
// (virtual thread vt = tid + 256 j holds i = vt + 1024 k), and the float64
// sums are reduced over the same butterflies and wave order, so both forms
// give the same bits.
template <bool SC1>  // SC1: agent-scope loads (global_load sc1: past the XCD's L2 to the coherence point)
__device__ __forceinline__ float fe_ld(const float* p) {
  if constexpr (SC1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

template <bool SC1>
__device__ __forceinline__ void fe_standardise_segment(float* db, bool keep_db, float* y, int count,
                                                       const float* bmax, int n_fb, float top_db, double* red) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float mx = -INFINITY;
  for (int b = 0; b < n_fb; ++b) mx = fmaxf(mx, fe_ld<SC1>(bmax + b));
  const float floor_db = top_db >= 0.f ? mx - top_db : -INFINITY;
  // one virtual thread's 32 values at a time (the segment is re-read from L2
  // per pass rather than held: 128 registers would spill)
  auto load = [&](int j, float (&v)[kNormRegs]) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k) {
      const int i = tid + 256 * j + 1024 * k;
      v[k] = i < count ? fmaxf(fe_ld<SC1>(db + i), floor_db) : 0.f;
    }
  };
  auto reduce = [&](double (&p)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      for (int o = 32; o > 0; o >>= 1) p[j] += __shfl_xor(p[j], o, 64);
    __syncthreads();
    if (lane == 0)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[wave + 4 * j] = p[j];
    __syncthreads();
    double t = 0.0;
    for (int w = 0; w < 16; ++w) t += red[w];
    return t;
  };
  double part[4];
  float v[kNormRegs];
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    load(j, v);
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k)
      if (tid + 256 * j + 1024 * k < count) s += (double)v[k];
    part[j] = s;
  }
  const double mean = reduce(part) / count;
  const float mean_f = (float)mean;
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    load(j, v);
    double ss = 0.0;
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k)
      if (tid + 256 * j + 1024 * k < count) {
        const double d = (double)v[k] - mean;
        ss += d * d;
      }
    part[j] = ss;
  }
  const double var = reduce(part) / (count - 1);
  const float denom = (float)sqrt(var) + 1e-6f;
  // the last pass reads a value before it (in place, y == db) overwrites it
#pragma unroll 1
  for (int j = 0; j < 4; ++j) {
    load(j, v);
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k) {
      const int i = tid + 256 * j + 1024 * k;
      if (i < count) {
        if (keep_db) db[i] = v[k];  // caller asked for the clamped dB map
        y[i] = (v[k] - mean_f) / denom;
      }
    }
  }
}

// FM (frame-major, round 6, the default; SAD_FE_FM=0 selects the staged
// form): the dB map goes out as [seg][frame][mel] -- each frame's 128 values
// are one 512-B row, so a lane stores its mel rows straight from registers --
// and fe_normalize_fm transposes it while standardising.  Without the dB
// staging (16.9 KB) a workgroup needs 52 KB of LDS, so three fit on a CU and
// each SIMD holds three waves (__launch_bounds__(256, 3): 154 VGPRs, no
// spills, the PCM prefetch kept; the step-2 twiddles and the window are
// re-read per frame).  With the per-bin recovery twiddles tabled per plan
// (fe_rtw) it runs at 1.62-1.66 ms per 2,048 segments against the staged
// form's 1.85-1.88 and round 6's first 1.97 (same box, 3 rounds,
// profiles/r06_fe_fm_ab.log).  Bit-identical to the staged form
// (tests/test_gpu_frontend_fused.py).
template <typename IT, bool FM = false>  // int16_t PCM (scaled by 1/32768, torchaudio.load normalize) or float
__global__ __launch_bounds__(256, FM ? 3 : 2) void fe_mel_db_kernel(
    const IT* __restrict__ pcm, int64_t seg_stride, const int64_t* __restrict__ seg_offs, int64_t max_off,
    int n_samples,
    int n_frames, int hop,
    const float2* __restrict__ tw1024, const float2* __restrict__ rtw, const float* __restrict__ window,
    const int* __restrict__ mel_start,
    const int* __restrict__ mel_len, const int* __restrict__ mel_off, const float* __restrict__ mel_w, int nnz,
    int n_mels, int bin_lo, int bin_hi, const int* __restrict__ lane_tab, const float* __restrict__ lane_w, int ml0,
    int ml1, float* __restrict__ out, int64_t n_seg, int xcd_map, int fuse, float top_db, float* __restrict__ map_out,
    unsigned* __restrict__ seg_cnt, float* __restrict__ seg_bmax) {
  // recovery twiddles of bins bin_lo.. (FE_RTWN of them; a wider bank reads them from global memory)
  __shared__ float2 s_rtw[FE_RTWN];
  __shared__ float2 s_buf[FE_WAVES][FE_ZBUF];
  __shared__ float2 s_tw3[64];  // W64^{q k2} at [k2][q]
  __shared__ float s_pow[FE_WAVES][FE_POW];
  __shared__ float s_db[FM ? 1 : FE_STAGE_MELS][FE_FRAMES_PER_WG + 1];
  __shared__ double s_red[16];
  __shared__ int s_last;
  // the 1024-point twiddle table (register and LDS tables' set-up, FM's step 2)
  auto twl = [&](int i) __attribute__((always_inline)) { return tw1024[i]; };

  // (the wave index through readfirstlane: the compiler then knows every
  // per-frame quantity -- t, its PCM base, the reflection test -- is uniform and
  // keeps it in SGPRs with scalar branches)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // 1-D grid.  xcd_map: workgroup L -> segment 8 (L / 8 / n_fb) + L % 8, frame
  // block (L / 8) % n_fb, so a segment's blocks share L mod 8 (one XCD);
  // else segment L / n_fb, block L % n_fb
  const int n_fb = (n_frames + FE_FRAMES_PER_WG - 1) / FE_FRAMES_PER_WG;
  const int64_t L = blockIdx.x;
  const int64_t L8 = L >> 3;
  const int64_t seg = xcd_map ? (L8 / n_fb) * 8 + (L & 7) : L / n_fb;
  const int fb = (int)(xcd_map ? L8 % n_fb : L % n_fb);
  if (seg >= n_seg) return;  // the grid is padded to a multiple of 8 segments
  // segment `seg` starts at sample seg_offs[seg] (windows of a long waveform,
  // sad_frontend_run_windows) or at seg * seg_stride
  // (offsets are clamped to [0, max_off]: a bad table cannot read out of bounds)
  int64_t x0 = seg * seg_stride;
  if (seg_offs) {
    const int64_t o = seg_offs[seg];
    x0 = o < 0 ? 0 : (o > max_off ? max_off : o);
  }
  const IT* x = pcm + x0;
  // (int16: the window carries torchaudio.load's 1/32768 -- a power of two, so
  // e * (w / 32768) rounds exactly as (e / 32768) * w)
  // staged: the mel rows by lane table (plan_create builds it when n_mels <=
  // FE_STAGE_MELS and the padded rows fit the power buffer), dB rows through LDS
  const bool staged = FM || lane_w != nullptr;
  const bool rtw_lds = bin_hi - bin_lo < FE_RTWN;  // uniform
  if (rtw_lds)
    for (int i = tid; i <= bin_hi - bin_lo; i += 256) s_rtw[i] = rtw[bin_lo + i];
  // this lane's mel rows (staged path) from the lane table: mm = the row (-1:
  // none), mk0 = its first bin - bin_lo; the power buffer's tail past bin_hi is
  // read (times a zero weight) by the padded rows: zero it once, the frames
  // never write it
  int mm[2] = {-1, -1}, mk0[2] = {0, 0};
  if (staged) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      mm[q] = lane_tab[q * 64 + lane];
      mk0[q] = lane_tab[128 + q * 64 + lane];
    }
    for (int i = bin_hi - bin_lo + 1 + FE_PWPAD + lane; i < FE_POW; i += 64) s_pow[wave][i] = 0.f;
    if (lane < FE_PWPAD) s_pow[wave][lane] = 0.f;
  }
  __syncthreads();

  // step 2's per-lane twiddles W1024^{l k1} (l = lane) in registers for all
  // frames; step 3's W64^{q k2} (q = lane & 3) as a [k2][q] LDS table
  // (FM: re-read per frame from the global table instead, 30 registers fewer)
  float2 tw2[FM ? 1 : 16];
  if constexpr (!FM) {
#pragma unroll
    for (int k = 1; k < 16; ++k) tw2[k] = twl((lane * k) & (FE_NC - 1));
  }
  if (tid < 64) s_tw3[tid] = twl((16 * (tid & 3) * (tid >> 2)) & (FE_NC - 1));  // [k2][q]
  __syncthreads();
  const int fg4 = lane >> 2, fq = lane & 3;
  const int fbr = (fq == 1 ? 2 : fq == 2 ? 1 : fq);  // bit-reversed q (output block of the lane)

  const int f_begin = fb * FE_FRAMES_PER_WG;
  const int f_end = min(n_frames, f_begin + FE_FRAMES_PER_WG);
  float2* buf = s_buf[wave];
  float* pw = s_pow[wave];
  const int pad = FE_NFFT / 2;
  // aligned pair loads need an even sample offset for every frame and pair:
  // even hop, and an even segment start (seg_stride in strided mode; this
  // segment's own offset in windows mode, where seg_stride is 0 and an odd
  // window hop gives odd starts) -- else the scalar path
  const bool pairs = ((hop & 1) == 0) && ((seg_stride & 1) == 0) && ((x0 & 1) == 0) &&
                     ((((uintptr_t)pcm) & (2 * sizeof(IT) - 1)) == 0);

  // int16 path: the next frame's PCM pairs are loaded while this frame is
  // transformed (software pipeline: a frame's HBM latency no longer stalls its
  // wave).  The prefetch address is clamped into the segment, so it is always
  // valid; frames needing reflection (the first / last ones) take the slow path.
  // (FM too since round 6: without the per-frame twiddle arithmetic the form
  // needs 154 VGPRs with the pipeline, inside its three-wave budget of 168)
  // The loop's prefetch is unconditional (a conditional one joins two paths with
  // different loads in flight, and the waitcnt pass then waits for all of them
  // at the next use of an older load): past the last frame it re-reads a clamped
  // frame, and where the pairs path is off (odd hop or offsets, a segment
  // shorter than one frame) it reads the window table instead -- never used.
  constexpr bool PREF = sizeof(IT) == 2;
  uint32_t pre[PREF ? 16 : 1];
  auto frame_inside = [&](int tt) { return pairs && tt * hop - pad >= 0 && tt * hop - pad + FE_NFFT <= n_samples; };
  const bool pf_ok = pairs && n_samples >= FE_NFFT;
  const IT* pfx = pf_ok ? x : (const IT*)window;  // the window table: 2,048 floats, at least 4 KB
  auto prefetch = [&](int tt) __attribute__((always_inline)) {
    if constexpr (PREF) {
      int b0 = tt * hop - pad;
      b0 = b0 < 0 ? 0 : (b0 + FE_NFFT > n_samples ? (n_samples - FE_NFFT) & ~1 : b0);
      b0 = (b0 < 0 || !pf_ok) ? 0 : b0;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = lane + 64 * (q & 3) + 256 * (q >> 2);
        pre[q] = *(const uint32_t*)(pfx + b0 + 2 * m);
      }
    }
  };
  prefetch(f_begin + wave);

  for (int t = f_begin + wave; t < f_end; t += FE_WAVES) {
    // FM: an opaque zero per frame keeps the window and twiddle loads inside
    // the loop (hoisted, they held 60 VGPRs across it and spilled)
    int oz = 0;
    if constexpr (FM) asm volatile("v_mov_b32 %0, 0" : "=v"(oz));
    float2 x16[16];  // z[lane + 64 t'], t' = b + 4 r
    // ---- pass 0 input: z[m] = (y[2m], y[2m+1]) windowed, m = j + 256 r; one
    // 2-sample load per lane (coalesced) where the frame needs no reflection
    const int base = t * hop - pad;
    const bool inside = frame_inside(t);
    float2 wvs[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) wvs[q] = *(const float2*)(window + oz + 2 * (lane + 64 * (q & 3) + 256 * (q >> 2)));
    // (one uniform branch around all 16 pairs: per-pair lane masks made the
    // waitcnt pass wait for every load in flight, the next frame's prefetch
    // included, at the first pair)
    // (float PCM keeps the per-pair branch: hoisted, its 16 pair loads spill)
    // sample indices of pair q of a frame that needs reflection (center=True
    // reflect padding at both ends of the segment)
    auto refl = [&](int q, int& i0, int& i1) __attribute__((always_inline)) {
      const int m = lane + 64 * (q & 3) + 256 * (q >> 2);
      i0 = base + 2 * m;
      i1 = i0 + 1;
      i0 = i0 < 0 ? -i0 : i0;
      i0 = i0 >= n_samples ? 2 * (n_samples - 1) - i0 : i0;
      i1 = i1 < 0 ? -i1 : i1;
      i1 = i1 >= n_samples ? 2 * (n_samples - 1) - i1 : i1;
    };
    if constexpr (PREF) {
      // a frame needing reflection packs its pairs into the prefetch
      // registers, so both kinds of frame share one conversion (two arms each
      // converting were merged below the join by 16 register copies)
      if (!inside) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          int i0, i1;
          refl(q, i0, i1);
          pre[PREF ? q : 0] = (uint32_t)(uint16_t)x[i0] | ((uint32_t)(uint16_t)x[i1] << 16);
        }
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t u = pre[PREF ? q : 0];
        x16[q] = make_float2((float)(short)(u & 0xFFFF) * wvs[q].x, (float)(short)(u >> 16) * wvs[q].y);
      }
    } else {  // float PCM
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (inside) {
          const float2 f = *(const float2*)(x + base + 2 * (lane + 64 * (q & 3) + 256 * (q >> 2)));
          x16[q] = make_float2(f.x * wvs[q].x, f.y * wvs[q].y);
        } else {
          int i0, i1;
          refl(q, i0, i1);
          x16[q] = make_float2((float)x[i0] * wvs[q].x, (float)x[i1] * wvs[q].y);
        }
      }
    }
    // ---- four-step FFT, N = 16 x 64: Z[k1 + 16 k2] = sum_l W64^{l k2} W1024^{l k1}
    // sum_t z[l + 64 t] W16^{t k1}.  Step 1 (16-point DFT over t) and its twiddle
    // in registers; ONE LDS transpose (XOR-swizzled: conflict-free both ways);
    // step 3's 64-point DFTs as 4 lanes x 16 registers: a 16-point DFT in
    // registers, twiddle, then a 4-point DFT across the lanes of a quad (DPP).
    dft16(x16);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1)
      x16[fe_p16(k1)] = cmul(x16[fe_p16(k1)], FM ? tw1024[oz + ((lane * k1) & (FE_NC - 1))] : tw2[FM ? 0 : k1]);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) buf[k1 * 64 + (lane ^ (4 * k1))] = x16[fe_p16(k1)];
    // the next frame's PCM, into the registers this frame's pairs left (after
    // the windowing's last use and its path join: no copies, and no wait on
    // these loads before the next frame)
    prefetch(t + FE_WAVES);
    wave_lds_sync();
    // lane (g, q) = (lane >> 2, lane & 3): B[l = q + 4 s][k1 = g], s = 0..15
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) x16[s2] = buf[fg4 * 64 + ((fq + 4 * s2) ^ (4 * fg4))];
    wave_lds_sync();
    dft16(x16);
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
      float2 d = x16[fe_p16(k2)];
      if (k2 > 0) d = cmul(d, s_tw3[4 * k2 + fq]);
      // 4-point DFT over q across the quad: radix-2 stages with partners q^2, q^1
      const float px = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d.x), 0x4E, 0xF, 0xF, true));
      const float py = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(d.y), 0x4E, 0xF, 0xF, true));
      float2 u = fq < 2 ? make_float2(d.x + px, d.y + py) : make_float2(px - d.x, py - d.y);
      if (fq == 3) u = make_float2(u.y, -u.x);  // x W4^1 = -i
      const float qx = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(u.x), 0xB1, 0xF, 0xF, true));
      const float qy = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(u.y), 0xB1, 0xF, 0xF, true));
      // lane (g, q) holds Z[g + 16 k2 + 256 br(q)]
      buf[fe_zslot(fg4 + 16 * k2 + 256 * fbr)] =
          (fq & 1) == 0 ? make_float2(u.x + qx, u.y + qy) : make_float2(qx - u.x, qy - u.y);
    }
    wave_lds_sync();
    // ---- real-spectrum recovery + power for bins [bin_lo, bin_hi]
    // Every lane runs the same trip count (the last round's surplus lanes
    // compute a clamped bin and do not store it), so no lane finishes the loop
    // in a one-active-lane remainder.  (Round 6 first blamed that remainder for
    // a wrong bin 705 beside the stem; the cause was the packed-FP32
    // instructions, which the library no longer uses: csrc/Makefile NOPK)
    const int n_kit = (bin_hi - bin_lo + 64) / 64;
    // e^{-2 pi i k / 2048} of bin k (fe_rtw, tabled per plan): from LDS, or
    // from global memory for a bank wider than FE_RTWN bins (two loop copies:
    // a select between the two loads issued both)
    // FAST (twiddles in LDS, bins 1..1023: no wrap of k or N/2 - k): bin k + 64
    // reads slots 65 on / 65 back and twiddle / power slots 64 on, so every
    // address is a per-lane base plus a constant; lanes past bin_hi read
    // unclamped (garbage, in or past the workgroup's LDS: zero) and store nothing
    auto recover = [&](auto from_lds, auto fast) __attribute__((always_inline)) {
      constexpr bool FAST = decltype(fast)::value;
      const float2* pa = buf + fe_zslot(bin_lo + lane);
      const float2* pb = buf + fe_zslot(FE_NC - bin_lo - lane);
      for (int it = 0; it < n_kit; ++it) {
        const int k_raw = bin_lo + lane + 64 * it;
        const int k = FAST ? k_raw : (k_raw <= bin_hi ? k_raw : bin_hi);
        const float2 A = FAST ? pa[65 * it] : buf[fe_zslot(k & (FE_NC - 1))];
        const float2 Bc = FAST ? pb[-65 * it] : buf[fe_zslot((FE_NC - k) & (FE_NC - 1))];
        const float2 B = make_float2(Bc.x, -Bc.y);  // conj(Z[N/2-k])
        // 2 X_k = (A + B) - i W (A - B): the recovery's 1/2 factors are left
        // out (exact powers of two), so pw holds 4 |X_k|^2 and the mel weights
        // carry the 1/4 -- the same bits as before, four VALU fewer per bin
        // (the fused operations spelled out as the compiler formed them with
        // the halvings in place: W O with O = -i (A - B), then each half-sum
        // added -- so every rounding is the earlier one's, times 2)
        const float2 E = make_float2(A.x + B.x, A.y + B.y);
        const float2 D = make_float2(A.x - B.x, A.y - B.y);
        const float ox = D.y, oy = -D.x;  // O = -i (A - B)
        const float2 w2 = decltype(from_lds)::value ? s_rtw[k - bin_lo] : rtw[k];
        const float wy_oy = w2.y * oy, wy_ox = w2.y * ox;
        const float wox = __builtin_fmaf(w2.x, ox, -wy_oy), woy = __builtin_fmaf(w2.x, oy, wy_ox);
        const float re = E.x + wox, im = E.y + woy;
        const float im2 = im * im;
        if (k_raw <= bin_hi) pw[k - bin_lo + FE_PWPAD] = __builtin_fmaf(re, re, im2);
      }
    };
    if (rtw_lds && bin_lo >= 1 && bin_hi < FE_NC)
      recover(std::true_type{}, std::true_type{});
    else if (rtw_lds)
      recover(std::true_type{}, std::false_type{});
    else
      recover(std::false_type{}, std::false_type{});
    wave_lds_sync();
    if (staged) {
      // every lane runs ml0 + ml1 steps (no divergence, independent loads):
      // zero weights, the row's bins in order, zero weights -- the same sums as
      // the CSR loop, bit for bit; each 32-lane group's window starts are
      // distinct mod 32, so every step's ds_read_b32 is bank-conflict-free
      // (plan_create's matching)
      const float* pa = pw + mk0[0];
      const float* pb = pw + mk0[1];
      const float* wa = lane_w + lane;
      const float* wb = lane_w + ml0 * 64 + lane;
      float a0 = 0.f, a1 = 0.f;
#pragma unroll 4
      for (int i = 0; i < ml0; ++i) a0 = fmaf(pa[i], wa[i * 64], a0);
#pragma unroll 4
      for (int i = 0; i < ml1; ++i) a1 = fmaf(pb[i], wb[i * 64], a1);
      if constexpr (FM) {  // frame-major: this frame's row of n_mels values
        float* row = out + (seg * n_frames + t) * n_mels;
        if (mm[0] >= 0) row[mm[0]] = 10.0f * log10f(fmaxf(a0, 1e-10f));
        if (mm[1] >= 0) row[mm[1]] = 10.0f * log10f(fmaxf(a1, 1e-10f));
      } else {
        if (mm[0] >= 0) s_db[mm[0]][t - f_begin] = 10.0f * log10f(fmaxf(a0, 1e-10f));
        if (mm[1] >= 0) s_db[mm[1]][t - f_begin] = 10.0f * log10f(fmaxf(a1, 1e-10f));
      }
    } else {
      for (int m = lane; m < n_mels; m += 64) {
        const int k0 = mel_start[m], len = mel_len[m], off = mel_off[m];
        float acc = 0.f;
        for (int q = 0; q < len; ++q) acc = fmaf(pw[k0 + q - bin_lo + FE_PWPAD], mel_w[off + q], acc);
        out[(seg * n_mels + m) * n_frames + t] = 10.0f * log10f(fmaxf(acc, 1e-10f));
      }
    }
    wave_lds_sync();  // pw / buf are rewritten by the next frame
  }
  if (!FM && staged) {
    // [n_mels][frames of this block] -> rows of up to 32 consecutive frames
    __syncthreads();
    const int nf = f_end - f_begin;
    for (int i = tid; i < n_mels * FE_FRAMES_PER_WG; i += 256) {
      const int m = i / FE_FRAMES_PER_WG, f = i - m * FE_FRAMES_PER_WG;
      if (f < nf) {
        float* o = out + (seg * n_mels + m) * n_frames + f_begin + f;
        if (fuse == 2)  // agent-scope store: at the coherence point when it completes
          __hip_atomic_store(o, s_db[m][f], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
          *o = s_db[m][f];
      }
    }
    // (fuse is a kernel argument, not a template parameter: the same binary
    // runs both forms, so their dB maps are bit-identical)
    if (fuse) {
      // the block's maximum, then publish (release) and count the arrival
      float bm = -INFINITY;
      for (int i = tid; i < n_mels * FE_FRAMES_PER_WG; i += 256) {
        const int m = i / FE_FRAMES_PER_WG, f = i - m * FE_FRAMES_PER_WG;
        if (f < nf) bm = fmaxf(bm, s_db[m][f]);
      }
      for (int o = 32; o > 0; o >>= 1) bm = fmaxf(bm, __shfl_xor(bm, o, 64));
      float* s_bm = s_pow[0];  // the frames are done with the power buffers
      __syncthreads();
      if (lane == 0) s_bm[wave] = bm;
      __syncthreads();
      if (tid == 0)
        __hip_atomic_store(seg_bmax + seg * n_fb + fb, fmaxf(fmaxf(s_bm[0], s_bm[1]), fmaxf(s_bm[2], s_bm[3])),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // fuse 1: agent-scope release (L2 write-back); fuse 2: the tile went out
      // by agent-scope stores, so waiting for their completion is the release
      if (fuse == 2)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      else
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __syncthreads();
      if (tid == 0)
        s_last = __hip_atomic_fetch_add(seg_cnt + seg, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                 (unsigned)(n_fb - 1);
      __syncthreads();
      if (!s_last) return;
      if (fuse != 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (tid == 0) __hip_atomic_store(seg_cnt + seg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int count = n_mels * n_frames;
      float* db = out + seg * count;
      float* y = map_out + seg * count;
      if (fuse == 2)
        fe_standardise_segment<true>(db, db != y, y, count, seg_bmax + seg * n_fb, n_fb, top_db, s_red);
      else
        fe_standardise_segment<false>(db, db != y, y, count, seg_bmax + seg * n_fb, n_fb, top_db, s_red);
    }
  }
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

__global__ __launch_bounds__(1024) void fe_normalize_kernel(float* db_io, int count,
                                                             float top_db, float* map_out) {
  __shared__ double red[16];
  __shared__ float redf[16];
  const int64_t seg = blockIdx.x;
  float* x = db_io + seg * count;
  float* y = map_out + seg * count;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (count <= kNormRegs * (int)blockDim.x) {
    // one HBM read: the segment's values stay in registers (32 per thread for
    // the 128 x 251 map); every reduction visits them in the same per-thread
    // order as the multi-pass loop below, so the results are identical
    float v[kNormRegs];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k) {
      const int i = tid + k * (int)blockDim.x;
      v[k] = i < count ? x[i] : -INFINITY;
      mx = fmaxf(mx, v[k]);
    }
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    mx = redf[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) mx = fmaxf(mx, redf[i]);
    const float floor_db = top_db >= 0.f ? mx - top_db : -INFINITY;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k) {
      const int i = tid + k * (int)blockDim.x;
      if (i < count) {
        v[k] = fmaxf(v[k], floor_db);
        if (x != y) x[i] = v[k];  // caller asked for the clamped dB map
        s += (double)v[k];
      }
    }
    const double mean = block_sum_d(s, red) / count;
    const float mean_f = (float)mean;
    double ss = 0.0;
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k) {
      const int i = tid + k * (int)blockDim.x;
      if (i < count) {
        const double d = (double)v[k] - mean;
        ss += d * d;
      }
    }
    const double var = block_sum_d(ss, red) / (count - 1);
    const float denom = (float)sqrt(var) + 1e-6f;
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k) {
      const int i = tid + k * (int)blockDim.x;
      if (i < count) y[i] = (v[k] - mean_f) / denom;
    }
    return;
  }
  float mx = -INFINITY;
  for (int i = tid; i < count; i += blockDim.x) mx = fmaxf(mx, x[i]);
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) redf[wave] = mx;
  __syncthreads();
  mx = redf[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) mx = fmaxf(mx, redf[i]);
  const float floor_db = top_db >= 0.f ? mx - top_db : -INFINITY;
  double s = 0.0;
  for (int i = tid; i < count; i += blockDim.x) {
    float v = fmaxf(x[i], floor_db);
    if (x != y) x[i] = v;  // caller asked for the clamped dB map
    s += (double)v;
  }
  const double mean = block_sum_d(s, red) / count;
  const float mean_f = (float)mean;
  double ss = 0.0;
  for (int i = tid; i < count; i += blockDim.x) {
    const double d = (double)fmaxf(x[i], floor_db) - mean;
    ss += d * d;
  }
  const double var = block_sum_d(ss, red) / (count - 1);
  const float denom = (float)sqrt(var) + 1e-6f;
  for (int i = tid; i < count; i += blockDim.x) {
    const float v = fmaxf(x[i], floor_db);
    y[i] = (v - mean_f) / denom;
  }
}

// fe_normalize for the frame-major dB map of fe_mel_db<IT, true>: the same
// statistics (max -> top-db clamp -> float64 mean / unbiased variance), then the
// clamped dB map (db_out, optional) and the standardised map (map_out) written
// mel-major [n_mels][n_frames] through a transpose in LDS (count floats of
// dynamic LDS: one workgroup per CU, coalesced reads and writes).  In place:
// every value is in registers before the first store (the reductions' barriers).
__global__ __launch_bounds__(1024) void fe_normalize_fm_kernel(float* db_io, int n_mels, int n_frames, float top_db,
                                                                float* db_out, float* map_out) {
  extern __shared__ __attribute__((aligned(16))) float s_t[];
  __shared__ double red[16];
  __shared__ float redf[16];
  const int count = n_mels * n_frames;
  const int64_t seg = blockIdx.x;
  const float* x = db_io + seg * count;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float v[kNormRegs];
  float mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < kNormRegs; ++k) {
    const int i = tid + k * 1024;
    v[k] = i < count ? x[i] : -INFINITY;
    mx = fmaxf(mx, v[k]);
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) redf[wave] = mx;
  __syncthreads();
  mx = redf[0];
  for (int i = 1; i < 16; ++i) mx = fmaxf(mx, redf[i]);
  const float floor_db = top_db >= 0.f ? mx - top_db : -INFINITY;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < kNormRegs; ++k) {
    if (tid + k * 1024 < count) {
      v[k] = fmaxf(v[k], floor_db);
      s += (double)v[k];
    }
  }
  const double mean = block_sum_d(s, red) / count;
  const float mean_f = (float)mean;
  double ss = 0.0;
#pragma unroll
  for (int k = 0; k < kNormRegs; ++k)
    if (tid + k * 1024 < count) {
      const double d = (double)v[k] - mean;
      ss += d * d;
    }
  const double var = block_sum_d(ss, red) / (count - 1);
  const float denom = (float)sqrt(var + 0.0) + 1e-6f;
  // frame-major i = frame * n_mels + mel -> mel-major mel * n_frames + frame
  // (frame / mel of i = tid + 1024 k stepped from k - 1's by the uniform
  // quotient and remainder of 1024 / n_mels: one integer division per thread)
  // (the LDS slot m * n_frames + f steps the same way: uniform increments)
  const int dq = 1024 / n_mels, dr = 1024 - dq * n_mels;
  const int dslot = dr * n_frames + dq, wrap = n_mels * n_frames - 1;
  // (v - mean) / denom, correctly rounded without a division per value:
  // Markstein's step from the correctly rounded reciprocal (q = x y within an
  // ulp of x / denom, the FMA residual exact, q + r y rounds to x / denom; no
  // overflow or subnormal range here: |x| >= ulp of a dB value or 0, denom >= 1e-6).
  // The step turns x = -0 into +0, so the sign is x's (denom > 0).  A CPU check
  // of 4e8 sampled pairs found no other difference outside subnormal quotients.
  const float rden = 1.0f / denom;
  auto put = [&](float* dst, bool std) __attribute__((always_inline)) {
    const int f0 = tid / n_mels, m0 = tid - f0 * n_mels;
    int m = m0, slot = m0 * n_frames + f0;
#pragma unroll
    for (int k = 0; k < kNormRegs; ++k) {
      if (tid + k * 1024 < count) {
        if (std) {
          const float xm = v[k] - mean_f;
          const float q0 = xm * rden;
          s_t[slot] = __builtin_copysignf(__builtin_fmaf(__builtin_fmaf(-q0, denom, xm), rden, q0), xm);
        } else {
          s_t[slot] = v[k];
        }
      }
      slot += dslot;
      m += dr;
      if (m >= n_mels) {
        m -= n_mels;
        slot -= wrap;
      }
    }
    __syncthreads();
    float* o = dst + seg * count;
    for (int i = tid; i < count; i += 1024) o[i] = s_t[i];
    __syncthreads();
  };
  if (db_out) put(db_out, false);
  put(map_out, true);
}

// Bilinear resize, align_corners=False (torchvision Resize on tensors; antialias
// is a no-op for upsampling).  One thread per output pixel.
template <typename OT>
__global__ void resize_kernel(const float* __restrict__ in, int h, int w, int oh, int ow,
                              OT* __restrict__ out, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int ox = i % ow;
  const int oy = (i / ow) % oh;
  const int64_t n = i / ((int64_t)ow * oh);
  const float sh = (float)h / oh, sw = (float)w / ow;
  float fy = sh * (oy + 0.5f) - 0.5f;
  fy = fy < 0.f ? 0.f : fy;
  float fx = sw * (ox + 0.5f) - 0.5f;
  fx = fx < 0.f ? 0.f : fx;
  const int y0 = min((int)floorf(fy), h - 1), x0 = min((int)floorf(fx), w - 1);
  const int y1 = min(y0 + 1, h - 1), x1 = min(x0 + 1, w - 1);
  const float ly = fminf(fmaxf(fy - y0, 0.f), 1.f), lx = fminf(fmaxf(fx - x0, 0.f), 1.f);
  const float* p = in + n * h * w;
  const float v = (1.f - ly) * ((1.f - lx) * p[y0 * w + x0] + lx * p[y0 * w + x1]) +
                  ly * ((1.f - lx) * p[y1 * w + x0] + lx * p[y1 * w + x1]);
  if constexpr (sizeof(OT) == 2)
    out[i] = f2bf(v);
  else
    out[i] = v;
}

// ---- host: mel filterbank (torchaudio melscale_fbanks, htk), float64 then f32
static std::vector<float> mel_fbank(int n_freqs, double f_min, double f_max, int n_mels, int sr, bool slaney) {
  auto hz2mel = [](double f) { return 2595.0 * log10(1.0 + f / 700.0); };
  auto mel2hz = [](double m) { return 700.0 * (pow(10.0, m / 2595.0) - 1.0); };
  std::vector<double> fpts(n_mels + 2);
  const double mmin = hz2mel(f_min), mmax = hz2mel(f_max);
  for (int i = 0; i < n_mels + 2; ++i) fpts[i] = mel2hz(mmin + (mmax - mmin) * i / (n_mels + 1));
  std::vector<float> fb((size_t)n_freqs * n_mels, 0.f);
  for (int k = 0; k < n_freqs; ++k) {
    const double f = (double)(sr / 2) * k / (n_freqs - 1);
    for (int m = 0; m < n_mels; ++m) {
      const double down = (f - fpts[m]) / (fpts[m + 1] - fpts[m]);
      const double up = (fpts[m + 2] - f) / (fpts[m + 2] - fpts[m + 1]);
      double v = fmax(0.0, fmin(down, up));
      if (slaney) v *= 2.0 / (fpts[m + 2] - fpts[m]);
      fb[(size_t)k * n_mels + m] = (float)v;
    }
  }
  return fb;
}

}  // namespace sad

using namespace sad;

struct sad_frontend_plan : sad::FrontendPlan {};

// fb: [n_fft / 2 + 1][n_mels] fp32, the mel filterbank the plan projects on
// SAD_FE_FUSED: 0 the two-kernel form (fe_mel_db + fe_normalize); 1 fused,
// agent-scope release / acquire fences; 2 fused, the tiles stored and re-read
// at agent scope (sc1) with no cache write-back / invalidate
static int fe_fused() {
  static const int v = [] {
    const char* e = getenv("SAD_FE_FUSED");
    return e ? atoi(e) : 0;
  }();
  return v;
}

static int frontend_plan_build(const sad_frontend_cfg* cfg, const float* fb_in, sad_frontend_plan** out) {
  SAD_REQUIRE(cfg && out, "null cfg/out");
  SAD_REQUIRE(cfg->n_fft == FE_NFFT, "only n_fft = 2048 is supported");
  SAD_REQUIRE(cfg->hop_length > 0 && cfg->n_mels > 0 && cfg->n_mels <= 1024, "hop/n_mels");
  SAD_REQUIRE(cfg->n_samples > FE_NFFT / 2, "n_samples must exceed n_fft/2 (reflect pad)");
  const int n_freqs = FE_NFFT / 2 + 1;
  std::vector<float> fb = fb_in ? std::vector<float>(fb_in, fb_in + (size_t)n_freqs * cfg->n_mels)
                                : mel_fbank(n_freqs, cfg->f_min, cfg->f_max, cfg->n_mels, cfg->sample_rate,
                                            cfg->norm_slaney != 0);
  for (float v : fb) SAD_REQUIRE(v >= 0.f && v < 1e30f, "filterbank weights must be finite and >= 0");
  auto* p = new sad_frontend_plan();
  p->cfg = *cfg;
  p->n_frames = 1 + cfg->n_samples / cfg->hop_length;
  (void)hipGetDevice(&p->device);
  std::vector<int> st(cfg->n_mels), ln(cfg->n_mels), off(cfg->n_mels);
  std::vector<float> w;
  int lo = n_freqs, hi = -1;
  for (int m = 0; m < cfg->n_mels; ++m) {
    int a = -1, b = -1;
    for (int k = 0; k < n_freqs; ++k)
      if (fb[(size_t)k * cfg->n_mels + m] != 0.f) {
        if (a < 0) a = k;
        b = k;
      }
    if (a < 0) a = b = 0;  // empty filter: contributes 0 (weight 0 at bin 0)
    st[m] = a;
    ln[m] = b - a + 1;
    off[m] = (int)w.size();
    // x 1/4: the kernels' power is 4 |X_k|^2 (the real-spectrum recovery's two
    // halvings dropped); both factors are powers of two, so every product and
    // sum of the projection rounds exactly as before
    for (int k = a; k <= b; ++k) w.push_back(0.25f * fb[(size_t)k * cfg->n_mels + m]);
    lo = std::min(lo, a);
    hi = std::max(hi, b);
  }
  p->bin_lo = lo;
  p->bin_hi = hi;
  p->nnz = (int)w.size();
  // lane table of the staged mel projection: the shorter half of the rows on
  // q = 0, the longer on q = 1, each run over a window of its longest row's
  // length ml[q].  A lane reads pw[start + i], i < ml[q], with one ds_read_b32
  // per step; its 32-lane group (the instruction's bank group, bank = dword
  // mod 32) is conflict-free when the group's window starts are distinct mod 32.
  // Rows sorted by start bin alternate between the two groups, and each row's
  // window may start d bins before the row (d <= ml[q] - len, zero weights in
  // front; the power buffer has FE_PWPAD zero slots before bin_lo): a bipartite
  // matching of rows to residues picks the d's.  For the reference's banks it
  // matches every row (bank-conflict cycles of the projection 2.4x -> 1x, CPU
  // model); an unmatched row keeps d = 0.  Leading zero products leave the fp32
  // sums bit-identical.
  std::vector<int> lane_tab(256, 0);
  std::vector<float> lane_w;
  bool lanes_ok = cfg->n_mels <= FE_STAGE_MELS && hi - lo + FE_PWPAD < FE_POW;
  if (lanes_ok) {
    std::vector<int> ord(cfg->n_mels);
    for (int m = 0; m < cfg->n_mels; ++m) ord[m] = m;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return ln[x] < ln[y]; });
    const int nA = std::min(cfg->n_mels, 64);
    int ml[2] = {0, 0};
    std::vector<int> lane_d(128, 0);
    const char* me = getenv("SAD_FE_MATCH");  // 0: round 4's greedy split (A/B)
    const bool match = !(me && atoi(me) == 0);
    for (int q = 0; q < 2; ++q) {
      std::vector<int> rows(q == 0 ? ord.begin() : ord.begin() + nA, q == 0 ? ord.begin() + nA : ord.end());
      for (int m : rows) ml[q] = std::max(ml[q], ln[m]);
      std::stable_sort(rows.begin(), rows.end(), [&](int x, int y) { return st[x] < st[y]; });
      std::vector<int> grps[2];
      if (match) {
        for (size_t k = 0; k < rows.size(); ++k) grps[k & 1].push_back(rows[k]);
      } else {  // round 4: longest first into the half with fewer same-bank starts
        std::stable_sort(rows.begin(), rows.end(), [&](int x, int y) { return ln[x] > ln[y]; });
        for (int m : rows) {
          int best = -1, bc = 1 << 30;
          for (int g = 0; g < 2; ++g) {
            if ((int)grps[g].size() >= 32) continue;
            int c = 0;
            for (int x : grps[g]) c += ((st[x] - lo) % 32 == (st[m] - lo) % 32) && st[x] != st[m];
            if (c < bc) bc = c, best = g;
          }
          grps[best].push_back(m);
        }
      }
      for (int g = 0; g < 2; ++g) {
        const std::vector<int>& grp = grps[g];
        // augmenting-path matching: row j -> residue (st - lo + PAD - d) mod 32
        const int n = (int)grp.size();
        std::vector<int> own(32, -1);
        auto dmax = [&](int j) { return std::min(ml[q] - ln[grp[j]], st[grp[j]] - lo + FE_PWPAD); };
        auto base = [&](int j) { return st[grp[j]] - lo + FE_PWPAD; };
        std::vector<char> seen(32);
        std::function<bool(int)> aug = [&](int j) {
          for (int d = 0; d <= dmax(j); ++d) {
            const int r = (base(j) - d) & 31;
            if (seen[r]) continue;
            seen[r] = 1;
            if (own[r] < 0 || aug(own[r])) {
              own[r] = j;
              return true;
            }
          }
          return false;
        };
        for (int j = 0; j < n && match; ++j) {
          std::fill(seen.begin(), seen.end(), 0);
          aug(j);
        }
        std::vector<int> dsel(n, 0);  // unmatched rows: d = 0
        for (int r = 0; r < 32; ++r)
          if (own[r] >= 0) dsel[own[r]] = (base(own[r]) - r) & 31;  // the least d with that residue
        for (int j = 0; j < n; ++j) {
          const int l = 32 * g + j;
          lane_tab[q * 64 + l] = grp[j];
          lane_tab[128 + q * 64 + l] = base(j) - dsel[j];
          lane_d[q * 64 + l] = dsel[j];
        }
        for (int j = n; j < 32; ++j) {
          lane_tab[q * 64 + 32 * g + j] = -1;
          lane_tab[128 + q * 64 + 32 * g + j] = 0;
        }
      }
    }
    for (int q = 0; q < 2 && lanes_ok; ++q)
      for (int l = 0; l < 64; ++l) lanes_ok = lanes_ok && lane_tab[128 + q * 64 + l] + ml[q] <= FE_POW;
    if (lanes_ok) {
      lane_w.assign((size_t)(ml[0] + ml[1]) * 64, 0.f);
      for (int q = 0; q < 2; ++q)
        for (int l = 0; l < 64; ++l) {
          const int m = lane_tab[q * 64 + l];
          if (m < 0) continue;
          const int d = lane_d[q * 64 + l];
          for (int i = 0; i < ln[m]; ++i) lane_w[(size_t)((q ? ml[0] : 0) + d + i) * 64 + l] = w[off[m] + i];
        }
      p->ml0 = ml[0];
      p->ml1 = ml[1];
    }
  }
  std::vector<float2> tw(FE_NC), tw2(FE_NC + 1);
  for (int m = 0; m < FE_NC; ++m) {
    const double a = -2.0 * M_PI * m / FE_NC;
    tw[m] = make_float2((float)cos(a), (float)sin(a));
  }
  for (int k = 0; k <= FE_NC; ++k) {
    const double a = -2.0 * M_PI * k / FE_NFFT;
    tw2[k] = make_float2((float)cos(a), (float)sin(a));
  }
  std::vector<float> win(FE_NFFT);
  for (int n = 0; n < FE_NFFT; ++n) win[n] = (float)(0.5 - 0.5 * cos(2.0 * M_PI * n / FE_NFFT));
#define UP(dst, vec)                                                                   \
  SAD_CHECK_HIP(hipMalloc((void**)&dst, vec.size() * sizeof(vec[0])));                 \
  SAD_CHECK_HIP(hipMemcpy(dst, vec.data(), vec.size() * sizeof(vec[0]), hipMemcpyHostToDevice));
  UP(p->d_tw1024, tw);
  UP(p->d_tw2048, tw2);
  UP(p->d_window, win);
  std::vector<float> win16(FE_NFFT);
  for (int n = 0; n < FE_NFFT; ++n) win16[n] = win[n] * (1.0f / 32768.0f);  // exact: a power of two
  UP(p->d_window_s16, win16);
  SAD_CHECK_HIP(hipMalloc((void**)&p->d_rtw, (FE_NC + 1) * sizeof(float2)));
  hipLaunchKernelGGL(fe_rtw_kernel, dim3((FE_NC + 256) / 256), dim3(256), 0, 0, p->d_tw1024, p->d_rtw);
  SAD_CHECK_HIP(hipGetLastError());
  SAD_CHECK_HIP(hipStreamSynchronize(nullptr));
  UP(p->d_mel_start, st);
  UP(p->d_mel_len, ln);
  UP(p->d_mel_off, off);
  UP(p->d_mel_w, w);
  if (lanes_ok) {
    UP(p->d_lane_tab, lane_tab);
    UP(p->d_lane_w, lane_w);
  }
  if (lanes_ok && fe_fused()) {
    // only the one-kernel form (SAD_FE_FUSED=1/2, off by default) needs the
    // fused normalisation's counters (zero; each launch leaves them zero) and
    // block maxima, for one launch chunk; the default plan stays immutable
    const int n_fb = (p->n_frames + FE_FRAMES_PER_WG - 1) / FE_FRAMES_PER_WG;
    std::vector<unsigned> zeros(FE_CHUNK, 0u);
    UP(p->d_seg_cnt, zeros);
    SAD_CHECK_HIP(hipMalloc((void**)&p->d_seg_bmax, (size_t)FE_CHUNK * n_fb * sizeof(float)));
  }
#undef UP
  *out = p;
  return SAD_OK;
}

extern "C" int sad_frontend_plan_create(const sad_frontend_cfg* cfg, sad_frontend_plan** out) {
  return frontend_plan_build(cfg, nullptr, out);
}

extern "C" int sad_frontend_plan_create_fb(const sad_frontend_cfg* cfg, const float* fbank, sad_frontend_plan** out) {
  SAD_REQUIRE(fbank, "null filterbank");
  return frontend_plan_build(cfg, fbank, out);
}

extern "C" int sad_frontend_plan_destroy(sad_frontend_plan* p) {
  if (!p) return SAD_OK;
  (void)hipFree(p->d_tw1024);
  (void)hipFree(p->d_tw2048);
  (void)hipFree(p->d_window);
  (void)hipFree(p->d_window_s16);
  (void)hipFree(p->d_rtw);
  (void)hipFree(p->d_mel_start);
  (void)hipFree(p->d_mel_len);
  (void)hipFree(p->d_mel_off);
  (void)hipFree(p->d_mel_w);
  if (p->d_lane_tab) (void)hipFree(p->d_lane_tab);
  if (p->d_lane_w) (void)hipFree(p->d_lane_w);
  if (p->d_seg_cnt) (void)hipFree(p->d_seg_cnt);
  if (p->d_seg_bmax) (void)hipFree(p->d_seg_bmax);
  delete p;
  return SAD_OK;
}

extern "C" int sad_frontend_frames(const sad_frontend_plan* p, int32_t* n) {
  SAD_REQUIRE(p && n, "null");
  *n = p->n_frames;
  return SAD_OK;
}

// SAD_FE_XCD_MAP=1: the XCD-aware block order (a segment's blocks on one XCD)
static int fe_xcd_map() {
  static const int v = [] {
    const char* e = getenv("SAD_FE_XCD_MAP");
    return e ? atoi(e) : 0;
  }();
  return v;
}

// SAD_FE_FM (default 1): the frame-major form (three workgroups per CU; see
// fe_mel_db_kernel); 0: the staged form (dB rows through LDS, two per CU)
static int fe_fm() {
  static const int v = [] {
    const char* e = getenv("SAD_FE_FM");
    return e ? atoi(e) : 1;
  }();
  return v;
}

template <typename IT>
static int frontend_run(const sad_frontend_plan* p, const IT* pcm, int64_t n_seg, int64_t seg_stride,
                        const int64_t* seg_offs, int64_t max_off, float* out_db, float* out_map,
                        void* stream) {
  SAD_REQUIRE(p, "null plan");
  SAD_REQUIRE(n_seg >= 0, "n_seg < 0");
  SAD_REQUIRE(out_map, "out_map is required");
  SAD_REQUIRE(seg_offs || seg_stride >= p->cfg.n_samples, "seg_stride < n_samples");
  if (n_seg == 0) return SAD_OK;
  SAD_REQUIRE(pcm, "null pcm");
  hipStream_t s = (hipStream_t)stream;
  float* dbbuf = out_db ? out_db : out_map;
  const int n_fb = (p->n_frames + FE_FRAMES_PER_WG - 1) / FE_FRAMES_PER_WG;
  const int count = p->cfg.n_mels * p->n_frames;
  const int fuse = p->d_seg_cnt != nullptr && count <= kNormRegs * 1024 ? fe_fused() : 0;
  const size_t fm_lds = (size_t)count * sizeof(float);
  const bool fm = !fuse && p->d_lane_w != nullptr && count <= kNormRegs * 1024 && fm_lds <= 150 * 1024 && fe_fm();
  if (fm) {
    static bool attr = [] {
      return hipFuncSetAttribute((const void*)fe_normalize_fm_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 150 * 1024) == hipSuccess;
    }();
    SAD_REQUIRE(attr, "fe_normalize_fm: dynamic LDS attribute");
  }
  int64_t done = 0;
  while (done < n_seg) {
    const int64_t chunk = std::min<int64_t>(FE_CHUNK, n_seg - done);
    const size_t off = (size_t)done * count;
    const int xmap = fe_xcd_map();
    const unsigned blocks = (unsigned)((xmap ? (chunk + 7) / 8 * 8 : chunk) * n_fb);
    auto kfn = fm ? fe_mel_db_kernel<IT, true> : fe_mel_db_kernel<IT, false>;
    hipLaunchKernelGGL(kfn, dim3(blocks), dim3(256), 0, s,
                       seg_offs ? pcm : pcm + done * seg_stride, seg_stride, seg_offs ? seg_offs + done : nullptr,
                       max_off, p->cfg.n_samples, p->n_frames, p->cfg.hop_length, p->d_tw1024, p->d_rtw,
                       sizeof(IT) == 2 ? p->d_window_s16 : p->d_window,
                       p->d_mel_start, p->d_mel_len, p->d_mel_off, p->d_mel_w, p->nnz, p->cfg.n_mels, p->bin_lo,
                       p->bin_hi, p->d_lane_tab, p->d_lane_w, p->ml0, p->ml1, dbbuf + off, chunk, xmap, fuse, p->cfg.top_db,
                       out_map + off, p->d_seg_cnt, p->d_seg_bmax);
    SAD_CHECK_HIP(hipGetLastError());
    if (fm) {
      hipLaunchKernelGGL(fe_normalize_fm_kernel, dim3((unsigned)chunk), dim3(1024), fm_lds, s, dbbuf + off,
                         p->cfg.n_mels, p->n_frames, p->cfg.top_db, out_db ? out_db + off : nullptr, out_map + off);
      SAD_CHECK_HIP(hipGetLastError());
    } else if (!fuse) {
      hipLaunchKernelGGL(fe_normalize_kernel, dim3((unsigned)chunk), dim3(1024), 0, s, dbbuf + off, count,
                         p->cfg.top_db, out_map + off);
      SAD_CHECK_HIP(hipGetLastError());
    }
    done += chunk;
  }
  return SAD_OK;
}

extern "C" int sad_frontend_run(const sad_frontend_plan* p, const int16_t* pcm, int64_t n_seg,
                                int64_t seg_stride, float* out_db, float* out_map, void* stream) {
  return frontend_run(p, pcm, n_seg, seg_stride, nullptr, 0, out_db, out_map, stream);
}

extern "C" int sad_frontend_run_f32(const sad_frontend_plan* p, const float* wav, int64_t n_seg,
                                    int64_t seg_stride, float* out_db, float* out_map, void* stream) {
  return frontend_run(p, wav, n_seg, seg_stride, nullptr, 0, out_db, out_map, stream);
}

extern "C" int sad_frontend_run_windows(const sad_frontend_plan* p, const float* wav, int64_t wav_len,
                                        const int64_t* offsets, int64_t n_seg, float* out_db, float* out_map,
                                        void* stream) {
  SAD_REQUIRE(p, "null plan");
  SAD_REQUIRE(wav_len >= p->cfg.n_samples, "waveform shorter than one segment");
  SAD_REQUIRE(n_seg == 0 || offsets, "null offsets");
  // the offsets live on the device (not checked here); the kernel clamps each
  // to [0, wav_len - n_samples]
  return frontend_run(p, wav, n_seg, 0, offsets, wav_len - p->cfg.n_samples, out_db, out_map, stream);
}

extern "C" int sad_resize_run(const float* map, int64_t n, int32_t h, int32_t w, int32_t oh,
                              int32_t ow, int32_t dtype, void* img, void* stream) {
  SAD_REQUIRE(h > 0 && w > 0 && oh > 0 && ow > 0 && n >= 0, "bad shape");
  SAD_REQUIRE(dtype == SAD_F32 || dtype == SAD_BF16, "dtype");
  const int64_t total = n * oh * ow;
  if (total == 0) return SAD_OK;
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (dtype == SAD_F32)
    hipLaunchKernelGGL(resize_kernel<float>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, map, h, w,
                       oh, ow, (float*)img, total);
  else
    hipLaunchKernelGGL(resize_kernel<u16>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, map, h, w,
                       oh, ow, (u16*)img, total);
  SAD_CHECK_HIP(hipGetLastError());
  return SAD_OK;
}
