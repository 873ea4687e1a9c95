/*
 * sad.h -- C ABI of libsad.so, the MI355X (gfx950) hot path of the
 * synthetic-audio-detection pipeline:
 *
 *   int16 PCM (4 s @ 32 kHz) -> STFT -> mel -> dB -> standardise      [frontend]
 *   -> bilinear 512x512 -> ResNet-18 backbone -> global avg pool        [backbone]
 *   -> N binary heads -> real-logit-averaging ensemble merge            [heads]
 *
 * The reference (TtesseractT/Synthetic-Audio-Detection @ 2025-05-23) has no
 * FFI: its hot path is Python calling torchaudio / torchvision / timm.  Each
 * entry point below names the reference interface (file:line) it replaces; the
 * Python host layer (synthetic-audio-detection_amd/sad/_lib.py) binds them with
 * ctypes, exactly as INTEGRATION.md shows.
 *
 * Conventions:
 *   - every call returns 0 on success, a negative sad_status otherwise;
 *     sad_last_error() returns a thread-local message for the last failure;
 *   - all tensors are caller-owned device pointers (PyTorch caching allocator);
 *     the library never frees caller memory;
 *   - plans are opaque, immutable after creation, freed by *_destroy (one
 *     exception: the experimental fused front end's counters, see
 *     sad_frontend_run);
 *   - *_run calls are asynchronous on the given hipStream_t (passed as void*),
 *     never allocate, never synchronise (graph-capturable);
 *   - distinct plans / streams may be used from different threads;
 *   - cross-stream hand-offs need only the usual event: an output written on
 *     one stream (a libsad call, or a collective on the NCCL/RCCL stream) may
 *     be consumed by a *_run on another stream after hipStreamWaitEvent (or a
 *     host wait) on an event recorded after the producer.  Kernels of
 *     different streams may run concurrently and co-reside on a CU; the
 *     outputs do not depend on it (tests/test_gpu_handoff.py: the front end
 *     beside the stem, and heads / AdamW / backbone fed from a side stream).
 *     The device code holds no packed-FP32 VALU instructions: on MI355X they
 *     returned wrong values while another kernel's MFMAs ran on the same CU
 *     (csrc/Makefile NOPK, tests/test_isa_scan.py).
 */
#ifndef SAD_H_
#define SAD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum sad_status {
  SAD_OK = 0,
  SAD_ERR_ARG = -1,      /* bad argument / shape */
  SAD_ERR_HIP = -2,      /* HIP runtime error */
  SAD_ERR_STATE = -3,    /* not initialised / wrong plan */
  SAD_ERR_NOMEM = -4,    /* workspace too small or device allocation failed */
};

enum sad_dtype {
  SAD_F32 = 0,   /* fp32 activations, f32 MFMA (v_mfma_f32_16x16x4_f32): parity mode */
  SAD_BF16 = 1,  /* bf16 activations, bf16 MFMA (v_mfma_f32_16x16x32_bf16), f32 accumulate */
  SAD_BF16X3 = 2 /* split-bf16 parity mode: every value v stored as hi = bf16(v), lo = bf16(v - hi)
                    (channels interleaved [hi 32 | lo 32] per group of 32, 4 B per value like fp32);
                    each product = W_hi.X_hi + W_lo.X_hi + W_hi.X_lo on bf16 MFMA, f32 accumulate:
                    ~2^-17 relative operands, 3x the bf16 MFMA work, 16/3 x the f32 MFMA rate */
};

/* ---------------------------------------------------------------- runtime */
/* Select the device for this thread's subsequent plan creation. */
int sad_init(int device);
/* Wait for the device, then release the launch-timing events of an
 * unfinished sad_profile_begin.  The small per-device constant buffers the
 * library allocates once (zero biases; stamp buffers of diagnostic builds) stay
 * allocated until the process exits.  Plans are caller-owned: destroy them
 * first.  sad_init may be called again after it. */
int sad_shutdown(void);
const char* sad_last_error(void);
/* Library / kernel build identification (for provenance in bench output). */
const char* sad_version(void);

/* --------------------------------------------------------------- frontend */
/* Replaces torchaudio.transforms.MelSpectrogram + AmplitudeToDB + the
 * standardisation at inference_runner.py:157-171 (and the norm=None trainer
 * variant at submodel_trainer.py:97-105,191-199). */
typedef struct sad_frontend_cfg {
  int32_t sample_rate;   /* 32000 */
  int32_t n_fft;         /* 2048 (only value supported) */
  int32_t hop_length;    /* 512 */
  int32_t n_mels;        /* 128 */
  float f_min;           /* 20 */
  float f_max;           /* 12000 */
  int32_t norm_slaney;   /* 1 = 'slaney' (inference), 0 = None (trainer) */
  float top_db;          /* 80; <0 disables the clamp */
  int32_t n_samples;     /* samples per segment, 128000 */
} sad_frontend_cfg;

typedef struct sad_frontend_plan sad_frontend_plan;

/* The mel filterbank built on the host in float64 from cfg (htk triangles,
 * optional slaney area norm), rounded once to fp32. */
int sad_frontend_plan_create(const sad_frontend_cfg* cfg, sad_frontend_plan** out);
/* The same with the caller's filterbank: fbank = HOST fp32 [n_fft/2 + 1][n_mels]
 * (finite, >= 0; copied).  torchaudio builds its bank in fp32 arithmetic
 * (melscale_fbanks, called by MelSpectrogram at inference_runner.py:158-166);
 * the host layer passes that exact bank, so the device projects on the
 * reference's weights, not on a more accurate rounding of the same triangles
 * (which moves a mel bin next to a strong tone at a triangle's edge by up to
 * 6e-3 dB). */
int sad_frontend_plan_create_fb(const sad_frontend_cfg* cfg, const float* fbank, sad_frontend_plan** out);
int sad_frontend_plan_destroy(sad_frontend_plan* plan);
/* Number of STFT frames per segment (1 + n_samples / hop = 251). */
int sad_frontend_frames(const sad_frontend_plan* plan, int32_t* n_frames);

/* Two kernels: fe_mel_db writes the dB map, fe_normalize standardises it.
 * (SAD_FE_FUSED=1/2 selects an experimental one-kernel form in which the last
 * workgroup of a segment standardises it, counting arrivals in the plan's
 * per-segment counters; it measured 1.7-2.2x slower, DESIGN.md 5c.  With it,
 * runs of ONE plan must not execute concurrently.)
 *
 * pcm: int16 mono segments, segment i at pcm + i*seg_stride (elements),
 *      n_samples each.  There is no n_ch argument: multi-channel audio goes
 *      through sad_pcm_mono_run first, once per file, as the reference
 *      averages the whole waveform before slicing it (inference_runner.py:145-146);
 *      averaging per segment would redo it for every overlapping window;
 * out_db:  optional [n_seg, n_mels, n_frames] fp32 dB map after the top-db
 *          clamp (NULL to skip);
 * out_map: [n_seg, n_mels, n_frames] fp32 standardised map
 *          (x - mean) / (std_unbiased + 1e-6), per segment. */
int sad_frontend_run(const sad_frontend_plan* plan, const int16_t* pcm, int64_t n_seg,
                     int64_t seg_stride, float* out_db, float* out_map, void* stream);
/* Same on fp32 waveforms already in [-1, 1) (the reference's tensor after
 * mono averaging / resampling, preprocess_waveform at inference_runner.py:144-155). */
int sad_frontend_run_f32(const sad_frontend_plan* plan, const float* wav, int64_t n_seg,
                         int64_t seg_stride, float* out_db, float* out_map, void* stream);
/* Windows of ONE long fp32 waveform wav[wav_len], read in place: segment i
 * starts at sample offsets[i] (DEVICE int64 array; each clamped to
 * [0, wav_len - n_samples]).  Replaces the per-window tensors of slice_waveform
 * (inference_runner.py:176-190) + torch.cat(specs) (:276-289): overlapping
 * windows are never copied. */
int sad_frontend_run_windows(const sad_frontend_plan* plan, const float* wav, int64_t wav_len,
                             const int64_t* offsets, int64_t n_seg, float* out_db, float* out_map,
                             void* stream);

/* -------------------------------------------------------------- ingestion */
/* preprocess_waveform (inference_runner.py:144-155) on the device: the WAV's
 * samples go to HBM as stored (int16) or host-decoded fp32, interleaved
 * [frames][channels]. */
enum sad_pcm_format {
  SAD_PCM_I16 = 0, /* int16, scaled by 1/32768 (torchaudio.load normalize=True) */
  SAD_PCM_F32 = 1  /* fp32 (other WAV encodings, decoded on the host) */
};
/* out[i] = mean_c pcm[i][c] (waveform.mean(dim=0): channels summed in order, / C) for
 * i < frames, 0 for frames <= i < out_len (the zero pad to one window, :151-154). */
int sad_pcm_mono_run(const void* pcm, int32_t format, int64_t frames, int32_t channels, float* out,
                     int64_t out_len, void* stream);

/* Replaces torchaudio.transforms.Resample(orig_freq, new_freq) with its
 * defaults (sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99), as built
 * at inference_runner.py:148 (and submodel_trainer.py:150-153): the plan holds
 * the polyphase kernel table (float64 on the host, rounded once to fp32). */
typedef struct sad_resample_plan sad_resample_plan;
int sad_resample_plan_create(int32_t orig_freq, int32_t new_freq, sad_resample_plan** out);
int sad_resample_plan_destroy(sad_resample_plan* plan);
/* ceil(new * n_in / orig) with the rates reduced by their gcd (torchaudio's target_length) */
int sad_resample_out_len(const sad_resample_plan* plan, int64_t n_in, int64_t* n_out);
/* x [n_in] fp32 -> y [y_len] fp32: the resampled signal, then zeros up to
 * y_len (>= sad_resample_out_len) */
int sad_resample_run(const sad_resample_plan* plan, const float* x, int64_t n_in, float* y, int64_t y_len,
                     void* stream);

/* out[w] = max |wav[w*hop, w*hop + window)| (window clipped at n; NaN
 * propagates as in torch.max), w < n_windows: the silence test of
 * slice_waveform (inference_runner.py:182-184) without moving windows to the host. */
int sad_window_absmax_run(const float* wav, int64_t n, int64_t window, int64_t hop, int64_t n_windows,
                          float* out, void* stream);

/* Replaces torchvision.transforms.Resize((512,512)) + repeat(3,1,1)
 * (inference_runner.py:172-174) for callers that want the image itself:
 * map [n, h, w] fp32 -> img [n, out_h, out_w] in `dtype` (one channel: the
 * reference's three channels are identical and are folded into conv1). */
int sad_resize_run(const float* map, int64_t n, int32_t h, int32_t w, int32_t out_h,
                   int32_t out_w, int32_t dtype, void* img, void* stream);

/* --------------------------------------------------------------- backbone */
/* Replaces timm.create_model('resnet18', num_classes=0).forward_features +
 * head[0:2] (AdaptiveAvgPool2d + Flatten) at inference_runner.py:35,49-51:
 * standardised map -> (fused) resize -> ResNet-18 -> pooled [B, 512] fp32. */
typedef struct sad_backbone_plan sad_backbone_plan;

/* params: host fp32 arrays in timm state-dict order, for each conv:
 *   conv weight [Cout, Cin, KH, KW], then its BN: weight, bias, running_mean,
 *   running_var  (5 pointers per conv+BN; conv1 has Cin = 3).
 * Order: conv1/bn1, then for layer1..4, block 0..1: conv1/bn1, conv2/bn2,
 * [downsample.0/downsample.1 for block 0 of layer2..4].  n_params must be
 * 5 * 20 = 100.  BN is folded (eps 1e-5) and weights are re-laid out
 * [Cout][KH][KW][Cin] in `dtype` on the current device. */
int sad_backbone_plan_create(const float* const* params, int32_t n_params, int32_t dtype,
                             int32_t map_h, int32_t map_w, sad_backbone_plan** out);
int sad_backbone_plan_destroy(sad_backbone_plan* plan);
/* Device workspace bytes needed by sad_backbone_run for a micro-batch of
 * `micro_batch` segments (the run processes B in chunks of micro_batch). */
int sad_backbone_workspace_size(const sad_backbone_plan* plan, int64_t micro_batch, size_t* bytes);
/* map: [B, map_h, map_w] fp32 standardised maps; feats: [B, 512] fp32. */
int sad_backbone_run(const sad_backbone_plan* plan, const float* map, int64_t B,
                     int64_t micro_batch, float* feats, void* workspace, size_t ws_bytes,
                     void* stream);
/* Same from already-resized images: img [B, 512, 512] fp32 = ONE channel of
 * the reference's [B, 3, 512, 512] input (its 3 channels are identical,
 * inference_runner.py:173; the caller checks that). */
int sad_backbone_run_img(const sad_backbone_plan* plan, const float* img, int64_t B,
                         int64_t micro_batch, float* feats, void* workspace, size_t ws_bytes,
                         void* stream);
/* Same from images whose 3 channels may DIFFER: img3 [B, 3, 512, 512] fp32, the
 * reference's general model input (its load-time check feeds
 * torch.randn(2,3,512,512), inference_runner.py:119-122 / model_merger.py:
 * 148-151); conv1 runs per channel in fp32 (not folded), the rest as above. */
int sad_backbone_run_img3(const sad_backbone_plan* plan, const float* img3, int64_t B,
                          int64_t micro_batch, float* feats, void* workspace, size_t ws_bytes,
                          void* stream);
/* Debug/parity entry: run only the fused resize+stem (conv1+bn1+relu+maxpool)
 * on B maps, writing NHWC [B,128,128,64] in the plan's dtype. */
int sad_backbone_stem_run(const sad_backbone_plan* plan, const float* map, int64_t B,
                          void* out, void* stream);
/* Debug/parity entry: layer4 output NHWC [B,16,16,512] (plan dtype) for B <=
 * micro_batch, in addition to the pooled features. */
int sad_backbone_run_debug(const sad_backbone_plan* plan, const float* map, int64_t B,
                           float* feats, void* layer4_out, void* workspace, size_t ws_bytes,
                           void* stream);

/* Deeper timm ResNets (resnet34/50/101/152, the
 * `--model-name` choices of submodel_trainer.py:51 / model_merger.py:24 /
 * inference_runner.py:77 backbone_name), on the same kernels: fused
 * resize+stem, block-conv GEMMs (downsample folded into the block's last GEMM
 * as extra K columns), the implicit-GEMM conv for Bottleneck identity adds,
 * then the average pool.  Replaces timm.create_model(name, num_classes=0)
 * .forward_features + global pool:  map -> pooled [B, num_features] fp32.
 * block: SAD_BASIC_BLOCK (resnet18/34: conv1/bn1, conv2/bn2 per block) or
 * SAD_BOTTLENECK (resnet50/101/152: conv1/bn1, conv2/bn2, conv3/bn3, width =
 * planes, expansion 4, stride on conv2 as timm).  layers: blocks per stage
 * ([3,4,6,3] for resnet34/50).  params: 5 pointers per conv+BN in timm
 * state-dict order (conv1/bn1 first; per block its convs, then
 * downsample.0/downsample.1 where present).  dtype SAD_BF16X3 with
 * SAD_BOTTLENECK runs every conv with the fourth split product W_lo.X_lo too
 * (|dlogit| <= 1e-3 on resnet50; environment SAD_DEEP_X4=0: three products). */
#define SAD_BASIC_BLOCK 0
#define SAD_BOTTLENECK 1
typedef struct sad_resnet_plan sad_resnet_plan;
int sad_resnet_plan_create(const float* const* params, int32_t n_params, int32_t block,
                           const int32_t* layers, int32_t dtype, int32_t map_h, int32_t map_w,
                           sad_resnet_plan** out);
int sad_resnet_plan_destroy(sad_resnet_plan* plan);
/* pooled feature width: 512 (BasicBlock) or 2048 (Bottleneck) */
int sad_resnet_num_features(const sad_resnet_plan* plan, int32_t* n);
int sad_resnet_workspace_size(const sad_resnet_plan* plan, int64_t micro_batch, size_t* bytes);
/* map: [B, map_h, map_w] fp32; feats: [B, num_features] fp32 */
int sad_resnet_run(const sad_resnet_plan* plan, const float* map, int64_t B, int64_t micro_batch,
                   float* feats, void* workspace, size_t ws_bytes, void* stream);
/* same from resized images img [B, 512, 512] fp32 (one of the 3 identical channels) */
int sad_resnet_run_img(const sad_resnet_plan* plan, const float* img, int64_t B, int64_t micro_batch,
                       float* feats, void* workspace, size_t ws_bytes, void* stream);

/* same from [B, 3, 512, 512] fp32 images with possibly distinct channels */
int sad_resnet_run_img3(const sad_resnet_plan* plan, const float* img3, int64_t B, int64_t micro_batch,
                        float* feats, void* workspace, size_t ws_bytes, void* stream);

/* Kernel-level timing of the backbone's block-conv launches (bench.py's
 * roofline of the dominant kernel): between begin and end, every block-conv
 * launch of sad_backbone_run* is bracketed by HIP events on its stream.  end()
 * synchronises those events and returns, for the launches of tile `variant`
 * (0 = all), the summed kernel time, the number of KERNEL launches (a conv
 * whose operands pass the 2 GiB buffer range runs as several image-range
 * launches inside one bracket; each counts, so total_ms / launches is the
 * average kernel duration rocprofv3 reports) and their algorithmic FLOPs
 * (2*M*Cout*K with K the conv taps [+ the downsample], never the identity
 * shortcut's columns). */
int sad_profile_begin(void);
int sad_profile_end(int32_t variant, double* total_ms, int64_t* launches, double* flops);

/* ------------------------------------------------------------------ heads */
/* Replaces BinaryClassifier.head (inference_runner.py:36-48) for N sub-models
 * and ModularMultiHeadClassifier.forward (inference_runner.py:62-73).
 * params: per head, host fp32, in nn.Sequential index order:
 *   2.weight [512,512], 2.bias, 3.{weight,bias,running_mean,running_var},
 *   6.weight [256,512], 6.bias, 7.{weight,bias,running_mean,running_var},
 *   10.weight [2,256], 10.bias            (14 pointers per head)
 * feat_index[h]: which backbone's pooled features head h reads (0..n_feat-1). */
typedef struct sad_heads_plan sad_heads_plan;

int sad_heads_plan_create(const float* const* params, int32_t n_heads, const int32_t* feat_index,
                          int32_t n_feat, sad_heads_plan** out);
/* Same with the backbone feature width feat_dim (2.weight is [512, feat_dim];
 * 2048 for Bottleneck ResNets, whose head is Linear(2048, 512),
 * inference_runner.py:39 with base.num_features); feats are [B, feat_dim]. */
int sad_heads_plan_create_dim(const float* const* params, int32_t n_heads, const int32_t* feat_index,
                              int32_t n_feat, int32_t feat_dim, sad_heads_plan** out);
int sad_heads_plan_destroy(sad_heads_plan* plan);
int sad_heads_workspace_size(const sad_heads_plan* plan, int64_t B, size_t* bytes);
/* feats: n_feat pointers to [B,512] fp32; logits: [B, N, 2] fp32 (per head
 * [Real, Synthetic]); merged: [B, N+1] fp32 = [syn_1..syn_N, mean_i real_i]. */
int sad_heads_merge_run(const sad_heads_plan* plan, const float* const* feats, int64_t B,
                        float* logits, float* merged, void* workspace, size_t ws_bytes,
                        void* stream);

/* ------------------------------------------------------------- operators */
/* One NHWC convolution (+ folded-BN bias, optional residual add, optional
 * ReLU) on the implicit-GEMM MFMA kernel the backbone uses: the building block
 * of timm's BasicBlock (conv -> bn -> [+ shortcut] -> act).  Exposed for op-level
 * parity tests and tile tuning.
 * in [N,H,W,Cin], wt [Cout,k,k,Cin] (dtype), bias [Cout] fp32, res/out
 * [N,Ho,Wo,Cout] (dtype; res may be NULL), Ho = (H + 2 pad - k)/stride + 1.
 * variant: 0 = the backbone's choice, 1..8 = tile variants (csrc/conv.hip). */
int sad_conv2d_run(const void* in, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* wt,
                   const float* bias, const void* res, void* out, int32_t Cout, int32_t k,
                   int32_t stride, int32_t pad, int32_t relu, int32_t dtype, int32_t variant,
                   void* stream);

/* One GEMM = conv(in0) + 1x1 shortcut(in1) (+ bias [+ res], optional ReLU) on
 * the block-conv kernels the backbone uses for timm's BasicBlock (conv2 -> bn2
 * -> + shortcut -> act2, the shortcut being the identity or downsample.0/1).
 * wt: [Cout][wt_ld] with wt_ld >= k*k*Cin + Cin1 (0 = exactly that): the conv
 * taps, then the shortcut's weights (identity matrix or folded 1x1 conv) as the
 * next Cin1 K columns; in1 may be NULL (plain conv).  Shortcut pixel =
 * (oy*ss1, ox*ss1) of in1 [N,H1,W1,Cin1].  res (NULL or NHWC [N,Ho,Wo,Cout],
 * same dtype) is an identity shortcut added in the epilogue instead; it needs
 * the halo kernel (bf16, 3x3/s1/p1, H and W multiples of 16).
 * variant: 0 = default, 9..18 = implicit-GEMM tiles, 20 = halo (block.hip, halo.hip);
 * | SAD_CONV_FOUR_PRODUCTS with dtype SAD_BF16X3: also W_lo.X_lo (the deep
 * Bottleneck plans' form, on variants 9 / 13 / 15; 0 picks among them). */
#define SAD_CONV_FOUR_PRODUCTS 0x10000
int sad_block_conv_run(const void* in0, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* in1,
                       int32_t H1, int32_t W1, int32_t Cin1, int32_t ss1, const void* wt, int32_t wt_ld,
                       const float* bias, const void* res, void* out, int32_t Cout, int32_t k,
                       int32_t stride, int32_t pad, int32_t relu, int32_t dtype, int32_t variant,
                       void* stream);

/* One whole layer1 BasicBlock (timm resnet18 layer1.{0,1} with BN folded:
 * out = relu(conv3x3(relu(conv3x3(x; w1) + b1); w2) + b2 + x), 64 channels,
 * stride 1) as ONE fused kernel (csrc/l1block.hip, variant 40): the
 * intermediate stays in LDS and the identity comes from the input patch.
 * Replaces the two sad_block_conv_run launches (conv1; conv2 + res) of a
 * layer1 block -- reference inference_runner.py:49-51 (timm forward_features).
 * bf16 only.  x, out: NHWC [N,H,W,64] bf16 (must not overlap), H and W
 * multiples of 16; w1, w2: [64][w_ld] bf16, k = tap * 64 + ci; b1, b2: [64]
 * fp32.  ablate: reserved, pass 0.  Async on `stream`. */
int sad_l1_block_run(const void* x, int64_t N, int32_t H, int32_t W, const void* w1, int32_t w1_ld,
                     const float* b1, const void* w2, int32_t w2_ld, const float* b2, void* out,
                     int32_t ablate, void* stream);

/* --------------------------------------------------------------- training */
/* The submodel_trainer.py hot path: the train-mode
 * front end of SpectrogramDataset.__getitem__ (:139-214, transforms :463-471),
 * and the train-mode ResNet-18 forward (BatchNorm with batch statistics) plus
 * the backward / clip / AdamW of train() (:250-302, setup :606-660).  These are
 * op-level entries; sad/train.py composes them into the step.  Activations are
 * NHWC in `dtype`; statistics, gradients and master weights are fp32. */

/* FrequencyMasking(15) + TimeMasking(35) (fill 0.0) on the top-db clamped dB
 * map, then (x - mean) / (std_unbiased + 1e-6)  (:107-114,191-199).
 * masks: device int32 [n,4] = {f0, f1, t0, t1} (rows [f0,f1), columns [t0,t1)
 * zeroed; f0 == f1 = no mask) or NULL.  db, out_map: [n, n_mels, n_frames]. */
int sad_specaug_norm_run(const float* db, int64_t n, int32_t n_mels, int32_t n_frames, const int32_t* masks,
                         float* out_map, void* stream);
/* transforms.Resize((512,512)) (:200) then RandomResizedCrop's
 * resized_crop(i, j, h, w, (out_hw, out_hw)) (:466), one plane of the three
 * identical channels (:203).  boxes: device int32 [n,4] = {i, j, h, w} in the
 * 512x512 image, or NULL (= the val transform Resize((512,512)), :470). */
int sad_crop_resize_run(const float* map, int64_t n, int32_t h, int32_t w, const int32_t* boxes, int32_t out_hw,
                        int32_t dtype, void* img, void* stream);
/* fp32 OIHW conv weight -> compute layout in dtype.  mode 0: [Cout][k][k][Cin]
 * (forward); 1: [Cin][k][k][Cout] with flipped taps (stride-1 dgrad as a conv of
 * dy); 2: [Cout][64], k = ky*7+kx, input channels summed (fp32 stem); 3: OIHW
 * copy; 4: [Cout][64], k = ky*8+kx (7x7 in an 8x8 grid), channels summed (bf16
 * training stem). */
int sad_pack_conv_weight_run(const float* w, int32_t cout, int32_t cin, int32_t k, int32_t mode, int32_t dtype,
                             void* out, void* stream);
/* timm conv1 7x7/2/p3 WITHOUT bn1 (train-mode BN needs the raw output):
 * img [n, ih, iw] (dtype) -> out NHWC [n, oh, ow, 64]; col_ws >= n*oh*ow*64
 * elements of dtype; w_packed from mode 2. */
int sad_stem_conv_run(const void* img, int64_t n, int32_t ih, int32_t iw, const void* w_packed, void* col_ws,
                      size_t ws_bytes, void* out, int32_t dtype, void* stream);
/* bf16 training stem in one pass (conv.hip stem_bf16_kernel<false, true>):
 * conv1 7x7/2 of the bf16 image with w_packed (pack mode 4), bn1 in train mode
 * (batch statistics -> stats, running stats updated as sad_bn_stats_run), ReLU,
 * maxpool 3x3/2 -> out NHWC [n, 128, 128, 64] bf16.  The raw 256x256 conv map
 * is never stored: the kernel pools sign(gamma) * conv and sums conv, conv^2
 * per channel.  ws: sad_stem_train_workspace_size bytes. */
int sad_stem_train_workspace_size(int64_t n, size_t* bytes);
int sad_stem_train_run(const void* img, int64_t n, const void* w_packed, const float* gamma, const float* beta,
                       float eps, float momentum, float* running_mean, float* running_var, float* stats, void* out,
                       void* ws, size_t ws_bytes, void* stream);
/* Train-mode conv + BatchNorm statistics: out NHWC [N, Ho, Wo, Cout] = raw conv
 * (no bias) of x with w_packed (pack mode 0), and stats / running stats as
 * sad_bn_stats_run computes them on out.  bf16 on the block-conv variants 13,
 * 15, 20 and 25 sums the statistics in the conv epilogue from the fp32
 * accumulators (out is not re-read; *fused_out = 1); otherwise (fp32, other
 * shapes) the conv is followed by the bn_reduce pass over out (*fused_out = 0).
 * ws: sad_conv_bn_train_workspace_size bytes. */
int sad_conv_bn_train_workspace_size(int64_t N, int32_t H, int32_t W, int32_t Cout, int32_t k, int32_t stride,
                                     int32_t pad, size_t* bytes);
int sad_conv_bn_train_run(const void* x, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* w_packed,
                          int32_t Cout, int32_t k, int32_t stride, int32_t pad, int32_t dtype, const float* gamma,
                          const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                          float* stats, void* out, float* ws, size_t ws_bytes, int32_t* fused_out, void* stream);
/* Workspace (bytes) of the BN entries for a [P, C] tensor. */
int sad_bn_workspace_size(int64_t P, int32_t C, size_t* bytes);
/* BatchNorm2d train-mode statistics of x NHWC [P, C]: stats = [mean | invstd |
 * scale = gamma*invstd | shift = beta - mean*scale] (4*C floats); running
 * stats (optional, both or neither) updated with momentum and the unbiased var. */
int sad_bn_stats_run(const void* x, int64_t P, int32_t C, int32_t dtype, const float* gamma, const float* beta,
                     float eps, float momentum, float* running_mean, float* running_var, float* stats, float* ws,
                     size_t ws_bytes, void* stream);
/* out = act(x*scale + shift [+ res] ) where res is added as-is (identity
 * shortcut) or, with res_stats, as res*rscale + rshift (downsample BN). */
int sad_bn_apply_run(const void* x, int64_t P, int32_t C, int32_t dtype, const float* stats, const void* res,
                     const float* res_stats, int32_t relu, void* out, void* stream);
/* bn1 + ReLU + maxpool 3x3/2/p1: x NHWC [n, H, W, C] raw conv1 -> out [n, Ho, Wo, C]. */
int sad_bn_relu_maxpool_run(const void* x, int64_t n, int32_t H, int32_t W, int32_t C, int32_t dtype,
                            const float* stats, void* out, void* stream);
/* CrossEntropyLoss on logits [B, C] fp32 (the trainer's pooled features, quirk
 * C1): dlogits = (softmax - onehot(target)) * scale; out[0] = sum of row
 * losses, out[1] = count of rows with argmax == target; pred (optional) [B] =
 * argmax (first maximum, outputs.max(1) at :281,346). */
int sad_ce_loss_run(const float* logits, const int64_t* target, int64_t B, int32_t C, float scale, float* dlogits,
                    float* out, int32_t* pred, void* stream);
/* The BinaryClassifier head in train mode (optional --head-loss of
 * submodel_trainer.py; the reference builds it at :613-625 and never calls it,
 * quirk C1): Linear(nf,512) -> BatchNorm1d(512) -> ReLU -> Dropout(p1) ->
 * Linear(512,256) -> BatchNorm1d(256) -> ReLU -> Dropout(p2) -> Linear(256,2).
 * Parameters are the head.* tensors (nn.Sequential indices 2, 3, 6, 7, 10),
 * fp32, device.  Dropout keeps element i of layer L (1, 2) when
 * u(seed, L, i) >= p, u from a splitmix64 hash (headtrain.hip hkeep), so the
 * backward regenerates the forward's masks from the same seed. */
typedef struct {
  const float *w2, *b2, *g3, *be3, *w6, *b6, *g7, *be7, *w10, *b10;
  float *rm3, *rv3, *rm7, *rv7; /* BN running statistics (updated in train mode) */
  int32_t in_features;          /* the backbone's num_features (512 / 2048) */
  float eps, momentum, p1, p2;  /* 1e-5, 0.1, 0.5, 0.3 in the reference */
} sad_head_params;
int sad_head_workspace_size(int64_t B, int32_t in_features, size_t* bytes);
/* feats [B, nf] -> logits [B, 2].  train: batch statistics (running stats
 * updated) and dropout; 0: eval (running stats, no dropout).  ws keeps the
 * activations the backward needs. */
int sad_head_train_forward_run(const sad_head_params* h, const float* feats, int64_t B, int32_t train, uint64_t seed,
                               float* logits, void* ws, size_t ws_bytes, void* stream);
/* After a train-mode forward with the same feats / seed / ws: dlogits [B, 2]
 * -> dfeats [B, nf] and grads = the head's parameter gradients, flat fp32 in
 * parameters() order (2.w, 2.b, 3.w, 3.b, 6.w, 6.b, 7.w, 7.b, 10.w, 10.b). */
int sad_head_train_backward_run(const sad_head_params* h, const float* feats, int64_t B, uint64_t seed,
                                const float* dlogits, float* dfeats, float* grads, void* ws, size_t ws_bytes,
                                void* stream);
/* BatchNorm2d train-mode backward through an optional ReLU:
 * dz = (dy | dpool[n][c]/pool_hw broadcast) * [y > 0 if y];  dbeta = sum dz,
 * dgamma = sum dz*xhat (written, or added if accumulate);  dx = gamma*invstd*
 * (dz - mean dz - xhat * mean(dz*xhat)).  x is the raw (pre-BN) tensor, stats
 * from sad_bn_stats_run; dz_out (optional) receives dz. */
int sad_bn_backward_run(const void* x, int64_t P, int32_t C, int32_t dtype, const float* stats, const float* gamma,
                        const void* dy, const float* dpool, int32_t pool_hw, const void* y, float* dgamma,
                        float* dbeta, int32_t accumulate, void* dz_out, void* dx, float* ws, size_t ws_bytes,
                        void* stream);
/* Conv weight gradient (wgrad.hip, hand-written MFMA, no im2col): dw
 * [Cout][Cin][k][k] fp32 = beta*dw + sum_p dy[p] (x) x[src(p, tap)], the
 * activation gathered per tap straight from NHWC x; split-K partials in ws
 * (sad_conv_wgrad_workspace_size bytes), reduced in a fixed order
 * (deterministic).  Cin, Cout multiples of 8 (bf16) / 4 (fp32). */
int sad_conv_wgrad_workspace_size(int64_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t k,
                                  int32_t stride, int32_t pad, int32_t dtype, size_t* bytes);
int sad_conv_wgrad_run(const void* x, int64_t N, int32_t H, int32_t W, int32_t Cin, const void* dy, int32_t Cout,
                       int32_t k, int32_t stride, int32_t pad, int32_t dtype, float beta, float* dw, void* ws,
                       size_t ws_bytes, void* stream);
/* Conv input gradient for any stride (wgrad.hip): dcol[p][j] = sum_co dy[p][co]
 * W[co][j] on the same MFMA kernel (w_oihw from pack mode 3, dy transposed
 * into ws), then the col2im gather into dx NHWC [N, H, W, Cin] (added to dx
 * if accumulate).  ws: sad_conv_dgrad_workspace_size bytes.  (Stride-1 3x3
 * dgrad runs as a block conv over dy with pack mode 1 weights instead.) */
int sad_conv_dgrad_workspace_size(int64_t N, int32_t Ho, int32_t Wo, int32_t Cout, int32_t Cin, int32_t k,
                                  int32_t dtype, size_t* bytes);
int sad_conv_dgrad_run(const void* dy, int64_t N, int32_t Ho, int32_t Wo, int32_t Cout, const void* w_oihw,
                       int32_t Cin, int32_t H, int32_t W, int32_t k, int32_t stride, int32_t pad, int32_t dtype,
                       int32_t accumulate, void* dx, void* ws, size_t ws_bytes, void* stream);
/* torch.nn.utils.clip_grad_norm_(params, max_norm) over one flat fp32 gradient
 * buffer (:276): norm_coef[0] = ||g||, norm_coef[1] = min(max_norm/(||g||+1e-6), 1);
 * g *= norm_coef[1].  ws >= 1024 doubles. */
int sad_clip_grad_norm_run(float* g, int64_t n, float max_norm, float* norm_coef, void* ws, size_t ws_bytes,
                           void* stream);
/* One conv weight inside the flat parameter buffer and its cached compute
 * copies (pack modes 0 / 1, either may be NULL) for sad_adamw_pack_run. */
typedef struct {
  int64_t offset; /* element offset of the OIHW weight in p */
  int32_t cout, cin, k, reserved;
  void* mode0;    /* [Cout][k][k][Cin] in dtype, or NULL */
  void* mode1;    /* [Cin][k][k][Cout], taps flipped, or NULL */
} sad_pack_seg;
/* sad_adamw_run + the updated conv weights written into their packed copies
 * (<= 16 segments): the trainer's next step needs no pack launches. */
int sad_adamw_pack_run(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                       float eps, float weight_decay, int64_t step, const sad_pack_seg* segs, int32_t nseg,
                       int32_t dtype, void* stream);
/* torch.optim.AdamW step `step` (1-based) over flat fp32 buffers (:648-652,278). */
int sad_adamw_run(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                  float eps, float weight_decay, int64_t step, void* stream);
/* y += alpha * x (fp32): folds a step's layer3 gradient into its never-zeroed
 * .grad (quirk C4: layer3 is unfrozen at epochs//3 but not in the optimizer). */
int sad_axpy_run(float* y, const float* x, int64_t n, float alpha, void* stream);
/* Element-wise dtype conversion fp32 <-> bf16 (RNE) of n values: the mixed
 * trainer's hand-over between its fp32 frozen prefix (stem, layers 1-3) and
 * its bf16 layer4 (sad/train.py, submodel_trainer.py --precision mixed). */
int sad_cast_run(const void* src, int32_t src_dtype, void* dst, int32_t dst_dtype, int64_t n, void* stream);
/* timm global average pool: x NHWC [B, hw, C] (dtype) -> out [B, C] fp32 (the
 * trainer's model(inputs), quirk C1). */
int sad_avgpool_run(const void* x, int64_t B, int32_t hw, int32_t C, int32_t dtype, float* out, void* stream);

/* -------------------------------------------------------------- synthetic */
/* Deterministic synthetic segments; bit-identical to
 * sad/synth.py up to rare 1-LSB float64 libm differences in the tone term.
 * pcm: [count, n_samples] int16, segments first_seg .. first_seg+count-1. */
int sad_synth_pcm(uint64_t seed, int64_t first_seg, int64_t count, int32_t n_samples,
                  int16_t* pcm, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SAD_H_ */
