"""ctypes binding of libsad.so (include/sad.h).

torch is imported first on purpose: torch ships its own ``libamdhip64.so.7``;
loading it before libsad makes the dynamic linker resolve libsad's
``libamdhip64.so.7`` dependency to the SAME runtime instance, so torch's device
pointers and streams are valid inside libsad.

There is no fallback: if the library is missing or fails to load, every entry
point raises.  (The product path never routes to a CPU implementation.)
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SAD_LIB', os.path.join(_HERE, 'libsad.so'))

SAD_F32 = 0
SAD_BF16 = 1
SAD_BF16X3 = 2  # split-bf16 parity mode (include/sad.h)
SAD_CONV_FOUR_PRODUCTS = 0x10000  # sad_block_conv_run variant flag (include/sad.h)
DTYPES = {'fp32': SAD_F32, 'bf16': SAD_BF16, 'bf16x3': SAD_BF16X3}
SAD_PCM_I16 = 0  # sad_pcm_format
SAD_PCM_F32 = 1

# name -> (restype, argtypes); exactly the symbols include/sad.h declares.
P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
SZ = ctypes.c_size_t
FPP = ctypes.POINTER(ctypes.c_void_p)


class FrontendCfg(ctypes.Structure):
    _fields_ = [('sample_rate', I32), ('n_fft', I32), ('hop_length', I32), ('n_mels', I32),
                ('f_min', ctypes.c_float), ('f_max', ctypes.c_float), ('norm_slaney', I32),
                ('top_db', ctypes.c_float), ('n_samples', I32)]


class PackSeg(ctypes.Structure):
    """sad_pack_seg (include/sad.h)."""
    _fields_ = [('offset', I64), ('cout', I32), ('cin', I32), ('k', I32), ('reserved', I32),
                ('mode0', P), ('mode1', P)]


class HeadParams(ctypes.Structure):
    """sad_head_params (include/sad.h): the train-mode head's device tensors."""
    _fields_ = [(n, P) for n in ('w2', 'b2', 'g3', 'be3', 'w6', 'b6', 'g7', 'be7', 'w10', 'b10',
                                 'rm3', 'rv3', 'rm7', 'rv7')] + \
               [('in_features', I32), ('eps', ctypes.c_float), ('momentum', ctypes.c_float),
                ('p1', ctypes.c_float), ('p2', ctypes.c_float)]


SIGNATURES = {
    'sad_init': (ctypes.c_int, [ctypes.c_int]),
    'sad_shutdown': (ctypes.c_int, []),
    'sad_last_error': (ctypes.c_char_p, []),
    'sad_version': (ctypes.c_char_p, []),
    'sad_frontend_plan_create': (ctypes.c_int, [ctypes.POINTER(FrontendCfg), ctypes.POINTER(P)]),
    'sad_frontend_plan_create_fb': (ctypes.c_int, [ctypes.POINTER(FrontendCfg), P, ctypes.POINTER(P)]),
    'sad_frontend_plan_destroy': (ctypes.c_int, [P]),
    'sad_frontend_frames': (ctypes.c_int, [P, ctypes.POINTER(I32)]),
    'sad_frontend_run': (ctypes.c_int, [P, P, I64, I64, P, P, P]),
    'sad_frontend_run_f32': (ctypes.c_int, [P, P, I64, I64, P, P, P]),
    'sad_frontend_run_windows': (ctypes.c_int, [P, P, I64, P, I64, P, P, P]),
    'sad_resize_run': (ctypes.c_int, [P, I64, I32, I32, I32, I32, I32, P, P]),
    # ingestion (include/sad.h "ingestion")
    'sad_pcm_mono_run': (ctypes.c_int, [P, I32, I64, I32, P, I64, P]),
    'sad_resample_plan_create': (ctypes.c_int, [I32, I32, ctypes.POINTER(P)]),
    'sad_resample_plan_destroy': (ctypes.c_int, [P]),
    'sad_resample_out_len': (ctypes.c_int, [P, I64, ctypes.POINTER(I64)]),
    'sad_resample_run': (ctypes.c_int, [P, P, I64, P, I64, P]),
    'sad_window_absmax_run': (ctypes.c_int, [P, I64, I64, I64, I64, P, P]),
    'sad_backbone_plan_create': (ctypes.c_int, [FPP, I32, I32, I32, I32, ctypes.POINTER(P)]),
    'sad_backbone_plan_destroy': (ctypes.c_int, [P]),
    'sad_backbone_workspace_size': (ctypes.c_int, [P, I64, ctypes.POINTER(SZ)]),
    'sad_backbone_run': (ctypes.c_int, [P, P, I64, I64, P, P, SZ, P]),
    'sad_backbone_run_img': (ctypes.c_int, [P, P, I64, I64, P, P, SZ, P]),
    'sad_backbone_run_img3': (ctypes.c_int, [P, P, I64, I64, P, P, SZ, P]),
    'sad_backbone_stem_run': (ctypes.c_int, [P, P, I64, P, P]),
    'sad_backbone_run_debug': (ctypes.c_int, [P, P, I64, P, P, P, SZ, P]),
    'sad_resnet_plan_create': (ctypes.c_int, [FPP, I32, I32, ctypes.POINTER(I32), I32, I32, I32,
                                              ctypes.POINTER(P)]),
    'sad_resnet_plan_destroy': (ctypes.c_int, [P]),
    'sad_resnet_num_features': (ctypes.c_int, [P, ctypes.POINTER(I32)]),
    'sad_resnet_workspace_size': (ctypes.c_int, [P, I64, ctypes.POINTER(SZ)]),
    'sad_resnet_run': (ctypes.c_int, [P, P, I64, I64, P, P, SZ, P]),
    'sad_resnet_run_img': (ctypes.c_int, [P, P, I64, I64, P, P, SZ, P]),
    'sad_resnet_run_img3': (ctypes.c_int, [P, P, I64, I64, P, P, SZ, P]),
    'sad_profile_begin': (ctypes.c_int, []),
    'sad_profile_end': (ctypes.c_int, [I32, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(I64),
                                       ctypes.POINTER(ctypes.c_double)]),
    'sad_heads_plan_create': (ctypes.c_int, [FPP, I32, ctypes.POINTER(I32), I32, ctypes.POINTER(P)]),
    'sad_heads_plan_create_dim': (ctypes.c_int, [FPP, I32, ctypes.POINTER(I32), I32, I32, ctypes.POINTER(P)]),
    'sad_heads_plan_destroy': (ctypes.c_int, [P]),
    'sad_heads_workspace_size': (ctypes.c_int, [P, I64, ctypes.POINTER(SZ)]),
    'sad_heads_merge_run': (ctypes.c_int, [P, FPP, I64, P, P, P, SZ, P]),
    'sad_conv2d_run': (ctypes.c_int, [P, I64, I32, I32, I32, P, P, P, P, I32, I32, I32, I32, I32, I32, I32, P]),
    'sad_block_conv_run': (ctypes.c_int, [P, I64, I32, I32, I32, P, I32, I32, I32, I32, P, I32, P, P, P, I32, I32,
                                          I32, I32, I32, I32, I32, P]),
    'sad_l1_block_run': (ctypes.c_int, [P, I64, I32, I32, P, I32, P, P, I32, P, P, I32, P]),
    'sad_synth_pcm': (ctypes.c_int, [ctypes.c_uint64, I64, I64, I32, P, P]),
    # training (include/sad.h "training")
    'sad_specaug_norm_run': (ctypes.c_int, [P, I64, I32, I32, P, P, P]),
    'sad_crop_resize_run': (ctypes.c_int, [P, I64, I32, I32, P, I32, I32, P, P]),
    'sad_pack_conv_weight_run': (ctypes.c_int, [P, I32, I32, I32, I32, I32, P, P]),
    'sad_stem_conv_run': (ctypes.c_int, [P, I64, I32, I32, P, P, SZ, P, I32, P]),
    'sad_stem_train_workspace_size': (ctypes.c_int, [I64, ctypes.POINTER(SZ)]),
    'sad_stem_train_run': (ctypes.c_int, [P, I64, P, P, P, ctypes.c_float, ctypes.c_float, P, P, P, P, P, SZ, P]),
    'sad_conv_bn_train_workspace_size': (ctypes.c_int, [I64, I32, I32, I32, I32, I32, I32, ctypes.POINTER(SZ)]),
    'sad_conv_bn_train_run': (ctypes.c_int, [P, I64, I32, I32, I32, P, I32, I32, I32, I32, I32, P, P, ctypes.c_float,
                                             ctypes.c_float, P, P, P, P, P, SZ, P, P]),
    'sad_bn_workspace_size': (ctypes.c_int, [I64, I32, ctypes.POINTER(SZ)]),
    'sad_bn_stats_run': (ctypes.c_int, [P, I64, I32, I32, P, P, ctypes.c_float, ctypes.c_float, P, P, P, P, SZ,
                                        P]),
    'sad_bn_apply_run': (ctypes.c_int, [P, I64, I32, I32, P, P, P, I32, P, P]),
    'sad_bn_relu_maxpool_run': (ctypes.c_int, [P, I64, I32, I32, I32, I32, P, P, P]),
    'sad_ce_loss_run': (ctypes.c_int, [P, P, I64, I32, ctypes.c_float, P, P, P, P]),
    'sad_bn_backward_run': (ctypes.c_int, [P, I64, I32, I32, P, P, P, P, I32, P, P, P, I32, P, P, P, SZ, P]),
    'sad_conv_wgrad_workspace_size': (ctypes.c_int, [I64, I32, I32, I32, I32, I32, I32, I32, I32,
                                                     ctypes.POINTER(SZ)]),
    'sad_conv_dgrad_workspace_size': (ctypes.c_int, [I64, I32, I32, I32, I32, I32, I32, ctypes.POINTER(SZ)]),
    'sad_conv_wgrad_run': (ctypes.c_int, [P, I64, I32, I32, I32, P, I32, I32, I32, I32, I32, ctypes.c_float, P, P,
                                          SZ, P]),
    'sad_conv_dgrad_run': (ctypes.c_int, [P, I64, I32, I32, I32, P, I32, I32, I32, I32, I32, I32, I32, I32, P, P,
                                          SZ, P]),
    'sad_clip_grad_norm_run': (ctypes.c_int, [P, I64, ctypes.c_float, P, P, SZ, P]),
    'sad_head_workspace_size': (ctypes.c_int, [I64, I32, ctypes.POINTER(SZ)]),
    'sad_head_train_forward_run': (ctypes.c_int, [ctypes.POINTER(HeadParams), P, I64, I32, ctypes.c_uint64, P, P,
                                                  SZ, P]),
    'sad_head_train_backward_run': (ctypes.c_int, [ctypes.POINTER(HeadParams), P, I64, ctypes.c_uint64, P, P, P,
                                                   P, SZ, P]),
    'sad_adamw_run': (ctypes.c_int, [P, P, P, P, I64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_float, ctypes.c_float, I64, P]),
    'sad_adamw_pack_run': (ctypes.c_int, [P, P, P, P, I64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float, I64, ctypes.POINTER(PackSeg), I32, I32,
                                          P]),
    'sad_axpy_run': (ctypes.c_int, [P, P, I64, ctypes.c_float, P]),
    'sad_cast_run': (ctypes.c_int, [P, I32, P, I32, I64, P]),
    'sad_avgpool_run': (ctypes.c_int, [P, I64, I32, I32, I32, P, P]),
}

_lib = None


def load():
    """Load libsad.so (once) and attach prototypes; raises if unavailable."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f'libsad.so not found at {LIB_PATH}; build it with '
                               f'`python -c "import __graft_entry__ as g; g.build()"`')
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            # (an older build loaded for a same-box A/B may lack newer entry
            # points: they fail when called; tests/test_abi.py checks the
            # in-tree build exports every one)
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str = ''):
    if rc != 0:
        msg = load().sad_last_error().decode(errors='replace')
        raise RuntimeError(f'libsad {what} failed ({rc}): {msg}')


def call(name: str, *args):
    check(getattr(load(), name)(*args), name)


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def pointer_array(arrays):
    """Keep-alive list + C array of host pointers to contiguous fp32 numpy arrays."""
    arr = (ctypes.c_void_p * len(arrays))(*[a.ctypes.data for a in arrays])
    return arr
