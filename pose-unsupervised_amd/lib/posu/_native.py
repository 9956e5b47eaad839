"""ctypes binding of libposeu.so (the C ABI declared in include/posu.h).

The library is built in-tree (``make -C pose-unsupervised_amd`` or
``__graft_entry__.build()``) and loaded from this directory.  There is no
fallback: if the library is missing, or no GPU is visible when an op runs,
the op raises.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  -- loads PyTorch's HIP runtime before libposeu.so binds to it

F32 = 0
BF16 = 1
F64 = 2
F16 = 3
F16X3 = 4   # split fp16 (hi + lo pairs, three MFMAs per product): include/posu.h

# the ABI revision this binding declares (include/posu.h); load() refuses any other library
ABI_VERSION = 16

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libposeu.so')
_lock = threading.Lock()
_lib = None

_p = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_ll = ctypes.c_longlong
_d = ctypes.c_double

# name -> argtypes (restype is int unless listed in _RESTYPES)
_SIGNATURES = {
    'posu_last_error': [],
    'posu_abi_version': [],
    'posu_pack_nchw_to_nhwc': [_i, _p, _i, _i, _i, _i, _p, _i, _i, _p],
    'posu_pack_job_blocks': [_i, _i, _i, _i, _i, _i, _i, _i],
    'posu_pack_weights': [_i, _p, _i, _ll, _p],
    'posu_pack_s2d_nchw': [_i, _p, _i, _i, _i, _i, _p, _i, _i, _p],
    'posu_nhwc_to_nchw_f32': [_i, _p, _i, _i, _i, _i, _p, _p],
    'posu_conv1x1_dual_fwd': [_i, _p, _i, _i, _i, _i, _p, _i, _i, _i, _i, _p, _i, _p, _p, _i, _p, _i, _p],
    'posu_conv_bk': [_i],
    'posu_stem_pool_fwd': [_i, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p],
    'posu_stem_pool_views_fwd': [_i, _p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p],
    'posu_bottleneck_fwd': [_i, _p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    'posu_bottleneck_tail_stream_fwd': [_i, _p, _p, _i, _i, _i, _i, _i, _p, _ll, _p, _p, _p, _p, _p, _p],
    'posu_bottleneck_tail_stream_next_fwd': [_i, _p, _p, _i, _i, _i, _i, _i, _p, _ll, _p, _p, _p, _p, _p, _p, _p,
                                             _p, _p],
    'posu_bottleneck_tail_stream_chain_fwd': [_i, _p, _p, _i, _i, _i, _i, _i, _i, _p, _ll, _p, _p, _p, _p, _p, _p,
                                              _p, _p, _p],
    'posu_bottleneck_down_tail_stream_fwd': [_i, _p, _p, _i, _i, _i, _i, _i, _p, _ll, _p, _p, _p, _p, _p, _p, _p,
                                             _p, _p],
    'posu_bottleneck_s2_tail_fwd': [_i, _p, _p, _i, _i, _i, _i, _i, _p, _ll, _p, _p, _p, _i, _p, _p],
    'posu_bottleneck_s2_tail_next_fwd': [_i, _p, _p, _i, _i, _i, _i, _i, _p, _ll, _p, _p, _p, _i, _p, _p, _p, _p, _p],
    'posu_bottleneck_down_fwd': [_i, _p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    'posu_conv2d_fwd': [_i, _p, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _p, _p, _p, _i, _p, _i, _i, _i, _p],
    'posu_deconv4x4s2_fwd': [_i, _p, _i, _i, _i, _i, _p, _i, _p, _p, _i, _p, _i, _p],
    'posu_deconv4x4s2_head_fwd': [_i, _p, _i, _i, _i, _i, _p, _i, _p, _p, _p, _p, _p, _i, _p, _p, _p],
    'posu_head1x1_nchw_fwd': [_i, _p, _i, _i, _i, _i, _p, _i, _p, _p, _p],
    'posu_maxpool3x3s2_fwd': [_i, _p, _i, _i, _i, _i, _p, _p],
    'posu_softargmax2d_fwd': [_p, _i, _i, _i, _i, _f, _p, _p, _p, _p],
    'posu_softargmax2d_bwd': [_p, _p, _i, _i, _i, _i, _f, _p, _p, _p, _p],
    'posu_argmax2d_fwd': [_p, _i, _i, _i, _i, _i, _p, _p, _p, _p],
    'posu_affine2d_apply': [_p, _p, _i, _i, _i, _p, _p],
    'posu_epipolar_loss_fwd': [_p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p],
    'posu_epipolar_loss_bwd': [_p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p],
    'posu_triangulate_dlt': [_p, _p, _p, _i, _i, _i, _p, _i, _i, _i, _i, _p, _p],
    'posu_joints_mse_fwd': [_p, _p, _p, _i, _i, _i, _p, _p, _p],
    'posu_joints_mse_bwd': [_p, _p, _p, _i, _i, _i, _p, _p, _p],
    'posu_ransac_inliers': [_p, _p, _p, _p, _i, _i, _i, _i, _d, _i, _p, _p],
    'posu_reproject': [_p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p],
    'posu_pack_view_rows': [_i, _p, _i, _i, _i, _p, _p],
    'posu_gemm_rows_f32': [_i, _p, _i, _i, _p, _i, _i, _p, _p],
    'posu_gaussian_targets': [_p, _p, _i, _i, _i, _i, _i, _i, _d, _p, _p, _p, _p],
    'posu_integral2d_fwd': [_p, _i, _i, _i, _i, _p, _p],
    'posu_crop_warp': [_p, _p, _p, _i, _p, _i, _i, _i, _i, _p, _p, _p, _p],
    'posu_flip_back': [_p, _p, _p, _i, _i, _i, _i, _i, _p, _p],
    # training path
    'posu_conv2d_dgrad': [_i, _p, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _p, _p, _i, _i, _p],
    'posu_conv2d_dgrad_tile': [_i, _p, _i, _i, _i, _i, _p, _i, _i, _i, _i, _i, _p, _p, _i, _i, _i, _p],
    'posu_conv2d_wgrad_workspace': [_i, _i, _i, _i, _i, _i, _i, _i, _i, _i],
    'posu_conv2d_wgrad': [_i, _p, _p, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _p, _p, _ll, _p],
    'posu_bn_workspace': [_i, _i],
    'posu_bn_train_fwd': [_i, _p, _i, _i, _i, _p, _p, _f, _f, _p, _p, _p, _p, _p, _p, _p, _ll, _p],
    'posu_bn_apply_mask': [_i, _p, _i, _i, _i, _p, _p, _p, _p, _p, _p],
    'posu_bn_train_bwd_mask': [_i, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _ll, _p],
    'posu_bn_relu_maxpool3x3s2_fwd': [_i, _p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p],
    'posu_maxpool3x3s2_bwd_idx': [_i, _p, _p, _i, _i, _i, _i, _p, _p],
    'posu_stem_conv_views_fwd': [_i, _p, _i, _i, _i, _i, _p, _p, _p],
    'posu_stem_wgrad_workspace': [_i, _i, _i],
    'posu_stem_wgrad_views': [_i, _p, _i, _i, _i, _i, _p, _p, _p, _ll, _p],
    'posu_bn_apply': [_i, _p, _i, _i, _i, _p, _p, _p, _i, _p, _p],
    'posu_bn_train_bwd': [_i, _p, _p, _p, _p, _p, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _ll, _p],
    'posu_channel_sum': [_i, _p, _i, _i, _p, _p, _ll, _p],
    'posu_maxpool3x3s2_bwd_workspace': [_i, _i, _i, _i],
    'posu_maxpool3x3s2_bwd': [_i, _p, _i, _i, _i, _i, _p, _p, _p, _ll, _p],
    'posu_adam_step': [_p, _i, _d, _d, _d, _d, _d, _ll, _p],
}
_RESTYPES = {'posu_last_error': ctypes.c_char_p, 'posu_conv2d_wgrad_workspace': ctypes.c_longlong,
             'posu_pack_job_blocks': ctypes.c_longlong,
             'posu_bn_workspace': ctypes.c_longlong, 'posu_maxpool3x3s2_bwd_workspace': ctypes.c_longlong,
             'posu_stem_wgrad_workspace': ctypes.c_longlong}


def library_path():
    return _LIB_PATH


def load():
    """Load libposeu.so once and declare every exported signature."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(
                'libposeu.so is not built (%s); run `make -C pose-unsupervised_amd` '
                'or __graft_entry__.build()' % _LIB_PATH)
        lib = ctypes.CDLL(_LIB_PATH)
        for name, args in _SIGNATURES.items():
            fn = getattr(lib, name)  # AttributeError = a declared symbol is missing
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        if lib.posu_abi_version() != ABI_VERSION:
            raise RuntimeError('libposeu.so has ABI %d, the binding expects %d: rebuild it'
                               % (lib.posu_abi_version(), ABI_VERSION))
        _lib = lib
        return lib


def exported_symbols():
    return sorted(_SIGNATURES)


def last_error():
    return load().posu_last_error().decode('utf-8', 'replace')


def call(name, *args):
    """Invoke an entry point and raise on a non-zero status."""
    status = getattr(load(), name)(*args)
    if status != 0:
        raise RuntimeError('%s failed (status %d): %s' % (name, status, last_error()))


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_of(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_cuda(*tensors):
    """The product path runs only on the GPU: refuse CPU tensors loudly."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                'pose-unsupervised_amd ops run only on the MI355X HIP path; '
                'got a CPU tensor (move inputs to a cuda device)')


def dtype_code_of(t):
    """Storage dtype code of an activation tensor."""
    codes = {torch.float32: F32, torch.bfloat16: BF16, torch.float16: F16}
    if t.dtype not in codes:
        raise TypeError('unsupported activation dtype %s' % t.dtype)
    return codes[t.dtype]
