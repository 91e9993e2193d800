"""ctypes binding of libscd.so (include/scd.h) — the only way the Python host reaches the GPU kernels.

Every function here takes torch tensors that already live on the current HIP device, converts them
to the C-ABI views (plain pointers + sizes) and launches on ``torch.cuda.current_stream()``.  There
is no fallback: if the library is missing or the device is not gfx950 the first call raises.
"""
from __future__ import annotations

import contextlib
import contextvars
import ctypes
import os
from ctypes import POINTER, c_char_p, c_float, c_int, c_int8, c_int32, c_int64, c_size_t, c_uint8, c_uint32, c_void_p

import torch

LIB_PATH = os.environ.get("SCD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libscd.so")


class NHWC(ctypes.Structure):
    """scd_nhwc_t: channel-slice view of an NHWC fp32 or bf16 tensor (dtype: SCD_DT_F32 0 / SCD_DT_BF16 1, ABI 6)."""

    _fields_ = [("data", c_void_p), ("n", c_int32), ("h", c_int32), ("w", c_int32), ("c", c_int32), ("ldc", c_int32),
                ("dtype", c_int32)]


# element types of NHWC views (enum scd_dtype); activations and gradients of the bf16 configs are stored as bf16
DT_F32, DT_BF16 = 0, 1
_VIEW_DTYPES = {torch.float32: (DT_F32, 4), torch.bfloat16: (DT_BF16, 2)}


class BNBWD(ctypes.Structure):
    """scd_bn_bwd_tiles_t: fused BatchNorm-backward partial sums in a data-grad conv epilogue."""

    _fields_ = [("y", NHWC), ("nseg", c_int32), ("save_mean", c_void_p), ("save_invstd", c_void_p),
                ("scale", c_void_p), ("shift", c_void_p), ("rec", c_void_p)]


class IGEMM(ctypes.Structure):
    _fields_ = [
        ("src", NHWC),
        ("out_h", c_int32),
        ("out_w", c_int32),
        ("stride", c_int32),
        ("ntaps", c_int32),
        ("dy", c_int8 * 9),
        ("dx", c_int8 * 9),
        ("wpk", c_void_p),
        ("n_out", c_int32),
        ("bias", c_void_p),
        ("dst", NHWC),
        ("store_mode", c_int32),
        ("wsplit", c_void_p),
        ("stat_rec", c_void_p),
        ("in_scale", c_void_p),
        ("in_shift", c_void_p),
        ("in_nseg", c_int32),
        ("bn_bwd", POINTER(BNBWD)),
        ("src_bound", c_void_p),
        ("dst_bound", c_void_p),
        ("math", c_int32),
        ("tune", c_uint32),
        ("dst_bound_seed", c_void_p),  # ABI 9
    ]


class WGRAD(ctypes.Structure):
    _fields_ = [
        ("rows", NHWC),
        ("src", NHWC),
        ("stride", c_int32),
        ("ntaps", c_int32),
        ("dy", c_int8 * 9),
        ("dx", c_int8 * 9),
        ("src_scale", c_void_p),
        ("src_shift", c_void_p),
        ("src_nseg", c_int32),
        ("rows_bound", c_void_p),
        ("src_bound", c_void_p),
        ("rows_y", NHWC),
        ("rows_nseg", c_int32),
        ("rows_mean", c_void_p),
        ("rows_invstd", c_void_p),
        ("rows_gamma", c_void_p),
        ("rows_scale", c_void_p),
        ("rows_shift", c_void_p),
        ("rows_coef", c_void_p),
        ("math", c_int32),
        ("tune", c_uint32),
        ("src_colsum", c_void_p),
        ("rows_out", NHWC),
        ("rows_out_bound", c_void_p),
    ]


# Tap sets (dy, dx) used by the network.
TAPS_3X3 = ([-1, -1, -1, 0, 0, 0, 1, 1, 1], [-1, 0, 1, -1, 0, 1, -1, 0, 1])  # t = ky*3 + kx
TAPS_1 = ([0], [0])
TAPS_2X2 = ([0, 0, 1, 1], [0, 1, 0, 1])  # t = i*2 + j

_NULL = NHWC(None, 0, 0, 0, 0, 0, 0)

_lib = None
_dev_checked: set = set()

_SIGS = {
    "scd_version": ([], c_char_p),
    "scd_abi_version": ([], c_int),
    "scd_last_error": ([], c_char_p),
    "scd_device_check": ([c_int], c_int),
    "scd_pack_nchw": ([c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, NHWC, c_void_p, c_void_p], c_int),
    "scd_pack_conv3x3": ([c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p], c_int),
    "scd_pack_conv3x3_multi": ([c_void_p, c_int32, c_void_p], c_int),
    "scd_pack_convT2x2_multi": ([c_void_p, c_int32, c_void_p], c_int),
    "scd_pack_convT2x2": ([c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p], c_int),
    "scd_split_bf16x3": ([c_void_p, c_int64, c_void_p, c_void_p], c_int),
    "scd_split_frag_bytes": ([c_int32, c_int32], c_size_t),
    "scd_split_bf16x3_frag": ([c_void_p, c_int32, c_int32, c_void_p, c_void_p], c_int),
    "scd_split_h2_frag": ([c_void_p, c_int32, c_int32, c_void_p, c_void_p], c_int),
    "scd_absmax_bound": ([NHWC, c_int32, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "scd_conv_igemm": ([POINTER(IGEMM), c_void_p], c_int),
    "scd_igemm_arith": ([POINTER(IGEMM)], c_int),
    "scd_igemm_input_bn_supported": ([POINTER(IGEMM)], c_int),
    "scd_igemm_bn_bwd_tiles": ([POINTER(IGEMM), POINTER(c_int32)], c_int),
    "scd_wgrad_src_bn_supported": ([POINTER(WGRAD)], c_int),
    "scd_igemm_stat_tiles": ([POINTER(IGEMM), POINTER(c_int32)], c_int),
    "scd_wgrad_plan": ([POINTER(WGRAD), POINTER(c_int32), POINTER(c_size_t)], c_int),
    "scd_conv_wgrad": ([POINTER(WGRAD), c_void_p, c_size_t, c_void_p], c_int),
    "scd_wgrad_arith": ([POINTER(WGRAD)], c_int),
    "scd_wgrad_rows_per_block": ([POINTER(WGRAD)], c_int),
    "scd_wgrad_rows_bn_supported": ([POINTER(WGRAD)], c_int),
    "scd_wgrad_finalize": ([c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p], c_int),
    "scd_wgrad_colsum_supported": ([POINTER(WGRAD)], c_int),
    "scd_wgrad_colsum_finalize": ([c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p], c_int),
    "scd_bn_workspace_bytes": ([c_int32, c_int32, c_int32, c_int32, c_int32], c_size_t),
    "scd_bn_train_stats": (
        [NHWC, c_int32, c_void_p, c_void_p, c_float, c_float, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
        c_int,
    ),
    "scd_bn_tile_stats_workspace_bytes": ([c_int32, c_int32, c_int32], c_size_t),
    "scd_bn_stats_from_tiles": (
        [c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_float, c_float, c_int32, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
        c_int,
    ),
    "scd_bn_eval_coeffs": ([c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p], c_int),
    "scd_bn_relu_apply": ([NHWC, c_int32, c_void_p, c_void_p, NHWC, c_void_p], c_int),
    "scd_bn_relu_backward": (
        [NHWC, NHWC, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, NHWC,
         c_void_p, c_void_p, c_size_t, c_void_p],
        c_int,
    ),
    "scd_bn_relu_backward_pooled": ([NHWC, NHWC, c_void_p, NHWC, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, NHWC, c_void_p, c_void_p,
                                     c_size_t, c_void_p], c_int),
    "scd_bn_relu_backward_pooled2": ([NHWC, NHWC, c_void_p, NHWC, c_int32, NHWC, c_int32, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, NHWC, c_void_p, c_void_p,
                                      c_size_t, c_void_p], c_int),
    "scd_bn_head_workspace_bytes": ([c_int32, c_int32, c_int32, c_int32, c_int32, c_int32], c_size_t),
    "scd_bn_relu_backward_head": ([NHWC, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, NHWC, c_void_p, c_void_p, c_void_p,
                                   c_size_t, c_void_p], c_int),
    "scd_bn_relu_backward_tiles": (
        [NHWC, NHWC, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
         c_void_p, c_void_p, NHWC, c_void_p, c_void_p, c_size_t, c_void_p],
        c_int,
    ),
    "scd_bn_relu_backward_coef": (
        [NHWC, NHWC, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
        c_int,
    ),
    "scd_channel_sum": ([NHWC, c_void_p, c_void_p, c_size_t, c_void_p], c_int),
    "scd_maxpool2_fwd": ([NHWC, NHWC, c_void_p, c_void_p], c_int),
    "scd_bn_relu_maxpool2_fwd": ([NHWC, c_int32, c_void_p, c_void_p, NHWC, c_void_p, c_void_p], c_int),
    "scd_bn_relu_siamese_diff": ([NHWC, c_void_p, c_void_p, NHWC, c_void_p], c_int),
    "scd_bn_relu_pool_diff": ([NHWC, c_void_p, c_void_p, NHWC, NHWC, c_void_p, c_void_p], c_int),
    "scd_bn_relu_pool_out": ([NHWC, c_int32, c_void_p, c_void_p, c_int32, NHWC, NHWC, NHWC, c_void_p, c_void_p], c_int),
    "scd_feature_grad": ([NHWC, c_void_p, NHWC, c_int32, NHWC, c_int32, c_void_p], c_int),
    "scd_siamese_diff": ([NHWC, NHWC, c_void_p], c_int),
    "scd_conv1x1_fwd": ([NHWC, c_void_p, c_void_p, c_int32, c_void_p, c_void_p], c_int),
    "scd_conv1x1_fwd_bn": ([NHWC, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p], c_int),
    "scd_conv1x1_fwd_bn2": ([NHWC, c_void_p, c_void_p, NHWC, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32,
                             c_void_p, c_void_p], c_int),
    "scd_conv1x1_bwd_bn": ([NHWC, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p,
                            c_void_p, c_size_t, c_void_p], c_int),
    "scd_conv1x1_workspace_bytes": ([NHWC, c_int32], c_size_t),
    "scd_conv1x1_bwd": (
        [NHWC, c_void_p, c_void_p, c_int32, NHWC, c_int32, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p],
        c_int,
    ),
    "scd_pjaccard_workspace_bytes": ([c_int64], c_size_t),
    "scd_pjaccard_fwd": ([c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p], c_int),
    "scd_pjaccard_bwd": ([c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p], c_int),
    "scd_pjaccard_loss_from_sums": ([c_void_p, c_void_p, c_void_p], c_int),
    "scd_jaccard_multi_loss_from_sums": ([c_void_p, c_int32, c_void_p, c_void_p, c_void_p], c_int),
    "scd_window_copy": ([NHWC, NHWC, c_int32, c_int32, c_void_p], c_int),
    "scd_window_label_sums": ([c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p], c_int),
    "scd_augment_apply": ([c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p], c_int),
    "scd_jaccard_multi_workspace_bytes": ([c_int32], c_size_t),
    "scd_jaccard_multi_fwd": ([c_void_p, c_int32, c_void_p, c_int32, c_int64, c_void_p, c_void_p, c_void_p, c_size_t,
                               c_void_p], c_int),
    "scd_jaccard_multi_bwd": ([c_void_p, c_int32, c_void_p, c_int32, c_int64, c_void_p, c_void_p, c_void_p], c_int),
    "scd_threshold_counts_workspace_bytes": ([c_int64, c_int32], c_size_t),
    "scd_threshold_counts": (
        [c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_size_t, c_void_p], c_int),
}

EXPORTED_SYMBOLS = tuple(_SIGS)
ABI_VERSION = 9  # SCD_ABI_VERSION of include/scd.h


def load_library(path: str = LIB_PATH):
    """Load libscd.so and bind every C-ABI symbol (no GPU work is done here)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"libscd.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback."
        )
    lib = ctypes.CDLL(path)
    abi = getattr(lib, 'scd_abi_version', None)
    got = abi() if abi is not None else None
    if got != ABI_VERSION:
        raise RuntimeError(f"{path}: libscd ABI {got}, this binding needs ABI {ABI_VERSION} (rebuild: "
                           "`python -c 'import __graft_entry__ as g; g.build()'`)")
    for name, (argtypes, restype) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load_library()


def version() -> str:
    return lib().scd_version().decode()


def _check(rc: int, what: str):
    if rc != 0:
        msg = lib().scd_last_error().decode()
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ensure_device(t: torch.Tensor):
    """Fail loudly unless `t` lives on a gfx950 HIP device."""
    if t.device.type != "cuda":
        raise RuntimeError(
            "multimodal_siamese_cd_amd runs only on MI355X (gfx950) HIP devices; got a tensor on "
            f"{t.device}. The CPU restatement under oracle/ is test infrastructure, not a fallback."
        )
    idx = t.device.index if t.device.index is not None else torch.cuda.current_device()
    if idx not in _dev_checked:
        _check(lib().scd_device_check(idx), "scd_device_check")
        _dev_checked.add(idx)


def _ptr(t):
    return None if t is None else t.data_ptr()


def nhwc(t: torch.Tensor, c_off: int = 0, c: int | None = None) -> NHWC:
    """View a 4-D [n, h, w, C] fp32 or bf16 tensor (stride(3) == 1, rows of ldc = stride(2)) as scd_nhwc_t."""
    if t is None:
        return _NULL
    if t.dim() != 4 or t.dtype not in _VIEW_DTYPES or t.stride(3) != 1:
        raise ValueError(f"expected an fp32 / bf16 NHWC tensor with unit channel stride, got {tuple(t.shape)} "
                         f"{t.dtype} {t.stride()}")
    n, h, w, cc = t.shape
    ldc = t.stride(2)
    if (h > 1 and t.stride(1) != w * ldc) or (n > 1 and t.stride(0) != h * w * ldc):
        raise ValueError(f"tensor is not an NHWC channel slice: shape {tuple(t.shape)} stride {t.stride()}")
    if c is None:
        c = cc - c_off
    dt, eb = _VIEW_DTYPES[t.dtype]
    v = NHWC(t.data_ptr() + eb * c_off, n, h, w, c, ldc, dt)
    v._owner = t  # keep the storage alive at least until the view has been handed to a launch
    return v


def _taps(taps):
    dy, dx = taps
    a = (c_int8 * 9)(*dy, *([0] * (9 - len(dy))))
    b = (c_int8 * 9)(*dx, *([0] * (9 - len(dx))))
    return len(dy), a, b


# ------------------------------------------------------------------------------------------------
# thin wrappers
# ------------------------------------------------------------------------------------------------
def pack_nchw(src: torch.Tensor, c_begin: int, c_count: int, dst: torch.Tensor, dst_c_off: int = 0, dst_c=None,
              bound=None):
    """`bound` (a device float): raised to max |value| packed (the input layer's h2 operand bound)."""
    n, c, h, w = src.shape
    src = src.contiguous()
    cc = dst.shape[3] - dst_c_off if dst_c is None else dst_c
    dt, eb = _VIEW_DTYPES[dst.dtype]
    v = NHWC(dst.data_ptr() + eb * dst_c_off, dst.shape[0], dst.shape[1], dst.shape[2], cc, dst.stride(2), dt)
    _check(lib().scd_pack_nchw(src.data_ptr(), n, c, h, w, c_begin, c_count, v, _ptr(bound), _stream()),
           "scd_pack_nchw")


def pack_conv3x3(w: torch.Tensor, mode: int, ci_pad: int | None = None) -> torch.Tensor:
    co, ci = w.shape[0], w.shape[1]
    ci_pad = ci if ci_pad is None else ci_pad
    out = torch.empty((co * 9 * ci_pad) if mode == 0 else (ci * 9 * co), device=w.device, dtype=torch.float32)
    _check(lib().scd_pack_conv3x3(w.contiguous().data_ptr(), co, ci, ci_pad, mode, out.data_ptr(), _stream()),
           "scd_pack_conv3x3")
    return _attach_split(out, co, 9 * ci_pad, 9) if mode == 0 else _attach_split(out, ci, 9 * co, 9)


class PACKJOB(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("out", c_void_p), ("split", c_void_p), ("co", c_int32), ("ci", c_int32),
                ("ci_pad", c_int32), ("mode", c_int32), ("math", c_int32)]


def pack_conv3x3_multi(jobs) -> list:
    """jobs: [(weight OIHW, mode, ci_pad)] -> packed tensors as pack_conv3x3 returns them (split planes
    attached under the split conv arithmetics), all prepared in one launch per 48 weights."""
    if not jobs:
        return []
    split = conv_math() != 'f32'
    m = _MATH_NAMES[conv_math()]
    outs, keep, arr = [], [], (PACKJOB * len(jobs))()
    for i, (w, mode, ci_pad) in enumerate(jobs):
        co, ci = w.shape[0], w.shape[1]
        w = w.contiguous()
        rows, K = (co, 9 * ci_pad) if mode == 0 else (ci, 9 * co)
        out = torch.empty(rows * K, device=w.device, dtype=torch.float32)
        sp = None
        if split and K % 16 == 0:
            sp = torch.empty(lib().scd_split_frag_bytes(rows, K) // 2, dtype=torch.int16, device=w.device)
            out._x3 = sp
        keep.append(w)
        arr[i] = PACKJOB(w.data_ptr(), out.data_ptr(), _ptr(sp), co, ci, ci_pad, mode, m)
        outs.append(out)
    _check(lib().scd_pack_conv3x3_multi(ctypes.cast(arr, c_void_p), len(jobs), _stream()), "scd_pack_conv3x3_multi")
    return outs


def pack_convT2x2(w: torch.Tensor, mode: int) -> torch.Tensor:
    ci, co = w.shape[0], w.shape[1]
    out = torch.empty(ci * co * 4, device=w.device, dtype=torch.float32)
    _check(lib().scd_pack_convT2x2(w.contiguous().data_ptr(), ci, co, mode, out.data_ptr(), _stream()),
           "scd_pack_convT2x2")
    return _attach_split(out, 4 * co, ci, 1) if mode == 0 else _attach_split(out, ci, 4 * co, 4)


def pack_convT2x2_multi(jobs) -> list:
    """jobs: [(weight [ci][co][2][2], mode)] -> packed tensors as pack_convT2x2 returns them (split planes attached
    under the split conv arithmetics), all prepared in three launches per 8 weights."""
    if not jobs:
        return []
    split = conv_math() != 'f32'
    m = _MATH_NAMES[conv_math()]
    outs, keep, arr = [], [], (PACKJOB * len(jobs))()
    for i, (w, mode) in enumerate(jobs):
        ci, co = w.shape[0], w.shape[1]
        w = w.contiguous()
        n_out, K = (4 * co, ci) if mode == 0 else (ci, 4 * co)
        out = torch.empty(ci * co * 4, device=w.device, dtype=torch.float32)
        sp = None
        if split and K % 16 == 0:
            sp = torch.empty(lib().scd_split_frag_bytes(n_out, K) // 2, dtype=torch.int16, device=w.device)
            out._x3 = sp
        keep.append(w)
        arr[i] = PACKJOB(w.data_ptr(), out.data_ptr(), _ptr(sp), co, ci, ci, mode, m)
        outs.append(out)
    _check(lib().scd_pack_convT2x2_multi(ctypes.cast(arr, c_void_p), len(jobs), _stream()), "scd_pack_convT2x2_multi")
    return outs


def split_bf16x3(src: torch.Tensor) -> torch.Tensor:
    """Exact 3-way bf16 split of an fp32 tensor: int16 planes [3][numel] (bit patterns of h, m, l)."""
    n = src.numel()
    dst = torch.empty(3 * n, dtype=torch.int16, device=src.device)
    _check(lib().scd_split_bf16x3(src.data_ptr(), n, dst.data_ptr(), _stream()), "scd_split_bf16x3")
    return dst


def split_h2_frag(wpk: torch.Tensor, n_out: int, K: int) -> torch.Tensor:
    """SCD_MATH_H2 weight split of a packed [n_out][K] fp32 matrix: fp16 h, m planes of the per-row power-of-two
    scaled rows, then the float inverse row scales (see scd.h)."""
    nbytes = lib().scd_split_frag_bytes(n_out, K)
    dst = torch.empty(nbytes // 2, dtype=torch.int16, device=wpk.device)
    _check(lib().scd_split_h2_frag(wpk.data_ptr(), n_out, K, dst.data_ptr(), _stream()), "scd_split_h2_frag")
    return dst


def split_bf16x3_frag(wpk: torch.Tensor, n_out: int, K: int) -> torch.Tensor:
    """Fragment-major exact 3-way bf16 split of a packed [n_out][K] fp32 weight matrix (see scd.h)."""
    nbytes = lib().scd_split_frag_bytes(n_out, K)
    dst = torch.empty(nbytes // 2, dtype=torch.int16, device=wpk.device)
    _check(lib().scd_split_bf16x3_frag(wpk.data_ptr(), n_out, K, dst.data_ptr(), _stream()), "scd_split_bf16x3_frag")
    return dst


def h2_weight_format(K: int, ntaps: int) -> bool:
    """Whether the library expects the h2 split for a conv of this contraction (mirrors h2_weight_format in
    conv_common.h: 3x3, 1-tap and 4-tap convs whose source channels are a multiple of 32, and the 16-channel 3x3
    input layer, under SCD_MATH_H2)."""
    if conv_math() != 'h2' or ntaps not in (9, 1, 4) or K % ntaps:
        return False
    c = K // ntaps
    return c % 32 == 0 or (ntaps == 9 and c == 16)


def _attach_split(wpk: torch.Tensor, n_out: int, K: int, ntaps: int) -> torch.Tensor:
    """Under the split conv arithmetics, pre-split packed weights once so every workgroup stages them by copy."""
    if K % 16 == 0 and conv_math() != 'f32':  # x3, x5, bf16 and h2 all read split planes
        wpk._x3 = split_h2_frag(wpk, n_out, K) if h2_weight_format(K, ntaps) else split_bf16x3_frag(wpk, n_out, K)
    return wpk


MATH_F32, MATH_X3, MATH_BF16, MATH_X5, MATH_H2 = 0, 1, 2, 3, 4
_MATH_NAMES = {'f32': MATH_F32, 'x3': MATH_X3, 'bf16': MATH_BF16, 'x5': MATH_X5, 'h2': MATH_H2}
_MATH_BY_ID = {v: k for k, v in _MATH_NAMES.items()}

# SCD_TUNE_* kernel-variant bits (include/scd.h): 0 = the library's measured defaults.
# (SCD_TUNE_X3_TILE bits also force the ConvT gather kernel's tile: an x3 tile study must not time ConvT launches.)
TUNE_HALO16_OFF = 0xF
TUNE_HALO16_WRING = 0x8  # automatic tiles, the h2 1 x N tiles' weight fragments through an LDS ring (A/B)
TUNE_H2_TILE_2X2 = 1 << 4
TUNE_H2_TILE64_2X2 = 1 << 5
TUNE_H2_NO_PRESCALE = 1 << 6
TUNE_NO_XCD_REMAP = 1 << 7
TUNE_HALO_ORDER_M = 1 << 8
TUNE_W16_LAYOUT_2X2 = 1 << 9
TUNE_WGRAD_R64 = 1 << 10
TUNE_BF16_1XN = 1 << 11  # flips the bf16 tile layout (1 x N with bf16 storage by default, 2 x 2 with fp32)
TUNE_HALO16_DB_OFF = 1 << 20
TUNE_HALO16_DB_ON = 1 << 21
TUNE_NO_GATHER16 = 1 << 22
TUNE_NO_WGRAD_C16 = 1 << 23
TUNE_NO_WGRAD_H2 = 1 << 24
TUNE_NO_HALO16_C16 = 1 << 25
TUNE_NO_HALO = 1 << 26
TUNE_HALO16_LATE_LOAD = 1 << 27
TUNE_H2_TILE64_128 = 1 << 28
TUNE_HALO16_WS = 1 << 29
TUNE_WGRAD16_REGSTAGE = 1 << 30  # bf16 halo weight grad: register staging instead of the LDS-DMA ring (A/B)
TUNE_WGRAD16_DB = 1 << 31


def tune_halo16_cfg(tile_id: int) -> int:
    return tile_id + 1


def tune_x3_tile(t: int) -> int:
    return (t & 15) << 12


def tune_c16_tiles(k: int) -> int:
    return (k & 15) << 16


# The arithmetic and kernel-variant bits every conv descriptor is built with.  libscd keeps no mode: these are
# host-side values stamped into each scd_igemm_t / scd_wgrad_t / scd_pack_job_t.  A model carries its own
# arithmetic (utils.networks.create_network: MODEL.PRECISION / CONV_MATH) and runs its forward and backward inside
# conv_scope(model math); code outside any scope (kernel tests, tools) uses the process default.
_DEFAULT = {'math': MATH_X3, 'tune': 0}
_SCOPE: contextvars.ContextVar = contextvars.ContextVar('scd_conv_scope', default=None)


def _cur():
    sc = _SCOPE.get()
    return sc if sc is not None else (_DEFAULT['math'], _DEFAULT['tune'])


def _math_id(mode) -> int:
    if isinstance(mode, str):
        if mode not in _MATH_NAMES:
            raise ValueError(f"conv arithmetic {mode!r}: expected one of {sorted(_MATH_NAMES)}")
        return _MATH_NAMES[mode]
    m = int(mode)
    if m not in _MATH_BY_ID:
        raise ValueError(f"conv arithmetic {mode!r}")
    return m


def conv_math() -> str:
    """The arithmetic of descriptors built now: the innermost conv_scope's, else the process default."""
    return _MATH_BY_ID[_cur()[0]]


def conv_tune() -> int:
    return _cur()[1]


@contextlib.contextmanager
def conv_scope(math=None, tune=None):
    """Build every conv descriptor inside with this arithmetic ('f32', 'x3', 'x5', 'bf16', 'h2') and tune bits
    (None: inherit the enclosing value).  Context-local, so models with different arithmetic coexist."""
    m0, t0 = _cur()
    tok = _SCOPE.set((m0 if math is None else _math_id(math), t0 if tune is None else int(tune)))
    try:
        yield
    finally:
        _SCOPE.reset(tok)


def set_conv_math(mode) -> str:
    """Set the process-default arithmetic for descriptors built outside any conv_scope ('f32' = fp32 MFMA, 'x3' =
    exact 3-way split-bf16 MFMA, 'x5', 'bf16', 'h2'); returns the previous default."""
    prev = _MATH_BY_ID[_DEFAULT['math']]
    _DEFAULT['math'] = _math_id(mode)
    return prev


def set_tune(bits: int) -> int:
    """Set the process-default SCD_TUNE_* bits (kernel variants for tests / A/B); returns the previous default."""
    prev = _DEFAULT['tune']
    _DEFAULT['tune'] = int(bits)
    return prev


def get_tune() -> int:
    return _DEFAULT['tune']


def set_halo16(mode: int) -> int:
    """Tile selection of the 16x16x32-MFMA halo conv kernel through the default tune bits: 0 = off (32x32x16 halo
    kernel), 1 = automatic, 2 + id = force tile id.  Returns the previous mode."""
    t = _DEFAULT['tune']
    v = t & 0xF
    prev = 0 if v == TUNE_HALO16_OFF else 1 if v in (0, TUNE_HALO16_WRING) else v + 1
    new = TUNE_HALO16_OFF if mode == 0 else 0 if mode == 1 else tune_halo16_cfg(int(mode) - 2)
    _DEFAULT['tune'] = (t & ~0xF) | new
    return prev


def halo16_tile_width_pref() -> int:
    """The tile width the 16x16x32 halo kernel tries first (halo16_pick in conv_halo16.hip)."""
    return 16


def _igemm_desc(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode, stat_rec=None, in_bn=None,
                bn_bwd=None, src_bound=None, dst_bound=None, dst_bound_seed=None):
    nt, dy, dx = _taps(taps)
    sc, sh, nseg = in_bn if in_bn is not None else (None, None, 0)
    bb = None
    if bn_bwd is not None:  # (y, nseg, save_mean, save_invstd, scale, shift, rec)
        y, bseg, mu, iv, bsc, bsh, rec = bn_bwd
        bb = ctypes.pointer(BNBWD(nhwc(y), bseg, _ptr(mu), _ptr(iv), _ptr(bsc), _ptr(bsh), _ptr(rec)))
    m, t = _cur()
    return IGEMM(src, out_h, out_w, stride, nt, dy, dx, wpk.data_ptr(), n_out, _ptr(bias), dst, store_mode,
                 _ptr(getattr(wpk, '_x3', None)), _ptr(stat_rec), _ptr(sc), _ptr(sh), nseg, bb, _ptr(src_bound),
                 _ptr(dst_bound), m, t, _ptr(dst_bound_seed))


def conv_igemm(src: NHWC, out_h: int, out_w: int, stride: int, taps, wpk: torch.Tensor, n_out: int,
               bias, dst: NHWC, store_mode: int = 0, stat_rec: torch.Tensor | None = None, in_bn=None, bn_bwd=None,
               src_bound: torch.Tensor | None = None, dst_bound: torch.Tensor | None = None,
               dst_bound_seed: torch.Tensor | None = None):
    """`in_bn` = (scale, shift, nseg): read src through the producing layer's BatchNorm-apply + ReLU.
    `bn_bwd` = (y, nseg, save_mean, save_invstd, scale, shift, rec): also emit the BatchNorm-backward partial
    sums of the stored output into rec (see scd_bn_bwd_tiles_t).
    `src_bound`: device float >= max |src as read| (SCD_MATH_H2 operand scaling; see scd_igemm_t.src_bound).
    `dst_bound`: device float raised to max |stored output| (ConvTranspose forward, store_mode 1).
    `dst_bound_seed` (ABI 9, with dst_bound): a device float whose value the launch also folds into dst_bound."""
    d = _igemm_desc(src, out_h, out_w, stride, taps, wpk, n_out, bias, dst, store_mode, stat_rec, in_bn, bn_bwd,
                    src_bound, dst_bound, dst_bound_seed)
    _check(lib().scd_conv_igemm(ctypes.byref(d), _stream()), "scd_conv_igemm")


def igemm_bn_bwd_tiles(src: NHWC, out_h: int, out_w: int, stride: int, taps, wpk: torch.Tensor, n_out: int,
                       dst: NHWC, src_bound=None) -> tuple[int, int]:
    """(tiles, pixels per tile) of the fused BatchNorm-backward partial sums for this conv, (0, 0) if unavailable."""
    d = _igemm_desc(src, out_h, out_w, stride, taps, wpk, n_out, None, dst, 0, src_bound=src_bound)
    tp = c_int32(0)
    n = lib().scd_igemm_bn_bwd_tiles(ctypes.byref(d), ctypes.byref(tp))
    return (n, tp.value) if n > 0 else (0, 0)


def igemm_arith(src: NHWC, out_h: int, out_w: int, stride: int, taps, wpk: torch.Tensor, n_out: int,
                dst: NHWC, store_mode: int = 0, src_bound=None) -> str:
    """The arithmetic ('f32', 'x3', 'x5', 'bf16', 'h2') scd_conv_igemm will use for this conv (descriptor built with
    the current conv_math())."""
    d = _igemm_desc(src, out_h, out_w, stride, taps, wpk, n_out, None, dst, store_mode, src_bound=src_bound)
    rc = lib().scd_igemm_arith(ctypes.byref(d))
    _check(min(rc, 0), "scd_igemm_arith")
    return _MATH_BY_ID[rc]


def wgrad_arith(d: 'WGRAD') -> str:
    """The arithmetic scd_conv_wgrad will use for this descriptor."""
    rc = lib().scd_wgrad_arith(ctypes.byref(d))
    _check(min(rc, 0), "scd_wgrad_arith")
    return _MATH_BY_ID[rc]


# Algorithmic bytes of a conv launch: every operand read once, every output written once.  The ONE definition behind
# bench.py's roofline.traffic.algorithmic_bytes_per_step and tools/traffic_table.py's per-launch table.
_WEIGHT_PLANES = {'h2': 2, 'x3': 3, 'x5': 2, 'bf16': 1, 'f32': 2}


def _view_bytes(v: NHWC) -> int:
    return int(v.n) * int(v.h) * int(v.w) * int(v.c) * (2 if v.dtype == DT_BF16 else 4)


def igemm_alg_bytes(src: NHWC, out_h: int, out_w: int, taps, n_out: int, dst: NHWC, arith: str,
                    bn_bwd_y: torch.Tensor | None = None) -> int:
    """scd_conv_igemm: src (n h_s w_s c) + the output (n out_h out_w n_out; a ConvT's pixel-shuffled store holds the
    same elements) + the split weights (planes of the arithmetic `arith` x K x n_out x 2 B) + the y a fused
    BatchNorm-backward epilogue reads."""
    eb = 2 if dst.dtype == DT_BF16 else 4
    k = len(taps[0]) * int(src.c)
    out = int(src.n) * out_h * out_w * n_out * eb
    yb = 0 if bn_bwd_y is None else bn_bwd_y.numel() * bn_bwd_y.element_size()
    return _view_bytes(src) + out + _WEIGHT_PLANES[arith] * k * n_out * 2 + yb


def wgrad_alg_bytes(d: 'WGRAD', slab_bytes: int) -> int:
    """scd_conv_wgrad: dY rows (n h w R) + X (n h_s w_s C) + the fp32 split-K slabs written [+ the y of a rows BatchNorm
    transform] [+ the dy it stores for the data grad (ABI 8)]."""
    return (_view_bytes(d.rows) + _view_bytes(d.src) + int(slab_bytes)
            + (_view_bytes(d.rows_y) if d.rows_y.data else 0) + (_view_bytes(d.rows_out) if d.rows_out.data else 0))


def wgrad_rows_per_block(d: 'WGRAD') -> int:
    """dY rows per workgroup of the halo weight-grad kernel for this descriptor (64 / 128; 0: another kernel)."""
    rc = lib().scd_wgrad_rows_per_block(ctypes.byref(d))
    _check(min(rc, 0), "scd_wgrad_rows_per_block")
    return rc


def igemm_input_bn_supported(src: NHWC, out_h: int, out_w: int, stride: int, taps, wpk: torch.Tensor, n_out: int,
                             dst: NHWC, in_bn, src_bound=None) -> bool:
    d = _igemm_desc(src, out_h, out_w, stride, taps, wpk, n_out, None, dst, 0, None, in_bn, src_bound=src_bound)
    return lib().scd_igemm_input_bn_supported(ctypes.byref(d)) == 1


def igemm_stat_tiles(src: NHWC, out_h: int, out_w: int, stride: int, taps, wpk: torch.Tensor, n_out: int,
                     dst: NHWC, src_bound=None) -> tuple[int, int]:
    """(tiles, pixels per tile) of the conv-fused BatchNorm statistics for this conv, (0, 0) if unavailable."""
    d = _igemm_desc(src, out_h, out_w, stride, taps, wpk, n_out, None, dst, 0, src_bound=src_bound)
    tp = c_int32(0)
    n = lib().scd_igemm_stat_tiles(ctypes.byref(d), ctypes.byref(tp))
    return (n, tp.value) if n > 0 else (0, 0)


def wgrad_desc(rows: NHWC, src: NHWC, stride: int, taps, src_bn=None, rows_bound=None, src_bound=None) -> 'WGRAD':
    """An scd_wgrad_t stamped with the current arithmetic and tune bits."""
    nt, dy, dx = _taps(taps)
    sc, sh, nseg = src_bn if src_bn is not None else (None, None, 0)
    d = WGRAD(rows, src, stride, nt, dy, dx, _ptr(sc), _ptr(sh), nseg, _ptr(rows_bound), _ptr(src_bound))
    d.math, d.tune = _cur()
    return d


def _rows_bn_fields(d: 'WGRAD', rows_bn):
    """rows_bn = (y NHWC, nseg, save_mean, save_invstd, gamma or None, scale, shift, coef): the rows are dL/da and
    the kernel forms dy through the BatchNorm backward while staging (scd_wgrad_t.rows_y)."""
    y, nseg, mean, inv, gamma, sc, sh, coef = rows_bn
    d.rows_y = y
    d.rows_nseg = nseg
    d.rows_mean, d.rows_invstd, d.rows_gamma = _ptr(mean), _ptr(inv), _ptr(gamma)
    d.rows_scale, d.rows_shift, d.rows_coef = _ptr(sc), _ptr(sh), _ptr(coef)


def wgrad_plan(rows: NHWC, src: NHWC, stride: int, taps, src_bn=None, rows_bound=None, src_bound=None,
               rows_bn=None, rows_out: NHWC | None = None, rows_out_bound=None):
    """`src_bn` = (scale, shift, nseg): read src through its BatchNorm-apply + ReLU (see scd_wgrad_t).
    `rows_bound` / `src_bound`: device floats bounding |rows| and |src as read| (SCD_MATH_H2; both or neither).
    `rows_bn`: see _rows_bn_fields (only where wgrad_rows_bn_supported); with it, `rows_out` (a view shaped as rows)
    receives the formed dY and `rows_out_bound` (device float) is raised to max |dY| (ABI 8, halo weight grads)."""
    d = wgrad_desc(rows, src, stride, taps, src_bn, rows_bound, src_bound)
    if rows_bn is not None:
        _rows_bn_fields(d, rows_bn)
    if rows_out is not None:
        d.rows_out = rows_out
        d.rows_out_bound = _ptr(rows_out_bound)
    d._keep = (rows_bound, src_bound, rows_bn, rows_out_bound)
    ns = c_int32(0)
    nb = c_size_t(0)
    _check(lib().scd_wgrad_plan(ctypes.byref(d), ctypes.byref(ns), ctypes.byref(nb)), "scd_wgrad_plan")
    return d, ns.value, nb.value


def wgrad_src_bn_supported(rows: NHWC, src: NHWC, stride: int, taps, src_bn) -> bool:
    d = wgrad_desc(rows, src, stride, taps, src_bn)
    return lib().scd_wgrad_src_bn_supported(ctypes.byref(d)) == 1


def wgrad_rows_bn_supported(rows: NHWC, src: NHWC, stride: int, taps, src_bn=None, rows_bound=None,
                            src_bound=None) -> bool:
    """Whether the weight grad for (rows, src) can form its rows through the fused BatchNorm backward (with the
    operand bounds and src transform the launch will carry: they select the arithmetic)."""
    d = wgrad_desc(rows, src, stride, taps, src_bn, rows_bound, src_bound)
    return lib().scd_wgrad_rows_bn_supported(ctypes.byref(d)) == 1


def conv_wgrad(d: WGRAD, slabs: torch.Tensor):
    _check(lib().scd_conv_wgrad(ctypes.byref(d), slabs.data_ptr(), slabs.numel() * 4, _stream()), "scd_conv_wgrad")


def wgrad_finalize(slabs, nsplit, R, ntaps, C, mode, c_valid, out: torch.Tensor):
    _check(lib().scd_wgrad_finalize(slabs.data_ptr(), nsplit, R, ntaps, C, mode, c_valid, out.data_ptr(), _stream()),
           "scd_wgrad_finalize")


def wgrad_colsum_supported(d: 'WGRAD') -> bool:
    """Whether the weight-grad kernel for `d` also writes the src column sums (scd_wgrad_t.src_colsum)."""
    return bool(lib().scd_wgrad_colsum_supported(ctypes.byref(d)))


def wgrad_colsum_finalize(colsum: torch.Tensor, nsplit: int, ntaps: int, C: int, out: torch.Tensor):
    """out[c] = sum over splits and taps of colsum[s][t*C + c] (the ConvTranspose bias grad)."""
    _check(lib().scd_wgrad_colsum_finalize(colsum.data_ptr(), nsplit, ntaps, C, out.data_ptr(), _stream()),
           "scd_wgrad_colsum_finalize")


def bn_workspace_bytes(n, h, w, c, nseg) -> int:
    return lib().scd_bn_workspace_bytes(n, h, w, c, nseg)


def bn_train_stats(y: NHWC, nseg, gamma, beta, eps, momentum, update, rmean, rvar, smean, sinv, scale, shift, ws,
                   act_bound=None):
    """`act_bound`: device float raised to a bound of |relu(BN(y))| (SCD_MATH_H2 operand scaling)."""
    _check(
        lib().scd_bn_train_stats(y, nseg, _ptr(gamma), _ptr(beta), eps, momentum, int(update), _ptr(rmean), _ptr(rvar),
                                 smean.data_ptr(), sinv.data_ptr(), scale.data_ptr(), shift.data_ptr(), _ptr(act_bound),
                                 ws.data_ptr(), ws.numel(), _stream()),
        "scd_bn_train_stats")


def bn_tile_stats_workspace_bytes(ntiles, c, nseg) -> int:
    return lib().scd_bn_tile_stats_workspace_bytes(ntiles, c, nseg)


def bn_stats_from_tiles(tile_rec, ntiles, tile_px, c, nseg, gamma, beta, eps, momentum, update, rmean, rvar, smean,
                        sinv, scale, shift, ws, act_bound=None):
    _check(
        lib().scd_bn_stats_from_tiles(tile_rec.data_ptr(), ntiles, tile_px, c, nseg, _ptr(gamma), _ptr(beta), eps,
                                      momentum, int(update), _ptr(rmean), _ptr(rvar), smean.data_ptr(),
                                      sinv.data_ptr(), scale.data_ptr(), shift.data_ptr(), _ptr(act_bound),
                                      ws.data_ptr(), ws.numel(), _stream()),
        "scd_bn_stats_from_tiles",
    )


def bn_eval_coeffs(c, gamma, beta, rmean, rvar, eps, scale, shift):
    _check(lib().scd_bn_eval_coeffs(c, _ptr(gamma), _ptr(beta), rmean.data_ptr(), rvar.data_ptr(), eps,
                                    scale.data_ptr(), shift.data_ptr(), _stream()), "scd_bn_eval_coeffs")


def absmax_bound(x: NHWC, bound: torch.Tensor, nseg: int = 1, scale=None, shift=None):
    """bound = max(bound, max |x|) (or of relu(x * scale + shift) per segment); bound is a device float."""
    _check(lib().scd_absmax_bound(x, nseg, _ptr(scale), _ptr(shift), bound.data_ptr(), _stream()), "scd_absmax_bound")


def bn_relu_apply(y: NHWC, nseg, scale, shift, a: NHWC):
    _check(lib().scd_bn_relu_apply(y, nseg, scale.data_ptr(), shift.data_ptr(), a, _stream()), "scd_bn_relu_apply")


def bn_relu_backward(y: NHWC, da: NHWC, nseg, smean, sinv, gamma, scale, shift, dgamma, dbeta, dbias, dy: NHWC, ws,
                     dy_bound=None):
    """`dy_bound`: device float raised to max |dy| (SCD_MATH_H2 operand scaling of the convs reading dy)."""
    _check(
        lib().scd_bn_relu_backward(y, da, nseg, smean.data_ptr(), sinv.data_ptr(), _ptr(gamma), scale.data_ptr(),
                                   shift.data_ptr(), _ptr(dgamma), _ptr(dbeta), _ptr(dbias), dy, _ptr(dy_bound),
                                   ws.data_ptr(), ws.numel(), _stream()),
        "scd_bn_relu_backward")


def bn_relu_backward_pooled(y: NHWC, gy: NHWC, idx, gskip: NHWC, skip_mode: int, nseg, smean, sinv, gamma, scale,
                            shift, dgamma, dbeta, dbias, dy: NHWC, ws, dy_bound=None):
    """bn_relu_backward of da = maxpool_bwd(gy, idx) -/+ gskip (feature_grad's operand, never materialised)."""
    _check(
        lib().scd_bn_relu_backward_pooled(y, gy, _ptr(idx), gskip, skip_mode, nseg, smean.data_ptr(), sinv.data_ptr(),
                                          _ptr(gamma), scale.data_ptr(), shift.data_ptr(), _ptr(dgamma), _ptr(dbeta),
                                          _ptr(dbias), dy, _ptr(dy_bound), ws.data_ptr(), ws.numel(), _stream()),
        "scd_bn_relu_backward_pooled")


def bn_relu_backward_pooled2(y: NHWC, gy: NHWC, idx, gskip: NHWC, skip_mode: int, gskip2: NHWC, nseg, smean, sinv,
                             gamma, scale, shift, dgamma, dbeta, dbias, dy: NHWC, ws, dy_bound=None):
    """bn_relu_backward_pooled with the dual-task second skip gradient (skip_mode 2: gskip2 = the semantic decoder's
    [t2; t1] skip gradient, added to the -/+ difference gradient before the pooled term)."""
    _check(
        lib().scd_bn_relu_backward_pooled2(y, gy, _ptr(idx), gskip, skip_mode, gskip2, nseg, smean.data_ptr(),
                                           sinv.data_ptr(), _ptr(gamma), scale.data_ptr(), shift.data_ptr(),
                                           _ptr(dgamma), _ptr(dbeta), _ptr(dbias), dy, _ptr(dy_bound), ws.data_ptr(),
                                           ws.numel(), _stream()),
        "scd_bn_relu_backward_pooled2")


def bn_head_workspace_bytes(n, h, w, c, nseg, n_out) -> int:
    return lib().scd_bn_head_workspace_bytes(n, h, w, c, nseg, n_out)


def bn_relu_backward_head(y: NHWC, gout: torch.Tensor, w_head: torch.Tensor, n_out: int, nseg, smean, sinv, gamma,
                          scale, shift, dgamma, dbeta, dbias, dy: NHWC, ws, dy_bound=None, w_grad=None):
    """bn_relu_backward of da = gout . w_head, the 1x1 head's input gradient (conv1x1_bwd's gx, never materialised);
    gout NCHW [n][n_out][h][w], w_head [n_out][C].  `w_grad` ([n_out][C]): also the head's weight grad from the same
    pass (workspace bn_head_workspace_bytes)."""
    _check(
        lib().scd_bn_relu_backward_head(y, gout.data_ptr(), w_head.data_ptr(), n_out, nseg, smean.data_ptr(),
                                        sinv.data_ptr(), _ptr(gamma), scale.data_ptr(), shift.data_ptr(), _ptr(dgamma),
                                        _ptr(dbeta), _ptr(dbias), dy, _ptr(dy_bound), _ptr(w_grad), ws.data_ptr(),
                                        ws.numel(), _stream()),
        "scd_bn_relu_backward_head")


def bn_relu_backward_tiles(y: NHWC, da: NHWC, nseg, smean, sinv, gamma, scale, shift, tile_rec, ntiles, dgamma, dbeta,
                           dbias, dy: NHWC, ws, dy_bound=None):
    """bn_relu_backward with the partial sums from conv-epilogue tile records (conv_igemm(..., bn_bwd=...))."""
    _check(
        lib().scd_bn_relu_backward_tiles(y, da, nseg, smean.data_ptr(), sinv.data_ptr(), _ptr(gamma), scale.data_ptr(),
                                         shift.data_ptr(), tile_rec.data_ptr(), ntiles, _ptr(dgamma), _ptr(dbeta),
                                         _ptr(dbias), dy, _ptr(dy_bound), ws.data_ptr(), ws.numel(), _stream()),
        "scd_bn_relu_backward_tiles")


def bn_relu_backward_coef(y: NHWC, da: NHWC, nseg, smean, sinv, gamma, scale, shift, tile_rec, ntiles, coef, dgamma,
                          dbeta, dbias, ws, da_bound=None, dy_bound=None):
    """The statistics half of bn_relu_backward(_tiles): coef [nseg][C][2], dgamma, dbeta, dbias (sum dy, from the
    sums) for a consumer that forms dy itself (wgrad_plan(..., rows_bn=...)).  tile_rec None: a pass over (y, da).
    `dy_bound` (with `da_bound`, a bound of |da|): raised to a bound of |dy| from the statistics (the h2 rows bound of
    that consumer)."""
    _check(
        lib().scd_bn_relu_backward_coef(y, da, nseg, smean.data_ptr(), sinv.data_ptr(), _ptr(gamma), scale.data_ptr(),
                                        shift.data_ptr(), _ptr(tile_rec), ntiles, coef.data_ptr(), _ptr(dgamma),
                                        _ptr(dbeta), _ptr(dbias), _ptr(da_bound), _ptr(dy_bound), ws.data_ptr(),
                                        ws.numel(), _stream()),
        "scd_bn_relu_backward_coef")


def channel_sum(x: NHWC, out: torch.Tensor, ws: torch.Tensor):
    _check(lib().scd_channel_sum(x, out.data_ptr(), ws.data_ptr(), ws.numel(), _stream()), "scd_channel_sum")


def maxpool2_fwd(x: NHWC, y: NHWC, idx: torch.Tensor):
    _check(lib().scd_maxpool2_fwd(x, y, idx.data_ptr(), _stream()), "scd_maxpool2_fwd")


def bn_relu_maxpool2_fwd(x: NHWC, nseg: int, scale, shift, y: NHWC, idx: torch.Tensor):
    """MaxPool2d(2) of max(fma(x, scale, shift), 0) per segment (BatchNorm-apply + ReLU fused into the pool)."""
    _check(lib().scd_bn_relu_maxpool2_fwd(x, nseg, scale.data_ptr(), shift.data_ptr(), y, idx.data_ptr(), _stream()),
           "scd_bn_relu_maxpool2_fwd")


def bn_relu_siamese_diff(a: NHWC, scale, shift, d: NHWC):
    """d = relu(bn_t2(a[n:])) - relu(bn_t1(a[:n])) with per-branch coefficients [2][C]."""
    _check(lib().scd_bn_relu_siamese_diff(a, scale.data_ptr(), shift.data_ptr(), d, _stream()),
           "scd_bn_relu_siamese_diff")


def bn_relu_pool_diff(a: NHWC, scale, shift, d: NHWC, y: NHWC, idx: torch.Tensor):
    """bn_relu_siamese_diff(a, ..., d) and bn_relu_maxpool2_fwd(a, 2, ..., y, idx) in one read of a (even h, w)."""
    _check(lib().scd_bn_relu_pool_diff(a, scale.data_ptr(), shift.data_ptr(), d, y, idx.data_ptr(), _stream()),
           "scd_bn_relu_pool_diff")


POOL_DIFF, POOL_COPY, POOL_DIFF_COPY = 0, 1, 2  # scd_bn_relu_pool_out modes


def bn_relu_pool_out(a: NHWC, nseg: int, scale, shift, mode: int, d: NHWC, o: NHWC, y: NHWC, idx):
    """One pass over an encoder level's conv output a (even h, w): mode 0 the Siamese difference d, 1 the activation
    into o (a concat-buffer slice), 2 both with o = [a_t2; a_t1]; plus MaxPool2d(2) into y / idx unless y is _NULL."""
    _check(lib().scd_bn_relu_pool_out(a, nseg, scale.data_ptr(), shift.data_ptr(), mode, d, o, y, _ptr(idx),
                                      _stream()), "scd_bn_relu_pool_out")


def feature_grad(gy: NHWC, idx, gskip: NHWC, skip_mode: int, gx: NHWC, accumulate: bool = False):
    _check(lib().scd_feature_grad(gy, _ptr(idx), gskip, skip_mode, gx, int(accumulate), _stream()), "scd_feature_grad")


def siamese_diff(a: NHWC, d: NHWC):
    _check(lib().scd_siamese_diff(a, d, _stream()), "scd_siamese_diff")


def conv1x1_fwd(x: NHWC, w, b, n_out, out: torch.Tensor):
    _check(lib().scd_conv1x1_fwd(x, w.data_ptr(), _ptr(b), n_out, out.data_ptr(), _stream()), "scd_conv1x1_fwd")


def conv1x1_fwd_bn(y: NHWC, scale, shift, nseg, w, b, n_out, out: torch.Tensor):
    """conv1x1_fwd of relu(fma(y, scale, shift)) (the head reading its input through the last BatchNorm + ReLU)."""
    _check(lib().scd_conv1x1_fwd_bn(y, scale.data_ptr(), shift.data_ptr(), nseg, w.data_ptr(), _ptr(b), n_out,
                                    out.data_ptr(), _stream()), "scd_conv1x1_fwd_bn")


def conv1x1_fwd_bn2(ya: NHWC, sa, ha, yb: NHWC, sb, hb, nseg, w, b, n_out, out: torch.Tensor):
    """The heads over cat([relu(bn_a(ya)), relu(bn_b(yb))]) without the cat (w [n_out][ya.c + yb.c]); coefficients for
    both sources or for neither (sa = None: the sources are plain activations)."""
    _check(lib().scd_conv1x1_fwd_bn2(ya, _ptr(sa), _ptr(ha), yb, _ptr(sb), _ptr(hb), nseg, w.data_ptr(), _ptr(b), n_out,
                                     out.data_ptr(), _stream()), "scd_conv1x1_fwd_bn2")


def conv1x1_bwd_bn(y: NHWC, scale, shift, nseg, w, gout, n_out, gw, gb, ws):
    """The head's weight / bias grads with its input read through the last BatchNorm + ReLU."""
    _check(lib().scd_conv1x1_bwd_bn(y, scale.data_ptr(), shift.data_ptr(), nseg, w.data_ptr(), gout.data_ptr(), n_out,
                                    _ptr(gw), _ptr(gb), ws.data_ptr(), ws.numel(), _stream()), "scd_conv1x1_bwd_bn")


def conv1x1_workspace_bytes(x: NHWC, n_out) -> int:
    return lib().scd_conv1x1_workspace_bytes(x, n_out)


def conv1x1_bwd(x: NHWC, w, gout, n_out, gx: NHWC, accumulate, gw, gb, ws):
    _check(lib().scd_conv1x1_bwd(x, w.data_ptr(), gout.data_ptr(), n_out, gx, int(accumulate), _ptr(gw), _ptr(gb),
                                 ws.data_ptr(), ws.numel(), _stream()), "scd_conv1x1_bwd")


def pjaccard_workspace_bytes(n) -> int:
    return lib().scd_pjaccard_workspace_bytes(n)


def pjaccard_fwd(logits, target, sums, loss, ws):
    _check(lib().scd_pjaccard_fwd(logits.data_ptr(), target.data_ptr(), logits.numel(), sums.data_ptr(),
                                  loss.data_ptr(), ws.data_ptr(), ws.numel(), _stream()), "scd_pjaccard_fwd")


def pjaccard_bwd(logits, target, sums, gloss, glogits, gtarget=None):
    _check(lib().scd_pjaccard_bwd(logits.data_ptr(), target.data_ptr(), logits.numel(), sums.data_ptr(),
                                  _ptr(gloss), glogits.data_ptr(), _ptr(gtarget), _stream()), "scd_pjaccard_bwd")


def pjaccard_loss_from_sums(sums, loss):
    """Re-form D and the loss from (all-reduced) sums {I, sum(p^2 + t^2), D} in place (exact-DataParallel loss)."""
    _check(lib().scd_pjaccard_loss_from_sums(sums.data_ptr(), loss.data_ptr(), _stream()), "scd_pjaccard_loss_from_sums")


def window_copy(src: NHWC, dst: NHWC, oy: int, ox: int):
    """dst[n, y, x] = src[n, y + oy, x + ox] where it exists, else 0 (Up's F.pad and its backward crop)."""
    _check(lib().scd_window_copy(src, dst, oy, ox, _stream()), "scd_window_copy")


THRESHOLD_MAX = 16  # thresholds per scd_threshold_counts launch


def threshold_counts_workspace_bytes(n: int, n_thr: int) -> int:
    return lib().scd_threshold_counts_workspace_bytes(n, n_thr)


def threshold_counts(pred: torch.Tensor, truth: torch.Tensor, thresholds: torch.Tensor, from_logits: bool,
                     counts: torch.Tensor, ws: torch.Tensor):
    """counts (int64[1 + 2T]) = {#label, per threshold: TP, #positive} of utils/metrics.py:22-31."""
    n = pred.numel()
    if truth.numel() != n or counts.numel() != 1 + 2 * thresholds.numel() or counts.dtype != torch.int64:
        raise ValueError("threshold_counts: pred/truth sizes or counts buffer mismatch")
    _check(lib().scd_threshold_counts(pred.data_ptr(), truth.data_ptr(), n, thresholds.data_ptr(), thresholds.numel(),
                                      int(from_logits), counts.data_ptr(), ws.data_ptr(), ws.numel(), _stream()),
           "scd_threshold_counts")


class JTERM(ctypes.Structure):
    _fields_ = [("logits", c_void_p), ("target", c_void_p), ("glogits", c_void_p), ("gtarget", c_void_p),
                ("coef", c_float), ("select", c_int32), ("soft_target", c_int32), ("zero_unselected", c_int32)]


def _jterms(terms):
    arr = (JTERM * len(terms))()
    for i, t in enumerate(terms):
        arr[i] = JTERM(_ptr(t['logits']), _ptr(t['target']), _ptr(t.get('glogits')), _ptr(t.get('gtarget')),
                       float(t['coef']), int(t['select']), int(t.get('soft', 0)), int(t.get('zero', 0)))
    return arr


def jaccard_multi_fwd(terms, labeled: torch.Tensor, n_samples: int, pixels: int, sums, loss):
    """terms: dicts {logits, target, coef, select, soft}; labeled: device uint8 [n_samples]."""
    ws = torch.empty(lib().scd_jaccard_multi_workspace_bytes(len(terms)), dtype=torch.uint8, device=labeled.device)
    arr = _jterms(terms)
    _check(lib().scd_jaccard_multi_fwd(ctypes.cast(arr, c_void_p), len(terms), labeled.data_ptr(), n_samples, pixels,
                                       sums.data_ptr(), loss.data_ptr(), ws.data_ptr(), ws.numel(), _stream()),
           "scd_jaccard_multi_fwd")


def jaccard_multi_bwd(terms, labeled: torch.Tensor, n_samples: int, pixels: int, sums, gloss):
    """terms as jaccard_multi_fwd plus {glogits, gtarget, zero}."""
    arr = _jterms(terms)
    _check(lib().scd_jaccard_multi_bwd(ctypes.cast(arr, c_void_p), len(terms), labeled.data_ptr(), n_samples, pixels,
                                       sums.data_ptr(), _ptr(gloss), _stream()), "scd_jaccard_multi_bwd")


def _ptr_table(tensors, device):
    return torch.tensor([t.data_ptr() for t in tensors], dtype=torch.int64).to(device)


def window_label_sums(labels: list, yx: torch.Tensor, crop: int) -> torch.Tensor:
    """labels: per-sample device HW(1) fp32 tiles; yx: int32 [B][ncand][2] -> sums float [B][ncand]."""
    dev = labels[0].device
    B, ncand = yx.shape[0], yx.shape[1]
    hw = torch.tensor([[t.shape[0], t.shape[1]] for t in labels], dtype=torch.int32).to(dev)
    ptrs = _ptr_table(labels, dev)
    yx = yx.to(device=dev, dtype=torch.int32).contiguous()
    out = torch.empty((B, ncand), dtype=torch.float32, device=dev)
    _check(lib().scd_window_label_sums(ptrs.data_ptr(), hw.data_ptr(), yx.data_ptr(), B, ncand, crop, out.data_ptr(),
                                       _stream()), "scd_window_label_sums")
    return out


def augment_apply(tiles: list, crop: int, params: torch.Tensor, scale=None, gamma=None) -> torch.Tensor:
    """tiles: per-sample device HWC fp32 (same C); params int32 [B][5]; scale/gamma float64 [B][C] or None."""
    dev = tiles[0].device
    B, C = len(tiles), tiles[0].shape[2]
    for t in tiles:
        if t.dim() != 3 or t.shape[2] != C or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("augment_apply: tiles must be contiguous HWC fp32 with the same channel count")
    hw = torch.tensor([[t.shape[0], t.shape[1]] for t in tiles], dtype=torch.int32).to(dev)
    ptrs = _ptr_table(tiles, dev)
    params = params.to(device=dev, dtype=torch.int32).contiguous()
    sc = None if scale is None else scale.to(device=dev, dtype=torch.float64).contiguous()
    gm = None if gamma is None else gamma.to(device=dev, dtype=torch.float64).contiguous()
    out = torch.empty((B, C, crop, crop), dtype=torch.float32, device=dev)
    _check(lib().scd_augment_apply(ptrs.data_ptr(), hw.data_ptr(), B, C, crop, params.data_ptr(), _ptr(sc), _ptr(gm),
                                   out.data_ptr(), _stream()), "scd_augment_apply")
    return out


def jaccard_multi_loss_from_sums(terms, sums, loss):
    """The multi-term loss re-formed from (all-reduced) per-term sums [n_terms][4] (exact-DataParallel loss)."""
    arr = _jterms(terms)
    _check(lib().scd_jaccard_multi_loss_from_sums(ctypes.cast(arr, c_void_p), len(terms), sums.data_ptr(),
                                                  loss.data_ptr(), _stream()), "scd_jaccard_multi_loss_from_sums")
