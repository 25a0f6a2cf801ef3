"""ctypes binding of ``libnos_hip.so`` (gfx950 kernels + CU-mask streams).

The library is linked against PyTorch's own HIP runtime, so ``torch`` is
imported first and raw device pointers / ``hipStream_t`` handles from torch
are passed straight through.  On a machine with a GPU the library MUST load:
:func:`lib` raises instead of silently falling back to eager PyTorch
(``NOS_AMD_ALLOW_FALLBACK=1`` relaxes that for debugging only).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

# NOS_AMD_HIP_LIB: load an experimental kernel variant (tools/build_variant.py) instead
_LIB_PATH = Path(os.environ.get("NOS_AMD_HIP_LIB") or
                 Path(__file__).resolve().parent.parent / "_native" / "libnos_hip.so")
_lock = threading.Lock()
_lib: ctypes.CDLL | None = None
_err: str | None = None

c_int, c_ll, c_float, c_void_p, c_double = (ctypes.c_int, ctypes.c_longlong, ctypes.c_float,
                                            ctypes.c_void_p, ctypes.c_double)

_SIGS = {
    "nos_attn_fwd_d64": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                         c_ll, c_int, c_ll, c_float, c_void_p],
    "nos_attn_fwd_f32_d64": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                             c_ll, c_int, c_ll, c_float, c_void_p],
    "nos_attn_fwd_f32x6_d64": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                               c_ll, c_int, c_ll, c_float, c_void_p, c_ll, c_void_p],
    "nos_attn_f32x6_workspace": [c_int, c_int, c_int, c_int],
    "nos_attn_fwd_f32x6_presplit_d64": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_ll, c_int, c_ll,
                                        c_float, c_void_p, c_ll, c_void_p],
    "nos_gemm_ln_f32x6_qkv": [c_void_p, c_int, c_void_p, c_int, c_ll, c_void_p, c_void_p, c_void_p, c_int, c_int,
                              c_int, c_int, c_int, c_float, c_void_p, c_int, c_int, c_void_p],
    "nos_gemm_ln_f32x6_qkv_h3": [c_void_p, c_int, c_void_p, c_int, c_ll, c_void_p, c_void_p, c_void_p, c_int,
                                 c_int, c_int, c_int, c_int, c_float, c_void_p, c_int, c_int, c_void_p, c_void_p],
    "nos_attn_fwd_f32h3_presplit_d64": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_ll, c_int, c_ll,
                                        c_float, c_void_p, c_void_p, c_ll, c_void_p, c_ll, c_float, c_void_p],
    "nos_attn_f32x6_set_kvsplit": [c_int],
    "nos_split_cols_h3": [c_void_p, c_int, c_ll, c_int, c_int, c_int, c_void_p, c_int, c_ll, c_void_p, c_void_p,
                          c_void_p],
    "nos_split_rows_h3": [c_void_p, c_int, c_void_p, c_int, c_ll, c_void_p, c_int, c_int, c_int, c_float, c_int,
                          c_void_p],
    "nos_gemm_f32h3": [c_void_p, c_int, c_ll, c_void_p, c_float, c_void_p, c_int, c_ll, c_void_p, c_void_p,
                       c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                       c_void_p, c_int, c_ll, c_float, c_void_p],
    "nos_gemm_f32h3_set_layout": [c_int],
    "nos_attn_f32h3_set_waves": [c_int],
    "nos_gemm_bf16": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int,
                      c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nos_gemm_f32": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int,
                     c_int, c_int, c_void_p],
    "nos_gemm_ln_f32": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                        c_int, c_float, c_void_p],
    "nos_gemm_f32x6": [c_void_p, c_int, c_void_p, c_int, c_ll, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                       c_int, c_int, c_int, c_void_p],
    "nos_gemm_ln_f32x6": [c_void_p, c_int, c_void_p, c_int, c_ll, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                          c_int, c_int, c_float, c_void_p],
    "nos_gemm_f32_pick_tile": [c_int, c_int],
    "nos_gemm_f32x6_set_stage": [c_int],
    "nos_gemm_f32x6_set_tile": [c_int],
    "nos_gemm_f32x6_set_pipeline": [c_int],
    "nos_gemm_set_policy": [c_int],
    "nos_gemm_set_persistent": [c_int],
    "nos_gemm_f32_set_policy": [c_int],
    "nos_attn_f32_set_variant": [c_int],
    "nos_gemm_ln_bf16": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                         c_int, c_int, c_float, c_int, c_void_p],
    "nos_layernorm_bf16": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                           c_int, c_int, c_int, c_int, c_float, c_void_p],
    "nos_probe_placement": [c_void_p, c_int, c_int, c_void_p],
    "nos_probe_hbm_copy": [c_void_p, c_void_p, c_ll, c_int, c_void_p],
    "nos_probe_hbm": [c_void_p, c_ll, c_int, c_int, ctypes.POINTER(c_double)],
    "nos_probe_hbm_mode": [c_void_p, c_ll, c_int, c_int, c_int, ctypes.POINTER(c_double)],
    "nos_probe_mfma_peak": [c_void_p, c_int, c_int, ctypes.POINTER(c_double)],
    "nos_probe_mfma_peak_launch": [c_void_p, c_int, c_int, c_void_p],
    "nos_probe_gemm": [c_void_p, c_int, c_int, c_int, ctypes.POINTER(c_double)],
    "nos_stream_create_cumask": [ctypes.POINTER(ctypes.c_uint), c_int, ctypes.POINTER(c_void_p)],
    "nos_stream_get_cumask": [c_void_p, c_int, ctypes.POINTER(ctypes.c_uint)],
    "nos_stream_destroy": [c_void_p],
    "nos_stream_sync": [c_void_p],
    "nos_device_info": [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_ll), ctypes.POINTER(c_int),
                        ctypes.c_char_p, c_int],
    "nos_runtime_version": [ctypes.POINTER(c_int)],
    "nos_set_cu_budget": [c_int],
    "nos_get_cu_budget": [],
    # general tenant programs (tenant_ops.hip, attention_h3g.hip, gemm_f32h.hip)
    "nos_gemm_f32h3_batched": [c_void_p, c_int, c_ll, c_ll, c_void_p, c_ll, c_float, c_void_p, c_int, c_ll, c_ll,
                               c_void_p, c_ll, c_void_p, c_ll, c_void_p, c_int, c_ll, c_void_p, c_int, c_ll, c_int,
                               c_int, c_int, c_int, c_int, c_void_p],
    "nos_embedding": [c_void_p, c_void_p, c_void_p, c_ll, c_int, c_int, c_void_p],
    "nos_rmsnorm": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_int, c_void_p],
    "nos_softmax": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nos_rotary": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_ll, c_int, c_void_p],
    "nos_im2col_h3": [c_void_p, c_void_p, c_ll, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                      c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nos_im2col": [c_void_p, c_ll, c_ll, c_ll, c_void_p, c_ll, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                   c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nos_unary": [c_void_p, c_int, c_void_p, c_int, c_ll, c_int, c_void_p],
    "nos_unary_rows": [c_void_p, c_ll, c_int, c_void_p, c_int, c_ll, c_int, c_int, c_void_p],
    "nos_glu": [c_void_p, c_int, c_void_p, c_int, c_void_p, c_ll, c_int, c_int, c_int, c_void_p],
    # decode.hip: stateful decoding (K / V caches and positions on the device) and skinny GEMMs
    "nos_kv_write": [c_void_p, c_int, c_int, c_ll, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                     c_int, c_int, c_int, c_void_p, c_int, c_ll, c_void_p, c_void_p],
    "nos_rotary_pos": [c_void_p, c_int, c_ll, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                       c_int, c_int, c_void_p],
    "nos_attn_decode_workspace": [c_int, c_int, c_int, c_int, c_int, c_int],
    "nos_attn_decode": [c_void_p, c_int, c_int, c_ll, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                        c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_ll,
                        c_void_p, c_void_p, c_int, c_int, c_ll, c_int, c_ll, c_int, c_void_p, c_ll, c_int, c_void_p],
    "nos_pos_update": [c_void_p, c_int, c_int, c_int, c_void_p],
    "nos_argmax": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p],
    "nos_gemv": [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                 c_int, c_int, c_int, c_float, c_void_p],
    "nos_gemv_partials": [c_void_p, c_ll, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p,
                          c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "nos_attn_h3g_workspace": [c_int, c_int, c_int, c_int, c_int, c_int],
    # LayerNorm hand-off (gemm_f32h.hip): producer row statistics, LN in the consumer's A load
    "nos_gemm_f32h3_stats": [c_void_p, c_int, c_ll, c_void_p, c_float, c_void_p, c_int, c_ll, c_void_p, c_void_p,
                             c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p],
    "nos_gemm_f32h3_lna": [c_void_p, c_int, c_void_p, c_int, c_int, c_float, c_int, c_void_p, c_int, c_ll, c_void_p,
                           c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                           c_int, c_void_p, c_void_p, c_int, c_ll, c_float, c_void_p],
    "nos_row_stats": [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p],
    "nos_gemm_f32h3_set_lds_epilogue": [c_int],
    "nos_gemm_f32h3_set_hot_ring": [c_int],
    "nos_gemm_f32h3_set_hot_bn": [c_int],
    "nos_gemm_f32h3_hot_bn": [],
    "nos_gemm_f32h3_set_lna_wide": [c_int],
    "nos_attn_h3g_set_kvsplit": [c_int],
    "nos_attn_h3g": [c_void_p, c_int, c_ll, c_void_p, c_int, c_ll, c_void_p, c_int, c_ll, c_void_p, c_int, c_ll,
                     c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_float, c_void_p,
                     c_ll, c_void_p],
}


_RESTYPES = {"nos_attn_f32x6_workspace": c_ll, "nos_attn_h3g_workspace": c_ll, "nos_attn_decode_workspace": c_ll}


class NativeUnavailable(RuntimeError):
    pass


def lib_path() -> Path:
    return _LIB_PATH


def _load() -> ctypes.CDLL:
    import torch  # noqa: F401  -- binds the process's HIP runtime first

    if not _LIB_PATH.exists():
        raise NativeUnavailable(
            f"{_LIB_PATH} missing: run `python -m nos_amd._native.build` (hipcc, gfx950)")
    L = ctypes.CDLL(str(_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    override = bool(os.environ.get("NOS_AMD_HIP_LIB"))
    for name, argtypes in _SIGS.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            # an older library named by NOS_AMD_HIP_LIB (A/B runs against the previous build):
            # a config setter it lacks leaves that config at its default, any other entry
            # point it lacks raises when called
            if override:
                if "_set_" in name:
                    setattr(L, name, lambda *a: 0)
                else:
                    def _missing(*a, _n=name):
                        raise NativeUnavailable(f"{_LIB_PATH} has no {_n}")

                    setattr(L, name, _missing)
                continue
            raise
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, c_int)
    return L


def lib() -> ctypes.CDLL:
    global _lib, _err
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            try:
                _lib = _load()
            except Exception as e:  # pragma: no cover - depends on build state
                _err = str(e)
                raise NativeUnavailable(_err) from e
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def require_native_on_gpu() -> None:
    """Raise if a GPU is present but the native library cannot be loaded."""
    import torch

    if torch.cuda.is_available() and not available() and os.environ.get("NOS_AMD_ALLOW_FALLBACK") != "1":
        raise NativeUnavailable(f"GPU present but libnos_hip.so not loadable: {_err}")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")
