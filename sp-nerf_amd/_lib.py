"""ctypes binding of libspnerf_amd.so (the C ABI declared in include/spnerf_amd.h).

The library is built in-tree (``make -C sp-nerf_amd`` or ``__graft_entry__.build()``).  There
is no fallback: every compute entry point raises if the library is missing or if it is handed
CPU tensors — the render path runs on the MI355X HIP kernels or not at all.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int32, c_int64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
# SPNERF_AMD_LIB: another in-tree build of the same sources (A/B runs of compile-time variants)
LIB_PATH = os.path.join(HERE, os.environ.get("SPNERF_AMD_LIB", "libspnerf_amd.so"))

SPNERF_MLP_SAVE = 1
SPNERF_MLP_SIGMA_ONLY = 2
SPNERF_MLP_SUN_ONLY = 4
SPNERF_MLP_ACCUMULATE = 8
SPNERF_MLP_DEFER_TRUNK_WGRAD = 16
SPNERF_COMP_WEIGHTS_ONLY = 1
SPNERF_COMP_SUN_COLUMN = 2


class ModelCfg(ctypes.Structure):
    """spnerf_model_cfg (include/spnerf_amd.h)."""
    _fields_ = [("width", c_int32), ("layers", c_int32), ("skip", c_int32), ("n_freq", c_int32),
                ("sem_classes", c_int32), ("sem_dim", c_int32), ("beta", c_int32), ("t_dim", c_int32),
                ("dtype", c_int32), ("reserved", c_int32 * 7)]

    def key(self):
        return tuple(getattr(self, f) for f, _ in self._fields_[:-1])


class Rng(ctypes.Structure):
    """spnerf_rng (include/spnerf_amd.h): on-device Philox draws keyed by the device state
    {seed, step}, the call's first global ray id and a draw slot."""
    _fields_ = [("state", c_void_p), ("ray0", c_int64), ("slot", c_int32), ("reserved", c_int32)]


def rng_ref(r):
    """ctypes argument for an optional spnerf_rng (None = NULL)."""
    return None if r is None else ctypes.byref(r)


# name → (restype, argtypes); the exact export list of include/spnerf_amd.h
SIGNATURES = {
    "spnerf_last_error": (c_char_p, []),
    "spnerf_abi_version": (c_int32, []),
    "spnerf_param_count": (c_int32, [POINTER(ModelCfg)]),
    "spnerf_param_info": (c_int32, [POINTER(ModelCfg), c_int32, c_char_p, c_int32, POINTER(c_int64), POINTER(c_int64)]),
    "spnerf_packed_bytes": (c_int64, [POINTER(ModelCfg)]),
    "spnerf_pack_params": (c_int32, [POINTER(ModelCfg), POINTER(c_void_p), c_void_p, c_void_p]),
    "spnerf_mlp_workspace_bytes": (c_int64, [POINTER(ModelCfg), c_int64, c_int32, c_int32]),
    "spnerf_mlp_forward": (c_int32, [POINTER(ModelCfg), c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int32, c_void_p,
                                     c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p]),
    "spnerf_mlp_forward_window": (c_int32, [POINTER(ModelCfg), c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int64,
                                            c_int64, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_void_p,
                                            c_void_p, c_void_p]),
    "spnerf_mlp_backward": (c_int32, [POINTER(ModelCfg), c_void_p, c_void_p, c_int32, c_int64, c_int32, c_void_p, c_void_p,
                                      c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "spnerf_composite_forward": (c_int32, [c_int64, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_float, c_int32,
                                           c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                           POINTER(Rng), c_void_p]),
    "spnerf_composite_backward": (c_int32, [c_int64, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_float, c_int32,
                                            c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                            POINTER(Rng), c_void_p]),
    "spnerf_render_loss_workspace_bytes": (c_int64, [c_int64]),
    "spnerf_render_loss_forward": (c_int32, [c_int64, c_int32, c_int32, c_void_p, c_void_p, c_float, c_void_p, c_int32,
                                             c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_int32, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_int64,
                                             c_int32, c_void_p, c_void_p, c_void_p]),
    "spnerf_render_loss_backward": (c_int32, [c_int64, c_int32, c_int32, c_void_p, c_void_p, c_float, c_void_p, c_int32,
                                              c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_int32, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "spnerf_sample_stratified": (c_int32, [c_int64, c_int32, c_void_p, c_int32, c_void_p, c_void_p, POINTER(Rng), c_void_p]),
    "spnerf_sample_guided": (c_int32, [c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, POINTER(Rng), c_void_p]),
    "spnerf_sample_pdf": (c_int32, [c_int64, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_float, c_void_p,
                                    POINTER(Rng), c_void_p]),
    "spnerf_sample_3sigma": (c_int32, [c_int64, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "spnerf_sort_rows": (c_int32, [c_int64, c_int32, c_void_p, c_void_p, c_void_p]),
    "spnerf_merge_samples": (c_int32, [c_int64, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                       c_void_p]),
    "spnerf_merge_samples_backward": (c_int32, [c_int64, c_int32, c_int32, c_void_p, c_void_p, c_int32, c_void_p,
                                                c_void_p, c_void_p]),
    "spnerf_rpc_rays": (c_int32, [POINTER(c_double), c_double, c_double, c_double, c_int32, c_int32, c_int32, c_int32,
                                  c_void_p, c_int64, POINTER(c_float), c_float, POINTER(c_float), c_void_p, c_int32,
                                  c_void_p]),
    "spnerf_dsm_points": (c_int32, [c_void_p, c_int32, c_int64, c_void_p, POINTER(c_double), c_double, c_int32, c_int32,
                                    c_void_p, c_void_p, c_void_p]),
    "spnerf_dsm_rasterize": (c_int32, [c_void_p, c_int64, c_double, c_double, c_double, c_int32, c_int32, c_int32,
                                       c_double, c_void_p, c_void_p, c_void_p]),
    "spnerf_set_option": (c_int32, [c_char_p, c_int32]),
    "spnerf_get_option": (c_int32, [c_char_p, POINTER(c_int32)]),
    "spnerf_adam_step": (c_int32, [c_int32, POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p), POINTER(c_void_p),
                                   POINTER(c_int64), c_double, c_double, c_double, c_double, c_int32, c_void_p]),
    "spnerf_gather_rows": (c_int32, [c_void_p, c_int64, c_int32, POINTER(c_void_p), POINTER(c_int64), POINTER(c_int32),
                                     POINTER(c_void_p), c_void_p]),
    "spnerf_rng_begin": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "spnerf_prof_enable": (c_int32, [c_int32]),
    "spnerf_prof_reset": (c_int32, []),
    "spnerf_prof_read": (c_int32, [c_char_p, POINTER(c_int64), POINTER(c_double), POINTER(c_double), POINTER(c_double)]),
    "spnerf_prof_classes": (c_int32, [c_char_p, c_int32]),
    "spnerf_mlp_trunk_wgrad": (c_int32, [POINTER(ModelCfg), c_int32, POINTER(c_void_p), POINTER(c_int64),
                                         POINTER(c_int32), POINTER(c_int32), c_void_p, c_void_p]),
    "spnerf_grad_marks": (c_int32, [POINTER(ModelCfg), POINTER(c_int32), c_int32]),
    "spnerf_grad_marks_arm": (c_int32, [c_int32]),
    "spnerf_grad_mark_wait": (c_int32, [c_int32, c_void_p]),
    "spnerf_grad_mark_query": (c_int32, [c_int32, c_int32]),
}

_lib = None


class SpnerfError(RuntimeError):
    pass


def lib():
    """Load the HIP library (once).  Raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SpnerfError(f"{LIB_PATH} is missing: build it with `make -C sp-nerf_amd` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().spnerf_last_error().decode(errors="replace")
        raise SpnerfError(f"spnerf_amd {what}: error {rc}: {msg}")


def ptr(t) -> c_void_p:
    return c_void_p(0) if t is None else c_void_p(t.data_ptr())


def stream_of(t) -> c_void_p:
    import torch
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*tensors) -> None:
    """The product path runs only on the GPU; CPU tensors are an error, not a fallback."""
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise SpnerfError("spnerf_amd runs the render path on the MI355X (HIP) only; got a tensor on "
                              f"{t.device}. Move rays / models to the GPU.")


class OptionUnavailable(SpnerfError):
    """A kernel switch the loaded library does not have: the A/B switches of kernels measured
    slower than the defaults exist only in a -DSPN_ABLATIONS build."""


def has_option(name: str) -> bool:
    v = ctypes.c_int32()
    return lib().spnerf_get_option(name.encode(), ctypes.byref(v)) == 0


def set_option(name: str, value: int) -> None:
    """Kernel-selection switch (spnerf_set_option): "fused_trunk", "nt_f32_variant", ..."""
    if not has_option(name):
        raise OptionUnavailable(f"set_option: the library has no option {name!r} (ablation build only?)")
    check(lib().spnerf_set_option(name.encode(), int(value)), f"set_option({name})")


def get_option(name: str) -> int:
    if not has_option(name):
        raise OptionUnavailable(f"get_option: the library has no option {name!r} (ablation build only?)")
    v = ctypes.c_int32()
    check(lib().spnerf_get_option(name.encode(), ctypes.byref(v)), f"get_option({name})")
    return v.value


def prof_enable(on: bool = True) -> None:
    check(lib().spnerf_prof_enable(1 if on else 0), "prof_enable")


def prof_reset() -> None:
    check(lib().spnerf_prof_reset(), "prof_reset")


def prof_classes() -> list:
    buf = ctypes.create_string_buffer(8192)
    check(lib().spnerf_prof_classes(buf, len(buf)), "prof_classes")
    return [c for c in buf.value.decode().split(",") if c]


def grad_marks(cfg: ModelCfg, n_params: int):
    """(mark of each parameter, number of marks): spnerf_grad_marks"""
    arr = (c_int32 * n_params)()
    n = lib().spnerf_grad_marks(ctypes.byref(cfg), arr, n_params)
    if n < 0:
        check(n, "grad_marks")
    return list(arr), n


def grad_marks_arm(on: bool) -> None:
    check(lib().spnerf_grad_marks_arm(1 if on else 0), "grad_marks_arm")


def grad_mark_query(device: int, mark: int):
    """Device ``device``'s gradient mark ``mark`` (spnerf_grad_mark_query): True when its latest
    record has completed, False while pending, None when it was never recorded on that device."""
    r = lib().spnerf_grad_mark_query(int(device), int(mark))
    if r < 0:
        check(r, "grad_mark_query")
    return None if r == 2 else r == 1


def grad_mark_wait(mark: int, stream) -> None:
    """``stream`` (a torch.cuda.Stream) waits for the latest record of gradient mark ``mark``."""
    check(lib().spnerf_grad_mark_wait(int(mark), c_void_p(stream.cuda_stream)), "grad_mark_wait")


def prof_read(kernel_class: str) -> dict:
    n, ms, fl, by = c_int64(), c_double(), c_double(), c_double()
    check(lib().spnerf_prof_read(kernel_class.encode(), ctypes.byref(n), ctypes.byref(ms), ctypes.byref(fl),
                                 ctypes.byref(by)), "prof_read")
    return {"launches": n.value, "ms": ms.value, "flop": fl.value, "bytes": by.value}
