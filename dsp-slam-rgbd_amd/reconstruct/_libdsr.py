"""ctypes binding of libdsr (include/dsr.h).

The library is the product path: there is no Python/PyTorch fallback.  If
``libdsr.so`` is missing or no gfx950 device is visible, every entry point
raises ``DsrError`` ("Use ctypes.CDLL, which releases the GIL
during a foreign call").
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
DEFAULT_LIB = os.path.join(_PKG, "csrc", "libdsr.so")

MAX_LAYERS = 16
CODE_LEN = 64
FAIL_REASONS = {0: "ok", 1: "sdf loss is NaN", 2: "fewer than 10 ray samples in the unit ball",
                3: "render loss is NaN (no render points)"}


class DsrError(RuntimeError):
    pass


FP = C.POINTER(C.c_float)
IP = C.POINTER(C.c_int)


class DecoderDesc(C.Structure):
    _fields_ = [("code_len", C.c_int), ("n_layers", C.c_int),
                ("out_dim", C.c_int * MAX_LAYERS), ("in_dim", C.c_int * MAX_LAYERS),
                ("latent_in", C.c_int), ("use_tanh", C.c_int), ("xyz_in_all", C.c_int),
                ("norm_mask", C.c_int)]


class OptimParams(C.Structure):
    _fields_ = [("k1", C.c_float), ("k2", C.c_float), ("k3", C.c_float), ("k4", C.c_float),
                ("b1", C.c_float), ("b2", C.c_float), ("lr", C.c_float), ("s_damp", C.c_float),
                ("num_iterations", C.c_int), ("code_len", C.c_int),
                ("num_depth_samples", C.c_int), ("cut_off", C.c_float),
                ("pose_only_iterations", C.c_int)]


class ObjectIn(C.Structure):
    _fields_ = [("t_cam_obj", C.c_float * 16), ("pts", FP), ("n_pts", C.c_int),
                ("rays", FP), ("n_rays", C.c_int), ("depth", FP), ("n_depth", C.c_int),
                ("code", FP), ("pose_is_obj_cam", C.c_int)]


class ObjectOut(C.Structure):
    _fields_ = [("t_cam_obj", C.c_float * 16), ("code", C.c_float * CODE_LEN),
                ("loss", C.c_float), ("is_good", C.c_int), ("fail_reason", C.c_int),
                ("iters_done", C.c_int), ("n_valid_last", C.c_int), ("k_last", C.c_int)]


class PoseIn(C.Structure):
    _fields_ = [("t_co_se3", C.c_float * 16), ("scale", C.c_float), ("pts", FP), ("n_pts", C.c_int),
                ("code", FP)]


class Trace(C.Structure):
    _fields_ = [("H", FP), ("b", FP), ("dx", FP), ("loss", FP), ("sdf_loss", FP),
                ("render_loss", FP), ("n_valid", IP), ("k", IP), ("t_obj_cam", FP), ("z", FP),
                ("n_decoded", IP), ("n_refined", IP)]


ABI_VERSION = 11         # include/dsr.h DSR_ABI_VERSION
BATCH_GRAPH = 1          # include/dsr.h DSR_BATCH_GRAPH
GATHER_HOST, GATHER_RCCL = 0, 1   # include/dsr.h DSR_GATHER_* (dsr_reconstruct_multi_ex)


class Stats(C.Structure):
    _fields_ = [("fwd_ms", C.c_double), ("jac_ms", C.c_double), ("total_ms", C.c_double),
                ("fwd_points", C.c_int64), ("jac_points", C.c_int64),
                ("fwd_launches", C.c_int), ("jac_launches", C.c_int), ("inball_points", C.c_int64),
                ("lite", C.c_int), ("refine_launches", C.c_int), ("refine_ms", C.c_double),
                ("refine_points", C.c_int64), ("lite_max_err", C.c_double),
                ("lite_min_margin", C.c_double), ("jac_surface_points", C.c_int64),
                ("jac_render_points", C.c_int64), ("keep_masks", C.c_int),
                ("lite_audit_violations", C.c_int), ("lite_redo_objects", C.c_int),
                ("surface_in_exact", C.c_int), ("audit_points", C.c_int64),
                ("lite_broken_blocks", C.c_int), ("test_hooks", C.c_int),
                ("lite_eligible", C.c_int), ("audit", C.c_int), ("audit_shell", C.c_float),
                ("audit_log2", C.c_int), ("lite_margin0", C.c_float), ("lite_floor", C.c_float),
                ("lite_safety", C.c_float), ("graph_captures", C.c_int), ("graph_replays", C.c_int),
                ("n_groups", C.c_int), ("graph_mode", C.c_int), ("fwd_variant", C.c_int),
                ("jac_variant", C.c_int), ("lite_variant", C.c_int), ("split_ring", C.c_int),
                ("prescan", C.c_int)]


class DecoderInfo(C.Structure):
    """dsr_decoder_info: the decoder's load-time lite qualification (include/dsr.h)."""
    _fields_ = [("code_len", C.c_int), ("lite_eligible", C.c_int), ("lite_probe_ratio", C.c_double),
                ("lite_probe_max_err", C.c_double), ("lite_probe_max_err_all", C.c_double),
                ("probe_points", C.c_int), ("probe_codes", C.c_int), ("probe_ms", C.c_double)]

#: dsr_batch_lite_diag record layout (csrc/dsr_dev.hpp: STD_*)
LITE_DIAG_FIELDS = ("broken_blocks", "recorded", "block", "wave", "counter", "target", "observed", "tile_iter",
                    "hw_id", "xcc_id", "polls", "real_ticks")
#: the counter index (``counter``) names the LiteStShared event counter that was waited on
LITE_DIAG_COUNTERS = ("ovf0", "ovf1", "cH0", "cH1", "cRlo", "cRhi", "cP", "cT0", "cT1", "cE", "broken")
LITE_DIAG_INTS = len(LITE_DIAG_FIELDS)


#: every function declared in include/dsr.h, with its ctypes signature
SIGNATURES = {
    "dsr_abi_version": (C.c_int, []),
    "dsr_device_count": (C.c_int, [IP]),
    "dsr_ctx_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "dsr_ctx_destroy": (C.c_int, [C.c_void_p]),
    "dsr_last_error": (C.c_char_p, [C.c_void_p]),
    "dsr_decoder_load": (C.c_int, [C.c_void_p, C.POINTER(DecoderDesc), FP, C.c_size_t,
                                   C.POINTER(C.c_void_p)]),
    "dsr_decoder_free": (C.c_int, [C.c_void_p, C.c_void_p]),
    "dsr_decoder_info_get": (C.c_int, [C.c_void_p, C.POINTER(DecoderInfo)]),
    "dsr_reconstruct_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(OptimParams), C.c_int,
                                        C.POINTER(ObjectIn), C.POINTER(ObjectOut),
                                        C.POINTER(Trace)]),
    "dsr_batch_create": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(OptimParams), C.c_int,
                                   C.POINTER(ObjectIn), C.POINTER(C.c_void_p)]),
    "dsr_batch_run": (C.c_int, [C.c_void_p]),
    "dsr_batch_graph": (C.c_int, [C.c_void_p]),
    "dsr_batch_sync": (C.c_int, [C.c_void_p]),
    "dsr_batch_query": (C.c_int, [C.c_void_p]),
    "dsr_batch_download": (C.c_int, [C.c_void_p, C.POINTER(ObjectOut)]),
    "dsr_batch_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "dsr_batch_lite_diag": (C.c_int, [C.c_void_p, IP, C.c_int]),
    "dsr_batch_destroy": (C.c_int, [C.c_void_p]),
    "dsr_batch_create_capacity": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(OptimParams), C.c_int, C.c_int,
                                            C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "dsr_batch_refill": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(ObjectIn)]),
    "dsr_sdf_eval": (C.c_int, [C.c_void_p, C.c_void_p, FP, FP, C.c_int, FP, FP]),
    "dsr_pose_only": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(OptimParams), FP, C.c_float,
                                FP, C.c_int, FP, FP]),
    "dsr_pose_only_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(OptimParams), C.c_int,
                                      C.POINTER(PoseIn), FP]),
    "dsr_reconstruct_multi": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int,
                                        C.POINTER(OptimParams), C.c_int, C.POINTER(ObjectIn),
                                        C.POINTER(ObjectOut)]),
    "dsr_reconstruct_multi_ex": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(C.c_void_p), C.c_int,
                                           C.POINTER(OptimParams), C.c_int, C.POINTER(ObjectIn),
                                           C.POINTER(ObjectOut), IP]),
    "dsr_gather_layout": (C.c_int, [C.c_int, C.POINTER(ObjectIn), C.c_int, C.c_int, IP, IP, IP]),
    "dsr_mesher_create": (C.c_int, [C.c_void_p, C.c_void_p, FP, C.c_int, C.POINTER(C.c_void_p)]),
    "dsr_mesher_run": (C.c_int, [C.c_void_p, FP, C.c_float, FP, C.c_int, IP, C.c_int, IP, IP]),
    "dsr_mesher_destroy": (C.c_int, [C.c_void_p]),
    "dsr_mc_volume": (C.c_int, [C.c_void_p, FP, C.c_int, C.c_float, FP, C.c_int, IP, C.c_int, IP, IP]),
}

_lib = None
_lock = threading.RLock()       # re-entrant: Context.get holds it while load_library takes it


def lib_path() -> str:
    return os.environ.get("DSR_LIB", DEFAULT_LIB)


def load_library(path: str | None = None):
    """Load libdsr.so (once) and attach the ctypes signatures."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or lib_path()
        if not os.path.isfile(p):
            raise DsrError(f"libdsr not built: {p} is missing (run `make -C dsp-slam-rgbd_amd/csrc` "
                           "or __graft_entry__.build()); there is no CPU fallback")
        lib = C.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dsr_abi_version() != ABI_VERSION:
            raise DsrError("libdsr ABI version mismatch")
        if path is None:
            _lib = lib
        return lib


def fptr(a: np.ndarray | None):
    if a is None:
        return None
    return a.ctypes.data_as(FP)


def iptr(a: np.ndarray | None):
    if a is None:
        return None
    return a.ctypes.data_as(IP)


class Context:
    """One libdsr context per HIP device (dsr_ctx_create)."""

    _cache: dict[int, "Context"] = {}

    def __init__(self, device: int = 0):
        self.lib = load_library()
        h = C.c_void_p()
        rc = self.lib.dsr_ctx_create(int(device), C.byref(h))
        if rc != 0:
            msgs = {-3: "no HIP device visible", -4: "device is not gfx950 (MI355X)",
                    -2: "bad device index", -1: "HIP runtime error"}
            raise DsrError(f"dsr_ctx_create(device={device}) failed: {msgs.get(rc, rc)}")
        self.handle = h
        self.device = device

    @classmethod
    def get(cls, device: int | None = None) -> "Context":
        if device is None:
            device = int(os.environ.get("DSR_DEVICE", os.environ.get("LOCAL_RANK", "0")))
        with _lock:            # one context per device even when threads race to create it
            if device not in cls._cache:
                cls._cache[device] = Context(device)
            return cls._cache[device]

    def check(self, rc: int, what: str):
        if rc != 0:
            msg = self.lib.dsr_last_error(self.handle)
            raise DsrError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def lite_diag(lib, handle):
    """The last run's staggered-lite-pass record (dsr_batch_lite_diag) as a dict."""
    rec = (C.c_int * LITE_DIAG_INTS)()
    rc = lib.dsr_batch_lite_diag(handle, rec, LITE_DIAG_INTS)
    if rc != 0:
        raise DsrError(f"dsr_batch_lite_diag failed ({rc})")
    v = list(rec)
    d = dict(zip(LITE_DIAG_FIELDS, v))
    if d["recorded"] and 0 <= d["counter"] < len(LITE_DIAG_COUNTERS):
        d["counter"] = LITE_DIAG_COUNTERS[d["counter"]]
    d["real_us"] = (d.pop("real_ticks") & 0xffffffff) / 100.0      # 100 MHz counter
    return d


def optim_params(cfg) -> OptimParams:
    """configs.optimizer block (optimizer.py:27-43) -> OptimParams."""
    jo = cfg["joint_optim"]
    po = cfg.get("pose_only_optim", {"num_iterations": 5}) if hasattr(cfg, "get") else \
        {"num_iterations": 5}
    return OptimParams(float(jo["k1"]), float(jo["k2"]), float(jo["k3"]), float(jo["k4"]),
                       float(jo["b1"]), float(jo["b2"]), float(jo["learning_rate"]),
                       float(jo["scale_damping"]), int(jo["num_iterations"]), int(cfg["code_len"]),
                       int(cfg["num_depth_samples"]), float(cfg["cut_off_threshold"]),
                       int(po["num_iterations"]))
