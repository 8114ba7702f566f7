"""ctypes binding of libgossip_hip.so (C-ABI: include/gossip_hip.h).

The product path: there is no CPU fallback.  If the in-tree HIP library is
missing, loading raises -- build it with ``python -c "import __graft_entry__ as g; g.build()"``.
"""
from __future__ import annotations

import ctypes as C
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libgossip_hip.so")
# The experiments build (-DGP_EXPERIMENTS: kernel variants and GP_* environment
# overrides) -- loaded only by the kernel-variant tests and tools/, never by default.
EXP_LIB_PATH = os.path.join(PKG_DIR, "libgossip_hip_exp.so")
# tools/ablate.py may point the experiments slot at an ablation build
EXP_LIB_PATH = os.environ.get("GOSSIP_HIP_LIB_EXPERIMENT", EXP_LIB_PATH)

GP_LINE, GP_FULL, GP_3D, GP_IMP3D = 0, 1, 2, 3
GP_GOSSIP, GP_PUSHSUM = 0, 1
GP_STATUS_CONVERGED, GP_STATUS_MAX_ROUNDS = 0, 1
GP_FLAG_KERNEL_TIMING = 1
GP_FLAG_VIRTUAL_RANKS = 2
ERRORS = {-1: "GP_EINVAL", -2: "GP_ENOMEM", -3: "GP_EHIP", -4: "GP_ENCCL", -5: "GP_ESTATE", -6: "GP_ENODEV"}


class GpConfig(C.Structure):
    _fields_ = [("num_nodes", C.c_int64), ("topology", C.c_int32), ("algorithm", C.c_int32),
                ("seed", C.c_uint64), ("num_gpus", C.c_int32), ("device", C.c_int32),
                ("max_rounds", C.c_int64), ("flags", C.c_int32), ("reserved", C.c_int32)]


class GpResult(C.Structure):
    _fields_ = [("rounds", C.c_int64), ("converged", C.c_int64), ("population", C.c_int64),
                ("threshold", C.c_int64), ("elapsed_ms", C.c_double), ("node_updates_per_s", C.c_double),
                ("hbm_bytes_alg", C.c_double), ("status", C.c_int32), ("reserved", C.c_int32)]


class GpInfo(C.Structure):
    _fields_ = [("population", C.c_int64), ("threshold", C.c_int64), ("grid", C.c_int64),
                ("seed_node", C.c_int64), ("rounds", C.c_int64), ("alerts_total", C.c_int64),
                ("active", C.c_int64), ("topology", C.c_int32), ("algorithm", C.c_int32),
                ("device", C.c_int32), ("num_gpus", C.c_int32), ("slab_first", C.c_int64),
                ("slab_count", C.c_int64)]


# (name, restype, argtypes) for every symbol include/gossip_hip.h declares
_vp, _i64, _i32 = C.c_void_p, C.c_int64, C.c_int32
SIGNATURES = [
    ("gp_version", _i32, []),
    ("gp_last_error", C.c_char_p, []),
    ("gp_parse_topology", _i32, [C.c_char_p]),
    ("gp_parse_algorithm", _i32, [C.c_char_p]),
    ("gp_resolve", _i32, [_i64, _i32, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64)]),
    ("gp_create", _i32, [C.POINTER(GpConfig), C.POINTER(_vp)]),
    ("gp_get_unique_id", _i32, [C.c_char_p]),
    ("gp_rendezvous_id", _i32, [_i32, C.c_char_p, _i32, C.c_char_p]),
    ("gp_create_rank", _i32, [C.POINTER(GpConfig), _i32, _i32, C.c_char_p, C.POINTER(_vp)]),
    ("gp_run", _i32, [_vp, C.POINTER(GpResult)]),
    ("gp_step", _i64, [_vp, _i64, C.POINTER(_i64)]),
    ("gp_read_state", _i32, [_vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    ("gp_neighbors", _i32, [_vp, _i64, C.POINTER(_i64), _i64]),
    ("gp_get_info", _i32, [_vp, C.POINTER(GpInfo)]),
    ("gp_sync", _i32, [_vp]),
    ("gp_kernel_stats", _i32, [_vp, C.POINTER(C.c_double), C.POINTER(_i64), C.c_char_p, _i32, _i32]),
    ("gp_alg_bytes_per_node", C.c_double, [_vp]),
    ("gp_destroy", None, [_vp]),
]

_libs = {}


class GossipError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib(experimental: bool = False):
    """Load the in-tree HIP library (raises if it has not been built).
    experimental=True loads the experiments build instead (tests / tools only)."""
    path = EXP_LIB_PATH if experimental else LIB_PATH
    L = _libs.get(path)
    if L is None:
        if not os.path.exists(path):
            raise ImportError(f"{path} not built: run __graft_entry__.build() (no CPU fallback exists)")
        L = C.CDLL(path)
        for name, res, args in SIGNATURES:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _libs[path] = L
    return L


def check(rc, L=None):
    if rc < 0:
        raise GossipError(rc, (L or lib()).gp_last_error().decode(errors="replace"))
    return rc
