"""ctypes binding of the C oracle (oracle/libsrs_oracle.so).

Test infrastructure: used by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg only.  Builds the oracle with make if the .so is missing.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "libsrs_oracle.so")

TOPO = {"line": 0, "full": 1, "3D": 2, "Imp3D": 3}
ALG = {"gossip": 0, "push-sum": 1}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = C.CDLL(LIB_PATH)
        vp, i64, i32, u64, u32 = C.c_void_p, C.c_int64, C.c_int, C.c_uint64, C.c_uint32
        L.or_create.restype = vp
        L.or_create.argtypes = [i64, i32, i32, u64, i64, i32]
        L.or_destroy.argtypes = [vp]
        L.or_step.restype = i64
        L.or_step.argtypes = [vp, i64, C.POINTER(i64)]
        for f in ("or_rounds_done", "or_alerts_total", "or_population", "or_threshold",
                  "or_seed_node", "or_active_count", "or_activate_all"):
            getattr(L, f).restype = i64
            getattr(L, f).argtypes = [vp]
        L.or_neighbors.restype = i32
        L.or_neighbors.argtypes = [vp, i64, C.POINTER(i64)]
        L.or_read_state.restype = i32
        L.or_read_state.argtypes = [vp, i64, i64, vp, vp, vp, vp]
        L.or_philox4x32_10.argtypes = [C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)]
        L.or_uniform.restype = u32
        L.or_uniform.argtypes = [u64, u32, u64, u32, u32]
        L.or_icbrt_ceil.restype = i64
        L.or_icbrt_ceil.argtypes = [i64]
        L.or_pushsum_receivers.restype = i64
        L.or_pushsum_receivers.argtypes = [i32, i64, u64, u32, vp, vp, vp, vp, i64, vp, vp, vp, i32]
        _lib = L
    return _lib


def philox(ctr, key):
    L = lib()
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    L.or_philox4x32_10(c, k, o)
    return tuple(o)


def pushsum_receivers(topology, num_nodes, seed, rnd, s, w, flags, ids, threads=0):
    """Round `rnd` of push-sum for the receivers `ids`, from the full round-start
    state (s, w, flags of all P nodes): or_pushsum_receivers.  Returns
    (s_out, w_out, flags_out, converging) for the ids."""
    topology = "Imp3D" if topology.lower() == "imp3d" else topology
    s = np.ascontiguousarray(s, np.float64)
    w = np.ascontiguousarray(w, np.float64)
    flags = np.ascontiguousarray(flags, np.uint8)
    ids = np.ascontiguousarray(ids, np.int64)
    so = np.zeros(len(ids), np.float64)
    wo = np.zeros(len(ids), np.float64)
    fo = np.zeros(len(ids), np.uint8)
    a = lib().or_pushsum_receivers(TOPO[topology], num_nodes, seed, rnd, s.ctypes.data, w.ctypes.data,
                                   flags.ctypes.data, ids.ctypes.data, len(ids), so.ctypes.data, wo.ctypes.data,
                                   fo.ctypes.data, threads)
    if a < 0:
        raise ValueError("or_pushsum_receivers: bad input")
    return so, wo, fo, a


class Oracle:
    def __init__(self, num_nodes, topology, algorithm, seed=1, max_rounds=0, threads=0):
        topology = "Imp3D" if topology.lower() == "imp3d" else topology
        self.topology, self.algorithm = topology, algorithm
        self._h = lib().or_create(num_nodes, TOPO[topology], ALG[algorithm], seed, max_rounds, threads)
        if not self._h:
            raise ValueError("or_create failed")

    def close(self):
        if self._h:
            lib().or_destroy(self._h)
            self._h = None

    __del__ = close

    def step(self, nrounds):
        buf = (C.c_int64 * max(1, nrounds))()
        n = lib().or_step(self._h, nrounds, buf)
        return [buf[i] for i in range(n)]

    def run(self, max_rounds=10**7, chunk=4096):
        alerts = []
        while len(alerts) < max_rounds:
            a = self.step(min(chunk, max_rounds - len(alerts)))
            alerts += a
            if not a or self.alerts_total >= self.T:
                break
        return alerts

    @property
    def P(self):
        return lib().or_population(self._h)

    @property
    def T(self):
        return lib().or_threshold(self._h)

    @property
    def rounds(self):
        return lib().or_rounds_done(self._h)

    @property
    def alerts_total(self):
        return lib().or_alerts_total(self._h)

    @property
    def seed_node(self):
        return lib().or_seed_node(self._h)

    def active_count(self):
        return lib().or_active_count(self._h)

    def activate_all(self):
        """bench.py cpu_baseline timing only: every push-sum node active (skips the
        activation pre-roll; not an SRS v1 transition)."""
        return lib().or_activate_all(self._h)

    def neighbors(self, i):
        d = lib().or_neighbors(self._h, i, None)
        out = (C.c_int64 * max(1, d))()
        lib().or_neighbors(self._h, i, out)
        return [out[k] for k in range(d)]

    def state(self, first=0, count=None):
        count = self.P - first if count is None else count
        c = np.zeros(count, np.int32)
        s = np.zeros(count, np.float64)
        w = np.zeros(count, np.float64)
        f = np.zeros(count, np.uint8)
        rc = lib().or_read_state(self._h, first, count, c.ctypes.data, s.ctypes.data,
                                 w.ctypes.data, f.ctypes.data)
        assert rc == 0
        return {"c": c, "s": s, "w": w, "flags": f}
