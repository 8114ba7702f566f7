"""Host-side mirror of the reference's entry point over the C-ABI.

The reference's only interface to the hot path is ``main`` in
/root/reference/Project2/Program.fs (Program.fs:31-283): parse
``num_nodes topology algorithm`` (Program.fs:32-34), build actors and topology
(Program.fs:169-261), start the seed (Program.fs:193-205), wait for the
scheduler's ``nodes`` alerts (Program.fs:41-61).  :class:`Simulation` exposes
the same steps -- create / run -- plus round stepping and state readback for
tests.  Every call goes to libgossip_hip.so; there is no CPU path here.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _lib as L

TOPOLOGIES = ("line", "full", "3D", "Imp3D")
ALGORITHMS = ("gossip", "push-sum")


def parse_topology(name: str) -> int:
    """Case-sensitive like Program.fs:180,209,238; 'imp3D' accepted as an alias."""
    return L.check(L.lib().gp_parse_topology(name.encode()))


def parse_algorithm(name: str) -> int:
    return L.check(L.lib().gp_parse_algorithm(name.encode()))


def resolve(num_nodes: int, topology: str):
    """(P, T, g) -- population, alert threshold, grid edge (Program.fs:170-171,53,239-240)."""
    P, T, g = C.c_int64(), C.c_int64(), C.c_int64()
    L.check(L.lib().gp_resolve(num_nodes, parse_topology(topology), C.byref(P), C.byref(T), C.byref(g)))
    return P.value, T.value, g.value


class Simulation:
    """One simulated network on one MI355X (handle over gp_sim)."""

    def __init__(self, num_nodes: int, topology: str, algorithm: str, seed: int = 1,
                 max_rounds: int = 0, device: int = 0, kernel_timing: bool = False,
                 rank: int = 0, world: int = 1, dist=None, virtual_ranks: int = 1, experimental: bool = False,
                 rendezvous: str | None = None, rendezvous_timeout_ms: int = 600000):
        """world > 1: this process is rank `rank` of a one-process-per-GPU run
        (RCCL; rank 0's RCCL id is shared once, through `dist` -- a
        torch.distributed group -- or through the file `rendezvous`
        (gp_rendezvous_id; gossipprotocol_amd.launch sets GOSSIP_RDV)).  virtual_ranks > 1: that many slabs in this process on `device`,
        exchanging through device copies (the multi-GPU path on one GPU).
        experimental: use the experiments build (kernel variants selected by
        GP_* environment variables; tests and tools only)."""
        self._L = L.lib(experimental)
        cfg = L.GpConfig()
        cfg.num_nodes = num_nodes
        cfg.topology = parse_topology(topology)
        cfg.algorithm = parse_algorithm(algorithm)
        cfg.seed = seed
        cfg.num_gpus = max(1, virtual_ranks)
        cfg.device = device
        cfg.max_rounds = max_rounds
        cfg.flags = (L.GP_FLAG_KERNEL_TIMING if kernel_timing else 0) | \
            (L.GP_FLAG_VIRTUAL_RANKS if virtual_ranks > 1 else 0)
        self.topology, self.algorithm = topology, algorithm
        h = C.c_void_p()
        if world > 1 or (world == 1 and dist is not None and experimental and os.environ.get("GP_FORCE_RCCL") == "1"):
            # one process per GPU: rank 0 makes the RCCL id, the caller's process
            # group (gloo is enough) broadcasts it, every rank joins its slab
            uid = C.create_string_buffer(128)
            if dist is None and rendezvous:
                self._chk(self._L.gp_rendezvous_id(rank, rendezvous.encode(), rendezvous_timeout_ms, uid))
            elif dist is None:
                raise ValueError("world > 1 needs a torch.distributed group or a rendezvous path to share the RCCL id")
            else:
                if rank == 0:
                    self._chk(self._L.gp_get_unique_id(uid))
                box = [uid.raw if rank == 0 else None]
                dist.broadcast_object_list(box, src=0)
                uid = C.create_string_buffer(box[0], 128)
            from .launch import stdout_to_stderr
            with stdout_to_stderr():  # (RCCL's version line)
                rc = self._L.gp_create_rank(C.byref(cfg), rank, world, uid, C.byref(h))
            self._chk(rc)
        else:
            self._chk(self._L.gp_create(C.byref(cfg), C.byref(h)))
        self._h = h

    def _chk(self, rc):
        return L.check(rc, self._L)

    # -- lifecycle -------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._L.gp_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()

    # -- the hot path ----------------------------------------------------
    def step(self, nrounds: int):
        """Run up to nrounds synchronous rounds; returns the per-round alert counts."""
        buf = (C.c_int64 * max(1, nrounds))()
        n = self._chk(self._L.gp_step(self._h, nrounds, buf))
        return [buf[i] for i in range(n)]

    def run(self) -> L.GpResult:
        """Run to convergence (or max_rounds): the reference's whole propagation."""
        res = L.GpResult()
        self._chk(self._L.gp_run(self._h, C.byref(res)))
        return res

    def sync(self):
        self._chk(self._L.gp_sync(self._h))

    # -- inspection ------------------------------------------------------
    def info(self) -> L.GpInfo:
        out = L.GpInfo()
        self._chk(self._L.gp_get_info(self._h, C.byref(out)))
        return out

    @property
    def population(self):
        return self.info().population

    @property
    def local_population(self):
        """Nodes owned by this handle (its slab; all P for a single GPU)."""
        return self.info().slab_count

    @property
    def threshold(self):
        return self.info().threshold

    @property
    def seed_node(self):
        return self.info().seed_node

    @property
    def rounds(self):
        return self.info().rounds

    @property
    def alerts_total(self):
        return self.info().alerts_total

    def neighbors(self, node: int):
        deg = self._chk(self._L.gp_neighbors(self._h, node, None, 0))
        out = (C.c_int64 * max(1, deg))()
        self._chk(self._L.gp_neighbors(self._h, node, out, deg))
        return [out[k] for k in range(deg)]

    def state(self, first: int = 0, count: int | None = None):
        count = self.population - first if count is None else count
        c = np.zeros(count, np.int32)
        s = np.zeros(count, np.float64)
        w = np.zeros(count, np.float64)
        f = np.zeros(count, np.uint8)
        self._chk(self._L.gp_read_state(self._h, first, count, c.ctypes.data, s.ctypes.data,
                                      w.ctypes.data, f.ctypes.data))
        return {"c": c, "s": s, "w": w, "flags": f}

    def kernel_stats(self, reset: bool = False):
        ms, n = C.c_double(), C.c_int64()
        name = C.create_string_buffer(128)
        self._chk(self._L.gp_kernel_stats(self._h, C.byref(ms), C.byref(n), name, 128, int(reset)))
        return ms.value, n.value, name.value.decode()

    def alg_bytes_per_node(self) -> float:
        return self._L.gp_alg_bytes_per_node(self._h)


def run(num_nodes: int, topology: str, algorithm: str, seed: int = 1, max_rounds: int = 0, device: int = 0):
    """`dotnet run num_nodes topology algorithm` as a function: returns the gp_result."""
    with Simulation(num_nodes, topology, algorithm, seed=seed, max_rounds=max_rounds, device=device) as sim:
        return sim.run()
