"""bench.py -- headline benchmark (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Workload: push-sum on the imperfect-3D lattice with 1e9 nodes (g = 1000,
BASELINE config 4 = C5), which fits one MI355X (46 GB of state).  A "step" is one
synchronous round over all P nodes; the metric is node-updates/s = P * rounds /
wall time of the K timed rounds (max over ranks), with the state already
resident in HBM.  Before the timed region the simulation is advanced until
every node is active (steady state: every node sends a message each round),
then W warmup rounds; convergence is never reached inside the timed window.

One JSON line on stdout (rank 0).  `roofline` is measured live: HIP events on
the library's stream bracket every round kernel; `achieved` counts SURVEY.md
§8(d)'s algorithmic bytes per node-round (B_ps = 34 + 4 [Imp3D] + 32 a + 8 a_x:
71.1 B at C5's steady state, survey_bytes_per_node), and `design_*` the fewer
bytes this design must move (no message is staged
through HBM).  `traffic` is
measured in the same run: before the bench, the workload is re-run as a child
under three rocprofv3 --pmc passes and the round kernel's HBM bytes are read
from the L2's request-size counters (tools/hbm_traffic.py).  `cpu_baseline` times the SRS v1 C oracle on the host cores over a
bounded sample of the same workload (steady state, smaller lattice).

Multi-GPU (N > 1): one process per GPU, contiguous plane-aligned node slabs,
RCCL exchange inside libgossip_hip.  Under torch.distributed.run the ranks come
from the environment; `python bench.py --gpus N` without a launcher starts the N
rank processes itself (launch_ranks) before anything touches a GPU -- it never
measures fewer GPUs than asked for.  GP_BENCH_DEVICE=d pins every rank to device
d (the one-GPU rehearsal: RCCL over sockets, recorded as such in the JSON line).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "node-updates/sec (whole node) + achieved HBM GB/s %, imp3D push-sum 1e9 nodes"
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def survey_bytes_per_node(topology, algorithm, g):
    """SURVEY.md §8(d)'s algorithmic bytes per node-round in steady state (every node
    active, a = 1): push-sum B_ps = 34 + 4 [Imp3D] + 32 a + 8 a_x, a_x the fraction of
    messages on a random (Imp3D) or full-topology link.  Imp3D: a node with d lattice
    neighbours picks its random link with probability 1 / (d + 1) (Program.fs:125-128);
    along each axis a node has 2 neighbours, or 1 on the lattice's two end planes, so
    a_x = sum_k C(3, k) (2/g)^k ((g-2)/g)^(3-k) / (7 - k) (1/7 in the interior)."""
    if algorithm != "push-sum":
        return None
    imp = topology == "Imp3D"
    if topology == "full":
        ax = 1.0
    elif imp:
        from math import comb
        pe = 2.0 / g if g > 2 else 1.0
        ax = sum(comb(3, k) * pe ** k * (1.0 - pe) ** (3 - k) / (7 - k) for k in range(4))
    else:
        ax = 0.0
    return 34.0 + (4.0 if imp else 0.0) + 32.0 + 8.0 * ax


def preroll(sim, population, cap=2000):
    """Advance until every node is active (push-sum activation front has swept the lattice)."""
    rounds = 0
    while rounds < cap:
        info = sim.info()
        if info.active >= population:
            return rounds
        rounds += len(sim.step(8))
    raise RuntimeError("activation did not complete within %d rounds" % cap)


def measure_traffic(args):
    """HBM bytes per launch of the round kernel, measured in this run: the same
    workload re-run as a child under three rocprofv3 --pmc passes (request-size
    counters, tools/hbm_traffic.py; calibrated on known byte counts in
    profiles/r02/calib/).  Runs before this process touches the GPU.  Returns
    (record, None) or (None, reason)."""
    import shutil
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import hbm_traffic
    if shutil.which("rocprofv3") is None:
        return None, "rocprofv3 not found"
    steps = 6
    cmd = [sys.executable, os.path.abspath(__file__), "--no-cpu", "--no-traffic", "--steps", str(steps), "--warmup",
           "0", "--nodes", str(args.nodes), "--topology", args.topology, "--algorithm", args.algorithm,
           "--seed", str(args.seed)]
    root = tempfile.mkdtemp(prefix="gp_traffic_", dir=os.environ.get("TMPDIR", "/tmp"))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    try:
        dirs = hbm_traffic.run_passes(cmd, root, timeout=args.traffic_timeout, env=env)
        rec = hbm_traffic.bytes_per_dispatch(dirs, args.traffic_kernel, last=steps)
    except Exception as e:  # noqa: BLE001 -- reported in the JSON line, never fatal
        return None, f"{type(e).__name__}: {e}"
    finally:
        shutil.rmtree(root, ignore_errors=True)
    if rec is None:
        return None, f"no '{args.traffic_kernel}' dispatches in the counter output"
    return rec, None


def cpu_baseline(args):
    """SRS v1 C oracle on the host cores, steady-state rounds: at least cpu_rounds (3) and
    ~cpu_seconds.

    Default sample: the benchmarked workload itself (--nodes, P = 1e9 for C5).  The
    activation pre-roll at that size would take minutes of full-population passes, so
    every node is set active directly (Oracle.activate_all, timing only) -- a round then
    does what a steady-state round does, every node sends.  Small samples (--cpu-nodes,
    or a host without memory for ~70 B/node) run the real pre-roll instead."""
    from tests.oracle_ctypes import Oracle
    # every core this process may run on (OpenMP over all host cores), not the
    # box's OMP_NUM_THREADS (16 on the GPU boxes) -- unless --cpu-threads asks for a count
    sched = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp_env = os.environ.get("OMP_NUM_THREADS")
    threads = args.cpu_threads or sched
    n = args.cpu_nodes or args.nodes
    note = ""
    try:
        host_bytes = os.sysconf("SC_PAGE_SIZE") * os.sysconf("SC_PHYS_PAGES")
    except (ValueError, OSError):
        host_bytes = 0
    if n > 200**3 and host_bytes and 70 * n > host_bytes // 2:
        note = f" (host memory {host_bytes / 2**30:.0f} GiB too small for n={n}: sample reduced)"
        n = 200**3
    t0 = time.perf_counter()
    orc = Oracle(n, args.topology, args.algorithm, args.seed, threads=threads)
    P = orc.P
    direct = args.algorithm == "push-sum" and P > 2**24
    if direct:
        orc.activate_all()
        pre = "every node set active directly (no pre-roll)"
    else:
        while orc.active_count() < P:
            orc.step(5)
            if time.perf_counter() - t0 > 120:
                break
        pre = f"after a {orc.rounds}-round activation pre-roll"
    t_setup = time.perf_counter() - t0
    log(f"[bench] cpu baseline: oracle P={P} ready ({t_setup:.1f} s, {threads} threads)")
    rounds, t = 0, 0.0
    while (t < args.cpu_seconds or rounds < args.cpu_rounds) and rounds < 400:
        t1 = time.perf_counter()
        rounds += len(orc.step(1 if direct else 2))
        t += time.perf_counter() - t1
        if direct:
            log(f"[bench] cpu baseline: {rounds} round(s), {t:.1f} s")
    orc.close()
    return {
        "value": P * rounds / t,
        "unit": "node-updates/s",
        "cores": threads,
        "kind": "port",
        "sample": f"SRS v1 C oracle (oracle/srs_oracle.c, OpenMP), {args.topology} {args.algorithm} "
                  f"n={n} (P={P}), {rounds} steady-state round(s) {pre}, {t:.1f} s timed "
                  f"({t_setup:.1f} s setup untimed){note}; {threads} OpenMP threads "
                  f"({'--cpu-threads' if args.cpu_threads else 'all scheduler cores'}: {sched} available, "
                  f"OMP_NUM_THREADS={omp_env if omp_env is not None else 'unset'} in the environment)",
    }


def launch_ranks(args):
    """`--gpus N` outside torch.distributed.run: start N rank processes of this
    script (gossipprotocol_amd/launch.py; device = rank, or GP_BENCH_DEVICE for
    all), wait for all of them, and return the first failing exit code (the
    others are stopped) or rank 0's.  This process never touches a GPU; rank 0
    prints the JSON line."""
    from gossipprotocol_amd.launch import run_ranks
    return run_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus,
                     env_for_rank=lambda r: {"GP_BENCH_LAUNCHED": "1"}, log=log)


def akka_baseline():
    """north_star's "original Akka reference timed on the box's host cores": needs a
    .NET SDK (and the reference tree, which the GPU box does not have); recorded as
    unavailable with the host's core count and CPU model (tools/akka_timing.py runs
    it where dotnet exists)."""
    import shutil
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    rec = {"nproc": os.cpu_count(), "cpu_model": model,
           "sched_cores": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None}
    if shutil.which("dotnet") is None:
        rec["status"] = "unavailable (no dotnet)"
    else:
        rec["status"] = "unavailable (dotnet present; run tools/akka_timing.py where the reference tree is)"
    return rec


@contextlib.contextmanager
def stdout_to_stderr():
    """File descriptor 1 -> 2 for the block (messages libraries write to stdout themselves)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nodes", type=int, default=10**9)
    ap.add_argument("--topology", default="Imp3D")
    ap.add_argument("--algorithm", default="push-sum")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-nodes", type=int, default=0, help="CPU-baseline sample size (0: --nodes)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-rounds", type=int, default=3,
                    help="CPU-baseline rounds at least (a 10^9-node round takes ~16 s on 256 cores)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline OpenMP threads (0: every core in the scheduler affinity mask)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--converge", action="store_true", help="also run a fresh simulation to convergence")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 HBM-traffic passes")
    ap.add_argument("--traffic-kernel", default="auto",
                    help="round-kernel name substring in the counters (auto: the kernel that writes the most)")
    ap.add_argument("--traffic-timeout", type=float, default=240.0)
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: refusing to measure another GPU count")
    traffic, traffic_note = None, "not measured (multi-GPU run)" if world > 1 else "not measured (--no-traffic)"
    if world == 1 and not args.no_traffic:
        t_tr = time.perf_counter()
        traffic, traffic_note = measure_traffic(args)
        log(f"[bench] HBM traffic passes: {time.perf_counter() - t_tr:.1f} s, "
            f"{'ok' if traffic else traffic_note}")
    from gossipprotocol_amd import Simulation
    from gossipprotocol_amd import _lib as L

    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo: host-side barrier / max only; data path is RCCL in the library
        with stdout_to_stderr():  # gloo announces its connections on stdout: the JSON line stays alone there
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x):
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # GP_BENCH_DEVICE pins every rank to one device (multi-process rehearsal on a one-GPU box).
    # RCCL refuses two ranks on one device of one host, so each rank then claims a host id of
    # its own: the ranks talk over RCCL's socket transport on loopback instead of xGMI.
    device = int(os.environ.get("GP_BENCH_DEVICE", local_rank))
    rehearsal = world > 1 and "GP_BENCH_DEVICE" in os.environ
    if rehearsal:  # every rank on one device: only RCCL's socket transport can connect them
        os.environ.setdefault("NCCL_HOSTID", f"gp-rehearsal-{rank}")
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    transport = ("none (one GPU)" if world == 1 else
                 f"RCCL sockets on loopback: one-GPU rehearsal, all {world} ranks on device {device} "
                 "(not a multi-GPU number)" if rehearsal else "RCCL, one process per GPU (xGMI)")
    sim = Simulation(args.nodes, args.topology, args.algorithm, seed=args.seed, device=device,
                     kernel_timing=True, rank=rank, world=world, dist=dist)
    P = sim.population
    t_pre = time.perf_counter()
    pre = preroll(sim, P) if args.algorithm == "push-sum" else 0
    log(f"[bench] rank {rank}: P={P} activation pre-roll {pre} rounds ({time.perf_counter() - t_pre:.1f} s)")
    sim.step(args.warmup)
    sim.sync()
    sim.kernel_stats(reset=True)
    barrier()
    t0 = time.perf_counter()
    got = sim.step(args.steps)
    sim.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if len(got) != args.steps:
        raise RuntimeError(f"only {len(got)} of {args.steps} timed rounds ran (converged inside the window)")
    elapsed = max_over_ranks(elapsed)
    kms, launches, kname = sim.kernel_stats()
    design_bytes = sim.alg_bytes_per_node()
    g_edge = round(P ** (1.0 / 3.0)) if args.topology in ("3D", "Imp3D") else 0
    local_nodes = sim.local_population
    sim.close()

    value = P * args.steps / elapsed
    avg_ms = kms / max(1, launches)
    bytes_per_node = survey_bytes_per_node(args.topology, args.algorithm, g_edge) or design_bytes
    achieved = bytes_per_node * local_nodes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    design_achieved = design_bytes * local_nodes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "node-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"push-sum rounds, {args.topology} lattice, n={args.nodes} (P={P}), steady state "
                        f"(all nodes active), seed {args.seed}",
            "num_nodes": args.nodes, "population": P, "topology": args.topology, "algorithm": args.algorithm,
            "parallelism": f"slab{world}", "transport": transport,
            "launcher": ("bench.py --gpus (rank processes)" if os.environ.get("GP_BENCH_LAUNCHED") else
                         "torch.distributed.run" if world > 1 else "single process"),
            "activation_preroll_rounds": pre,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": kname,
            "achieved": achieved,
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "traffic": traffic["total_bytes"] if traffic else None,
            "alg_bytes_per_node_round": bytes_per_node,
            "alg_bytes_source": "SURVEY.md §8(d) B_ps (steady state)",
            "design_bytes_per_node_round": design_bytes,
            "design_achieved": design_achieved,
            "design_frac": design_achieved / HBM_PEAK_GBPS,
            "kernel_avg_ms": avg_ms,
        },
        "cpu_baseline": None,
    }
    if traffic:
        alg = bytes_per_node * local_nodes
        out["roofline"]["traffic_detail"] = {
            "method": "this run: rocprofv3 --pmc request-size counters (128/64/32-B TCC_EA0_RDREQ) + WRITE_SIZE, "
                      "3 passes over the same workload, last %d round kernels (tools/hbm_traffic.py)" % traffic["dispatches"],
            "read_bytes": traffic["read_bytes"], "write_bytes": traffic["write_bytes"],
            "traffic_over_algorithmic": traffic["total_bytes"] / alg,
            "traffic_over_design_bytes": traffic["total_bytes"] / (design_bytes * local_nodes),
            "traffic_gbps": traffic["total_bytes"] / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None,
            "fetch_size_equivalent_bytes": traffic["fetch_size_equivalent_bytes"],
        }
    else:
        out["roofline"]["traffic_detail"] = {"method": traffic_note}
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args)
    out["akka_baseline"] = akka_baseline()
    if rank == 0 and world == 1 and args.converge:
        with Simulation(args.nodes, args.topology, args.algorithm, seed=args.seed, device=device) as s2:
            res = s2.run()
            out["config"]["convergence"] = {"rounds": res.rounds, "converged": res.status == L.GP_STATUS_CONVERGED,
                                            "elapsed_ms": res.elapsed_ms}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
