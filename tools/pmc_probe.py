"""Per-node instruction / cycle counters of the round kernel for variants
(experiment tool; run on the GPU box).

    python tools/pmc_probe.py <n> <topology> <algorithm> <kernel_substr> "ENV=V[,ENV=V]" ...

Every variant runs tools/perf_round.py under the counter passes below (one
rocprofv3 --pmc run each, at most 8 SQ counters per pass); values are the mean
over the last 8 round kernels, divided by the wave-node count P / 64 where they
count wave-instructions (so "VALU 420" = 420 VALU instructions per node and
lane), or printed raw for cycle counters.
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import hbm_traffic  # noqa: E402

PASSES = [
    ("i1", ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
            "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_FMA_F64"]),
    ("c1", ["SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
            "SQ_WAIT_INST_ANY", "SQ_INST_CYCLES_VMEM_RD", "SQ_INSTS_VALU_INT32"]),
]


def run(cmd, env, root):
    dirs = {}
    for name, counters in PASSES:
        d = os.path.join(root, name)
        argv = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", name, "--", *cmd]
        subprocess.run(argv, env=env, check=True, timeout=300, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                       start_new_session=True)
        dirs[name] = d
    return dirs


def main():
    n, topo, alg, sub = sys.argv[1:5]
    variants = sys.argv[5:] or ["default"]
    rounds = 8
    cmd = [sys.executable, os.path.join(HERE, "perf_round.py"), n, topo, alg, str(rounds)]
    P = float(n) if topo in ("line", "full") else round(float(n) ** (1 / 3)) ** 3
    wn = P / 64.0
    for v in variants:
        env = dict(os.environ, GP_NOEV="0")
        if v != "default":
            for kv in v.split(","):
                k, val = kv.split("=", 1)
                env[k] = val
        root = tempfile.mkdtemp(prefix="gp_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        dirs = run(cmd, env, root)
        vals = {}
        for name, counters in PASSES:
            rows = hbm_traffic.per_dispatch(dirs[name], sub)
            for c in counters:
                vals[c], _ = hbm_traffic.mean_last(rows, c, rounds)
        inst = {c[9:]: vals[c] / wn for c in PASSES[0][1] if vals.get(c) is not None}
        print(f"{v:40s} per node: " + " ".join(f"{k} {x:.1f}" for k, x in inst.items()), flush=True)
        print(f"{'':40s} waves {vals['SQ_WAVES']:.0f} busy {vals['SQ_BUSY_CYCLES']:.3e} wave_cyc {vals['SQ_WAVE_CYCLES']:.3e} "
              f"valu_act {vals['SQ_ACTIVE_INST_VALU']:.3e} any_act {vals['SQ_ACTIVE_INST_ANY']:.3e} "
              f"wait_inst {vals['SQ_WAIT_INST_ANY']:.3e} vmem_rd_cyc {vals['SQ_INST_CYCLES_VMEM_RD']:.3e} "
              f"int32/node {vals['SQ_INSTS_VALU_INT32'] / wn:.1f}", flush=True)


if __name__ == "__main__":
    main()
