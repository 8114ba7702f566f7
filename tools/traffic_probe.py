"""Round time + HBM bytes per node-round of the round kernel for variants
(experiment tool; run on the GPU box).

    python tools/traffic_probe.py <n> <topology> <algorithm> <kernel_substr> "ENV=V[,ENV=V]" ...

Every variant (environment overrides, experiments build via GP_EXP=1) runs
tools/perf_round.py once for the time, then under the three rocprofv3 passes
of tools/hbm_traffic.py; bytes are the mean over the last 8 round kernels.
"""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import hbm_traffic  # noqa: E402


def main():
    n, topo, alg, sub = sys.argv[1:5]
    variants = sys.argv[5:] or ["default"]
    rounds = 8
    cmd = [sys.executable, os.path.join(HERE, "perf_round.py"), n, topo, alg, str(rounds)]
    for v in variants:
        env = dict(os.environ, GP_NOEV="0")
        if v != "default":
            for kv in v.split(","):
                k, val = kv.split("=", 1)
                env[k] = val
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(v, "FAILED", out.stderr[-400:], flush=True)
            sys.exit(1)
        line = [x for x in out.stdout.splitlines() if "ms/round kernel" in x][-1]
        ms = float(line.split("ms/round kernel")[0].split()[-1])
        root = tempfile.mkdtemp(prefix="gp_probe_", dir=os.environ.get("TMPDIR", "/tmp"))
        dirs = hbm_traffic.run_passes(cmd, root, timeout=300, env=env)
        rec = hbm_traffic.bytes_per_dispatch(dirs, sub, last=rounds)
        P = float(n) if topo in ("line", "full") else round(float(n) ** (1 / 3)) ** 3
        print(f"{v:40s} {ms:8.3f} ms/round  read {rec['read_bytes'] / P:6.2f} B/node  write "
              f"{rec['write_bytes'] / P:6.2f} B/node  ({rec['total_bytes'] / (ms * 1e-3) / 1e9:.0f} GB/s; "
              f"128B {rec['rdreq_128b'] / P:.3f} 64B {rec['rdreq_64b'] / P:.3f} 32B {rec['rdreq_32b'] / P:.3f} req/node)",
              flush=True)


if __name__ == "__main__":
    main()
