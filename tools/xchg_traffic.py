"""HBM bytes per dispatch of the multi-rank kernels at world W (experiment tool;
run on the GPU box).

    python tools/xchg_traffic.py <n> <topology> <algorithm> <W> <rounds> [kernel_substr ...]

Runs `tools/mgpu_model.py run` (W in-process virtual ranks on one device: the
slab plan, kernels and exchange of W processes) under the three rocprofv3 --pmc
passes of tools/hbm_traffic.py and prints, per kernel, the mean read / write
bytes of its last W * rounds dispatches (one per slab and round), per node of a
slab.  Default kernels: the pack / unpack of the random-edge exchange and the
round kernels.
"""
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import hbm_traffic  # noqa: E402


def main():
    n, topo, alg, W, rounds = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    kernels = sys.argv[6:] or ["k_pack", "k_unpack", "k_ps_tile", "k_gossip_col"]
    cmd = [sys.executable, os.path.join(HERE, "mgpu_model.py"), "run", n, topo, alg, str(W), str(rounds)]
    root = tempfile.mkdtemp(prefix="gp_xt_", dir=os.environ.get("TMPDIR", "/tmp"))
    dirs = hbm_traffic.run_passes(cmd, root, timeout=900)
    P = float(n) if topo in ("line", "full") else round(float(n) ** (1 / 3)) ** 3
    per_slab = P / W
    out = {"workload": f"{alg} {topo} n={n} W={W}", "rounds": rounds, "nodes_per_slab": per_slab, "kernels": {}}
    for k in kernels:
        rec = hbm_traffic.bytes_per_dispatch(dirs, k, last=W * rounds)
        if rec is None:
            continue
        out["kernels"][k] = {"read_B_per_node": rec["read_bytes"] / per_slab, "write_B_per_node": rec["write_bytes"] / per_slab,
                             "read_bytes": rec["read_bytes"], "write_bytes": rec["write_bytes"],
                             "dispatches": rec["dispatches"], "kernel": rec["kernel"]}
        print(f"{k:14s} read {rec['read_bytes'] / per_slab:7.2f} B/node  write {rec['write_bytes'] / per_slab:7.2f} B/node"
              f"  ({rec['dispatches']} dispatches)", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
