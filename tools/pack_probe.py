"""HBM bytes and SQ cycle counters of one kernel of the several-rank round, on
virtual ranks (experiment tool; run on the GPU box).

    python tools/pack_probe.py <n> <topology> <algorithm> <W> <kernel_substr> ...

Runs tools/mgpu_model.py's virtual-rank round under the three rocprofv3 --pmc
passes of tools/hbm_traffic.py and the two SQ passes of tools/pmc_probe.py; prints
per-dispatch means over the last 2 W dispatches of each kernel (the pack: every
slab and region of the last round; a per-slab kernel: the last two rounds).
"""
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import hbm_traffic  # noqa: E402
import pmc_probe  # noqa: E402


def main():
    n, topo, alg, W = sys.argv[1:5]
    subs = sys.argv[5:]
    last = 2 * int(W)
    cmd = [sys.executable, os.path.join(HERE, "mgpu_model.py"), "run", n, topo, alg, W, "6"]
    env = dict(os.environ, GP_EXP="1")
    root = tempfile.mkdtemp(prefix="gp_pack_", dir=os.environ.get("TMPDIR", "/tmp"))
    hdirs = hbm_traffic.run_passes(cmd, os.path.join(root, "hbm"), env=env)
    sdirs = pmc_probe.run(cmd, env, os.path.join(root, "sq"))
    for sub in subs:
        rec = hbm_traffic.bytes_per_dispatch(hdirs, sub, last=last)
        print("%s: read %.4g B write %.4g B per dispatch (128B req %.4g, 64B %.4g, 32B %.4g)" % (
            sub, rec["read_bytes"], rec["write_bytes"], rec["rdreq_128b"], rec["rdreq_64b"], rec["rdreq_32b"]),
            flush=True)
        for name, counters in pmc_probe.PASSES:
            rows = hbm_traffic.per_dispatch(sdirs[name], sub)
            print("  " + " ".join("%s %.4g" % (c[3:], hbm_traffic.mean_last(rows, c, last)[0] or 0.0)
                                  for c in counters), flush=True)

if __name__ == "__main__":
    main()
