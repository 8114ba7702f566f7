"""HBM-byte calibration table from tools/calib.hip (experiment tool).

    python tools/calib_summary.py <calib.log> <pass_root> [out.json]

calib.log is build/calib's stdout (one line per shape: algorithmic bytes read
and written, time); pass_root holds the rocprofv3 passes of
tools/hbm_traffic.PASSES over the same program (rdA / rdB / wr).  For every
shape: read bytes from the request-size counters (128 / 64 / 32-B requests)
and the FETCH_SIZE-equivalent (its gfx950 formula, 128-B requests at 64 B),
each divided by the shape's algorithmic bytes; WRITE_SIZE likewise.  The
distinct-line gathers give the memory-side bytes of one random 16-B read.
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from hbm_traffic import PASSES, per_dispatch  # noqa: E402

SHAPE_KERNEL = {  # shape (calib.log) -> kernel name in the PMC csv
    "rd16": "k_rd16(", "rd16_nt": "k_rd16_nt(", "rd4_nt": "k_rd4_nt(",
    "dma16": "k_dma16<0>", "dma16_nt": "k_dma16<2>",
    "gat16_line": "k_gat16<true>", "gatdma_nt_line": "k_gatdma_nt<true>",
    "gat16": "k_gat16<false>", "gatdma_nt": "k_gatdma_nt<false>",
    "st16_nt": "k_st16_nt(", "st4_nt": "k_st4_nt(",
}
SHAPE_KERNEL.update({"gat16_uc": "k_gat16_uc(", "sc16_uc": "k_sc16_uc(", "sc16": "k_sc16("})
for _a in (0, 1, 3, 16, 17, 19):
    SHAPE_KERNEL[f"gatdma_aux{_a}"] = f"k_gatdma_aux<{_a}>"


def largest(rows, key):
    """the dispatch with the largest value of key (the flush kernel is k_st16_nt too)"""
    vals = [r.get(key, 0.0) for _, r in rows]
    return max(vals) if vals else 0.0


def main():
    log, root = sys.argv[1:3]
    outp = sys.argv[3] if len(sys.argv) > 3 else None
    dirs = {name: os.path.join(root, name) for name, _ in PASSES}
    table = {}
    with open(log) as f:
        for line in f:
            p = line.split()
            if len(p) < 9 or p[0] not in SHAPE_KERNEL:
                continue
            shape, rd, wr, ms = p[0], float(p[2]), float(p[4]), float(p[6])
            sub = SHAPE_KERNEL[shape]
            a, b, w = (per_dispatch(dirs[n], sub) for n in ("rdA", "rdB", "wr"))
            u = per_dispatch(os.path.join(root, "rdU"), sub) if os.path.isdir(os.path.join(root, "rdU")) else []
            nall, n32 = largest(a, "TCC_EA0_RDREQ_sum"), largest(a, "TCC_EA0_RDREQ_32B_sum")
            n64, n128 = largest(b, "TCC_EA0_RDREQ_64B_sum"), largest(b, "TCC_EA0_RDREQ_128B_sum")
            wbytes = largest(w, "WRITE_SIZE") * 1024.0
            rbytes = 128.0 * n128 + 64.0 * n64 + 32.0 * n32
            fetch_eq = 64.0 * (nall - n32) + 32.0 * n32
            rec = {"alg_read_bytes": rd, "alg_write_bytes": wr, "ms": ms,
                   "rdreq": nall, "rdreq_32b": n32, "rdreq_64b": n64, "rdreq_128b": n128,
                   "read_bytes_by_size": rbytes, "fetch_size_bytes": fetch_eq, "write_size_bytes": wbytes}
            if rd:
                rec["read_factor_by_size"] = rbytes / rd
                rec["fetch_size_factor"] = fetch_eq / rd
            if wr:
                rec["write_factor"] = wbytes / wr
            q = per_dispatch(os.path.join(root, "wrq"), sub) if os.path.isdir(os.path.join(root, "wrq")) else []
            if q:
                rec["wrreq"] = largest(q, "TCC_EA0_WRREQ_sum")
                rec["wrreq_64b"] = largest(q, "TCC_EA0_WRREQ_64B_sum")
            if u:
                rec["rd_uncached_32b"] = largest(u, "TCC_EA0_RD_UNCACHED_32B_sum")
                rec["rdreq_dram"] = largest(u, "TCC_EA0_RDREQ_DRAM_sum")
            if shape.startswith("gat"):
                g = rd / 16.0
                rec["requests_per_gather"] = nall / g
                rec["read_bytes_per_gather"] = rbytes / g
            table[shape] = rec
    text = json.dumps(table, indent=1)
    print(text)
    if outp:
        with open(outp, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
