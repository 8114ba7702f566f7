"""HBM bytes of a kernel from rocprofv3 request-size counters (measurement helper,
used by bench.py and tools/calib_summary.py).

rocprofv3's FETCH_SIZE on gfx950 is
    (TCC_BUBBLE*128 + (TCC_EA0_RDREQ - TCC_BUBBLE - TCC_EA0_RDREQ_32B)*64 + TCC_EA0_RDREQ_32B*32) / 1024
(its --list-avail expression): a 128-byte request is tallied at 64 B unless
TCC_BUBBLE counts it, which on this part it does not -- hence the guide's
"FETCH_SIZE reports 1/2 of a streaming read".  The L2's memory-side request
counters split by size instead:
    read bytes  = 128 * TCC_EA0_RDREQ_128B + 64 * TCC_EA0_RDREQ_64B + 32 * TCC_EA0_RDREQ_32B
    write bytes = WRITE_SIZE (exact for 16-B stores per the guide; 64-B and 32-B requests)
calibrated per access shape on known byte counts in profiles/r02/calib/
(tools/calib.hip): streaming 16-B and 4-B loads, LDS-DMA, non-temporal
variants, random 16-B gathers.  Infinity-Cache hits are counted (they are
memory-side requests of the L2), so this is an upper bound on DRAM bytes.

One rocprofv3 pass per group below (the TCC block collects at most 4 counters
per pass; these groups use 2 each).
"""
import csv
import glob
import os
import signal
import subprocess

PASSES = [
    ("rdA", ["TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum"]),
    ("rdB", ["TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum"]),
    ("wr", ["WRITE_SIZE"]),
]


def per_dispatch(root, sub):
    """[(dispatch id, {counter: value})] of the kernels whose name contains sub, in order."""
    disp = {}
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as f:
            for row in csv.DictReader(f):
                if sub not in row["Kernel_Name"]:
                    continue
                d = disp.setdefault(int(row["Dispatch_Id"]), {})
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return [(k, disp[k]) for k in sorted(disp)]


def mean_last(rows, key, last):
    vals = [r[key] for _, r in rows if key in r]
    vals = vals[-last:] if last else vals
    return sum(vals) / len(vals) if vals else None, len(vals)


def dominant_kernel(root):
    """Name of the kernel with the largest total WRITE_SIZE in a pass directory
    (the round kernel: it writes the next state)."""
    tot = {}
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] == "WRITE_SIZE":
                    tot[row["Kernel_Name"]] = tot.get(row["Kernel_Name"], 0.0) + float(row["Counter_Value"])
    return max(tot, key=tot.get) if tot else None


def bytes_per_dispatch(dirs, sub, last=None):
    """dirs: {pass name: output dir}.  Mean bytes per dispatch over the last
    `last` dispatches of the matching kernel in every pass.  sub == "auto": the
    kernel that writes the most (dominant_kernel); its name is returned too."""
    if sub == "auto":
        sub = dominant_kernel(dirs["wr"])
        if sub is None:
            return None
    rows = {name: per_dispatch(d, sub) for name, d in dirs.items()}
    n32, c1 = mean_last(rows["rdA"], "TCC_EA0_RDREQ_32B_sum", last)
    nall, _ = mean_last(rows["rdA"], "TCC_EA0_RDREQ_sum", last)
    n64, c2 = mean_last(rows["rdB"], "TCC_EA0_RDREQ_64B_sum", last)
    n128, _ = mean_last(rows["rdB"], "TCC_EA0_RDREQ_128B_sum", last)
    wkib, c3 = mean_last(rows["wr"], "WRITE_SIZE", last)
    if None in (n32, nall, n64, n128, wkib):
        return None
    rd = 128.0 * n128 + 64.0 * n64 + 32.0 * n32
    return {
        "read_bytes": rd,
        "write_bytes": wkib * 1024.0,
        "total_bytes": rd + wkib * 1024.0,
        "rdreq": nall, "rdreq_32b": n32, "rdreq_64b": n64, "rdreq_128b": n128,
        # requests of no size class (should be ~0: the three classes cover RDREQ)
        "rdreq_unclassified": nall - n32 - n64 - n128,
        "fetch_size_equivalent_bytes": (64.0 * (nall - n32) + 32.0 * n32),
        "dispatches": min(c1, c2, c3),
        "kernel": sub,
    }


def run_passes(cmd, outroot, timeout=300, env=None):
    """Run `cmd` (argv list, the program itself -- no launcher) under one
    rocprofv3 --pmc pass per counter group.  Returns {pass: dir} or raises."""
    dirs = {}
    for name, counters in PASSES:
        d = os.path.join(outroot, name)
        argv = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", name, "--", *cmd]
        # own process group: a timeout kills the profiled program too
        p = subprocess.Popen(argv, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env,
                             start_new_session=True)
        try:
            _, err = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            p.communicate()
            raise RuntimeError(f"rocprofv3 pass {name} timed out after {timeout} s")
        if p.returncode:
            raise RuntimeError(f"rocprofv3 pass {name} failed ({p.returncode}): {err.decode(errors='replace')[-300:]}")
        dirs[name] = d
    return dirs
