"""Steady-state per-kernel durations from a rocprofv3 kernel trace (experiment tool).

    python tools/kt_steady.py <trace dir> [substr] [--last N]

Takes the last N dispatches of every kernel whose name contains substr (default
all), ignoring dispatches shorter than 5 % of the kernel's median (rounds after
convergence exit at once).
"""
import csv
import glob
import statistics
import sys


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 10
    rows = []
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    by = {}
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        if sub in r["Kernel_Name"]:
            by.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, v in by.items():
        med = statistics.median(v)
        v = [x for x in v if x > 0.05 * med][-last:]
        print("%-60s n %3d mean %8.4f ms  min %8.4f  max %8.4f" % (k[:60], len(v), statistics.mean(v), min(v), max(v)))


if __name__ == "__main__":
    main()
