#!/bin/bash
# Kernel-trace stats of the headline config (per-kernel avg durations); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o kt -- python3 tools/perf_round.py ${N:-1000000000} ${TOPO:-Imp3D} ${ALG:-push-sum} 10 > gpurun_out/kt.log 2>&1 || exit 1
python3 - <<'PY'
import csv,glob
for f in glob.glob("gpurun_out/kt/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        print(f"{row['Name'][:70]:70s} calls {row['Calls']:>6s} avg {float(row['AverageNs'])/1e6:9.3f} ms  total {float(row['TotalDurationNs'])/1e6:9.1f} ms")
PY
