#!/bin/bash
# Steady-state round time + rocprofv3 kernel stats of the other BASELINE configs
# (C2 3D push-sum 1e6, C3 Imp3D gossip 1e8, C4 full push-sum 1e8); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out/configs
for cfg in "1000000 3D push-sum 200" "100000000 Imp3D gossip 20" "100000000 full push-sum 10"; do
  set -- $cfg
  n=$3_$2_$1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/configs/$n -o kt -- python3 tools/perf_round.py $1 $2 $3 $4 > gpurun_out/configs/$n.log 2>&1 || { tail -20 gpurun_out/configs/$n.log; exit 1; }
  echo "== $n"; tail -3 gpurun_out/configs/$n.log
done
