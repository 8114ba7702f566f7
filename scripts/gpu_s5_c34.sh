#!/bin/bash
# C3 (gossip Imp3D 1e8: random-edge delivery pass + column march) and C4 (full push-sum
# 1e8: LDS binning) steady-state rounds with kernel traces + C3 HBM bytes, then the
# full GPU suite; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out/c34
for cfg in "100000000 Imp3D gossip 20" "100000000 full push-sum 10"; do
  set -- $cfg
  n=$3_$2_$1
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c34/$n -o kt -- python3 tools/perf_round.py $1 $2 $3 $4 > gpurun_out/c34/$n.log 2>&1 || { tail -20 gpurun_out/c34/$n.log; exit 1; }
  echo "== $n"; grep -v "^E2\|^W2" gpurun_out/c34/$n.log | tail -2
done
N=100000000 TOPO=Imp3D ALG=gossip KSUB=k_gossip VARIANTS="default" bash scripts/gpu_probe.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
exit $rc
