#!/bin/bash
# L2 miss calibration: 3D (no random edges) vs Imp3D push-sum at P = 1e9, walk 2 vs 0; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "3D 2" "3D 0" "Imp3D 2"; do
  set -- $cfg
  n=$1_w$2
  GP_WALK=$2 timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/l2b_$n -o p -- python3 tools/perf_round.py 1000000000 $1 push-sum 10 > gpurun_out/l2b_$n.log 2>&1 || exit 1
  GP_WALK=$2 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/l2f_$n -o p -- python3 tools/perf_round.py 1000000000 $1 push-sum 10 > gpurun_out/l2f_$n.log 2>&1 || exit 1
  echo "== $n $(grep -o 'k_ps_tile<[A-Z0-9]*>: [0-9.]* ms' gpurun_out/l2b_$n.log) $(python3 tools/pmc_summary.py gpurun_out/l2b_$n 'k_ps_tile' --last=10 | tr -d '\n ') $(python3 tools/pmc_summary.py gpurun_out/l2f_$n 'k_ps_tile' --last=10 | tr -d '\n ')"
done
