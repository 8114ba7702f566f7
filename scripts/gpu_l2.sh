#!/bin/bash
# L2 hit/miss + time per walk/grid config of the headline round kernel; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-"2 8 16384" "0 8 16384" "2 8 1280" "2 4 16384" "2 16 2560"}; do
  set -- $cfg
  n=w$1x$2g$3
  GP_WALK=$1 GP_WX=$2 GP_GRID=$3 timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/l2_$n -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/l2_$n.log 2>&1 || exit 1
  echo "== $n $(grep -o 'k_ps_tile<IMP3D>: [0-9.]* ms' gpurun_out/l2_$n.log) $(python3 tools/pmc_summary.py gpurun_out/l2_$n 'k_ps_tile<3' --last=10 | tr -d '\n ')"
done
