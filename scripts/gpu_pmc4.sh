#!/bin/bash
# FETCH/WRITE/L2 hit passes for the round kernels under given env; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
name=${NAME:-cur}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc4_$name/p$i -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/pmc4_${name}_$i.log 2>&1 || exit 1
done
for k in k_ps_edges "k_ps_tile<3"; do echo "== $name $k"; python3 tools/pmc_summary.py gpurun_out/pmc4_$name "$k" --last=10; done
