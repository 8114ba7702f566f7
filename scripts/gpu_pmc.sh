#!/bin/bash
# PMC passes (one counter group per run, as the pool requires) over the steady-state
# round kernel: tools/perf_round.py (default 1e9 Imp3D push-sum, 10 timed rounds).
# OUT names the output directory under gpurun_out/ (default pmc); extra env (GP_KERNEL, ...) passes through.
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:-pmc}
mkdir -p $OUT
[ -f gpurun_out/counters_list.txt ] || rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
N=${N:-1000000000}; TOPO=${TOPO:-Imp3D}; ALG=${ALG:-push-sum}
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES" \
  "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ${EXTRA_GROUPS} ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc ${grp//+/ } --output-format csv -d $OUT/p$i -o p -- python3 tools/perf_round.py $N $TOPO $ALG 10 > $OUT/p$i.log 2>&1 || exit 1
done
