#!/bin/bash
# Two PMC passes (SQ timing, SQ instruction mix) per kernel variant over the headline
# steady state; summary of the last 10 dispatches per kernel; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARS:-1 0}; do
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    GP_EDGES=$v timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc2_e$v/p$i -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/pmc2_e$v_$i.log 2>&1 || exit 1
  done
  for k in k_ps_edges "k_ps_tile<3"; do
    echo "== GP_EDGES=$v $k"; python3 tools/pmc_summary.py gpurun_out/pmc2_e$v "$k" --last=10
  done
done
