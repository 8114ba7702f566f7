#!/bin/bash
# Bottleneck counters of the push-sum tile kernel (1e9 Imp3D, steady state), one
# counter group per rocprofv3 pass; summary per pass over the last 10 dispatches.
export TMPDIR=/tmp
mkdir -p gpurun_out
K=${KERNEL:-k_ps_tile<3}
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
  "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
  "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_BUSY_sum GRBM_GUI_ACTIVE" \
  "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmck2/p$i -o p -- python3 tools/perf_round.py ${N:-1000000000} ${TOPO:-Imp3D} ${ALG:-push-sum} 10 > gpurun_out/pmck2_$i.log 2>&1 || { tail -5 gpurun_out/pmck2_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmck2 "$K" --last=10
