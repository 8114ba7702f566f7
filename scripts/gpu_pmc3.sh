#!/bin/bash
# SQ timing + instruction-mix passes over: edge-split round (product), single-kernel round,
# and the no_ephilox ablation; summaries of the last 10 dispatches; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name env...
  name=$1; shift
  i=0
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"; do
    i=$((i+1))
    env "$@" timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc3_$name/p$i -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/pmc3_${name}_$i.log 2>&1 || exit 1
  done
  echo "== $name"; python3 tools/pmc_summary.py gpurun_out/pmc3_$name "k_ps_tile<3" --last=10
}
run edges GP_EDGES=1
run single GP_EDGES=0
run noeph GP_EDGES=0 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_no_ephilox.so
