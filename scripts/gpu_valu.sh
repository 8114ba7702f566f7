#!/bin/bash
# Dynamic VALU instruction count + VALU-busy cycles per ablation variant (one SQ pass each); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/valu_$v -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/valu_$v.log 2>&1 || exit 1
  echo "== $v $(grep -o 'k_ps_tile<IMP3D>: [0-9.]* ms' gpurun_out/valu_$v.log)"
  python3 tools/pmc_summary.py gpurun_out/valu_$v "k_ps_tile<3" --last=10 | tr -d '\n '; echo
done
