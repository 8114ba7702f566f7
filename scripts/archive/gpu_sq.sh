#!/bin/bash
# SQ counters (issue vs wave cycles) of the push-sum tile kernel at P = 1e9, for the
# product library and experiments variants.   VARIANTS="lgm4 ..." (build/ablate/lib_<v>.so)
export TMPDIR=/tmp
O=${O:-gpurun_out/sq}
mkdir -p $O
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES"
C2="SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_COUNT"
for v in product $VARIANTS; do
  if [ $v = product ]; then L=""; else L="build/ablate/lib_$v.so"; fi
  for pass in 1 2; do
    if [ $pass = 1 ]; then CC=$C; else CC=$C2; fi
    GOSSIP_HIP_LIB_EXPERIMENT=$L GP_EXP=${L:+1} timeout -s KILL 200 rocprofv3 --pmc $CC --output-format csv -d $O/$v/p$pass -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > $O/$v.p$pass.log 2>&1 || { tail -20 $O/$v.p$pass.log; exit 1; }
  done
  echo "== $v"; python3 tools/pmc_summary.py $O/$v "k_ps_tile<3" --last=10
done
