#!/bin/bash
# Alternating same-box timing of experiments-build libraries (VARIANTS: build/ablate/lib_<v>.so),
# REPS rounds, then SQ instruction counters of each (one pass).
export TMPDIR=/tmp
O=${O:-gpurun_out/ab2}
CFG=${CFG:-"1000000000 Imp3D push-sum 20"}
mkdir -p $O
for rep in $(seq ${REPS:-3}); do
  for v in $VARIANTS; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 200 python3 tools/perf_round.py $CFG > $O/perf_$v.$rep.log 2>&1 || { tail -5 $O/perf_$v.$rep.log; exit 1; }
    echo "$v: $(grep -o 'k_[a-z_+<>A-Z0-9]*: [0-9.]* ms/round kernel' $O/perf_$v.$rep.log)"
  done
done
if [ -n "$SQ" ]; then
  for v in $VARIANTS; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/sq_$v -o p -- python3 tools/perf_round.py $CFG > $O/sq_$v.log 2>&1 || { tail -20 $O/sq_$v.log; exit 1; }
    echo "== $v"; python3 tools/pmc_summary.py $O/sq_$v "$SQ" --last=10 | grep -v "^{\|^}"
  done
fi
