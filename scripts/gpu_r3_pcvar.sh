#!/bin/bash
# Push-sum column kernel variants at P = 1e9 (ms/round), then HBM traffic and SQ counters of the product kernel.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_pcvar}
mkdir -p $O
for v in ${VARIANTS:-nr2m4 nr4m3 nr4m4 nr2m5}; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_pc_$v.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$v.log 2>&1 || { tail -5 $O/perf_$v.log; exit 1; }
  echo "$v: $(grep -o 'k_ps_col<IMP3D>: [0-9.]* ms/round kernel' $O/perf_$v.log)"
done
timeout -k 10 400 python3 tools/traffic_probe.py 1000000000 Imp3D push-sum k_ps_col GP_EXP=1,GP_KERNEL=col > $O/traffic.log 2>&1 || { tail -5 $O/traffic.log; exit 1; }
cat $O/traffic.log
GP_EXP=1 GP_KERNEL=col timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/valu -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > $O/valu.log 2>&1 || { tail -20 $O/valu.log; exit 1; }
python3 tools/pmc_summary.py $O/valu "k_ps_col<3" --last=10
