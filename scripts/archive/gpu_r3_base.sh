#!/bin/bash
# Round-3 start: the headline bench on a fresh box + one SQ counter pass on the
# round kernel (VALU issue vs wave cycles) to split compute from memory time.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_base}
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $O/valu -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > $O/valu.log 2>&1 || { tail -20 $O/valu.log; exit 1; }
grep -v "^E2\|^W2" $O/valu.log | tail -3
python3 tools/pmc_summary.py $O/valu "k_ps_tile<3" --last=10
