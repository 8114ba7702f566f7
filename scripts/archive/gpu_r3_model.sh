#!/bin/bash
# Multi-GPU cost model inputs (virtual ranks on one GPU under a kernel trace) for C5 and C4,
# and the C3 round: kernel vs wall over 200 rounds, with the kernel trace of every kernel.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_model}
mkdir -p $O
for cfg in "1000000000 Imp3D push-sum 8" "1000000000 Imp3D push-sum 4" "1000000000 Imp3D push-sum 2" "100000000 full push-sum 8" "100000000 full push-sum 4" "100000000 full push-sum 2"; do
  set -- $cfg; d=$O/vr_$3_$2_$1_w$4
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $1 $2 $3 $4 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  grep '^{' $d.log
done
d=$O/c3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o kt -- python3 tools/perf_round.py 100000000 Imp3D gossip 200 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
grep -v "^W2\|^E2" $d.log | tail -2
python3 tools/kt_steady.py $d k_ --last 200
