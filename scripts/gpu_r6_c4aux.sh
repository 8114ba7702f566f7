#!/bin/bash
# C4 one rank: the fold reads each message's receiver offset (written by the split) instead of
# drawing the sender's target again.  Parity (one rank: boundary sizes, the three-pass form, the
# whole 624-round run at 1e8; several ranks), then A/B against the previous commit, same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_c4aux}; mkdir -p $O
OLD=${OLD:-build/ab/exp_303c4e4.so}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_multirank.py -k "full" -x -v --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_full.log | tail -1; grep -E "FAILED|Error" $O/pytest_full.log | head; [ $rc = 0 ] || exit $rc
for i in 1 2 3; do
  for lib in new old; do
    if [ $lib = new ]; then L=gossipprotocol_amd/libgossip_hip_exp.so; else L=$OLD; fi
    GOSSIP_HIP_LIB_EXPERIMENT=$L timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 40 > $O/c4_${lib}_$i.log 2>&1 || { tail $O/c4_${lib}_$i.log; exit 1; }
    echo "C4 one rank, $lib: $(tail -1 $O/c4_${lib}_$i.log)"
  done
done
timeout -k 10 500 python3 tools/traffic_probe.py 100000000 full push-sum k_fb_fold default > $O/fold_traffic.txt 2>&1 && cat $O/fold_traffic.txt
timeout -k 10 500 python3 tools/traffic_probe.py 100000000 full push-sum k_fb_split default > $O/split_traffic.txt 2>&1 && cat $O/split_traffic.txt
