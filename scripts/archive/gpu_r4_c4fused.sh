#!/bin/bash
# C4: the fold bins the next round's messages (one rank, k_fb_fold<true>) against the three-pass round
# (experiments build, GP_FB_FUSED=0): full push-sum parity, ms/round at P = 1e8 (same box), HBM bytes.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4fused}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread -k "full or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in f p f p; do
  if [ $v = p ]; then export GP_EXP=1 GP_FB_FUSED=0; else unset GP_EXP GP_FB_FUSED; fi
  timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 40 > $O/perf_$v.log 2>&1 || { tail -5 $O/perf_$v.log; exit 1; }
  echo "$v: $(grep -o 'wall [0-9.]* ms/round' $O/perf_$v.log | head -1) $(grep -o 'kernel [0-9.]* ms/round' $O/perf_$v.log | head -1)"
done
unset GP_EXP GP_FB_FUSED
timeout -k 10 600 python3 tools/traffic_probe.py 100000000 full push-sum k_fb_fold > $O/fold_traffic.txt 2>&1 || { tail -5 $O/fold_traffic.txt; exit 1; }
cat $O/fold_traffic.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/perf_round.py 100000000 full push-sum 20 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 tools/kt_steady.py $O/kt k_fb_ --last 60 || true
