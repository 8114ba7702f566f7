#!/bin/bash
# C4 fused with coarse bins one size below the rule: full push-sum parity, ms/round against the
# three-pass round (same box), per-pass HBM bytes, kernel trace.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "full or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o 'wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
run f1 GP_X=0 && run p1 GP_EXP=1 GP_FB_FUSED=0 && run f2 GP_X=0 && run p2 GP_EXP=1 GP_FB_FUSED=0 || exit 1
timeout -k 10 600 python3 tools/traffic_probe.py 100000000 full push-sum k_fb_split > $O/split_traffic.txt 2>&1 || { tail -5 $O/split_traffic.txt; exit 1; }
cat $O/split_traffic.txt
timeout -k 10 600 python3 tools/traffic_probe.py 100000000 full push-sum k_fb_fold > $O/fold_traffic.txt 2>&1 || { tail -5 $O/fold_traffic.txt; exit 1; }
cat $O/fold_traffic.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/perf_round.py 100000000 full push-sum 20 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 tools/kt_steady.py $O/kt k_fb_ --last 20 || true
