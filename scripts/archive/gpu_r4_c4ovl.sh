#!/bin/bash
# C4 fused fold: next-round targets drawn while the tile's loads are in flight, reservation atomics
# overlapping the LDS scatter -- parity, then A/B against the previous commit's build
# (build/ablate/lib_c4prev.so), same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4ovl}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "full or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o 'wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2 3; do
  run new$k GP_X=0 && run prev$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_c4prev.so GP_EXP=1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 tools/perf_round.py 100000000 full push-sum 20 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 tools/kt_steady.py $O/kt k_fb_ --last 20 || true
