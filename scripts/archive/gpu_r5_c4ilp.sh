#!/bin/bash
# C4 fused fold: a thread's receivers folded two at a time in lock step (GP_FB_ILP=2, the in-tree
# build) against one after the other (build/ablate/lib_ilp1.so), same box, alternated; C4 parity first.
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c4ilp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "full or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000001 full push-sum 80 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o '[0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2 3; do
  run ilp2_$k GP_X=0 && run ilp1_$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_ilp1.so GP_EXP=1 || exit 1
done
