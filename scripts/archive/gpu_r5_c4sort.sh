#!/bin/bash
# C4 fused fold: the receivers' insertion sort moving (sender, payload) pairs (GP_FB_SORTMSG=1, the
# product) against sorting slot indices (build/ablate/lib_sm0.so), same box, alternated; C4 parity
# first; then the per-phase stamps of the new form (build/ablate/lib_fbst.so).
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c4sort}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "full or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000001 full push-sum 80 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o '[0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2; do
  run sortmsg$k GP_X=0 && run sortidx$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_sm0.so GP_EXP=1 || exit 1
done
GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbst.so timeout -k 10 300 python3 tools/fold_stamps.py 100000001 20 > $O/stamps.txt 2>&1 || { tail -5 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
