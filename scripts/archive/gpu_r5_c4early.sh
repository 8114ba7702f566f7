#!/bin/bash
# C4 fused fold: the send phase's counts and reservations issued before the fold (GP_FB_EARLY=1, the
# product) against the round-4/5 order (build/ablate/lib_fbe0.so, -DGP_FB_EARLY=0), same box; C4 parity first.
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c4early}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "full or c4" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
V=build/ablate/lib_fbe0.so
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000001 full push-sum 80 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o '[0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2; do
  run early$k GP_X=0 && run old$k GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/perf_round.py 100000001 full push-sum 20 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 tools/kt_steady.py $O/kt k_fb_ --last 20 || true
