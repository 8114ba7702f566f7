# Round 6: parity of the product build (C5 / C4 kernels changed), then same-box alternated A/B:
# C5 round-kernel libraries and C4 whole experiments libraries.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_ab3
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_baseline_sizes.py::test_run_to_convergence_matches_oracle_record" -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  for v in wv sc scep; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 240 python3 tools/perf_round.py 1000000000 Imp3D push-sum 30 > $O/c5_$v.$rep.log 2>&1 || { tail -5 $O/c5_$v.$rep.log; exit 1; }
    echo "c5 $v: $(grep -o 'k_[a-z_+<>A-Z0-9, ]*: [0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/c5_$v.$rep.log)"
  done
  for v in c4base c4new; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 240 python3 tools/perf_round.py 100000000 full push-sum 40 > $O/c4_$v.$rep.log 2>&1 || { tail -5 $O/c4_$v.$rep.log; exit 1; }
    echo "c4 $v: $(grep -o 'wall [0-9.]* ms/round' $O/c4_$v.$rep.log | head -1)"
  done
done
