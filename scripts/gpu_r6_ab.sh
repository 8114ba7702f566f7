# Same-box alternating A/B of round-kernel libraries (build/ablate/lib_<v>.so, scripts/build_round_ab.sh)
# on the C5 workload, then optional parity tests of the product build.  VARIANTS, REPS, O, CFG, TESTS.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_ab}
CFG=${CFG:-"1000000000 Imp3D push-sum 30"}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
for rep in $(seq ${REPS:-3}); do
  for v in $VARIANTS; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 240 python3 tools/perf_round.py $CFG > $O/perf_$v.$rep.log 2>&1 || { tail -5 $O/perf_$v.$rep.log; exit 1; }
    echo "$v: $(grep -o 'k_[a-z_+<>A-Z0-9, ]*: [0-9.]* ms/round kernel' $O/perf_$v.$rep.log)"
  done
done
