# Same-box alternated A/B: C5 round-kernel libraries (C5V) and C4 whole libraries (C4V).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_ab4}
mkdir -p $O
for rep in $(seq ${REPS:-3}); do
  for v in $C5V; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 240 python3 tools/perf_round.py 1000000000 Imp3D push-sum 60 > $O/c5_$v.$rep.log 2>&1 || { tail -5 $O/c5_$v.$rep.log; exit 1; }
    echo "c5 $v: $(grep -o 'k_[a-z_+<>A-Z0-9, ]*: [0-9.]* ms/round kernel' $O/c5_$v.$rep.log)"
  done
  for v in $C4V; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 240 python3 tools/perf_round.py 100000000 full push-sum 60 > $O/c4_$v.$rep.log 2>&1 || { tail -5 $O/c4_$v.$rep.log; exit 1; }
    echo "c4 $v: $(grep -o 'wall [0-9.]* ms/round' $O/c4_$v.$rep.log | head -1)"
  done
done
