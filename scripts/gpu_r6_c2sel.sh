set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_c2sel}; mkdir -p $O
c2() {
  local l=$1; shift
  env "$@" GP_KERNEL=block timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_$l.log 2>&1 || { tail -5 $O/c2_$l.log; return 1; }
  echo "c2 $l: $(grep -o '[0-9.]* ms/round kernel' $O/c2_$l.log | head -1) $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_$l.log | head -1)"
}
for i in 1 2 3; do
  c2 pf$i GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_c2pf.so || exit 1
  c2 sel$i GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_c2sel.so || exit 1
done
