#!/bin/bash
# C2 on the LDS-resident kernel: a face node.s (s, w) as one 16-byte sc1 buffer store / load (GP_BK_B128=0,
# build/ablate/lib_b128.so) against two 8-byte agent-scope atomic stores / loads (the product) (build/ablate/lib_b128.so), same box; block parity first.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c2b128}; mkdir -p $O
for c in "27000 3D push-sum 3000" "1000000 3D push-sum 600"; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_b128.so GP_EXP=1 GP_KERNEL=block timeout -k 10 300 python3 tools/variant_parity.py $c > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
  tail -1 $O/parity.log
done
c2() {
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_$l.log 2>&1 || { tail -5 $O/c2_$l.log; return 1; }
  echo "c2 $l: $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_$l.log | head -1)"
}
for k in 1 2; do
  c2 b128_$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_b128.so GP_KERNEL=block && c2 atomics$k GP_X=0 || exit 1
done
