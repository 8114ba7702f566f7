#!/bin/bash
# C2 on the LDS-resident kernel: every lattice slot folded with non-senders reading the zero sentinel (GP_BK_SENTINEL=1,
# the product build) against a branch per slot (build/ablate/lib_sent0.so), same box; block parity first.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c2sent}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "block" > $O/block_pytest.log 2>&1 || { tail -30 $O/block_pytest.log; exit 1; }
tail -1 $O/block_pytest.log
c2() {
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_$l.log 2>&1 || { tail -5 $O/c2_$l.log; return 1; }
  echo "c2 $l: $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_$l.log | head -1)"
}
for k in 1 2; do
  c2 sentinel$k GP_X=0 && c2 branches$k GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_sent0.so GP_KERNEL=block || exit 1
done
