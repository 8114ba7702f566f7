#!/bin/bash
# C2 (3D push-sum, n = 1e6): the LDS-resident kernel -- parity, then timing against the tile kernel
# and its no-node-work ablation (same box).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_c2}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "block" > $O/block_pytest.log 2>&1 || { tail -30 $O/block_pytest.log; exit 1; }
tail -1 $O/block_pytest.log
c2() {
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_$l.log 2>&1 || { tail -5 $O/c2_$l.log; return 1; }
  echo "c2 $l: $(grep -o '[0-9.]* ms/round kernel' $O/c2_$l.log | head -1) $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_$l.log | head -1)"
}
c2 block GP_X=0 && c2 ablation GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_bkabl.so GP_KERNEL=block && c2 tile GP_EXP=1 GP_KERNEL=tile && c2 block2 GP_X=0 || exit 1
# C2 to convergence on the product's kernel (the LDS-resident one): rounds and wall time
timeout -k 10 300 python3 tools/converge.py 1000000 3D push-sum 1 $O/c2_converge.json > $O/c2_converge.log 2>&1 || { tail -5 $O/c2_converge.log; exit 1; }
tail -2 $O/c2_converge.log
