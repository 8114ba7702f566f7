#!/bin/bash
# Round 5: the LDS-resident 3D push-sum kernel (gp_block.hip) -- parity, then C2 timing against
# the tile kernel (same box).  Then the exchange A/B (scripts/gpu_r5_xchg.sh).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_block}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "block" > $O/block_pytest.log 2>&1 || { tail -30 $O/block_pytest.log; exit 1; }
tail -1 $O/block_pytest.log
c2() {
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_$l.log 2>&1 || { tail -5 $O/c2_$l.log; return 1; }
  echo "c2 $l: $(grep -o 'wall [0-9.]* ms/round' $O/c2_$l.log | head -1) $(grep -o '[0-9.]* ms/round kernel' $O/c2_$l.log | head -1) $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_$l.log | head -1)"
}
c2 block GP_X=0 && c2 tile GP_EXP=1 GP_KERNEL=tile && c2 block2 GP_X=0 || exit 1
if [ -n "$WITH_XCHG" ]; then O=gpurun_out/r5_xchg bash scripts/gpu_r5_xchg.sh; fi
