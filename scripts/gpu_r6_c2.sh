#!/bin/bash
# Round 6, C2: the LDS-resident kernel with neighbour flags inside 16-round epochs (one grid
# barrier per epoch, checkpoint replay of the converging epoch) -- parity, the C2 whole-run
# record, then timing against the round-5 form (build/ab/exp_old.so, same box).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_c2}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "block" > $O/block_pytest.log 2>&1 || { tail -30 $O/block_pytest.log; exit 1; }
tail -1 $O/block_pytest.log
c2() {
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_$l.log 2>&1 || { tail -5 $O/c2_$l.log; return 1; }
  echo "c2 $l: $(grep -o '[0-9.]* ms/round kernel' $O/c2_$l.log | head -1) $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_$l.log | head -1)"
}
c2 new GP_EXP=1 && c2 old GOSSIP_HIP_LIB_EXPERIMENT=build/ab/exp_old.so && c2 new2 GP_EXP=1 || exit 1
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_baseline_sizes.py -k "record and c2" > $O/record_pytest.log 2>&1 || { tail -30 $O/record_pytest.log; exit 1; }
tail -1 $O/record_pytest.log
