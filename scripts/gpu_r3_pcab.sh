#!/bin/bash
# Push-sum column kernel vs the tile kernel at P = 1e9 (same box): parity of the column
# variants on the small cases, then ms/round of the tile kernel, the default column
# kernel and its build variants.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_pcab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "kernel_variant and col" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_tile.log 2>&1 || { tail -5 $O/perf_tile.log; exit 1; }
echo "tile: $(grep -o 'k_ps_tile<IMP3D>: [0-9.]* ms/round kernel' $O/perf_tile.log)"
GP_EXP=1 GP_KERNEL=col timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_col.log 2>&1 || { tail -5 $O/perf_col.log; exit 1; }
echo "col: $(grep -o 'k_ps_col<IMP3D>: [0-9.]* ms/round kernel' $O/perf_col.log)"
for v in ${VARIANTS:-nr2m4 nr4m3 nr2m5 nr2a2 nr2a3 nr4m3a2}; do
  GP_KERNEL=col GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_pc_$v.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$v.log 2>&1 || { tail -5 $O/perf_$v.log; exit 1; }
  echo "$v: $(grep -o 'k_ps_col<IMP3D>: [0-9.]* ms/round kernel' $O/perf_$v.log)"
done
