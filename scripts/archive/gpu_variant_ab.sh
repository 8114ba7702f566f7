#!/bin/bash
# A/B of experiments-build variants of the push-sum tile kernel against the product kernel
# (same box): parity of each variant (kernel-variant tests through the variant library),
# then ms/round at P = 1e9.   VARIANTS="lg ..." (build/ablate/lib_<v>.so)
export TMPDIR=/tmp
O=${O:-gpurun_out/variant_ab}
mkdir -p $O
for v in $VARIANTS; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread \
    -k "tile or walk or stage or wide or fuse or imp3d or Imp3D" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v parity: $(tail -1 $O/pytest_$v.log)"
done
timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_product.log 2>&1 || { tail -5 $O/perf_product.log; exit 1; }
echo "product: $(grep -o 'k_ps_tile<IMP3D>: [0-9.]* ms/round kernel' $O/perf_product.log)"
for v in $VARIANTS; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$v.log 2>&1 || { tail -5 $O/perf_$v.log; exit 1; }
  echo "$v: $(grep -o 'preroll.*ms/round kernel' $O/perf_$v.log)"
done
