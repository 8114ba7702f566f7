#!/bin/bash
# C4 fused fold in 2048-receiver tiles with 512-thread blocks (two blocks per CU: 73 KB of LDS each;
# build/ablate/lib_tb11.so, -DGP_FB_TB=11 -DGP_FBF_THREADS=512) against the product, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c4tb11}
mkdir -p $O
V=build/ablate/lib_tb11.so
GOSSIP_HIP_LIB_EXPERIMENT=$V timeout -k 10 400 python3 -u tools/c4_variant_check.py > $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
tail -2 $O/check.log
run() {  # label, env...
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/perf_$l.log 2>&1 || { tail -5 $O/perf_$l.log; return 1; }
  echo "$l: $(grep -o 'wall [0-9.]* ms/round' $O/perf_$l.log | head -1)"
}
for k in 1 2; do
  run p$k GP_X=0 && run t$k GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 && run t${k}m GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 GP_FB_S1D=-1 && run t${k}p GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 GP_FB_S1D=1 || exit 1
done
GOSSIP_HIP_LIB_EXPERIMENT=$V GP_EXP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 tools/perf_round.py 100000000 full push-sum 20 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 tools/kt_steady.py $O/kt k_fb_ --last 20 || true
