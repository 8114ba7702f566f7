#!/bin/bash
# (1) wave-end neighbours in LDS: push-sum parity + headline A/B vs the previous build;
# (2) LDS-ordered full-topology binning: variant parity + C4 time; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_s5_zb.sh || exit 1
GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbord.so timeout -k 10 300 python -u tools/variant_parity.py 30000 full push-sum 300 || exit 1
GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbord.so timeout -k 10 300 python -u tools/variant_parity.py 200000 full push-sum 60 3 || exit 1
for v in lib_base lib_fbord; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab2/$v -o kt -- python3 tools/perf_round.py 100000000 full push-sum 10 > gpurun_out/ab2_$v.log 2>&1 || { tail -20 gpurun_out/ab2_$v.log; exit 1; }
  echo "== $v"; grep -v "^E2\|^W2" gpurun_out/ab2_$v.log | tail -1
done
