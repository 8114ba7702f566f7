#!/bin/bash
# Push-sum tile-kernel variants (build/ablate/lib_<v>.so): bit-exact vs the oracle on
# Imp3D / 3D / line, then round time + HBM bytes at P = 1e9; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${PAR_VARIANTS:-rnew}; do
  for c in "1000000 Imp3D push-sum 200" "125000 3D push-sum 100" "20000 line push-sum 100"; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 300 python -u tools/variant_parity.py $c || exit 1
  done
done
V=""; for v in ${TIME_VARIANTS:-rhead rnew}; do V="$V GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so"; done
N=${N:-1000000000} TOPO=${TOPO:-Imp3D} VARIANTS="$V" bash scripts/gpu_probe.sh
