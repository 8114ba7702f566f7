#!/bin/bash
# Gossip Imp3D (C3) variants (build/ablate/lib_<v>.so): bit-exact vs the oracle, then
# kernel traces at P = 1.005e8; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out/c3
for v in ${PAR_VARIANTS:-cnew}; do
  for c in "1000000 Imp3D gossip 60" "8000000 Imp3D gossip 40"; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 300 python -u tools/variant_parity.py $c || exit 1
  done
done
for v in ${TIME_VARIANTS:-chead cnew}; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3/$v -o kt -- python3 tools/perf_round.py 100000000 Imp3D gossip 20 > gpurun_out/c3/$v.log 2>&1 || { tail -20 gpurun_out/c3/$v.log; exit 1; }
  echo "== $v $(grep -v '^E2\|^W2' gpurun_out/c3/$v.log | tail -1)"
  python3 tools/kt_steady.py gpurun_out/c3/$v k_gossip
done
