#!/bin/bash
# Full-topology push-sum binning variants (scripts/build_fb_variants.sh): bit-exact vs
# the oracle, then C4 round time per variant and HBM bytes per kernel; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out/fb
for v in ${PAR_VARIANTS:-fbv2}; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 300 python -u tools/variant_parity.py 30000 full push-sum 300 || exit 1
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 300 python -u tools/variant_parity.py 200000 full push-sum 60 3 || exit 1
done
for v in ${TIME_VARIANTS:-fbv1 fbv2}; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fb/$v -o kt -- python3 tools/perf_round.py 100000000 full push-sum 10 > gpurun_out/fb/$v.log 2>&1 || { tail -20 gpurun_out/fb/$v.log; exit 1; }
  echo "== $v $(grep -v '^E2\|^W2' gpurun_out/fb/$v.log | tail -1)"
  python3 - gpurun_out/fb/$v <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_fb" in row["Name"]:
            print("   %-40s calls %5s avg %8.3f ms" % (row["Name"][:40], row["Calls"], float(row["AverageNs"]) / 1e6))
PY
done
for k in ${PROBE_KERNELS:-k_fb_send k_fb_split}; do
  for v in ${PROBE_VARIANTS:-fbv1 fbv2}; do
    echo "== $k $v"; N=100000000 TOPO=full ALG=push-sum KSUB=$k VARIANTS="GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so" bash scripts/gpu_probe.sh || exit 1
  done
done
