#!/bin/bash
# Same-box alternated A/B of exchange-kernel libraries on the C5 W = 8 virtual-rank run: per-kernel
# averages from the rocprofv3 kernel-trace stats (k_list_pack and the rest).  VARIANTS, REPS, O.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_lpab}; mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for v in $VARIANTS; do
    d=$O/$v.$rep
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    python3 - "$d" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/kt_kernel_stats.csv', recursive=True)[0]
rows = {r['Name'][:40]: (float(r['AverageNs']) / 1e6, int(r['Calls'])) for r in csv.DictReader(open(f))}
print(sys.argv[2], {k: '%.4f ms x %d' % v for k, v in rows.items() if any(s in k for s in ('k_list_pack', 'k_ps_tile', 'k_halo', 'k_pack'))})
PY
    rm -f $d/*/kt_kernel_trace.csv $d/kt_kernel_trace.csv 2>/dev/null
  done
done
