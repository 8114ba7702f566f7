#!/bin/bash
# Walk-3 work stealing (tools/ablate.py steal, -DGP_STEAL=1): oracle parity at walk-3 sizes, then the
# headline kernel against base (product form) alternated, and C5 at W = 8 virtual ranks (kernel trace).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_steal}
mkdir -p $O
V=build/ablate/lib_steal.so
for c in "512000 Imp3D push-sum 300 3" "1000000 3D push-sum 200 4" "2744000 Imp3D push-sum 120 5"; do
  GOSSIP_HIP_LIB_EXPERIMENT=$V timeout -k 10 300 python3 tools/variant_parity.py $c >> $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
done
tail -3 $O/parity.log
for k in 1 2 3; do
  for v in base steal; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 40 > $O/perf_${v}_$k.log 2>&1 || { tail -5 $O/perf_${v}_$k.log; exit 1; }
    echo "$v $k: $(grep -o '[0-9.]* ms/round kernel' $O/perf_${v}_$k.log | head -1)"
  done
done
for v in base steal; do
  d=$O/vr_$v
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum 8 10 $O/m_$v.json > /dev/null || exit 1
  python3 -c "import json; d=json.load(open('$O/m_$v.json')); print('$v W=8', {k:round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()})"
done
