#!/bin/bash
# k_pack with wave priority raised while it issues its loads (-DGP_XCHG_PRIO=1, lib_xp1.so) against the
# same build without (lib_xp0.so): C5 at W = 8 virtual ranks, kernel traces, alternated, same box.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_xprio}
mkdir -p $O
for k in 1 2; do
  for v in xp0 xp1; do
    d=$O/vr_${v}_$k
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
    python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum 8 10 $O/m_${v}_$k.json > /dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/m_${v}_$k.json')); print('$v $k', {k:round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'])"
  done
done
