#!/bin/bash
# C5 at W = 8 virtual ranks: HBM bytes and SQ cycle counters per dispatch of k_list_pack and of the
# REMOTE round kernel (tools/pack_probe.py: three HBM passes + two SQ passes, each its own rocprofv3 run).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_packpmc}; mkdir -p $O
timeout -k 10 900 python3 -u tools/pack_probe.py 1000000000 Imp3D push-sum 8 k_list_pack "k_ps_tile<3, true>" > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
# C5 on 2 and 4 virtual ranks with the round-5 exchange (lists), for the DESIGN 7.1 table
model() {  # model <tag> <W>
  local t=$1 W=$2
  local d=$O/vr_$t
  GP_EXP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 20 $O/model_$t.json > /dev/null
}
model c5w2 2 && model c5w4 4 || exit 1
bash scripts/gpu_r5_pack4.sh
