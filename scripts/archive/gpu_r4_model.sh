#!/bin/bash
# Multi-GPU model inputs at W = 8 (virtual ranks under a kernel trace) for C5 and C3, and the HBM
# traffic of the exchange kernels (k_pack / k_unpack) at W = 8 (tools/xchg_traffic.py).
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_model}
mkdir -p $O
for cfg in "1000000000 Imp3D push-sum 8" "100000000 Imp3D gossip 8"; do
  set -- $cfg; d=$O/vr_$3_$2_$1_w$4
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $1 $2 $3 $4 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  grep '^{' $d.log
  python3 tools/mgpu_model.py model $d $1 $2 $3 $4 10 $O/model_$3_$2_w$4.json > /dev/null || exit 1
done
timeout -k 10 600 python3 tools/xchg_traffic.py 1000000000 Imp3D push-sum 8 4 k_pack k_unpack k_ps_tile > $O/xt_c5_w8.txt 2>&1 || { tail -20 $O/xt_c5_w8.txt; exit 1; }
cat $O/xt_c5_w8.txt | grep -v '^{'
# rejected headline variant (in-edge pass as its own kernel): HBM bytes of both kernels
timeout -k 10 600 python3 tools/traffic_probe.py 1000000000 Imp3D push-sum k_ps_gather "GP_INBOX=1,GP_EXP=1" > $O/inbox_gather_traffic.txt 2>&1 || { tail -5 $O/inbox_gather_traffic.txt; exit 1; }
cat $O/inbox_gather_traffic.txt
timeout -k 10 600 python3 tools/traffic_probe.py 1000000000 Imp3D push-sum "k_ps_tile<3, false, true>" "GP_INBOX=1,GP_EXP=1" > $O/inbox_tile_traffic.txt 2>&1 || { tail -5 $O/inbox_tile_traffic.txt; exit 1; }
cat $O/inbox_tile_traffic.txt
