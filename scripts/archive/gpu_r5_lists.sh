#!/bin/bash
# Round 5: sender-ordered lists for Imp3D push-sum across ranks (no k_unpack).
#  1. virtual-rank parity (1-16 ranks) and RCCL rank-process parity (incl. C5 at 1e9, W = 2);
#  2. C5 W = 8 per-rank model (tools/mgpu_model.py), the new build and the round-4 build
#     (build/ablate/lib_r4.so) on the same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_lists}; mkdir -p $O
timeout -k 10 560 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py > $O/multirank.log 2>&1 || { tail -30 $O/multirank.log; exit 1; }
tail -2 $O/multirank.log
[ -n "$SKIP_MPROC" ] || timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_multiproc.py > $O/mproc.log 2>&1 || { tail -30 $O/mproc.log; exit 1; }
[ -n "$SKIP_MPROC" ] || tail -2 $O/mproc.log
for v in new rkearly r4; do
  d=$O/vr_c5_w8_$v
  if [ $v = new ]; then export GP_EXP=1; else export GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum 8 10 > $d.log 2>&1 || { tail -20 $d.log; exit 1; }
  unset GOSSIP_HIP_LIB_EXPERIMENT GP_EXP
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum 8 10 $O/model_c5_w8_$v.json > $O/model_$v.txt || exit 1
  grep -E '"rank_compute_ms"|round_ms_as_scheduled|node_updates_per_s_overlapped' -A0 $O/model_c5_w8_$v.json | head -12
done
