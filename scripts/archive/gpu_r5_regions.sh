#!/bin/bash
# Imp3D push-sum exchange in 4 regions (XREGIONS) instead of 2: virtual-rank parity, RCCL rank-process
# parity (incl. the BASELINE sizes), then the C5 W = 8 model against 2 regions (GP_XREGIONS=2), same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_regions}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py > $O/multirank.log 2>&1 || { grep -E "FAILED|Error" $O/multirank.log | head; tail -30 $O/multirank.log; exit 1; }
tail -1 $O/multirank.log
GP_MPROC_FULL=1 timeout -k 10 700 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_rccl_multiproc.py > $O/mproc.log 2>&1 || { tail -30 $O/mproc.log; exit 1; }
tail -1 $O/mproc.log
model() {  # model <tag> <W> <env...>
  local t=$1 W=$2; shift 2
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank max %.3f ms' % max(d['rank_compute_ms']), 'halo B/dir', d['halo_bytes_per_direction'], d['global_kernel_ms'])
for m in d['model']: print('   %g GB/s: exchange %.3f sched %.3f ms -> %.3g' % (m['link_gbps'], m['exchange_ms'], m['round_ms_as_scheduled'], m['node_updates_per_s_overlapped']))"
}
model c5w8_r4 8 GP_EXP=1 && model c5w8_r2 8 GP_EXP=1 GP_XREGIONS=2 && model c5w8_r4b 8 GP_EXP=1 && model c5w8_r2b 8 GP_EXP=1 GP_XREGIONS=2
