#!/bin/bash
# Round 5: k_list_pack with static ranks (xdr / lwt) -- parity (virtual ranks, RCCL rank
# processes incl. C5 at 1e9), C5 W = 8 model against the previous build (lib_r5a); the
# LDS-resident C2 kernel with coherent face I/O and the grouped barrier (+ its no-work ablation).
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_static}; mkdir -p $O
timeout -k 10 560 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py > $O/multirank.log 2>&1 || { tail -30 $O/multirank.log; exit 1; }
tail -1 $O/multirank.log
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_multiproc.py > $O/mproc.log 2>&1 || { tail -30 $O/mproc.log; exit 1; }
tail -1 $O/mproc.log
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "block" > $O/block_pytest.log 2>&1 || { tail -30 $O/block_pytest.log; exit 1; }
tail -1 $O/block_pytest.log
model() {  # model <tag> <W> <env...>
  local t=$1 W=$2; shift 2
  local d=$O/vr_$t
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 1000000000 Imp3D push-sum $W 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 1000000000 Imp3D push-sum $W 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank max %.3f ms' % max(d['rank_compute_ms']), {k[:24]: round(sum(v)/len(v),3) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'])
for m in d['model']: print('   %g GB/s: sched %.3f ms -> %.3g' % (m['link_gbps'], m['round_ms_as_scheduled'], m['node_updates_per_s_overlapped']))"
}
model c5w8_static 8 GP_EXP=1 && model c5w8_r5a 8 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_r5a.so || exit 1
c2() {
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 1000000 3D push-sum 4000 > $O/c2_$l.log 2>&1 || { tail -5 $O/c2_$l.log; return 1; }
  echo "c2 $l: $(grep -o '[0-9.]* ms/round kernel' $O/c2_$l.log | head -1) $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_$l.log | head -1)"
}
c2 block GP_X=0 && c2 ablation GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_bkabl.so GP_KERNEL=block && c2 tile GP_EXP=1 GP_KERNEL=tile || exit 1
