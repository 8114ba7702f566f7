#!/bin/bash
# Round 5: exchange rework A/B.  Parity first (virtual ranks, RCCL rank processes), then the
# per-rank models (tools/mgpu_model.py) of C5 (Imp3D push-sum, lists) and C3 (Imp3D gossip,
# bitmaps) for this build and the round-4 build (build/ablate/lib_r4.so), same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r5_xchg}; mkdir -p $O
timeout -k 10 560 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py > $O/multirank.log 2>&1 || { tail -30 $O/multirank.log; exit 1; }
tail -1 $O/multirank.log
[ -n "$SKIP_MPROC" ] || timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rccl_multiproc.py > $O/mproc.log 2>&1 || { tail -30 $O/mproc.log; exit 1; }
[ -n "$SKIP_MPROC" ] || tail -1 $O/mproc.log
model() {  # model <tag> <n> <topo> <alg> <W> <lib: new|r4>
  local d=$O/vr_$1_w$5_$6
  if [ $6 = new ]; then export GP_EXP=1; else export GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$6.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $2 $3 $4 $5 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  unset GOSSIP_HIP_LIB_EXPERIMENT GP_EXP
  python3 tools/mgpu_model.py model $d $2 $3 $4 $5 20 $O/model_$1_w$5_$6.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$1_w$5_$6.json'))
print('$1 W=$5 $6: rank max %.3f ms' % max(d['rank_compute_ms']), {k[:24]: round(sum(v)/len(v),3) for k,v in d['per_slab_kernel_ms'].items()}, d['global_kernel_ms'])
for m in d['model']: print('   %g GB/s: sched %.3f ms -> %.3g' % (m['link_gbps'], m['round_ms_as_scheduled'], m['node_updates_per_s_overlapped']))"
}
for v in new r4; do model c5 1000000000 Imp3D push-sum 8 $v || exit 1; done
for W in 2 8; do for v in new r4; do model c3 100000000 Imp3D gossip $W $v || exit 1; done; done
# C4: the fused fold's message prefetch (GP_FB_PF) -- parity, then alternated timing against GP_FB_PF=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread -k "full or c4" > $O/c4_pytest.log 2>&1 || { tail -30 $O/c4_pytest.log; exit 1; }
tail -1 $O/c4_pytest.log
c4() {
  local l=$1; shift
  env "$@" timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 80 > $O/c4_$l.log 2>&1 || { tail -5 $O/c4_$l.log; return 1; }
  echo "c4 $l: $(grep -o 'wall [0-9.]* ms/round' $O/c4_$l.log | head -1)"
}
c4 pf1 GP_X=0 && c4 pf0 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbpf0.so && c4 pf1b GP_X=0 && c4 pf0b GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbpf0.so || exit 1
