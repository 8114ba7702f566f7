#!/bin/bash
# C4 across ranks, round 6 (the fold bins the next round's messages by destination rank and
# coarse bin into the exchange buffers): parity on virtual ranks and RCCL rank processes (the
# BASELINE-size C4 case included), the modelled rounds at W = 2 / 4 / 8, and the one-rank C4
# round A/B against the round-5 end state (build/ab/exp_<old>.so), same box, alternated.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_c4multi}; mkdir -p $O
OLD=${OLD:-build/ab/exp_d36cf59.so}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl_multiproc.py -k "full" -x -v --timeout 300 --timeout-method thread > $O/pytest_full.log 2>&1
rc=$?; grep -E "passed|failed" $O/pytest_full.log | tail -1; grep -E "FAILED|Error" $O/pytest_full.log | head; [ $rc = 0 ] || exit $rc
model() {  # model <tag> <W>
  local t=$1 w=$2
  local d=$O/vr_$t
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run 100000000 full push-sum $w 20 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d 100000000 full push-sum $w 20 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
print('$t: rank compute max %.3f ms, regions %s, sched %.3f (128) / %.3f (64) ms, %.3g / %.3g node-updates/s' % (max(d['rank_compute_ms']), d['full_fused_regions'], d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled'], d['model'][1]['node_updates_per_s_overlapped'], d['model'][0]['node_updates_per_s_overlapped']))
print('   per-slab kernels', {k: round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()})"
  rm -f $d/*/kt_kernel_trace.csv 2>/dev/null; true
}
model c4w2 2 && model c4w4 4 && model c4w8 8 || exit 1
for i in 1 2; do
  for lib in new old; do
    if [ $lib = new ]; then L=gossipprotocol_amd/libgossip_hip_exp.so; else L=$OLD; fi
    GOSSIP_HIP_LIB_EXPERIMENT=$L timeout -k 10 200 python3 tools/perf_round.py 100000000 full push-sum 40 > $O/c4_${lib}_$i.log 2>&1 || { tail $O/c4_${lib}_$i.log; exit 1; }
    echo "C4 one rank, $lib: $(tail -1 $O/c4_${lib}_$i.log)"
  done
done
