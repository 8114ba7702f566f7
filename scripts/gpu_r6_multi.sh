#!/bin/bash
# Round 6, several ranks: parity of the multi-rank paths (virtual ranks, RCCL rank processes incl.
# the BASELINE-size runs), then the modelled C5 / C4 rounds at W = 8 for the HEAD experiments
# library before the global-store / uniform-resource change (lib_xbase) and after, same box.
set -o pipefail
export TMPDIR=/tmp
O=${O:-gpurun_out/r6_multi}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl_multiproc.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_multi.log 2>&1 || { tail -30 $O/pytest_multi.log; exit 1; }
tail -1 $O/pytest_multi.log
model() {  # model <tag> <n> <topo> <W> <lib>
  local t=$1 n=$2 topo=$3 w=$4 lib=$5
  local d=$O/vr_$t
  GOSSIP_HIP_LIB_EXPERIMENT=$lib timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/mgpu_model.py run $n $topo push-sum $w 10 > $d.log 2>&1 || { tail -20 $d.log; return 1; }
  python3 tools/mgpu_model.py model $d $n $topo push-sum $w 10 $O/model_$t.json > /dev/null || return 1
  python3 -c "
import json; d=json.load(open('$O/model_$t.json'))
P=$n if '$topo'!='Imp3D' else round($n**(1/3))**3
print('$t: rank compute max %.3f ms, sched %.3f (128) / %.3f (64) ms' % (max(d['rank_compute_ms']), d['model'][1]['round_ms_as_scheduled'], d['model'][0]['round_ms_as_scheduled']))
print('   per-slab kernels', {k: round(sum(v)/len(v),4) for k,v in d['per_slab_kernel_ms'].items()})"
  rm -f $d/*/kt_kernel_trace.csv $d/kt_kernel_trace.csv 2>/dev/null; true
}
NEW=gossipprotocol_amd/libgossip_hip_exp.so; OLD=build/ablate/lib_xbase.so
model c5w8_old 1000000000 Imp3D 8 $OLD && model c5w8_new 1000000000 Imp3D 8 $NEW && model c4w8_old 100000000 full 8 $OLD && model c4w8_new 100000000 full 8 $NEW
