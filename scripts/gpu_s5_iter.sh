#!/bin/bash
# Session-5 iteration: headline variants (time + HBM bytes), C3 after the redraw-first
# in-edge decisions, then the full GPU parity suite; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== C3 gossip Imp3D 1e8 (col)"
N=100000000 TOPO=Imp3D ALG=gossip KSUB=k_gossip VARIANTS="default" bash scripts/gpu_probe.sh || exit 1
echo "== headline variants"
VARIANTS="${HV:-GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so}" bash scripts/gpu_probe.sh || exit 1
echo "== GPU suite"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
