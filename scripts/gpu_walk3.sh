#!/bin/bash
# walk 3 (per-XCD tile queue): push-sum parity, then time + HBM bytes vs walk 2; lattice-gather ablations (walk 2 build); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_baseline_sizes.py -x -v --timeout 200 --timeout-method thread -k "push or golden or live or c5" > gpurun_out/pytest_walk3.log 2>&1 || { tail -30 gpurun_out/pytest_walk3.log; exit 1; }
tail -2 gpurun_out/pytest_walk3.log
VARIANTS="GP_EXP=1 GP_EXP=1,GP_WALK=2" bash scripts/gpu_probe.sh || exit 1
TOPO=3D VARIANTS="GP_EXP=1 GP_EXP=1,GP_WALK=2 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_nolat.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_nox.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_noy.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_noz.so" bash scripts/gpu_probe.sh
