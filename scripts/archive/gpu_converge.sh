#!/bin/bash
# Headline configuration run to convergence (C5 on one GPU) + the activation-phase
# round time; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "Imp3D or golden or live" > gpurun_out/pytest_act.log 2>&1 || { tail -20 gpurun_out/pytest_act.log; exit 1; }
tail -2 gpurun_out/pytest_act.log
timeout -k 10 300 python -u tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/perf.log 2>&1 || { cat gpurun_out/perf.log; exit 1; }
cat gpurun_out/perf.log
timeout -k 10 900 python -u tools/converge.py ${N:-1000000000} Imp3D push-sum 1 gpurun_out/converge.json 2> gpurun_out/converge.err
rc=$?
tail -3 gpurun_out/converge.err
exit $rc
