#!/bin/bash
# Report-curve harness: GPU-vs-oracle parity of the sweep, then the full sweep
# (n = 100..1000, 5 seeds, all 8 pairs); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_report_curves.py -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/pytest_report.log 2>&1 || { tail -30 gpurun_out/pytest_report.log; exit 1; }
tail -2 gpurun_out/pytest_report.log
timeout -k 10 600 python -u tools/report_curves.py --seeds ${SEEDS:-5} --out gpurun_out/report_curves > gpurun_out/report_curves.log 2>&1 || { tail -30 gpurun_out/report_curves.log; exit 1; }
tail -30 gpurun_out/report_curves.log
