#!/bin/bash
# Round-kernel ablation (tools/ablate.py variants built on the CPU beforehand) +
# one SQ counter pass over the product kernel; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 600 python -u tools/ablate.py run ${N:-1000000000} ${VARIANTS} > gpurun_out/ablate.log 2>&1 || exit 1
mkdir -p gpurun_out/pmc_sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o p -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > gpurun_out/pmc_sq.log 2>&1
