#!/bin/bash
# C4 full push-sum: HBM bytes per kernel (request-size counters) and SQ/TCC counters of
# the three binning kernels; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in k_fb_send k_fb_split k_fb_fold; do
  echo "== $k"; N=100000000 TOPO=full ALG=push-sum KSUB=$k VARIANTS="default" bash scripts/gpu_probe.sh || exit 1
done
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/c4_sq -o p -- python3 tools/perf_round.py 100000000 full push-sum 10 > gpurun_out/c4_sq.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/c4_tcc -o p -- python3 tools/perf_round.py 100000000 full push-sum 10 > gpurun_out/c4_tcc.log 2>&1 || exit 1
for k in k_fb_send k_fb_split k_fb_fold; do echo "== $k"; python3 tools/pmc_summary.py gpurun_out/c4_sq "$k" --last=10 | tr -d '\n '; echo; python3 tools/pmc_summary.py gpurun_out/c4_tcc "$k" --last=10 | tr -d '\n '; echo; done
