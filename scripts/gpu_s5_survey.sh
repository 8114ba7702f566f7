#!/bin/bash
# Round-2 session-5 survey at HEAD: other BASELINE configs (kernel trace), C3 HBM bytes +
# SQ counters of the column-march gossip kernel vs the tiled one, and the headline
# kernel's lattice-gather traffic by direction (ablation builds); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_configs.sh || exit 1
echo "== C3 traffic (col default, tile walk 2)"
N=100000000 TOPO=Imp3D ALG=gossip KSUB=k_gossip VARIANTS="GP_EXP=1 GP_EXP=1,GP_KERNEL=tile" bash scripts/gpu_probe.sh || exit 1
echo "== C3 SQ counters k_gossip_col"
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/c3_sq -o p -- python3 tools/perf_round.py 100000000 Imp3D gossip 10 > gpurun_out/c3_sq.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/c3_sq "k_gossip_col" --last=10 | tr -d '\n '; echo
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/c3_tcc -o p -- python3 tools/perf_round.py 100000000 Imp3D gossip 10 > gpurun_out/c3_tcc.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/c3_tcc "k_gossip_col" --last=10 | tr -d '\n '; echo
echo "== Imp3D push-sum 1e9 lattice-direction ablations (wrong results, timing + bytes only)"
VARIANTS="GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_base.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_nolat.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_nox.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_noy.so GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_noz.so" bash scripts/gpu_probe.sh
