export TMPDIR=/tmp
mkdir -p gpurun_out/r4_state
timeout -k 10 120 build/scatter_bench > gpurun_out/r4_state/scatter_bench.txt 2>&1 && cat gpurun_out/r4_state/scatter_bench.txt && bash scripts/gpu_r4_bench.sh
