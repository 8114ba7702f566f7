#!/bin/bash
# Full GPU suite on the current product library, then full-topology fine tiles of
# 1024 vs 2048 receivers (variant parity + C4 kernel traces); run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out/tb
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbtb11.so timeout -k 10 300 python -u tools/variant_parity.py 30000 full push-sum 300 || exit 1
GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_fbtb11.so timeout -k 10 300 python -u tools/variant_parity.py 200000 full push-sum 60 3 || exit 1
for v in lib_fbtb10 lib_fbtb11; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/$v.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tb/$v -o kt -- python3 tools/perf_round.py 100000000 full push-sum 10 > gpurun_out/tb_$v.log 2>&1 || { tail -20 gpurun_out/tb_$v.log; exit 1; }
  echo "== $v"; grep -v "^E2\|^W2" gpurun_out/tb_$v.log | tail -1
done
