#!/bin/bash
# Gossip column kernel occupancy (waves/SIMD 5..8) on C3 and 3D gossip 1e8, the
# nibble wide-tile fallback parity test; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "wide_tile or kernel_variant" > gpurun_out/pytest_colw.log 2>&1 || { tail -30 gpurun_out/pytest_colw.log; exit 1; }
tail -1 gpurun_out/pytest_colw.log
for w in 5 6 7 8; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_colw$w.so timeout -k 10 300 python -u tools/variant_parity.py 1000000 Imp3D gossip 60 || exit 1
  for t in Imp3D 3D; do echo "colw$w $(GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_colw$w.so timeout -k 10 200 python -u tools/perf_round.py 100000000 $t gossip 20 | tail -1)"; done
done
