#!/bin/bash
# Same-box A/B: GPU parity of the product library (TESTS, a pytest -k expression over
# test_gpu_parity.py + test_gpu_baseline_sizes.py), then ms/round of the product and of
# experiments-build variants (VARIANTS: build/ablate/lib_<v>.so) on CONFIGS.
export TMPDIR=/tmp
O=${O:-gpurun_out/ab}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py -x -q --timeout 300 --timeout-method thread \
    -k "$TESTS" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  echo "parity: $(tail -1 $O/pytest.log)"
fi
for cfg in ${CONFIGS:-"1000000000 Imp3D push-sum 20"}; do :; done
IFS=';' read -ra CFGS <<< "${CONFIGS:-1000000000 Imp3D push-sum 20}"
for cfg in "${CFGS[@]}"; do
  tag=$(echo $cfg | tr ' ' '_')
  for rep in 1 2; do
    for v in product $VARIANTS; do
      if [ $v = product ]; then
        timeout -k 10 200 python3 tools/perf_round.py $cfg > $O/perf_${tag}_$v.$rep.log 2>&1 || { tail -5 $O/perf_${tag}_$v.$rep.log; exit 1; }
      else
        GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 200 python3 tools/perf_round.py $cfg > $O/perf_${tag}_$v.$rep.log 2>&1 || { tail -5 $O/perf_${tag}_$v.$rep.log; exit 1; }
      fi
      echo "$cfg | $v: $(grep -o '| .*' $O/perf_${tag}_$v.$rep.log | head -1)"
    done
  done
done
