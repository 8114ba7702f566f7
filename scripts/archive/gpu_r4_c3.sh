#!/bin/bash
# C3 (gossip Imp3D 1e8): random-edge delivery counts as bytes (GP_RQ8=1) vs words -- parity, then same-box
# ms/round and the column kernel's HBM bytes.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_c3}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_multirank.py -k "byte_counters" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in 0 1; do
    GP_EXP=1 GP_RQ8=$v timeout -k 10 200 python3 tools/perf_round.py 100000000 Imp3D gossip 200 > $O/perf_$v.$rep.log 2>&1 || { tail -5 $O/perf_$v.$rep.log; exit 1; }
    echo "rq8=$v: $(grep -o 'k_[a-z_+<>A-Z0-9]*: [0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$v.$rep.log)"
  done
done
timeout -k 10 600 python3 tools/traffic_probe.py 100000000 Imp3D gossip k_gossip_col "GP_EXP=1,GP_RQ8=0" "GP_EXP=1,GP_RQ8=1" > $O/traffic.txt 2>&1 || { tail -5 $O/traffic.txt; exit 1; }
cat $O/traffic.txt
# C2 (3D push-sum, 1e6: launch / latency bound): tile-shape variants of the round kernel, wall per round
for v in base t1024m8 npt2 n2m6 t512m6; do
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 120 python3 tools/variant_parity.py 64000 3D push-sum 300 3 > $O/c2_parity_$v.log 2>&1 || { tail -5 $O/c2_parity_$v.log; exit 1; }
  GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 120 python3 tools/perf_round.py 1000000 3D push-sum 2000 > $O/c2_perf_$v.log 2>&1 || { tail -5 $O/c2_perf_$v.log; exit 1; }
  echo "C2 $v: $(grep -o 'no events: wall [0-9.]* ms/round' $O/c2_perf_$v.log) $(tail -1 $O/c2_parity_$v.log | cut -c1-40)"
done
