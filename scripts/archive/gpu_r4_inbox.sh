#!/bin/bash
# Headline kernel experiment: the in-edge pass as a kernel of its own (GP_INBOX=1, experiments build;
# build/ablate/lib_inb6.so: the round kernel at 6 waves/SIMD) -- parity, then same-box ms/round at
# P = 1e9 alternating with the product kernel, then HBM bytes of both kernels.
export TMPDIR=/tmp
O=${O:-gpurun_out/r4_inbox}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_parity.py -k "inbox" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
GP_INBOX=1 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_inb6.so timeout -k 10 300 python3 tools/variant_parity.py 512000 Imp3D push-sum 120 4 > $O/parity_inb6.log 2>&1 || { tail -5 $O/parity_inb6.log; exit 1; }
tail -1 $O/parity_inb6.log
for rep in 1 2; do
  for v in product inbox inb6; do
    case $v in
      product) env -u GP_INBOX -u GP_EXP -u GOSSIP_HIP_LIB_EXPERIMENT timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$v.$rep.log 2>&1 ;;
      inbox) GP_INBOX=1 GP_EXP=1 timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$v.$rep.log 2>&1 ;;
      inb6) GP_INBOX=1 GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_inb6.so timeout -k 10 200 python3 tools/perf_round.py 1000000000 Imp3D push-sum 20 > $O/perf_$v.$rep.log 2>&1 ;;
    esac
    [ $? -eq 0 ] || { tail -5 $O/perf_$v.$rep.log; exit 1; }
    echo "$v: $(grep -o 'k_[a-z_+<>A-Z0-9]*: [0-9.]* ms/round kernel, wall [0-9.]* ms/round' $O/perf_$v.$rep.log)"
  done
done
GP_INBOX=1 GP_EXP=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_inbox -o kt -- python3 tools/perf_round.py 1000000000 Imp3D push-sum 10 > $O/kt_inbox.log 2>&1 || { tail -5 $O/kt_inbox.log; exit 1; }
python3 tools/kt_steady.py $O/kt_inbox k_ps --last 20
