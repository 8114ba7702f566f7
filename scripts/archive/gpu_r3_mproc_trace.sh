#!/bin/bash
# Kernel traces of two RCCL rank processes on one GPU (per-rank NCCL_HOSTID, socket transport):
# each rank worker runs under its own rocprofv3 --kernel-trace --stats, C5 workload (n = 1e9) for 100 rounds.
export TMPDIR=/tmp
O=${O:-gpurun_out/r3_mproc_trace}
mkdir -p $O/out
pids=()
for r in 0 1; do
  RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 GP_BENCH_DEVICE=0 \
  NCCL_HOSTID=gp-rehearsal-$r NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1 \
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rank$r -o kt -- \
    python3 tests/helpers/rccl_worker.py $O/out ${NODES:-1000000000} Imp3D push-sum 1 ${ROUNDS:-100} > $O/rank$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { tail -30 $O/rank0.log $O/rank1.log; exit $rc; }
for r in 0 1; do echo "rank $r:"; f=$(find $O/rank$r -name '*kernel_stats.csv' | head -1); head -12 "$f" | cut -d, -f1-5; done
