# C3 (Imp3D gossip, P = 1.005e8) column kernel A/B, same box, alternated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6_c3ab; mkdir -p $O
for rep in 1 2 3; do
  for v in colbase colp5 colp4; do
    GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so GP_EXP=1 timeout -k 10 240 python3 tools/perf_round.py 100544625 Imp3D gossip 100 > $O/c3_$v.$rep.log 2>&1 || { tail -5 $O/c3_$v.$rep.log; exit 1; }
    echo "c3 $v: $(grep -o 'k_[a-z_+<>A-Z0-9, ]*: [0-9.]* ms/round kernel' $O/c3_$v.$rep.log)"
  done
done
