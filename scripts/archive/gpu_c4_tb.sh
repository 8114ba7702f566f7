export TMPDIR=/tmp
for v in tb11 tb11f tb12f; do GOSSIP_HIP_LIB_EXPERIMENT=build/ablate/lib_$v.so timeout -k 10 200 python3 tools/variant_parity.py 200000 full push-sum 400 3 || exit 1; done
O=gpurun_out/c4tb VARIANTS="cur tb11 tb11f tb12f" REPS=2 CFG="100000000 full push-sum 20" bash scripts/gpu_ab2.sh
