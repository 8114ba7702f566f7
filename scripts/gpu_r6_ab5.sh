# window-prefetch confirmation: A/B (win1 first) then the product build's parity tests.
set -o pipefail
export TMPDIR=/tmp
C5V="win1 cur" C4V="" REPS=4 O=gpurun_out/r6_ab9 bash scripts/gpu_r6_ab3.sh || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_baseline_sizes.py::test_run_to_convergence_matches_oracle_record" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_ab9/tests.log 2>&1 || { tail -30 gpurun_out/r6_ab9/tests.log; exit 1; }
tail -2 gpurun_out/r6_ab9/tests.log
