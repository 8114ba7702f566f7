#!/bin/bash
# Round 4: the multi-GPU launchers rehearsed on one GPU, the 16-rank exchange, Imp3D gossip counts
# across ranks (column kernel), the 1e9 alert-phase parity.
set -o pipefail
O=gpurun_out/r4_launch
mkdir -p $O
# does loading libgossip_hip.so (no HIP call) open the GPU?  (the CLI launcher forks after loading it)
timeout -k 10 60 python3 -c "
import ctypes, os
ctypes.CDLL('gossipprotocol_amd/libgossip_hip.so')
fds = []
for f in os.listdir('/proc/self/fd'):
    try:
        fds.append(os.readlink('/proc/self/fd/' + f))
    except OSError:
        pass
print('fds after load:', [f for f in fds if 'kfd' in f or 'dri' in f])
" > $O/kfd_on_load.txt 2>&1; cat $O/kfd_on_load.txt
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread --durations=30 \
  tests/test_gpu_launcher.py tests/test_gpu_multirank.py::test_virtual_ranks_max_world \
  "tests/test_gpu_multirank.py::test_virtual_ranks_parity" -k "col or max_world or launcher or rccl_processes or full_size_1e9" \
  "tests/test_gpu_rccl_multiproc.py::test_rccl_processes_match_single" \
  "tests/test_gpu_parity.py" > $O/pytest.log 2>&1
rc=$?; tail -45 $O/pytest.log; exit $rc
