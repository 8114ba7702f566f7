#!/bin/bash
# HBM-byte calibration of the tile kernel's access shapes (tools/calib.hip) with the
# request-size counter passes of tools/hbm_traffic.py; run via gpurun.
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
timeout -k 10 120 ./build/calib > gpurun_out/calib/calib.log 2>&1 || { cat gpurun_out/calib/calib.log; exit 1; }
cat gpurun_out/calib/calib.log
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/calib/rdA -o rdA -- ./build/calib > gpurun_out/calib/rdA.log 2>&1 || { tail gpurun_out/calib/rdA.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d gpurun_out/calib/rdB -o rdB -- ./build/calib > gpurun_out/calib/rdB.log 2>&1 || { tail gpurun_out/calib/rdB.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/wr -o wr -- ./build/calib > gpurun_out/calib/wr.log 2>&1 || { tail gpurun_out/calib/wr.log; exit 1; }
python3 tools/calib_summary.py gpurun_out/calib/calib.log gpurun_out/calib gpurun_out/calib/calib.json
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RD_UNCACHED_32B_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d gpurun_out/calib/rdU -o rdU -- ./build/calib > gpurun_out/calib/rdU.log 2>&1 || { tail gpurun_out/calib/rdU.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d gpurun_out/calib/wrq -o wrq -- ./build/calib > gpurun_out/calib/wrq.log 2>&1 || { tail gpurun_out/calib/wrq.log; exit 1; }
python3 tools/calib_summary.py gpurun_out/calib/calib.log gpurun_out/calib gpurun_out/calib/calib.json > /dev/null
