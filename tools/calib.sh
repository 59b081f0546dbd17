#!/bin/bash
# FETCH_SIZE calibration of gather widths (tools/gather_calib.hip)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o gpurun_out/gather_calib tools/gather_calib.hip || exit 1
timeout -k 10 60 gpurun_out/gather_calib > gpurun_out/calib_time.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib1 -o run --output-format csv -- gpurun_out/gather_calib > gpurun_out/calib1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d gpurun_out/calib2 -o run --output-format csv -- gpurun_out/gather_calib > gpurun_out/calib2.log 2>&1
exit 0
