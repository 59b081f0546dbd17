export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/step_profile.py 128 6 > gpurun_out/dev_sp.log 2>&1 || exit 1
timeout -k 10 200 python tools/small_profile.py > gpurun_out/dev_small.log 2>&1 || exit 1
