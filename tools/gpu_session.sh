#!/bin/bash
# One GPU-box session: parity tests, then a short bench.  Stops at the first
# step that ends in anything but success/test-failure (fault, abort, timeout).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" >> gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc" >> gpurun_out/session.log; exit $rc; fi
  return 0
}
: > gpurun_out/session.log
for step in "$@"; do
  case "$step" in
    tests) run gpu_tests 800 python -m pytest tests -q -m gpu --timeout 300 -p no:cacheprovider ;;
    bench) run bench 900 python bench.py --steps 3 --warmup 1 ;;
    benchfast) run bench 600 python bench.py --steps 3 --warmup 1 --no-cpu ;;
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    curve) run gpu_curve 600 python -u -m pytest tests/test_gpu_curve.py -x -v --timeout 300 -p no:cacheprovider ;;
    stats) run step_stats 300 python tools/step_stats.py 128 6 ;;
    pmcf) run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu ;;
    pmcw) run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu ;;
  esac
done
