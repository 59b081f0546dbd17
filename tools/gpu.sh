#!/bin/bash
# One GPU-box session, parametrised: each argument is a step, run in order
# under its own time limit; the session stops at the first step that ends in
# anything but success (or a plain test failure, rc 1, for test steps).
#
#   bash tools/gpu.sh tests bench:128 bench:203 sp:128 prof:128 ...
#
# steps (name[:arg[:arg]]):
#   tests              every -m gpu test (stop at the first failure)
#   test:<path>        one test file / node id
#   smoke              __graft_entry__.smoke()
#   bench[:G[:lib]]    bench.py --no-cpu at G marks (default 128), 10 timed passes;
#                      lib: an in-tree variant (TNP_LIB)
#   benchfull          the default bench line (CPU baseline and legs included)
#   sp[:G[:lib]]       tools/step_profile.py G 6 (per-step kernel times)
#   small[:lib]        tools/small_profile.py (bunny-scale latency)
#   finish[:lib]       tools/finish_profile.py
#   prof[:G]           rocprofv3 --kernel-trace --stats of a short bench
#   proffinish         rocprofv3 --kernel-trace --stats of tools/finish64.py
#   pmc:<counters>     one rocprofv3 --pmc pass (counters comma-separated) of a short bench
#   pmcsession         tools/pmc_session.sh (kernel trace + the four counter passes -> pmc_table.json)
#   rehearsal[:N]      bench at 161^3 on one rank, then N (default 2) gloo ranks sharing the GPU
#   ranks[:N]          only the N gloo ranks sharing the GPU (rc 1 does not stop the session)
#   diag:<cases>       tools/descend_diag.py on descend fixtures (comma-separated)
#   env:<VAR=val>      export a variable for the following steps
# Logs: gpurun_out/<tag>_<n>_<step>.log, summary gpurun_out/<tag>_session.log
# (tag = $TNP_TAG, default "s").
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${TNP_TAG:-s}
sess=gpurun_out/${tag}_session.log
: > "$sess"
n=0
run() {  # limit okrc cmd...
  local t=$1 ok=$2; shift 2
  n=$((n + 1))
  local log="gpurun_out/${tag}_${n}_${name//[:\/=]/_}.log"
  echo "== $n $step" >> "$sess"
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  echo "== $n $step rc=$rc" >> "$sess"
  if [ $rc -ne 0 ] && ! { [ "$ok" = 1 ] && [ $rc -eq 1 ]; }; then
    echo "stopping after $step rc=$rc" >> "$sess"
    tail -30 "$log"
    cat "$sess"
    exit $rc
  fi
  return 0
}
lib() { if [ -n "${1:-}" ]; then echo "TNP_LIB=$1"; else echo "TNP_LIB=libtropical_hip.so"; fi; }
for step in "$@"; do
  IFS=: read -r name a1 a2 <<< "$step"
  case "$name" in
    tests) run 900 1 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    test) run 400 1 python -u -m pytest "$a1" -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    smoke) run 300 0 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 400 0 env "$(lib "$a2")" python -u bench.py --marks "${a1:-128}" --steps 10 --warmup 3 --no-cpu ;;
    benchfull) run 900 0 python -u bench.py ;;
    sp) run 300 0 env "$(lib "$a2")" python -u tools/step_profile.py "${a1:-128}" 6 ;;
    small) run 300 0 env "$(lib "$a1")" python -u tools/small_profile.py ;;
    finish) run 300 0 env "$(lib "$a1")" python -u tools/finish_profile.py ;;
    proffinish) run 600 0 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_proffinish" -o run --output-format csv \
            -- python tools/finish64.py ;;
    prof) run 600 0 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof${a1:-128}" -o run --output-format csv \
            -- python bench.py --marks "${a1:-128}" --steps 2 --warmup 1 --no-cpu ;;
    pmc) run 120 0 rocprofv3 --pmc ${a1//,/ } -d "gpurun_out/${tag}_pmc_${a1//,/_}" -o run --output-format csv \
            -- python bench.py --marks "${a2:-128}" --steps 1 --warmup 1 --no-cpu ;;
    pmcsession) run 900 0 bash tools/pmc_session.sh ;;
    rehearsal) run 300 0 python -u bench.py --marks 161 --steps 2 --warmup 1 --no-cpu &&
               run 400 0 env TNP_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
                 --nproc-per-node "${a1:-2}" --master-addr 127.0.0.1 --master-port 29517 bench.py \
                 --gpus "${a1:-2}" --steps 2 --warmup 1 --no-cpu ;;
    ranks) run 400 1 env TNP_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
             --nproc-per-node "${a1:-2}" --master-addr 127.0.0.1 --master-port 29518 bench.py \
             --gpus "${a1:-2}" --steps 2 --warmup 1 --no-cpu ;;
    diag) run 240 0 python -u tools/descend_diag.py ${a1//,/ } ;;
    env) export "$a1"; echo "== env $a1" >> "$sess" ;;
    *) echo "unknown step $step" >> "$sess"; exit 2 ;;
  esac
done
cat "$sess"
