#!/bin/bash
# rocprofv3 session on the bench workload: kernel-trace stats, then one
# counter set per pass (gfx950 does not multiplex; limits per block in
# MI355X_MICROARCH.md).  Each pass under its own kill timer; stops at the
# first failure.
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python bench.py --steps 2 --warmup 1 --no-cpu"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $B > gpurun_out/prof.log 2>&1 || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SMEM" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" \
    "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc$i -o run --output-format csv -- $B > gpurun_out/pmc$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 gpurun_out/pmc$i.log; exit 1; }
done
python tools/pmc_table.py gpurun_out/pmc_table.json gpurun_out/pmc1 gpurun_out/pmc2 gpurun_out/pmc3 gpurun_out/pmc4 \
  gpurun_out/pmc5 > /dev/null
