#!/usr/bin/env bash
# LDS-side counters of the render kernels (run on the GPU box from the repo root): LDS busy cycles
# (SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / XCDs x CUs) = LDS utilisation), bank conflicts, issue
# stalls on LDS, bytes loaded.  Output: gpurun_out/<tag>_lds/.
set -euo pipefail
tag=${1:-rNN}
root=$(pwd)
export TMPDIR=/tmp
out=$root/gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS_LOAD_BANDWIDTH \
    SQ_LDS_DATA_FIFO_FULL SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --kernel-include-regex 'k_render' --output-format csv -d "$out/${tag}_lds" -o pmc -- \
    python3 "$root/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$out/${tag}_lds.log" 2>&1
