#!/usr/bin/env bash
# Issue/wait counters of the kernels matching a regex over a short bench (run on the GPU box from
# the repo root): tools/pmc_kernel.sh <tag> <kernel regex>  ->  gpurun_out/<tag>_pmc/
set -euo pipefail
tag=${1:-k}
re=${2:-k_depth_bucket_sort}
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE \
    --kernel-include-regex "$re" --output-format csv -d "$(pwd)/gpurun_out/${tag}_pmc" -o pmc -- \
    python3 "$(pwd)/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "gpurun_out/${tag}_pmc.log" 2>&1
