#!/usr/bin/env bash
# Issue-side counters of the render kernels (run on the GPU box from the repo root): one PMC pass
# of 8 SQ counters + GRBM_GUI_ACTIVE over a short bench.  Output: gpurun_out/<tag>_sq/.
set -euo pipefail
tag=${1:-rNN}
root=$(pwd)
export TMPDIR=/tmp
out=$root/gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
    --kernel-include-regex 'k_render|k_preprocess' --output-format csv -d "$out/${tag}_sq" -o pmc -- \
    python3 "$root/bench.py" --steps 3 --warmup 2 --no-cpu-baseline > "$out/${tag}_sq.log" 2>&1
