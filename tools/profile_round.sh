#!/usr/bin/env bash
# Profiling recipe for the bench workload of one config (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes (they do not fit
#   one pass on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots"), then the SQ issue counters, and
#   the summaries bench.py reads (gpurun_out/<tag>_<cfg>_{summary,valu}.json: copy them into profiles/).
#     tools/profile_round.sh r03 C3
set -euo pipefail
tag=${1:-rNN}
cfg=${2:-C3}
root=$(pwd)
export TMPDIR=/tmp
export LSR_BENCH_RGB=0  # the RGB step is reported beside the bench line, not profiled here
export LSR_PIPELINE=0   # serial forms only: overlapped kernels would stretch the per-kernel averages
out=$root/gpurun_out
b="$root/bench.py --config $cfg --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${tag}_${cfg}_trace" -o trace -- \
    python3 $b --steps 20 --warmup 5 > "$out/${tag}_${cfg}_trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/${tag}_${cfg}_fetch" -o pmc -- \
    python3 $b --steps 3 --warmup 2 > "$out/${tag}_${cfg}_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/${tag}_${cfg}_write" -o pmc -- \
    python3 $b --steps 3 --warmup 2 > "$out/${tag}_${cfg}_write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE \
    --kernel-include-regex 'k_render|k_preprocess' --output-format csv -d "$out/${tag}_${cfg}_sq" -o pmc -- \
    python3 $b --steps 3 --warmup 2 > "$out/${tag}_${cfg}_sq.log" 2>&1
python3 tools/prof_summary.py --trace "$out/${tag}_${cfg}_trace/trace_kernel_trace.csv" \
    --fetch "$out/${tag}_${cfg}_fetch/pmc_counter_collection.csv" \
    --write "$out/${tag}_${cfg}_write/pmc_counter_collection.csv" --out "$out/${tag}_${cfg}_summary.json"
python3 tools/valu_summary.py --sq "$out/${tag}_${cfg}_sq/pmc_counter_collection.csv" \
    --out "$out/${tag}_${cfg}_valu.json"
cp "$out/${tag}_${cfg}_trace/trace_kernel_stats.csv" "$out/${tag}_${cfg}_kernel_stats.csv"
