set -e
tools/gpu_tests.sh r04_t12.log tests/test_gpu_forward_only.py tests/test_gpu_captured_forms.py tests/test_gpu_parity.py tests/test_gpu_timed_step.py tests/test_gpu_graph.py tests/test_gpu_dist_step.py
for m in "" --nowait "" --nowait; do timeout -k 10 200 python3 tools/pg_host.py --steps 300 $m > gpurun_out/pgh.log 2>&1; echo "mode=$m $(grep 'rep 2' gpurun_out/pgh.log)" >> gpurun_out/pgh_wait.txt; done
timeout -k 10 300 python3 bench.py --json-out gpurun_out/r04_bench5.json > gpurun_out/r04_bench5.log 2>&1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gap -o t -- python3 tools/graph_gap_probe.py > gpurun_out/gap.log 2>&1
python3 tools/graph_gap_probe.py --report gpurun_out/gap/t_kernel_trace.csv > gpurun_out/gap_report.txt
for r in 2 3 4; do LSR_PG_ROT=$r timeout -k 10 200 python3 tools/pg_host.py --steps 300 --nowait > gpurun_out/pgh.log 2>&1; echo "rot=$r $(grep 'rep 2' gpurun_out/pgh.log)" >> gpurun_out/pgh_wait.txt; done
timeout -k 10 400 python3 bench.py --config C5 --steps 20 --warmup 5 --no-cpu-baseline --json-out gpurun_out/r04_bench_C5.json > gpurun_out/r04_bench_C5.log 2>&1
LSR_PG_ROT=4 timeout -k 10 300 python3 bench.py --no-cpu-baseline --json-out gpurun_out/r04_bench_rot4.json > gpurun_out/r04_bench_rot4.log 2>&1
