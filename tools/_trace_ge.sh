set -e
export TMPDIR=/tmp
for m in graph eager; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tge_$m -o t -- python3 tools/step_trace.py $m > gpurun_out/tge_$m.log 2>&1
done
python3 tools/step_trace.py --compare gpurun_out/tge_eager/t_kernel_trace.csv gpurun_out/tge_graph/t_kernel_trace.csv > gpurun_out/tge_compare.txt
python3 tools/step_trace.py --timeline gpurun_out/tge_graph/t_kernel_trace.csv > gpurun_out/tge_graph_timeline.txt
python3 tools/step_trace.py --timeline gpurun_out/tge_eager/t_kernel_trace.csv > gpurun_out/tge_eager_timeline.txt
