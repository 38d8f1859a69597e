set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/st_pg -o t -- python3 tools/step_trace.py pgraph > gpurun_out/stpg.log 2>&1
python3 tools/step_trace.py --timeline gpurun_out/st_pg/t_kernel_trace.csv > gpurun_out/st_pg.txt
