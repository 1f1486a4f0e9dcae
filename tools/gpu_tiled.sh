# usage: bash tools/gpu_tiled.sh TAG — gpu tests then the tiled-path timings at C4's shape
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tiled_$TAG -o run --output-format csv -- python tools/bench_tiled.py 256 1e7 2 > gpurun_out/tiled_$TAG.log 2>&1 || { tail gpurun_out/tiled_$TAG.log; exit 1; }
grep N= gpurun_out/tiled_$TAG.log
python3 - <<PY
import csv
for r in csv.DictReader(open('gpurun_out/prof_tiled_$TAG/run_kernel_stats.csv')):
    print(r['Name'][:50], r['Calls'], '%.2f ms avg' % (float(r['AverageNs'])/1e6))
PY
