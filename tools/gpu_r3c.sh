# usage: bash tools/gpu_r3c.sh TAG — full -m gpu suite, then the default bench (C3 + other configs + CPU baselines)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=8 \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -12 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json 2>/dev/null || head -c 1500 gpurun_out/bench_$TAG.json
timeout -k 10 120 python3 tools/bench_overhead.py 200 64 65536 || exit 1
OMP_NUM_THREADS=1 timeout -k 10 120 python3 tools/bench_overhead.py 200 64 65536 || exit 1
