# usage: bash tools/gpu_r3.sh TAG — round-3 GPU check: new tests verbose, full -m gpu suite,
# traced C3 bench (line-search screens) — each step time-limited, logs in gpurun_out/
set -o pipefail
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_screen32.py tests/test_gpu_group.py -m gpu -x -v -s --timeout 240 \
  --timeout-method thread > gpurun_out/pytest_new_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_new_$TAG.log; exit 1; }
grep -E "v_exp_f32|PASS|FAIL" gpurun_out/pytest_new_$TAG.log | head -40
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=5 \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -8 gpurun_out/pytest_gpu_$TAG.log
PICARD_TRACE=1 timeout -k 10 300 python -u bench.py --configs 0 --cpu-baseline 0 > gpurun_out/bench_trace_$TAG.json \
  2> gpurun_out/bench_trace_$TAG.err || { tail -20 gpurun_out/bench_trace_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_trace_$TAG.json'));print(d['value'],d['ms_per_step'],d['kernels_per_step'])"
