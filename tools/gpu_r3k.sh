# usage: bash tools/gpu_r3k.sh TAG — whole -m gpu suite, per-call overhead at N = 64, C2 three times
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 120 python3 tools/bench_overhead.py 200 64 65536 | tee gpurun_out/overhead_$TAG.txt || exit 1
for i in 1 2 3; do
  timeout -k 10 120 python3 tools/run_configs.py C2 > gpurun_out/c2_$TAG.$i.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('C2', d['iterations_s'], d['samples_per_s_per_iter'])" gpurun_out/c2_$TAG.$i.json
done | tee gpurun_out/c2_$TAG.txt
