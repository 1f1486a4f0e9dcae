# usage: bash tools/gpu_g8ab.sh TAG — the full-size tests with the digit G stage, then the C3 bench
# (driver window) with and without it, on one box
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PICARD_G8=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_fullsize_fit.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/full_$TAG.log 2>&1 || { tail -40 gpurun_out/full_$TAG.log; exit 1; }
tail -2 gpurun_out/full_$TAG.log
for g in 1 0; do
  PICARD_G8=$g timeout -k 10 400 python -u bench.py --warmup 5 --steps 20 --configs 0 --cpu-baseline 0 \
    > gpurun_out/bench_${TAG}_g$g.json 2> gpurun_out/bench_${TAG}_g$g.err || { tail -20 gpurun_out/bench_${TAG}_g$g.err; exit 1; }
  echo "== PICARD_G8=$g"; python3 tools/bench_summary.py gpurun_out/bench_${TAG}_g$g.json | head -4
done
