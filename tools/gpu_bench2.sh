# usage: bash tools/gpu_bench2.sh TAG — the default bench.py twice (box-to-box / run-to-run check)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.$i.json 2> gpurun_out/bench_$TAG.$i.err || { tail -20 gpurun_out/bench_$TAG.$i.err; exit 1; }
  python3 tools/bench_summary.py gpurun_out/bench_$TAG.$i.json | grep -E "value|whole|C2|C5 "
done
