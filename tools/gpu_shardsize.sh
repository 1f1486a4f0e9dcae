# usage: bash tools/gpu_shardsize.sh TAG — fused-pass kernel time against the shard size at N = 128
# (fixed per-launch cost), then the one-rank-of-8 proxy bench (bench.py --t 1.25e7) with the trace
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in 1.25e7 2.5e7 5e7 1e8; do
  timeout -k 10 120 python3 tools/bench_pass.py 128 $t tanh 10 || exit 1
done 2>&1 | tee gpurun_out/shardsize_$TAG.txt
PICARD_TRACE=1 timeout -k 10 300 python -u bench.py --t 1.25e7 > gpurun_out/proxy_$TAG.json 2> gpurun_out/proxy_trace_$TAG.log || { tail -20 gpurun_out/proxy_trace_$TAG.log; exit 1; }
python3 tools/bench_summary.py gpurun_out/proxy_$TAG.json
