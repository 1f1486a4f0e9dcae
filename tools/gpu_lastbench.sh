# usage: bash tools/gpu_lastbench.sh TAG — the default bench.py, then the one-rank-of-8 proxy
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json
PICARD_TRACE=1 timeout -k 10 300 python -u bench.py --t 1.25e7 --configs 0 --cpu-baseline 0 > gpurun_out/proxy_$TAG.json 2> gpurun_out/proxy_$TAG.err || { tail -20 gpurun_out/proxy_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/proxy_$TAG.json | head -4
grep step_ms gpurun_out/proxy_$TAG.err | sed -E 's/.*step_ms ([0-9.]+) eval_ms ([0-9.]+) host_ms ([0-9.]+).*/\3/' \
  | sort -n | awk '{h[NR]=$1; s+=$1} END {printf "proxy host ms per iteration: n %d mean %.3f median %.3f p90 %.3f max %.3f\n", NR, s/NR, h[int(NR/2)+1], h[int(NR*0.9)], h[NR]}'
