# usage: bash tools/gpu_profset.sh TAG — the round's measurement set in one call:
#   1. the one-rank-of-8 proxy (bench.py --t 1.25e7) traced: host ms per iteration summary
#   2. the C3 bench traced (policy cells, screens, curvature skips, [picard-host] phases)
#   3. tools/prof_c3.sh: --kernel-trace --stats of the default C3 bench, FETCH_SIZE, WRITE_SIZE
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PICARD_TRACE=1 timeout -k 10 300 python -u bench.py --t 1.25e7 --configs 0 --cpu-baseline 0 > gpurun_out/proxy_$TAG.json 2> gpurun_out/proxy_$TAG.err || { tail -20 gpurun_out/proxy_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/proxy_$TAG.json | head -4
grep "picard-trace\] iter" gpurun_out/proxy_$TAG.err | sed -E 's/.*host_ms ([0-9.]+).*/\1/' \
  | sort -n | awk '{h[NR]=$1; s+=$1} END {printf "proxy host ms per iteration: n %d mean %.3f median %.3f p90 %.3f max %.3f\n", NR, s/NR, h[int(NR/2)+1], h[int(NR*0.9)], h[NR]}'
PICARD_TRACE=1 timeout -k 10 400 python -u bench.py --configs 0 --cpu-baseline 0 > gpurun_out/c3trace_$TAG.json 2> gpurun_out/c3trace_$TAG.err || { tail -20 gpurun_out/c3trace_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/c3trace_$TAG.json | head -4
bash tools/prof_c3.sh $TAG
