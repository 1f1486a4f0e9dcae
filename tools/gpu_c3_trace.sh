# usage: bash tools/gpu_c3_trace.sh TAG — the default C3 bench (no CPU baseline, no other configs)
# with PICARD_TRACE=1: per-iteration policy cells, screens, model full passes, curvature skips
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PICARD_TRACE=1 timeout -k 10 400 python -u bench.py --configs 0 --cpu-baseline 0 > gpurun_out/c3trace_$1.json 2> gpurun_out/c3trace_$1.err || { tail -20 gpurun_out/c3trace_$1.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/c3trace_$1.json | head -4
