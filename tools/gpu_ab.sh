# usage: bash tools/gpu_ab.sh TAG ENVVAR — A/B of a kernel knob: screen / loss / fused timing at
# N=128, T=2e7 with and without ENVVAR=1, then the C3 bench (configs 0, no CPU baseline)
TAG=$1; KNOB=$2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 auto || exit 1
env $KNOB=1 timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 auto || exit 1
timeout -k 10 400 python bench.py --cpu-baseline 0 --configs 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 tools/bench_summary.py gpurun_out/bench_$TAG.json
