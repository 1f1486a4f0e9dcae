# usage: bash tools/gpu_c4stage.sh TAG [GROUPS…] — C4 end to end with PICARD_TRACE=1 (which try each
# search accepted) for the one-pass multi-try schedule, then with the first pass capped at each
# given group size (PICARD_MULTI_GROUP)
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for g in 0 "$@"; do
  PICARD_MULTI_GROUP=$g PICARD_TRACE=1 timeout -k 10 300 python -u tools/run_configs.py C4 \
    > gpurun_out/c4s_${TAG}_g$g.json 2> gpurun_out/c4s_${TAG}_g$g.err || { tail -20 gpurun_out/c4s_${TAG}_g$g.err; exit 1; }
  echo "== group $g"; cut -c1-400 gpurun_out/c4s_${TAG}_g$g.json
done
