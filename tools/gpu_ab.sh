# usage: bash tools/gpu_ab.sh TAG ROUNDS "ENV=V ..." "ENV=V ..." ... — alternating A/B of the fused
# pass (tools/bench_pass.py 128 2e7) and the line-search screen (tools/screen_time.py) under each
# environment setting, ROUNDS times; log in gpurun_out/ab_TAG.log
TAG=$1; ROUNDS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/ab_$TAG.log
: > $O
for r in $(seq 1 $ROUNDS); do
  for cfg in "$@"; do
    echo "[ab] round $r: $cfg" | tee -a $O
    timeout -k 10 120 env $cfg python3 -u tools/bench_pass.py 128 2e7 tanh 10 >> $O 2>&1 || { echo "[ab] fused failed: $cfg"; tail -20 $O; exit 1; }
    timeout -k 10 120 env $cfg python3 -u tools/screen_time.py 10 >> $O 2>&1 || { echo "[ab] screen failed: $cfg"; tail -20 $O; exit 1; }
  done
done
grep -E "^\[ab\]|kernel|screen" $O
