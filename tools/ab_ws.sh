# usage: bash tools/ab_ws.sh — fused pass A/B: warp-specialised (default) vs 8-wave k_eval_fused<8>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2; do
  echo "== ws"; timeout -k 10 120 python tools/bench_split.py 128 5e7 5 tanh 0.3 || exit 1
  echo "== 8-wave"; PICARD_FUSED_WS=0 timeout -k 10 120 python tools/bench_split.py 128 5e7 5 tanh 0.3 || exit 1
done
