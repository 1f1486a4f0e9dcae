# usage: bash tools/ab_loss2.sh — loss-only pass A/B: k_eval_loss2 (default) vs k_eval_loss<8>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PICARD_NO_YSTORE=1
for r in 1 2; do
  echo "== loss2"; timeout -k 10 120 python tools/bench_split.py 128 5e7 5 tanh 0.3 || exit 1
  echo "== loss<8>"; PICARD_LOSS2=0 timeout -k 10 120 python tools/bench_split.py 128 5e7 5 tanh 0.3 || exit 1
done
