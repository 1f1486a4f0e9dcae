# usage: bash tools/gpu_pair_fill.sh TAG — single and paired screen times at (128, 2e7) for the
# PICARD_SCREEN2_FILL variants 1 / 2 / 0, alternating twice on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/pairfill_$1.txt
: > $O
for rep in 1 2; do
  for f in 1 2 0; do
    echo "== FILL=$f rep $rep" >> $O
    PICARD_SCREEN2_FILL=$f timeout -k 10 120 python -u tools/bench_loss.py 128 2e7 5 auto >> $O 2>&1 || exit 1
  done
done
grep -E "^==|screen" $O
