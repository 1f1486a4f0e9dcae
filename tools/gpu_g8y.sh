# usage: bash tools/gpu_g8y.sh TAG — k_eval_fused_g8y (PICARD_G8Y=1) against k_eval_fused_g8x: the
# digit-G tests under the variant, then the fused pass at (128, 2e7) both ways
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PICARD_G8Y=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_g8.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/g8y_$TAG.log 2>&1; rc=$?
tail -5 gpurun_out/g8y_$TAG.log
[ $rc -eq 0 ] || exit 1
for v in "PICARD_G8Y=1" "PICARD_G8Y=0" "PICARD_G8Y=1"; do
  echo "== $v"; env $v timeout -k 10 120 python -u tools/bench_pass.py 128 2e7 tanh 5 || exit 1
done
