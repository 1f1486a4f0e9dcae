# usage: bash tools/gpu_g8var.sh TAG — the digit-G, int8 and parity tests, the full-size tests,
# then the fused pass at (128, 2e7) with the G stage on digits and on fp64 MFMA
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_g8.py tests/test_gpu_int8.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/g8x_$TAG.log 2>&1; rc=$?
tail -6 gpurun_out/g8x_$TAG.log
[ $rc -le 1 ] || exit 1
for v in "PICARD_G8=1" "PICARD_G8=0"; do
  echo "== $v"; env $v timeout -k 10 120 python -u tools/bench_pass.py 128 2e7 tanh 5 || exit 1
done
