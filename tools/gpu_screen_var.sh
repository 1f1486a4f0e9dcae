# usage: bash tools/gpu_screen_var.sh TAG — the screen kernels at (128, 2e7) and (64, 1e7): k_screen_oz2
# with PICARD_SCREEN2_FILL 2 (default) / 1 / 0 and k_screen_oz (PICARD_SCREEN_V2=0), then the screen /
# int8 tests on the default
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/svar_$TAG
mkdir -p $O
run() {  # name, env...
  local nm=$1; shift
  env "$@" timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 auto > $O/$nm.txt 2>&1 || { cat $O/$nm.txt; return 1; }
  env "$@" timeout -k 10 120 python3 tools/bench_loss.py 64 1e7 5 auto >> $O/$nm.txt 2>&1 || { cat $O/$nm.txt; return 1; }
  echo "$nm: $(grep screen $O/$nm.txt | sed 's/auto  //' | tr '\n' ' ')"
}
run oz2_fill2 PICARD_SCREEN2_FILL=2 && run oz2_fill1 PICARD_SCREEN2_FILL=1 && run oz2_fill0 PICARD_SCREEN2_FILL=0 && \
  run oz PICARD_SCREEN_V2=0 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_screen32.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
