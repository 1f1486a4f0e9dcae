# usage: bash tools/gpu_screen_ab.sh TAG — the line-search screen k_screen_oz (PICARD_SCREEN_V2=0)
# against k_screen_oz2 (default): screen kernel time at (128, 2e7) and (64, 1e7), then the
# screen / int8 / group tests; log in gpurun_out/sab_TAG/
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/sab_$TAG
mkdir -p $O
for V in 0 1; do
  PICARD_SCREEN_V2=$V timeout -k 10 120 python3 tools/bench_loss.py 128 2e7 5 auto > $O/v$V.txt 2>&1 || { cat $O/v$V.txt; exit 1; }
  PICARD_SCREEN_V2=$V timeout -k 10 120 python3 tools/bench_loss.py 64 1e7 5 auto >> $O/v$V.txt 2>&1 || { cat $O/v$V.txt; exit 1; }
  echo "== V2=$V"; grep screen $O/v$V.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_int8.py tests/test_gpu_screen32.py tests/test_gpu_group.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
