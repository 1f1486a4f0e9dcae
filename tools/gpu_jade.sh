# usage: bash tools/gpu_jade.sh TAG — JADE GPU tests, then C5 (host vs device sweeps) with PICARD_TRACE timings
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/jade_$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_jade.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
PICARD_HOST_JADE=1 PICARD_TRACE=1 timeout -k 10 200 python tools/run_configs.py C5 --max-iter=2 > $O/c5_host.json 2> $O/c5_host.err || { tail -20 $O/c5_host.err; exit 1; }
grep "jade:" $O/c5_host.err
PICARD_TRACE=1 timeout -k 10 200 python tools/run_configs.py C5 --max-iter=2 > $O/c5_dev.json 2> $O/c5_dev.err || { tail -20 $O/c5_dev.err; exit 1; }
grep "jade:" $O/c5_dev.err
