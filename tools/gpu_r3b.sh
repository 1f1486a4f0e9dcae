# usage: bash tools/gpu_r3b.sh TAG — screen tests + int8 tests, then traced C3 bench (default screen)
# and the same with PICARD_SCREEN_DMAX=4; each step time-limited, logs in gpurun_out/
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_screen32.py tests/test_gpu_int8.py tests/test_gpu_group.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > gpurun_out/pytest_scr_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_scr_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_scr_$TAG.log
for D in 3 4; do
  PICARD_SCREEN_DMAX=$D PICARD_TRACE=1 timeout -k 10 300 python -u bench.py --configs 0 --cpu-baseline 0 \
    > gpurun_out/bench_d${D}_$TAG.json 2> gpurun_out/bench_d${D}_$TAG.err || { tail -20 gpurun_out/bench_d${D}_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_d${D}_$TAG.json'));k=d['kernels_per_step'];print('D<=$D', d['value'],d['ms_per_step'],d['whole_fit']['samples_per_s_per_iter'],k['fused']['avg_ms'],k['screen']['avg_ms'],k['screen']['launches'])"
  grep -c reject gpurun_out/bench_d${D}_$TAG.err; grep picard-screen gpurun_out/bench_d${D}_$TAG.err | grep -c exact
done
