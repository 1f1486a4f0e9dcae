cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PICARD_TRACE=1 timeout -k 10 300 python -u bench.py --t 1.25e7 --configs 0 --cpu-baseline 0 > gpurun_out/pred_proxy.json 2> gpurun_out/pred_proxy.err && \
PICARD_TRACE=1 timeout -k 10 400 python -u bench.py --configs 0 --cpu-baseline 0 > gpurun_out/pred_c3.json 2> gpurun_out/pred_c3.err && \
PICARD_TRACE=1 timeout -k 10 300 python -u tools/run_configs.py C2 > gpurun_out/pred_c2.json 2> gpurun_out/pred_c2.err
