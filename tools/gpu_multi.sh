# usage: bash tools/gpu_multi.sh TAG — bounded multi-try tests, int8 multi tests, C4 end to end with the
# bounded multi-try pass and with the exact one (PICARD_MULTI_F64=1)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multi_bound.py tests/test_gpu_int8.py tests/test_gpu_parity.py tests/test_gpu_fullsize_c4.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_multi_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_multi_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_multi_$TAG.log
timeout -k 10 200 python3 tools/run_configs.py C4 > gpurun_out/c4_$TAG.json || exit 1
PICARD_MULTI_F64=1 timeout -k 10 200 python3 tools/run_configs.py C4 > gpurun_out/c4_${TAG}_f64.json || exit 1
python3 - << PY
import json
for f in ("gpurun_out/c4_$TAG.json", "gpurun_out/c4_${TAG}_f64.json"):
    d = json.load(open(f)); print(f, {k: d[k] for k in ("iterations_s", "n_iterations", "samples_per_s_per_iter", "passes", "amari")}, {k: v for k, v in d["kernels"].items() if v[1]})
PY
