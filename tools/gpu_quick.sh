# usage: bash tools/gpu_quick.sh TAG — gpu tests then a bench line without the CPU baseline
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('value %.4g ms/step %.1f passes/iter %.2f' % (d['value'], d['ms_per_step'], d['passes_per_iter']))
print({k: (round(v['avg_ms'],2) if v['avg_ms'] else None, v['launches']) for k,v in d['kernels_per_step'].items()})
print('roof', d['roofline']['achieved'], d['roofline']['frac'])"
