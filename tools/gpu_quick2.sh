# usage: bash tools/gpu_quick2.sh TAG — gpu tests, C3 bench line (no CPU baseline), C2 end to end
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_$TAG.json'))
print('C3 value %.4g ms/step %.1f passes/iter %.2f in-eval %.1f' % (d['value'], d['ms_per_step'], d['passes_per_iter'], d['ms_in_eval_calls_per_step']))
print({k: (round(v['avg_ms'],2) if v['avg_ms'] else None, v['launches']) for k,v in d['kernels_per_step'].items()})"
timeout -k 10 100 python tools/run_configs.py C2 > gpurun_out/c2_$TAG.json || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/c2_$TAG.json'))
print('C2 iters_s %.3f n_it %d passes %d sps/iter %.4g' % (d['iterations_s'], d['n_iterations'], d['passes'], d['samples_per_s_per_iter']), {k:(round(v[0],1),v[1]) for k,v in d['kernels'].items()})"
