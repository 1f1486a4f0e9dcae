# usage: bash tools/gpu_configs.sh TAG [configs...] — BASELINE configs end to end (default C2 C4 C5)
TAG=$1; shift
CFGS=${@:-C2 C4 C5}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in $CFGS; do
  timeout -k 10 240 python tools/run_configs.py $c >> gpurun_out/configs_$TAG.jsonl 2> gpurun_out/configs_${TAG}_$c.err || { echo "$c failed/timeout"; tail -5 gpurun_out/configs_${TAG}_$c.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/configs_$TAG.jsonl').read().strip().split('\n')[-1])
print(d['config'], 'setup %.2f iters_s %.2f n_it %d passes %d conv %s amari %.2e sps/iter %.3g'%(d['setup_s'],d['iterations_s'],d['n_iterations'],d['passes'],d['converged'],d['amari'],d['samples_per_s_per_iter']), {k:(round(v[0],1),v[1]) for k,v in d['kernels'].items()})"
done
