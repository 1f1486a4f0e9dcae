# usage: bash tools/exp_policy.sh — bench the line-search evaluation schedules + split kernel timings
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 100 python tools/bench_split.py 128 1e8 3 || exit 1
for v in "PICARD_NONE=1" "PICARD_KEEP_Y=1" "PICARD_SPLIT_FIRST=1" "PICARD_KEEP_Y=1 PICARD_SPLIT_FIRST=1"; do
  env $v timeout -k 10 300 python bench.py --cpu-baseline 0 --to-tol 1 > gpurun_out/bench_pol.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_pol.json'))
print('$v', 'value %.4g'%d['value'], 'ms/step %.1f'%d['ms_per_step'], 'iters', d['iters_to_tol'], 'to_tol_s %.2f'%d['timings_s']['to_tol_untimed'], {k:(round(v['ms'],1),v['launches']) for k,v in d['kernels_per_step'].items()})"
done
