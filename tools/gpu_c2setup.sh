# usage: bash tools/gpu_c2setup.sh TAG — C2's setup time after the C3 context is released, with and
# without the CPU-baseline leg before it (bench.py --steps 2)
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cb in 0 1 0 1; do
  timeout -k 10 400 python -u bench.py --steps 2 --cpu-baseline $cb > gpurun_out/c2s_$TAG.$cb.json 2> gpurun_out/c2s_$TAG.$cb.err || { tail -20 gpurun_out/c2s_$TAG.$cb.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print('cpu_baseline', sys.argv[2], 'gen', round(d['timings_s']['generate'],2), {k:round(v['setup_s'],3) for k,v in d['other_configs'].items()})" gpurun_out/c2s_$TAG.$cb.json $cb
done
