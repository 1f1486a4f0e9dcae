# usage: bash tools/gpu_c2stall.sh TAG — the default bench.py twice with PICARD_TRACE=1 (the
# Solver's setup phases per config), to locate the intermittent C2 setup stall
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  PICARD_TRACE=1 timeout -k 10 600 python -u bench.py > gpurun_out/stall_$TAG.$i.json 2> gpurun_out/stall_$TAG.$i.err || { tail -20 gpurun_out/stall_$TAG.$i.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print('value', d['value'], {k:round(v['setup_s'],3) for k,v in d['other_configs'].items()})" gpurun_out/stall_$TAG.$i.json
  grep "setup ms" gpurun_out/stall_$TAG.$i.err
done
