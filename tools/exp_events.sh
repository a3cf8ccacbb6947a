set -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 300 python bench.py --no-cpu --no-kernel-events > gpurun_out/exp/noev.json 2>gpurun_out/exp/noev.err || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/exp/ev.json 2>gpurun_out/exp/ev.err || exit 1
python -c "
import json
for f in ['noev','ev']:
    d=json.loads(open('gpurun_out/exp/'+f+'.json').read().strip().splitlines()[-1]); print(f, d['ms_per_step'], d['cg_iterations'], d.get('phase_ms_per_step'))
"
