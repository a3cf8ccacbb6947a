set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gap
timeout -k 10 300 python bench.py --no-cpu --steps 50 > gpurun_out/gap/bench.json 2> gpurun_out/gap/bench.err || { tail -5 gpurun_out/gap/bench.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/gap/bench.json')); print(d['ms_per_step'], d['ms_per_step_without_kernel_events'], d['cg_iterations'])"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gap/ev -o run --output-format csv -- python3 bench.py --no-cpu --steps 30 > gpurun_out/gap/ev.json 2> gpurun_out/gap/ev.err || { tail -5 gpurun_out/gap/ev.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/gap/noev -o run --output-format csv -- python3 bench.py --no-cpu --steps 30 --no-kernel-events > gpurun_out/gap/noev.json 2> gpurun_out/gap/noev.err || { tail -5 gpurun_out/gap/noev.err; exit 1; }
echo done
