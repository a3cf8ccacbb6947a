set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bf3d
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bf3d/tests.log 2>&1; tail -3 gpurun_out/bf3d/tests.log
for K in 32 64 128; do bash tools/ab_gram.sh "--k $K" f32k$K:MR_GRAM_BF3=0 bf3k$K: || exit 1; done
bash tools/ab_variants.sh "--steps 60" f32:MR_GRAM_BF3=0 bf3: || exit 1
bash tools/ab_variants.sh "--steps 20 --k 128" f32k128:MR_GRAM_BF3=0 bf3k128:
