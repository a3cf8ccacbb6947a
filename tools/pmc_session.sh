#!/bin/bash
# PMC counter passes over the Gram + CG microbenchmark (tools/gram_bench.py).
set -o pipefail
OUT=gpurun_out/${1:-pmc}; shift
mkdir -p $OUT; export TMPDIR=/tmp
ARGS="$@"
i=0
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
         "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCC_EA0_RDREQ_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace -d $OUT/p$i -o run --output-format csv -- python3 tools/gram_bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_kernels.py $OUT/p1 $OUT/p2 $OUT/p3
