#!/bin/bash
# GPU-box run of the host-sanitizer driver (build first: make -C tools/asan).
set -o pipefail
mkdir -p gpurun_out/asan
export ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0:halt_on_error=1:abort_on_error=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
timeout -k 10 300 tools/asan/_out/asan_driver > gpurun_out/asan/asan.log 2>&1
rc=$?
grep -v "^  0x\|^Shadow\|^  [A-Z][a-z]* [a-z]*:\|^  [A-Z][a-z]*:" gpurun_out/asan/asan.log | head -60
exit $rc
