#!/bin/bash
# conv / deformable bias gradients on the column-sum kernels: tests + SSD-512 bench + window
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_kpad.py tests/test_deform_conv.py tests/test_conv_dilated.py tests/test_ssd.py tests/test_hip_kernels.py -k "conv or deform or ssd or dilat or kpad or multibox" > gpurun_out/r6aa_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r6aa_tests.log; exit 1; }
tail -1 gpurun_out/r6aa_tests.log
timeout -k 10 400 python -u tools/bench_ssd.py --steps 20 --warmup 5 > gpurun_out/r6aa_ssd.log 2>&1 || { echo SSD FAILED; tail -20 gpurun_out/r6aa_ssd.log; exit 1; }
tail -1 gpurun_out/r6aa_ssd.log | cut -c1-160
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6aa_prof -o trace -- python3 -u tools/bench_ssd.py --steps 8 --warmup 4 > gpurun_out/r6aa_prof.log 2>&1 || { echo PROF FAILED; tail -5 gpurun_out/r6aa_prof.log; exit 1; }
python tools/trace_window.py gpurun_out/r6aa_prof --steps 4 --top 70 > gpurun_out/r6aa_window.txt 2>&1; head -11 gpurun_out/r6aa_window.txt | cut -c1-160
grep -E "direct_copy|copyBuffer|CUDAFunctor_add|Fill|reduce_kernel|float32_copy|float16_copy" gpurun_out/r6aa_window.txt | cut -c1-150
rm -rf gpurun_out/r6aa_prof
