set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread -k "layernorm or gelu or softmax_fwd or dropout or adam or lamb or all_finite or linear" > gpurun_out/nlp_tests.log 2>&1
