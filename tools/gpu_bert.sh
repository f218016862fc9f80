set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "layernorm or linear" > gpurun_out/ln_tests.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 > gpurun_out/bench_bert.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --optimizer adamw > gpurun_out/bench_bert_adamw.log 2>&1
