#!/bin/bash
# round 6d: RNN backward GEMMs in-tree + learnable LSTM LM; then the ResNet-50 bench + window
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rnn_kernels.py > gpurun_out/r6d_rnn_tests.log 2>&1 || { echo RNN TESTS FAILED; tail -40 gpurun_out/r6d_rnn_tests.log; exit 1; }
tail -2 gpurun_out/r6d_rnn_tests.log
timeout -k 10 300 python -u tools/bench_lstm_lm.py --dtype bfloat16 --steps 30 --warmup 5 > gpurun_out/r6d_lstm650_bf16.log 2>&1 && tail -1 gpurun_out/r6d_lstm650_bf16.log
timeout -k 10 300 python -u tools/bench_lstm_lm.py --dtype bfloat16 --steps 30 --warmup 5 --hidden 1024 > gpurun_out/r6d_lstm1024_bf16.log 2>&1 && tail -1 gpurun_out/r6d_lstm1024_bf16.log
bash tools/gpu_bench.sh r6d
