#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_lstm_lm.py --dtype bfloat16 --steps 30 --warmup 5 > gpurun_out/r6e_lstm650_bf16.log 2>&1 && tail -1 gpurun_out/r6e_lstm650_bf16.log
timeout -k 10 300 python -u tools/bench_lstm_lm.py --dtype bfloat16 --steps 30 --warmup 5 --hidden 1024 > gpurun_out/r6e_lstm1024_bf16.log 2>&1 && tail -1 gpurun_out/r6e_lstm1024_bf16.log
bash tools/gpu_bench.sh r6e
