set -o pipefail
mkdir -p gpurun_out
# 2 ranks on one GPU over gloo (last step) rehearses the multi-process GPU path: arena buckets, backward hooks, direct grads
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv or bottleneck or resnet" > gpurun_out/conv_tests.log 2>&1 && \
timeout -k 10 400 env MXAMD_BENCH_VERBOSE=1 python -u bench.py --steps 20 --warmup 10 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 400 env MXAMD_DIST_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --batch 64 > gpurun_out/bench_2rank_gloo.log 2>&1
