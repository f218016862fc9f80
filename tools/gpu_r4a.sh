set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_resnet_gpu.py tests/test_engine_device.py "tests/test_hip_kernels.py::test_lamb_arena_kernel_matches_per_segment_reference" > gpurun_out/r4a_tests.log 2>&1
