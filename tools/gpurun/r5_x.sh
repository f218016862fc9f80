# round 5: A/B of non-temporal LDS-DMA operand loads in the weight-gradient kernels (alternate build)
set -o pipefail
TAG=${1:-r5x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SO=mxnet_maintenance_amd/_lib/_hip_kernels.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/base.so || exit 1
for run in base alt base alt; do
  if [ $run = alt ]; then cp alt_build/_hip_kernels_wgrad_nt.so $SO; else cp /tmp/base.so $SO; fi
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$run.log 2>&1 || exit $?
  echo "$run $(tail -1 gpurun_out/${TAG}_bench_$run.log | grep -o '"value": [0-9.]*')"
done
cp alt_build/_hip_kernels_wgrad_nt.so $SO
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -- \
  python bench.py --steps 8 --warmup 6 > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python tools/trace_window.py gpurun_out/${TAG}_prof --steps 5 --top 60 > gpurun_out/${TAG}_window.txt
head -4 gpurun_out/${TAG}_window.txt | cut -c1-160
grep -E "wgrad" gpurun_out/${TAG}_window.txt | cut -c1-110
