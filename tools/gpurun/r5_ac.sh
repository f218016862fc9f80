# round 5: A/B of non-temporal optimizer-state traffic (alternate builds, MXAMD_OPT_NT 1 / 2) on BERT and ResNet
set -o pipefail
TAG=${1:-r5ac}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SO=mxnet_maintenance_amd/_lib/_hip_kernels.cpython-310-x86_64-linux-gnu.so
cp $SO /tmp/base.so || exit 1
for run in base nt1 nt2 base nt1 nt2; do
  if [ $run = base ]; then cp /tmp/base.so $SO; else cp alt_build/_hip_kernels_opt_$run.so $SO; fi
  timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_$run.log 2>&1 || exit $?
  echo "bert $run $(tail -1 gpurun_out/${TAG}_bert_$run.log | grep -o '"value": [0-9.]*')"
done
for run in base nt2; do
  if [ $run = base ]; then cp /tmp/base.so $SO; else cp alt_build/_hip_kernels_opt_$run.so $SO; fi
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_resnet_$run.log 2>&1 || exit $?
  echo "resnet $run $(tail -1 gpurun_out/${TAG}_resnet_$run.log | grep -o '"value": [0-9.]*' | head -1)"
done
