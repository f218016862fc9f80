# round 5: hipBLASLt/rocBLAS solution tuning (PyTorch TunableOp) for the library GEMMs: BERT and ResNet A/B
set -o pipefail
TAG=${1:-r5o}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_base.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert_base.log | cut -c1-200
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/${TAG}_tunable_bert%d.csv \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 \
  timeout -k 10 600 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_tuned.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert_tuned.log | cut -c1-200
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/${TAG}_tunable_bert%d.csv \
  timeout -k 10 300 python -u tools/bench_bert.py --steps 20 --warmup 5 --graph > gpurun_out/${TAG}_bert_tuned_reuse.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bert_tuned_reuse.log | cut -c1-200
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/${TAG}_tunable_resnet%d.csv \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 \
  timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_resnet_tuned.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_resnet_tuned.log | cut -c1-200
ls -la gpurun_out/${TAG}_tunable_* 
