set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for opt in lamb lamb lamb adamw adamw adamw; do
  echo "== $opt"
  timeout -k 10 300 python -u tools/bench_bert.py --steps 3 --trace-loss --graph --batch 8 --warmup 3 --optimizer $opt > gpurun_out/dbg_env.log 2>&1; grep "^step" gpurun_out/dbg_env.log | tail -2
done
