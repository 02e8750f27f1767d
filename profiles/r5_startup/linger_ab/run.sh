#!/bin/bash
# A/B: default vs --linger, interleaved (A B A B), 8 bring-ups each
set -o pipefail
export PYTHONPATH="$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5_ab}
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-pod-workload --no-sweep > $O/a$r.json 2> $O/a$r.err || exit 1
  echo a$r done
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-pod-workload --no-sweep $2 > $O/b$r.json 2> $O/b$r.err || exit 1
  echo b$r done
done
