#!/bin/bash
# End-of-round GPU check at HEAD, as the driver runs it: the GPU test tier,
# smoke() and a driver-style N=1 bench.  Usage (from the repo root, on the
# box): gpurun --timeout 1100 -- bash tools/gpu_round_check.sh [tag] [steps] [warmup]
# Results under gpurun_out/round_check_<tag>/.  Every GPU step has its own
# time limit and the steps stop at the first failure.
set -u
tag=${1:-head}
steps=${2:-20}
warmup=${3:-5}
out=gpurun_out/round_check_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 420 python -u -m pytest tests -m gpu -v -rs --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$out/pytest_gpu.log"
[ $rc -eq 0 ] || { echo "pytest -m gpu rc=$rc"; exit $rc; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1
rc=$?
tail -2 "$out/smoke.log"
[ $rc -eq 0 ] || { echo "smoke rc=$rc"; exit $rc; }
timeout -k 10 420 python -u bench.py --gpus 1 --steps "$steps" --warmup "$warmup" --detail "$out/bench_detail.json" \
    > "$out/bench.json" 2> "$out/bench.err"
rc=$?
cat "$out/bench.json"
[ $rc -eq 0 ] || { tail -20 "$out/bench.err"; echo "bench rc=$rc"; exit $rc; }
