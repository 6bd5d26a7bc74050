#!/bin/bash
# GPU parity suite, then interleaved bench runs with env A vs env B
# (A/B: space-separated VAR=VALUE lists), REPS times each.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -40 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
for rep in $(seq ${REPS:-3}); do
  for v in A B; do
    envs=${!v}
    env $envs timeout -k 10 120 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    echo "$v [$envs] $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"stitch_ms": [0-9.]*' gpurun_out/ab.json | tr '\n' ' ')"
  done
done
