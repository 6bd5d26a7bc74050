#!/bin/bash
# GPU parity suite, then the default bench line (no CPU leg); prints the
# pytest tail and the bench's value / kernel_ms / stitch_ms.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1
rc=$?
tail -3 gpurun_out/verify_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/verify_bench.json 2> gpurun_out/verify_bench.err || { tail gpurun_out/verify_bench.err; exit 1; }
grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"stitch_ms": [0-9.]*' gpurun_out/verify_bench.json | tr '\n' ' '
echo
