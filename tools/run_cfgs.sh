set -o pipefail
timeout -k 10 120 ./tools/ubench_valu > gpurun_out/ubench_valu2.txt 2>&1 || exit 1
for cv in 0:0 3:0 4:0 5:0 4:4 3:4 0:0; do
  c=${cv%:*}; v=${cv#*:}
  r=$(DSX_SCAN_CFG=$c DSX_SCAN_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu 2>/dev/null | grep -o '"kernel_ms": [0-9.]*\|"value": [0-9.]*\|"stitch_ms": [0-9.]*' | tr '\n' ' ') || exit 1
  echo "cfg=$c variant=$v $r"
done
