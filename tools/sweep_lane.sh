#!/bin/bash
# Lane-segment size / regions-per-slot sweep of the line-aligned scan at 1 and
# 4 GiB (full kernel and the staging-only / compute-only ablations).
bash tools/sweep2.sh DSX_REGIONS_PER_SLOT=1 DSX_REGIONS_PER_SLOT=2 DSX_REGIONS_PER_SLOT=4 \
  "DSX_REGIONS_PER_SLOT=4 DSX_SCAN_VARIANT=3" "DSX_REGIONS_PER_SLOT=4 DSX_SCAN_VARIANT=4" \
  DSX_LANE_BYTES=8448 DSX_LANE_BYTES=2304 DSX_LANE_BYTES=4224 \
  "DSX_LANE_BYTES=8448 DSX_SCAN_VARIANT=3" "DSX_LANE_BYTES=4224 DSX_SCAN_VARIANT=3" \
  "DSX_LANE_BYTES=8448 DSX_SCAN_VARIANT=4"
