#!/bin/bash
# Samples board power, shader clock and temperature of every GPU hwmon
# (sysfs, readable as an ordinary user) every ~5 ms while a command runs:
#   tools/power_sample.sh OUT.txt -- python bench.py ...
# Each line: unix time, then {power uW, sclk Hz, temp mC} per hwmon.
OUT=$1; shift; [ "$1" = "--" ] && shift
# this job's GPU only (tools/gpu_hwmon.py: HIP device 0's PCI function); all
# cards if it cannot be found
HW=$(python3 "$(dirname "$0")/gpu_hwmon.py" 2>/dev/null) || HW=""
[ -n "$HW" ] || HW="/sys/class/drm/card*/device/hwmon/hwmon*"
( while :; do
    line="$(date +%s.%N)"
    for h in $HW; do
      line="$line $(cat $h/power1_input 2>/dev/null || echo -) $(cat $h/freq1_input 2>/dev/null || echo -) $(cat $h/temp2_input 2>/dev/null || echo -)"
    done
    echo "$line"
    sleep 0.005
  done ) > "$OUT" &
SP=$!
"$@"
rc=$?
kill $SP 2>/dev/null
wait $SP 2>/dev/null
exit $rc
