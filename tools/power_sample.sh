#!/bin/bash
# Samples board power, shader clock and temperature of every GPU hwmon
# (sysfs, readable as an ordinary user) every ~5 ms while a command runs:
#   tools/power_sample.sh OUT.txt -- python bench.py ...
# Each line: unix time, then {power uW, sclk Hz, temp mC} per hwmon.
OUT=$1; shift; [ "$1" = "--" ] && shift
( while :; do
    line="$(date +%s.%N)"
    for h in /sys/class/drm/card*/device/hwmon/hwmon*; do
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
