#!/bin/bash
# isa_scan.sh ASM KERNEL_SUBSTR: list s_barrier / scratch / loop headers of one kernel in an -S dump
f=$1; k=$2
start=$(grep -n "^_Z[^ ]*${k}[^ ]*:" $f | head -1 | cut -d: -f1)
end=$(awk -v s=$start 'NR>s && /s_endpgm/ {print NR; exit}' $f)
sed -n "${start},${end}p" $f | grep -n "s_barrier\|scratch_\|Loop Header" | sed 's/;.*Loop Header: Depth=/LOOP/' | awk '{printf "%s ", $0} END {print ""}' | fold -w 220
