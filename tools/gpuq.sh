#!/bin/bash
# gpurun with waiting for a free slot: repeats ONLY while gpurun reports "no box/slot free" (exit 3,
# nothing ran, nothing charged).  Usage: gpuq.sh OUTFILE TIMEOUT CMD
OUT=$1; T=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@" > $OUT 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc" >> $OUT; exit $rc; fi
  sleep 90
done
exit 3
