#!/bin/bash
# retry gpurun only while it reports "no slot / no box" (exit 3); any other status ends it
log="$1"; shift
for i in $(seq 1 20); do
  timeout 2400 /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "rc=$rc" >> "$log"; exit $rc; fi
  sleep 150
done
echo "rc=3 (gave up)" >> "$log"
