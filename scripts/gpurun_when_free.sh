#!/bin/bash
# scripts/gpurun_when_free.sh OUTFILE TIMEOUT 'command': one gpurun call,
# re-issued only while gpurun reports status=transient (no box or slot free:
# nothing ran, nothing was charged), at most 12 times, 4 minutes apart. Any
# other outcome (the command ran, failed or was refused) ends it.
out=$1 lim=$2 cmd=$3
for i in $(seq 1 12); do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  grep -q "status=transient" "$out" || break
  echo "attempt $i: transient (rc $rc), waiting" >> "$out.tries"
  sleep 240
done
echo "done rc=$rc" >> "$out.tries"
