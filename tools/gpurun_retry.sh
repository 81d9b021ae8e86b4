#!/bin/bash
# Dev tool: run one gpurun call, retrying ONLY while the pool reports no free box / backoff ("status=transient":
# nothing ran, nothing charged), at most $TRIES times, $WAIT s apart.  Usage: tools/gpurun_retry.sh OUT TIMEOUT 'CMD'
out=$1; to=$2; cmd=$3
for i in $(seq 1 ${TRIES:-8}); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if ! grep -q "status=transient" "$out"; then echo "rc=$rc try=$i" >> "$out"; exit $rc; fi
  sleep ${WAIT:-540}
done
echo "gave up after $i tries" >> "$out"
exit 3
