#!/bin/bash
# Client-side helper: run one gpurun call, re-submitting it only when gpurun
# reports an infrastructure event before the command ran (status=transient:
# no box free, box lost while being prepared, backoff).  A call whose command
# ran is never repeated, whatever its exit code.
# usage: [RETRIES=N] scripts/gpurun_retry.sh LOGFILE TIMEOUT 'command'
log=$1; to=$2; cmd=$3
for i in $(seq 1 ${RETRIES:-8}); do
    /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
    rc=$?
    if grep -q "status=transient" "$log" && ! grep -q "run [1-9][0-9.]*s of limit" "$log"; then
        sleep 75
        continue
    fi
    exit $rc
done
exit 3
