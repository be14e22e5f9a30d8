#!/bin/bash
# Host-side helper (this container, not the GPU box): submit one gpurun call and resubmit it only while the
# pool reports a transient condition (no free box / slot, box taken away before the command ran) -- never after
# the command itself ran.  Up to 8 submissions, 150 s apart.
#   tools/gpurun_retry.sh TIMEOUT 'command'
T=$1
shift
for i in 1 2 3 4 5 6 7 8; do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
    rc=$?
    st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status', ''))" 2>/dev/null)
    if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
    echo "[gpurun_retry] transient (attempt $i), retrying in 150 s"
    sleep 150
done
exit 3
