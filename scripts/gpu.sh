#!/bin/bash
# Run a command on the GPU box via gpurun; re-submit ONLY when the box failed
# to come up (status=transient: nothing ran, nothing charged).  Never retries
# a command that ran and failed.
# usage: scripts/gpu.sh <timeout-seconds> '<command>'
T=$1; shift
for attempt in 1 2 3 4 5; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient\|backing off\|no box\|slot"; then
    if echo "$out" | grep -q "status=ok\|rc=[0-9]"; then break; fi
    sleep 45; continue
  fi
  break
done
