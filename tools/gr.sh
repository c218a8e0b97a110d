#!/bin/bash
# gpurun with a resubmit when the call never ran (box lost while being prepared / taken away):
# only transient infrastructure outcomes are resubmitted, never a command that ran and failed
T=$1; shift
for i in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gr.out 2>&1
  rc=$?
  if grep -q 'status=transient\|taken away\|rc=3\|no box' /tmp/gr.out && ! grep -q 'status=ok' /tmp/gr.out; then
    sleep 45; continue
  fi
  break
done
grep -v 'every call sends' /tmp/gr.out | tail -6
exit $rc
