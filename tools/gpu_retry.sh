#!/bin/bash
# (development helper: run from the container, not on the GPU box)
# retry a gpurun call only while the pool reports an infrastructure transient (no box / backoff); stop on any run
LOG=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout 1100 -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && ! grep -q "run [1-9]" $LOG; then
    w=$(grep -o "retry in [0-9]*s" $LOG | grep -o "[0-9]*" | head -1)
    sleep $(( ${w:-120} + 10 ))
    continue
  fi
  break
done
echo "__done rc=$rc attempts=$i" >> $LOG
