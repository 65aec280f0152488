#!/bin/bash
# retry a gpurun call only while the pool reports no free slot/box (nothing ran, nothing charged)
out=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout 2700 /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  if grep -q "nothing was charged\|no free box right now\|stopped responding while being prepared\|is backing off" $out && ! grep -q "status=ok\|status=fail" $out; then
    sleep 150; continue
  fi
  break
done
