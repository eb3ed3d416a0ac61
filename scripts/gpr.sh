#!/bin/bash
# usage: gpr.sh <logfile> <timeout> <command...> : resubmit while gpurun reports no free box (exit 3 / transient)
log=$1; to=$2; shift 2
for i in $(seq 1 40); do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout $to -- "$@" > "$log" 2>&1
  rc=$?
  if grep -q "no free box\|backing off\|stopped responding\|retry" "$log" && ! grep -q "status=ok\|status=fail" "$log"; then sleep 120; continue; fi
  break
done
echo "GPR_DONE rc=$rc" >> "$log"
