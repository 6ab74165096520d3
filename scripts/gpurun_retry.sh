#!/bin/bash
# Local helper (runs HERE, not on the GPU box): submit one gpurun call and, only
# when gpurun reports that no box could be prepared (rc 3, or a "transient"
# status before anything ran), submit the same call again a few minutes later —
# at most N attempts.  A call that ran (any exit code of the command itself) is
# never repeated.
#   bash scripts/gpurun_retry.sh OUT.txt TIMEOUT 'command ...'
OUT=$1; TMO=$2; CMD=$3; N=${4:-6}
for i in $(seq 1 "$N"); do
  timeout $((TMO + 900)) /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if grep -q "stopped responding while being prepared\|backing off\|no box\|no free box\|are busy\|status=transient rc=None" "$OUT" && ! grep -q "merged" "$OUT"; then
    echo "attempt $i: no box (rc=$rc); retrying in 150 s" >> "$OUT.attempts"
    sleep 150
    continue
  fi
  echo "attempt $i: rc=$rc" >> "$OUT.attempts"
  exit $rc
done
exit 3
