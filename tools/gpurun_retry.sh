# run one gpurun call; on exit 3 (no box / transient, nothing ran, nothing charged) wait and
# try again, at most 6 times.  Any other exit code is final.
# usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for k in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  echo "exit=$rc try=$k" >> $LOG
  [ $rc -ne 3 ] && exit $rc
  sleep 75
done
exit 3
