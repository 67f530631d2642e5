# Submit one gpurun call, re-submitting only while the pod reports no free slot (exit 3: nothing ran, nothing
# charged).  Any other exit (including a failed GPU step) ends the loop.   usage: tools/gpurun_wait.sh <out> <timeout> <cmd>
out=$1; to=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
