# Run GPU steps in order, each under its own time limit; test failures (rc 1) go on to the
# next step, anything else (a timeout 124/137, an abort 134, a fault 139, ...) ends the
# session there, so nothing more touches a GPU that may be in a bad state.
#   bash tools/gpu_steps.sh <outdir> "<seconds> <command>" ["<seconds> <command>" ...]
O=$1; shift
mkdir -p $O
i=0
for step in "$@"; do
  i=$((i + 1))
  secs=${step%% *}; cmd=${step#* }
  timeout -k 10 $secs bash -c "$cmd" > $O/step$i.log 2>&1
  rc=$?
  echo "step $i rc=$rc: $cmd" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
