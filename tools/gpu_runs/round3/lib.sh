# Helpers for round-3 GPU command files: run a step under its own time limit, log it
# under gpurun_out/, and stop the whole script on a fault / abort / timeout (exit
# status other than 0 = ok or 1 = test / check failure).
set -u
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <command...>
  local name="$1" secs="$2"; shift 2
  echo "[step] $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[step] $name rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 4 ]; then
    echo "[step] stopping after rc=$rc"; exit $rc
  fi
}
PYT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
