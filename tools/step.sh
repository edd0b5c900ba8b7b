#!/bin/bash
# Run GPU steps in sequence on the box, each under its own time limit, stopping at the first failure that is not
# a plain test failure (rc 1). Usage: bash tools/step.sh NAME SECONDS CMD... [-- NAME SECONDS CMD...]...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
while [ $# -gt 0 ]; do
  name=$1 secs=$2
  shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do cmd+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  echo "== $name: ${cmd[*]}"
  timeout -k 10 "$secs" "${cmd[@]}" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -n 15 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "== stopping (rc=$rc)"; exit $rc; fi
done
