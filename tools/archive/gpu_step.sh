#!/bin/bash
# run one GPU step under its own time limit; stop the whole script on a hang / crash
# (124 / 137 timeout, 134 abort, 139 segfault): usage  step NAME SECONDS cmd...
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -3 "gpurun_out/$name.txt" >&2
  case $rc in 124|137|134|139) echo "stopping after $name (rc $rc)" >&2; exit $rc;; esac
  return 0
}
