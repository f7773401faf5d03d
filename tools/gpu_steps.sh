#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# fault / abort / timeout (exit 124, 134, 137, 139) so nothing else touches the
# GPU after one.  Usage: tools/gpu_steps.sh SECONDS 'cmd1' 'cmd2' ...
lim=$1; shift
for c in "$@"; do
  echo "== $c"
  timeout -k 10 "$lim" bash -c "$c"
  e=$?
  echo "== exit $e"
  case $e in 124|134|137|139) echo "stopping after exit $e"; exit $e;; esac
done
