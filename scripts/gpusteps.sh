#!/bin/bash
# Run GPU steps one after another on the gpurun box: each line of the steps
# file is "<name> <timeout seconds> <command...>".  Output goes to
# gpurun_out/<name>.out / .err.  A step that passes or fails normally (exit 0
# or 1) lets the next one run; anything else (a time limit, an abort, a
# segfault, a GPU fault) ends the call there.
set -u
mkdir -p gpurun_out
while read -r name limit cmd; do
    [ -z "${name:-}" ] && continue
    case "$name" in \#*) continue ;; esac
    start=$(date +%s)
    timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    rc=$?
    echo "$name rc=$rc $(( $(date +%s) - start ))s"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit "$rc"
    fi
done < "$1"
