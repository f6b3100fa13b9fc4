#!/bin/bash
# Runs GPU steps on the gpurun box, each under its own time limit; stops at the first step that
# faults, aborts, segfaults, times out or is killed (exit 124/134/137/139 or a signal), and keeps
# going after an ordinary failure (e.g. a failing test, exit 1) so later measurements still run.
#   tools/gpu_steps.sh "300:name:cmd ..." "600:name2:cmd2 ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
    limit=${spec%%:*}
    rest=${spec#*:}
    name=${rest%%:*}
    cmd=${rest#*:}
    echo "=== [$name] limit ${limit}s: $cmd"
    start=$(date +%s)
    timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "=== [$name] exit $rc after $(( $(date +%s) - start ))s"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ]; then status=$rc; fi
    case $rc in
        124|134|137|139) echo "=== stopping: fatal exit $rc"; exit $rc ;;
    esac
    if [ $rc -gt 128 ]; then echo "=== stopping: signal exit $rc"; exit $rc; fi
done
exit $status
