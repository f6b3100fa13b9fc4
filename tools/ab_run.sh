#!/bin/bash
# On the GPU box: alternate the two builds of tools/ab_build.sh through bench.py (same box, same
# clocks), ROUNDS times each, printing Msamples/s per run.  Extra args go to bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROUNDS=${ROUNDS:-3}
for r in $(seq "$ROUNDS"); do
    for v in A B; do
        out=$(MCPT_LIB_PATH=ab/lib$v.so timeout -k 10 200 python bench.py --no-cpu "$@" 2>/dev/null | grep '^{') || exit 1
        echo "$v $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_ms"])')"
    done
done
