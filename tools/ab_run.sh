#!/bin/bash
# On the GPU box: alternate the builds ab/lib<V>.so (tools/ab_build.sh makes A = HEAD and B = the
# working tree; more variants can be dropped into ab/ by hand) through bench.py (same box, same
# clocks), ROUNDS times each, printing Msamples/s and the light-prep launch time per run.
# VARIANTS="A B C" selects the builds; extra args go to bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROUNDS=${ROUNDS:-3}
VARIANTS=${VARIANTS:-A B}
for r in $(seq "$ROUNDS"); do
    for v in $VARIANTS; do
        err=$(mktemp)
        out=$(MCPT_LIB_PATH=ab/lib$v.so timeout -k 10 200 python bench.py --no-cpu "$@" 2>"$err" | grep '^{') || exit 1
        # the exact pick's listed nodes over the timed steps, from the rank-0 totals log line
        exact=$(grep -o '"prep_exact_nodes": [0-9]*' "$err" | tail -1 | grep -o '[0-9]*$')
        rm -f "$err"
        echo "$v $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); p=d.get("roofline_prep") or {}; t=d.get("roofline_trace") or {}; print(d["value"], "prep_ms", p.get("avg_launch_ms"), "trace_ms", t.get("avg_launch_ms"), "visits", t.get("node_visits_per_ray"), "tests", t.get("tri_tests_per_ray"))') exact_nodes ${exact:-?}"
    done
done
