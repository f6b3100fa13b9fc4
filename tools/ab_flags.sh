#!/bin/bash
# Same-binary A/B over mcpt_render_opts debug flags: FLAGS="0 0x100000 ..." alternated ROUNDS times through
# bench.py (extra args passed on), printing Msamples/s and the light-prep / traversal launch times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for r in $(seq "${ROUNDS:-2}"); do
    for fl in ${FLAGS:-0}; do
        out=$(timeout -k 10 300 python bench.py --no-cpu --debug-flags "$fl" "$@" 2>/dev/null | grep '^{') || exit 1
        echo "$fl $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); p=d.get("roofline_prep") or {}; t=d.get("roofline_trace") or {}; print(d["value"], "prep_ms", p.get("avg_launch_ms"), "trace_ms", t.get("avg_launch_ms"), "visits/ray", t.get("node_visits_per_ray"), "tests/ray", t.get("tri_tests_per_ray"))')"
    done
done
