#!/bin/bash
# Same-binary A/B of the C5 traversal: k_rays_cw8 (8-wide, MCPT_DEBUG_RAYS_CW8 = 0x200000) vs
# k_rays_persistent (4-wide, the default), ROUNDS alternations of bench.py --scene cornell1m.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for r in $(seq "${ROUNDS:-2}"); do
    for v in cw8 bvh4; do
        fl=0x200000; [ $v = bvh4 ] && fl=0
        out=$(timeout -k 10 300 python bench.py --scene cornell1m --no-cpu --debug-flags $fl "$@" 2>/dev/null | grep '^{') || exit 1
        echo "$v $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); t=d.get("roofline_trace") or {}; print(d["value"], "trace_ms", t.get("avg_launch_ms"), "visits/ray", t.get("node_visits_per_ray"), "tests/ray", t.get("tri_tests_per_ray"))')"
    done
done
