#!/bin/bash
# Builds compile-time variants of the library into ab/lib<NAME>.so for same-box A/B timing
# (tools/ab_run.sh):  tools/ab_variants.sh "C:-DMCPT_RAY_TOP=21" "D:-DMCPT_RAY_TOP=85 -DMCPT_RAY_LDS=8"
set -e
cd "$(dirname "$0")/.."
mkdir -p ab
for spec in "$@"; do
    name=${spec%%:*}
    defs=${spec#*:}
    obj=/tmp/mcpt_ab_$name
    make -s -C monte_carlo_path_tracing_amd/csrc -j8 OBJ="$obj" LIB="$PWD/ab/lib$name.so" CLI="$obj/cli" EXTRA="$defs" \
        "$PWD/ab/lib$name.so" >/dev/null
    echo "ab/lib$name.so: $defs"
done
