#!/bin/bash
# Builds the library at git revision/stash state A (HEAD) and at the working tree (B) into ab/
# for same-box A/B timing:  MCPT_LIB_PATH=ab/libA.so python bench.py ... vs ab/libB.so
set -e
cd "$(dirname "$0")/.."
mkdir -p ab
make -C monte_carlo_path_tracing_amd/csrc -j8 >/dev/null
cp monte_carlo_path_tracing_amd/libmcpt_hip.so ab/libB.so
git stash -q
make -C monte_carlo_path_tracing_amd/csrc -j8 >/dev/null
cp monte_carlo_path_tracing_amd/libmcpt_hip.so ab/libA.so
git stash pop -q
make -C monte_carlo_path_tracing_amd/csrc -j8 >/dev/null
echo "ab/libA.so (HEAD) ab/libB.so (working tree)"
