#!/bin/bash
# round 5 final build (16-byte kept tiles, compact OUTK image): full GPU suite + smoke, then
# rocprof around bench.py for every config (+ PMC HBM passes) and the training steps
set -o pipefail
bash tools/gpu_suite.sh r05suite2 || exit $?
bash tools/profile_bench.sh r05i --pmc cfg2 cfg2:125000 cfg3 cfg3:125000 cfg4 cfg5f cfg5i cfg5i:1024 || exit $?
bash tools/profile_bench.sh r05i cfg4t+graph cfg2t+graph cfg3t+graph || exit $?
