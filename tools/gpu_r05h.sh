#!/bin/bash
# round 5 final build: rocprof around bench.py for every BASELINE config (+ PMC HBM passes) and the training steps
set -o pipefail
bash tools/profile_bench.sh r05h --pmc cfg2 cfg2:125000 cfg3 cfg3:125000 cfg4 cfg5f cfg5i cfg5i:1024 || exit $?
bash tools/profile_bench.sh r05h cfg4t+graph cfg2t+graph cfg3t+graph || exit $?
