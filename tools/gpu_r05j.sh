#!/bin/bash
# round 5 final build (+ num_batches_tracked counted in the running-statistics kernel): full GPU
# suite + smoke, then rocprof around bench.py for every config (+ PMC HBM passes) and the training steps
set -o pipefail
bash tools/gpu_suite.sh r05suite4 || exit $?
bash tools/profile_bench.sh r05j cfg2t+graph || exit $?
bash tools/profile_bench.sh r05j --pmc cfg2 cfg2:125000 cfg3 cfg3:125000 cfg4 cfg5f cfg5i cfg5i:1024 || exit $?
bash tools/profile_bench.sh r05j cfg4t+graph cfg3t+graph || exit $?
