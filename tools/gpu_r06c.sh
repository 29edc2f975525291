#!/bin/bash
# Round 6: push-kernel near-slot ablation (the chain wave's share of a two-wave split: timing
# only) against the shipped kernel, then the relational seeds on both train paths.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06c; mkdir -p $O; cd $R
timeout -k 10 300 python -u tools/seq_batch_sweep.py 256 1024 > $O/sweep_base.jsonl 2>&1 || exit $?
NFX_LIB=$R/normalizing-flows-study_amd/nfs_amd/libnfx_near.so timeout -k 10 300 python -u tools/seq_batch_sweep.py 256 1024 > $O/sweep_near.jsonl 2>&1 || exit $?
cat $O/sweep_base.jsonl $O/sweep_near.jsonl | grep '^{'
NFX_TRAIN_KEEP=1 timeout -k 10 400 python -u tools/relational_seeds.py > $O/keep1.jsonl 2>&1 || exit $?
NFX_TRAIN_KEEP=0 timeout -k 10 400 python -u tools/relational_seeds.py > $O/keep0.jsonl 2>&1 || exit $?
