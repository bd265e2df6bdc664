#!/bin/bash
# Per-step kernel durations of the first 65 training steps under rocprofv3
# (profiles/r03/warm/).  Variants B (no synchronize after the warmup), D (the
# ranking section before the warmup) and E (100 extra training steps first)
# used temporary diagnostic switches of bench.py that were removed after the
# measurement; A and C run on the current bench.py.
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/warm
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-A B C}; do
  case $v in
    A) E="KGE_X=0"; X="--no-rank";;
    B) E="KGE_DBG_NOSYNC_WARMUP=1"; X="--no-rank";;
    C) E="KGE_X=0"; X="--no-stage-timer --no-rank";;
    D) E="KGE_BENCH_RANK_FIRST=1"; X="";;
    E) E="KGE_DBG_PRESTEPS=100"; X="--no-rank";;
  esac
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/warm/$v -o run -- python3 $R/bench.py --steps 60 --warmup 5 --no-cpu-baseline $X > $R/gpurun_out/warm/$v.json 2> $R/gpurun_out/warm/$v.err || exit $?
done
