# round 5: the entity pass with its Adam moments loaded straight into LDS
# (KGE_ENT_MOML was read only by a temporary diagnostic build; rejected, code removed)
# (global_load_lds, 74 VGPRs / 6 waves per SIMD instead of 92 / 5;
# KGE_ENT_MOML=1, A/B diagnostic) — the parity suites with it on, then the
# bench alternated, then rocprofv3 traces of both
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r05u"
mkdir -p "$O"
cd "$ROOT"
KGE_ENT_MOML=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_edge_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > "$O/gpu_tests.log" 2>&1 || exit $?
for k in 1 2; do
  KGE_ENT_MOML=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-rank --steps 200 --warmup 100 > "$O/bench_moml_$k.json" 2>> "$O/bench.err" || exit $?
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-rank --steps 200 --warmup 100 > "$O/bench_regs_$k.json" 2>> "$O/bench.err" || exit $?
done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  KGE_ENT_MOML=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_moml$v" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-rank --steps 60 --warmup 20 > "$O/bench_prof_moml$v.json" 2>> "$O/bench.err" || exit $?
done
