# round 6: the occurrence CSR's bucket offsets from one workgroup (k_csr_scan1) instead of rocPRIM's
# decoupled look-back scan beside k_row: training parity suites, 200-step windows alternated
# (KGE_CSR_SCAN1=0 restores rocPRIM), rocprofv3 kernel stats of both
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06q"
mkdir -p "$O"
cd "$ROOT"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_dp_factors_gpu.py tests/test_dp_owner_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/parity.log" 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_scan1_$i.json" 2> "$O/err_scan1_$i.txt" || exit $?
  KGE_CSR_SCAN1=0 timeout -k 10 200 python3 bench.py --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_rocprim_$i.json" 2> "$O/err_rocprim_$i.txt" || exit $?
done
timeout -k 10 300 python3 bench.py --workload yago3-10-rowpart --no-rank --no-cpu-baseline --steps 100 --warmup 20 > "$O/yago_scan1.json" 2> "$O/err_yago1.txt" || exit $?
KGE_CSR_SCAN1=0 timeout -k 10 300 python3 bench.py --workload yago3-10-rowpart --no-rank --no-cpu-baseline --steps 100 --warmup 20 > "$O/yago_rocprim.json" 2> "$O/err_yago0.txt" || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_scan1" -o run -- \
  python3 "$ROOT/bench.py" --no-rank --no-cpu-baseline --steps 100 --warmup 20 > "$O/bench_prof_scan1.json" 2> "$O/err_prof1.txt" || exit $?
KGE_CSR_SCAN1=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_rocprim" -o run -- \
  python3 "$ROOT/bench.py" --no-rank --no-cpu-baseline --steps 100 --warmup 20 > "$O/bench_prof_rocprim.json" 2> "$O/err_prof0.txt" || exit $?
