# round 6: the whole GPU suite (incl. the CSR look-ahead, the two-direction ranking, the config-5
# world-8 test with per-step replica fingerprints), then the CSR look-ahead A/B on the bench and the
# pRotatE tile staging A/B on the ranking tool
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(pwd)}"
O="$ROOT/gpurun_out/r06e"
mkdir -p "$O"
cd "$ROOT"
( while true; do date >> "$O/heartbeat.txt"; sleep 30; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  --durations=15 > "$O/gpu_tests.log" 2>&1
rc=$?
kill $HB
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_ahead_$i.json" 2> "$O/err_ahead_$i.txt" || exit $?
  KGE_CSR_AHEAD=0 timeout -k 10 200 python3 bench.py --no-rank --no-cpu-baseline --steps 200 --warmup 20 > "$O/bench_noahead_$i.json" 2> "$O/err_noahead_$i.txt" || exit $?
done
for i in 1 2; do
  timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_spl.jsonl" 2>> "$O/err_prot.txt" || exit $?
  KGE_TILE_SPL=0 timeout -k 10 200 python3 tools/bench_rank.py --models pRotatE --gamma 6 --reps 3 >> "$O/prot_old.jsonl" 2>> "$O/err_prot.txt" || exit $?
done
