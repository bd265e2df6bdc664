# round 4: the early-step phase with an in-kernel clock probe beside the training step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/hump_trace.py --bursts 0:150,1000:60,50:60,3000:60 > gpurun_out/r04f_hump_probe.jsonl 2> gpurun_out/r04f_hump_probe.err || exit $?
