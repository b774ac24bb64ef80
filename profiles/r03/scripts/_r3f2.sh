set -uo pipefail
TAG=r3f WL=c5 STEPS="pmc" bash tools/gpu_round.sh || exit 1
TAG=r3f2 STEPS="bench" WL=c3 BSTEPS=5 bash tools/gpu_round.sh || exit 1
TAG=r3f2 STEPS="bench" WL=c4 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
TAG=r3f2 STEPS="bench" WL=big13 BSTEPS=5 BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_round.sh || exit 1
