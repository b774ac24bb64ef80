# Round-3 final GPU session: bench lines, rocprofv3 kernel stats and the PMC
# passes the bench's roofline reads (separate passes), per workload.
set -uo pipefail
for wl in c3 c4; do
  TAG=r3f WL=$wl STEPS="prof pmc" bash tools/gpu_round.sh || exit 1
done
TAG=r3f WL=c5 STEPS="pmc" bash tools/gpu_round.sh || exit 1
