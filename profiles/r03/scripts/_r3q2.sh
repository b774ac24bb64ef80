# A/B: issue priority for the bands of a job's longest pairs (span-bound big13)
set -uo pipefail
export REPS=5
for V in base3 prio base3 prio; do
  timeout -k 10 200 python3 -u tools/fill_timeit.py tools/abv/$V 2>&1 | grep timeit || exit 1
done
for V in base3 prio; do
  timeout -k 10 200 python3 -u tools/ab_wl.py tools/abv/$V c3 3 2>&1 | grep "^ab" || exit 1
done
