set -o pipefail
for v in old old_prio rowrun rowrun_prio; do
  timeout -k 10 120 python3 tools/ab_wl.py tools/libvariants/$v c3 2 || exit 1
done
