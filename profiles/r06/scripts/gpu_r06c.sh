set -u
O=gpurun_out/r6c; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.out 2>&1; local rc=$?; tail -3 $O/$name.out; echo "$name rc=$rc"; if [ $rc -gt 1 ]; then exit $rc; fi; }
NWK_GUARD_LOG=1 NWK_GOTOH=0 NWK_BITS_WIN=40 step flake 400 python -u profiles/r06/scripts/pka_flake_guard.py 300
NWK_GOTOH=0 step ab_new 300 python -u tools/ab_wl.py multiple-sequence-alignment-openmp-openmpi_amd/lib c5 1
NWK_GOTOH=0 step ab_old 300 python -u tools/ab_wl.py variants/asmpf c5 1
step pytest 900 python -u -m pytest tests/ -m gpu -q --timeout 150 --timeout-method thread -p no:cacheprovider
