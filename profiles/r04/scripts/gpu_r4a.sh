set -uo pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4a
timeout -k 10 120 ./tools/probe/col_probe > gpurun_out/r4a/col_probe.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_bench.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1
echo rc=$?
