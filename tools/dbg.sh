cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dbgprof -o dbg -- python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/dbg.log 2>&1
tail -2 gpurun_out/dbg.log
find gpurun_out/dbgprof -name "*kernel_trace.csv" | head -1 | xargs cat | cut -d, -f1-30 | head -20
