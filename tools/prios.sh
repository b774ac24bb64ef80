cd $GRAFT_REPO_ROOT
for p in 0 1 2 0; do echo "== NWK_PRIO=$p"; NWK_PRIO=$p timeout -k 10 100 bash tools/timeline.sh 2>&1 | tail -2; done
