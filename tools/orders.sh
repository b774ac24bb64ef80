cd $GRAFT_REPO_ROOT
for o in 0 1 4 16; do echo "== NWK_ORDER=$o"; NWK_ORDER=$o timeout -k 10 100 bash tools/timeline.sh 2>&1 | tail -2; done
