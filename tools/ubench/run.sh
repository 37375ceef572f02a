cd $GRAFT_REPO_ROOT/tools/ubench
for t in 128 16384; do for m in 0 1 2; do for w in 2 4 8; do timeout -k 5 60 ./gather $t $m 200 $w || exit 1; done; done; done
