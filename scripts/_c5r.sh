cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04c5r; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/c5_attraction.py --relabel degree > $O/c5_relabel.json 2> $O/c5_relabel.err || { tail -5 $O/c5_relabel.err; exit 1; }
cat $O/c5_relabel.json; cat $O/c5_relabel.err
