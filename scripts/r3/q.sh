# round 3, lease q: more scan tile shapes on the fixed look-back (scan7: 384/768-thread tiles)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3q_scan7.log 2>&1
