# round 3, lease k: scan tile shapes with several workgroups per CU on the fixed look-back (scan7)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 scripts/ubench/scan7 > gpurun_out/r3k_scan7.log 2>&1
