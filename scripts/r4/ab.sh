# round 4, lease ab: copy_if one-hop look-back, group 64/32 x poll sleep 1/3 (scan and int32 rows ride along)
cd $GRAFT_REPO_ROOT
for b in oh_g64_s1 oh_g32_s1 oh_g64_s3 oh_g32_s3 oh_g64_s1 oh_g32_s1; do
  timeout -k 10 150 scripts/r4/lb/$b >> gpurun_out/r4ab_onehop_group.log 2>&1 || exit $?
done
