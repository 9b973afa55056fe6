cd $GRAFT_REPO_ROOT
for c in c1_w512 c3_w512 c3_w64 beta_w64 nomap_w64 c3_test_w64 c5_w512; do
timeout -k 10 200 python tools/zsave_check.py $c zsave=0 zsave=1 2>/dev/null | grep grad | sed "s/^/$c /" | cut -c1-60
done
