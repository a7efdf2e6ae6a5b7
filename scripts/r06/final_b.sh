# Round-6 evidence, call B: the 1M / 10M profile set and the README scene's (scripts/round_profiles.sh 2, 3).
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash scripts/round_profiles.sh 2 && mkdir -p gpurun_out/round2 && cp gpurun_out/round/* gpurun_out/round2/ &&
bash scripts/round_profiles.sh 3
