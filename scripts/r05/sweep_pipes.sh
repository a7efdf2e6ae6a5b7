# pipelines (iterations in flight) and trace waves per CU re-swept at the 4-wide code (one process per setting)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp &&
bash scripts/envsweep.sh 2 "--steps 20 --warmup 5" "" "PT_PIPES=12" "PT_PIPES=20" "PT_PIPES=24" "PT_TRACE_WAVES_PER_CU=6" "PT_PIPES=24 PT_TRACE_WAVES_PER_CU=6" &&
bash scripts/envsweep.sh 1 "--steps 16 --warmup 2 --ntri 10000000 --bounces 16 --inmem" "" "PT_PIPES=24" "PT_TRACE_WAVES_PER_CU=6"
