cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp PYTHONUNBUFFERED=1
BENCH_ARGS="--variant fa_tc_v1a --d 32 --H 32" bash tools/pmc_sq.sh r04f16sq/default || exit 1
QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/f16pj/libqmha.so BENCH_ARGS="--variant fa_tc_v1a --d 32 --H 32" bash tools/pmc_sq.sh r04f16sq/pipe || exit 1
