cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp PYTHONUNBUFFERED=1; O=gpurun_out/r04sync; mkdir -p $O
for rep in 1 2 3; do for lib in default sync1 sync2; do
  if [ $lib = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
  echo "== $lib rep $rep"; env QMHA_LIB_PATH=$LP timeout -k 10 120 python tools/probe_calls.py --reps 10 --bursts async1,solve 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done; done 2>&1 | tee $O/summary.txt
