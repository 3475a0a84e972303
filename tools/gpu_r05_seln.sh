# Round 5: the NULL-able selection's one structural experiment (VERDICT r4
# item 6): 6 loaders + 6 storers (MBX_SR_NL=6) vs the default 8 loaders + 4
# storers.  First the NULL-able selection tests under the 6+6 form, then the
# A/B as rocprofv3 kernel-trace averages over 7 launches per run, alternated twice.
set -o pipefail
mkdir -p gpurun_out/r05s
R=$PWD
MBX_SR_NL=6 timeout -k 10 400 python -u -m pytest tests/test_gpu_compact.py -m gpu -x -q -k "nullable" --timeout 200 --timeout-method thread > gpurun_out/r05s/tests_nl6.log 2>&1 || exit 51
export MBX_EXPERIMENTS=1 NULLABLE=1 SHAPES=seln_out,seln_pred REPS=7
for rep in 1 2; do
  for nl in 8 6; do
    ( cd /tmp && export TMPDIR=/tmp && MBX_SR_NL=$nl timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05s/nl${nl}_$rep -o t -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/r05s/nl${nl}_$rep.log 2>&1 ) || exit 52
    rm -f $R/gpurun_out/r05s/nl${nl}_$rep/*kernel_trace.csv  # (the stats CSV is what is kept)
  done
done
du -sh gpurun_out/r05s
echo DONE
