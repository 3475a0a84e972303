# select_rounds storer store flavour A/B (MBX_SR_NT_OFF: bit 0 plain value
# stores, bit 1 plain validity stores) on the NULL-able output shape and sel:
# kernel medians, then WRITE_SIZE per launch for the default and the
# plain-validity form.
set -o pipefail
mkdir -p gpurun_out/nt
R=${GRAFT_REPO_ROOT:-$PWD}
export MBX_EXPERIMENTS=1 NULLABLE=1 REPS=7
for nt in 0 2 1 3 0 2; do
  echo "NT_OFF=$nt" >> gpurun_out/nt/shapes.log
  MBX_SR_NT_OFF=$nt SHAPES=seln_out,sel timeout -k 10 200 python -u tools/shape_bench.py 1000000000 >> gpurun_out/nt/shapes.log 2>> gpurun_out/nt/err.log || exit 51
done
for nt in 0 2; do
  ( cd /tmp && export TMPDIR=/tmp MBX_SR_NT_OFF=$nt SHAPES=seln_out REPS=4 && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/nt/w$nt -o w -- python3 $R/tools/shape_bench.py 1000000000 >> $R/gpurun_out/nt/pmc.log 2>&1 ) || exit 52
done
echo NT_OK
