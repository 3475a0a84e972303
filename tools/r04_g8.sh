# storer copy-form A/B on the NULL-able output shape (MBX_SR_COPY1: 0 = 4 rows
# per lane with partial passes and 4-byte validity stores, 1 = one row per
# lane, 2 = 4 rows per lane with byte validity stores), with the role split.
set -o pipefail
mkdir -p gpurun_out/g8
export MBX_EXPERIMENTS=1 NULLABLE=1
for c in 0 1 2 0 1 2; do
  echo "== COPY1=$c" >> gpurun_out/g8/ab.log
  MBX_SR_COPY1=$c REPS=5 SHAPES=seln_out,seln_pred timeout -k 10 200 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g8/ab.log 2>&1 || exit 101
done
for c in 0 1 2; do
  echo "== DEBUG COPY1=$c" >> gpurun_out/g8/dbg.log
  MBX_SR_DEBUG=1 MBX_SR_COPY1=$c REPS=2 SHAPES=seln_out timeout -k 10 200 python -u tools/shape_bench.py 1000000000 >> gpurun_out/g8/dbg.log 2>&1 || exit 102
done
echo G8_OK
