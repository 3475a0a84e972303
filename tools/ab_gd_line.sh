# A/B of the C3 flush inside the C2 line (C3's table built after C2's): records
# (default) vs global atomics (MBX_EXPERIMENTS=1 MBX_GD_ATOMIC_FLUSH=1), alternated.
set -o pipefail
mkdir -p gpurun_out/gdl
for rep in 1 2; do
  for m in parts atomic; do
    if [ $m = atomic ]; then X="MBX_EXPERIMENTS=1 MBX_GD_ATOMIC_FLUSH=1"; else X=""; fi
    env $X timeout -k 10 300 python bench.py --no-cpu --steps 20 > gpurun_out/gdl/c2_${m}_$rep.json 2> gpurun_out/gdl/c2_${m}_$rep.err || exit 12
  done
done
echo AB_OK
