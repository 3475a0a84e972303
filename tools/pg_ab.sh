# A/B of a partitioned GROUP BY knob: c3h / c3s at each PG_GROUPS, the default
# plan vs MBX_EXPERIMENTS=1 $PG_KNOB (kernel split per step from the bench line)
set -o pipefail
mkdir -p gpurun_out/pgab
for g in ${PG_GROUPS:-100000 1000000}; do
  for c in c3h c3s; do
    for m in default knob; do
      if [ $m = knob ]; then X="MBX_EXPERIMENTS=1 $PG_KNOB"; else X=""; fi
      env $X timeout -k 10 300 python bench.py --config $c --groups $g --steps 10 --warmup 2 --extra "" --no-cpu > gpurun_out/pgab/${c}_${g}_$m.json 2> gpurun_out/pgab/${c}_${g}_$m.err || exit 3
    done
  done
done
echo ok
