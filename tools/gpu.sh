# One GPU pass on the box (gpurun): the steps named in STEPS run in this order,
# each under its own time limit; the chain stops at the first failure.
#   tests     the -m gpu suite (PYTEST_K narrows it)      smoke   __graft_entry__.smoke()
#   bench     the headline line (C2 + C3/sel extras, CPU baseline)
#   configs   bench.py --config c3 / c5 / sel / c4        shards  --shards-per-gpu 2 (c2, c5, c3)
#   c1        bench.py --config c1 (native per-cell and stream loops)
#   overhead  tools/shard_overhead.py                      shapes  tools/shape_bench.py (SHAPES, NULLABLE)
#   layout    tools/c3_layout_probe.py                     rehearse  2 gloo ranks on one GPU (--ranks)
#   prof      rocprofv3 --kernel-trace --stats of bench.py (c2 line with extras)
#   pmc       rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py (C2 line with c3, sel; one counter set per run)
#   pmc5      the same passes of bench.py --config c5 (1.25e9 rows per launch)
#   link      tools/link8_probe (8 MB D2H variants; build it first: see its header)
#   pmcshape  rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE of tools/shape_bench.py (PMC_SHAPES)
#   clock     C3 / C2 / two-array ring with in-kernel clock stamps at 4 launch cadences (tools/c3_clock.py;
#             needs libduckdb_mb_amd_clk.so: make -C duckdb.mbt_amd clockdiag), then a GRBM_GUI_ACTIVE pass
#   seln      NULL-able selection A/B: the default plan vs MBX_SR_NL=$SELN_NL (rocprofv3 stats, alternated twice)
#   apitrace  HIP API + kernel trace of the C2 query loop at 1e6 rows (tools/query_overhead.py)
#   rccl      the RCCL-combine loopback tests and the sharded tests
#   gpuonly   the -m gpu suite alone (as tests, no smoke)
#   gdab      C3 table flush A/B (records vs global atomics), alone and in the C2 line
#   overheadq per-query overhead of the C2 / C3 shapes at 1e6 rows (tools/query_overhead.py)
#   profcost  the per-kernel event profile's cost on the C2 query (tools/profile_cost.py)
#   chunk     the C harness's append_data_chunk ingest under each pinned-staging copy form (MBX_CHUNK_COPY)
#   newcfg    bench.py --config c3n (C3 with NULLs), c3h (wide dense keys) and c3s (sparse keys), HASH_GROUPS keys
#   gdvar     c3n / c3 under each group_direct_lds launch shape (GD_VARIANTS)
#   profh     rocprofv3 kernel trace + stats of the c3h and c3n lines (PROFH_CONFIGS, PROFH_GROUPS)
#   hashab    c3h partitioned (default) vs the hash path (MBX_PART_GROUP=0)
#   pmcnew    FETCH_SIZE / WRITE_SIZE passes of the c3n, c3h and c3s lines
#   inlibn    the in-library --gpus 8 (c2) / 4 (c5, c3) line on one GPU (MBX_BENCH_DEVICE_MOD=1)
# Results go to gpurun_out/ (merged back by gpurun); copy what is judged into profiles/.
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$PWD}
STEPS=${STEPS:-tests,smoke,bench}
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1 || exit 11
fi
if has smoke; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 12
fi
if has bench; then
  timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 13
fi
if has c1; then
  timeout -k 10 200 python bench.py --config c1 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err || exit 24
fi
if has configs; then
  for c in c3 c5 sel; do
    timeout -k 10 300 python bench.py --config $c --extra "" > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 14
  done
  timeout -k 10 400 python bench.py --config c4 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || exit 15
fi
if has shards; then
  for c in c2 c5 c3; do
    timeout -k 10 240 python bench.py --shards-per-gpu 2 --config $c --no-cpu > gpurun_out/bench_${c}_s2.json 2> gpurun_out/bench_${c}_s2.err || exit 16
  done
fi
if has overhead; then
  timeout -k 10 240 python tools/shard_overhead.py > gpurun_out/shard_overhead.json 2> gpurun_out/shard_overhead.err || exit 17
fi
if has shapes; then
  SHAPES=${SHAPES:-seln_out,seln_pred,seln_both,sel,compact,compact2} NULLABLE=1 timeout -k 10 400 python tools/shape_bench.py ${SHAPE_ROWS:-1000000000} > gpurun_out/shapes.json 2> gpurun_out/shapes.err || exit 18
fi
if has layout; then
  timeout -k 10 300 python tools/c3_layout_probe.py > gpurun_out/c3_layout.json 2> gpurun_out/c3_layout.err || exit 19
fi
if has rehearse; then
  for c in c2 c5 c3; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2951${#c} bench.py --ranks --gpus 2 --config $c --dist-backend gloo --no-cpu --steps 10 > gpurun_out/rehearse_n2_$c.json 2> gpurun_out/rehearse_n2_$c.err || exit 20
  done
fi
if has prof; then
  mkdir -p gpurun_out/prof
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/c2 -o c2 -- python3 $R/bench.py --steps 10 --no-cpu > $R/gpurun_out/prof_c2.log 2>&1 ) || exit 21
fi
if has pmc; then
  mkdir -p gpurun_out/pmc
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmc/$ctr -o $ctr -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --extra c3,sel > $R/gpurun_out/pmc_$ctr.log 2>&1 ) || exit 22
  done
fi
if has pmc5; then  # the same two passes of the C5 line (1.25e9 rows per launch: the filter_agg@1250000000 entry)
  mkdir -p gpurun_out/pmc5
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmc5/$ctr -o $ctr -- python3 $R/bench.py --config c5 --steps 5 --warmup 1 --no-cpu > $R/gpurun_out/pmc5_$ctr.log 2>&1 ) || exit 33
  done
fi
if has pmcshape; then  # kernel trace + FETCH_SIZE / WRITE_SIZE passes of tools/shape_bench.py (PMC_SHAPES, 1e9 rows)
  mkdir -p gpurun_out/pmcshape
  export SHAPES=${PMC_SHAPES:-seln_out} NULLABLE=1
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmcshape/trace -o trace -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/pmcshape_trace.log 2>&1 ) || exit 25
  for ctr in FETCH_SIZE WRITE_SIZE; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmcshape/$ctr -o $ctr -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/pmcshape_$ctr.log 2>&1 ) || exit 26
  done
fi
if has clock; then
  mkdir -p gpurun_out/clock
  DUCKDB_MB_AMD_LIB=$R/duckdb.mbt_amd/libduckdb_mb_amd_clk.so timeout -k 10 300 python -u tools/c3_clock.py 15 > gpurun_out/clock/c3_clock.jsonl 2> gpurun_out/clock/c3_clock.err || exit 27
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/clock/grbm -o grbm -- python3 $R/tools/c3_clock.py pmc 15 > $R/gpurun_out/clock/grbm.log 2>&1 ) || exit 28
fi
if has seln; then
  mkdir -p gpurun_out/seln
  for rep in 1 2; do
    for nl in default ${SELN_NL:-4}; do
      ( cd /tmp && export TMPDIR=/tmp MBX_EXPERIMENTS=1 NULLABLE=1 SHAPES=${SHAPES:-seln_out,seln_pred} REPS=7 && if [ $nl != default ]; then export MBX_SR_NL=$nl; fi && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/seln/nl${nl}_$rep -o t -- python3 $R/tools/shape_bench.py 1000000000 > $R/gpurun_out/seln/nl${nl}_$rep.log 2>&1 ) || exit 29
      rm -f $R/gpurun_out/seln/nl${nl}_$rep/*kernel_trace.csv
    done
  done
fi
if has apitrace; then
  mkdir -p gpurun_out/apitrace
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $R/gpurun_out/apitrace/tr -o tr -- python3 $R/tools/query_overhead.py 1000000 > $R/gpurun_out/apitrace/qo.log 2>&1 ) || exit 30
fi
if has rccl; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_rccl_loopback.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rccl_tests.log 2>&1 || exit 31
fi
if has gpuonly; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 32
fi
if has gdab; then  # C3 table flush A/B: per-workgroup records (default) vs global atomics (MBX_GD_ATOMIC_FLUSH=1),
  # alternated, alone (--config c3) and inside the C2 line; results in gpurun_out/gd/
  mkdir -p gpurun_out/gd
  for rep in 1 2; do
    for m in parts atomic; do
      if [ $m = atomic ]; then X="MBX_EXPERIMENTS=1 MBX_GD_ATOMIC_FLUSH=1"; else X=""; fi
      env $X timeout -k 10 200 python bench.py --config c3 --steps 60 --warmup 5 --no-cpu --extra "" > gpurun_out/gd/c3_${m}_$rep.json 2> gpurun_out/gd/c3_${m}_$rep.err || exit 34
      env $X timeout -k 10 300 python bench.py --no-cpu --steps 20 > gpurun_out/gd/c2line_${m}_$rep.json 2> gpurun_out/gd/c2line_${m}_$rep.err || exit 35
    done
  done
fi
if has overheadq; then  # per-query overhead of the C2 and C3 shapes at 1e6 rows (tools/query_overhead.py), twice
  mkdir -p gpurun_out/qo
  for rep in 1 2; do
    timeout -k 10 100 python tools/query_overhead.py 1000000 > gpurun_out/qo/qo_$rep.json 2> gpurun_out/qo/qo_$rep.err || exit 36
  done
fi
if has profcost; then  # what the per-kernel event profile costs the C2 query (tools/profile_cost.py)
  timeout -k 10 300 python tools/profile_cost.py > gpurun_out/profile_cost.json 2> gpurun_out/profile_cost.err || exit 37
fi
if has chunk; then  # the reference-ABI chunk ingest (C harness) under each copy form of the pinned staging
  mkdir -p gpurun_out/chunk
  gcc -O2 -std=c11 -Iinclude tests/c_harness/mb_harness.c -o gpurun_out/chunk/mbh -Lduckdb.mbt_amd -lduckdb_mb_amd -Wl,-rpath,$R/duckdb.mbt_amd || exit 38
  for m in default memcpy sse avx512; do
    if [ $m = default ]; then X=""; else X="MBX_EXPERIMENTS=1 MBX_CHUNK_COPY=$m"; fi
    env $X timeout -k 10 200 gpurun_out/chunk/mbh c4chunk ${CHUNK_ROWS:-100000000} > gpurun_out/chunk/$m.json 2> gpurun_out/chunk/$m.err || exit 39
  done
fi
if has newcfg; then  # the C3-with-NULLs and hash GROUP BY configs
  timeout -k 10 300 python bench.py --config c3n --extra "" > gpurun_out/bench_c3n.json 2> gpurun_out/bench_c3n.err || exit 40
  for g in ${HASH_GROUPS:-100000 1000000}; do
    for c in c3h c3s; do
      timeout -k 10 400 python bench.py --config $c --groups $g --steps ${HASH_STEPS:-10} --warmup 2 --extra "" --cpu-seconds 4 > gpurun_out/bench_${c}_$g.json 2> gpurun_out/bench_${c}_$g.err || exit 41
    done
  done
fi
if has gdvar; then  # C3 / C3-with-NULLs under group_direct_lds launch shapes (MBX_GD_VARIANT), rocprof stats each
  mkdir -p gpurun_out/gdvar
  for v in ${GD_VARIANTS:-d2_g1 d3_g1 d2_g2 d3_g2}; do
    for c in c3n c3; do
      ( cd /tmp && export TMPDIR=/tmp MBX_EXPERIMENTS=1 MBX_GD_VARIANT=$v && timeout -k 10 200 python3 $R/bench.py --config $c --extra "" --no-cpu --steps 20 > $R/gpurun_out/gdvar/${c}_$v.json 2> $R/gpurun_out/gdvar/${c}_$v.err ) || exit 42
    done
  done
fi
if has profh; then  # rocprofv3 kernel trace + stats of the c3h (F3 partitioned GROUP BY) and c3n lines
  mkdir -p gpurun_out/profh
  for c in ${PROFH_CONFIGS:-c3h c3s c3n}; do
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profh/$c -o $c -- python3 $R/bench.py --config $c --groups ${PROFH_GROUPS:-100000} --extra "" --no-cpu --steps 10 > $R/gpurun_out/profh/$c.json 2> $R/gpurun_out/profh/$c.err ) || exit 43
    python3 $R/tools/rocpd_stats.py $R/gpurun_out/profh/$c/${c}_results.db $R/gpurun_out/profh/${c}_kernel_stats.csv || true
  done
fi
if has hashab; then  # the wide-key GROUP BY: partitioned (default) vs the hash path (MBX_PART_GROUP=0), 1e5 keys
  mkdir -p gpurun_out/hashab
  timeout -k 10 300 python bench.py --config c3h --groups 100000 --steps 10 --warmup 2 --extra "" --no-cpu > gpurun_out/hashab/part.json 2> gpurun_out/hashab/part.err || exit 44
  MBX_EXPERIMENTS=1 MBX_PART_GROUP=0 timeout -k 10 300 python bench.py --config c3h --groups 100000 --steps 3 --warmup 1 --extra "" --no-cpu > gpurun_out/hashab/hash.json 2> gpurun_out/hashab/hash.err || exit 45
fi
if has pmcnew; then  # FETCH_SIZE / WRITE_SIZE passes of the c3n, c3h and c3s (1e5 keys) lines
  mkdir -p gpurun_out/pmcnew
  for c in c3n c3h c3s; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $R/gpurun_out/pmcnew/${c}_$ctr -o $ctr -- python3 $R/bench.py --config $c --extra "" --steps 5 --warmup 1 --no-cpu > $R/gpurun_out/pmcnew/${c}_$ctr.log 2>&1 ) || exit 46
    done
  done
fi
if has inlibn; then  # the in-library N-GPU line rehearsed on one GPU (MBX_BENCH_DEVICE_MOD=1: all shards on device 0)
  mkdir -p gpurun_out/inlibn
  MBX_BENCH_DEVICE_MOD=1 timeout -k 10 400 python bench.py --gpus 8 --no-cpu --steps 10 > gpurun_out/inlibn/c2_n8.json 2> gpurun_out/inlibn/c2_n8.err || exit 47
  for c in c5 c3; do
    MBX_BENCH_DEVICE_MOD=1 timeout -k 10 400 python bench.py --gpus 4 --config $c --no-cpu --steps 10 > gpurun_out/inlibn/${c}_n4.json 2> gpurun_out/inlibn/${c}_n4.err || exit 48
  done
fi
if has link; then
  timeout -k 10 200 ./tools/link8_probe ${LINK_MB:-8} 200 > gpurun_out/link8_probe.log 2>&1 || exit 23
fi
echo ALL_OK
