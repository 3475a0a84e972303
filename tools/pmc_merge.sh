# Copies the FETCH_SIZE / WRITE_SIZE counter collections of `STEPS=pmc,pmc5,pmcnew tools/gpu.sh`
# from gpurun_out/ into profiles/r06_final/pmc/ (our kernels' rows only) and merges them into
# profiles/pmc_traffic.json (tools/pmc_traffic.py, stamped with the sources' digest)
set -e
P=profiles/r06_final/pmc
mkdir -p $P
for d in pmc pmc5; do for c in FETCH_SIZE WRITE_SIZE; do cp gpurun_out/$d/$c/${c}_counter_collection.csv $P/${d}_${c,,}.csv; done; done
for c3 in c3n c3h c3s; do for c in FETCH_SIZE WRITE_SIZE; do cp gpurun_out/pmcnew/${c3}_$c/${c}_counter_collection.csv $P/${c3}_${c,,}.csv; done; done
python3 - <<'PY'
import csv, glob
keep = ("filter_agg_lds", "group_direct_lds", "select_rounds", "pg_hist", "pg_scatter", "pg_reduce", "pg_hscatter", "pg_hreduce")
for f in glob.glob("profiles/r06_final/pmc/*.csv"):
    rows = list(csv.DictReader(open(f)))
    fn = rows[0].keys()
    rows = [r for r in rows if any(k in r["Kernel_Name"] for k in keep)]
    with open(f, "w", newline="") as o:
        w = csv.DictWriter(o, fieldnames=fn)
        w.writeheader()
        w.writerows(rows)
PY
for c in fetch write; do
  python3 tools/pmc_traffic.py $P/pmc_${c}_size.csv filter_agg=filter_agg_lds_kernel group_direct=group_direct_lds_kernel select_rounds=select_rounds_kernel > /dev/null
  python3 tools/pmc_traffic.py $P/pmc5_${c}_size.csv filter_agg@1250000000=filter_agg_lds_kernel > /dev/null
  python3 tools/pmc_traffic.py $P/c3n_${c}_size.csv group_direct_nulls=group_direct_lds_kernel > /dev/null
  python3 tools/pmc_traffic.py $P/c3h_${c}_size.csv pg_hist=pg_hist_kernel pg_scatter=pg_scatter_kernel pg_reduce=pg_reduce_kernel > /dev/null
  python3 tools/pmc_traffic.py $P/c3s_${c}_size.csv pg_hist_hashed=pg_hist_kernel pg_hscatter=pg_hscatter_kernel pg_hreduce=pg_hreduce_kernel > /dev/null
done
echo merged
