set -o pipefail
mkdir -p gpurun_out/shapes
JIT_WAIT=3 SHAPES=c2_count,c3,c3_where,c3_where2,filter_multi,filter_multi3,multi_key,c3_jit,c3_where_jit,sel,sel2,sel3,compact,compact2 timeout -k 10 500 python -u tools/shape_bench.py 1000000000 > gpurun_out/shapes/shapes_1e9.log 2>&1 || exit 11
NULLABLE=1 SHAPES=c2n,c5n,c5n_sumv,c3n,c3n_where,seln_pred,seln_out,seln_both timeout -k 10 500 python -u tools/shape_bench.py 1000000000 > gpurun_out/shapes/shapes_nullable_1e9.log 2>&1 || exit 12
