# C3 placement with the VMM-backed pool blocks (MBX_VMM_MIN_MB=1024) vs
# hipMalloc, alone and after the C2 table, alternated; the hot-path tests with
# the VMM blocks on.
set -o pipefail
mkdir -p gpurun_out/g17
export MBX_EXPERIMENTS=1
MBX_VMM_MIN_MB=1024 timeout -k 10 400 python -u -m pytest tests/test_gpu_hotpath.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/g17/tests_vmm.log 2>&1 || exit 191
for rep in 1 2; do
  for vmm in 0 1024; do
    for mode in alone after_c2; do
      echo "vmm=$vmm" >> gpurun_out/g17/times.jsonl
      MBX_VMM_MIN_MB=$vmm timeout -k 10 200 python -u tools/c3_tlb_probe.py $mode 10 >> gpurun_out/g17/times.jsonl 2>> gpurun_out/g17/err.log || exit 192
    done
  done
done
echo G17_OK
