set -o pipefail
mkdir -p gpurun_out/probe
export C4P_GRID=1
timeout -k 10 300 python3 -u tools/c4_probe.py > gpurun_out/probe/c4_probe.log 2>&1 || exit 12
