set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 120 ./tools/c3_probe 1000000000 w > gpurun_out/probe/c3_probe_w.log 2>&1 || exit 11
