set -o pipefail
mkdir -p gpurun_out/r2p
MBX_SR_MIN_ROWS=0 GRID='[{}, {"MBX_SR_PW":4}, {"MBX_SR_PW":1}, {"MBX_SR_S":1}, {"MBX_SR_S":1,"MBX_SR_PW":4}, {"MBX_SR_DEPTH":4}, {"MBX_SR_DEPTH":4,"MBX_SR_PW":4}, {"MBX_SR_SLEEP":0,"MBX_SR_PW":4}]' MBX_SR_DEBUG=1 timeout -k 10 400 python -u tools/sweep_rounds.py 1000000000 sel sel2 sel3 > gpurun_out/r2p/sweep.log 2>gpurun_out/r2p/sweep.err || exit 12
