# parity (all strategies), then bench variants at the full config
set -o pipefail
mkdir -p gpurun_out
B="python bench.py --steps 2 --warmup 0 --no-cpu-baseline"
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/parity.log 2>&1 &&
timeout -k 10 300 $B > gpurun_out/v_default.json 2> gpurun_out/err.log &&
RT_IOW_NARROW=1 timeout -k 10 300 $B > gpurun_out/v_narrow.json 2>> gpurun_out/err.log &&
timeout -k 10 300 $B --occupancy > gpurun_out/v_default_occ.json 2>> gpurun_out/err.log
