set -o pipefail
mkdir -p gpurun_out
(lscpu | head -20; nproc; grep -c processor /proc/cpuinfo; grep -m1 -o -w fma /proc/cpuinfo) > gpurun_out/host.txt 2>&1
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 1000 python -m pytest tests/test_gpu_parity.py -q -s -p no:cacheprovider > gpurun_out/t1.log 2>&1
