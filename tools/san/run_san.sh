#!/bin/bash
# The CPU test suite's host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only;
# no GPU code runs under a sanitizer).  Builds the host-sanitized product library
# (raytracing-tests_amd/librt_hip_san.so: the scene library, packers, LBVH / SAH / 4-wide builders,
# RI grid, presets, tile spiral) and the oracle (oracle/librt_oracle_san.so), both with the ROCm
# clang so that one sanitizer runtime serves both, then runs the CPU tests that exercise them.
#   bash tools/san/run_san.sh [log]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
LOG=${1:-$ROOT/profiles/r04_sanitizer_cpu.log}
make -C "$ROOT/raytracing-tests_amd" -j8 san > /dev/null || exit 1
make -C "$ROOT/oracle" san > /dev/null || exit 1
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
[ -f "$RT" ] || RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
{
  echo "# $(date -u) host sanitizer run: ASan + UBSan (-fno-sanitize-recover=undefined), runtime $RT"
  echo "# libraries: raytracing-tests_amd/librt_hip_san.so, oracle/librt_oracle_san.so"
  cd "$ROOT" && LD_PRELOAD="$RT" LD_LIBRARY_PATH=/opt/rocm/lib/llvm/lib:$LD_LIBRARY_PATH \
    ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1:detect_odr_violation=0 \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    RT_HIP_LIB="$ROOT/raytracing-tests_amd/librt_hip_san.so" RT_ORACLE_LIB="$ROOT/oracle/librt_oracle_san.so" \
    OMP_NUM_THREADS=4 \
    timeout -k 10 1500 python -m pytest -q -p no:cacheprovider -m "not gpu" \
      tests/test_host_logic.py tests/test_oracle_golden.py tests/test_oracle_kat.py tests/test_progressive.py \
      tests/test_textures.py tests/test_stages_oracle.py tests/test_abi.py tests/test_multiproc.py tests/test_time_bins.py 2>&1
  echo "# exit status $?"
} > "$LOG" 2>&1
tail -3 "$LOG"
grep -c "ERROR: AddressSanitizer\|runtime error:" "$LOG" && exit 1
exit 0
