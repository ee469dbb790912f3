#!/bin/bash
# Rebuild the product library and the diagnostic / experiment variants used by tools/gpu/r04_*.sh
set -e
cd "$(dirname "$0")/.."
make -C raytracing-tests_amd -j8 2>&1 | grep -E " error|warning: (?!failed to meet)" || true
make -C raytracing-tests_amd -j8 variant VARIANT=occ VDEFS=-DRT_DIAG_OCC > /dev/null 2>&1
ls -la raytracing-tests_amd/*.so
make -C raytracing-tests_amd -j8 variant VARIANT=park VDEFS=-DRT_INW_PARK > /dev/null 2>&1
make -C raytracing-tests_amd -j8 variant VARIANT=park16 VDEFS="-DRT_INW_PARK -DRT_INW_PARK_LANES=16" > /dev/null 2>&1
make -C raytracing-tests_amd -j8 variant VARIANT=park4m8 VDEFS="-DRT_INW_PARK -DRT_INW_PARK_LANES=4 -DRT_INW_PARK_MIN=8" > /dev/null 2>&1
ls -la raytracing-tests_amd/*.so
