"""normalize(v) == v * RN(1/RN(sqrt(dot(v, v)))) under the numerics contract.
The device computes the reciprocal there with a shortened form of the compiler's correctly
rounded 1.0f / s sequence (raytracing-tests_amd/csrc/rt_math.hpp rcp_sqrt_domain), valid for s
the square root of a float.  It must equal 1.0f / sqrtf(x) for every one of the 2^32 float bit
patterns x (NaN payloads aside), checked on the device by rt_debug_check_fastmath(0)."""
import ctypes as C

import pytest

pytestmark = pytest.mark.gpu


def test_rcp_of_sqrt_matches_correctly_rounded_division_for_all_inputs(gpu):
    import rt_amd as R
    lib = R.load()
    bad = C.c_uint64(0)
    first = C.c_uint32(0)
    assert lib.rt_debug_check_fastmath(0, C.byref(bad), C.byref(first)) == 0
    assert bad.value == 0, f"{bad.value} mismatches, first at bit pattern {first.value:#010x}"
    assert first.value == 0xFFFFFFFF

