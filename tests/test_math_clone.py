"""The device's glibc-clone logf/sinf/cosf equal the host glibc on every input the integrator can
produce: x = 1 - u and phi = 2*pi*u for every value of uniform<float>() (random.hpp:107-111)."""
import pytest

import hostsim_lib as HS


@pytest.mark.parametrize("which,name", [(0, "logf(1-u)"), (1, "sinf(2*pi*u)"), (2, "cosf(2*pi*u)"),
                                       (3, "sincosf(2*pi*u) fused")])
def test_clone_equals_glibc_exhaustive(which, name):
    assert HS.lib().vpths_math_mismatches(which) == 0, name


@pytest.mark.slow
def test_pow2_is_square():
    # std::pow(x, 2.0f) (random.hpp:58,64,66; utils.hpp:45,50) == x*x for all finite floats
    assert HS.lib().vpths_pow2_mismatches() == 0
