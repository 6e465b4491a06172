"""Device self-tests of building blocks whose exact behaviour the parity depends on."""
import ctypes as C

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("which", [0, 1, 2, 3, 4],
                         ids=["chain_cmp_by_pos", "chain_cmp_by_MEM_score", "chain_cmp_by_score",
                              "Anchor_cmp_by_chr_ID_and_pos", "MEM_rst_cmp_by_match_len"])
@pytest.mark.parametrize("n", [2, 3, 7, 64, 400])
def test_glibc_msort_restatement_same_on_device_and_host(pyd, which, n):
    """dsb_msort (glibc 2.35 msort_with_tmp restated) gives the host permutation on gfx950.
    which=0 pins the hipcc mis-scheduling of the early-return comparator form."""
    f = pyd.lib().dsb_gpu_selftest_sort
    f.argtypes = [C.c_uint32, C.c_uint32, C.c_int, C.c_uint32]
    f.restype = C.c_int
    assert f(n, 512, which, 1000 + n) == 0
