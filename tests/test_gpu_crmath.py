"""GPU verification of the correctly rounded division / sqrt cores the exact kernel uses
(black_hole_ray_marching_amd/csrc/bh_crmath.hpp) against hipcc's IEEE operations, on device.

Exhaustive where the domain is 1-D (sqrt over every non-negative float bit pattern; x/6 over all
2^32 patterns); for n/d, every numerator significand against blocks of denominator significands
(the whole 2^46 square is tools/ubench/cr_forms.hip, log in profiles/r01_cr_forms.log), plus 2^31
random pairs over the guarded exponent range and 2^30 near-exact quotients."""
import ctypes as C

import pytest

import black_hole_ray_marching_amd as bh

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return bh.load()


def run(lib, op, base, count):
    mism = C.c_uint64()
    ex = (C.c_uint32 * 8)()
    st = lib.bh_selftest_crmath(op, base, count, C.byref(mism), ex, 0)
    assert st == 0
    return mism.value, [hex(v) for v in ex]


def test_sqrt_core_exhaustive(lib):
    # every non-negative pattern from +0 up to +inf (the guard sends x < 2^-96 and +inf to IEEE sqrt)
    m, ex = run(lib, 0, 0, 0x7F800001)
    assert m == 0, ex


def test_div6_exhaustive(lib):
    m, ex = run(lib, 1, 0, 1 << 32)
    assert m == 0, ex


def test_div_core_random(lib):
    m, ex = run(lib, 2, 12345, 1 << 31)
    assert m == 0, ex


@pytest.mark.parametrize("d0", [0, 0x3A5F00, 0x7FFFC0])
def test_div_core_significand_blocks(lib, d0):
    # 64 denominator significands (incl. 1.0, and the all-ones fraction at 0x7FFFFF) x all 2^23
    # numerator significands
    m, ex = run(lib, 7, d0, 64 << 23)
    assert m == 0, ex


def test_rcp_from_rsq_is_not_exact(lib):
    """A measured negative result kept as a guard against reusing it: the reciprocal of rd_derivative's Q
    seeded from the square-root core's v_rsq (y^5, one refinement; BH_RCP_SEED, off) is RN(1/Q) except for a
    few hundred near-midpoint Q (op 12), and with those the one-correction division misses the IEEE quotient
    for some numerators (op 13) -- which is why the march keeps the v_rcp form (bh_crmath.hpp)."""
    lo, hi = 0x37000000, 0x4C000000  # bits of 2^-17 and 2^25: every q whose Q passes the division guard
    m12, _ = run(lib, 12, lo, hi - lo)
    m13, ex = run(lib, 13, lo, hi - lo)
    assert 0 < m12 < 4096 and m13 > 0, (m12, m13, ex)


def test_div_core_near_exact_quotients(lib):
    m, ex = run(lib, 3, 777, 1 << 30)
    assert m == 0, ex


def test_srgb_encode_exhaustive(lib):
    # the BGRA8 encoder (hardware log2/exp2 estimate + threshold fix-up) over all 2^32 patterns
    m, ex = run(lib, 4, 0, 1 << 32)
    assert m == 0, ex


def test_div12_exhaustive(lib):
    # x / 12 of the bloom chain's up-sampling filter, over all 2^32 patterns in the guarded domain
    m, ex = run(lib, 5, 0, 1 << 32)
    assert m == 0, ex


def test_srgb_encode_table_form_exhaustive(lib):
    # the bloom chain's log-free encoder (bucket base codes + one threshold) over all 2^32 patterns
    m, ex = run(lib, 6, 0, 1 << 32)
    assert m == 0, ex


def test_srgb_encode_code_table_form_exhaustive(lib):
    # the code-table form (one read per channel: base code | the bucket's threshold low bits) over all 2^32
    # patterns; a bucket holding two thresholds would also count as a mismatch
    m, ex = run(lib, 10, 0, 1 << 32)
    assert m == 0, ex


def test_atan2_core_against_the_library(lib):
    """The shading's f32-rounded atan2 (bh_crmath.hpp atan2_core + the library fallback where it flags a
    near-midpoint angle) equals (float)atan2((double)y, (double)x) on 2^29 pairs: unit vectors as the
    shading sees them, random magnitudes, zeros, axes and diagonals."""
    m, ex = run(lib, 8, 20261016, 1 << 29)
    assert m == 0, ex


def test_atan2_core_fallback_is_rare(lib):
    """Unit vectors handed to the library call: ~2e-6 of them (2^28 x 10/16 pairs; profiles/r02b)."""
    n = 1 << 28
    m, _ = run(lib, 9, 7, n)
    assert m < n * 10 // 16 * 1e-5, m


def test_wave_max_dpp(lib):
    # the tile-cost reduction of the march kernel (bh_common.hpp wave_max_u32: DPP row_shr / row_bcast
    # scan) against a serial max over the 64 lanes, 64 rounds of random values on every wave of the grid
    m, ex = run(lib, 11, 0x5EED, 64)
    assert m == 0, ex
