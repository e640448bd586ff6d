"""CPU-only checks of the product boundary: the gfx950 library builds, loads without a GPU and exports
every entry point include/scotty_mi355x.h declares (no compute calls)."""
import ctypes
import os
import subprocess

import pytest

from helpers import product, ROOT


@pytest.fixture(scope="module")
def pkg():
    p = product()
    if not os.path.exists(p.LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(p.LIB_PATH)])
    return p


def test_library_exports_every_header_symbol(pkg):
    names = pkg.header_functions()
    assert len(names) >= 15
    L = ctypes.CDLL(pkg.LIB_PATH)
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_library_is_gfx950_code_object(pkg):
    blob = open(pkg.LIB_PATH, "rb").read()
    assert b".hip_fatbin" in blob and b"hipv4-amdgcn-amd-amdhsa--gfx950" in blob


def test_no_cpu_fallback_without_gpu(pkg):
    """The product path must fail loudly instead of computing on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg.ScottyError):
        pkg.SlicingWindowOperator()


def test_header_constants_match_oracle():
    import specs
    from oracle import oracle as O
    txt = open(os.path.join(ROOT, "include", "scotty_mi355x.h")).read()
    for name, val in [("SCOTTY_AGG_SUM_I32", specs.SUM), ("SCOTTY_AGG_COUNT", specs.COUNT),
                      ("SCOTTY_AGG_MIN_I32", specs.MIN), ("SCOTTY_AGG_MAX_I32", specs.MAX),
                      ("SCOTTY_AGG_SUM_F64", O.AGG_SUM_F64), ("SCOTTY_WIN_SLIDING", O.WIN_SLIDING),
                      ("SCOTTY_WIN_FIXED_BAND", O.WIN_FIXED_BAND)]:
        assert "#define %s %d" % (name, val) in txt, name


def test_java_random_restatement():
    """java.util.Random known answers: new Random(42).nextInt() == -1170105035, nextInt(10) sequence,
    and the C2 window sizes start like BenchmarkRunner.randomTumbling(1000,1,20) with Random(10)."""
    w = product().workloads
    r = w.JavaRandom(42)
    assert r.nextInt() == -1170105035
    assert r.nextInt() == 234785527
    r = w.JavaRandom(42)
    assert [r.nextInt(10) for _ in range(5)] == [0, 3, 8, 4, 0]
    r = w.JavaRandom(0)
    assert abs(r.nextDouble() - 0.730967787376657) < 1e-15
    sizes = w.random_tumbling_sizes()
    assert len(sizes) == 1000 and min(sizes) >= 1000 and max(sizes) < 20000
