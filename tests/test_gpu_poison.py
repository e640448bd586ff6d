"""No kernel reads device memory its engine never wrote.

Every engine allocation is filled with a poison byte (internal scotty_debug_alloc_poison, the run-time form of the
SCOTTY_ALLOC_POISON knob, csrc/dev_alloc.h) while these tests create their operators, so a read of never-written
state yields wild indices and values at its first use instead of the zeros a fresh mapping happens to hold.

Regression: the quiet path's ingest kernel read the cell-index metadata (cix_meta) even when the prep kernel had
refused the batch -- the cell-index build then writes no index, so the ingest's window search went to a cix entry
computed from a previous push's index or from never-written memory (slicing_kernels.hip, ingest_kernel; DESIGN.md
§4).  That was the illegal address of test_session_streams_match_oracle[11] in round 3
(profiles/r03/r03r_fault_before_zero_fill.txt), masked by zero-filled allocations until it was found.  The same cases
run here under the poison, with the engines' other paths (grid, count, keyed, event-exact) beside them."""
import ctypes

import pytest

import test_gpu_count
import test_gpu_exact
import test_gpu_parity
from helpers import product

pytestmark = pytest.mark.gpu

POISON = 0xA5


@pytest.fixture
def poisoned():
    L = product().lib()
    f = L.scotty_debug_alloc_poison
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_int]
    prev = f(POISON)
    try:
        yield
    finally:
        f(prev)


@pytest.mark.parametrize("seed", [11, 0, 3, 7, 13, 21])
def test_session_streams_under_poison(poisoned, seed):
    test_gpu_exact.test_session_streams_match_oracle(seed)


@pytest.mark.parametrize("seed", [0, 1, 5])
def test_quiet_and_event_exact_paths_under_poison(poisoned, seed):
    test_gpu_exact.test_quiet_path_equals_event_exact_path_and_replay(product(), seed)


@pytest.mark.parametrize("seed", [0, 2, 3])
def test_lazy_and_count_windows_under_poison(poisoned, seed):
    test_gpu_exact.test_lazy_session_slices_match_oracle(seed)
    test_gpu_exact.test_out_of_order_count_windows_match_oracle(seed)


@pytest.mark.parametrize("seed", [0, 1, 3])
def test_keyed_under_poison(poisoned, seed):
    test_gpu_exact.test_keyed_streams_match_per_key_oracles(product(), seed)
    test_gpu_exact.test_keyed_out_of_order_count_windows_match_per_key_oracles(product(), seed)


def test_grid_and_count_paths_under_poison(poisoned):
    test_gpu_parity.test_config3_sliding_1000_concurrent_out_of_order_min_max()
    test_gpu_parity.test_slice_compaction_keeps_window_assembly_exact()
    test_gpu_count.test_count_path_matches_oracle(0)
    test_gpu_count.test_count_and_time_windows_on_count_path_match_oracle(product(), 1)


def test_poison_knob_round_trip():
    """The internal setter returns the previous setting; -1 switches the poison off."""
    L = product().lib()
    f = L.scotty_debug_alloc_poison
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_int]
    prev = f(0x5A)
    assert f(-1) == 0x5A
    assert f(prev) == -1
