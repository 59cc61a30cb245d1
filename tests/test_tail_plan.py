"""Host logic of the last-generation spreading planner (UWVK_OPT_TAIL_SLOTS,
csrc/uwvk_psp_k.hip plan_tail), through the host-only C-ABI query; no device
work.  A Python twin of the planner's cost model (count / (2 C) + 0.75 C (C - 1)
epochs of ramp + extra block overhead, against count / 2 unspread) and of the
kernel's block layout (tail_unit)."""
import os

import pytest

from uwvk import engine


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(engine.LIB_PATH):
        pytest.skip("libuwvk.so not built")
    return engine.lib()


def twin_chunks(n, s, count):
    if s <= 0 or count < 4:
        return 1
    best, ch = 0.45 * count, 1
    for c in range(2, 9):
        if 2 * c > count or n < (c + 1) * s:
            break
        cost = count / (2.0 * c) + 0.75 * c * (c - 1)
        if cost < best:
            best, ch = cost, c
    return ch


def layout(n, s, c):
    """(local instance, chunk) per XCD block position, as tail_unit decodes it."""
    if c <= 1:
        return [(i, -1) for i in range(n)]
    m = c * s
    t0 = n - m
    return [(i, -1) if i < t0 else (t0 + (i - t0) % m, (i - t0) // m) for i in range(n + (c - 1) * m)]


def test_no_spreading_when_it_cannot_pay(L):
    assert L.uwvk_pose_tail_chunks(8192, 384, 3) == 1     # too few epochs to split
    assert L.uwvk_pose_tail_chunks(700, 384, 200) == 1    # under 3 generations
    assert L.uwvk_pose_tail_chunks(8192, 0, 200) == 1     # unknown occupancy


@pytest.mark.parametrize("n,s,count", [(8192, 384, 200), (8192, 384, 20), (8192, 384, 5), (16384, 384, 2000),
                                       (20, 3, 200), (12, 3, 20), (12, 2, 600), (16, 3, 37), (16, 3, 363),
                                       (9, 2, 9), (1200, 384, 200)])
def test_planner_matches_its_twin(L, n, s, count):
    assert L.uwvk_pose_tail_chunks(n, s, count) == twin_chunks(n, s, count)


def test_bench_shapes(L):
    # 65,536 instances: 8,192 per XCD over 384 slots (12 per CU x 32 CUs)
    assert L.uwvk_pose_tail_chunks(8192, 384, 20) == 2
    assert L.uwvk_pose_tail_chunks(8192, 384, 200) == 4


@pytest.mark.parametrize("n,s,c", [(8192, 384, 3), (8192, 384, 8), (20, 3, 5), (9, 2, 2)])
def test_layout_covers_every_epoch_once_in_order(n, s, c):
    seen = {}
    for i, (j, k) in enumerate(layout(n, s, c)):
        assert (j, k) not in seen
        if k > 0:
            assert i - seen[(j, k - 1)] == c * s  # predecessor one chunk group (m blocks) earlier
        seen[(j, k)] = i
    whole = {j for (j, k) in seen if k < 0}
    chunked = {j for (j, k) in seen if k >= 0}
    assert whole | chunked == set(range(n)) and not whole & chunked
    for j in chunked:
        assert all((j, k) in seen for k in range(c))
