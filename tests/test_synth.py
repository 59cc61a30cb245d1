"""Synthetic-log noise (uwvk_synth_normal, csrc/uwvk_synth.cpp): the C generator
agrees with its numpy restatement, is counter-based (a shard draws bitwise the
rows of the full batch, which the instance-sharded multi-GPU runs rely on) and
has standard-normal moments.  CPU only (host code of libuwvk.so)."""
import os

import numpy as np
import pytest

from uwvk import engine, synth

pytestmark = pytest.mark.skipif(not os.path.exists(engine.LIB_PATH), reason="libuwvk.so not built")


def test_c_generator_matches_numpy_twin():
    a = synth._normal_lib(synth.SEED, 3, 257, 5, 101)
    b = synth._normal_np(synth.SEED, np.arange(3, 260), 5, 101)
    np.testing.assert_allclose(a, b, rtol=0, atol=1e-14)


@pytest.mark.parametrize("lo,hi", [(0, 1), (17, 300), (4095, 4097)])
def test_shard_rows_are_bitwise_the_full_batch(lo, hi):
    full = synth.normals(synth.SEED, 0, 4100, 2, (7, 3))
    part = synth.normals(synth.SEED, lo, hi - lo, 2, (7, 3))
    np.testing.assert_array_equal(part, full[lo:hi])


def test_streams_and_instances_differ():
    a = synth.normals(synth.SEED, 0, 2, 0, (1000,))
    b = synth.normals(synth.SEED, 0, 2, 1, (1000,))
    assert abs(np.corrcoef(a[0], a[1])[0, 1]) < 0.1 and abs(np.corrcoef(a[0], b[0])[0, 1]) < 0.1


def test_moments():
    x = synth.normals(1, 0, 500, 0, (8000,)).ravel()
    n = x.size
    assert abs(x.mean()) < 5 / np.sqrt(n)
    assert abs(x.var() - 1) < 5 * np.sqrt(2 / n)
    assert abs((x ** 4).mean() - 3) < 5 * np.sqrt(96 / n)


def test_log_shards_concatenate():
    full = synth.make_pose_log(12, 30, "C4", dropout_on=0.01, dropout_off=0.01)
    a = synth.make_pose_log(5, 30, "C4", dropout_on=0.01, dropout_off=0.01)
    b = synth.make_pose_log(7, 30, "C4", dropout_on=0.01, dropout_off=0.01, first_instance=5)
    for k in ("gyro", "acc", "dvl", "pressure", "efforts"):
        np.testing.assert_array_equal(np.concatenate([a[k], b[k]], axis=-2 if k != "pressure" else -1), full[k])
