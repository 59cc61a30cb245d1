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


@pytest.mark.parametrize("offset,records,group", [(0, 7, 3), (1, 5, 1), (3, 4, 6), (8, 3, 8)])
def test_record_major_window_is_the_stream(offset, records, group):
    """uwvk_synth_normal_at: a window of each instance's stream, written
    [record][instance][group], is bitwise the same variates as the full rows."""
    full = synth.normals(synth.SEED, 5, 9, 4, (offset + records * group,))
    rec = synth.normals_rec(synth.SEED, 5, 9, 4, offset, records, group)
    want = full[:, offset:].reshape(9, records, group).transpose(1, 0, 2)
    np.testing.assert_array_equal(rec, want)


def test_log_segments_are_slices_of_the_mission():
    """make_pose_log(epoch0=...) draws epochs [epoch0, epoch0 + n) of the whole
    mission: the same flags, IMU rows and low-rate samples (re-indexed from the
    segment's first sample) -- the long C4 window is generated in segments."""
    kw = dict(dropout_on=0.3, dropout_off=0.2, adcp_every=250)
    full = synth.make_pose_log(6, 1200, "C4", **kw)
    for e0, n in ((0, 400), (400, 401), (801, 399)):
        s = synth.make_pose_log(6, n, "C4", epoch0=e0, **kw)
        for k in ("flags", "gyro", "acc"):
            np.testing.assert_array_equal(s[k], full[k][e0:e0 + n])
        for key, ix in (("dvl", "dvl_index"), ("pressure", "pressure_index"), ("adcp", "adcp_index"),
                        ("efforts", "efforts_index")):
            fi, si = full[ix][e0:e0 + n], s[ix]
            np.testing.assert_array_equal(si >= 0, fi >= 0)
            sel = fi >= 0
            np.testing.assert_array_equal(s[key][si[sel]], full[key][fi[sel]])
        np.testing.assert_array_equal(s["pos0"], full["pos0"])
