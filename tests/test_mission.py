"""Recorded-mission ingestion (uwvk_schedule_streams, uwvk_adcp_cell_weighting,
uwvk.mission): the stream-aligner replay the reference leaves to its caller
(DESIGN.md §11).

CPU: the native scheduler is integer/index work and is held bit-exact to
  (a) the synthetic logs' own epoch schedule (stamps k*dt, C3 and C4), and
  (b) an independent numpy restatement on random jittered stamps with
      collisions, early and late samples.
GPU (-m gpu): a jittered recording replayed through the HIP engine matches the
oracle replaying the same scheduled log (fp64 log tolerance 1e-7)."""
import os

import numpy as np
import pytest

import oracle_ctypes as O
from helpers import cov_err, state_err
from uwvk import abi, engine, mission, synth

LIB = os.path.exists(engine.LIB_PATH)
pytestmark = pytest.mark.skipif(not LIB, reason="libuwvk.so not built")


def ref_place(imu, t, eps):
    """numpy restatement of the per-sensor placement rule."""
    E = len(imu)
    idx = np.full(E, -1, np.int32)
    nxt, row, dropped = 0, 0, 0
    for ts in t:
        if not ts >= imu[0] - eps:
            dropped += 1
            continue
        e = int(np.searchsorted(imu, ts - eps, side="left"))
        at = max(e, nxt)
        if at >= E:
            dropped += 1
            continue
        idx[at] = row
        row += 1
        nxt = at + 1
    return idx, dropped


def stamps_of(log, bit):
    k = np.arange(1, log["epochs"] + 1)
    return k[(log["flags"] & bit) != 0] * log["dt"]


@pytest.mark.parametrize("mode", ["C3", "C4"])
def test_schedule_reproduces_synthetic_log(mode):
    log = synth.make_pose_log(2, 6000, mode, dropout_on=2.0, dropout_off=1.0, efforts_velocity_only=True)
    E, dt = log["epochs"], log["dt"]
    t = np.arange(1, E + 1) * dt
    eff = (log["flags"] & abi.EV_EFFORTS) != 0
    s = mission.schedule(t, stamps_of(log, abi.EV_DVL), stamps_of(log, abi.EV_PRESSURE),
                         stamps_of(log, abi.EV_ADCP), stamps_of(log, abi.EV_EFFORTS),
                         efforts_velocity_only=((log["flags"][eff] & abi.EV_EFFORTS_VELOCITY_ONLY) != 0))
    assert s["epochs"] == E and abs(s["dt"] - dt) < 1e-15
    np.testing.assert_array_equal(s["flags"], log["flags"])
    for k in mission.SENSORS:
        np.testing.assert_array_equal(s[k + "_index"], log[k + "_index"])
    assert not s["dropped"].any()
    if mode == "C4":
        assert s["kept"].all()


def test_schedule_matches_numpy_restatement():
    rng = np.random.default_rng(7)
    E, dt = 3000, 1e-3
    imu = 100.0 + np.arange(E) * dt + rng.uniform(-2e-5, 2e-5, E)
    streams = {}
    for k, n in (("dvl", 30), ("pressure", 80), ("adcp", 6), ("efforts", 40)):
        t = np.sort(rng.uniform(imu[0] - 0.01, imu[-1] + 0.01, n))
        t[5:8] = t[5]  # three samples in one epoch: queued
        t[-3:] = imu[-1] + 0.005  # past the end: queued beyond the last epoch -> dropped
        streams[k] = t
    evo = rng.integers(0, 2, len(streams["efforts"])).astype(bool)
    s = mission.schedule(imu, streams["dvl"], streams["pressure"], streams["adcp"], streams["efforts"],
                         efforts_velocity_only=evo, dt_tolerance=0.05, time_epsilon=1e-9)
    flags = np.full(E, abi.EV_ACC, np.uint32)
    for j, (k, bit) in enumerate((("dvl", abi.EV_DVL), ("pressure", abi.EV_PRESSURE), ("adcp", abi.EV_ADCP),
                                  ("efforts", abi.EV_EFFORTS))):
        idx, dropped = ref_place(imu, streams[k], 1e-9)
        np.testing.assert_array_equal(s[k + "_index"], idx)
        assert s["dropped"][j] == dropped and s["kept"][j] == len(streams[k]) - dropped
        flags[idx >= 0] |= bit
        if k == "efforts":
            first = int(np.searchsorted(streams[k], imu[0] - 1e-9))
            rows = idx[idx >= 0]
            flags[np.flatnonzero(idx >= 0)[evo[first + rows]]] |= abi.EV_EFFORTS_VELOCITY_ONLY
        # queueing keeps every placed sample at or after its own stamp
        at = np.flatnonzero(idx >= 0)
        assert (np.diff(at) > 0).all()
    np.testing.assert_array_equal(s["flags"], flags)
    assert s["dropped"].min() >= 3


def test_schedule_rejects_bad_streams():
    t = np.arange(100) * 1e-3
    bad = t.copy()
    bad[50:] += 5e-3  # a 6 ms gap in a 1 kHz stream
    with pytest.raises(engine.UWVKError) as e:
        mission.schedule(bad)
    assert e.value.code == 1
    with pytest.raises(engine.UWVKError):
        mission.schedule(t, dvl_t=np.array([0.05, 0.01]))  # not ascending
    with pytest.raises(engine.UWVKError):
        mission.schedule(t[::-1])
    s = mission.schedule(t[:1], dvl_t=np.array([0.0, 0.0]))  # one epoch: second sample queued out
    assert s["epochs"] == 1 and s["kept"][0] == 1 and s["dropped"][0] == 1


def test_cell_weighting():
    wv = synth.default_pose_config().water_velocity
    wv.cell_size, wv.first_cell_blank, wv.minimum_correlation = 2.0, 0.5, 0.6
    w, v = mission.cell_weighting(wv, 4, correlation=[0.9, 0.6, 0.59, 1.0])
    np.testing.assert_allclose(w, [0.0, 1.0 / 3.0, 2.0 / 3.0, 1.0], rtol=0, atol=1e-15)
    np.testing.assert_array_equal(v, [True, True, False, True])
    w1, v1 = mission.cell_weighting(wv, 1)
    assert w1[0] == 0.0 and v1.all()
    with pytest.raises(engine.UWVKError):
        mission.cell_weighting(wv, 0)


def jittered_mission(batch, epochs, seed=3, collide=True):
    """A C4 synthetic log re-expressed as stamped sensor streams with clock
    jitter: every sample stamped up to 0.9 dt before its epoch's IMU stamp."""
    log = synth.make_pose_log(batch, epochs, "C4", dropout_on=0.5, dropout_off=0.2, adcp_every=200)
    rng = np.random.default_rng(seed)
    E, dt = log["epochs"], log["dt"]
    imu = 50.0 + np.arange(1, E + 1) * dt + rng.uniform(-1e-5, 1e-5, E)

    def st(bit):
        at = np.flatnonzero((log["flags"] & bit) != 0)
        return imu[at] - rng.uniform(0.0, 0.9 * dt, len(at))

    dvl_t, dvl_mu = st(abi.EV_DVL), log["dvl"]
    if collide:  # one extra DVL ping right behind the 3rd: the scheduler queues it one epoch later
        dvl_t = np.insert(dvl_t, 3, dvl_t[2] + 1e-6)
        dvl_mu = np.insert(dvl_mu, 3, dvl_mu[2] + 0.01, axis=0)
    m = mission.build_pose_log(
        batch, imu, log["gyro"], log["acc"], log["acc_cov"],
        dvl=(dvl_t, dvl_mu, log["dvl_cov"]),
        pressure=(st(abi.EV_PRESSURE), log["pressure"], log["pressure_cov"]),
        adcp=(st(abi.EV_ADCP), log["adcp"], log["adcp_cov"]),
        efforts=(st(abi.EV_EFFORTS), log["efforts"], log["efforts_cov"]),
        adcp_cell_weighting=log["adcp_cell_weighting"])
    return log, m


def test_mission_roundtrip_and_save(tmp_path):
    log, m = jittered_mission(2, 3000, collide=False)
    for k in ("flags", "dvl_index", "pressure_index", "adcp_index", "efforts_index"):
        np.testing.assert_array_equal(m[k], log[k])
    for k in ("gyro", "acc", "dvl", "pressure", "adcp", "efforts"):
        np.testing.assert_array_equal(m[k], log[k])
    p = os.path.join(tmp_path, "m.npz")
    mission.save(p, m)
    r = mission.load(p)
    for k in mission._ARRAYS:
        np.testing.assert_array_equal(np.asarray(r[k]), np.asarray(m[k]))
    assert r["epochs"] == m["epochs"] and r["dt"] == m["dt"]


def test_mission_collision_queues_one_epoch():
    log, m = jittered_mission(2, 3000, collide=True)
    d = np.flatnonzero(m["dvl_index"] >= 0)
    d0 = np.flatnonzero(log["dvl_index"] >= 0)
    assert len(d) == len(d0) + 1
    assert d[3] == d[2] + 1 and m["dvl_index"][d[3]] == 3
    np.testing.assert_array_equal(m["dvl"][3], log["dvl"][2] + 0.01)


def test_oracle_replays_broadcast_payload():
    """Broadcast payloads ([n][m], one recording for the whole ensemble) equal
    the per-instance copy."""
    B, E = 3, 400
    log = synth.make_pose_log(1, E, "C3")
    t = np.arange(1, E + 1) * log["dt"]
    dvl_t = stamps_of(log, abi.EV_DVL)
    a = mission.build_pose_log(B, t, log["gyro"][:, 0], log["acc"][:, 0], log["acc_cov"],
                               dvl=(dvl_t, log["dvl"][:, 0], log["dvl_cov"]))
    b = mission.build_pose_log(B, t, np.repeat(log["gyro"], B, 1), np.repeat(log["acc"], B, 1), log["acc_cov"],
                               dvl=(dvl_t, np.repeat(log["dvl"], B, 1), log["dvl_cov"]))
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    pos0 = np.repeat(log["pos0"], B, 0)
    rot0 = np.repeat(log["rot0"], B, 0)
    out = []
    for lg in (a, b):
        o = O.OraclePoseBatch(B, 53)
        o.init_from_config(pos0, np.repeat(log["pos_cov"], B, 0), rot0, np.repeat(log["rot_cov"], B, 0), cfg, uwv)
        o.set_process_noise_from_config(cfg, lg["dt"])
        o.run_log(lg)
        out.append(o.get_state())
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


@pytest.mark.gpu
def test_gpu_replays_jittered_mission():
    B, E = 16, 3000
    log, m = jittered_mission(B, E, collide=True)
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    f = engine.PoseUKFBatch(B, 53)
    o = O.OraclePoseBatch(B, 53)
    for h in (f, o):
        h.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
        h.set_process_noise_from_config(cfg, m["dt"])
    cnt_o = o.run_log(m)
    f.run_log(f.upload_log(m))
    (xg, Pg), (xo, Po) = f.get_state(), o.get_state()
    assert state_err(xg, xo, Po, 53).max() < 1e-7
    assert cov_err(Pg, Po).max() < 1e-7
    assert not f.get_status().any()
