#!/usr/bin/env python3
"""Rehearsal of the native RCCL ensemble all-reduce (uwvk_comm_* C ABI) with
N ranks as processes, rank r on device r.  Prints OK when the RCCL sum equals
the sum of the per-shard statistics.  (--same-device puts every rank on device
0: RCCL refuses that with "Duplicate GPU detected" and uwvk_comm_init returns
UWVK_EDEVICE, which this reports; on a one-GPU box the one-rank case is
tests/test_distributed.py::test_rccl_allreduce_through_c_abi.)"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))

B, E = 96, 30


def worker(rank, world, dev, uid, q):
    try:
        _work(rank, world, dev, uid, q)
    except Exception as e:  # report instead of leaving the parent waiting
        q.put((rank, None, repr(e)))


def _work(rank, world, dev, uid, q):
    from uwvk import engine, ensemble, synth
    lo, hi = ensemble.shard_range(rank, world, B)
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(hi - lo, E, "C3", first_instance=lo)
    f = engine.PoseUKFBatch(hi - lo, device=dev)
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    f.run_log(f.upload_log(log))
    truth = log["truth"].state(E)
    comm = engine.RcclComm(world, uid, rank, dev)
    q.put((rank, f.ensemble_stats(truth), f.ensemble_stats(truth, comm)))
    comm.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--same-device", action="store_true")
    a = ap.parse_args()
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    from uwvk import engine
    uid = engine.RcclComm.unique_id()
    ps = [ctx.Process(target=worker, args=(r, a.ranks, 0 if a.same_device else r, uid, q)) for r in range(a.ranks)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(a.ranks))
    for p in ps:
        p.join(timeout=60)
    bad = [r for r in res if r[1] is None]
    if bad:
        print("FAILED: %s" % bad)  # e.g. RCCL's duplicate-GPU check with --same-device
        sys.exit(1)
    local = sum(r[1] for r in res)
    for r in res:
        np.testing.assert_allclose(r[2], local, rtol=1e-12, atol=1e-12)
    print("OK: %d ranks, RCCL sum of %d stats == sum of the shard stats" % (a.ranks, len(local)))


if __name__ == "__main__":
    main()
