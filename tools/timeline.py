#!/usr/bin/env python3
"""Per-wave timeline of one k_psp_epoch<53> launch (diagnostic build
libuwvk_timeline.so, -DUWVK_TIMELINE): entry, Sigma loaded, epochs done,
stored, and the CU, for every wave.  Prints where a short launch's time goes:
prologue/epilogue per wave, the generation structure and the idle tail.
usage: UWVK_LIB=.../libuwvk_timeline.so python tools/timeline.py [--steps 20] [--out file.npz]"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-uwv_kalman_filters_amd", "python"))
from uwvk import engine, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--out", default="")
    ap.add_argument("--tail-slots", type=int, default=0)
    ap.add_argument("--persist", type=int, default=0, help="UWVK_OPT_PERSIST (records are then per work unit)")
    a = ap.parse_args()
    B, E = a.batch, a.steps
    cfg, uwv = synth.default_pose_config(), synth.default_uwv()
    log = synth.make_pose_log(B, E + 5, "C3")
    f = engine.PoseUKFBatch(B)
    f.set_tail_slots(a.tail_slots)
    f.set_persist(a.persist)
    L0 = engine.lib()
    s_x = L0.uwvk_pose_resident_slots(53, 0)
    ch = L0.uwvk_pose_tail_chunks(B // 8, a.tail_slots or s_x, E) if a.tail_slots >= 0 else 1
    print("resident slots per XCD (runtime): %d; tail_slots %d; chunks %d" % (s_x, a.tail_slots, ch))
    f.init_from_config(log["pos0"], log["pos_cov"], log["rot0"], log["rot_cov"], cfg, uwv)
    f.set_process_noise_from_config(cfg, log["dt"])
    d = f.upload_log(log)
    f.run_log(d, 0, 5)
    f.timer_start()
    f.run_log(d, 5, E, sync=False)
    ms = f.timer_stop()
    L = engine.lib()
    n = min(B + 8 * (ch - 1) * ch * (a.tail_slots or s_x), 131072)  # spread launches: 8 (c - 1) r_x more blocks
    buf = np.zeros(n * 8, np.uint64)
    # the default (right) side's kernels record into the SR = 1 object's buffer
    assert L.uwvk_debug_read_timeline_r(buf.ctypes.data_as(C.c_void_p), C.c_longlong(n * 8)) == 0
    t = buf.reshape(n, 8)
    t = t[t[:, 3] != 0]  # blocks that ran
    n = len(t)
    ts = t[:, :4].astype(np.int64)
    t0 = ts[:, 0].min()
    rel = (ts - t0) * 10e-3  # 100 MHz realtime counter -> us
    cu = (t[:, 4] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 4] >> 32).astype(np.int64)
    pro, body, epi = rel[:, 1] - rel[:, 0], rel[:, 2] - rel[:, 1], rel[:, 3] - rel[:, 2]
    span = rel[:, 3].max()
    print("kernel %.3f ms (HIP events), wave span %.3f ms, %d waves" % (ms, span * 1e-3, n))
    for name, v in (("prologue (load)", pro), ("epochs", body), ("epilogue (fold+store)", epi)):
        print("  %-22s mean %8.2f us  p50 %8.2f  p95 %8.2f  max %8.2f" % (name, v.mean(), np.median(v),
                                                                          np.percentile(v, 95), v.max()))
    # concurrency over time
    grid = np.linspace(0, span, 400)
    act = np.array([((rel[:, 0] <= g) & (rel[:, 3] > g)).sum() for g in grid])
    print("  active waves: max %d, mean %.0f; time with < 2/3 of max active: %.1f us" %
          (act.max(), act.mean(), (act < act.max() * 2 / 3).sum() * span / 400))
    # gaps: per CU, time between one wave's end and the next start on that CU
    key = xcc * 1024 + cu
    gaps = []
    for k in np.unique(key):
        m = key == k
        s = np.sort(rel[m, 0])
        e = np.sort(rel[m, 3])
        if len(s) > 12:
            gaps.append(np.median(s[12:] - e[:len(s) - 12]))
    if gaps:
        print("  per-CU refill gap (end of wave -> start of the 12th-next): median %.2f us" % np.median(gaps))
    print("  start spread of the first 3072 waves: %.2f us" % np.sort(rel[:, 0])[3071])
    for x in range(8):
        m = xcc == x
        if m.any():
            e = np.sort(rel[m, 3])
            print("  XCC %d: %5d blocks, last end %8.1f us, 95%% of ends by %8.1f us, mean duration %6.1f us" %
                  (x, m.sum(), e[-1], e[int(0.95 * (len(e) - 1))], (rel[m, 3] - rel[m, 0]).mean()))
    if a.out:
        np.savez_compressed(a.out, rel=rel.astype(np.float32), cu=cu, xcc=xcc, inst=t[:, 5].astype(np.int64), ms=ms)


if __name__ == "__main__":
    main()
