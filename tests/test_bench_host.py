"""Host-side logic of bench.py (no GPU): the roofline it reports is computed
from the committed counter passes of the timed launch shape, stays <= 1, and
the CPU baseline sizes itself to the cores this process may use."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


# committed counter passes: the default (right SO3 side) kernel and the left option's
PMC_WORKLOADS = ["C3-dof53-b65536", "C3-dof53-b65536-left"]


@pytest.mark.parametrize("workload", PMC_WORKLOADS)
@pytest.mark.parametrize("steps", [20, 200])
def test_committed_counter_passes_give_executed_roofline(steps, workload):
    e = bench.pmc_entry(workload, steps)
    assert e.get("epochs_per_launch") == steps, "no counter pass of the %d-epoch launch committed" % steps
    pw = e["per_wave_epoch"]
    # the counters come from the timed launch of 65,536 instances (normalised per
    # instance-epoch; the tail spreading adds chunk waves beyond one per instance)
    assert e["instances"] == 65536
    assert 65536 <= e["waves"] <= 65536 + 8 * 7 * 8 * 384
    assert 0 < pw["valu_fma_f64"] < pw["valu"]
    # a plausible kernel time for that shape (0.43-0.5 ms per epoch): frac stays in (0, 1)
    for ms in (0.43 * steps, 0.5 * steps):
        cr = bench.counter_roofline(e, 65536, steps, ms)
        frac = cr["achieved_tflops"] / bench.PEAK_FP64_TFLOPS
        assert 0.1 < frac < 1.0
    assert 0 < e["valu_busy"]["model_frac"] <= e["valu_busy"]["frac"] <= 1.0
    # traffic: at least the packed Sigma + mu round trip of every instance
    assert e["bytes_per_launch"] >= 65536 * 2 * (1431 + 54) * 8 * 0.95


def test_pmc_entry_falls_back_without_exact_shape():
    assert bench.pmc_entry("C3-dof53-b65536", 12345).get("epochs_per_launch") != 12345
    assert bench.pmc_entry("no-such-workload", 20) == {}


def test_available_cores_and_torchrun_detection(monkeypatch):
    n = bench.available_cores()
    assert 1 <= n <= (os.cpu_count() or 1)
    for k in ("TORCHELASTIC_RUN_ID", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    assert not bench.launched_by_torchrun()
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "x")
    assert bench.launched_by_torchrun()


def test_flop_models():
    assert bench.F_STEP == 1_554_084  # SURVEY 8(d), frozen
    assert 40_000 < bench.F_STEP_PSP < 70_000  # the PSP engine's own model


def test_bench_line_fields_documented():
    """The keys the driver and the judge read are the ones DESIGN.md section 6 documents."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    for key in ('"roofline"', '"cpu_baseline"', '"achieved"', '"peak"', '"frac"', '"traffic"',
                '"effective_tflops"', '"counters"', '"timing"'):
        assert key in src
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    assert "C3-dof53-b65536-e20" in d and "C3-dof53-b65536-left-e20" in d


# ---- multi-GPU launch logic (no GPU: spawned scripts stand in for the ranks) ----

class _Args:
    def __init__(self, gpus, mode="auto", batch_per_gpu=0):
        self.gpus, self.mode, self.batch_per_gpu = gpus, mode, batch_per_gpu


def test_workload_defaults_c3_single_c5_multi():
    assert bench.workload_of(_Args(1), 1) == ("C3", 65536)
    mode, b = bench.workload_of(_Args(8), 8)
    assert (mode, b * 8) == ("C5", 1_048_576)  # BASELINE.json config 5
    assert bench.workload_of(_Args(2), 2) == ("C5", 131072)
    assert bench.workload_of(_Args(2, batch_per_gpu=1000), 2) == ("C5", 1000)
    assert bench.workload_of(_Args(1, mode="C2"), 1) == ("C2", 4096)


def test_resolve_world_checks_the_launcher():
    assert bench.resolve_world(_Args(1), env={}) == (1, 0, 0)
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}
    assert bench.resolve_world(_Args(4), env=env) == (4, 2, 2)
    with pytest.raises(SystemExit):
        bench.resolve_world(_Args(8), env=env)
    with pytest.raises(SystemExit):
        bench.resolve_world(_Args(1), env=env)


def test_rank_env():
    e = bench.rank_env({"X": "1"}, 3, 8, 12345)
    assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["MASTER_ADDR"], e["MASTER_PORT"]) == \
        ("3", "3", "8", "127.0.0.1", "12345")
    assert e["X"] == "1" and e["UWVK_BENCH_SPAWNED"] == "1"


def test_spawn_ranks_runs_every_rank(tmp_path):
    script = tmp_path / "rank.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text("import os, sys\n"
                      "open(os.path.join(sys.argv[1], os.environ['RANK']), 'w').write(os.environ['WORLD_SIZE'])\n")
    assert bench.spawn_ranks([str(out)], 3, timeout=60, script=str(script)) == 0
    assert sorted(os.listdir(out)) == ["0", "1", "2"]
    assert all((out / r).read_text() == "3" for r in "012")


def test_spawn_ranks_stops_the_others_when_one_fails(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1':\n    sys.exit(7)\n"
                      "time.sleep(120)\n")
    import time
    t0 = time.time()
    assert bench.spawn_ranks([], 3, timeout=60, script=str(script)) == 7
    assert time.time() - t0 < 30


def test_gloo_control_plane_two_ranks(tmp_path):
    """The self-launched ranks form the gloo process group bench.py uses
    (barrier, broadcast of the RCCL id, max of the times) on 127.0.0.1."""
    script = tmp_path / "rank.py"
    script.write_text(
        "import os, sys\n"
        "sys.path.insert(0, %r)\n"
        "import bench, torch\n"
        "dist = bench.init_dist(int(os.environ['WORLD_SIZE']))\n"
        "uid = [b'id' if dist.get_rank() == 0 else None]\n"
        "dist.broadcast_object_list(uid, src=0)\n"
        "w = torch.tensor([float(dist.get_rank())], dtype=torch.float64)\n"
        "dist.all_reduce(w, op=dist.ReduceOp.MAX)\n"
        "dist.barrier()\n"
        "sys.exit(0 if (uid[0] == b'id' and float(w[0]) == 1.0) else 5)\n" % ROOT)
    assert bench.spawn_ranks([], 2, timeout=120, script=str(script)) == 0


@pytest.mark.parametrize("fail", ["none", "rank1", "uid"])
def test_make_rccl_agrees_on_a_fallback(tmp_path, fail):
    """make_rccl over the gloo control plane with a stand-in engine: every rank
    gets the communicator, or every rank gets (None, reason) when one rank
    (or rank 0's id) failed, so the bench falls back to the gloo sum together."""
    script = tmp_path / "rank.py"
    script.write_text(
        "import os, sys\n"
        "sys.path.insert(0, %r)\n"
        "import bench, torch\n"
        "FAIL = %r\n"
        "class Comm:\n"
        "    closed = False\n"
        "    def __init__(self, world, uid, rank, local):\n"
        "        if FAIL == 'rank1' and rank == 1:\n"
        "            raise RuntimeError('no device')\n"
        "        assert uid == b'uid'\n"
        "    def close(self):\n"
        "        Comm.closed = True\n"
        "    @staticmethod\n"
        "    def unique_id():\n"
        "        if FAIL == 'uid':\n"
        "            raise RuntimeError('no rccl')\n"
        "        return b'uid'\n"
        "class Eng:\n"
        "    RcclComm = Comm\n"
        "world = int(os.environ['WORLD_SIZE'])\n"
        "dist = bench.init_dist(world)\n"
        "comm, err = bench.make_rccl(dist, Eng, world, dist.get_rank(), 0)\n"
        "ok = (comm is not None and err is None) if FAIL == 'none' else (comm is None and err is not None)\n"
        "if FAIL == 'rank1' and dist.get_rank() == 0:\n"
        "    ok = ok and Comm.closed\n"
        "dist.barrier()\n"
        "sys.exit(0 if ok else 5)\n" % (ROOT, fail))
    assert bench.spawn_ranks([], 2, timeout=120, script=str(script)) == 0


@pytest.mark.parametrize("fail", ["none", "rank5"])
def test_eight_rank_spawn_and_collective_text(tmp_path, fail):
    """C5's launch shape on CPU: bench.spawn_ranks starts 8 stand-in ranks,
    they form the gloo control plane, make_rccl agrees on the engine's
    communicator (stand-in) or, when rank 5 cannot make it, on the gloo
    fallback on every rank; each rank reports config.collective as bench.py
    would and the job's exit code is 0 either way.  (RCCL with N > 1 itself
    runs only in the driver's 8-GPU bench: DESIGN.md section 8.)"""
    script = tmp_path / "rank.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text(
        "import os, sys\n"
        "sys.path.insert(0, %r)\n"
        "import bench\n"
        "FAIL = %r\n"
        "class Comm:\n"
        "    def __init__(self, world, uid, rank, local):\n"
        "        if FAIL == 'rank5' and rank == 5:\n"
        "            raise RuntimeError('ncclCommInitRank failed')\n"
        "    def close(self):\n"
        "        pass\n"
        "    @staticmethod\n"
        "    def unique_id():\n"
        "        return b'uid'\n"
        "class Eng:\n"
        "    RcclComm = Comm\n"
        "world = int(os.environ['WORLD_SIZE'])\n"
        "dist = bench.init_dist(world)\n"
        "rank = dist.get_rank()\n"
        "comm, err = bench.make_rccl(dist, Eng, world, rank, rank)\n"
        "open(os.path.join(sys.argv[1], str(rank)), 'w').write(bench.collective_desc(dist, world, comm, err, False))\n"
        "dist.barrier()\n"
        "dist.destroy_process_group()\n" % (ROOT, fail))
    assert bench.spawn_ranks([str(out)], 8, timeout=240, script=str(script)) == 0
    texts = [(out / str(r)).read_text() for r in range(8)]
    # every rank agrees on the collective (the reason names the failing rank or "another rank")
    assert len(set(t.split(" failed (")[0] for t in texts)) == 1
    if fail == "none":
        assert all(t.startswith("RCCL all_reduce") for t in texts)
    else:
        assert all(t.startswith("gloo all_reduce") and "RCCL communicator failed" in t for t in texts)


def test_collective_desc_one_gpu_rehearsals(monkeypatch):
    """N = 1 names the communicator rehearsal UWVK_BENCH_COLL asks for (the
    one-rank communicator through the window, or made around each all-reduce),
    and no collective without one."""
    monkeypatch.delenv("UWVK_BENCH_COLL", raising=False)
    assert bench.collective_desc(None, 1, None, None, False) is None
    monkeypatch.setenv("UWVK_BENCH_COLL", "rccl1")
    assert "through the timed region" in bench.collective_desc(None, 1, None, None, False)
    monkeypatch.setenv("UWVK_BENCH_COLL", "scoped")
    assert "around each statistics all-reduce" in bench.collective_desc(None, 1, None, None, False)
