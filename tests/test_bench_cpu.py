"""bench.py's multi-rank control flow on CPU (world-size-2 gloo; VERDICT r2 "make bench.py safe at
N > 1"): the untimed clock ramp and the layout tuning must make the SAME decisions on every rank —
one extra 100-iteration trip on one rank spins the in-launch exchange into a timeout (or mis-pairs
RCCL collectives), and ranks that keep different layouts launch different kernels.

The plan is a stand-in whose launches only sleep (rank-dependent speeds, and per-rank layout
timings whose individual winners differ), so the test exercises exactly bench.clock_ramp and
MUPlan.tune's collective choice.  The real launches are covered by tests/test_gpu_bench_dist.py.
"""
import os
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from cnmf_amd import _lib
from cnmf_amd.solver import MUPlan


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _SleepPlan(MUPlan):
    """A persistent k = 4 fp32 plan whose iterations sleep: rank r is (r + 1)× slower."""

    def __init__(self, rank, group):  # noqa: D107 — no super(): no HIP buffers
        self.rank = rank
        self.group = group
        self.world = dist.get_world_size(group)
        self.device = torch.device("cpu")
        self.persistent = True
        self.k, self.xdt = 4, _lib.F32
        self.layout = 0
        self.W = torch.zeros(8, 4)
        self.H64 = torch.zeros(4, 81, dtype=torch.float64)
        self.calls = 0

    def iterate(self, n_iter, update_H=True, pass_events=None):
        self.calls += 1
        self.W += 1.0  # state that the ramp / tune must restore
        time.sleep(0.004 * (self.rank + 1))

    def refresh_basis(self):
        pass

    def _time_iterations(self, n_iter):
        self.iterate(n_iter)
        # per-rank timings with DIFFERENT winners: rank 0 prefers layout 1, rank 1 layout 2; the
        # slowest rank's time per layout is 4: 60/70, 1: 50/90, 2: 80/55 -> collective pick 4
        table = {0: {4: 60.0, 1: 50.0, 2: 80.0}, 1: {4: 70.0, 1: 90.0, 2: 55.0}}
        return table[self.rank][self.layout] * n_iter / 1e6


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        plan = _SleepPlan(rank, dist.group.WORLD)
        W0 = plan.W.clone()
        el, trips = bench.clock_ramp(plan, 0.25, world, torch.device("cpu"), lambda: None)
        ramp_calls = plan.calls
        assert torch.equal(plan.W, W0)  # the ramp restored the state
        tuned = plan.tune(n_iter=100, rounds=2, variants=(4, 1, 2))
        assert torch.equal(plan.W, W0)  # and so did the tuning
        flags = [bench.any_rank(rank == 1, world, torch.device("cpu")),
                 bench.rank0_says(rank == 0, world, torch.device("cpu"))]
        out[rank] = (trips, ramp_calls, tuned, plan.layout, flags, el)
    finally:
        dist.destroy_process_group()


def test_ramp_and_tune_decisions_are_collective():
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r0, r1 = out[0], out[1]
    assert r0[0] == r1[0] and r0[1] == r1[1] and r0[0] >= 1  # same number of ramp trips / launches
    assert r0[2] == r1[2] == {4: 70.0, 1: 90.0, 2: 80.0}      # the slowest rank's time per layout
    assert r0[3] == r1[3] == 4                                 # one layout on every rank
    assert r0[4] == r1[4] == [True, True]                      # any_rank / rank0_says agree


def test_single_rank_helpers_need_no_group():
    assert bench.any_rank(True, 1, None) and not bench.any_rank(False, 1, None)
    assert bench.rank0_says(True, 1, None)


def test_cpu_model_is_named():
    assert isinstance(bench.cpu_model(), str) and bench.cpu_model()


@pytest.mark.parametrize("argv", [["--backend", "gloo"], ["--backend", "nccl"]])
def test_backend_flag_parses(argv, monkeypatch):
    monkeypatch.setattr("sys.argv", ["bench.py"] + argv)
    assert bench.parse().backend == argv[1]


def test_launcher_decision():
    """`--gpus N` never runs fewer ranks than it reports."""
    d = bench.launcher_decision
    assert d(1, {}, 0, "nccl") == ("run", None)
    assert d(8, {}, 8, "nccl") == ("spawn", None)
    assert d(2, {}, 1, "gloo") == ("spawn", None)  # gloo ranks may share a device
    assert d(8, {}, 1, "nccl")[0] == "refuse"  # RCCL: one device per rank
    assert d(2, {"WORLD_SIZE": "2"}, 0, "nccl") == ("run", None)  # the driver's torchrun line
    assert d(8, {"WORLD_SIZE": "1"}, 8, "nccl")[0] == "refuse"
    assert d(1, {"WORLD_SIZE": "4"}, 8, "nccl")[0] == "refuse"
    # --gpus omitted takes the launcher's WORLD_SIZE (torchrun without a matching --gpus)
    assert d(None, {"WORLD_SIZE": "4"}, 8, "nccl") == ("run", None)
    assert d(None, {}, 0, "nccl") == ("run", None)


def test_line_value_and_unit():
    """VERDICT r4 item 5 / ADVICE r4: the value is an iteration rate of the problem actually run,
    and the unit says which — no rescaling by rows / 1e6 (the 1e7-row cfg3 line once printed
    12,377 'it/s' for a 1,238 it/s fit)."""
    v, u = bench.line_value("weak", 1, 10_000_000, 500, 500 / 1238.0)
    assert abs(v - 1238.0) < 1e-6 and u == "1e7-row it/s"
    v, u = bench.line_value("weak", 1, 1_000_000, 500, 500 / 17800.0)
    assert abs(v - 17800.0) < 1e-6 and u == "1e6-row it/s"  # cfg2 at N = 1: unchanged value
    v, u = bench.line_value("weak", 8, 1_000_000, 500, 500 / 17000.0)
    assert abs(v - 8 * 17000.0) < 1e-6 and u == "1e6-row it/s"  # the 1e6-row shards' iterations, summed
    v, u = bench.line_value("strong", 8, 124_992, 500, 500 / 60000.0)
    assert abs(v - 60000.0) < 1e-6 and u == "it/s"
    assert bench.row_unit(16384) == "16384"


def test_state_problem_flags_nan_and_negative():
    import numpy as np
    W, H = np.ones((4, 2), np.float32), np.ones((2, 3))
    assert bench.state_problem(1.0, W, H) is None
    assert "error" in bench.state_problem(float("nan"), W, H)
    assert "error" in bench.state_problem(float("inf"), W, H)
    Wn = W.copy(); Wn[1, 1] = np.nan
    assert "W" in bench.state_problem(1.0, Wn, H)
    Hn = H.copy(); Hn[0, 2] = -1e-30
    assert "negative" in bench.state_problem(1.0, W, Hn)


class _NaNPlan:
    """A stand-in plan whose final state is broken on one rank only."""

    def __init__(self, broken):
        self.broken = broken
        self.W = torch.ones(8, 4)
        self.H64 = torch.ones(4, 81, dtype=torch.float64)
        if broken:
            self.W[3, 2] = float("nan")

    def frobenius_error(self):
        return float("nan") if self.broken else 1.0


def _verdict_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        err, problem = bench.final_verdict(_NaNPlan(broken=rank == 1), world, torch.device("cpu"))
        code = None
        try:
            if problem:
                bench.refuse_result(problem, rank)
        except SystemExit as e:
            code = e.code
        out[rank] = (problem, code)
    finally:
        dist.destroy_process_group()


def test_forced_nan_plan_refuses_on_every_rank():
    """a NaN state on ANY rank makes EVERY rank exit non-zero without a line."""
    manager = mp.Manager()
    out = manager.dict()
    mp.spawn(_verdict_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in (0, 1):
        problem, code = out[r]
        assert problem and code == bench.EXIT_BROKEN != 0
    assert "another rank" in out[0][0] and "error" in out[1][0]
    # one rank, no group: the same verdict
    err, problem = bench.final_verdict(_NaNPlan(broken=True), 1, None)
    assert problem and err != err
    with pytest.raises(SystemExit) as e:
        bench.refuse_result(problem, 0)
    assert e.value.code == bench.EXIT_BROKEN


def _bench_cmd(extra, env):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in dict(os.environ, **env).items() if v is not None}
    return subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--no-cpu"] + extra, env=env,
                          cwd=root, capture_output=True, text=True, timeout=240)


@pytest.mark.timeout(300)
def test_gpus_flag_without_launcher_never_reports_one_rank():
    """`bench.py --gpus 2` without torchrun starts two ranks itself (here, without a GPU, they fail
    — the point is that no line claiming n_gpus 1 is printed and the exit status is non-zero);
    a WORLD_SIZE that disagrees with --gpus is refused before anything runs."""
    r = _bench_cmd(["--gpus", "2", "--backend", "gloo", "--steps", "1", "--warmup", "1"],
                   {"WORLD_SIZE": None, "RANK": None, "LOCAL_RANK": None})
    assert "starting 2 ranks" in r.stderr, r.stderr[-2000:]
    assert '"n_gpus": 1' not in r.stdout
    if not torch.cuda.is_available():
        assert r.returncode != 0
    r = _bench_cmd(["--gpus", "2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "refused" in r.stderr and '"n_gpus"' not in r.stdout
