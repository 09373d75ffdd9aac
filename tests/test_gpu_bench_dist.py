"""bench.py at N = 2 on ONE GPU: two ranks launched as the driver launches them
(RANK / WORLD_SIZE / MASTER_* in the environment), sharing cuda:0 over the gloo backend (RCCL needs
distinct devices; the kernels, the in-launch exchange through IPC and every collective decision
of the bench are the same).  The run must finish, validate the in-launch exchange against the
host-collective path, time it, and report the same layout on both ranks.

The problem is small enough (32768 rows: 64 workgroups per rank) that both ranks' persistent grids
are co-resident on the one GPU, as the exchange requires.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_two_ranks(extra, timeout=240, rank_env=None):
    """bench.py's two ranks on cuda:0; rank_env: {rank: {VAR: value}} added to that rank's environment
    (the fault-injection switches of cnmf_amd/solver.py).  Without --strong-rows the bench records the
    default 1e6-row split as not measured (ranks sharing a GPU)."""
    port = _free_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE="2",
                   LOCAL_WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.update((rank_env or {}).get(rank, {}))
        cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
               "--steps", "20", "--warmup", "20", "--no-cpu", "--ramp-seconds", "0.2", "--scaling", "strong"] + extra
        procs.append(subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            outs.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, o, e in outs:
        assert rc == 0, e[-3000:]
    lines = [ln for ln in outs[0][1].splitlines() if ln.startswith("{")]
    assert len(lines) == 1, outs[0][1][-2000:]
    assert not [ln for ln in outs[1][1].splitlines() if ln.startswith("{")]  # rank 0 prints alone
    return json.loads(lines[0]), outs


@pytest.mark.timeout(300)
def test_bench_two_ranks_one_gpu_exchange():
    res, outs = _run_two_ranks(["--rows", "32768"])
    cfg = res["config"]
    assert res["ranks"] == 2 and res["n_gpus"] == 1 and res["value"] > 0  # two ranks sharing one GPU
    assert cfg["exchange"].startswith("validated"), cfg["exchange"]
    lay = cfg["layout_per_rank"]
    assert len(lay) == 2 and lay[0] == lay[1]
    assert cfg["clock_ramp_trips"] >= 1
    assert res["roofline"]["iterations_per_launch"] == 20  # the 20 steps as ONE launch per rank
    # the default 1e6-row strong split is not co-resident when ranks share a GPU
    assert res["strong"] == {"skipped": res["strong"]["skipped"]} and "not measured" in res["strong"]["skipped"]


@pytest.mark.timeout(300)
def test_bench_exchange_setup_fault_moves_every_rank_to_rccl():
    """one rank's exchange setup fails (CNMF_FAULT_XCHG_SETUP on rank 1 only):
    enable_exchange agrees collectively, so BOTH ranks time the shard-step + collective path and the
    line's config.exchange names the failing rank."""
    res, outs = _run_two_ranks(["--rows", "32768"], rank_env={1: {"CNMF_FAULT_XCHG_SETUP": "1"}})
    cfg = res["config"]
    assert cfg["exchange"].startswith("unavailable") and "rank 1: fault injected" in cfg["exchange"], cfg["exchange"]
    assert "RCCL path timed" in cfg["exchange"]
    assert res["roofline"]["launches_timed"] == 20 and res["value"] > 0  # one shard step per iteration
    assert "in-launch over xGMI" not in cfg["parallelism"]
    for _, _, err in outs:  # both ranks reported the same decision
        assert "in-launch exchange (16384 rows): unavailable" in err


@pytest.mark.timeout(300)
def test_bench_exchange_poisoned_launch_moves_every_rank_to_rccl():
    """One rank's launch fails inside the exchange (CNMF_FAULT_XCHG_POISON on rank 1: its error word
    set before its first exchange launch, so its top combiner tags its words XPOISON): the peer's
    launch must fail in the same iteration (no 2 s timeout per iteration), validation fails on both
    ranks together and both time the collective path; the results stay a valid factorisation."""
    res, outs = _run_two_ranks(["--rows", "32768"], rank_env={1: {"CNMF_FAULT_XCHG_POISON": "1"}})
    cfg = res["config"]
    assert cfg["exchange"].startswith("failed validation"), cfg["exchange"]
    assert res["roofline"]["launches_timed"] == 20 and res["value"] > 0
    assert res["final_frobenius_error"] > 0
    for _, _, err in outs:
        assert "in-launch exchange (16384 rows): failed validation" in err


@pytest.mark.timeout(300)
def test_bench_two_ranks_weighted_with_strong_split():
    """--weighted at N = 2 through the whole bench, the strong split included (its plan is
    released after the measurement): one line, the exchange validated for the weighted launch."""
    res, outs = _run_two_ranks(["--rows", "16384", "--scaling", "weak", "--weighted", "--strong-rows", "32768"])
    assert res["ranks"] == 2 and res["value"] > 0
    assert res["config"]["exchange"].startswith("validated"), res["config"]["exchange"]
    assert res["strong"]["rows"] == 32768 and res["strong"]["speedup_vs_n1"] > 0
    assert "weighted" in res["metric"]


@pytest.mark.timeout(300)
def test_bench_two_ranks_one_gpu_host_collective_path():
    """--exchange off: one shard step + one all_reduce per iteration on both ranks."""
    res, _ = _run_two_ranks(["--rows", "32768", "--exchange", "off", "--no-tune"])
    assert res["ranks"] == 2 and res["value"] > 0
    assert res["config"]["exchange"] is None
    assert res["roofline"]["launches_timed"] == 20


@pytest.mark.timeout(300)
def test_bench_two_ranks_one_gpu_weak_scaling():
    """The default scaling (weak): every rank owns --rows rows; the line's value is the 1e6-row
    iterations all ranks completed per second, the exchange validated as at strong scaling."""
    res, _ = _run_two_ranks(["--rows", "16384", "--scaling", "weak"])
    assert res["scaling"] == "weak" and res["ranks"] == 2
    assert res["config"]["n_rows_per_gpu"] == 16384 and res["config"]["n_rows_total"] == 32768
    assert res["config"]["exchange"].startswith("validated"), res["config"]["exchange"]
    it_s = res["steps"] / (res["ms_per_step"] * res["steps"] / 1e3)
    # ranks x it/s of the problem run, in a unit that names the shard's rows
    assert abs(res["value"] - 2 * it_s) <= 0.02 * res["value"]
    assert res["unit"] == "16384-row it/s"
    assert res["n_gpus"] == 1 and res["ranks"] == 2  # two ranks sharing one GPU are not two GPUs


@pytest.mark.timeout(300)
def test_bench_two_ranks_strong_split_beside_the_weak_line():
    """at N > 1 the line carries the fixed problem (here 32768 rows, the metric's
    V = 1e6 on the driver's nodes) split over the same ranks and timed in the same run, and the same
    problem on rank 0's GPU alone: it/s, us per iteration, HBM fraction, speed-up over one GPU."""
    res, outs = _run_two_ranks(["--rows", "16384", "--scaling", "weak", "--strong-rows", "32768"])
    assert res["unit"] == "16384-row it/s" and res["scaling"] == "weak"
    st = res["strong"]
    assert st["rows"] == 32768 and st["ranks"] == 2 and st["rows_per_gpu_max"] == 16384
    for key in ("it_s", "us_per_iteration", "frac", "speedup_vs_n1", "n1_it_s", "n1_us_per_iteration"):
        assert st[key] > 0, (key, st)
    assert abs(st["it_s"] * st["us_per_iteration"] / 1e6 - 1.0) < 0.01
    assert abs(st["speedup_vs_n1"] - st["n1_us_per_iteration"] / st["us_per_iteration"]) < 0.01
    assert st["exchange"].startswith("validated"), st["exchange"]
    assert outs[0][2].count("in-launch exchange (16384 rows): validated") == 2  # the weak and the split plan


@pytest.mark.timeout(300)
def test_bench_one_gpu_line_carries_strong_as_itself():
    """At N = 1 on the metric's rows the `strong` key is the line itself (speed-up 1)."""
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "20",
                        "--no-cpu", "--ramp-seconds", "0.1", "--rows", "65536", "--strong-rows", "65536"],
                       cwd=ROOT, capture_output=True, text=True, timeout=240,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert res["unit"] == "65536-row it/s" and res["n_gpus"] == 1
    assert res["strong"]["speedup_vs_n1"] == 1.0 and res["strong"]["rows"] == 65536
    assert abs(res["strong"]["it_s"] - res["value"]) <= 0.01 * res["value"]
