"""The in-process collectives of `factorise(..., devices=[...])` (cnmf_amd.multidevice.LocalGroup) on
CPU: shard-order sums that are bit-identical on every shard, max, all-gather, and a failing shard
releasing the others instead of leaving them waiting."""
import threading

import pytest
import torch

from cnmf_amd.multidevice import LocalGroup
from cnmf_amd.solver import agree_max, plan_world


def _run(P, fn):
    g = LocalGroup(P)
    out, errs = [None] * P, [None] * P

    def body(r):
        try:
            out[r] = fn(g.view(r), r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
            g.abort()
    ts = [threading.Thread(target=body, args=(r,)) for r in range(P)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out, errs


def test_sum_max_gather_are_identical_on_every_shard():
    def fn(v, r):
        t = torch.tensor([0.1 * (r + 1), 1e16, -1e16 + r], dtype=torch.float64)
        v.all_reduce(t, "sum")
        m = agree_max([r, -r], v, None)
        return t.tolist(), m, v.all_gather(("rank", r)), plan_world(v)
    out, errs = _run(3, fn)
    assert not any(errs)
    assert out[0] == out[1] == out[2]
    s, m, g, w = out[0]
    assert s[0] == (0.1 + 0.2) + 0.30000000000000004 or abs(s[0] - 0.6) < 1e-15
    assert m == [2.0, 0.0] and g == [("rank", 0), ("rank", 1), ("rank", 2)] and w == 3


def test_a_failing_shard_releases_the_others():
    def fn(v, r):
        if r == 1:
            raise RuntimeError("shard 1 failed")
        v.all_gather(r)
    out, errs = _run(3, fn)
    assert isinstance(errs[1], RuntimeError)
    assert all(isinstance(errs[r], threading.BrokenBarrierError) for r in (0, 2))


def test_devices_argument_validation():
    from cnmf_amd.multidevice import MultiDeviceFit
    with pytest.raises(ValueError):
        MultiDeviceFit(torch.zeros(4, 3), None, 2, (0, 0, 0, 0), [])


def test_host_all_reduce_works_after_a_failed_exchange_setup(monkeypatch):
    """a failed enable_exchange aborts the group's barrier; the fallback (the host
    all-reduce of the same group) must still work afterwards instead of raising BrokenBarrierError."""
    import contextlib
    import types

    from cnmf_amd import _lib
    from cnmf_amd import multidevice as md

    class _Plan:
        def __init__(self, r):
            self.device, self.exchange, self.r = torch.device("cpu"), False, r

        def enable_exchange(self):
            if self.r == 1:  # one shard cannot map its peers; the others would wait in a rendezvous
                raise _lib.HipLibraryError("in-launch exchange unavailable: no peer access")
            fit.group.view(self.r).all_gather(self.r)

    fit = object.__new__(md.MultiDeviceFit)
    fit.plans = [_Plan(r) for r in range(3)]
    fit.group = LocalGroup(3)
    fit.streams = [None] * 3
    fit.shared_device_exchange, fit.exchange = False, False
    monkeypatch.setattr(md.torch.cuda, "set_device", lambda d: None)
    monkeypatch.setattr(md.torch.cuda, "stream", lambda s: contextlib.nullcontext())
    monkeypatch.setattr(md.torch.cuda, "current_stream", lambda: types.SimpleNamespace(synchronize=lambda: None))
    monkeypatch.setattr(md, "_exchange_fits", lambda plans, shared=False: True)
    with pytest.warns(RuntimeWarning):
        assert fit.enable_exchange() is False
    out = [None] * 3

    def go(r, plan):
        t = torch.tensor([float(r + 1)], dtype=torch.float64)
        fit.group.view(r).all_reduce(t, "sum")
        out[r] = float(t[0])
    fit._run(go)
    assert out == [6.0, 6.0, 6.0]
