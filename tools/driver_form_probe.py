"""Where does the driver's short bench form lose time?  

The driver runs `bench.py --gpus 1 --steps 20 --warmup 5`: warmup, clock ramp, MUPlan.tune() (100-
iteration launches), then ONE timed 20-iteration launch after a host synchronisation.  In r03 the
timed launch averaged 63.5 us/iteration while tune() in the same process measured 57.8.  This probe
replays that sequence and then separates the candidates:

  seq      : the bench's own sequence (tune -> describe -> events -> prepare -> sync -> launch)
  gap      : a 20-iteration launch after a host sync and an idle gap of G ms (clock drop while idle?)
  chained  : an n-iteration launch enqueued behind a busy 100-iteration launch, no host sync
             (the fixed per-launch cost at warm clocks: t(n) = a + b n)
  synced   : the same n after a host sync (the GPU idle for the host's launch latency only)

Every line is one JSON object (us per launch and per iteration).
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from cnmf_amd.solver import MUPlan
    from cnmf_amd.synthetic import iop_spectra, random_init
    import bench

    X = iop_spectra(1_000_000, 81, seed=0, dtype=np.float32)
    W0, H0 = random_init(X, 4, 42)
    plan = MUPlan(torch.from_numpy(X).cuda(), 4)
    plan.set_W(torch.from_numpy(W0))
    plan.set_H(torch.from_numpy(H0))
    sync = torch.cuda.synchronize
    stream = torch.cuda.current_stream()

    def ev2():
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for x in e:
            x.record(stream)
        return e

    def out(**kw):
        print(json.dumps(kw), flush=True)

    plan.iterate(5)
    sync()
    ramp_s, trips = bench.clock_ramp(plan, 0.5, 1, plan.device, sync)
    tuned = plan.tune(n_iter=100, rounds=2) if os.environ.get("NO_TUNE") is None else {}
    out(what="tune", tuned=tuned, ramp_s=ramp_s, trips=trips)

    # the bench's own sequence, repeated (each after a tune-like 100-iteration launch + sync)
    for rep in range(4):
        plan.layout = 4
        plan._time_iterations(100)
        plan.describe()
        e = ev2()
        run = plan.prepare(20, pass_events=e)
        sync()
        sync()
        t0 = time.perf_counter()
        run()
        sync()
        wall = time.perf_counter() - t0
        us = e[0].elapsed_time(e[1]) * 1e3
        out(what="seq", rep=rep, us_launch=round(us, 2), us_it=round(us / 20, 2), wall_us=round(wall * 1e6, 1))

    # idle gap before the timed launch
    for rep in range(3):
        for gap_ms in (0, 0.2, 1, 3, 10, 30, 100, 300):
            plan._time_iterations(100)
            e = ev2()
            run = plan.prepare(20, pass_events=e)
            sync()
            if gap_ms:
                time.sleep(gap_ms / 1e3)
            run()
            sync()
            us = e[0].elapsed_time(e[1]) * 1e3
            out(what="gap", rep=rep, gap_ms=gap_ms, us_launch=round(us, 2), us_it=round(us / 20, 2))

    # launch length scan: chained behind a busy launch (no idle) vs after a sync
    for rep in range(3):
        for n in (1, 2, 5, 10, 20, 50, 100, 500):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            plan.iterate(100)  # busy, no sync
            e[0].record(stream)
            plan.iterate(n)
            e[1].record(stream)
            sync()
            us = e[0].elapsed_time(e[1]) * 1e3
            out(what="chained", rep=rep, n=n, us_launch=round(us, 2), us_it=round(us / n, 2))
            plan.iterate(100)
            sync()
            e = ev2()
            run = plan.prepare(n, pass_events=e)
            sync()
            run()
            sync()
            us = e[0].elapsed_time(e[1]) * 1e3
            out(what="synced", rep=rep, n=n, us_launch=round(us, 2), us_it=round(us / n, 2))
    plan.check_sync_error()


if __name__ == "__main__":
    main()
