"""Host orchestration of the MU hot path on PyTorch-ROCm device memory.

`MUPlan` owns the device buffers of one (shard of a) factorisation and issues the C-ABI launches;
`run_mu` is the driver loop of sklearn's `_fit_multiplicative_update` (SK:731-893, loop SK:831-884):
W then H every iteration, the Frobenius error every 10 iterations when tol > 0, and the relative
decrease test (SK:872-884).  Iterations between two error checks go to the library in one call
(`cnmf_mu_iterations`) — no host synchronisation inside a stretch.

Multi-GPU: the rows of X/W are sharded over the ranks of a torch.distributed
group; after each rank's pass, the per-rank fp64 accumulators [WᵀX | WᵀW] (k·(F+k) doubles) are
summed with ONE all_reduce (RCCL over xGMI for backend "nccl"), and every rank applies the identical
basis update.  The error check all-reduces one double.

SK:<line> = sklearn/decomposition/_nmf.py (1.7.2).
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from . import _lib
from ._lib import check
from ._trace import trace_range

_XDT = {torch.float32: _lib.F32, torch.float64: _lib.F64, torch.bfloat16: _lib.BF16}


# Fault injection for the multi-GPU tests (SURVEY §5 "failure detection"; never set in a measured
# run): CNMF_FAULT_XCHG_SETUP=1 makes THIS rank report its in-launch exchange setup as failed, so
# every rank must agree to take the RCCL path; CNMF_FAULT_XCHG_POISON=1 sets this rank's error word
# before its first exchange launch, so its top combiner tags its words XPOISON and every peer's
# launch fails in the same iteration (tests/test_gpu_bench_dist.py).
def _fault(name: str) -> bool:
    return os.environ.get(name, "0") == "1"


def _ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def plan_world(group) -> int:
    """Ranks a plan's accumulators are summed over: the size of `group` when one is given, else 1.
    A plan built without a group is a single-process fit even inside an initialised default group
    (independent per-rank fits under torchrun, e.g. cNMF replicates, must not all-reduce)."""
    if group is None:
        return 1
    if getattr(group, "is_local", False):  # shards of one process (cnmf_amd.multidevice)
        return group.size()
    return torch.distributed.get_world_size(group)


def collective_tensor(values, group, device):
    """A float64 tensor of `values` on the device the group's backend reduces (host memory for
    gloo, the plan's GPU for RCCL)."""
    dev = "cpu" if torch.distributed.get_backend(group) == "gloo" else device
    return torch.tensor([float(v) for v in values], dtype=torch.float64, device=dev)


def agree_max(values, group, device):
    """Element-wise maximum of `values` over the ranks of `group` (identity without a group)."""
    if group is None or plan_world(group) == 1:
        return [float(v) for v in values]
    if getattr(group, "is_local", False):
        return group.all_reduce_values(values, "max")
    t = collective_tensor(values, group, device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
    return [float(v) for v in t.tolist()]


def _event_array(events):
    if events is None:
        return None, 0
    handles = [int(e.cuda_event) for e in events]
    if not all(handles):
        raise ValueError("record each event once before passing it (creates the HIP event)")
    return (ctypes.c_void_p * len(handles))(*handles), len(handles)


def _prepared_call(fn, name, args, device):
    """fn(*args) with the arguments converted once to their ctypes types (fn.argtypes); the call
    itself runs on `device` (the current device when the plan's is already current)."""
    if len(args) != len(fn.argtypes):
        raise TypeError(f"{name}: {len(args)} arguments for {len(fn.argtypes)} parameters")
    cargs = tuple(None if a is None else t(a) if not isinstance(a, ctypes.Array) else a
                  for a, t in zip(args, fn.argtypes))

    def run():
        if torch.cuda.current_device() != device.index:
            with torch.cuda.device(device):
                check(fn(*cargs), name)
        else:
            check(fn(*cargs), name)
    return run


class MUPlan:
    """Device state for the MU iterations on X (n_rows × F, samples-major, already on the GPU)."""

    def __init__(self, X: torch.Tensor, n_components: int, l1_W=0.0, l2_W=0.0, l1_H=0.0,
                 l2_H=0.0, group=None):
        if X.device.type != "cuda":
            raise ValueError("MUPlan needs X on a HIP device")
        if X.dtype not in _XDT:
            raise TypeError(f"unsupported X dtype {X.dtype}")
        if X.dim() != 2:
            raise ValueError("X must be 2-D")
        self.lib = _lib.load()
        self.X = X.contiguous()
        self.device = X.device
        self.n_rows, self.F = (int(s) for s in self.X.shape)
        self.k = int(n_components)
        self.xdt = _XDT[X.dtype]
        self.tc = torch.float64 if X.dtype == torch.float64 else torch.float32
        self.l1_W, self.l2_W, self.l1_H, self.l2_H = map(float, (l1_W, l2_W, l1_H, l2_H))
        self.group = group
        self.world = plan_world(group)
        KP = self.lib.cnmf_padded_k(self.k)
        if KP < 0:
            raise _lib.HipLibraryError(f"n_components={self.k} is not supported (1..16)")
        self.KP = KP
        self.V = self.F + self.k
        self.n_out = self.k * self.V
        with torch.cuda.device(self.device):
            nb = self.lib.cnmf_pass_blocks(self.n_rows, self.F, self.k, self.xdt)
        check(nb, "cnmf_pass_blocks")
        self.n_parts = int(nb)
        dev, f64 = self.device, torch.float64
        self.W = torch.empty((self.n_rows, self.k), dtype=self.tc, device=dev)
        self.H64 = torch.zeros((self.k, self.F), dtype=f64, device=dev)
        self.Ht = torch.zeros((self.F, KP), dtype=f64, device=dev)
        self.HHt = torch.zeros((KP, KP), dtype=f64, device=dev)
        # partial rows, stage and AB leave room for the loss column of the device tolerance test
        # (cnmf_mu_fit_tol: rows of n_out + 2 — the loss and a pad, ABI 302; the ALS form: n_out + 1);
        # the other launches use rows of n_out in the same memory
        self._partials = torch.zeros(max(self.n_parts, 1) * (self.n_out + 2), dtype=f64, device=dev)
        self.partials = self._partials[:max(self.n_parts, 1) * self.n_out].view(max(self.n_parts, 1), self.n_out)
        self.stage = torch.zeros(int(self.lib.cnmf_stage_doubles(self.n_out + 2)), dtype=f64, device=dev)
        self.counter = torch.zeros(int(self.lib.cnmf_counter_words()), dtype=torch.int32, device=dev)
        self.err_word = int(self.lib.cnmf_counter_err_word())
        with torch.cuda.device(self.device):
            p = self.lib.cnmf_mu_persistent(self.n_rows, self.F, self.k, self.xdt)
        self.persistent_shape = bool(check(p, "cnmf_mu_persistent"))  # the persistent kernel serves it
        # ...and its in-launch cross-rank exchange (the wave-tile shapes; cfg4's bf16 launch is one GPU only)
        with torch.cuda.device(self.device):
            xg = self.lib.cnmf_persist_workgroups(self.n_rows, self.F, self.k, self.xdt, 0, 1) if self.persistent_shape else 0
        self.exchange_shape = self.persistent_shape and int(xg) > 0
        # the persistent layouts tune() chooses between for this shape (include/cnmf_hip.h `layout`):
        # cfg4's bf16 shape: the per-iteration launches (4) or ONE persistent launch (6).  k = 8 fp32
        # takes the VALU wave tiles (4); the matrix-core tiles (5) lost on every box measured (cfg3
        # shard 150.6 vs 110.7 us, profiles/r05/) and live in the diagnostic library only (round 6)
        self.layouts = ()
        if self.xdt == _lib.BF16 and self.world == 1 and not self.persistent_shape:
            with torch.cuda.device(self.device):
                if int(self.lib.cnmf_persist_workgroups(self.n_rows, self.F, self.k, self.xdt, 6, 0)) > 0:
                    self.layouts = (4, 6)
        self.persistent = self.persistent_shape and self.world == 1  # ...as one multi-iteration launch
        self.layout = 0  # layout of the persistent launch (include/cnmf_hip.h; 0 = default); tune() sets it
        self.shard_steps = False  # True: the multi-GPU iteration (shard step + all_reduce) at any world
        self.exchange = False  # True: multi-GPU iterations as one launch per rank (enable_exchange)
        self._AB = torch.zeros(self.n_out + 2, dtype=f64, device=dev)
        self.AB = self._AB[:self.n_out]
        self.loss_buf = torch.zeros(1, dtype=f64, device=dev)
        self.stats = torch.zeros(2, dtype=f64, device=dev)
        self._wsnap = None  # the device tolerance test's W snapshot (streamed W), allocated on first use

    # -- multi-GPU with the all-reduce inside the launch ------------------------------------------
    def enable_exchange(self):
        """Set up the in-launch cross-rank all-reduce (cnmf_mu_iterations_multi): one fine-grained
        exchange buffer per rank, IPC-shared with every peer (handles via all_gather_object on the
        plan's group).  Collective: every rank of the group calls it.  Afterwards `iterate` runs
        n iterations as ONE launch per rank.  Raises (on every rank) when any rank's shard is not a
        persistent shape or any buffer cannot be shared; the plan then stays on the RCCL path."""
        dist = torch.distributed
        if self.group is None:
            raise RuntimeError("enable_exchange needs the plan's torch.distributed group (MUPlan(..., group=...))")
        if getattr(self.group, "is_local", False):
            return self._enable_exchange_local()
        rank = dist.get_rank(self.group)
        ok = torch.tensor([1.0 if self.exchange_shape else 0.0])
        handle, ptr, err = None, ctypes.c_void_p(), ""
        # peer reachability first: every peer's GPU that this process can see must be mappable
        devs = [None] * self.world
        dist.all_gather_object(devs, (rank, self._pci_bus_id(self.device.index)), group=self.group)
        local = {self._pci_bus_id(j): j for j in range(torch.cuda.device_count())}
        for r, bus in devs:
            j = local.get(bus)
            if r != rank and j is not None and j != self.device.index and \
                    self.lib.cnmf_device_can_access_peer(self.device.index, j) != 1:
                ok[0], err = 0.0, f"no peer access from device {self.device.index} to {j} ({bus})"
        if _fault("CNMF_FAULT_XCHG_SETUP"):
            ok[0], err = 0.0, "fault injected (CNMF_FAULT_XCHG_SETUP)"
        if self.exchange_shape and ok[0] != 0.0:
            hb = int(self.lib.cnmf_xbuf_handle_bytes())
            hbuf = ctypes.create_string_buffer(hb)
            with torch.cuda.device(self.device):
                st = self.lib.cnmf_xbuf_alloc(self.world, ctypes.byref(ptr), hbuf)
            if st < 0:
                ok[0], err = 0.0, self.lib.cnmf_last_error().decode()
            else:
                handle = hbuf.raw
        handles = [None] * self.world
        dist.all_gather_object(handles, (rank, float(ok[0]), handle, err), group=self.group)
        bad = [h for h in handles if h[1] == 0.0]
        if bad:
            if ptr.value:
                self.lib.cnmf_xbuf_free(ptr)
            raise _lib.HipLibraryError("in-launch exchange unavailable: " + "; ".join(
                f"rank {r}: {e or 'shard is not a persistent shape'}" for r, _, _, e in bad))
        opened, peers, err = [], [], ""
        with torch.cuda.device(self.device):
            for r, _, h, _ in sorted(handles, key=lambda x: x[0]):
                if r == rank:
                    peers.append(ptr.value)
                    continue
                q = ctypes.c_void_p()
                if self.lib.cnmf_xbuf_open(h, ctypes.byref(q)) < 0:
                    err = f"rank {rank} cannot open rank {r}'s buffer: " + self.lib.cnmf_last_error().decode()
                    break
                opened.append(q.value)
                peers.append(q.value)
        res = [None] * self.world
        dist.all_gather_object(res, err, group=self.group)
        if any(res):
            for q in opened:
                self.lib.cnmf_xbuf_close(ctypes.c_void_p(q))
            self.lib.cnmf_xbuf_free(ptr)
            raise _lib.HipLibraryError("in-launch exchange unavailable: " + "; ".join(e for e in res if e))
        self._xbuf, self._xopened = ptr.value, opened
        self.xctl = torch.zeros(int(check(self.lib.cnmf_xctl_words(self.world), "cnmf_xctl_words")),
                                dtype=torch.int64, device=self.device)
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_xctl_init(_ptr(self.xctl), (ctypes.c_void_p * self.world)(*peers),
                                          rank, self.world), "cnmf_xctl_init")
        self.xrank = rank
        self.exchange = True
        self.persistent = True
        self.shard_steps = False

    def _enable_exchange_local(self):
        """enable_exchange for shards driven by threads of ONE process (cnmf_amd.multidevice): the
        exchange buffers are mapped directly (peer access enabled between distinct devices), no IPC.
        Collective over the local group: raises on every shard when any shard cannot take part."""
        grp = self.group
        ptr, err = ctypes.c_void_p(), ""
        if not self.exchange_shape:
            err = f"shard {grp.rank()}: not a persistent shape with the in-launch exchange"
        else:
            hbuf = ctypes.create_string_buffer(int(self.lib.cnmf_xbuf_handle_bytes()))
            with torch.cuda.device(self.device):
                if self.lib.cnmf_xbuf_alloc(self.world, ctypes.byref(ptr), hbuf) < 0:
                    err = self.lib.cnmf_last_error().decode()
        infos = grp.all_gather((ptr.value, self.device.index, err))
        errs = [e for _, _, e in infos if e]
        if not errs:
            with torch.cuda.device(self.device):
                for _, d, _ in infos:
                    if d != self.device.index and self.lib.cnmf_enable_peer_access(self.device.index, d) < 0:
                        errs.append(f"device {self.device.index} -> {d}: " + self.lib.cnmf_last_error().decode())
        errs = [e for e in grp.all_gather("; ".join(errs)) if e]
        if errs:
            if ptr.value:
                self.lib.cnmf_xbuf_free(ptr)
            raise _lib.HipLibraryError("in-launch exchange unavailable: " + "; ".join(errs))
        peers = [p for p, _, _ in infos]
        self._xbuf, self._xopened = ptr.value, []
        self.xctl = torch.zeros(int(check(self.lib.cnmf_xctl_words(self.world), "cnmf_xctl_words")),
                                dtype=torch.int64, device=self.device)
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_xctl_init(_ptr(self.xctl), (ctypes.c_void_p * self.world)(*peers),
                                          grp.rank(), self.world), "cnmf_xctl_init")
        self.xrank = grp.rank()
        self.exchange = True
        self.persistent = True
        self.shard_steps = False

    def _pci_bus_id(self, dev: int) -> str:
        buf = ctypes.create_string_buffer(64)
        check(self.lib.cnmf_device_pci_bus_id(dev, buf, 64), "cnmf_device_pci_bus_id")
        return buf.value.decode().lower()

    def _inject_poison(self):
        """CNMF_FAULT_XCHG_POISON=1 (tests only): this rank's error word set before its first exchange
        launch — the launch's top combiner then tags its exchange words XPOISON (xchg_allreduce_n)."""
        if _fault("CNMF_FAULT_XCHG_POISON") and not getattr(self, "_poisoned", False):
            self._poisoned = True
            self.counter[self.err_word] = 1

    def disable_exchange(self):
        """Back to shard steps + RCCL (the buffers stay mapped until the plan is released)."""
        self.exchange = False
        self.persistent = self.persistent_shape and self.world == 1

    def release(self):
        """Unmap / free the exchange buffers (not collective; the GPU must be idle)."""
        if getattr(self, "_xbuf", None):
            torch.cuda.synchronize(self.device)
            for q in self._xopened:
                self.lib.cnmf_xbuf_close(ctypes.c_void_p(q))
            self.lib.cnmf_xbuf_free(ctypes.c_void_p(self._xbuf))
            self._xbuf, self._xopened = None, []
            self.exchange = False

    def use_shard_steps(self):
        """Run the multi-GPU iteration (one shard step + one all_reduce per iteration) even on a
        single rank — a diagnostic of that path's per-iteration cost."""
        self.shard_steps = True
        self.persistent = False
        if 6 in getattr(self, "layouts", ()):
            self.set_layout(4)

    # -- plumbing ------------------------------------------------------------------------------
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def set_W(self, W):
        self.W.copy_(torch.as_tensor(W).to(device=self.device, dtype=self.tc))

    def set_H(self, H):
        """Load H (k × F) into the fp64 master copy and derive Ht/HHt (no update)."""
        self.H64.copy_(torch.as_tensor(H).to(device=self.device, dtype=torch.float64))
        self.refresh_basis()

    def refresh_basis(self):
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_basis_update(None, _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                                             self.F, self.k, 0.0, 0.0, 0, None, self._stream()),
                  "cnmf_basis_update")

    # -- launches ------------------------------------------------------------------------------
    def sample_pass(self, flags: int):
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_mu_sample_pass(
                _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.Ht), _ptr(self.HHt),
                _ptr(self.partials), self.n_rows, self.F, self.k, self.l1_W, self.l2_W, flags,
                self._stream()), "cnmf_mu_sample_pass")

    def reduce(self, n_out: int, out: torch.Tensor):
        if self.n_rows == 0:  # an empty shard contributes zeros to the all-reduce
            out.zero_()
            return
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_reduce_partials(_ptr(self.partials), self.n_parts, n_out,
                                                _ptr(self.stage), _ptr(self.counter), _ptr(out),
                                                self._stream()), "cnmf_reduce_partials")

    def basis_update(self):
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_basis_update(_ptr(self.AB), _ptr(self.H64), _ptr(self.Ht),
                                             _ptr(self.HHt), self.F, self.k, self.l1_H, self.l2_H, 1,
                                             None, self._stream()), "cnmf_basis_update")

    def shard_step(self, apply_first: bool):
        if self.n_rows == 0:  # an empty shard (world > rows): the pending update, then zeros
            if apply_first:
                self.basis_update()
            self.AB.zero_()
            return
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_mu_shard_step(
                _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                _ptr(self.partials), self.n_parts, _ptr(self.stage), _ptr(self.counter),
                _ptr(self.AB), self.n_rows, self.F, self.k, self.l1_W, self.l2_W, self.l1_H,
                self.l2_H, int(apply_first), self.layout, self._stream()), "cnmf_mu_shard_step")

    def _allreduce(self, t: torch.Tensor):
        if self.world > 1 or (self.shard_steps and self.group is not None):
            if getattr(self.group, "is_local", False):
                self.group.all_reduce(t, "sum")
            else:
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=self.group)

    def check_sync_error(self):
        """Raise if a persistent launch gave up waiting for a workgroup (its results are invalid);
        synchronises the stream."""
        if getattr(self, "persistent", False) and int(self.counter[self.err_word].item()) != 0:
            code = int(self.counter[self.err_word].item())
            self.counter.zero_()  # tickets, pools and the error word: at rest for the next launch
            if getattr(self, "exchange", False):
                self.disable_exchange()  # the buffer set's flags are poisoned: never reuse it
                raise _lib.HipLibraryError(
                    f"multi-GPU persistent launch failed (code {code}: 1 = a local workgroup, 2 = a "
                    "peer rank timed out, 3 = a peer failed); the plan is back on the RCCL path and "
                    "the results of that launch are invalid")
            raise _lib.HipLibraryError("persistent MU launch timed out waiting for a workgroup "
                                       "(grid not co-resident?); results of that launch are invalid")

    def describe(self) -> str:
        """The persistent launch this plan's shape takes (kernel, layout, W residency, grid)."""
        buf = ctypes.create_string_buffer(256)
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_persist_describe(self.n_rows, self.F, self.k, self.xdt, self.layout, buf, 256),
                  "cnmf_persist_describe")
        return buf.value.decode()

    def counters_at_rest(self) -> bool:
        """Every ticket, flag, pool and the error word back at zero."""
        return int(self.counter.cpu().numpy().astype("int64").sum()) == 0

    def prepare(self, n_iter: int, pass_events=None):
        """A zero-argument callable that runs `iterate(n_iter, pass_events=...)`: for the one-launch
        paths the library call with its arguments marshalled up front (so a timed region holds the
        launch itself, not the host's argument conversion), else a plain call of iterate."""
        ev = _event_array(pass_events)
        if getattr(self, "exchange", False):
            fn, name = self.lib.cnmf_mu_iterations_multi, "cnmf_mu_iterations_multi"
            args = (n_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                    _ptr(self.partials), self.n_parts, _ptr(self.stage), _ptr(self.counter), _ptr(self.AB),
                    self.n_rows, self.F, self.k, self.l1_W, self.l2_W, self.l1_H, self.l2_H, _ptr(self.xctl),
                    self.layout, *ev, self._stream())
        elif self.world == 1 and not self.shard_steps and self.persistent:
            fn, name = self.lib.cnmf_mu_iterations, "cnmf_mu_iterations"
            args = (n_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                    _ptr(self.partials), self.n_parts, _ptr(self.stage), _ptr(self.counter), _ptr(self.AB), None,
                    self.n_rows, self.F, self.k, self.l1_W, self.l2_W, self.l1_H, self.l2_H, self.layout, *ev,
                    self._stream())
        else:
            return lambda: self.iterate(n_iter, pass_events=pass_events)
        return _prepared_call(fn, name, args, self.device)

    def iterate(self, n_iter: int, update_H: bool = True, pass_events=None):
        """n_iter MU iterations (SK:831-870) without host synchronisation.  pass_events: optional
        recorded-once torch.cuda.Event(enable_timing=True) list (single GPU only): 2 events around
        the one launch when self.persistent, else 2*n_iter events around each sample pass."""
        if n_iter <= 0:
            return
        if not update_H:
            for _ in range(n_iter):  # transform: W only, H (and Ht/HHt) fixed (SK:854 skipped)
                self.sample_pass(_lib.PASS_UPDATE_W)
            return
        if getattr(self, "exchange", False):
            self._inject_poison()
            with torch.cuda.device(self.device):
                check(self.lib.cnmf_mu_iterations_multi(
                    n_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht),
                    _ptr(self.HHt), _ptr(self.partials), self.n_parts, _ptr(self.stage),
                    _ptr(self.counter), _ptr(self.AB), self.n_rows, self.F, self.k,
                    self.l1_W, self.l2_W, self.l1_H, self.l2_H, _ptr(self.xctl), self.layout,
                    *_event_array(pass_events), self._stream()), "cnmf_mu_iterations_multi")
            return
        if self.world == 1 and not self.shard_steps and self.persistent_shape and not self.persistent:
            # kept off the persistent kernel (a launch of it failed): pass + reduce + update launches;
            # pass_events as documented (unrecorded events read ~0 s and an absurd rate)
            ev = list(pass_events) if pass_events is not None else None
            stream = torch.cuda.current_stream(self.device) if ev is not None else None
            whole = ev is not None and len(ev) == 2
            if ev is not None and not whole and len(ev) != 2 * n_iter:
                raise ValueError(f"pass_events: 2 or 2*n_iter events, got {len(ev)}")
            if whole:
                ev[0].record(stream)
            for i in range(n_iter):
                if ev is not None and not whole:
                    ev[2 * i].record(stream)
                self.sample_pass(_lib.PASS_UPDATE_W | _lib.PASS_ACCUMULATE)
                self.reduce(self.n_out, self.AB)
                self.basis_update()
                if ev is not None and not whole:
                    ev[2 * i + 1].record(stream)
            if whole:
                ev[1].record(stream)
            return
        if self.world == 1 and not self.shard_steps:
            with torch.cuda.device(self.device):
                check(self.lib.cnmf_mu_iterations(
                    n_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht),
                    _ptr(self.HHt), _ptr(self.partials), self.n_parts, _ptr(self.stage),
                    _ptr(self.counter), _ptr(self.AB), None, self.n_rows, self.F, self.k,
                    self.l1_W, self.l2_W, self.l1_H, self.l2_H, self.layout, *_event_array(pass_events),
                    self._stream()), "cnmf_mu_iterations")
            return
        # multi-GPU: per iteration ONE shard step (pending basis update from the all-reduced AB,
        # then this shard's W update and local [WᵀX | WᵀW] into AB) and ONE all_reduce of AB
        ev = list(pass_events) if pass_events is not None else None
        stream = torch.cuda.current_stream(self.device) if ev is not None else None
        for i in range(n_iter):
            if ev is not None:
                ev[2 * i].record(stream)
            self.shard_step(apply_first=i > 0)
            if ev is not None:
                ev[2 * i + 1].record(stream)
            self._allreduce(self.AB)
        self.basis_update()

    def tune(self, n_iter: int = 100, rounds: int = 2, variants=None) -> dict:
        """Time the layouts of the persistent launch (the `layout` argument, include/cnmf_hip.h:
        at k = 8, 4 = the VALU wave tiles and 5 = the matrix-core wave tiles; k = 4 has one layout in
        the product library, so there is nothing to time unless `variants` names some) on this
        plan's shape and keep the fastest for THIS plan.  Runs on copies of W and H: the plan's state is
        unchanged.  Collective over the plan's group: every rank times the same launches in the
        same order, the per-layout times are max-reduced over the ranks and every rank keeps the
        same layout (the ranks' launches must match: the in-launch exchange, and the shard steps'
        partial sums).  Call after the GPU has been busy for a while (the clock ramps up over the
        first ~35 ms of work).  Returns {layout: µs per iteration, the slowest rank's}.  No-op
        (empty dict) for non-persistent plans."""
        if variants is None:
            variants = self.layouts
        if len(variants) < 2 or (self.world > 1 and not self.persistent):
            return {}
        W0, H0 = self.W.clone(), self.H64.clone()
        keep = self.layout
        times = {v: [] for v in variants}
        try:
            for _ in range(rounds):
                for v in variants:
                    self.set_layout(v)
                    times[v].append(self._time_iterations(n_iter) * 1e6 / n_iter)
        finally:
            self.W.copy_(W0)
            self.H64.copy_(H0)
            self.refresh_basis()
            self.set_layout(keep)
        mean = [sum(times[v]) / len(times[v]) for v in variants]
        mean = dict(zip(variants, agree_max(mean, self.group if self.world > 1 else None, self.device)))
        self.set_layout(min(variants, key=lambda v: (mean[v], variants.index(v))))
        return mean

    def set_layout(self, layout: int):
        """The persistent layout of this plan's launches; layout 6 (cfg4's shape) makes the plan a
        one-launch persistent one, layout 4 there keeps the per-iteration launches."""
        self.layout = int(layout)
        if 6 in getattr(self, "layouts", ()):
            self.persistent = self.layout == 6

    def _time_iterations(self, n_iter: int) -> float:
        """Seconds of one n_iter launch on the plan's stream (HIP events); raises on a failed launch."""
        stream = torch.cuda.current_stream(self.device)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(stream)
        self.iterate(n_iter)
        ev[1].record(stream)
        torch.cuda.synchronize(self.device)
        self.check_sync_error()
        return ev[0].elapsed_time(ev[1]) / 1e3

    # -- the tolerance test on the device (cnmf_mu_fit_tol) -----------------------------------------
    _TC = {"tol": 0, "it0": 1, "init": 2, "prev": 3, "done": 4, "stopped": 5, "in_snap": 6, "wsnap": 7,
           "cap": 8, "nerr": 9, "errs": 16}

    def prepare_device_tol(self, max_iter: int, tol: float, pass_events=None):
        """(run, finish) for a max_iter fit with the tolerance test on the device (cnmf_mu_fit_tol):
        run() issues the ONE launch (arguments marshalled and the control block on the device
        beforehand), finish() synchronises and returns (n_iter, [(g, error)] for g = 0, 10, ...
        checked), restoring W from the snapshot when the test stopped a streamed-W fit.  None when
        the library does not serve this plan's shape (the caller runs the host loop)."""
        import numpy as np
        if not self.persistent or tol <= 0 or max_iter <= 0:  # the same on every rank
            return None
        xctl = _ptr(self.xctl) if getattr(self, "exchange", False) else None
        # this shard's eligibility, asked of the TOL kernel's own plan (bit 1), then agreed over the
        # plan's group: ranks that launched the exchange-plus-tol kernel would wait in
        # the exchange for a rank that took the host loop
        ok = self.n_rows > 0 and self._tol_served(xctl is not None)
        if self.world > 1 and agree_max([0.0 if ok else 1.0], self.group, self.device)[0] != 0.0:
            return None
        if not ok:
            return None  # not a wave-tile shape / layout: the host loop
        n_tc = int(check(self.lib.cnmf_tolctl_doubles(max_iter), "cnmf_tolctl_doubles"))
        if self._wsnap is None or self._wsnap.shape != self.W.shape:
            self._wsnap = torch.empty_like(self.W)
        host = np.zeros(n_tc, dtype=np.float64)
        host[self._TC["tol"]] = tol
        host[self._TC["cap"]] = n_tc - self._TC["errs"]
        host[self._TC["wsnap"]] = np.array([self._wsnap.data_ptr()], dtype=np.uint64).view(np.float64)[0]
        tolctl = torch.from_numpy(host).to(self.device)
        fn, args = self._tol_call(max_iter, tolctl, xctl, pass_events)
        cargs = tuple(None if a is None else t(a) if not isinstance(a, ctypes.Array) else a
                      for a, t in zip(args, fn.argtypes))
        state = {}

        def run():
            if torch.cuda.current_device() != self.device.index:
                with torch.cuda.device(self.device):
                    state["st"] = fn(*cargs)
            else:
                state["st"] = fn(*cargs)

        def finish(raise_on_error: bool = True):
            """(n_iter, errors); with raise_on_error=False a refused launch gives None (the caller
            agrees the fallback with its peers, as after a failed launch)."""
            if not raise_on_error and state.get("st", -1) < 0:
                import warnings
                warnings.warn(f"{fn.__name__}: {self.lib.cnmf_last_error().decode()}", RuntimeWarning)
                return None
            check(state.get("st", -1), fn.__name__)
            out = tolctl.cpu().numpy()
            if out[self._TC["stopped"]] != 0 and out[self._TC["in_snap"]] != 0:
                self.W.copy_(self._wsnap)
            nerr = min(int(out[self._TC["nerr"]]), n_tc - self._TC["errs"])
            return int(out[self._TC["done"]]), [(10 * i, float(out[self._TC["errs"] + i])) for i in range(nerr)]
        return run, finish

    def _tol_served(self, multi: bool) -> bool:
        """The TOL launch's own plan serves this shape (and layout, and the exchange when multi)."""
        with torch.cuda.device(self.device):
            probe = self.lib.cnmf_persist_workgroups(self.n_rows, self.F, self.k, self.xdt, self.layout,
                                                     (1 if multi else 0) | 2)
        return probe > 0 and "wave tiles" in self.describe()

    def _tol_call(self, max_iter, tolctl, xctl, pass_events):
        args = (max_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                _ptr(self._partials), self.n_parts, _ptr(self.stage), _ptr(self.counter), _ptr(self._AB),
                _ptr(tolctl), self.n_rows, self.F, self.k, self.l1_W, self.l2_W, self.l1_H, self.l2_H,
                self.layout, xctl, *_event_array(pass_events), self._stream())
        return self.lib.cnmf_mu_fit_tol, args

    def fit_device_tol(self, max_iter: int, tol: float, pass_events=None):
        """max_iter MU iterations with sklearn's tolerance test (SK:872-884) evaluated on the device:
        ONE launch, no host round trip per 10 iterations (cnmf_mu_fit_tol).  Returns
        (n_iter, [(g, error)] for g = 0, 10, ... checked), or None when the library does not serve
        this plan's shape (the caller then runs the host loop).  Synchronises once, at the end."""
        prep = self.prepare_device_tol(max_iter, tol, pass_events)
        if prep is None:
            return None
        run, finish = prep
        run()
        return finish()

    _NORMS = {"l1": 1, "l2": 2, "max": 3}

    def normalise(self, norm: str = "l2") -> torch.Tensor:
        """Normalisation projection: unit-norm basis rows, scales folded into W's
        columns (W·H unchanged).  Returns the k scales (fp64, on the device)."""
        if norm not in self._NORMS:
            raise ValueError(f"normalise must be one of {sorted(self._NORMS)} or None, got {norm!r}")
        scale = torch.empty(self.k, dtype=torch.float64, device=self.device)
        wdt = _lib.F64 if self.tc == torch.float64 else _lib.F32
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_normalise(_ptr(self.W), wdt, _ptr(self.H64), _ptr(self.Ht),
                                          _ptr(self.HHt), _ptr(scale), self.n_rows, self.F, self.k,
                                          self._NORMS[norm], self._stream()), "cnmf_normalise")
        return scale

    def frobenius_error(self) -> float:
        """sqrt(‖X − W·H‖²) over all ranks (SK:85-129 with square_root=True); synchronises."""
        if self.n_rows == 0:
            self.loss_buf.zero_()
        else:
            self.sample_pass(_lib.PASS_LOSS)
            self.reduce(1, self.loss_buf)
        self._allreduce(self.loss_buf)
        return math.sqrt(max(float(self.loss_buf.item()), 0.0))

    def H(self, dtype=None) -> torch.Tensor:
        return self.H64.to(dtype or self.tc)


def sync_failed(plan, local_failure: bool = False) -> bool:
    """check_sync_error() as a collective verdict: True on EVERY rank of the plan's group when the
    last launch failed on ANY rank (a rank deciding the fallback from its own error word
    alone re-runs a stretch its peers do not, and the collectives stop matching).  local_failure:
    this rank's launch was refused before it ran.  Synchronises."""
    import warnings
    failed = bool(local_failure)
    try:
        plan.check_sync_error()
    except _lib.HipLibraryError as e:
        failed = True
        warnings.warn(f"{e}; the stretch is re-run on the per-iteration path", RuntimeWarning)
    if plan.world > 1:
        failed = agree_max([1.0 if failed else 0.0], plan.group, plan.device)[0] != 0.0
    return failed


def _iterate_guarded(plan, n_iter: int, update_H: bool):
    """plan.iterate(n_iter) for a persistent plan, with a way back: W and H are snapshotted before
    the launch; if it reports a synchronisation failure on any rank (a workgroup never co-resident,
    a peer rank timed out: results invalid), EVERY rank restores its snapshot and re-runs the
    stretch on the per-iteration path (single GPU) or the RCCL path (multi-GPU).  Synchronises."""
    import warnings
    W0, H0 = plan.W.clone(), plan.H64.clone()
    plan.iterate(n_iter, update_H)
    if sync_failed(plan):
        if plan.world > 1:
            warnings.warn("a rank's persistent launch failed: every rank re-runs the stretch on the "
                          "RCCL path", RuntimeWarning)
        plan.W.copy_(W0)
        plan.H64.copy_(H0)
        plan.refresh_basis()
        if getattr(plan, "exchange", False):
            plan.disable_exchange()
        plan.exchange = False
        plan.persistent = False
        if 6 in getattr(plan, "layouts", ()):  # cfg4's persistent layout: back to its launches
            plan.set_layout(4)
        plan.iterate(n_iter, update_H)
        plan.check_sync_error()


def _run_mu_device_tol(plan, max_iter, tol, verbose, return_errors):
    """run_mu's tol > 0 fit as ONE launch with the test on the device; None when not served.  On a
    failed launch (any rank) every rank restores its state and returns None (the host loop runs)."""
    prep = plan.prepare_device_tol(max_iter, tol)  # collective: None on every rank or on none
    if prep is None:  # not served: nothing was launched
        return None
    W0, H0 = plan.W.clone(), plan.H64.clone()
    run, finish = prep
    with trace_range(f"cnmf:iterations 1..{max_iter} (device tol)"):
        run()
        res = finish(raise_on_error=False)
    if sync_failed(plan, local_failure=res is None):
        plan.W.copy_(W0)
        plan.H64.copy_(H0)
        plan.refresh_basis()
        if getattr(plan, "exchange", False):
            plan.disable_exchange()
        plan.exchange = False
        plan.persistent = False
        if 6 in getattr(plan, "layouts", ()):
            plan.set_layout(4)
        return None
    n_iter, errors = res
    if (verbose or return_errors) and n_iter == max_iter and max_iter % 10 == 0:
        errors.append((max_iter, plan.frobenius_error()))  # sklearn's check after the last iteration
    if verbose:
        for it, e in errors[1:]:
            print(f"Epoch {it:02d} reached, error: {e:f}")
    return n_iter, errors


def run_mu(plan: MUPlan, max_iter: int = 200, tol: float = 1e-4, update_H: bool = True,
           verbose: int = 0, return_errors: bool = False):
    """The driver of `_fit_multiplicative_update` (SK:731-893).  Returns n_iter (and the error
    trajectory [(n_iter, error)] when return_errors).  tol > 0 on a wave-tile persistent plan: ONE
    launch with the tolerance test on the device (MUPlan.fit_device_tol); else stretches of 10
    iterations with the error checked on the host between them."""
    if tol > 0 and update_H and hasattr(plan, "prepare_device_tol") and getattr(plan, "persistent", False):
        res = _run_mu_device_tol(plan, max_iter, tol, verbose, return_errors)
        if res is not None:
            return res if return_errors else res[0]
    errors = []
    if tol > 0:
        with trace_range("cnmf:loss it=0"):
            error_at_init = plan.frobenius_error()  # SK:827
        previous_error = error_at_init
        errors.append((0, error_at_init))
    it = 0
    while it < max_iter:
        stop = min(max_iter, (it // 10 + 1) * 10) if tol > 0 else max_iter
        with trace_range(f"cnmf:iterations {it + 1}..{stop}"):
            if getattr(plan, "persistent", False) and update_H:
                _iterate_guarded(plan, stop - it, update_H)
            else:
                plan.iterate(stop - it, update_H)
                if tol > 0 or stop >= max_iter:
                    plan.check_sync_error()
        it = stop
        if tol > 0 and it % 10 == 0:  # SK:872-884
            with trace_range(f"cnmf:loss it={it}"):
                error = plan.frobenius_error()
            errors.append((it, error))
            if verbose:
                print(f"Epoch {it:02d} reached, error: {error:f}")
            if (previous_error - error) / error_at_init < tol:
                break
            previous_error = error
    if return_errors:
        return it, errors
    return it


class ALSPlan(MUPlan):
    """Device state of the constrained-ALS variant (spec and oracle:
    oracle/als_ref.py, DESIGN.md §Constrained ALS).

    Per iteration: the W-step pass (exact per-sample FCLS, δ = sum_to_one; one HBM pass that also
    accumulates [WᵀX | WᵀW] of the new W), the deterministic fp64 reduction, (multi-GPU: one
    all_reduce of the k(F+k) accumulators,) and the H-step (one Gauss-Seidel sweep of exact
    smoothness-penalised NNLS rows, λ = smoothness) that also rebuilds the W-step's table."""

    def __init__(self, X: torch.Tensor, n_components: int, sum_to_one=0.0, smoothness=0.0, group=None):
        super().__init__(X, n_components, group=group)
        if self.k > 4:
            raise _lib.HipLibraryError(f"constrained ALS supports n_components <= 4 (got {self.k})")
        self.delta = float(sum_to_one or 0.0)
        self.lam = float(smoothness or 0.0)
        if self.delta < 0 or self.lam < 0:
            raise ValueError("sum_to_one and smoothness must be >= 0")
        self.table = torch.zeros(int(self.lib.cnmf_als_table_doubles()), dtype=torch.float64,
                                 device=self.device)
        with torch.cuda.device(self.device):
            p = self.lib.cnmf_als_persistent(self.n_rows, self.F, self.k, self.xdt)
        # one persistent launch per stretch of iterations (als_iter_wt_kernel), single GPU
        self.persistent_shape = bool(check(p, "cnmf_als_persistent"))
        self.exchange_shape = self.persistent_shape
        self.persistent = self.persistent_shape and self.world == 1

    def refresh_basis(self):
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_als_prepare(_ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                                            _ptr(self.table), self.F, self.k, self.delta,
                                            self._stream()), "cnmf_als_prepare")

    def w_step(self, accumulate: bool = True):
        if self.n_rows == 0:  # an empty shard (world > rows): reduce() then contributes zeros
            return
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_als_sample_pass(
                _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.Ht), _ptr(self.table),
                _ptr(self.partials), self.n_rows, self.F, self.k, self.delta, int(accumulate),
                self._stream()), "cnmf_als_sample_pass")

    def h_step(self):
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_als_basis_update(
                _ptr(self.AB), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt), _ptr(self.table),
                self.F, self.k, self.lam, self.delta, self._stream()), "cnmf_als_basis_update")

    def describe(self) -> str:
        if self.persistent:
            return ("als_iter_wt_kernel<PD=2, 2 workgroups per CU, MX>: wave tiles of 16 samples, "
                    "the W-step on the matrix cores (c = Hx and the 16 passive sets in fp64 MFMA), "
                    "in-launch reduction and H-step (one-wave BPP NNLS rows: Jacobi sweeps when "
                    "10*lambda <= B_jj/20, else block cyclic reduction; every workgroup)")
        return "ALS W-step pass + cnmf_reduce_partials + als_basis_kernel per iteration"

    def tune(self, *args, **kwargs) -> dict:
        return {}  # one layout

    def _tol_served(self, multi: bool) -> bool:
        """cnmf_als_fit_tol's plan serves this shard (the persistent shape with >= 5 tiles per wave;
        multi: the exchange form, tests/test_gpu_als.py::test_persistent_als_two_ranks_device_tol)."""
        with torch.cuda.device(self.device):
            probe = self.lib.cnmf_als_persist_workgroups(self.n_rows, self.F, self.k, self.xdt,
                                                         (1 if multi else 0) | 2)
        return probe > 0

    def _tol_call(self, max_iter, tolctl, xctl, pass_events):
        # the TOL launch writes the loss column: rows of n_out + 1 in the same memory
        args = (max_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                _ptr(self.table), _ptr(self._partials), self.n_parts, _ptr(self.stage), _ptr(self.counter),
                _ptr(self._AB), _ptr(tolctl), self.n_rows, self.F, self.k, self.delta, self.lam, xctl,
                *_event_array(pass_events), self._stream())
        return self.lib.cnmf_als_fit_tol, args

    def prepare(self, n_iter: int, pass_events=None):
        """As MUPlan.prepare, for the persistent ALS launch."""
        if not self.persistent:
            return lambda: self.iterate(n_iter, pass_events=pass_events)
        args = (n_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                _ptr(self.table), _ptr(self.partials), self.n_parts, _ptr(self.stage), _ptr(self.counter),
                _ptr(self.AB), self.n_rows, self.F, self.k, self.delta, self.lam)
        ev = _event_array(pass_events)
        if self.exchange:
            return _prepared_call(self.lib.cnmf_als_iterations_multi, "cnmf_als_iterations_multi",
                                  args + (_ptr(self.xctl), *ev, self._stream()), self.device)
        return _prepared_call(self.lib.cnmf_als_iterations, "cnmf_als_iterations",
                              args + (*ev, self._stream()), self.device)

    def iterate(self, n_iter: int, update_H: bool = True, pass_events=None):
        """n_iter ALS iterations; pass_events: 2 events around the one launch when self.persistent,
        else 2·n_iter events around each W-step pass."""
        if n_iter <= 0:
            return
        if self.persistent and update_H:
            args = (n_iter, _ptr(self.X), self.xdt, _ptr(self.W), _ptr(self.H64), _ptr(self.Ht),
                    _ptr(self.HHt), _ptr(self.table), _ptr(self.partials), self.n_parts,
                    _ptr(self.stage), _ptr(self.counter), _ptr(self.AB), self.n_rows, self.F, self.k,
                    self.delta, self.lam)
            with torch.cuda.device(self.device):
                if self.exchange:  # several GPUs: the AB all-reduce inside the launch (enable_exchange)
                    check(self.lib.cnmf_als_iterations_multi(*args, _ptr(self.xctl), *_event_array(pass_events),
                                                             self._stream()), "cnmf_als_iterations_multi")
                else:
                    check(self.lib.cnmf_als_iterations(*args, *_event_array(pass_events), self._stream()),
                          "cnmf_als_iterations")
            return
        ev = list(pass_events) if pass_events is not None else None
        stream = torch.cuda.current_stream(self.device) if ev is not None else None
        for i in range(max(n_iter, 0)):
            if ev is not None:
                ev[2 * i].record(stream)
            self.w_step(accumulate=update_H)
            if ev is not None:
                ev[2 * i + 1].record(stream)
            if not update_H:
                continue
            self.reduce(self.n_out, self.AB)
            self._allreduce(self.AB)
            self.h_step()


class WeightedMUPlan:
    """Device state of the weighted / masked MU (spec: oracle/wmu_ref.py).

    Per iteration: one pass over X and the weights M (`cnmf_wmu_sample_pass`: the W-step and the
    per-workgroup fp64 rows [W'ᵀ(M∘X) | W'ᵀ(M∘(W'H))]), the deterministic fp64 reduction, (multi-GPU:
    one all_reduce of the 2kF accumulators,) and the H-step (`cnmf_wmu_basis_update`).  The same
    driver (`run_mu`) runs it: W then H, the weighted error every 10 iterations when tol > 0.

    Single GPU at the served shape (fp32, F = 81, k = 4, rows a multiple of 16, W fits in LDS;
    `cnmf_wmu_persistent`): n iterations are ONE launch of the persistent weighted kernel
    (`cnmf_wmu_iterations`: pass, in-launch reduction and H-step per iteration)."""

    persistent = persistent_shape = exchange_shape = exchange = False

    def __init__(self, X: torch.Tensor, M: torch.Tensor, n_components: int, group=None):
        self.lib = _lib.load()
        if X.dtype != torch.float32 or M.dtype != torch.float32:
            raise TypeError("weighted MU takes float32 X and weights")
        if X.shape != M.shape or X.dim() != 2:
            raise ValueError(f"weights must have X's shape {tuple(X.shape)}, got {tuple(M.shape)}")
        if X.device.type != "cuda" or M.device.type != "cuda":
            raise _lib.HipLibraryError("WeightedMUPlan needs X and the weights in HIP device memory")
        self.X, self.M = X.contiguous(), M.contiguous()
        self.device = X.device
        self.n_rows, self.F = map(int, X.shape)
        self.k = int(n_components)
        self.tc = torch.float32
        self.group = group
        self.world = plan_world(group)
        with torch.cuda.device(self.device):
            nb = self.lib.cnmf_wmu_pass_blocks(self.n_rows, self.F, self.k)
        check(nb, "cnmf_wmu_pass_blocks")
        self.n_parts = int(nb)
        self.n_out = 2 * self.k * self.F
        dev, f64 = self.device, torch.float64
        self.W = torch.empty((self.n_rows, self.k), dtype=torch.float32, device=dev)
        self.H64 = torch.zeros((self.k, self.F), dtype=f64, device=dev)
        self.partials = torch.zeros((max(self.n_parts, 1), self.n_out), dtype=f64, device=dev)
        self.stage = torch.zeros(int(self.lib.cnmf_stage_doubles(self.n_out)), dtype=f64, device=dev)
        self.counter = torch.zeros(int(self.lib.cnmf_counter_words()), dtype=torch.int32, device=dev)
        self.AD = torch.zeros(self.n_out, dtype=f64, device=dev)
        self.loss_buf = torch.zeros(1, dtype=f64, device=dev)
        self.err_word = int(self.lib.cnmf_counter_err_word())
        with torch.cuda.device(self.device):
            p = self.lib.cnmf_wmu_persistent(self.n_rows, self.F, self.k)
        self.persistent_shape = bool(check(p, "cnmf_wmu_persistent"))
        self.exchange_shape = self.persistent_shape
        self.persistent = self.persistent_shape and self.world == 1

    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def set_W(self, W):
        self.W.copy_(torch.as_tensor(W).to(device=self.device, dtype=torch.float32))

    def set_H(self, H):
        self.H64.copy_(torch.as_tensor(H).to(device=self.device, dtype=torch.float64))

    def H(self, dtype=None) -> torch.Tensor:
        return self.H64.to(dtype or self.tc)

    def sample_pass(self, flags: int):
        if self.n_rows == 0:  # an empty shard: reduce() contributes zeros
            return
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_wmu_sample_pass(
                _ptr(self.X), _ptr(self.M), _ptr(self.W), _ptr(self.H64), _ptr(self.partials),
                self.n_parts, self.n_rows, self.F, self.k, flags, self._stream()), "cnmf_wmu_sample_pass")

    def reduce(self, n_out: int, out: torch.Tensor):
        if self.n_parts == 0:  # an empty shard contributes zeros to the all_reduce
            out.zero_()
            return
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_reduce_partials(_ptr(self.partials), self.n_parts, n_out,
                                                _ptr(self.stage), _ptr(self.counter), _ptr(out),
                                                self._stream()), "cnmf_reduce_partials")

    def _allreduce(self, t: torch.Tensor):
        if self.world > 1:
            if getattr(self.group, "is_local", False):
                self.group.all_reduce(t, "sum")
            else:
                torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=self.group)

    def refresh_basis(self):
        pass  # the weighted kernels read H64 itself

    def describe(self) -> str:
        if self.persistent:
            return ("wmu_iter_wt_kernel<k=4, W resident in LDS, PD=2>: wave tiles of 16 samples, X and the "
                    "weights prefetched together, one 4-wave workgroup per CU, in-launch reduction and H-step")
        return "wmu_pass_kernel + cnmf_reduce_partials + wmu_basis_kernel per iteration"

    def prepare(self, n_iter: int, pass_events=None):
        """As MUPlan.prepare, for the persistent weighted launch."""
        if not self.persistent:
            return lambda: self.iterate(n_iter, pass_events=pass_events)
        args = (n_iter, _ptr(self.X), _ptr(self.M), _ptr(self.W), _ptr(self.H64), _ptr(self.partials),
                self.n_parts, _ptr(self.stage), _ptr(self.counter), _ptr(self.AD), self.n_rows, self.F, self.k)
        ev = _event_array(pass_events)
        if self.exchange:
            return _prepared_call(self.lib.cnmf_wmu_iterations_multi, "cnmf_wmu_iterations_multi",
                                  args + (_ptr(self.xctl), *ev, self._stream()), self.device)
        return _prepared_call(self.lib.cnmf_wmu_iterations, "cnmf_wmu_iterations",
                              args + (*ev, self._stream()), self.device)

    def iterate(self, n_iter: int, update_H: bool = True, pass_events=None):
        """n_iter weighted MU iterations; pass_events: 2 events around the one launch when
        self.persistent, else 2·n_iter events recorded around each pass."""
        if n_iter <= 0:
            return
        if self.persistent and update_H:
            args = (n_iter, _ptr(self.X), _ptr(self.M), _ptr(self.W), _ptr(self.H64), _ptr(self.partials),
                    self.n_parts, _ptr(self.stage), _ptr(self.counter), _ptr(self.AD), self.n_rows, self.F,
                    self.k)
            with torch.cuda.device(self.device):
                if self.exchange:  # several GPUs: the [A | D] all-reduce inside the launch
                    check(self.lib.cnmf_wmu_iterations_multi(*args, _ptr(self.xctl), *_event_array(pass_events),
                                                             self._stream()), "cnmf_wmu_iterations_multi")
                else:
                    check(self.lib.cnmf_wmu_iterations(*args, *_event_array(pass_events), self._stream()),
                          "cnmf_wmu_iterations")
            return
        ev = list(pass_events) if pass_events is not None else None
        stream = torch.cuda.current_stream(self.device) if ev is not None else None
        for i in range(max(n_iter, 0)):
            if ev is not None:
                ev[2 * i].record(stream)
            self.sample_pass(_lib.PASS_UPDATE_W | (_lib.PASS_ACCUMULATE if update_H else 0))
            if ev is not None:
                ev[2 * i + 1].record(stream)
            if not update_H:
                continue
            self.reduce(self.n_out, self.AD)
            self._allreduce(self.AD)
            self.basis_update()

    def basis_update(self):
        """H <- H ∘ A / D from the (all-reduced) accumulators AD = [A | D]."""
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_wmu_basis_update(_ptr(self.AD), _ptr(self.H64), self.F, self.k,
                                                 self._stream()), "cnmf_wmu_basis_update")

    def check_sync_error(self):
        """Raise if the persistent launch gave up waiting for a workgroup (results invalid)."""
        if self.persistent_shape and int(self.counter[self.err_word].item()) != 0:
            self.counter.zero_()
            if self.exchange:
                self.disable_exchange()  # the buffer set's flags are poisoned: never reuse it
                raise _lib.HipLibraryError("multi-GPU persistent weighted MU launch failed; the plan is back "
                                           "on the RCCL path and the results of that launch are invalid")
            raise _lib.HipLibraryError("persistent weighted MU launch timed out waiting for a workgroup "
                                       "(grid not co-resident?); results of that launch are invalid")

    # the in-launch cross-rank exchange (MUPlan's: IPC-shared buffers, cnmf_xctl_init), for the
    # persistent weighted launch; collective over the plan's group
    enable_exchange = MUPlan.enable_exchange
    _enable_exchange_local = MUPlan._enable_exchange_local
    disable_exchange = MUPlan.disable_exchange
    release = MUPlan.release
    _pci_bus_id = MUPlan._pci_bus_id

    def frobenius_error(self) -> float:
        """sqrt(Σ m·(x − w·h)²) over all ranks; synchronises."""
        self.sample_pass(_lib.PASS_LOSS)
        self.reduce(1, self.loss_buf)
        self._allreduce(self.loss_buf)
        return math.sqrt(max(float(self.loss_buf.item()), 0.0))
