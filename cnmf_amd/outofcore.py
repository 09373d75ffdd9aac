"""Out-of-core MU: X stays in host memory and streams through HBM every iteration (SURVEY.md
§8(f3), "chunked streaming when N·F exceeds HBM").

An IOP cube larger than one GPU's HBM (or than a caller's memory budget) is fitted without ever
holding all of X on the device.  The rows are cut into chunks of `chunk_rows` (a multiple of 64,
the kernels' sample tile); `n_buffers` device buffers hold the chunks in flight.  Per iteration:

    for each chunk c (in row order):
        wait until chunk c's host->device copy has landed in its buffer
        cnmf_mu_shard_step(chunk c, apply_first=0)   W rows of c updated (W stays on the device:
                                                     N·k is 1/20 of X at F = 81, k = 4), the
                                                     chunk's [WᵀX | WᵀW] reduced into AB_chunks[c]
        release the buffer (an event) -> the copy stream refills it with the chunk n_buffers ahead
    cnmf_reduce_partials(AB_chunks)                  fixed chunk order: deterministic
    (multi-GPU: one all_reduce of AB, as MUPlan)
    cnmf_basis_update(AB)                            H, Hᵀ, HHᵀ for the next iteration

The copies run on their own stream, `n_buffers - 1` chunks ahead of the compute, so the PCIe
transfer of chunk c+1 overlaps the pass over chunk c; the iteration is bound by the host->device
rate (a pass over a resident chunk moves the same bytes ~100x faster).  The copy source is X's own
memory, page-locked in place with cnmf_host_register when it can be (an ordinary array); when it
cannot (a read-only file mapping, np.load(mmap_mode='r')) each chunk is first copied into one of
`n_buffers` pinned staging buffers on the host, which then bounds host memory to
n_buffers·chunk_rows rows as well.

The summation order depends only on the chunking, not on the copies: a plan whose chunks all fit
in its buffers (`n_buffers >= n_chunks`: loaded once, no per-iteration copy) gives the same
factors bit for bit — tests/test_gpu_outofcore.py uses that to check the streaming schedule.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from ._lib import check
from .solver import _XDT, _ptr, plan_world

__all__ = ["StreamedMUPlan", "chunk_bounds", "chunk_rows_for_budget"]

TILE = 64  # rows per sample tile of every pass kernel


def chunk_rows_for_budget(memory_budget: int, n_features: int, itemsize: int, n_buffers: int = 2) -> int:
    """Rows per chunk so that `n_buffers` chunk buffers of X fit `memory_budget` bytes (a multiple
    of the 64-row tile, at least one tile)."""
    rows = int(memory_budget) // (n_buffers * n_features * itemsize)
    return max(TILE, rows // TILE * TILE)


def chunk_bounds(n_rows: int, chunk_rows: int) -> list[tuple[int, int]]:
    """[lo, hi) row ranges of the chunks: `chunk_rows` each, the last one ragged."""
    if chunk_rows < 1:
        raise ValueError("chunk_rows must be >= 1")
    return [(lo, min(lo + chunk_rows, n_rows)) for lo in range(0, n_rows, chunk_rows)]


def _as_host_array(X):
    if isinstance(X, torch.Tensor):
        if X.device.type != "cpu":
            raise ValueError("StreamedMUPlan streams a host X; a device X fits in HBM already (MUPlan)")
        X = X.numpy()
    X = np.asarray(X)
    if X.ndim != 2:
        raise ValueError("X must be 2-D")
    if X.dtype not in (np.float32, np.float64):
        raise TypeError(f"unsupported X dtype {X.dtype} (float32 / float64)")
    if not X.flags.c_contiguous:
        raise ValueError("X must be C-contiguous (row-major samples)")
    return X


class StreamedMUPlan:
    """MU iterations over a host-resident X (n_rows × F), streamed through HBM in row chunks.
    Same interface as MUPlan for run_mu / the API: W (device), H64 / Ht / HHt, iterate,
    frobenius_error, normalise, H."""

    persistent = False
    exchange = False
    shard_steps = False

    def __init__(self, X, n_components: int, l1_W=0.0, l2_W=0.0, l1_H=0.0, l2_H=0.0, group=None,
                 device=None, memory_budget: int | None = None, chunk_rows: int | None = None,
                 n_buffers: int = 2, register: bool = True):
        self.src = _as_host_array(X)
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.n_rows, self.F = (int(s) for s in self.src.shape)
        self.k = int(n_components)
        tdt = torch.float32 if self.src.dtype == np.float32 else torch.float64
        self.xdt = _XDT[tdt]
        self.tc = tdt
        self.l1_W, self.l2_W, self.l1_H, self.l2_H = map(float, (l1_W, l2_W, l1_H, l2_H))
        self.group = group
        self.world = plan_world(group)
        KP = self.lib.cnmf_padded_k(self.k)
        if KP < 0:
            raise _lib.HipLibraryError(f"n_components={self.k} is not supported (1..16)")
        self.KP, self.V = KP, self.F + self.k
        self.n_out = self.k * self.V
        if n_buffers < 1:
            raise ValueError("n_buffers must be >= 1")
        itemsize = self.src.dtype.itemsize
        if chunk_rows is None:
            if memory_budget is None:
                raise ValueError("give memory_budget (bytes of device memory for X) or chunk_rows")
            chunk_rows = chunk_rows_for_budget(memory_budget, self.F, itemsize, n_buffers)
        self.chunk_rows = int(chunk_rows)
        if self.chunk_rows % TILE:
            raise ValueError(f"chunk_rows must be a multiple of {TILE}")
        self.chunks = chunk_bounds(self.n_rows, self.chunk_rows) if self.n_rows else []
        self.n_chunks = len(self.chunks)
        self.n_buffers = max(1, min(int(n_buffers), self.n_chunks))
        self.resident = self.n_chunks <= self.n_buffers  # every chunk has its own buffer: load once
        dev, f64 = self.device, torch.float64
        with torch.cuda.device(dev):
            nb = [int(check(self.lib.cnmf_pass_blocks(hi - lo, self.F, self.k, self.xdt), "cnmf_pass_blocks"))
                  for lo, hi in self.chunks]
        self.chunk_parts = nb
        self.n_parts = max(nb + [1])
        rows = min(self.chunk_rows, self.n_rows) if self.n_rows else 1
        self.bufs = [torch.empty((rows, self.F), dtype=tdt, device=dev) for _ in range(self.n_buffers)]
        self.W = torch.empty((self.n_rows, self.k), dtype=tdt, device=dev)
        self.H64 = torch.zeros((self.k, self.F), dtype=f64, device=dev)
        self.Ht = torch.zeros((self.F, KP), dtype=f64, device=dev)
        self.HHt = torch.zeros((KP, KP), dtype=f64, device=dev)
        self.partials = torch.zeros((self.n_parts, self.n_out), dtype=f64, device=dev)
        self.stage = torch.zeros(int(self.lib.cnmf_stage_doubles(self.n_out)), dtype=f64, device=dev)
        self.counter = torch.zeros(int(self.lib.cnmf_counter_words()), dtype=torch.int32, device=dev)
        self.AB_chunks = torch.zeros((max(self.n_chunks, 1), self.n_out), dtype=f64, device=dev)
        self.loss_chunks = torch.zeros(max(self.n_chunks, 1), dtype=f64, device=dev)
        self.AB = torch.zeros(self.n_out, dtype=f64, device=dev)
        self.AB_step = torch.zeros(self.n_out, dtype=f64, device=dev)
        self.loss_buf = torch.zeros(1, dtype=f64, device=dev)
        self.copy_stream = torch.cuda.Stream(dev)
        self._registered = False
        self._staging = None
        if not self.resident and self.n_rows:
            if register and self.src.flags.writeable:
                with torch.cuda.device(dev):
                    self._registered = self.lib.cnmf_host_register(self.src.ctypes.data, self.src.nbytes) == 0
            if not self._registered:  # pinned staging ring (host memory bounded to n_buffers chunks)
                self._staging = [torch.empty((rows, self.F), dtype=tdt, pin_memory=True) for _ in range(self.n_buffers)]
        self.mode = "resident" if self.resident else ("registered" if self._registered else "staged")
        self._ready = [None] * self.n_buffers     # event: the buffer's copy has landed
        self._consumed = [None] * self.n_buffers  # event: the compute reading the buffer is done
        self._staged = [None] * self.n_buffers    # event: the staging buffer's copy has drained
        self._next_seq = 0  # next chunk sequence number to copy (chunk = seq % n_chunks)
        self._use_seq = 0   # next chunk sequence number the compute reads
        with torch.cuda.device(dev):
            self.copy_stream.wait_stream(torch.cuda.current_stream(dev))  # buffers allocated there
        if self.resident and self.n_rows:
            with torch.cuda.device(dev):
                for c in range(self.n_chunks):
                    self._issue_copy(c, c)
                torch.cuda.current_stream(dev).wait_stream(self.copy_stream)

    # -- copies ---------------------------------------------------------------------------------
    def _issue_copy(self, seq: int, slot: int):
        lo, hi = self.chunks[seq % self.n_chunks]
        nbytes = (hi - lo) * self.F * self.src.dtype.itemsize
        dst = self.bufs[slot]
        if self.mode == "staged" and self._staging is None:  # after release(): a pinned ring, lazily
            self._staging = [torch.empty_like(b, device="cpu", pin_memory=True) for b in self.bufs]
        with torch.cuda.stream(self.copy_stream):
            if self._consumed[slot] is not None:
                self.copy_stream.wait_event(self._consumed[slot])
            if self._staging is not None:
                if self._staged[slot] is not None:
                    self._staged[slot].synchronize()  # the staging buffer's previous copy drained
                st = self._staging[slot]
                st[:hi - lo].numpy()[...] = self.src[lo:hi]
                src_ptr = st.data_ptr()
            else:
                src_ptr = self.src.ctypes.data + lo * self.F * self.src.dtype.itemsize
            check(self.lib.cnmf_copy_h2d_async(dst.data_ptr(), src_ptr, nbytes, self.copy_stream.cuda_stream),
                  "cnmf_copy_h2d_async")
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        self._ready[slot] = ev
        if self._staging is not None:
            self._staged[slot] = ev

    def _acquire(self, c: int) -> torch.Tensor:
        """The device buffer holding chunk c for the compute stream (copies issued ahead)."""
        if self.resident:
            return self.bufs[c]
        seq = self._use_seq
        assert seq % self.n_chunks == c
        while self._next_seq < seq + self.n_buffers:  # keep n_buffers chunks in flight
            self._issue_copy(self._next_seq, self._next_seq % self.n_buffers)
            self._next_seq += 1
        slot = seq % self.n_buffers
        torch.cuda.current_stream(self.device).wait_event(self._ready[slot])
        return self.bufs[slot]

    def _release(self, c: int):
        if self.resident:
            return
        slot = self._use_seq % self.n_buffers
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._consumed[slot] = ev
        self._use_seq += 1

    # -- plumbing (MUPlan's interface) ------------------------------------------------------------
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def set_W(self, W):
        self.W.copy_(torch.as_tensor(W).to(device=self.device, dtype=self.tc))

    def set_H(self, H):
        self.H64.copy_(torch.as_tensor(H).to(device=self.device, dtype=torch.float64))
        self.refresh_basis()

    def refresh_basis(self):
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_basis_update(None, _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
                                             self.F, self.k, 0.0, 0.0, 0, None, self._stream()),
                  "cnmf_basis_update")

    def basis_update(self):
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_basis_update(_ptr(self.AB), _ptr(self.H64), _ptr(self.Ht),
                                             _ptr(self.HHt), self.F, self.k, self.l1_H, self.l2_H, 1,
                                             None, self._stream()), "cnmf_basis_update")

    def _allreduce(self, t: torch.Tensor):
        if self.world > 1:
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=self.group)

    def check_sync_error(self):
        pass  # no persistent launch: every wait is a stream dependency

    def counters_at_rest(self) -> bool:
        return int(self.counter.cpu().numpy().astype("int64").sum()) == 0

    # -- iterations -----------------------------------------------------------------------------
    def _chunk_step(self, c: int, Xc: torch.Tensor):
        lo, hi = self.chunks[c]
        check(self.lib.cnmf_mu_shard_step(
            _ptr(Xc), self.xdt, _ptr(self.W[lo:hi]), _ptr(self.H64), _ptr(self.Ht), _ptr(self.HHt),
            _ptr(self.partials), self.n_parts, _ptr(self.stage), _ptr(self.counter),
            _ptr(self.AB_step), hi - lo, self.F, self.k, self.l1_W, self.l2_W, self.l1_H,
            self.l2_H, 0, 0, self._stream()), "cnmf_mu_shard_step")
        self.AB_chunks[c].copy_(self.AB_step)  # rows of n_out doubles need not be 16-byte aligned

    def _chunk_transform(self, c: int, Xc: torch.Tensor):
        lo, hi = self.chunks[c]
        check(self.lib.cnmf_mu_sample_pass(
            _ptr(Xc), self.xdt, _ptr(self.W[lo:hi]), _ptr(self.Ht), _ptr(self.HHt), _ptr(self.partials),
            hi - lo, self.F, self.k, self.l1_W, self.l2_W, _lib.PASS_UPDATE_W, self._stream()),
            "cnmf_mu_sample_pass")

    def _chunk_loss(self, c: int, Xc: torch.Tensor):
        lo, hi = self.chunks[c]
        check(self.lib.cnmf_mu_sample_pass(
            _ptr(Xc), self.xdt, _ptr(self.W[lo:hi]), _ptr(self.Ht), _ptr(self.HHt), _ptr(self.partials),
            hi - lo, self.F, self.k, 0.0, 0.0, _lib.PASS_LOSS, self._stream()), "cnmf_mu_sample_pass")
        check(self.lib.cnmf_reduce_partials(_ptr(self.partials), self.chunk_parts[c], 1, _ptr(self.stage),
                                            _ptr(self.counter), _ptr(self.loss_chunks[c:c + 1]),
                                            self._stream()), "cnmf_reduce_partials")

    def _sweep(self, fn):
        for c in range(self.n_chunks):
            Xc = self._acquire(c)
            fn(c, Xc)
            self._release(c)

    def iterate(self, n_iter: int, update_H: bool = True, pass_events=None):
        """n_iter MU iterations (SK:831-870), each one sweep over the chunks; no host
        synchronisation except for the staging copies (staged mode)."""
        if n_iter <= 0:
            return
        with torch.cuda.device(self.device):
            for _ in range(n_iter):
                if not update_H:
                    self._sweep(self._chunk_transform)
                    continue
                if self.n_chunks:
                    self._sweep(self._chunk_step)
                    check(self.lib.cnmf_reduce_partials(_ptr(self.AB_chunks), self.n_chunks, self.n_out,
                                                        _ptr(self.stage), _ptr(self.counter), _ptr(self.AB),
                                                        self._stream()), "cnmf_reduce_partials")
                else:
                    self.AB.zero_()
                self._allreduce(self.AB)
                self.basis_update()

    def frobenius_error(self) -> float:
        """sqrt(‖X − W·H‖²) over all chunks (and ranks), one streamed sweep; synchronises."""
        with torch.cuda.device(self.device):
            if self.n_chunks:
                self._sweep(self._chunk_loss)
                self.loss_buf.copy_(self.loss_chunks[:self.n_chunks].sum().reshape(1))
            else:
                self.loss_buf.zero_()
        self._allreduce(self.loss_buf)
        return math.sqrt(max(float(self.loss_buf.item()), 0.0))

    _NORMS = {"l1": 1, "l2": 2, "max": 3}

    def normalise(self, norm: str = "l2") -> torch.Tensor:
        if norm not in self._NORMS:
            raise ValueError(f"normalise must be one of {sorted(self._NORMS)} or None, got {norm!r}")
        scale = torch.empty(self.k, dtype=torch.float64, device=self.device)
        wdt = _lib.F64 if self.tc == torch.float64 else _lib.F32
        with torch.cuda.device(self.device):
            check(self.lib.cnmf_normalise(_ptr(self.W), wdt, _ptr(self.H64), _ptr(self.Ht),
                                          _ptr(self.HHt), _ptr(scale), self.n_rows, self.F, self.k,
                                          self._NORMS[norm], self._stream()), "cnmf_normalise")
        return scale

    def H(self, dtype=None) -> torch.Tensor:
        return self.H64.to(dtype or self.tc)

    def release(self):
        """Drain the copies and unlock X's pages (the plan keeps working in staged mode; its pinned
        staging ring is allocated only if it streams again)."""
        torch.cuda.synchronize(self.device)
        if self._registered:
            self.lib.cnmf_host_unregister(self.src.ctypes.data)
            self._registered = False
            self._staging = None
            self.mode = "staged"

    def __del__(self):
        try:
            if self._registered:
                torch.cuda.synchronize(self.device)
                self.lib.cnmf_host_unregister(self.src.ctypes.data)
        except Exception:
            pass
